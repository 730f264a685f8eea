# JPEG on-GPU path: span-size sweep + kernel profile (round 6)
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_jpeg_gpu.py -x -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/jpeg_test.log 2>&1 || exit 1
for S in 4096 2048 1024; do
  timeout -k 10 200 python -u bench/jpeg_ingest_bench.py --gpu --threads 16 --seconds 4 --span-bits $S --json-out gpurun_out/jpeg_gpu_s$S.json > gpurun_out/jpeg_bench_s$S.log 2>&1 || exit 2
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/jpeg_prof -o jpeg -- python3 $R/bench/jpeg_ingest_bench.py --gpu --threads 16 --seconds 2 > $R/gpurun_out/jpeg_prof.log 2>&1 || exit 3
