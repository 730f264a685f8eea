set -o pipefail
mkdir -p gpurun_out
T=aiforearth_api_platform_amd/ops/conv_tiles.json
cp $T gpurun_out/tiles_old.json
timeout -k 10 400 python -u bench/conv_tune_model.py resnet --write > gpurun_out/tune.log 2>&1 || exit 5
cp $T gpurun_out/tiles_new.json
for i in 1 2; do
timeout -k 10 200 python bench.py --steps 60 --warmup 5 > gpurun_out/bench_new$i.log 2>&1 || exit 6
cp gpurun_out/tiles_old.json $T
timeout -k 10 200 python bench.py --steps 60 --warmup 5 > gpurun_out/bench_old$i.log 2>&1 || exit 7
cp gpurun_out/tiles_new.json $T
done
grep -h '^{' gpurun_out/bench_*.log | cut -c100-200
