set -o pipefail
mkdir -p gpurun_out/k9
export TMPDIR=/tmp
timeout -k 10 240 python -u bench/race_screen_256.py --reps 40 > gpurun_out/k9/race.log 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "tile" > gpurun_out/k9/pytest.log 2>&1 && \
B=250 timeout -k 10 400 python -u bench/conv_tune_model.py resnet > gpurun_out/k9/tune.log 2>&1
rc=$?; tail -3 gpurun_out/k9/race.log; tail -3 gpurun_out/k9/pytest.log; tail -15 gpurun_out/k9/tune.log; [ $rc -eq 0 ] || exit $rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 100 --warmup 10 --json-out gpurun_out/k9/bench.json > gpurun_out/k9/bench.log 2>&1
rc=$?; tail -2 gpurun_out/k9/bench.log; [ $rc -eq 0 ] || exit $rc
