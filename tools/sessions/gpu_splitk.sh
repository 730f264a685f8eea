set -o pipefail
mkdir -p gpurun_out/sk
export TMPDIR=/tmp
timeout -k 10 300 python -u bench/race_screen_256.py --reps 40 > gpurun_out/sk/race.log 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "tile" > gpurun_out/sk/pytest.log 2>&1 && \
B=250 timeout -k 10 400 python -u bench/conv_tune_model.py resnet > gpurun_out/sk/tune.log 2>&1 && \
B=250 TUNE_PAIR=1 timeout -k 10 400 python -u bench/conv_tune_model.py resnet > gpurun_out/sk/tune_pair.log 2>&1
rc=$?; tail -3 gpurun_out/sk/race.log; tail -3 gpurun_out/sk/pytest.log; grep '^{' gpurun_out/sk/tune.log | tail -14; grep '^{' gpurun_out/sk/tune_pair.log | tail -14; exit $rc
