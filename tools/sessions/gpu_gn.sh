set -o pipefail
mkdir -p gpurun_out/gn
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels2_gpu.py -k "groupnorm or gn" > gpurun_out/gn/pytest.log 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_models_gpu.py -k "unet or spatial" > gpurun_out/gn/pytest_models.log 2>&1 && \
timeout -k 10 300 python -u bench/landcover_bench.py > gpurun_out/gn/landcover.log 2>&1
rc=$?; tail -3 gpurun_out/gn/pytest.log; tail -3 gpurun_out/gn/pytest_models.log; tail -2 gpurun_out/gn/landcover.log; exit $rc
