set -o pipefail
mkdir -p gpurun_out/pair
export TMPDIR=/tmp
B=250 TUNE_PAIR=1 timeout -k 10 400 python -u bench/conv_tune_model.py resnet > gpurun_out/pair/tune_pair.log 2>&1
rc=$?; grep '^{' gpurun_out/pair/tune_pair.log | tail -20; exit $rc
