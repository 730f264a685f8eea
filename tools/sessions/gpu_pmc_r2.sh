set -o pipefail
bash tools/pmc_resnet.sh > gpurun_out/pmc_run.log 2>&1
rc=$?; cat gpurun_out/pmc_run.log | tail -8; [ $rc -eq 0 ] || exit $rc
python tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc_summary.txt 2>&1; rc=$?; head -70 gpurun_out/pmc_summary.txt; exit $rc
