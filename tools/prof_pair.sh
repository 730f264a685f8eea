#!/bin/bash
# Kernel traces of eager batch-250 forwards with the K1p pair on and off (per-dispatch durations in situ).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail gpurun_out/build.log; exit 3; }
for v in ${PAIR_VARIANTS:-1 0}; do
  export AI4E_PAIR=$v
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_pair$v -o run -- python bench/profile_resnet.py 250 3 > gpurun_out/prof_pair$v.log 2>&1 || { echo "rocprof rc=$?"; tail gpurun_out/prof_pair$v.log; exit 1; }
  f=$(find gpurun_out/prof_pair$v -name 'run_kernel_trace.csv' | head -1)
  python tools/step_breakdown.py "$f" -v > gpurun_out/pair$v.breakdown.txt
  head -30 gpurun_out/pair$v.breakdown.txt
done
echo "=== done"
