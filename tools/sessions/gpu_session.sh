#!/bin/bash
# One GPU-box session: tests, bench, kernel-trace profile. Each GPU step has its own time limit;
# a fault/abort/timeout (rc not in {0,1}) stops the session (no further GPU work).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
MODE=${1:-all}
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo build failed; tail gpurun_out/build.log; exit 3; }
if [[ $MODE == all || $MODE == test ]]; then
  step pytest_gpu 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider
fi
if [[ $MODE == all || $MODE == bench ]]; then
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
  step bench 600 python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench.json
fi
if [[ $MODE == all || $MODE == prof ]]; then
  step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 5 --warmup 2
fi
echo "=== session done"
