#!/bin/bash
# Focused GPU check: given test files first, then the whole GPU suite, bench and a kernel-trace profile.
# Each GPU step has its own time limit; any fault/abort/timeout stops the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail gpurun_out/build.log; exit 3; }
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -n 30 "gpurun_out/$name.log"
  echo "=== $name rc=$rc"
  if [ $rc -ne 0 ]; then echo "STOP after $name"; exit $rc; fi
}
if [ -n "${TESTS:-}" ]; then
  run focus 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider $TESTS
fi
if [ -n "${FULL:-}" ]; then
  run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
fi
if [ -n "${BENCH:-}" ]; then
  run bench 300 python bench.py --steps 30 --warmup 5 --json-out gpurun_out/bench.json
fi
if [ -n "${PROF:-}" ]; then
  run prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 5 --warmup 2
fi
echo "=== done"
