#!/bin/bash
# Round-2 GPU session: focused tests, smoke, bench (production serving path), optional full suite + profile.
# Each GPU step has its own time limit; any failure/fault/timeout stops the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -n 25 "gpurun_out/$name.log"
  echo "=== $name rc=$rc"
  if [ $rc -ne 0 ]; then echo "STOP after $name"; exit $rc; fi
}
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail gpurun_out/build.log; exit 3; }
if [ -n "${TESTS:-}" ]; then
  run focus 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider $TESTS
fi
if [ -n "${SMOKE:-}" ]; then
  run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
fi
if [ -n "${BENCH:-}" ]; then
  run bench 400 python -u bench.py ${BENCH_ARGS:-} --json-out gpurun_out/bench.json
fi
if [ -n "${FULL:-}" ]; then
  run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider
fi
if [ -n "${PROF:-}" ]; then
  run prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 20 --warmup 3 --http 0
fi
echo "=== done"
