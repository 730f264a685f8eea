#!/bin/bash
# Round-3 GPU session: smoke, benches at several step counts, extra command, focused tests, optional full
# suite + profile.
# Each GPU step has its own time limit; any failure/fault/timeout stops the session.
#   TESTS="tests/x.py"   focused pytest
#   SMOKE=1              __graft_entry__.smoke()
#   BENCHES="20:5 200:10"  bench.py --steps S --warmup W (--http 0 unless BENCH_HTTP=1), one JSON per run
#   FULL=1               pytest -m gpu
#   PROF=1               rocprofv3 kernel-trace stats of a short bench
#   EXTRA="cmd ..."      one more command (e.g. a bench/ script), 400 s limit
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
if [ -n "${SMOKE:-}" ]; then
  run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
fi
for sw in ${BENCHES:-}; do
  s=${sw%%:*}; w=${sw##*:}
  run "bench_s${s}_w${w}" 400 python -u bench.py --steps "$s" --warmup "$w" --http "${BENCH_HTTP:-0}" \
      --json-out "gpurun_out/bench_s${s}_w${w}.json"
done
if [ -n "${EXTRA:-}" ]; then
  run extra 400 $EXTRA
fi
if [ -n "${TESTS:-}" ]; then
  run focus 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider $TESTS
fi
if [ -n "${FULL:-}" ]; then
  run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider
fi
if [ -n "${PROF:-}" ]; then
  run prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 20 --warmup 3 --http 0
fi
echo "=== done"
