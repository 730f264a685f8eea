#!/bin/bash
# K1p session: numerics tests, the layer3/4 pair micro-bench, forward A/B with the pair on/off.
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
run pair_tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_pair_gpu.py
run pair_micro 200 python -u bench/pair_micro.py 250
run pair_ab 400 env B=250 python -u bench/forward_ab.py ${AB_VARIANTS:-pair=0 pair=1 pair=1,pairtile=64}
if [ -n "${BENCH:-}" ]; then
  run bench 400 python -u bench.py --steps 200 --warmup 10 --http 0 --json-out gpurun_out/bench.json
fi
echo "=== done"
