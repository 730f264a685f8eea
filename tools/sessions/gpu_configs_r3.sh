#!/bin/bash
# BASELINE configs 1, 3, 4, 5 through the API path on one GPU box at HEAD (each GPU step time-limited; stop on a
# fault / abort / time limit). Results -> gpurun_out/r3_configs/*.json
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3_configs
mkdir -p $O
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > $O/build.log 2>&1 || exit 3
run() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
  grep '^{' $O/$name.log | tail -1 | cut -c1-400; [ $rc -ne 0 ] && tail -5 $O/$name.log;
  if [ $rc -ne 0 ]; then echo "STOP rc=$rc"; exit $rc; fi; }
run cfg3_detector 400 python bench/api_bench.py --model detector --steps 20 --json-out $O/cfg3_detector_api.json
run cfg5_ensemble 400 python bench/api_bench.py --model ensemble --steps 20 --json-out $O/cfg5_ensemble_api.json
run cfg4_landcover 400 python bench/api_bench.py --model landcover --steps 10 --json-out $O/cfg4_landcover_api.json
run cfg1_echo 300 python bench/echo_bench.py --json-out $O/cfg1_echo.json
echo "=== done"
