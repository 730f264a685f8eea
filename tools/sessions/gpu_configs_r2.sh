#!/bin/bash
# BASELINE configs 3-5 through the API path + the stock PyTorch comparator + the control-plane load test.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2_configs
export TMPDIR=/tmp
O=gpurun_out/r2_configs
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  tail -n 3 "$O/$name.log" | cut -c1-1500
  echo "=== $name rc=$rc"
  if [ $rc -ne 0 ]; then echo "STOP after $name"; exit $rc; fi
}
python -c "import __graft_entry__ as g; g.build()" > $O/build.log 2>&1 || exit 3
run cp_loadtest 120 python tools/cp_loadtest.py --workers 8 --seconds 5 --ingest-threads 8 --json-out $O/cp_loadtest.json
run detector 400 python bench/api_bench.py --model detector --steps 20 --json-out $O/cfg3_detector_api.json
run ensemble 400 python bench/api_bench.py --model ensemble --steps 20 --json-out $O/cfg5_ensemble_api.json
run landcover 400 python bench/api_bench.py --model landcover --steps 10 --json-out $O/cfg4_landcover_api.json
run torch_baseline 300 python bench/torch_baseline.py 250 20
echo "=== done"
