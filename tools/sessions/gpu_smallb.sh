#!/bin/bash
# Tile tuning of the low-load ResNet-50 buckets (batch 8 / 32 / 128) and a latency A/B of the merged table.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -n 6 "gpurun_out/$name.log"
  echo "=== $name rc=$rc"
  if [ $rc -ne 0 ]; then echo "STOP after $name"; exit $rc; fi
}
for b in ${SMALLB:-8 32 128}; do
  run "tune_b$b" 300 env B=$b TUNE_OUT=gpurun_out/tiles_b$b.json python -u bench/conv_tune_model.py resnet
done
python - <<'EOF' || exit 3
import glob, json
m = json.load(open("aiforearth_api_platform_amd/ops/conv_tiles.json"))
for p in sorted(glob.glob("gpurun_out/tiles_b*.json")):
    m.update(json.load(open(p)))
json.dump(m, open("gpurun_out/conv_tiles_smallb.json", "w"), indent=1, sort_keys=True)
EOF
run lat_repo 200 python -u bench/resnet_batch_latency.py
run lat_tuned 200 env AI4E_CONV_TILES=gpurun_out/conv_tiles_smallb.json python -u bench/resnet_batch_latency.py
run lat_repo2 200 python -u bench/resnet_batch_latency.py
run lat_tuned2 200 env AI4E_CONV_TILES=gpurun_out/conv_tiles_smallb.json python -u bench/resnet_batch_latency.py
echo "=== done"
