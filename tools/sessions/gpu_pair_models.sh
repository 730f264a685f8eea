#!/bin/bash
# K1p on the other ResNet-backbone APIs: detector (config 3) and ensemble (config 5) through the API path,
# pair off/on alternating on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/pair_models; mkdir -p $O
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > $O/build.log 2>&1 || exit 3
for round in 1 2; do
  for m in detector ensemble; do
    for v in 0 1; do
      AI4E_PAIR=$v timeout -k 10 300 python bench/api_bench.py --model $m --steps 20 --json-out $O/${m}_pair${v}_r$round.json > $O/${m}_pair${v}_r$round.log 2>&1
      rc=$?
      echo "$m pair=$v r$round rc=$rc $(python -c "import json; d=json.load(open('$O/${m}_pair${v}_r$round.json')); print(d['value'], d.get('unit'), d.get('p50_task_latency_ms'))" 2>/dev/null)"
      if [ $rc -ne 0 ]; then tail -5 $O/${m}_pair${v}_r$round.log; exit $rc; fi
    done
  done
done
echo "=== done"
