#!/bin/bash
# A/B bench/api_bench.py under alternating environment settings on one box: ab_api.sh MODEL "VAR=a" "VAR=b" [rounds]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
M=$1; A=$2; B=$3; R=${4:-2}
for i in $(seq $R); do
  for e in "$A" "$B"; do
    env $e timeout -k 10 300 python bench/api_bench.py --model $M --steps 30 --warmup 3 > gpurun_out/ab_api.log 2>&1
    rc=$?
    echo "$e: $(grep '^{' gpurun_out/ab_api.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['p50_task_latency_ms'])")"
    if [ $rc -ne 0 ]; then echo "STOP rc=$rc"; tail -5 gpurun_out/ab_api.log; exit $rc; fi
  done
done
