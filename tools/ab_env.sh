#!/bin/bash
# A/B bench.py under alternating environment settings on one box: ab_env.sh "VAR=a" "VAR=b" [rounds]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 3
A=$1; B=$2; R=${3:-2}
for i in $(seq $R); do
  for e in "$A" "$B"; do
    env $e timeout -k 10 200 python bench.py --steps 60 --warmup 5 --http 0 > gpurun_out/ab.log 2>&1
    rc=$?
    echo "$e: $(grep '^{' gpurun_out/ab.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], 'gfx_mhz', d.get('gpu_telemetry', {}).get('gfx_mhz', {}).get('mean'), 'W', d.get('gpu_telemetry', {}).get('power_w', {}).get('mean'))")"
    if [ $rc -ne 0 ]; then echo "STOP rc=$rc"; tail -5 gpurun_out/ab.log; exit $rc; fi
  done
done
