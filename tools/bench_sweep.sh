#!/bin/bash
# Sweep bench.py settings on one GPU (each run time-limited; stop on fault).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 3
for cfg in "$@"; do
  echo "=== $cfg"
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 $cfg > gpurun_out/sweep.log 2>&1
  rc=$?
  grep '^{' gpurun_out/sweep.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], 'img/s p50', d['p50_task_latency_ms'], 'ms/step', d['ms_per_step'])" || tail -5 gpurun_out/sweep.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo STOP rc=$rc; exit $rc; fi
done
