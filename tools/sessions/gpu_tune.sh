#!/bin/bash
# Conv tile sweep (winners -> gpurun_out/conv_tiles.json) + bench.py sweep of the given option sets.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail gpurun_out/build.log; exit 3; }
TILES_OUT=gpurun_out/conv_tiles.json timeout -k 10 300 python bench/conv_tune.py --write > gpurun_out/conv_tune.log 2>&1
rc=$?; cat gpurun_out/conv_tune.log | tail -40
if [ $rc -ne 0 ]; then echo STOP tune rc=$rc; exit $rc; fi
for cfg in "$@"; do
  echo "=== $cfg"
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 $cfg > gpurun_out/sweep.log 2>&1
  rc=$?
  grep '^{' gpurun_out/sweep.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], 'img/s p50', d['p50_task_latency_ms'], 'ms/step', d['ms_per_step'])" || tail -5 gpurun_out/sweep.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo STOP rc=$rc; exit $rc; fi
done
