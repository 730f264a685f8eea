#!/bin/bash
# All BASELINE configs on one GPU box (each GPU step time-limited; stop on fault). Results -> gpurun_out/*.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 3
run() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?;
  grep '^{' gpurun_out/$name.log | tail -1 | cut -c1-600; [ $rc -ne 0 ] && tail -5 gpurun_out/$name.log;
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP rc=$rc"; exit $rc; fi; }
run cfg2_resnet50 300 python bench.py --steps 60 --warmup 5 --json-out gpurun_out/cfg2_resnet50.json
run cfg3_detector 300 python bench/detector_bench.py --json-out gpurun_out/cfg3_detector.json
run cfg4_landcover 300 python bench/landcover_bench.py --json-out gpurun_out/cfg4_landcover.json
run cfg5_pipeline 300 python bench/pipeline_bench.py --json-out gpurun_out/cfg5_pipeline.json
run cfg1_echo 300 python bench/echo_bench.py --json-out gpurun_out/cfg1_echo.json
run comparator 300 python bench/comparator_refstyle.py --json-out gpurun_out/comparator.json
echo "=== done"
