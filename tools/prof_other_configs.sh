#!/bin/bash
# Kernel-trace + stats of the non-headline BASELINE configs (detector, land-cover, ensemble), one rocprofv3 run each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out && export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 3
for c in "detector bench/detector_bench.py --steps 5 --warmup 2" \
         "landcover bench/landcover_bench.py --steps 2 --warmup 1" \
         "pipeline bench/pipeline_bench.py --steps 5 --warmup 2"; do
  set -- $c; name=$1; shift
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$name -o run -- python "$@" \
    > gpurun_out/prof_$name.log 2>&1
  rc=$?; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/prof_$name.log; exit $rc; fi
done
