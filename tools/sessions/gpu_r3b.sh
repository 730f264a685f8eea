#!/bin/bash
# Round-3 session B: build, focused chain tests, chain tile A/B (CHAIN_CFGS), bench, kernel-trace profile.
# Each GPU step has its own time limit; any failure stops the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail gpurun_out/build.log; exit 3; }
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -n 12 "gpurun_out/$name.log"
  echo "=== $name rc=$rc"
  if [ $rc -ne 0 ]; then echo "STOP after $name"; exit $rc; fi
}
[ -n "${TESTS:-}" ] && run focus 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider $TESTS
[ -n "${FULL:-}" ] && run pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider
[ -n "${SMOKE:-}" ] && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[ -n "${CHAIN_CFGS:-}" ] && run chain_ab 300 python -u bench/chain_patch_ab.py
[ -n "${MICRO:-}" ] && run micro 300 env CFGS=${MICRO_CFGS:-9,10} TWO=1 python -u bench/conv_micro.py $MICRO
[ -n "${RETUNE:-}" ] && run retune 900 env B=250 TUNE_PAIR=1 TUNE_REPS=${TUNE_REPS:-12} TUNE_OUT=gpurun_out/conv_tiles_retuned.json python -u bench/conv_tune_model.py resnet
[ -n "${PAIRMICRO:-}" ] && run pairmicro 300 env PAIR_TILES=$PAIRMICRO python -u bench/pair_micro.py
[ -n "${PAIRST:-}" ] && run pairst 300 python -u tools/pair_stamps.py
[ -n "${K256ST:-}" ] && run k256st 300 python -u tools/k256_stamps.py
[ -n "${CUSPLIT:-}" ] && run cusplit 400 python -u bench/cu_split_probe.py $CUSPLIT
[ -n "${BIGB:-}" ] && for bb in $BIGB; do run "bigb_$bb" 400 env B=$bb NO_SPLIT=1 NB=30 python -u bench/cu_split_probe.py; done
[ -n "${BENCH:-}" ] && run bench 300 python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench.json
[ -n "${BENCH2:-}" ] && run bench2 300 env $BENCH2 python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench2.json
[ -n "${PROF:-}" ] && run prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 5 --warmup 2
[ -n "${HBM:-}" ] && run hbm 200 python -u bench/hbm_probe.py
[ -n "${PROF2:-}" ] && run prof2 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof2 -o run -- python bench.py --steps 120 --warmup 10 --http 0
# AB="label:ENV=v ...|--bench-args;..." -> bench runs in that order (either part may be empty)
if [ -n "${AB:-}" ]; then
  IFS=';' read -ra CASES <<< "$AB"
  for c in "${CASES[@]}"; do
    lab=${c%%:*}; a=${c#*:}; envs=${a%%|*}; bargs=${a#*|}; [ "$bargs" = "$a" ] && bargs=""
    run "ab_$lab" 300 env $envs python bench.py --steps 20 --warmup 5 $bargs --json-out "gpurun_out/ab_$lab.json"
  done
fi
if [ -n "${PMC:-}" ]; then
  run pmc 700 bash tools/pmc_resnet.sh
  python tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc_summary.txt 2>&1; tail -3 gpurun_out/pmc_summary.txt
fi
echo "=== done"
