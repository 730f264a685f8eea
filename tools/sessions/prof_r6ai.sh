# Round 6, session AI: HEAD ResNet-50 PMC passes + the serving bench under a kernel trace (per-kernel stats)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 900 bash tools/pmc_resnet.sh > gpurun_out/pmc_ai.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/serve_prof -o serve -- python3 $R/bench.py --steps 50 --warmup 5 --http 0 > $R/gpurun_out/serve_prof.log 2>&1 || exit 2
