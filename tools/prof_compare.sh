#!/bin/bash
# Kernel-trace profiles of bench.py and of a bare graph-replay forward, for per-kernel comparison.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pb -o run -- python bench.py --steps 20 --warmup 5 > gpurun_out/pb.log 2>&1 || { echo pb failed; tail gpurun_out/pb.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pf -o run -- python bench/forward_ab.py chain64=1 > gpurun_out/pf.log 2>&1 || { echo pf failed; tail gpurun_out/pf.log; exit 1; }
tail -2 gpurun_out/pb.log gpurun_out/pf.log
