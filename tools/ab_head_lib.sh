#!/bin/bash
# Same-box A/B of the kernel library at HEAD against the build of commit 03cb0bc (before the fused RPN head's
# epilogue option in the 256-wide conv): ResNet-50 bench and land-cover bench, alternating, two rounds each.
#   aiforearth_api_platform_amd/_lib/libai4e_kernels_old03cb.so = `git archive 03cb0bc csrc/kernels` compiled with the _build.py flags
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail gpurun_out/build.log; exit 3; }
OLD=$PWD/aiforearth_api_platform_amd/_lib/libai4e_kernels_old03cb.so
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/hl_rn_new$i.log 2>&1 || exit 5
  AI4E_KERNEL_LIB=$OLD timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/hl_rn_old$i.log 2>&1 || exit 6
  timeout -k 10 300 python bench/landcover_bench.py > gpurun_out/hl_lc_new$i.log 2>&1 || exit 7
  AI4E_KERNEL_LIB=$OLD timeout -k 10 300 python bench/landcover_bench.py > gpurun_out/hl_lc_old$i.log 2>&1 || exit 8
done
for f in gpurun_out/hl_*.log; do echo "$f $(grep '^{' $f | tail -1 | cut -c1-140)"; done
