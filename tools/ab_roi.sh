#!/bin/bash
# Detection-kernel change (RoIAlign, NMS): numerics, then detector bench A/B of two kernel-library builds on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels2_gpu.py -k "roi or detector or nms" tests/test_models_gpu.py > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 4; }
tail -3 gpurun_out/t.log
for i in 1 2; do
  timeout -k 10 200 python bench/detector_bench.py > gpurun_out/det_new$i.log 2>&1 || exit 5
  AI4E_KERNEL_LIB=$PWD/build/ab/libai4e_kernels_old.so timeout -k 10 200 python bench/detector_bench.py > gpurun_out/det_old$i.log 2>&1 || exit 6
done
for f in gpurun_out/det_*.log; do echo "$f $(grep '^{' $f | cut -c1-110)"; done
