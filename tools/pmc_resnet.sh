#!/bin/bash
# PMC counter passes over eager ResNet-50 forwards (bench/profile_resnet.py), one rocprofv3 run per pass;
# PMC_MODEL=detector|unet profiles the config-3 / config-4 forwards instead (bench/profile_model.py),
# output in gpurun_out/pmc_<model>.
# Each pass stays within the per-block limits (<= 8 SQ, <= 4 TCC: FETCH_SIZE takes 3, WRITE_SIZE 2).
# Summarize with: python tools/pmc_summary.py gpurun_out/pmc  (detector/unet: --start spin_kernel --by-kernel)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pmc
PROG="bench/profile_resnet.py ${B:-250} 2"
if [ -n "${PMC_MODEL:-}" ]; then OUT=gpurun_out/pmc_$PMC_MODEL; PROG="bench/profile_model.py $PMC_MODEL"; fi
mkdir -p $OUT && export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 3
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES" \
           "SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
           "FETCH_SIZE TCC_HIT_sum" \
           "WRITE_SIZE TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $set --output-format csv -d $OUT -o pass$i -- python $PROG > $OUT/pass$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $OUT/pass$i.log; exit $rc; fi
done
ls $OUT
