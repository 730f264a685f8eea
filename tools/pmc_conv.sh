#!/bin/bash
# PMC counters for one K1 conv shape under two tile configs (kernel-trace + pmc only, no sys/runtime traces).
# usage: bash tools/pmc_conv.sh "N H W C K ks s" cfgA cfgB
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc_conv && export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 3
SHAPE=$1; shift
for cfg in "$@"; do
  i=0
  for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
             "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_MFMA"; do
    i=$((i+1))
    timeout -k 10 240 rocprofv3 --kernel-trace --pmc $set --output-format csv -d gpurun_out/pmc_conv -o cfg${cfg}_p$i -- python bench/conv_one.py $SHAPE $cfg 10 > gpurun_out/pmc_conv/cfg${cfg}_p$i.log 2>&1
    rc=$?; echo "cfg $cfg pass $i rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc_conv/cfg${cfg}_p$i.log; exit $rc; fi
  done
done
find gpurun_out/pmc_conv -name "*counter_collection.csv" | head
