#!/bin/bash
# PMC passes over tools/conv_pmc.py for one shape: tools/conv_pmc.sh TAG B C N k s p H W
set -o pipefail
tag=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out/cpmc_$tag
i=0
for p in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS" \
         "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
         "TCC_HIT_sum TCC_MISS_sum TA_TA_BUSY_sum TD_TD_BUSY_sum" "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_WAVES"; do
  timeout -s KILL 90 rocprofv3 --pmc $p -d gpurun_out/cpmc_$tag/p$i -o pmc --output-format csv -- python3 tools/conv_pmc.py "$@" 10 \
      > gpurun_out/cpmc_$tag/p$i.log 2>&1 || exit 1
  i=$((i+1))
done
