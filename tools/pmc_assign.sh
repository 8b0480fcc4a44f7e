#!/bin/bash
# PMC counters of the KMeans assign kernel (separate rocprofv3 passes).
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
export TMPDIR=/tmp AB_ONLY=${AB_ONLY:-3}
OUT=$R/gpurun_out/pmc_assign
mkdir -p $OUT
cd /tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-include-regex k_kmeans_assign3 -T -d $OUT/p$i -o run --output-format csv -- python3 $R/tools/kmeans_ab.py ${AB_ROWS:-2000000} > $OUT/p$i.log 2>&1 || exit $?
done
