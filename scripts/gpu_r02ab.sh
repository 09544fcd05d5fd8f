#!/bin/bash
# PMC passes over the kernel microbenchmark (configs[2] shapes): MFMA busy / co-exec, wait shares,
# instruction-type activity, LDS conflicts -- one rocprofv3 --pmc pass per group
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_pmc_mb2.sh ab "262144 256 8" \
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE" \
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL GRBM_GUI_ACTIVE" &&
python3 scripts/pmc_summary.py gpurun_out/ab_pmc_summary.csv $(ls gpurun_out/pmcmb_ab_*/*counter_collection.csv gpurun_out/pmcmb_ab_*/*/*counter_collection.csv 2>/dev/null)
