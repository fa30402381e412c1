#!/bin/bash
# r03m: SQ/LDS counter passes of the patch engine (layer 11), the direct engine (layers 2, 6)
# and the strip engine (layer 1) at HEAD (conv_probe, 3 launches each).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-r03m}
export PMC_SETS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU;SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE;SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_FLAT"
bash tools/gpu_pmc.sh $TAG/l11 tools/conv_probe.py --layer 11 --codes 1 && \
bash tools/gpu_pmc.sh $TAG/l6 tools/conv_probe.py --layer 6 --codes 1 && \
bash tools/gpu_pmc.sh $TAG/l2 tools/conv_probe.py --layer 2 --codes 1 --residual && \
bash tools/gpu_pmc.sh $TAG/l1 tools/conv_probe.py --layer 1 --codes 1
