#!/bin/bash
# Ring-engine timing ablations (tools/variant.sh builds libtq_hip_<name>.so) on chosen layers,
# then PMC passes of the product kernel on one layer.
# Usage: bash tools/gpu_ring_ab.sh <tag> "<layers>" "<variants>" [pmc layer]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=$1; LAYERS=$2; VARS=$3; PL=${4:-}
O=$R/gpurun_out/$TAG; mkdir -p $O
for L in $LAYERS; do
  timeout -k 10 120 python -u tools/conv_probe.py --layer $L --config 0 --codes 1 --residual --iters 30 2>/dev/null | grep layer | sed "s/^/default /" || exit 1
  for v in default $VARS; do
    lib=""; [ "$v" != default ] && lib=$R/term-quantization_amd/lib/libtq_hip_$v.so
    TQ_LIB_PATH=$lib timeout -k 10 120 python -u tools/conv_probe.py --layer $L --config 13 --codes 1 --residual --iters 30 2>/dev/null | grep layer | sed "s/^/$v /" || exit 1
  done
done
if [ -n "$PL" ]; then
  PMC_SETS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU;SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE;TCC_HIT_sum TCC_MISS_sum;FETCH_SIZE;WRITE_SIZE" \
    bash tools/gpu_pmc.sh $TAG/pmc tools/conv_probe.py --layer $PL --config 13 --codes 1 --residual --iters 10
fi
