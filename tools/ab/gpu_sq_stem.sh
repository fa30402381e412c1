#!/bin/bash
# SQ counters of the fused stem kernel (tools/stem_probe.py), one PMC pass per set.
set -u
TAG=${1:-sq_stem}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
cd "$R"
timeout -k 10 120 python tools/stem_probe.py > "$O/probe.txt" 2>&1 || { cat "$O/probe.txt"; exit 1; }
cat "$O/probe.txt"
i=0
for SET in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $SET --output-format csv -d "$O/p$i" -o p -- \
      python3 "$R/tools/stem_probe.py" --iters 3 > "$O/p$i.log" 2>&1 || { tail -5 "$O/p$i.log"; exit 1; }
done
echo done
