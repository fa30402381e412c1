#!/bin/bash
# Memory-path counters (TA / TCP / TCC) of one fused conv (tools/conv_probe.py), one pass each.
set -u
TAG=${1:-memctr}; shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
cd "$R"
i=0
for SET in "TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE" \
           "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
           "TCC_HIT_sum TCC_MISS_sum TCC_READ_REQ_LATENCY_sum TCC_READ_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $SET --output-format csv -d "$O/p$i" -o p -- \
      python3 "$R/tools/conv_probe.py" --iters 3 "$@" > "$O/p$i.log" 2>&1 || { tail -5 "$O/p$i.log"; exit 1; }
done
echo done
