#!/bin/bash
# PMC passes (one rocprofv3 run per counter set) over a probe command.
# Usage: bash tools/gpu_pmc.sh <tag> <python script> [args...]
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python3 "$@" > $O/probe.txt 2>&1 || { cat $O/probe.txt; exit 1; }
cat $O/probe.txt
i=0
DEFAULT_SETS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU;SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE;FETCH_SIZE;WRITE_SIZE;TA_BUSY_avr TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"
IFS=';' read -ra SETS <<< "${PMC_SETS:-$DEFAULT_SETS}"  # PMC_SETS: counter sets separated by ';'
for SET in "${SETS[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $SET --output-format csv -d $O/p$i -o p -- python3 "$@" --iters 3 > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $O/p$i.log; }
done
python3 - <<PY
import csv, glob, collections
tot = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob('$O/p*/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name']
        if 'dwconv' not in k and 'conv2d' not in k: continue
        tot[r['Counter_Name']] += float(r['Counter_Value']); n[r['Counter_Name']] += 1
for c in sorted(tot): print("%-32s %16.0f per-dispatch-avg %14.0f" % (c, tot[c], tot[c] / max(1, n[c])))
PY
