#!/bin/bash
# SQ counter passes (three) of a probe command, summed per dispatch over the kernels whose
# name matches a pattern.  Usage: bash tools/gpu_pmc_cmd.sh <tag> <kernel substring> "<cmd>"
set -u
TAG=$1; PAT=$2; CMD=$3
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
S1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES"
S2="SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"
S3="SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
j=0
for S in "$S1" "$S2" "$S3"; do
  j=$((j+1))
  timeout -s KILL 90 rocprofv3 --pmc $S --output-format csv -d $O/p_$j -o p -- $CMD > $O/p_$j.log 2>&1 || { echo "pmc $j failed"; tail -3 $O/p_$j.log; }
done
python3 - "$O" "$PAT" <<'PY'
import csv, glob, collections, sys
O, pat = sys.argv[1], sys.argv[2]
tot = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob('%s/p_*/**/*counter_collection.csv' % O, recursive=True):
    for r in csv.DictReader(open(f)):
        if pat not in r['Kernel_Name']: continue
        tot[r['Counter_Name']] += float(r['Counter_Value']); n[r['Counter_Name']] += 1
for c in sorted(tot): print("  %-28s %14.0f" % (c, tot[c] / max(1, n[c])))
PY
