#!/bin/bash
# Layer-1 conv baseline at HEAD: per-launch times of the fused executor, the layer-1 conv
# forms on their default engines (conv_probe), and one SQ counter pass per form.
# Usage: bash tools/ab/gpu_l1_base.sh <tag>
set -u
TAG=${1:-l1base}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 240 python3 tools/layer_times.py --steps 3 > $O/layers.txt 2>&1 || { tail -20 $O/layers.txt; exit 1; }
head -12 $O/layers.txt
FORMS=("--codes 1 --no-out" "--codes 1 --residual" "--codes 1 --residual --no-out")
for i in 0 1 2; do
  timeout -k 10 120 python3 tools/conv_probe.py --layer 1 --nonneg ${FORMS[$i]} --iters 30 > $O/probe$i.txt 2>&1 || { tail -5 $O/probe$i.txt; exit 1; }
  echo "form $i (${FORMS[$i]}): $(tail -1 $O/probe$i.txt)"
done
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
SQ2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC"
for i in 0 1; do
  for j in 1 2; do
    S=$SQ; [ $j = 2 ] && S=$SQ2
    timeout -s KILL 90 rocprofv3 --pmc $S --output-format csv -d $O/pmc${i}_$j -o p -- python3 tools/conv_probe.py --layer 1 --nonneg ${FORMS[$i]} --iters 3 > $O/pmc${i}_$j.log 2>&1 || { echo "pmc $i $j failed"; tail -3 $O/pmc${i}_$j.log; exit 1; }
  done
done
python3 - <<PY
import csv, glob, collections
for i in (0, 1):
    tot = collections.defaultdict(float); n = collections.Counter()
    for f in glob.glob('$O/pmc%d_*/**/*counter_collection.csv' % i, recursive=True):
        for r in csv.DictReader(open(f)):
            if 'conv2d' not in r['Kernel_Name']: continue
            tot[r['Counter_Name']] += float(r['Counter_Value']); n[r['Counter_Name']] += 1
    print("form", i)
    for c in sorted(tot): print("  %-30s per-dispatch %14.0f" % (c, tot[c] / max(1, n[c])))
PY
