#!/bin/bash
# SQ counter passes of the c64 engine (conv_probe, layer 1) for the product build and variant
# builds.  Usage: bash tools/gpu_c64_pmc.sh <tag> <form 0|1|2> <variant>...
set -u
TAG=$1; F=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
FORMS=("--codes 1 --no-out" "--codes 1 --residual" "--codes 1 --residual --no-out")
S1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES"
S2="SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"
S3="SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_SALU GRBM_GUI_ACTIVE"
for v in base "$@"; do
  if [ $v = base ]; then unset TQ_LIB_PATH; else export TQ_LIB_PATH=$R/term-quantization_amd/lib/libtq_hip_$v.so; fi
  j=0
  for S in "$S1" "$S2" "$S3"; do
    j=$((j+1))
    timeout -s KILL 90 rocprofv3 --pmc $S --output-format csv -d $O/${v}_$j -o p -- python3 tools/conv_probe.py --layer 1 --nonneg --config 15 ${FORMS[$F]} --iters 3 > $O/${v}_$j.log 2>&1 || { echo "pmc $v $j failed"; tail -3 $O/${v}_$j.log; }
  done
done
python3 - "$O" base "$@" <<'PY'
import csv, glob, collections, sys
O = sys.argv[1]
for v in sys.argv[2:]:
    tot = collections.defaultdict(float); n = collections.Counter()
    for f in glob.glob('%s/%s_*/**/*counter_collection.csv' % (O, v), recursive=True):
        for r in csv.DictReader(open(f)):
            if 'c64' not in r['Kernel_Name']: continue
            tot[r['Counter_Name']] += float(r['Counter_Value']); n[r['Counter_Name']] += 1
    print("==", v)
    for c in sorted(tot): print("  %-28s %14.0f" % (c, tot[c] / max(1, n[c])))
PY
