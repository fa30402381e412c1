#!/bin/bash
# r03o: streaming depthwise kernel + stem contiguous tile order: tests, dw shapes A/B,
# MobileNet-V2 / EfficientNet-b0 D4 A/B, bench A/B vs lib/libtq_hip_base.so, stem FETCH.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-r03o}; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
BASE=$R/term-quantization_amd/lib/libtq_hip_base.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_stem.py \
    tests/test_gpu_fused_mbv2.py tests/test_gpu_fused_effnet.py -m gpu -x -q --timeout 300 \
    --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for A in "32 112 1" "96 112 2" "144 56 1" "144 56 2" "192 28 1" "192 28 2" "384 14 1" "576 14 1" "576 14 2" "960 7 1"; do
  set -- $A
  for M in 0 1 6; do
    echo -n "stream=$M "
    TQ_DW_STREAM=$M timeout -k 10 120 python tools/dw_probe.py --c $1 --hw $2 --stride $3 --iters 20 2>>$O/err.log | tail -1 || exit 1
  done
done | tee $O/dw_probe.txt
for M in 1 0; do
  echo "== TQ_DW_STREAM=$M"
  TQ_DW_STREAM=$M timeout -k 10 300 python tools/bench_d4.py --only mobilenet_v2 --steps 5 2>>$O/err.log | tail -1 | cut -c1-400 || exit 1
  TQ_DW_STREAM=$M timeout -k 10 300 python tools/bench_d4.py --only efficientnet_b0 --steps 5 2>>$O/err.log | tail -1 | cut -c1-400 || exit 1
done | tee $O/d4_ab.txt
for V in cur base cur base; do
  if [ $V = base ]; then export TQ_LIB_PATH=$BASE; else unset TQ_LIB_PATH; fi
  echo -n "$V "; timeout -k 10 300 python bench.py --no-cpu-baseline --no-d1 --no-d4 --steps 20 2>>$O/err.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('%.0f img/s conv %.1f us frac %.3f stem %.1f' % (d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['roofline_tr']['avg_launch_us']))" || exit 1
done | tee $O/bench_ab.txt
unset TQ_LIB_PATH
for V in cur base; do
  if [ $V = base ]; then export TQ_LIB_PATH=$BASE; else unset TQ_LIB_PATH; fi
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_$V -o pmc -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-d1 --no-d4 --streams 1 --launch eager > $O/pmc_$V.log 2>&1 || { tail $O/pmc_$V.log; exit 1; }
  python3 - $O/pmc_$V $V <<'PY'
import csv, glob, sys
tot = n = 0
for f in glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'stem_conv_pool' in r['Kernel_Name'] and r['Counter_Name'] == 'FETCH_SIZE':
            tot += float(r['Counter_Value']); n += 1
print(sys.argv[2], 'stem FETCH_SIZE records', n, 'KiB sum', tot)
PY
  find $O/pmc_$V -name '*.csv' -size +2M -delete
done | tee $O/stem_fetch.txt
