#!/bin/bash
# Kernel traces of the D4 MobileNet-V2 / EfficientNet-b0 runs (true kernel durations; the
# D4 events include host gaps when the GPU is starved), row-blocked dw vs flat.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r02dw2; mkdir -p $O; export TMPDIR=/tmp
for v in rows flat; do
  if [ $v = flat ]; then export TQ_DW_ROWS=0; else unset TQ_DW_ROWS; fi
  for m in mobilenet_v2 efficientnet_b0; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_${m}_$v -o kt -- python3 tools/bench_d4.py --only $m --steps 3 --warmup 1 > $O/kt_${m}_$v.log 2>&1 || { tail $O/kt_${m}_$v.log; exit 1; }
  done
done
find $O -name "*kernel_trace.csv" -delete; find $O -name "*.csv" ! -name "*kernel_stats.csv" -delete; du -sh $O; echo done
