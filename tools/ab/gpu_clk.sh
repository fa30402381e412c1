#!/bin/bash
# Sample shader clock / power / utilisation (rocm-smi, read-only) while bench.py runs a long
# timed region -- tells whether the MFMA loops run at full clock.
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --steps ${1:-8000} --warmup 5 > gpurun_out/clk_bench.log 2>&1 &
P=$!
for i in $(seq 1 30); do
  rocm-smi --showclocks --showpower --showuse 2>&1 | grep -E "sclk|Power \(W\)|GPU use" | tr -s ' ' | tr '\n' ' ' >> gpurun_out/clk.log
  echo >> gpurun_out/clk.log
  sleep 2
done
wait $P
