#!/bin/bash
# A/B of the in-tree library against lib/libtq_hip_old.so (a build of an earlier commit):
# GPU tests, per-launch layer times and two interleaved bench runs each.  TAG=<dir> names
# the gpurun_out/ subdirectory.
mkdir -p gpurun_out/${TAG:-ab1}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG:-ab1}/gputests.log 2>&1 && tail -2 gpurun_out/${TAG:-ab1}/gputests.log && \
TQ_LIB_PATH=$PWD/term-quantization_amd/lib/libtq_hip_old.so timeout -k 10 200 python tools/layer_times.py > gpurun_out/${TAG:-ab1}/lt_old.txt 2>&1 && \
timeout -k 10 200 python tools/layer_times.py > gpurun_out/${TAG:-ab1}/lt_new.txt 2>&1 && \
TQ_LIB_PATH=$PWD/term-quantization_amd/lib/libtq_hip_old.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/${TAG:-ab1}/b_old.json 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/${TAG:-ab1}/b_new.json 2>&1 && \
TQ_LIB_PATH=$PWD/term-quantization_amd/lib/libtq_hip_old.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/${TAG:-ab1}/b_old2.json 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/${TAG:-ab1}/b_new2.json 2>&1; echo rc=$?
