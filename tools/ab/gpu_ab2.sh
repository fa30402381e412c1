#!/bin/bash
# Interleaved bench A/B (new first): in-tree library vs lib/libtq_hip_old.so, R rounds.
T=gpurun_out/${TAG:-ab}
mkdir -p $T
OLD=$PWD/term-quantization_amd/lib/libtq_hip_old.so
for i in $(seq 1 ${R:-3}); do
  for v in new old; do
    if [ $v = old ]; then export TQ_LIB_PATH=$OLD; else unset TQ_LIB_PATH; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps ${STEPS:-50} > $T/b_${v}_$i.json 2> $T/b_${v}_$i.err || exit $?
    python3 -c "import json; d=json.loads(open('$T/b_${v}_$i.json').read().strip().splitlines()[-1]); print('$v', round(d['value']), round(d['roofline']['avg_launch_us'],1), round(d['roofline_tr']['avg_launch_us'],1))"
  done
done
