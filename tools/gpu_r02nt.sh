#!/bin/bash
# Non-temporal fp32 output stores (ntA) / + non-temporal residual loads (ntB) vs base, bench
# interleaved: keep the next conv's codes in L2 / MALL instead of the fp32 tensors.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r02nt; mkdir -p $O
L=$R/term-quantization_amd/lib
for rep in 1 2 3; do for v in base ntA ntB; do
  if [ $v = base ]; then unset TQ_LIB_PATH; else export TQ_LIB_PATH=$L/libtq_hip_$v.so; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 40 > $O/b_${v}_$rep.json 2>$O/b.err || { tail $O/b.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/b_${v}_$rep.json').read().splitlines()[-1]); print('$v', round(d['value']), round(d['roofline']['avg_launch_us'],1))"
done; done
