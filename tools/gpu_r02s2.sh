#!/bin/bash
# Stem A/B: v3 (2-row passes + x prefetch, in-tree) vs ab2 (2-row, no prefetch) vs ab1 (4-row
# passes, committed r02_final): probe and bench, interleaved; stem tests on v3.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r02s2; mkdir -p $O
L=$R/term-quantization_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_gpu_stem.py tests/test_gpu_fused_parity.py -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1; rc=$?
tail -1 $O/t.log; [ $rc -ne 0 ] && { grep -E "Error|assert" $O/t.log | head; exit $rc; }
for rep in 1 2; do for v in v3 ab2 ab1; do
  if [ $v = v3 ]; then unset TQ_LIB_PATH; else export TQ_LIB_PATH=$L/libtq_hip_$v.so; fi
  echo -n "$v: "; timeout -k 10 120 python tools/stem_probe.py --iters 30 2>&1 | tail -1 || exit 1
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 > $O/b_${v}_$rep.json 2>$O/b.err || { tail $O/b.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/b_${v}_$rep.json').read().splitlines()[-1]); print('   bench', round(d['value']), round(d['roofline_tr']['avg_launch_us'],1))"
done; done
