# Exact-stem A/B: in-tree build vs lib/libtq_hip_sepfix.so (built with the option under test:
# FIX_FUSED=0, STEM_NRM_MFMA=1, a two-ahead fetch, the flat 2^-12 flag slack in turn): exact-mode
# tests, stem call times, then interleaved
# bench runs with the exact stem.
set -u
O=gpurun_out/fixfused_ab; mkdir -p $O
OLD=$PWD/term-quantization_amd/lib/libtq_hip_sepfix.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_stem.py tests/test_gpu_fused_parity.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for v in new old; do
  L=$PWD/term-quantization_amd/lib/libtq_hip.so; [ $v = old ] && L=$OLD
  TQ_LIB_PATH=$L timeout -k 10 300 python3 tools/ab/stem_fix_count.py 128 256 > $O/count_$v.txt 2>&1
  rc=$?; echo "== $v"; grep -E "==|listed|us per" $O/count_$v.txt; [ $rc -ne 0 ] && exit $rc
done
for r in 1 2 3; do for v in new old; do
  L=$PWD/term-quantization_amd/lib/libtq_hip.so; [ $v = old ] && L=$OLD
  TQ_LIB_PATH=$L timeout -k 10 300 python3 bench.py --stem exact --no-d4 --no-d1 --no-cpu-baseline --no-stem-leg > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err
  rc=$?; [ $rc -ne 0 ] && { tail -5 $O/b_${v}_$r.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('$O/b_${v}_$r.json').read().strip().splitlines()[-1]); print('$v', round(d['value']), round(d['ms_per_step'],4), 'conv', round(d['roofline']['avg_launch_us'],2), 'stem', round(d['roofline_tr']['avg_launch_us'],1))"
done; done
echo done
