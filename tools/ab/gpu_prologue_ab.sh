# Workgroup-prologue A/B: every setup load in flight before the first store (in-tree build)
# vs the load-store loops (lib/libtq_hip_oldpro.so: -DC64_WSTAGE=0 -DSETUP_UNROLL=0).
# Parity tests of the touched kernels first, then stem (+ exact fix-up) call times, then
# interleaved bench runs (default stem, then --stem exact).
set -u
O=gpurun_out/prologue_ab; mkdir -p $O
OLD=$PWD/term-quantization_amd/lib/libtq_hip_oldpro.so
timeout -k 10 900 python -u -m pytest tests/test_gpu_c64.py tests/test_gpu_stem.py tests/test_gpu_fused_parity.py -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for v in new old; do
  L=$PWD/term-quantization_amd/lib/libtq_hip.so; [ $v = old ] && L=$OLD
  TQ_LIB_PATH=$L timeout -k 10 300 python3 tools/ab/stem_fix_count.py 64 256 > $O/count_$v.txt 2>&1
  rc=$?; echo "== $v"; grep -E "==|us per" $O/count_$v.txt; [ $rc -ne 0 ] && exit $rc
done
for stem in fused exact; do
for r in 1 2 3; do for v in new old; do
  L=$PWD/term-quantization_amd/lib/libtq_hip.so; [ $v = old ] && L=$OLD
  TQ_LIB_PATH=$L timeout -k 10 300 python3 bench.py --stem $stem --no-d4 --no-d1 --no-cpu-baseline --no-stem-leg > $O/b_${stem}_${v}_$r.json 2> $O/b_${stem}_${v}_$r.err
  rc=$?; [ $rc -ne 0 ] && { tail -5 $O/b_${stem}_${v}_$r.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('$O/b_${stem}_${v}_$r.json').read().strip().splitlines()[-1]); print('$stem', '$v', round(d['value']), round(d['ms_per_step'],4), 'conv', round(d['roofline']['avg_launch_us'],2), 'stem', round(d['roofline_tr']['avg_launch_us'],1))"
done; done; done
echo done
