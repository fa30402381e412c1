# Where the fix-up kernel's time goes: timing-only builds (lib/libtq_hip_fab{1,2,3}.so:
# FIXUP_AB 1 no sums, 2 no window staging, 3 setup only) vs the product build, stem + fix-up
# call times at 64 and 256 images (results of the timing-only builds are not codes).
set -u
O=gpurun_out/fixup_diag; mkdir -p $O
for v in base fab1 fab2 fab3; do
  L=$PWD/term-quantization_amd/lib/libtq_hip.so; [ $v != base ] && L=$PWD/term-quantization_amd/lib/libtq_hip_$v.so
  TQ_LIB_PATH=$L timeout -k 10 300 python3 tools/ab/stem_fix_count.py 64 256 > $O/count_$v.txt 2>&1
  rc=$?; echo "== $v"; grep -E "==|us per" $O/count_$v.txt; [ $rc -ne 0 ] && exit $rc
done
echo done
