# The FIX stem kernel's own cost: timing-only builds (STEM_FIXAB 1 no window norms, 2 no
# flags) and the VALU window norms (STEM_NRM_MFMA=0, a product option) vs the in-tree build;
# stem (+ its fix-up tail) per call at 256 images.
set -u
O=gpurun_out/fixdiag2; mkdir -p $O
for v in base fixab1 fixab2 nrm0; do
  L=$PWD/term-quantization_amd/lib/libtq_hip.so; [ $v != base ] && L=$PWD/term-quantization_amd/lib/libtq_hip_$v.so
  TQ_LIB_PATH=$L timeout -k 10 300 python3 tools/ab/stem_fix_count.py 256 > $O/count_$v.txt 2>&1
  rc=$?; echo "== $v"; grep -E "listed|us per" $O/count_$v.txt; [ $rc -ne 0 ] && exit $rc
done
echo done
