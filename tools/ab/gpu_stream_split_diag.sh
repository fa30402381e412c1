# tools/ab/stream_split_diag.py with the in-tree build and lib/libtq_hip_sepfix.so
set -u
O=gpurun_out/ssdiag; mkdir -p $O
for v in new old; do
  L=$PWD/term-quantization_amd/lib/libtq_hip.so; [ $v = old ] && L=$PWD/term-quantization_amd/lib/libtq_hip_sepfix.so
  echo "== $v"
  TQ_LIB_PATH=$L timeout -k 10 400 python3 tools/ab/stream_split_diag.py 4 > $O/$v.txt 2>&1
  rc=$?; grep -v amdgpu.ids $O/$v.txt | tail -8; [ $rc -ne 0 ] && exit $rc
done
echo done
