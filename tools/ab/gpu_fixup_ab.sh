# Channel-grouped fix-up: exact-mode tests, then the per-call stem time with and without the
# fix-up for the default build and the variant libraries named as arguments, then a kernel
# trace of the default build.
set -u
O=gpurun_out/fixup_ab; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_stem.py tests/test_gpu_fused_parity.py -k "exact or correctly_rounded or seam" -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -4 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for v in base "$@"; do
  L=$PWD/term-quantization_amd/lib/libtq_hip.so; [ $v != base ] && L=$PWD/term-quantization_amd/lib/libtq_hip_$v.so
  echo "== $v"
  TQ_LIB_PATH=$L timeout -k 10 300 python3 tools/ab/stem_fix_count.py 64 256 > $O/count_$v.txt 2>&1
  rc=$?; grep -v amdgpu.ids $O/count_$v.txt; [ $rc -ne 0 ] && exit $rc
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/ab/stem_fix_count.py 64 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1
rc=$?; [ $rc -ne 0 ] && { tail -5 $GRAFT_REPO_ROOT/$O/prof.log; exit $rc; }
f=$(find $GRAFT_REPO_ROOT/$O/prof -name 'run_kernel_stats.csv' | head -1)
head -4 $f | cut -c1-200
echo done
