set -u
O=gpurun_out/r06g; mkdir -p $O
export TMPDIR=/tmp
for v in base fixab1 fixab2; do
  L=$PWD/term-quantization_amd/lib/libtq_hip.so; [ $v != base ] && L=$PWD/term-quantization_amd/lib/libtq_hip_$v.so
  TQ_LIB_PATH=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$v -o kt -- python3 tools/ab/stem_fix_count.py > $O/fix_count_$v.log 2>&1
  rc=$?; echo "== $v"; grep -E "listed|exact=" $O/fix_count_$v.log; [ $rc -ne 0 ] && { tail -5 $O/fix_count_$v.log; exit $rc; }
  python3 -c "
import csv
for r in csv.DictReader(open('$O/kt_$v/kt_kernel_stats.csv')):
    if 'stem' in r['Name']: print(r['Name'][:75], r['Calls'], round(float(r['AverageNs'])/1000,1))
"
done
echo done
