# Kernel trace (rocprofv3 --kernel-trace --stats) of the C5 encode per libgcow.so build: usage var1d_kt.sh LIB...
set -e
export TMPDIR=/tmp
for lib in "$@"; do
  n=$(basename $lib .so)
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_$n -o kt --output-format csv -- python tools/prof_cases.py c5 --reps 5 --lib $lib > gpurun_out/kt_$n.log 2>&1
  python3 -c "
import csv,sys
for r in csv.DictReader(open('gpurun_out/kt_$n/kt_kernel_stats.csv')):
    if 'gcow' in r['Name'] and 'fill' not in r['Name']: print('$n', r['Name'].split('(')[0][-34:], r['Calls'], round(float(r['AverageNs'])/1000,1), 'us')
"
done
