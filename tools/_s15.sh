export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_INSTS_VALU SQ_WAVES -d gpurun_out/ic -o pmc --output-format csv -- python tools/prof_cases.py c3 c5 dmean --reps 2 > gpurun_out/ic.log 2>&1 && python tools/pmc_summary.py gpurun_out/ic > gpurun_out/ic.json
