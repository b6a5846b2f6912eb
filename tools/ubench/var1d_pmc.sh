#!/bin/bash
# SQ instruction counts of the 1-D variable-rate encoder builds (product + ab/v1ab_*.so) on C5 (prof_cases.py c5).
export TMPDIR=/tmp
for lib in product "$@"; do
  extra=""; [ "$lib" != product ] && extra="--lib ab/v1ab_$lib.so"
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU -d gpurun_out/pmc_$lib -o pmc --output-format csv -- python tools/prof_cases.py c5 --reps 2 $extra > gpurun_out/pmc_$lib.log 2>&1 || exit $?
  python tools/pmc_summary.py gpurun_out/pmc_$lib > gpurun_out/pmc_$lib.json
done
