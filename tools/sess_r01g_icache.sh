#!/bin/bash
# instruction-cache behaviour of the C3 kernels (one counter block per pass)
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && tools/gpu_session.sh \
  "90|ic1|timeout -s KILL 60 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS --output-format csv -d gpurun_out/ic1 -o pmc -- python3 tools/prof_cases.py c3 --reps 2" \
  "90|ic2|timeout -s KILL 60 rocprofv3 --pmc SQ_IFETCH SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/ic2 -o pmc -- python3 tools/prof_cases.py c3 --reps 2"
