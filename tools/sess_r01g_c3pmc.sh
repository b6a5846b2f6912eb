#!/bin/bash
# C3 (512^3 3-D) kernel stats + HBM traffic passes (FETCH_SIZE, WRITE_SIZE in separate runs)
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && tools/gpu_session.sh \
  "200|c3kt|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c3kt -o kt -- python3 tools/prof_cases.py c3" \
  "120|c3f|timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/c3f -o pmc -- python3 tools/prof_cases.py c3 --reps 3" \
  "120|c3w|timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/c3w -o pmc -- python3 tools/prof_cases.py c3 --reps 3"
