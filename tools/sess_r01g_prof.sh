#!/bin/bash
# C3/C5 kernel stats + SQ instruction/cycle counters (one PMC pass, no tracing combined)
cd "$(dirname "$0")/.." && R=$PWD && cd /tmp && export TMPDIR=/tmp && cd $R && tools/gpu_session.sh \
  "200|cfg|python tools/bench_configs.py c3 c5" \
  "200|pkt|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pkt -o kt -- python3 tools/prof_cases.py" \
  "120|psq|timeout -s KILL 100 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/psq -o pmc -- python3 tools/prof_cases.py --reps 2"
