#!/bin/bash
# single-pass variable-rate 1-D encoder: GPU suite, C5 / var_f32 timings (single pass vs two-pass), kernel trace
cd "$(dirname "$0")/.." && tools/gpu_session.sh \
  "600|pytest_gpu|python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread" \
  "300|cfg_sp|python tools/bench_configs.py c5 var_f32" \
  "300|cfg_2p|GCOW_VAR1D_2PASS=1 python tools/bench_configs.py c5 var_f32" \
  "300|kt_c5|rocprofv3 --kernel-trace --stats -d gpurun_out/kt_c5 -o kt --output-format csv -- python3 tools/bench_configs.py c5"
