#!/bin/bash
# single-pass variable-rate 1-D encoder: GPU suite, C5 / var_f32 timings (single pass vs two-pass), kernel trace
cd "$(dirname "$0")/.." && tools/gpu_session.sh \
  "600|pytest_gpu|python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread" \
  "300|cfg_sp|python tools/bench_configs.py c5 var_f32" \
  "300|cfg_2p|GCOW_VAR1D_MODE=2pass python tools/bench_configs.py c5 var_f32" \
  "300|cfg_lb|GCOW_VAR1D_MODE=lookback python tools/bench_configs.py c5"
