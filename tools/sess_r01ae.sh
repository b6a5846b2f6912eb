#!/bin/bash
# table-driven variable-rate 1-D decoder: GPU suite, decode timings vs the generic bit-serial decoder
cd "$(dirname "$0")/.." && tools/gpu_session.sh \
  "600|pytest_gpu|python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread" \
  "300|vdec|python tools/bench_configs.py var_decode" \
  "300|vdec_generic|GCOW_GENERIC_DECODE=1 python tools/bench_configs.py var_decode"
