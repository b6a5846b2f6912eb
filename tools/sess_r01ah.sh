#!/bin/bash
# 3-D variable rate: private-word writer in the encode tiles, LDS-staged generic decoder; GPU suite, C3 timings
cd "$(dirname "$0")/.." && tools/gpu_session.sh \
  "600|pytest_gpu|python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread" \
  "300|c3|python tools/bench_configs.py c3" \
  "300|c3_glob|GCOW_DECODE_GLOBAL=1 python tools/bench_configs.py c3"
