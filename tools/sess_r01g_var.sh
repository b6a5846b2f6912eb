#!/bin/bash
cd "$(dirname "$0")/.." && tools/gpu_session.sh \
  "400|pytest_gpu|python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread" \
  "300|cfg|python tools/bench_configs.py c3 c5"
