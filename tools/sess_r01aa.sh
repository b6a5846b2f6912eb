#!/bin/bash
# append API + overlapped host path: GPU suite, C5 configs (sequential vs overlapped host path), bench host_e2e
cd "$(dirname "$0")/.." && tools/gpu_session.sh \
  "600|pytest_gpu|python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread" \
  "300|c5|python tools/bench_configs.py c5" \
  "300|bench|python bench.py --no-cpu-baseline"
