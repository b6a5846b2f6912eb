#!/bin/bash
cd "$(dirname "$0")/.." && tools/gpu_session.sh \
  "900|pytest_gpu|python -m pytest tests -m gpu -q -x -p no:cacheprovider" \
  "300|configs|python tools/bench_configs.py c3 c2_decode"
