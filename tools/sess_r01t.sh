#!/bin/bash
# lean-5 1-D coder: full GPU suite (default coder = lean-5), A/B ablation vs lean-4, bench
cd "$(dirname "$0")/.." && tools/gpu_session.sh \
  "600|pytest_gpu|python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread" \
  "300|ablate|python tools/ubench/ablate.py 54:12,55:12,51:12,56:12,57:12,58:12,56:8,56:16,8:8,9:8 12" \
  "300|bench|python bench.py --no-host-e2e" \
  "300|bench_l4|GCOW_FIXED1D_VARIANT=4 python bench.py --no-cpu-baseline --no-host-e2e"
