#!/bin/bash
cd "$(dirname "$0")/.." && tools/gpu_session.sh \
  "600|pytest_fast|python -m pytest tests/test_gpu_parity.py -m gpu -q -x -k 'fast1d or c2 or rate or bf16 or tiny or drop'" \
  "200|ablate9|python tools/ubench/ablate.py 12:32,46:12,51:8,51:12,51:16,52:12,53:12,50:12,8:8 8" \
  "300|bench|python bench.py --no-cpu-baseline"
