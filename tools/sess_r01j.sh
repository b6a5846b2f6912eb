#!/bin/bash
# DDP hooks + reference gtest suites through libgcow.so
cd "$(dirname "$0")/.." && tools/gpu_session.sh \
  "900|pytest_new|python -m pytest tests/test_reference_suites.py tests/test_gpu_parity.py -k 'reference or ddp' -m gpu -q -rs"
