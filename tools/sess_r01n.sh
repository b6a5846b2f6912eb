#!/bin/bash
cd "$(dirname "$0")/.." && tools/gpu_session.sh \
  "600|pytest_dec|python -m pytest tests/test_gpu_parity.py tests/test_header_product.py -m gpu -q -x -k 'fast1d or c2 or rate or fixture or golden or header or zfpy or drop or ddp'" \
  "300|configs|python tools/bench_configs.py c2_decode"
