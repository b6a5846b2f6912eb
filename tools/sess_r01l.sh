#!/bin/bash
cd "$(dirname "$0")/.." && tools/gpu_session.sh \
  "300|hdr_gpu|python -m pytest tests/test_header_product.py -m gpu -q -x" \
  "200|ablate4|python tools/ubench/ablate.py 12,24,25,26,27 32 && python tools/ubench/ablate.py 12,24,25,26,27 8 && python tools/ubench/ablate.py 12,25,26,27 16"
