#!/bin/bash
cd "$(dirname "$0")/.." && tools/gpu_session.sh \
  "900|pytest_var|python -m pytest tests/test_gpu_parity.py tests/test_header_product.py -m gpu -q -x -k 'var1d or c5 or random or fixture or golden or bf16 or stitch or acc or prec or ddp or zfpy or drop'" \
  "300|configs|python tools/bench_configs.py var_f32 c5"
