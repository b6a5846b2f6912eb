#!/bin/bash
cd "$(dirname "$0")/.." && tools/gpu_session.sh \
  "300|pytest_dec|python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k 'var1d or decode or c5 or ddp or append or host or libzfp'" \
  "300|vdec|python tools/bench_configs.py var_decode" \
  "300|vdec128|GCOW_VDEC=staged128 python tools/bench_configs.py var_decode" \
  "300|vdec_glob|GCOW_VDEC=global python tools/bench_configs.py var_decode"
