#!/bin/bash
# 3-D fixed rate: per-lane word writer + LDS-staged decoder; GPU suite, C3 A/B against the generic tile path
cd "$(dirname "$0")/.." && tools/gpu_session.sh \
  "600|pytest_gpu|python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread" \
  "300|c3|python tools/bench_configs.py c3" \
  "300|c3_generic|GCOW_GENERIC_3D=1 python tools/bench_configs.py c3" \
  "300|kt_c3|rocprofv3 --kernel-trace --stats -d gpurun_out/kt_c3 -o kt --output-format csv -- python3 tools/bench_configs.py c3"
