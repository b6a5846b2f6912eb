#!/bin/bash
cd "$(dirname "$0")/.." && tools/gpu_session.sh \
  "900|pytest_3d|python -m pytest tests/test_gpu_parity.py tests/test_reference_suites.py -m gpu -q -x -p no:cacheprovider -k '3d or c3 or random or fixture or stage or block or 16x or reference'" \
  "300|configs|python tools/bench_configs.py c3"
