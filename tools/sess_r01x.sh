#!/bin/bash
# one-shot encoder + decoder: GPU suite, steady-state bench A/B (encoder U, persistent), decoder A/B
B="python bench.py --no-cpu-baseline --no-host-e2e"
cd "$(dirname "$0")/.." && tools/gpu_session.sh \
  "600|pytest_gpu|python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread" \
  "120|b8|GCOW_FIXED1D_VARIANT=8 $B" \
  "120|b12|GCOW_FIXED1D_VARIANT=12 $B" \
  "120|b16|GCOW_FIXED1D_VARIANT=16 $B" \
  "120|b5|GCOW_FIXED1D_VARIANT=5 $B" \
  "120|b8b|GCOW_FIXED1D_VARIANT=8 $B" \
  "120|dec0|GCOW_DECODE1D_VARIANT=0 python tools/bench_configs.py c2_decode" \
  "120|dec8|GCOW_DECODE1D_VARIANT=8 python tools/bench_configs.py c2_decode" \
  "120|dec16|GCOW_DECODE1D_VARIANT=16 python tools/bench_configs.py c2_decode" \
  "300|pytest_dec8|GCOW_DECODE1D_VARIANT=8 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k 'fast1d or c2_full or decode or other_rates'"
