#!/bin/bash
# one-shot lean-5 encoder (U blocks per lane): GPU suite under the new default, bench A/B over U and the old pipe
B="python bench.py --no-cpu-baseline --no-host-e2e"
cd "$(dirname "$0")/.." && tools/gpu_session.sh \
  "600|pytest_gpu|python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread" \
  "120|b8|GCOW_FIXED1D_VARIANT=8 $B" \
  "120|b12|GCOW_FIXED1D_VARIANT=12 $B" \
  "120|b16|GCOW_FIXED1D_VARIANT=16 $B" \
  "120|b5|GCOW_FIXED1D_VARIANT=5 $B" \
  "120|b8r8|GCOW_FIXED1D_VARIANT=8 $B --rate 8" \
  "120|b5r8|GCOW_FIXED1D_VARIANT=5 $B --rate 8" \
  "120|b8_again|GCOW_FIXED1D_VARIANT=8 $B" \
  "300|pytest_u16|GCOW_FIXED1D_VARIANT=16 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k 'fast1d or c2_full or bf16 or empty or other_rates'"
