#!/bin/bash
# lean-5 launch-shape ablation: grid-stride pipe vs non-persistent vs contiguous-chunk persistent
cd "$(dirname "$0")/.." && tools/gpu_session.sh \
  "300|ablate|python tools/ubench/ablate.py 49:12,49:8,56:12,59:8,60:8,61:8,62:8,62:12,63:8,9:8 12"
