#!/bin/bash
# why does the one-shot encoder time differently in bench.py and in the ablation tool: kernel traces of both
B="python3 bench.py --no-cpu-baseline --no-host-e2e"
cd "$(dirname "$0")/.." && tools/gpu_session.sh \
  "300|kt_bench|rocprofv3 --kernel-trace --stats -d gpurun_out/kt_bench -o kt --output-format csv -- $B --steps 40" \
  "300|kt_abl|rocprofv3 --kernel-trace --stats -d gpurun_out/kt_abl -o kt --output-format csv -- python3 tools/ubench/ablate.py 61:8,56:12 12" \
  "120|b8_100|python bench.py --no-cpu-baseline --no-host-e2e --steps 200 --warmup 20"
