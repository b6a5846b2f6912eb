#!/bin/bash
# profiles for the one-shot encoder: kernel stats, PMC HBM traffic (separate passes), then the full bench line
B="python3 bench.py --no-cpu-baseline --no-host-e2e"
cd "$(dirname "$0")/.." && tools/gpu_session.sh \
 "300|prof_kt|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kt -o kt --output-format csv -- $B" \
 "300|prof_fetch|rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_fetch -o pmc --output-format csv -- $B" \
 "300|prof_write|rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_write -o pmc --output-format csv -- $B" \
 "120|summ|python3 tools/pmc_traffic.py k_encode_fixed1d_np c2_1d_fp32_fixed_rate16_256Mi_per_gpu gpurun_out/prof_kt gpurun_out/prof_fetch gpurun_out/prof_write gpurun_out/r01d" \
 "400|bench_full|python bench.py"
