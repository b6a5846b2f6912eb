#!/bin/bash
# bench kernel: kernel trace + stats, then separate FETCH_SIZE and WRITE_SIZE passes (never combined with tracing);
# C5 kernel split (count / scan / encode)
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
B="python3 bench.py --steps 200 --warmup 100 --no-cpu-baseline --no-host-e2e"
tools/gpu_session.sh \
 "300|prof_kt|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kt -o kt --output-format csv -- $B" \
 "300|prof_fetch|timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_fetch -o pmc --output-format csv -- $B" \
 "300|prof_write|timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_write -o pmc --output-format csv -- $B" \
 "120|summ|python3 tools/pmc_traffic.py k_encode_fixed1d_np c2_1d_fp32_fixed_rate16_256Mi_per_gpu gpurun_out/prof_kt gpurun_out/prof_fetch gpurun_out/prof_write gpurun_out/r01g 200" \
 "200|c5kt|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5kt -o kt -- python3 tools/prof_cases.py c5"
