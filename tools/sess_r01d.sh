B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-e2e"
tools/gpu_session.sh \
 "600|pytest_gpu|python -m pytest tests -m gpu -q -x -p no:cacheprovider -k 'fast1d or c2 or fixture or golden or subnormal or bf16 or tiny'" \
 "200|b_v2|GCOW_FIXED1D_VARIANT=2 $B" \
 "200|b_v3_w8|GCOW_FIXED1D_VARIANT=3 $B" \
 "200|b_v3_w4|GCOW_FIXED1D_VARIANT=3 GCOW_FIXED1D_WGS=4 $B" \
 "200|b_v3_w16|GCOW_FIXED1D_VARIANT=3 GCOW_FIXED1D_WGS=16 $B" \
 "200|b_v3_w64|GCOW_FIXED1D_VARIANT=3 GCOW_FIXED1D_WGS=64 $B" \
 "300|prof_sq3|rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY -d gpurun_out/prof_sq3 -o pmc --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-e2e"
