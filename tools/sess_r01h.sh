B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-e2e"
T="python -m pytest tests -m gpu -q -x -p no:cacheprovider -k 'fast1d or c2 or fixture or golden or subnormal or bf16 or tiny'"
tools/gpu_session.sh \
 "600|t_v8|GCOW_FIXED1D_VARIANT=8 $T" \
 "200|b_v8_16|GCOW_FIXED1D_VARIANT=8 GCOW_FIXED1D_WGS=16 $B" \
 "200|b_v8_8|GCOW_FIXED1D_VARIANT=8 GCOW_FIXED1D_WGS=8 $B" \
 "200|b_v8_32|GCOW_FIXED1D_VARIANT=8 GCOW_FIXED1D_WGS=32 $B" \
 "200|b_v3_16|GCOW_FIXED1D_VARIANT=3 GCOW_FIXED1D_WGS=16 $B"
