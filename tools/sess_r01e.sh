B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-e2e"
T="python -m pytest tests -m gpu -q -x -p no:cacheprovider -k 'fast1d or c2 or fixture or golden or subnormal or bf16 or tiny'"
tools/gpu_session.sh \
 "600|t_v4|GCOW_FIXED1D_VARIANT=4 $T" \
 "600|t_v5|GCOW_FIXED1D_VARIANT=5 $T" \
 "200|b_v3_w16|GCOW_FIXED1D_VARIANT=3 GCOW_FIXED1D_WGS=16 $B" \
 "200|b_v4_w4|GCOW_FIXED1D_VARIANT=4 GCOW_FIXED1D_WGS=4 $B" \
 "200|b_v4_w8|GCOW_FIXED1D_VARIANT=4 GCOW_FIXED1D_WGS=8 $B" \
 "200|b_v4_w16|GCOW_FIXED1D_VARIANT=4 GCOW_FIXED1D_WGS=16 $B" \
 "200|b_v5_w2|GCOW_FIXED1D_VARIANT=5 GCOW_FIXED1D_WGS=2 $B" \
 "200|b_v5_w4|GCOW_FIXED1D_VARIANT=5 GCOW_FIXED1D_WGS=4 $B" \
 "200|b_v5_w8|GCOW_FIXED1D_VARIANT=5 GCOW_FIXED1D_WGS=8 $B"
