B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-e2e"
T="python -m pytest tests -m gpu -q -x -p no:cacheprovider -k 'fast1d or c2 or fixture or golden or subnormal or bf16 or tiny'"
tools/gpu_session.sh \
 "600|t_v6|GCOW_FIXED1D_VARIANT=6 $T" \
 "200|b_v6_w8|GCOW_FIXED1D_VARIANT=6 GCOW_FIXED1D_WGS=8 $B" \
 "200|b_v6_w16|GCOW_FIXED1D_VARIANT=6 GCOW_FIXED1D_WGS=16 $B" \
 "200|b_v6_w4|GCOW_FIXED1D_VARIANT=6 GCOW_FIXED1D_WGS=4 $B" \
 "300|abl|python tools/ubench/ablate.py 0,4,5,6,7,8,9 8"
