export GPU_SESSION_STRICT=1
K="-k 'fixed1d or c2 or rate8 or fast1d or encode_fixed'"
T="python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread $K"
tools/gpu_session.sh "300|t_lazy|$T" \
 "120|a_lazy|python tools/c2_lib_time.py --rate 8" \
 "120|a_nolazy|python tools/c2_lib_time.py --rate 8 --lib abv/libgcow_nolazy.so" \
 "120|b_lazy|python tools/c2_lib_time.py --rate 8" \
 "120|b_nolazy|python tools/c2_lib_time.py --rate 8 --lib abv/libgcow_nolazy.so" \
 "120|c_lazy|python tools/c2_lib_time.py --rate 8" \
 "120|c_nolazy|python tools/c2_lib_time.py --rate 8 --lib abv/libgcow_nolazy.so" \
 "120|d_lazy|python tools/c2_lib_time.py --rate 8" \
 "120|d_nolazy|python tools/c2_lib_time.py --rate 8 --lib abv/libgcow_nolazy.so"
