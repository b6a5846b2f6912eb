export GPU_SESSION_STRICT=1
K="-k 'fixed1d or c2 or decode or hook or fast1d or var1d or c5_full or host_encoder'"
T="python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_exchange.py -m gpu -x -q --timeout 120 --timeout-method thread $K"
tools/gpu_session.sh "300|t_prod|$T" \
 "150|a_new|python tools/dec_lib_time.py" \
 "150|a_old|python tools/dec_lib_time.py --lib abv/libgcow_prev.so" \
 "150|b_new|python tools/dec_lib_time.py" \
 "150|b_old|python tools/dec_lib_time.py --lib abv/libgcow_prev.so"
