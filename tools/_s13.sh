export GPU_SESSION_STRICT=1
K="-k 'var1d or c5_full or host_encoder or decode_mean or hook or decode'"
T="python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_exchange.py -m gpu -x -q --timeout 120 --timeout-method thread $K"
tools/gpu_session.sh "300|t_prod|$T" \
 "120|a_new|python tools/c5_lib_time.py" \
 "120|a_old|python tools/c5_lib_time.py --lib abv/libgcow_prev.so" \
 "120|b_new|python tools/c5_lib_time.py" \
 "120|b_old|python tools/c5_lib_time.py --lib abv/libgcow_prev.so" \
 "120|c_new|python tools/c5_lib_time.py" \
 "120|c_old|python tools/c5_lib_time.py --lib abv/libgcow_prev.so"
