export GPU_SESSION_STRICT=1
K="-k 'var1d or c5_full or host_encoder or decode_mean_vs'"
T="python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_exchange.py -m gpu -x -q --timeout 120 --timeout-method thread $K"
tools/gpu_session.sh "300|t_prod|$T" \
 "120|a_ol2|python tools/c5_lib_time.py" \
 "120|a_ol1|python tools/c5_lib_time.py --lib abv/libgcow_ol1.so" \
 "120|a_ol0|python tools/c5_lib_time.py --lib abv/libgcow_ol0.so" \
 "120|b_ol2|python tools/c5_lib_time.py" \
 "120|b_ol1|python tools/c5_lib_time.py --lib abv/libgcow_ol1.so" \
 "120|b_ol0|python tools/c5_lib_time.py --lib abv/libgcow_ol0.so" \
 "120|c_ol2|python tools/c5_lib_time.py" \
 "120|c_ol1|python tools/c5_lib_time.py --lib abv/libgcow_ol1.so" \
 "120|c_ol0|python tools/c5_lib_time.py --lib abv/libgcow_ol0.so"
