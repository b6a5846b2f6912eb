export GPU_SESSION_STRICT=1
K="-k '3d or c3 or fixed3d or libzfp or staged or tiles'"
T="python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread $K"
tools/gpu_session.sh "300|t_prod|$T" \
 "120|a_new|python tools/c3_time.py" \
 "120|a_old|python tools/c3_time.py --lib abv/libgcow_prev.so" \
 "120|b_new|python tools/c3_time.py" \
 "120|b_old|python tools/c3_time.py --lib abv/libgcow_prev.so" \
 "120|c_new|python tools/c3_time.py" \
 "120|c_old|python tools/c3_time.py --lib abv/libgcow_prev.so"
