export GPU_SESSION_STRICT=1
K="-k 'var1d or c5_full or host_encoder or decode_mean_vs'"
T="python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_exchange.py -m gpu -x -q --timeout 120 --timeout-method thread $K"
tools/gpu_session.sh "300|t_prod|$T" \
 "300|t_pf2|GCOW_TEST_LIB=abv/libgcow_pf2.so $T" \
 "300|t_pf3|GCOW_TEST_LIB=abv/libgcow_pf3.so $T" \
 "300|t_zall|GCOW_TEST_LIB=abv/libgcow_zall.so $T" \
 "120|a_prod|python tools/c5_lib_time.py" \
 "120|a_pf2|python tools/c5_lib_time.py --lib abv/libgcow_pf2.so" \
 "120|a_pf3|python tools/c5_lib_time.py --lib abv/libgcow_pf3.so" \
 "120|a_zall|python tools/c5_lib_time.py --lib abv/libgcow_zall.so" \
 "120|b_prod|python tools/c5_lib_time.py" \
 "120|b_pf2|python tools/c5_lib_time.py --lib abv/libgcow_pf2.so" \
 "120|b_pf3|python tools/c5_lib_time.py --lib abv/libgcow_pf3.so" \
 "120|b_zall|python tools/c5_lib_time.py --lib abv/libgcow_zall.so" \
 "120|c_prod|python tools/c5_lib_time.py" \
 "120|c_pf2|python tools/c5_lib_time.py --lib abv/libgcow_pf2.so" \
 "120|c_pf3|python tools/c5_lib_time.py --lib abv/libgcow_pf3.so" \
 "120|c_zall|python tools/c5_lib_time.py --lib abv/libgcow_zall.so"
