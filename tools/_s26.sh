export GPU_SESSION_STRICT=1
tools/gpu_session.sh "500|gp|python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_exchange.py -m gpu -x -q --timeout 120 --timeout-method thread" \
 "150|a32|python tools/c5_lib_time.py" \
 "150|a0|python tools/c5_lib_time.py --lib abv/libgcow_s0.so" \
 "150|a24|python tools/c5_lib_time.py --lib abv/libgcow_s24.so" \
 "150|a40|python tools/c5_lib_time.py --lib abv/libgcow_s40.so" \
 "150|b32|python tools/c5_lib_time.py" \
 "150|b0|python tools/c5_lib_time.py --lib abv/libgcow_s0.so" \
 "150|b24|python tools/c5_lib_time.py --lib abv/libgcow_s24.so" \
 "150|b40|python tools/c5_lib_time.py --lib abv/libgcow_s40.so"
