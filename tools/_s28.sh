export GPU_SESSION_STRICT=1
tools/gpu_session.sh "500|gp|python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k 'var or acc or c5 or decode or exact'" \
 "150|a1|python tools/c5_lib_time.py" \
 "150|a0|python tools/c5_lib_time.py --lib abv/libgcow_na.so" \
 "150|ac|python tools/c5_lib_time.py --capacity" \
 "150|b1|python tools/c5_lib_time.py" \
 "150|b0|python tools/c5_lib_time.py --lib abv/libgcow_na.so" \
 "150|bc|python tools/c5_lib_time.py --capacity"
