export GPU_SESSION_STRICT=1
tools/gpu_session.sh "300|gx|python -u -m pytest tests/test_gpu_exchange.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k 'decode_mean or sharded'" \
 "150|a1|python tools/dmean_stride_time.py --stride 8" \
 "150|a0|python tools/dmean_stride_time.py --stride 8 --lib abv/libgcow_sc0.so" \
 "150|b1|python tools/dmean_stride_time.py --stride 8" \
 "150|b0|python tools/dmean_stride_time.py --stride 8 --lib abv/libgcow_sc0.so"
