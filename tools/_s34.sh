export GPU_SESSION_STRICT=1
tools/gpu_session.sh "300|gx|python -u -m pytest tests/test_gpu_exchange.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k 'decode_mean or sharded or hook'" \
 "150|c16|python tools/dmean_stride_time.py --stride 16" \
 "150|c8|python tools/dmean_stride_time.py --stride 8"
