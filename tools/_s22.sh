export GPU_SESSION_STRICT=1
tools/gpu_session.sh "400|gx|python -u -m pytest tests/test_gpu_exchange.py -m gpu -x -v --timeout 120 --timeout-method thread" \
 "150|a16|python tools/dmean_stride_time.py --stride 16" \
 "150|a8|python tools/dmean_stride_time.py --stride 8" \
 "150|b16|python tools/dmean_stride_time.py --stride 16" \
 "150|b8|python tools/dmean_stride_time.py --stride 8" \
 "500|bench|python bench.py"
