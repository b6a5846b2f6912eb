export GPU_SESSION_STRICT=1
tools/gpu_session.sh "150|a4|python tools/dmean_stride_time.py --stride 16" \
 "150|a3|python tools/dmean_stride_time.py --stride 16 --lib abv/libgcow_w3.so" \
 "150|a3lp|python tools/dmean_stride_time.py --stride 16 --lib abv/libgcow_w3lp.so" \
 "150|b4|python tools/dmean_stride_time.py --stride 16" \
 "150|b3|python tools/dmean_stride_time.py --stride 16 --lib abv/libgcow_w3.so" \
 "150|b3lp|python tools/dmean_stride_time.py --stride 16 --lib abv/libgcow_w3lp.so"
