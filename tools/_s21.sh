export GPU_SESSION_STRICT=1
tools/gpu_session.sh "150|a4|python tools/dmean_stride_time.py --stride 8" \
 "150|a5|python tools/dmean_stride_time.py --stride 8 --lib abv/libgcow_w5.so" \
 "150|a6|python tools/dmean_stride_time.py --stride 8 --lib abv/libgcow_w6.so" \
 "150|b4|python tools/dmean_stride_time.py --stride 8" \
 "150|b5|python tools/dmean_stride_time.py --stride 8 --lib abv/libgcow_w5.so" \
 "150|b6|python tools/dmean_stride_time.py --stride 8 --lib abv/libgcow_w6.so"
