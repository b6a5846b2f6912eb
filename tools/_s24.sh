export GPU_SESSION_STRICT=1
tools/gpu_session.sh "150|a0|python tools/c5_lib_time.py" \
 "150|a1|python tools/c5_lib_time.py --lib abv/libgcow_vlp1.so" \
 "150|a2|python tools/c5_lib_time.py --lib abv/libgcow_vlp1c48.so" \
 "150|b0|python tools/c5_lib_time.py" \
 "150|b1|python tools/c5_lib_time.py --lib abv/libgcow_vlp1.so" \
 "150|b2|python tools/c5_lib_time.py --lib abv/libgcow_vlp1c48.so"
