export GPU_SESSION_STRICT=1
tools/gpu_session.sh "400|dpp_tests|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "200|c5_dpp|python tools/c5_lib_time.py" \
 "200|c5_nodpp|python tools/c5_lib_time.py --lib abv/libgcow_nodpp.so" \
 "200|c5_dpp_b|python tools/c5_lib_time.py" \
 "200|c5_nodpp_b|python tools/c5_lib_time.py --lib abv/libgcow_nodpp.so" \
 "200|c3_dpp|python tools/c3_time.py" \
 "200|c3_nodpp|python tools/c3_time.py --lib abv/libgcow_nodpp.so" \
 "200|c3_dpp_b|python tools/c3_time.py" \
 "200|c3_nodpp_b|python tools/c3_time.py --lib abv/libgcow_nodpp.so"
