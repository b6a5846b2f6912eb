export GPU_SESSION_STRICT=1
K="-k 'fixed1d or c2 or rate8 or fast1d or encode_fixed or host_encoder or lean'"
T="python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread $K"
tools/gpu_session.sh "300|t_p1|$T" \
 "120|a_new|python tools/c2_lib_time.py" \
 "120|a_old|python tools/c2_lib_time.py --lib abv/libgcow_p1vote.so" \
 "120|b_new|python tools/c2_lib_time.py" \
 "120|b_old|python tools/c2_lib_time.py --lib abv/libgcow_p1vote.so" \
 "120|c_new|python tools/c2_lib_time.py" \
 "120|c_old|python tools/c2_lib_time.py --lib abv/libgcow_p1vote.so" \
 "120|d_new|python tools/c2_lib_time.py" \
 "120|d_old|python tools/c2_lib_time.py --lib abv/libgcow_p1vote.so" \
 "120|e_new8|python tools/c2_lib_time.py --rate 8" \
 "120|e_old8|python tools/c2_lib_time.py --rate 8 --lib abv/libgcow_p1vote.so" \
 "120|f_new8|python tools/c2_lib_time.py --rate 8" \
 "120|f_old8|python tools/c2_lib_time.py --rate 8 --lib abv/libgcow_p1vote.so"
