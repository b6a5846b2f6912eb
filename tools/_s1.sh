export GPU_SESSION_STRICT=1
tools/gpu_session.sh "200|r05_dm_tests|python -u -m pytest tests/test_gpu_exchange.py -m gpu -x -q --timeout 120 --timeout-method thread -k decode_mean" \
 "200|c2v_tests|for v in c2v7 c2u4 c2v7u4; do GCOW_TEST_LIB=abv/libgcow_\$v.so python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k 'c2_full or fast1d or fixed1d or smoke or golden' || exit 1; done" \
 "120|dm_new|python tools/bench_configs.py decode_mean" \
 "120|dm_old|python tools/bench_configs.py decode_mean --lib abv/libgcow_dm_old.so" \
 "120|dm_noskew|python tools/bench_configs.py decode_mean --lib abv/libgcow_dm_noskew.so" \
 "120|dm_new2|python tools/bench_configs.py decode_mean" \
 "300|c2ab|for r in 1 2 3; do for v in '' c2v7 c2u4 c2v7u4; do if [ -z \"\$v\" ]; then python tools/c2_lib_time.py; else python tools/c2_lib_time.py --lib abv/libgcow_\$v.so; fi || exit 1; done; done"
