tools/gpu_session.sh \
 "600|pytest_gpu|python -m pytest tests -m gpu -q -x -p no:cacheprovider" \
 "600|configs|python tools/bench_configs.py c2_decode var_f32 c5 c3" \
 "400|bench_full|python bench.py"
