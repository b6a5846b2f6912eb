export GPU_SESSION_STRICT=1
tools/gpu_session.sh "300|r05_sharded_tests|python -u -m pytest tests/test_gpu_exchange.py -m gpu -x -q --timeout 120 --timeout-method thread -k 'sharded or world1 or multi_legs or multiprocess'" \
 "400|r05_pytest_gpu_d|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "900|r05_measure|bash tools/measure_round.sh r05"
