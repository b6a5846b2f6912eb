export GPU_SESSION_STRICT=1
tools/gpu_session.sh "300|t_arb|python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k 'arbitrary'"
