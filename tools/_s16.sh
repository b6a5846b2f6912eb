export GPU_SESSION_STRICT=1
tools/gpu_session.sh "420|r05_pytest_gpu_e|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "900|r05_measure_b|bash tools/measure_round.sh r05b"
