export GPU_SESSION_STRICT=1
tools/gpu_session.sh "420|bench|python -u bench.py"
