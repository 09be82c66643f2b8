cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 720 env KCEP_FUZZ_SEEDS=300:520 python -u -m pytest tests/test_fuzz_gpu.py -v --timeout 120 --timeout-method thread -m gpu -k "test_random_pattern_parity and mixed" --durations=5 > gpurun_out/fuzz11.log 2>&1
