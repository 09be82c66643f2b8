cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 450 env KCEP_FUZZ_SEEDS=150:280 python -u -m pytest tests/test_fuzz_gpu.py -v --timeout 120 --timeout-method thread -m gpu -k "test_random_rich_parity" --durations=3 > gpurun_out/fuzz12.log 2>&1
