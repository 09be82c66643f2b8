cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 1080 env KCEP_FUZZ_SEEDS=0:110 python -u -m pytest tests/test_fuzz_gpu.py -v --timeout 120 --timeout-method thread -m gpu -k "rich_carry" --durations=5 > gpurun_out/fuzz10.log 2>&1
