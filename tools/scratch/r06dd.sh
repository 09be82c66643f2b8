cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof/r06dd_c2carry -o t -- python3 bench.py --config c2 --steps 2 --warmup 1 --no-cpu-baseline --no-host-input --processor-batch , --handoff-cap 0 > gpurun_out/r06dd.log 2>&1 && tail -1 gpurun_out/r06dd.log | cut -c1-300
echo done
