cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_prof.sh r06 "c2 c3 c5 c4" || exit 1
timeout -k 10 300 python3 -u tools/flush_probe.py 65536 200 > gpurun_out/flush_probe_r06final.log 2>&1; grep "us/batch" gpurun_out/flush_probe_r06final.log
echo done
