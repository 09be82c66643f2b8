cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 10 --warmup 2 > gpurun_out/torchrun_1.log 2>&1 || { tail -20 gpurun_out/torchrun_1.log; exit 1; }
tail -1 gpurun_out/torchrun_1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["n_gpus"], d["value"], d["ms_per_step"], d["config"].get("parallelism"), d["checksum"])'
timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 1 > gpurun_out/launch_2.log 2>&1; echo "launcher --gpus 2 on a 1-GPU box: exit $?"; tail -3 gpurun_out/launch_2.log
echo done
