cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for o in interp_lane interp_wave jit_wave jit_lane; do
  timeout -k 5 45 python -u tools/dbg_fuzz.py 206 0:1 $o >> gpurun_out/gg.log 2>&1
  rc=$?; echo "$o rc=$rc" >> gpurun_out/gg.log
  if [ $rc -ne 0 ]; then exit 0; fi
done
