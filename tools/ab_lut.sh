set -o pipefail
cd $GRAFT_REPO_ROOT
for c in c2 c5; do
for i in 1 2 3; do
  KCEP_LIB=build_variants/libkcep_nolut.so timeout -k 10 200 python -u bench.py --config $c --steps 30 --warmup 5 --no-cpu-baseline --no-host-input --carry-batches 1 > gpurun_out/lut_old_${c}_$i.log 2>&1 || exit 1
  timeout -k 10 200 python -u bench.py --config $c --steps 30 --warmup 5 --no-cpu-baseline --no-host-input --carry-batches 1 > gpurun_out/lut_new_${c}_$i.log 2>&1 || exit 1
done
done
echo done
