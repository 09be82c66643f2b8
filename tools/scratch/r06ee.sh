cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out/ee
for i in 1 2; do
for v in base sub2 sub3; do
  if [ $v = base ]; then L=""; else L="KCEP_LIB=build_variants/$v/libkcep.so"; fi
  env $L timeout -k 10 200 python -u bench.py --config c2 --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/ee/${v}_$i.log 2>&1 || exit 1
  echo "$v $i done"
done; done
