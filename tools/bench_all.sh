set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for c in cfg3 cfg5 cfg4; do
  timeout -k 10 400 python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_$c.log 2>&1
  rc=$?; tail -n 2 gpurun_out/bench_$c.log; echo "== $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
