mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -8 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" || exit 1
for c in cfg2 cfg3 cfg5; do timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_$c.log 2>&1 || exit 1; tail -1 gpurun_out/bench_$c.log | cut -c1-400; done
LIBS="pymhealth_amd/libmhfeat.so pymhealth_amd/libmhfeat_r2.so" CONFIGS="cfg2 cfg3" REPS=2 bash tools/ab_bench.sh
for w in 65536 262144; do timeout -k 10 120 python bench.py --config cfg3 --windows $w --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/b.log 2>&1 || exit 1; python -c "import json; d=json.loads(open('gpurun_out/b.log').read().strip().split('\n')[-1]); print('cfg3 nw=$w', d['roofline']['kernel_ms'], 'ms', d['roofline']['kernel_ms']*1e7/$w, 'ms-per-1e7')"; done
