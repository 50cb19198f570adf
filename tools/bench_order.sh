set -u
mkdir -p gpurun_out
for f in median "median,interquartile_range,mode" "sampen" "mean,var,skewness,kurtosis,zero_crossings,median"; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 --config cfg2 --features "$f" --no-cpu-baseline > gpurun_out/bench_feat.log 2>&1 || exit $?
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench_feat.log').read().strip().splitlines()[-1]); print('$f', d['ms_per_step'], d['config']['kernel'], d['roofline']['kernel_ms'])"
done
