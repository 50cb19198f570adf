#!/bin/bash
# Round-6 GPU sessions: each step "name timeout env cmd..." runs under its own time limit;
# the session stops at the first failure (SOFT=1: a plain test / probe failure, exit 1, does
# not end it; a fault, abort, crash or time limit always does). No retries.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
SOFT=0
run() {  # run <name> <timeout> <env assignments or -> <cmd...>
  local name=$1 t=$2 envs=$3; shift 3
  echo "=== $name"
  if [ "$envs" = "-" ]; then timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  else env $envs timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; fi
  local rc=$?
  tail -n 2 "gpurun_out/$name.log" | cut -c1-1500
  echo "=== $name rc=$rc"
  if [ $rc -ne 0 ] && ! { [ $SOFT = 1 ] && [ $rc = 1 ]; }; then exit $rc; fi
}
# profile <tag> <summary args> -- <bench args>: tools/profile.sh passes, then the summary on
# the box (the raw traces exceed gpurun's 64 MiB pull): profiles/<tag>_* and traffic.json
# copied to gpurun_out/summ/, the raw directory removed
profile() {
  local tag=$1; shift
  local sargs=()
  while [ "$1" != "--" ]; do sargs+=("$1"); shift; done; shift
  local envs="-"
  [ -n "${KRE:-}" ] && envs="KRE=$KRE"
  run prof_$tag 600 "$envs" bash tools/profile.sh $tag "$@"
  python tools/prof_summary.py $tag "${sargs[@]}" > gpurun_out/summ_$tag.log 2>&1 || true
  mkdir -p gpurun_out/summ && cp profiles/${tag}_* profiles/traffic.json gpurun_out/summ/ 2>/dev/null
  rm -rf gpurun_out/prof_$tag
}
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu"
PYTNX="python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu"
B="python bench.py --no-cpu-baseline"
# quick profile: kernel trace + the two SQ passes, summarised on the box
qprof() {  # qprof <tag> <kernel regex> <summary args> -- <bench args>
  local tag=$1 kre=$2; shift 2
  local sargs=()
  while [ "$1" != "--" ]; do sargs+=("$1"); shift; done; shift
  QUICK=1 run prof_q_$tag 400 "KRE=$kre" bash tools/profile.sh $tag "$@"
  python tools/prof_summary.py $tag "${sargs[@]}" > gpurun_out/summ_$tag.log 2>&1 || true
  mkdir -p gpurun_out/summ && cp profiles/${tag}_* gpurun_out/summ/ 2>/dev/null; rm -rf gpurun_out/prof_$tag
}
case "${1:-}" in
  a)
    # fast var default + exact opt-in: the whole GPU suite, the BASELINE benches, cfg3 profile
    SOFT=1
    run tests_gpu 900 - $PYTNX tests
    SOFT=0
    run bench_cfg2 200 - $B --config cfg2 --steps 20 --warmup 3
    run bench_cfg3 200 - $B --config cfg3 --steps 10 --warmup 2
    run bench_cfg4 300 - $B --config cfg4 --steps 5 --warmup 1
    qprof r06a_cfg3 tile_kernel --config cfg3 --plan tile_w256_c1 -- --config cfg3 --steps 5 --warmup 1
    ;;
  ab1)
    # same box, alternating: round-5 library (base), fast-var HEAD, HEAD without DMA (pure
    # instruction time, results garbage); then the cfg3 feature dissection at HEAD
    for rep in 1 2; do
      for v in base new nodma; do
        L=""; [ $v != new ] && L="MHF_DIAGNOSTICS=1 MHF_LIB=_ab/libmhfeat_$v.so"
        for c in cfg3 cfg2; do
          run ab_${c}_${v}_$rep 200 "${L:--}" $B --config $c --steps 10 --warmup 2
        done
        run ab_cfg4_${v}_$rep 300 "${L:--}" $B --config cfg4 --steps 3 --warmup 1
      done
    done
    for f in mean mean,var,skewness,kurtosis band_power band_power,spectral_entropy mean,var,skewness,kurtosis,band_power; do
      run dis_cfg3_${f//,/_} 200 - $B --config cfg3 --features $f --steps 10 --warmup 2
      run dis_cfg3_nodma_${f//,/_} 200 MHF_LIB=_ab/libmhfeat_nodma.so $B --config cfg3 --features $f --steps 10 --warmup 2
    done
    ;;
  ab2)
    # L2 warm-up of chunks 4-7 in the SPEC tiles (HEAD) vs without (_ab/libmhfeat_nowarm.so)
    SOFT=1
    run warm_parity 600 - $PYTNX tests/test_gpu_parity.py -k "fast_var or full_size_workload_every_window_vs_oracle_and_halves and (cfg3 or cfg4) or spectral_vs_oracle or fused"
    SOFT=0
    for rep in 1 2; do
      for v in new nowarm; do
        L=""; [ $v != new ] && L="MHF_DIAGNOSTICS=1 MHF_LIB=_ab/libmhfeat_$v.so"
        run ab_cfg3_${v}_$rep 200 "${L:--}" $B --config cfg3 --steps 10 --warmup 2
        run ab_cfg4_${v}_$rep 300 "${L:--}" $B --config cfg4 --steps 3 --warmup 1
      done
    done
    ;;
  b)
    # split FFT (HEAD) vs fast var only (_ab/libmhfeat_fv.so): the GPU suite, then A/B
    SOFT=1
    run tests_gpu 900 - $PYTNX tests
    SOFT=0
    for rep in 1 2; do
      for v in new fv; do
        L=""; [ $v != new ] && L="MHF_DIAGNOSTICS=1 MHF_LIB=_ab/libmhfeat_$v.so"
        run ab_cfg3_${v}_$rep 200 "${L:--}" $B --config cfg3 --steps 10 --warmup 2
        run ab_cfg4_${v}_$rep 300 "${L:--}" $B --config cfg4 --steps 3 --warmup 1
        run ab_cfg2_${v}_$rep 200 "${L:--}" $B --config cfg2 --steps 20 --warmup 3
      done
    done
    qprof r06b_cfg3 tile_kernel --config cfg3 --plan tile_w256_c1 -- --config cfg3 --steps 5 --warmup 1
    ;;
  diag1)
    # which library faults on the tile_fix golden case: fast-var build (last green), the
    # current tree with the pre-refactor tile_idx.hip.h, the current tree. Stops at the
    # first GPU fault (a fault inside pytest is a failed test: the log is checked)
    export HIP_LAUNCH_BLOCKING=1 AMD_SERIALIZE_KERNEL=3
    for v in fv oldidx new; do
      L="-"; [ $v != new ] && L="MHF_DIAGNOSTICS=1 MHF_LIB=_ab/libmhfeat_$v.so"
      run diag_$v 300 "$L" python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py -k "golden and (one_window or ragged or w3_s1)"
      if grep -q "illegal memory access\|HIP error" gpurun_out/diag_$v.log; then echo "FAULT with $v"; exit 3; fi
    done
    ;;
  b2)
    # after the s_nop 4 hazard fix: the faulting golden case first (stop on a fault), then
    # the whole suite, the split-FFT A/B, the cfg3 profile
    run diag_new 300 - python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py -k "golden and (one_window or ragged or w3_s1)"
    if grep -q "illegal memory access\|HIP error" gpurun_out/diag_new.log; then echo "FAULT"; exit 3; fi
    SOFT=1
    run tests_gpu 900 - $PYTNX tests
    if grep -q "illegal memory access" gpurun_out/tests_gpu.log; then echo "FAULT in suite"; exit 3; fi
    SOFT=0
    for rep in 1 2; do
      for v in new fv; do
        L=""; [ $v != new ] && L="MHF_DIAGNOSTICS=1 MHF_LIB=_ab/libmhfeat_$v.so"
        run ab_cfg3_${v}_$rep 200 "${L:--}" $B --config cfg3 --steps 10 --warmup 2
        run ab_cfg4_${v}_$rep 300 "${L:--}" $B --config cfg4 --steps 3 --warmup 1
      done
    done
    qprof r06b_cfg3 tile_kernel --config cfg3 --plan tile_w256_c1 -- --config cfg3 --steps 5 --warmup 1
    ;;
  c)
    # the whole suite; BASELINE bench lines with the CPU baseline; cfg4 / cfg5 profiles
    SOFT=1
    run tests_gpu 900 - $PYTNX tests
    if grep -q "illegal memory access" gpurun_out/tests_gpu.log; then echo "FAULT in suite"; exit 3; fi
    SOFT=0
    run bench_default 300 - python bench.py
    for c in cfg3 cfg4 cfg5; do
      run bench_$c 400 - python bench.py --config $c --steps 10 --warmup 2
    done
    qprof r06c_cfg4 tile_kernel --config cfg4 --plan tile_w256_c3 -- --config cfg4 --steps 3 --warmup 1
    qprof r06c_cfg5 spectral_reg --config cfg5 --plan spectral_reg -- --config cfg5 --steps 5 --warmup 1
    ;;
  d)
    # cfg5 scalar-stream cut (HEAD: scalar wave index, row-base selects, one-DMA chunks,
    # row lane masks, branch-free min_lanep) vs round-6 c (_ab/libmhfeat_base.so): the W = 1024
    # parity tests, the A/B, the cfg5 profile
    run par_w1024 600 - python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py -k "w1024 or edge_windows or spectral_vs_oracle or full_size_workload_every_window_vs_oracle_and_halves and cfg5"
    if grep -q "illegal memory access" gpurun_out/par_w1024.log; then echo "FAULT"; exit 3; fi
    for rep in 1 2; do
      for v in new base; do
        L=""; [ $v != new ] && L="MHF_DIAGNOSTICS=1 MHF_LIB=_ab/libmhfeat_$v.so"
        run ab_cfg5_${v}_$rep 300 "${L:--}" $B --config cfg5 --steps 10 --warmup 2
      done
    done
    qprof r06d_cfg5 spectral_reg --config cfg5 --plan spectral_reg -- --config cfg5 --steps 5 --warmup 1
    # tile_fix with the default cache policy instead of nt (_ab/libmhfeat_fixpol.so): does L2
    # catch the overlapping windows' second read (ovl250 FETCH 2.72 x distinct with nt)?
    for rep in 1 2; do
      for v in new fixpol; do
        L=""; [ $v != new ] && L="MHF_DIAGNOSTICS=1 MHF_LIB=_ab/libmhfeat_$v.so"
        run ab_ovl250_${v}_$rep 300 "${L:--}" $B --config ovl250 --steps 10 --warmup 2
      done
    done
    for v in new fixpol; do
      L="TMPDIR=/tmp"; [ $v != new ] && L="TMPDIR=/tmp MHF_DIAGNOSTICS=1 MHF_LIB=_ab/libmhfeat_$v.so"
      run fetch_ovl250_$v 300 "$L" rocprofv3 --kernel-trace --pmc FETCH_SIZE --kernel-include-regex tile_idx_kernel --output-format csv -d gpurun_out/pf_$v -o f -- python3 bench.py --no-cpu-baseline --config ovl250 --steps 3 --warmup 1
      python - "$v" <<'PY' >> gpurun_out/fetch_ovl250.txt
import csv, glob, statistics, sys
v = sys.argv[1]
vals = [float(r["Counter_Value"]) for f in glob.glob("gpurun_out/pf_%s/*counter_collection.csv" % v) + glob.glob("gpurun_out/pf_%s/*/*counter_collection.csv" % v)
        for r in csv.DictReader(open(f)) if r["Counter_Name"] == "FETCH_SIZE"]
print(v, "FETCH_SIZE KiB per launch", statistics.mean(vals) if vals else None, "read B", 2 * 1024 * statistics.mean(vals) if vals else None)
PY
      rm -rf gpurun_out/pf_$v
    done
    cat gpurun_out/fetch_ovl250.txt
    ;;
  e)
    # tile_fix span image (HEAD) for overlapping fixed windows: parity first (stop on a
    # fault), then the ovl250 A/B against round-6 c (_ab/libmhfeat_base.so: per-window chunk
    # DMA, nt) and the default-policy chunk DMA (_ab/libmhfeat_fixpol.so), the profile
    run par_span 600 - python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py -k "tile_span or tile_fix or high_address or (full_size and ovl250)"
    if grep -q "illegal memory access\|HIP error" gpurun_out/par_span.log; then echo "FAULT"; exit 3; fi
    for rep in 1 2; do
      for v in new span1 stg8 base; do
        L=""; [ $v != new ] && L="MHF_DIAGNOSTICS=1 MHF_LIB=_ab/libmhfeat_$v.so"
        run ab_ovl250_${v}_$rep 300 "${L:--}" $B --config ovl250 --steps 10 --warmup 2
      done
    done
    KRE=tile_idx_kernel profile r06e_ovl250 --config ovl250 --plan tile_fix -- --config ovl250 --steps 5 --warmup 1
    ;;
  f)
    # fast var with the centering guard (HEAD): its parity tests and the full-size register
    # tile workloads; then what the span kernel's wait is made of: no span wait / no stores
    # (diagnostic builds, results garbage) against HEAD
    run par_fv 900 - python -u -m pytest -x -q --timeout 600 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py -k "fast_var or (full_size and (cfg2 or cfg3 or cfg4))"
    if grep -q "illegal memory access\|HIP error" gpurun_out/par_fv.log; then echo "FAULT"; exit 3; fi
    run smoke 300 - python -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')"
    for rep in 1 2; do
      for v in new nowait nostore; do
        L=""; [ $v != new ] && L="MHF_DIAGNOSTICS=1 MHF_LIB=_ab/libmhfeat_$v.so"
        run ab_ovl250_${v}_$rep 300 "${L:--}" $B --config ovl250 --steps 10 --warmup 2
      done
      run ab_cfg3_new_$rep 300 - $B --config cfg3 --steps 10 --warmup 2
    done
    ;;
  g)
    # spectral_reg with bin-ordered lanes after transpose 2 (HEAD) against the round-6 d
    # build (_ab/libmhfeat_span1.so): the W = 1024 parity tests, the cfg5 A/B, the profile
    run par_w1024 600 - python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py -k "w1024 or edge_windows or spectral_vs_oracle or full_size_workload_every_window_vs_oracle_and_halves and cfg5"
    if grep -q "illegal memory access" gpurun_out/par_w1024.log; then echo "FAULT"; exit 3; fi
    for rep in 1 2; do
      for v in new span1; do
        L=""; [ $v != new ] && L="MHF_DIAGNOSTICS=1 MHF_LIB=_ab/libmhfeat_$v.so"
        run ab_cfg5_${v}_$rep 300 "${L:--}" $B --config cfg5 --steps 10 --warmup 2
      done
    done
    qprof r06g_cfg5 spectral_reg --config cfg5 --plan spectral_reg -- --config cfg5 --steps 5 --warmup 1
    ;;
  final1)
    # round-end validation at HEAD: the whole GPU suite, smoke, every bench line with its CPU
    # baseline (the default line first)
    SOFT=1
    run tests_gpu 900 - $PYTNX tests
    if grep -q "illegal memory access" gpurun_out/tests_gpu.log; then echo "FAULT in suite"; exit 3; fi
    SOFT=0
    run smoke 300 - python -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')"
    run bench_default 300 - python bench.py
    for c in cfg3 cfg4 cfg5 ovl250 cfgidx cfg2f64; do
      run bench_$c 400 - python bench.py --config $c --steps 10 --warmup 2
    done
    ;;
  final2)
    for c in cfg3f64 filt cfg2med cfg2ord sampen256 cfg5m ovl256; do
      run bench_$c 400 - python bench.py --config $c --steps 10 --warmup 2
    done
    KRE=tile_kernel profile ${P:-r06h}_cfg2 --config cfg2 --plan tile_w256_c3 -- --config cfg2 --steps 10 --warmup 2
    KRE=tile_kernel profile ${P:-r06h}_cfg3 --config cfg3 --plan tile_w256_c1 -- --config cfg3 --steps 5 --warmup 1
    ;;
  final3)
    KRE=tile_kernel profile ${P:-r06h}_cfg4 --config cfg4 --plan tile_w256_c3 -- --config cfg4 --steps 3 --warmup 1
    KRE=spectral_reg profile ${P:-r06h}_cfg5 --config cfg5 --plan spectral_reg -- --config cfg5 --steps 5 --warmup 1
    KRE=tile_idx_kernel profile ${P:-r06h}_ovl250 --config ovl250 --plan tile_fix -- --config ovl250 --steps 5 --warmup 1
    KRE=tile_idx_kernel profile ${P:-r06h}_cfgidx --config cfgidx --plan tile_idx -- --config cfgidx --steps 5 --warmup 1
    ;;
  h)
    # tile_idx / tile_fix wave reductions through DPP (HEAD) against the round-end build
    # (_ab/libmhfeat_r6i.so): their parity tests, then cfgidx / ovl250 A/B
    run par_idx 900 - python -u -m pytest -x -q --timeout 600 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py -k "indexed or tile_idx or tile_fix or tile_span or high_address or cfgidx or (full_size and ovl250) or division or aos or single_channel"
    if grep -q "illegal memory access\|HIP error" gpurun_out/par_idx.log; then echo "FAULT"; exit 3; fi
    for rep in 1 2; do
      for v in new dpp; do
        L=""; [ $v != new ] && L="MHF_DIAGNOSTICS=1 MHF_LIB=_ab/libmhfeat_$v.so"
        run ab_cfgidx_${v}_$rep 300 "${L:--}" $B --config cfgidx --steps 10 --warmup 2
        run ab_ovl250_${v}_$rep 300 "${L:--}" $B --config ovl250 --steps 10 --warmup 2
      done
    done
    ;;
  i)
    # order statistics: HEAD against HEAD with round 5's order.hip (_ab/libmhfeat_ord5.so):
    # is the cfg2med / cfg2ord round-end reading (1.37 / 4.74 ms vs 1.22 / 4.44 at round 5) a
    # regression or the box?
    for rep in 1 2; do
      for v in new ord5; do
        L=""; [ $v != new ] && L="MHF_DIAGNOSTICS=1 MHF_LIB=_ab/libmhfeat_$v.so"
        run ab_cfg2med_${v}_$rep 300 "${L:--}" $B --config cfg2med --steps 10 --warmup 2
        run ab_cfg2ord_${v}_$rep 300 "${L:--}" $B --config cfg2ord --steps 10 --warmup 2
      done
    done
    ;;
  j)
    # order_sel_kernel with one special-value ballot per key (HEAD): order parity tests, then
    # the session-i A/B against round 5's order.hip
    run par_ord 900 - python -u -m pytest -x -q --timeout 600 --timeout-method thread -p no:cacheprovider -m gpu tests -k "order or median or percentile or iqr or quantile or mode or special or nan or zero"
    if grep -q "illegal memory access\|HIP error" gpurun_out/par_ord.log; then echo "FAULT"; exit 3; fi
    for rep in 1 2; do
      for v in new ord5; do
        L=""; [ $v != new ] && L="MHF_DIAGNOSTICS=1 MHF_LIB=_ab/libmhfeat_$v.so"
        run ab_cfg2med_${v}_$rep 300 "${L:--}" $B --config cfg2med --steps 10 --warmup 2
        run ab_cfg2ord_${v}_$rep 300 "${L:--}" $B --config cfg2ord --steps 10 --warmup 2
      done
    done
    ;;
  k)
    # fast var on the any-length fixed tile (HEAD) against the r06m build (_ab/libmhfeat_r6m.so):
    # the tile_fix parity tests (exact replay and default numerics, full-size ovl250), then
    # the ovl250 A/B
    run par_fix 900 - python -u -m pytest -x -q --timeout 600 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py -k "tile_fix or fast_var or tile_span or high_address or division or (full_size and ovl250)"
    if grep -q "illegal memory access\|HIP error" gpurun_out/par_fix.log; then echo "FAULT"; exit 3; fi
    for rep in 1 2; do
      for v in new r6m; do
        L=""; [ $v != new ] && L="MHF_DIAGNOSTICS=1 MHF_LIB=_ab/libmhfeat_$v.so"
        run ab_ovl250_${v}_$rep 300 "${L:--}" $B --config ovl250 --steps 10 --warmup 2
      done
    done
    ;;
  *)
    echo "usage: $0 a|ab1|ab2|b|diag1|b2|c|d|e|f|g|h|i|j|k|final1|final2|final3" >&2; exit 2;;
esac
