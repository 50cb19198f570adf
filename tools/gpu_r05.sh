#!/bin/bash
# Round-5 GPU sessions (historical record of the round-5 measurements; the round-4
# experimental switches and the exp / tile modes that set them are gone): each step "name timeout env cmd..." runs under its own time limit;
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
case "${1:-}" in
  order)
    # order kernel: DPP / permlane register bitonic, ballot counts, 4 waves per SIMD; the
    # sampen match-word walk; parity of both, then their benches
    SOFT=1
    run order_parity 600 - $PYT tests -k "median or order or percentile or mode or iqr or interquartile or sort"
    run sampen_parity 600 - $PYT tests -k "sampen or rqa"
    run bench_cfg2med 200 - $B --config cfg2med --steps 10 --warmup 2
    run bench_sampen256 200 - $B --config sampen256 --steps 5 --warmup 1
    ;;
  profo)
    run prof_cfg2med 600 "KRE=order_kernel" bash tools/profile.sh r05a_cfg2med --config cfg2med --steps 5 --warmup 1
    run prof_sampen 600 "KRE=sampen_kernel" bash tools/profile.sh r05a_sampen256 --config sampen256 --steps 3 --warmup 1
    ;;
  meas)
    # the whole GPU suite at HEAD, smoke, then one bench line per workload
    run tests_gpu 900 - python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests
    run smoke 300 - python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')"
    run bench_default 400 - python bench.py
    for c in cfg3 cfg4 cfg5 cfgidx ovl250 cfg2med cfg2ord sampen256 cfg2f64 cfg3f64; do
      run bench_$c 300 - $B --config $c --steps 10 --warmup 2
    done
    run bench_filt 300 - $B --config filt --steps 5 --warmup 1
    QUICK=1 run prof_q_cfg2med 300 "KRE=order_" bash tools/profile.sh r05o_cfg2med --config cfg2med --steps 3 --warmup 1
    python tools/prof_summary.py r05o_cfg2med --config cfg2med --sum-kernels > gpurun_out/summ_r05o_cfg2med.log 2>&1 || true
    mkdir -p gpurun_out/summ && cp profiles/r05o_cfg2med_* gpurun_out/summ/ 2>/dev/null; rm -rf gpurun_out/prof_r05o_cfg2med
    ;;
  profb)
    # HEAD profiles of the BASELINE workloads and the promoted register tiles
    M5="--features mean,var,skewness,kurtosis,zero_crossings"
    KRE= profile r05b_cfg2 --config cfg2 --plan tile_w256_c3 $M5 -- --config cfg2 --steps 10 --warmup 2
    KRE= profile r05b_cfg4 --config cfg4 --plan tile_w256_c3 -- --config cfg4 --steps 3 --warmup 1
    KRE= profile r05b_cfg5 --config cfg5 --plan spectral_reg -- --config cfg5 --steps 5 --warmup 1
    KRE=tile_idx_kernel profile r05b_cfgidx --config cfgidx --plan tile_idx $M5 -- --config cfgidx --steps 5 --warmup 1
    KRE=tile_idx_kernel profile r05b_ovl250 --config ovl250 --plan tile_fix -- --config ovl250 --steps 5 --warmup 1
    KRE= profile r05b_cfg3 --config cfg3 --plan tile_w256_c1 -- --config cfg3 --steps 5 --warmup 1
    ;;
  sampen)
    run sampen_parity 600 - $PYT tests -k "sampen or rqa"
    run bench_sampen256 200 - $B --config sampen256 --steps 5 --warmup 1
    KRE=sampen_kernel profile r05c_sampen256 --config sampen256 --plan sampen --features sampen -- --config sampen256 --steps 3 --warmup 1
    ;;
  filt)
    # the LDS-streamed filtfilt passes: parity first (small records), then the bench and
    # the profile
    run filt_parity 300 - $PYT tests/test_gpu_parity.py -k "filtfilt or filter or n2"
    run bench_filt 200 - $B --config filt --steps 5 --warmup 1
    run bench_filt_old 200 MHF_NO_IIR_TILE=1 $B --config filt --steps 5 --warmup 1
    KRE=iir_tile_kernel profile r05d_filt --config filt --plan filtfilt --windows 100000000 --sum-kernels -- --config filt --steps 3 --warmup 1
    ;;
  fdbg)
    run filt_debug 120 - python tools/filt_debug.py 70001
    run filt_debug_big 120 - python tools/filt_debug.py 3000001
    ;;
  sel)
    # order selection without sorting; the LDS-streamed filtfilt as the default
    run order_parity 600 - $PYT tests -k "median or order or percentile or mode or iqr or interquartile or sort"
    run filt_parity 300 - $PYT tests -k "filtfilt or filter or n2 or accel"
    run bench_cfg2med 200 - $B --config cfg2med --steps 10 --warmup 2
    run bench_filt 200 - $B --config filt --steps 5 --warmup 1
    QUICK=1 run prof_q_cfg2med 300 "KRE=order_kernel" bash tools/profile.sh r05e_cfg2med --config cfg2med --steps 3 --warmup 1
    python tools/prof_summary.py r05e_cfg2med --config cfg2med > gpurun_out/summ_r05e_cfg2med.log 2>&1 || true
    mkdir -p gpurun_out/summ && cp profiles/r05e_cfg2med_* gpurun_out/summ/ 2>/dev/null; rm -rf gpurun_out/prof_r05e_cfg2med
    ;;
  samp)
    # sampen: cyclic-diagonal walk (MHF_NO_SAMPEN_CYC=1: the straight-diagonal pairs)
    run sampen_parity 600 - $PYT tests -k "sampen or rqa"
    run bench_sampen256 200 - $B --config sampen256 --steps 5 --warmup 1
    run bench_sampen256_old 200 MHF_NO_SAMPEN_CYC=1 $B --config sampen256 --steps 5 --warmup 1
    QUICK=1 run prof_q_sampen 300 "KRE=sampen_kernel" bash tools/profile.sh r05f_sampen256 --config sampen256 --steps 3 --warmup 1
    python tools/prof_summary.py r05f_sampen256 --config sampen256 > gpurun_out/summ_r05f_sampen256.log 2>&1 || true
    mkdir -p gpurun_out/summ && cp profiles/r05f_sampen256_* gpurun_out/summ/ 2>/dev/null; rm -rf gpurun_out/prof_r05f_sampen256
    ;;
  tidx)
    # tile_idx / tile_fix with the pieces past each window's end redirected (no reach into
    # the next window's lines): parity, benches, the HBM read of cfgidx
    run tidx_parity 600 - $PYT tests/test_gpu_parity.py -k "tile or indexed or cfgidx or aos or division or single_channel or ovl250 or fixed"
    run bench_cfgidx 200 - $B --config cfgidx --steps 10 --warmup 2
    run bench_ovl250 200 - $B --config ovl250 --steps 10 --warmup 2
    KRE=tile_idx_kernel profile r05g_cfgidx --config cfgidx --plan tile_idx --windows 1000000 -- --config cfgidx --steps 3 --warmup 1
    ;;
  combo1)
    bash tools/gpu_r05.sh tidx || exit $?
    run order_parity 600 - $PYT tests -k "median or order or percentile or mode or iqr or interquartile or non_current"
    run bench_cfg2med 200 - $B --config cfg2med --steps 10 --warmup 2
    run sampen_parity 600 - $PYT tests -k "sampen or rqa"
    run bench_sampen256 200 - $B --config sampen256 --steps 5 --warmup 1
    ;;
  combo2)
    run order_parity 600 - $PYT tests -k "median or order or percentile or mode or iqr or interquartile or non_current"
    run bench_cfg2med 200 - $B --config cfg2med --steps 10 --warmup 2
    run sampen_parity 600 - $PYT tests -k "sampen or rqa"
    run bench_sampen256 200 - $B --config sampen256 --steps 5 --warmup 1
    run tidx_parity 600 - $PYT tests/test_gpu_parity.py -k "tile or indexed or cfgidx or aos or division or single_channel or ovl250 or fixed"
    run bench_ovl250 200 - $B --config ovl250 --steps 10 --warmup 2
    run bench_cfgidx 200 - $B --config cfgidx --steps 10 --warmup 2
    ;;
  abtidx)
    # tile_idx at HEAD vs before the DMA redirect / exactness-tracking change
    for rep in 1 2; do
      run bench_ovl250_$rep 200 - $B --config ovl250 --steps 10 --warmup 2
      run bench_ovl250_old_$rep 200 MHF_LIB=_ab/libmhfeat_tidxold.so $B --config ovl250 --steps 10 --warmup 2
      run bench_cfgidx_$rep 200 - $B --config cfgidx --steps 10 --warmup 2
      run bench_cfgidx_old_$rep 200 MHF_LIB=_ab/libmhfeat_tidxold.so $B --config cfgidx --steps 10 --warmup 2
    done
    ;;
  ab2)
    run tidx_parity 600 - $PYT tests/test_gpu_parity.py -k "tile or indexed or cfgidx or aos or division or single_channel or ovl250 or fixed"
    for rep in 1 2; do
      run bench_ovl250_$rep 200 - $B --config ovl250 --steps 10 --warmup 2
      run bench_ovl250_old_$rep 200 MHF_LIB=_ab/libmhfeat_tidxold.so $B --config ovl250 --steps 10 --warmup 2
      run bench_cfgidx_$rep 200 - $B --config cfgidx --steps 10 --warmup 2
    done
    KRE=iir_tile_kernel profile r05h_filt --config filt --plan filtfilt --windows 100000000 --sum-kernels -- --config filt --steps 3 --warmup 1
    ;;
  med)
    run order_parity 600 - $PYTNX tests -k "median or order or percentile or mode or iqr or interquartile or rolling or golden"
    run bench_cfg2med_1 200 - $B --config cfg2med --steps 10 --warmup 2
    run bench_cfg2med_2 200 - $B --config cfg2med --steps 10 --warmup 2
    QUICK=1 run prof_q_cfg2med 300 "KRE=order_" bash tools/profile.sh r05n_cfg2med --config cfg2med --steps 3 --warmup 1
    python tools/prof_summary.py r05n_cfg2med --config cfg2med --sum-kernels > gpurun_out/summ_r05n_cfg2med.log 2>&1 || true
    mkdir -p gpurun_out/summ && cp profiles/r05n_cfg2med_* gpurun_out/summ/ 2>/dev/null; rm -rf gpurun_out/prof_r05n_cfg2med
    ;;
  ab5)
    for rep in 1 2; do
      run bench_cfg5_$rep 200 - $B --config cfg5 --steps 10 --warmup 2
      run bench_cfg5_old_$rep 200 MHF_LIB=_ab/libmhfeat_r05a.so $B --config cfg5 --steps 10 --warmup 2
    done
    run bench_cfg3 200 - $B --config cfg3 --steps 10 --warmup 2
    run bench_cfg3_old 200 MHF_LIB=_ab/libmhfeat_r05a.so $B --config cfg3 --steps 10 --warmup 2
    ;;
  profmed)
    QUICK=1 run prof_q_cfg2med 300 "KRE=order_" bash tools/profile.sh r05o_cfg2med --config cfg2med --steps 3 --warmup 1
    python tools/prof_summary.py r05o_cfg2med --config cfg2med --sum-kernels > gpurun_out/summ_r05o_cfg2med.log 2>&1 || true
    mkdir -p gpurun_out/summ && cp profiles/r05o_cfg2med_* gpurun_out/summ/ 2>/dev/null; rm -rf gpurun_out/prof_r05o_cfg2med
    ;;
  ordt)
    run order_parity 600 - $PYTNX tests -k "median or order or percentile or mode or iqr or interquartile or rolling or golden"
    ;;
  c5m)
    run bench_cfg5m 300 - $B --config cfg5m --steps 10 --warmup 2
    run bench_ovl256 300 - $B --config ovl256 --steps 10 --warmup 2
    ;;
  selgrid)
    for b in 16384 32768 65536 250000 8192; do
      run bench_cfg2med_b$b 200 MHF_ORDER_SEL_BLOCKS=$b $B --config cfg2med --steps 10 --warmup 2
    done
    run bench_cfg2med_b32768_2 200 MHF_ORDER_SEL_BLOCKS=32768 $B --config cfg2med --steps 10 --warmup 2
    run bench_cfg2ord_b32768 200 MHF_ORDER_SEL_BLOCKS=32768 $B --config cfg2ord --steps 10 --warmup 2
    run bench_cfg2ord_b8192 200 MHF_ORDER_SEL_BLOCKS=8192 $B --config cfg2ord --steps 10 --warmup 2
    ;;
  fin)
    run tests_gpu 900 - python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests
    run smoke 300 - python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')"
    run bench_default 400 - python bench.py
    run bench_cfg2med 300 - $B --config cfg2med --steps 10 --warmup 2
    run bench_cfg2ord 300 - $B --config cfg2ord --steps 10 --warmup 2
    QUICK=1 run prof_q_cfg2med 300 "KRE=order_" bash tools/profile.sh r05r_cfg2med --config cfg2med --steps 3 --warmup 1
    python tools/prof_summary.py r05r_cfg2med --config cfg2med --sum-kernels > gpurun_out/summ_r05r_cfg2med.log 2>&1 || true
    mkdir -p gpurun_out/summ && cp profiles/r05r_cfg2med_* gpurun_out/summ/ 2>/dev/null; rm -rf gpurun_out/prof_r05r_cfg2med
    ;;
  nostore)
    for rep in 1 2; do
      run bench_cfg2_$rep 200 - $B --config cfg2 --steps 20 --warmup 3
      run bench_cfg2_nostore_$rep 200 MHF_LIB=_ab/libmhfeat_nostore.so $B --config cfg2 --steps 20 --warmup 3
    done
    ;;
  ninterp)
    run order_parity 600 MHF_LIB=_ab/libmhfeat_n3.so $PYTNX tests -k "median or order or percentile or iqr or interquartile"
    for rep in 1 2; do
      for v in base n3 n4; do
        run bench_cfg2med_${v}_$rep 200 MHF_LIB=_ab/libmhfeat_$v.so $B --config cfg2med --steps 10 --warmup 2
        run bench_cfg2ord_${v}_$rep 200 MHF_LIB=_ab/libmhfeat_$v.so $B --config cfg2ord --steps 10 --warmup 2
      done
    done
    ;;
  gen)
    run order_parity 600 - $PYTNX tests -k "median or order or percentile or mode or iqr or interquartile or rolling or golden"
    run order_parity_nosel 600 MHF_NO_ORDER_SEL=1 $PYTNX tests -k "median or order or percentile or iqr or interquartile"
    for rep in 1 2; do
      run bench_cfg2med_gen_$rep 200 MHF_NO_ORDER_SEL=1 $B --config cfg2med --steps 10 --warmup 2
      run bench_cfg2med_gen_old_$rep 200 "MHF_NO_ORDER_SEL=1 MHF_LIB=_ab/libmhfeat_base.so" $B --config cfg2med --steps 10 --warmup 2
    done
    ;;
  vcnt)
    run order_parity 600 - $PYTNX tests -k "median or order or percentile or mode or iqr or interquartile or rolling or golden"
    run bench_cfg2ord 200 - $B --config cfg2ord --steps 10 --warmup 2
    run bench_cfg2ord_old 200 MHF_LIB=_ab/libmhfeat_base.so $B --config cfg2ord --steps 10 --warmup 2
    for rep in 1 2; do
      run bench_cfg2med_$rep 200 - $B --config cfg2med --steps 10 --warmup 2
      run bench_cfg2med_old_$rep 200 MHF_LIB=_ab/libmhfeat_base.so $B --config cfg2med --steps 10 --warmup 2
    done
    ;;
  sel2)
    run order_parity 600 - $PYT tests -k "median or order or percentile or mode or iqr or interquartile"
    run bench_cfg2med 200 - $B --config cfg2med --steps 10 --warmup 2
    run bench_cfg2med_b 200 - $B --config cfg2med --steps 10 --warmup 2
    ;;
  ovlp)
    run tidx_parity 600 - $PYT tests/test_gpu_parity.py -k "tile or indexed or cfgidx or aos or division or single_channel or ovl250 or fixed"
    run bench_cfgidx_1 200 - $B --config cfgidx --steps 10 --warmup 2
    run bench_cfgidx_2 200 - $B --config cfgidx --steps 10 --warmup 2
    run bench_ovl250 200 - $B --config ovl250 --steps 10 --warmup 2
    ;;
  warm)
    run filt_parity 300 - $PYT tests -k "filtfilt or filter or n2 or accel or non_current"
    run bench_filt_1 200 - $B --config filt --steps 5 --warmup 1
    run bench_filt_2 200 - $B --config filt --steps 5 --warmup 1
    KRE=iir_tile_kernel profile r05k_filt --config filt --plan filtfilt --windows 100000000 --sum-kernels -- --config filt --steps 3 --warmup 1
    ;;
  s64)
    run s64_parity 300 - $PYT tests -k "f64 or float64 or spectral64"
    run bench_cfg3f64 300 - $B --config cfg3f64 --steps 5 --warmup 1
    KRE=spectral64_kernel QUICK=1 run prof_q_cfg3f64 300 "KRE=spectral64_kernel|tile64_kernel" bash tools/profile.sh r05l_cfg3f64 --config cfg3f64 --steps 3 --warmup 1
    python tools/prof_summary.py r05l_cfg3f64 --config cfg3f64 > gpurun_out/summ_r05l_cfg3f64.log 2>&1 || true
    mkdir -p gpurun_out/summ && cp profiles/r05l_cfg3f64_* gpurun_out/summ/ 2>/dev/null; rm -rf gpurun_out/prof_r05l_cfg3f64
    ;;
  groups)
    for g in 256 384 512 768 1024 1536; do
      run bench_filt_g$g 200 MHF_IIR_TILE_GROUPS=$g $B --config filt --steps 5 --warmup 1
    done
    ;;
  pol)
    # register tiles with the default DMA cache policy instead of nt (_ab/libmhfeat_pol.so):
    # overlapping / adjacent windows re-read lines another window of the tile just fetched
    for rep in 1 2; do
      run bench_ovl250_$rep 200 - $B --config ovl250 --steps 10 --warmup 2
      run bench_ovl250_pol_$rep 200 MHF_LIB=_ab/libmhfeat_pol.so $B --config ovl250 --steps 10 --warmup 2
      run bench_cfgidx_$rep 200 - $B --config cfgidx --steps 10 --warmup 2
      run bench_cfgidx_pol_$rep 200 MHF_LIB=_ab/libmhfeat_pol.so $B --config cfgidx --steps 10 --warmup 2
    done
    ;;
  *)
    echo "usage: $0 order|profo|meas|profb|sampen|filt|pol|..." >&2; exit 2;;
esac
