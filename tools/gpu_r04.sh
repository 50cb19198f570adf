#!/bin/bash
# HISTORICAL (round 4): kept as the record of that round's sessions. The switches it sets
# (MHF_EXPERIMENTAL, MHF_TILE_IDX / MHF_TILE_FIX, MHF_IIR_RING, ...) were removed in round 5;
# running it today compares the default build with itself.
# Round-4 GPU sessions: each step "name timeout env cmd..." runs under its own time limit,
# the session stops at the first failure (no retries).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
SOFT=0   # 1: a plain failure (exit 1: a test / probe mismatch) does not end the session
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
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu"
B="python bench.py --no-cpu-baseline"
case "${1:-}" in
  abi7)
    # ABI 7 (caller workspaces), fp64 spectral, every-window parity: the whole GPU suite,
    # smoke, the default bench, the strong-scaling pipeline (N = 1 RCCL, N = 2 gloo rehearsal)
    run tests_gpu 1000 - $PYT tests
    run smoke 300 - python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')"
    run bench_default 400 - python bench.py
    run strong1_cfg5 300 - $B --strong --config cfg5 --steps 5 --warmup 1
    run strong1_cfg2 300 - $B --strong --config cfg2 --steps 5 --warmup 1
    run strong2_gloo_cfg5 300 - $B --gpus 2 --backend gloo --strong --config cfg5 --windows 200000 --steps 3 --warmup 1
    run weak2_gloo_cfg2 300 - $B --gpus 2 --backend gloo --steps 5 --warmup 1
    run bench_cfgidx 300 - $B --config cfgidx --steps 10 --warmup 2
    run bench_ovl250 300 - $B --config ovl250 --steps 5 --warmup 1
    run bench_generic 300 MHF_FORCE_GENERIC=1 $B --config cfg2 --steps 5 --warmup 1 --windows 200000
    ;;
  benches)
    run strong1_cfg5 300 - $B --strong --config cfg5 --steps 5 --warmup 1
    run strong1_cfg2 300 - $B --strong --config cfg2 --steps 5 --warmup 1
    run strong2_gloo_cfg5 300 - $B --gpus 2 --backend gloo --strong --config cfg5 --windows 200000 --steps 3 --warmup 1
    run weak2_gloo_cfg2 300 - $B --gpus 2 --backend gloo --steps 5 --warmup 1
    run bench_cfgidx 300 - $B --config cfgidx --steps 10 --warmup 2
    run bench_ovl250 300 - $B --config ovl250 --steps 5 --warmup 1
    run bench_generic 300 MHF_FORCE_GENERIC=1 $B --config cfg2 --steps 5 --warmup 1 --windows 200000
    run order_parity 900 - $PYT tests -k "sampen or rqa or median or order or percentile or mode or iqr"
    run bench_sampen256 300 - $B --config sampen256 --steps 5 --warmup 1
    run bench_cfg2med 300 - $B --config cfg2med --steps 10 --warmup 2
    run bench_cfg5 300 - $B --config cfg5 --steps 10 --warmup 2
    # A/B builds of spectral_reg (ab/, built beside the tree's library): both transposes in
    # LDS (the round-3 kernel), transpose 1 only in registers, both in registers at 5 waves
    # per SIMD with one window per iteration; and this build with one window per iteration
    run bench_cfg5_lds 300 MHF_LIB=ab/libmhfeat_lds.so $B --config cfg5 --steps 10 --warmup 2
    run bench_cfg5_t1 300 MHF_LIB=ab/libmhfeat_t1.so $B --config cfg5 --steps 10 --warmup 2
    run bench_cfg5_x5 300 "MHF_LIB=ab/libmhfeat_x5.so MHF_SPECREG_NW2=0" $B --config cfg5 --steps 10 --warmup 2
    run bench_cfg5_nw1 300 MHF_SPECREG_NW2=0 $B --config cfg5 --steps 10 --warmup 2
    run bench_cfg5_again 300 - $B --config cfg5 --steps 10 --warmup 2
    run bench_cfg3 300 - $B --config cfg3 --steps 10 --warmup 2
    ;;
  f8)
    # §8f kernels measured on their own: bench lines, then rocprofv3 kernel
    # trace + PMC passes (tools/profile.sh) for each, and the cfgidx traffic refresh
    run bench_filt 300 - python bench.py --config filt --steps 5 --warmup 1
    run bench_cfg2med 300 - python bench.py --config cfg2med --steps 10 --warmup 2
    run bench_sampen256 300 - python bench.py --config sampen256 --steps 5 --warmup 1
    run prof_filt 600 "KRE=iir_chunk_kernel" bash tools/profile.sh r04d_filt --config filt --steps 3 --warmup 1
    run prof_cfg2med 600 "KRE=order_kernel" bash tools/profile.sh r04d_cfg2med --config cfg2med --steps 5 --warmup 1
    run prof_sampen 600 "KRE=sampen_kernel" bash tools/profile.sh r04d_sampen256 --config sampen256 --steps 3 --warmup 1
    run prof_cfgidx 600 "KRE=moments_indexed" bash tools/profile.sh r04d_cfgidx --config cfgidx --steps 5 --warmup 1
    ;;
  filt)
    # filtfilt with ~2 waves per SIMD of chunk lanes (was ~8k lanes: 129 waves)
    run filt_parity 600 - $PYT tests/test_gpu_parity.py -k "filtfilt or filter or n2"
    run bench_filt 300 - $B --config filt --steps 5 --warmup 1
    for l in 16384 65536 131072; do
      run bench_filt_l$l 300 MHF_IIR_LANES=$l $B --config filt --steps 5 --warmup 1
    done
    ;;
  tidx)
    # the round-4 paths that are off by default (engine_common.h experimental()): parity of
    # each against the oracle and against its measured default, then A/B benches
    # (MHF_EXPERIMENTAL=1 turns every one on; MHF_TILE_IDX / MHF_TILE_FIX / MHF_IIR_RING /
    # MHF_ORDER_PREFETCH / MHF_SAMPEN_WALK2 one at a time) and kernel profiles
    SOFT=1
    run exp_parity 900 MHF_TEST_EXPERIMENTAL=1 $PYT tests/test_gpu_parity.py -k "tile_path or tile_fix or experimental_paths"
    run tidx_parity 900 MHF_EXPERIMENTAL=1 $PYT tests/test_gpu_parity.py -k "indexed or cfgidx or aos or division or single_channel or ovl250 or filtfilt or filter or n2 or sampen or median or order"
    run bench_cfgidx 300 - $B --config cfgidx --steps 10 --warmup 2
    run bench_cfgidx_tile 300 MHF_TILE_IDX=1 $B --config cfgidx --steps 10 --warmup 2
    run bench_ovl250 300 - $B --config ovl250 --steps 10 --warmup 2
    run bench_ovl250_tile 300 MHF_TILE_FIX=1 $B --config ovl250 --steps 10 --warmup 2
    run bench_filt 300 - $B --config filt --steps 5 --warmup 1
    run bench_filt_ring 300 MHF_IIR_RING=1 $B --config filt --steps 5 --warmup 1
    run bench_cfg2med 300 - $B --config cfg2med --steps 10 --warmup 2
    run bench_cfg2med_pf 300 MHF_ORDER_PREFETCH=1 $B --config cfg2med --steps 10 --warmup 2
    run bench_sampen256 300 - $B --config sampen256 --steps 5 --warmup 1
    run bench_sampen256_w2 300 MHF_SAMPEN_WALK2=1 $B --config sampen256 --steps 5 --warmup 1
    # spectral_reg transposes: A/B builds in ab/ (register exchanges at 4 / 5 waves per SIMD,
    # transpose 1 only) against the tree's (LDS) build
    run bench_cfg5 300 - $B --config cfg5 --steps 10 --warmup 2
    run bench_cfg5_xt 300 MHF_LIB=ab/libmhfeat_xt.so $B --config cfg5 --steps 10 --warmup 2
    run bench_cfg5_t1 300 MHF_LIB=ab/libmhfeat_t1.so $B --config cfg5 --steps 10 --warmup 2
    run bench_cfg5_x5 300 "MHF_LIB=ab/libmhfeat_x5.so MHF_SPECREG_NW2=0" $B --config cfg5 --steps 10 --warmup 2
    run prof_cfgidx 600 "MHF_TILE_IDX=1 KRE=tile_idx_kernel" bash tools/profile.sh r04e_cfgidx --config cfgidx --steps 5 --warmup 1
    run prof_ovl250 600 "MHF_TILE_FIX=1 KRE=tile_idx_kernel" bash tools/profile.sh r04e_ovl250 --config ovl250 --steps 5 --warmup 1
    ;;
  *)
    echo "usage: $0 abi7|benches|f8|filt|tidx" >&2; exit 2;;
esac
