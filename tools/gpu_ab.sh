#!/bin/bash
# A/B session: each STEP "name|env|timeout|command" runs under its own time limit; the
# session stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
run() {  # run <name> <timeout> <env assignments or -> <cmd...>
  local name=$1 t=$2 envs=$3; shift 3
  echo "=== $name"
  if [ "$envs" = "-" ]; then timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  else env $envs timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; fi
  local rc=$?
  tail -n 2 "gpurun_out/$name.log" | cut -c1-1200
  echo "=== $name rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu"
B="python bench.py --no-cpu-baseline"
case "${1:-}" in
  f64)
    run t64tests 600 - $PYT tests/test_gpu_parity.py -k "float64 or long_windows"
    run b64 300 - $B --config cfg2f64 --steps 10 --warmup 2
    run b64old 300 MHF_NO_TILE64=1 $B --config cfg2f64 --steps 5 --warmup 1
    ;;
  nw2)
    run nw2tests 600 MHF_SPECREG_NW2=1 $PYT tests/test_gpu_parity.py -k "w1024 or edge_windows or full_size"
    for i in 1 2; do
      run cfg5_nw1_$i 300 - $B --config cfg5 --steps 10 --warmup 2
      run cfg5_nw2_$i 300 MHF_SPECREG_NW2=1 $B --config cfg5 --steps 10 --warmup 2
    done
    ;;
  stores)
    for i in 1 2; do
      run cfg2_f64_$i 300 - $B --steps 20 --warmup 3
      run cfg2_f64_nostore_$i 300 MHF_LIB=pymhealth_amd/libmhfeat_nostore.so $B --steps 20 --warmup 3
      run cfg2_f32_$i 300 - $B --steps 20 --warmup 3 --out-dtype f32
      run cfg3_f64_$i 300 - $B --config cfg3 --steps 10 --warmup 2
      run cfg3_nostore_$i 300 MHF_LIB=pymhealth_amd/libmhfeat_nostore.so $B --config cfg3 --steps 10 --warmup 2
    done
    ;;
  swait)
    # price the scalar-load waits of the in-lane spectral code (diagnostic build, garbage results)
    export LIBS="pymhealth_amd/libmhfeat.so pymhealth_amd/libmhfeat_nosw.so"
    export CONFIGS="${CONFIGS:-cfg3 cfg4}" REPS=2
    run abrun 900 - bash tools/ab_bench.sh
    ;;
  spipe)
    # pipelined scalar table loads in the in-lane spectral code: parity, then A/B vs the
    # previous build and the no-wait diagnostic
    run spipe_parity 600 - $PYT tests/test_gpu_parity.py -k "spectral or fused or full_size or rolling_apply"
    export LIBS="pymhealth_amd/libmhfeat_prev.so pymhealth_amd/libmhfeat.so pymhealth_amd/libmhfeat_nosw.so"
    export CONFIGS="${CONFIGS:-cfg3 cfg4}" REPS=2
    run abrun 900 - bash tools/ab_bench.sh
    ;;
  contig)
    # contiguous tile runs per block (output partial lines merge in one L2) vs round robin
    run contig_parity 600 MHF_LIB=pymhealth_amd/libmhfeat_contig.so $PYT tests/test_gpu_parity.py -k "full_size or fused or multichannel or rolling_apply"
    export LIBS="pymhealth_amd/libmhfeat.so pymhealth_amd/libmhfeat_contig.so"
    export CONFIGS="${CONFIGS:-cfg2 cfg3 cfg4}" REPS=2
    run abrun 900 - bash tools/ab_bench.sh
    ;;
  idx)
    # time-indexed windows at bench size: parity of every window, then the bench line
    run idx_parity 600 - $PYT tests/test_gpu_parity.py -k "indexed"
    run bench_cfgidx 300 - $B --config cfgidx --steps 10 --warmup 2
    ;;
  idxshm)
    # indexed kernel occupancy cap (dynamic LDS per 256-thread block) on cfgidx
    run idx_parity 600 - $PYT tests/test_gpu_parity.py -k "indexed or nonuniform"
    for i in 1 2; do
      for k in 0 20 40 80; do
        run idx_shm${k}_$i 300 MHF_IDX_SHM=$k $B --config cfgidx --steps 10 --warmup 2
      done
    done
    ;;
  idxxl)
    # pass-1 extras levels in window_moments (zero crossings alone) and the hoisted-reciprocal
    # division: the exhaustive division probe, the full GPU suite, then A/B
    run div_probe 300 - ./tools/div_probe 65536
    run tests_gpu 900 - python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests
    for i in 1 2; do
      run idx_prev_$i 300 "MHF_IDX_SHM=40 MHF_LIB=pymhealth_amd/libmhfeat_prev.so" $B --config cfgidx --steps 10 --warmup 2
      run idx_new_$i 300 - $B --config cfgidx --steps 10 --warmup 2
    done
    ;;
  idxab)
    for i in 1 2; do
      run idx_prev_$i 300 "MHF_IDX_SHM=40 MHF_LIB=pymhealth_amd/libmhfeat_prev.so" $B --config cfgidx --steps 10 --warmup 2
      run idx_new_$i 300 - $B --config cfgidx --steps 10 --warmup 2
    done
    for i in 1 2; do
      run ovl250_prev_$i 300 "MHF_LIB=pymhealth_amd/libmhfeat_prev.so" $B --config ovl250 --steps 10 --warmup 2
      run ovl250_new_$i 300 - $B --config ovl250 --steps 10 --warmup 2
    done
    ;;
  generic)
    # lane-walk kernels remapped to (window, channel) lanes: whole GPU suite, then the
    # forced-generic cfg2 / cfg3 and the moments_f64_kernel cfg2f64 lines
    run tests_gpu 1000 - python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests
    for c in cfg2 cfg3; do run generic_$c 300 MHF_FORCE_GENERIC=1 $B --config $c --steps 5 --warmup 1 --windows 200000; done
    run f64_generic 300 MHF_NO_TILE64=1 $B --config cfg2f64 --steps 5 --warmup 1
    run bench_cfgidx 300 - $B --config cfgidx --steps 10 --warmup 2
    ;;
  nodma)
    # the tile kernels with every LDS-DMA skipped (diagnostic build, results garbage): the
    # pure instruction time of the bit-exact design at one wave per SIMD
    export LIBS="pymhealth_amd/libmhfeat.so pymhealth_amd/libmhfeat_nodma.so"
    export CONFIGS="${CONFIGS:-cfg2 cfg3 cfg4}" REPS=2
    run abrun 900 - bash tools/ab_bench.sh
    ;;
  walk)
    # loads in flight per lane in the global-memory walks (MHF_GLOB_WALK 8 / 16 / 32)
    run walk_parity 600 "MHF_LIB=pymhealth_amd/libmhfeat_w32.so" $PYT tests/test_gpu_parity.py -k "indexed or division or n3_n4 or edge_sizes or float64"
    for i in 1 2; do
      for l in libmhfeat libmhfeat_w16 libmhfeat_w32; do
        run idx_${l}_$i 300 "MHF_LIB=pymhealth_amd/$l.so" $B --config cfgidx --steps 10 --warmup 2
        run gen_${l}_$i 300 "MHF_LIB=pymhealth_amd/$l.so MHF_FORCE_GENERIC=1" $B --config cfg2 --steps 5 --warmup 1 --windows 200000
      done
    done
    ;;
  ldswalk)
    # samples per batch in the LDS walks (span kernel): 8 / 16
    run lw_parity 600 "MHF_LIB=pymhealth_amd/libmhfeat_l16.so" $PYT tests/test_gpu_parity.py -k "overlap or division or n3_n4 or sharded"
    for i in 1 2; do
      for l in libmhfeat libmhfeat_l16; do
        run ovl_${l}_$i 300 "MHF_LIB=pymhealth_amd/$l.so" $B --config ovl250 --steps 10 --warmup 2
        run c5m_${l}_$i 300 "MHF_LIB=pymhealth_amd/$l.so" $B --config cfg5m --steps 10 --warmup 2
      done
    done
    ;;
  ext)
    # lane-walk / span kernels specialised on the extended features (EXT = false for moment
    # sets), window_moments force-inlined (exti), LDS walk batch 16 (l16)
    run ext_parity 900 "MHF_LIB=pymhealth_amd/libmhfeat_exti.so" python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests
    for i in 1 2; do
      for l in libmhfeat libmhfeat_ext libmhfeat_exti libmhfeat_l16; do
        run ovl_${l}_$i 300 "MHF_LIB=pymhealth_amd/$l.so" $B --config ovl250 --steps 5 --warmup 1
        run idx_${l}_$i 300 "MHF_LIB=pymhealth_amd/$l.so" $B --config cfgidx --steps 5 --warmup 1
        run gen_${l}_$i 300 "MHF_LIB=pymhealth_amd/$l.so MHF_FORCE_GENERIC=1" $B --config cfg2 --steps 5 --warmup 1 --windows 200000
      done
    done
    ;;
  shm2)
    # occupancy cap of the lane-walk kernels after the inlining (61 VGPRs): 0/20/27/40/53 KiB
    for i in 1 2; do
      for k in 0 20 27 40 53; do
        run idxs_${k}_$i 300 MHF_IDX_SHM=$k $B --config cfgidx --steps 5 --warmup 1
        run gens_${k}_$i 300 "MHF_IDX_SHM=$k MHF_FORCE_GENERIC=1" $B --config cfg2 --steps 5 --warmup 1 --windows 200000
      done
      run idxg16_$i 300 "MHF_LIB=pymhealth_amd/libmhfeat_g16.so" $B --config cfgidx --steps 5 --warmup 1
      run geng16_$i 300 "MHF_LIB=pymhealth_amd/libmhfeat_g16.so MHF_FORCE_GENERIC=1" $B --config cfg2 --steps 5 --warmup 1 --windows 200000
    done
    ;;
  verify)
    # the final lane-walk settings: whole GPU suite, smoke, default bench, lane-walk workloads
    run tests_gpu 1000 - python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests
    run smoke 300 - python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')"
    run bench_default 400 - python bench.py
    for i in 1 2; do
      run vidx_$i 300 - $B --config cfgidx --steps 10 --warmup 2
      run vgen_$i 300 MHF_FORCE_GENERIC=1 $B --config cfg2 --steps 5 --warmup 1 --windows 200000
      run vovl_$i 300 - $B --config ovl250 --steps 5 --warmup 1
    done
    ;;
  finish)
    [ "${SKIP_PARITY:-0}" = "1" ] || run parity_new 600 - $PYT tests/test_gpu_parity.py -k "rolling_apply or full_size or fused or multichannel or single_channel or spectral"
    [ "${SKIP_PARITY:-0}" = "1" ] || run parity_raw 600 MHF_LIB=pymhealth_amd/libmhfeat_raw.so $PYT tests/test_gpu_parity.py -k "spectral or fused or full_size"
    export LIBS="pymhealth_amd/libmhfeat_prev.so pymhealth_amd/libmhfeat.so pymhealth_amd/libmhfeat_raw.so"
    export CONFIGS="cfg2 cfg3 cfg4" REPS=2
    run abrun 900 - bash tools/ab_bench.sh
    ;;
esac
