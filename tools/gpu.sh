#!/bin/bash
# The one GPU-box script: `gpurun -- bash tools/gpu.sh <recipe> [<recipe> ...]`, each recipe's
# steps under their own time limits, stopping at the first fault / abort / timeout (exit codes
# other than 0 and 1). Logs and rocprofv3 outputs land in gpurun_out/; the summaries that are
# judged are copied into profiles/rNN/ by tools/collect_profiles.py.
#
# Recipes (what produced which committed profile):
#   tests        pytest -m gpu (PYTEST_K=<expr> narrows it)             -> pytest_gpu.log
#   smoke        __graft_entry__.smoke()                                 -> smoke.log
#   bench        default bench line (N=1, Humanoid 4096)                 -> bench_default.log
#   prof         rocprofv3 --kernel-trace --stats of the default bench   -> kernel_stats_bench_default.*
#   fuse         obs/reward fuse sweeps Humanoid/Ant + rocprof at 1 M    -> fuse_roofline_*.json, kernel_stats_fuse_*
#   fuseab       fuse tile variants 32p vs 16p at 1 M / 2 M envs (alternating) -> DESIGN §6
#   fusepmc      FETCH_SIZE / WRITE_SIZE passes of the fuse at 1 M envs   -> traffic_fuse_*.json (tools/pmc_traffic.py)
#   traffic      env-count FETCH/WRITE sweep of the fused step (TASK=..)  -> traffic_<task>.json (tools/traffic_split.py)
#   sq           SQ issue / wait / occupancy counters of the fused step   -> sq_counters_<task>.txt
#   icache       SQC I-cache + instruction-fetch counters                  -> icache/
#   calib        FETCH_SIZE calibration kernels (tools/fetch_calib.hip)   -> fetch_calib.json
#   pstats       device-vs-oracle error distribution + oracle sensitivity -> parity_stats_<task>.log
#   freerun      free-running device vs oracle distributions              -> free_run_*.log
#   stamps       phase stamps (per-phase s_memtime accumulators)          -> stamps_<task>.log
#   tail         slowest-wave phase stamps of the paired kernel            -> tail/pair_tail_*.log
#   patha        INTEGRATION path (A): reference call sequence over ArticulationView -> path_a_humanoid.json
#   train        PPO frames/s (tools/bench_train.py)                       -> bench_train_*.log
#   curve        reference training schedule, per-epoch curve (tools/train_curve.py) -> train_curve_*.jsonl
#   sizes        env-count sweep of the fused step (tools/bw_sweep.py)     -> bw_sweep_*.json
#   ab           bench A/B: default library vs LIB_B (alternating passes)  -> DESIGN perf log
#   abn          bench A/B/C..: default library vs each of LIBS (alternating passes)
# Environment knobs: TASK (Humanoid), NS (env counts), BARGS (extra bench.py args), TAG (log suffix).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TASK=${TASK:-Humanoid}
TAG=${TAG:-cur}
RP="rocprofv3 --output-format csv"
B="python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --fuse-envs 0 --no-side --task $TASK ${BARGS:-}"

# the diagnostic stamps library stays off the box (.gpurunignore): the two stamps recipes build
# it there (a few minutes of hipcc on the box's CPU) when it is missing
stamps_lib() {
  [ -f omniisaacgymenvs_amd/libmi_sim_stamps.so ] && return 0
  ( for _ in $(seq 1 20); do sleep 30; echo "   building the stamps library ..."; done ) &   # bounded: 10 min
  local tick=$!
  trap "kill $tick 2>/dev/null" EXIT
  run build_stamps 600 python -c "import __graft_entry__ as g; g.build_hip_stamps()"
  kill $tick 2>/dev/null
}

run() {  # run <name> <timeout> <cmd...>; exit codes 0/1 (test failures) continue, others stop
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}

recipe() {
  case "$1" in
  tests)
    run pytest_gpu${PTAG:-} 900 python -u -m pytest tests -m gpu -q ${PYTEST_X--x} --timeout 200 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
    grep -E "^FAILED|^E  .*Error|passed|failed" gpurun_out/pytest_gpu${PTAG:-}.log | head -30 ;;
  smoke)
    run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
  bench)
    run bench_default 600 python -u bench.py ;;
  prof)
    run prof_bench 600 $RP --kernel-trace --stats -d gpurun_out/prof_bench -o run -- python3 bench.py ;;
  fuse)
    run fuse_h 300 python -u tools/fuse_roofline.py Humanoid 4096,65536,131072,262144,1048576,2097152
    run fuse_a 300 python -u tools/fuse_roofline.py Ant 4096,65536,131072,262144,1048576,2097152
    run prof_fuse 300 $RP --kernel-trace --stats -d gpurun_out/prof_fuse -o run -- python3 tools/fuse_roofline.py Humanoid 1048576 20 ;;
  fuseab)   # obs/reward fuse tile variants at 1 M envs, alternating (MI_POST_TILE 32p vs 16p)
    for k in 1 2 3; do
      for V in 32p 16p; do
        for T in Humanoid Ant; do run fab_${V}_${T}_$k 120 env MI_POST_TILE=$V python -u tools/fuse_roofline.py $T 1048576,2097152 30; done
      done
    done
    grep -h '"kernel"' gpurun_out/fab_*.log | cut -c1-200 ;;
  fusepmc)
    for T in Humanoid Ant; do
      run fpf_$T 120 timeout -s KILL 100 $RP --pmc FETCH_SIZE --kernel-trace -d gpurun_out/fpf_$T -o run -- python3 tools/fuse_roofline.py $T 1048576 10
      run fpw_$T 120 timeout -s KILL 100 $RP --pmc WRITE_SIZE --kernel-trace -d gpurun_out/fpw_$T -o run -- python3 tools/fuse_roofline.py $T 1048576 10
    done ;;
  traffic)
    for N in ${NS:-1024 2048 4096 8192 16384}; do
      BN="python3 bench.py --task $TASK --num-envs $N --steps 30 --warmup 5 --no-cpu-baseline --no-side --fuse-envs 0 ${BARGS:-}"
      run tsf_${TASK}_$N 100 timeout -s KILL 90 $RP --pmc FETCH_SIZE --kernel-trace -d gpurun_out/tsf_${TASK}_$N -o run -- $BN
      run tsw_${TASK}_$N 100 timeout -s KILL 90 $RP --pmc WRITE_SIZE --kernel-trace -d gpurun_out/tsw_${TASK}_$N -o run -- $BN
    done ;;
  sq)
    run sq1_${TASK}_$TAG 120 timeout -s KILL 100 $RP --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-trace -d gpurun_out/sq1_${TASK}_$TAG -o run -- $B
    run sq2_${TASK}_$TAG 120 timeout -s KILL 100 $RP --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD --kernel-trace -d gpurun_out/sq2_${TASK}_$TAG -o run -- $B
    run sq3_${TASK}_$TAG 120 timeout -s KILL 100 $RP --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace -d gpurun_out/sq3_${TASK}_$TAG -o run -- $B ;;
  icache)
    run ic1_$TAG 90 timeout -s KILL 80 $RP --kernel-trace --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE -d gpurun_out/ic1_$TAG -o run -- $B
    run ic2_$TAG 90 timeout -s KILL 80 $RP --kernel-trace --pmc SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU -d gpurun_out/ic2_$TAG -o run -- $B ;;
  calib)
    for N in ${NS:-4096 1048576}; do
      run calf_$N 60 $RP --pmc FETCH_SIZE --kernel-trace -d gpurun_out/calf_$N -o run -- tools/fetch_calib $N 6
      run calw_$N 60 $RP --pmc WRITE_SIZE --kernel-trace -d gpurun_out/calw_$N -o run -- tools/fetch_calib $N 6
    done ;;
  pstats)
    for T in ${TASKS:-Humanoid Ant}; do run pstats_${T}_$TAG 300 python -u tools/parity_stats.py $T 4096 4 ${SOLVER:-config}; done ;;
  freerun)
    for T in Humanoid Ant Cartpole; do run free_run_${T}_$TAG 300 python -u tools/free_run.py $T 4096; done ;;
  stamps)
    stamps_lib
    for T in ${TASKS:-Humanoid Ant}; do run stamps_${T}_$TAG 150 python -u tools/phase_stamps.py $T 4096; done ;;
  tail)   # slowest-wave phase stamps of the paired kernel
    stamps_lib
    for T in ${TASKS:-Humanoid}; do run tail_${T}_$TAG 150 python -u tools/pair_tail.py $T 4096 3 ${SOLVER:-config}; done ;;
  patha)
    run path_a 200 python -u tools/path_a_timing.py ;;
  pathaprof)   # kernel trace of path (A): every backend launch and its duration
    run prof_patha 300 $RP --kernel-trace --stats -d gpurun_out/prof_patha -o run -- python3 tools/path_a_timing.py Humanoid 4096 100 ;;
  train)
    for T in ${TASKS:-Humanoid}; do run train_${T}_$TAG 600 python -u tools/bench_train.py --task $T; done ;;
  curve)
    for T in ${TASKS:-Ant Humanoid}; do run curve_${T}_$TAG 900 python -u tools/train_curve.py --task $T ${CARGS:-}; done ;;
  sizes)
    run sizes_${TASK}_$TAG 300 python -u tools/bw_sweep.py $TASK ${NS// /,} ;;
  ab)   # A/B of the default library against LIB_B (another build of libmi_sim.so) or, with
        # ENV_B="VAR=value ...", against the default library under those variables; alternating
    for k in 1 2 3; do
      run ab_a_${TASK}_${TAG}_$k 200 python -u bench.py --task $TASK --steps 300 --warmup 30 --no-cpu-baseline --no-side --fuse-envs 0 ${BARGS:-}
      run ab_b_${TASK}_${TAG}_$k 200 env ${ENV_B:-MI_SIM_LIB=$LIB_B} python -u bench.py --task $TASK --steps 300 --warmup 30 --no-cpu-baseline --no-side --fuse-envs 0 ${BARGS:-}
    done
    for f in gpurun_out/ab_[ab]_${TASK}_${TAG}_*.log; do echo "$f $(grep -o '"kernel_ms": [0-9.]*\|"ms_per_step": [0-9.]*\|"lds_bytes_per_env": [0-9]*' $f | head -3 | tr '\n' ' ')"; done ;;
  abn)  # the default library and each of LIBS (space-separated paths to other builds), alternating
    for k in 1 2 3; do
      run abn_0_${TASK}_${TAG}_$k 200 python -u bench.py --task $TASK --steps 300 --warmup 30 --no-cpu-baseline --no-side --fuse-envs 0 ${BARGS:-}
      j=1
      for L in $LIBS; do
        run abn_${j}_${TASK}_${TAG}_$k 200 env MI_SIM_LIB=$L python -u bench.py --task $TASK --steps 300 --warmup 30 --no-cpu-baseline --no-side --fuse-envs 0 ${BARGS:-}
        j=$((j + 1))
      done
    done
    for f in gpurun_out/abn_*_${TASK}_${TAG}_*.log; do echo "$f $(grep -o '"kernel_ms": [0-9.]*' $f | head -1)"; done ;;
  *)
    echo "unknown recipe $1"; exit 2 ;;
  esac
}

for r in "$@"; do recipe "$r"; done
echo ALL_DONE
