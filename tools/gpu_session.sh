#!/bin/bash
# One GPU-box session made of steps, each under its own time limit, stopping at the first failure:
#   tests                       pytest -m gpu (tests/, one process)
#   testk:EXPR                  pytest -m gpu -k EXPR (a subset first, under a shorter limit)
#   calib                       tools/valu_calib (VALU issue-cost calibration, plain run)
#   logcheck                    tools/log_check (device logs vs glibc over all 2^24 draws) -> gpurun_out/log_check.json
#   uvcheck                     tools/uv_check (device sphere_uv vs host bits and glibc texel choice) -> gpurun_out/uv_check.json
#   ab:LIB1,LIB2[:ARGS]         tools/ab_quick.sh over in-tree libart builds (bench.py ARGS, default --spp 256)
#   abenv:ARGS:V1+V2+...        tools/ab_env.sh over LIB[@VAR=VAL,...] variants (bench.py ARGS)
#   abopt:ARGS:V1+V2+...        tools/ab_opts.sh over option variants of the current build ("base" or NAME=VALUE,...)
#   pmc:TAG:SCENE[:SPP[:OPTS]]  tools/pmc.sh counter passes + kernel trace of the current libart (ART_LIB honoured);
#                               OPTS: library options NAME=V,NAME=V (bench.py --option)
#   bench:TAG[:ARGS]            bench.py line -> gpurun_out/bench_TAG.log
#   prof:TAG[:ARGS]             rocprofv3 --kernel-trace --stats of a bench run -> gpurun_out/prof_TAG
#   configs:TAG                 tools/configs.sh (one bench line per BASELINE GPU config, plus the capsule)
#   defaultrun:TAG[:CPURUNS]    tools/default_run.py: the reference's default run (capsule, adaptive, 720x540x100) on the GPU and
#                               the reference itself on the host CPU (CPURUNS pinned 4-thread runs, default 9)
#   c5full:TAG                  C5 as configured on one GPU: dino 4096^2 x 8192 spp, one timed step after a warm-up
#   stats:TAG                   tools/stats_configs.sh over the four GPU configs (libart_stats.so: divergence counters
#                               and the per-phase cycle split) -> gpurun_out/stats_TAG.txt
# Usage (GPU box): bash tools/gpu_session.sh tests ab:libart_x.so,libart.so pmc:r2b:1
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; echo "== rc=$rc : $*"; [ $rc -eq 0 ] || exit $rc; }
PMC_ALL="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE;\
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC;\
SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT;\
SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_THREAD_CYCLES_VALU SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL GRBM_GUI_ACTIVE;\
TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE;FETCH_SIZE;WRITE_SIZE"
for step in "$@"; do
  IFS=':' read -r kind a b c <<< "$step"
  case "$kind" in
    tests)
      run 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
      tail -1 gpurun_out/gpu_tests.log ;;
    testk)
      run 200 python -u -m pytest tests -m gpu -x -v --timeout 60 --timeout-method thread -k "$a" > gpurun_out/gpu_testk.log 2>&1
      tail -1 gpurun_out/gpu_testk.log ;;
    calib)
      run 120 ./tools/valu_calib > gpurun_out/valu_calib.jsonl 2>&1
      cat gpurun_out/valu_calib.jsonl ;;
    logcheck)
      run 200 ./tools/log_check gpurun_out/log_exceptions.txt > gpurun_out/log_check.json 2>&1
      cat gpurun_out/log_check.json ;;
    uvcheck)
      run 300 ./tools/uv_check > gpurun_out/uv_check.json 2>&1
      cat gpurun_out/uv_check.json ;;
    ab)
      LIBS="${a//,/ }" ARGS="${b:---spp 256}" bash tools/ab_quick.sh || exit 1 ;;
    abenv)
      ARGS="$a" bash tools/ab_env.sh ${b//+/ } || exit 1 ;;
    abopt)
      ARGS="$a" bash tools/ab_opts.sh ${b//+/ } || exit 1 ;;
    pmc)
      IFS=':' read -r _k _a _b _c opts <<< "$step"
      spp=${c:-64}; spp=${spp%%:*}
      extra=""; for o in ${opts//,/ }; do extra="$extra --option $o"; done
      PMC_GROUPS="$PMC_ALL" TAG=$a SCENE=$b SPP=$spp BENCH_EXTRA="$extra" bash tools/pmc.sh || exit 1
      SEGS=$(grep -o '"segments_per_step": [0-9]*' gpurun_out/pmc_${a}_trace.log | grep -o '[0-9]*$')
      VAR=4; [ "$b" = "1" ] && VAR=3
      python tools/pmc_summary.py $a $b f64 $SEGS $VAR > gpurun_out/pmc_summary_$a.txt || exit 1
      cp profiles/${a}_pmc_scene${b}_f64.json gpurun_out/ && cat gpurun_out/pmc_summary_$a.txt ;;
    bench)
      run 600 python bench.py $b > gpurun_out/bench_$a.log 2>&1
      tail -1 gpurun_out/bench_$a.log ;;
    prof)
      run 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$a -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline $b > gpurun_out/rocprof_$a.log 2>&1
      tail -1 gpurun_out/rocprof_$a.log ;;
    configs)
      TAG=$a bash tools/configs.sh || exit 1 ;;
    defaultrun)
      run 900 python -u tools/default_run.py --cpu-runs ${b:-9} --json gpurun_out/default_run_$a.jsonl > gpurun_out/default_run_$a.log 2>&1
      tail -3 gpurun_out/default_run_$a.log ;;
    c5full)
      run 300 python bench.py --scene dino --width 4096 --height 4096 --spp 8192 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/c5full_$a.log 2>&1
      grep "^{" gpurun_out/c5full_$a.log | tail -1 > gpurun_out/c5full_$a.json; cut -c1-400 gpurun_out/c5full_$a.json ;;
    stats)
      CFGS="--scene 1 --spp 64|--scene cow --spp 64|--scene 8 --spp 64|--scene dino --width 4096 --height 4096 --spp 16" bash tools/stats_configs.sh \
        > gpurun_out/stats_$a.txt 2>&1 || exit 1
      cat gpurun_out/stats_$a.txt ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo SESSION OK
