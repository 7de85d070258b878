#!/bin/bash
# PMC passes over a short bench run (one counter group per rocprofv3 invocation; no tracing domains combined with
# --pmc).  Usage (on the GPU box): TAG=r1 SPP=64 [BENCH_EXTRA='--option NAME=V'] bash tools/pmc.sh
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
TAG=${TAG:-r1}; SPP=${SPP:-64}; SCENE=${SCENE:-1}; PREC=${PREC:-f64}
ARGS="--steps 1 --warmup 0 --no-cpu-baseline --no-parity --no-profile --spp $SPP --scene $SCENE --precision $PREC $BENCH_EXTRA"
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; echo "== rc=$rc : $*"; if [ $rc -ne 0 ]; then exit $rc; fi; }
mkdir -p gpurun_out
rocprofv3 -L > gpurun_out/pmc_list_$TAG.txt 2>&1 || true
DEFAULT_GROUPS=("FETCH_SIZE" "WRITE_SIZE"
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
  "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT"
  "TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE")
if [ -n "$PMC_GROUPS" ]; then IFS=';' read -ra GROUPS_ARR <<< "$PMC_GROUPS"; else GROUPS_ARR=("${DEFAULT_GROUPS[@]}"); fi
i=0
for group in "${GROUPS_ARR[@]}"; do
  i=$((i+1))
  run ${STEP_TIMEOUT:-180} rocprofv3 --pmc $group --output-format csv -d gpurun_out/pmc_${TAG}/g$i -o run -- python bench.py $ARGS > gpurun_out/pmc_${TAG}_g$i.log 2>&1
done
run ${STEP_TIMEOUT:-180} rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc_${TAG}/trace -o run -- python bench.py $ARGS > gpurun_out/pmc_${TAG}_trace.log 2>&1
echo done
