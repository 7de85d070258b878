#!/bin/bash
# VALU issue-cost calibration on the GPU box (tools/valu_calib.hip): one plain run (in-kernel cycles per
# wave-instruction per SIMD at 1 and 4 waves per SIMD) and one rocprofv3 --pmc pass per counter group, so the SQ
# counters' units are read off a known instruction stream.  Usage (GPU box): TAG=r2a bash tools/gpu_calib.sh
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
TAG=${TAG:-r2}
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; echo "== rc=$rc : $*"; [ $rc -eq 0 ] || exit $rc; }
mkdir -p gpurun_out
run 60 ./tools/valu_calib > gpurun_out/valu_calib_$TAG.jsonl 2>&1
cat gpurun_out/valu_calib_$TAG.jsonl
GROUPS_ARR=("SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_FMA_F64 GRBM_GUI_ACTIVE"
  "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_WAIT_INST_ANY")
i=0
for group in "${GROUPS_ARR[@]}"; do
  i=$((i+1))
  run 60 rocprofv3 --pmc $group --output-format csv -d gpurun_out/calib_${TAG}/g$i -o run -- ./tools/valu_calib > gpurun_out/calib_${TAG}_g$i.log 2>&1
done
echo calib done
