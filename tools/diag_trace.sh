#!/bin/bash
# Find where GPU and oracle part ways on a scene's sampled rows and trace the first diverging paths on both sides
# (GPU box).  Usage: bash tools/diag_trace.sh SCENE W H SPP STRIDE [NPIX]   -> gpurun_out/diag_SCENE.jsonl,
# gpurun_out/trace_SCENE_<pixel>_<sample>_{gpu,oracle}.txt
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
SC=$1; W=$2; H=$3; SPP=$4; STRIDE=$5; NPIX=${6:-2}
mkdir -p gpurun_out
timeout -k 10 600 python tools/diag_rows.py $SC $W $H $SPP $STRIDE $NPIX > gpurun_out/diag_$SC.jsonl || exit 1
cat gpurun_out/diag_$SC.jsonl
python - "$SC" "$W" > /tmp/diag_pairs.txt <<'PY'
import json, sys
for ln in open(f"gpurun_out/diag_{sys.argv[1]}.jsonl"):
    d = json.loads(ln)
    if "pixel" in d:
        y, x = d["pixel"]
        print(y * int(sys.argv[2]) + x, d["first_diverging_sample"])
PY
while read -r pix smp; do
  timeout -k 10 120 env ART_LIB=$PWD/another_raytracer_amd/libart_trace.so python tools/trace_path.py gpu $SC $W $H $pix $smp > gpurun_out/trace_${SC}_${pix}_${smp}_gpu.txt 2>&1 || exit 1
  timeout -k 10 120 python tools/trace_path.py oracle $SC $W $H $pix $smp > gpurun_out/trace_${SC}_${pix}_${smp}_oracle.txt 2>&1 || exit 1
  echo "== pixel $pix sample $smp"
  diff <(grep TRACE gpurun_out/trace_${SC}_${pix}_${smp}_gpu.txt | sed 's/ prim=.*//') <(grep TRACE gpurun_out/trace_${SC}_${pix}_${smp}_oracle.txt) | head -8
done < /tmp/diag_pairs.txt
echo diag done
