#!/bin/bash
# Throughput of every BASELINE.json GPU config on one GPU (one step each): C2 random spheres, C3 cow, C4 Next-Week
# final, C5 dino at 4096^2 (spp reduced to 512: per-segment cost does not depend on spp; C5 as configured, 8192 spp, is
# the c5full step of tools/gpu_session.sh and the 8-GPU round-end run), plus the capsule (scene 9, the reference's
# default scene: main.cpp:20) at 512 spp.  Output: gpurun_out/configs_<TAG>.jsonl
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
TAG=${TAG:-r1}
mkdir -p gpurun_out
out=gpurun_out/configs_$TAG.jsonl
: > $out
for cfg in "--scene 1 --spp 1024" "--scene cow --spp 512" "--scene 8 --spp 4096" "--scene dino --width 4096 --height 4096 --spp 512" "--scene 9 --spp 512"; do
  timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline $cfg > gpurun_out/cfg.log 2>&1
  rc=$?; echo "rc=$rc $cfg"
  [ $rc -eq 0 ] || { tail -5 gpurun_out/cfg.log; exit $rc; }
  tail -1 gpurun_out/cfg.log >> $out
done
python - <<'PY'
import json, os
for l in open(os.environ.get("OUT", "gpurun_out/configs_" + os.environ.get("TAG", "r1") + ".jsonl")):
    d = json.loads(l); c = d["config"]
    print(c["workload"], c["width"], c["height"], c["spp"], "->", d["value"], "Msamples/s", d["ms_per_step"], "ms/frame",
          "variant", d.get("roofline", {}).get("extend_variant"))
PY
