#!/bin/bash
# General-scene A/B: persistent HBM-scene paths (variant 4) over the libart builds in $LIBS, plus the per-depth
# wavefront reference (--wavefront) for the first lib, on cow / Next-Week final / dino configs (one step each;
# CFGS="args|args|..." overrides the configs).
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
LIBS=${LIBS:-libart.so}
CFGS=${CFGS:-"--scene cow --spp 512|--scene 8 --spp 1024|--scene dino --width 4096 --height 4096 --spp 128"}
IFS='|' read -ra CFG_ARR <<< "$CFGS"
for cfg in "${CFG_ARR[@]}"; do
  for lib in $LIBS; do
    timeout -k 10 300 env ART_LIB=$PWD/another_raytracer_amd/$lib python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-parity $cfg > gpurun_out/cfg.log 2>&1 || { tail -5 gpurun_out/cfg.log; exit 1; }
    echo "$lib $cfg: $(grep -o '"value": [0-9.]*' gpurun_out/cfg.log) $(grep -o '"extend_variant": [0-9]*' gpurun_out/cfg.log)"
  done
done
