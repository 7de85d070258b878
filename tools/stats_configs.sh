#!/bin/bash
# Traversal statistics and the per-phase cycle split of the path kernels (libart_stats.so: SPLIT=0 EXTRA=-DART_STATS)
# over the general-scene configs.  Usage (GPU box): bash tools/stats_configs.sh
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
CFGS=${CFGS:-"--scene cow --spp 64|--scene 8 --spp 64|--scene dino --width 4096 --height 4096 --spp 16|--scene 7 --spp 64|--scene 9 --spp 64"}
IFS='|' read -ra CFG_ARR <<< "$CFGS"
for cfg in "${CFG_ARR[@]}"; do
  timeout -k 10 200 env ART_LIB=$PWD/another_raytracer_amd/libart_stats.so python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-parity $cfg > gpurun_out/stats.log 2>&1 || exit 1
  echo "$cfg"; grep ART_STATS gpurun_out/stats.log | head -8
done
