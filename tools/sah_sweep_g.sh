#!/bin/bash
# BVH builder sweep over the general-scene configs: full-frame throughput per (options bvh.sah_ci, bvh.sah_leaf).
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in ${CFGS:-"1.5:4" "3:4" "0.75:4" "1.5:2" "1.5:8" "3:8"}; do
  ci=${cfg%%:*}; leaf=${cfg##*:}
  line="ci=$ci leaf=$leaf"
  for sc in "--scene cow --spp 256" "--scene 8 --spp 256" "--scene dino --width 4096 --height 4096 --spp 64" "--scene 9 --spp 128"; do
    timeout -k 10 120 python bench.py --option bvh.sah_ci=$ci --option bvh.sah_leaf=$leaf --steps 1 --warmup 1 --no-cpu-baseline $sc > gpurun_out/sahg.log 2>&1 || { tail -3 gpurun_out/sahg.log; exit 1; }
    line="$line | $(echo $sc | cut -d' ' -f2): $(grep -o '"value": [0-9.]*' gpurun_out/sahg.log | cut -d' ' -f2)"
  done
  echo "$line"
done
