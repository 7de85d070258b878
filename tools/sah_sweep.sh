#!/bin/bash
# BVH builder sweep: traversal statistics (stats build, spp 16) and full-frame throughput per (options bvh.sah_ci, bvh.sah_leaf).
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in ${CFGS:-"1.5:4" "0.75:4" "3:4" "1.5:2" "1.5:8" "3:8"}; do
  ci=${cfg%%:*}; leaf=${cfg##*:}
  timeout -k 10 120 env ART_LIB=$PWD/another_raytracer_amd/libart_stats.so python bench.py --option bvh.sah_ci=$ci --option bvh.sah_leaf=$leaf --spp 16 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/sah_stats_${ci}_${leaf}.log 2>&1 || exit 1
  echo "ci=$ci leaf=$leaf $(grep 'ART_STATS node' gpurun_out/sah_stats_${ci}_${leaf}.log | head -1 | sed 's/.*traversals/traversals/')"
  timeout -k 10 200 python bench.py --option bvh.sah_ci=$ci --option bvh.sah_leaf=$leaf --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/sah_bench_${ci}_${leaf}.log 2>&1 || exit 1
  echo "   value $(grep -o '"value": [0-9.]*' gpurun_out/sah_bench_${ci}_${leaf}.log)"
done
