#!/bin/bash
# A/B the bench across libart builds: LIBS="a.so b.so" ARGS="--spp 256" bash tools/ab_libs.sh
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
for round in 1 2; do
for lib in $LIBS; do
  timeout -k 10 300 env ART_LIB=$PWD/another_raytracer_amd/$lib python bench.py --steps 2 --warmup 1 --no-cpu-baseline $ARGS > gpurun_out/ab_${lib}_$round.log 2>&1
  rc=$?; echo "$lib round $round rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/ab_${lib}_$round.log | head -1) $(grep -o '"extend_ms_total": [0-9.]*' gpurun_out/ab_${lib}_$round.log)"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
done
