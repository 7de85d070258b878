#!/bin/bash
# Quick bench A/B over the libart builds in $LIBS (one short run each, 2 rounds), each run under its own time limit,
# stopping at the first failure.  LIBS="libart.so libart_x.so" ARGS="--spp 256" bash tools/ab_quick.sh
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
for round in 1 2; do
  for lib in $LIBS; do
    timeout -k 10 90 env ART_LIB=$PWD/another_raytracer_amd/$lib python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity $ARGS > gpurun_out/abq_${lib}_$round.log 2>&1
    rc=$?
    echo "$lib round $round rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/abq_${lib}_$round.log | head -1)"
    [ $rc -eq 0 ] || exit $rc
  done
done
