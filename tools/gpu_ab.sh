#!/bin/bash
# GPU tests (all of -m gpu), then the bench A/B over the libart builds in $LIBS (2 rounds each).
#   LIBS="libart.so libart_x.so" ARGS="--spp 256" bash tools/gpu_ab.sh
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -z "$NOTESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${TESTK:+-k "$TESTK"} > gpurun_out/gpu_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
fi
for round in 1 2; do
for lib in $LIBS; do
  timeout -k 10 300 env ART_LIB=$PWD/another_raytracer_amd/$lib python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity $ARGS > gpurun_out/ab_${lib}_$round.log 2>&1
  rc=$?; echo "$lib round $round rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/ab_${lib}_$round.log | head -1) $(grep -o '"extend_ms_total": [0-9.]*' gpurun_out/ab_${lib}_$round.log) $(grep -o "\"extend_variant\": [0-9]*" gpurun_out/ab_${lib}_$round.log) $(grep -o "\"segments_per_step\": [0-9]*" gpurun_out/ab_${lib}_$round.log)"
  [ $rc -eq 0 ] || { tail -5 gpurun_out/ab_${lib}_$round.log; exit $rc; }
done
done
