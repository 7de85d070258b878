#!/bin/bash
# One evidence session on the GPU box, stopping at the first fault/timeout:
#   parity tests -> traversal statistics (libart_stats.so, if built) -> PMC passes (tools/pmc.sh) -> official bench
#   line -> rocprofv3 kernel trace of the bench.  Usage: TAG=r1r bash tools/gpu_round.sh
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
TAG=${TAG:-r1}
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; echo "== rc=$rc : $*"; [ $rc -eq 0 ] || exit $rc; }
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  run 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
  tail -1 gpurun_out/gpu_tests_$TAG.log
fi
if [ -f another_raytracer_amd/libart_stats.so ]; then
  run 200 env ART_LIB=$PWD/another_raytracer_amd/libart_stats.so python bench.py --spp 16 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/stats_$TAG.log 2>&1
  grep ART_STATS gpurun_out/stats_$TAG.log
fi
if [ -z "$SKIP_PMC" ]; then
  TAG=$TAG SPP=64 bash tools/pmc.sh || exit 1
  SEGS=$(grep -o '"segments_per_step": [0-9]*' gpurun_out/pmc_${TAG}_trace.log | grep -o '[0-9]*$')
  VAR=$(grep -o '"extend_variant": [0-9]*' gpurun_out/pmc_${TAG}_trace.log | grep -o '[0-9]*$'); VAR=${VAR:-3}  # --no-profile runs print no variant: the persistent-path kernel
  # the summary lands in profiles/ here (so the bench below prices `traffic` with it) and in gpurun_out/ (to commit)
  python tools/pmc_summary.py $TAG 1 f64 $SEGS $VAR > gpurun_out/pmc_summary_$TAG.txt && cp profiles/${TAG}_pmc_scene1_f64.json gpurun_out/ || exit 1
fi
run 600 python bench.py $BENCH_ARGS > gpurun_out/bench_$TAG.log 2>&1
tail -1 gpurun_out/bench_$TAG.log
run 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline $BENCH_ARGS > gpurun_out/rocprof_$TAG.log 2>&1
tail -1 gpurun_out/rocprof_$TAG.log
echo all done
