#!/bin/bash
# r1p: A/B (packed LDS keys vs HEAD) + GPU tests, divergence stats, PMC passes, official bench line, kernel trace.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
LIBS="libart.so libart_spec.so" bash tools/gpu_ab.sh || exit $?
timeout -k 10 200 env ART_LIB=$PWD/another_raytracer_amd/libart_stats.so python bench.py --spp 16 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/stats_r1p.log 2>&1 || exit 1
grep ART_STATS gpurun_out/stats_r1p.log
TAG=r1p SPP=64 bash tools/pmc.sh || exit 1
timeout -k 10 600 python bench.py > gpurun_out/bench_r1p.log 2>&1 || exit 1
tail -1 gpurun_out/bench_r1p.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r1p -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/rocprof_r1p.log 2>&1 || exit 1
echo all done
