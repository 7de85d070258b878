#!/bin/bash
# r1q evidence: divergence stats, PMC passes (k_paths), official bench line, kernel trace of the same bench command.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 env ART_LIB=$PWD/another_raytracer_amd/libart_stats.so python bench.py --spp 16 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/stats_r1q.log 2>&1 || exit 1
grep ART_STATS gpurun_out/stats_r1q.log
TAG=r1q SPP=64 bash tools/pmc.sh || exit 1
timeout -k 10 600 python bench.py > gpurun_out/bench_r1q.log 2>&1 || exit 1
tail -1 gpurun_out/bench_r1q.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r1q -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/rocprof_r1q.log 2>&1 || exit 1
tail -1 gpurun_out/rocprof_r1q.log
echo all done
