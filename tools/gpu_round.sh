#!/bin/bash
# One GPU session: parity tests, full bench, rocprofv3 kernel trace.  Stops at the first fault/timeout.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
TAG=${TAG:-r1}
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; echo "== rc=$rc : $*"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
run 900 python -m pytest tests -q -m gpu -s > gpurun_out/gpu_tests_$TAG.log 2>&1
fi
run 600 python bench.py $BENCH_ARGS > gpurun_out/bench_$TAG.log 2>&1
run 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline $BENCH_ARGS > gpurun_out/rocprof_$TAG.log 2>&1
echo done
