#!/bin/bash
# Parity subset, then A/B of libart.so vs libart_prev.so (full bench frame), then the stats build.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py -m gpu -x -v --timeout 120 --timeout-method thread -s ${TESTK:+-k "$TESTK"} > gpurun_out/ab_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/ab_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
b() { local tag=$1; shift; timeout -k 10 300 "$@" > gpurun_out/ab_$tag.log 2>&1; local rc=$?; echo "$tag rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/ab_$tag.log | head -1) $(grep -o '"extend_ms_total": [0-9.]*' gpurun_out/ab_$tag.log)"; [ $rc -eq 0 ] || exit $rc; }
for r in 1 2; do
b new_$r python bench.py --steps 2 --warmup 1 --no-cpu-baseline $BARGS
b prev_$r env ART_LIB=$PWD/another_raytracer_amd/libart_prev.so python bench.py --steps 2 --warmup 1 --no-cpu-baseline $BARGS
done
if [ -f another_raytracer_amd/libart_stats.so ]; then
ART_LIB=$PWD/another_raytracer_amd/libart_stats.so timeout -k 10 200 python bench.py --spp 16 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/stats.log 2>&1; echo "stats rc=$?"; grep ART_STATS gpurun_out/stats.log
fi
