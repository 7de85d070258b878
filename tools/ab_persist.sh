#!/bin/bash
# Parity of the extend variants, then A/B of the persistent-lane kernel (refill thresholds) vs the batch kernel.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -s -k "variants or adaptive or f64_matches" > gpurun_out/ab_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/ab_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
b() { local tag=$1; shift; timeout -k 10 300 "$@" > gpurun_out/ab_$tag.log 2>&1; local rc=$?; echo "$tag rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/ab_$tag.log | head -1) $(grep -o '"extend_ms_total": [0-9.]*' gpurun_out/ab_$tag.log)"; [ $rc -eq 0 ] || exit $rc; }
for r in 1 2; do
b batch_$r python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-persist
b r32_$r python bench.py --steps 2 --warmup 1 --no-cpu-baseline
b r16_$r env ART_LIB=$PWD/another_raytracer_amd/libart_r16.so python bench.py --steps 2 --warmup 1 --no-cpu-baseline
b r48_$r env ART_LIB=$PWD/another_raytracer_amd/libart_r48.so python bench.py --steps 2 --warmup 1 --no-cpu-baseline
done
