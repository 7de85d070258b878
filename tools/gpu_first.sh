#!/bin/bash
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; echo "== rc=$rc : $*"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
rocm-smi --showproductname > gpurun_out/box.txt 2>&1 || true
run 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
run 900 python -m pytest tests/test_gpu_parity.py -q -m gpu -s -x -k "f64_matches and (c1 or 1 or cow)" > gpurun_out/gpu_tests_a.log 2>&1
run 300 python bench.py --spp 64 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench64.log 2>&1
run 300 python bench.py --spp 64 --steps 2 --warmup 1 --no-cpu-baseline --precision f64 > gpurun_out/bench64_f64.log 2>&1
echo done
