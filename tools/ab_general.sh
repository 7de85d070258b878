cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for cfg in "--scene cow --spp 512" "--scene 8 --spp 1024" "--scene dino --width 4096 --height 4096 --spp 128"; do
 for wf in "" "--wavefront"; do
  timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline $cfg $wf > gpurun_out/cfg.log 2>&1 || { tail -5 gpurun_out/cfg.log; exit 1; }
  echo "$cfg $wf: $(grep -o '"value": [0-9.]*' gpurun_out/cfg.log) $(grep -o '"extend_variant": [0-9]*' gpurun_out/cfg.log)"
 done
done
