export TMPDIR=/tmp
for cfg in "--scene cow --spp 64" "--scene 8 --spp 64" "--scene dino --width 4096 --height 4096 --spp 16"; do
  timeout -k 10 200 env ART_LIB=$PWD/another_raytracer_amd/libart_stats.so python bench.py --steps 1 --warmup 0 --no-cpu-baseline $cfg > gpurun_out/stats.log 2>&1 || exit 1
  echo "$cfg"; grep ART_STATS gpurun_out/stats.log | head -2
done
