cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
bash tools/gpu_session.sh "abenv:--scene 1 --spp 256:libart.so+libart_sortp.so+libart_ring96.so+libart.so" || exit 1
for v in libart.so:r3l_base libart_ring96.so:r3l_ring96; do
  lib=${v%%:*}; tag=${v##*:}
  ART_LIB=$PWD/another_raytracer_amd/$lib PMC_GROUPS="FETCH_SIZE;WRITE_SIZE" TAG=$tag SCENE=1 SPP=64 bash tools/pmc.sh || exit 1
done
echo S3 OK
