#!/bin/bash
# r3m: camera-ray ring layout / size A/B with HBM traffic per variant, and the leaf-test type statistics
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
bash tools/gpu_session.sh "abenv:--scene 1 --spp 256:libart.so+libart_ring96.so+libart_noxcd.so" || exit 1
for v in libart.so:r3m_xcd128 libart_ring96.so:r3m_xcd96 libart_noxcd.so:r3m_blk128; do
  lib=${v%%:*}; tag=${v##*:}
  ART_LIB=$PWD/another_raytracer_amd/$lib PMC_GROUPS="FETCH_SIZE;WRITE_SIZE" TAG=$tag SCENE=1 SPP=64 bash tools/pmc.sh || exit 1
done
bash tools/gpu_session.sh stats:r3m || exit 1
echo S4 OK
