#!/bin/bash
# r3w: A/B of the per-traversal |d|^2 reciprocal for leaf spheres in triangle-free k_paths_g kernels (ART_SPH_PRE_G),
# with the GPU parity suite run on that build (ART_LIB)
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
ART_LIB=$PWD/another_raytracer_amd/libart_sph.so bash tools/gpu_session.sh tests || exit 1
bash tools/gpu_session.sh "abenv:--scene 8 --spp 256:libart.so+libart_sph.so" "abenv:--scene 7 --spp 256:libart.so+libart_sph.so" || exit 1
echo S14 OK
