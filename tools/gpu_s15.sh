#!/bin/bash
# r3x: A/B of 112-B LDS nodes in cow's LM 2 kernel (ART_LM2_COMPACT), with the GPU parity suite on that build
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
ART_LIB=$PWD/another_raytracer_amd/libart_cmp.so bash tools/gpu_session.sh tests || exit 1
bash tools/gpu_session.sh "abenv:--scene cow --spp 128:libart.so+libart_cmp.so" || exit 1
echo S15 OK
