#!/bin/bash
# r3v: leaf triangles from TriRec112 records (plane precomputed) in the LM 1 kernels: GPU suite, then A/B vs r3t
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
bash tools/gpu_session.sh tests || exit 1
bash tools/gpu_session.sh "abenv:--scene dino --width 4096 --height 4096 --spp 32:libart.so+libart_r3t.so" "abenv:--scene cow --spp 128:libart.so+libart_r3t.so" || exit 1
echo S13 OK
