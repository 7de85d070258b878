#!/bin/bash
# r3t: A/B of the per-traversal near-plane offsets in dino's LM 1 kernel (ART_NF_HOIST) and of cow's suspend threshold
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
bash tools/gpu_session.sh "abenv:--scene dino --width 4096 --height 4096 --spp 32:libart.so+libart_nfh.so" "abenv:--scene cow --spp 128:libart.so+libart_s16.so+libart_s32.so" || exit 1
echo S11 OK
