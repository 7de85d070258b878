#!/bin/bash
# r3s: XOR near/far node addressing and the explicit-LDS node path for LM 1: parity suite, then A/B against r3q
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
bash tools/gpu_session.sh tests || exit 1
V="libart.so+libart_r3q.so"
bash tools/gpu_session.sh "abenv:--scene cow --spp 128:$V" "abenv:--scene 8 --spp 256:$V" "abenv:--scene dino --width 4096 --height 4096 --spp 32:$V" || exit 1
echo S10 OK
