#!/bin/bash
# r3p: packed 16-bit-code keys (F_CODE16) and byte-addressed stacks in k_paths_g: parity suite on the default build,
# then A/B against the stack-only and the r3o builds on the general-scene configs
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
bash tools/gpu_session.sh tests || exit 1
V="libart.so+libart_noc16.so+libart_base.so"
bash tools/gpu_session.sh "abenv:--scene cow --spp 128:$V" "abenv:--scene 8 --spp 256:$V" "abenv:--scene dino --width 4096 --height 4096 --spp 32:$V" || exit 1
echo S7 OK
