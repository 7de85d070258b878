#!/bin/bash
# r3r evidence for the benched build: build-stamped PMC summaries of k_paths (scene 1) and k_paths_g (cow, Next-Week
# final, dino), the four GPU configs, then the bench line (which reads the scene-1 summary of the same build)
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
bash tools/gpu_session.sh tests pmc:r3r:1 pmc:r3r:cow pmc:r3r:8 pmc:r3r:dino:16 configs:r3r bench:r3r prof:r3r || exit 1
echo S6 OK
