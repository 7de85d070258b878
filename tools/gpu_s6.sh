#!/bin/bash
# r3o evidence for the benched build: build-stamped PMC summaries of k_paths (scene 1) and k_paths_g (cow, Next-Week
# final, dino), the four GPU configs, then the bench line (which reads the scene-1 summary of the same build)
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
bash tools/gpu_session.sh pmc:r3o:1 pmc:r3o:cow pmc:r3o:8 pmc:r3o:dino:16 configs:r3o bench:r3o || exit 1
echo S6 OK
