#!/bin/bash
# r3u evidence for the benched build: GPU suite, build-stamped PMC summaries of k_paths (scene 1) and k_paths_g (cow,
# Next-Week final, dino), the four GPU configs, the bench line (reads the scene-1 summary of the same build), a
# rocprofv3 kernel trace of the bench, and C5 as configured on one GPU (dino 4096^2 x 8192 spp, one job)
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
bash tools/gpu_session.sh tests pmc:r3u:1 pmc:r3u:cow pmc:r3u:8 pmc:r3u:dino:16 configs:r3u bench:r3u prof:r3u || exit 1
timeout -k 10 300 python bench.py --scene dino --width 4096 --height 4096 --spp 8192 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/c5_r3u.log 2>&1 || exit 1
tail -1 gpurun_out/c5_r3u.log
echo S12 OK
