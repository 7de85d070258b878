#!/bin/bash
# Final r3 evidence for the benched build (tag $1, default r3zf): the same steps as gpu_s12.sh -- GPU suite,
# build-stamped PMC summaries of k_paths (scene 1) and k_paths_g (cow, Next-Week final, dino), the four GPU configs,
# the bench line, a rocprofv3 kernel trace of the bench, and C5 as configured on one GPU (dino 4096^2 x 8192 spp)
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
T=${1:-r3zf}
bash tools/gpu_session.sh tests pmc:$T:1 pmc:$T:cow pmc:$T:8 pmc:$T:dino:16 configs:$T bench:$T prof:$T || exit 1
timeout -k 10 300 python bench.py --scene dino --width 4096 --height 4096 --spp 8192 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/c5_$T.log 2>&1 || exit 1
tail -1 gpurun_out/c5_$T.log
echo S16 OK
