#!/bin/bash
# r3n: parity suite on the 96-entry XCD rings, leaf-test type stats of the Next-Week final and cow, bench + rocprof
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
bash tools/gpu_session.sh tests || exit 1
CFGS="--scene 8 --spp 64|--scene cow --spp 64|--scene 1 --spp 64" bash tools/stats_configs.sh > gpurun_out/stats_r3n.txt 2>&1 || exit 1
cat gpurun_out/stats_r3n.txt
bash tools/gpu_session.sh bench:r3n prof:r3n || exit 1
echo S5 OK
