#!/bin/bash
# Bench A/B over library-option variants of one build (rt_option_set via bench.py --option), 2 rounds, each run under
# its own time limit, stopping at the first failure.  Each argument is "base" or NAME=VALUE[,NAME=VALUE...]:
#   ARGS="--scene 9 --spp 256" bash tools/ab_opts.sh base render.leaf2=0 render.leaf2=0,render.tex_bary=0
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
ARGS="${ARGS:---spp 256}"
for round in 1 2; do
  i=0
  for v in "$@"; do
    i=$((i + 1))
    opts=""
    if [ "$v" != "base" ]; then
      for o in ${v//,/ }; do opts="$opts --option $o"; done
    fi
    timeout -k 10 150 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity $ARGS $opts > gpurun_out/abo_${i}_$round.log 2>&1
    rc=$?
    echo "$v round $round rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/abo_${i}_$round.log | head -1) $(grep -o '"extend_variant": [0-9]*' gpurun_out/abo_${i}_$round.log | head -1)"
    [ $rc -eq 0 ] || exit $rc
  done
done
