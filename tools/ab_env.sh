#!/bin/bash
# Bench A/B over (library, environment) variants, 2 rounds, each run under its own time limit, stopping at the first
# failure.  Each argument is LIB[@VAR=VAL[,VAR=VAL...]]:
#   ARGS="--spp 256" bash tools/ab_env.sh libart.so libart_exp.so@ART_EXP_X=1
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
ARGS="${ARGS:---spp 256}"
for round in 1 2; do
  i=0
  for v in "$@"; do
    i=$((i + 1))
    lib="${v%%@*}"
    envs=""
    [ "$lib" != "$v" ] && envs="${v#*@}"
    timeout -k 10 120 env ART_LIB=$PWD/another_raytracer_amd/$lib ${envs//,/ } python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity $ARGS \
      > gpurun_out/abe_${i}_$round.log 2>&1
    rc=$?
    echo "$v round $round rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/abe_${i}_$round.log | head -1)"
    [ $rc -eq 0 ] || exit $rc
  done
done
