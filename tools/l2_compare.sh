#!/bin/bash
# L2 miss / HBM fetch of the dominant kernel for several builds on one box: one rocprofv3 --pmc pass each.
# Usage: bash tools/l2_compare.sh "DIR:LIB" ... (DIR holds bench.py; LIB is relative to DIR/another_raytracer_amd)
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
ROOT=$PWD
ARGS=${ARGS:-"--steps 1 --warmup 0 --no-cpu-baseline --spp 64 --scene cow"}
i=0
for spec in "$@"; do
  i=$((i+1)); dir=${spec%%:*}; lib=${spec#*:}
  (cd $ROOT/$dir && ART_LIB=$ROOT/$dir/another_raytracer_amd/$lib timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TCC_MISS_sum --output-format csv -d $ROOT/gpurun_out/l2c/$i -o run -- \
     python bench.py $ARGS > $ROOT/gpurun_out/l2c_$i.log 2>&1) || { echo "fail $spec"; tail -5 gpurun_out/l2c_$i.log; exit 1; }
  echo "$spec: $(python3 - $ROOT/gpurun_out/l2c/$i <<'PY'
import csv, glob, sys
out = {}
for f in glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'paths' in r['Kernel_Name']:
            out[r['Counter_Name']] = out.get(r['Counter_Name'], 0) + float(r['Counter_Value'])
print(out)
PY
)"
done
