#!/bin/bash
# HBM write / read bytes per segment of the path kernel and of k_accum, per libart build and scene (one rocprofv3 --pmc
# pass per counter, nothing else traced).  LIBS="libart.so libart_x.so" SCENES="1 8" SPP=64 bash tools/write_traffic.sh
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
SPP=${SPP:-64}
for lib in ${LIBS:-libart.so}; do
  for sc in ${SCENES:-1 8}; do
    for ctr in WRITE_SIZE FETCH_SIZE; do
      d=gpurun_out/wt_${lib}_${sc}_${ctr}
      ART_LIB=$PWD/another_raytracer_amd/$lib timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $d -o run -- python bench.py \
        --steps 1 --warmup 0 --no-cpu-baseline --no-parity --no-profile --spp $SPP --scene $sc > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
    done
    python - "$lib" "$sc" <<'PY'
import csv, glob, json, re, sys
lib, sc = sys.argv[1], sys.argv[2]
out = {"lib": lib, "scene": sc}
segs = None
for ctr in ("WRITE_SIZE", "FETCH_SIZE"):
    d = f"gpurun_out/wt_{lib}_{sc}_{ctr}"
    line = [l for l in open(d + ".log") if l.startswith("{")][-1]
    segs = json.loads(line)["config"]["segments_per_step"]
    tot = {}
    for p in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            k = re.sub(r"\(.*", "", r["Kernel_Name"])
            tot[k] = tot.get(k, 0.0) + float(r["Counter_Value"])
    for k, v in tot.items():
        if "k_paths" in k or "k_accum" in k:
            # WRITE_SIZE x 1024 = bytes written; reads = 2 x FETCH_SIZE x 1024 (MI355X_MICROARCH.md "HBM", gfx950)
            b = v * 1024 * (2 if ctr == "FETCH_SIZE" else 1)
            out[("write" if ctr == "WRITE_SIZE" else "read") + "_B_per_segment." + k.split("::")[-1].split("<")[0]] = round(b / segs, 3)
out["segments"] = segs
print(json.dumps(out))
PY
  done
done
