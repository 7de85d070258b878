"""Summarise tools/pmc.sh output into profiles/<tag>_pmc_<scene>_<prec>.json (per-kernel counter totals, and per-
segment HBM bytes of k_extend for bench.py's roofline `traffic`).

gfx950 corrections (MI355X_MICROARCH.md "HBM"): FETCH_SIZE (KB) counts 64 B per TCC_EA0_RDREQ and reads exactly half
of a wide coalesced stream, so HBM read bytes = 2 x FETCH_SIZE x 1024 (an upper estimate for narrower accesses);
WRITE_SIZE x 1024 = bytes written."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d):
    out = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(set)
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"]
            out[k][r["Counter_Name"]] += float(r["Counter_Value"])
            calls[k].add(r["Dispatch_Id"])
    return out, {k: len(v) for k, v in calls.items()}


def main(tag, scene, prec, segments_per_step, variant=2, root="gpurun_out"):
    base = os.path.join(root, f"pmc_{tag}")
    agg = defaultdict(dict)
    ncalls = {}
    for g in sorted(glob.glob(os.path.join(base, "g*"))):
        c, n = load(g)
        for k, v in c.items():
            agg[k].update(v)
            ncalls[k] = max(ncalls.get(k, 0), n.get(k, 0))
    kernels = {}
    for k, v in agg.items():
        short = k.split("(")[0].replace("void ", "")
        e = dict(v)
        e["dispatches"] = ncalls.get(k, 0)
        if "FETCH_SIZE" in v:
            e["hbm_read_bytes_corrected"] = 2 * v["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in v:
            e["hbm_write_bytes"] = v["WRITE_SIZE"] * 1024
        if "SQ_INSTS_VALU" in v and "SQ_WAVES" in v and v["SQ_WAVES"]:
            e["valu_insts_per_wave"] = v["SQ_INSTS_VALU"] / v["SQ_WAVES"]
        if "SQ_INSTS_VALU" in v and v.get("GRBM_GUI_ACTIVE"):
            # VALU issue share: 4 cycles per wave64 instruction over 1024 SIMDs x per-XCD busy cycles (GRBM_GUI_ACTIVE
            # is summed over the 8 XCDs); transcendentals take longer, so this is a lower estimate
            e["valu_busy"] = v["SQ_INSTS_VALU"] * 4 / (1024 * v["GRBM_GUI_ACTIVE"] / 8)
        kernels[short] = e
    ext = {k: v for k, v in kernels.items() if k.startswith("art::k_extend") or k.startswith("art::k_paths")}
    total = lambda key: sum(v.get(key, 0) for v in ext.values())
    res = {"tag": tag, "scene": scene, "precision": prec, "segments": segments_per_step, "extend_variant": variant,
           "kernels": kernels,
           "note": "hbm_read_bytes_corrected = 2*FETCH_SIZE*1024 (gfx950 half-count correction), hbm_write_bytes = WRITE_SIZE*1024"}
    busy = [v["valu_busy"] for v in ext.values() if "valu_busy" in v]
    if busy:
        res["valu_busy"] = round(max(busy), 4)
    if segments_per_step and ext:
        res["extend_bytes_per_segment"] = (total("hbm_read_bytes_corrected") + total("hbm_write_bytes")) / segments_per_step
        res["extend_read_bytes_per_segment"] = total("hbm_read_bytes_corrected") / segments_per_step
        res["extend_write_bytes_per_segment"] = total("hbm_write_bytes") / segments_per_step
    os.makedirs("profiles", exist_ok=True)
    out = os.path.join("profiles", f"{tag}_pmc_scene{scene}_{prec}.json")
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    print(out)
    for k, v in sorted(kernels.items()):
        print(k, {kk: round(vv, 3) if isinstance(vv, float) else vv for kk, vv in v.items()})


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]), int(sys.argv[5]) if len(sys.argv) > 5 else 2)
