"""Summarise tools/pmc.sh output into profiles/<tag>_pmc_scene<scene>_<prec>.json: per-kernel counter totals plus, for
the path kernels (k_paths / k_paths_g / k_extend), the derived bound analysis and per-segment HBM bytes that bench.py's
roofline reads.

Units, pinned on a known instruction stream (tools/valu_calib.hip; profiles/r2a_valu_calib*.json*):
  * SQ_INSTS_VALU counts wave-instructions; SQ_ACTIVE_INST_VALU counts VALU issue units: 1 per ordinary VALU
    instruction (f32, packed f32, f64 add/mul/fma, integer, conversions), 2 per f32 transcendental (v_rcp_f32,
    v_sqrt_f32), 4 per f64 transcendental (v_rsq_f64); SQ_THREAD_CYCLES_VALU = 64 x ACTIVE_INST_VALU at full EXEC, so
    THREAD_CYCLES_VALU / (64 x ACTIVE_INST_VALU) is the VALU lane utilization.
  * measured issue rate with 4 waves per SIMD (k_paths' occupancy) and 8 independent chains per wave: one unit per
    ~3.0-3.3 shader cycles per SIMD (f32 fma 3.01, packed f32 fma 3.31, f64 fma 3.29, f64 add/mul 3.34, u32 max 3.27);
    trans f32 2x, rsq_f64 4x.  With 8 waves per SIMD the same streams reach ~2.1-2.6 cycles (the pipe's peak is near
    MI355X_MICROARCH.md's 2 cycles per wave64 VALU instruction, also reported), so at 4 waves part of the gap to the
    pipe is latency that more waves would hide.
  * SQ_WAVE_CYCLES / SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY count quad-cycles per wave (they sum to
    WAVE_CYCLES); GRBM_GUI_ACTIVE is summed over the 8 XCDs (cycles = GRBM_GUI_ACTIVE / 8).

gfx950 HBM corrections (MI355X_MICROARCH.md "HBM"): FETCH_SIZE (KB) counts 64 B per TCC_EA0_RDREQ and reads exactly half
of a wide coalesced stream, so HBM read bytes = 2 x FETCH_SIZE x 1024 (an upper estimate for narrower accesses);
WRITE_SIZE x 1024 = bytes written."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

SIMDS = 1024          # 256 CUs x 4
CUS = 256
XCDS = 8
GUIDE_CYC = 2.0       # MI355X_MICROARCH.md: wave64 VALU on SIMD-32, >= 2 waves per SIMD
NORMAL_OPS = ("v_fma_f32", "v_pk_fma_f32", "v_fma_f64", "v_add_f64", "v_mul_f64", "v_max_u32")


def calibrated_cycles(root="profiles", waves=4):
    """Median measured cycles per VALU issue unit at `waves` waves per SIMD over the ordinary ops, from the newest
    tools/valu_calib run committed under profiles/ that has them (None when there is none)."""
    best = None
    for path in sorted(glob.glob(os.path.join(root, "*valu_calib.jsonl"))):
        vals = []
        for ln in open(path):
            try:
                d = json.loads(ln)
            except ValueError:
                continue
            if d.get("op") in NORMAL_OPS and d.get("waves_per_simd") == waves:
                vals.append(d["cycles_per_inst_per_simd"])
        if vals:
            vals.sort()
            best = (vals[len(vals) // 2], os.path.basename(path))
    return best


def load(d):
    out = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(set)
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"]
            out[k][r["Counter_Name"]] += float(r["Counter_Value"])
            calls[k].add(r["Dispatch_Id"])
    return out, {k: len(v) for k, v in calls.items()}


def derive(v, segments, cyc_unit, cyc_unit8=None):
    """Bound analysis of one kernel's counters (see the module docstring for the units)."""
    e = {}
    grbm = v.get("GRBM_GUI_ACTIVE")
    cycles = grbm / XCDS if grbm else None
    if cycles:
        e["cycles_per_xcd"] = cycles
    units = v.get("SQ_ACTIVE_INST_VALU")
    if units and cycles:
        per_simd = units / SIMDS / cycles
        e["valu_units_per_simd_cycle"] = per_simd
        if cyc_unit:
            e["valu_issue_util_calibrated"] = per_simd * cyc_unit[0]
            e["valu_calibration"] = f"{cyc_unit[0]:.3f} cycles per unit at 4 waves/SIMD ({cyc_unit[1]})"
        if cyc_unit8:
            e["valu_issue_util_vs_8wave_peak"] = per_simd * cyc_unit8[0]
        e["valu_issue_util_guide_2cyc"] = per_simd * GUIDE_CYC
    if units and v.get("SQ_THREAD_CYCLES_VALU"):
        e["valu_lane_util"] = v["SQ_THREAD_CYCLES_VALU"] / (64.0 * units)
    wc = v.get("SQ_WAVE_CYCLES")
    if wc:
        for key, name in (("SQ_ACTIVE_INST_ANY", "wave_frac_issuing"), ("SQ_WAIT_INST_ANY", "wave_frac_wait_inst_dependency"),
                          ("SQ_WAIT_ANY", "wave_frac_wait_waitcnt")):
            if key in v:
                e[name] = v[key] / wc
        if "SQ_WAIT_INST_LDS" in v:
            e["wave_frac_wait_inst_lds"] = v["SQ_WAIT_INST_LDS"] / wc
    if v.get("SQ_LDS_IDX_ACTIVE") and cycles:
        e["lds_busy"] = v["SQ_LDS_IDX_ACTIVE"] / CUS / cycles
        e["lds_conflict_share"] = v.get("SQ_LDS_BANK_CONFLICT", 0.0) / v["SQ_LDS_IDX_ACTIVE"]
    if segments:
        mix = {}
        for key in ("SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_INT64",
                    "SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_ADD_F64",
                    "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_TRANS_F32", "SQ_INSTS_VALU_TRANS_F64", "SQ_INSTS_VALU_CVT"):
            if key in v:
                mix[key.replace("SQ_", "").lower()] = v[key] / segments
        e["per_segment_wave_instructions"] = mix
    return e


def main(tag, scene, prec, segments_per_step, variant=2, root="gpurun_out"):
    base = os.path.join(root, f"pmc_{tag}")
    agg = defaultdict(dict)
    ncalls = {}
    for g in sorted(glob.glob(os.path.join(base, "g*"))):
        c, n = load(g)
        for k, v in c.items():
            agg[k].update(v)
            ncalls[k] = max(ncalls.get(k, 0), n.get(k, 0))
    cyc_unit = calibrated_cycles()
    cyc_unit8 = calibrated_cycles(waves=8)
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
        is_path = short.startswith("art::k_extend") or short.startswith("art::k_paths")
        e.update(derive(v, segments_per_step if is_path else 0, cyc_unit, cyc_unit8))
        kernels[short] = e
    ext = {k: v for k, v in kernels.items() if k.startswith("art::k_extend") or k.startswith("art::k_paths")}
    total = lambda key: sum(v.get(key, 0) for v in ext.values())
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from another_raytracer_amd._lib import LIB_PATH, kernel_build_id
    res = {"tag": tag, "scene": scene, "precision": prec, "segments": segments_per_step, "extend_variant": variant,
           "libart_build": kernel_build_id(LIB_PATH),  # bench.py uses this summary only with the same device code
           "kernels": kernels,
           "note": "hbm_read_bytes_corrected = 2*FETCH_SIZE*1024 (gfx950 half-count correction), hbm_write_bytes = WRITE_SIZE*1024; "
                   "bound analysis units: tools/pmc_summary.py docstring"}
    dom = max(ext.items(), key=lambda kv: kv[1].get("SQ_WAVE_CYCLES", 0), default=None)
    if dom:
        res["dominant_kernel"] = dom[0]
        for key in ("valu_issue_util_calibrated", "valu_issue_util_vs_8wave_peak", "valu_issue_util_guide_2cyc", "valu_lane_util", "wave_frac_issuing",
                    "wave_frac_wait_inst_dependency", "wave_frac_wait_waitcnt", "lds_busy", "lds_conflict_share", "valu_calibration"):
            if key in dom[1]:
                res[key] = round(dom[1][key], 4) if isinstance(dom[1][key], float) else dom[1][key]
    if segments_per_step and ext:
        res["extend_bytes_per_segment"] = (total("hbm_read_bytes_corrected") + total("hbm_write_bytes")) / segments_per_step
        res["extend_read_bytes_per_segment"] = total("hbm_read_bytes_corrected") / segments_per_step
        res["extend_write_bytes_per_segment"] = total("hbm_write_bytes") / segments_per_step
    os.makedirs("profiles", exist_ok=True)
    out = os.path.join("profiles", f"{tag}_pmc_scene{scene}_{prec}.json")
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    print(out)
    for k in ("dominant_kernel", "valu_issue_util_calibrated", "valu_issue_util_vs_8wave_peak", "valu_issue_util_guide_2cyc", "valu_lane_util", "wave_frac_issuing",
              "wave_frac_wait_inst_dependency", "wave_frac_wait_waitcnt", "lds_busy", "lds_conflict_share"):
        if k in res:
            print(f"  {k}: {res[k]}")


if __name__ == "__main__":
    # argv: tag scene precision segments_per_render [variant [renders]]: renders = path-kernel renders the profiled
    # process ran (counters are summed over all of them)
    renders = int(sys.argv[6]) if len(sys.argv) > 6 else 1
    main(sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]) * renders, int(sys.argv[5]) if len(sys.argv) > 5 else 2)
