"""Markdown rows for DESIGN.md §4 / §6 from committed evidence (no GPU needed):

    python tools/design_tables.py pmc r5f            # bound-analysis rows from profiles/r5f_pmc_scene*_f64.json
    python tools/design_tables.py configs r5f        # one row per config line of profiles/r5f_configs.jsonl
"""
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NAMES = {"1": "k_paths (1)", "8": "k_paths_g LM 1 (final)", "cow": "k_paths_g LM 2 (cow)", "dino": "k_paths_g LM 1 (dino)",
         "9": "k_paths_g LM 2 (capsule)"}


def pmc_rows(tag):
    for scene in ("1", "cow", "8", "dino", "9"):
        path = os.path.join(ROOT, "profiles", f"{tag}_pmc_scene{scene}_f64.json")
        if not os.path.exists(path):
            continue
        d = json.load(open(path))
        k = d["kernels"][d["dominant_kernel"]]
        per = k["per_segment_wave_instructions"]
        print(f"| {NAMES[scene]}, {tag} | {per['insts_valu']:.1f} | {d['valu_issue_util_calibrated']:.2f} | "
              f"{d['valu_issue_util_guide_2cyc']:.2f} | {d['valu_lane_util']:.2f} | {d['wave_frac_wait_waitcnt']:.2f} | "
              f"{d['wave_frac_wait_inst_dependency']:.2f} | {d['extend_bytes_per_segment']:.1f} |")


def config_rows(tag):
    for line in open(os.path.join(ROOT, "profiles", f"{tag}_configs.jsonl")):
        d = json.loads(line)
        c, r = d["config"], d["roofline"]
        traffic = r.get("traffic")
        print(f"| {c['workload']} {c['width']}x{c['height']}x{c['spp']} | {d['value']:.0f} | {r.get('kernel')} | "
              f"{r['frac']:.3f} | {'%.1f GB' % (traffic / 1e9) if traffic else 'null'} |")


if __name__ == "__main__":
    {"pmc": pmc_rows, "configs": config_rows}[sys.argv[1]](sys.argv[2])
