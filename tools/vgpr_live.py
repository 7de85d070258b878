"""Per-source-line VGPR live-range report of one kernel, from hipcc's gfx950 assembly (`-S --cuda-device-only
-gline-tables-only`).  No GPU needed.

    python tools/vgpr_live.py kernels.s KERNEL_SUBSTRING [--top N] [--window LINES]

The function's instructions are parsed into basic blocks (labels, s_branch / s_cbranch_* / s_endpgm), every VALU /
memory operand into the VGPRs (v / a) it defines and uses, and a backward liveness pass over the linearised CFG gives
the number of live VGPRs at every instruction -- the register pressure the allocator had to fit, which is what sets
`.vgpr_count` and so the waves per SIMD.  Spill slots (scratch_store / scratch_load offsets) count as pseudo-registers,
so on a spilling build "demand" = live VGPRs + live spilled dwords is what the code needed at once.  Printed: the
peak demand, the demand per source line (max over the line's instructions, with its instruction count), what is live
at the peak (and at --at PATTERN) grouped by the source line that last defined it, and where the scratch
instructions sit (innermost enclosing loop).

This is standard liveness on physical registers: a register written under a partial exec mask in one arm of a
branch and rewritten in the other is not counted live in the second arm before its write (the allocator gave both
arms the same register, so the count of registers in use is unaffected)."""
import argparse
import re
import sys
from collections import defaultdict

REG = re.compile(r"\b([va])(\d+)\b|\b([va])\[(\d+):(\d+)\]")
LABEL = re.compile(r"^(\.?[A-Za-z_][\w.$]*):")
# first operand is not a destination
NO_DEF = re.compile(r"^(global_store|buffer_store|flat_store|scratch_store|ds_write|ds_store|ds_(add|sub|min|max|and|or|xor|inc|dec)_(u|i|f|b)\d+\b"
                    r"|global_atomic(?!.*\bsc0\b)|flat_atomic(?!.*\bsc0\b)|buffer_atomic(?!.*\bsc0\b)|s_|exp\b)")
# the destination is also read (partial writes)
DEF_USE = re.compile(r"^(v_writelane|v_mov_b32_dpp|v_.*_dpp\b)")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(1):
            out.add((m.group(1), int(m.group(2))))
        else:
            k, a, b = m.group(3), int(m.group(4)), int(m.group(5))
            out.update((k, i) for i in range(a, b + 1))
    return out


def bits(rs):
    x = 0
    for k, i in rs:
        x |= 1 << (i + {"v": 0, "a": 256, "s": 512}[k])
    return x


def parse(path, name_sub):
    """Instructions of the first function whose label contains name_sub: list of (mnemonic, defs, uses, file, line, text)
    and a map label -> instruction index."""
    lines = open(path).read().split("\n")
    start = None
    for i, l in enumerate(lines):
        if l.endswith(":") and not l.startswith((".", "\t", " ")) and name_sub in l.split(":")[0]:
            start = i + 1
            break
        if ":" in l and not l.startswith((".", "\t", " ")) and name_sub in l.split(":")[0] and "@" in l:
            start = i + 1
            break
    if start is None:
        sys.exit(f"no function matching {name_sub}")
    fname = lines[start - 1].split(":")[0]
    files = {}
    for l in lines:
        m = re.match(r'\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', l)
        if m:
            files[int(m.group(1))] = m.group(2)
    ins, labels = [], {}
    cur_file, cur_line = "?", 0
    for l in lines[start:]:
        s = l.strip()
        if s.startswith(".Lfunc_end"):
            break
        m = LABEL.match(s)
        if m and not s.startswith("\t"):
            labels[m.group(1)] = len(ins)
            continue
        if s.startswith(".loc"):
            p = s.split()
            cur_file, cur_line = files.get(int(p[1]), p[1]), int(p[2])
            continue
        if not s or s.startswith((";", ".", "//")):
            continue
        s = s.split(";")[0].split("//")[0].strip()
        if not s:
            continue
        mn, _, ops = s.partition(" ")
        ops = ops.strip()
        parts = [o.strip() for o in ops.split(",")] if ops else []
        defs, uses = set(), set()
        sm = re.search(r"offset:(\d+)", ops)
        so = int(sm.group(1)) // 4 if sm else 0
        width = {"dword": 1, "dwordx2": 2, "dwordx3": 3, "dwordx4": 4}.get(mn.split("_", 2)[-1], 1)
        if mn.startswith("scratch_store"):  # a spill slot (dword offset) is a pseudo-register: demand = registers + slots
            defs = {("s", so + k) for k in range(width)}
            uses = regs(ops)
            ins.append((mn, bits(defs), bits(uses), cur_file, cur_line, s))
            continue
        if mn.startswith("scratch_load"):
            defs = regs(parts[0])
            uses = {("s", so + k) for k in range(width)}
            ins.append((mn, bits(defs), bits(uses), cur_file, cur_line, s))
            continue
        if parts and not NO_DEF.match(mn):
            defs = regs(parts[0])
            uses = regs(",".join(parts[1:]))
            if DEF_USE.match(mn):
                uses |= defs
        else:
            uses = regs(ops)
        ins.append((mn, bits(defs), bits(uses), cur_file, cur_line, s))
    return fname, ins, labels


def blocks(ins, labels):
    """Basic blocks [start, end) and successor lists."""
    starts = sorted(set([0] + list(labels.values()) + [i + 1 for i, x in enumerate(ins) if x[0].startswith(("s_branch", "s_cbranch", "s_endpgm", "s_setpc"))]))
    starts = [s for s in starts if s < len(ins)]
    bl = [(s, starts[k + 1] if k + 1 < len(starts) else len(ins)) for k, s in enumerate(starts)]
    idx = {s: k for k, (s, _) in enumerate(bl)}
    succ = []
    for k, (s, e) in enumerate(bl):
        last = ins[e - 1]
        mn = last[0]
        out = []
        if mn.startswith(("s_branch", "s_cbranch")):
            tgt = last[5].split()[-1]
            if tgt in labels and labels[tgt] in idx:
                out.append(idx[labels[tgt]])
            if mn.startswith("s_cbranch") and k + 1 < len(bl):
                out.append(k + 1)
        elif mn.startswith(("s_endpgm", "s_setpc")):
            pass
        elif k + 1 < len(bl):
            out.append(k + 1)
        succ.append(out)
    return bl, succ


def liveness(ins, bl, succ):
    live_in = [0] * len(bl)
    gen, kill = [], []
    for s, e in bl:
        g = k = 0
        for i in range(e - 1, s - 1, -1):
            _, d, u, *_ = ins[i]
            g = (g & ~d) | u
            k |= d
        gen.append(g)
        kill.append(k)
    changed = True
    while changed:
        changed = False
        for b in range(len(bl) - 1, -1, -1):
            out = 0
            for t in succ[b]:
                out |= live_in[t]
            new = gen[b] | (out & ~kill[b])
            if new != live_in[b]:
                live_in[b] = new
                changed = True
    # per-instruction live-after sets
    live_at = [0] * len(ins)
    for b, (s, e) in enumerate(bl):
        cur = 0
        for t in succ[b]:
            cur |= live_in[t]
        for i in range(e - 1, s - 1, -1):
            _, d, u, *_ = ins[i]
            live_at[i] = cur | d  # registers occupied while instruction i executes (its defs included)
            cur = (cur & ~d) | u
    return live_at


def popv(x):
    """(live VGPRs, live AGPRs + spill-slot dwords)"""
    return bin(x & ((1 << 256) - 1)).count("1"), bin(x >> 256).count("1")


def loops_of(ins, labels):
    """Back edges (a branch at i to a label at j <= i) as [j, i] instruction ranges, innermost first."""
    out = []
    for i, x in enumerate(ins):
        if x[0].startswith(("s_branch", "s_cbranch")):
            t = x[5].split()[-1]
            if t in labels and labels[t] <= i:
                out.append((labels[t], i))
    return sorted(out, key=lambda l: l[1] - l[0])


def breakdown(ins, live, i_at):
    """Live registers / spill slots at instruction i_at grouped by the source line of their last linear def (values
    defined only later in the linear order are loop-carried: 'LC')."""
    lastdef = {}
    for i, x in enumerate(ins[:i_at + 1]):
        d, r = x[1], 0
        while d:
            if d & 1:
                lastdef[r] = i
            d >>= 1
            r += 1
    groups = defaultdict(int)
    x, r = live[i_at], 0
    while x:
        if x & 1:
            i = lastdef.get(r)
            kind = "slot" if r >= 512 else ("agpr" if r >= 256 else "vgpr")
            groups[(kind, f"{ins[i][3]}:{ins[i][4]}" if i is not None else "LC (loop-carried)")] += 1
        x >>= 1
        r += 1
    return sorted(groups.items(), key=lambda kv: -kv[1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("kernel")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--at", default=None, help="breakdown at the highest-demand instruction whose text or file:line contains this")
    ap.add_argument("--window", type=int, default=0, help="also print the instructions around the peak")
    a = ap.parse_args()
    fname, ins, labels = parse(a.asm, a.kernel)
    bl, succ = blocks(ins, labels)
    live = liveness(ins, bl, succ)
    pv = [popv(x) for x in live]
    dem = [v + s for v, s in pv]  # registers + spilled values live in scratch slots: what the code needed at once
    nspill = sum(1 for x in ins if x[0].startswith("scratch_"))
    print(f"{fname}\n  {len(ins)} instructions, {len(bl)} blocks, {nspill} scratch instructions; peak live VGPRs {max(v for v, _ in pv)}, "
          f"peak demand (VGPRs + live spill-slot dwords) {max(dem)}")
    per_line = defaultdict(lambda: [0, 0])
    for d, x in zip(dem, ins):
        key = (x[3], x[4])
        per_line[key][0] = max(per_line[key][0], d)
        per_line[key][1] += 1
    print(f"\n  source lines by peak demand (top {a.top}):  demand  insts  file:line")
    for (f, ln), (v, n) in sorted(per_line.items(), key=lambda kv: (-kv[1][0], kv[0]))[:a.top]:
        print(f"    {v:4d} {n:6d}  {f}:{ln}")
    hist = defaultdict(int)
    for d in dem:
        hist[(d // 16) * 16] += 1
    print("\n  instructions by demand band: " + ", ".join(f"{k}-{k + 15}: {hist[k]}" for k in sorted(hist)))
    i_peak = max(range(len(ins)), key=lambda i: dem[i])
    points = [("peak", i_peak)]
    if a.at:
        hits = [i for i, x in enumerate(ins) if a.at in f"{x[3]}:{x[4]}" or a.at in x[5]]
        if hits:
            points.append((f"--at {a.at}", max(hits, key=lambda i: dem[i])))
    for what, i_at in points:
        print(f"\n  at the {what} (instruction {i_at}, {ins[i_at][3]}:{ins[i_at][4]}: {ins[i_at][5]}; demand {dem[i_at]}), by defining line:")
        for (kind, where), n in breakdown(ins, live, i_at):
            print(f"    {n:3d} {kind:4s} {where}")
    if nspill:
        loops = loops_of(ins, labels)
        agg = defaultdict(list)
        for i, x in enumerate(ins):
            if x[0].startswith("scratch_"):
                inner = next(((s, e) for s, e in loops if s <= i <= e), None)
                agg[inner].append(x[0].split("_")[1])
        print("\n  scratch instructions by innermost enclosing loop (instruction range, size):")
        for l, v in sorted(agg.items(), key=lambda kv: (kv[0][1] - kv[0][0]) if kv[0] else 1 << 30):
            where = f"[{l[0]}, {l[1]}] {l[1] - l[0]} insts, head {ins[l[0]][3]}:{ins[l[0]][4]}" if l else "outside every loop"
            print(f"    {v.count('store'):3d} stores {v.count('load'):3d} loads  {where}")
    if a.window:
        for i in range(max(0, i_peak - a.window), min(len(ins), i_peak + a.window)):
            print(f"    {dem[i]:4d} {ins[i][3]}:{ins[i][4]}  {ins[i][5]}")


if __name__ == "__main__":
    main()
