"""Per-depth breakdown of a rocprofv3 --kernel-trace run of bench.py (extend dispatch i of a pass = depth i % max_depth).

Usage: python tools/trace_depth.py gpurun_out/<trace dir> [max_depth]"""
import collections
import csv
import glob
import sys


def main(d, max_depth=50):
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3  # us
    ext = [r for r in rows if "k_extend" in r["Kernel_Name"]]
    print(len(ext), "extend dispatches")
    bydepth = collections.defaultdict(list)
    for i, r in enumerate(ext):
        bydepth[i % max_depth].append(dur(r))
    tot = sum(sum(v) for v in bydepth.values())
    acc = 0.0
    for dd in range(max_depth):
        v = bydepth[dd]
        s = sum(v)
        acc += s
        if dd < 12 or dd % 5 == 0 or dd == max_depth - 1:
            print(f"depth {dd:2d} avg {s / len(v):8.1f} us  sum {s / 1e3:7.1f} ms  cum {acc / tot * 100:5.1f}%")
    gaps = sum(max(0, int(rows[i + 1]["Start_Timestamp"]) - int(rows[i]["End_Timestamp"])) for i in range(len(rows) - 1)) / 1e6
    busy = sum(dur(r) for r in rows) / 1e3
    print(f"kernels {len(rows)}  busy {busy:.1f} ms  gaps {gaps:.1f} ms")
    byk = collections.defaultdict(lambda: [0.0, 0])
    for r in rows:
        k = byk[r["Kernel_Name"].split("(")[0].replace("void ", "")[:70]]
        k[0] += dur(r) / 1e3
        k[1] += 1
    for k, (ms, n) in sorted(byk.items(), key=lambda x: -x[1][0])[:12]:
        print(f"{ms:9.1f} ms {n:6d} x {ms / n * 1e3:8.1f} us  {k}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 50)
