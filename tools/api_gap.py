#!/usr/bin/env python3
"""Where the time between two searches goes: the HIP API calls, kernels and
copies from one pair_kernel's end to the next one's start, from a
rocprofv3 --kernel-trace --hip-runtime-trace --memory-copy-trace run
(tools/runs.sh api_trace).  usage: api_gap.py <trace dir> [which gap, default -2]"""
import csv
import glob
import os
import sys


def rows(d, pat):
    fs = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return list(csv.DictReader(open(fs[0]))) if fs else []


def main():
    d = sys.argv[1]
    gi = int(sys.argv[2]) if len(sys.argv) > 2 else -2
    ks = rows(d, "*kernel_trace.csv")
    api = rows(d, "*hip_api_trace.csv")
    cp = rows(d, "*memory_copy_trace.csv")
    ev = []
    for r in ks:
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K", r["Kernel_Name"][:70]))
    for r in api:
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "A", r["Function"]))
    for r in cp:
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C", r.get("Direction", "copy")))
    ev.sort()
    pairs = [e for e in ev if e[2] == "K" and "pair_kernel" in e[3]]
    gaps = sorted((pairs[i][0] - pairs[i - 1][1]) / 1e3 for i in range(1, len(pairs)))
    if gaps:
        print(f"all {len(gaps)} gaps between pair launches (us): median {gaps[len(gaps) // 2]:.1f}, "
              f"min {gaps[0]:.1f}, max {gaps[-1]:.1f}")
    durs = {}
    for s_, e_, kind, name in ev:
        if kind == "K":
            durs.setdefault(name, []).append((e_ - s_) / 1e3)
    print("kernel durations (us, median over the run):",
          ", ".join(f"{n.split('(')[0].split('::')[-1]} {sorted(v)[len(v) // 2]:.1f}"
                    for n, v in sorted(durs.items(), key=lambda x: -sum(x[1])) if len(v) > 2))
    a, b = pairs[gi - 1], pairs[gi]
    t0 = a[1]
    print(f"gap between pair launches ending {a[1]} and starting {b[0]}: {(b[0] - a[1]) / 1e3:.1f} us")
    tot = {}
    for s, e, kind, name in ev:
        if e < a[1] - 1000 or s > b[0] + 1000:
            continue
        if kind == "K" and "pair_kernel" in name:
            continue
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {kind} {name}")
        if kind == "A":
            tot[name] = tot.get(name, 0) + (e - s) / 1e3
    print("API time by function (us):")
    for k, v in sorted(tot.items(), key=lambda x: -x[1]):
        print(f"  {v:8.1f}  {k}")


if __name__ == "__main__":
    main()
