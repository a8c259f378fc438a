#!/usr/bin/env python3
"""The gap between consecutive pair launches cut at the device events inside
it (medians over every gap of a rocprofv3 --kernel-trace --memory-copy-trace
run, tools/runs.sh kgap): pair end -> filter_block start (the long-stream
joins and the kernel-end marker), the filter chain, the result copy, copy end
-> next upload start (host: result, return, next call, plan, launches), upload,
upload end -> tables start, tables, tables end -> pair start.
usage: gap_split.py <trace dir> [...]"""
import csv
import glob
import os
import sys


def rows(d, pat):
    fs = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return list(csv.DictReader(open(fs[0]))) if fs else []


def med(v):
    v = sorted(v)
    return v[len(v) // 2] if v else float("nan")


def split(d):
    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows(d, "*kernel_trace.csv")]
    ev += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy") for r in rows(d, "*memory_copy_trace.csv")]
    ev.sort()
    pairs = [e for e in ev if "pair_kernel" in e[2]]
    seg = {}
    for a, b in zip(pairs, pairs[1:]):
        inside = [e for e in ev if e[0] >= a[1] and e[1] <= b[0]]

        def first(key, after=0):
            for e in inside:
                if key in e[2] and e[0] >= after:
                    return e
            return None
        # (the filter's first and last kernels: filter_block .. filter_select,
        # or the one launch filter_onepass)
        fb = first("filter_block") or first("filter_onepass")
        fs = first("filter_select") or first("filter_onepass")
        cp = first("copyBuffer", fs[1] if fs else 0) or first("copy", fs[1] if fs else 0)
        up = first("upload_kernel", cp[1] if cp else 0)
        tb = first("pair_tables_kernel", up[1] if up else 0)
        if not (fb and fs and cp and up and tb):
            continue
        parts = {
            "pair_end->filter": fb[0] - a[1],
            "filter chain": fs[1] - fb[0],
            "select->copy end": cp[1] - fs[1],
            "copy end->upload (host)": up[0] - cp[1],
            "upload": up[1] - up[0],
            "upload->tables": tb[0] - up[1],
            "tables": tb[1] - tb[0],
            "tables->pair": b[0] - tb[1],
            "total": b[0] - a[1],
        }
        for k, v in parts.items():
            seg.setdefault(k, []).append(v / 1e3)
    return seg


def main():
    for d in sys.argv[1:]:
        seg = split(d)
        n = len(seg.get("total", []))
        print(f"{os.path.basename(d.rstrip('/'))} ({n} gaps): " +
              ", ".join(f"{k} {med(v):.1f}" for k, v in seg.items()))


if __name__ == "__main__":
    main()
