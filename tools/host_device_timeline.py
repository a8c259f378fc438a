#!/usr/bin/env python3
"""Host marks (SSA_AMD_TRACE "trace: host us" lines, steady_clock) laid over
the device's kernel and copy trace (rocprofv3 --kernel-trace
--memory-copy-trace, same clock) for each search of a run: where the time
between one search's result copy and the next search's first kernel goes.

Per search (medians over the run, us):
  copy end -> host synced      the host's wake-up after the result copy
  synced -> return             candidates, replay, the hit list
  return -> next entry         the caller (bench.py's loop)
  entry -> upload issued       plan, staging, the upload launch call
  upload issued -> upload start  the launch's way to the device
usage: host_device_timeline.py <trace dir> <stderr log>"""
import csv
import glob
import os
import re
import sys


def rows(d, pat):
    fs = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return list(csv.DictReader(open(fs[0]))) if fs else []


def med(v):
    v = sorted(v)
    return v[len(v) // 2] if v else float("nan")


def main(d, log):
    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows(d, "*kernel_trace.csv")]
    ev += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy") for r in rows(d, "*memory_copy_trace.csv")]
    ev.sort()
    searches = []
    for ln in open(log):
        m = re.match(r"trace: host us \(entry at (\d+) ns\): caller ([-\d.]+)(.*)", ln)
        if not m:
            continue
        t0 = int(m.group(1))
        marks = {k.strip(): float(v) for k, v in re.findall(r", ([a-z ]+) ([-\d.]+)", m.group(3))}
        searches.append((t0, marks))
    uploads = [e for e in ev if "upload_kernel" in e[2]]
    copies = [e for e in ev if e[2] == "copy" or "copyBuffer" in e[2]]
    out = {k: [] for k in ("copy end -> host synced", "synced -> return", "return -> next entry",
                           "entry -> upload issued", "upload issued -> upload start")}
    for i, (t0, mk) in enumerate(searches):
        if "upload issued" not in mk or "synced" not in mk:
            continue
        t_up = t0 + mk["upload issued"] * 1e3
        nxt = [u for u in uploads if u[0] >= t0]
        if nxt:
            out["upload issued -> upload start"].append((nxt[0][0] - t_up) / 1e3)
        out["entry -> upload issued"].append(mk["upload issued"])
        t_sync = t0 + mk["synced"] * 1e3
        prev = [c for c in copies if c[1] <= t_sync]
        if prev:
            out["copy end -> host synced"].append((t_sync - prev[-1][1]) / 1e3)
        out["synced -> return"].append(mk["return"] - mk["synced"])
        if i + 1 < len(searches):
            out["return -> next entry"].append((searches[i + 1][0] - (t0 + mk["return"] * 1e3)) / 1e3)
    print(f"{len(searches)} traced searches, {len(uploads)} upload kernels, {len(copies)} copies")
    for k, v in out.items():
        print(f"  {k:32s} median {med(v):8.1f} us  (n={len(v)}, min {min(v) if v else float('nan'):.1f})")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
