#!/usr/bin/env python3
"""Per workload (a tools/profile_pmc.sh directory with the stats, valu and
lds passes): the pair kernel's mean duration, effective clock (GRBM_GUI_ACTIVE
/ 8 XCDs / duration), VALU lane-instructions per cell, and LDS bank-conflict
cycles per LDS instruction; plus the same VALU figure over every DP kernel of
the search (pair + long-entry kernels).  Cells come from the pass's own bench
line (config.cells_per_step).

usage: python tools/pmc_shapes.py <dir> [<dir> ...]
"""
import collections
import csv
import json
import os
import sys


def per_dispatch(path):
    """{kernel: [{counter: value, "_ns": duration}, ...]} of one pass."""
    rows = collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        key = (r["Dispatch_Id"], r["Kernel_Name"])
        rows[key][r["Counter_Name"]] = float(r["Counter_Value"])
        rows[key]["_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    out = collections.defaultdict(list)
    for (_, k), v in sorted(rows.items(), key=lambda x: int(x[0][0])):
        out[k].append(v)
    return out


def bench_line(log):
    for line in reversed(open(log).read().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    return None


def is_pair(k):
    return "pair_kernel<" in k


def is_dp(k):
    return "pair_kernel<" in k or "long16_kernel<" in k or "long_kernel<" in k


def mean(x):
    return sum(x) / len(x) if x else float("nan")


for d in sys.argv[1:]:
    name = os.path.basename(d.rstrip("/"))
    b = bench_line(os.path.join(d, "valu.log"))
    cells = b["config"]["cells_per_step"] if b else float("nan")
    valu = per_dispatch(os.path.join(d, "valu", "run_counter_collection.csv"))
    lds = per_dispatch(os.path.join(d, "lds", "run_counter_collection.csv"))
    pk = [k for k in valu if is_pair(k)]
    # skip the warm-up dispatch (first) of every kernel
    pv = [x for k in pk for x in valu[k][1:]]
    dur_ns = mean([x["_ns"] for x in pv])
    clk = mean([x["GRBM_GUI_ACTIVE"] / 8 / x["_ns"] for x in pv])       # GHz
    pair_valu = mean([x["SQ_INSTS_VALU"] for x in pv])
    dp_valu = sum(mean([x["SQ_INSTS_VALU"] for x in valu[k][1:]]) for k in valu if is_dp(k))
    busy = mean([x["SQ_BUSY_CYCLES"] / x["GRBM_GUI_ACTIVE"] for x in pv])
    lv = [x for k in lds if is_pair(k) for x in lds[k][1:]]
    conf = mean([x["SQ_LDS_BANK_CONFLICT"] / x["SQ_INSTS_LDS"] for x in lv]) if lv else float("nan")
    ldsa = mean([x["SQ_LDS_IDX_ACTIVE"] / x["SQ_INSTS_LDS"] for x in lv]) if lv else float("nan")
    # wave-instructions per SIMD and cycle at that clock
    ipc = pair_valu / 1024 / (clk * dur_ns) if dur_ns else float("nan")
    # (cycles, not milliseconds, compare passes: the chip's clock under load
    # differs from pass to pass -- MI355X_MICROARCH.md 'DVFS give-back')
    print(f"{name:10s} pair {dur_ns / 1e6:7.3f} ms  clock {clk:5.3f} GHz  Mcycles {dur_ns * clk / 1e6:6.2f}  "
          f"VALU/cell pair {pair_valu * 64 / cells:5.3f} all-DP {dp_valu * 64 / cells:5.3f}  "
          f"cycles/VALU-instr per SIMD {1 / ipc:5.2f}  LDS conflict cyc/instr {conf:5.2f}  "
          f"LDS active cyc/instr {ldsa:5.2f}  busy {busy:4.2f}  kernel TCUPS {b['kernel']['kernel_gcups'] / 1e3:6.2f}")
