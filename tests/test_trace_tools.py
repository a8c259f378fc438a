"""The per-search gap tools (tools/gap_split.py, tools/host_device_timeline.py)
on a synthetic rocprofv3 kernel/copy trace and SSA_AMD_TRACE host lines: the
segments they report are the ones the timestamps define (DESIGN.md §7 cites
their output)."""
import csv
import os
import subprocess
import sys

from tests.conftest import ROOT

TOOLS = os.path.join(ROOT, "tools")


def _write_trace(d, searches):
    """`searches` loops of device events (ns): pair kernel, one-launch filter,
    the result copy, then the next search's upload and tables; a last pair
    kernel closes the trace."""
    rows, copies = [], []
    for s in range(searches):
        t = 1_000_000_000 + s * 20_000_000
        rows.append((t, t + 10_000_000, "void ssa::pair_kernel<24, false, 8>(ssa::StripArgs)"))
        rows.append((t + 10_011_000, t + 10_036_000, "void ssa::filter_onepass<16>(ssa::FilterArgs)"))
        copies.append((t + 10_036_000, t + 10_040_000))
        rows.append((t + 10_076_000, t + 10_080_000, "ssa::upload_kernel(unsigned int*, unsigned int const*, unsigned int)"))
        rows.append((t + 10_086_000, t + 10_099_000, "ssa::pair_tables_kernel(ssa::TableArgs)"))
    # the next search's pair kernel starts 6 us after the tables
    rows.append((1_000_000_000 + searches * 20_000_000 - 9_895_000, 1_000_000_000 + searches * 20_000_000,
                 "void ssa::pair_kernel<24, false, 8>(ssa::StripArgs)"))
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "run_kernel_trace.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        for a, b, n in rows:
            w.writerow([n, a, b])
    with open(os.path.join(d, "run_memory_copy_trace.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Start_Timestamp", "End_Timestamp"])
        for a, b in copies:
            w.writerow([a, b])
    return rows, copies


def test_gap_split_on_a_synthetic_trace(tmp_path):
    d = str(tmp_path / "trace")
    _write_trace(d, 1)
    out = subprocess.run([sys.executable, os.path.join(TOOLS, "gap_split.py"), d], capture_output=True, text=True,
                         check=True).stdout
    assert "(1 gaps)" in out
    seg = dict(x.rsplit(" ", 1) for x in out.split(": ", 1)[1].strip().split(", "))
    assert float(seg["pair_end->filter"]) == 11.0
    assert float(seg["filter chain"]) == 25.0
    assert float(seg["select->copy end"]) == 4.0
    assert float(seg["copy end->upload (host)"]) == 36.0
    assert float(seg["tables"]) == 13.0


def test_host_device_timeline_on_a_synthetic_trace(tmp_path):
    d = str(tmp_path / "trace")
    rows, copies = _write_trace(d, 3)
    uploads = [a for a, _, n in rows if "upload_kernel" in n]
    # search j (j = 0, 1) enters 10 us before upload j, issues it 4 us later,
    # runs pair kernel j + 1 and wakes 3 us after that kernel's result copy
    # (copy j + 1); it returns 12 us after the wake
    lines = []
    for j in range(2):
        entry = uploads[j] - 10_000
        synced = (copies[j + 1][1] + 3_000 - entry) / 1e3
        lines.append(f"trace: host us (entry at {entry} ns): caller 1.0, views 0.1, planned 2.0, "
                     f"upload issued 4.0, pair issued 10.0, issued 20.0, synced {synced:.1f}, "
                     f"candidates {synced + 4:.1f}, searched {synced + 7:.1f}, return {synced + 12:.1f}\n")
    log = tmp_path / "trace.log"
    log.write_text("trace: sync-wait 1.0\n" + "".join(lines))
    out = subprocess.run([sys.executable, os.path.join(TOOLS, "host_device_timeline.py"), d, str(log)],
                         capture_output=True, text=True, check=True).stdout
    assert out.startswith("2 traced searches, 3 upload kernels, 3 copies")
    med = {ln.split(" median")[0].strip(): float(ln.split("median")[1].split("us")[0]) for ln in out.splitlines()[1:]}
    assert med["copy end -> host synced"] == 3.0
    assert med["synced -> return"] == 12.0
    # search 0 returns 15 us after copy 1's end (10 040 us into its loop);
    # search 1 enters 10 us before upload 1 (10 076 us into the same loop)
    assert med["return -> next entry"] == 11.0
    assert med["entry -> upload issued"] == 4.0
    assert med["upload issued -> upload start"] == 6.0
