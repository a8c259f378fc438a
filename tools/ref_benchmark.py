#!/usr/bin/env python3
"""The reference's own thread-sweep benchmark program, unchanged, on the GPU.

benchmark/src/benchmark_threads.c + benchmark_util.c, compiled against this
repository's libssa.h and linked to libssa_amd (oracle/Makefile
benchmark_threads_amd), times sw_align / nw_align of its query P18080 (513
aa, BLOSUM50, gaps -3/-1) at 8, 16 and 64 bits, 10 times each, for
set_thread_count 2, 3, 5, 6, 0, 0 -- the program behind the numbers
BASELINE.md quotes (benchmark/results/31_03_2015_threads).  Its DB path is
fixed (data/uniprot_sprot.fasta): the Swiss-Prot form of bench.py (548 208
synthetic sequences in Swiss-Prot's 25 letters plus 300 entries of 5-35 k
residues; no network for UniProt) stands in, and data/P18080 is the query
file the reference ships (tests/golden/data/P18080.fasta).

usage (on the GPU box, after make -C oracle ref):
    python tools/ref_benchmark.py <out dir> [SSA_AMD_DEVICES value]
Writes the program's stdout and results/ log to <out dir> and a summary:
per row the median of its 10 times and GCUPS = 513 x DB residues / time
(the reference's formula, benchmark/scripts/evaluate_threads.r:111-117)."""
import os
import shutil
import statistics
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from libssa_amd import synthetic as syn  # noqa: E402
from libssa_amd import workloads as W  # noqa: E402

BIN = os.path.join(ROOT, "oracle", "_ref", "benchmark_threads_amd")


def main(out, devices=None):
    os.makedirs(out, exist_ok=True)
    cfg = W.CONFIGS["sprot"]
    q = W.query(cfg)
    total = cfg["seqs"]
    codes, off = W.slice_db(cfg, q, total, 0, total, cfg["alphabet"])
    codes, off = syn.with_long_tail(codes, off, cfg["long_tail"], 77, cfg["alphabet"])
    residues = int(off[-1])
    with tempfile.TemporaryDirectory(prefix="ssa_refbench_") as tmp:
        os.makedirs(os.path.join(tmp, "data"))
        os.makedirs(os.path.join(tmp, "results"))
        syn.write_fasta(os.path.join(tmp, "data", "uniprot_sprot.fasta"), codes, off)
        shutil.copy(os.path.join(ROOT, "tests", "golden", "data", "P18080.fasta"), os.path.join(tmp, "data", "P18080"))
        env = dict(os.environ)
        if devices:
            env["SSA_AMD_DEVICES"] = devices
        r = subprocess.run([BIN], cwd=tmp, capture_output=True, text=True, timeout=900, env=env)
        open(os.path.join(out, "stdout.txt"), "w").write(r.stdout)
        open(os.path.join(out, "stderr.txt"), "w").write(r.stderr)
        for f in os.listdir(os.path.join(tmp, "results")):
            shutil.copy(os.path.join(tmp, "results", f), os.path.join(out, "results_" + f))
        if r.returncode != 0:
            raise SystemExit(f"benchmark_threads exited with {r.returncode}: {r.stderr[-2000:]}")
    cells = 513 * residues
    lines = [f"DB {total + 0} sequences, {residues} residues; cells per search {cells:.4g}",
             "row: median of 10 sw_align/nw_align times (s), GCUPS"]
    for ln in r.stdout.splitlines():
        if not ln.startswith("P18080,"):
            continue
        f = ln.split(",")
        t = statistics.median(float(x) for x in f[5:])
        lines.append(f"{','.join(f[:5]):34s} {t:9.5f} s {cells / t / 1e9:9.1f}")
    open(os.path.join(out, "summary.txt"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
