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
    python tools/ref_benchmark.py <out dir> [SSA_AMD_DEVICES value] [--queries]
--pairwise runs benchmark_pairwise.c (one entry, one query, 10 x 10 000 calls per
row: the per-call latency); --queries runs its query-length sweep instead (benchmark_queries.c: 36 queries of
24-5478 residues, SW and NW at 8 and 16 bits, 10 times each; synthetic proteins
of the published queries' lengths under their IDs).
Writes the program's stdout and results/ log to <out dir> and a summary:
per row the median of its 10 times and GCUPS = 513 x DB residues / time
(the reference's formula, benchmark/scripts/evaluate_threads.r:111-117)."""
import os
import shutil
import statistics
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from libssa_amd import synthetic as syn  # noqa: E402
from libssa_amd import workloads as W  # noqa: E402

BIN = os.path.join(ROOT, "oracle", "_ref", "benchmark_threads_amd")
BIN_Q = os.path.join(ROOT, "oracle", "_ref", "benchmark_queries_amd")
BIN_P = os.path.join(ROOT, "oracle", "_ref", "benchmark_pairwise_amd")
# benchmark_queries.c's 36 query IDs and their lengths (residues of the
# reference's benchmark/data/<ID> files, read there); synthetic proteins of
# these lengths stand in for them on the GPU box
QUERY_LENS = {"Q9UKN1": 5478, "P33450": 5147, "Q7TMA5": 4743, "P08519": 4548, "P20930": 4061, "P0C6B8": 3564,
              "P28167": 3005, "P19096": 2504, "P04775": 2005, "Q8LLD0": 1046, "P27895": 1000, "P21177": 729,
              "P42357": 657, "P03435": 567, "P25705": 553, "P18080": 513, "P58229": 511, "P10635": 497,
              "P01008": 464, "Q3ZAI3": 390, "P07327": 375, "P03989": 362, "Q8ZGB4": 361, "P53765": 255,
              "Q60341": 287, "P00762": 246, "P14942": 222, "P19930": 195, "P05013": 189, "P01111": 189,
              "P02232": 144, "P03630": 127, "O74807": 110, "P07765": 70, "O29181": 63, "P56980": 24}


def main(out, devices=None, program="threads"):
    os.makedirs(out, exist_ok=True)
    cfg = W.CONFIGS["sprot"]
    total = cfg["seqs"]
    if program != "pairwise":      # (its DB is one query file)
        q = W.query(cfg)
        codes, off = W.slice_db(cfg, q, total, 0, total, cfg["alphabet"])
        codes, off = syn.with_long_tail(codes, off, cfg["long_tail"], 77, cfg["alphabet"])
        residues = int(off[-1])
    with tempfile.TemporaryDirectory(prefix="ssa_refbench_") as tmp:
        os.makedirs(os.path.join(tmp, "data"))
        os.makedirs(os.path.join(tmp, "results"))
        if program != "pairwise":
            syn.write_fasta(os.path.join(tmp, "data", "uniprot_sprot.fasta"), codes, off)
        shutil.copy(os.path.join(ROOT, "tests", "golden", "data", "P18080.fasta"), os.path.join(tmp, "data", "P18080"))
        if program == "queries":
            for i, (qid, n) in enumerate(QUERY_LENS.items()):
                if qid != "P18080":
                    with open(os.path.join(tmp, "data", qid), "w") as f:
                        f.write(f">{qid} synthetic, {n} residues\n{syn.query_string(syn.protein_query(n, 500 + i))}\n")
        if program == "pairwise":
            # (its DB is the one query file, its query Q3ZAI3: 10 x 10 000 calls per row)
            shutil.copy(os.path.join(ROOT, "tests", "golden", "data", "P18080.fasta"),
                        os.path.join(tmp, "data", "P18080.fasta"))
            shutil.copy(os.path.join(ROOT, "tests", "golden", "data", "Q3ZAI3.fasta"),
                        os.path.join(tmp, "data", "Q3ZAI3.fasta"))
        env = dict(os.environ)
        if devices:
            env["SSA_AMD_DEVICES"] = devices
        binary = {"queries": BIN_Q, "pairwise": BIN_P}.get(program, BIN)
        # (the program's stdout straight into the out dir: a long run shows progress)
        # (a heartbeat line every 30 s: the program's own output is block-buffered
        # into the file until it ends)
        with open(os.path.join(out, "stdout.txt"), "w") as fo, open(os.path.join(out, "stderr.txt"), "w") as fe:
            proc = subprocess.Popen([binary], cwd=tmp, stdout=fo, stderr=fe, env=env)
            t0 = time.time()
            while True:
                try:
                    proc.wait(timeout=30)
                    break
                except subprocess.TimeoutExpired:
                    print(f"{os.path.basename(binary)} running, {time.time() - t0:.0f} s", flush=True)
                    if time.time() - t0 > 1100:
                        proc.kill()
                        proc.wait()
                        raise SystemExit(f"{binary} did not finish in 1100 s")
        r = subprocess.CompletedProcess([binary], proc.returncode, open(os.path.join(out, "stdout.txt")).read(),
                                        open(os.path.join(out, "stderr.txt")).read())
        for f in os.listdir(os.path.join(tmp, "results")):
            shutil.copy(os.path.join(tmp, "results", f), os.path.join(out, "results_" + f))
        if r.returncode != 0:
            raise SystemExit(f"benchmark_threads exited with {r.returncode}: {r.stderr[-2000:]}")
    if program == "pairwise":
        # rows "<SIMD>,<type>,<bits>_bit,t1..t10", each t the time of 10 000 calls
        lines = ["one 513-residue DB entry (P18080) against Q3ZAI3 (390 aa); per row the median over 10 of",
                 "the time of 10 000 sw_align/nw_align calls, and the time per call"]
        for ln in r.stdout.splitlines():
            f = ln.split(",")
            if len(f) < 4 or not f[2].endswith("_bit"):
                continue
            t = statistics.median(float(x) for x in f[3:])
            lines.append(f"{','.join(f[:3]):24s} {t:9.4f} s per 10 000 calls  {t / 1e4 * 1e6:8.1f} us per call")
        open(os.path.join(out, "summary.txt"), "w").write("\n".join(lines) + "\n")
        print("\n".join(lines))
        return
    lines = [f"DB {total + 0} sequences, {residues} residues",
             "row: median of 10 sw_align/nw_align times (s), GCUPS (query length x DB residues / time)"]
    nkey = 4 if program == "queries" else 5
    for ln in r.stdout.splitlines():
        f = ln.split(",")
        if len(f) <= nkey or f[0] not in QUERY_LENS:
            continue
        t = statistics.median(float(x) for x in f[nkey:])
        cells = QUERY_LENS[f[0]] * residues
        lines.append(f"{','.join(f[:nkey]):34s} q {QUERY_LENS[f[0]]:5d} {t:9.5f} s {cells / t / 1e9:9.1f}")
    open(os.path.join(out, "summary.txt"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    prog = "queries" if "--queries" in sys.argv else "pairwise" if "--pairwise" in sys.argv else "threads"
    main(args[0], args[1] if len(args) > 1 else None, prog)
