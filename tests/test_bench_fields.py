"""The bench line's derived fields follow the build: roofline.traffic and the
VALU roofline's instructions per cell and clock come from a PMC record of the
same workload AND the same kernel sources (profiles/traffic.json keyed by
libssa_amd.workloads.kernel_src_hash); another build's record is reported as
stale, never as this build's figures."""
import json
import os
import shutil

from libssa_amd import workloads as W
from tests.conftest import ROOT

KEY = "c2:sw:blosum62:bg20:gamma:tail0:seqs1000000:q400:rows48"


def _tree(tmp_path):
    for rel in W.KERNEL_SOURCES:
        dst = tmp_path / rel
        dst.parent.mkdir(parents=True, exist_ok=True)
        shutil.copy(os.path.join(ROOT, rel), dst)
    return str(tmp_path)


def test_kernel_src_hash_is_the_repo_sources():
    assert W.kernel_src_hash() == W.kernel_src_hash(ROOT)
    assert len(W.kernel_src_hash()) == 16


def test_profiled_figures_follow_the_kernel_sources(tmp_path):
    root = _tree(tmp_path / "tree")
    h1 = W.kernel_src_hash(root)
    assert h1 == W.kernel_src_hash()
    path = str(tmp_path / "traffic.json")
    json.dump({KEY: {"bytes_per_launch": 2.9e10, "read_bytes": 1.8e10, "write_bytes": 1.1e10, "kernel_src": h1,
                     "valu_instr_per_cell": 2.96, "clock_ghz": 2.15, "source": "profiles/r06/pmc/c2",
                     "kernel": "pair_kernel"}}, open(path, "w"))
    pf = W.profiled_figures(KEY, h1, path)
    assert pf["stale"] is False and pf["traffic"] == 2.9e10 and pf["valu_instr_per_cell"] == 2.96
    assert pf["clock_ghz"] == 2.15 and pf["source"] == "profiles/r06/pmc/c2"
    # one byte of one kernel source changes: the same record is now stale
    p = os.path.join(root, "libssa_amd/csrc/pair_kernel.h")
    with open(p, "a") as f:
        f.write(" ")
    h2 = W.kernel_src_hash(root)
    assert h2 != h1
    pf = W.profiled_figures(KEY, h2, path)
    assert pf["stale"] is True and pf["stale_source"] == "profiles/r06/pmc/c2"
    assert pf["traffic"] is None and pf["valu_instr_per_cell"] is None and pf["clock_ghz"] is None
    # no record for the workload: nothing, and not stale either
    pf = W.profiled_figures("c3:nw", h1, path)
    assert pf["stale"] is None and pf["traffic"] is None
    assert W.profiled_figures(KEY, h1, str(tmp_path / "absent.json"))["traffic"] is None


def test_committed_records_carry_their_build():
    """Every record bench.py can report names the sources it was measured on
    (rounds 1-5's records, which do not, read as stale)."""
    data = json.load(open(os.path.join(ROOT, "profiles", "traffic.json")))
    for key, rec in data.items():
        pf = W.profiled_figures(key, W.kernel_src_hash(), os.path.join(ROOT, "profiles", "traffic.json"))
        if "kernel_src" not in rec:
            assert pf["stale"] is True and pf["traffic"] is None, key
        else:
            assert pf["stale"] == (rec["kernel_src"] != W.kernel_src_hash()), key
