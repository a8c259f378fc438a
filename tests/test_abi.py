"""CPU-side checks of the drop-in boundary: the shared libraries load, export
every symbol include/*.h declares, keep the reference's struct layouts, and
the host-only entry points behave like the reference (no GPU compute here)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import libssa_amd as S
from tests.conftest import DATA, ROOT


def declared(header):
    txt = open(os.path.join(ROOT, "include", header)).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    names = re.findall(r"\b([a-z_][a-z0-9_]*)\s*\(", txt)
    skip = {"if", "while", "for", "sizeof", "return", "defined"}
    return sorted({n for n in names if n not in skip})


def exported(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", os.path.join(S.LIB_DIR, lib)], capture_output=True,
                         text=True, check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if " T " in line}


def test_libraries_built():
    assert os.path.exists(S.LIB_PATH) and os.path.exists(S.DB_LIB_PATH)
    S.load()


@pytest.mark.parametrize("obj", ["kernels", "pair_sw", "pair_nw", "counters"])
def test_hip_objects_hold_every_registered_kernel(obj):
    """Every kernel the host half of a HIP object registers is in its gfx950
    code object (tools/check_kernels.sh, also run by the Makefile): a launch
    of a host-only stub aborts the process on the GPU."""
    path = os.path.join(ROOT, "libssa_amd", "build", obj + ".o")
    if not os.path.exists(path):
        pytest.skip("no in-tree build objects")
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "check_kernels.sh"), path], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


@pytest.mark.parametrize("header,lib", [("libssa.h", "libssa_amd.so"), ("libssa_amd.h", "libssa_amd.so"),
                                        ("libssa_extern_db.h", "libssa_fasta_db.so")])
def test_every_declared_symbol_is_exported(header, lib):
    names = declared(header)
    assert names, header
    missing = [n for n in names if n not in exported(lib)]
    assert not missing, missing
    for n in names:
        assert n in S.EXPORTS[lib], n


def test_c_header_compiles_and_struct_layout(tmp_path):
    """A C caller compiled against include/libssa.h sees the reference's
    struct sizes and offsets (x86-64: db_seq_t 32, q_seq_t 24,
    alignment_t 112 with score at 72, alignment_list_t 16)."""
    src = tmp_path / "layout.c"
    src.write_text(r'''
#include <stdio.h>
#include <stddef.h>
#include "libssa.h"
#include "libssa_amd.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu\n", sizeof(db_seq_t), sizeof(q_seq_t), sizeof(alignment_t),
         offsetof(alignment_t, score), sizeof(alignment_list_t), sizeof(ssa_hit_t));
  return 0;
}''')
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), str(src), "-o",
                    str(exe)], check=True)
    assert subprocess.run([str(exe)], capture_output=True, text=True).stdout.split() == \
        ["32", "24", "112", "72", "16", "24"]


def test_stats_struct_layout_matches_ctypes(tmp_path):
    """ssa_amd_stats_t as a C caller sees it (include/libssa_amd.h) and as
    the Python mirror declares it: same size, same offsets of the last
    fields (the per-slot arrays of the multi-device path)."""
    src = tmp_path / "stats.c"
    src.write_text(r'''
#include <stdio.h>
#include <stddef.h>
#include "libssa_amd.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu\n", sizeof(ssa_amd_stats_t), offsetof(ssa_amd_stats_t, slots),
         offsetof(ssa_amd_stats_t, slot_device), offsetof(ssa_amd_stats_t, slot_kernel_ms),
         offsetof(ssa_amd_stats_t, slot_search_ms));
  return 0;
}''')
    exe = tmp_path / "stats"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), str(src), "-o",
                    str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True).stdout.split()]
    T = S.ssa_amd_stats_t
    assert got == [ctypes.sizeof(T), T.slots.offset, T.slot_device.offset, T.slot_kernel_ms.offset,
                   T.slot_search_ms.offset]


def test_device_query_without_gpu():
    """ssa_amd_get_devices on a machine without a HIP device: one slot, the
    current device unresolved (-1); nothing is fatal before a search."""
    assert S.get_devices() in ([-1], [0])


def test_reference_example_caller_links(tmp_path):
    """The reference's CLI (src/libssa_example.c) is the drop-in caller; a
    caller written against the same API links against libssa_amd.so."""
    src = tmp_path / "caller.c"
    src.write_text(r'''
#include <stdio.h>
#include "libssa.h"
int main(int argc, char** argv) {
  set_output_mode(OUTPUT_ERROR); set_thread_count(4); set_chunk_size(1000);
  set_simd_compute_mode(COMPUTE_ON_AVX2);
  init_score_matrix(MATRIX_BUILDIN, BLOSUM62); init_gap_penalties(-11, -1);
  init_symbol_translation(AMINOACID, FORWARD_STRAND, 1, 1);
  init_db(argv[1]);
  p_query q = init_sequence_fasta(READ_FROM_FILE, argv[2]);
  if (!q) return 3;
  if (argc > 3) { p_alignment_list l = sw_align(q, 5, BIT_WIDTH_16, COMPUTE_SCORE);
    for (size_t i = 0; i < l->len; i++) printf("%ld %zu\n", l->alignments[i]->score, l->alignments[i]->db_seq.ID);
    free_alignment(l); }
  free_sequence(q); ssa_exit(); puts("ok"); return 0;
}''')
    exe = tmp_path / "caller"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe),
                    "-L", S.LIB_DIR, "-lssa_amd", "-lssa_fasta_db", f"-Wl,-rpath,{S.LIB_DIR}"], check=True)
    r = subprocess.run([str(exe), os.path.join(DATA, "AF091148.fas"), os.path.join(DATA, "Q3ZAI3.fasta")],
                       capture_output=True, text=True)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stderr


def _run_c(tmp_path, body, args=()):
    src = tmp_path / "t.c"
    src.write_text('#include <stdio.h>\n#include <string.h>\n#include "libssa.h"\n#include "libssa_extern_db.h"\n'
                   "int main(int argc, char** argv) {" + body + "}\n")
    exe = tmp_path / "t"
    subprocess.run(["gcc", "-std=c99", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe), "-L",
                    S.LIB_DIR, "-lssa_amd", "-lssa_fasta_db", f"-Wl,-rpath,{S.LIB_DIR}"], check=True)
    return subprocess.run([str(exe), *args], capture_output=True, text=True)


def test_fasta_provider_contract(tmp_path):
    """tests/test_libssa_extern_db.c:12-55: counts, ID == index, NULL past end."""
    body = r'''
  ssa_db_init(argv[1]); printf("%zu\n", ssa_db_get_sequence_count());
  for (size_t i = 0; i < ssa_db_get_sequence_count(); i++) if (ssa_db_get_sequence(i)->ID != i) return 5;
  printf("%d %d\n", ssa_db_get_sequence(1403) == NULL, ssa_db_get_sequence(1404) == NULL);
  ssa_db_close();
  ssa_db_init(argv[2]); printf("%zu %zu\n", ssa_db_get_sequence_count(), ssa_db_get_sequence(0)->seqlen);
  printf("%d\n", ssa_db_get_sequence(1) == NULL); ssa_db_close();
  ssa_db_init(argv[3]); printf("%zu %zu\n", ssa_db_get_sequence_count(), ssa_db_get_sequence(4)->ID);
  return 0;'''
    r = _run_c(tmp_path, body, [os.path.join(DATA, f) for f in ("AF091148.fas", "one_seq.fas", "test.fas")])
    assert r.returncode == 0
    assert r.stdout.split() == ["1403", "1", "1", "1", "54", "1", "5", "4"]


def test_fasta_provider_empty_and_multiline_records(tmp_path):
    db = tmp_path / "db.fas"
    db.write_bytes(b">a\nAC\nGT\n>empty\n>b desc\n  AC GT\t\n\n>c\nMKV")
    body = r'''
  ssa_db_init(argv[1]);
  for (size_t i = 0; i < ssa_db_get_sequence_count(); i++) {
    p_seqinfo s = ssa_db_get_sequence(i); printf("%zu:%zu:%.*s\n", s->ID, s->seqlen, (int)s->seqlen, s->seq); }
  return 0;'''
    r = _run_c(tmp_path, body, [str(db)])
    assert r.stdout.split() == ["0:4:ACGT", "1:0:", "2:4:ACGT", "3:3:MKV"]


def test_fatal_paths_exit_1(tmp_path):
    """Configuration errors end the process with status 1 (util.c:36-46,
    tests/test_util.c:152-176 check this through fork+wait)."""
    cases = {
        'init_score_matrix(MATRIX_BUILDIN, "blosum99");': "Unknown matrix: blosum99",
        "init_score_matrix(7, \"x\");": "Unknown mode for reading score matrices: 7",
        'init_score_matrix(READ_FROM_FILE, "/nonexistent");': "Cannot open score matrix file.",
        "init_symbol_translation(AMINOACID, FORWARD_STRAND, 7, 1);": "Illegal database genetic code specified.",
        "init_symbol_translation(AMINOACID, FORWARD_STRAND, 1, 99);": "Illegal query genetic code specified.",
        "init_symbol_translation(9, FORWARD_STRAND, 1, 1);": "Illegal symbol type specified.",
        "init_sequence_fasta(5, \"x\");": "Unknown mode for reading query sequences: 5",
        "sw_align(NULL, 5, 16, 0);": "Scoring not initialized.",
        "init_constant_scores(1,-1); sw_align(NULL, 5, 16, 0);": "Query not initialized.",
        "init_score_matrix(MATRIX_BUILDIN, BLOSUM62); init_symbol_translation(NUCLEOTIDE, 1, 1, 1);"
        "sw_align(init_sequence_fasta(READ_FROM_STRING, \"ACGT\"), 5, 16, 0);":
            "Nucleotide sequences can only be aligned using constant scores.",
    }
    for body, msg in cases.items():
        r = _run_c(tmp_path, "set_output_mode(OUTPUT_SILENT);" + body + " return 0;")
        assert r.returncode == 1, (body, r.returncode, r.stderr)
        assert msg in r.stderr, (body, r.stderr)


def test_query_file_errors_return_null(tmp_path):
    empty = tmp_path / "empty.fas"
    empty.write_text("")
    body = r'''
  set_output_mode(OUTPUT_ERROR);
  printf("%d\n", init_sequence_fasta(READ_FROM_FILE, "-") == NULL);
  printf("%d\n", init_sequence_fasta(READ_FROM_FILE, "/nonexistent/q.fas") == NULL);
  printf("%d\n", init_sequence_fasta(READ_FROM_FILE, argv[1]) == NULL);
  return 0;'''
    r = _run_c(tmp_path, body, [str(empty)])
    lines = r.stdout.splitlines()
    assert [ln for ln in lines if ln in ("0", "1")] == ["1", "1", "1"]
    assert "libssa ERROR: Query not specified" in r.stdout
    assert "libssa ERROR: Cannot open query file: /nonexistent/q.fas" in r.stdout
    assert "libssa ERROR: Could not initialise from query sequence" in r.stdout


def test_chunk_size_zero_message(tmp_path):
    r = _run_c(tmp_path, "set_chunk_size(0); return 0;")
    assert "libssa ERROR: Only non zero chunk sizes are allowed. Using the default size of 1000 sequences." \
        in r.stdout


def test_replay_entry_point_is_host_only():
    """ssa_amd_replay is the reference heap over a log (no GPU needed)."""
    from oracle import pyoracle as po
    rng = np.random.default_rng(0)
    sc = rng.integers(0, 40, 5000)
    ids = np.arange(5000, dtype=np.uint64)
    for k in (1, 3, 10, 100, 6000):
        assert S.replay(list(zip(sc.tolist(), ids.tolist())), k) == po.topk(sc, ids, k)


def test_packed_db_refuses_foreign_files(tmp_path):
    """ssa_amd_load_db checks magic, version and settings before any device
    work (so this runs without a GPU)."""
    import libssa_amd as S
    S.set_output_mode(S.OUTPUT_SILENT)
    S.init_symbol_translation(S.AMINOACID, S.FORWARD_STRAND, 1, 1)
    bad = tmp_path / "bad.ssapack"
    bad.write_bytes(b"NOTAPACK" + bytes(200))
    assert S.load_db(str(bad)) != 0
    assert S.load_db(str(tmp_path / "missing.ssapack")) != 0
    import struct
    hdr = b"SSAPACK1" + struct.pack("<4I", 1, S.NUCLEOTIDE, 1, 1) + struct.pack("<5Q", 0, 0, 0, 0, 0) + bytes(40)
    other = tmp_path / "other.ssapack"
    other.write_bytes(hdr)
    assert S.load_db(str(other)) != 0
    S.set_output_mode(S.OUTPUT_WARNING)


REF = "/root/reference"


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "benchmark", "src")), reason="reference tree absent")
@pytest.mark.parametrize("main", ["src/libssa_example.c", "benchmark/src/benchmark_base_test_run.c",
                                  "benchmark/src/benchmark_chunks.c", "benchmark/src/benchmark_pairwise.c",
                                  "benchmark/src/benchmark_queries.c", "benchmark/src/benchmark_threads.c"])
def test_reference_callers_compile_and_link_unchanged(tmp_path, main):
    """SURVEY §8b "callers to keep linking": the reference's own CLI and
    benchmark drivers, compiled from their sources where they lie (never
    copied) and linked against libssa_amd.so with every symbol resolved.
    (The benchmark drivers include ../../src/libssa.h, the reference's
    header, whose ABI include/libssa.h reproduces.)"""
    srcs = [os.path.join(REF, main)]
    if main.startswith("benchmark/"):
        srcs.append(os.path.join(REF, "benchmark", "src", "benchmark_util.c"))
    exe = tmp_path / "caller"
    r = subprocess.run(["gcc", "-std=gnu99", "-w", "-I", os.path.join(ROOT, "include"), *srcs, "-o", str(exe),
                        "-L", S.LIB_DIR, "-lssa_amd", "-lssa_fasta_db", f"-Wl,-rpath,{S.LIB_DIR}",
                        "-Wl,--no-undefined"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    assert exe.exists()
