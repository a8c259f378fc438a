/*
 * ref_harness.c -- drives the reference's own C sources (compiled from
 * /root/reference/src by oracle/Makefile into oracle/_ref/) so that:
 *   - golden fixtures can be generated from the reference itself
 *     (tools/gen_golden.py), pinning oracle/ssa_oracle.c;
 *   - bench.py's cpu_baseline leg can time the reference's AVX2 int16
 *     kernel (search_16_chunk -> search_16_avx2_sw) on the host cores.
 *
 * TEST INFRASTRUCTURE ONLY: never linked into the product.  It calls the
 * reference's internal per-chunk functions directly, the way the
 * reference's kernel-level tests do (tests/algo/16/test_16_simd_*), so it
 * needs no DB plugin: chunks are assembled here from a request file.
 *
 * Request (little endian), see tools/refharness.py:
 *   char[4] "SSAR"; u32 mode; u32 algo; u32 threads; u64 k; u64 chunk;
 *   i32 gapO; i32 gapE; u32 repeat; u32 pad; i64 matrix[1024];
 *   u64 qlen; u8 q[qlen]; u64 nseq; u64 off[nseq+1]; u8 db[off[nseq]]
 * modes: 0 = per-sequence full_sw/full_nw (int64),
 *        1 = 64-bit search (search_64_chunk, heap replay),
 *        2 = 16-bit AVX2 search (search_16_chunk), 3 = 16-bit SSE2 search
 *        4 = dump built-in matrices and maps
 *        5 = translate every DB sequence (mapped NT codes) with the query
 *            table (genetic code k) and the DB table (genetic code chunk):
 *            for side 0/1, strand 0/1, frame 0..2: u64 len, u8 codes[len]
 *        6 = COMPUTE_ALIGNMENT traceback (align.c align_sequences) of the
 *            query against every DB sequence: u64 region[4] (q begin, q end,
 *            d begin, d end), u64 cigar length, cigar bytes
 *        7 = 8-bit AVX2 search: per chunk the reference's int8 kernel for
 *            every query, its overflow chunk re-run by search_16_chunk
 *            (the cascade of search_8.c:94-124, restated here because
 *            search_8_chunk is static)
 * Search modes (1, 2, 3, 7) answer: u64 count, (i64 score, u64 id) x count,
 * u64 16-bit overflows, u64 non-empty sequences, f64 best seconds, u64
 * 8-bit overflows, u64 nchunks, (u64 o8, u64 o16) per chunk (with chunk = 1:
 * per-sequence overflow flags), u64 repeats, f64 seconds of every repeat.
 * The header's pad field is the number of query views (0 or 1: one); the
 * query blob then holds that many views of qlen / views residues each
 * (e.g. both strands of a nucleotide query, searcher.c:42-90).
 */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>
#include <pthread.h>
#include <time.h>

#include "libssa.h"
#include "libssa_datatypes.h"
#include "matrices.h"
#include "cpu_config.h"
#include "db_adapter.h"
#include "util/minheap.h"
#include "util/util.h"
#include "util/util_sequence.h"
#include "algo/searcher.h"
#include "algo/gap_costs.h"
#include "algo/16/search_16.h"
#include "algo/8/search_8.h"
#include "algo/8/search_8_util.h"
#include "algo/64/search_64.h"
#include "algo/align.h"

int64_t full_sw(sequence_t* dseq, sequence_t* qseq, int64_t* hearray);
int64_t full_nw(sequence_t* dseq, sequence_t* qseq, int64_t* hearray);

static void die(const char* m) { fprintf(stderr, "ref_harness: %s\n", m); exit(2); }

static void rd(void* p, size_t n, FILE* f) { if (n && fread(p, 1, n, f) != n) die("short read"); }

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

typedef struct {
    uint32_t mode, algo, threads; uint64_t k, chunk; int32_t gO, gE; uint32_t repeat, views;
    int64_t mat[1024];
    uint64_t qlen; uint8_t* q;
    uint64_t nseq; uint64_t* off; uint8_t* db;
} req_t;

/* --------------------------------------------------- chunked search state */
static req_t R;
static p_search_data SDP;
static p_sdb_sequence* SEQS;      /* one sdb_sequence_t per non-empty DB sequence */
static size_t NSEQS;              /* number of non-empty sequences */
static size_t* CHUNK_BEGIN;       /* chunk c covers SEQS[CHUNK_BEGIN[c] .. CHUNK_BEGIN[c+1]) */
static size_t NCHUNKS;
static size_t NEXT_CHUNK;
static pthread_mutex_t MTX = PTHREAD_MUTEX_INITIALIZER;

typedef struct { p_minheap heap; size_t ovf, ovf8; } tres_t;
static uint64_t* CH_OVF;          /* per chunk: (8-bit, 16-bit) overflow counts */

static size_t claim(void) {
    pthread_mutex_lock(&MTX);
    size_t c = NEXT_CHUNK++;
    pthread_mutex_unlock(&MTX);
    return c;
}

static void* worker(void* arg) {
    tres_t* res = (tres_t*)arg;
    res->heap = minheap_init(R.k);
    res->ovf = res->ovf8 = 0;
    db_chunk_t chunk;
    p_s16info s16 = NULL;
    p_s8info s8 = NULL;
    int64_t* he = NULL;
    if (R.mode == 2 || R.mode == 3 || R.mode == 7) s16 = search_16_init(SDP);
    if (R.mode == 7) s8 = search_8_init(SDP);
    if (!s16) he = search_64_alloc_hearray(SDP);
    for (;;) {
        size_t c = claim();
        if (c >= NCHUNKS) break;
        chunk.seq = SEQS + CHUNK_BEGIN[c];
        chunk.fill_pointer = CHUNK_BEGIN[c + 1] - CHUNK_BEGIN[c];
        chunk.size = chunk.fill_pointer;
        uint64_t o8 = 0, o16 = 0;
        if (s8) {
            /* search_8.c:94-124 */
            p_db_chunk ovf = adp_alloc_chunk(chunk.size * SDP->q_count + 1);
            for (uint8_t q = 0; q < SDP->q_count; q++) {
                if (R.algo == 0) search_8_avx2_sw(s8, &chunk, res->heap, ovf, q);
                else search_8_avx2_nw(s8, &chunk, res->heap, ovf, q);
            }
            if (ovf->fill_pointer) {
                o8 = ovf->fill_pointer;
                o16 = search_16_chunk(s16, res->heap, ovf, SDP);
            }
            adp_free_chunk_no_sequences(ovf);
        } else if (s16) {
            o16 = search_16_chunk(s16, res->heap, &chunk, SDP);
        } else {
            search_64_chunk(res->heap, &chunk, SDP, he);
        }
        res->ovf8 += o8;
        res->ovf += o16;
        CH_OVF[2 * c] = o8;
        CH_OVF[2 * c + 1] = o16;
    }
    if (s8) search_8_exit(s8);
    if (s16) search_16_exit(s16);
    if (he) free(he);
    return NULL;
}

static void run_search(FILE* out) {
    /* query buffer (AMINOACID-style single query; symbol type does not
     * matter below the searcher for pre-mapped codes) */
    SDP = (p_search_data)calloc(1, sizeof(search_data_t));
    const uint32_t nq = R.views > 1 ? R.views : 1;
    SDP->q_count = (uint8_t)nq;
    SDP->maxqlen = R.qlen / nq;
    for (uint32_t v = 0; v < nq; v++) {
        SDP->queries[v].seq.seq = (char*)R.q + v * (R.qlen / nq);
        SDP->queries[v].seq.len = R.qlen / nq;
    }

    score_matrix_64 = (int64_t*)aligned_alloc(64, sizeof(int64_t) * 1024);
    score_matrix_16 = (int16_t*)aligned_alloc(64, sizeof(int16_t) * 1024);
    score_matrix_8 = (int8_t*)aligned_alloc(64, sizeof(int8_t) * 1024);
    for (int i = 0; i < 1024; i++) {
        score_matrix_64[i] = R.mat[i];
        score_matrix_16[i] = (int16_t)R.mat[i];
        score_matrix_8[i] = (int8_t)R.mat[i];
    }
    gapO = (int8_t)R.gO;
    gapE = (int8_t)R.gE;

    reset_compute_capability();
    if (R.mode == 3) set_max_compute_capability(COMPUTE_ON_SSE2);
    search_64_init_algo(R.algo);
    search_16_init_algo(R.algo);
    search_8_init_algo(R.algo);

    /* non-empty sequences in ID order; chunks are ID ranges of R.chunk IDs
     * with empty sequences skipped (db_adapter.c:212-239) */
    SEQS = (p_sdb_sequence*)malloc(sizeof(p_sdb_sequence) * (R.nseq + 1));
    NCHUNKS = (R.nseq + R.chunk - 1) / R.chunk;
    CHUNK_BEGIN = (size_t*)malloc(sizeof(size_t) * (NCHUNKS + 1));
    NSEQS = 0;
    for (uint64_t i = 0; i < R.nseq; i++) {
        if (i % R.chunk == 0) CHUNK_BEGIN[i / R.chunk] = NSEQS;
        uint64_t len = R.off[i + 1] - R.off[i];
        if (len == 0) continue;
        p_sdb_sequence s = (p_sdb_sequence)calloc(1, sizeof(sdb_sequence_t));
        s->ID = i;
        s->seq.seq = (char*)(R.db + R.off[i]);
        s->seq.len = len;
        SEQS[NSEQS++] = s;
    }
    CHUNK_BEGIN[NCHUNKS] = NSEQS;
    CH_OVF = (uint64_t*)calloc(2 * NCHUNKS + 2, sizeof(uint64_t));

    int T = R.threads ? (int)R.threads : 1;
    tres_t* res = (tres_t*)calloc(T, sizeof(tres_t));
    pthread_t* th = (pthread_t*)calloc(T, sizeof(pthread_t));
    double best = 1e30;
    const uint32_t nrep = R.repeat ? R.repeat : 1;
    double* times = (double*)calloc(nrep, sizeof(double));
    p_minheap merged = NULL;
    size_t ovf = 0, ovf8 = 0;
    for (uint32_t rep = 0; rep < nrep; rep++) {
        if (merged) minheap_exit(merged);
        for (int t = 0; t < T; t++) if (res[t].heap) { minheap_exit(res[t].heap); res[t].heap = NULL; }
        NEXT_CHUNK = 0;
        double t0 = now();
        for (int t = 0; t < T; t++) pthread_create(&th[t], NULL, worker, &res[t]);
        for (int t = 0; t < T; t++) pthread_join(th[t], NULL);
        /* merge in thread order (manager.c:141-145) */
        merged = minheap_init(R.k);
        ovf = ovf8 = 0;
        for (int t = 0; t < T; t++) {
            for (size_t j = 0; j < res[t].heap->count; j++) minheap_add(merged, &res[t].heap->array[j]);
            ovf += res[t].ovf;
            ovf8 += res[t].ovf8;
        }
        minheap_sort(merged);
        double dt = now() - t0;
        times[rep] = dt;
        if (dt < best) best = dt;
    }
    uint64_t cnt = merged->count;
    fwrite(&cnt, 8, 1, out);
    for (size_t i = 0; i < merged->count; i++) {
        int64_t sc = merged->array[i].score;
        uint64_t id = merged->array[i].db_id;
        fwrite(&sc, 8, 1, out);
        fwrite(&id, 8, 1, out);
    }
    uint64_t o = ovf;
    fwrite(&o, 8, 1, out);
    uint64_t ns = NSEQS;
    fwrite(&ns, 8, 1, out);
    fwrite(&best, 8, 1, out);
    uint64_t o8 = ovf8, nch = NCHUNKS;
    fwrite(&o8, 8, 1, out);
    fwrite(&nch, 8, 1, out);
    fwrite(CH_OVF, 8, 2 * NCHUNKS, out);
    uint64_t nr = nrep;
    fwrite(&nr, 8, 1, out);
    fwrite(times, 8, nrep, out);
    free(times);
}

static void run_scores(FILE* out) {
    score_matrix_64 = (int64_t*)aligned_alloc(64, sizeof(int64_t) * 1024);
    for (int i = 0; i < 1024; i++) score_matrix_64[i] = R.mat[i];
    gapO = (int8_t)R.gO;
    gapE = (int8_t)R.gE;
    int64_t* he = (int64_t*)malloc(sizeof(int64_t) * 2 * (R.qlen + 1));
    sequence_t q = {(char*)R.q, R.qlen};
    for (uint64_t i = 0; i < R.nseq; i++) {
        sequence_t d = {(char*)(R.db + R.off[i]), R.off[i + 1] - R.off[i]};
        int64_t s = R.algo == 0 ? full_sw(&d, &q, he) : full_nw(&d, &q, he);
        fwrite(&s, 8, 1, out);
    }
    free(he);
}

static void dump_tables(FILE* out) {
    static const char* names[8] = {BLOSUM45, BLOSUM50, BLOSUM62, BLOSUM80, BLOSUM90, PAM30, PAM70, PAM250};
    for (int k = 0; k < 8; k++) {
        mat_init_buildin(names[k]);
        fwrite(score_matrix_64, sizeof(int64_t), 1024, out);
        mat_free();
    }
    fwrite(map_ncbi_aa, 1, 256, out);
    fwrite(map_ncbi_nt16, 1, 256, out);
}

static void run_translate(FILE* out) {
    us_init_translation((int)R.k, (int)R.chunk);
    sequence_t prot = {(char*)malloc(1), 0};
    for (uint64_t i = 0; i < R.nseq; i++) {
        sequence_t dna = {(char*)(R.db + R.off[i]), R.off[i + 1] - R.off[i]};
        for (int side = 0; side < 2; side++)
            for (int strand = 0; strand < 2; strand++)
                for (int frame = 0; frame < 3; frame++) {
                    us_translate_sequence(side, dna, strand, frame, &prot);
                    uint64_t n = prot.len;
                    fwrite(&n, 8, 1, out);
                    fwrite(prot.seq, 1, n, out);
                }
    }
    free(prot.seq);
}

static void run_align(FILE* out) {
    score_matrix_64 = (int64_t*)aligned_alloc(64, sizeof(int64_t) * 1024);
    for (int i = 0; i < 1024; i++) score_matrix_64[i] = R.mat[i];
    gapO = (int8_t)R.gO;
    gapE = (int8_t)R.gE;
    for (uint64_t i = 0; i < R.nseq; i++) {
        alignment_t al;
        memset(&al, 0, sizeof al);
        al.query.seq = (char*)R.q;
        al.query.len = R.qlen;
        al.db_seq.seq = (char*)(R.db + R.off[i]);
        al.db_seq.len = R.off[i + 1] - R.off[i];
        align_sequences(R.algo == 0 ? SMITH_WATERMAN : NEEDLEMAN_WUNSCH, &al);
        uint64_t v[5] = {al.align_q_start, al.align_q_end, al.align_d_start, al.align_d_end, al.alignment_len};
        fwrite(v, 8, 5, out);
        fwrite(al.alignment, 1, al.alignment_len, out);
        free(al.alignment);
    }
}

int main(int argc, char** argv) {
    if (argc < 3) die("usage: ref_harness <request|-> <response>");
    FILE* f = strcmp(argv[1], "-") ? fopen(argv[1], "rb") : stdin;
    if (!f) die("cannot open request");
    char magic[4];
    rd(magic, 4, f);
    if (memcmp(magic, "SSAR", 4)) die("bad magic");
    rd(&R.mode, 4, f); rd(&R.algo, 4, f); rd(&R.threads, 4, f);
    rd(&R.k, 8, f); rd(&R.chunk, 8, f);
    rd(&R.gO, 4, f); rd(&R.gE, 4, f); rd(&R.repeat, 4, f);
    rd(&R.views, 4, f);
    rd(R.mat, 8 * 1024, f);
    rd(&R.qlen, 8, f);
    R.q = (uint8_t*)malloc(R.qlen + 1);
    rd(R.q, R.qlen, f);
    R.q[R.qlen] = 0;
    rd(&R.nseq, 8, f);
    R.off = (uint64_t*)malloc(8 * (R.nseq + 1));
    rd(R.off, 8 * (R.nseq + 1), f);
    R.db = (uint8_t*)malloc(R.off[R.nseq] + 1);
    rd(R.db, R.off[R.nseq], f);
    if (f != stdin) fclose(f);
    if (R.chunk == 0) R.chunk = 1000;
    set_output_mode(OUTPUT_ERROR);

    FILE* out = fopen(argv[2], "wb");
    if (!out) die("cannot open response");
    if (R.mode == 0) run_scores(out);
    else if (R.mode == 4) dump_tables(out);
    else if (R.mode == 5) run_translate(out);
    else if (R.mode == 6) run_align(out);
    else run_search(out);
    fclose(out);
    return 0;
}
