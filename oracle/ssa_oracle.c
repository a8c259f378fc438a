/*
 * ssa_oracle.c -- CPU restatement of libssa's scoring path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (libssa_amd/) links,
 * loads or calls this file.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py use it, and only as the checker.
 *
 * It restates, in plain C99, the reference's exact 64-bit semantics:
 *   - residue alphabets  (reference src/util/util_sequence.c:44-88)
 *   - DB residue mapping, unknown -> 0      (util_sequence.c:298-318)
 *   - query mapping, unknown symbols dropped (src/query.c:102-130)
 *   - score-matrix text parser + constant scoring, default cell -1
 *                                           (src/matrices.c:335-460)
 *   - full_sw, int64 Gotoh local alignment  (src/algo/64/smith_waterman_63.c:32-98)
 *   - full_nw, int64 Gotoh global alignment (src/algo/64/needleman_wunsch_64.c:32-98)
 *   - bounded min-heap top-k with the reference's tie behaviour
 *                                           (src/util/minheap.c:50-106, util.h:12)
 *
 * Parity of this restatement is pinned two ways (see tests/test_oracle.py):
 * the known-answer vectors in the reference's own tests, and
 * fixtures produced by the reference sources themselves, compiled by
 * oracle/Makefile into oracle/_ref/ (tools/gen_golden.py).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#include <pthread.h>

#define DIM 32

/* ---------------------------------------------------------------- alphabets */
/* Code order of the reference alphabets (util_sequence.c:40-61 and 63-88). */
static const char AA_ORDER[] = "-ABCDEFGHIKLMNPQRSTVWXYZU*OJ";
static const char NT_ORDER[] = "-ACMGRSVTWYHKDBN";

/* Builds the 256-entry ASCII->code map.  AA: '-' is NOT mapped (it is
 * unknown), letters in either case.  NT: '-' maps to 0, U is T. */
void oracle_build_map(int nucleotide, signed char out[256]) {
    for (int c = 0; c < 256; c++) out[c] = -1;
    const char* order = nucleotide ? NT_ORDER : AA_ORDER;
    int n = (int)strlen(order);
    for (int code = 0; code < n; code++) {
        char ch = order[code];
        if (ch == '-') {
            if (nucleotide) out[(unsigned char)'-'] = 0;
            continue;
        }
        out[(unsigned char)ch] = (signed char)code;
        if (ch >= 'A' && ch <= 'Z') out[(unsigned char)(ch - 'A' + 'a')] = (signed char)code;
    }
    if (nucleotide) {
        out[(unsigned char)'U'] = out[(unsigned char)'T'];
        out[(unsigned char)'u'] = out[(unsigned char)'T'];
    }
}

/* DB mapping: every residue kept, unknown -> 0 (util_sequence.c:298-318).
 * Returns the number of unknown residues. */
size_t oracle_map_db(int nucleotide, const char* s, size_t len, uint8_t* out) {
    signed char map[256];
    oracle_build_map(nucleotide, map);
    size_t unknown = 0;
    for (size_t i = 0; i < len; i++) {
        signed char m = map[(unsigned char)s[i]];
        if (m >= 0) out[i] = (uint8_t)m;
        else { out[i] = 0; unknown++; }
    }
    return unknown;
}

/* Query mapping: unknown symbols are dropped (query.c:102-130).
 * Returns the mapped length. */
size_t oracle_map_query(int nucleotide, const char* s, size_t len, uint8_t* out) {
    signed char map[256];
    oracle_build_map(nucleotide, map);
    size_t n = 0;
    for (size_t i = 0; i < len; i++) {
        signed char m = map[(unsigned char)s[i]];
        if (m >= 0) out[n++] = (uint8_t)m;
    }
    return n;
}

/* ------------------------------------------------------------------ matrix */
/* M[x][y] = m[(x<<5)+y]; x = DB residue, y = query residue
 * (smith_waterman_63.c:57).  Unset cells are -1 (matrices.c:344). */
void oracle_matrix_reset(int64_t* m) {
    for (int i = 0; i < DIM * DIM; i++) m[i] = -1;
}

/* Constant scoring: cells with both codes >= 1 (matrices.c:447-460). */
void oracle_matrix_constant(int match, int mismatch, int64_t* m) {
    oracle_matrix_reset(m);
    for (int a = 1; a < DIM; a++)
        for (int b = 1; b < DIM; b++)
            m[(a << 5) + b] = (a == b) ? match : mismatch;
}

/* One line of the NCBI-style text format (matrices.c:388-437).
 * Header lines start with blank/tab; symbols are mapped with the AA map
 * even for nucleotide work (matrices.c:408,418). */
static void parse_line(const char* line, int* nsym, signed char* order, int64_t* m) {
    signed char map[256];
    oracle_build_map(0, map);
    char c = line[0];
    if (c == '\n' || c == '#' || c == 0) return;
    if (c == ' ' || c == '\t') {
        int k = 0;
        for (const char* p = line + 1; *p; p++)
            if (*p != ' ' && *p != '\t' && *p != '\n') { order[k++] = map[(unsigned char)*p]; (*nsym)++; }
        return;
    }
    int a = map[(unsigned char)c];
    const char* p = line + 1;
    for (int i = 0; i < *nsym; i++) {
        char* end;
        long v = strtol(p, &end, 10);
        if (end == p) break;
        int b = order[i];
        if (a >= 0 && b >= 0 && a < DIM && b < DIM) m[(a << 5) + b] = v;
        p = end;
    }
}

/* Parses a whole matrix text (string or file contents). */
void oracle_matrix_parse(const char* text, int64_t* m) {
    oracle_matrix_reset(m);
    signed char order[4096];
    int nsym = 0;
    const char* s = text;
    char line[4096];
    while (*s) {
        const char* nl = strchr(s, '\n');
        size_t n = nl ? (size_t)(nl - s) : strlen(s);
        if (n >= sizeof(line)) n = sizeof(line) - 1;
        memcpy(line, s, n);
        line[n] = 0;
        parse_line(line, &nsym, order, m);
        s = nl ? nl + 1 : s + strlen(s);
    }
}

/* --------------------------------------------------------------- scorers */
/* full_sw restated: column j over DB, row i over query; H,E per row kept in
 * hearray; F and the diagonal carried down the column; H clamped at 0;
 * score = max over all cells (smith_waterman_63.c:32-98). */
int64_t oracle_full_sw(const uint8_t* d, size_t dlen, const uint8_t* q, size_t qlen,
                       const int64_t* m, int gapO, int gapE, int64_t* hearray) {
    int64_t s = 0;
    for (size_t i = 0; i < 2 * qlen; i++) hearray[i] = 0;
    for (size_t j = 0; j < dlen; j++) {
        int64_t h = 0, f = 0;
        int64_t* hep = hearray;
        const int64_t* row = m + ((size_t)d[j] << 5);
        for (size_t i = 0; i < qlen; i++) {
            int64_t n = hep[0];
            int64_t e = hep[1];
            h += row[q[i]];
            if (e > h) h = e;
            if (f > h) h = f;
            if (h < 0) h = 0;
            if (h > s) s = h;
            hep[0] = h;
            e += gapE;
            f += gapE;
            h += gapO + gapE;
            if (h > e) e = h;
            if (h > f) f = h;
            hep[1] = e;
            h = n;
            hep += 2;
        }
    }
    return s;
}

/* full_nw restated: boundary H(i,-1)=Q+(i+1)R, incoming E at column 0 =
 * 2Q+(i+2)R; per column F into row 0 = 2Q+(j+2)R and diagonal of row 0 =
 * H(-1,j-1) (0 for j=0, else Q+jR); score = H(qlen-1, dlen-1)
 * (needleman_wunsch_64.c:32-98).  qlen must be > 0. */
int64_t oracle_full_nw(const uint8_t* d, size_t dlen, const uint8_t* q, size_t qlen,
                       const int64_t* m, int gapO, int gapE, int64_t* hearray) {
    for (size_t i = 0; i < qlen; i++) {
        hearray[2 * i] = gapO + (int64_t)(i + 1) * gapE;
        hearray[2 * i + 1] = 2 * (int64_t)gapO + (int64_t)(i + 2) * gapE;
    }
    for (size_t j = 0; j < dlen; j++) {
        int64_t* hep = hearray;
        int64_t f = 2 * (int64_t)gapO + (int64_t)(j + 2) * gapE;
        int64_t h = (j == 0) ? 0 : (gapO + (int64_t)j * gapE);
        const int64_t* row = m + ((size_t)d[j] << 5);
        for (size_t i = 0; i < qlen; i++) {
            int64_t n = hep[0];
            int64_t e = hep[1];
            h += row[q[i]];
            if (f > h) h = f;
            if (e > h) h = e;
            hep[0] = h;
            e += gapE;
            f += gapE;
            h += gapO + gapE;
            if (f < h) f = h;
            if (e < h) e = h;
            hep[1] = e;
            h = n;
            hep += 2;
        }
    }
    return hearray[2 * qlen - 2];
}

/* ------------------------------------------------- 8/16-bit overflow flags */
/* Whether the reference's w-bit SIMD NW kernel (w = 8 or 16) sends one
 * (query, DB sequence) pair to the next width, i.e. counts it in
 * overflow_{w}_bit_count.  Replays, for one channel, the saturated int_w
 * recurrence of search_simd_nw.c:180-503:
 *   - the DB sequence runs in blocks of CDEPTH = 4 columns, the last one
 *     padded with code 0 (move_db_sequence_window_*, search_16_util.h:66-80);
 *   - first block: top diagonals H0..H3 = 0, Q+R, Q+2R, Q+3R and top F
 *     F0..F3 = Q+R .. Q+4R, computed in int and truncated to int_w
 *     (:445-453); later blocks continue both with saturating +R (:494-502);
 *     the F entering row 0 is F_k + QR (:211-214);
 *   - left boundary (new sequence): H(i,-1) = QR + i*R and the incoming E
 *     = H(i,-1) + QR, both saturating chains (:233-240);
 *   - ALIGNCORE (:180-191) with saturating adds; h_min / h_max start at 0
 *     (:202-203) and collect every H of every processed cell;
 *   - overflow iff h_min < trunc(I_MIN - Q - R - 1) or h_max == I_MAX
 *     (:372-373, 483-485), or the score H(qlen-1, dlen-1) is not strictly
 *     inside (I_MIN, I_MAX) (:426).
 * V = (int_w) M[d][q] (the 8/16-bit score tables truncate, matrices.c:375-376).
 * work: 2 * qlen int64.  qlen and dlen must be > 0. */
static int64_t trunc_w(int64_t v, int w) { return w == 8 ? (int64_t)(int8_t)v : (int64_t)(int16_t)v; }

static int64_t sat_w(int64_t v, int w) {
    const int64_t lo = -((int64_t)1 << (w - 1)), hi = ((int64_t)1 << (w - 1)) - 1;
    return v < lo ? lo : (v > hi ? hi : v);
}

int oracle_nw_overflow(int w, const uint8_t* d, size_t dlen, const uint8_t* q, size_t qlen,
                       const int64_t* m, int gapO, int gapE, int64_t* work) {
    const int64_t IMIN = -((int64_t)1 << (w - 1)), IMAX = ((int64_t)1 << (w - 1)) - 1;
    const int64_t QR = trunc_w(gapO + gapE, w), R = trunc_w(gapE, w);
    const int64_t T = trunc_w(IMIN - gapO - gapE - 1, w);
    int64_t* hep = work;
    int64_t mge = QR;
    for (size_t i = 0; i < qlen; i++) {
        hep[2 * i] = sat_w(mge, w);
        hep[2 * i + 1] = sat_w(sat_w(mge, w) + QR, w);
        mge = sat_w(mge + R, w);
    }
    int64_t Ht[4], Ft[4];
    for (int k = 0; k < 4; k++) {
        Ht[k] = k == 0 ? 0 : trunc_w(gapO + (int64_t)k * gapE, w);
        Ft[k] = trunc_w(gapO + (int64_t)(k + 1) * gapE, w);
    }
    int64_t hmin = 0, hmax = 0, score = 0;
    const size_t nblocks = (dlen + 3) / 4;
    for (size_t b = 0; b < nblocks; b++) {
        int64_t h[4], f[4], V[4];
        const int64_t* row[4];
        for (int k = 0; k < 4; k++) {
            const size_t j = 4 * b + k;
            row[k] = m + ((size_t)(j < dlen ? d[j] : 0) << 5);
            h[k] = Ht[k];
            f[k] = sat_w(Ft[k] + QR, w);
        }
        for (size_t i = 0; i < qlen; i++) {
            const int64_t h4 = hep[2 * i];
            int64_t E = hep[2 * i + 1], N[4];
            for (int k = 0; k < 4; k++) V[k] = trunc_w(row[k][q[i]], w);
            for (int k = 0; k < 4; k++) {
                int64_t H = sat_w(h[k] + V[k], w);
                if (f[k] > H) H = f[k];
                if (E > H) H = E;
                if (H < hmin) hmin = H;
                if (H > hmax) hmax = H;
                N[k] = H;
                H = sat_w(H + QR, w);
                f[k] = sat_w(f[k] + R, w);
                if (H > f[k]) f[k] = H;
                E = sat_w(E + R, w);
                if (H > E) E = H;
            }
            hep[2 * i] = N[3];
            hep[2 * i + 1] = E;
            if (i + 1 == qlen && b + 1 == nblocks) score = N[(dlen + 3) % 4];
            h[0] = h4; h[1] = N[0]; h[2] = N[1]; h[3] = N[2];
        }
        const int64_t F3 = Ft[3], H3 = Ht[3];
        Ft[0] = sat_w(F3 + R, w); Ft[1] = sat_w(Ft[0] + R, w); Ft[2] = sat_w(Ft[1] + R, w); Ft[3] = sat_w(Ft[2] + R, w);
        Ht[0] = sat_w(H3 + R, w); Ht[1] = sat_w(Ht[0] + R, w); Ht[2] = sat_w(Ht[1] + R, w); Ht[3] = sat_w(Ht[2] + R, w);
    }
    return hmin < T || hmax == IMAX || score <= IMIN || score >= IMAX;
}

/* Same for the w-bit SIMD SW kernel (search_simd_sw.c:172-441): values
 * biased by -2^(w-1) so the local floor is the saturation floor; every
 * block starts its top row and F at I_MIN (:188-189); a new sequence's left
 * column H and E are I_MIN (:205-212); S = max of every H incl. the padding
 * columns; overflow iff S reaches I_MAX (:372-378, 422-423).  With Q, R <= 0,
 * Q + R and the matrix inside int_w this is "score >= 2^w - 1"; large or
 * positive penalties make the truncated Q+R behave differently. */
int oracle_sw_overflow(int w, const uint8_t* d, size_t dlen, const uint8_t* q, size_t qlen,
                       const int64_t* m, int gapO, int gapE, int64_t* work) {
    const int64_t IMIN = -((int64_t)1 << (w - 1)), IMAX = ((int64_t)1 << (w - 1)) - 1;
    const int64_t QR = trunc_w(gapO + gapE, w), R = trunc_w(gapE, w);
    int64_t* hep = work;
    for (size_t i = 0; i < 2 * qlen; i++) hep[i] = IMIN;
    int64_t S = IMIN;
    const size_t nblocks = (dlen + 3) / 4;
    for (size_t b = 0; b < nblocks; b++) {
        int64_t h[4], f[4];
        const int64_t* row[4];
        for (int k = 0; k < 4; k++) {
            const size_t j = 4 * b + k;
            row[k] = m + ((size_t)(j < dlen ? d[j] : 0) << 5);
            h[k] = IMIN;
            f[k] = IMIN;
        }
        for (size_t i = 0; i < qlen; i++) {
            const int64_t h4 = hep[2 * i];
            int64_t E = hep[2 * i + 1], N[4];
            for (int k = 0; k < 4; k++) {
                int64_t H = sat_w(h[k] + trunc_w(row[k][q[i]], w), w);
                if (f[k] > H) H = f[k];
                if (E > H) H = E;
                if (H > S) S = H;
                N[k] = H;
                H = sat_w(H + QR, w);
                f[k] = sat_w(f[k] + R, w);
                if (H > f[k]) f[k] = H;
                E = sat_w(E + R, w);
                if (H > E) E = H;
            }
            hep[2 * i] = N[3];
            hep[2 * i + 1] = E;
            h[0] = h4; h[1] = N[0]; h[2] = N[1]; h[3] = N[2];
        }
        if (S == IMAX) return 1;
    }
    return 0;
}

/* The reference's overflow counters of one search (m_run's INFO line,
 * manager.c:157-160), from per-(view, sequence) scores or flags.  For
 * every DB sequence e with views v: a8(e) = #v overflowing at 8 bits,
 * a16(e) = #v overflowing at 16 bits.  SW overflows at w bits iff the
 * score is >= 2^w - 1 under ordinary penalties (oracle_sw_overflow); NW per
 * oracle_nw_overflow.
 *   width 16: o16 = sum a16(e)                        (search_16.c:92-114)
 *   width 8:  o8 = sum a8(e), o16 = sum a8(e) * a16(e) -- the 8-bit overflow
 *             chunk holds e once per overflowing view and search_16_chunk
 *             re-runs every copy for every view (search_8.c:94-124).
 * flags: [views][nseq] bytes, bit 0 = 8-bit, bit 1 = 16-bit overflow. */
void oracle_overflow_counts(int width, const uint8_t* flags, size_t views, size_t nseq, uint64_t out[2]) {
    uint64_t o8 = 0, o16 = 0;
    for (size_t e = 0; e < nseq; e++) {
        uint64_t a8 = 0, a16 = 0;
        for (size_t v = 0; v < views; v++) {
            a8 += flags[v * nseq + e] & 1;
            a16 += (flags[v * nseq + e] >> 1) & 1;
        }
        if (width == 8) {
            o8 += a8;
            o16 += a8 * a16;
        } else if (width == 16) {
            o16 += a16;
        }
    }
    out[0] = o8;
    out[1] = o16;
}

/* Per-sequence overflow flags of every DB sequence (bit 0: 8-bit, bit 1:
 * 16-bit), multithreaded.  algo 0 = SW, 1 = NW (saturated replays). */
typedef struct {
    int algo; const uint8_t* db; const uint64_t* off; const uint8_t* q; size_t qlen;
    const int64_t* m; int gO, gE; uint8_t* out; size_t begin, end;
} flag_job_t;

static void* run_flag_job(void* p) {
    flag_job_t* J = (flag_job_t*)p;
    int64_t* he = (int64_t*)malloc(sizeof(int64_t) * 2 * (J->qlen + 1));
    for (size_t k = J->begin; k < J->end; k++) {
        const uint8_t* d = J->db + J->off[k];
        size_t dl = (size_t)(J->off[k + 1] - J->off[k]);
        uint8_t f = 0;
        if (dl > 0 && J->qlen > 0) {
            if (J->algo == 0) {
                f = (uint8_t)(oracle_sw_overflow(8, d, dl, J->q, J->qlen, J->m, J->gO, J->gE, he) |
                              (oracle_sw_overflow(16, d, dl, J->q, J->qlen, J->m, J->gO, J->gE, he) << 1));
            } else {
                f = (uint8_t)(oracle_nw_overflow(8, d, dl, J->q, J->qlen, J->m, J->gO, J->gE, he) |
                              (oracle_nw_overflow(16, d, dl, J->q, J->qlen, J->m, J->gO, J->gE, he) << 1));
            }
        }
        J->out[k] = f;
    }
    free(he);
    return NULL;
}

void oracle_overflow_flags(int algo, const uint8_t* db, const uint64_t* offsets, size_t nseq,
                           const uint8_t* q, size_t qlen, const int64_t* m, int gapO, int gapE,
                           uint8_t* out, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    if ((size_t)nthreads > nseq) nthreads = nseq ? (int)nseq : 1;
    pthread_t th[256];
    flag_job_t jobs[256];
    size_t per = (nseq + nthreads - 1) / nthreads;
    for (int t = 0; t < nthreads; t++) {
        flag_job_t J = {algo, db, offsets, q, qlen, m, gapO, gapE, out, t * per, (t + 1) * per};
        if (J.begin > nseq) J.begin = nseq;
        if (J.end > nseq) J.end = nseq;
        jobs[t] = J;
        pthread_create(&th[t], NULL, run_flag_job, &jobs[t]);
    }
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
}

/* Scores every DB sequence (concatenated codes, offsets[k]..offsets[k+1])
 * against one query.  algo: 0 = SW, 1 = NW.  Multithreaded, order-free. */
typedef struct {
    int algo; const uint8_t* db; const uint64_t* off; size_t nseq;
    const uint8_t* q; size_t qlen; const int64_t* m; int gO, gE;
    int64_t* out; size_t begin, end;
} job_t;

static void* run_job(void* p) {
    job_t* J = (job_t*)p;
    int64_t* he = (int64_t*)malloc(sizeof(int64_t) * 2 * (J->qlen + 1));
    for (size_t k = J->begin; k < J->end; k++) {
        const uint8_t* d = J->db + J->off[k];
        size_t dl = (size_t)(J->off[k + 1] - J->off[k]);
        J->out[k] = J->algo == 0 ? oracle_full_sw(d, dl, J->q, J->qlen, J->m, J->gO, J->gE, he)
                                 : oracle_full_nw(d, dl, J->q, J->qlen, J->m, J->gO, J->gE, he);
    }
    free(he);
    return NULL;
}

void oracle_scores(int algo, const uint8_t* db, const uint64_t* offsets, size_t nseq,
                   const uint8_t* q, size_t qlen, const int64_t* m, int gapO, int gapE,
                   int64_t* out, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if ((size_t)nthreads > nseq) nthreads = nseq ? (int)nseq : 1;
    pthread_t th[256];
    job_t jobs[256];
    if (nthreads > 256) nthreads = 256;
    size_t per = (nseq + nthreads - 1) / nthreads;
    for (int t = 0; t < nthreads; t++) {
        job_t J = {algo, db, offsets, nseq, q, qlen, m, gapO, gapE, out, t * per, (t + 1) * per};
        if (J.begin > nseq) J.begin = nseq;
        if (J.end > nseq) J.end = nseq;
        jobs[t] = J;
        pthread_create(&th[t], NULL, run_job, &jobs[t]);
    }
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
}

/* ----------------------------------------------------------------- top-k */
/* Bounded min-heap with the reference's exact structure (minheap.c:50-91):
 * sift-up on insert with strict '<'; when full, replace the root only when
 * root.score < new.score; sift-down picks child c+1 only if strictly
 * smaller than child c.  Final order: score desc, then db_id desc
 * (CMP_ASC in util.h:12 sorts descending; minheap.c:93-106). */
typedef struct { int64_t score; uint64_t id; } ent_t;

static int heap_add(ent_t* a, size_t* count, size_t alloc, ent_t n) {
    if (alloc == 0) return 0;
    if (*count < alloc) {
        size_t i = (*count)++;
        while (i > 0) {
            size_t p = (i - 1) / 2;
            if (!(n.score < a[p].score)) break;
            a[i] = a[p];
            i = p;
        }
        a[i] = n;
        return 1;
    } else if (a[0].score < n.score) {
        size_t p = 0, c = 1;
        while (c < *count) {
            if (c + 1 < *count && a[c + 1].score < a[c].score) c++;
            if (a[c].score < n.score) a[p] = a[c];
            else break;
            p = c;
            c = 2 * p + 1;
        }
        a[p] = n;
        return 1;
    }
    return 0;
}

static int ent_cmp(const void* x, const void* y) {
    const ent_t* a = (const ent_t*)x;
    const ent_t* b = (const ent_t*)y;
    if (a->score != b->score) return a->score > b->score ? -1 : 1;
    if (a->id != b->id) return a->id > b->id ? -1 : 1;
    return 0;
}

/* Replays the insertions in the given order (= ascending DB ID for the
 * 64-bit single-thread reference) and returns the sorted top-k. */
size_t oracle_topk(const int64_t* scores, const uint64_t* ids, size_t n, size_t k,
                   int64_t* out_scores, uint64_t* out_ids) {
    ent_t* a = (ent_t*)malloc(sizeof(ent_t) * (k ? k : 1));
    size_t count = 0;
    for (size_t i = 0; i < n; i++) {
        ent_t e = {scores[i], ids[i]};
        heap_add(a, &count, k, e);
    }
    qsort(a, count, sizeof(ent_t), ent_cmp);
    for (size_t i = 0; i < count; i++) { out_scores[i] = a[i].score; out_ids[i] = a[i].id; }
    free(a);
    return count;
}

/* Insertion log: the elements the heap accepts, in insertion order (used to
 * check the sharded exchange: any globally accepted element is accepted by
 * its shard's heap). Returns the log length. */
size_t oracle_topk_log(const int64_t* scores, const uint64_t* ids, size_t n, size_t k,
                       int64_t* log_scores, uint64_t* log_ids) {
    ent_t* a = (ent_t*)malloc(sizeof(ent_t) * (k ? k : 1));
    size_t count = 0, m = 0;
    for (size_t i = 0; i < n; i++) {
        ent_t e = {scores[i], ids[i]};
        if (heap_add(a, &count, k, e)) { log_scores[m] = e.score; log_ids[m] = e.id; m++; }
    }
    free(a);
    return m;
}
