// pair_kernel.h -- the pair-symbol f16-pattern DP kernel,
// instantiated by pair_sw.hip (SW) and pair_nw.hip (NW), which compile in
// parallel.
#pragma once
#include <type_traits>

#include "dp_common.h"

namespace ssa {

// ---------------------------------------------------------------------------
// SW and NW on f16 bit patterns with a PAIR-SYMBOL profile (the fast path).
//
// Values are 16-bit patterns v + base that order like the positive f16
// numbers they encode (see kernels.hip strip_f16m_kernel): SW uses base = kF16Floor and
// the local-alignment floor inside E's max3.  NW works on diagonal-relative
// values X^(i,j) = X(i,j) - (i+j)R: the gap-extension adds
// of E and F cancel (E^ <- max(E^, h^+Q), F^ <- max(F^, h^+Q)), the profile
// carries -2R, all boundaries become constants, and the score is
// H^(m-1,len-1) + (m+len-2)R.  Its base a.nw_base is chosen on the host so
// that every real value and intermediate of entries up to a.nmax16 columns
// stays inside [0x0400, 0x7BFF] -- NW needs no floor and no
// saturation.  Padding rows/columns may leave that range;
// nothing real depends on them (dependencies only run down and right, and a
// borrow only runs from a low half into the high half, whose cell is at the
// same or a later column and row).
//
// The packed profile operand of one column is (QP[d_j][r], QP[d_{j-1}][r+NP]):
// low half for the current residue, high half for the previous one (the
// skew).  Indexing the LDS table by the residue pair (d_j, d_{j-1}) returns
// it directly -- no v_bfi_b32 per cell and no VGPR copy of the previous row.
// The table has (alpha+1)^2 rows of NP dwords in global memory (alpha =
// compact DB alphabet, +1 for padding); LDS holds the (alpha+1)alpha+1 of
// them a column after column 0 can meet (kernels.h pair_lds_row): 421 rows /
// 46 KiB at stride NP+4 for a 20-letter DB.  It is shared by
// the workgroup's waves, so they step through the strips together (one
// barrier per strip; groups of a workgroup are adjacent in the length order,
// so their strips take nearly the same time).
//
// One launch covers the whole query: a.nstrips strips of 2*NP rows from row
// 0, then -- when NPT > 0 -- one final strip of 2*NPT rows with its own table
// (a.qpt_tail).  The host (engine.cpp) picks NPT as the smallest multiple of 4
// (8 rows) that holds the remainder, so a 400-row query runs 8 strips of 48
// rows and one of 16 instead of a half-empty 48-row strip, and without a
// second launch (a separate launch of the short strip cost its
// own grid ramp and prologue: ~20 % above its instruction count).  NW always
// runs its last strip as the tail: it captures H(m-1, len-1), a per-column
// select that only the tail's instantiation carries (in the main strips'
// code it raised the register allocation past the 3-waves limit).
//
// Columns are processed up to GroupDesc::ncols (a multiple of 4, >= the
// group's longest entry + 1) in 16-column residue blocks with a uniform exit
// inside the last block.
// ---------------------------------------------------------------------------
// row groups of the SW anti-diagonal maxima: 16, then 8, then 4 rows
constexpr int ad_size_at(int s, int np) { return np - s >= 16 ? 16 : (np - s >= 8 ? 8 : (np - s >= 4 ? 4 : 2)); }
constexpr int ad_start(int r, int np) {
    int s = 0;
    while (r >= s + ad_size_at(s, np)) s += ad_size_at(s, np);
    return s;
}
constexpr int ad_size(int r, int np) { return ad_size_at(ad_start(r, np), np); }
constexpr int ad_index(int r, int np) {
    int s = 0, i = 0;
    while (r >= s + ad_size_at(s, np)) s += ad_size_at(s, np), i++;
    return i;
}
constexpr int ad_ngroups(int np) { return ad_index(np - 1, np) + 1; }

// waves per workgroup (they share the pair table) and waves per SIMD the
// register budget is sized for.  (64-row strips, NP = 32, were tried: their
// 63.5 KiB table allows two workgroups per CU, and at 3-4 waves/SIMD the
// strip's state no longer fits the registers -- they spill in the DP loop.)
constexpr int pair_waves(int, bool) { return kPairWaves; }
constexpr int pair_occupancy(int np, bool) { return np <= 16 ? 4 : (np <= 24 ? 3 : 2); }

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) const uint32_t lds_u32;
typedef __attribute__((address_space(3))) const u32x4 lds_u4;
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) const u32x2 lds_u2;

// Strip parts (StripArgs::nparts = 2 or 3) hand a group's boundary rows from
// the workgroup of part p-1 (XCD A) to that of part p (maybe XCD B; the XCDs'
// L2s are not coherent).  Part p-1 keeps its strip boundaries in its row
// buffer as usual, but writes its LAST boundary -- the one part p reads --
// with device-scope 16-byte stores (a buffer store with the sc1 bit:
// write-through past A's L2, full lines), then waits for them (vmcnt 0)
// before the flag.  Part p reads that boundary with ordinary loads (B's L1/L2
// never held these lines in this kernel: dispatch invalidates them, and only
// part p-1 wrote them) and keeps its own boundaries in a buffer of its own
// (rowbuf2 for part 1, rowbuf3 for part 2), so no dirty line of another
// part's buffer left in another XCD's L2 can ever be written back over newer
// data.  No cache-wide writeback/invalidate (those stalled every XCD: -3 %
// on C2); the row-buffer traffic is unchanged.  One buffer per part, so at
// most three parts.
__device__ __forceinline__ void store_row(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t soff, uint4 v, bool dev) {
    const u32x4 x = {v.x, v.y, v.z, v.w};
    if (dev) __builtin_amdgcn_raw_buffer_store_b128(x, rs, voff, soff, 16 /* sc1 */);
    else __builtin_amdgcn_raw_buffer_store_b128(x, rs, voff, soff, 2 /* nt */);
}
// The per-group streams (row buffers, pair rows, top boundary) are read and
// written through buffer resources based at the group's first block: the
// lane's offset is a constant VGPR and the quad's a scalar, so no 64-bit
// address arithmetic runs per quad.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t group_rsrc(const void* base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
}
// (aux: cache policy; the row buffer is written once and read once, so its
// loads and stores are non-temporal: C2 +1 %, profiles/r03/stream/nt_pf_variants.txt;
// the pair-row stream is re-read by every strip and keeps the default)
// (w & 0xffff) << 4 in one instruction (an SDWA word select of the shifted
// operand; left to itself the compiler emits a shift and a mask)
__device__ __forceinline__ uint32_t lo16x16(uint32_t w) {
    uint32_t r;
    asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0"
        : "=v"(r) : "v"(4u), "v"(w));
    return r;
}
template <int AUX = 0>
__device__ __forceinline__ uint4 load_quad(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t soff) {
    const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, AUX);
    return make_uint4(x.x, x.y, x.z, x.w);
}

template <int NP, bool NW, int NPT>
__global__ void __launch_bounds__(64 * pair_waves(NP, NW), pair_occupancy(NP, NW))
pair_kernel(const StripArgs a) {
    constexpr int W = pair_waves(NP, NW);
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t wg = blockIdx.x;
    if (a.ticket) {
        // (through the table's first LDS dword: the first strip's staging
        // starts behind a barrier, after every wave has read it; a static
        // __shared__ word would not fit beside a 160 KiB table)
        if (threadIdx.x == 0) lds[0] = __hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        wg = __builtin_amdgcn_readfirstlane(lds[0]);
    }
    // several queries (StripArgs::nq): unit = (part, quad, query), query innermost
    const uint32_t nqs = a.nq > 1 ? a.nq : 1u;
    uint32_t qi = 0;
    if (nqs > 1) {
        const uint32_t u = wg;
        wg = u / nqs;
        qi = u - wg * nqs;
    }
    // strip parts (StripArgs::nparts): units 0 .. nquads-1 are part 0 (or
    // the whole) of quad wg, later units the later parts of the split quads
    uint32_t part = 0;
    bool split = false;
    if (a.nparts > 1) {
        const uint32_t ns = a.split_q1 - a.split_q0;
        if (wg >= a.nquads) {
            const uint32_t u = wg - a.nquads;
            part = 1 + u / ns;
            wg = a.split_q0 + u % ns;
        }
        split = wg >= a.split_q0 && wg < a.split_q1;
        if (part > 0) {
            // the group's previous part must be done: its strip boundary rows
            // (row buffer) and running maxima come from that workgroup.  Its
            // unit had a lower start-order ticket (tickets are always on with
            // parts), so it is resident or finished: the wait ends.  Bounded
            // anyway (a.part_wait): a timeout is reported and the host runs
            // the search again without parts -- never a hang
            if (threadIdx.x == 0) {
                const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
                while (__hip_atomic_load(a.part_done + (size_t)wg * nqs + qi, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT) != a.part_epoch + part - 1) {
                    if (__builtin_amdgcn_s_memrealtime() - t0 >= a.part_wait) {
                        __hip_atomic_store(a.part_err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(4);
                }
            }
            __syncthreads();
        }
    }
    const uint32_t g = a.g_first + wg * W + wave;
    const bool active = g < a.ngroups;
    if (g < a.g_prio) __builtin_amdgcn_s_setprio(2);
    const uint32_t t_start = a.timeline ? (uint32_t)__builtin_amdgcn_s_memrealtime() : 0u;
    const uint32_t gg = active ? g : a.g_first;

    // this unit's query: rows, tables, outputs
    const uint32_t m = nqs > 1 ? a.qm[qi] : a.m;
    const uint32_t* const qpt = a.qpt + qi * a.q_tab_stride;
    const uint32_t* const qpt_tail = a.qpt_tail + qi * a.q_tab_stride;
    int32_t* const scores = a.scores + qi * a.q_score_stride;
    uint32_t* const ovf_list = a.ovf_list + qi * a.q_ovf_stride;
    uint32_t* const ovf_count = a.ovf_count + qi * a.q_ovf_stride;

    const GroupDesc gd = a.groups[gg];
    const uint32_t nquads = gd.ncols >> 2;
    const uint32_t nblk = (gd.ncols + 15) >> 4;
    const uint4* resp = a.res + (size_t)gd.blk * 64 + lane;
    // row buffers: part p's own boundaries in rowbuf / rowbuf2 / rowbuf3
    // (rowbuf also for every strip without parts); rbr / rbw: where the
    // current strip reads its top boundary (part p > 0 first: part p-1's
    // buffer, the handoff) and writes its bottom one
    // (quad q of a group at byte q * 1024 + lane * 16, as the pair-row stream)
    // (scalar selects: part is wave-uniform)
    const size_t roff = qi * a.q_rowbuf_stride + (size_t)gd.blk * 256;
    const uint4* const own = part == 0 ? a.rowbuf : part == 1 ? a.rowbuf2 : a.rowbuf3;
    const uint4* const prev = part <= 1 ? a.rowbuf : a.rowbuf2;
    __amdgpu_buffer_rsrc_t rbr = group_rsrc(prev + roff);
    __amdgpu_buffer_rsrc_t rbw = group_rsrc(own + roff);
    const uint32_t lane16 = (uint32_t)lane * 16;
    // a non-last part's last strip stores its boundary at device scope (the handoff)
    bool handoff = false;
    // the pair-row stream: per 16-column block two octs of 64 lanes x 16 B,
    // eight 16-bit offsets (LDS byte offset / 16) per lane and oct
    const __amdgpu_buffer_rsrc_t pap = group_rsrc(a.paddr + (size_t)gd.blk * 128);
    const uint32_t nocts = (nquads + 1) >> 1;
    const uint32_t gl = gg * 64 + lane;
    const uint32_t prow = a.alpha + 1;
    const uint32_t len = a.lane_len[gl];

    constexpr uint32_t FL = (uint32_t)kF16Floor * 0x10001u;
    const int Q = a.gap_open, R = a.gap_extend;
    const int BASE = NW ? (int)a.nw_base : kF16Floor;
    const uint32_t cQ = (uint32_t)(Q * 65536 + Q);      // "combined": one v_add_u32 updates both halves
    auto pat = [&](int v) -> uint32_t { return (uint32_t)(v + BASE) & 0xffffu; };

    // SW: running max of x = sat(h - floor(next column)) = max(H - |R|, 0),
    // an exact H_max + (-|R|) unless it is 0 (then the lane is re-scored)
    const uint32_t Rabs = (uint32_t)(-R);
    const uint32_t cRabs = Rabs * 0x10001u;
    uint32_t* const smax = a.part_smax + (size_t)qi * a.ngroups * 64;
    uint32_t S = (!NW && part > 0 && active) ? __hip_atomic_load(smax + gl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                             : 0u;

    // NW: H(m-1, len-1) as captured by the tail strip, and which half of it
    uint32_t cap = 0;
    int cap_half = 0;

    // One strip of height 2*NPS from query row i0, table at src.  CAPS: the
    // strip holding row m-1 of an NW search (captures its H).
    // Every strip's LDS table has rows of ROWW dwords: the main strips' NP + 4
    // (the tail's NPT rows at the same stride), or the tail's own NPT + 4 when
    // the query has no main strip -- the width a.paddr was built for.
    auto strip = [&](auto np_c, auto cap_c, int i0, const uint32_t* tab) {
        constexpr int NPS = decltype(np_c)::value;
        constexpr bool CAPS = decltype(cap_c)::value;
        const uint32_t ROWW = NPS == NP || a.nstrips > 0 ? NP + 4 : NPS + 4;
        // ---- the whole workgroup stages this strip's pair table: the rows a
        // column after column 0 can meet (kernels.h pair_lds_row), from the
        // global table's (A+1)^2 rows (row c1 * prow + c0)
        __syncthreads();
        const uint32_t A_ = a.alpha;
        // (table rows of NPS dwords at a pitch of whole 16-byte units: a tail
        // of NPS = 2 mod 4 rows has a padded global pitch, pair_tables_kernel)
        constexpr uint32_t NP4 = (NPS + 3) / 4;
        const uint32_t ntab4 = pair_lds_rows(A_) * NP4;
        const uint4* src = (const uint4*)tab;
        for (uint32_t i = threadIdx.x; i < ntab4; i += 64 * W) {
            const uint32_t lrow = i / NP4, k = i % NP4;
            const uint32_t c1 = lrow < (A_ + 1) * A_ ? lrow / A_ : A_;
            const uint32_t c0 = lrow < (A_ + 1) * A_ ? lrow - c1 * A_ : A_;
            *(uint4*)(lds + lrow * ROWW + 4 * k) = src[(c1 * prow + c0) * NP4 + k];
        }
        __syncthreads();
        if (!active) return;
        const bool first = (i0 == 0);
        // the last strip's boundary row has no reader
        const bool keep = i0 + 2 * NPS < (int)m;
        const int rr = (int)m - 1 - i0;          // strip row of the last query row (CAPS)
        if (CAPS) cap_half = rr >= NPS ? 1 : 0;
        const int cap_row = rr - cap_half * NPS;
        const uint32_t cap_col = len - 1 + cap_half;
        // the wave's capture columns span [cmin, cmax] (lengths are sorted, so
        // the span is narrow): the select runs only there, behind a scalar test
        uint32_t cmin = 0, cmax = 0;
        if (CAPS) {
            uint32_t lo = len ? cap_col : 0xffffffffu, hi = len ? cap_col : 0u;
            for (int o = 32; o > 0; o >>= 1) {
                lo = min(lo, (uint32_t)__shfl_xor((int)lo, o));
                hi = max(hi, (uint32_t)__shfl_xor((int)hi, o));
            }
            cmin = __builtin_amdgcn_readfirstlane(lo);
            cmax = __builtin_amdgcn_readfirstlane(hi);
        }

        // ---- left boundary (column -1).  SW: 0.  NW, diagonal-relative
        // (X^(i,j) = X(i,j) - (i+j)R): H^(i,-1) = Q+2R, E^ into column 0 =
        // 2Q+2R, H^(-1,j) = Q+2R, F^ into row 0 = 2Q+2R, H^(-1,-1) = 2R --
        // constants.  High halves: step 0 runs them over the virtual column
        // -1, and the initial values make that step produce the boundary by
        // itself: diagonal input Q+4R plus the padding profile -2R, E and F at
        // the pattern minimum, so h = Q+2R and E leaves it as h+Q.
        // SW, also diagonal-relative: true 0 is the pattern of (i+j)|R|, so
        // the local-alignment floor differs per row and column: row r's
        // floor of the next column, both halves, is fl0 + r|R| (fl0: row 0's,
        // wave-uniform, +|R| per column) -- walked down the rows by one
        // scalar add per row (flr), so one SGPR holds the floors instead of
        // NPS (the column loop's SGPRs are the tight resource: spilled ones
        // come back as v_readlane in the loop).  Boundary H(i,-1) = 0 ->
        // (i-1)|R|; high halves at step 0: E at the boundary value, the
        // diagonal input and F low, so h = (i-1)|R|.
        uint32_t H[NPS], E[NPS];
        uint32_t fl0 = NW ? 0u : __builtin_amdgcn_readfirstlane(pat((i0 + 1) * (int)Rabs) |
                                                                (pat((i0 + NPS) * (int)Rabs) << 16));
#pragma unroll
        for (int r = 0; r < NPS; r++) {
            if (NW) {
                H[r] = pat(Q + 2 * R) | (pat(Q + 4 * R) << 16);
                E[r] = pat(2 * Q + 2 * R) | (0x0400u << 16);
            } else {
                H[r] = pat((i0 + r - 1) * (int)Rabs) | (pat(0) << 16);
                E[r] = pat((i0 + r) * (int)Rabs) | (pat((i0 + NPS + r - 1) * (int)Rabs) << 16);
            }
        }
        // diagonal input of row i0 at column 0, H(i0-1, -1); high half low
        uint32_t hd0 = NW ? pat(first ? 2 * R : Q + 2 * R) | (pat(Q + 4 * R) << 16)
                          : pat((i0 - 2) * (int)Rabs) | (pat(0) << 16);
        uint32_t Fprev = 0x0400u;
        // the boundary row above the strip: the previous strip's row buffer,
        // or for the first strip the lane-independent top boundary a.top
        // (a broadcast read; no per-column select between the two)
        const __amdgpu_buffer_rsrc_t qsrc = first ? group_rsrc(a.top) : rbr;
        const uint32_t qvoff = first ? 0u : lane16, qstride = first ? 16u : 1024u;

        // SW, anti-diagonal maxima (AD): cells (r, j) and (r+1, j-1) have the
        // same diagonal-relative offset i0+r+j, so the running maximum needs no
        // per-cell floor subtraction when it is taken along anti-diagonals.
        // The strip's rows are split into groups of 16/8/4 rows (ad_group);
        // in a group of G rows from row g, A[g + (a - g) % G] collects
        // anti-diagonal a: at column j every even local row adds its new h and
        // the previous column's H of the row below (one max3 per two cells);
        // the group's anti-diagonal g+j is complete after its first row at
        // column j and is flushed into S with one saturating subtract of its
        // floor (= that row's floor).  G divides the 16-column block, so
        // every register index is static.
        constexpr bool AD = !NW;
        constexpr int NG = ad_ngroups(NPS);
        uint32_t A[AD ? NPS : 1];
#pragma unroll
        for (int p = 0; p < (AD ? NPS : 1); p++) A[p] = 0;
        uint32_t xa[2] = {0, 0};

        uint32_t ob[4] = {0, 0, 0, 0};
        // row-buffer quads, prefetched PF quads ahead (NW's shorter steps
        // need the longer distance to cover HBM latency).  SW: two buffers
        // used alternately (quad q in buffer q & 1; a block is four quads), so
        // no register copies; NW: a shift register.  The pair-row octs (eight
        // columns) alternate between two buffers: oct 2b in ao[0] (quads 0, 1
        // of block b), 2b + 1 in ao[1]; each is loaded two quads before use.
        constexpr int PF = NW ? 2 : 1;
        constexpr int NB = PF == 1 ? 2 : PF;
        uint4 qn[NB], ao[2];
#pragma unroll
        for (int p = 0; p < PF; p++) {
            const uint32_t nq = min((uint32_t)p, nquads - 1);
            qn[p] = load_quad<2>(qsrc, qvoff, nq * qstride);
        }
        ao[0] = load_quad(pap, lane16, 0u);
        // P: the current column's profile operands, first the pair row
        // (d_0, pad) of column 0 (LDS byte d_0 * prow * rowB + pad * rowB);
        // the next column's row is loaded into P in place behind the row
        // loop, four rows at a time (no second buffer: the registers pay for
        // the SW accumulators A)
        uint32_t P[NPS];
        {
            // column 0's pair (d_0, pad) is not in LDS (pair_lds_row): the
            // row (d_0, 0) with its high halves replaced by the padding
            // value -- a combined constant lo + 65536 hi with a signed low
            // half, so lo is the sign-extended low 16 bits
            const uint32_t d0 = resp[0].x & 0xffu;
            load_row<NPS>(P, (const uint32_t*)((const char*)lds + pair_lds_row(a.alpha, d0, 0) * (ROWW * 4)));
            const uint32_t hi = (uint32_t)(int32_t)(int16_t)(a.pad_word & 0xffffu) << 16;
#pragma unroll
            for (int r = 0; r < NPS; r++) P[r] = (uint32_t)(int32_t)(int16_t)(P[r] & 0xffffu) + hi;
        }

        for (uint32_t b = 0; b < nblk; b++) {
#pragma unroll
            for (int t = 0; t < 4; t++) {
                if (b * 4 + t >= nquads) break;      // uniform: the group's last columns
                const int cb = PF == 1 ? (t & 1) : 0;
                const uint4 qcur = qn[cb];
#pragma unroll
                for (int p = 0; p + 1 < PF; p++) qn[p] = qn[p + 1];
                {
                    // unconditional (past the group's last quad / oct: its last
                    // one again, never used), so the wait for a quad's data can
                    // count exactly the loads issued after it
                    const uint32_t nq = min(b * 4 + t + PF, nquads - 1);
                    const int nb = PF == 1 ? ((t + 1) & 1) : PF - 1;
                    qn[nb] = load_quad<2>(qsrc, qvoff, nq * qstride);
                    if ((t & 1) == 0) {
                        const uint32_t no = min(b * 2 + (t >> 1) + 1, nocts - 1);
                        ao[(t >> 1) ^ 1] = load_quad(pap, lane16, no * 1024u);
                    }
                }
                const uint32_t qw[4] = {qcur.x, qcur.y, qcur.z, qcur.w};
                // this quad's four offsets (16 bits each, in 16-byte units)
                const uint32_t w0 = (t & 1) ? ao[t >> 1].z : ao[t >> 1].x;
                const uint32_t w1 = (t & 1) ? ao[t >> 1].w : ao[t >> 1].y;
                const uint32_t aw[4] = {lo16x16(w0), (w0 >> 16) << 4, lo16x16(w1), (w1 >> 16) << 4};
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const int k = t * 4 + u;
                    const uint32_t j = b * 16 + k;
                    // the next column's pair row: the stream's offsets are LDS
                    // addresses as they stand (the table is the kernel's only
                    // LDS, dynamic, at 0; an address-space-3 pointer keeps the
                    // compiler from adding that base per column)
                    const lds_u32* nrow = (const lds_u32*)(uintptr_t)aw[u];
                    const uint32_t rbv = qw[u];
                    uint32_t F = perm(Fprev, rbv, SEL_LO_BHI_HI_ALO);
                    uint32_t hd = hd0;
                    uint32_t xs[2];
                    uint32_t flr = fl0;          // row r's floor (SW), advanced row by row
#pragma unroll
                    for (int r = 0; r < NPS; r++) {
                        // the diagonal step: P holds combined signed constants
                        // (pair_tables_kernel), so one full-rate v_add_u32
                        // replaces the half-rate v_pk_add_u16 (-5 % per row,
                        // profiles/r01/ubench_mix_rates.txt)
                        const uint32_t h = fmax3(hd + P[r], E[r], F);
                        if ((r & 3) == 3) {
                            const u32x4 v = *(const lds_u4*)(nrow + r - 3);
                            P[r - 3] = v.x;
                            P[r - 2] = v.y;
                            P[r - 1] = v.z;
                            P[r] = v.w;
                        } else if (NPS % 4 == 2 && r == NPS - 1) {
                            // (a tail of NPS = 2 mod 4 rows: its last two)
                            const u32x2 v = *(const lds_u2*)(nrow + r - 1);
                            P[r - 1] = v.x;
                            P[r] = v.y;
                        }
                        hd = H[r];
                        const int g0 = ad_start(r, NPS), G = ad_size(r, NPS);
                        if (AD && ((r - g0) & 1) == 0) {
                            // H[r + 1] still holds column j-1
                            const int ai = g0 + (r - g0 + k) % G;
                            A[ai] = (r - g0 == G - 2) ? fmax2(h, H[r + 1]) : fmax3(A[ai], h, H[r + 1]);
                        }
                        H[r] = h;
                        if (NW) {
                            // diagonal-relative: E and F need no extension add
                            const uint32_t tt = h + cQ;
                            E[r] = fmax2(E[r], tt);
                            F = fmax2(F, tt);
                        } else {
                            const uint32_t tt = h + cQ;
                            E[r] = fmax3(E[r], tt, flr);
                            F = fmax2(F, tt);
                            if (!AD) {
                                // x = max(H - |R|, 0) into H[r]'s slot of the S tree
                                xs[r & 1] = psubsat16(h, flr);
                                if (r & 1) S = fmax3(S, xs[0], xs[1]);
                            }
                            if (AD && r == g0) {
                                // the group's anti-diagonal g0+j is complete:
                                // x = max(H - |R|, 0).  One group: S takes two
                                // columns' x per max3; several: two groups'.
                                const uint32_t x = psubsat16(A[g0 + k % G], flr);   // (r == g0)
                                const int gi = ad_index(r, NPS);
                                if (NG == 1) {
                                    xa[k & 1] = x;
                                    if (k & 1) S = fmax3(S, xa[0], xa[1]);
                                } else if (gi & 1) {
                                    S = fmax3(S, xa[0], x);
                                } else if (gi == NG - 1) {
                                    S = fmax2(S, x);
                                } else {
                                    xa[0] = x;
                                }
                            }
                            // the next row's floor (a chain the compiler
                            // must not turn into NPS precomputed values)
                            flr += cRabs;
                            asm volatile("" : "+s"(flr));
                        }
                    }
                    if (!NW) fl0 += cRabs;
                    hd0 = perm(hd, rbv, SEL_LO_BLO_HI_ALO);
                    Fprev = F;
                    // a per-step anchor the scheduler cannot move work across
                    // (without it NW's schedule grows past 128 VGPRs and spills)
                    if (!NW) asm volatile("" : "+v"(S));
                    else asm volatile("" : "+v"(Fprev));
                    // step 0's high half is the virtual column -1: no output
                    if (b != 0 || k != 0) {
                        ob[(k + 3) & 3] = perm(F, H[NPS - 1], SEL_LO_BHI_HI_AHI);
                        if ((k & 3) == 0 && keep)
                            store_row(rbw, lane16, (b * 4 + (k >> 2) - 1) * 1024u, make_uint4(ob[0], ob[1], ob[2], ob[3]),
                                      handoff);
                    }
                    if (CAPS && j >= cmin && j <= cmax) {
                        uint32_t hsel = H[0];
#pragma unroll
                        for (int r = 1; r < NPS; r++) hsel = (cap_row == r) ? H[r] : hsel;
                        cap = (j == cap_col) ? hsel : cap;
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        }
        ob[3] = FL;
        if (keep)
            store_row(rbw, lane16, (nquads - 1) * 1024u, make_uint4(ob[0], ob[1], ob[2], ob[3]), handoff);
        // the next strip reads what this one wrote (part 1 after its first
        // strip: its own buffer)
        rbr = rbw;
        if (AD) {
            // drain after the last column J = ncols-1: the odd local rows'
            // cells of column J, and each group's anti-diagonals J+1 ..
            // J+G-1 (partial).  fl0 now holds column J+1's floor of row 0;
            // register g+p holds the group's anti-diagonal J+1+d, d = (p -
            // ncols) mod G, floor fl0 + (g + d)|R| (d = G-1 is anti-diagonal
            // J, already flushed: skipped).
#pragma unroll
            for (int r = 0; r < NPS; r++) {
                const int g0 = ad_start(r, NPS), G = ad_size(r, NPS);
                // (fl0 + r|R|: row r's floor of column J+1)
                if ((r - g0) & 1) S = fmax2(S, psubsat16(H[r], fl0 + (uint32_t)(r - 1) * cRabs));
                const uint32_t d = ((uint32_t)(r - g0) - gd.ncols) & (G - 1);
                const uint32_t f = d == (uint32_t)G - 1 ? 0xffffffffu : fl0 + ((uint32_t)g0 + d) * cRabs;
                S = fmax2(S, psubsat16(A[r], __builtin_amdgcn_readfirstlane(f)));
            }
        }
    };

    using MainNP = std::integral_constant<int, NP>;
    using TailNP = std::integral_constant<int, NPT ? NPT : 8>;
    // this unit's strips [s0, s1) of the nstrips main strips + the tail strip
    const uint32_t T = a.nstrips + (NPT > 0 ? 1u : 0u);
    const uint32_t s0 = split ? part * a.part_strips : 0u;
    const uint32_t s1 = split ? min(T, s0 + a.part_strips) : T;
    for (uint32_t s = s0; s < min(s1, a.nstrips); s++) {
        handoff = split && part + 1 < a.nparts && s + 1 == s1;
        strip(MainNP{}, std::false_type{}, (int)s * 2 * NP, qpt + (size_t)s * prow * prow * NP);
    }
    if (NPT > 0 && s1 == T) {
        handoff = false;
        strip(TailNP{}, std::integral_constant<bool, NW>{}, (int)a.nstrips * 2 * NP, qpt_tail);
    }

    if (split && part + 1 < a.nparts) {
        // hand the group on: running maxima, then (after every wave's row
        // buffer stores and maxima are visible at agent scope) the part count
        if (!NW && active) __hip_atomic_store(smax + gl, S, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // every wave's device-scope stores complete, then one flag store
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __syncthreads();
        if (threadIdx.x == 0)
            __hip_atomic_store(a.part_done + (size_t)wg * nqs + qi, a.part_epoch + part, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    if (!active) return;
    if (a.timeline && lane == 0)
        a.timeline[g - a.g_first] = make_uint4(g, t_start, (uint32_t)__builtin_amdgcn_s_memrealtime(), hw_place());
    const uint32_t o = a.lane_out[gl];
    if (o == 0xffffffffu) return;
    if (len == 0) {
        scores[o] = NW ? (int32_t)(a.gap_open + (int64_t)m * a.gap_extend) : 0;
        return;
    }
    int32_t score;
    bool ovf = len > a.nmax16;
    if (!NW) {
        const uint32_t slo = S & 0xffffu, shi = S >> 16;
        const uint32_t smax = slo > shi ? slo : shi;
        // 0 leaves H_max in [0, |R|] undecided: re-score exactly
        ovf = ovf || (smax == 0 && Rabs != 0);
        score = (int32_t)smax + (int32_t)Rabs;
    } else {
        // back from the diagonal-relative value: + (i + j) R at (m-1, len-1)
        score = (int32_t)(cap_half ? cap >> 16 : cap & 0xffffu) - BASE + ((int32_t)m + (int32_t)len - 2) * R;
    }
    if (ovf) {
        const uint32_t idx = atomicAdd(ovf_count, 1u);
        if (idx < a.ovf_cap) ovf_list[idx] = gl;
        scores[o] = INT32_MIN;
    } else {
        scores[o] = score;
    }
}

template <int NP, bool NW, int NPT>
static hipError_t launch_pair_t(const StripArgs& a, size_t lds_bytes, hipStream_t st, int* occ) {
    static std::atomic<uint64_t> attr{0};
    const hipError_t e = lds_attr_once((const void*)pair_kernel<NP, NW, NPT>, attr, (int)kPairLdsMax);
    if (e != hipSuccess) return e;
    constexpr int W = pair_waves(NP, NW);
    if (occ) return hipOccupancyMaxActiveBlocksPerMultiprocessor(occ, (const void*)pair_kernel<NP, NW, NPT>, 64 * W,
                                                                 lds_bytes);
    const uint32_t quads = (a.ngroups - a.g_first + W - 1) / W;
    if (a.nparts > 1 && (a.nquads != quads || a.split_q0 >= a.split_q1 || a.split_q1 > quads))
        return hipErrorInvalidValue;
    if (a.nq > (uint32_t)kMaxFuse) return hipErrorInvalidValue;
    const uint32_t units = a.nparts > 1 ? quads + (a.nparts - 1) * (a.split_q1 - a.split_q0) : quads;
    const uint32_t blocks = units * std::max(a.nq, 1u);
    (void)ssa_launch((const void*)&pair_kernel<NP, NW, NPT>, dim3(blocks), dim3(64 * W), lds_bytes, st, a);
    return hipGetLastError();
}

template <int NP, bool NW, int NPT = 2>
static hipError_t launch_pair_np(const StripArgs& a, int npt, size_t lds_bytes, hipStream_t st, int* occ) {
    // npt in {0} + multiples of 4 up to NP, and for the default strip heights
    // (pair_tail_fine) the multiples of 2
    // (discarded branches, not early returns: a kernel named only behind a
    // return is still instantiated by the device pass)
    constexpr int STEP = pair_tail_fine(NP, NW) ? 2 : 4;
    if constexpr (NPT == 2 && STEP == 4) {
        if (npt == 0) return launch_pair_t<NP, NW, 0>(a, lds_bytes, st, occ);
        return launch_pair_np<NP, NW, 4>(a, npt, lds_bytes, st, occ);
    } else {
        if constexpr (NPT == 2)
            if (npt == 0) return launch_pair_t<NP, NW, 0>(a, lds_bytes, st, occ);
        if (npt == NPT) return launch_pair_t<NP, NW, NPT>(a, lds_bytes, st, occ);
        if constexpr (NPT + STEP <= NP) return launch_pair_np<NP, NW, NPT + STEP>(a, npt, lds_bytes, st, occ);
        else return hipErrorInvalidValue;
    }
}

}  // namespace ssa
