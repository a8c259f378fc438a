// counters.hip -- the reference's 8/16-bit overflow counters (kernels.h
// FlagArgs / CountArgs).
//
// Every width returns exact scores here, so the counters are not a by-product
// of the scoring: they say how many (query view, DB sequence) pairs the
// reference's saturated w-bit SIMD kernels would have handed on to the next
// width (m_run's INFO line, manager.c:157-160).  Per lane:
//
//   flags_decide_kernel  decides from the exact score and bounds wherever
//                        that is provable ("ordinary" regime, checked on the
//                        host: Q, R <= 0, Q + R inside int_w, every profile
//                        value inside int_w):
//     SW  (search_simd_sw.c:172-441, biased so the floor is I_MIN): overflow
//         iff the maximum H over the sequence padded to a multiple of 4
//         columns with code 0 (move_db_sequence_window_*) reaches 2^w - 1;
//         that maximum lies in [score, score + 3 * padmax].
//     NW  (search_simd_nw.c:180-516): overflow iff some H < I_MIN - Q - R - 1,
//         some H == I_MAX or the score is not strictly inside (I_MIN, I_MAX).
//         No overflow is certain when every H of the padded matrix is >= the
//         two-gap bound 2Q + (m + n4)R >= I_MIN - Q - R - 1, no H can reach
//         I_MAX (min(m, n4) * maxM < I_MAX) and the score is inside: then no
//         value of the saturated run ever saturates where it matters, so it
//         equals the exact run.  An exact score >= I_MAX always overflows.
//   flags_replay_kernel  replays the reference's saturated w-bit recurrence
//                        for the remaining lanes (oracle_nw_overflow /
//                        oracle_sw_overflow restate it), stopping at the
//                        first cell that decides the flag.  In practice:
//                        NW at 8 bits with a query longer than ~10 rows
//                        (overflows within the first block's first ~120
//                        rows), lanes whose exact value lives in the int64
//                        list, and pathological penalties.
//   count_kernel         sums the flags into the reference's two counters.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"

namespace ssa {

namespace {

__device__ __forceinline__ int32_t trunc_w(int64_t v, int w) {
    return w == 8 ? (int32_t)(int8_t)v : (int32_t)(int16_t)v;
}

__device__ __forceinline__ int32_t sat_w(int32_t v, int32_t lo, int32_t hi) { return v < lo ? lo : (v > hi ? hi : v); }

// -1: undecided (replay), else the flag.  hmm: the exact (min, max) of H
// over the lane's real cells when long_kernel scored it (NW), else null.
__device__ __forceinline__ int decide(const FlagArgs& a, int w, int32_t s, uint32_t len, const int2* hmm,
                                      bool long_lane) {
    if (!((a.ordinary >> (w == 8 ? 0 : 1)) & 1) || s == INT32_MIN) return -1;
    const int64_t IMIN = -(1ll << (w - 1)), IMAX = (1ll << (w - 1)) - 1;
    if (a.nw && hmm) {
        // exact extremes: when no boundary chain of the saturated run leaves
        // int_w (H(-1,j), F into row 0, H(i,-1), E into column 0 all >= 2Q +
        // (max(m, n4) + 2)R), the saturated run equals the exact one up to the
        // first cell below T or at I_MAX (earlier values never saturate where
        // it matters), and there the saturated value is <= max(exact, I_MIN) <
        // T or == I_MAX -- so a real cell beyond the limits decides "flagged";
        // padding cells (code 0, at most 3 columns) lie within [min + Q + 3R,
        // max + 3 padmax], so real extremes that far inside decide "clear"
        const int64_t n4 = (len + 3) & ~3u;
        const int64_t Q = a.gap_open, R = a.gap_extend;
        const int64_t T = IMIN - Q - R - 1;
        if (2 * Q + ((int64_t)max((int64_t)a.m, n4) + 2) * R >= IMIN) {
            const int2 mm = *hmm;
            if (mm.x < T || mm.y >= IMAX || s <= IMIN || s >= IMAX) return 1;
            if ((int64_t)mm.x + Q + 3 * R >= T && (int64_t)mm.y + 3ll * a.padmax < IMAX) return 0;
        }
    }
    if (!a.nw) {
        const int64_t lim = (1ll << w) - 1;
        if (s >= lim) return 1;
        if ((int64_t)s + 3ll * a.padmax < lim) return 0;
        return -1;
    }
    if (s >= IMAX) return 1;
    const int64_t n4 = (len + 3) & ~3u;
    const int64_t Q = a.gap_open, R = a.gap_extend;
    const int64_t L = 2 * Q + ((int64_t)a.m + n4) * R;
    const int64_t T = IMIN - Q - R - 1;
    int64_t U = (int64_t)min((int64_t)a.m, n4) * a.maxm;
    // a lane the pair or int16 strip kernel scored exactly never held an H
    // of 32767 or more: their admissibility bounds (engine.cpp nw_f16_limit,
    // nw_int16_limit) cap every value of the matrix below it
    if (w == 16 && a.nw_hmax16_ok && !long_lane) U = min(U, IMAX - 1);
    if (L >= T && U < IMAX && s > IMIN) return 0;
    return -1;
}

// a lane's flags into the search's two counters (single view: FlagArgs::direct)
__device__ __forceinline__ void count_direct(const FlagArgs& a, uint32_t f) {
    unsigned long long c8 = 0, c16 = 0;
    if (a.bw == 8) {
        c8 = f & 1;
        c16 = (f & 1) & (f >> 1);
    } else {
        c16 = (f >> 1) & 1;
    }
    for (int o = 32; o > 0; o >>= 1) {
        c8 += __shfl_xor(c8, o);
        c16 += __shfl_xor(c16, o);
    }
    if ((threadIdx.x & 63) == 0) {
        if (c8) atomicAdd(&a.direct[0], c8);
        if (c16) atomicAdd(&a.direct[1], c16);
    }
}

// one thread per entry (coalesced reads of the score and the entry's length
// and lane)
__global__ void __launch_bounds__(256) flags_decide_kernel(const FlagArgs a) {
    const uint32_t o = blockIdx.x * 256 + threadIdx.x;
    uint32_t f = 0;
    bool undecided = false;
    if (o < a.entries) {
        const uint2 ll = a.entry_lane[o];
        const uint32_t len = ll.x, gl = ll.y;
        if (len > 0 && a.m > 0) {
            const int32_t s = a.scores[o];
            for (int b = 0; b < 2; b++) {
                if (!((a.widths >> b) & 1)) continue;
                const int d = decide(a, b ? 16 : 8, s, len, gl < a.hmm_lanes ? a.hmm + gl : nullptr,
                                     gl < a.long_lanes);
                if (d < 0) undecided = true;
                else f |= (uint32_t)d << b;
            }
        }
        if (undecided) {
            // NW, ordinary penalties: which boundary chain first falls below the
            // threshold T = I_MIN - Q - R - 1 -- the left one (H(i,-1) = Q + (i+1)R,
            // met after ~4 i_L cells column by column) or the top one (H(-1,j) =
            // Q + (j+1)R, met after ~j_T cells row by row); the flag is almost
            // always decided where the first one crosses
            bool rows = false;
            if (a.nw && a.rlist && a.gap_extend < 0 && (a.ordinary & 2)) {
                const int w = (a.widths & 1) ? 8 : 16;
                const int64_t T = -(1ll << (w - 1)) - a.gap_open - a.gap_extend - 1;
                const int64_t Rm = -(int64_t)a.gap_extend;
                const int64_t cross = ((int64_t)a.gap_open - T) / Rm + 2;     // i_L ~ j_T
                const int64_t n4 = (len + 3) & ~3u, full = (int64_t)a.m * n4;
                const int64_t cost_col = a.m > cross ? 4 * cross : full;
                const int64_t cost_row = n4 > cross && n4 <= a.rstride ? cross : full;
                rows = cost_row * 16 < cost_col;
            }
            uint32_t* L = rows ? a.rlist : a.list;
            const uint32_t i = atomicAdd(L, 1u);
            L[1 + i] = gl;             // capacity: every lane
        } else if (!a.direct) {
            a.flags[o] = (uint8_t)f;
        }
    }
    if (a.direct) count_direct(a, undecided ? 0u : f);     // (whole waves: the shuffles need every lane)
}


// The lane's residue at column j (compact code) and its matrix row; columns
// past the end are the reference's code-0 padding.
struct LaneSeq {
    const uint8_t* base;
    uint32_t len;
    __device__ const int64_t* row(const FlagArgs& a, uint32_t j) const {
        if (j >= len) return a.padrow;
        return a.matrix + ((uint32_t)base[(size_t)(j >> 4) * 1024 + (j & 15)] << 5);
    }
};

// search_simd_nw.c:180-503 for one channel at w bits (oracle_nw_overflow)
__device__ int replay_nw(const FlagArgs& a, const LaneSeq& d, int w, int32_t* hep, uint32_t stride) {
    const int32_t IMIN = -(1 << (w - 1)), IMAX = (1 << (w - 1)) - 1;
    const int64_t Q = a.gap_open, R0 = a.gap_extend;
    const int32_t QR = trunc_w(Q + R0, w), R = trunc_w(R0, w);
    const int32_t T = trunc_w(IMIN - Q - R0 - 1, w);
    const uint32_t m = a.m;
    int32_t mge = QR;
    for (uint32_t i = 0; i < m; i++) {
        const int32_t h = sat_w(mge, IMIN, IMAX);
        hep[(size_t)(2 * i) * stride] = h;
        hep[(size_t)(2 * i + 1) * stride] = sat_w(h + QR, IMIN, IMAX);
        mge = sat_w(mge + R, IMIN, IMAX);
    }
    int32_t Ht[4], Ft[4];
    for (int k = 0; k < 4; k++) {
        Ht[k] = k == 0 ? 0 : trunc_w(Q + k * R0, w);
        Ft[k] = trunc_w(Q + (k + 1) * R0, w);
    }
    int32_t hmin = 0, hmax = 0, score = 0;
    const uint32_t nblocks = (d.len + 3) / 4;
    for (uint32_t b = 0; b < nblocks; b++) {
        int32_t h[4], f[4];
        const int64_t* row[4];
        for (int k = 0; k < 4; k++) {
            row[k] = d.row(a, 4 * b + k);
            h[k] = Ht[k];
            f[k] = sat_w(Ft[k] + QR, IMIN, IMAX);
        }
        for (uint32_t i = 0; i < m; i++) {
            const uint32_t qc = a.query[i];
            const int32_t h4 = hep[(size_t)(2 * i) * stride];
            int32_t E = hep[(size_t)(2 * i + 1) * stride], N[4];
            for (int k = 0; k < 4; k++) {
                int32_t H = sat_w(h[k] + trunc_w(row[k][qc], w), IMIN, IMAX);
                H = max(H, f[k]);
                H = max(H, E);
                hmin = min(hmin, H);
                hmax = max(hmax, H);
                N[k] = H;
                H = sat_w(H + QR, IMIN, IMAX);
                f[k] = max(sat_w(f[k] + R, IMIN, IMAX), H);
                E = max(sat_w(E + R, IMIN, IMAX), H);
            }
            hep[(size_t)(2 * i) * stride] = N[3];
            hep[(size_t)(2 * i + 1) * stride] = E;
            if (i + 1 == m && b + 1 == nblocks) score = N[(d.len + 3) % 4];
            h[0] = h4; h[1] = N[0]; h[2] = N[1]; h[3] = N[2];
            if (hmin < T || hmax == IMAX) return 1;     // decided: the flag is an OR
        }
        const int32_t F3 = Ft[3], H3 = Ht[3];
        Ft[0] = sat_w(F3 + R, IMIN, IMAX);
        Ft[1] = sat_w(Ft[0] + R, IMIN, IMAX);
        Ft[2] = sat_w(Ft[1] + R, IMIN, IMAX);
        Ft[3] = sat_w(Ft[2] + R, IMIN, IMAX);
        Ht[0] = sat_w(H3 + R, IMIN, IMAX);
        Ht[1] = sat_w(Ht[0] + R, IMIN, IMAX);
        Ht[2] = sat_w(Ht[1] + R, IMIN, IMAX);
        Ht[3] = sat_w(Ht[2] + R, IMIN, IMAX);
    }
    return score <= IMIN || score >= IMAX;
}

// search_simd_sw.c:172-441 for one channel at w bits (oracle_sw_overflow)
__device__ int replay_sw(const FlagArgs& a, const LaneSeq& d, int w, int32_t* hep, uint32_t stride) {
    const int32_t IMIN = -(1 << (w - 1)), IMAX = (1 << (w - 1)) - 1;
    const int32_t QR = trunc_w((int64_t)a.gap_open + a.gap_extend, w), R = trunc_w(a.gap_extend, w);
    const uint32_t m = a.m;
    for (uint32_t i = 0; i < 2 * m; i++) hep[(size_t)i * stride] = IMIN;
    int32_t S = IMIN;
    const uint32_t nblocks = (d.len + 3) / 4;
    for (uint32_t b = 0; b < nblocks; b++) {
        int32_t h[4], f[4];
        const int64_t* row[4];
        for (int k = 0; k < 4; k++) {
            row[k] = d.row(a, 4 * b + k);
            h[k] = IMIN;
            f[k] = IMIN;
        }
        for (uint32_t i = 0; i < m; i++) {
            const uint32_t qc = a.query[i];
            const int32_t h4 = hep[(size_t)(2 * i) * stride];
            int32_t E = hep[(size_t)(2 * i + 1) * stride], N[4];
            for (int k = 0; k < 4; k++) {
                int32_t H = sat_w(h[k] + trunc_w(row[k][qc], w), IMIN, IMAX);
                H = max(H, f[k]);
                H = max(H, E);
                S = max(S, H);
                N[k] = H;
                H = sat_w(H + QR, IMIN, IMAX);
                f[k] = max(sat_w(f[k] + R, IMIN, IMAX), H);
                E = max(sat_w(E + R, IMIN, IMAX), H);
            }
            hep[(size_t)(2 * i) * stride] = N[3];
            hep[(size_t)(2 * i + 1) * stride] = E;
            h[0] = h4; h[1] = N[0]; h[2] = N[1]; h[3] = N[2];
        }
        if (S == IMAX) return 1;
    }
    return 0;
}

// search_simd_nw.c's saturated w-bit NW recurrence for one channel, the same
// cell values as replay_nw but computed row by row (the DP is a function of
// each cell's neighbours; the processing order is free): boundaries are the
// reference's saturating chains -- H(-1, j-1) = 0, trunc(Q + jR) (j = 1..3),
// then +R; F into row 0 = sat(Ft(j) + Q + R), Ft(j) = trunc(Q + (j+1)R) (j <
// 4), then +R; H(i, -1) = QR, then +R; E into column 0 = H(i, -1) + QR.
// Scratch per lane: H(i-1, j) and F(i, j) for the entry's n4 columns.
__device__ int replay_nw_rows(const FlagArgs& a, const LaneSeq& d, int w, int32_t* hep, uint32_t stride) {
    const int32_t IMIN = -(1 << (w - 1)), IMAX = (1 << (w - 1)) - 1;
    const int64_t Q = a.gap_open, R0 = a.gap_extend;
    const int32_t QR = trunc_w(Q + R0, w), R = trunc_w(R0, w);
    const int32_t T = trunc_w(IMIN - Q - R0 - 1, w);
    const uint32_t m = a.m, n4 = (d.len + 3) & ~3u;
    int32_t score = 0;
    int32_t Lprev = 0;                                   // H(i-1, -1); row 0: H(-1,-1) = 0
    int32_t L = QR;                                      // H(i, -1)
    for (uint32_t i = 0; i < m; i++) {
        const uint32_t qc = a.query[i];
        int32_t diag = Lprev;                            // H(i-1, j-1) for j = 0
        int32_t E = sat_w(L + QR, IMIN, IMAX);           // E into column 0
        int32_t top = 0, Ft = 0;                         // row 0: H(-1, j-1) chain and Ft chain
        // the next column's profile value is fetched one column ahead
        int32_t vnext = trunc_w(d.row(a, 0)[qc], w);
        for (uint32_t j = 0; j < n4; j++) {
            const int32_t v = vnext;
            if (j + 1 < n4) vnext = trunc_w(d.row(a, j + 1)[qc], w);
            int32_t Fin, up;
            if (i == 0) {
                // H(-1, j) (the next column's diagonal) and F into row 0
                Ft = j < 4 ? trunc_w(Q + (int64_t)(j + 1) * R0, w) : sat_w(Ft + R, IMIN, IMAX);
                Fin = sat_w(Ft + QR, IMIN, IMAX);
                const uint32_t jn = j + 1;
                top = jn < 4 ? trunc_w(Q + (int64_t)jn * R0, w) : sat_w(top + R, IMIN, IMAX);
                up = top;
            } else {
                Fin = hep[(size_t)(2 * j + 1) * stride];
                up = hep[(size_t)(2 * j) * stride];
            }
            int32_t H = sat_w(diag + v, IMIN, IMAX);
            H = max(H, Fin);
            H = max(H, E);
            if (H < T || H == IMAX) return 1;            // decided: the flag is an OR
            if (i + 1 == m && j + 1 == d.len) score = H;
            const int32_t t = sat_w(H + QR, IMIN, IMAX);
            hep[(size_t)(2 * j + 1) * stride] = max(sat_w(Fin + R, IMIN, IMAX), t);
            hep[(size_t)(2 * j) * stride] = H;
            E = max(sat_w(E + R, IMIN, IMAX), t);
            diag = up;
        }
        Lprev = L;
        L = sat_w(L + R, IMIN, IMAX);
    }
    return score <= IMIN || score >= IMAX;
}

__global__ void __launch_bounds__(64) flags_replay_rows_kernel(const FlagArgs a) {
    const uint32_t n = *a.rlist;
    const uint32_t tid = blockIdx.x * 64 + threadIdx.x;
    int32_t* hep = a.rwork + tid;
    for (uint32_t i = tid; i < n; i += a.rthreads) {
        const uint32_t gl = a.rlist[1 + i];
        const uint32_t g = gl >> 6, lane = gl & 63;
        LaneSeq d{(const uint8_t*)a.res + (size_t)a.groups[g].blk * 1024 + lane * 16, a.lane_len[gl]};
        uint32_t f = 0;
        for (int b = 0; b < 2; b++) {
            if (!((a.widths >> b) & 1)) continue;
            f |= (uint32_t)replay_nw_rows(a, d, b ? 16 : 8, hep, a.rthreads) << b;
        }
        if (a.direct) {
            const unsigned long long c8 = a.bw == 8 ? (f & 1) : 0;
            const unsigned long long c16 = a.bw == 8 ? ((f & 1) & (f >> 1)) : ((f >> 1) & 1);
            if (c8) atomicAdd(&a.direct[0], c8);
            if (c16) atomicAdd(&a.direct[1], c16);
        } else {
            a.flags[a.lane_out[gl]] = (uint8_t)f;
        }
    }
}

__global__ void __launch_bounds__(64) flags_replay_kernel(const FlagArgs a) {
    const uint32_t n = *a.list;
    const uint32_t tid = blockIdx.x * 64 + threadIdx.x;
    int32_t* hep = a.work + tid;                       // row r at hep[r * threads]
    for (uint32_t i = tid; i < n; i += a.threads) {
        const uint32_t gl = a.list[1 + i];
        const uint32_t g = gl >> 6, lane = gl & 63;
        LaneSeq d{(const uint8_t*)a.res + (size_t)a.groups[g].blk * 1024 + lane * 16, a.lane_len[gl]};
        uint32_t f = 0;
        for (int b = 0; b < 2; b++) {
            if (!((a.widths >> b) & 1)) continue;
            const int w = b ? 16 : 8;
            const int x = a.nw ? replay_nw(a, d, w, hep, a.threads) : replay_sw(a, d, w, hep, a.threads);
            f |= (uint32_t)x << b;
        }
        if (a.direct) {
            const unsigned long long c8 = a.bw == 8 ? (f & 1) : 0;
            const unsigned long long c16 = a.bw == 8 ? ((f & 1) & (f >> 1)) : ((f >> 1) & 1);
            if (c8) atomicAdd(&a.direct[0], c8);
            if (c16) atomicAdd(&a.direct[1], c16);
        } else {
            a.flags[a.lane_out[gl]] = (uint8_t)f;
        }
    }
}

__global__ void __launch_bounds__(256) count_kernel(const CountArgs a) {
    const uint32_t e = blockIdx.x * 256 + threadIdx.x;
    unsigned long long c8 = 0, c16 = 0;
    if (e < a.entries) {
        uint32_t a8 = 0, a16 = 0;
        for (uint32_t v = 0; v < a.views; v++) {
            const uint32_t f = a.flags[(size_t)v * a.entries + e];
            a8 += f & 1;
            a16 += (f >> 1) & 1;
        }
        if (a.bw == 8) {
            c8 = a8;
            c16 = (unsigned long long)a8 * a16;
        } else {
            c16 = a16;
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        c8 += __shfl_xor(c8, o);
        c16 += __shfl_xor(c16, o);
    }
    if ((threadIdx.x & 63) == 0) {
        if (c8) atomicAdd(&a.out[0], c8);
        if (c16) atomicAdd(&a.out[1], c16);
    }
}

}  // namespace

hipError_t launch_flags(const FlagArgs& a, hipStream_t st) {
    if (a.nlanes == 0) return hipSuccess;
    hipError_t e = hipSuccess;
    if (!a.lists_zeroed) {
        if ((e = op_set(a.list, 0, 4, st)) != hipSuccess) return e;
        if (a.rlist && (e = op_set(a.rlist, 0, 4, st)) != hipSuccess) return e;
    }
    if (a.entries > 0) (void)ssa_launch((const void*)&flags_decide_kernel, dim3((a.entries + 255) / 256), dim3(256), 0, st, a);
    if (a.m > 0) (void)ssa_launch((const void*)&flags_replay_kernel, dim3(a.threads / 64), dim3(64), 0, st, a);
    if (a.m > 0 && a.rlist) (void)ssa_launch((const void*)&flags_replay_rows_kernel, dim3(a.rthreads / 64), dim3(64), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_count(const CountArgs& a, hipStream_t st) {
    if (a.entries == 0) return hipSuccess;
    (void)ssa_launch((const void*)&count_kernel, dim3((a.entries + 255) / 256), dim3(256), 0, st, a);
    return hipGetLastError();
}

}  // namespace ssa
