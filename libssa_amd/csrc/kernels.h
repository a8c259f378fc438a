// kernels.h -- argument blocks of the HIP kernels (kernels.hip, counters.hip,
// pair_kernel.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "launch.h"

namespace ssa {

constexpr int kWaves = 4;          // waves (= 64-sequence groups) per workgroup
constexpr int kPairWaves = 4;      // waves per pair_kernel workgroup (they share one pair table)
constexpr size_t kPairLdsMax = 160 * 1024;  // pair table budget: one workgroup per CU (47 KiB for 20-letter proteins: 3)

// The pair kernel's LDS table holds the residue pairs (current c1, previous
// c0) a column after column 0 can meet: c0 a real code (c1 any, padding
// included) and (pad, pad) -- a padding column is followed only by padding,
// and (c1, pad) with c1 real occurs only at column 0, whose operand the
// kernel reads from the global table instead.  (A + 1) A + 1 rows for A real
// codes instead of (A + 1)^2: 421 for 20 letters, 463 for 21.
__host__ __device__ constexpr uint32_t pair_lds_rows(uint32_t A) { return (A + 1) * A + 1; }
__host__ __device__ constexpr uint32_t pair_lds_row(uint32_t A, uint32_t c1, uint32_t c0) {
    return c0 < A ? c1 * A + c0 : (A + 1) * A;
}
// Workgroups of `bytes` dynamic LDS that one gfx950 CU keeps resident (LDS
// alone): allocations are rounded up to 1 280 B (measured, tools/ubench/
// lds_occ.hip, profiles/r05/lds_occ.txt: 40 960 B -> 4, 53 760 B -> 3,
// 54 208 B -> 2, 75 776 B -> 2 -- 160 KiB / 3 = 54 613 B is not reachable).
// gfx950's granule: the library holds gfx950 code only and refuses any other
// device at its first use of it (engine.cpp upload_pack), so the plan never
// meets another architecture's allocation rule.
constexpr size_t kLdsGranule = 1280;
constexpr size_t pair_wgs_per_cu(size_t bytes) {
    return bytes == 0 ? 4 : kPairLdsMax / ((bytes + kLdsGranule - 1) / kLdsGranule * kLdsGranule);
}
constexpr int kF16Floor = 0x0800;  // pattern of the SW zero in strip_f16m_kernel

// pair_kernel tail strips of 2*npt rows: npt a multiple of 4, or of 2 for the
// default strip heights (SW 48 rows, NW 64/80) after at least one main strip
// -- the tail's table then has a padded global pitch of round4(npt) dwords
__host__ __device__ constexpr bool pair_tail_fine(int np, bool nw) { return nw ? (np == 32 || np == 40) : np == 24; }
__host__ __device__ constexpr uint32_t pair_tail_pitch(uint32_t npt) { return (npt + 3) & ~3u; }

constexpr int kMaxFuse = 16;       // queries one pair_kernel launch may score (StripArgs::nq)

struct GroupDesc {
    uint32_t blk;     // residue offset in 1 KiB blocks (16 columns x 64 lanes)
    uint32_t ncols;   // columns to compute: multiple of 4, >= longest + 1 (blocks: ceil(ncols/16))
};

struct StripArgs {
    const uint4* res;          // packed residues
    uint4* rowbuf;             // strip boundary buffer (4 B per lane and column)
    const GroupDesc* groups;
    const uint32_t* lane_len;  // [ngroups * 64]
    const uint32_t* lane_out;  // [ngroups * 64] dense output index
    const uint32_t* qpt;       // [nstrips][32][np] packed query profile
    int32_t* scores;           // [entries]
    uint32_t* ovf_list;        // lanes that need the exact int64 re-score
    uint32_t* ovf_count;
    uint32_t ngroups, nstrips, m;
    int32_t gap_open, gap_extend;
    uint32_t nmax16;           // longest DB entry proven int16-safe
    uint32_t ovf_cap;          // capacity of ovf_list
    uint32_t pad_word;         // profile dword of the padding residue (both halves)
    uint32_t alpha;            // compact alphabet size; code alpha = padding column
    uint32_t nw_base;          // NW pattern offset of pair_kernel (value + nw_base)
    // pair_kernel: the tail strip's table (launch_pair's npt > 0)
    const uint32_t* qpt_tail;
    // pair_kernel: top boundary of the first strip, (H(-1,j), F into row 0)
    // as diagonal-relative patterns in row-buffer quads, the same for every
    // lane ([ceil(max ncols / 4)] uint4)
    const uint4* top;
    // pair_kernel: first group it scores (groups before it go to long_kernel)
    uint32_t g_first;
    // pair_kernel: groups [g_first, g_prio) issue at raised wave priority --
    // the longest groups, which set the launch's critical path when the DB
    // fills the chip only a few times over (engine.cpp device_search)
    uint32_t g_prio;
    // wave timeline (option "timeline", ssa_amd_get_timeline): per pair-kernel
    // group g - g_first, (g, start, end, place) -- s_memrealtime ticks
    // (100 MHz) and (XCC << 16 | HW_ID & 0xffff); null: off
    uint4* timeline;
    // pair_kernel: workgroup -> groups by a start-order ticket (an atomic
    // counter the tables kernel zeroes) instead of blockIdx: the workgroups'
    // XCD is fixed by blockIdx round robin, so with blockIdx order a slower
    // XCD still gets an equal share; tickets hand the next-longest groups to
    // whichever workgroup starts next on any XCD.  Null: blockIdx order.
    uint32_t* ticket;
    // pair_kernel: each group's strips in `nparts` consecutive parts of
    // `part_strips` strips (the tail strip counts as one), run as separate
    // work units: unit u = part (u / nquads) of quad (u % nquads), so the
    // units of all groups' first parts come first (longest groups first),
    // then all second parts.  A part waits until its group's previous part
    // is done (part_done[quad]); the handoff boundary crosses workgroups,
    // maybe XCDs, through device-scope stores, and part p keeps its own
    // boundaries in its own buffer -- rowbuf (part 0), rowbuf2, rowbuf3 --
    // so no buffer is written from two XCDs (pair_kernel.h store_row: the
    // coherence argument; at most 3 parts); the SW running maximum travels in
    // part_smax (one dword per lane).  The launch's last units are then
    // the shortest groups' last parts -- a fraction of a whole group's work
    // -- so the SIMDs drain closer together.
    // nparts 1: whole groups, no carry.
    uint32_t nparts, part_strips, nquads;
    // only quads [split_q0, split_q1) are split (the others run whole as
    // units 0 .. nquads-1 like part 0): units nquads .. are the later parts
    // of the split quads, part by part
    uint32_t split_q0, split_q1;
    uint32_t* part_done;       // [nquads] part_epoch + q once the quad's part q is done (never cleared)
    uint32_t part_epoch;       // this launch's flag base: a multiple of 4, above every earlier launch's values
    uint32_t* part_smax;       // [ngroups * 64]
    uint32_t* part_err;        // set when a wait timed out (the host then runs the search again without parts)
    uint32_t part_wait;        // bound of that wait, s_memrealtime ticks (100 MHz)
    uint4* rowbuf2;            // part 1's own strip boundaries (same layout as rowbuf)
    uint4* rowbuf3;            // part 2's (nparts 3)
    // pair_kernel: several queries of one plan in one launch (a batch of
    // short queries, ssa_amd_search_batch): unit order part, quad (longest
    // first), query; query qi reads its tables at qpt / qpt_tail + qi *
    // q_tab_stride and writes scores / overflow list / row buffer at the
    // strides below.  Parts and strip counts are the same for every query;
    // its row count is qm[qi] (device memory: a select chain over an array
    // in the argument block measured 2.5 % slower on C2 -- register
    // allocation).  nq 0/1: one query (a.m).
    uint32_t nq;
    const uint32_t* qm;
    size_t q_tab_stride, q_score_stride, q_ovf_stride, q_rowbuf_stride;
    // pair_kernel: the pair-row stream (pair_addr_kernel), the LDS offset of
    // each column's next pair row in 16-byte units, 16 bits per column, in
    // octs of 8 columns (2 KiB per residue block), built for this launch's
    // table row width ((NP + 4) dwords, or (NPT + 4) when nstrips = 0) and
    // code count
    const uint4* paddr;
};

// Long DB entries (long_kernel): the query rows split over the lanes of W
// waves (RL consecutive rows per lane, passes of W*64*RL rows), DB columns
// swept as a lane-skewed wavefront; exact int32 arithmetic.  Serves the
// entries of the first nseq/64 (longest) groups, which pair_kernel then
// skips (StripArgs::g_first).
struct LongArgs {
    const uint4* res;
    const GroupDesc* groups;
    const uint32_t* lane_len;
    const uint32_t* lane_out;
    const uint8_t* query;      // [m]
    const int64_t* matrix;     // [1024] compact code x query code
    int32_t* scores;
    int64_t* scratch;          // [nseq][stride] (H, F) of a pass's last row (multi-pass only)
    uint32_t stride;
    uint32_t seq0, nseq;       // entries served: lanes [seq0, seq0 + nseq) of the group order
    uint32_t* gate;            // every workgroup increments it when it starts (TableArgs::gate)
    int2* hmm;                 // NW: per lane (min, max) of H over the entry's real cells, or null
                               // (the overflow counters' exact decision, counters.hip)
    uint32_t m, alpha;
    int32_t gap_open, gap_extend;
    uint4* timeline;           // per entry s: (0x80000000 | s, start, end, place), like StripArgs
    // dynamic LDS of a workgroup at least this: the concurrent pair kernel's
    // (engine.cpp), so the hole a finished long workgroup leaves in a CU's
    // LDS takes a pair workgroup (allocations are contiguous: a smaller hole
    // beside the pair workgroups' would stay empty until one of those ends)
    uint32_t lds_min;
    // long16_kernel (SW on 16-bit patterns): pattern of score 0, and the
    // padding profile value (int16 in the low half)
    uint32_t base16, pad16;
    // long16_kernel: the query's last extra16 rows are not in any pass (m -
    // extra16 is a whole number of 64 x RL-row passes); the wave scores them
    // one row at a time after its passes (a prefix maximum over 64 columns
    // per step, kernels.hip long16_rows), from the last pass's bottom row
    uint32_t extra16;
    uint32_t low_prio;         // long16_kernel: 1 = no raised wave priority (option "long_prio" 0)
    // long_kernel (W = 1) as the exact int32 re-score tier of the DP kernels'
    // overflowed lanes (engine.cpp): when `list` is set the entries are the
    // lanes list[0 .. min(*list_count, nseq)), in a grid of `blocks`
    // workgroups that loops over them; entry i's exact score goes to
    // list_out[i] (the int64 slot wide_kernel would fill), its multi-pass
    // scratch row is its wave's slot
    const uint32_t* list;
    const uint32_t* list_count;
    int64_t* list_out;
    uint32_t blocks;
    // (list mode) block 0 clears these as wide_kernel would (WideArgs::zero,
    // zero2): the tier replaces its launch
    uint32_t* zero;
    uint32_t nzero;
    uint32_t* zero2[2];
};
constexpr int kLongWaves = 4;

struct WideArgs {
    const uint4* res;
    const GroupDesc* groups;
    const uint32_t* lane_len;
    const uint32_t* ovf_list;
    const uint32_t* ovf_count;
    const uint8_t* query;      // [m]
    const int64_t* matrix;     // [1024]
    int64_t* work;             // [threads][2m]
    int64_t* wide_scores;      // [ovf_count]
    uint32_t m;
    int32_t gap_open, gap_extend;
    int32_t nw;
    uint32_t ovf_cap;
    uint32_t* zero;            // nzero dwords cleared by block 0 (the next filter pass's counters)
    uint32_t nzero;
    uint32_t* zero2[2];        // and these two dwords (the overflow-flag replay lists' counts), if set
};

// Device-side top-k candidate filter (single query view, k <= kFilterMaxK).
// Every entry gets a lower bound of the reference heap's root at the time
// it is offered (k-th largest of maxima of earlier 64-entry runs, see
// kernels.hip); only entries above it (or overflowed, INT32_MIN) can change
// the heap.  They are compacted into cand[] for the host replay.
constexpr int kFilterBlock = 4096;
constexpr int kFilterMaxK = 64;
constexpr int kFilterMaxViews = 12;   // query views one filter pass covers
constexpr int kFilterHeader = 16;     // dwords before the candidates in the counters buffer
struct FilterArgs {
    const int32_t* scores;     // per-entry scores, INT32_MIN = overflowed (exact value elsewhere)
    const uint32_t* order;     // [n] score index of insertion position p (null: identity) -- the
                               // chunk-interleaved order of multi-view searches
    uint32_t n, k, nblocks;
    int32_t* summary;          // [nblocks][kFilterMaxK] top-k mini maxima per block, descending
    int32_t* thresh;           // [nblocks] bound from earlier blocks
    int32_t* thresh_local;     // [nblocks * 64] bound from earlier minis of the same block
    int32_t* before;           // [nblocks][kFilterMaxK] scan scratch
    const uint32_t* ovf_count; // view v's count at ovf_count[v * ovf_stride], copied into counters[3 + v]
    uint32_t ovf_stride, nviews;
    uint32_t* counters;        // [0] candidates, [2] *status, [3 + v] overflowed lanes of view v
                               // (one host copy fetches everything)
    const uint32_t* status;    // the pair launch's strip-part wait status word (copied into
                               // counters[2]: no separate read-back); null: none
    uint2* cand;               // [n] (insertion position, score) of the candidates, unordered;
                               // at counters + kFilterHeader
    // several independent queries in one pass (a fused batch): blockIdx.y =
    // query q reads scores + q * q_scores and ovf_count + q * q_ovf, writes
    // counters (and cand) + q * q_counters, and uses the q-th nblocks-sized
    // slice of the scratch arrays.  nq 0/1: one.
    uint32_t nq;
    size_t q_scores, q_ovf, q_counters;
    // single pass (nq <= 1): the result straight into pinned host memory
    // instead of a D2H copy -- the last filter_select block to finish (done:
    // a device word, 0 between searches, reset by that block) writes header
    // words 0..14 and the first host_cap candidates to host_out, then
    // host_seq into host_out[kFilterSeqWord] at system scope (the host spins
    // on that word).  host_out null: none.
    uint32_t* host_out;
    uint32_t host_cap;
    uint32_t host_seq;
    uint32_t* done;
    uint32_t host_fence;       // 1: system-scope release before the sequence word (an L2 writeback);
                               // 0: system-scope relaxed stores, each thread waits for its own
                               // stores' completion before the block's barrier and the sequence word;
                               // 2: plain stores, no ordering (the host synchronises with the stream)
    // rare-code merge (single pass, identity order): an entry whose codes
    // (emask[e]) meet merge_mask holds an UPPER BOUND of its score (the
    // merged class scores the maximum of its members).  It is left out of
    // the maxima like an overflowed entry; when forwarded, its lane
    // (entry_lane[e].y) is appended to exact_lanes (count: counters[1]) for
    // the exact re-score.  emask null: none.
    const uint32_t* emask;
    uint32_t merge_mask;
    const uint2* entry_lane;
    uint32_t* exact_lanes;
    uint32_t exact_lane0;      // lanes below it (the long-entry kernels') are scored exactly anyway
    // one pass (filter_onepass): the three steps in one launch.  Blocks take
    // their block index from a start-order ticket (pass[2q]) and chain the
    // prefix by a decoupled look-back through summary, read as 8-byte words
    // [nq][nblocks][kFilterMaxK] (the allocation is sized for them): per lane
    // (1 << 31 | epoch << 2 | 1 aggregate / 2 inclusive) << 32 | list element
    // (epoch < 2^29) -- stale
    // epochs read as not ready, so nothing is cleared between searches; the
    // last block to finish (pass[2q + 1]) resets both pass words.  pass
    // null: the three launches.
    uint32_t* pass;
    uint32_t epoch;
};
constexpr int kFilterSeqWord = 15;    // header word that carries FilterArgs::host_seq
hipError_t launch_filter(const FilterArgs& a, hipStream_t st);


hipError_t launch_strip16(const StripArgs& a, int np, bool nw, hipStream_t st);
hipError_t launch_sw_f16(const StripArgs& a, int np, hipStream_t st);
// a.nstrips strips of 2*np rows, then one of 2*npt rows (npt 0: none;
// required for NW, whose score is captured in the last strip)
// occ: when set, nothing is launched -- *occ receives the kernel's resident
// workgroups per CU at lds_bytes (hipOccupancyMaxActiveBlocksPerMultiprocessor)
hipError_t launch_pair(const StripArgs& a, int np, int npt, bool nw, size_t lds_bytes, hipStream_t st,
                       int* occ = nullptr);
hipError_t launch_wide(const WideArgs& a, uint32_t threads, hipStream_t st);
// rl: rows per lane (4, 8, 12 or 16; 64*rl rows per pass)
// w: waves per entry (1: four entries per workgroup; 4: one entry, its
// rows over the workgroup's waves); rl: rows per lane (w 1: 4, 8, 12 or 16;
// w 4: 2 or 4); w * 64 * rl rows per pass
hipError_t launch_long(const LongArgs& a, int w, int rl, bool nw, hipStream_t st);
size_t long_lds_bytes(uint32_t alpha, int w, int rl);
// SW long entries on packed 16-bit patterns, one wave per entry; rl (rows
// per lane) 4, 6, 8, 10, 12 or 16, 64*rl rows per pass
hipError_t launch_long16(const LongArgs& a, int rl, hipStream_t st);
// filter_prefix with the scan states in registers for DBs of <= 256 filter
// blocks (1, default) or always the general kernel (0; option "filter_prefix_regs")
void set_filter_prefix_regs(int on);
size_t long16_lds_bytes(uint32_t alpha, int rl);

// The reference's 8/16-bit overflow counters (counters.hip).  m_run reports
// how many (query view, DB sequence) pairs its w-bit SIMD kernels sent on to
// the next width (manager.c:157-160, search_8.c:94-124, search_16.c:92-114);
// the scores here are exact at every width, so whether the reference's
// saturated w-bit run would have overflowed is decided per lane: from the
// exact score and bounds where that is provable (flags_decide_kernel), else
// by replaying the reference's saturated w-bit recurrence for that lane
// (flags_replay_kernel).  Per (view, entry) flag byte: bit 0 = 8-bit
// overflow, bit 1 = 16-bit overflow.
struct FlagArgs {
    const uint4* res;
    const GroupDesc* groups;
    const uint32_t* lane_len;
    const uint32_t* lane_out;
    const uint2* entry_lane;   // [entries] (length, lane) in entry order
    uint32_t entries;
    const int32_t* scores;     // this view's exact scores (INT32_MIN: value elsewhere -> replay)
    const uint8_t* query;      // [m]
    const int64_t* matrix;     // [1024] compact code x query code
    const int64_t* padrow;     // [32] M[0][y]: the reference pads a sequence to 4 columns with code 0
    uint8_t* flags;            // this view's [entries]
    uint32_t* list;            // [0] count, [1..nlanes] lanes left to the replay (column-major)
    int32_t* work;             // replay scratch, [2m][threads] (thread-interleaved)
    uint32_t nlanes, m, threads;
    // NW lanes whose top boundary crosses the flag threshold within the
    // entry (entries of ~16 k+ residues at 16 bits): row-major replay, which
    // meets the flagging cell within the first row instead of m x that
    uint32_t* rlist;           // [0] count, [1..nlanes] lanes
    int32_t* rwork;            // [2 rstride][rthreads]
    uint32_t rstride, rthreads;
    int32_t gap_open, gap_extend;
    int32_t nw;
    int32_t widths;            // bit 0: 8-bit flags wanted, bit 1: 16-bit
    int32_t ordinary;          // bit 0/1: 8/16-bit decidable from exact values (host-checked regime)
    int32_t maxm;              // max(0, M over the DB's codes and code 0 x the query's residues)
    int32_t padmax;            // max(0, max_i M[0][q_i])
    // NW lanes [0, hmm_lanes) scored by long_kernel: exact (min, max) of H
    const int2* hmm;
    uint32_t hmm_lanes;
    uint32_t long_lanes;       // lanes [0, long_lanes) were scored by long_kernel
    int32_t nw_hmax16_ok;      // NW: the other lanes' kernel kept every H below 32767
    // single-view searches: the two counters are summed here directly (width
    // 8: o8 += f8, o16 += f8 * f16; width 16: o16 += f16) and no count pass
    // follows; null: flags only (multi-view, CountArgs)
    unsigned long long* direct;
    int32_t bw;
    int32_t lists_zeroed;      // list counts were cleared by the wide kernel (WideArgs::zero2)
};
hipError_t launch_flags(const FlagArgs& a, hipStream_t st);

// counters of one search: out[0] += sum_e a8(e), out[1] += width 8 ?
// sum_e a8(e) * a16(e) : sum_e a16(e), a_w(e) = #views whose flag w is set
// (oracle_overflow_counts restates it)
struct CountArgs {
    const uint8_t* flags;      // [views][entries]
    uint32_t entries, views;
    int32_t bw;
    unsigned long long* out;   // [2]
};
hipError_t launch_count(const CountArgs& a, hipStream_t st);

// Residue recode (per-query residue classes, engine.cpp device_search):
// out byte = map[in byte] over n16 16-byte words of the packed layout.
struct RecodeArgs {
    const uint4* in;
    uint4* out;
    size_t n16;
    uint8_t map[64];
};
hipError_t launch_recode(const RecodeArgs& a, hipStream_t st);

// pair_kernel's strips read, per column j, the LDS byte offset of the
// pair row of column j+1, (d_{j+1} * prow + d_j) * row_bytes, from this
// stream instead of forming it from the residue bytes (two 24-bit
// multiplies and an add per column, ~3 % of the strip's issue time).  The
// offset is stored in 16-byte units in 16 bits (every table row is 16-byte
// aligned and the LDS holds at most 160 KiB): per residue block,
// [oct][lane][8 columns] (2 KiB, half the row buffer's block) -- a shift per
// column in the kernel for half the stream's HBM traffic; the column after
// a group's last one takes the padding code.
struct PairAddrArgs {
    const uint4* res;          // residue blocks (compact or class codes)
    uint4* out;                // [blocks * 256] uint4
    const GroupDesc* groups;
    uint32_t ngroups;
    uint32_t prow;             // codes + 1 (the padding code is prow - 1)
    uint32_t row_bytes;        // table row stride: (NP + 4) * 4, or (NPT + 4) * 4 without main strips
};
hipError_t launch_pair_addr(const PairAddrArgs& a, hipStream_t st);

// Per DB entry, the set of compact residue codes it holds (bit c: code c
// occurs), from the packed residue blocks: one wave per group, one lane per
// entry (engine.cpp: the rare-code merge's flags).
struct EntryMaskArgs {
    const uint4* res;          // residue blocks, compact codes
    const GroupDesc* groups;
    const uint32_t* lane_out;  // lane -> entry (0xffffffff: padding lane)
    uint32_t ngroups;
    uint32_t pad;              // the padding code (not reported)
    uint32_t* out;             // [entries]
};
hipError_t launch_entry_mask(const EntryMaskArgs& a, hipStream_t st);

// pair_kernel's per-search pair tables, built on the device from the query
// and the compact-code matrix: main strips (count x (alpha+1)^2 x np dwords)
// then the tail strip ((alpha+1)^2 x npt dwords).  Dword (c1*(alpha+1)+c0, r)
// of a strip from row i0 = (P(c1, i0+r), P(c0, i0+np+r)), P(c, i) =
// clamp16(M[c][q_i] + rel) for a real code and row, pad otherwise.
struct TableArgs {
    const uint8_t* query;      // [m] query codes
    const int64_t* matrix;     // [1024] compact-code matrix (x = DB code)
    uint32_t* out;             // main tables, then the tail table
    uint32_t m, alpha;
    uint32_t np, nmain;        // main strip half-height and count
    uint32_t npt, tail_row0;   // tail strip half-height (0: none) and first row
    int32_t rel;               // added to every real profile value (-2R)
    uint32_t pad;              // 16-bit padding value
    uint32_t* zero;            // cleared by thread 0 (the search's overflow count), may be null
    // dispatch gate (null: none): block 0 waits, bounded, until gate_target
    // long_kernel workgroups have started, so the pair kernel that follows
    // on the stream cannot fill the CUs before the long entries are placed
    const uint32_t* gate;
    uint32_t gate_target;
    uint32_t* zero_ticket;     // StripArgs::ticket, cleared by thread 0 (may be null)
    uint32_t* zero_hdr;        // nzero_hdr dwords cleared by block 0 (the filter pass's counters,
    uint32_t nzero_hdr;        // when the re-score tier runs beside the filter instead of before it)
};
hipError_t launch_pair_tables(const TableArgs& a, hipStream_t st);
// dst (device) <- src (pinned host), bytes a multiple of 4: a kernel on st
hipError_t launch_upload(void* dst, const void* src, size_t bytes, hipStream_t st);

}  // namespace ssa
