// engine.h -- device-resident packed DB and the per-device search.
#pragma once
#include <hip/hip_runtime.h>

#include <memory>
#include <unordered_map>
#include <vector>

#include "common.h"
#include "kernels.h"

namespace ssa {

// One DB "entry" = one scored sequence: a non-empty DB record, or one of its
// strands (NUCLEOTIDE with the complementary strand) -- the reference's
// sdb_sequence_t (libssa_datatypes.h:88-96, db_adapter.c:47-110).
struct EntryMeta {
    std::vector<uint64_t> id;       // local record ID per entry (ascending)
    std::vector<uint8_t> strand;
    std::vector<uint8_t> frame;
    std::vector<uint32_t> len;
    uint64_t residues = 0;
    size_t records = 0;             // IDs the plugin handed out
    size_t size() const { return id.size(); }
};

struct PlanCache;   // engine.cpp: plan_view results of the last queries

struct DeviceDB {
    int device = -1;
    uint64_t generation = ~0ull;
    int symtype = -1, strands = -1, dgencode = -1;
    hipStream_t stream = nullptr;
    hipEvent_t ev[9] = {};                // [8]: the int32 tier's end when it runs beside the filter
    hipEvent_t ev_fork = nullptr;         // a recorded search's fork to the long-entry streams
    // graph-eligible searches' stream operations as instantiated HIP graphs
    // (engine.cpp run_ops), a few launch plans at once (least recently used
    // replaced): a search whose operations have the shape of a cached graph's
    // replays it with its changed arguments set on the nodes
    struct SearchGraph {
        hipGraph_t g = nullptr;
        hipGraphExec_t exec = nullptr;
        std::vector<StreamOp> ops;
        std::vector<hipGraphNode_t> nodes;   // per op: its node (kernels, copies, sets)
        uint64_t used = 0;
        void reset();
    };
    static constexpr size_t kGraphs = 8;
    struct SearchGraphs {
        SearchGraph slot[kGraphs];
        bool broken = false;                 // a capture or instantiation failed: call by call from then on
        uint64_t clock = 0;
        void reset() {
            for (auto& x : slot) x.reset();
        }
    } graph;
    EntryMeta meta;
    uint32_t ngroups = 0;
    uint64_t nblocks = 0;                 // 1 KiB residue blocks
    GroupDesc* d_groups = nullptr;
    uint4* d_res = nullptr;
    uint4* d_rowbuf = nullptr;
    uint32_t* d_lane_len = nullptr;
    uint32_t* d_lane_out = nullptr;
    // top-k candidate filter (kernels.h FilterArgs)
    uint32_t* d_fbuf = nullptr;           // [4] counters, then (index, score) x entries
    int32_t* d_summary = nullptr;
    int32_t* d_before = nullptr;
    int32_t* d_thresh = nullptr;
    int32_t* d_thresh_local = nullptr;
    uint32_t* h_fbuf = nullptr;           // pinned: counters + h_cand_cap candidates
    size_t h_cand_cap = 0;
    size_t cand_first = 0;                // candidates the last single-view search copied with its counters
    uint32_t cand_hint = 0;               // the last single-view search's candidate count (sizes that copy)
    uint8_t* h_up = nullptr;              // pinned staging for per-search uploads
    size_t h_up_cap = 0;
    int32_t* d_scores = nullptr;
    int32_t* h_scores = nullptr;          // pinned, [views][entries]
    size_t h_scores_cap = 0;
    // overflow lists: per view slice [0] = count, [1..lanes] = lanes to re-score
    // exactly (room for every lane: no cap), their int64 scores in d_wide
    uint32_t* d_ovf = nullptr;
    int64_t* d_wide = nullptr;
    size_t ovf_slices = 0;                // view slices d_ovf / d_wide hold
    uint32_t* h_ovf = nullptr;            // pinned, kOvfPinned + 1
    int64_t* h_wide = nullptr;            // pinned, kOvfPinned
    uint32_t* d_qpt = nullptr;
    size_t qpt_cap = 0;
    size_t scores_cap = 0;                // d_scores entries
    size_t filter_cap = 0;                // entries the filter buffers cover
    size_t filter_blocks_cap = 0;         // 4096-entry blocks the filter scratch covers
    // multi-view searches: insertion order of (view, entry) scores for the
    // device filter (search_64.c:44-56 chunk interleave), device and host
    uint32_t* d_order = nullptr;
    std::vector<uint32_t> h_order;
    uint64_t order_key = ~0ull;
    std::vector<hipEvent_t> vev;          // per-view kernel start/end events
    size_t fbuf_bytes = 0;                // d_fbuf capacity
    size_t h_fbuf_regions = 1;            // pinned h_fbuf regions (one per pipelined query)
    // per-search uploads in one device block (one H2D copy): the compact-code
    // matrix, the pair kernel's first-strip boundary quads, the query codes;
    // d_matrix / d_top / d_query point into it (not separately owned)
    uint8_t* d_upblk = nullptr;
    size_t upblk_cap = 0;
    uint32_t* d_top = nullptr;
    // SW's first-strip boundary depends only on R and the longest group: kept
    // on the device (d_topc, key topc_key) instead of built and uploaded per
    // search (140 KB for a 35 k-residue entry); d_top then points here
    uint32_t* d_topc = nullptr;
    size_t topc_cap = 0;
    uint64_t topc_key = ~0ull;
    uint8_t* d_query = nullptr;
    int64_t* d_matrix = nullptr;
    int64_t* d_work = nullptr;
    size_t work_cap = 0;
    // the reference's 8/16-bit overflow counters (counters.hip): per (view,
    // entry) flags, the replay's lane list, per-query (o8, o16) sums
    uint8_t* d_flags = nullptr;
    size_t flags_cap = 0;
    uint32_t* d_flist = nullptr;          // [0] count, then up to ngroups * 64 lanes
    uint32_t* d_frlist = nullptr;         // the same for the row-major NW replay
    int32_t* d_frwork = nullptr;          // its scratch
    size_t frwork_cap = 0;                // int32 elements
    int2* d_hmm = nullptr;                // NW long entries: exact (min, max) of H per lane
    uint4* d_timeline = nullptr;          // option "timeline": [long lanes][pair groups] wave rows
    size_t timeline_cap = 0, timeline_rows = 0;
    uint32_t* d_entry_lane = nullptr;     // [entries] (length, lane) in entry order
    // rare-code merge (engine.cpp plan_view): per entry the
    // compact codes it holds, and per compact code the entries holding it
    // (computed on first use; empty: not yet)
    uint32_t* d_emask = nullptr;
    std::vector<uint64_t> code_entries;
    // the exact re-score of forwarded merged-code entries: lanes [exact_cap],
    // then their int64 scores; pinned mirror of the first kExactPinned of each
    uint32_t* d_exact = nullptr;
    size_t exact_cap = 0;
    uint8_t* h_exact = nullptr;
    size_t hmm_cap = 0;                   // lanes
    unsigned long long* d_cnt = nullptr;  // [kMaxBatchPipe][2]
    unsigned long long* h_cnt = nullptr;  // pinned mirror (+ 16 B: the gate block's error word)
    // pair_kernel strip parts (StripArgs::nparts): per quad parts done, per lane running maxima
    uint32_t* d_part = nullptr;
    size_t part_cap = 0;
    uint32_t part_epoch = 0;              // the last pair launch's handoff flag value (StripArgs::part_epoch)
    // the long-entry dispatch gate (d_cnt's gate word) is never cleared per
    // search: it counts every long workgroup launched since d_cnt was last
    // zeroed, and the tables kernel waits for this search's share above
    // gate_count.  cnt_dirty: zero the whole block before the next search
    // (fresh memory, or a strip part's wait-timeout word was raised)
    uint32_t gate_count = 0;
    // the largest overflow list of the last search: sizes the re-score tier's
    // grid (a hint only -- the tier loops over any list length)
    uint32_t tier_hint = 0;
    bool cnt_dirty = true;
    uint32_t filter_seq = 0;              // the last FilterArgs::host_seq (never 0)
    uint32_t filter_epoch = 0;            // the last FilterArgs::epoch (one-pass filter)
    uint32_t* d_smax = nullptr;
    size_t smax_cap = 0;
    uint4* d_rowbuf2 = nullptr;           // part 1's row buffer (StripArgs::rowbuf2), as d_rowbuf
    uint4* d_rowbuf3 = nullptr;           // part 2's (StripArgs::rowbuf3; three parts only)
    // fused batches (StripArgs::nq): one row buffer per query
    uint8_t* d_rowbuf_q = nullptr;
    size_t rowbuf_q_cap = 0;
    // long entries (long_kernel, launched on stream_long beside the pair
    // kernel): the groups' column counts (longest first), their sum, the
    // device's SIMD count, the multi-pass scratch
    std::vector<uint32_t> group_ncols;
    uint64_t ncols_sum = 0;
    uint32_t nsimd = 1024;
    hipStream_t stream_long = nullptr;    // long_kernel, 4 waves per entry (event ev[7])
    hipStream_t stream_long1 = nullptr;   // long_kernel, 1 wave per entry (event ev[6])
    int64_t* d_lscratch = nullptr;
    size_t lscratch_cap = 0;              // int64 elements
    int64_t* d_rscratch = nullptr;        // the int32 re-score tier's multi-pass rows (LongArgs::list)
    size_t rscratch_cap = 0;              // int64 elements
    std::vector<uint32_t> lane_out;       // host copy for overflow mapping
    std::vector<uint32_t> len_sorted;     // entry lengths, ascending
    // residues are stored in a compact alphabet: device code c < alpha stands
    // for residue code code_of[c]; code alpha is the padding column
    std::vector<uint8_t> code_of;
    uint32_t alpha = 0;
    // per-query residue classes (device_search): class-coded copy of d_res
    // and the class map it was made with
    uint4* d_res_cls = nullptr;
    std::vector<uint8_t> cls_key;
    // pair_kernel's pair-row streams (StripArgs::paddr, as d_rowbuf) and
    // what each was built from: residue copy (class map), code count + 1,
    // row width.  Two slots (the second only while memory is plentiful), so
    // queries alternating between two strip heights (32-row strips for
    // q <= 32 or 49..64, 48-row ones otherwise) or class maps rebuild none.
    struct PairRows {
        uint4* d = nullptr;
        std::vector<uint8_t> cls;
        bool valid = false, use_cls = false;
        uint32_t prow = 0, row_bytes = 0;
        uint64_t used = 0;                 // search counter at last use (LRU)
    };
    PairRows prs[2];
    uint64_t pr_clock = 0;
    size_t rec_begin = 0, rec_end = 0;    // plugin records [rec_begin, rec_end) of this shard
    std::shared_ptr<PlanCache> plans;
    void release();
};

// One slot per device the library searches on: slot 0 alone (the current
// HIP device or ssa_amd_set_device) by default; with ssa_amd_set_devices the
// DB is split into contiguous record ranges, one per device, cut at
// chunk_size boundaries (so the reference's insertion order is the
// concatenation of the slots' orders) and balanced by residues.
struct SlotPlan {
    int device;
    size_t rec_begin, rec_end;
};
std::vector<SlotPlan> device_plan();
DeviceDB& device_db(size_t slot = 0);
bool ensure_device_db(size_t slot, const SlotPlan& p);   // (re)packs from the plugin when stale
void ensure_device_db();                  // every slot of device_plan()
int save_packed_db(const char* path);     // 0 on success (single device)
int load_packed_db(const char* path);     // 0 on success; replaces packing from the plugin
std::vector<uint8_t> fetch_entry_codes(uint64_t local_id, int strand, int frame);

// Exact scores of every entry for every query view.  Scores live in the
// pinned int32 buffer (view-major); entries re-scored by the int64 kernel
// read INT32_MIN there and have their value in `wide`.
struct SearchScores {
    const int32_t* s32 = nullptr;
    size_t entries = 0, views = 0;
    // sparse: only the entries in `cand` (ascending) were copied back -- the
    // device filter proved every other entry leaves the top-k heap unchanged;
    // o8/o16 then come from the device counters (non-overflowed entries)
    bool sparse = false;
    std::vector<uint32_t> cand;
    uint64_t dev_o8 = 0, dev_o16 = 0;
    std::unordered_map<uint64_t, int64_t> wide;   // key = view * entries + entry
    uint64_t cells = 0;
    // device-side timing and counts of this search (published to stats())
    double kernel_ms = 0, wide_ms = 0, d2h_ms = 0, prep_ms = 0, upload_ms = 0, sync_wait_ms = 0;
    uint64_t wide_count = 0, kernel_bytes = 0;
    const char* kernel = "";
    uint32_t strip_rows = 0;             // pair kernel main strip height
    uint32_t long_entries = 0;           // entries the long-entry kernels scored (view 0)
    char long_kernel[24] = {};           // which (ssa_amd_stats_t::long_kernel)
    uint32_t fused_views = 0;            // views one fused pair_kernel launch scored (0: not fused)
    uint32_t part_retries = 0;           // 1: a strip-part wait timed out, the search ran again without parts
    uint32_t rare_merged = 0;            // compact codes scored through one upper-bound class (0: none)
    uint32_t rare_rescored = 0;          // forwarded merged-code entries re-scored exactly
    uint32_t graph = 0;                  // 0 direct, 1 captured into a new graph, 2 replayed (stats graph)
    int64_t get(size_t v, size_t e) const {
        const int32_t x = s32[v * entries + e];
        if (x != INT32_MIN) return x;
        auto it = wide.find((uint64_t)v * entries + e);
        return it == wide.end() ? (int64_t)INT32_MIN : it->second;
    }
};
// k / bit_width decide whether the device top-k filter applies
// indep != null: every view is an independent single-view query
// (ssa_amd_search_batch): the queries are enqueued back to back, each with its
// own device filter pass, and (*indep)[v] receives query v's scores; `out`
// then only carries the batch's aggregate timing.  Callers check
// batch_pipelinable() first.
void device_search(DeviceDB& D, const std::vector<QueryView>& views, int algo, size_t k, int bw, SearchScores& out,
                   std::vector<SearchScores>* indep = nullptr);
bool batch_pipelinable(size_t nqueries, size_t k);
constexpr size_t kMaxBatchPipe = 16;    // queries per pipelined sub-batch (one fused launch when their plans agree)
static_assert(kMaxBatchPipe == (size_t)kMaxFuse, "a sub-batch fuses into one pair_kernel launch");

ssa_amd_stats_t& stats();
void dist_overlay_stats(ssa_amd_stats_t* out);   // dist.cpp
void check(hipError_t e, const char* what);
double now_ms();
void host_mark(const char* what);
void host_marks_begin(bool on);
const std::vector<std::pair<const char*, double>>& host_marks();

}  // namespace ssa
