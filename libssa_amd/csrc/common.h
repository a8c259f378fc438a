// common.h -- internal declarations shared by the libssa_amd host sources.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include "libssa.h"
#include "libssa_amd.h"
#include "libssa_extern_db.h"

namespace ssa {

constexpr int kDim = 32;          // score matrix is 32 x 32, M(x,y) = m[(x << 5) + y]
constexpr int kAlgoSW = 0;
constexpr int kAlgoNW = 1;
constexpr size_t kMaxSlots = 16;   // devices one process can search on

// ------------------------------------------------------------------ config
struct Config {
    // bumped by every setter of the scoring or the options (api.cpp): the
    // per-DB plan cache (engine.cpp cached_plan) keys on it
    uint64_t plan_gen = 0;
    int output_mode = OUTPUT_WARNING;     // reference util.c:34
    size_t chunk_size = 1000;             // reference util.h:31 DEFAULT_CHUNK_SIZE
    size_t thread_count = 0;              // 0 = all host cores
    int symtype = AMINOACID;              // reference util_sequence.c:178
    int strands = FORWARD_STRAND;         // util_sequence.c:179
    int q_gencode = 1, d_gencode = 1;
    int8_t gap_open = 0, gap_extend = 0;  // libssa.c:35-36
    int device = -1;                      // -1: current HIP device
    std::vector<int> devices;             // ssa_amd_set_devices: shard the DB over these
    bool device_chosen = false;           // the caller called ssa_amd_set_device(s): SSA_AMD_DEVICES is not read
    bool device_env_read = false;         // SSA_AMD_DEVICES was applied (at the first init_db)
    std::vector<int> env_devices;         // the devices SSA_AMD_DEVICES (or its default, all) lists; the search
                                          // uses the first set_thread_count() of them (api.cpp refresh_env_devices)
    size_t id_offset = 0;                 // global ID of local record 0
    uint64_t db_generation = 0;           // bumped by init_db
    // tuning knobs (ssa_amd_set_option)
    int strip_np = 16;                    // packed rows per strip (2*np query rows)
    int waves_per_block = 4;
    int force_wide = 0;                   // 1: score everything with the int64 kernel
    int sw_kernel = 0;                    // 0: f16-pattern kernel when applicable, 1: int16 kernel
    int no_filter = 0;                    // 1: copy every score back (no device top-k filter)
    int pair_np = 0;                      // pair kernel main strip: 2 x pair_np rows; 0 auto (engine.cpp pair_strip_np)
    int long_groups = -1;                 // leading groups scored by long_kernel: -1 auto, 0 never, N forced
    int long_share_pct = 50;              // auto: groups longer than this % of a SIMD's share of all columns
    int long_waves = 0;                   // waves per long entry: 0 auto, 4 (rows over a workgroup) or 1
    int long4_share_pct = 1500;           // auto: 4 waves for groups longer than this % of a SIMD's share
                                          // (400 until round 6: NW's Swiss-Prot form +11 % at 1500, engine.cpp)
    int long16 = 1;                       // SW long entries on packed 16-bit patterns (long16_kernel) when exact
    int graph = 0;                        // 1: the usual single-view search runs as cached HIP graphs (engine.cpp
                                          // run_ops; measured slower than the direct calls on ROCm 7.2,
                                          // profiles/r06/graph); 0 (default): every operation issued on its own
    int upload_kernel = 1;                // 1: the per-search upload block is read from pinned memory by a kernel
                                          // on the search's stream instead of a copy-engine transfer (-14 us
                                          // between searches, profiles/r05/host_gap/kgap_upk*.txt)
    int tier_defer = 1;                   // single-view searches: the int32 re-score tier runs after the result's
                                          // copy, only when the search has overflowed lanes
    int tail_rows4 = 1;                   // pair kernel tail strips at 4-row granularity (default heights)
    int long_prio = 1;                    // long16 waves at raised issue priority (s_setprio 3)
    int long_pad = 1;
    int filter_onepass = 1;               // kernels.hip filter_onepass (0: three launches)
    int long_latency = 1;                 // engine.cpp long_plan: a tiny DB's groups all go to the long kernels
    int plan_cache = 1;                   // engine.cpp cached_plan (0: plan every search)                     // 1: long-entry workgroups pad their LDS to the pair kernel's (a finished
                                          // one leaves exactly a pair workgroup's hole); 0: their own LDS only
    int long_gate = 1;                    // the tables kernel holds the pair kernel until the long-entry
                                          // workgroups have started (TableArgs::gate)
    int long16_rows = 1;                  // long16_kernel may leave up to 8 query rows to its row scan (LongArgs::extra16)
    int pair_parts = 0;                   // pair_kernel: each group's strips in 2 dependent parts (StripArgs::nparts):
                                          // 0 auto (groups of >= 4 strips), 1 whole groups, 2 always
    int batch_fuse = 1;                   // ssa_amd_search_batch: queries of one pair-kernel plan in one launch
    int pair_ticket = 1;                  // pair_kernel workgroups take groups in start order (StripArgs::ticket)
    int rescore32 = 1;                    // overflowed lanes re-scored in int32 (long_kernel list mode) when exact
    long part_wait_us = 2000000;          // bound of a strip part's wait for its group's first part (then the
                                          // search runs again without parts; never a hang, never fatal)
    int timeline = 0;                     // record the DP waves' start/end (ssa_amd_get_timeline)
    int counters = -1;                    // the reference's 8/16-bit overflow counters: -1 auto (output mode
                                          // >= INFO, when m_run prints them), 0 never, 1 always
    int pair_prio_groups = 0;             // pair_kernel groups at raised wave priority: -1 one per SIMD, 0 none (measured neutral)
    int sync_spin = 1;                    // 1: hipDeviceScheduleSpin for this library's devices (set at the first
                                          // pack on a device): the host spins, not yields, while a search runs
                                          // (-15 us between searches, profiles/r05/host_gap/kgap_spin.txt)
    int lean_events = 1;                  // 1 (default): no timing markers around the upload, the tier and the filter
                                          // (stats upload_ms / wide_ms / d2h_ms stay 0; kernel_ms kept;
                                          // C2 +0.5 %, profiles/r05/ab/lean_events)
    int side_tier = 0;                    // 1: the int32 re-score tier runs beside the device filter (a second
                                          // stream) instead of in front of it (single-view sparse searches;
                                          // measured no gain, profiles/r05/ab/side_tier)
    int pair_split = 0;                   // strip parts for all quads (0) or only the first P % (P > 0, the longest)
                                          // or the last -P % (P < 0) of the quads
    int rare_merge = 0;                   // 1: when the query's residue classes leave the pair table too big for
                                          // three workgroups per CU, the rarest classes share one upper-bound
                                          // class and the forwarded entries holding them are re-scored exactly
                                          // (default off: Swiss-Prot form kernel +0.8 %, end to end -4 %,
                                          // profiles/r05/ab/merge_sprot2)
    int filter_host = 0;                  // 1/2: the top-k filter writes its result into pinned host memory and
                                          // the host spins on its sequence word (no D2H copy, no stream
                                          // synchronisation; 1 with a system-scope release, 2 with system-
                                          // scope stores and a store-completion wait); 3: the filter writes
                                          // it with plain stores, the host synchronises with the stream (no
                                          // copy); 0 (default: 1 and 2 measured slower,
                                          // profiles/r05/ab/filter_host*): copy + hipStreamSynchronize
};
Config& cfg();
// whether a search computes the overflow counters (Config::counters)
inline bool counters_on(const Config& C) {
    return C.counters > 0 || (C.counters < 0 && C.output_mode >= OUTPUT_INFO);
}

// SSA_AMD_TRACE=1: per-search host/device timing lines on stderr
bool trace_on();

// --------------------------------------------------------------- messages
// Same channels and prefixes as the reference (util.c:36-89): errors and
// warnings and infos go to stdout gated by the output mode, fatal goes to
// stderr and exits with status 1.
[[noreturn]] void fatal(const char* fmt, ...);
void print_info(const char* fmt, ...);
void print_warning(const char* fmt, ...);
void print_error(const char* fmt, ...);

// --------------------------------------------------------------- alphabets
extern const signed char* map_aa();   // 256-entry ASCII -> code, -1 unknown
extern const signed char* map_nt();
uint8_t nt_complement(uint8_t code);
void revcompl(const uint8_t* in, size_t len, uint8_t* out);
void init_translation(int q_gencode, int d_gencode);
bool gencode_valid(int code);
// translate mapped NT codes, strand 0 = forward, 1 = reverse complement
std::vector<uint8_t> translate(bool db_side, const uint8_t* dna, size_t len, int strand, int frame);

// ----------------------------------------------------------------- matrix
struct Matrix {
    bool ready = false;
    bool constant = false;                // reference never clears this flag
    int64_t m[kDim * kDim];
};
Matrix& matrix();
void matrix_builtin(const char* name);
void matrix_from_string(const char* text);
void matrix_from_file(const char* path);
void matrix_constant(int match, int mismatch);
void matrix_free();

// ------------------------------------------------------------------ query
struct SeqBuf {
    std::vector<uint8_t> seq;   // codes, plus a trailing 0 kept for C callers
    size_t len() const { return seq.empty() ? 0 : seq.size() - 1; }
};
}  // namespace ssa

struct _query {
    ssa::SeqBuf nt[2];
    ssa::SeqBuf aa[6];
    std::string header;
    int symtype;
};

namespace ssa {
struct QueryView {                // one search "query buffer" (searcher.c:42-90)
    const uint8_t* seq;
    size_t len;
    int strand, frame;
    char* cseq;                   // pointer handed out in q_seq_t.seq
};
std::vector<QueryView> query_views(p_query q);

// ---------------------------------------------------------------- top-k
struct Hit {
    int64_t score;
    uint64_t id;
    uint8_t qid, strand, frame;
};
// Reference min-heap (minheap.c:50-106) with exact tie behaviour.
class TopK {
public:
    explicit TopK(size_t k) : k_(k) { a_.reserve(k); }
    // returns true when the element entered the heap
    bool add(const Hit& h);
    size_t size() const { return a_.size(); }
    bool full() const { return a_.size() >= k_; }
    int64_t root_score() const { return a_.empty() ? INT64_MIN : a_[0].score; }
    std::vector<Hit> sorted() const;
private:
    size_t k_;
    std::vector<Hit> a_;
};
void sort_hits(std::vector<Hit>& v);   // score desc, id desc (util.h:12)

// ------------------------------------------------------ COMPUTE_ALIGNMENT
// align.cpp: region {q begin, q end, db begin, db end} and CIGAR of a pair
std::string traceback(int algo, const uint8_t* q, size_t qn, const uint8_t* d, size_t dn, size_t region[4]);
void compute_alignments(p_alignment_list L, int algo);

}  // namespace ssa
