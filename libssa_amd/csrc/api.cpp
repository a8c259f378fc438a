// api.cpp -- the exported C ABI: every function of include/libssa.h (the
// reference's src/libssa.h:122-263, implemented in src/libssa.c) plus the
// MI355X extensions of include/libssa_amd.h.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <numeric>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "engine.h"

using namespace ssa;

namespace ssa {
p_query query_from_string(const char* s);
p_query query_from_file(const char* path);
}

namespace {

// The environment's device list as the search uses it: its first
// set_thread_count() devices -- the reference's thread count is its number of
// search workers (thread_pool.c:39-47), a device slot's analogue here; 0 (the
// default) = all of them.  An explicit ssa_amd_set_device(s) is left alone.
void refresh_env_devices() {
    Config& C = cfg();
    if (C.device_chosen || !C.device_env_read || C.env_devices.empty()) return;
    std::vector<int> d = C.env_devices;
    if (C.thread_count > 0 && d.size() > C.thread_count) d.resize(C.thread_count);
    if (d.size() > 1) {
        C.devices = d;
    } else {
        C.devices.clear();
        C.device = d[0];
    }
}

// SSA_AMD_DEVICES (include/libssa_amd.h), applied once -- at the first
// init_db or device query -- unless the caller chose devices itself.  The
// reference's default is every core (src/util/thread_pool.c:39-47); here it
// is every visible GPU.
void apply_device_env() {
    Config& C = cfg();
    if (C.device_chosen || C.device_env_read) return;
    C.device_env_read = true;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess) {
        (void)hipGetLastError();
        return;                           // no device: the first search reports it
    }
    const char* e = getenv("SSA_AMD_DEVICES");
    std::vector<int> devs;
    if (!e || !*e || !strcmp(e, "all")) {
        for (int i = 0; i < count && devs.size() < kMaxSlots; i++) devs.push_back(i);
        // (one device: the current-device path, unchanged)
        if (devs.size() > 1) {
            C.env_devices = devs;
            refresh_env_devices();
        }
        return;
    }
    if (!strcmp(e, "current")) return;
    for (const char* p = e; *p;) {
        char* end = nullptr;
        const long d = strtol(p, &end, 10);
        if (end == p || d < 0 || d >= count || devs.size() >= kMaxSlots) {
            print_error("SSA_AMD_DEVICES=%s: not a list of at most %d of the %d visible devices; using the current "
                        "device", e, (int)kMaxSlots, count);
            return;
        }
        devs.push_back((int)d);
        p = end;
        if (*p == ',') p++;
        else if (*p) {
            print_error("SSA_AMD_DEVICES=%s: not a comma-separated device list; using the current device", e);
            return;
        }
    }
    C.env_devices = devs;
    refresh_env_devices();
}

// Persistent per-slot host threads for multi-device searches (SURVEY.md §8b
// "one host thread per GPU inside sw_align"; the reference keeps its worker
// pool across searches too, thread_pool.c:50-86).  run(n, fn) runs fn(0) on
// the calling thread and fn(s) for 0 < s < n on worker s, and returns when
// all are done.  A worker spins for a few ms after each job (a benchmark's
// back-to-back searches hand over without a wake-up), then sleeps.  The pool
// is never destroyed: its threads are detached and idle at process exit.
class SlotPool {
public:
    void run(size_t n, const std::function<void(size_t)>& fn) {
        if (n > 1) {
            while (workers_ + 1 < n) {
                const size_t s = ++workers_;
                const uint64_t g0 = gen_.load(std::memory_order_acquire);
                std::thread([this, s, g0]() { loop(s, g0); }).detach();
            }
            {
                std::lock_guard<std::mutex> g(m_);
                job_ = &fn;
                njob_ = n;
                pending_.store(n - 1, std::memory_order_relaxed);
                gen_.fetch_add(1, std::memory_order_release);
            }
            cv_.notify_all();
        }
        fn(0);
        while (n > 1 && pending_.load(std::memory_order_acquire) != 0) __builtin_ia32_pause();
    }

private:
    void loop(size_t s, uint64_t seen) {
        using clk = std::chrono::steady_clock;
        for (;;) {
            const auto t0 = clk::now();
            for (uint32_t it = 0; gen_.load(std::memory_order_acquire) == seen; it++) {
                if ((it & 255) == 0 && clk::now() - t0 > std::chrono::milliseconds(5)) {
                    std::unique_lock<std::mutex> lk(m_);
                    cv_.wait(lk, [&]() { return gen_.load(std::memory_order_acquire) != seen; });
                    break;
                }
                __builtin_ia32_pause();
            }
            // a consistent (generation, job) snapshot: run() writes both
            // under the lock, and a job this worker belongs to is never
            // replaced before the worker has finished it
            const std::function<void(size_t)>* job;
            size_t n;
            {
                std::lock_guard<std::mutex> g(m_);
                seen = gen_.load(std::memory_order_acquire);
                job = job_;
                n = njob_;
            }
            if (s < n) {
                (*job)(s);
                pending_.fetch_sub(1, std::memory_order_acq_rel);
            }
        }
    }
    std::mutex m_;
    std::condition_variable cv_;
    std::atomic<uint64_t> gen_{0};
    std::atomic<size_t> pending_{0};
    const std::function<void(size_t)>* job_ = nullptr;
    size_t njob_ = 0;
    size_t workers_ = 0;                 // (grown by the caller's thread only)
};

SlotPool& slot_pool() {
    static SlotPool* p = new SlotPool();   // (leaked on purpose: detached workers wait on it at exit)
    return *p;
}

// test_configuration (libssa.c:196-219)
void test_configuration(p_query q) {
    if (!cfg().gap_open && !cfg().gap_extend)
        print_warning("Gap opening and gap extension cost set to zero. Possible error.");
    if (!matrix().ready) fatal("Scoring not initialized.");
    if (!q) fatal("Query not initialized.");
    if (ssa_db_get_sequence_count() == 0) print_warning("Database contains zero sequences. Possible error.");
    if (!matrix().constant && cfg().symtype == NUCLEOTIDE)
        fatal("Nucleotide sequences can only be aligned using constant scores.");
}

void check_width(int bw) {
    if (bw != BIT_WIDTH_8 && bw != BIT_WIDTH_16 && bw != BIT_WIDTH_64)
        fatal("\nunknown bit width provided: %d\n\n", bw);
}

// Feeds every (view, entry) score to the reference heap in the 64-bit
// single-thread insertion order: ID chunks of chunk_size, and inside a chunk
// query view by query view, entries in ID order (search_64.c:44-56,
// db_adapter.c:212-239).  Optionally records the accepted insertions.
void replay(const SearchScores& sc, const EntryMeta& meta, const std::vector<QueryView>& views, TopK& heap,
            std::vector<Hit>* log) {
    const size_t V = sc.views, E = sc.entries;
    const uint64_t off = cfg().id_offset;
    auto visit = [&](size_t v, size_t e) {
        const int64_t s = sc.get(v, e);
        if (heap.full() && s <= heap.root_score()) return;
        Hit h{s, meta.id[e] + off, (uint8_t)v, meta.strand[e], meta.frame[e]};
        if (heap.add(h) && log) log->push_back(h);
    };
    (void)views;
    if (sc.sparse) {
        // candidates in insertion order, as view * entries + entry
        for (const uint32_t x : sc.cand) visit(x / E, x % E);
        return;
    }
    if (V == 1) {
        if (sc.wide.empty()) {
            // hot loop: plain int32 scan with the root cached
            const int32_t* s32 = sc.s32;
            for (size_t e = 0; e < E; e++) {
                if (heap.full() && (int64_t)s32[e] <= heap.root_score()) continue;
                visit(0, e);
            }
        } else {
            for (size_t e = 0; e < E; e++) visit(0, e);
        }
        return;
    }
    const uint64_t cs = cfg().chunk_size;
    size_t e0 = 0;
    while (e0 < E) {
        const uint64_t chunk_end = (meta.id[e0] / cs + 1) * cs;
        size_t e1 = e0;
        while (e1 < E && meta.id[e1] < chunk_end) e1++;
        for (size_t v = 0; v < V; v++)
            for (size_t e = e0; e < e1; e++) visit(v, e);
        e0 = e1;
    }
}

struct SearchResult {
    std::vector<QueryView> views;
    std::vector<Hit> hits;      // sorted top-k, or the insertion log
};

// scores the device top-k filter let through to the host (every score of a
// search that ran without the filter)
uint64_t candidates(const SearchScores& x) { return x.sparse ? x.cand.size() : (uint64_t)x.entries * x.views; }

void publish_stats(const std::vector<SearchScores>& sc, const std::vector<SlotPlan>& plan,
                   const std::vector<double>& slot_ms) {
    ssa_amd_stats_t& S = stats();
    S.kernel_ms = S.wide_ms = S.d2h_ms = S.prep_ms = S.upload_ms = S.sync_wait_ms = 0;
    S.cells = S.entries = S.wide_count = S.kernel_bytes = S.filter_candidates = 0;
    S.slots = (uint32_t)std::min(sc.size(), (size_t)16);
    S.graph = sc.empty() ? 0u : sc[0].graph;
    for (size_t i = 0; i < 16; i++) {
        S.slot_device[i] = i < S.slots ? plan[i].device : -1;
        S.slot_kernel_ms[i] = i < S.slots ? sc[i].kernel_ms : 0;
        S.slot_search_ms[i] = i < S.slots ? slot_ms[i] : 0;
    }
    for (size_t i = 0; i < sc.size(); i++) {
        S.filter_candidates += candidates(sc[i]);
        // devices run concurrently: times are the slowest device's
        S.kernel_ms = std::max(S.kernel_ms, sc[i].kernel_ms);
        S.wide_ms = std::max(S.wide_ms, sc[i].wide_ms);
        S.d2h_ms = std::max(S.d2h_ms, sc[i].d2h_ms);
        S.prep_ms = std::max(S.prep_ms, sc[i].prep_ms);
        S.upload_ms = std::max(S.upload_ms, sc[i].upload_ms);
        S.sync_wait_ms = std::max(S.sync_wait_ms, sc[i].sync_wait_ms);
        S.cells += sc[i].cells;
        S.entries += sc[i].entries;
        S.wide_count += sc[i].wide_count;
        S.kernel_bytes += sc[i].kernel_bytes;
    }
    S.kernel_launches = (uint32_t)(sc.empty() ? 0 : sc[0].views);
    S.device = plan.empty() ? -1 : plan[0].device;
    snprintf(S.kernel, sizeof S.kernel, "%s", sc.empty() ? "" : sc[0].kernel);
    S.strip_rows = sc.empty() ? 0 : sc[0].strip_rows;
    S.long_entries = sc.empty() ? 0 : sc[0].long_entries;
    snprintf(S.long_kernel, sizeof S.long_kernel, "%s", sc.empty() ? "" : sc[0].long_kernel);
    S.part_retries = 0;
    S.rare_merged = S.rare_rescored = 0;
    for (const SearchScores& x : sc) {
        S.part_retries += x.part_retries;
        S.rare_merged = std::max(S.rare_merged, x.rare_merged);
        S.rare_rescored += x.rare_rescored;
    }
}

void run_search(p_query q, int algo, size_t k, int bw, bool want_log, SearchResult& R) {
    const double t0 = now_ms();
    check_width(bw);
    ensure_device_db();
    const std::vector<SlotPlan> plan = device_plan();
    R.views = query_views(q);
    host_mark("views");
    std::vector<SearchScores> sc(plan.size());
    std::vector<std::vector<Hit>> logs(plan.size());
    std::vector<double> slot_ms(plan.size(), 0.0);
    if (plan.size() == 1) {
        device_search(device_db(0), R.views, algo, k, bw, sc[0]);
        slot_ms[0] = now_ms() - t0;
    } else {
        // one persistent host thread per device slot (the caller's for slot
        // 0); each replays its shard into a log of the elements its own heap
        // accepts
        slot_pool().run(plan.size(), [&](size_t s) {
            const double ts = now_ms();
            device_search(device_db(s), R.views, algo, k, bw, sc[s]);
            TopK h(k);
            replay(sc[s], device_db(s).meta, R.views, h, &logs[s]);
            slot_ms[s] = now_ms() - ts;
        });
    }
    const double t1 = now_ms();
    host_mark("searched");
    TopK heap(k);
    if (plan.size() == 1) {
        replay(sc[0], device_db(0).meta, R.views, heap, want_log ? &R.hits : nullptr);
    } else {
        for (const auto& L : logs)
            for (const Hit& h : L)
                if (heap.add(h) && want_log) R.hits.push_back(h);
    }
    if (!want_log) R.hits = heap.sorted();
    const double t2 = now_ms();
    // the reference's overflow counters, counted on the device
    // (counters.hip): what its 8/16-bit kernels would have re-run
    uint64_t o8 = 0, o16 = 0;
    for (const SearchScores& x : sc) {
        o8 += x.dev_o8;
        o16 += x.dev_o16;
    }
    publish_stats(sc, plan, slot_ms);
    ssa_amd_stats_t& S = stats();
    S.overflow_8 = o8;
    S.overflow_16 = o16;
    S.counters = (bw == BIT_WIDTH_64 || counters_on(cfg())) ? 1 : 0;
    S.replay_ms = t2 - t1;
    S.search_ms = now_ms() - t0;
    if (trace_on()) fprintf(stderr, "trace: run_search on %zu device slots: to device_search end %.3f, replay %.3f, total %.3f\n",
                            plan.size(), t1 - t0, t2 - t1, S.search_ms);
    S.total_searches++;
    S.total_kernel_ms += S.kernel_ms;
    S.total_search_ms += S.search_ms;
    // m_run's bookkeeping messages (manager.c:147-170)
    const size_t cs = cfg().chunk_size;
    size_t records = 0, entries = 0;
    for (size_t s = 0; s < plan.size(); s++) {
        const EntryMeta& M = device_db(s).meta;
        print_info("Device %d - Processed chunks: %ld and sequences: %ld\n", device_db(s).device,
                   (long)((M.records + cs - 1) / cs), (long)M.size());
        records += M.records;
        entries += M.size();
    }
    if (o8 || o16)
        print_info("Overflow occurred: %ld sequences were re-aligned with 16 bit, and %ld sequences with 64 bit\n",
                   (long)o8, (long)o16);
    if (records != entries)
        print_warning("# Number of processed sequences differs! Expected: %ld - Actual: %ld\n", (long)records,
                      (long)entries);
}

// create_score_alignment_list (aligner.c:62-99): one alignment_t per hit,
// the DB sequence re-fetched through the plugin as a mapped-code copy, the
// query borrowed from the p_query.  Note the reference's field swap
// (aligner.c:76-77): db_seq.strand <- frame, db_seq.frame <- strand.
p_alignment_list build_list(const SearchResult& R) {
    p_alignment_list L = (p_alignment_list)malloc(sizeof(alignment_list_t));
    L->len = R.hits.size();
    L->alignments = (p_alignment*)malloc(sizeof(p_alignment) * (L->len ? L->len : 1));
    for (size_t i = 0; i < L->len; i++) {
        const Hit& h = R.hits[i];
        p_alignment a = (p_alignment)calloc(1, sizeof(alignment_t));
        const uint64_t local = h.id - cfg().id_offset;
        std::vector<uint8_t> codes = fetch_entry_codes(local, h.strand, h.frame);
        const size_t n = codes.empty() ? 0 : codes.size() - 1;
        a->db_seq.seq = (char*)malloc(n + 1);
        if (n) memcpy(a->db_seq.seq, codes.data(), n);
        a->db_seq.seq[n] = 0;
        a->db_seq.len = n;
        a->db_seq.ID = h.id;
        a->db_seq.strand = h.frame;
        a->db_seq.frame = h.strand;
        const QueryView& qv = R.views[h.qid];
        a->query.seq = qv.cseq;
        a->query.len = qv.len;
        a->query.strand = qv.strand;
        a->query.frame = qv.frame;
        a->score = (long)h.score;
        L->alignments[i] = a;
    }
    return L;
}

p_alignment_list align(p_query q, size_t k, int bw, int at, int algo) {
    // (SSA_AMD_TRACE: the host's timeline of the call, from the previous
    // call's return -- the caller's own time -- to this one's)
    static double last_return = 0;
    if (trace_on()) {
        host_marks_begin(true);
        host_mark("entry");
    }
    test_configuration(q);
    SearchResult R;
    run_search(q, algo, k, bw, false, R);
    p_alignment_list L = build_list(R);
    if (at == COMPUTE_ALIGNMENT) compute_alignments(L, algo);   // align.cpp (aligner.c:163-181)
    if (trace_on()) {
        host_mark("return");
        const auto& m = host_marks();
        const double t0 = m.front().second;
        fprintf(stderr, "trace: host us (entry at %.0f ns): caller %.1f", t0 * 1e6, last_return > 0 ? (t0 - last_return) * 1e3 : -1.0);
        for (size_t i = 1; i < m.size(); i++) fprintf(stderr, ", %s %.1f", m[i].first, (m[i].second - t0) * 1e3);
        fprintf(stderr, "\n");
        last_return = now_ms();
        host_marks_begin(false);
    }
    return L;
}

}  // namespace

extern "C" {

// ---------------------------------------------------------- technical setup
void set_output_mode(int mode) { cfg().output_mode = mode; }
void set_simd_compute_mode(int mode) { (void)mode; }
void set_chunk_size(size_t size) {
    if (size == 0) {
        print_error("Only non zero chunk sizes are allowed. Using the default size of 1000 sequences.", size);
        size = 1000;
    }
    cfg().chunk_size = size;
}
// (libssa.c:58-60: the number of search workers; here it caps the device
// slots an unchanged caller gets from SSA_AMD_DEVICES / all devices)
void set_thread_count(size_t count) {
    cfg().thread_count = count;
    refresh_env_devices();
}

// ------------------------------------------------------------ initialisation
void init_score_matrix(int mode, const char* m) {
    cfg().plan_gen++;
    if (mode == READ_FROM_FILE) matrix_from_file(m);
    else if (mode == READ_FROM_STRING) matrix_from_string(m);
    else if (mode == MATRIX_BUILDIN) matrix_builtin(m);
    else fatal("Unknown mode for reading score matrices: %d", mode);
}

void init_gap_penalties(const int8_t gapO, const int8_t gapE) {
    cfg().plan_gen++;
    cfg().gap_open = gapO;
    cfg().gap_extend = gapE;
}

void init_constant_scores(const int8_t p, const int8_t m) {
    cfg().plan_gen++;
    matrix_constant(p, m);
}

// MI355X: validates the NEW type and strands (the reference checks the old
// global symtype twice, libssa.c:146-151, and so rejects any call made after
// TRANS_DB/TRANS_BOTH was selected).
void init_symbol_translation(int type, int strands, int d_gencode, int q_gencode) {
    if (!gencode_valid(q_gencode)) fatal("Illegal query genetic code specified.");
    if (!gencode_valid(d_gencode)) fatal("Illegal database genetic code specified.");
    if (type < 0 || type > 4) fatal("Illegal symbol type specified.");
    if (strands < 1 || strands > 3) fatal("Illegal strands specified.");
    cfg().plan_gen++;
    cfg().symtype = type;
    cfg().strands = strands;
    cfg().q_gencode = q_gencode;
    cfg().d_gencode = d_gencode;
    init_translation(q_gencode, d_gencode);
}

void init_db(const char* db_file) {
    apply_device_env();
    ssa_db_close();
    ssa_db_init(db_file);
    cfg().db_generation++;
    print_info("DB read %lu sequences\n", (unsigned long)ssa_db_get_sequence_count());
}

p_query init_sequence_fasta(int mode, const char* s) {
    if (mode == READ_FROM_FILE) return query_from_file(s);
    if (mode == READ_FROM_STRING) return query_from_string(s);
    fatal("Unknown mode for reading query sequences: %d", mode);
}

void free_sequence(p_query p) { delete p; }

// ------------------------------------------------------------------ searches
p_alignment_list sw_align(p_query p, size_t hitcount, int bit_width, int align_type) {
    return align(p, hitcount, bit_width, align_type, kAlgoSW);
}

p_alignment_list nw_align(p_query p, size_t hitcount, int bit_width, int align_type) {
    return align(p, hitcount, bit_width, align_type, kAlgoNW);
}

void free_alignment(p_alignment_list alist) {
    if (!alist) return;
    if (alist->alignments) {
        for (size_t i = 0; i < alist->len; i++) {
            p_alignment a = alist->alignments[i];
            if (!a) continue;
            free(a->db_seq.seq);
            free(a->alignment);
            free(a);
        }
        free(alist->alignments);
    }
    free(alist);
}

// (libssa.c:266-271 frees the matrix, closes the DB and ends its thread
// pool; here the device copies of the DB are released too)
void ssa_exit(void) {
    matrix_free();
    ssa_db_close();
    cfg().db_generation++;
    for (size_t s = 0; s < kMaxSlots; s++) {
        DeviceDB& D = device_db(s);
        if (D.device < 0) continue;
        // (a runtime already shut down -- ssa_exit from an atexit handler --
        // leaves the memory to the process's end)
        if (hipSetDevice(D.device) != hipSuccess) {
            (void)hipGetLastError();
            continue;
        }
        D.release();
    }
}

// ------------------------------------------------------------- extensions
int ssa_amd_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

void ssa_amd_set_device(int device) {
    cfg().device = device;
    cfg().devices.clear();
    cfg().device_chosen = true;
}

int ssa_amd_set_devices(const int* devices, int n) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess) count = 0;
    cfg().device_chosen = true;
    if (n <= 0 || !devices) {
        cfg().devices.clear();
        return 0;
    }
    if ((size_t)n > kMaxSlots) {
        print_error("At most %d devices per process", (int)kMaxSlots);
        return 1;
    }
    for (int i = 0; i < n; i++)
        if (devices[i] < 0 || devices[i] >= count) {
            print_error("No HIP device %d (%d visible)", devices[i], count);
            return 1;
        }
    cfg().devices.assign(devices, devices + n);
    return 0;
}

int ssa_amd_get_devices(int* out, int cap) {
    apply_device_env();
    const Config& C = cfg();
    std::vector<int> d = C.devices;
    if (d.size() <= 1) {
        int dev = d.empty() ? C.device : d[0];
        if (dev < 0 && hipGetDevice(&dev) != hipSuccess) {
            (void)hipGetLastError();
            dev = -1;
        }
        d.assign(1, dev);
    }
    for (int i = 0; out && i < cap && i < (int)d.size(); i++) out[i] = d[i];
    return (int)d.size();
}
void ssa_amd_set_id_offset(size_t offset) { cfg().id_offset = offset; }

int ssa_amd_prepare_db(void) {
    ensure_device_db();
    return 0;
}

size_t ssa_amd_get_timeline(uint32_t* out, size_t cap) {
    DeviceDB& D = device_db(0);
    if (!D.d_timeline || D.timeline_rows == 0) return 0;
    const size_t n = std::min(cap, D.timeline_rows);
    if (out && n) {
        check(hipSetDevice(D.device), "hipSetDevice");
        check(hipMemcpy(out, D.d_timeline, n * sizeof(uint4), hipMemcpyDeviceToHost), "timeline copy");
    }
    return D.timeline_rows;
}

void ssa_amd_get_stats(ssa_amd_stats_t* out) {
    if (!out) return;
    *out = stats();
    dist_overlay_stats(out);      // a fake rank's own gather time (dist.cpp)
}

int ssa_amd_save_db(const char* path) {
    if (!path) return 1;
    return save_packed_db(path);
}

int ssa_amd_load_db(const char* path) {
    if (!path) return 1;
    return load_packed_db(path);
}

size_t ssa_amd_align_pair(int algo, const char* query, size_t qlen, const char* db, size_t dlen, size_t region[4],
                          char* cigar, size_t cap) {
    if (!matrix().ready) fatal("Scoring matrix not initialized");
    if (algo != SSA_AMD_SW && algo != SSA_AMD_NW) fatal("ssa_amd_align_pair: unknown algorithm %d", algo);
    size_t rg[4];
    const std::string c = traceback(algo == SSA_AMD_SW ? kAlgoSW : kAlgoNW, (const uint8_t*)query, qlen,
                                    (const uint8_t*)db, dlen, rg);
    if (region) memcpy(region, rg, sizeof rg);
    if (cigar && cap) {
        const size_t n = std::min(c.size(), cap - 1);
        memcpy(cigar, c.data(), n);
        cigar[n] = 0;
    }
    return c.size();
}

size_t ssa_amd_query_views(p_query query, q_seq_t* out, size_t cap) {
    if (!query) return 0;
    const std::vector<QueryView> v = query_views(query);
    for (size_t i = 0; i < v.size() && i < cap; i++)
        out[i] = q_seq_t{v[i].cseq, v[i].len, v[i].strand, v[i].frame};
    return v.size();
}

size_t ssa_amd_translate(int db_side, const char* nt_codes, size_t len, int strand, int frame, char* out,
                         size_t cap) {
    if (frame < 0 || frame > 2 || strand < 0 || strand > 1) fatal("ssa_amd_translate: bad strand/frame");
    const std::vector<uint8_t> p = translate(db_side != 0, (const uint8_t*)nt_codes, len, strand, frame);
    const size_t n = p.size() - 1;
    if (out) memcpy(out, p.data(), std::min(n, cap));
    return n;
}

void ssa_amd_set_option(const char* name, long value) {
    if (!name) return;
    cfg().plan_gen++;
    if (!strcmp(name, "strip_np")) cfg().strip_np = (int)value;
    else if (!strcmp(name, "force_wide")) cfg().force_wide = (int)value;
    else if (!strcmp(name, "sw_kernel")) cfg().sw_kernel = (int)value;
    else if (!strcmp(name, "no_filter")) cfg().no_filter = (int)value;
    else if (!strcmp(name, "pair_np")) cfg().pair_np = (int)value;
    else if (!strcmp(name, "long_groups")) cfg().long_groups = (int)value;
    else if (!strcmp(name, "long_share_pct")) cfg().long_share_pct = (int)value;
    else if (!strcmp(name, "long_waves")) cfg().long_waves = (int)value;
    else if (!strcmp(name, "long4_share_pct")) cfg().long4_share_pct = (int)value;
    else if (!strcmp(name, "long16")) cfg().long16 = (int)value;
    else if (!strcmp(name, "pair_prio_groups")) cfg().pair_prio_groups = (int)value;
    else if (!strcmp(name, "timeline")) cfg().timeline = (int)value;
    else if (!strcmp(name, "pair_ticket")) cfg().pair_ticket = (int)value;
    else if (!strcmp(name, "pair_parts")) cfg().pair_parts = (int)value;
    else if (!strcmp(name, "batch_fuse")) cfg().batch_fuse = (int)value;
    else if (!strcmp(name, "counters")) cfg().counters = (int)value;
    else if (!strcmp(name, "part_wait_us")) cfg().part_wait_us = std::max(0L, value);
    else if (!strcmp(name, "rescore32")) cfg().rescore32 = (int)value;
    else if (!strcmp(name, "filter_host")) cfg().filter_host = (int)value;
    else if (!strcmp(name, "rare_merge")) cfg().rare_merge = (int)value;
    else if (!strcmp(name, "pair_split")) cfg().pair_split = (int)value;
    else if (!strcmp(name, "side_tier")) cfg().side_tier = (int)value;
    else if (!strcmp(name, "sync_spin")) cfg().sync_spin = (int)value;
    else if (!strcmp(name, "lean_events")) cfg().lean_events = (int)value;
    else if (!strcmp(name, "long16_rows")) cfg().long16_rows = (int)value;
    else if (!strcmp(name, "long_gate")) cfg().long_gate = (int)value;
    else if (!strcmp(name, "long_pad")) cfg().long_pad = (int)value;
    else if (!strcmp(name, "long_prio")) cfg().long_prio = (int)value;
    else if (!strcmp(name, "tail_rows4")) cfg().tail_rows4 = (int)value;
    else if (!strcmp(name, "tier_defer")) cfg().tier_defer = (int)value;
    else if (!strcmp(name, "upload_kernel")) cfg().upload_kernel = (int)value;
    else if (!strcmp(name, "graph")) cfg().graph = (int)value;
    else if (!strcmp(name, "plan_cache")) cfg().plan_cache = (int)value;
    else if (!strcmp(name, "long_latency")) cfg().long_latency = (int)value;
    else if (!strcmp(name, "filter_onepass")) cfg().filter_onepass = (int)value;
    else if (!strcmp(name, "filter_prefix_regs")) set_filter_prefix_regs((int)value);
    else print_warning("unknown option %s", name);
}

size_t ssa_amd_search(p_query query, int algo, size_t hitcount, int bit_width, int mode, ssa_hit_t* out,
                      size_t cap) {
    test_configuration(query);
    SearchResult R;
    run_search(query, algo == SSA_AMD_NW ? kAlgoNW : kAlgoSW, hitcount, bit_width, mode == SSA_AMD_LOG, R);
    const size_t n = std::min(cap, R.hits.size());
    for (size_t i = 0; i < n; i++) {
        const Hit& h = R.hits[i];
        out[i] = ssa_hit_t{h.score, h.id, h.qid, h.strand, h.frame, {0, 0, 0, 0, 0}};
    }
    return n;
}

size_t ssa_amd_search_batch(const p_query* queries, size_t nq, int algo, size_t hitcount, int bit_width,
                            ssa_hit_t* out, size_t* counts) {
    size_t total = 0;
    const double t0 = now_ms();
    double kms = 0;
    uint64_t cells = 0;
    // the running totals as the batch found them: a lone query below goes
    // through run_search, which adds itself, so the batch sets them once
    const ssa_amd_stats_t before = stats();
    // single-device, single-view queries with a small k: pipelined sub-batches
    // (device_search's independent mode) -- the host prepares query i+1 while
    // query i runs, one synchronisation per sub-batch
    const int al = algo == SSA_AMD_NW ? kAlgoNW : kAlgoSW;
    bool piped = nq > 1 && batch_pipelinable(nq, hitcount);
    std::vector<std::vector<QueryView>> qviews(piped ? nq : 0);
    for (size_t i = 0; piped && i < nq; i++) {
        test_configuration(queries[i]);
        qviews[i] = query_views(queries[i]);
        piped = qviews[i].size() == 1 && qviews[i][0].len > 0;
    }
    if (piped) {
        check_width(bit_width);
        ensure_device_db();
        piped = device_plan().size() == 1;
    }
    if (piped) {
        DeviceDB& D = device_db(0);
        // sub-batches of queries of similar length (stable order by length):
        // a sub-batch whose pair-kernel plans agree runs as one fused launch
        std::vector<size_t> ord(nq);
        std::iota(ord.begin(), ord.end(), (size_t)0);
        std::stable_sort(ord.begin(), ord.end(),
                         [&](size_t x, size_t y) { return qviews[x][0].len < qviews[y][0].len; });
        uint32_t launches = 0, retries = 0;
        uint64_t ncand = 0;
        for (size_t b0 = 0; b0 < nq; b0 += kMaxBatchPipe) {
            const size_t b1 = std::min(nq, b0 + kMaxBatchPipe);
            std::vector<QueryView> vs;
            for (size_t i = b0; i < b1; i++) vs.push_back(qviews[ord[i]][0]);
            if (vs.size() == 1) {
                // a lone last query: the ordinary path
                const size_t qi = ord[b0];
                SearchResult R;
                run_search(queries[qi], al, hitcount, bit_width, false, R);
                kms += stats().kernel_ms;
                cells += stats().cells;
                retries += stats().part_retries;
                ncand += stats().filter_candidates;
                launches++;
                const size_t n = std::min(hitcount, R.hits.size());
                for (size_t j = 0; j < n; j++) {
                    const Hit& h = R.hits[j];
                    out[qi * hitcount + j] = ssa_hit_t{h.score, h.id, h.qid, h.strand, h.frame, {0, 0, 0, 0, 0}};
                }
                if (counts) counts[qi] = n;
                total += n;
                continue;
            }
            SearchScores agg;
            std::vector<SearchScores> sc;
            device_search(D, vs, al, hitcount, bit_width, agg, &sc);
            kms += agg.kernel_ms;
            retries += agg.part_retries;
            launches += agg.fused_views ? 1u : (uint32_t)vs.size();
            for (size_t bi = b0; bi < b1; bi++) {
                const size_t i = ord[bi];
                const SearchScores& x = sc[bi - b0];
                cells += x.cells;
                ncand += candidates(x);
                TopK heap(hitcount);
                replay(x, D.meta, qviews[i], heap, nullptr);
                const std::vector<Hit> hits = heap.sorted();
                const size_t n = std::min(hitcount, hits.size());
                for (size_t j = 0; j < n; j++) {
                    const Hit& h = hits[j];
                    out[i * hitcount + j] = ssa_hit_t{h.score, h.id, h.qid, h.strand, h.frame, {0, 0, 0, 0, 0}};
                }
                if (counts) counts[i] = n;
                total += n;
            }
        }
        ssa_amd_stats_t& S = stats();
        S.kernel_ms = kms;
        S.cells = cells;
        S.kernel_launches = launches;
        S.part_retries = retries;
        S.filter_candidates = ncand;
        S.search_ms = now_ms() - t0;
        S.total_searches = before.total_searches + nq;
        S.total_kernel_ms = before.total_kernel_ms + kms;
        S.total_search_ms = before.total_search_ms + S.search_ms;
        return total;
    }
    uint32_t retries = 0, launches = 0;
    uint64_t ncand = 0;
    for (size_t i = 0; i < nq; i++) {
        test_configuration(queries[i]);
        SearchResult R;
        run_search(queries[i], algo == SSA_AMD_NW ? kAlgoNW : kAlgoSW, hitcount, bit_width, false, R);
        kms += stats().kernel_ms;
        cells += stats().cells;
        retries += stats().part_retries;
        ncand += stats().filter_candidates;
        launches += stats().kernel_launches;
        const size_t n = std::min(hitcount, R.hits.size());
        for (size_t j = 0; j < n; j++) {
            const Hit& h = R.hits[j];
            out[i * hitcount + j] = ssa_hit_t{h.score, h.id, h.qid, h.strand, h.frame, {0, 0, 0, 0, 0}};
        }
        if (counts) counts[i] = n;
        total += n;
    }
    // batch aggregates, like the pipelined path (the running totals were
    // advanced by run_search, once per query)
    ssa_amd_stats_t& S = stats();
    S.kernel_ms = kms;
    S.cells = cells;
    S.part_retries = retries;
    S.filter_candidates = ncand;
    S.kernel_launches = launches;
    S.search_ms = now_ms() - t0;
    return total;
}

size_t ssa_amd_replay(const ssa_hit_t* log, size_t n, size_t hitcount, ssa_hit_t* out) {
    TopK heap(hitcount);
    for (size_t i = 0; i < n; i++) {
        if (heap.full() && log[i].score <= heap.root_score()) continue;
        heap.add(Hit{log[i].score, log[i].db_id, log[i].query_id, log[i].db_strand, log[i].db_frame});
    }
    std::vector<Hit> v = heap.sorted();
    for (size_t i = 0; i < v.size(); i++)
        out[i] = ssa_hit_t{v[i].score, v[i].id, v[i].qid, v[i].strand, v[i].frame, {0, 0, 0, 0, 0}};
    return v.size();
}

}  // extern "C"
