// engine.cpp -- packs the plugin's DB into the device layout once (cached
// until init_db / a symbol-type change), then runs searches on one device.
//
// Replaces the reference's per-search chunk pipeline (db_adapter.c:212-239
// re-fetches and re-maps every sequence on every search) and its per-thread
// SIMD drivers (search_16.c:92-134, search_8.c:94-146).
#include <algorithm>
#include <functional>
#include <array>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <numeric>
#include <thread>

#include "bulk_alloc.h"
#include "engine.h"

namespace ssa {

// (events: see upload_pack)
static const unsigned kEventFlags = hipEventReleaseToDevice;

ssa_amd_stats_t& stats() {
    static ssa_amd_stats_t s;
    return s;
}

double now_ms() {
    using namespace std::chrono;
    return duration<double, std::milli>(steady_clock::now().time_since_epoch()).count();
}

// SSA_AMD_TRACE: the host's timeline of one call (host_mark at the points
// below), recorded on the calling thread between host_marks_begin and the
// print in api.cpp align(); other threads (device slots) record nothing
namespace {
thread_local std::vector<std::pair<const char*, double>> t_marks;
thread_local bool t_marks_on = false;
}  // namespace
const std::vector<std::pair<const char*, double>>& host_marks() { return t_marks; }
void host_marks_begin(bool on) {
    t_marks.clear();
    t_marks_on = on;
}
void host_mark(const char* what) {
    if (t_marks_on) t_marks.emplace_back(what, now_ms());
}

void check(hipError_t e, const char* what) {
    if (e != hipSuccess) fatal("HIP error in %s: %s", what, hipGetErrorString(e));
}

DeviceDB& device_db(size_t slot) {
    static DeviceDB slots[kMaxSlots];
    if (slot >= kMaxSlots) fatal("device slot %zu out of range", slot);
    return slots[slot];
}

static void dfree(void* p) {
    if (p) (void)hipFree(p);
}

void DeviceDB::SearchGraph::reset() {
    if (exec) (void)hipGraphExecDestroy(exec);
    if (g) (void)hipGraphDestroy(g);
    exec = nullptr;
    g = nullptr;
    ops.clear();
    nodes.clear();
    used = 0;
}

void DeviceDB::release() {
    // the buffers belong to `device`: free them there (a failure here means
    // the device is gone -- fatal, as every other HIP error of the library)
    if (device >= 0) check(hipSetDevice(device), "hipSetDevice");
    // (the cached graph names the buffers freed below)
    graph.reset();
    graph.broken = false;
    plans.reset();
    dfree(d_groups); dfree(d_res); dfree(d_rowbuf); dfree(d_lane_len); dfree(d_lane_out);
    dfree(d_scores); dfree(d_ovf); dfree(d_wide); dfree(d_qpt); dfree(d_upblk);
    dfree(d_work); dfree(d_order); dfree(d_lscratch); dfree(d_rscratch);
    d_rscratch = nullptr;
    rscratch_cap = 0;
    dfree(d_flags); dfree(d_flist); dfree(d_cnt); dfree(d_res_cls); dfree(d_frlist); dfree(d_frwork);
    d_frlist = nullptr; d_frwork = nullptr; frwork_cap = 0;
    dfree(d_hmm);
    d_hmm = nullptr;
    dfree(d_part);
    dfree(d_smax);
    d_part = d_smax = nullptr;
    part_cap = smax_cap = 0;
    dfree(d_rowbuf_q);
    d_rowbuf_q = nullptr;
    rowbuf_q_cap = 0;
    dfree(d_rowbuf2);
    d_rowbuf2 = nullptr;
    dfree(d_rowbuf3);
    d_rowbuf3 = nullptr;
    for (auto& pr : prs) {
        dfree(pr.d);
        pr = PairRows();
    }
    dfree(d_timeline);
    d_timeline = nullptr;
    timeline_cap = timeline_rows = 0;
    dfree(d_entry_lane);
    d_entry_lane = nullptr;
    dfree(d_emask);
    d_emask = nullptr;
    code_entries.clear();
    dfree(d_exact);
    d_exact = nullptr;
    exact_cap = 0;
    if (h_exact) (void)hipHostFree(h_exact);
    h_exact = nullptr;
    hmm_cap = 0;
    d_res_cls = nullptr;
    cls_key.clear();
    if (h_cnt) (void)hipHostFree(h_cnt);
    d_flags = nullptr; d_flist = nullptr; d_cnt = nullptr; h_cnt = nullptr;
    flags_cap = 0;
    cnt_dirty = true;                     // a new d_cnt block starts unzeroed
    gate_count = 0;
    d_lscratch = nullptr;
    lscratch_cap = 0;
    d_upblk = nullptr;
    upblk_cap = 0;
    d_order = nullptr;
    h_order.clear();
    order_key = ~0ull;
    scores_cap = filter_cap = 0;
    for (auto& e : vev) (void)hipEventDestroy(e);
    vev.clear();
    d_top = nullptr;
    dfree(d_topc);
    d_topc = nullptr;
    topc_cap = 0;
    topc_key = ~0ull;
    dfree(d_fbuf); dfree(d_summary); dfree(d_before); dfree(d_thresh); dfree(d_thresh_local);
    if (h_fbuf) (void)hipHostFree(h_fbuf);
    if (h_up) (void)hipHostFree(h_up);
    h_up = nullptr;
    h_up_cap = 0;
    d_fbuf = nullptr; d_summary = nullptr; d_before = nullptr; d_thresh = nullptr;
    d_thresh_local = nullptr;
    h_fbuf = nullptr; h_cand_cap = 0;
    if (h_scores) (void)hipHostFree(h_scores);
    if (h_ovf) (void)hipHostFree(h_ovf);
    if (h_wide) (void)hipHostFree(h_wide);
    d_groups = nullptr; d_res = nullptr; d_rowbuf = nullptr; d_lane_len = nullptr; d_lane_out = nullptr;
    d_scores = nullptr; d_ovf = nullptr; d_wide = nullptr; d_qpt = nullptr; d_query = nullptr;
    d_matrix = nullptr; d_work = nullptr; h_scores = nullptr; h_ovf = nullptr; h_wide = nullptr;
    h_scores_cap = qpt_cap = work_cap = 0;
    generation = ~0ull;
    meta = EntryMeta();
    lane_out.clear();
}

constexpr size_t kOvfPinned = 4096;      // overflow entries the pinned mirrors hold (more: pageable copies)
// per-search device upload block: [kernel-code matrix 8 KiB][code-0 row 256 B][top boundary][query]
// per-search upload block: kernel-code matrix (8 KB), code 0's row (256 B),
// the compact-code matrix of the rare-code merge's exact re-score (8 KB)
constexpr size_t kUpExactMat = 8192 + 256;
constexpr size_t kUpHeader = 8192 + 256 + 8192;
constexpr size_t kExactPinned = 1024;    // exact re-score results the pinned mirror holds

// ------------------------------------------------------------ entry codes
// Mapped residues of one entry, as db_adapter.c:47-110 builds them: NT codes
// (reverse complement for strand 1), translated frames for TRANS_DB/BOTH,
// amino-acid codes otherwise; unknown symbols become 0.
static size_t map_record(const char* s, size_t n, const signed char* map, uint8_t* out) {
    size_t unknown = 0;
    for (size_t i = 0; i < n; i++) {
        const signed char m = map[(unsigned char)s[i]];
        if (m >= 0) out[i] = (uint8_t)m;
        else { out[i] = 0; unknown++; }
    }
    return unknown;
}

std::vector<uint8_t> fetch_entry_codes(uint64_t local_id, int strand, int frame) {
    p_seqinfo si = ssa_db_get_sequence(local_id);
    if (!si) fatal("Could not get sequence from DB: %ld", (long)local_id);
    const int st = cfg().symtype;
    std::vector<uint8_t> v(si->seqlen + 1, 0);
    if (st == NUCLEOTIDE) {
        map_record(si->seq, si->seqlen, map_nt(), v.data());
        (void)strand;  // reference aligner.c:76 / util_sequence.c:394-402 never flips it here
    } else if (st == TRANS_DB || st == TRANS_BOTH) {
        map_record(si->seq, si->seqlen, map_nt(), v.data());
        return translate(true, v.data(), si->seqlen, strand, frame);
    } else {
        map_record(si->seq, si->seqlen, map_aa(), v.data());
    }
    return v;
}

// ---------------------------------------------------------------- packing
namespace {
struct Staged {
    EntryMeta meta;
    std::vector<uint64_t> off;       // entry -> offset into codes
    Bytes codes;
    std::array<uint8_t, 256> seen{};     // codes that occur
    std::vector<std::pair<size_t, size_t>> unknown;   // (record, count) with unknown symbols
};

// Records [r0, r1) -> entries, as db_adapter.c:47-110 + 212-239 build them.
void stage_range(size_t r0, size_t r1, Staged& S) {
    const int st = cfg().symtype, strands = cfg().strands;
    EntryMeta& M = S.meta;
    std::vector<uint8_t> nt;
    for (size_t id = r0; id < r1; id++) {
        p_seqinfo si = ssa_db_get_sequence(id);
        if (!si) break;
        if (si->seqlen == 0) continue;
        const size_t n = si->seqlen;
        const size_t cb = S.codes.size();
        auto add = [&](const uint8_t* c, size_t len, int strand, int frame) {
            M.id.push_back(id);
            M.strand.push_back((uint8_t)strand);
            M.frame.push_back((uint8_t)frame);
            M.len.push_back((uint32_t)len);
            S.off.push_back(S.codes.size());
            S.codes.insert(S.codes.end(), c, c + len);
            M.residues += len;
        };
        size_t unknown;
        if (st == NUCLEOTIDE) {
            nt.resize(n);
            unknown = map_record(si->seq, n, map_nt(), nt.data());
            add(nt.data(), n, 0, 0);
            if (strands & 2) {
                std::vector<uint8_t> rc(n);
                revcompl(nt.data(), n, rc.data());
                add(rc.data(), n, 1, 0);
            }
        } else if (st == TRANS_DB || st == TRANS_BOTH) {
            nt.resize(n);
            unknown = map_record(si->seq, n, map_nt(), nt.data());
            if (strands == BOTH_STRANDS) {
                for (int s = 0; s < 2; s++)
                    for (int f = 0; f < 3; f++) {
                        auto p = translate(true, nt.data(), n, s, f);
                        add(p.data(), p.size() - 1, s, f);
                    }
            } else {
                // reference quirk (db_adapter.c:85-93): strand field = strands
                for (int f = 0; f < 3; f++) {
                    auto p = translate(true, nt.data(), n, strands - 1, f);
                    add(p.data(), p.size() - 1, strands, f);
                }
            }
        } else {
            const size_t base = S.codes.size();
            S.codes.resize(base + n);
            unknown = map_record(si->seq, n, map_aa(), S.codes.data() + base);
            M.id.push_back(id);
            M.strand.push_back(0);
            M.frame.push_back(0);
            M.len.push_back((uint32_t)n);
            S.off.push_back(base);
            M.residues += n;
        }
        if (unknown > 0) S.unknown.push_back({id, unknown});
        // the codes that occur (the compact alphabet), marked while the
        // record's codes are still in cache
        const uint8_t* cw = S.codes.data();
        for (size_t i = cb, e = S.codes.size(); i < e; i++) S.seen[cw[i]] = 1;
    }
}

unsigned host_threads() { return std::max(1u, std::min(16u, std::thread::hardware_concurrency())); }

// The parse threads' parts, merged by reference: one metadata array over all
// entries, and per entry a pointer to its codes inside its part (the parts'
// code buffers are never concatenated: 3.6 GB for the 10 M DB).
struct StagedDB {
    EntryMeta meta;
    std::vector<const uint8_t*> src;
    std::vector<Staged> parts;
};

// The plugin is called from several threads at once, as the reference's
// own search threads do (adp_next_chunk runs in every worker).
void stage_from_plugin(StagedDB& S, size_t rb, size_t re) {
    const size_t count = re - rb;
    const unsigned nth = count < 20000 ? 1u : host_threads();
    S.parts.assign(nth, Staged());
    std::vector<std::thread> pool;
    for (unsigned t = 0; t < nth; t++)
        pool.emplace_back([&, t]() { stage_range(rb + count * t / nth, rb + count * (t + 1) / nth, S.parts[t]); });
    for (auto& th : pool) th.join();
    S.meta.records = count;
    // the parts' entries at their prefix offsets, one thread per part
    std::vector<size_t> at(nth + 1, 0);
    for (unsigned t = 0; t < nth; t++) at[t + 1] = at[t] + S.parts[t].meta.size();
    const size_t ne = at[nth];
    S.meta.id.resize(ne); S.meta.strand.resize(ne); S.meta.frame.resize(ne); S.meta.len.resize(ne);
    S.src.resize(ne);
    pool.clear();
    for (unsigned t = 0; t < nth; t++)
        pool.emplace_back([&, t]() {
            Staged& P = S.parts[t];
            const size_t b = at[t], n = P.meta.size();
            std::copy(P.meta.id.begin(), P.meta.id.end(), S.meta.id.begin() + b);
            std::copy(P.meta.strand.begin(), P.meta.strand.end(), S.meta.strand.begin() + b);
            std::copy(P.meta.frame.begin(), P.meta.frame.end(), S.meta.frame.begin() + b);
            std::copy(P.meta.len.begin(), P.meta.len.end(), S.meta.len.begin() + b);
            for (size_t i = 0; i < n; i++) S.src[b + i] = P.codes.data() + P.off[i];
        });
    for (auto& th : pool) th.join();
    for (auto& P : S.parts) {
        S.meta.residues += P.meta.residues;
        for (auto& u : P.unknown) print_warning("%ld unknown symbols found and set to zero", (long)u.second);
        P.meta = EntryMeta();
        P.off = std::vector<uint64_t>();
    }
}

// Device layout built on the host; also the on-disk format.
struct HostPack {
    EntryMeta meta;
    std::vector<GroupDesc> groups;
    std::vector<uint32_t> lane_len, lane_out;
    Bytes res;                          // blocks * 1 KiB
    std::vector<uint8_t> code_of;
    uint64_t blocks = 0;
};

void build_host_pack(HostPack& H, size_t rb, size_t re) {
    const double t0 = now_ms();
    StagedDB S;
    stage_from_plugin(S, rb, re);
    const size_t E = S.meta.size();
    const double t1 = now_ms();

    // length-sorted groups of 64 lanes (longest first: long waves start
    // early); a stable counting sort by length, entry order within a length
    uint32_t maxlen = 0;
    for (uint32_t l : S.meta.len) maxlen = std::max(maxlen, l);
    std::vector<uint32_t> order(E);
    if (maxlen < (1u << 24)) {
        std::vector<uint64_t> start((size_t)maxlen + 2, 0);
        for (uint32_t l : S.meta.len) start[(size_t)(maxlen - l) + 1]++;
        for (size_t i = 1; i < start.size(); i++) start[i] += start[i - 1];
        for (uint32_t e = 0; e < E; e++) order[start[maxlen - S.meta.len[e]]++] = e;
    } else {
        std::iota(order.begin(), order.end(), 0u);
        std::stable_sort(order.begin(), order.end(),
                         [&](uint32_t a, uint32_t b) { return S.meta.len[a] > S.meta.len[b]; });
    }
    const uint32_t ngroups = (uint32_t)((E + 63) / 64);
    H.groups.resize(ngroups);
    uint64_t blocks = 0;
    for (uint32_t g = 0; g < ngroups; g++) {
        const uint32_t longest = S.meta.len[order[(size_t)g * 64]];
        // columns to compute: longest + 1 (the high half lags one column),
        // rounded to the 4-column row-buffer quad; residues in 16-column blocks
        const uint32_t ncols = ((longest + 1) + 3) / 4 * 4;
        H.groups[g].blk = (uint32_t)blocks;
        H.groups[g].ncols = ncols;
        blocks += (ncols + 15) / 16;
    }
    if (blocks >= (1ull << 32)) fatal("DB shard too large for one device (%llu KiB of residues)", (unsigned long long)blocks);
    H.blocks = blocks;
    const double t2 = now_ms();
    const unsigned nth = host_threads();
    // compact alphabet: the residue codes that occur, in code order; the
    // padding column gets the next code.  Pair-symbol profiles scale with
    // (alpha+1)^2, so a 20-letter DB uses 441 rows instead of 1024.
    uint8_t remap[256] = {0};
    H.code_of.clear();
    for (int c = 0; c < 256; c++) {
        bool any = false;
        for (auto& P : S.parts) any |= P.seen[c] != 0;
        if (any) {
            remap[c] = (uint8_t)H.code_of.size();
            H.code_of.push_back((uint8_t)c);
        }
    }
    if (H.code_of.size() > 31) fatal("residue alphabet too large (%d codes)", (int)H.code_of.size());
    const uint8_t pad = (uint8_t)H.code_of.size();
    H.lane_len.assign((size_t)ngroups * 64, 0);
    H.lane_out.assign((size_t)ngroups * 64, 0xffffffffu);
    const double t3 = now_ms();
    // (no serial fill: every group's thread pads its own blocks)
    H.res.resize((size_t)blocks * 1024);
    const double t4 = now_ms();
    std::vector<std::thread> pool;
    for (unsigned t = 0; t < nth; t++) {
        pool.emplace_back([&, t]() {
            for (uint32_t g = t; g < ngroups; g += nth) {
                uint8_t* gbase = H.res.data() + (size_t)H.groups[g].blk * 1024;
                memset(gbase, pad, (size_t)(H.groups[g].ncols + 15) / 16 * 1024);
                for (uint32_t l = 0; l < 64; l++) {
                    const size_t pos = (size_t)g * 64 + l;
                    if (pos >= E) break;
                    const uint32_t e = order[pos];
                    const uint32_t n = S.meta.len[e];
                    H.lane_len[pos] = n;
                    H.lane_out[pos] = e;
                    const uint8_t* src = S.src[e];
                    for (uint32_t c = 0; c < n; c++) gbase[(size_t)(c / 16) * 1024 + l * 16 + (c & 15)] = remap[src[c]];
                }
            }
        });
    }
    for (auto& th : pool) th.join();
    H.meta = std::move(S.meta);
    if (trace_on())
        fprintf(stderr, "trace: pack stage %.1f ms, sort %.1f, alphabet %.1f, fill %.1f, scatter %.1f ms\n", t1 - t0,
                t2 - t1, t3 - t2, t4 - t3, now_ms() - t4);
}

void upload_pack(DeviceDB& D, HostPack& H, int dev) {
    const Config& C = cfg();
    const double t_al0 = now_ms();
    D.release();
    check(hipSetDevice(dev), "hipSetDevice");
    D.device = dev;
    if (!D.stream) {
        // how the host waits for a search (option "sync_spin"): HIP's default
        // on a machine with more CPUs than contexts yields the waiting thread;
        // spinning keeps it on its core -- 15 us less from the result's copy
        // to the next search's first launch (profiles/r05/host_gap/kgap_spin.txt
        // vs kgap_nospin.txt, one box).  Set before this library's first use
        // of the device; a context another runtime user made first keeps its
        // flags (the call's error is cleared)
        if (C.sync_spin && hipSetDeviceFlags(hipDeviceScheduleSpin) != hipSuccess) (void)hipGetLastError();
        // the code object holds gfx950 kernels only, and the launch plans use
        // gfx950's measured LDS allocation rule (kernels.h pair_wgs_per_cu)
        hipDeviceProp_t prop;
        check(hipGetDeviceProperties(&prop, dev), "hipGetDeviceProperties");
        if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
            fatal("libssa_amd is built for gfx950 (MI355X) only; device %d is %s", dev, prop.gcnArchName);
        check(hipStreamCreateWithFlags(&D.stream, hipStreamNonBlocking), "hipStreamCreate");
        // the long-entry kernels' streams at the device's highest priority:
        // their workgroups are the search's critical path (see also the gate,
        // TableArgs::gate)
        int prio_lo = 0, prio_hi = 0;
        if (hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi) != hipSuccess) {
            (void)hipGetLastError();
            prio_hi = 0;
        }
        check(hipStreamCreateWithPriority(&D.stream_long, hipStreamNonBlocking, prio_hi), "hipStreamCreate");
        check(hipStreamCreateWithPriority(&D.stream_long1, hipStreamNonBlocking, prio_hi), "hipStreamCreate");
        // every event of a search orders work on this device (timing
        // markers, the long kernels' join, the staging buffer's reuse): a
        // device-scope release, not a system-scope one (an L2 writeback of
        // the search's row-buffer lines each time, ~5 us on the path)
        for (auto& e : D.ev) check(hipEventCreateWithFlags(&e, kEventFlags), "hipEventCreate");
        check(hipEventCreateWithFlags(&D.ev_fork, hipEventDisableTiming), "hipEventCreate");
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && cus > 0)
            D.nsimd = (uint32_t)cus * 4;
    }
    const size_t E = H.meta.size();
    auto dalloc = [&](void** p, size_t bytes, const char* what) {
        check(hipMalloc(p, bytes ? bytes : 16), what);
    };
    dalloc((void**)&D.d_groups, H.groups.size() * sizeof(GroupDesc), "groups");
    dalloc((void**)&D.d_res, H.res.size(), "residues");
    dalloc((void**)&D.d_rowbuf, H.res.size() * 4, "row buffer");
    dalloc((void**)&D.d_lane_len, H.lane_len.size() * 4, "lane_len");
    dalloc((void**)&D.d_lane_out, H.lane_out.size() * 4, "lane_out");
    {
        const size_t nb = (E + kFilterBlock - 1) / kFilterBlock;
        dalloc((void**)&D.d_fbuf, kFilterHeader * 4 + std::max<size_t>(E, 1) * 8, "filter candidates");
        D.filter_cap = std::max<size_t>(E, 1);
        D.fbuf_bytes = kFilterHeader * 4 + std::max<size_t>(E, 1) * 8;
        D.h_fbuf_regions = 1;
        dalloc((void**)&D.d_summary, std::max<size_t>(nb, 1) * kFilterMaxK * 8, "filter summaries");   // (8 B: the one-pass look-back words)
        dalloc((void**)&D.d_before, std::max<size_t>(nb, 1) * kFilterMaxK * 4, "filter scan");
        dalloc((void**)&D.d_thresh_local, std::max<size_t>(nb, 1) * 64 * 4, "filter local thresholds");
        dalloc((void**)&D.d_thresh, std::max<size_t>(nb, 1) * 4, "filter thresholds");
        D.filter_blocks_cap = std::max<size_t>(nb, 1);
        D.h_cand_cap = 4096;
        check(hipHostMalloc((void**)&D.h_fbuf, kFilterHeader * 4 + D.h_cand_cap * 8, hipHostMallocDefault), "pinned");
    }
    dalloc((void**)&D.d_scores, std::max<size_t>(E, 1) * 4, "scores");
    D.scores_cap = std::max<size_t>(E, 1);
    // one view slice of the overflow list (grown per search for pipelined views)
    dalloc((void**)&D.d_ovf, (H.lane_len.size() + 1) * 4, "overflow list");
    dalloc((void**)&D.d_wide, std::max<size_t>(H.lane_len.size(), 1) * 8, "wide scores");
    D.ovf_slices = 1;
    dalloc((void**)&D.d_flist, (H.lane_len.size() + 1) * 4, "overflow-flag replay list");
    dalloc((void**)&D.d_frlist, (H.lane_len.size() + 1) * 4, "overflow-flag replay list");
    // overflow counters, then the long-entry dispatch gate (TableArgs::gate)
    // (+ the one-pass filter's ticket and done words, two per query of a
    // fused batch: zero between searches, FilterArgs::pass)
    dalloc((void**)&D.d_cnt, 16 * kMaxBatchPipe + 16 + 8 * kMaxFuse, "overflow counters");
    check(hipMemset(D.d_cnt, 0, 16 * kMaxBatchPipe + 16 + 8 * kMaxFuse), "memset");
    check(hipHostMalloc((void**)&D.h_cnt, 16 * kMaxBatchPipe + 16, hipHostMallocDefault), "pinned");
    const double t_up0 = now_ms();
    if (trace_on()) fprintf(stderr, "trace: pack device allocations %.1f ms\n", t_up0 - t_al0);
    D.upblk_cap = kUpHeader + 16384 + 4096;
    dalloc((void**)&D.d_upblk, D.upblk_cap, "per-search uploads");
    D.d_matrix = (int64_t*)D.d_upblk;
    check(hipHostMalloc((void**)&D.h_ovf, (kOvfPinned + 1) * 4, hipHostMallocDefault), "pinned");
    check(hipHostMalloc((void**)&D.h_wide, kOvfPinned * 8, hipHostMallocDefault), "pinned");
    check(hipMemcpy(D.d_groups, H.groups.data(), H.groups.size() * sizeof(GroupDesc), hipMemcpyHostToDevice), "H2D");
    check(hipMemcpy(D.d_res, H.res.data(), H.res.size(), hipMemcpyHostToDevice), "H2D residues");
    check(hipMemcpy(D.d_lane_len, H.lane_len.data(), H.lane_len.size() * 4, hipMemcpyHostToDevice), "H2D");
    check(hipMemcpy(D.d_lane_out, H.lane_out.data(), H.lane_out.size() * 4, hipMemcpyHostToDevice), "H2D");
    {
        // entry-ordered (length, lane): the overflow-flag pass reads them
        // coalesced, entry by entry (lane order would gather the scores)
        std::vector<uint32_t> el(std::max<size_t>(2 * E, 2), 0);
        for (size_t l = 0; l < H.lane_out.size(); l++) {
            const uint32_t e = H.lane_out[l];
            if (e != 0xffffffffu) {
                el[2 * (size_t)e] = H.lane_len[l];
                el[2 * (size_t)e + 1] = (uint32_t)l;
            }
        }
        dalloc((void**)&D.d_entry_lane, el.size() * 4, "entry lanes");
        check(hipMemcpy(D.d_entry_lane, el.data(), el.size() * 4, hipMemcpyHostToDevice), "H2D");
    }
    if (trace_on()) fprintf(stderr, "trace: pack upload %.1f ms (%zu B residues)\n", now_ms() - t_up0, H.res.size());
    D.ngroups = (uint32_t)H.groups.size();
    D.group_ncols.resize(H.groups.size());
    D.ncols_sum = 0;
    for (size_t g = 0; g < H.groups.size(); g++) {
        D.group_ncols[g] = H.groups[g].ncols;
        D.ncols_sum += H.groups[g].ncols;
    }
    D.nblocks = H.blocks;
    // ascending lengths: the lanes hold the entries longest first (padding
    // lanes of the last group at the end, length 0), so reversed
    D.len_sorted.assign(H.lane_len.rbegin() + (H.lane_len.size() - E), H.lane_len.rend());
    D.meta = std::move(H.meta);
    D.lane_out = std::move(H.lane_out);
    D.code_of = std::move(H.code_of);
    D.alpha = (uint32_t)D.code_of.size();
    D.generation = C.db_generation;
    D.symtype = C.symtype;
    D.strands = C.strands;
    D.dgencode = C.d_gencode;
}

// ------------------------------------------------------ packed DB files
// "SSAPACK1" | u32 version, symtype, strands, dgencode | u64 records,
// entries, residues, ngroups, blocks | u32 alpha, 0 | u8 code_of[32] |
// u64 id[E] | u8 strand[E] | u8 frame[E] | u32 len[E] | GroupDesc[ngroups]
// | u32 lane_len[64 ngroups] | u32 lane_out[64 ngroups] | u8 res[1 KiB * blocks]
constexpr char kPackMagic[8] = {'S', 'S', 'A', 'P', 'A', 'C', 'K', '1'};
constexpr uint32_t kPackVersion = 1;

template <class T>
bool wr(FILE* f, const T* p, size_t n) { return n == 0 || fwrite(p, sizeof(T), n, f) == n; }
template <class T>
bool rd(FILE* f, T* p, size_t n) { return n == 0 || fread(p, sizeof(T), n, f) == n; }

}  // namespace

std::vector<SlotPlan> device_plan() {
    const Config& C = cfg();
    const size_t count = ssa_db_get_sequence_count();
    if (C.devices.size() <= 1) {
        int dev = C.devices.empty() ? C.device : C.devices[0];
        if (dev < 0) check(hipGetDevice(&dev), "hipGetDevice");
        return {{dev, 0, count}};
    }
    // cut at chunk boundaries, balancing residues (cached per DB generation)
    static uint64_t gen = ~0ull;
    static std::vector<int> devs;
    static size_t chunk = 0, cnt = 0;
    static std::vector<SlotPlan> plan;
    if (gen == C.db_generation && devs == C.devices && chunk == C.chunk_size && cnt == count) return plan;
    const size_t n = C.devices.size();
    // one residue sum per chunk_size chunk (the cuts fall on chunk
    // boundaries anyway): 8 B per chunk, not per record (50 M records would
    // otherwise hold 400 MB of lengths for the duration of the cut)
    const size_t cs = std::max<size_t>(C.chunk_size, 1);
    const size_t nch = (count + cs - 1) / cs;
    std::vector<uint64_t> sums(nch, 0);
    for (size_t i = 0; i < count; i++) {
        p_seqinfo si = ssa_db_get_sequence(i);
        if (si) sums[i / cs] += si->seqlen;
    }
    std::vector<size_t> bounds(n + 1);
    ssa_amd_shard_bounds(sums.data(), nch, n, 1, bounds.data());
    plan.clear();
    for (size_t s = 0; s < n; s++)
        plan.push_back({C.devices[s], std::min(count, bounds[s] * cs), std::min(count, bounds[s + 1] * cs)});
    gen = C.db_generation;
    devs = C.devices;
    chunk = C.chunk_size;
    cnt = count;
    return plan;
}

bool ensure_device_db(size_t slot, const SlotPlan& p) {
    DeviceDB& D = device_db(slot);
    const Config& C = cfg();
    if (D.generation == C.db_generation && D.device == p.device && D.symtype == C.symtype &&
        D.strands == C.strands && D.dgencode == C.d_gencode && D.rec_begin == p.rec_begin && D.rec_end == p.rec_end)
        return false;
    check(hipSetDevice(p.device), "hipSetDevice");
    const double t0 = now_ms();
    {
        HostPack H;
        build_host_pack(H, p.rec_begin, p.rec_end);
        upload_pack(D, H, p.device);
        if (trace_on()) fprintf(stderr, "trace: pack build+upload %.1f ms\n", now_ms() - t0);
    }
    if (trace_on()) fprintf(stderr, "trace: pack incl. host frees %.1f ms\n", now_ms() - t0);
    D.rec_begin = p.rec_begin;
    D.rec_end = p.rec_end;
    return true;
}

void ensure_device_db() {
    const std::vector<SlotPlan> plan = device_plan();
    const double t0 = now_ms();
    bool packed = false;
    if (plan.size() == 1) {
        packed = ensure_device_db(0, plan[0]);
    } else {
        std::vector<char> did(plan.size(), 0);
        std::vector<std::thread> pool;
        for (size_t s = 0; s < plan.size(); s++) pool.emplace_back([&, s]() { did[s] = ensure_device_db(s, plan[s]); });
        for (auto& t : pool) t.join();
        for (char d : did) packed |= d != 0;
    }
    if (packed) stats().pack_ms = now_ms() - t0;
}

int save_packed_db(const char* path) {
    if (device_plan().size() != 1) {
        print_error("Packed DB files are written from a single-device DB (ssa_amd_set_device, or SSA_AMD_DEVICES=current)");
        return 1;
    }
    ensure_device_db();
    DeviceDB& D = device_db(0);
    FILE* f = fopen(path, "wb");
    if (!f) {
        print_error("Cannot open packed DB file for writing: %s", path);
        return 1;
    }
    const uint64_t E = D.meta.size();
    std::vector<uint8_t> res((size_t)D.nblocks * 1024);
    std::vector<GroupDesc> groups(D.ngroups);
    std::vector<uint32_t> lane_len((size_t)D.ngroups * 64);
    check(hipSetDevice(D.device), "hipSetDevice");
    check(hipMemcpy(res.data(), D.d_res, res.size(), hipMemcpyDeviceToHost), "D2H residues");
    check(hipMemcpy(groups.data(), D.d_groups, groups.size() * sizeof(GroupDesc), hipMemcpyDeviceToHost), "D2H");
    check(hipMemcpy(lane_len.data(), D.d_lane_len, lane_len.size() * 4, hipMemcpyDeviceToHost), "D2H");
    const uint32_t hdr32[4] = {kPackVersion, (uint32_t)D.symtype, (uint32_t)D.strands, (uint32_t)D.dgencode};
    const uint64_t hdr64[5] = {(uint64_t)D.meta.records, E, D.meta.residues, D.ngroups, D.nblocks};
    const uint32_t alpha[2] = {D.alpha, 0};
    uint8_t code_of[32] = {0};
    std::copy(D.code_of.begin(), D.code_of.end(), code_of);
    bool ok = wr(f, kPackMagic, 8) && wr(f, hdr32, 4) && wr(f, hdr64, 5) && wr(f, alpha, 2) && wr(f, code_of, 32) &&
              wr(f, D.meta.id.data(), E) && wr(f, D.meta.strand.data(), E) && wr(f, D.meta.frame.data(), E) &&
              wr(f, D.meta.len.data(), E) && wr(f, groups.data(), groups.size()) &&
              wr(f, lane_len.data(), lane_len.size()) && wr(f, D.lane_out.data(), D.lane_out.size()) &&
              wr(f, res.data(), res.size());
    ok = (fclose(f) == 0) && ok;
    if (!ok) print_error("Writing packed DB file failed: %s", path);
    return ok ? 0 : 1;
}

int load_packed_db(const char* path) {
    const Config& C = cfg();
    FILE* f = fopen(path, "rb");
    if (!f) {
        print_error("Cannot open packed DB file: %s", path);
        return 1;
    }
    char magic[8];
    uint32_t hdr32[4], alpha[2];
    uint64_t hdr64[5];
    uint8_t code_of[32];
    HostPack H;
    auto fail = [&](const char* why) {
        fclose(f);
        print_error("Packed DB file %s: %s", path, why);
        return 1;
    };
    if (!rd(f, magic, 8) || memcmp(magic, kPackMagic, 8) || !rd(f, hdr32, 4) || !rd(f, hdr64, 5) ||
        !rd(f, alpha, 2) || !rd(f, code_of, 32))
        return fail("not a packed DB");
    if (hdr32[0] != kPackVersion) return fail("unsupported version");
    if ((int)hdr32[1] != C.symtype || (int)hdr32[2] != C.strands || (int)hdr32[3] != C.d_gencode)
        return fail("packed for another symbol type / strands / genetic code");
    if (hdr64[0] != ssa_db_get_sequence_count()) return fail("record count differs from the open DB");
    const std::vector<SlotPlan> plan = device_plan();
    if (plan.size() != 1) return fail("packed DB files load into a single device (ssa_amd_set_device, or SSA_AMD_DEVICES=current)");
    const uint64_t E = hdr64[1], ng = hdr64[3];
    if (alpha[0] > 31 || E > ng * 64 || ng > E / 64 + 1) return fail("corrupt header");
    H.meta.records = hdr64[0];
    H.meta.residues = hdr64[2];
    H.blocks = hdr64[4];
    H.code_of.assign(code_of, code_of + alpha[0]);
    H.meta.id.resize(E); H.meta.strand.resize(E); H.meta.frame.resize(E); H.meta.len.resize(E);
    H.groups.resize(ng);
    H.lane_len.resize(ng * 64);
    H.lane_out.resize(ng * 64);
    H.res.resize(H.blocks * 1024);
    if (!rd(f, H.meta.id.data(), E) || !rd(f, H.meta.strand.data(), E) || !rd(f, H.meta.frame.data(), E) ||
        !rd(f, H.meta.len.data(), E) || !rd(f, H.groups.data(), ng) || !rd(f, H.lane_len.data(), ng * 64) ||
        !rd(f, H.lane_out.data(), ng * 64) || !rd(f, H.res.data(), H.res.size()))
        return fail("truncated");
    fclose(f);
    // structural checks before anything reaches the device
    for (uint64_t g = 0; g < ng; g++) {
        const GroupDesc& G = H.groups[g];
        if ((uint64_t)G.blk + (G.ncols + 15) / 16 > H.blocks || G.ncols % 4) return fail("corrupt group table");
        for (int l = 0; l < 64; l++) {
            const uint32_t o = H.lane_out[g * 64 + l];
            if (o != 0xffffffffu && (o >= E || H.lane_len[g * 64 + l] != H.meta.len[o] ||
                                     H.lane_len[g * 64 + l] + 1 > G.ncols))
                return fail("corrupt lane table");
        }
    }
    const double t0 = now_ms();
    DeviceDB& D = device_db(0);
    upload_pack(D, H, plan[0].device);
    D.rec_begin = 0;
    D.rec_end = hdr64[0];
    stats().pack_ms = now_ms() - t0;
    return 0;
}

// ----------------------------------------------------------------- search
// Largest DB entry length n for which int16 NW provably never saturates:
// every H is bounded below by the two-gap path 2Q+(i+j+2)R and above by
// min(m,n)*maxM, and E/F/diagonal intermediates stay within one extra gap or
// score of those bounds.
static uint32_t nw_int16_limit(size_t m, int Q, int R, int64_t minM, int64_t maxM) {
    if (Q > 0 || R > 0) return 0;
    const int64_t up = std::max<int64_t>(maxM, 0), lo = std::min<int64_t>(minM, 0);
    auto ok = [&](uint64_t n) {
        const int64_t U = (int64_t)std::min<uint64_t>(m, n) * up + up;
        const int64_t L = 3 * (int64_t)Q + (int64_t)(m + n + 4) * R + lo;
        return U <= 32766 && L >= -32767;
    };
    if (!ok(0)) return 0;
    uint64_t a = 0, b = 0xffffffffull;
    if (ok(b)) return 0xffffffffu;
    while (b - a > 1) {
        const uint64_t c = (a + b) / 2;
        if (ok(c)) a = c; else b = c;
    }
    return (uint32_t)a;
}

// NW on f16 bit patterns (pair_kernel<.., NW=true>) works on diagonal-
// relative values X^ = X - (i+j)R stored as X^ + base; every real value and
// intermediate of an entry of length n (and of its +1 padding column) must
// stay inside [0x0400, 0x7BFF].  Lower bound (constant): H^ >= 2Q+2R (two-gap
// path), E^/F^/h^+Q >= 3Q+2R, diagonal input + profile >= 2Q+minM, the
// step-0 boundary input Q+4R; it fixes base.  Upper bound:
// H^ <= min(m, n+1) maxM + (m+n)|R| (+ one profile value and 2|R| for the
// diagonal input); it limits n.  Returns the largest admissible n (0 when the
// query cannot use the f16 path at all) and the base.
static uint32_t nw_f16_limit(size_t m, int Q, int R, int64_t minM, int64_t maxM, uint32_t* base) {
    *base = 0;
    if (Q > 0 || R > 0) return 0;
    const int64_t up = std::max<int64_t>(maxM, 0), lo = std::min<int64_t>(minM, 0);
    const int64_t L = std::min({3 * (int64_t)Q + 2 * (int64_t)R, 2 * (int64_t)Q + lo, (int64_t)Q + 4 * (int64_t)R,
                                2 * (int64_t)R}) - 2;
    const int64_t b = 0x0400 - L;
    auto ok = [&](uint64_t n) {
        const int64_t U = (int64_t)std::min<uint64_t>(m, n + 1) * up + (int64_t)(m + n + 2) * (-(int64_t)R) + up + 2;
        return U + b <= 0x7BFF;
    };
    if (!ok(0)) return 0;
    *base = (uint32_t)b;
    if (R == 0 && ok(0xffffffffull)) return 0xffffffffu;
    uint64_t a = 0, c = 0xffffffffull;
    while (c - a > 1) {
        const uint64_t x = (a + c) / 2;
        if (ok(x)) a = x; else c = x;
    }
    return (uint32_t)a;
}

// SW on the pair kernel: diagonal-relative patterns H + (i+j)|R| + 0x0800
// must stay below 0x7BFF for every real cell and the +1 padding column:
// H <= min(m,n) maxM, plus one profile value and 2|R| for the diagonal
// input.  The lower side holds by construction (floor >= 0x0800, minM and
// Q >= -1024).  Returns the largest admissible entry length (0: never).
static uint32_t sw_rel_limit(size_t m, int Q, int R, int64_t minM, int64_t maxM) {
    if (Q > 0 || R > 0 || Q < -1024 || minM < -1024 || maxM > 1024) return 0;
    const int64_t up = std::max<int64_t>(maxM, 0), rabs = -(int64_t)R;
    auto ok = [&](uint64_t n) {
        const int64_t U = (int64_t)std::min<uint64_t>(m, n) * up + (int64_t)(m + n + 4) * rabs + up + kF16Floor;
        return U <= 0x7BFF;
    };
    if (!ok(0)) return 0;
    if (R == 0) return 0xffffffffu;
    uint64_t a = 0, c = 0xffffffffull;
    while (c - a > 1) {
        const uint64_t x = (a + c) / 2;
        if (ok(x)) a = x; else c = x;
    }
    return (uint32_t)a;
}

// Leading (longest-first) groups that long_kernel scores instead of
// pair_kernel.  One pair_kernel lane scores a whole entry, so a group whose
// column count is a large part of one SIMD's share of the launch's columns
// keeps its wave running after the rest of the chip has drained (a 548 k-entry
// DB: 8.2 instead of 11.8 TCUPS); long_kernel spreads such an entry's query
// rows over a wave.  Also every group holding an entry beyond the pair
// kernel's f16 length bound (`beyond` entries, longest first).  Returns
// UINT32_MAX when `beyond` cannot be covered; 0 when the int32 bound of
// long_kernel does not hold or the option is off.
static constexpr uint32_t kLongMaxGroups = 256;
// pair kernel main strip half-height: the option when it names an
// instantiated one; else SW 24 (48 rows, three waves per SIMD) and NW the
// tallest of 40/32/24 whose table (prow^2 x (np+4) dwords) lets two
// workgroups share a CU.  At two waves per SIMD the kernel issues nearly as
// fast as at three (the wave timeline of a 548 k DB whose CUs held two pair
// workgroups beside a long one for a third of the launch: -1.5 % overall),
// and NW's 80-row strips (fewer boundary rows, per-strip and per-column work
// over more rows) gain more than that: C3 +5 %.  SW's taller strips carry
// the anti-diagonal accumulators too and measured 1-3 % slower (C2, C5;
// same box, alternating runs).
static int pair_strip_np(int opt, bool nw, uint32_t prow, size_t m) {
    if (opt == 16 || opt == 24 || opt == 32 || opt == 40 || (opt == 36 && !nw)) return opt;
    auto tbl = [&](int np) { return (size_t)pair_lds_rows(prow - 1) * (np + 4) * 4; };
    if (!nw) {
        // short SW queries whose rows fill 32-row strips better than 48-row
        // ones run at four waves per SIMD when four tables fit a CU
        // (profiles/r02/short_query_np.txt: q = 30 +1.4 %, q = 64 +2.1 %;
        // q = 100 is 5 % faster at 48 rows)
        const bool short_q = m <= 32 || (m > 48 && m <= 64);
        return short_q && pair_wgs_per_cu(tbl(16)) >= 4 ? 16 : 24;
    }
    // an NW query of at most 48 rows runs only the capture strip: at three
    // waves per SIMD rather than the 80-row strips' two (q = 30: +4.8 %,
    // profiles/r02/short_query_np.txt)
    if (m <= 48) return 24;
    for (int np : {40, 32})
        if (pair_wgs_per_cu(tbl(np)) >= 2) return np;
    return 24;
}

// strip parts of a pair-kernel launch of T strips (StripArgs::nparts; at
// most three: one row buffer per part, pair_kernel.h store_row's coherence
// argument).  Auto: two parts for groups of at least 4 strips -- C2 (9
// strips) +1.1 %, C3 (13) +1.1 %, the reference's benchmark shape (11)
// +6-8 %, q = 200 (5) +1 %; q = 100 (3) -2.3 % (profiles/r03/parts_sweep.txt)
static uint32_t strip_parts(uint32_t T) {
    const int o = cfg().pair_parts;
    const uint32_t p = o == 0 ? (T >= 4 ? 2u : 1u) : o >= 3 ? 3u : o == 2 ? 2u : 1u;
    return std::min(p, T);
}

// long_kernel at 4 waves per entry: rows per lane for an m-row query
// The rows per lane of a long-entry pass: the instantiated RL whose passes
// over the query cost the fewest row steps per column, ceil(m / (lanes RL))
// (RL + 1) (ties: the larger RL, fewer passes) -- an entry's latency is that times
// its columns, and the longest entries' latency is the long kernels'
// critical path (until round 6 the plan took the smallest single-pass RL of
// 4, 8, 9, 12, 16, else 16: q = 1046 ran two 16-row passes, 32 row steps,
// where two 9-row passes take 18 -- NW on the Swiss-Prot form 10.5 against
// 13.3 TCUPS beside it -- and q = 287 one 8-row pass where 5 rows do)
template <size_t N>
static int long_rl_fewest(size_t m, size_t lanes, const int (&rls)[N]) {
    int best = rls[0];
    size_t best_cost = SIZE_MAX;
    for (int rl : rls) {
        // (+1 row step per pass: its ramp, boundary row and profile)
        const size_t cost = (m + lanes * rl - 1) / (lanes * rl) * (rl + 1);
        if (cost <= best_cost) {
            best_cost = cost;
            best = rl;
        }
    }
    return best;
}
// ... at four waves per entry (its rows over the workgroup: 256 RL rows a pass)
static int long_rl4(size_t m) {
    static constexpr int kRl[] = {2, 3, 4};
    return long_rl_fewest(std::max<size_t>(m, 1), 256, kRl);
}
// ... at one wave per entry
static int long_rl1(size_t m) {
    static constexpr int kRl[] = {4, 5, 6, 7, 8, 9, 12, 16};   // (kernels.hip launch_long)
    return long_rl_fewest(std::max<size_t>(m, 1), 64, kRl);
}

// The exact int32 re-score tier (kernels.h LongArgs::list): the DP kernels'
// overflowed lanes are re-scored by long_kernel (one wave per entry, the
// reference's recurrences in int32) instead of wide_kernel (one thread per
// entry, int64, its H/E column in HBM) whenever int32 is exact for every
// entry of the DB: R, Q <= 0 (its SW clamps E and F at 0), the profile fits
// its int16 LDS table, and (m + n + 2)(max|M| + |Q| + |R|) < 2^30 for the
// longest entry n (long_plan's bound).  Returns the rows per lane, or 0.
static int rescore32_rl(const DeviceDB& D, size_t m, uint32_t A, int Q, int R, int64_t minM, int64_t maxM) {
    const Config& C = cfg();
    if (!C.rescore32 || C.force_wide || Q > 0 || R > 0 || A > 31 || D.len_sorted.empty() || m == 0) return 0;
    if (minM < -32768 || maxM > 32767) return 0;
    const int64_t amp = std::max(std::abs(minM), std::abs(maxM)) + std::abs((int64_t)Q) + std::abs((int64_t)R);
    if ((int64_t)(m + D.len_sorted.back() + 2) * amp >= (1ll << 30)) return 0;
    return long_rl1(m);
}
constexpr uint32_t kRescoreBlocks = 1024;    // the tier's grid: 4 workgroups per CU, looping over the list
constexpr uint32_t kTierMinBlocks = 256;     // ... or fewer when the last search's list was short

// long16_kernel (SW long entries on packed 16-bit patterns): the pattern of
// score 0 -- high enough that h + Q + R and E + R never borrow across the
// halves -- and the rows per lane for an m-row query (the fewest rows >= m
// of 64 x {4, 6, 8, 10, 12, 16}, passes of 1024 rows beyond), or 0 when the
// kernel does not apply: NW, the option off, or min(m, n) maxM (the largest
// SW score) beyond the patterns' finite range (kernels.hip long16_kernel)
static uint32_t long16_base(int Q, int R) { return 0x0400u + (uint32_t)std::max(0, -(Q + R)); }
static int long16_rl(const DeviceDB& D, size_t m, bool nw, int Q, int R, int64_t minM, int64_t maxM);

// long16_kernel's rows per lane RL and the query rows it leaves to its row
// scan (LongArgs::extra16, *extra).  Up to 1 024 rows: the smallest RL that
// holds the query in one pass (q = 513 at RL 8 + 1 scanned row instead of RL
// 10 issues 18 % less but measured no faster on the Swiss-Prot form,
// profiles/r05/ab/rows_sprot: the long waves' issue is not what the search
// waits on there).  Beyond, by issue cost per DB column: a pass step ~10.7 wave
// instructions per register (RL / 2 registers; hotloop census of the 16-step
// body) plus kPass for a pass's ramp and profile staging, a scanned row ~1 --
// q = 1025 one RL 16 pass + 1 row instead of two passes, q = 1500 two RL 12
// passes instead of two RL 16 ones (RL >= 8).  Ties go to the larger RL.
static int long16_plan(const DeviceDB& D, size_t m, bool nw, int Q, int R, int64_t minM, int64_t maxM,
                       uint32_t* extra) {
    *extra = 0;
    const int rl = long16_rl(D, m, nw, Q, R, minM, maxM);
    if (rl == 0 || !cfg().long16_rows || (m <= (size_t)64 * 16 && cfg().long16_rows != 2)) return rl;
    // (a pass's ramp, 2 x 63 steps, and profile staging: ~5 % of its steps
    // on a long entry; RL >= 8 keeps the pass count low)
    constexpr double kStep = 10.7, kRow = 1.0, kRamp = 1.05;
    constexpr size_t kExtraMax = 8;
    double best = 1e300;
    int brl = rl;
    for (int r : {16, 12, 10, 8, 6, 4}) {
        if (r < 8 && m > (size_t)64 * 16) continue;
        const size_t rp = (size_t)64 * r, full = m / rp, e = m - full * rp;
        const double step = r / 2 * kStep * kRamp;
        const double c = (double)((m + rp - 1) / rp) * step;
        if (c < best) {
            best = c;
            brl = r;
            *extra = 0;
        }
        if (full > 0 && e > 0 && e <= kExtraMax && (double)full * step + (double)e * kRow < best) {
            best = (double)full * step + (double)e * kRow;
            brl = r;
            *extra = (uint32_t)e;
        }
    }
    return brl;
}

static int long16_rl(const DeviceDB& D, size_t m, bool nw, int Q, int R, int64_t minM, int64_t maxM) {
    // (minM: a diagonal sum hd + M, hd >= base16, must stay a positive
    // pattern; a matrix value below -base16 could wrap it into the NaN
    // patterns 0xFC01..0xFFFF, which the maxima propagate)
    if (nw || !cfg().long16 || Q > 0 || R > 0 || Q + R < -16384 || minM < 1 - (int64_t)long16_base(Q, R) ||
        D.len_sorted.empty())
        return 0;
    const int64_t mp = std::max<int64_t>(maxM, 0);
    const int64_t hmax = (int64_t)std::min<size_t>(m, D.len_sorted.back()) * mp;
    if ((int64_t)long16_base(Q, R) + hmax + mp > 0x7BFF) return 0;
    for (int rl : {4, 6, 8, 10, 12})
        if (m <= (size_t)64 * rl) return rl;
    return 16;
}

constexpr double kLongTypical = 4.0;   // long_plan: the length tail's multiple of the median group
// long_plan's latency rule (tools/pairwise_probe.py, profiles/r06/ref_pairwise):
// pair_kernel's single wave per group takes about kPairNsPerCell ns per cell
// of its group's longest entry and its strips' rows; the long-entry kernels
// score about kLong16CellsPerNs (SW, packed) or kLong32CellsPerNs (int32)
// cells per ns over the whole chip, counted on the rows they pad the query to
constexpr double kPairNsPerCell = 6.0;
constexpr double kLong16CellsPerNs = 3400.0;
constexpr double kLong32CellsPerNs = 2200.0;
static uint32_t long_plan(const DeviceDB& D, size_t m, size_t beyond, int Q, int R, int64_t minM, int64_t maxM,
                          uint32_t scale = 1, bool nw = false, int strip_rows = 0) {
    const Config& C = cfg();
    const uint32_t need = (uint32_t)((beyond + 63) / 64);
    if (C.long_groups == 0 || D.ngroups == 0 || D.alpha > 32) return need ? UINT32_MAX : 0;
    // long_kernel's SW clamps E and F at 0: exact only for R <= 0
    if (Q > 0 || R > 0) return need ? UINT32_MAX : 0;
    const int64_t amp = std::max(std::abs(minM), std::abs(maxM)) + std::abs((int64_t)Q) + std::abs((int64_t)R);
    if ((int64_t)(m + D.len_sorted.back() + 2) * amp >= (1ll << 30)) return need ? UINT32_MAX : 0;
    uint32_t g = 0;
    if (C.long_groups > 0) {
        g = std::min<uint32_t>((uint32_t)C.long_groups, D.ngroups);
    } else {
        // A group is routed when its pair-kernel wave -- one lane per entry,
        // every column of its longest entry, strip after strip -- would
        // outlast the launch: on a DB that fills the chip twice over, when it
        // is longer than long_share_pct % of one SIMD's share of all columns
        // (a lower threshold costs more than it gains: long_kernel's cost per
        // cell is several times pair_kernel's -- the 548 k-entry DB: 40 %
        // 9.7, 50 % 10.9, 65 % 10.9 TCUPS); and on any DB never unless it is
        // kLongTypical times the median group's length -- a length tail (UniProt's
        // 5-35 k-residue entries) then goes to the long kernels even when the
        // DB is too small for the share rule (a 30 k-entry DB with such a tail
        // ran 48 ms in one pair wave), while a DB without a tail keeps its
        // groups (a moderate DB's share is shorter than its typical group:
        // the share rule alone routed half of a 150 k-entry DB's groups)
        double thr = kLongTypical * (double)D.group_ncols[D.ngroups / 2];
        if (D.ngroups >= 2 * D.nsimd)
            thr = std::max(thr, (double)D.ncols_sum / D.nsimd * C.long_share_pct / 100.0 * scale);
        while (g < D.ngroups && g < kLongMaxGroups && D.group_ncols[g] > thr) g++;
        // a DB too small to fill the chip (at most kLongMaxGroups groups): the
        // pair launch lasts as long as its longest group's one wave walking
        // every strip, while the long-entry kernels spread each entry over a
        // wave of its own -- with a query of two strips or more, every group
        // goes to them when their throughput estimate is the shorter
        // (P18080 as the one DB entry, query Q3ZAI3: SW 1.48 -> 0.14 ms)
        if (C.long_latency && g < D.ngroups && D.ngroups <= kLongMaxGroups && D.ngroups <= D.nsimd && strip_rows > 0 &&
            m > (size_t)strip_rows) {
            const size_t T = (m + strip_rows - 1) / strip_rows;
            const double pair_ns = kPairNsPerCell * D.group_ncols[0] * (double)(T * strip_rows);
            const int rl16 = long16_rl(D, m, nw, Q, R, minM, maxM);
            const size_t span = rl16 > 0 ? (size_t)64 * rl16 : (size_t)256 * long_rl4(m);
            const double padded = (double)((m + span - 1) / span * span);
            const double long_ns = 64.0 * (double)D.ncols_sum * padded / (rl16 > 0 ? kLong16CellsPerNs : kLong32CellsPerNs);
            if (long_ns < pair_ns) g = D.ngroups;
        }
    }
    g = std::max(g, need);
    return need > kLongMaxGroups ? UINT32_MAX : g;
}

// The kernels and bounds that score one query view (device_search):
// residue classes, profile bounds, pair-kernel admissibility and strip plan,
// long-entry groups.  Host only, no device work.  `force` (a fused batch,
// one pair_kernel launch for several queries): the profile bounds and the
// row count the length limits are computed for, shared by all its queries,
// and the factor by which the launch outlasts one query's (long groups).
struct ViewPlan {
    std::vector<uint8_t> cls_of, cls_rep;
    bool use_cls = false;
    // the kernels' codes' profile rows: crow[c * 32 + y] = score of kernel
    // code c against query code y (a class's representative row)
    std::vector<int64_t> crow;
    uint32_t A = 0, prow = 0;
    int64_t minM = 0, maxM = 0;
    uint32_t nmax16 = 0, nw_base = 0, long_groups = 0;
    int pnp = 0;
    size_t pair_lds = 0;
    bool use_pair = false, use_f16 = false;
    uint32_t nstrips = 0;
    int rel = 0;
    int16_t padv = 0;
    uint32_t main_strips = 0;
    int tail_np = 0;
    size_t tail_off = 0, qpt_words = 0;   // pair tables: tail offset, total dwords
    // rare-code merge: compact codes scored through the upper-bound class
    // (bit c), an upper bound of the entries that hold one, the int32 tier's
    // rows per lane for their exact re-score
    uint32_t merge_mask = 0;
    uint64_t merge_entries = 0;
    int merge_rl = 0;
    // the compact codes' profile bounds (the exact re-score's and, with a
    // merge, the long-entry kernels', which score the compact codes exactly)
    int64_t xminM = 0, xmaxM = 0;
};
struct PlanForce {
    int64_t minM, maxM;
    size_t m;
    uint32_t long_scale;
};

static void plan_view(const DeviceDB& D, const QueryView& qv, bool nw, int np, const PlanForce* force, ViewPlan& vp,
                      bool allow_merge = false, bool batch = false) {
    const Config& C = cfg();
    const int Q = C.gap_open, R = C.gap_extend;
    const int64_t* M = matrix().m;
    const size_t m = qv.len;
    const size_t ml = force ? force->m : m;        // row count of the length limits
    vp = ViewPlan();
    std::vector<uint8_t>& cls_of = vp.cls_of;
    std::vector<uint8_t>& cls_rep = vp.cls_rep;
    // residue classes of this view: DB codes whose matrix rows agree on
    // every residue of the query score identically, so the kernels may
    // see one code per class.  Used when it lets more pair-kernel
    // workgroups share a CU's LDS (the reference generator's uniform
    // 28-symbol DB: '-', U, O and X score alike against a standard-residue
    // query -> 25 classes, a 75.7 KiB table, two workgroups per CU instead
    // of none); the class-coded residues are cached per class map.
    {
        uint32_t qset = 0;
        for (size_t i = 0; i < m; i++) qset |= 1u << (qv.seq[i] & 31);
        cls_of.resize(D.alpha);
        for (uint32_t c = 0; c < D.alpha; c++) {
            const int64_t* rc = M + ((size_t)D.code_of[c] << 5);
            size_t k = 0;
            for (; k < cls_rep.size(); k++) {
                const int64_t* rk = M + ((size_t)cls_rep[k] << 5);
                bool same = true;
                for (int y = 0; y < 32 && same; y++) same = !((qset >> y) & 1) || rc[y] == rk[y];
                if (same) break;
            }
            if (k == cls_rep.size()) cls_rep.push_back(D.code_of[c]);
            cls_of[c] = (uint8_t)k;
        }
    }
    // (workgroups per CU, strip height) of the pair kernel for a compact
    // alphabet of a codes
    auto pair_wgs = [&](size_t a) {
        const int pn = pair_strip_np(C.pair_np, nw, (uint32_t)a + 1, m);
        const size_t b = (size_t)pair_lds_rows((uint32_t)a) * (pn + 4) * 4;
        const size_t w = std::min<size_t>(pn <= 24 ? 3 : 2, pair_wgs_per_cu(b));
        return std::make_pair(w, pn);
    };
    bool use_cls = C.sw_kernel == 0 && np == 16 && cls_rep.size() < D.alpha &&
                   pair_wgs(cls_rep.size()) > pair_wgs(D.alpha);
    // Rare-code merge (Swiss-Prot's X, B, Z, U, O: ~0.04 % of the residues,
    // in ~12 % of the entries): when the classes leave the pair table too big
    // for the best plan (SW: three workgroups per CU; NW: 80-row strips at
    // two), the fewest rarest classes that reach it share ONE class
    // that scores the element-wise maximum of their rows.  An entry holding
    // one of them then scores an upper bound of its true score (max-plus DP
    // is monotone in the profile); the device filter leaves such entries out
    // of its heap-root bounds and forwards every one whose bound could enter
    // the heap to an exact re-score (the int32 tier over the compact codes),
    // so the result is unchanged.  Only while those entries stay a small
    // share (a quarter of the DB at most) and the tier is exact for them.
    int ub = -1;
    if (allow_merge && C.rare_merge && C.sw_kernel == 0 && np == 16 && !D.code_entries.empty() && m > 0) {
        const size_t A0 = cls_rep.size();
        int64_t xlo = INT64_MAX, xhi = INT64_MIN;        // the exact re-score's profile bounds
        for (size_t i = 0; i < m; i++)
            for (uint32_t c = 0; c < D.alpha; c++) {
                const int64_t x = M[((size_t)D.code_of[c] << 5) + qv.seq[i]];
                xlo = std::min(xlo, x);
                xhi = std::max(xhi, x);
            }
        const int rlx = rescore32_rl(D, m, D.alpha, C.gap_open, C.gap_extend, xlo, xhi);
        if (rlx > 0 && A0 >= 3) {
            std::vector<uint64_t> ce(A0, 0);
            for (uint32_t c = 0; c < D.alpha; c++) ce[cls_of[c]] += D.code_entries[c];
            std::vector<uint32_t> ord(A0);
            std::iota(ord.begin(), ord.end(), 0u);
            std::stable_sort(ord.begin(), ord.end(), [&](uint32_t x, uint32_t y) { return ce[x] < ce[y]; });
            uint64_t fl = ce[ord[0]];
            for (size_t k = 2; k < A0; k++) {
                fl += ce[ord[k - 1]];
                if (fl * 4 > D.meta.size()) break;
                // (workgroups per CU, then strip height: SW 2 -> 3 workgroups
                // per CU, NW 64 -> 80-row strips at two per CU)
                if (!(pair_wgs(A0 - k + 1) > pair_wgs(A0))) continue;
                // classes ord[0..k) become one: the others keep their order,
                // the merged class comes last
                std::vector<uint8_t> merged(A0, 0), idx(A0, 0);
                for (size_t i = 0; i < k; i++) merged[ord[i]] = 1;
                std::vector<uint8_t> rep2;
                for (size_t j = 0; j < A0; j++)
                    if (!merged[j]) {
                        idx[j] = (uint8_t)rep2.size();
                        rep2.push_back(cls_rep[j]);
                    }
                ub = (int)rep2.size();
                for (size_t j = 0; j < A0; j++)
                    if (merged[j]) idx[j] = (uint8_t)ub;
                for (uint32_t c = 0; c < D.alpha; c++) {
                    if (merged[cls_of[c]]) vp.merge_mask |= 1u << c;
                    cls_of[c] = idx[cls_of[c]];
                }
                rep2.push_back(0);               // (the merged class has no representative row)
                cls_rep = std::move(rep2);
                vp.merge_entries = fl;
                vp.merge_rl = rlx;
                vp.xminM = xlo;
                vp.xmaxM = xhi;
                use_cls = true;
                break;
            }
        }
    }
    // kernel codes: the classes, or the compact codes themselves
    uint32_t A = use_cls ? (uint32_t)cls_rep.size() : D.alpha;
    std::vector<int64_t>& crow = vp.crow;
    crow.assign((size_t)std::max<uint32_t>(A, 1) * 32, -1);
    for (uint32_t c = 0; c < A; c++)
        if ((int)c != ub) memcpy(&crow[(size_t)c * 32], M + ((size_t)(use_cls ? cls_rep[c] : D.code_of[c]) << 5), 32 * 8);
    if (ub >= 0) {
        // the upper-bound class: the maximum of its members' rows
        for (int y = 0; y < 32; y++) {
            int64_t mx = INT64_MIN;
            for (uint32_t c = 0; c < D.alpha; c++)
                if ((vp.merge_mask >> c) & 1) mx = std::max(mx, M[((size_t)D.code_of[c] << 5) + y]);
            crow[(size_t)ub * 32 + y] = mx;
        }
    }
    vp.use_cls = use_cls;
    // profile bounds over the kernel codes
    int64_t minM = INT64_MAX, maxM = INT64_MIN;
    for (size_t i = 0; i < m; i++)
        for (uint32_t c = 0; c < A; c++) {
            const int64_t x = crow[(size_t)c * 32 + qv.seq[i]];
            minM = std::min(minM, x);
            maxM = std::max(maxM, x);
        }
    if (A == 0) minM = maxM = 0;
    if (force) {
        minM = force->minM;
        maxM = force->maxM;
    }
    const bool fits16 = minM >= -32768 && maxM <= 32767;
    uint32_t nmax16 = fits16 ? (nw ? nw_int16_limit(ml, Q, R, minM, maxM) : 0xffffffffu) : 0;
    // SW with a positive gap increment (R > 0 or Q + R > 0): E would keep
    // growing through the strip kernels' padding columns past an entry's
    // end and leak into its maximum -- every lane goes to the exact int64
    // kernel (the reference's full_sw recurrence)
    if (!nw && (R > 0 || Q + R > 0)) nmax16 = 0;
    if (C.force_wide) nmax16 = 0;
    // SW on f16 bit patterns needs non-positive gaps and scores within
    // +-1024 so no pattern can leave [0x0400, 0x7C7F] (kernels.hip)
    const uint32_t prow = A + 1;
    // pair kernel main strip height: 2 * pair_np rows (16 -> 32 rows, 24 -> 48)
    const int pnp = pair_strip_np(C.pair_np, nw, prow, m);
    const size_t pair_lds = (size_t)pair_lds_rows(A) * (pnp + 4) * 4;
    // pair kernel (diagonal-relative f16 patterns): only when no more than
    // a handful of entries exceed its length bound (those are re-scored
    // by the int64 kernel); otherwise the strip kernels
    uint32_t nw_base = 0;
    bool use_pair = false;
    uint32_t long_groups = 0;            // leading groups scored by long_kernel
    if (C.sw_kernel == 0 && np == 16 && pair_lds <= kPairLdsMax && nmax16 > 0) {
        uint32_t lim = nw ? nw_f16_limit(ml, Q, R, minM, maxM, &nw_base) : sw_rel_limit(ml, Q, R, minM, maxM);
        lim = std::min(lim, nmax16);
        if (lim > 0) {
            const size_t beyond = (size_t)(D.len_sorted.end() -
                                           std::upper_bound(D.len_sorted.begin(), D.len_sorted.end(), lim));
            // (with a merge the long-entry kernels score the compact codes:
            // their bound covers both profiles)
            const int64_t lminM = vp.merge_mask ? std::min(minM, vp.xminM) : minM;
            const int64_t lmaxM = vp.merge_mask ? std::max(maxM, vp.xmaxM) : maxM;
            const uint32_t lg = long_plan(D, ml, beyond, Q, R, lminM, lmaxM, force ? force->long_scale : 1u, nw,
                                        force ? 0 : 2 * pnp);
            // (an entry beyond the bound would also corrupt its group's
            // other lanes, whose padding columns run to its length: the
            // group must go to long_kernel, or the strip kernels run)
            if (lg != UINT32_MAX) {
                use_pair = true;
                nmax16 = lim;
                long_groups = lg == UINT32_MAX ? 0 : lg;
            }
        }
    }
    // SW on f16 patterns without the pair table (strip_f16m_kernel) needs
    // non-positive gaps and scores within +-1024
    const bool use_f16 = use_pair || (!nw && C.sw_kernel != 1 && Q <= 0 && R <= 0 && minM >= -1024 && maxM <= 1024);
    // strip profile table, dword (s, c, r) = (QP[c][s*2np+r], QP[c][s*2np+np+r]);
    // pair table of a strip of height 2P from row i0,
    //   dword (c1*prow+c0, r) = (QP[c1][i0+r], QP[c0][i0+P+r])
    const uint32_t nstrips = (uint32_t)((m + 2 * np - 1) / (2 * np));
    // NW on the pair kernel is diagonal-relative: every profile value (and
    // the padding value 0) carries -2R
    const int rel = use_pair ? -2 * R : 0;
    const int16_t padv = nw ? (int16_t)rel : (use_f16 ? (int16_t)(-1024 + rel) : -32768);
    // pair kernel plan (one launch): main strips of 2*pnp rows, then a
    // tail strip of the smallest height (multiple of 8 rows) that holds the
    // remainder; NW always ends in a tail strip, which captures its score
    size_t qpt_words = 0;                // device table size (dwords)
    uint32_t main_strips = 0;
    int tail_np = 0;
    size_t tail_off = 0;
    if (use_pair) {
        const uint32_t Hm = 2 * pnp;
        uint32_t full = (uint32_t)(m / Hm);
        const uint32_t rem = (uint32_t)(m % Hm);
        if (rem > 0) {
            tail_np = (int)(rem + 7) / 8 * 4;     // 8-row granularity
            // 4-row granularity after a main strip, for the default heights
            // (q = 513: a 36-row tail instead of 40 for the last 33 rows); a
            // fused batch keeps 8-row tails (its queries share one plan, and
            // finer tails would split batches of nearby lengths)
            if (C.tail_rows4 && !batch && full > 0 && pair_tail_fine(pnp, nw)) tail_np = (int)(rem + 3) / 4 * 2;
        } else if (nw) {
            full--;
            tail_np = pnp;
        }
        main_strips = full;
        tail_off = (size_t)full * prow * prow * pnp;
        qpt_words = tail_off + (size_t)prow * prow * pair_tail_pitch((uint32_t)tail_np);
    }
    vp.A = A;
    vp.prow = prow;
    vp.minM = minM;
    vp.maxM = maxM;
    vp.nmax16 = nmax16;
    vp.nw_base = nw_base;
    vp.long_groups = long_groups;
    vp.pnp = pnp;
    vp.pair_lds = pair_lds;
    vp.use_pair = use_pair;
    vp.use_f16 = use_f16;
    vp.nstrips = nstrips;
    vp.rel = rel;
    vp.padv = padv;
    vp.main_strips = main_strips;
    vp.tail_np = tail_np;
    vp.tail_off = tail_off;
    vp.qpt_words = qpt_words;
}

// plan_view's result for the last few (query, kind) pairs of a packed DB: a
// search repeats its predecessor's plan when the query and every setting it
// reads are unchanged (Config::plan_gen; the DB's own state is the
// DeviceDB's, whose release() drops the cache) -- ~7 us of host time per
// search on the path between two searches (profiles/r06/htrace)
struct PlanCache {
    struct Entry {
        std::vector<uint8_t> seq;
        uint64_t gen = 0, used = 0;
        int np = 0;
        bool nw = false, merge = false, batch = false;
        ViewPlan vp;
    };
    std::vector<Entry> e;
    uint64_t clock = 0;
};

static void cached_plan(DeviceDB& D, const QueryView& qv, bool nw, int np, ViewPlan& vp, bool allow_merge) {
    if (!cfg().plan_cache) return plan_view(D, qv, nw, np, nullptr, vp, allow_merge);   // (option "plan_cache" 0)
    if (!D.plans) D.plans = std::make_shared<PlanCache>();
    PlanCache& P = *D.plans;
    const uint64_t gen = cfg().plan_gen;
    for (auto& x : P.e)
        if (x.gen == gen && x.np == np && x.nw == nw && x.merge == allow_merge && !x.batch && x.seq.size() == qv.len &&
            (qv.len == 0 || !memcmp(x.seq.data(), qv.seq, qv.len))) {
            x.used = ++P.clock;
            vp = x.vp;
            return;
        }
    plan_view(D, qv, nw, np, nullptr, vp, allow_merge);
    constexpr size_t kPlans = 4;
    PlanCache::Entry* slot = nullptr;
    if (P.e.size() < kPlans) {
        slot = &P.e.emplace_back();
    } else {
        slot = &P.e[0];
        for (auto& x : P.e)
            if (x.used < slot->used) slot = &x;
    }
    slot->seq.assign(qv.seq, qv.seq + qv.len);
    slot->gen = gen;
    slot->np = np;
    slot->nw = nw;
    slot->merge = allow_merge;
    slot->batch = false;
    slot->used = ++P.clock;
    slot->vp = vp;
}

// per entry the compact codes it holds and per code the entries holding it
// (the rare-code merge's decision and flags), once per packed DB
static void ensure_entry_masks(DeviceDB& D) {
    if (!D.code_entries.empty()) return;
    const size_t E = D.meta.size();
    check(hipMalloc((void**)&D.d_emask, std::max<size_t>(E, 1) * 4), "entry code masks");
    EntryMaskArgs a{};
    a.res = D.d_res;
    a.groups = D.d_groups;
    a.lane_out = D.d_lane_out;
    a.ngroups = D.ngroups;
    a.pad = D.alpha;
    a.out = D.d_emask;
    check(launch_entry_mask(a, D.stream), "entry mask launch");
    std::vector<uint32_t> h(E);
    check(hipMemcpyAsync(h.data(), D.d_emask, E * 4, hipMemcpyDeviceToHost, D.stream), "D2H entry masks");
    check(hipStreamSynchronize(D.stream), "entry masks");
    D.code_entries.assign(std::max<uint32_t>(D.alpha, 1), 0);
    for (uint32_t x : h)
        for (; x; x &= x - 1) D.code_entries[__builtin_ctz(x)]++;
}

// ---------------------------------------------------------- search graph
// A search's stream operations, recorded (launch.h), are replayed as one
// HIP graph: the cached graph when the operations have the same shape as
// the ones it was captured from (kinds, streams, kernels, grids, events,
// argument sizes), with every changed argument block or copy set on its node
// (hipGraphExecKernelNodeSetParams: the tables kernel's gate target, the pair
// kernel's strip-part epoch, the candidate copy's length change per search);
// otherwise the operations are captured into a new graph.  One graph launch
// instead of ~12 calls: less host issue time and fewer barrier packets
// between the kernels (tools/graph_probe.hip).
static bool same_shape(const StreamOp& a, const StreamOp& b) {
    if (a.kind != b.kind || a.stream != b.stream) return false;
    switch (a.kind) {
    case StreamOp::kKernel:
        return a.func == b.func && a.grid.x == b.grid.x && a.grid.y == b.grid.y && a.grid.z == b.grid.z &&
               a.block.x == b.block.x && a.block.y == b.block.y && a.block.z == b.block.z && a.lds == b.lds &&
               a.args.size() == b.args.size() && a.arg_off == b.arg_off;
    case StreamOp::kCopy:
        return a.ck == b.ck;
    case StreamOp::kSet:
        return a.dst == b.dst && a.value == b.value && a.bytes == b.bytes;
    case StreamOp::kRecord:
        return a.event == b.event && a.timing == b.timing;
    case StreamOp::kWait:
        return a.event == b.event;
    }
    return false;
}

static void issue_all(const std::vector<StreamOp>& ops) {
    for (const StreamOp& op : ops) check(issue_op(op, false), "stream operation");
}

// A sync point inside the recording window: what was recorded is issued as
// it stands and the rest of the search runs call by call.
static void sync_point(hipStream_t s, const char* what) {
    if (OpRecorder* r = op_recorder()) {
        if (trace_on()) fprintf(stderr, "trace: search graph: sync point (%s) after %zu ops\n", what, r->ops.size());
        op_recorder() = nullptr;
        issue_all(r->ops);
        r->ops.clear();
    }
    check(hipStreamSynchronize(s), what);
}

static bool capture_ops(DeviceDB::SearchGraph& G, const std::vector<StreamOp>& ops, hipStream_t st) {
    G.reset();
    auto fail = [&](const char* what, size_t i, hipError_t e) {
        if (trace_on())
            fprintf(stderr, "trace: search graph: %s failed at op %zu of %zu (kind %d): %s\n", what, i, ops.size(),
                    i < ops.size() ? (int)ops[i].kind : -1, hipGetErrorString(e));
        return false;
    };
    hipError_t e = hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal);
    if (e != hipSuccess) return fail("begin capture", 0, e);
    std::vector<hipGraphNode_t> nodes(ops.size(), nullptr);
    bool ok = true;
    for (size_t i = 0; i < ops.size() && ok; i++) {
        const StreamOp& op = ops[i];
        e = issue_op(op, true);
        ok = e == hipSuccess || fail("capture", i, e);
        if (ok && (op.kind == StreamOp::kKernel || op.kind == StreamOp::kCopy || op.kind == StreamOp::kSet)) {
            hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
            const hipGraphNode_t* deps = nullptr;
            size_t nd = 0;
            e = hipStreamGetCaptureInfo_v2(op.stream, &cs, nullptr, nullptr, &deps, &nd);
            ok = (e == hipSuccess && cs == hipStreamCaptureStatusActive && nd == 1 && deps) ||
                 fail(e != hipSuccess ? "capture info" : cs != hipStreamCaptureStatusActive ? "capture status"
                                                                                             : "node count", i, e);
            if (ok) nodes[i] = deps[0];
        }
    }
    hipGraph_t g = nullptr;
    e = hipStreamEndCapture(st, &g);
    if (ok && (e != hipSuccess || !g)) ok = fail("end capture", ops.size(), e);
    if (ok) {
        e = hipGraphInstantiate(&G.exec, g, nullptr, nullptr, 0);
        if (e != hipSuccess) ok = fail("instantiate", ops.size(), e);
    }
    if (!ok) {
        if (g) (void)hipGraphDestroy(g);
        G.exec = nullptr;
        (void)hipGetLastError();
        return false;
    }
    G.g = g;
    G.ops = ops;
    G.nodes = std::move(nodes);
    return true;
}

// One segment of a search's operations (no timing record inside) as a
// cached graph.  Returns 0: issued call by call, 1: captured, 2: replayed.
static uint32_t run_segment(DeviceDB& D, const std::vector<StreamOp>& ops, hipStream_t st) {
    auto shape_of = [&](const DeviceDB::SearchGraph& x) {
        bool same = x.exec && x.ops.size() == ops.size();
        for (size_t i = 0; same && i < ops.size(); i++) same = same_shape(x.ops[i], ops[i]);
        return same;
    };
    DeviceDB::SearchGraph* pg = nullptr;
    for (auto& x : D.graph.slot)
        if (shape_of(x)) pg = &x;
    bool same = pg != nullptr;
    if (!pg) {
        // a free slot, else the least recently used
        for (auto& x : D.graph.slot)
            if (!x.exec) {
                pg = &x;
                break;
            }
        if (!pg) {
            pg = &D.graph.slot[0];
            for (auto& x : D.graph.slot)
                if (x.used < pg->used) pg = &x;
        }
    }
    DeviceDB::SearchGraph& G = *pg;
    const double t0 = now_ms();
    uint32_t nset = 0;
    if (same) {
        for (size_t i = 0; same && i < ops.size(); i++) {
            const StreamOp &a = ops[i], &b = G.ops[i];
            if (a.kind == StreamOp::kKernel && a.args != b.args) {
                void* p[32];
                for (size_t j = 0; j < a.arg_off.size() && j < 32; j++) p[j] = (void*)(a.args.data() + a.arg_off[j]);
                hipKernelNodeParams kp{};
                kp.blockDim = a.block;
                kp.gridDim = a.grid;
                kp.func = const_cast<void*>(a.func);
                kp.kernelParams = p;
                kp.sharedMemBytes = a.lds;
                same = hipGraphExecKernelNodeSetParams(G.exec, G.nodes[i], &kp) == hipSuccess;
                nset++;
            } else if (a.kind == StreamOp::kCopy && (a.dst != b.dst || a.src != b.src || a.bytes != b.bytes)) {
                same = hipGraphExecMemcpyNodeSetParams1D(G.exec, G.nodes[i], a.dst, a.src, a.bytes, a.ck) == hipSuccess;
            }
        }
        if (same) G.ops = ops;
        else (void)hipGetLastError();
    }
    if (!same && !capture_ops(G, ops, st)) {
        // (this device searches call by call from now on)
        D.graph.reset();
        D.graph.broken = true;
        if (trace_on()) fprintf(stderr, "trace: search graph capture failed; direct launches\n");
        issue_all(ops);
        return 0;
    }
    G.used = ++D.graph.clock;
    const double t1 = now_ms();
    check(hipGraphLaunch(G.exec, st), "graph launch");
    if (trace_on())
        fprintf(stderr, "trace: search graph: segment of %zu ops, %s, %u kernel arguments set, %.1f us, launch %.1f us\n",
                ops.size(), same ? "replayed" : "captured", nset, (t1 - t0) * 1e3, (now_ms() - t1) * 1e3);
    return same ? 2u : 1u;
}

// A recorded search: its timing records (kernel_ms: after the upload, after
// the DP kernels' join) are issued on the stream as they are -- their
// timestamps then mark exactly what they mark in a direct search -- and the
// operations between them run as cached graphs (a lone operation directly).
// Returns 0: issued call by call, 1: some segment captured, 2: all replayed.
static uint32_t run_ops(DeviceDB& D, OpRecorder& rec, hipStream_t st) {
    const std::vector<StreamOp>& ops = rec.ops;
    if (ops.empty()) return 0;
    uint32_t mode = 2;
    bool any = false;
    size_t i = 0;
    while (i < ops.size()) {
        if (ops[i].kind == StreamOp::kRecord && ops[i].timing) {
            check(issue_op(ops[i], false), "event");
            i++;
            continue;
        }
        size_t j = i;
        while (j < ops.size() && !(ops[j].kind == StreamOp::kRecord && ops[j].timing)) j++;
        if (j - i == 1 || D.graph.broken) {
            for (size_t x = i; x < j; x++) check(issue_op(ops[x], false), "stream operation");
        } else {
            const std::vector<StreamOp> seg(ops.begin() + i, ops.begin() + j);
            mode = std::min(mode, run_segment(D, seg, st));
            any = true;
        }
        i = j;
    }
    return any ? mode : 0u;
}

bool batch_pipelinable(size_t nqueries, size_t k) {
    return nqueries > 1 && k > 0 && k <= (size_t)kFilterMaxK && !cfg().no_filter;
}

// One search (device_search below).  no_parts: every group as one work unit
// (StripArgs::nparts = 1).  Returns false when a strip part's wait for its
// group's first part ran into its bound (StripArgs::part_wait): the scores
// of that launch are not used and the caller runs the search again without
// parts.
static bool device_search_once(DeviceDB& D, const std::vector<QueryView>& views, int algo, size_t k, int bw,
                               SearchScores& out, std::vector<SearchScores>* indep, bool no_parts) {
    check(hipSetDevice(D.device), "hipSetDevice");
    const Config& C = cfg();
    const size_t E = D.meta.size();
    const size_t V = views.size();
    const int np = (C.strip_np == 8 || C.strip_np == 32) ? C.strip_np : 16;
    const bool nw = algo == kAlgoNW;
    const int Q = C.gap_open, R = C.gap_extend;
    const int64_t* M = matrix().m;

    if (D.h_scores_cap < V * E) {
        if (D.h_scores) (void)hipHostFree(D.h_scores);
        check(hipHostMalloc((void**)&D.h_scores, std::max<size_t>(V * E, 1) * 4, hipHostMallocDefault), "pinned scores");
        D.h_scores_cap = V * E;
    }
    out.s32 = D.h_scores;
    out.entries = E;
    out.views = V;
    out.wide.clear();
    out.cells = 0;
    out.cand.clear();
    out.dev_o8 = out.dev_o16 = 0;
    // the reference's overflow counters (counters.hip): per (view, entry)
    // flags, summed on the device after the last view -- only when someone
    // observes them (m_run prints them at OUTPUT_INFO, manager.c:157-160;
    // option "counters")
    const bool want_counts = bw != BIT_WIDTH_64 && E > 0 && V > 0 && counters_on(cfg());
    bool counted = false;
    if (want_counts && D.flags_cap < V * E) {
        dfree(D.d_flags);
        check(hipMalloc((void**)&D.d_flags, V * E), "overflow flags");
        D.flags_cap = V * E;
    }
    // counters and the long-entry dispatch gate start at 0
    uint32_t* const gate = (uint32_t*)(D.d_cnt + 2 * kMaxBatchPipe);
    // option "filter_onepass": the filter as one launch (kernels.hip
    // filter_onepass), its flags told apart from the last pass's by an epoch
    auto one_pass = [&](FilterArgs& f) {
        if (!C.filter_onepass) return;
        f.pass = gate + 4;
        if (++D.filter_epoch >= 0x20000000u) D.filter_epoch = 1;
        f.epoch = D.filter_epoch;
    };
    uint32_t gate_total = 0, gate_base = 0;   // long workgroups launched in all views / before this view
    // (no per-search memset: the gate word only grows, see DeviceDB::gate_count;
    // the counters are zeroed only when this search computes them)
    if (E > 0) {
        if (D.cnt_dirty) {
            check(op_set(D.d_cnt, 0, 16 * kMaxBatchPipe + 16, D.stream), "memset");
            D.gate_count = 0;
            D.cnt_dirty = false;
        } else if (want_counts) {
            check(op_set(D.d_cnt, 0, 16 * kMaxBatchPipe, D.stream), "memset");
        }
    }
    const uint32_t gate0 = D.gate_count;
    // single query view and a small k: only heap-changing candidates come back
    const double t_prep0 = now_ms();
    double prep = 0, sync_wait = 0;
    float upload = 0;
    bool all_rows = V > 0;
    for (const auto& qv : views) all_rows = all_rows && qv.len > 0;
    // (a batch runs one filter pass per query; one pass over several views
    // covers at most kFilterMaxViews)
    out.sparse = (indep != nullptr || V <= (size_t)kFilterMaxViews) && k > 0 && k <= (size_t)kFilterMaxK && E > 0 &&
                 all_rows && !cfg().no_filter;
    // several views: enqueued back to back (host preparation of view v+1
    // overlaps view v on the GPU), each into its own score and overflow
    // slice, then one filter pass over all (view, entry) scores in the
    // reference's chunk-interleaved insertion order -- no per-view sync,
    // copy or host scan of every score
    // independent queries (a batch): the same back-to-back enqueue, but
    // every query gets its own filter pass, candidate region and result
    const bool ind = indep != nullptr;
    if (ind && !(out.sparse && V > 1 && V <= kMaxBatchPipe)) fatal("device_search: batch not pipelinable");
    const bool multi = out.sparse && V > 1 && !ind;
    const bool piped = multi || ind;
    const bool lean = C.lean_events != 0;   // (option "lean_events": no upload/tier/filter markers)
    // the sparse single-pass filter hands its result straight to the host
    // (FilterArgs::host_out) unless something else still has to be copied
    // back on the stream (the overflow counters)
    bool host_direct = C.filter_host && out.sparse && !ind && !want_counts;
    // the rare-code merge (plan_view) needs the single-pass filter and no
    // counters (they decide from exact scores)
    const bool allow_merge = C.rare_merge && V == 1 && !ind && out.sparse && !want_counts && E > 0;
    // option "graph": the usual search -- one query view, the device filter,
    // no counters, the result copied back -- runs as a cached HIP graph
    const bool use_graph = C.graph && !D.graph.broken && V == 1 && out.sparse && !ind && !want_counts &&
                           !host_direct && !C.timeline && !C.side_tier && !allow_merge;
    OpRecorder rec;
    if (allow_merge && D.alpha > 21) ensure_entry_masks(D);
    // every lane fits a view's overflow list (reference: no limit on the
    // sequences search_16.c:101-109 re-runs at 64 bits)
    const size_t ovf_capv = std::max<size_t>((size_t)D.ngroups * 64, 1);
    if (D.ovf_slices < (piped ? V : 1)) {
        dfree(D.d_ovf);
        dfree(D.d_wide);
        D.ovf_slices = piped ? V : 1;
        check(hipMalloc((void**)&D.d_ovf, D.ovf_slices * (ovf_capv + 1) * 4), "overflow list");
        check(hipMalloc((void**)&D.d_wide, D.ovf_slices * ovf_capv * 8), "wide scores");
    }
    // pipelined: per-query candidate regions (device and pinned host)
    const size_t dreg = ind ? ((size_t)kFilterHeader * 4 + E * 8 + 255) & ~(size_t)255 : 0;
    const size_t hreg = (size_t)kFilterHeader * 4 + D.h_cand_cap * 8;
    if (piped) {
        if (D.scores_cap < V * E) {
            dfree(D.d_scores);
            check(hipMalloc((void**)&D.d_scores, V * E * 4), "scores");
            D.scores_cap = V * E;
        }
        while (D.vev.size() < 2 * V + 1) {
            hipEvent_t e;
            check(hipEventCreateWithFlags(&e, kEventFlags), "hipEventCreate");
            D.vev.push_back(e);
        }
    }
    if (ind) {
        if (D.fbuf_bytes < V * dreg) {
            dfree(D.d_fbuf);
            check(hipMalloc((void**)&D.d_fbuf, V * dreg), "filter candidates");
            D.fbuf_bytes = V * dreg;
        }
        if (D.h_fbuf_regions < V) {
            if (D.h_fbuf) (void)hipHostFree(D.h_fbuf);
            check(hipHostMalloc((void**)&D.h_fbuf, V * hreg, hipHostMallocDefault), "pinned candidates");
            D.h_fbuf_regions = V;
        }
        indep->assign(V, SearchScores{});
    }
    if (multi) {
        if (D.filter_cap < V * E) {
            const size_t nb = (V * E + kFilterBlock - 1) / kFilterBlock;
            dfree(D.d_fbuf); dfree(D.d_summary); dfree(D.d_before); dfree(D.d_thresh_local); dfree(D.d_thresh);
            check(hipMalloc((void**)&D.d_fbuf, kFilterHeader * 4 + V * E * 8), "filter candidates");
            D.fbuf_bytes = kFilterHeader * 4 + V * E * 8;
            check(hipMalloc((void**)&D.d_summary, nb * kFilterMaxK * 8), "filter summaries");
            check(hipMalloc((void**)&D.d_before, nb * kFilterMaxK * 4), "filter scan");
            check(hipMalloc((void**)&D.d_thresh_local, nb * 64 * 4), "filter local thresholds");
            check(hipMalloc((void**)&D.d_thresh, nb * 4), "filter thresholds");
            D.filter_cap = V * E;
            D.filter_blocks_cap = nb;
        }
        // insertion order (replay() in api.cpp): ID chunks of chunk_size,
        // views outer inside a chunk, entries in ID order
        const uint64_t cs = C.chunk_size;
        const uint64_t key = (uint64_t)V << 48 ^ cs << 20 ^ E;
        if (D.order_key != key) {
            D.h_order.resize(V * E);
            size_t p = 0, e0 = 0;
            while (e0 < E) {
                const uint64_t chunk_end = (D.meta.id[e0] / cs + 1) * cs;
                size_t e1 = e0;
                while (e1 < E && D.meta.id[e1] < chunk_end) e1++;
                for (size_t v = 0; v < V; v++)
                    for (size_t e = e0; e < e1; e++) D.h_order[p++] = (uint32_t)(v * E + e);
                e0 = e1;
            }
            dfree(D.d_order);
            check(hipMalloc((void**)&D.d_order, V * E * 4), "insertion order");
            check(hipMemcpy(D.d_order, D.h_order.data(), V * E * 4, hipMemcpyHostToDevice), "H2D order");
            D.order_key = key;
        }
    }
    // a batch of single-view queries whose pair-kernel plans agree (strip
    // heights and counts; no residue classes) runs as ONE pair_kernel launch
    // over all of them (StripArgs::nq): the launch's ramp and drain are paid
    // once per batch instead of once per query, and a short query's strips
    // share the chip with the others'.  The profile bounds (and so the f16
    // length limit, NW base and long-entry routing) are the batch's union;
    // each query keeps its own tables, scores, overflow list, filter pass.
    bool fused = false;
    std::vector<ViewPlan> fplans;
    size_t fstride = 0;                  // per-query upload block / staging stride
    StripArgs fb{};                      // view 0's pair-kernel arguments
    size_t qm_off0 = 0;                  // the row counts' offset in view 0's upload block
    std::vector<std::function<void()>> deferred;
    if (ind && V > 1 && V <= (size_t)kMaxFuse && C.batch_fuse && !C.timeline && E > 0) {
        fplans.resize(V);
        fused = true;
        int64_t lo = INT64_MAX, hi = INT64_MIN;
        size_t mmax = 0;
        for (size_t v = 0; v < V && fused; v++) {
            plan_view(D, views[v], nw, np, nullptr, fplans[v], false, true);
            const ViewPlan &p = fplans[v], &p0 = fplans[0];
            fused = p.use_pair && !p.use_cls && p.pnp == p0.pnp && p.main_strips == p0.main_strips &&
                    p.tail_np == p0.tail_np;
            lo = std::min(lo, p.minM);
            hi = std::max(hi, p.maxM);
            mmax = std::max(mmax, views[v].len);
        }
        if (fused) {
            const PlanForce f{lo, hi, mmax, (uint32_t)V};
            for (size_t v = 0; v < V && fused; v++) {
                plan_view(D, views[v], nw, np, &f, fplans[v], false, true);
                const ViewPlan &p = fplans[v], &p0 = fplans[0];
                fused = p.use_pair && !p.use_cls && p.pnp == p0.pnp && p.main_strips == p0.main_strips &&
                        p.tail_np == p0.tail_np && p.long_groups == p0.long_groups && p.nmax16 == p0.nmax16 &&
                        p.nw_base == p0.nw_base && p.qpt_words == p0.qpt_words;
            }
            // NW counters read the long entries' exact extremes from one
            // buffer per search: not shared between deferred views
            if (fused && want_counts && nw && fplans[0].long_groups > 0) fused = false;
        }
        if (fused) {
            const size_t ncols_max = ((size_t)(D.len_sorted.empty() ? 0 : D.len_sorted.back()) + 1 + 3) & ~(size_t)3;
            const size_t top_bytes = (std::max<size_t>(ncols_max, 4) * 4 + 15) & ~(size_t)15;
            fstride = (kUpHeader + top_bytes + mmax + 16 + 4 * V + 255) & ~(size_t)255;
            const size_t qw = fplans[0].qpt_words;
            const uint32_t T0 = fplans[0].main_strips + (fplans[0].tail_np > 0 ? 1u : 0u);
            const bool rows_cross = T0 > 1;
            // one row buffer per query, two with strip parts (rowbuf2 after all first ones)
            const size_t rb = rows_cross ? V * (size_t)D.nblocks * 4096 * (strip_parts(T0) > 1 ? 2 : 1) : 0;
            if (rb > D.rowbuf_q_cap) {
                // one row buffer per query: only within a third of the free memory
                size_t fr = 0, tot = 0;
                check(hipMemGetInfo(&fr, &tot), "hipMemGetInfo");
                if (rb > fr / 3) fused = false;
            }
            if (fused) {
                check(hipStreamSynchronize(D.stream), "sync");
                if (D.upblk_cap < V * fstride) {
                    dfree(D.d_upblk);
                    D.upblk_cap = V * fstride;
                    check(hipMalloc((void**)&D.d_upblk, D.upblk_cap), "per-search uploads");
                }
                if (D.h_up_cap < V * fstride) {
                    if (D.h_up) (void)hipHostFree(D.h_up);
                    check(hipHostMalloc((void**)&D.h_up, V * fstride, hipHostMallocDefault), "pinned uploads");
                    D.h_up_cap = V * fstride;
                }
                if (D.qpt_cap < V * qw) {
                    dfree(D.d_qpt);
                    check(hipMalloc((void**)&D.d_qpt, V * qw * 4), "qpt");
                    D.qpt_cap = V * qw;
                }
                if (rb > D.rowbuf_q_cap) {
                    dfree(D.d_rowbuf_q);
                    check(hipMalloc((void**)&D.d_rowbuf_q, rb), "per-query row buffers");
                    D.rowbuf_q_cap = rb;
                }
                // one filter pass over every query (FilterArgs::nq): a scratch
                // slice per query
                const size_t nb = V * ((E + kFilterBlock - 1) / kFilterBlock);
                if (D.filter_blocks_cap < nb) {
                    dfree(D.d_summary); dfree(D.d_before); dfree(D.d_thresh_local); dfree(D.d_thresh);
                    check(hipMalloc((void**)&D.d_summary, nb * kFilterMaxK * 8), "filter summaries");
                    check(hipMalloc((void**)&D.d_before, nb * kFilterMaxK * 4), "filter scan");
                    check(hipMalloc((void**)&D.d_thresh_local, nb * 64 * 4), "filter local thresholds");
                    check(hipMalloc((void**)&D.d_thresh, nb * 4), "filter thresholds");
                    D.filter_blocks_cap = nb;
                    D.filter_cap = std::min(D.filter_cap, nb * kFilterBlock);
                }
            }
        }
    }
    float kms = 0, wms = 0, dms = 0;
    uint64_t wide_total = 0;
    uint32_t tier_max = 0;           // the longest overflow list this search (DeviceDB::tier_hint)
    uint64_t kernel_bytes = 0;
    const char* kname = "";
    uint32_t srows = 0;
    char lkname[24] = "";                // long-entry kernel(s) of view 0 (stats)
    uint32_t lentries = 0;
    bool parts_used = false;                 // some view ran strip parts (their wait-timeout word is read back)

    for (size_t v = 0; v < V; v++) {
        const QueryView& qv = views[v];
        const size_t m = qv.len;
        out.cells += (uint64_t)m * D.meta.residues;
        int32_t* hs = D.h_scores + v * E;
        if (E == 0) continue;
        if (m == 0) {
            // no query rows: SW scores 0, NW the boundary value H(-1, n-1);
            // the reference skips the pair (no overflow)
            for (size_t e = 0; e < E; e++)
                hs[e] = nw ? (int32_t)(Q + (int64_t)D.meta.len[e] * R) : 0;
            if (want_counts) check(op_set(D.d_flags + v * E, 0, E, D.stream), "memset");
            continue;
        }
        // which kernels, bounds and strip plan (plan_view); a fused batch
        // planned every query up front with shared bounds
        ViewPlan vpl;
        if (fused) vpl = fplans[v];
        else cached_plan(D, qv, nw, np, vpl, allow_merge);
        if (v == 0) host_mark("planned");
        const ViewPlan& vp = vpl;
        const bool merge = vp.merge_mask != 0;
        if (merge) {
            host_direct = false;           // (the exact re-score follows the filter)
            // lanes, then int64 scores, for every entry that holds a merged code
            const size_t cap = std::max<uint64_t>(vp.merge_entries, 1);
            if (D.exact_cap < cap) {
                dfree(D.d_exact);
                check(hipMalloc((void**)&D.d_exact, cap * 12 + 16), "exact re-score list");
                D.exact_cap = cap;
            }
            if (!D.h_exact) check(hipHostMalloc((void**)&D.h_exact, kExactPinned * 12, hipHostMallocDefault), "pinned");
        }
        const bool use_cls = vp.use_cls;
        const std::vector<uint8_t>& cls_of = vp.cls_of;
        const uint4* dres = D.d_res;
        if (use_cls) {
            if (D.cls_key != cls_of) {
                // earlier views of a pipelined search may still read the buffer
                if (piped && v > 0) check(hipStreamSynchronize(D.stream), "sync");
                if (!D.d_res_cls) check(hipMalloc((void**)&D.d_res_cls, D.nblocks * 1024), "class-coded residues");
                RecodeArgs ra{};
                ra.in = D.d_res;
                ra.out = D.d_res_cls;
                ra.n16 = D.nblocks * 64;
                for (int c = 0; c < 64; c++) ra.map[c] = (uint8_t)vp.A;   // padding / unused codes
                for (uint32_t c = 0; c < D.alpha; c++) ra.map[c] = cls_of[c];
                check(launch_recode(ra, D.stream), "recode launch");
                D.cls_key = cls_of;
            }
            dres = D.d_res_cls;
        }
        const uint32_t A = vp.A;
        const int64_t minM = vp.minM, maxM = vp.maxM;
        const uint32_t nmax16 = vp.nmax16, nw_base = vp.nw_base, long_groups = vp.long_groups;
        const int pnp = vp.pnp;
        const size_t pair_lds = vp.pair_lds;
        const bool use_pair = vp.use_pair, use_f16 = vp.use_f16;
        const uint32_t nstrips = vp.nstrips;
        const int rel = vp.rel;
        const int16_t padv = vp.padv;
        // profile values P[c][i] (16-bit, clamped), padding rows/codes = padv;
        // rows up to the last strip's end so table builders need no bounds test
        const size_t mpad = std::max<size_t>((size_t)nstrips * 2 * np, m + 2 * pnp) + 64;
        // (the pair kernel's tables are built on the device: pair_tables_kernel)
        std::vector<uint16_t> P(use_pair ? 0 : (size_t)(A + 1) * mpad, (uint16_t)padv);
        for (uint32_t c = 0; c < (use_pair ? 0u : A); c++) {
            const int64_t* row = vp.crow.data() + (size_t)c * 32;
            uint16_t* pc = P.data() + (size_t)c * mpad;
            for (size_t i = 0; i < m; i++)
                pc[i] = (uint16_t)(int16_t)std::max<int64_t>(-32768, std::min<int64_t>(32767, row[qv.seq[i]] + rel));
        }
        auto prow_of = [&](uint32_t c) { return P.data() + (size_t)std::min(c, A) * mpad; };
        auto val = [&](uint32_t c, size_t i) -> int16_t { return (int16_t)prow_of(c)[i]; };
        std::vector<uint32_t> qpt;
        size_t qpt_words = vp.qpt_words;     // device table size (dwords)
        const uint32_t main_strips = vp.main_strips;
        const int tail_np = vp.tail_np;
        const size_t tail_off = vp.tail_off;
        if (!use_pair) {
            qpt.resize((size_t)nstrips * 32 * np);
            qpt_words = qpt.size();
            for (uint32_t s = 0; s < nstrips; s++)
                for (uint32_t c = 0; c < 32; c++)
                    for (int r = 0; r < np; r++) {
                        const size_t i = (size_t)s * 2 * np + r;
                        qpt[((size_t)s * 32 + c) * np + r] =
                            (uint32_t)(uint16_t)val(c, i) | ((uint32_t)(uint16_t)val(c, i + np) << 16);
                    }
        }
        // the kernel codes' matrix (every kernel reads residues in kernel codes)
        int64_t Mc[1024];
        for (int x = 0; x < 32; x++)
            for (int y = 0; y < 32; y++) Mc[(x << 5) + y] = (uint32_t)x < A ? vp.crow[(size_t)x * 32 + y] : -1;
        const uint32_t wide_threads = (uint32_t)(std::max<size_t>(64, std::min<size_t>(16384, (64ull << 20) / (16 * m))) / 64 * 64);
        // a multi-view search's earlier views may still be queued on the
        // stream: drain it before a device buffer they read is reallocated
        if (piped && v > 0 && ((!fused && D.qpt_cap < qpt_words) || D.work_cap < (size_t)wide_threads * 2 * m))
            check(hipStreamSynchronize(D.stream), "sync");
        if (!fused && D.qpt_cap < qpt_words) {
            dfree(D.d_qpt);
            check(hipMalloc((void**)&D.d_qpt, qpt_words * 4), "qpt");
            D.qpt_cap = qpt_words;
        }
        if (D.work_cap < (size_t)wide_threads * 2 * m) {
            dfree(D.d_work);
            check(hipMalloc((void**)&D.d_work, (size_t)wide_threads * 2 * m * 8), "wide scratch");
            D.work_cap = (size_t)wide_threads * 2 * m;
        }
        hipStream_t st = D.stream;
        // pair kernel: the first strip's top boundary (H(-1,j), F into row
        // 0), diagonal-relative patterns, one dword per column up to the
        // longest group's ncols (kernels.h StripArgs::top)
        std::vector<uint32_t> top;
        const bool top_cached = use_pair && !nw && !fused;
        if (use_pair) {
            const size_t ncols_max = ((size_t)(D.len_sorted.empty() ? 0 : D.len_sorted.back()) + 1 + 3) & ~(size_t)3;
            const uint64_t tkey = (uint64_t)(uint32_t)R << 32 ^ (uint64_t)ncols_max;
            // (cached and current: nothing to build or upload)
            if (!top_cached || D.topc_key != tkey) top.resize(std::max<size_t>(ncols_max, 4));
            if (top.empty()) {
            } else if (nw) {
                auto pat = [&](int v) { return (uint32_t)(v + (int)nw_base) & 0xffffu; };
                std::fill(top.begin(), top.end(), pat(Q + 2 * R) | (pat(2 * Q + 2 * R) << 16));
            } else {
                // 32-bit wrapping, exactly the kernel's combined adds
                const uint32_t rabs = (uint32_t)(-R);
                uint32_t v = (((uint32_t)(kF16Floor - (int)rabs)) & 0xffffu) * 0x10001u;
                for (auto& t : top) {
                    t = v;
                    v += rabs * 0x10001u;
                }
            }
            if (top_cached && !top.empty()) {
                // (every search before this one has drained the stream; the
                // views of one search share the key)
                if (D.topc_cap < top.size()) {
                    check(hipStreamSynchronize(st), "sync");
                    dfree(D.d_topc);
                    check(hipMalloc((void**)&D.d_topc, (top.size() + 4) * 4), "first-strip boundary");
                    D.topc_cap = top.size() + 4;
                }
                check(hipMemcpy(D.d_topc, top.data(), top.size() * 4, hipMemcpyHostToDevice), "H2D boundary");
                D.topc_key = tkey;
                top.clear();
            }
        }
        // device upload block: [matrix 8 KB][top boundary][query codes]
        // (+ a fused batch's row counts, view 0: StripArgs::qm)
        const size_t top_bytes = (top.size() * 4 + 15) & ~(size_t)15;
        const size_t qm_off = (kUpHeader + top_bytes + m + 3) & ~(size_t)3;
        const size_t blk_bytes = (fused && v == 0) ? qm_off + 4 * V : kUpHeader + top_bytes + m;
        const size_t up_bytes = blk_bytes + 16 + qpt.size() * 4;
        // the staging buffer is reused: in a multi-view search the previous
        // view's copies may still be queued behind its predecessor's kernel
        // (waited for before the buffer is refilled or reallocated); growing
        // the device block drains the stream (its kernels read the old one)
        // (a fused batch: every query its own regions, allocated up front --
        // all of them are read by the one pair launch after the last view)
        uint8_t* dup = D.d_upblk;
        uint8_t* hup = D.h_up;
        uint32_t* dqpt = D.d_qpt;
        if (fused) {
            dup = D.d_upblk + v * fstride;
            hup = D.h_up + v * fstride;
            dqpt = D.d_qpt + v * qpt_words;
        } else {
            if (piped && v > 0) {
                if (D.upblk_cap < blk_bytes) check(hipStreamSynchronize(st), "sync");
                else check(hipEventSynchronize(D.ev[5]), "staging");
            }
            if (D.upblk_cap < blk_bytes) {
                dfree(D.d_upblk);
                D.upblk_cap = blk_bytes + 4096;
                check(hipMalloc((void**)&D.d_upblk, D.upblk_cap), "per-search uploads");
            }
            // one pinned staging buffer for the per-search uploads (pageable
            // sources would make each copy a synchronous staged transfer)
            if (D.h_up_cap < up_bytes) {
                if (D.h_up) (void)hipHostFree(D.h_up);
                check(hipHostMalloc((void**)&D.h_up, up_bytes, hipHostMallocDefault), "pinned uploads");
                D.h_up_cap = up_bytes;
            }
            dup = D.d_upblk;
            hup = D.h_up;
            dqpt = D.d_qpt;
        }
        D.d_matrix = (int64_t*)dup;
        D.d_top = top_cached ? D.d_topc : (uint32_t*)(dup + kUpHeader);
        D.d_query = dup + kUpHeader + top_bytes;
        // staging mirrors the device block, then the strip kernels' table
        uint8_t* up_m = hup;
        uint8_t* up_t = up_m + kUpHeader;
        uint8_t* up_s = up_t + top_bytes;
        uint8_t* up_q = hup + ((blk_bytes + 15) & ~(size_t)15);
        memcpy(up_m, Mc, 1024 * 8);
        for (int y = 0; y < 32; y++) memcpy(up_m + 8192 + 8 * y, &M[y], 8);   // code 0's row, M[0][y]
        if (merge) {
            // the compact codes' matrix: the exact re-score of merged-code entries
            int64_t* mx = (int64_t*)(up_m + kUpExactMat);
            for (int x = 0; x < 32; x++)
                for (int y = 0; y < 32; y++)
                    mx[(x << 5) + y] = (uint32_t)x < D.alpha ? M[((size_t)D.code_of[x] << 5) + y] : -1;
        }
        if (!top.empty()) memcpy(up_t, top.data(), top.size() * 4);
        memcpy(up_s, qv.seq, m);
        if (fused && v == 0)
            for (size_t i = 0; i < V; i++) {
                const uint32_t mi = (uint32_t)views[i].len;
                memcpy(up_m + qm_off + 4 * i, &mi, 4);
            }
        if (!qpt.empty()) memcpy(up_q, qpt.data(), qpt.size() * 4);
        // a graph-eligible search records its stream operations from here to
        // the result's copy and replays them as one HIP graph (run_ops)
        if (use_graph) {
            rec.ops.clear();
            op_recorder() = &rec;
        }
        if (!lean) check(op_record(D.ev[4], st, true), "event");
        if (!qpt.empty())
            check(op_copy(dqpt, up_q, qpt.size() * 4, hipMemcpyHostToDevice, st), "H2D qpt");
        if (C.upload_kernel)
            check(launch_upload(dup, up_m, (blk_bytes + 3) & ~(size_t)3, st), "upload kernel");
        else
            check(op_copy(dup, up_m, blk_bytes, hipMemcpyHostToDevice, st), "H2D uploads");
        if (piped) check(op_record(D.ev[5], st), "event");   // staging buffer free again
        // overflow list of this view: the whole list, or in a multi-view
        // search its own slice (all views stay on the device until the end)
        uint32_t* ovf = D.d_ovf + (piped ? v * (ovf_capv + 1) : 0);
        int64_t* wide = D.d_wide + (piped ? v * ovf_capv : 0);
        StripArgs a{};
        a.res = dres;
        a.rowbuf = D.d_rowbuf;
        a.groups = D.d_groups;
        a.lane_len = D.d_lane_len;
        a.lane_out = D.d_lane_out;
        a.qpt = dqpt;
        a.scores = D.d_scores + (piped ? v * E : 0);
        a.ovf_list = ovf + 1;
        a.ovf_count = ovf;
        a.ngroups = D.ngroups;
        a.nstrips = nstrips;
        a.m = (uint32_t)m;
        a.gap_open = Q;
        a.gap_extend = R;
        a.nmax16 = nmax16;
        a.ovf_cap = (uint32_t)ovf_capv;
        a.pad_word = (uint32_t)(uint16_t)padv * 0x10001u;
        a.alpha = A;
        a.nw_base = nw_base;

        WideArgs w{};
        w.res = dres;
        w.groups = D.d_groups;
        w.lane_len = D.d_lane_len;
        w.ovf_list = ovf + 1;
        w.ovf_count = ovf;
        w.query = D.d_query;
        w.matrix = D.d_matrix;
        w.work = D.d_work;
        w.wide_scores = wide;
        w.m = (uint32_t)m;
        w.gap_open = Q;
        w.gap_extend = R;
        w.nw = nw ? 1 : 0;
        w.ovf_cap = (uint32_t)ovf_capv;
        // the counters of the filter pass that follows this wide kernel
        if (ind) w.zero = (uint32_t*)((uint8_t*)D.d_fbuf + v * dreg);
        else if (out.sparse && v + 1 == V) w.zero = D.d_fbuf;
        w.nzero = w.zero ? kFilterHeader : 0;
        if (want_counts) {
            // the overflow-flag replay lists start empty (flags pass below)
            w.zero2[0] = D.d_flist;
            w.zero2[1] = D.d_frlist;
        }

        // the int32 re-score tier for this view's overflowed lanes, when exact
        const int rl32 = rescore32_rl(D, m, A, Q, R, minM, maxM);
        // the int32 tier beside the filter (on stream_long1, after the DP
        // kernels) instead of in front of it: the filter does not read its
        // output, so the tier leaves the path from the pair kernel's end to
        // the result; the tables kernel then clears the filter header
        const bool side_tier = C.side_tier && rl32 > 0 && use_pair && out.sparse && !piped && !want_counts;
        // (the host then waits for the stream's end, which covers the tier:
        // a filter result handed straight to pinned memory would let the
        // host read d_wide, and the tier's end event, before the tier ran)
        if (side_tier) host_direct = false;
        // ... or after it, only when the search has overflowed lanes: the
        // filter forwards every overflowed lane (INT32_MIN) and leaves it out
        // of its bounds, so the tier's exact scores are needed only by the
        // host, which sees the list's length in the candidate header -- the
        // usual search (no overflow) then skips the tier's launch (~5 us on
        // the path from the pair kernel to the result, profiles/r05/host_gap)
        const bool defer_tier = C.tier_defer && !side_tier && rl32 > 0 && use_pair && out.sparse && !piped &&
                                !want_counts && !merge;
        LongArgs ra{};
        if (rl32 > 0) {
            ra.res = dres;
            ra.groups = D.d_groups;
            ra.lane_len = D.d_lane_len;
            ra.lane_out = D.d_lane_out;
            ra.query = D.d_query;
            ra.matrix = D.d_matrix;
            ra.m = (uint32_t)m;
            ra.alpha = A;
            ra.gap_open = Q;
            ra.gap_extend = R;
            ra.list = ovf + 1;
            ra.list_count = ovf;
            ra.list_out = wide;
            ra.nseq = (uint32_t)ovf_capv;
            // grid: one workgroup per four entries of the last search's list
            // (the list is usually empty: a full 1024-workgroup grid that only
            // reads the count costs ~4 us), at least one per CU
            ra.blocks = (uint32_t)std::min<size_t>(
                std::min<size_t>(kRescoreBlocks, (ovf_capv + kLongWaves - 1) / kLongWaves),
                std::max<size_t>(kTierMinBlocks, ((size_t)D.tier_hint + kLongWaves - 1) / kLongWaves));
            if (m > (size_t)64 * rl32) {
                ra.stride = D.group_ncols[0] + 16;
                const size_t need = (size_t)ra.blocks * kLongWaves * ra.stride;
                if (D.rscratch_cap < need) {
                    if (piped && v > 0) sync_point(D.stream, "sync");
                    dfree(D.d_rscratch);
                    check(hipMalloc((void**)&D.d_rscratch, need * 8), "re-score scratch");
                    D.rscratch_cap = need;
                }
                ra.scratch = D.d_rscratch;
            }
        }
        kname = use_pair ? (nw ? "pair_f16_nw" : "pair_f16_sw")
                         : use_f16 ? "strip_f16m_sw" : (nw ? "strip16_nw" : "strip16_sw");
        if (nmax16 == 0) kname = "wide_i64";
        srows = use_pair ? 2 * (uint32_t)pnp : 0;
        if (v == 0) prep = now_ms() - t_prep0;
        if (v == 0) host_mark("upload issued");
        hipEvent_t ev_k0 = piped ? D.vev[2 * v] : D.ev[0], ev_k1 = piped ? D.vev[2 * v + 1] : D.ev[1];
        // option "timeline": one row per long_kernel lane and pair_kernel group
        uint4* tl = nullptr;
        D.timeline_rows = 0;
        if (C.timeline && use_pair) {
            const size_t rows = (size_t)long_groups * 64 + (D.ngroups - long_groups);
            if (D.timeline_cap < rows) {
                dfree(D.d_timeline);
                check(hipMalloc((void**)&D.d_timeline, rows * sizeof(uint4)), "timeline");
                D.timeline_cap = rows;
            }
            check(op_set(D.d_timeline, 0, rows * sizeof(uint4), st), "memset");
            D.timeline_rows = rows;
            tl = D.d_timeline;
        }
        check(op_record(ev_k0, st, true), "event");
        // the long-entry streams fork here: in a recorded search through an
        // event of its own, recorded inside the graph segment that follows
        // (ev_k0 is issued on the stream between two graphs, run_ops)
        hipEvent_t fork_ev = ev_k0;
        if (op_recorder()) {
            fork_ev = D.ev_fork;
            check(op_record(fork_ev, st), "event");
        }
        std::vector<std::function<void()>> long_launch;   // the long-entry kernels' launches
        uint32_t long4 = 0;        // leading groups at 4 waves per entry, the rest of long_groups at 1
        bool long_hmm = false;     // long_kernel wrote the NW extremes (D.d_hmm)
        bool long_only = false;    // the long-entry kernels on the search stream (below)
        size_t lds_long = pair_lds;   // LDS of a long workgroup (the pair tables' gate)
        if (long_groups > 0) {
            // a merge: the long entries are scored exactly on the compact codes
            // (a 35 k-residue entry re-scored by one wave would cost
            // milliseconds), so they never need the exact re-score
            uint32_t extra16 = 0;
            const int rl16 = merge ? long16_plan(D, m, nw, Q, R, std::min(minM, vp.xminM), std::max(maxM, vp.xmaxM), &extra16)
                                   : long16_plan(D, m, nw, Q, R, minM, maxM, &extra16);
            // the longest groups on their own streams, concurrently with the
            // pair kernel (enqueued first, so their waves start first): one
            // wave per entry (RL rows per lane, 64*RL rows per pass), or --
            // for the groups so long that one wave's latency would outlast
            // the pair kernel -- one workgroup per entry, its rows over 4
            // waves (RL 2 up to 512 rows, else 4, passes of 1024 rows)
            if (rl16 > 0) {
                long4 = 0;                 // (one wave per entry)
            } else if (C.long_waves == 4) {
                long4 = long_groups;
            } else if (C.long_waves == 0) {
                // (the 4-wave kernel cuts an entry's latency ~3x at more total
                // issue: worth it only where one wave would outlast the pair
                // kernel -- an entry's one-wave time per column and query row
                // against the pair kernel's per column and strip makes that
                // ~15x a SIMD's share for q = 513 (NW's Swiss-Prot form: one
                // wave 12.7 against four 11.4 TCUPS at its 11.7x; a 30 k- or
                // 150 k-entry DB with that tail, 140x / 39x: four waves ahead,
                // profiles/r06/kshapes))
                const double thr4 = (double)D.ncols_sum / D.nsimd * C.long4_share_pct / 100.0;
                while (long4 < long_groups && D.group_ncols[long4] > thr4) long4++;
            }
            LongArgs la{};
            la.res = merge ? D.d_res : dres;
            la.groups = D.d_groups;
            la.lane_len = D.d_lane_len;
            la.lane_out = D.d_lane_out;
            la.query = D.d_query;
            la.matrix = merge ? (const int64_t*)(dup + kUpExactMat) : D.d_matrix;
            la.scores = a.scores;
            la.m = (uint32_t)m;
            la.alpha = merge ? D.alpha : A;
            la.gap_open = Q;
            la.gap_extend = R;
            // NW: the exact extremes of H the overflow counters decide from,
            // needed only when some long entry is too long for the bounds
            // (2Q + (m + n4)R below the flag threshold, or min(m, n4) maxM at
            // I_MAX: the decide kernel's bounds, counters.hip)
            bool need_hmm = false;
            if (want_counts && nw) {
                const int64_t n4max = (int64_t)D.group_ncols[0];
                int64_t hi = maxM;                         // incl. the padding code 0 (as FlagArgs::maxm)
                for (size_t i = 0; i < m; i++) hi = std::max(hi, M[qv.seq[i]]);
                for (int b = 0; b < 2; b++) {
                    const int64_t imin = b ? -32768 : -128, imax = b ? 32767 : 127;
                    if ((bw == BIT_WIDTH_8) || b == 1)
                        need_hmm = need_hmm || 2 * (int64_t)Q + ((int64_t)m + n4max) * R < imin - Q - R - 1 ||
                                   std::min<int64_t>((int64_t)m, n4max) * std::max<int64_t>(hi, 0) >= imax;
                }
            }
            if (need_hmm) {
                if (D.hmm_cap < (size_t)long_groups * 64) {
                    sync_point(D.stream_long, "sync");
                    sync_point(D.stream_long1, "sync");
                    if (piped && v > 0) sync_point(st, "sync");
                    dfree(D.d_hmm);
                    check(hipMalloc((void**)&D.d_hmm, (size_t)long_groups * 64 * sizeof(int2)), "long-entry extremes");
                    D.hmm_cap = (size_t)long_groups * 64;
                }
                la.hmm = D.d_hmm;
                long_hmm = true;
            }
            // rows per lane: the fewest computed rows for this query (a
            // wave of W waves x 64 lanes x RL rows per pass; waves past the
            // query idle): q = 513 computes 576 rows at RL 3, 768 at RL 4
            const int rl4 = long_rl4(m);
            const int rl1 = long_rl1(m);
            if (rl16 > 0 ? m > (size_t)64 * rl16 : (m > (size_t)4 * 64 * rl4 || m > (size_t)64 * rl1)) {
                la.stride = D.group_ncols[0] + 16;
                const size_t need = (size_t)long_groups * 64 * la.stride;
                if (D.lscratch_cap < need) {
                    sync_point(D.stream_long, "sync");
                    sync_point(D.stream_long1, "sync");
                    dfree(D.d_lscratch);
                    check(hipMalloc((void**)&D.d_lscratch, need * 8), "long-entry scratch");
                    D.lscratch_cap = need;
                }
                la.scratch = D.d_lscratch;
            }
            la.gate = gate;
            la.timeline = tl;
            if (use_pair && C.long_pad) la.lds_min = (uint32_t)pair_lds;
            gate_base = gate_total;
            // (issued right after the tables kernel below: the host issues
            // the next GPU step first, and the tables kernel's gate holds the
            // pair kernel until these workgroups have started)
            // (every group on them and of one kind: no pair work to overlap,
            // so they run on the search stream itself, without the gate and
            // the events across streams -- 16 us of a one-entry search's 180)
            long_only = long_groups == D.ngroups && !fused && (long4 == 0 || long4 == long_groups);
            if (long4 > 0) {
                la.seq0 = 0;
                la.nseq = long4 * 64;
                gate_total += la.nseq;                         // one workgroup per entry
                D.gate_count += la.nseq;
                long_launch.push_back([=, &D]() {
                    if (long_only) {
                        check(launch_long(la, 4, rl4, nw, st), "long kernel launch");
                        return;
                    }
                    check(op_wait(D.stream_long, fork_ev), "event wait");
                    check(launch_long(la, 4, rl4, nw, D.stream_long), "long kernel launch");
                    check(op_record(D.ev[7], D.stream_long), "event");
                });
            }
            if (long4 < long_groups) {
                la.seq0 = long4 * 64;
                la.nseq = (long_groups - long4) * 64;
                gate_total += (la.nseq + kLongWaves - 1) / kLongWaves;   // four entries per workgroup
                D.gate_count += (la.nseq + kLongWaves - 1) / kLongWaves;
                if (rl16 > 0) {
                    la.base16 = long16_base(Q, R);
                    la.extra16 = extra16;
                    la.low_prio = C.long_prio ? 0u : 1u;
                    la.pad16 = (uint32_t)(uint16_t)(int16_t)(std::max<int64_t>(maxM, 0) - 32767);
                }
                long_launch.push_back([=, &D]() {
                    const hipStream_t ls = long_only ? st : D.stream_long1;
                    if (!long_only) check(op_wait(ls, fork_ev), "event wait");
                    if (rl16 > 0) check(launch_long16(la, rl16, ls), "long kernel launch");
                    else check(launch_long(la, 1, rl1, nw, ls), "long kernel launch");
                    if (!long_only) check(op_record(D.ev[6], ls), "event");
                });
            }
            if (v == 0) {
                lentries = long_groups * 64;
                if (rl16 > 0 && extra16) snprintf(lkname, sizeof lkname, "long16_rl%d+%u", rl16, extra16);
                else if (rl16 > 0) snprintf(lkname, sizeof lkname, "long16_rl%d", rl16);
                else if (long4 == 0) snprintf(lkname, sizeof lkname, "long32_w1_rl%d", rl1);
                else if (long4 == long_groups) snprintf(lkname, sizeof lkname, "long32_w4_rl%d", rl4);
                else snprintf(lkname, sizeof lkname, "long32_w4_rl%d+w1_rl%d", rl4, rl1);
            }
            lds_long = std::max(C.long_pad ? pair_lds : 0,
                                rl16 > 0 ? long16_lds_bytes(la.alpha, rl16)
                                         : long4 > 0 ? long_lds_bytes(la.alpha, 4, rl4) : long_lds_bytes(la.alpha, 1, rl1));
        }
        // the pair tables, then the long entries' launches: the tables kernel
        // runs while the host issues them, and its gate (block 0) holds the
        // pair kernel until their workgroups have started -- they are the
        // critical path and must be placed before the pair kernel's fill the
        // CUs' LDS
        if (use_pair) {
            TableArgs ta{};
            ta.query = D.d_query;
            ta.matrix = D.d_matrix;
            ta.out = dqpt;
            ta.m = (uint32_t)m;
            ta.alpha = A;
            ta.np = (uint32_t)pnp;
            ta.nmain = main_strips;
            ta.npt = (uint32_t)tail_np;
            ta.tail_row0 = main_strips * 2 * (uint32_t)pnp;
            ta.rel = rel;
            ta.pad = (uint32_t)(uint16_t)padv;
            ta.zero = ovf;
            if (side_tier || defer_tier) {
                ta.zero_hdr = D.d_fbuf;
                ta.nzero_hdr = kFilterHeader;
            }
            // the start-order ticket (StripArgs::ticket): always with strip
            // parts, whose waits rely on it
            {
                const uint32_t T = main_strips + (tail_np > 0 ? 1u : 0u);
                if (C.pair_ticket || (!no_parts && strip_parts(T) > 1)) ta.zero_ticket = gate + 1;
            }
            if (long_groups > 0 && C.long_gate && !long_only) {
                // (at most what can be resident at once: every long workgroup
                // pads its LDS to the pair table's size, so a CU holds
                // floor(160 KiB / that) of them -- beyond it the target is
                // reached only as early ones retire, and the wait would run
                // into its 20 ms bound; and at most 512, the rest follow the
                // first in order)
                const uint32_t resident = (uint32_t)std::max<size_t>(1, pair_wgs_per_cu(lds_long)) *
                                          (D.nsimd / 4);
                uint32_t want = std::min<uint32_t>(gate_total - gate_base, std::min<uint32_t>(512, resident));
                // (option long_gate P > 1: only the first P % of them)
                if (C.long_gate > 1 && C.long_gate < 100) want = std::max<uint32_t>(1, want * (uint32_t)C.long_gate / 100);
                ta.gate = gate;
                ta.gate_target = gate0 + gate_base + want;
                if (trace_on() && v == 0)
                    fprintf(stderr, "trace: long gate: groups %u (4-wave %u), workgroups %u, resident %u, want %u, lds %zu\n",
                            long_groups, long4, gate_total - gate_base, resident, want, lds_long);
            }
            check(launch_pair_tables(ta, st), "pair tables kernel");
        } else {
            check(op_set(ovf, 0, 4, st), "memset");
        }
        for (auto& f : long_launch) f();

        if (use_pair) {
            StripArgs b = a;
            b.nstrips = main_strips;
            b.qpt_tail = dqpt + tail_off;
            b.top = (const uint4*)D.d_top;
            b.g_first = long_groups;
            if (C.pair_ticket) b.ticket = gate + 1;    // zeroed by the tables kernel just before
            b.timeline = tl ? tl + (size_t)long_groups * 64 : nullptr;
            // the first wave on every SIMD holds one of the longest groups; it
            // shares the SIMD with two other waves, so at equal priority it
            // runs at a third of the issue rate and, on a DB that fills the chip
            // only a few times over, outlasts the rest of the launch
            {
                const uint32_t pg = C.pair_prio_groups < 0 ? D.nsimd : (uint32_t)C.pair_prio_groups;
                b.g_prio = (uint32_t)std::min<uint64_t>((uint64_t)long_groups + pg, D.ngroups);
            }
            // a fused batch: view 0's arguments plus per-query strides cover
            // every view, launched once after the last view's tables
            if (fused && v == 0) {
                fb = b;
                qm_off0 = qm_off;
            }
            if (fused && v + 1 == V) {
                b = fb;
                b.nq = (uint32_t)V;
                b.qm = (const uint32_t*)(D.d_upblk + qm_off0);
                b.q_tab_stride = qpt_words;
                b.q_score_stride = E;
                b.q_ovf_stride = ovf_capv + 1;
                if (main_strips + (tail_np > 0 ? 1u : 0u) > 1) {
                    b.rowbuf = (uint4*)D.d_rowbuf_q;
                    b.q_rowbuf_stride = (size_t)D.nblocks * 256;
                }
                b.timeline = nullptr;
            }
            // strip parts: the launch's last work units become a fraction of a
            // group (kernels.h StripArgs::nparts)
            if (!fused || v + 1 == V) {
                const uint32_t T = main_strips + (tail_np > 0 ? 1u : 0u);
                const size_t nqf = fused ? V : 1;
                uint32_t parts = no_parts ? 1u : strip_parts(T);
                if (fused) parts = std::min(parts, 2u);   // (a fused batch's layout holds two row buffers)
                if (parts > 2 && !D.d_rowbuf3 && D.ngroups > long_groups) {
                    // the third part's row buffer (4 B per residue slot); without
                    // the memory for it the search runs two parts
                    if (piped && v > 0) sync_point(st, "sync");
                    if (hipMalloc((void**)&D.d_rowbuf3, (size_t)D.nblocks * 4096) != hipSuccess) {
                        (void)hipGetLastError();
                        D.d_rowbuf3 = nullptr;
                        parts = 2;
                    }
                }
                if (parts > 1 && D.ngroups > long_groups) {
                    const uint32_t quads = (D.ngroups - long_groups + kPairWaves - 1) / kPairWaves;
                    const uint32_t ps = (T + parts - 1) / parts;
                    parts = (T + ps - 1) / ps;
                    if (D.part_cap < quads * nqf || D.smax_cap < (size_t)D.ngroups * 64 * nqf) {
                        if (piped && v > 0) sync_point(st, "sync");
                        if (D.part_cap < quads * nqf) {
                            dfree(D.d_part);
                            check(hipMalloc((void**)&D.d_part, (size_t)quads * nqf * 4), "strip parts");
                            check(op_set(D.d_part, 0, (size_t)quads * nqf * 4, st), "memset");
                            D.part_cap = quads * nqf;
                        }
                        if (D.smax_cap < (size_t)D.ngroups * 64 * nqf) {
                            dfree(D.d_smax);
                            check(hipMalloc((void**)&D.d_smax, (size_t)D.ngroups * 64 * nqf * 4), "strip-part maxima");
                            D.smax_cap = (size_t)D.ngroups * 64 * nqf;
                        }
                    }
                    // this launch's handoff flag value (no per-launch clearing:
                    // older launches left smaller or different values; never 0,
                    // the value of fresh memory)
                    // (a multiple of 4: part q's flag is part_epoch + q)
                    D.part_epoch += 4;
                    if (D.part_epoch < 4) D.part_epoch = 4;
                    b.part_epoch = D.part_epoch;
                    b.nparts = parts;
                    b.part_strips = ps;
                    b.nquads = quads;
                    // option pair_split: only the first P % of the quads (the
                    // longest, P > 0) or the last -P % (P < 0) are split
                    b.split_q0 = 0;
                    b.split_q1 = quads;
                    if (C.pair_split > 0 && C.pair_split < 100)
                        b.split_q1 = std::max<uint32_t>(1, (uint32_t)((uint64_t)quads * C.pair_split / 100));
                    else if (C.pair_split < 0 && C.pair_split > -100)
                        b.split_q0 = quads - std::max<uint32_t>(1, (uint32_t)((uint64_t)quads * -C.pair_split / 100));
                    b.part_done = D.d_part;
                    b.part_smax = D.d_smax;
                    b.part_err = gate + 2;
                    // (ticks of the 100 MHz s_memrealtime clock)
                    b.part_wait = (uint32_t)std::min<uint64_t>(0xffffffffull, (uint64_t)C.part_wait_us * 100);
                    // a part waits only for a unit that holds an earlier
                    // start-order ticket, i.e. one already resident or done
                    b.ticket = gate + 1;
                    if (fused) {
                        b.rowbuf2 = (uint4*)(D.d_rowbuf_q + nqf * (size_t)D.nblocks * 4096);
                    } else {
                        if (!D.d_rowbuf2) {
                            if (piped && v > 0) sync_point(st, "sync");
                            check(hipMalloc((void**)&D.d_rowbuf2, (size_t)D.nblocks * 4096), "second row buffer");
                        }
                        b.rowbuf2 = D.d_rowbuf2;
                        if (parts > 2) b.rowbuf3 = D.d_rowbuf3;
                    }
                    parts_used = true;
                }
            }
            const int lnp = main_strips ? pnp : tail_np;
            if (!fused || v + 1 == V) {
                // the pair-row stream (StripArgs::paddr) for the launch's table
                // row width, rebuilt when the residue copy, code count or row
                // width it was made for changes (a fused batch shares view 0's
                // plan; on this stream any earlier pair launch has finished
                // reading it before it is rewritten)
                const uint32_t rowB = (uint32_t)(lnp + 4) * 4;
                auto same = [&](const DeviceDB::PairRows& r) {
                    return r.valid && r.use_cls == use_cls && r.prow == A + 1 && r.row_bytes == rowB &&
                           (!use_cls || r.cls == cls_of);
                };
                DeviceDB::PairRows* pr = same(D.prs[0]) ? &D.prs[0] : same(D.prs[1]) ? &D.prs[1] : nullptr;
                if (!pr) {
                    // a free slot (the second only if a stream is at most a
                    // quarter of the free memory), else the least recently used
                    const size_t bytes = (size_t)D.nblocks * 2048;
                    pr = &D.prs[0];
                    if (D.prs[0].d) {
                        if (!D.prs[1].d) {
                            size_t fr = 0, tot = 0;
                            check(hipMemGetInfo(&fr, &tot), "hipMemGetInfo");
                            if (bytes <= fr / 4) pr = &D.prs[1];
                        } else if (D.prs[1].used < D.prs[0].used) {
                            pr = &D.prs[1];
                        }
                    }
                    if (!pr->d) check(hipMalloc((void**)&pr->d, bytes), "pair-row stream");
                    PairAddrArgs pa{};
                    pa.res = dres;
                    pa.out = pr->d;
                    pa.groups = D.d_groups;
                    pa.ngroups = D.ngroups;
                    pa.prow = A + 1;
                    pa.row_bytes = rowB;
                    check(launch_pair_addr(pa, st), "pair-row stream launch");
                    pr->valid = true;
                    pr->use_cls = use_cls;
                    pr->prow = A + 1;
                    pr->row_bytes = rowB;
                    pr->cls = use_cls ? cls_of : std::vector<uint8_t>();
                }
                pr->used = ++D.pr_clock;
                b.paddr = pr->d;
            }
            // a fused batch's DP time runs from this one launch (not from view
            // 0's start: the host prepared the other views in between)
            if (fused && v + 1 == V) check(op_record(D.vev[2 * V], st, true), "event");
            if (!fused || v + 1 == V) {
                check(launch_pair(b, pnp, tail_np, nw, (size_t)pair_lds_rows(A) * (lnp + 4) * 4, st), "pair kernel launch");
                host_mark("pair issued");
            }
        } else {
            check(use_f16 ? launch_sw_f16(a, np, st) : launch_strip16(a, np, nw, st), "strip kernel launch");
        }
        // what follows the DP kernels for this view: the exact re-score, the
        // overflow flags, its filter pass (a fused batch defers it until the
        // one pair launch that covers every view)
        auto post = [=, &D, &kernel_bytes, &counted]() {
            if (long4 > 0 && !long_only) check(op_wait(st, D.ev[7]), "event wait");
            if (long4 < long_groups && !long_only) check(op_wait(st, D.ev[6]), "event wait");
            check(op_record(ev_k1, st, true), "event");
            if (side_tier) {
                // (header cleared by the tables kernel; no counters)
                check(op_wait(D.stream_long1, ev_k1), "event wait");
                check(launch_long(ra, 1, rl32, nw, D.stream_long1), "int32 re-score launch");
                check(op_record(D.ev[8], D.stream_long1), "event");
            } else if (defer_tier) {
                // (after the result's copy, if the header reports overflowed lanes)
            } else if (rl32 > 0) {
                // the int32 tier clears what wide_kernel would have (one launch)
                LongArgs rz = ra;
                rz.zero = w.zero;
                rz.nzero = w.nzero;
                rz.zero2[0] = w.zero2[0];
                rz.zero2[1] = w.zero2[1];
                check(launch_long(rz, 1, rl32, nw, st), "int32 re-score launch");
            } else {
                check(launch_wide(w, wide_threads, st), "wide kernel launch");
            }
            if (want_counts) {
                // 8/16-bit overflow flags of this view's lanes (counters.hip);
                // "ordinary" widths are decided from exact values and bounds
                int64_t lo = minM, hi = maxM, pm = INT64_MIN;
                for (size_t i = 0; i < m; i++) {
                    const int64_t x = M[qv.seq[i]];           // padding code 0
                    lo = std::min(lo, x);
                    hi = std::max(hi, x);
                    pm = std::max(pm, x);
                }
                int ordinary = 0;
                for (int b = 0; b < 2; b++) {
                    const int64_t imin = b ? -32768 : -128, imax = b ? 32767 : 127;
                    const bool ok = Q <= 0 && R <= 0 && Q + R >= imin && (!nw || Q + R <= -1) && lo >= imin && hi <= imax;
                    ordinary |= (int)ok << b;
                }
                FlagArgs fa{};
                fa.res = dres;
                fa.groups = D.d_groups;
                fa.lane_len = D.d_lane_len;
                fa.lane_out = D.d_lane_out;
                fa.entry_lane = (const uint2*)D.d_entry_lane;
                fa.entries = (uint32_t)E;
                fa.scores = a.scores;
                // this view's own uploads (D.d_query / D.d_matrix name the
                // last view's when a fused batch runs its posts deferred)
                fa.query = w.query;
                fa.matrix = w.matrix;
                fa.padrow = (const int64_t*)(dup + 8192);
                fa.flags = D.d_flags + v * E;
                fa.list = D.d_flist;
                fa.work = (int32_t*)D.d_work;
                fa.nlanes = D.ngroups * 64;
                fa.m = (uint32_t)m;
                fa.threads = wide_threads;
                fa.gap_open = Q;
                fa.gap_extend = R;
                fa.nw = nw ? 1 : 0;
                fa.widths = bw == BIT_WIDTH_8 ? 3 : 2;
                fa.ordinary = ordinary;
                fa.maxm = (int32_t)std::max<int64_t>(0, std::min<int64_t>(hi, INT32_MAX));
                fa.padmax = (int32_t)std::max<int64_t>(0, std::min<int64_t>(pm, INT32_MAX));
                if (nw && long_groups > 0 && long_hmm) {
                    fa.hmm = D.d_hmm;
                    fa.hmm_lanes = long_groups * 64;
                }
                fa.long_lanes = long_groups * 64;
                fa.bw = bw;
                fa.lists_zeroed = 1;                       // by the wide kernel just before
                // a single view (or a batch query): counted as decided, no flags
                // array and no count pass
                if (ind || V == 1) fa.direct = D.d_cnt + (ind ? 2 * v : 0);
                // pair kernel (nw_f16_limit) and int16 strip kernel (nw_int16_limit):
                // every H of an exactly scored lane stays below 32767
                fa.nw_hmax16_ok = nw && (use_pair || !use_f16) && nmax16 > 0 ? 1 : 0;
                if (nw && D.ngroups > 0) {
                    // row-major NW replay: scratch for the longest entry's
                    // columns, 64..1024 lanes within 64 MiB
                    fa.rstride = D.group_ncols[0];
                    fa.rthreads = (uint32_t)std::max<size_t>(64, std::min<size_t>(1024, (64ull << 20) / (8ull * fa.rstride)) / 64 * 64);
                    const size_t need = (size_t)fa.rthreads * 2 * fa.rstride;
                    if (D.frwork_cap < need) {
                        if (piped && v > 0) sync_point(st, "sync");
                        dfree(D.d_frwork);
                        check(hipMalloc((void**)&D.d_frwork, need * 4), "row-major replay scratch");
                        D.frwork_cap = need;
                    }
                    fa.rlist = D.d_frlist;
                    fa.rwork = D.d_frwork;
                }
                check(launch_flags(fa, st), "overflow flags launch");
                if (!fa.direct && v + 1 == V) {
                    // the search's counters over all views
                    CountArgs ca{};
                    ca.flags = D.d_flags;
                    ca.entries = (uint32_t)E;
                    ca.views = (uint32_t)V;
                    ca.bw = bw;
                    ca.out = D.d_cnt;
                    check(launch_count(ca, st), "overflow count launch");
                }
                if (v + 1 == V) {
                    check(op_copy(D.h_cnt, D.d_cnt, 16 * (ind ? V : 1), hipMemcpyDeviceToHost, st), "D2H counters");
                    counted = true;
                }
            }
            kernel_bytes += D.meta.residues + 4ull * E + qpt_words * 4;
            if (ind && !fused) {
                // this query's own filter pass into its own candidate region
                uint32_t* reg = (uint32_t*)((uint8_t*)D.d_fbuf + v * dreg);
                FilterArgs f{};
                f.scores = D.d_scores + v * E;
                f.order = nullptr;
                f.n = (uint32_t)E;
                f.k = (uint32_t)k;
                f.nblocks = (uint32_t)((E + kFilterBlock - 1) / kFilterBlock);
                f.summary = D.d_summary;
                f.thresh = D.d_thresh;
                f.thresh_local = D.d_thresh_local;
                f.before = D.d_before;
                f.ovf_count = ovf;
                f.ovf_stride = 0;
                f.nviews = 1;
                f.counters = reg;
                f.status = gate + 2;
                f.cand = (uint2*)(reg + kFilterHeader);
                one_pass(f);
                check(launch_filter(f, st), "filter launch");
                check(op_copy((uint8_t*)D.h_fbuf + v * hreg, reg, kFilterHeader * 4 + 8 * std::min(D.h_cand_cap, E),
                                     hipMemcpyDeviceToHost, st), "D2H candidates");
            }
        };
        if (fused && v + 1 < V) {
            deferred.push_back(post);
            continue;
        }
        for (auto& f : deferred) f();
        deferred.clear();
        post();
        if (fused) {
            // every query's filter pass in one (FilterArgs::nq), then each
            // query's candidates back into its pinned region
            FilterArgs f{};
            f.scores = D.d_scores;
            f.n = (uint32_t)E;
            f.k = (uint32_t)k;
            f.nblocks = (uint32_t)((E + kFilterBlock - 1) / kFilterBlock);
            f.summary = D.d_summary;
            f.thresh = D.d_thresh;
            f.thresh_local = D.d_thresh_local;
            f.before = D.d_before;
            f.ovf_count = D.d_ovf;
            f.ovf_stride = 0;
            f.nviews = 1;
            f.counters = (uint32_t*)D.d_fbuf;
            f.status = gate + 2;
            f.cand = (uint2*)(f.counters + kFilterHeader);
            f.nq = (uint32_t)V;
            f.q_scores = E;
            f.q_ovf = ovf_capv + 1;
            f.q_counters = dreg / 4;
            one_pass(f);
            check(launch_filter(f, st), "filter launch");
            for (size_t vv = 0; vv < V; vv++)
                check(op_copy((uint8_t*)D.h_fbuf + vv * hreg, (uint8_t*)D.d_fbuf + vv * dreg,
                                     kFilterHeader * 4 + 8 * std::min(D.h_cand_cap, E), hipMemcpyDeviceToHost, st),
                      "D2H candidates");
        }
        if (piped && v + 1 < V) continue;
        if (!lean) check(op_record(D.ev[2], st, true), "event");
        if (ind) {
            // (filters already enqueued per query)
        } else if (out.sparse) {
            FilterArgs f{};
            f.scores = D.d_scores;
            f.order = multi ? D.d_order : nullptr;
            f.n = (uint32_t)(multi ? V * E : E);
            f.k = (uint32_t)k;
            f.nblocks = (uint32_t)((f.n + kFilterBlock - 1) / kFilterBlock);
            f.summary = D.d_summary;
            f.thresh = D.d_thresh;
            f.thresh_local = D.d_thresh_local;
            f.before = D.d_before;
            f.ovf_count = D.d_ovf;
            f.ovf_stride = (uint32_t)(ovf_capv + 1);
            f.nviews = (uint32_t)(multi ? V : 1);
            f.counters = D.d_fbuf;
            f.status = gate + 2;
            f.cand = (uint2*)(D.d_fbuf + kFilterHeader);
            if (host_direct) {
                // the filter writes header + first candidates into h_fbuf and
                // then the sequence word the host spins on below
                if (++D.filter_seq == 0) D.filter_seq = 1;
                __atomic_store_n(&D.h_fbuf[kFilterSeqWord], 0u, __ATOMIC_RELEASE);
                f.host_out = D.h_fbuf;
                f.host_cap = (uint32_t)std::min<size_t>(D.h_cand_cap, f.n);
                f.host_seq = D.filter_seq;
                f.done = gate + 3;
                f.host_fence = C.filter_host == 1 ? 1u : C.filter_host == 3 ? 2u : 0u;
            }
            const size_t xcap_al = (D.exact_cap + 1) & ~(size_t)1;     // (int64 scores 8-byte aligned)
            if (merge) {
                f.emask = D.d_emask;
                f.merge_mask = vp.merge_mask;
                f.entry_lane = (const uint2*)D.d_entry_lane;
                f.exact_lanes = D.d_exact;
                f.exact_lane0 = long_groups * 64;
            }
            one_pass(f);
            check(launch_filter(f, st), "filter launch");
            // (the stream's end, and so the host's wake-up, covers the tier)
            if (side_tier) check(op_wait(st, D.ev[8]), "event wait");
            if (merge) {
                // the forwarded merged-code entries, exactly: the int32 tier
                // over their lanes (count: the filter header's word 1) on the
                // compact-code residues and matrix
                LongArgs xa{};
                xa.res = D.d_res;
                xa.groups = D.d_groups;
                xa.lane_len = D.d_lane_len;
                xa.lane_out = D.d_lane_out;
                xa.query = D.d_query;
                xa.matrix = (const int64_t*)(dup + kUpExactMat);
                xa.m = (uint32_t)m;
                xa.alpha = D.alpha;
                xa.gap_open = Q;
                xa.gap_extend = R;
                xa.list = D.d_exact;
                xa.list_count = D.d_fbuf + 1;
                xa.list_out = (int64_t*)(D.d_exact + xcap_al);
                xa.nseq = (uint32_t)D.exact_cap;
                xa.blocks = (uint32_t)std::min<size_t>(kRescoreBlocks, (D.exact_cap + kLongWaves - 1) / kLongWaves);
                if (m > (size_t)64 * vp.merge_rl) {
                    xa.stride = D.group_ncols[0] + 16;
                    const size_t need = (size_t)xa.blocks * kLongWaves * xa.stride;
                    if (D.rscratch_cap < need) {
                        sync_point(st, "sync");
                        dfree(D.d_rscratch);
                        check(hipMalloc((void**)&D.d_rscratch, need * 8), "re-score scratch");
                        D.rscratch_cap = need;
                    }
                    xa.scratch = D.d_rscratch;
                }
                check(launch_long(xa, 1, vp.merge_rl, nw, st), "exact re-score launch");
                const size_t nx = std::min(kExactPinned, D.exact_cap);
                check(op_copy(D.h_exact, D.d_exact, nx * 4, hipMemcpyDeviceToHost, st), "D2H exact lanes");
                check(op_copy(D.h_exact + kExactPinned * 4, D.d_exact + xcap_al, nx * 8, hipMemcpyDeviceToHost, st),
                      "D2H exact scores");
            }
            if (!host_direct) {
                // one copy: counters (incl. the overflow counts) + the first
                // candidates -- twice the last search's count, at least 256
                // (a short copy is most of a copy's latency; more candidates
                // than that come in a second copy after the synchronisation)
                const size_t first = std::min<size_t>(std::min<size_t>(D.h_cand_cap, f.n),
                                                      std::max<size_t>(256, 2 * (size_t)D.cand_hint + 64));
                D.cand_first = first;
                check(op_copy(D.h_fbuf, D.d_fbuf, kFilterHeader * 4 + 8 * first, hipMemcpyDeviceToHost, st),
                      "D2H candidates");
            }
        } else {
            check(op_copy(hs, D.d_scores, E * 4, hipMemcpyDeviceToHost, st), "D2H scores");
            // (the first kOvfPinned entries; d_ovf holds ovf_capv + 1 dwords)
            const size_t pre = std::min(kOvfPinned, ovf_capv);
            check(op_copy(D.h_ovf, D.d_ovf, 4 * (pre + 1), hipMemcpyDeviceToHost, st), "D2H overflow");
            check(op_copy(D.h_wide, D.d_wide, 8 * pre, hipMemcpyDeviceToHost, st), "D2H wide");
        }
        // the strip-part wait status: the filter passes copy it into their
        // candidate headers (word 2); only a search without them reads it back
        uint32_t* const h_perr = (uint32_t*)(D.h_cnt + 2 * kMaxBatchPipe) + 2;
        const bool perr_in_header = ind || out.sparse;
        if (parts_used && !perr_in_header)
            check(op_copy(h_perr, gate + 2, 4, hipMemcpyDeviceToHost, st), "D2H part status");
        out.graph = 0;
        if (op_recorder()) {
            op_recorder() = nullptr;
            out.graph = run_ops(D, rec, st);
        }
        if (trace_on()) fprintf(stderr, "trace: search graph: eligible %d, ops %zu, mode %u\n", (int)use_graph, rec.ops.size(), out.graph);
        const double t_sync0 = now_ms();
        host_mark("issued");
        // filter_host 3: the filter's own stores, made visible by the end of
        // its dispatch -- an ordinary synchronisation, no copy, no spin
        const bool spin = host_direct && C.filter_host != 3;
        if (spin) {
            // spin on the filter's sequence word in pinned memory: the result is
            // here as soon as the last filter block has written it, before the
            // kernel's end-of-dispatch cache writeback and completion signal
            // (the stream keeps that tail; the next search queues behind it).
            // A drained stream without the word is a library bug: fatal.
            const volatile uint32_t* seqw = D.h_fbuf + kFilterSeqWord;
            for (uint64_t it = 1; __atomic_load_n(seqw, __ATOMIC_ACQUIRE) != D.filter_seq; it++) {
                if ((it & 1023) == 0) {
                    const hipError_t q = hipStreamQuery(st);
                    if (q == hipSuccess) {
                        if (__atomic_load_n(seqw, __ATOMIC_ACQUIRE) != D.filter_seq)
                            fatal("device filter result did not reach the host");
                        break;
                    }
                    if (q != hipErrorNotReady) check(q, "search");
                }
                __builtin_ia32_pause();
            }
        } else {
            if (!lean) check(hipEventRecord(D.ev[3], st), "event");
            check(hipStreamSynchronize(st), "search");
        }
        sync_wait += now_ms() - t_sync0;
        // a strip part gave up waiting for its group's first part: this
        // launch's scores are incomplete -- the caller runs the search again
        // without parts (never fatal: a slow predecessor is a timing event)
        if (parts_used) {
            uint32_t perr = 0;
            if (ind) {
                for (size_t vv = 0; vv < V; vv++) perr |= ((const uint32_t*)((const uint8_t*)D.h_fbuf + vv * hreg))[2];
            } else {
                perr = out.sparse ? D.h_fbuf[2] : *h_perr;
            }
            if (perr) {
                D.cnt_dirty = true;          // (the wait-timeout word is cleared before the re-run)
                return false;
            }
        }
        const double t_post0 = now_ms();

        if (!lean) {
            float u;
            check(hipEventElapsedTime(&u, D.ev[4], ev_k0), "elapsed");
            upload += u;
        }
        if (trace_on()) fprintf(stderr, "trace: sync-wait %.3f\n", now_ms() - t_sync0);
        host_mark("synced");
        // exact int64 scores of overflowed lanes: view vv's list and scores
        auto take_wide = [&](size_t vv, uint32_t nov, SearchScores& dst, size_t key_view) {
            const uint32_t* ov = D.d_ovf + (piped ? vv * (ovf_capv + 1) : 0);
            const int64_t* wd = D.d_wide + (piped ? vv * ovf_capv : 0);
            const uint32_t* hov = D.h_ovf;
            const int64_t* hwd = D.h_wide;
            std::vector<uint32_t> big_ovf;
            std::vector<int64_t> big_wide;
            if (nov > kOvfPinned) {
                big_ovf.resize((size_t)nov + 1);
                big_wide.resize(nov);
                check(hipMemcpy(big_ovf.data(), ov, 4 * ((size_t)nov + 1), hipMemcpyDeviceToHost), "D2H overflow");
                check(hipMemcpy(big_wide.data(), wd, 8 * (size_t)nov, hipMemcpyDeviceToHost), "D2H wide");
                hov = big_ovf.data();
                hwd = big_wide.data();
            } else if (out.sparse) {
                check(hipMemcpy(D.h_ovf, ov, 4 * ((size_t)nov + 1), hipMemcpyDeviceToHost), "D2H overflow");
                check(hipMemcpy(D.h_wide, wd, 8 * (size_t)nov, hipMemcpyDeviceToHost), "D2H wide");
            }
            dst.wide.reserve(dst.wide.size() + nov);
            for (uint32_t i = 0; i < nov; i++) {
                const uint32_t e = D.lane_out[hov[1 + i]];
                dst.wide[(uint64_t)key_view * E + e] = hwd[i];
            }
            wide_total += nov;
            tier_max = std::max(tier_max, nov);
        };
        if (ind) {
            for (size_t vv = 0; vv < V; vv++) {
                SearchScores& o = (*indep)[vv];
                const uint32_t* hf = (const uint32_t*)((const uint8_t*)D.h_fbuf + vv * hreg);
                const uint32_t nc = hf[0];
                const uint2* cand = (const uint2*)(hf + kFilterHeader);
                std::vector<uint2> more;
                if (nc > D.h_cand_cap) {
                    more.resize(nc);
                    check(hipMemcpy(more.data(), (const uint8_t*)D.d_fbuf + vv * dreg + kFilterHeader * 4, 8 * (size_t)nc,
                                    hipMemcpyDeviceToHost), "D2H candidates");
                    cand = more.data();
                }
                o.s32 = D.h_scores + vv * E;
                o.entries = E;
                o.views = 1;
                o.sparse = true;
                o.cells = (uint64_t)views[vv].len * D.meta.residues;
                o.cand.resize(nc);
                for (uint32_t i = 0; i < nc; i++) {
                    o.cand[i] = cand[i].x;
                    D.h_scores[vv * E + cand[i].x] = (int32_t)cand[i].y;
                }
                std::sort(o.cand.begin(), o.cand.end());
                o.dev_o8 = want_counts ? D.h_cnt[2 * vv] : 0;
                o.dev_o16 = want_counts ? D.h_cnt[2 * vv + 1] : 0;
                if (hf[3]) take_wide(vv, hf[3], o, 0);
                o.kernel = kname;
                o.strip_rows = srows;
                o.long_entries = lentries;
                memcpy(o.long_kernel, lkname, sizeof lkname);
            }
        } else if (out.sparse) {
            const uint32_t nc = D.h_fbuf[0];
            const uint2* cand = (const uint2*)(D.h_fbuf + kFilterHeader);
            std::vector<uint2> more;
            // (the filter wrote its result to pinned memory itself: up to h_cand_cap)
            const size_t have = host_direct ? D.h_cand_cap : D.cand_first;
            D.cand_hint = nc;
            if (nc > have) {
                more.resize(nc);
                check(hipMemcpy(more.data(), D.d_fbuf + kFilterHeader, 8 * (size_t)nc, hipMemcpyDeviceToHost),
                      "D2H candidates");
                cand = more.data();
            }
            // candidates by insertion position; out.cand holds view * E + entry
            // (the scores land first, then the bare positions are sorted)
            out.cand.resize(nc);
            for (uint32_t i = 0; i < nc; i++) {
                out.cand[i] = cand[i].x;
                D.h_scores[multi ? D.h_order[cand[i].x] : cand[i].x] = (int32_t)cand[i].y;
            }
            std::sort(out.cand.begin(), out.cand.end());
            if (multi)
                for (uint32_t i = 0; i < nc; i++) out.cand[i] = D.h_order[out.cand[i]];
            for (size_t vv = 0; vv < (multi ? V : 1); vv++) {
                const uint32_t nov = D.h_fbuf[3 + vv];
                if (nov && defer_tier) {
                    check(launch_long(ra, 1, rl32, nw, st), "int32 re-score launch");
                    check(hipStreamSynchronize(st), "re-score");
                }
                if (nov) take_wide(multi ? vv : v, nov, out, multi ? vv : v);
            }
            if (merge) {
                // exact scores of the forwarded merged-code entries (after the
                // overflow re-score's, which scored them on the merged class)
                const uint32_t nx = D.h_fbuf[1];
                const uint32_t* xl = (const uint32_t*)D.h_exact;
                const int64_t* xs = (const int64_t*)(D.h_exact + kExactPinned * 4);
                std::vector<uint32_t> bl;
                std::vector<int64_t> bs;
                if (nx > kExactPinned) {
                    const size_t xcap_al = (D.exact_cap + 1) & ~(size_t)1;
                    bl.resize(nx);
                    bs.resize(nx);
                    check(hipMemcpy(bl.data(), D.d_exact, 4 * (size_t)nx, hipMemcpyDeviceToHost), "D2H exact lanes");
                    check(hipMemcpy(bs.data(), D.d_exact + xcap_al, 8 * (size_t)nx, hipMemcpyDeviceToHost),
                          "D2H exact scores");
                    xl = bl.data();
                    xs = bs.data();
                }
                for (uint32_t i = 0; i < nx; i++) {
                    const uint32_t e = D.lane_out[xl[i]];
                    out.wide[e] = xs[i];
                    D.h_scores[e] = INT32_MIN;
                }
                out.rare_rescored = nx;
                out.rare_merged = (uint32_t)__builtin_popcount(vp.merge_mask);
            }
        } else {
            take_wide(v, D.h_ovf[0], out, v);
        }
        if (trace_on()) fprintf(stderr, "trace: candidates %.3f (%zu)\n", now_ms() - t_post0, out.cand.size());
        host_mark("candidates");
        float t;
        if (fused) {
            // one launch for all views: from that launch to the join of the DP
            // kernels (view 0's post, the first to run after it; the long-entry
            // kernels started with their views and overlap the host's preparation)
            check(hipEventElapsedTime(&t, D.vev[2 * V], D.vev[1]), "elapsed");
            kms += t;
            for (size_t vv = 0; vv < V; vv++) (*indep)[vv].kernel_ms = t / V;
        } else if (piped) {
            for (size_t vv = 0; vv < V; vv++) {
                check(hipEventElapsedTime(&t, D.vev[2 * vv], D.vev[2 * vv + 1]), "elapsed");
                kms += t;
                if (ind) (*indep)[vv].kernel_ms = t;
            }
        } else {
            check(hipEventElapsedTime(&t, D.ev[0], D.ev[1]), "elapsed");
            kms += t;
        }
        if (!lean || side_tier) {
            check(hipEventElapsedTime(&t, ev_k1, side_tier ? D.ev[8] : D.ev[2]), "elapsed");
            wms += t;
        }
        if (!spin && !lean) {
            // (the spinning path has no copy: the filter's own time is in the
            // kernel trace, d2h_ms stays 0)
            check(hipEventElapsedTime(&t, D.ev[2], D.ev[3]), "elapsed");
            dms += t;
        }
        if (counted && !ind) {
            out.dev_o8 = D.h_cnt[0];
            out.dev_o16 = D.h_cnt[1];
        }
        if (trace_on()) fprintf(stderr, "trace: post-sync %.3f\n", now_ms() - t_post0);
    }
    if (want_counts && !counted) {
        // the last view had no query rows: sum the flags now
        CountArgs ca{};
        ca.flags = D.d_flags;
        ca.entries = (uint32_t)E;
        ca.views = (uint32_t)V;
        ca.bw = bw;
        ca.out = D.d_cnt;
        check(launch_count(ca, D.stream), "overflow count launch");
        check(hipMemcpyAsync(D.h_cnt, D.d_cnt, 16, hipMemcpyDeviceToHost, D.stream), "D2H counters");
        check(hipStreamSynchronize(D.stream), "counters");
        out.dev_o8 = D.h_cnt[0];
        out.dev_o16 = D.h_cnt[1];
    }
    if (trace_on())
        fprintf(stderr, "trace: prep %.3f sync %.3f total %.3f\n", prep, sync_wait, now_ms() - t_prep0);
    out.kernel_ms = kms;
    out.prep_ms = V == 1 ? prep : 0;
    out.upload_ms = upload;
    out.sync_wait_ms = sync_wait;
    out.wide_ms = wms;
    out.d2h_ms = dms;
    out.wide_count = wide_total;
    D.tier_hint = tier_max;
    out.kernel_bytes = kernel_bytes;
    out.kernel = kname;
    out.strip_rows = srows;
    out.long_entries = lentries;
    memcpy(out.long_kernel, lkname, sizeof lkname);
    out.fused_views = fused ? (uint32_t)V : 0u;
    return true;
}

void device_search(DeviceDB& D, const std::vector<QueryView>& views, int algo, size_t k, int bw, SearchScores& out,
                   std::vector<SearchScores>* indep) {
    if (device_search_once(D, views, algo, k, bw, out, indep, false)) {
        out.part_retries = 0;
        return;
    }
    // (every stream of the search has been synchronised; the counters and
    // the wait flag are zeroed again at the start of the search)
    if (!device_search_once(D, views, algo, k, bw, out, indep, true))
        fatal("pair kernel: strip-part wait timed out with strip parts off");
    out.part_retries = 1;
}

}  // namespace ssa
