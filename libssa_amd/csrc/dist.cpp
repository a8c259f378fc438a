// dist.cpp -- the multi-process shard gather over RCCL (include/libssa_amd.h
// ssa_amd_dist_* / ssa_amd_gather_logs / ssa_amd_merge_logs).
//
// One process per GPU searches its contiguous ID shard and produces its
// insertion log (ssa_amd_search(..., SSA_AMD_LOG)).  The reference merges its
// worker threads' heaps on one host (manager.c:141-145); here the shards'
// logs meet on rank 0 in ONE collective over xGMI: every rank contributes a
// fixed slot of a count row plus kSlotRows (score, id, ...) rows, gathered to
// rank 0 by a single ncclGather ((512 + 1) x 24 B = 12 KB per rank,
// latency-bound).  A log longer than its slot (hitcount in the hundreds, or a
// shard whose scores rise through its whole ID range) sends the rest of its
// rows point to point to rank 0 (ncclSend / ncclRecv): only that rank knows
// its count before the gather and only rank 0 after it, so exactly those two
// take part and every other rank's collective sequence is the one gather.
// Rank 0 then replays the logs in rank (= ID) order through the reference
// heap: the 64-bit single-thread result, ties included.
//
// The collectives go through a Transport: RCCL in production, and an
// in-process one (ssa_amd_dist_init_fake: W host threads of one process
// exchanging through shared memory) so that the slot addressing, the count
// rows and the point-to-point remainder run at W > 1 in the CPU tests too.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <condition_variable>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

#include "engine.h"

namespace ssa {
namespace {

constexpr size_t kSlotRows = 512;
constexpr size_t kRow = sizeof(ssa_hit_t);            // 24 bytes
static_assert(sizeof(ssa_hit_t) == 24, "ssa_hit_t layout");

constexpr size_t slot_bytes() { return (kSlotRows + 1) * kRow; }

// RCCL is resolved at run time, not linked: a Python host that imported
// torch first already holds torch's librccl.so.1 (same soname), and dlopen
// by soname returns that instance, so the library and the process group
// share one RCCL; a plain C caller gets the system's (/opt/rocm/lib).
struct Rccl {
    ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*comm_count)(const ncclComm_t, int*) = nullptr;
    ncclResult_t (*gather)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*group_start)() = nullptr;
    ncclResult_t (*group_end)() = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
};

const Rccl* rccl() {
    static Rccl r;
    static bool tried = false;
    if (tried) return r.comm_init_rank ? &r : nullptr;
    tried = true;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
        print_error("RCCL not found (librccl.so.1): %s", dlerror());
        return nullptr;
    }
    r.get_unique_id = (decltype(r.get_unique_id))dlsym(h, "ncclGetUniqueId");
    r.comm_init_rank = (decltype(r.comm_init_rank))dlsym(h, "ncclCommInitRank");
    r.comm_destroy = (decltype(r.comm_destroy))dlsym(h, "ncclCommDestroy");
    r.comm_count = (decltype(r.comm_count))dlsym(h, "ncclCommCount");
    r.gather = (decltype(r.gather))dlsym(h, "ncclGather");
    r.send = (decltype(r.send))dlsym(h, "ncclSend");
    r.recv = (decltype(r.recv))dlsym(h, "ncclRecv");
    r.group_start = (decltype(r.group_start))dlsym(h, "ncclGroupStart");
    r.group_end = (decltype(r.group_end))dlsym(h, "ncclGroupEnd");
    r.error_string = (decltype(r.error_string))dlsym(h, "ncclGetErrorString");
    if (!r.get_unique_id || !r.comm_init_rank || !r.comm_destroy || !r.comm_count || !r.gather || !r.send || !r.recv ||
        !r.group_start || !r.group_end || !r.error_string) {
        print_error("RCCL lacks a required symbol");
        r = Rccl();
        return nullptr;
    }
    return &r;
}

void nccl_check(ncclResult_t r, const char* what) {
    if (r != ncclSuccess) fatal("RCCL error in %s: %s", what, rccl()->error_string(r));
}

// ---------------------------------------------------------------- transports
// Host buffers in, host buffers out.  gather0 is collective (every rank, same
// byte count); send0 / recv0 are point to point between one rank and rank 0,
// called by exactly the two ranks involved.
struct Transport {
    virtual ~Transport() = default;
    // rank 0's recv gets rank r's `bytes` at recv + r * bytes; recv unused elsewhere
    virtual void gather0(const void* send, size_t bytes, uint8_t* recv) = 0;
    // this rank (not 0) sends `bytes` to rank 0
    virtual void send0(const void* send, size_t bytes) = 0;
    // rank 0 receives from[i].second bytes from rank from[i].first, in list
    // order, concatenated into recv
    virtual void recv0(const std::vector<std::pair<int, size_t>>& from, uint8_t* recv) = 0;
    virtual int ranks() = 0;      // ranks the communicator holds (ncclCommCount)
};

// RCCL: the rows are staged through pinned host and device buffers on the
// library's own stream of the rank's GPU.
struct RcclTransport final : Transport {
    ncclComm_t comm = nullptr;
    int rank = 0, world = 0, device = -1;
    hipStream_t stream = nullptr;
    size_t send_cap = 0, recv_cap = 0, stage_cap = 0;
    uint8_t* d_send = nullptr;
    uint8_t* d_recv = nullptr;
    uint8_t* h_stage = nullptr;           // pinned

    void grow(uint8_t** p, size_t* cap, size_t bytes, bool pinned, const char* what) {
        if (bytes <= *cap) return;
        (void)hipStreamSynchronize(stream);
        if (pinned) (void)hipHostFree(*p);
        else (void)hipFree(*p);
        *p = nullptr;
        *cap = std::max(bytes, 2 * *cap);
        if (pinned) check(hipHostMalloc((void**)p, *cap, hipHostMallocDefault), what);
        else check(hipMalloc((void**)p, *cap), what);
    }
    void reserve(size_t send, size_t recv) {
        grow(&d_send, &send_cap, send, false, "gather send buffer");
        grow(&d_recv, &recv_cap, recv, false, "gather receive buffer");
        grow(&h_stage, &stage_cap, std::max(send, recv), true, "pinned gather buffer");
    }
    void stage_in(const void* send, size_t bytes, size_t recv_bytes) {
        check(hipSetDevice(device), "hipSetDevice");
        reserve(bytes, recv_bytes);
        memcpy(h_stage, send, bytes);
        check(hipMemcpyAsync(d_send, h_stage, bytes, hipMemcpyHostToDevice, stream), "H2D log");
    }
    void stage_out(uint8_t* recv, size_t bytes) {
        check(hipMemcpyAsync(h_stage, d_recv, bytes, hipMemcpyDeviceToHost, stream), "D2H logs");
        check(hipStreamSynchronize(stream), "gather");
        memcpy(recv, h_stage, bytes);
    }
    void gather0(const void* send, size_t bytes, uint8_t* recv) override {
        stage_in(send, bytes, rank == 0 ? bytes * world : 0);
        nccl_check(rccl()->gather(d_send, d_recv, bytes, ncclUint8, 0, comm, stream), "ncclGather");
        if (rank == 0) stage_out(recv, bytes * world);
        else check(hipStreamSynchronize(stream), "gather");
    }
    void send0(const void* send, size_t bytes) override {
        stage_in(send, bytes, 0);
        nccl_check(rccl()->send(d_send, bytes, ncclUint8, 0, comm, stream), "ncclSend");
        check(hipStreamSynchronize(stream), "send");
    }
    void recv0(const std::vector<std::pair<int, size_t>>& from, uint8_t* recv) override {
        size_t total = 0;
        for (const auto& f : from) total += f.second;
        check(hipSetDevice(device), "hipSetDevice");
        reserve(0, total);
        nccl_check(rccl()->group_start(), "ncclGroupStart");
        size_t at = 0;
        for (const auto& f : from) {
            nccl_check(rccl()->recv(d_recv + at, f.second, ncclUint8, f.first, comm, stream), "ncclRecv");
            at += f.second;
        }
        nccl_check(rccl()->group_end(), "ncclGroupEnd");
        stage_out(recv, total);
    }
    int ranks() override {
        int n = 0;
        return rccl()->comm_count(comm, &n) == ncclSuccess ? n : -1;
    }
    ~RcclTransport() override {
        if (!comm) return;                // ncclCommInitRank failed: nothing was set up
        (void)hipSetDevice(device);
        (void)hipStreamSynchronize(stream);
        (void)rccl()->comm_destroy(comm);
        (void)hipFree(d_send);
        (void)hipFree(d_recv);
        (void)hipHostFree(h_stage);
        (void)hipStreamDestroy(stream);
    }
};

// In-process stand-in for the collectives: the W ranks are host threads of
// one process; a collective publishes every rank's send pointer, meets at a
// barrier, copies, and meets again before any sender may reuse its buffer.
struct FakeGroup {
    std::mutex mu;
    std::condition_variable cv;
    int world = 0, members = 0;
    int arrived = 0;
    uint64_t phase = 0;
    std::vector<const void*> send;
    // point to point: rank r's pending message to rank 0 (nullptr: none)
    std::vector<const void*> p2p;
    std::vector<size_t> p2p_bytes;

    void barrier() {
        std::unique_lock<std::mutex> lk(mu);
        const uint64_t ph = phase;
        if (++arrived == world) {
            arrived = 0;
            phase++;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return phase != ph; });
        }
    }
};

std::mutex g_fake_mu;
std::map<int, std::shared_ptr<FakeGroup>> g_fake_groups;

struct FakeTransport final : Transport {
    std::shared_ptr<FakeGroup> g;
    int rank = 0, key = 0;

    void exchange(const void* send, size_t bytes, uint8_t* recv, bool everyone) {
        g->send[rank] = send;
        g->barrier();
        if (everyone || rank == 0)
            for (int r = 0; r < g->world; r++) memcpy(recv + (size_t)r * bytes, g->send[r], bytes);
        g->barrier();
    }
    void gather0(const void* send, size_t bytes, uint8_t* recv) override { exchange(send, bytes, recv, false); }
    void send0(const void* send, size_t bytes) override {
        std::unique_lock<std::mutex> lk(g->mu);
        g->p2p[rank] = send;
        g->p2p_bytes[rank] = bytes;
        g->cv.notify_all();
        g->cv.wait(lk, [&] { return g->p2p[rank] == nullptr; });      // rank 0 has copied it
    }
    void recv0(const std::vector<std::pair<int, size_t>>& from, uint8_t* recv) override {
        std::unique_lock<std::mutex> lk(g->mu);
        for (const auto& f : from) {
            g->cv.wait(lk, [&] { return g->p2p[f.first] != nullptr; });
            if (g->p2p_bytes[f.first] != f.second)
                fatal("fake transport: rank %d sent %zu bytes, rank 0 expected %zu", f.first, g->p2p_bytes[f.first],
                      f.second);
            memcpy(recv, g->p2p[f.first], f.second);
            recv += f.second;
            g->p2p[f.first] = nullptr;
            g->cv.notify_all();
        }
    }
    int ranks() override { return g->world; }
    ~FakeTransport() override {
        std::lock_guard<std::mutex> lk(g_fake_mu);
        if (--g->members == 0) g_fake_groups.erase(key);
    }
};

struct DistState {
    std::unique_ptr<Transport> t;
    int rank = 0, world = 0;
    std::vector<uint8_t> slots;           // rank 0: the world slots of the gather
    std::vector<uint8_t> rest;            // rank 0: the rows beyond the slots, received point to point
};

// the process's communicator (one per process, as RCCL's one rank per GPU)
DistState& proc_state() {
    static DistState s;
    return s;
}
// a fake rank bound to the calling thread (ssa_amd_dist_init_fake)
thread_local DistState* t_fake = nullptr;

DistState& cur() { return t_fake ? *t_fake : proc_state(); }

// the last gather's time and rounds: the process's stats for the RCCL rank;
// per thread for a fake rank (its W threads gather concurrently), laid over
// the process's stats by ssa_amd_get_stats on that thread
thread_local double t_gather_ms = 0;
thread_local uint32_t t_gather_rounds = 0;

void record_gather(double ms, uint32_t rounds) {
    if (t_fake) {
        t_gather_ms = ms;
        t_gather_rounds = rounds;
    } else {
        stats().gather_ms = ms;
        stats().gather_rounds = rounds;
    }
}

Hit to_hit(const ssa_hit_t& x) { return Hit{x.score, x.db_id, x.query_id, x.db_strand, x.db_frame}; }

void init_state(DistState& S, std::unique_ptr<Transport> t, int rank, int world) {
    S.t = std::move(t);
    S.rank = rank;
    S.world = world;
    S.slots.assign(slot_bytes() * (size_t)world, 0);
}

}  // namespace

void dist_overlay_stats(ssa_amd_stats_t* out) {
    if (!t_fake) return;
    out->gather_ms = t_gather_ms;
    out->gather_rounds = t_gather_rounds;
}

}  // namespace ssa

using namespace ssa;

extern "C" {

int ssa_amd_dist_unique_id(void* id) {
    const Rccl* R = rccl();
    if (!id || !R) return 1;
    ncclUniqueId u;
    if (R->get_unique_id(&u) != ncclSuccess) return 1;
    memcpy(id, &u, sizeof u);
    return 0;
}

size_t ssa_amd_dist_unique_id_bytes(void) { return sizeof(ncclUniqueId); }

int ssa_amd_dist_available(void) {
    // everything ssa_amd_dist_init needs before it enters the collective
    // ncclCommInitRank: RCCL resolvable, the rank's device selectable
    if (!rccl()) return 1;
    int dev = cfg().device;
    if (dev < 0 && hipGetDevice(&dev) != hipSuccess) return 1;
    return hipSetDevice(dev) == hipSuccess ? 0 : 1;
}

int ssa_amd_dist_init(int rank, int world, const void* id) {
    DistState& S = proc_state();
    if (S.t) {
        print_error("ssa_amd_dist_init: already initialised (call ssa_amd_dist_finalize first)");
        return 1;
    }
    if (!id || world < 1 || rank < 0 || rank >= world) {
        print_error("ssa_amd_dist_init: bad rank %d / world %d", rank, world);
        return 1;
    }
    if (ssa_amd_dist_available() != 0) return 1;
    int dev = cfg().device;
    if (dev < 0) check(hipGetDevice(&dev), "hipGetDevice");
    auto t = std::make_unique<RcclTransport>();
    ncclUniqueId u;
    memcpy(&u, id, sizeof u);
    if (rccl()->comm_init_rank(&t->comm, world, u, rank) != ncclSuccess) {
        t->comm = nullptr;
        return 1;
    }
    t->rank = rank;
    t->world = world;
    t->device = dev;
    check(hipStreamCreateWithFlags(&t->stream, hipStreamNonBlocking), "hipStreamCreate");
    t->reserve(slot_bytes(), rank == 0 ? slot_bytes() * (size_t)world : 0);
    init_state(S, std::move(t), rank, world);
    return 0;
}

int ssa_amd_dist_init_fake(int rank, int world, int group) {
    if (t_fake) {
        print_error("ssa_amd_dist_init_fake: this thread already holds a rank");
        return 1;
    }
    if (world < 1 || rank < 0 || rank >= world) {
        print_error("ssa_amd_dist_init_fake: bad rank %d / world %d", rank, world);
        return 1;
    }
    auto t = std::make_unique<FakeTransport>();
    {
        std::lock_guard<std::mutex> lk(g_fake_mu);
        auto& g = g_fake_groups[group];
        if (!g) {
            g = std::make_shared<FakeGroup>();
            g->world = world;
            g->send.assign(world, nullptr);
            g->p2p.assign(world, nullptr);
            g->p2p_bytes.assign(world, 0);
        }
        if (g->world != world) {
            print_error("ssa_amd_dist_init_fake: group %d has world %d, not %d", group, g->world, world);
            if (g->members == 0) g_fake_groups.erase(group);
            return 1;
        }
        g->members++;
        t->g = g;
    }
    t->rank = rank;
    t->key = group;
    t_fake = new DistState();
    init_state(*t_fake, std::move(t), rank, world);
    return 0;
}

int ssa_amd_dist_ranks(void) {
    DistState& S = cur();
    return S.t ? S.t->ranks() : 0;
}

void ssa_amd_dist_finalize(void) {
    if (t_fake) {
        delete t_fake;
        t_fake = nullptr;
        return;
    }
    DistState& S = proc_state();
    S = DistState();
}

size_t ssa_amd_merge_logs(const ssa_hit_t* rows, const size_t* counts, size_t nlogs, size_t stride,
                          size_t hitcount, ssa_hit_t* out) {
    TopK heap(hitcount);
    for (size_t r = 0; r < nlogs; r++) {
        const ssa_hit_t* L = rows + r * stride;
        for (size_t i = 0; i < counts[r]; i++) {
            if (heap.full() && L[i].score <= heap.root_score()) continue;
            heap.add(to_hit(L[i]));
        }
    }
    const std::vector<Hit> v = heap.sorted();
    for (size_t i = 0; i < v.size(); i++)
        out[i] = ssa_hit_t{v[i].score, v[i].id, v[i].qid, v[i].strand, v[i].frame, {0, 0, 0, 0, 0}};
    return v.size();
}

int ssa_amd_shard_bounds(const uint64_t* lengths, size_t n, size_t world, size_t align, size_t* bounds) {
    if (world < 1 || !bounds) return 1;
    const size_t a = std::max<size_t>(align, 1), units = (n + a - 1) / a;
    std::vector<uint64_t> cum(units + 1, 0);           // residues before unit u
    for (size_t u = 0; u < units; u++) {
        uint64_t r = 0;
        for (size_t i = u * a; i < std::min(n, (u + 1) * a); i++) r += lengths[i];
        cum[u + 1] = cum[u] + r;
    }
    bounds[0] = 0;
    size_t c0 = 0;
    for (size_t s = 1; s < world; s++) {
        // the unit boundary whose prefix is nearest the ideal s/world share
        const long double target = (long double)cum[units] * s / world;
        size_t c1 = (size_t)(std::lower_bound(cum.begin(), cum.end(), (uint64_t)std::ceil(target)) - cum.begin());
        if (c1 > 0 && c1 <= units && target - cum[c1 - 1] < (long double)cum[std::min(c1, units)] - target) c1--;
        c1 = std::max(c0, std::min(c1, units));
        bounds[s] = std::min(n, c1 * a);
        c0 = c1;
    }
    bounds[world] = n;
    return 0;
}

size_t ssa_amd_gather_logs(const ssa_hit_t* log, size_t n, size_t hitcount, ssa_hit_t* out) {
    DistState& S = cur();
    if (!S.t) fatal("ssa_amd_gather_logs: ssa_amd_dist_init was not called");
    const double t0 = now_ms();
    const size_t W = (size_t)S.world;
    // the one collective: every rank's slot -- a count row, then up to
    // kSlotRows rows -- gathered to rank 0
    std::vector<uint8_t> mine(slot_bytes(), 0);
    const uint64_t cnt = n;
    memcpy(mine.data(), &cnt, 8);
    if (n) memcpy(mine.data() + kRow, log, std::min(n, kSlotRows) * kRow);
    S.t->gather0(mine.data(), slot_bytes(), S.rank == 0 ? S.slots.data() : nullptr);
    uint32_t rounds = 1;
    if (S.rank != 0) {
        // a log longer than the slot: its remaining rows, point to point
        if (n > kSlotRows) {
            S.t->send0(log + kSlotRows, (n - kSlotRows) * kRow);
            rounds = 2;
        }
        record_gather(now_ms() - t0, rounds);
        return 0;
    }
    std::vector<size_t> counts(W);
    std::vector<std::pair<int, size_t>> from;
    for (size_t r = 0; r < W; r++) {
        uint64_t c;
        memcpy(&c, S.slots.data() + r * slot_bytes(), 8);
        counts[r] = c;
        if (r > 0 && c > kSlotRows) from.emplace_back((int)r, (c - kSlotRows) * kRow);
    }
    size_t rest = 0;
    for (const auto& f : from) rest += f.second;
    S.rest.resize(std::max<size_t>(rest, 1));
    if (!from.empty()) {
        S.t->recv0(from, S.rest.data());
        rounds = 2;
    }
    // replay rank by rank, in rank (= ID) order: the slot rows, then the rest
    // (rank 0's own log is local)
    TopK heap(hitcount);
    auto offer = [&](const ssa_hit_t* L, size_t c) {
        for (size_t i = 0; i < c; i++) {
            if (heap.full() && L[i].score <= heap.root_score()) continue;
            heap.add(to_hit(L[i]));
        }
    };
    const uint8_t* rp = S.rest.data();
    for (size_t r = 0; r < W; r++) {
        if (r == 0) {
            offer(log, n);
            continue;
        }
        offer((const ssa_hit_t*)(S.slots.data() + r * slot_bytes() + kRow), std::min(counts[r], kSlotRows));
        if (counts[r] > kSlotRows) {
            offer((const ssa_hit_t*)rp, counts[r] - kSlotRows);
            rp += (counts[r] - kSlotRows) * kRow;
        }
    }
    const std::vector<Hit> v = heap.sorted();
    for (size_t i = 0; i < v.size(); i++)
        out[i] = ssa_hit_t{v[i].score, v[i].id, v[i].qid, v[i].strand, v[i].frame, {0, 0, 0, 0, 0}};
    record_gather(now_ms() - t0, rounds);
    return v.size();
}

}  // extern "C"
