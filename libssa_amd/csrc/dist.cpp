// dist.cpp -- the multi-process shard gather over RCCL (include/libssa_amd.h
// ssa_amd_dist_* / ssa_amd_gather_logs / ssa_amd_merge_logs).
//
// One process per GPU searches its contiguous ID shard and produces its
// insertion log (ssa_amd_search(..., SSA_AMD_LOG)).  The reference merges its
// worker threads' heaps on one host (manager.c:141-145); here the shards'
// logs meet on rank 0 in ONE collective over xGMI: every rank contributes a
// fixed slot of a count row plus kSlotRows (score, id, ...) rows, gathered by
// ncclAllGather ((512 + 1) x 24 B = 12 KB per rank: latency-bound, one call).
// Only when some log is longer than a slot (hitcount in the hundreds, or a
// shard whose scores rise through its whole ID range) is a second, exact-size
// ncclGather to rank 0 issued -- every rank knows whether it is needed from
// the first round's counts, so the ranks never disagree on the collective
// sequence.  Rank 0 then replays the logs in rank (= ID) order through the
// reference heap: the 64-bit single-thread result, ties included.
//
// The collectives go through a Transport: RCCL in production, and an
// in-process one (ssa_amd_dist_init_fake: W host threads of one process
// exchanging through shared memory) so that the slot addressing, the count
// rows and the exact-size round run at W > 1 in the CPU tests too.
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
    ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*gather)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
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
    r.all_gather = (decltype(r.all_gather))dlsym(h, "ncclAllGather");
    r.gather = (decltype(r.gather))dlsym(h, "ncclGather");
    r.error_string = (decltype(r.error_string))dlsym(h, "ncclGetErrorString");
    if (!r.get_unique_id || !r.comm_init_rank || !r.comm_destroy || !r.comm_count || !r.all_gather || !r.gather ||
        !r.error_string) {
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
// Host buffers in, host buffers out; every rank calls each collective in the
// same order with the same byte count.
struct Transport {
    virtual ~Transport() = default;
    // recv (every rank) gets rank r's `bytes` at recv + r * bytes
    virtual void all_gather(const void* send, size_t bytes, uint8_t* recv) = 0;
    // rank 0's recv gets rank r's `bytes` at recv + r * bytes; recv unused elsewhere
    virtual void gather0(const void* send, size_t bytes, uint8_t* recv) = 0;
    virtual int ranks() = 0;      // ranks the communicator holds (ncclCommCount)
};

// RCCL: the rows are staged through pinned host and device buffers on the
// library's own stream of the rank's GPU.
struct RcclTransport final : Transport {
    ncclComm_t comm = nullptr;
    int rank = 0, world = 0, device = -1;
    hipStream_t stream = nullptr;
    size_t cap = 0;                       // bytes per rank of the buffers below
    uint8_t* d_send = nullptr;
    uint8_t* d_recv = nullptr;            // world x cap
    uint8_t* h_stage = nullptr;           // pinned, world x cap

    void reserve(size_t bytes) {
        if (bytes <= cap) return;
        (void)hipStreamSynchronize(stream);
        (void)hipFree(d_send);
        (void)hipFree(d_recv);
        (void)hipHostFree(h_stage);
        cap = bytes;
        check(hipMalloc((void**)&d_send, cap), "gather send buffer");
        check(hipMalloc((void**)&d_recv, cap * world), "gather receive buffer");
        check(hipHostMalloc((void**)&h_stage, cap * world, hipHostMallocDefault), "pinned gather buffer");
    }
    void stage_in(const void* send, size_t bytes) {
        check(hipSetDevice(device), "hipSetDevice");
        reserve(bytes);
        memcpy(h_stage, send, bytes);
        check(hipMemcpyAsync(d_send, h_stage, bytes, hipMemcpyHostToDevice, stream), "H2D log");
    }
    void all_gather(const void* send, size_t bytes, uint8_t* recv) override {
        stage_in(send, bytes);
        nccl_check(rccl()->all_gather(d_send, d_recv, bytes, ncclUint8, comm, stream), "ncclAllGather");
        check(hipMemcpyAsync(h_stage, d_recv, bytes * world, hipMemcpyDeviceToHost, stream), "D2H logs");
        check(hipStreamSynchronize(stream), "gather");
        memcpy(recv, h_stage, bytes * world);
    }
    void gather0(const void* send, size_t bytes, uint8_t* recv) override {
        stage_in(send, bytes);
        nccl_check(rccl()->gather(d_send, d_recv, bytes, ncclUint8, 0, comm, stream), "ncclGather");
        if (rank == 0)
            check(hipMemcpyAsync(h_stage, d_recv, bytes * world, hipMemcpyDeviceToHost, stream), "D2H logs");
        check(hipStreamSynchronize(stream), "gather");
        if (rank == 0) memcpy(recv, h_stage, bytes * world);
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
    void all_gather(const void* send, size_t bytes, uint8_t* recv) override { exchange(send, bytes, recv, true); }
    void gather0(const void* send, size_t bytes, uint8_t* recv) override { exchange(send, bytes, recv, false); }
    int ranks() override { return g->world; }
    ~FakeTransport() override {
        std::lock_guard<std::mutex> lk(g_fake_mu);
        if (--g->members == 0) g_fake_groups.erase(key);
    }
};

struct DistState {
    std::unique_ptr<Transport> t;
    int rank = 0, world = 0;
    std::vector<uint8_t> slots;           // world slots of round 1
    std::vector<uint8_t> big_send, big_recv;
};

// the process's communicator (one per process, as RCCL's one rank per GPU)
DistState& proc_state() {
    static DistState s;
    return s;
}
// a fake rank bound to the calling thread (ssa_amd_dist_init_fake)
thread_local DistState* t_fake = nullptr;

DistState& cur() { return t_fake ? *t_fake : proc_state(); }

Hit to_hit(const ssa_hit_t& x) { return Hit{x.score, x.db_id, x.query_id, x.db_strand, x.db_frame}; }

void init_state(DistState& S, std::unique_ptr<Transport> t, int rank, int world) {
    S.t = std::move(t);
    S.rank = rank;
    S.world = world;
    S.slots.assign(slot_bytes() * (size_t)world, 0);
}

}  // namespace
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
    t->reserve(slot_bytes());
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
    const size_t W = (size_t)S.world;
    // round 1: every rank's slot -- a count row, then up to kSlotRows rows
    std::vector<uint8_t> mine(slot_bytes(), 0);
    const uint64_t cnt = n;
    memcpy(mine.data(), &cnt, 8);
    if (n) memcpy(mine.data() + kRow, log, std::min(n, kSlotRows) * kRow);
    S.t->all_gather(mine.data(), slot_bytes(), S.slots.data());
    std::vector<size_t> counts(W);
    size_t longest = 0;
    for (size_t r = 0; r < W; r++) {
        uint64_t c;
        memcpy(&c, S.slots.data() + r * slot_bytes(), 8);
        counts[r] = c;
        longest = std::max<size_t>(longest, c);
    }
    if (longest <= kSlotRows) {
        if (S.rank != 0) return 0;
        return ssa_amd_merge_logs((const ssa_hit_t*)(S.slots.data() + kRow), counts.data(), W, slot_bytes() / kRow,
                                  hitcount, out);
    }
    // round 2 (every rank saw the same counts): exact-size gather to rank 0
    S.big_send.assign(longest * kRow, 0);
    if (n) memcpy(S.big_send.data(), log, n * kRow);
    if (S.rank == 0) S.big_recv.resize(longest * kRow * W);
    S.t->gather0(S.big_send.data(), longest * kRow, S.rank == 0 ? S.big_recv.data() : nullptr);
    if (S.rank != 0) return 0;
    return ssa_amd_merge_logs((const ssa_hit_t*)S.big_recv.data(), counts.data(), W, longest, hitcount, out);
}

}  // extern "C"
