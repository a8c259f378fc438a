// dist.cpp -- the multi-process shard gather over RCCL (include/libssa_amd.h
// ssa_amd_dist_* / ssa_amd_gather_logs / ssa_amd_merge_logs).
//
// One process per GPU searches its contiguous ID shard and produces its
// insertion log (ssa_amd_search(..., SSA_AMD_LOG)).  The reference merges its
// worker threads' heaps on one host (manager.c:141-145); here the shards'
// logs meet on rank 0 in ONE collective over xGMI: every rank contributes a
// fixed slot of kSlotRows (score, id, ...) rows plus a count row, gathered by
// ncclAllGather (20 KB per rank: latency-bound, one call).  Only when some
// log is longer than a slot (hitcount in the hundreds, or a shard whose
// scores rise through its whole ID range) is a second, exact-size ncclGather
// to rank 0 issued -- every rank knows whether it is needed from the first
// round's counts, so the ranks never disagree on the collective sequence.
// Rank 0 then replays the logs in rank (= ID) order through the reference
// heap: the 64-bit single-thread result, ties included.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "engine.h"

namespace ssa {
namespace {

constexpr size_t kSlotRows = 512;
constexpr size_t kRow = sizeof(ssa_hit_t);            // 24 bytes
static_assert(sizeof(ssa_hit_t) == 24, "ssa_hit_t layout");

struct DistState {
    ncclComm_t comm = nullptr;
    int rank = 0, world = 0, device = -1;
    hipStream_t stream = nullptr;
    uint8_t* d_send = nullptr;   // slot: count row + kSlotRows rows
    uint8_t* d_recv = nullptr;   // world slots
    uint8_t* h_buf = nullptr;    // pinned, world slots
    size_t big_cap = 0;          // rows per rank of the exact-size buffers
    uint8_t* d_big_send = nullptr;
    uint8_t* d_big_recv = nullptr;
};

DistState& ds() {
    static DistState s;
    return s;
}

// RCCL is resolved at run time, not linked: a Python host that imported
// torch first already holds torch's librccl.so.1 (same soname), and dlopen
// by soname returns that instance, so the library and the process group
// share one RCCL; a plain C caller gets the system's (/opt/rocm/lib).
struct Rccl {
    ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
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
    r.all_gather = (decltype(r.all_gather))dlsym(h, "ncclAllGather");
    r.gather = (decltype(r.gather))dlsym(h, "ncclGather");
    r.error_string = (decltype(r.error_string))dlsym(h, "ncclGetErrorString");
    if (!r.get_unique_id || !r.comm_init_rank || !r.comm_destroy || !r.all_gather || !r.gather || !r.error_string) {
        print_error("RCCL lacks a required symbol");
        r = Rccl();
        return nullptr;
    }
    return &r;
}

void nccl_check(ncclResult_t r, const char* what) {
    if (r != ncclSuccess) fatal("RCCL error in %s: %s", what, rccl()->error_string(r));
}

constexpr size_t slot_bytes() { return (kSlotRows + 1) * kRow; }

Hit to_hit(const ssa_hit_t& x) { return Hit{x.score, x.db_id, x.query_id, x.db_strand, x.db_frame}; }

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

int ssa_amd_dist_init(int rank, int world, const void* id) {
    DistState& S = ds();
    const Rccl* R = rccl();
    if (!R) return 1;
    if (S.comm) {
        print_error("ssa_amd_dist_init: already initialised (call ssa_amd_dist_finalize first)");
        return 1;
    }
    if (!id || world < 1 || rank < 0 || rank >= world) {
        print_error("ssa_amd_dist_init: bad rank %d / world %d", rank, world);
        return 1;
    }
    int dev = cfg().device;
    if (dev < 0 && hipGetDevice(&dev) != hipSuccess) return 1;
    if (hipSetDevice(dev) != hipSuccess) return 1;
    ncclUniqueId u;
    memcpy(&u, id, sizeof u);
    if (R->comm_init_rank(&S.comm, world, u, rank) != ncclSuccess) {
        S.comm = nullptr;
        return 1;
    }
    S.rank = rank;
    S.world = world;
    S.device = dev;
    check(hipStreamCreateWithFlags(&S.stream, hipStreamNonBlocking), "hipStreamCreate");
    check(hipMalloc((void**)&S.d_send, slot_bytes()), "gather send slot");
    check(hipMalloc((void**)&S.d_recv, slot_bytes() * world), "gather receive slots");
    check(hipHostMalloc((void**)&S.h_buf, slot_bytes() * world, hipHostMallocDefault), "pinned gather");
    return 0;
}

void ssa_amd_dist_finalize(void) {
    DistState& S = ds();
    if (!S.comm) return;
    (void)hipSetDevice(S.device);
    (void)hipStreamSynchronize(S.stream);
    (void)rccl()->comm_destroy(S.comm);
    (void)hipFree(S.d_send);
    (void)hipFree(S.d_recv);
    (void)hipFree(S.d_big_send);
    (void)hipFree(S.d_big_recv);
    (void)hipHostFree(S.h_buf);
    (void)hipStreamDestroy(S.stream);
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

size_t ssa_amd_gather_logs(const ssa_hit_t* log, size_t n, size_t hitcount, ssa_hit_t* out) {
    DistState& S = ds();
    if (!S.comm) fatal("ssa_amd_gather_logs: ssa_amd_dist_init was not called");
    check(hipSetDevice(S.device), "hipSetDevice");
    const size_t W = (size_t)S.world;
    // round 1: every rank's slot (count row, then up to kSlotRows rows)
    uint8_t* mine = S.h_buf + (size_t)S.rank * slot_bytes();
    memset(mine, 0, kRow);
    const uint64_t cnt = n;
    memcpy(mine, &cnt, 8);
    if (n) memcpy(mine + kRow, log, std::min(n, kSlotRows) * kRow);
    check(hipMemcpyAsync(S.d_send, mine, kRow * (1 + std::min(n, kSlotRows)), hipMemcpyHostToDevice, S.stream),
          "H2D log");
    nccl_check(rccl()->all_gather(S.d_send, S.d_recv, slot_bytes(), ncclUint8, S.comm, S.stream), "ncclAllGather");
    check(hipMemcpyAsync(S.h_buf, S.d_recv, slot_bytes() * W, hipMemcpyDeviceToHost, S.stream), "D2H logs");
    check(hipStreamSynchronize(S.stream), "gather");
    std::vector<size_t> counts(W);
    size_t longest = 0;
    for (size_t r = 0; r < W; r++) {
        uint64_t c;
        memcpy(&c, S.h_buf + r * slot_bytes(), 8);
        counts[r] = c;
        longest = std::max<size_t>(longest, c);
    }
    if (longest <= kSlotRows) {
        if (S.rank != 0) return 0;
        return ssa_amd_merge_logs((const ssa_hit_t*)(S.h_buf + kRow), counts.data(), W, slot_bytes() / kRow,
                                  hitcount, out);
    }
    // round 2 (every rank saw the same counts): exact-size gather to rank 0
    if (S.big_cap < longest) {
        (void)hipFree(S.d_big_send);
        (void)hipFree(S.d_big_recv);
        S.big_cap = longest;
        check(hipMalloc((void**)&S.d_big_send, longest * kRow), "gather send");
        check(hipMalloc((void**)&S.d_big_recv, S.rank == 0 ? longest * kRow * W : kRow), "gather receive");
    }
    if (n) check(hipMemcpyAsync(S.d_big_send, log, n * kRow, hipMemcpyHostToDevice, S.stream), "H2D log");
    nccl_check(rccl()->gather(S.d_big_send, S.d_big_recv, longest * kRow, ncclUint8, 0, S.comm, S.stream),
               "ncclGather");
    std::vector<ssa_hit_t> all(S.rank == 0 ? longest * W : 0);
    if (S.rank == 0)
        check(hipMemcpyAsync(all.data(), S.d_big_recv, longest * kRow * W, hipMemcpyDeviceToHost, S.stream),
              "D2H logs");
    check(hipStreamSynchronize(S.stream), "gather");
    if (S.rank != 0) return 0;
    return ssa_amd_merge_logs(all.data(), counts.data(), W, longest, hitcount, out);
}

}  // extern "C"
