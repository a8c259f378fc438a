// launch.h -- every stream operation of a search goes through these calls, so
// a search's sequence can be recorded instead of issued and replayed as one
// HIP graph (engine.cpp SearchGraph, option "graph").  Without a recorder
// they issue the operation at once, exactly as the plain HIP calls would.
#pragma once
#include <hip/hip_runtime.h>

#include <cstring>
#include <type_traits>
#include <vector>

namespace ssa {

// One enqueued stream operation, with its arguments by value.
struct StreamOp {
    enum Kind : uint8_t { kKernel, kCopy, kSet, kRecord, kWait } kind = kKernel;
    hipStream_t stream = nullptr;
    // kernel
    const void* func = nullptr;
    dim3 grid, block;
    uint32_t lds = 0;
    std::vector<uint8_t> args;        // the arguments' bytes, each at its alignment
    std::vector<uint32_t> arg_off;    // where each argument starts
    // copy / set
    void* dst = nullptr;
    const void* src = nullptr;
    size_t bytes = 0;
    hipMemcpyKind ck = hipMemcpyDefault;
    int value = 0;
    // record / wait; timing: a record whose timestamp is read (kernel_ms)
    hipEvent_t event = nullptr;
    bool timing = false;
};

// The calling thread's recorder (null: operations are issued directly).
struct OpRecorder {
    std::vector<StreamOp> ops;
};
OpRecorder*& op_recorder();
hipError_t issue_op(const StreamOp& op, bool capturing);

template <class... A>
hipError_t ssa_launch(const void* func, dim3 grid, dim3 block, size_t lds, hipStream_t st, const A&... a) {
    if (OpRecorder* r = op_recorder()) {
        StreamOp op;
        op.kind = StreamOp::kKernel;
        op.stream = st;
        op.func = func;
        op.grid = grid;
        op.block = block;
        op.lds = (uint32_t)lds;
        size_t off = 0;
        auto put = [&](const auto& x) {
            constexpr size_t al = alignof(std::remove_reference_t<decltype(x)>);
            off = (off + al - 1) / al * al;
            op.arg_off.push_back((uint32_t)off);
            op.args.resize(off + sizeof x);
            memcpy(op.args.data() + off, &x, sizeof x);
            off += sizeof x;
        };
        (put(a), ...);
        r->ops.push_back(std::move(op));
        return hipSuccess;
    }
    void* p[] = {(void*)&a..., nullptr};
    return hipLaunchKernel(func, grid, block, p, lds, st);
}

hipError_t op_copy(void* dst, const void* src, size_t bytes, hipMemcpyKind kind, hipStream_t st);
hipError_t op_set(void* dst, int value, size_t bytes, hipStream_t st);
hipError_t op_record(hipEvent_t e, hipStream_t st, bool timing = false);
hipError_t op_wait(hipStream_t st, hipEvent_t e);

}  // namespace ssa
