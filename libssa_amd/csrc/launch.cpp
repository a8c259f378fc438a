// launch.cpp -- the recorder behind launch.h's stream operations.
#include "launch.h"

namespace ssa {

OpRecorder*& op_recorder() {
    thread_local OpRecorder* r = nullptr;
    return r;
}

// (inside a stream capture HIP turns an event record into an event record
// node -- its timestamp is taken when the graph runs, tools/graph_probe.hip --
// and a wait on it into the dependency between the streams)
hipError_t issue_op(const StreamOp& op, bool capturing) {
    (void)capturing;
    switch (op.kind) {
    case StreamOp::kKernel: {
        void* p[32];
        const size_t n = op.arg_off.size();
        if (n > 32) return hipErrorInvalidValue;
        for (size_t i = 0; i < n; i++) p[i] = (void*)(op.args.data() + op.arg_off[i]);
        return hipLaunchKernel(op.func, op.grid, op.block, p, op.lds, op.stream);
    }
    case StreamOp::kCopy:
        return hipMemcpyAsync(op.dst, op.src, op.bytes, op.ck, op.stream);
    case StreamOp::kSet:
        return hipMemsetAsync(op.dst, op.value, op.bytes, op.stream);
    case StreamOp::kRecord:
        return hipEventRecord(op.event, op.stream);
    case StreamOp::kWait:
        return hipStreamWaitEvent(op.stream, op.event, 0);
    }
    return hipErrorInvalidValue;
}

static hipError_t put(StreamOp&& op) {
    if (OpRecorder* r = op_recorder()) {
        r->ops.push_back(std::move(op));
        return hipSuccess;
    }
    return issue_op(op, false);
}

hipError_t op_copy(void* dst, const void* src, size_t bytes, hipMemcpyKind kind, hipStream_t st) {
    StreamOp op;
    op.kind = StreamOp::kCopy;
    op.stream = st;
    op.dst = dst;
    op.src = src;
    op.bytes = bytes;
    op.ck = kind;
    return put(std::move(op));
}

hipError_t op_set(void* dst, int value, size_t bytes, hipStream_t st) {
    StreamOp op;
    op.kind = StreamOp::kSet;
    op.stream = st;
    op.dst = dst;
    op.value = value;
    op.bytes = bytes;
    return put(std::move(op));
}

hipError_t op_record(hipEvent_t e, hipStream_t st, bool timing) {
    StreamOp op;
    op.kind = StreamOp::kRecord;
    op.stream = st;
    op.event = e;
    op.timing = timing;
    return put(std::move(op));
}

hipError_t op_wait(hipStream_t st, hipEvent_t e) {
    StreamOp op;
    op.kind = StreamOp::kWait;
    op.stream = st;
    op.event = e;
    return put(std::move(op));
}

}  // namespace ssa
