// graph_probe.hip -- does a HIP graph shorten the per-search launch sequence?
// (DESIGN.md §4, round-5 verdict item 6).  One "search" here is the library's
// fixed sequence with trivial kernels: upload, tables, a fork to a second
// stream (wait, kernel, record), the DP kernel, the join, three filter
// kernels, a 2 KB D2H copy into pinned memory and a spinning synchronize.
// Per iteration wall time (median of 2000) for
//   direct  -- the calls issued one by one, as engine.cpp does;
//   graph   -- the same sequence captured once, hipGraphLaunch per iteration;
//   graph+1 -- as graph, plus one kernel node's arguments updated per
//              iteration (the search's changing gate target).
// build: hipcc --offload-arch=gfx950 -O2 -o gpurun_out/graph_probe tools/graph_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                    \
        }                                                                               \
    } while (0)

__global__ void k_small(unsigned* p, unsigned v) {
    if (blockIdx.x == 0 && threadIdx.x == 0) p[0] += v;
}
// (mode "spin": the long-entry and DP kernels hold one workgroup for a fixed
// time, so the iteration shows whether the long branch overlaps the DP kernel)
__global__ void k_spin(unsigned* p, unsigned ticks) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
    if (threadIdx.x == 0) p[0] += 1;
}
static unsigned g_long_ticks = 0, g_pair_ticks = 0;   // 100 MHz ticks; 0: k_small

struct Ctx {
    hipStream_t s, s2;
    hipEvent_t e0, e1, ek0, ek1;
    unsigned* d;
    void* h;
};

static void issue(Ctx& c, unsigned v) {
    hipLaunchKernelGGL(k_small, dim3(64), dim3(256), 0, c.s, c.d, 1u);        // upload
    CK(hipEventRecord(c.ek0, c.s));                                          // kernel_ms start
    hipLaunchKernelGGL(k_small, dim3(64), dim3(256), 0, c.s, c.d + 1, v);      // tables (gate target)
    CK(hipStreamWaitEvent(c.s2, c.ek0, 0));                                   // long stream fork
    if (g_long_ticks) hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, c.s2, c.d + 2, g_long_ticks);
    else hipLaunchKernelGGL(k_small, dim3(64), dim3(256), 0, c.s2, c.d + 2, 1u);    // long kernel
    CK(hipEventRecord(c.e0, c.s2));
    if (g_pair_ticks) hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, c.s, c.d + 3, g_pair_ticks);
    else hipLaunchKernelGGL(k_small, dim3(1024), dim3(256), 0, c.s, c.d + 3, 1u);   // pair kernel
    CK(hipStreamWaitEvent(c.s, c.e0, 0));                                     // join
    CK(hipEventRecord(c.ek1, c.s));                                          // kernel_ms end
    hipLaunchKernelGGL(k_small, dim3(256), dim3(256), 0, c.s, c.d + 4, 1u);    // filter_block
    hipLaunchKernelGGL(k_small, dim3(1), dim3(1024), 0, c.s, c.d + 5, 1u);     // filter_prefix
    hipLaunchKernelGGL(k_small, dim3(256), dim3(256), 0, c.s, c.d + 6, 1u);    // filter_select
    CK(hipMemcpyAsync(c.h, c.d, 2048, hipMemcpyDeviceToHost, c.s));           // candidates
}

static double med(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main(int argc, char** argv) {
    (void)argv;
    if (argc > 1) {   // spin: long 200 us, DP 300 us
        g_long_ticks = 20000;
        g_pair_ticks = 30000;
    }
    CK(hipSetDeviceFlags(hipDeviceScheduleSpin));
    Ctx c;
    int lo, hi;
    CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    CK(hipStreamCreateWithFlags(&c.s, hipStreamNonBlocking));
    CK(hipStreamCreateWithPriority(&c.s2, hipStreamNonBlocking, hi));
    CK(hipEventCreateWithFlags(&c.e0, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&c.e1, hipEventDisableTiming));
    CK(hipEventCreate(&c.ek0));
    CK(hipEventCreate(&c.ek1));
    CK(hipMalloc((void**)&c.d, 4096));
    CK(hipMemset(c.d, 0, 4096));
    CK(hipHostMalloc(&c.h, 4096, hipHostMallocDefault));
    const int N = argc > 1 ? 300 : 2000;
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };

    // direct
    std::vector<double> td, tsub;
    for (int i = 0; i < N + 50; i++) {
        auto t0 = now();
        issue(c, (unsigned)i);
        auto t1 = now();
        CK(hipStreamSynchronize(c.s));
        auto t2 = now();
        if (i >= 50) {
            td.push_back(us(t0, t2));
            tsub.push_back(us(t0, t1));
        }
    }
    // graph: captured once (the fork/join through the events is captured too)
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(c.s, hipStreamCaptureModeGlobal));
    issue(c, 7u);
    CK(hipStreamEndCapture(c.s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    std::vector<double> tg, tgs;
    for (int i = 0; i < N + 50; i++) {
        auto t0 = now();
        CK(hipGraphLaunch(ge, c.s));
        auto t1 = now();
        CK(hipStreamSynchronize(c.s));
        auto t2 = now();
        if (i >= 50) {
            tg.push_back(us(t0, t2));
            tgs.push_back(us(t0, t1));
        }
    }
    // the kernel_ms markers recorded by the graph's event nodes: readable?
    float graph_kms = -1.0f;
    const hipError_t ee = hipEventElapsedTime(&graph_kms, c.ek0, c.ek1);
    if (ee != hipSuccess) graph_kms = -1.0f;
    (void)hipGetLastError();
    // graph + one node's arguments per iteration (the tables kernel: second kernel node)
    size_t nn = 0;
    CK(hipGraphGetNodes(g, nullptr, &nn));
    std::vector<hipGraphNode_t> nodes(nn);
    CK(hipGraphGetNodes(g, nodes.data(), &nn));
    hipGraphNode_t tables = nullptr;
    int seen = 0;
    for (auto n : nodes) {
        hipGraphNodeType t;
        CK(hipGraphNodeGetType(n, &t));
        if (t == hipGraphNodeTypeKernel && ++seen == 2) tables = n;
    }
    std::vector<double> tu, tus;
    if (tables) {
        hipKernelNodeParams kp;
        CK(hipGraphKernelNodeGetParams(tables, &kp));
        unsigned* dp = c.d + 1;
        for (int i = 0; i < N + 50; i++) {
            unsigned v = (unsigned)i;
            void* args[2] = {&dp, &v};
            kp.kernelParams = args;
            auto t0 = now();
            CK(hipGraphExecKernelNodeSetParams(ge, tables, &kp));
            CK(hipGraphLaunch(ge, c.s));
            auto t1 = now();
            CK(hipStreamSynchronize(c.s));
            auto t2 = now();
            if (i >= 50) {
                tu.push_back(us(t0, t2));
                tus.push_back(us(t0, t1));
            }
        }
    }
    // re-captured every iteration and swapped into the instantiated graph
    // (hipGraphExecUpdate: same topology, new arguments), then launched
    std::vector<double> tr, trs;
    for (int i = 0; i < N + 50; i++) {
        auto t0 = now();
        hipGraph_t g2;
        CK(hipStreamBeginCapture(c.s, hipStreamCaptureModeGlobal));
        issue(c, (unsigned)i);
        CK(hipStreamEndCapture(c.s, &g2));
        hipGraphExecUpdateResult ur;
        hipGraphNode_t en = nullptr;
        CK(hipGraphExecUpdate(ge, g2, &en, &ur));
        CK(hipGraphLaunch(ge, c.s));
        auto t1 = now();
        CK(hipStreamSynchronize(c.s));
        auto t2 = now();
        CK(hipGraphDestroy(g2));
        if (i >= 50) {
            tr.push_back(us(t0, t2));
            trs.push_back(us(t0, t1));
        }
    }
    printf("{\"recapture_us\": %.1f, \"recapture_issue_us\": %.1f, ", med(tr), med(trs));
    printf("\"mode\": \"%s\", \"iterations\": %d, \"direct_us\": %.1f, \"direct_issue_us\": %.1f, \"graph_us\": %.1f, "
           "\"graph_issue_us\": %.1f, \"graph_update_us\": %.1f, \"graph_update_issue_us\": %.1f, \"graph_event_elapsed_us\": %.1f, \"graph_event_status\": \"%s\"}\n",
           argc > 1 ? "spin: long 200 us, DP 300 us" : "trivial kernels", N, med(td), med(tsub), med(tg), med(tgs), tu.empty() ? -1.0 : med(tu), tus.empty() ? -1.0 : med(tus),
           graph_kms * 1000.0, hipGetErrorName(ee));
    return 0;
}
