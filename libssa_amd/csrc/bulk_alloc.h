// bulk_alloc.h -- allocator of the multi-GB host byte buffers of DB
// ingest (the FASTA provider's residue arena, the engine's staging and
// layout buffers).  Shared by libssa_amd.so and libssa_fasta_db.so.
#pragma once
#include <sys/mman.h>

#include <cstddef>
#include <cstdint>
#include <memory>
#include <new>
#include <vector>

namespace ssa {

// The staging and layout byte buffers (GBs for a 10 M DB):
// resize leaves new bytes uninitialised (their writers fill them, in
// parallel; a zeroing resize is a serial extra pass), and blocks from 32 MiB
// up are anonymous mappings advised onto transparent huge pages (2 MiB pages:
// 512x fewer page faults while they are filled, and a cheap unmap when they
// are freed -- 4 KiB pages made the frees alone ~0.8 s on the 10 M DB).
template <class T>
struct BulkAlloc {
    using value_type = T;
    static constexpr size_t kBig = 32u << 20;
    BulkAlloc() = default;
    template <class U>
    BulkAlloc(const BulkAlloc<U>&) noexcept {}
    T* allocate(size_t n) {
        const size_t bytes = n * sizeof(T);
        if (bytes < kBig) return std::allocator<T>().allocate(n);
        void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (p == MAP_FAILED) throw std::bad_alloc();
        (void)madvise(p, bytes, MADV_HUGEPAGE);
        return (T*)p;
    }
    void deallocate(T* p, size_t n) noexcept {
        const size_t bytes = n * sizeof(T);
        if (bytes < kBig) std::allocator<T>().deallocate(p, n);
        else munmap((void*)p, bytes);
    }
    template <class U>
    void construct(U* p) noexcept {
        ::new ((void*)p) U;
    }
    template <class U, class... A>
    void construct(U* p, A&&... a) {
        ::new ((void*)p) U(std::forward<A>(a)...);
    }
    template <class U>
    bool operator==(const BulkAlloc<U>&) const noexcept { return true; }
    template <class U>
    bool operator!=(const BulkAlloc<U>&) const noexcept { return false; }
};
using Bytes = std::vector<uint8_t, BulkAlloc<uint8_t>>;
using Chars = std::vector<char, BulkAlloc<char>>;

}  // namespace ssa
