// uncached_reuse_probe.hip -- why uncached exchange buffers diverged after earlier engines had
// used and freed cached memory (profiles/r02_uncached_exchange_bisect.txt).
//
// Hypothesis: plain stores leave dirty lines in the XCDs' L2s; hipFree does not write them back;
// a later uncached allocation (hipDeviceMallocUncached: the L2 is bypassed) that gets the same
// physical pages is written straight to memory -- and when the stale dirty lines are evicted
// later, they are written back OVER the uncached data.
//
// Each trial: allocate a cached buffer, fill it with pattern A by plain stores, free it; (with
// --writeback: launch the every-XCD L2 write-back kernel); allocate an uncached buffer of the same
// size, fill it with pattern B through uncached stores; then stream through a large unrelated
// cached buffer (evicts the L2s); read the uncached buffer back and count words that hold
// pattern A instead of B.  Diagnostic only.
//   build: hipcc --offload-arch=gfx950 -O2 experiments/uncached_reuse_probe.hip -o tools/_ab/uncached_reuse_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            printf("%s at line %d\n", hipGetErrorString(e_), __LINE__);        \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

__global__ void k_fill(unsigned long long *p, size_t n, unsigned long long tag) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = tag ^ i;
}

__global__ void k_fill_sys(unsigned long long *p, size_t n, unsigned long long tag) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        __hip_atomic_store(p + i, tag ^ i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void k_stream(unsigned long long *p, size_t n) {  // read-modify-write: fills the L2s with other lines
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] += 1;
}

__global__ void k_count(const unsigned long long *p, size_t n, unsigned long long tagA, unsigned long long tagB,
                        unsigned long long *out) {
    unsigned long long a = 0, other = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const unsigned long long v =
            __hip_atomic_load(const_cast<unsigned long long *>(p + i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (v == (tagA ^ i)) ++a;
        else if (v != (tagB ^ i)) ++other;
    }
    atomicAdd(out, a);
    atomicAdd(out + 1, other);
}

__global__ void k_l2_writeback() {
    if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
}

int main(int argc, char **argv) {
    const bool wb = argc > 1 && strcmp(argv[1], "--writeback") == 0;
    const size_t n = (size_t)4 << 20;  // 32 MiB per buffer (fits the 32 MiB of L2s)
    const size_t big = (size_t)64 << 20;  // 512 MiB eviction stream
    unsigned long long *ev, *cnt;
    CK(hipMalloc(&ev, big * 8));
    CK(hipMalloc(&cnt, 16));
    CK(hipMemset(ev, 0, big * 8));
    unsigned long long total_a = 0, total_o = 0, total = 0;
    for (int trial = 0; trial < 8; ++trial) {
        const unsigned long long A = 0xA5A5000000000000ull + trial, B = 0x5B5B000000000000ull + trial;
        unsigned long long *c;
        CK(hipMalloc(&c, n * 8));
        k_fill<<<2048, 256>>>(c, n, A);  // plain stores: dirty lines in the L2s
        CK(hipDeviceSynchronize());
        CK(hipFree(c));
        if (wb) {
            k_l2_writeback<<<4096, 64>>>();
            CK(hipDeviceSynchronize());
        }
        unsigned long long *u;
        CK(hipExtMallocWithFlags(reinterpret_cast<void **>(&u), n * 8, hipDeviceMallocUncached));
        const bool same = u == c;
        k_fill_sys<<<2048, 256>>>(u, n, B);
        CK(hipDeviceSynchronize());
        for (int k = 0; k < 3; ++k) k_stream<<<4096, 256>>>(ev, big);
        CK(hipDeviceSynchronize());
        CK(hipMemset(cnt, 0, 16));
        k_count<<<2048, 256>>>(u, n, A, B, cnt);
        unsigned long long h[2];
        CK(hipMemcpy(h, cnt, 16, hipMemcpyDeviceToHost));
        printf("trial %d (%s, uncached buffer %s the freed one's address): %llu of %zu words hold the freed "
               "buffer's pattern, %llu other mismatches\n",
               trial, wb ? "L2 written back before the uncached allocation" : "no write-back",
               same ? "AT" : "not at", h[0], n, h[1]);
        total_a += h[0];
        total_o += h[1];
        total += n;
        CK(hipFree(u));
    }
    printf("UNCACHED_REUSE %s: %llu stale words of %llu (%llu other)\n", wb ? "with-writeback" : "no-writeback",
           total_a, total, total_o);
    return 0;
}
