// msweep_probe.hip -- prototype of the batch sweep on the matrix cores (diagnostic).
//
// The sweep applies K pending pivots to every element, in slot order (solver.cu:34-46):
//   x = T[i][j];  for s < K:  x = fma(F[s][i], U[s][j], x)
// v_mfma_f64_16x16x4f64 computes a 16x16 tile's D = A B + C as the k-ordered chain of fused
// multiply-adds, bit for bit (experiments/mfma_f64_probe.hip), so K/4 MFMAs per tile are exactly the
// reference's K updates.  Layout: A (16 rows x 4 slots) lane l = F^T[s0 + l/16][r0 + l%16];
// B (4 slots x 16 columns) lane l = U[s0 + l/16][col(l%16)]; C/D lane l, register v =
// T[r0 + l/16 + 4v][col(l%16)].  Two tiles share a lane's 16-byte access: tile X takes the even
// columns 2j, tile Y the odd 2j+1, so every T access is one 16-byte load / store per lane (4 rows
// x 256 contiguous bytes per wave instruction).  A wave owns 64 columns (2 pairs of tiles) and
// walks 16-row strips; U fragments stay in registers, F fragments are loaded per strip (F stored
// [slot][row], so a fragment load is 4 rows of 128 contiguous bytes).
// This probe measures the in-place bandwidth at K = 32 and 64 and checks every element against
// the VALU chain.
//   build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off experiments/msweep_probe.hip -o tools/_ab/msweep_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                           \
    do {                                                                \
        hipError_t e_ = (x);                                            \
        if (e_ != hipSuccess) {                                         \
            printf("%s at line %d\n", hipGetErrorString(e_), __LINE__); \
            exit(1);                                                    \
        }                                                               \
    } while (0)

typedef double d4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// grid: (column tiles of 256 = 4 waves x 64, row slots G); block 256
template <int K>
__global__ __launch_bounds__(256) void k_msweep(double *T, int rows, int cols, size_t ld, const double *__restrict__ Ft,
                                                const double *__restrict__ U, int G) {
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c0 = (blockIdx.x * 4 + w) * 64;  // this wave's 64 columns
    if (c0 >= cols) return;
    const int jl = l & 15, rg = l >> 4;
    // U fragments: [k-block][pair] -> (even column, odd column) of slot 4 kb + rg
    double2 uf[K / 4][2];
#pragma unroll
    for (int kb = 0; kb < K / 4; ++kb)
#pragma unroll
        for (int p = 0; p < 2; ++p)
            uf[kb][p] = *reinterpret_cast<const double2 *>(U + (size_t)(4 * kb + rg) * ld + c0 + 32 * p + 2 * jl);
    const int nstrip = rows / 16;
    const int oob = 0x7fffffff;
    for (int g = blockIdx.y; g < nstrip; g += G) {
        const int r0 = g * 16;
        double ff[K / 4];
#pragma unroll
        for (int kb = 0; kb < K / 4; ++kb) ff[kb] = Ft[(size_t)(4 * kb + rg) * rows + r0 + jl];
        double2 cx[2][4];
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                    T + (size_t)(r0 + rg + 4 * v) * ld, 0, oob, 0x00020000);
                cx[p][v] = __builtin_bit_cast(double2,
                                              __builtin_amdgcn_raw_buffer_load_b128(rs, (c0 + 32 * p + 2 * jl) * 8, 0, 2));
            }
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            d4 ax = {cx[p][0].x, cx[p][1].x, cx[p][2].x, cx[p][3].x};
            d4 ay = {cx[p][0].y, cx[p][1].y, cx[p][2].y, cx[p][3].y};
#pragma unroll
            for (int kb = 0; kb < K / 4; ++kb) {
                ax = __builtin_amdgcn_mfma_f64_16x16x4f64(ff[kb], uf[kb][p].x, ax, 0, 0, 0);
                ay = __builtin_amdgcn_mfma_f64_16x16x4f64(ff[kb], uf[kb][p].y, ay, 0, 0, 0);
            }
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                    T + (size_t)(r0 + rg + 4 * v) * ld, 0, oob, 0x00020000);
                const double2 y = make_double2(ax[v], ay[v]);
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, y), rs, (c0 + 32 * p + 2 * jl) * 8, 0,
                                                       16);
            }
        }
    }
}

// the same, one pair of tiles at a time (fewer registers: 2 waves per SIMD at K = 64)
template <int K>
__global__ __launch_bounds__(256, 2) void k_msweep2(double *T, int rows, int cols, size_t ld,
                                                    const double *__restrict__ Ft, const double *__restrict__ U, int G) {
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c0 = (blockIdx.x * 4 + w) * 64;
    if (c0 >= cols) return;
    const int jl = l & 15, rg = l >> 4;
    double2 uf[K / 4][2];
#pragma unroll
    for (int kb = 0; kb < K / 4; ++kb)
#pragma unroll
        for (int p = 0; p < 2; ++p)
            uf[kb][p] = *reinterpret_cast<const double2 *>(U + (size_t)(4 * kb + rg) * ld + c0 + 32 * p + 2 * jl);
    const int nstrip = rows / 16;
    const int oob = 0x7fffffff;
    for (int g = blockIdx.y; g < nstrip; g += G) {
        const int r0 = g * 16;
        double ff[K / 4];
#pragma unroll
        for (int kb = 0; kb < K / 4; ++kb) ff[kb] = Ft[(size_t)(4 * kb + rg) * rows + r0 + jl];
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            double2 cx[4];
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                    T + (size_t)(r0 + rg + 4 * v) * ld, 0, oob, 0x00020000);
                cx[v] = __builtin_bit_cast(double2,
                                           __builtin_amdgcn_raw_buffer_load_b128(rs, (c0 + 32 * p + 2 * jl) * 8, 0, 2));
            }
            d4 ax = {cx[0].x, cx[1].x, cx[2].x, cx[3].x};
            d4 ay = {cx[0].y, cx[1].y, cx[2].y, cx[3].y};
#pragma unroll
            for (int kb = 0; kb < K / 4; ++kb) {
                ax = __builtin_amdgcn_mfma_f64_16x16x4f64(ff[kb], uf[kb][p].x, ax, 0, 0, 0);
                ay = __builtin_amdgcn_mfma_f64_16x16x4f64(ff[kb], uf[kb][p].y, ay, 0, 0, 0);
            }
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                    T + (size_t)(r0 + rg + 4 * v) * ld, 0, oob, 0x00020000);
                const double2 y = make_double2(ax[v], ay[v]);
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, y), rs, (c0 + 32 * p + 2 * jl) * 8, 0,
                                                       16);
            }
        }
    }
}

// the same with one wave-uniform buffer resource per strip (the per-lane row bases above compile
// to waterfall loops), as the engine's k_msweep
template <int K>
__global__ __launch_bounds__(256, 2) void k_msweep3(double *T, int rows, int cols, size_t ld,
                                                    const double *__restrict__ Ft, const double *__restrict__ U, int G) {
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c0 = (blockIdx.x * 4 + w) * 64;
    if (c0 >= cols) return;
    const int jl = l & 15, rg = l >> 4;
    double2 uf[K / 4][2];
#pragma unroll
    for (int kb = 0; kb < K / 4; ++kb)
#pragma unroll
        for (int p = 0; p < 2; ++p)
            uf[kb][p] = *reinterpret_cast<const double2 *>(U + (size_t)(4 * kb + rg) * ld + c0 + 32 * p + 2 * jl);
    const int nstrip = rows / 16;
    for (int g = blockIdx.y; g < nstrip; g += G) {
        const int r0 = g * 16;
        double ff[K / 4];
#pragma unroll
        for (int kb = 0; kb < K / 4; ++kb) ff[kb] = Ft[(size_t)(4 * kb + rg) * rows + r0 + jl];
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(T + (size_t)r0 * ld, 0, (int)(16 * ld * 8), 0x00020000);
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            double2 cx[4];
#pragma unroll
            for (int v = 0; v < 4; ++v)
                cx[v] = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(
                                                        rs, (int)(((rg + 4 * v) * ld + c0 + 32 * p + 2 * jl) * 8), 0, 2));
            d4 ax = {cx[0].x, cx[1].x, cx[2].x, cx[3].x};
            d4 ay = {cx[0].y, cx[1].y, cx[2].y, cx[3].y};
#pragma unroll
            for (int kb = 0; kb < K / 4; ++kb) {
                ax = __builtin_amdgcn_mfma_f64_16x16x4f64(ff[kb], uf[kb][p].x, ax, 0, 0, 0);
                ay = __builtin_amdgcn_mfma_f64_16x16x4f64(ff[kb], uf[kb][p].y, ay, 0, 0, 0);
            }
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const double2 y = make_double2(ax[v], ay[v]);
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, y), rs,
                                                       (int)(((rg + 4 * v) * ld + c0 + 32 * p + 2 * jl) * 8), 0, 16);
            }
        }
    }
}

// reference: the VALU chain, one element per thread
template <int K>
__global__ void k_ref(double *T, int rows, int cols, size_t ld, const double *Ft, const double *U) {
    const size_t n = (size_t)rows * cols;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x) {
        const int i = (int)(e / cols), j = (int)(e % cols);
        double x = T[(size_t)i * ld + j];
        for (int s = 0; s < K; ++s) x = fma(Ft[(size_t)s * rows + i], U[(size_t)s * ld + j], x);
        T[(size_t)i * ld + j] = x;
    }
}

__global__ void k_cmp(const double *A, const double *B, size_t n, unsigned long long *bad) {
    unsigned long long c = 0;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x)
        c += __double_as_longlong(A[e]) != __double_as_longlong(B[e]);
    atomicAdd(bad, c);
}

__global__ void k_init(double *p, size_t n, unsigned seed, double lo, double hi) {
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x) {
        unsigned long long x = (e + 1) * 0x9E3779B97F4A7C15ull ^ (unsigned long long)seed * 0xBF58476D1CE4E5B9ull;
        x ^= x >> 31;
        x *= 0x94D049BB133111EBull;
        x ^= x >> 29;
        p[e] = lo + (hi - lo) * (double)(x >> 11) * (1.0 / 9007199254740992.0);
    }
}

template <int K, int VAR>
void run(int rows, int cols, size_t ld_pad = 0) {
    auto kern = VAR == 2 ? k_msweep3<K> : VAR ? k_msweep2<K> : k_msweep<K>;
    const size_t ld = ld_pad ? ld_pad : cols;
    double *T, *T2, *Ft, *U;
    CK(hipMalloc(&T, (size_t)rows * ld * 8));
    CK(hipMalloc(&T2, (size_t)rows * ld * 8));
    CK(hipMalloc(&Ft, (size_t)K * rows * 8));
    CK(hipMalloc(&U, (size_t)K * ld * 8));
    k_init<<<4096, 256>>>(T, (size_t)rows * ld, 1, 1.0, 100.0);
    k_init<<<4096, 256>>>(Ft, (size_t)K * rows, 2, -1e-2, 1e-2);
    k_init<<<4096, 256>>>(U, (size_t)K * ld, 3, 1.0, 100.0);
    CK(hipMemcpy(T2, T, (size_t)rows * ld * 8, hipMemcpyDeviceToDevice));
    int per_cu = 0, cus = 0, dev = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 256, 0));
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const int cb = cols / 256;
    for (int mult : {1, 2}) {
        int G = per_cu * cus * mult / cb;
        if (G > rows / 16) G = rows / 16;
        if (G < 1) G = 1;
        dim3 grid(cb, G);
        // correctness: one sweep vs the VALU chain
        if (mult == 1) {
            CK(hipMemcpy(T2, T, (size_t)rows * ld * 8, hipMemcpyDeviceToDevice));
            kern<<<grid, 256>>>(T2, rows, cols, ld, Ft, U, G);
            k_ref<K><<<8192, 256>>>(T, rows, cols, ld, Ft, U);
            unsigned long long *bad;
            CK(hipMalloc(&bad, 8));
            CK(hipMemset(bad, 0, 8));
            k_cmp<<<4096, 256>>>(T, T2, (size_t)rows * ld, bad);
            unsigned long long h = 0;
            CK(hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost));
            printf("K=%d var %d %dx%d: MFMA sweep vs VALU chain: %llu of %zu elements differ\n", K, VAR, rows, cols, h,
                   (size_t)rows * ld);
            CK(hipFree(bad));
        }
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        for (int i = 0; i < 5; ++i) kern<<<grid, 256>>>(T2, rows, cols, ld, Ft, U, G);
        CK(hipEventRecord(e0));
        const int it = 30;
        for (int i = 0; i < it; ++i) kern<<<grid, 256>>>(T2, rows, cols, ld, Ft, U, G);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = 1e3 * ms / it, bytes = 16.0 * rows * cols;
        printf("K=%d var %d %dx%d blocks/CU %d grid %dx%d: %.1f us per sweep, %.0f GB/s (frac %.3f), %.2f us per pivot\n",
               K, VAR, rows, cols, per_cu, cb, G, us, bytes / us / 1e3, bytes / us / 1e3 / 8000.0, us / K);
    }
    CK(hipFree(T));
    CK(hipFree(T2));
    CK(hipFree(Ft));
    CK(hipFree(U));
}

int main() {
    for (int rep = 0; rep < 2; ++rep) {
        run<32, 2>(4096, 8192);
        run<64, 2>(4096, 8192);
        run<32, 2>(4096, 11008, 12304);
        run<64, 2>(4096, 11008, 12304);
        run<32, 2>(32768, 9216);
        run<64, 2>(32768, 9216);
        run<32, 2>(32768, 9216, 12288);
        run<64, 2>(32768, 9216, 12288);
    }
    return 0;
}
