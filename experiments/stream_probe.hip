// stream_probe.hip -- what bounds the sweep?  Streams an m x N fp64 matrix (row stride ld) the
// way k_sweep does (a thread owns two adjacent columns, 16-byte accesses, RB rows per step, a
// resident grid of column tiles x row slots) with K fmas per element against per-column
// registers and per-row scalar factors, writing either in place or to a second buffer.
// usage: stream_probe <m> <N> [iters]     prints GB/s (read + write bytes) per variant
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                   \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            printf("%s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);   \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int K, int RB, bool SC1>
__global__ __launch_bounds__(256) void k_stream(const double *Tin, double *Tout, int rows, size_t ld, int N,
                                                const double *__restrict__ F, const double *__restrict__ U) {
    const int cb = (N + 511) / 512;
    if ((int)blockIdx.x >= cb) return;
    const int j = ((int)blockIdx.x * 256 + (int)threadIdx.x) * 2;
    if (j >= N) return;
    double2 u[K > 0 ? K : 1];
#pragma unroll
    for (int s = 0; s < K; ++s) u[s] = *reinterpret_cast<const double2 *>(U + (size_t)s * ld + j);
    const int ng = (rows + RB - 1) / RB;
    const int oob = (int)(ld * 8);
    for (int g = blockIdx.y; g < ng; g += gridDim.y) {
        const int i0 = g * RB;
        double2 x[RB];
#pragma unroll
        for (int k = 0; k < RB; ++k) {
            const int i = i0 + k < rows ? i0 + k : i0;
            const __amdgpu_buffer_rsrc_t rs =
                __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(Tin) + (size_t)i * ld, 0, oob, 0x00020000);
            x[k] = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(rs, i0 + k < rows ? j * 8 : oob,
                                                                                      0, 0));
        }
#pragma unroll
        for (int k = 0; k < RB; ++k) {
            const int i = i0 + k;
            if (i >= rows) break;
            double2 y = x[k];
            if (K > 0) {
                const double *Fr = F + (size_t)i * 32;
                double f[K > 0 ? K : 1];
#pragma unroll
                for (int s = 0; s < K; ++s) f[s] = Fr[s];
#pragma unroll
                for (int s = 0; s < K; ++s) {
                    y.x = fma(f[s], u[s].x, y.x);
                    y.y = fma(f[s], u[s].y, y.y);
                }
            }
            const __amdgpu_buffer_rsrc_t rs =
                __builtin_amdgcn_make_buffer_rsrc(Tout + (size_t)i * ld, 0, oob, 0x00020000);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, y), rs, j * 8, 0, SC1 ? 16 : 0);
        }
    }
}

// reference: a flat grid-stride float4 copy (MI355X_MICROARCH.md's 6.29 TB/s form)
__global__ __launch_bounds__(256) void k_linear(const double2 *a, double2 *b, size_t n) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) b[i] = a[i];
}

// the 2-D walk with wider column tiles: each thread owns two adjacent columns in each of W
// 512-column chunks of one block-tile (W x 4 KB contiguous per row per block)
template <int W, int RB>
__global__ __launch_bounds__(256) void k_wide(const double *Tin, double *Tout, int rows, size_t ld, int N) {
    const int cw = 512 * W;
    const int cb = (N + cw - 1) / cw;
    if ((int)blockIdx.x >= cb) return;
    const int ng = (rows + RB - 1) / RB;
    const int oob = (int)(ld * 8);
    for (int g = blockIdx.y; g < ng; g += gridDim.y) {
        const int i0 = g * RB;
        double2 x[RB][W];
#pragma unroll
        for (int k = 0; k < RB; ++k) {
            const int i = i0 + k < rows ? i0 + k : i0;
            const __amdgpu_buffer_rsrc_t rs =
                __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(Tin) + (size_t)i * ld, 0, oob, 0x00020000);
#pragma unroll
            for (int w = 0; w < W; ++w) {
                const int j = (int)blockIdx.x * cw + w * 512 + (int)threadIdx.x * 2;
                x[k][w] = __builtin_bit_cast(
                    double2, __builtin_amdgcn_raw_buffer_load_b128(rs, (i0 + k < rows && j < N) ? j * 8 : oob, 0, 0));
            }
        }
#pragma unroll
        for (int k = 0; k < RB; ++k) {
            const int i = i0 + k;
            if (i >= rows) break;
            const __amdgpu_buffer_rsrc_t rs =
                __builtin_amdgcn_make_buffer_rsrc(Tout + (size_t)i * ld, 0, oob, 0x00020000);
#pragma unroll
            for (int w = 0; w < W; ++w) {
                const int j = (int)blockIdx.x * cw + w * 512 + (int)threadIdx.x * 2;
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, x[k][w]), rs, j < N ? j * 8 : oob, 0,
                                                       16);
            }
        }
    }
}

template <int W, int RB>
static void run_wide(double *A, int m, size_t ld, int N, int iters, float waves) {
    int per_cu = 0, cus = 0;
    CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_wide<W, RB>, 256, 0));
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int cb = (N + 512 * W - 1) / (512 * W);
    int G = (int)(waves * per_cu * cus) / cb;
    if (G < 1) G = 1;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    k_wide<W, RB><<<dim3(cb, G), 256>>>(A, A, m, ld, N);
    CHECK(hipEventRecord(e0));
    for (int it = 0; it < iters; ++it) k_wide<W, RB><<<dim3(cb, G), 256>>>(A, A, m, ld, N);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    printf("copy in place, %2d x 4 KB per row  RB=%d waves=%.1f occ=%d: %8.1f us/launch  %7.1f GB/s\n", W, RB, waves,
           per_cu, 1e3 * ms / iters, 16.0 * m * N * iters / (ms * 1e-3) / 1e9);
    fflush(stdout);
}

template <int K, int RB, bool SC1>
static void run(const char *name, double *A, double *B, bool inplace, int m, size_t ld, int N, const double *F,
                const double *U, int iters) {
    int per_cu = 0, cus = 0;
    CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_stream<K, RB, SC1>, 256, 0));
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int cb = (N + 511) / 512;
    int G = per_cu * cus / cb;
    if (G < 1) G = 1;
    dim3 grid(cb, G);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    k_stream<K, RB, SC1><<<grid, 256>>>(A, inplace ? A : B, m, ld, N, F, U);  // warm
    CHECK(hipEventRecord(e0));
    for (int it = 0; it < iters; ++it) {
        const double *src = inplace ? A : ((it & 1) ? B : A);
        double *dst = inplace ? A : ((it & 1) ? A : B);
        k_stream<K, RB, SC1><<<grid, 256>>>(src, dst, m, ld, N, F, U);
    }
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double bytes = 16.0 * (double)m * (double)N * iters;
    printf("%-34s K=%2d RB=%d sc1=%d occ=%d: %8.1f us/launch  %7.1f GB/s\n", name, K, RB, SC1 ? 1 : 0, per_cu,
           1e3 * ms / iters, bytes / (ms * 1e-3) / 1e9);
    fflush(stdout);
}

int main(int argc, char **argv) {
    const int m = argc > 1 ? atoi(argv[1]) : 32768;
    const int N = argc > 2 ? atoi(argv[2]) : 40961;
    const int iters = argc > 3 ? atoi(argv[3]) : 10;
    const size_t ld = ((size_t)N + 15) / 16 * 16;
    double *A, *B, *F, *U;
    CHECK(hipMalloc(&A, sizeof(double) * ld * m));
    CHECK(hipMalloc(&B, sizeof(double) * ld * m));
    CHECK(hipMalloc(&F, sizeof(double) * 32 * m));
    CHECK(hipMalloc(&U, sizeof(double) * 32 * ld));
    CHECK(hipMemset(A, 0, sizeof(double) * ld * m));
    CHECK(hipMemset(B, 0, sizeof(double) * ld * m));
    CHECK(hipMemset(F, 0, sizeof(double) * 32 * m));
    CHECK(hipMemset(U, 0, sizeof(double) * 32 * ld));
    printf("m=%d N=%d ld=%zu (%.2f GB per pass read+write)\n", m, N, ld, 16.0 * m * N / 1e9);
    {
        const size_t n2 = ld * m / 2;
        hipEvent_t e0, e1;
        CHECK(hipEventCreate(&e0));
        CHECK(hipEventCreate(&e1));
        for (int blocks : {2048, 8192, 32768}) {
            k_linear<<<blocks, 256>>>((const double2 *)A, (double2 *)B, n2);
            CHECK(hipEventRecord(e0));
            for (int it = 0; it < iters; ++it) k_linear<<<blocks, 256>>>((const double2 *)A, (double2 *)B, n2);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms = 0.f;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            printf("linear float4 copy, %6d blocks: %8.1f us/launch  %7.1f GB/s\n", blocks, 1e3 * ms / iters,
                   32.0 * n2 * iters / (ms * 1e-3) / 1e9);
        }
    }
    run_wide<1, 4>(A, m, ld, N, iters, 1.0f);
    run_wide<2, 4>(A, m, ld, N, iters, 1.0f);
    run_wide<4, 4>(A, m, ld, N, iters, 1.0f);
    run_wide<1, 8>(A, m, ld, N, iters, 1.0f);
    run_wide<1, 4>(A, m, ld, N, iters, 2.0f);
    run_wide<4, 2>(A, m, ld, N, iters, 1.0f);
    run<0, 4, true>("copy in place", A, B, true, m, ld, N, F, U, iters);
    run<0, 4, true>("copy out of place", A, B, false, m, ld, N, F, U, iters);
    run<0, 4, false>("copy out of place", A, B, false, m, ld, N, F, U, iters);
    run<32, 4, true>("sweep in place", A, B, true, m, ld, N, F, U, iters);
    run<32, 4, true>("sweep out of place", A, B, false, m, ld, N, F, U, iters);
    run<32, 4, false>("sweep out of place", A, B, false, m, ld, N, F, U, iters);
    run<16, 4, true>("sweep in place", A, B, true, m, ld, N, F, U, iters);
    run<8, 4, true>("sweep in place", A, B, true, m, ld, N, F, U, iters);
    return 0;
}
