// vsweep_probe.hip -- the 64-slot sweep on the vector units (diagnostic).  The fp64 vector FMA
// sustains 53-62 TFLOP/s on this chip against 47.6 for v_mfma_f64_16x16x4f64
// (profiles/r03_f64_rate_probe.txt); the obstacle is operand delivery: a factor F[i][s] is
// uniform across a row's columns.  Here a lane owns one column, keeps its 64 pivot-row values
// U[s][j] in registers, and takes F[i][s] from a register that holds 16 slots of the row (lane
// l: slot 16c + l % 16) broadcast by DPP inside each 16-lane row: v_fmac_f64_dpp ...
// row_newbcast:k -- x = fma(F[i][16c + k], U[16c + k][j], x), the reference's chain in slot order.
//   V0     the engine's matrix-core shape (two tile pairs per wave), for comparison
//   D<R>   R rows per step (R independent chains per lane), factors in the strip-major layout
// Every variant is checked against the sequential fma chain, bit for bit.
//   build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off experiments/vsweep_probe.hip -o tools/_ab/vsweep_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

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
constexpr int K = 64, NKB = 16;

__device__ __forceinline__ size_t fidx(long long i, int s) { return (size_t)(i >> 4) * (16 * K) + (size_t)s * 16 + (size_t)(i & 15); }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t strip_rsrc(double *T, int r0, size_t ld) {
    return __builtin_amdgcn_make_buffer_rsrc(T + (size_t)r0 * ld, 0, (int)(16 * ld * 8), 0x00020000);
}
__device__ __forceinline__ double2 ld16(__amdgpu_buffer_rsrc_t rs, int off) {
    return __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 2));
}
__device__ __forceinline__ void st16(__amdgpu_buffer_rsrc_t rs, int off, double x, double y) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, make_double2(x, y)), rs, off, 0, 16);
}

__global__ __launch_bounds__(256) void k_v0(double *T, int rows, int cols, size_t ld, const double *__restrict__ F,
                                            const double *__restrict__ U, int G) {
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6, jl = l & 15, rg = l >> 4;
    const int c0 = (blockIdx.x * 4 + w) * 64;
    if (c0 >= cols) return;
    double2 uf[NKB][2];
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
        for (int p = 0; p < 2; ++p)
            uf[kb][p] = *reinterpret_cast<const double2 *>(U + (size_t)(4 * kb + rg) * ld + c0 + 32 * p + 2 * jl);
    const int nstrip = rows / 16;
    for (int g = blockIdx.y; g < nstrip; g += G) {
        const int r0 = g * 16;
        const __amdgpu_buffer_rsrc_t rs = strip_rsrc(T, r0, ld);
        double2 cx[2][4];
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
            for (int v = 0; v < 4; ++v) cx[p][v] = ld16(rs, (int)(((rg + 4 * v) * ld + c0 + 32 * p + 2 * jl) * 8));
        double ff[NKB];
        const double *Fs = F + fidx(r0, 0) + l;
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb) ff[kb] = Fs[64 * kb];
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            d4 ax = {cx[p][0].x, cx[p][1].x, cx[p][2].x, cx[p][3].x};
            d4 ay = {cx[p][0].y, cx[p][1].y, cx[p][2].y, cx[p][3].y};
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb) {
                ax = __builtin_amdgcn_mfma_f64_16x16x4f64(ff[kb], uf[kb][p].x, ax, 0, 0, 0);
                ay = __builtin_amdgcn_mfma_f64_16x16x4f64(ff[kb], uf[kb][p].y, ay, 0, 0, 0);
            }
#pragma unroll
            for (int v = 0; v < 4; ++v) st16(rs, (int)(((rg + 4 * v) * ld + c0 + 32 * p + 2 * jl) * 8), ax[v], ay[v]);
        }
    }
}

// x = fma(f broadcast from lane K of each 16-lane row, u, x)
template <int KL>
__device__ __forceinline__ double fmac_bcast(double x, double f, double u) {
    asm("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf" : "+v"(x) : "v"(f), "v"(u), "n"(KL));
    return x;
}

template <int S0, int R>
__device__ __forceinline__ void chunk16(double (&x)[R], const double (&fv)[R], const double *u) {
#define SX_STEP(KL)                                                                   \
    _Pragma("unroll") for (int k = 0; k < R; ++k) x[k] = fmac_bcast<KL>(x[k], fv[k], u[S0 + KL]);
    SX_STEP(0) SX_STEP(1) SX_STEP(2) SX_STEP(3) SX_STEP(4) SX_STEP(5) SX_STEP(6) SX_STEP(7)
    SX_STEP(8) SX_STEP(9) SX_STEP(10) SX_STEP(11) SX_STEP(12) SX_STEP(13) SX_STEP(14) SX_STEP(15)
#undef SX_STEP
}

// D<R>: lane = column (64 per wave), R rows per step
template <int R>
__global__ __launch_bounds__(256, 2) void k_dpp(double *T, int rows, int cols, size_t ld, const double *__restrict__ F,
                                                const double *__restrict__ U, int G) {
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int j = (blockIdx.x * 4 + w) * 64 + l;
    if ((blockIdx.x * 4 + w) * 64 >= cols) return;
    double u[K];
#pragma unroll
    for (int s = 0; s < K; ++s) u[s] = U[(size_t)s * ld + j];
    const int ng = rows / R;
    for (int g = blockIdx.y; g < ng; g += G) {
        const int i0 = g * R;
        double x[R];
#pragma unroll
        for (int k = 0; k < R; ++k) x[k] = __builtin_nontemporal_load(T + (size_t)(i0 + k) * ld + j);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            double fv[R];
#pragma unroll
            for (int k = 0; k < R; ++k) fv[k] = F[fidx(i0 + k, 16 * c + (l & 15))];
            if (c == 0) chunk16<0, R>(x, fv, u);
            if (c == 1) chunk16<16, R>(x, fv, u);
            if (c == 2) chunk16<32, R>(x, fv, u);
            if (c == 3) chunk16<48, R>(x, fv, u);
        }
#pragma unroll
        for (int k = 0; k < R; ++k) T[(size_t)(i0 + k) * ld + j] = x[k];
    }
}

__global__ void k_ref(double *T, int rows, int cols, size_t ld, const double *F, const double *U) {
    const size_t n = (size_t)rows * cols;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x) {
        const int i = (int)(e / cols), j = (int)(e % cols);
        double x = T[(size_t)i * ld + j];
        for (int s = 0; s < K; ++s) x = fma(F[fidx(i, s)], U[(size_t)s * ld + j], x);
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

typedef void (*Kern)(double *, int, int, size_t, const double *, const double *, int);

void run(const char *name, Kern kern, int cols_per_block, int rows, int cols, int rows_per_slot) {
    const size_t ld = cols;
    double *T, *T2, *F, *U;
    CK(hipMalloc(&T, (size_t)rows * ld * 8));
    CK(hipMalloc(&T2, (size_t)rows * ld * 8));
    CK(hipMalloc(&F, (size_t)K * rows * 8));
    CK(hipMalloc(&U, (size_t)K * ld * 8));
    k_init<<<4096, 256>>>(T, (size_t)rows * ld, 1, 1.0, 100.0);
    k_init<<<4096, 256>>>(F, (size_t)K * rows, 2, -1e-2, 1e-2);
    k_init<<<4096, 256>>>(U, (size_t)K * ld, 3, 1.0, 100.0);
    int per_cu = 0, cus = 0, dev = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 256, 0));
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const int cb = cols / cols_per_block;
    int G = per_cu * cus / cb;
    if (G > rows / rows_per_slot) G = rows / rows_per_slot;
    if (G < 1) G = 1;
    dim3 grid(cb, G);
    CK(hipMemcpy(T2, T, (size_t)rows * ld * 8, hipMemcpyDeviceToDevice));
    kern<<<grid, 256>>>(T2, rows, cols, ld, F, U, G);
    k_ref<<<8192, 256>>>(T, rows, cols, ld, F, U);
    unsigned long long *bad;
    CK(hipMalloc(&bad, 8));
    CK(hipMemset(bad, 0, 8));
    k_cmp<<<4096, 256>>>(T, T2, (size_t)rows * ld, bad);
    unsigned long long h = 0;
    CK(hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost));
    CK(hipFree(bad));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 5; ++i) kern<<<grid, 256>>>(T2, rows, cols, ld, F, U, G);
    CK(hipEventRecord(e0));
    const int it = 30;
    for (int i = 0; i < it; ++i) kern<<<grid, 256>>>(T2, rows, cols, ld, F, U, G);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = 1e3 * ms / it, bytes = 16.0 * rows * cols;
    printf("%s %dx%d blocks/CU %d grid %dx%d: %s (%llu differ)  %.1f us per sweep, frac %.3f, %.1f TFLOP/s, %.2f us per pivot\n",
           name, rows, cols, per_cu, cb, G, h == 0 ? "bit-exact" : "WRONG", h, us, bytes / us / 1e3 / 8000.0,
           2.0 * K * rows * cols / us / 1e6, us / K);
    CK(hipFree(T));
    CK(hipFree(T2));
    CK(hipFree(F));
    CK(hipFree(U));
}

int main() {
    const int sizes[3][2] = {{32768, 9216}, {4096, 8192}, {32768, 10240}};
    for (int rep = 0; rep < 2; ++rep)
        for (auto &sz : sizes) {
            run("V0 matrix cores", k_v0, 256, sz[0], sz[1], 16);
            run("D4 vector, dpp ", k_dpp<4>, 256, sz[0], sz[1], 4);
            run("D8 vector, dpp ", k_dpp<8>, 256, sz[0], sz[1], 8);
        }
    return 0;
}
