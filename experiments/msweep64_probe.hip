// msweep64_probe.hip -- layouts of the 64-slot matrix-core sweep (diagnostic).  The engine's
// k_msweep<16> holds two tile pairs per wave (246 VGPRs, 2 waves per SIMD) and reaches ~0.55-0.58
// of 8 TB/s at 32768 rows; here the same update with
//   V0  the engine's shape: 64 columns per wave, both pairs' tiles + the strip's factors issued together
//   V1  one tile pair per wave (32 columns): half the U registers, more waves per SIMD
//   V2  V1 with the next strip's tiles and factors loaded before this strip's matrix steps
//   V3  V0 with the strip's factors loaded once per block into LDS (4 waves share them)
//   V4  V3 with the next strip's tiles and factors loaded before this strip's matrix steps
//   V6  V0 with the next strip's tiles loaded before this strip's matrix steps
// Factors in the engine's strip-major layout (16-row strips, slot-major inside: sx_fidx).  Every
// variant is checked against the vector fma chain, bit for bit.
//   build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off experiments/msweep64_probe.hip -o tools/_ab/msweep64_probe
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

// PAIRS tile pairs per wave (32 columns each); block = 4 waves
template <int PAIRS>
__device__ __forceinline__ void load_u(double2 (&uf)[NKB][PAIRS], const double *U, size_t ld, int c0, int rg, int jl) {
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
        for (int p = 0; p < PAIRS; ++p)
            uf[kb][p] = *reinterpret_cast<const double2 *>(U + (size_t)(4 * kb + rg) * ld + c0 + 32 * p + 2 * jl);
}

template <int PAIRS>
__global__ __launch_bounds__(256) void k_v01(double *T, int rows, int cols, size_t ld, const double *__restrict__ F,
                                             const double *__restrict__ U, int G) {
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6, jl = l & 15, rg = l >> 4;
    const int c0 = (blockIdx.x * 4 + w) * 32 * PAIRS;
    if (c0 >= cols) return;
    double2 uf[NKB][PAIRS];
    load_u<PAIRS>(uf, U, ld, c0, rg, jl);
    const int nstrip = rows / 16;
    for (int g = blockIdx.y; g < nstrip; g += G) {
        const int r0 = g * 16;
        const __amdgpu_buffer_rsrc_t rs = strip_rsrc(T, r0, ld);
        double2 cx[PAIRS][4];
#pragma unroll
        for (int p = 0; p < PAIRS; ++p)
#pragma unroll
            for (int v = 0; v < 4; ++v) cx[p][v] = ld16(rs, (int)(((rg + 4 * v) * ld + c0 + 32 * p + 2 * jl) * 8));
        double ff[NKB];
        const double *Fs = F + fidx(r0, 0) + l;
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb) ff[kb] = Fs[64 * kb];
#pragma unroll
        for (int p = 0; p < PAIRS; ++p) {
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

// V2: one pair per wave, the next strip's loads before this strip's matrix steps
__global__ __launch_bounds__(256) void k_v2(double *T, int rows, int cols, size_t ld, const double *__restrict__ F,
                                            const double *__restrict__ U, int G) {
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6, jl = l & 15, rg = l >> 4;
    const int c0 = (blockIdx.x * 4 + w) * 32;
    if (c0 >= cols) return;
    double2 uf[NKB][1];
    load_u<1>(uf, U, ld, c0, rg, jl);
    const int nstrip = rows / 16;
    int g = blockIdx.y;
    if (g >= nstrip) return;
    double2 cx[4];
    double ff[NKB];
    {
        const __amdgpu_buffer_rsrc_t rs = strip_rsrc(T, g * 16, ld);
#pragma unroll
        for (int v = 0; v < 4; ++v) cx[v] = ld16(rs, (int)(((rg + 4 * v) * ld + c0 + 2 * jl) * 8));
        const double *Fs = F + fidx(g * 16, 0) + l;
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb) ff[kb] = Fs[64 * kb];
    }
    for (; g < nstrip; g += G) {
        const int r0 = g * 16, gn = g + G;
        double2 cn[4];
        double fn[NKB];
        if (gn < nstrip) {
            const __amdgpu_buffer_rsrc_t rs = strip_rsrc(T, gn * 16, ld);
#pragma unroll
            for (int v = 0; v < 4; ++v) cn[v] = ld16(rs, (int)(((rg + 4 * v) * ld + c0 + 2 * jl) * 8));
            const double *Fs = F + fidx(gn * 16, 0) + l;
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb) fn[kb] = Fs[64 * kb];
        }
        d4 ax = {cx[0].x, cx[1].x, cx[2].x, cx[3].x};
        d4 ay = {cx[0].y, cx[1].y, cx[2].y, cx[3].y};
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb) {
            ax = __builtin_amdgcn_mfma_f64_16x16x4f64(ff[kb], uf[kb][0].x, ax, 0, 0, 0);
            ay = __builtin_amdgcn_mfma_f64_16x16x4f64(ff[kb], uf[kb][0].y, ay, 0, 0, 0);
        }
        const __amdgpu_buffer_rsrc_t rs = strip_rsrc(T, r0, ld);
#pragma unroll
        for (int v = 0; v < 4; ++v) st16(rs, (int)(((rg + 4 * v) * ld + c0 + 2 * jl) * 8), ax[v], ay[v]);
        if (gn < nstrip) {
#pragma unroll
            for (int v = 0; v < 4; ++v) cx[v] = cn[v];
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb) ff[kb] = fn[kb];
        }
    }
}

// V3: two pairs per wave, the strip's factors through LDS (double-buffered, one barrier per strip)
__global__ __launch_bounds__(256) void k_v3(double *T, int rows, int cols, size_t ld, const double *__restrict__ F,
                                            const double *__restrict__ U, int G) {
    __shared__ double s_f[2][16 * K];
    const int t = threadIdx.x, l = t & 63, w = t >> 6, jl = l & 15, rg = l >> 4;
    const int c0 = (blockIdx.x * 4 + w) * 64;
    const bool live = c0 < cols;
    double2 uf[NKB][2];
    if (live) load_u<2>(uf, U, ld, c0, rg, jl);
    const int nstrip = rows / 16;
    int buf = 0;
    for (int g = blockIdx.y; g < nstrip; g += G, buf ^= 1) {
        const int r0 = g * 16;
        const __amdgpu_buffer_rsrc_t rs = strip_rsrc(T, r0, ld);
        double2 cx[2][4];
        if (live)
#pragma unroll
            for (int p = 0; p < 2; ++p)
#pragma unroll
                for (int v = 0; v < 4; ++v) cx[p][v] = ld16(rs, (int)(((rg + 4 * v) * ld + c0 + 32 * p + 2 * jl) * 8));
        // the strip's 1024 factors: 4 per thread
        {
            const double2 *src = reinterpret_cast<const double2 *>(F + fidx(r0, 0));
            const double2 a = src[2 * t], b = src[2 * t + 1];
            reinterpret_cast<double2 *>(s_f[buf])[2 * t] = a;
            reinterpret_cast<double2 *>(s_f[buf])[2 * t + 1] = b;
        }
        __syncthreads();
        if (!live) continue;
        double ff[NKB];
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb) ff[kb] = s_f[buf][64 * kb + l];
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

// V4: V3 + the next strip's tableau tiles and factors loaded (to registers) before this strip's
// matrix steps; the factors go to the other LDS buffer after them (one barrier per strip)
__global__ __launch_bounds__(256, 2) void k_v4(double *T, int rows, int cols, size_t ld, const double *__restrict__ F,
                                               const double *__restrict__ U, int G) {
    __shared__ double s_f[2][16 * K];
    const int t = threadIdx.x, l = t & 63, w = t >> 6, jl = l & 15, rg = l >> 4;
    const int c0 = (blockIdx.x * 4 + w) * 64;
    const bool live = c0 < cols;
    double2 uf[NKB][2];
    if (live) load_u<2>(uf, U, ld, c0, rg, jl);
    const int nstrip = rows / 16;
    int g = blockIdx.y;
    if (g >= nstrip) return;
    double2 cx[2][4];
    {
        const __amdgpu_buffer_rsrc_t rs = strip_rsrc(T, g * 16, ld);
        if (live)
#pragma unroll
            for (int p = 0; p < 2; ++p)
#pragma unroll
                for (int v = 0; v < 4; ++v) cx[p][v] = ld16(rs, (int)(((rg + 4 * v) * ld + c0 + 32 * p + 2 * jl) * 8));
        const double2 *src = reinterpret_cast<const double2 *>(F + fidx(g * 16, 0));
        const double2 a = src[2 * t], b = src[2 * t + 1];
        reinterpret_cast<double2 *>(s_f[0])[2 * t] = a;
        reinterpret_cast<double2 *>(s_f[0])[2 * t + 1] = b;
    }
    for (int buf = 0; g < nstrip; g += G, buf ^= 1) {
        __syncthreads();
        const int gn = g + G;
        double2 cn[2][4], fa, fb;
        if (gn < nstrip) {
            const __amdgpu_buffer_rsrc_t rn = strip_rsrc(T, gn * 16, ld);
            if (live)
#pragma unroll
                for (int p = 0; p < 2; ++p)
#pragma unroll
                    for (int v = 0; v < 4; ++v)
                        cn[p][v] = ld16(rn, (int)(((rg + 4 * v) * ld + c0 + 32 * p + 2 * jl) * 8));
            const double2 *src = reinterpret_cast<const double2 *>(F + fidx(gn * 16, 0));
            fa = src[2 * t];
            fb = src[2 * t + 1];
        }
        if (live) {
            const __amdgpu_buffer_rsrc_t rs = strip_rsrc(T, g * 16, ld);
#pragma unroll
            for (int p = 0; p < 2; ++p) {
                d4 ax = {cx[p][0].x, cx[p][1].x, cx[p][2].x, cx[p][3].x};
                d4 ay = {cx[p][0].y, cx[p][1].y, cx[p][2].y, cx[p][3].y};
#pragma unroll
                for (int kb = 0; kb < NKB; ++kb) {
                    const double ff = s_f[buf][64 * kb + l];
                    ax = __builtin_amdgcn_mfma_f64_16x16x4f64(ff, uf[kb][p].x, ax, 0, 0, 0);
                    ay = __builtin_amdgcn_mfma_f64_16x16x4f64(ff, uf[kb][p].y, ay, 0, 0, 0);
                }
#pragma unroll
                for (int v = 0; v < 4; ++v) st16(rs, (int)(((rg + 4 * v) * ld + c0 + 32 * p + 2 * jl) * 8), ax[v], ay[v]);
            }
        }
        if (gn < nstrip) {
            reinterpret_cast<double2 *>(s_f[buf ^ 1])[2 * t] = fa;
            reinterpret_cast<double2 *>(s_f[buf ^ 1])[2 * t + 1] = fb;
            if (live)
#pragma unroll
                for (int p = 0; p < 2; ++p)
#pragma unroll
                    for (int v = 0; v < 4; ++v) cx[p][v] = cn[p][v];
        }
    }
}

// V6: V0 + the next strip's tableau tiles loaded before this strip's matrix steps (factors
// loaded per strip to registers, as V0)
__global__ __launch_bounds__(256, 2) void k_v6(double *T, int rows, int cols, size_t ld, const double *__restrict__ F,
                                               const double *__restrict__ U, int G) {
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6, jl = l & 15, rg = l >> 4;
    const int c0 = (blockIdx.x * 4 + w) * 64;
    if (c0 >= cols) return;
    double2 uf[NKB][2];
    load_u<2>(uf, U, ld, c0, rg, jl);
    const int nstrip = rows / 16;
    int g = blockIdx.y;
    if (g >= nstrip) return;
    double2 cx[2][4];
    {
        const __amdgpu_buffer_rsrc_t rs = strip_rsrc(T, g * 16, ld);
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
            for (int v = 0; v < 4; ++v) cx[p][v] = ld16(rs, (int)(((rg + 4 * v) * ld + c0 + 32 * p + 2 * jl) * 8));
    }
    for (; g < nstrip; g += G) {
        const int gn = g + G;
        double ff[NKB];
        const double *Fs = F + fidx(g * 16, 0) + l;
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb) ff[kb] = Fs[64 * kb];
        double2 cn[2][4];
        if (gn < nstrip) {
            const __amdgpu_buffer_rsrc_t rn = strip_rsrc(T, gn * 16, ld);
#pragma unroll
            for (int p = 0; p < 2; ++p)
#pragma unroll
                for (int v = 0; v < 4; ++v) cn[p][v] = ld16(rn, (int)(((rg + 4 * v) * ld + c0 + 32 * p + 2 * jl) * 8));
        }
        const __amdgpu_buffer_rsrc_t rs = strip_rsrc(T, g * 16, ld);
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
        if (gn < nstrip)
#pragma unroll
            for (int p = 0; p < 2; ++p)
#pragma unroll
                for (int v = 0; v < 4; ++v) cx[p][v] = cn[p][v];
    }
}

// V7<WPC>: the pivot rows U in LDS (the B operands read per 4-slot step with one ds_read_b128 for
// both tiles of a pair), freeing the 128 U registers for a prefetch: the next strip's tableau
// tiles and factors are loaded before this strip's matrix steps.  Block = 4 column groups of 64
// columns (256 columns, 128 KB of U) x WPC waves per group (the waves of a group take alternate
// strips); one block per CU, WPC waves per SIMD.
template <int WPC, bool SGB>
__global__ __launch_bounds__(256 * WPC, 1) void k_v7(double *T, int rows, int cols, size_t ld,
                                                    const double *__restrict__ F, const double *__restrict__ U, int G) {
    extern __shared__ double2 s_u[];  // [kb][cg][p][lane]: 16 x 4 x 2 x 64 double2
    const int t = threadIdx.x, l = t & 63, w = t >> 6, cg = w & 3, sub = w >> 2, jl = l & 15, rg = l >> 4;
    const int c0 = (blockIdx.x * 4 + cg) * 64;
    const bool live = c0 < cols;
    if (live)
        for (int kb = sub; kb < NKB; kb += WPC)
#pragma unroll
            for (int p = 0; p < 2; ++p)
                s_u[((kb * 4 + cg) * 2 + p) * 64 + l] =
                    *reinterpret_cast<const double2 *>(U + (size_t)(4 * kb + rg) * ld + c0 + 32 * p + 2 * jl);
    __syncthreads();
    if (!live) return;
    const int nstrip = rows / 16, GS = G * WPC;
    int g = blockIdx.y * WPC + sub;
    if (g >= nstrip) return;
    double2 cx[2][4];
    double ff[NKB];
    {
        const __amdgpu_buffer_rsrc_t rs = strip_rsrc(T, g * 16, ld);
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
            for (int v = 0; v < 4; ++v) cx[p][v] = ld16(rs, (int)(((rg + 4 * v) * ld + c0 + 32 * p + 2 * jl) * 8));
        const double *Fs = F + fidx(g * 16, 0) + l;
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb) ff[kb] = Fs[64 * kb];
    }
    for (; g < nstrip; g += GS) {
        const int gn = g + GS;
        double2 cn[2][4];
        double fn[NKB];
        if (gn < nstrip) {
            const __amdgpu_buffer_rsrc_t rn = strip_rsrc(T, gn * 16, ld);
#pragma unroll
            for (int p = 0; p < 2; ++p)
#pragma unroll
                for (int v = 0; v < 4; ++v) cn[p][v] = ld16(rn, (int)(((rg + 4 * v) * ld + c0 + 32 * p + 2 * jl) * 8));
            const double *Fs = F + fidx(gn * 16, 0) + l;
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb) fn[kb] = Fs[64 * kb];
        }
        const __amdgpu_buffer_rsrc_t rs = strip_rsrc(T, g * 16, ld);
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            d4 ax = {cx[p][0].x, cx[p][1].x, cx[p][2].x, cx[p][3].x};
            d4 ay = {cx[p][0].y, cx[p][1].y, cx[p][2].y, cx[p][3].y};
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb) {
                const double2 u = s_u[((kb * 4 + cg) * 2 + p) * 64 + l];
                ax = __builtin_amdgcn_mfma_f64_16x16x4f64(ff[kb], u.x, ax, 0, 0, 0);
                ay = __builtin_amdgcn_mfma_f64_16x16x4f64(ff[kb], u.y, ay, 0, 0, 0);
                if (SGB) {
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
                }
            }
#pragma unroll
            for (int v = 0; v < 4; ++v) st16(rs, (int)(((rg + 4 * v) * ld + c0 + 32 * p + 2 * jl) * 8), ax[v], ay[v]);
        }
        if (gn < nstrip) {
#pragma unroll
            for (int p = 0; p < 2; ++p)
#pragma unroll
                for (int v = 0; v < 4; ++v) cx[p][v] = cn[p][v];
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb) ff[kb] = fn[kb];
        }
    }
}

// V8<WPC>: V7 without the prefetch (U in LDS only): WPC waves per SIMD doing V0's strip
template <int WPC, bool SGB>
__global__ __launch_bounds__(256 * WPC, 1) void k_v8(double *T, int rows, int cols, size_t ld,
                                                    const double *__restrict__ F, const double *__restrict__ U, int G) {
    extern __shared__ double2 s_u[];
    const int t = threadIdx.x, l = t & 63, w = t >> 6, cg = w & 3, sub = w >> 2, jl = l & 15, rg = l >> 4;
    const int c0 = (blockIdx.x * 4 + cg) * 64;
    const bool live = c0 < cols;
    if (live)
        for (int kb = sub; kb < NKB; kb += WPC)
#pragma unroll
            for (int p = 0; p < 2; ++p)
                s_u[((kb * 4 + cg) * 2 + p) * 64 + l] =
                    *reinterpret_cast<const double2 *>(U + (size_t)(4 * kb + rg) * ld + c0 + 32 * p + 2 * jl);
    __syncthreads();
    if (!live) return;
    const int nstrip = rows / 16, GS = G * WPC;
    for (int g = blockIdx.y * WPC + sub; g < nstrip; g += GS) {
        const __amdgpu_buffer_rsrc_t rs = strip_rsrc(T, g * 16, ld);
        double2 cx[2][4];
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
            for (int v = 0; v < 4; ++v) cx[p][v] = ld16(rs, (int)(((rg + 4 * v) * ld + c0 + 32 * p + 2 * jl) * 8));
        double ff[NKB];
        const double *Fs = F + fidx(g * 16, 0) + l;
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb) ff[kb] = Fs[64 * kb];
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            d4 ax = {cx[p][0].x, cx[p][1].x, cx[p][2].x, cx[p][3].x};
            d4 ay = {cx[p][0].y, cx[p][1].y, cx[p][2].y, cx[p][3].y};
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb) {
                const double2 u = s_u[((kb * 4 + cg) * 2 + p) * 64 + l];
                ax = __builtin_amdgcn_mfma_f64_16x16x4f64(ff[kb], u.x, ax, 0, 0, 0);
                ay = __builtin_amdgcn_mfma_f64_16x16x4f64(ff[kb], u.y, ay, 0, 0, 0);
                if (SGB) {
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
                }
            }
#pragma unroll
            for (int v = 0; v < 4; ++v) st16(rs, (int)(((rg + 4 * v) * ld + c0 + 32 * p + 2 * jl) * 8), ax[v], ay[v]);
        }
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

void run(const char *name, Kern kern, int cols_per_block, int rows, int cols, int threads = 256, size_t lds = 0) {
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
    if (lds) CK(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, threads, lds));
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const int cb = cols / cols_per_block;
    int G = per_cu * cus / cb;
    if (G > rows / 16) G = rows / 16;
    if (G < 1) G = 1;
    dim3 grid(cb, G);
    CK(hipMemcpy(T2, T, (size_t)rows * ld * 8, hipMemcpyDeviceToDevice));
    kern<<<grid, threads, lds>>>(T2, rows, cols, ld, F, U, G);
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
    for (int i = 0; i < 5; ++i) kern<<<grid, threads, lds>>>(T2, rows, cols, ld, F, U, G);
    CK(hipEventRecord(e0));
    const int it = 30;
    for (int i = 0; i < it; ++i) kern<<<grid, threads, lds>>>(T2, rows, cols, ld, F, U, G);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = 1e3 * ms / it, bytes = 16.0 * rows * cols;
    printf("%s %dx%d blocks/CU %d grid %dx%d: %s (%llu differ)  %.1f us per sweep, frac %.3f, %.2f us per pivot\n", name,
           rows, cols, per_cu, cb, G, h == 0 ? "bit-exact" : "WRONG", h, us, bytes / us / 1e3 / 8000.0, us / K);
    CK(hipFree(T));
    CK(hipFree(T2));
    CK(hipFree(F));
    CK(hipFree(U));
}

int main() {
    const int sizes[3][2] = {{32768, 9216}, {4096, 8192}, {32768, 10240}};
    for (int rep = 0; rep < 1; ++rep)
        for (auto &sz : sizes) {
            run("V0 2 pairs/wave          ", k_v01<2>, 256, sz[0], sz[1]);
            run("V1 1 pair/wave           ", k_v01<1>, 128, sz[0], sz[1]);
            run("V2 1 pair/wave, prefetch ", k_v2, 128, sz[0], sz[1]);
            run("V3 2 pairs/wave, F in LDS", k_v3, 256, sz[0], sz[1]);
            run("V4 V3 + next strip loaded", k_v4, 256, sz[0], sz[1]);
            run("V6 V0 + next tiles loaded", k_v6, 256, sz[0], sz[1]);
            run("V7<1> U in LDS + prefetch", k_v7<1, false>, 256, sz[0], sz[1], 256, 131072);
            run("V7<1> ... sched groups   ", k_v7<1, true>, 256, sz[0], sz[1], 256, 131072);
            run("V7<2> ... sched groups   ", k_v7<2, true>, 256, sz[0], sz[1], 512, 131072);
            run("V7<3> ... sched groups   ", k_v7<3, true>, 256, sz[0], sz[1], 768, 131072);
            run("V8<1> U in LDS           ", k_v8<1, false>, 256, sz[0], sz[1], 256, 131072);
            run("V8<2> U in LDS           ", k_v8<2, false>, 256, sz[0], sz[1], 512, 131072);
            run("V8<2> ... sched groups   ", k_v8<2, true>, 256, sz[0], sz[1], 512, 131072);
            run("V8<3> ... sched groups   ", k_v8<3, true>, 256, sz[0], sz[1], 768, 131072);
            run("V8<4> ... sched groups   ", k_v8<4, true>, 256, sz[0], sz[1], 1024, 131072);
        }
    return 0;
}
