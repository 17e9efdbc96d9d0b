// bench_update.hip -- variant sweep of the rank-1 tableau update (development tool).
//
// Times several organisations of T[i][j] = fma(f_i, prow[j], T[i][j]) over an m x N fp64
// tableau (row stride ld) and checks each against variant 0 bit for bit after one launch.
// usage: bench_update <m> <N> [iters]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            printf("%s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);              \
            exit(1);                                                                          \
        }                                                                                     \
    } while (0)

typedef double d2 __attribute__((ext_vector_type(2)));

struct Args {
    double *T;
    int rows;
    size_t ld;
    int N;
    const double *prow;
    const double *f;
    int r;
    double p;
    int flip;
};

template <int RB, int CPT, bool NT, bool SNAKE, bool NTS = false, int TPB = 256>
__global__ __launch_bounds__(TPB) void k_var(Args a) {
    int bx = blockIdx.x, by = blockIdx.y;
    if (SNAKE && a.flip) {
        bx = gridDim.x - 1 - bx;
        by = gridDim.y - 1 - by;
    }
    const int i0 = by * RB;
    const int j = (bx * TPB + threadIdx.x) * (2 * CPT);
    if (j >= a.N) return;
    const int nrow = a.rows - i0 < RB ? a.rows - i0 : RB;
    d2 pr[CPT];
#pragma unroll
    for (int c = 0; c < CPT; ++c) pr[c] = *reinterpret_cast<const d2 *>(a.prow + j + 2 * c);
    double *base = a.T + (size_t)i0 * a.ld + j;
    if (nrow == RB && j + 2 * CPT <= a.N) {
        d2 x[RB][CPT];
#pragma unroll
        for (int k = 0; k < RB; ++k)
#pragma unroll
            for (int c = 0; c < CPT; ++c) {
                d2 *ptr = reinterpret_cast<d2 *>(base + (size_t)k * a.ld + 2 * c);
                x[k][c] = NT ? __builtin_nontemporal_load(ptr) : *ptr;
            }
#pragma unroll
        for (int k = 0; k < RB; ++k) {
            const double f = a.f[i0 + k];
#pragma unroll
            for (int c = 0; c < CPT; ++c) {
                d2 y;
                if (i0 + k == a.r) {
                    y.x = pr[c].x / a.p;
                    y.y = pr[c].y / a.p;
                } else {
                    y.x = fma(f, pr[c].x, x[k][c].x);
                    y.y = fma(f, pr[c].y, x[k][c].y);
                }
                d2 *ptr = reinterpret_cast<d2 *>(base + (size_t)k * a.ld + 2 * c);
                if (NT || NTS)
                    __builtin_nontemporal_store(y, ptr);
                else
                    *ptr = y;
            }
        }
    } else {
        for (int k = 0; k < nrow; ++k)
            for (int jj = j; jj < j + 2 * CPT && jj < a.N; ++jj) {
                double *x = base + (size_t)k * a.ld + (jj - j);
                *x = (i0 + k == a.r) ? a.prow[jj] / a.p : fma(a.f[i0 + k], a.prow[jj], *x);
            }
    }
}

// persistent: fixed grid, each block walks tiles (RB rows x 512 cols) with a stride
template <int RB, bool SNAKE>
__global__ __launch_bounds__(256) void k_persist(Args a, int tiles_x, int tiles_y) {
    const int ntiles = tiles_x * tiles_y;
    for (int t0 = blockIdx.x; t0 < ntiles; t0 += gridDim.x) {
        const int t = (SNAKE && a.flip) ? ntiles - 1 - t0 : t0;
        const int bx = t % tiles_x, by = t / tiles_x;
        const int i0 = by * RB;
        const int j = (bx * 256 + threadIdx.x) * 2;
        if (j >= a.N) continue;
        const int nrow = a.rows - i0 < RB ? a.rows - i0 : RB;
        const d2 pr = *reinterpret_cast<const d2 *>(a.prow + j);
        double *base = a.T + (size_t)i0 * a.ld + j;
        if (nrow == RB && j + 2 <= a.N) {
            d2 x[RB];
#pragma unroll
            for (int k = 0; k < RB; ++k) x[k] = *reinterpret_cast<const d2 *>(base + (size_t)k * a.ld);
#pragma unroll
            for (int k = 0; k < RB; ++k) {
                const double f = a.f[i0 + k];
                d2 y;
                if (i0 + k == a.r) {
                    y.x = pr.x / a.p;
                    y.y = pr.y / a.p;
                } else {
                    y.x = fma(f, pr.x, x[k].x);
                    y.y = fma(f, pr.y, x[k].y);
                }
                *reinterpret_cast<d2 *>(base + (size_t)k * a.ld) = y;
            }
        } else {
            for (int k = 0; k < nrow; ++k)
                for (int jj = j; jj < j + 2 && jj < a.N; ++jj) {
                    double *x = base + (size_t)k * a.ld + (jj - j);
                    *x = (i0 + k == a.r) ? a.prow[jj] / a.p : fma(a.f[i0 + k], a.prow[jj], *x);
                }
        }
    }
}

typedef unsigned int u4 __attribute__((ext_vector_type(4)));

// RB rows per block, 2 doubles per thread, stores write-through (sc1) via a buffer resource
template <int RB, bool SNAKE, int AUX>
__global__ __launch_bounds__(256) void k_sc1(Args a) {
    int bx = blockIdx.x, by = blockIdx.y;
    if (SNAKE && a.flip) {
        bx = gridDim.x - 1 - bx;
        by = gridDim.y - 1 - by;
    }
    const int i0 = by * RB;
    const int nrow = a.rows - i0 < RB ? a.rows - i0 : RB;
    double *blk = a.T + (size_t)i0 * a.ld;
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(blk, 0, (int)(nrow * a.ld * 8), 0x00020000);
    const int j = (bx * 256 + threadIdx.x) * 2;
    if (j >= a.N) return;
    const d2 pr = *reinterpret_cast<const d2 *>(a.prow + j);
    if (nrow == RB && j + 2 <= a.N) {
        d2 x[RB];
#pragma unroll
        for (int k = 0; k < RB; ++k) x[k] = *reinterpret_cast<const d2 *>(blk + (size_t)k * a.ld + j);
#pragma unroll
        for (int k = 0; k < RB; ++k) {
            const double f = a.f[i0 + k];
            d2 y;
            if (i0 + k == a.r) {
                y.x = pr.x / a.p;
                y.y = pr.y / a.p;
            } else {
                y.x = fma(f, pr.x, x[k].x);
                y.y = fma(f, pr.y, x[k].y);
            }
            u4 v = __builtin_bit_cast(u4, y);
            __builtin_amdgcn_raw_buffer_store_b128(v, rs, (int)(((size_t)k * a.ld + j) * 8), 0, AUX);
        }
    } else {
        for (int k = 0; k < nrow; ++k)
            for (int jj = j; jj < j + 2 && jj < a.N; ++jj) {
                double *x = blk + (size_t)k * a.ld + jj;
                *x = (i0 + k == a.r) ? a.prow[jj] / a.p : fma(a.f[i0 + k], a.prow[jj], *x);
            }
    }
}

template <int RB, bool SNAKE, int AUX>
void launch_sc1(Args a, hipStream_t s) {
    dim3 grid((a.N + 511) / 512, (a.rows + RB - 1) / RB);
    k_sc1<RB, SNAKE, AUX><<<grid, 256, 0, s>>>(a);
}

__global__ void k_tiny(const double *T, double *out) {
    if (threadIdx.x == 0) out[blockIdx.x] = T[blockIdx.x];
}
double *g_tiny_out;
template <void (*L)(Args, hipStream_t)>
void launch_pair(Args a, hipStream_t s) {
    k_tiny<<<4, 64, 0, s>>>(a.T, g_tiny_out);
    L(a, s);
}

struct Variant {
    const char *name;
    void (*launch)(Args, hipStream_t);
};

template <int RB, int CPT, bool NT, bool SNAKE, bool NTS = false, int TPB = 256>
void launch_var(Args a, hipStream_t s) {
    const int cols = TPB * 2 * CPT;
    dim3 grid((a.N + cols - 1) / cols, (a.rows + RB - 1) / RB);
    k_var<RB, CPT, NT, SNAKE, NTS, TPB><<<grid, TPB, 0, s>>>(a);
}

template <int RB, bool SNAKE, int BPC>
void launch_persist(Args a, hipStream_t s) {
    const int tx = (a.N + 511) / 512, ty = (a.rows + RB - 1) / RB;
    k_persist<RB, SNAKE><<<256 * BPC, 256, 0, s>>>(a, tx, ty);
}

int main(int argc, char **argv) {
    const int m = argc > 1 ? atoi(argv[1]) : 4096;
    const int N = argc > 2 ? atoi(argv[2]) : 16385;
    const int iters = argc > 3 ? atoi(argv[3]) : 40;
    const size_t ld = (N + 15) / 16 * 16;
    const double bytes = 16.0 * m * (double)N;
    std::vector<double> hT((size_t)m * ld), hp(ld), hf(m);
    srand(1);
    for (auto &x : hT) x = (rand() % 10000) / 100.0 + 1.0;
    for (auto &x : hp) x = (rand() % 10000) / 100.0 + 1.0;
    for (auto &x : hf) x = -((rand() % 1000) + 1) * 1e-7;
    double *T, *T0, *prow, *f;
    CHECK(hipMalloc(&T, sizeof(double) * m * ld));
    CHECK(hipMalloc(&T0, sizeof(double) * m * ld));
    CHECK(hipMalloc(&prow, sizeof(double) * ld));
    CHECK(hipMalloc(&f, sizeof(double) * m));
    CHECK(hipMemcpy(T0, hT.data(), sizeof(double) * m * ld, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(prow, hp.data(), sizeof(double) * ld, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(f, hf.data(), sizeof(double) * m, hipMemcpyHostToDevice));
    hipStream_t s;
    CHECK(hipStreamCreate(&s));
    CHECK(hipMalloc(&g_tiny_out, 64 * sizeof(double)));
    Args a{T, m, ld, N, prow, f, m / 3, 37.5, 0};
    Variant vs[] = {
        {"rb2_c1", launch_var<2, 1, false, false>},
        {"rb1_c1", launch_var<1, 1, false, false>},
        {"rb4_c1", launch_var<4, 1, false, false>},
        {"rb1_c1_snake", launch_var<1, 1, false, true>},
        {"rb2_c1_snake", launch_var<2, 1, false, true>},
        {"rb4_c1_snake", launch_var<4, 1, false, true>},
        {"rb8_c1_snake", launch_var<8, 1, false, true>},
        {"rb2_c1_t128_snake", launch_var<2, 1, false, true, false, 128>},
        {"rb2_c1_nts_snake", launch_var<2, 1, false, true, true>},
        {"buf_rb1_snake_sc1", launch_sc1<1, true, 16>},
        {"buf_rb2_snake_sc1", launch_sc1<2, true, 16>},
        {"buf_rb4_snake_sc1", launch_sc1<4, true, 16>},
        {"buf_rb1_sc1", launch_sc1<1, false, 16>},
        {"buf_rb2_sc1", launch_sc1<2, false, 16>},
    };
    const int nv = sizeof(vs) / sizeof(vs[0]);
    std::vector<double> ref((size_t)m * ld), out((size_t)m * ld);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    printf("m=%d N=%d ld=%zu bytes/launch=%.3f GB iters=%d\n", m, N, ld, bytes / 1e9, iters);
    for (int round = 0; round < 2; ++round) {
        for (int v = 0; v < nv; ++v) {
            // correctness: one launch from T0
            CHECK(hipMemcpy(T, T0, sizeof(double) * m * ld, hipMemcpyDeviceToDevice));
            a.flip = 0;
            vs[v].launch(a, s);
            CHECK(hipStreamSynchronize(s));
            CHECK(hipMemcpy(v == 0 ? ref.data() : out.data(), T, sizeof(double) * m * ld, hipMemcpyDeviceToHost));
            bool ok = true;
            if (v > 0) ok = memcmp(ref.data(), out.data(), sizeof(double) * m * ld) == 0;
            // timing
            for (int w = 0; w < 3; ++w) {
                a.flip = w & 1;
                vs[v].launch(a, s);
            }
            CHECK(hipEventRecord(e0, s));
            for (int it = 0; it < iters; ++it) {
                a.flip = it & 1;
                vs[v].launch(a, s);
            }
            CHECK(hipEventRecord(e1, s));
            CHECK(hipEventSynchronize(e1));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            const double us = ms * 1e3 / iters;
            if (round == 1)
                printf("%-20s %8.1f us  %7.1f GB/s  %5.1f%% of 8 TB/s  %s\n", vs[v].name, us, bytes / us / 1e3,
                       bytes / us / 1e3 / 80.0, ok ? "bit-exact" : "MISMATCH");
        }
    }
    return 0;
}
