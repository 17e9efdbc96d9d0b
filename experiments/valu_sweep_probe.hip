// valu_sweep_probe.hip -- can the vector units beat the matrix cores on the 64-slot sweep? (diagnostic)
//
// The sweep applies q <= 64 pending pivots to every element: x = fma(F[i][s], U[s][j], x), s in
// order (solver.cu:34-46).  k_msweep runs it on v_mfma_f64_16x16x4f64 (47.6 TFLOP/s measured ceiling,
// profiles/r03_f64_rate_probe.txt).  Here each lane owns one column and R rows of a strip: the
// row factors F[i][s] are wave-uniform -- scalar loads, SGPR operands of v_fma_f64 -- and the lane's
// U[s][j] stay in VGPRs for the whole sweep, so no cross-lane operand traffic at all.  Also the
// rate of v_mfma_f64_4x4x4f64 (4 blocks) next to 16x16x4.
//   build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off experiments/valu_sweep_probe.hip -o /tmp/vsp
#include <hip/hip_runtime.h>

#include <cmath>
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

#define KMAX 64
__host__ __device__ constexpr size_t fidx(long long i, int s) {
    return (size_t)(i >> 4) * (16 * KMAX) + (size_t)s * 16 + (size_t)(i & 15);
}

// R rows per strip (16 or 32), one column per lane, 64 columns per wave, 4 waves per block
template <int R, int K>
__global__ __launch_bounds__(256, 2) void k_vsweep(double *__restrict__ T, int rows, int cols, size_t ld,
                                                   const double *__restrict__ F, const double *__restrict__ U,
                                                   int G) {
    const int cb = (cols + 255) / 256;
    const int lin = blockIdx.x;
    const int tile = lin % cb, gy = lin / cb;
    if (gy >= G) return;
    const int c = tile * 256 + (int)threadIdx.x;
    const bool live = c < cols;
    double u[K];
#pragma unroll
    for (int s = 0; s < K; ++s) u[s] = live ? U[(size_t)s * ld + c] : 0.0;
    const int nstrip = (rows + R - 1) / R;
    for (int g = gy; g < nstrip; g += G) {
        const int r0 = g * R;
        double x[R];
#pragma unroll
        for (int k = 0; k < R; ++k) x[k] = live ? __builtin_nontemporal_load(T + (size_t)(r0 + k) * ld + c) : 0.0;
        const double *Fs = F + fidx(r0, 0);
#pragma unroll
        for (int s = 0; s < K; ++s) {
#pragma unroll
            for (int k = 0; k < R; ++k) {
                const double f = Fs[(size_t)(k >> 4) * (16 * KMAX) + 16 * s + (k & 15)];  // wave-uniform
                x[k] = fma(f, u[s], x[k]);
            }
        }
#pragma unroll
        for (int k = 0; k < R; ++k)
            if (live) T[(size_t)(r0 + k) * ld + c] = x[k];
    }
}

typedef double d4 __attribute__((ext_vector_type(4)));
template <int NM>
__global__ __launch_bounds__(256) void k_rate44(double *out, int iters, double a, double b) {
    const int l = threadIdx.x;
    double acc[NM];
#pragma unroll
    for (int k = 0; k < NM; ++k) acc[k] = (double)(l + k);
    const double fa = a + l * 1e-9, fb = b - l * 1e-9;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int k = 0; k < NM; ++k) acc[k] = __builtin_amdgcn_mfma_f64_4x4x4f64(fa, fb, acc[k], 0, 0, 0);
    }
    double s = 0;
#pragma unroll
    for (int k = 0; k < NM; ++k) s += acc[k];
    out[blockIdx.x * 256 + l] = s;
}
template <int NM>
__global__ __launch_bounds__(256) void k_rate16(double *out, int iters, double a, double b) {
    const int l = threadIdx.x;
    d4 acc[NM];
#pragma unroll
    for (int k = 0; k < NM; ++k) acc[k] = d4{(double)l, 1.0 * k, 2.0, 3.0};
    const double fa = a + l * 1e-9, fb = b - l * 1e-9;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int k = 0; k < NM; ++k) acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa, fb, acc[k], 0, 0, 0);
    }
    double s = 0;
#pragma unroll
    for (int k = 0; k < NM; ++k) s += acc[k][0] + acc[k][1] + acc[k][2] + acc[k][3];
    out[blockIdx.x * 256 + l] = s;
}

static float time_it(void (*launch)(void *), void *arg, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    launch(arg);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) launch(arg);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
}

struct SweepArg {
    double *T;
    int rows, cols;
    size_t ld;
    double *F, *U;
    int G, R;
};

template <int R>
static void launch_v(void *p) {
    SweepArg *a = (SweepArg *)p;
    const int cb = (a->cols + 255) / 256;
    k_vsweep<R, KMAX><<<cb * a->G, 256>>>(a->T, a->rows, a->cols, a->ld, a->F, a->U, a->G);
}

static void sweep_case(int rows, int cols, int R, float waves) {
    const size_t ld = ((size_t)cols + 15) / 16 * 16;
    double *T, *F, *U;
    CK(hipMalloc(&T, (size_t)rows * ld * 8));
    CK(hipMalloc(&F, ((size_t)rows + 32) * KMAX * 8));
    CK(hipMalloc(&U, (size_t)KMAX * ld * 8));
    std::vector<double> h((size_t)rows * ld);
    for (size_t i = 0; i < h.size(); ++i) h[i] = 1.0 + (double)(i % 97);
    CK(hipMemcpy(T, h.data(), h.size() * 8, hipMemcpyHostToDevice));
    std::vector<double> hf(((size_t)rows + 32) * KMAX), hu((size_t)KMAX * ld);
    for (size_t i = 0; i < hf.size(); ++i) hf[i] = -1e-3 * (double)(i % 13);
    for (size_t i = 0; i < hu.size(); ++i) hu[i] = 1.0 + (double)(i % 7);
    CK(hipMemcpy(F, hf.data(), hf.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(U, hu.data(), hu.size() * 8, hipMemcpyHostToDevice));
    int cus = 0, dev = 0, per_cu = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    if (R == 16)
        CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_vsweep<16, KMAX>, 256, 0));
    else
        CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_vsweep<32, KMAX>, 256, 0));
    const int cb = (cols + 255) / 256;
    int G = (int)(waves * per_cu * cus / cb);
    const int nstrip = (rows + R - 1) / R;
    if (G > nstrip) G = nstrip;
    if (G < 1) G = 1;
    SweepArg a{T, rows, cols, ld, F, U, G, R};
    // correctness of the chain on one element (row 5, column 3) after one sweep
    CK(hipMemcpy(T, h.data(), h.size() * 8, hipMemcpyHostToDevice));
    if (R == 16) launch_v<16>(&a); else launch_v<32>(&a);
    CK(hipDeviceSynchronize());
    double got = 0;
    CK(hipMemcpy(&got, T + 5 * ld + 3, 8, hipMemcpyDeviceToHost));
    double want = h[5 * ld + 3];
    for (int s = 0; s < KMAX; ++s) want = std::fma(hf[fidx(5, s)], hu[(size_t)s * ld + 3], want);
    const float ms = time_it(R == 16 ? launch_v<16> : launch_v<32>, &a, 10);
    const double bytes = 16.0 * rows * cols, flops = 2.0 * KMAX * rows * cols;
    printf("VALU sweep %5d x %5d  R=%d waves %.2f (G %d, %d blocks/CU): %8.1f us  %.3f of 8 TB/s  %5.1f TFLOP/s  %.2f us/pivot  %s\n",
           rows, cols, R, waves, G, per_cu, ms * 1e3, bytes / (ms * 1e-3) / 8e12, flops / (ms * 1e-3) / 1e12,
           ms * 1e3 / KMAX, got == want ? "bit-exact" : "MISMATCH");
    CK(hipFree(T));
    CK(hipFree(F));
    CK(hipFree(U));
}

template <int NM>
static void rate44(int wps) {
    int cus = 0, dev = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const int blocks = cus * wps, iters = 20000;
    double *out;
    CK(hipMalloc(&out, (size_t)blocks * 256 * 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float ms44 = 0, ms16 = 0;
    k_rate44<NM><<<blocks, 256>>>(out, 100, 0.999, 1e-3);
    CK(hipEventRecord(e0));
    k_rate44<NM><<<blocks, 256>>>(out, iters, 0.999, 1e-3);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms44, e0, e1));
    k_rate16<NM><<<blocks, 256>>>(out, 100, 0.999, 1e-3);
    CK(hipEventRecord(e0));
    k_rate16<NM><<<blocks, 256>>>(out, iters, 0.999, 1e-3);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms16, e0, e1));
    const double waves = blocks * 4.0;
    // 4x4x4 (4 blocks): 4 * 4*4*4 = 256 MACs per instruction; 16x16x4: 1024
    printf("MFMA f64 %d acc/wave, %d waves/SIMD: 4x4x4_4b %6.1f TFLOP/s   16x16x4 %6.1f TFLOP/s\n", NM, wps,
           waves * iters * NM * 512.0 / ms44 / 1e9, waves * iters * NM * 2048.0 / ms16 / 1e9);
    CK(hipFree(out));
}

int main() {
    rate44<4>(2);
    rate44<8>(2);
    rate44<8>(4);
    for (float w : {1.0f, 2.0f}) {
        sweep_case(4096, 8192, 16, w);
        sweep_case(32768, 9216, 16, w);
        sweep_case(4096, 8192, 32, w);
        sweep_case(32768, 9216, 32, w);
    }
    return 0;
}
