// f64_rate_probe.hip -- the fp64 arithmetic ceilings the 64-slot sweep runs against (diagnostic).
//   M  v_mfma_f64_16x16x4f64 only: 4 independent accumulators per wave
//   V  v_fma_f64 only: 8 independent chains per lane
//   MV both in one wave: per step 4 MFMAs and NV vector fmas (the matrix and vector pipes in parallel?)
// Every form runs on all CUs with WPS waves per SIMD; rates in TFLOP/s (MFMA 2048 flops, fma 2).
//   build: hipcc --offload-arch=gfx950 -O3 experiments/f64_rate_probe.hip -o tools/_ab/f64_rate_probe
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

template <int NM, int NV>
__global__ __launch_bounds__(256) void k_rate(double *out, int iters, double a, double b) {
    const int l = threadIdx.x;
    d4 acc[NM > 0 ? NM : 1];
    double v[NV > 0 ? NV : 1];
#pragma unroll
    for (int k = 0; k < (NM > 0 ? NM : 1); ++k) acc[k] = d4{(double)l, 1.0 * k, 2.0, 3.0};
#pragma unroll
    for (int k = 0; k < (NV > 0 ? NV : 1); ++k) v[k] = (double)(l + k);
    const double fa = a + l * 1e-9, fb = b - l * 1e-9;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int k = 0; k < NM; ++k) acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa, fb, acc[k], 0, 0, 0);
#pragma unroll
        for (int k = 0; k < NV; ++k) v[k] = fma(v[k], fa, fb);
    }
    double s = 0;
#pragma unroll
    for (int k = 0; k < NM; ++k) s += acc[k][0] + acc[k][1] + acc[k][2] + acc[k][3];
#pragma unroll
    for (int k = 0; k < NV; ++k) s += v[k];
    out[blockIdx.x * 256 + l] = s;
}

template <int NM, int NV>
void run(const char *name, int wps) {
    int cus = 0, dev = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const int blocks = cus * wps, iters = NM > 0 ? 20000 : 100000;
    double *out;
    CK(hipMalloc(&out, (size_t)blocks * 256 * 8));
    k_rate<NM, NV><<<blocks, 256>>>(out, 100, 0.999, 1e-3);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0));
    k_rate<NM, NV><<<blocks, 256>>>(out, iters, 0.999, 1e-3);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double waves = blocks * 4.0;
    const double fm = waves * iters * NM * 2048.0, fv = waves * iters * NV * 64 * 2.0;
    printf("%-28s waves/SIMD %d: %8.3f ms  matrix %6.1f TFLOP/s  vector %6.1f TFLOP/s  total %6.1f\n", name, wps, ms,
           fm / ms / 1e9, fv / ms / 1e9, (fm + fv) / ms / 1e9);
    CK(hipFree(out));
}

int main() {
    for (int wps = 1; wps <= 4; wps *= 2) {
        run<4, 0>("M  4 accumulators", wps);
        run<8, 0>("M  8 accumulators", wps);
        run<0, 8>("V  8 chains", wps);
        run<0, 16>("V  16 chains", wps);
        run<4, 16>("MV 4 mfma + 16 fma", wps);
        run<4, 32>("MV 4 mfma + 32 fma", wps);
        run<4, 64>("MV 4 mfma + 64 fma", wps);
    }
    return 0;
}
