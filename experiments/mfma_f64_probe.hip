// mfma_f64_probe.hip -- does v_mfma_f64_16x16x4f64 (D = A B + C) give, for every element, the
// bits of the sequential fused chain c = fma(a_k, b_k, c) for k = 0, 1, 2, 3 (the reference's
// per-pivot update order, solver.cu:34-46, applied 4 pivots at a time)?  If it does, a batch
// sweep can run on the matrix cores bit for bit.  Diagnostic only.
//   build: hipcc --offload-arch=gfx950 -O2 -ffp-contract=off experiments/mfma_f64_probe.hip -o tools/_ab/mfma_f64_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

typedef double double4_t __attribute__((ext_vector_type(4)));

// operand layout (checked below against a plain product; a first run with C/D row 4 (l / 16) + v
// matched only the 64 elements where the two formulas agree):
//   A 16x4: lane l holds A[l % 16][l / 16];  B 4x16: lane l holds B[l / 16][l % 16];
//   C/D 16x16: lane l, register v holds [l / 16 + 4 v][l % 16]
__global__ void k_mfma(const double *A, const double *B, const double *C, double *D, int reps) {
    const int l = threadIdx.x;
    const double a = A[(l % 16) * 4 + l / 16];
    const double b = B[(l / 16) * 16 + l % 16];
    double4_t c;
    for (int v = 0; v < 4; ++v) c[v] = C[(l / 16 + 4 * v) * 16 + l % 16];
    for (int r = 0; r < reps; ++r) c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    for (int v = 0; v < 4; ++v) D[(l / 16 + 4 * v) * 16 + l % 16] = c[v];
}

// the sequential chain in the order k = 0..3 (order 0) or 3..0 (order 1)
__global__ void k_chain(const double *A, const double *B, const double *C, double *D, int reps, int order) {
    const int t = threadIdx.x + blockIdx.x * blockDim.x;
    if (t >= 256) return;
    const int i = t / 16, j = t % 16;
    double c = C[t];
    for (int r = 0; r < reps; ++r)
        for (int kk = 0; kk < 4; ++kk) {
            const int k = order ? 3 - kk : kk;
            c = fma(A[i * 4 + k], B[k * 16 + j], c);
        }
    D[t] = c;
}

int main() {
    std::mt19937_64 g(12345);
    std::uniform_real_distribution<double> u(-1.0, 1.0), big(1.0, 100.0);
    int worst_bad = 0;
    for (int trial = 0; trial < 6; ++trial) {
        std::vector<double> A(64), B(64), C(256), D(256), S0(256), S1(256);
        for (auto &x : A) x = trial % 2 ? -u(g) / big(g) : u(g);           // factors -(a/p)
        for (auto &x : B) x = trial % 3 ? big(g) : u(g) * 1e-3;            // pivot-row values
        for (auto &x : C) x = trial % 2 ? big(g) : u(g) * std::ldexp(1.0, (int)(u(g) * 40));
        double *dA, *dB, *dC, *dD;
        hipMalloc(&dA, 64 * 8);
        hipMalloc(&dB, 64 * 8);
        hipMalloc(&dC, 256 * 8);
        hipMalloc(&dD, 256 * 8);
        hipMemcpy(dA, A.data(), 64 * 8, hipMemcpyHostToDevice);
        hipMemcpy(dB, B.data(), 64 * 8, hipMemcpyHostToDevice);
        hipMemcpy(dC, C.data(), 256 * 8, hipMemcpyHostToDevice);
        for (int reps : {1, 8}) {
            k_mfma<<<1, 64>>>(dA, dB, dC, dD, reps);
            hipMemcpy(D.data(), dD, 256 * 8, hipMemcpyDeviceToHost);
            k_chain<<<1, 256>>>(dA, dB, dC, dD, reps, 0);
            hipMemcpy(S0.data(), dD, 256 * 8, hipMemcpyDeviceToHost);
            k_chain<<<1, 256>>>(dA, dB, dC, dD, reps, 1);
            hipMemcpy(S1.data(), dD, 256 * 8, hipMemcpyDeviceToHost);
            int same0 = 0, same1 = 0, close = 0;
            double maxrel = 0;
            for (int t = 0; t < 256; ++t) {
                same0 += D[t] == S0[t];
                same1 += D[t] == S1[t];
                const double rel = std::fabs(D[t] - S0[t]) / std::fmax(std::fabs(S0[t]), 1e-300);
                close += rel < 1e-12;
                maxrel = std::fmax(maxrel, rel);
            }
            printf("trial %d reps %d: layout %s (%d/256 within 1e-12, max rel %.3g); bit-equal to fma chain k=0..3: "
                   "%d/256, k=3..0: %d/256\n",
                   trial, reps, close == 256 ? "ok" : "WRONG", close, maxrel, same0, same1);
            worst_bad += 256 - same0;
        }
        hipFree(dA);
        hipFree(dB);
        hipFree(dC);
        hipFree(dD);
    }
    printf("MFMA_F64 %s\n", worst_bad == 0 ? "BIT-EXACT vs sequential fma chain" : "DIFFERS from sequential fma chain");
    return 0;
}
