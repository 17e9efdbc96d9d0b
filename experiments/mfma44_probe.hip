// mfma44_probe.hip -- v_mfma_f64_4x4x4f64 (4 blocks): operand layout and arithmetic (diagnostic).
//
// The 64-slot sweep needs D = A B + C with every element the slot-ordered chain of fused
// multiply-adds, fma(a3, b3, fma(a2, b2, fma(a1, b1, fma(a0, b0, c)))) -- the reference's
// per-element operations (solver.cu:34-46).  experiments/mfma_f64_probe.hip showed it for
// v_mfma_f64_16x16x4f64; this probe checks it for the 4x4x4 (4-block) form -- 62-72 TFLOP/s on
// MI355X against 43-48 for 16x16x4 (experiments/valu_sweep_probe.hip) -- with the lane layout below,
// bit for bit on random operands and on edge-value pools (signed zeros, subnormals, overflow, inf,
// NaN), at 1 and 16 chained steps.
//   build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off experiments/mfma44_probe.hip -o tools/_ab/mfma44_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#define CK(x)                                                           \
    do {                                                                \
        hipError_t e_ = (x);                                            \
        if (e_ != hipSuccess) {                                         \
            printf("%s at line %d\n", hipGetErrorString(e_), __LINE__); \
            exit(1);                                                    \
        }                                                               \
    } while (0)

// steps chained MFMAs: lane l, step t uses A[t*64 + l], B[t*64 + l]; C is the lane's start value
__global__ void k_mfma44(const double *A, const double *B, const double *C, double *D, int steps) {
    const int l = threadIdx.x;
    double d = C[l];
    for (int t = 0; t < steps; ++t) d = __builtin_amdgcn_mfma_f64_4x4x4f64(A[t * 64 + l], B[t * 64 + l], d, 0, 0, 0);
    D[l] = d;
}

// The operand layout of the 4-block form, found on MI355X by one-hot operands
// (profiles/r05_mfma44_layout.txt): block a = (lane >> 2) & 3,
//   A[a][i][k] at lane 16k + 4a + i,   B[a][k][j] at lane 16k + 4a + j,   D[a][i][j] at lane 16i + 4a + j
// -- with A the same in every block, one instruction is a 4-row x 16-column tile over 4 slots:
// row i = lane >> 4 (D) / lane & 3 (A), column 4a + j = lane & 15 (B and D), slot k = lane >> 4 (A, B).
static bool same_bits(double a, double b) { return std::memcmp(&a, &b, 8) == 0; }

// reference: element (i, j) of block a = chain over steps t and k of fma(A_t[a][i][k], B_t[a][k][j], .)
static void reference(const std::vector<double> &A, const std::vector<double> &B, const std::vector<double> &C,
                      std::vector<double> &D, int steps) {
    for (int l = 0; l < 64; ++l) {
        const int i = l >> 4, a = (l >> 2) & 3, j = l & 3;
        double x = C[l];
        for (int t = 0; t < steps; ++t)
            for (int k = 0; k < 4; ++k) x = std::fma(A[t * 64 + 16 * k + 4 * a + i], B[t * 64 + 16 * k + 4 * a + j], x);
        D[l] = x;
    }
}

static void run(const std::vector<double> &A, const std::vector<double> &B, const std::vector<double> &C,
                std::vector<double> &D, int steps) {
    double *dA, *dB, *dC, *dD;
    CK(hipMalloc(&dA, A.size() * 8));
    CK(hipMalloc(&dB, B.size() * 8));
    CK(hipMalloc(&dC, 64 * 8));
    CK(hipMalloc(&dD, 64 * 8));
    CK(hipMemcpy(dA, A.data(), A.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, B.data(), B.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dC, C.data(), 64 * 8, hipMemcpyHostToDevice));
    k_mfma44<<<1, 64>>>(dA, dB, dC, dD, steps);
    CK(hipDeviceSynchronize());
    D.resize(64);
    CK(hipMemcpy(D.data(), dD, 64 * 8, hipMemcpyDeviceToHost));
    CK(hipFree(dA));
    CK(hipFree(dB));
    CK(hipFree(dC));
    CK(hipFree(dD));
}

static double pool_value(std::mt19937_64 &g, int pool) {
    std::uniform_real_distribution<double> u(-1.0, 1.0);
    const double x = u(g);
    switch (pool) {
        case 0: return x * 100.0;                                      // plain
        case 1: { const int k = (int)(g() % 6); return k == 0 ? 0.0 : k == 1 ? -0.0 : x; }  // signed zeros
        case 2: return x * 1e-310;                                     // subnormal operands
        case 3: return x * ((g() & 1) ? 1e-160 : 1e-150);              // products in the subnormal range
        case 4: return x * 1e300;                                      // overflow to +-inf
        case 5: { const int k = (int)(g() % 8); return k == 0 ? INFINITY : k == 1 ? -INFINITY : x; }
        case 6: { const int k = (int)(g() % 8);
                  if (k == 0) { uint64_t b = 0x7ff8000000000000ull | (g() & 0xfffffffffull); double q; std::memcpy(&q, &b, 8); return q; }
                  return x; }                                          // NaN payloads
        default: { const int k = (int)(g() % 5); return k == 0 ? x * 1e-300 : k == 1 ? -0.0 : k == 2 ? x * 1e-310 : x; }
    }
}

int main() {
    std::mt19937_64 g(12345);
    std::uniform_real_distribution<double> u(-1.0, 1.0);
    // 1. one step, random operands
    std::vector<double> A(64), B(64), C(64), D, R(64);
    for (int l = 0; l < 64; ++l) { A[l] = u(g); B[l] = u(g); C[l] = u(g); }
    run(A, B, C, D, 1);
    reference(A, B, C, R, 1);
    int ok = 0;
    for (int l = 0; l < 64; ++l) ok += same_bits(R[l], D[l]);
    printf("layout (A 16k+4a+i, B 16k+4a+j, D 16i+4a+j), one step: %d of 64 equal\n", ok);
    // 2. bit-exactness on pools, 1 and 16 steps
    long long total = 0, bad = 0, nan_payload = 0;
    for (int pool = 0; pool < 8; ++pool)
        for (int steps : {1, 16})
            for (int trial = 0; trial < 200; ++trial) {
                std::vector<double> a((size_t)steps * 64), b((size_t)steps * 64), c(64), d, r(64);
                for (auto &x : a) x = pool_value(g, pool);
                for (auto &x : b) x = pool_value(g, pool);
                for (auto &x : c) x = pool_value(g, pool);
                run(a, b, c, d, steps);
                reference(a, b, c, r, steps);
                for (int l = 0; l < 64; ++l) {
                    ++total;
                    if (!same_bits(r[l], d[l])) {
                        if (std::isnan(r[l]) && std::isnan(d[l])) {  // both NaN: only the payload differs
                            uint64_t gb, wb;
                            std::memcpy(&gb, &d[l], 8);
                            std::memcpy(&wb, &r[l], 8);
                            if (nan_payload < 3) printf("pool %d steps %d lane %d: NaN payload %016llx want %016llx\n", pool,
                                                        steps, l, (unsigned long long)gb, (unsigned long long)wb);
                            ++nan_payload;
                            continue;
                        }
                        if (bad < 5) printf("pool %d steps %d lane %d: got %a want %a\n", pool, steps, l, d[l], r[l]);
                        ++bad;
                    }
                }
            }
    printf("%lld elements, %lld differ from the sequential fma chain%s; %lld NaN results with another payload\n",
           total, bad, bad ? "" : " (every non-NaN result BIT-EXACT, NaN exactly where the chain gives NaN)", nan_payload);
    return bad ? 1 : 0;
}
