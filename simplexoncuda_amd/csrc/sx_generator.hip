// sx_generator.hip -- device-side synthesis of generateRandomProblem's instances
// (reference generator.cu:9-77, problem.cu:49-126).
//
// The reference draws A(i, j) = U(XORWOW(seed_A) draw #(i*n + j)) with one CUDA thread per
// constraint (curand_init(seed, 0, i*n) = jump i*n draws ahead).  Here every thread owns a
// chunk of consecutive draws of one constraint row and jumps straight to its first draw:
// the XORWOW v-state recurrence is linear over GF(2), so k steps are the 160x160 bit matrix
// M^k applied to the state, composed from precomputed M^(2^b); the Weyl counter d advances
// by 362437*k.  Values are written straight into the shard's tableau rows (row-major,
// column 1+j) -- or into the reference's column-major A for problem_t -- and are
// bit-identical to the host generator (uniform = fmaf((float)x, 2^-32, 2^-33), value =
// fma(u, max-min, min)).
#include <cstring>
#include <mutex>
#include <vector>

#include "sx_common.hpp"

namespace {

constexpr int kWords = 5;     // 160-bit v-state
constexpr int kBits = 160;
constexpr int kJumps = 48;    // M^(2^b), b < 48: offsets below 2^48

// host: one XORWOW step on the v-state (curand(): t = v0^(v0>>2); shift; v4 = ...)
void step_v(const uint32_t in[kWords], uint32_t out[kWords]) {
    const uint32_t t = in[0] ^ (in[0] >> 2);
    out[0] = in[1];
    out[1] = in[2];
    out[2] = in[3];
    out[3] = in[4];
    out[4] = (in[4] ^ (in[4] << 4)) ^ (t ^ (t << 1));
}

// bit matrix as 160 columns of 160 bits: y = M x = XOR of columns j with x_j = 1
struct BitMat {
    uint32_t col[kBits][kWords];
};

void matmul(const BitMat &A, const BitMat &B, BitMat &C) {  // C = A * B
    for (int j = 0; j < kBits; ++j) {
        uint32_t acc[kWords] = {0, 0, 0, 0, 0};
        for (int k = 0; k < kBits; ++k)
            if ((B.col[j][k >> 5] >> (k & 31)) & 1u)
                for (int w = 0; w < kWords; ++w) acc[w] ^= A.col[k][w];
        std::memcpy(C.col[j], acc, sizeof(acc));
    }
}

std::once_flag g_jump_once;
uint32_t *g_jump_dev = nullptr;  // kJumps matrices, column-major words

void build_jumps() {
    std::vector<BitMat> J(kJumps);
    for (int j = 0; j < kBits; ++j) {
        uint32_t e[kWords] = {0, 0, 0, 0, 0};
        e[j >> 5] = 1u << (j & 31);
        step_v(e, J[0].col[j]);
    }
    for (int b = 1; b < kJumps; ++b) matmul(J[b - 1], J[b - 1], J[b]);
    SX_HIP(hipMalloc(reinterpret_cast<void **>(&g_jump_dev), sizeof(BitMat) * kJumps));
    SX_HIP(hipMemcpy(g_jump_dev, J.data(), sizeof(BitMat) * kJumps, hipMemcpyHostToDevice));
}

struct Xw {
    uint32_t d, v[kWords];
};

__device__ __forceinline__ void xw_init(Xw &s, uint64_t seed) {  // curand_init(seed, 0, 0)
    const uint32_t s0 = ((uint32_t)seed) ^ 0xaad26b49u;
    const uint32_t s1 = ((uint32_t)(seed >> 32)) ^ 0xf7dcefddu;
    const uint32_t t0 = 1099087573u * s0;
    const uint32_t t1 = 2591861531u * s1;
    s.d = 6615241u + t1 + t0;
    s.v[0] = 123456789u + t0;
    s.v[1] = 362436069u ^ t0;
    s.v[2] = 521288629u + t1;
    s.v[3] = 88675123u ^ t1;
    s.v[4] = 5783321u + t0;
}

__device__ __forceinline__ uint32_t xw_next(Xw &s) {
    const uint32_t t = s.v[0] ^ (s.v[0] >> 2);
    s.v[0] = s.v[1];
    s.v[1] = s.v[2];
    s.v[2] = s.v[3];
    s.v[3] = s.v[4];
    s.v[4] = (s.v[4] ^ (s.v[4] << 4)) ^ (t ^ (t << 1));
    s.d += 362437u;
    return s.v[4] + s.d;
}

// skip k draws: v <- M^k v (one matrix per set bit of k), d += 362437 k
__device__ void xw_skip(Xw &s, uint64_t k, const uint32_t *__restrict__ jumps) {
    s.d += (uint32_t)(362437ull * k);
    for (int b = 0; k; ++b, k >>= 1) {
        if (!(k & 1)) continue;
        const uint32_t *M = jumps + (size_t)b * kBits * kWords;
        uint32_t y[kWords] = {0, 0, 0, 0, 0};
#pragma unroll 4
        for (int j = 0; j < kBits; ++j) {
            const uint32_t mask = 0u - ((s.v[j >> 5] >> (j & 31)) & 1u);
#pragma unroll
            for (int w = 0; w < kWords; ++w) y[w] ^= M[j * kWords + w] & mask;
        }
#pragma unroll
        for (int w = 0; w < kWords; ++w) s.v[w] = y[w];
    }
}

__device__ __forceinline__ double value_of(uint32_t x, double lo, double span) {
    const float u = __fmaf_rn((float)x, 2.3283064e-10f, 2.3283064e-10f / 2.0f);  // curand_uniform
    return __fma_rn((double)u, span, lo);                                      // generator.cu:18
}

// A for rows [row0, row0+rows) of an n-column problem: chunk c of row i covers columns
// [c*CH, c*CH+CH).  Output either the tableau (element (i, 1 + j) in the layout tl, region A) or
// column-major A_cm[j*m + row0+i].
template <int CH>
__global__ __launch_bounds__(256) void k_gen_A(uint32_t seed, int n, int m, int row0, int rows, double lo, double span,
                                               const uint32_t *__restrict__ jumps, double *T, TLay tl,
                                               double *A_cm) {
    const int chunks = (n + CH - 1) / CH;
    const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (tid >= (long long)rows * chunks) return;
    const int i = (int)(tid / chunks), c = (int)(tid % chunks);
    const int j0 = c * CH, j1 = min(n, j0 + CH);
    Xw s;
    xw_init(s, seed);
    xw_skip(s, (uint64_t)(row0 + i) * (uint64_t)n + (uint64_t)j0, jumps);
    if (T) {
        for (int j = j0; j < j1; ++j) T[tl.idx(i, 1 + j)] = value_of(xw_next(s), lo, span);
    } else {
        for (int j = j0; j < j1; ++j) A_cm[(size_t)j * m + row0 + i] = value_of(xw_next(s), lo, span);
    }
}

// draws #first .. #first+count-1 of one stream (b_i or c_j)
__global__ void k_gen_vec(uint32_t seed, long long first, int count, double lo, double span,
                          const uint32_t *__restrict__ jumps, double *out, int CH) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int i0 = t * CH;
    if (i0 >= count) return;
    Xw s;
    xw_init(s, seed);
    xw_skip(s, (uint64_t)(first + i0), jumps);
    const int i1 = min(count, i0 + CH);
    for (int i = i0; i < i1; ++i) out[i] = value_of(xw_next(s), lo, span);
}

}  // namespace

// problem.cu:63-67 with MSVC's rand(): seeds for b, c, A
void sx_crt_seeds(unsigned seed, int kind, uint32_t out[3]);

const uint32_t *sx_jump_tables() {
    std::call_once(g_jump_once, build_jumps);
    return g_jump_dev;
}

void sx_launch_gen_rows(uint32_t seedA, int n, int m, int row0, int rows, double lo, double hi, double *T, TLay tl,
                        double *A_cm, hipStream_t s) {
    if (rows <= 0 || n <= 0) return;
    constexpr int CH = 128;
    const long long threads = (long long)rows * ((n + CH - 1) / CH);
    const int blocks = (int)((threads + 255) / 256);
    k_gen_A<CH><<<blocks, 256, 0, s>>>(seedA, n, m, row0, rows, lo, hi - lo, sx_jump_tables(), T, tl, A_cm);
}

void sx_launch_gen_vector(uint32_t seed, long long first, int count, double lo, double hi, double *out,
                          hipStream_t s) {
    if (count <= 0) return;
    const int CH = 64;
    const int threads = (count + CH - 1) / CH;
    k_gen_vec<<<(threads + 255) / 256, 256, 0, s>>>(seed, first, count, lo, hi - lo, sx_jump_tables(), out, CH);
}
