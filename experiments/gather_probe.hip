// gather_probe.hip -- what one fused-batch pivot pays for its tableau reads, by layout (diagnostic).
//
// The fused batch (k_batch) reads, per pivot, the entering column of the tableau (one 8-byte
// element in each of the shard's rows, every ratio block its 512 rows) and the leaving row (one
// element per logical column, every objective block its 512 columns).  This probe times those two
// reads alone, round after round, each round a new random column (or row), with nothing else on
// the chip: every block loads its 512 elements, waits for them (one block barrier), and thread 0
// stamps s_memrealtime (100 MHz).  Layouts of a rows x ld fp64 matrix:
//   RM  row-major (the engine's): element (i, j) at i*ld + j
//   SM  16-row strips, column-contiguous inside a strip: (i/16)*16*ld + 16*j + i%16
//       (a column of 16 rows is one 128-byte line; a row's 16 consecutive columns are 16 lines)
//   CM  column-major: j*rows + i (a column of 512 rows is 4 KB contiguous)
//   B4  16-row strips of 4-column groups, each group 4 blocks of 4 rows x 4 columns (128 B):
//       (i/16)*16*ld + (j/4)*64 + ((i%16)/4)*16 + (i%4)*4 + j%4  (a 512-row column: 128 lines;
//       512 columns of a row: 128 lines)
//   B8  8 rows x 2 columns per 128-byte line: (i/16)*16*ld + (j/2)*32 + ((i%16)/8)*16 + (i%8)*2 + j%2
//   B2  2 rows x 8 columns per line: (i/16)*16*ld + (j/8)*128 + ((i%16)/2)*16 + (i%2)*8 + j%8
// With pollers > 0, that many extra blocks spin on 64 granule lines with sc1 loads and s_sleep(1)
// meanwhile (the fused batch's idle side polling the next records).
// Modes: G = column gather (block b: rows [512b, 512b+512), column c_k), R = row read (block b:
// columns [512b, 512b+512) of row r_k).
//   build: hipcc --offload-arch=gfx950 -O3 experiments/gather_probe.hip -o tools/_ab/gather_probe
//   run:   experiments/gather_probe [rows ld blocks_G blocks_R rounds]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
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

template <int LAY, int MODE>
__global__ __launch_bounds__(512) void k_probe(const double *__restrict__ T, int rows, long long ld, const int *idx,
                                               int R, unsigned long long *stamps, double *sink) {
    const int t = threadIdx.x;
    __shared__ int s_dep;
    if (t == 0) s_dep = 0;
    __syncthreads();
    double acc = 0.0;
    for (int k = 0; k < R; ++k) {
        const int x = idx[k] + s_dep;  // (s_dep stays 0; the compiler cannot hoist the load)
        long long i, j;
        if (MODE == 0) {
            i = (long long)blockIdx.x * 512 + t;
            j = x;
        } else {
            i = x;
            j = (long long)blockIdx.x * 512 + t;
        }
        size_t off;
        if (LAY == 0)
            off = (size_t)i * ld + j;
        else if (LAY == 1)
            off = (size_t)(i >> 4) * 16 * ld + (size_t)j * 16 + (size_t)(i & 15);
        else if (LAY == 2)
            off = (size_t)j * rows + i;
        else if (LAY == 3)
            off = (size_t)(i >> 4) * 16 * ld + (size_t)(j >> 2) * 64 + (size_t)((i & 15) >> 2) * 16 + (i & 3) * 4 + (j & 3);
        else if (LAY == 4)
            off = (size_t)(i >> 4) * 16 * ld + (size_t)(j >> 1) * 32 + (size_t)((i & 15) >> 3) * 16 + (i & 7) * 2 + (j & 1);
        else
            off = (size_t)(i >> 4) * 16 * ld + (size_t)(j >> 3) * 128 + (size_t)((i & 15) >> 1) * 16 + (i & 1) * 8 + (j & 7);
        const double v = T[off];
        acc += v;
        const int any = __syncthreads_or(v == 12345.0);  // every thread's load has landed
        if (t == 0) {
            stamps[(size_t)blockIdx.x * R + k] = __builtin_amdgcn_s_memrealtime();
            s_dep = any;
        }
        __syncthreads();
    }
    sink[(size_t)blockIdx.x * 512 + t] = acc;
}

// extra blocks polling 64 granule lines (never written) until *stop is set
__global__ void k_pollers(const unsigned long long *g, const unsigned *stop, unsigned long long *sink) {
    if (threadIdx.x >= 64) return;
    unsigned long long acc = 0;
    for (int it = 0; it < (1 << 22); ++it) {  // (bounded: ends within seconds even if the stop word is missed)
        const unsigned long long *p = g + (size_t)threadIdx.x * 16 + (size_t)(blockIdx.x & 7) * 1024;
        acc += __hip_atomic_load(const_cast<unsigned long long *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        acc += __hip_atomic_load(const_cast<unsigned long long *>(p + 8), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((it & 15) == 15 &&
            __builtin_amdgcn_readfirstlane(__hip_atomic_load(const_cast<unsigned *>(stop), __ATOMIC_RELAXED,
                                                              __HIP_MEMORY_SCOPE_SYSTEM)) != 0u)
            break;
        __builtin_amdgcn_s_sleep(1);
    }
    sink[blockIdx.x * 64 + threadIdx.x] = acc;
}

static int g_pollers = 0;
static unsigned long long *g_pg = nullptr, *g_psink = nullptr;
static unsigned *g_stop = nullptr;

template <int LAY, int MODE>
static void run(const char *name, const double *T, int rows, long long ld, int blocks, int R, int limit, int *d_idx,
                unsigned long long *d_st, double *d_sink) {
    std::mt19937 g(1234 + LAY * 7 + MODE);
    std::vector<int> idx(R);
    for (auto &v : idx) v = (int)(g() % (unsigned)limit);
    CK(hipMemcpy(d_idx, idx.data(), R * sizeof(int), hipMemcpyHostToDevice));
    k_probe<LAY, MODE><<<blocks, 512>>>(T, rows, ld, d_idx, R, d_st, d_sink);  // warm (code, TLB)
    CK(hipDeviceSynchronize());
    for (auto &v : idx) v = (int)(g() % (unsigned)limit);
    CK(hipMemcpy(d_idx, idx.data(), R * sizeof(int), hipMemcpyHostToDevice));
    hipStream_t ps = nullptr;
    if (g_pollers > 0) {  // (pollers on a second stream, running before and during the probe)
        CK(hipStreamCreateWithFlags(&ps, hipStreamNonBlocking));
        CK(hipMemset(g_stop, 0, 4));
        k_pollers<<<g_pollers, 64, 0, ps>>>(g_pg, g_stop, g_psink);
    }
    k_probe<LAY, MODE><<<blocks, 512>>>(T, rows, ld, d_idx, R, d_st, d_sink);
    CK(hipStreamSynchronize(nullptr));
    if (g_pollers > 0) {
        const unsigned one = 1;
        CK(hipMemcpy(g_stop, &one, 4, hipMemcpyHostToDevice));
        CK(hipStreamSynchronize(ps));
        CK(hipStreamDestroy(ps));
    }
    CK(hipDeviceSynchronize());
    std::vector<unsigned long long> st((size_t)blocks * R);
    CK(hipMemcpy(st.data(), d_st, st.size() * 8, hipMemcpyDeviceToHost));
    // per round: the median block's and the slowest block's round time (us)
    std::vector<double> med, mx;
    for (int k = 1; k < R; ++k) {
        std::vector<double> dt(blocks);
        for (int b = 0; b < blocks; ++b) dt[b] = (double)(st[(size_t)b * R + k] - st[(size_t)b * R + k - 1]) * 0.01;
        std::sort(dt.begin(), dt.end());
        med.push_back(dt[blocks / 2]);
        mx.push_back(dt[blocks - 1]);
    }
    std::sort(med.begin(), med.end());
    std::sort(mx.begin(), mx.end());
    printf("%-34s%s blocks %4d  round us: median block %6.3f (p10 %6.3f p90 %6.3f) | slowest block %6.3f (p90 %6.3f)\n",
           name, g_pollers ? " +pollers" : "", blocks, med[med.size() / 2], med[med.size() / 10], med[med.size() * 9 / 10], mx[mx.size() / 2],
           mx[mx.size() * 9 / 10]);
}

int main(int argc, char **argv) {
    const int rows = argc > 1 ? atoi(argv[1]) : 32768;
    const long long ld = argc > 2 ? atoll(argv[2]) : 12800;  // config 5 region A stride
    const int bg = argc > 3 ? atoi(argv[3]) : rows / 512;
    const int br = argc > 4 ? atoi(argv[4]) : 144;
    const int R = argc > 5 ? atoi(argv[5]) : 400;
    const int pollers = argc > 6 ? atoi(argv[6]) : 0;
    const size_t n = (size_t)rows * ld;
    printf("gather_probe: %d rows x %lld doubles (%.2f GB), %d gather blocks, %d row-read blocks, %d rounds\n", rows,
           ld, n * 8.0 / 1e9, bg, br, R);
    double *T, *sink;
    int *d_idx;
    unsigned long long *d_st;
    CK(hipMalloc(&T, n * 8));
    CK(hipMemset(T, 0, n * 8));
    CK(hipMalloc(&d_idx, R * sizeof(int)));
    CK(hipMalloc(&d_st, (size_t)std::max(bg, br) * R * 8));
    CK(hipMalloc(&sink, (size_t)std::max(bg, br) * 512 * 8));
    const int gl = (int)std::min<long long>(ld, 12288);  // gathered columns: the swept block
    const int rl = rows;
    const int rbr = (int)std::min<long long>(br, ld / 512);
    CK(hipMalloc(&g_pg, 8 * 1024 * 8 * 2));
    CK(hipMemset(g_pg, 0, 8 * 1024 * 8 * 2));
    CK(hipMalloc(&g_psink, 256 * 64 * 8));
    CK(hipMalloc(&g_stop, 4));
    for (int pass = 0; pass < (pollers > 0 ? 2 : 1); ++pass) {
        g_pollers = pass ? pollers : 0;
        run<0, 0>("G RM (row-major, engine)", T, rows, ld, bg, R, gl, d_idx, d_st, sink);
        run<1, 0>("G SM (16-row strips)", T, rows, ld, bg, R, gl, d_idx, d_st, sink);
        run<2, 0>("G CM (column-major)", T, rows, ld, bg, R, gl, d_idx, d_st, sink);
        run<3, 0>("G B4 (4x4 blocks)", T, rows, ld, bg, R, gl, d_idx, d_st, sink);
        run<4, 0>("G B8 (8 rows x 2 cols)", T, rows, ld, bg, R, gl, d_idx, d_st, sink);
        run<5, 0>("G B2 (2 rows x 8 cols)", T, rows, ld, bg, R, gl, d_idx, d_st, sink);
        run<0, 1>("R RM (row-major, engine)", T, rows, ld, rbr, R, rl, d_idx, d_st, sink);
        run<1, 1>("R SM (16-row strips)", T, rows, ld, rbr, R, rl, d_idx, d_st, sink);
        run<3, 1>("R B4 (4x4 blocks)", T, rows, ld, rbr, R, rl, d_idx, d_st, sink);
        run<4, 1>("R B8 (8 rows x 2 cols)", T, rows, ld, rbr, R, rl, d_idx, d_st, sink);
        run<5, 1>("R B2 (2 rows x 8 cols)", T, rows, ld, rbr, R, rl, d_idx, d_st, sink);
        run<0, 0>("G RM, one block", T, rows, ld, 1, R, gl, d_idx, d_st, sink);
        run<3, 0>("G B4, one block", T, rows, ld, 1, R, gl, d_idx, d_st, sink);
    }
    CK(hipFree(T));
    return 0;
}
