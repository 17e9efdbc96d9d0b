// sx_kernels.hip -- CDNA4 (gfx950) kernels of the dense two-phase simplex pivot path.
//
// Layout: the tableau T is row-major in HBM, one row per constraint, row
// stride ld doubles; column 0 = RHS b, column v+1 = variable v.  The objective row d is
// a separate vector, replicated on every shard.  Shards own contiguous row ranges whose
// starts are multiples of 512 (the reference's argmin tile).
//
// Every decision uses the reference's epsilon comparison (macro.h:28-42) and its exact
// argmin combine tree (reduction.cu:10-104): a 32-lane shuffle-down tree per "warp",
// then the 16 (pass 1, 512 threads) or 32 (pass 2, 1024 threads) warp winners combined
// by the same 32-lane tree.  On wave64 a reference warp is one 32-lane half of a wave:
// __shfl_down(x, off, 32) stays inside the half and returns the lane's own value past its
// end, exactly like the CUDA shuffle.  Compiled with -ffp-contract=off; every fused
// multiply-add of the reference is an explicit fma().

#include <float.h>

#include "sx_common.hpp"

namespace {

__device__ __forceinline__ int cmp_eps(double x, double y) {
    if (fabs(x - y) < SX_EPS) return 0;
    return x < y ? -1 : 1;
}

// Lane i takes lane i + OFF's value inside its 16-lane DPP row (row_shl:OFF); a lane whose
// source is past the row keeps its own value, as a CUDA shuffle past the warp's end does.
template <int OFF>
__device__ __forceinline__ int dpp_down(int x) {
    return __builtin_amdgcn_update_dpp(x, x, 0x100 + OFF, 0xF, 0xF, false);
}
template <int OFF>
__device__ __forceinline__ double dpp_down(double x) {
    const long long b = __double_as_longlong(x);
    const int lo = dpp_down<OFF>((int)b), hi = dpp_down<OFF>((int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}

template <int OFF>
__device__ __forceinline__ void argmin_step(double &v, int &i, double sv, int si) {
    if (cmp_eps(sv, v) < 0) {
        v = sv;
        i = si;
    }
}

// warpReduceMin (reduction.cu:10-22) on one 32-lane half of a wave64.  Every caller reads
// the result of lane 0 of the half, whose inputs at every step come from lanes inside the
// half (lanes 0..15 take 16..31, then 0..7 take 8..15, ...), so these are exactly the
// reference's combines.  The offset-16 step crosses DPP rows (a bpermute shuffle); offsets
// 8, 4, 2, 1 stay inside row 0 and use DPP row shifts (VALU, no LDS round trip).
__device__ __forceinline__ void half_argmin(double &v, int &i) {
    argmin_step<16>(v, i, __shfl_down(v, 16, 32), __shfl_down(i, 16, 32));
    argmin_step<8>(v, i, dpp_down<8>(v), dpp_down<8>(i));
    argmin_step<4>(v, i, dpp_down<4>(v), dpp_down<4>(i));
    argmin_step<2>(v, i, dpp_down<2>(v), dpp_down<2>(i));
    argmin_step<1>(v, i, dpp_down<1>(v), dpp_down<1>(i));
}

// blockReduceMin (reduction.cu:24-49) for a 512-thread block (8 waves = 16 halves).
// Result valid in thread 0.  The same tree is the reference's 1024-thread pass 2 whenever
// at most 512 partials exist: halves 16..31 of that block would hold only (DBL_MAX, -1),
// which is exactly the padding the 512-thread final stage inserts.
__device__ __forceinline__ void block_argmin512(double &v, int &i, double *s_v, int *s_i) {
    half_argmin(v, i);
    const int lane = threadIdx.x & 31;
    const int h = threadIdx.x >> 5;
    if (lane == 0) {
        s_v[h] = v;
        s_i[h] = i;
    }
    __syncthreads();
    if (threadIdx.x < 32) {
        v = (threadIdx.x < 16) ? s_v[threadIdx.x] : DBL_MAX;
        i = (threadIdx.x < 16) ? s_i[threadIdx.x] : -1;
        half_argmin(v, i);
    }
}

// Pass 2 (deviceReduceKernel<false><<<1,1024>>>, reduction.cu:239-241) over B <= 512 tile
// winners.  A partial equal to DBL_MAX is not taken (compare(DBL_MAX, DBL_MAX) == 0), so
// its index stays -1, as in the reference.
__device__ __forceinline__ void stage2_512(const TilePart *parts, int B, double &v, int &i, double *s_v,
                                           int *s_i) {
    v = DBL_MAX;
    i = -1;
    if ((int)threadIdx.x < B) {
        const double c = parts[threadIdx.x].v;
        if (cmp_eps(c, v) < 0) {
            v = c;
            i = parts[threadIdx.x].idx;
        }
    }
    block_argmin512(v, i, s_v, s_i);
}

// ---------------------------------------------------------------------------------------
// K1: entering-variable pass 1 over d[1..N) (minElement(costs+1, rows-1), solver.cu:87).
// Grid-stride exactly as the reference when L > 512*1024 (never for BASELINE sizes).
__global__ __launch_bounds__(512) void k_argmin_pass1(const double *__restrict__ v, int L, TilePart *out,
                                                      const DevState *st) {
    if (st != nullptr && st->status != SX_NOT_ENDED) return;
    __shared__ double s_v[16];
    __shared__ int s_i[16];
    double mv = DBL_MAX;
    int mi = -1;
    for (int i = blockIdx.x * SX_TILE + threadIdx.x; i < L; i += SX_TILE * gridDim.x) {
        const double c = v[i];
        if (cmp_eps(c, mv) < 0) {
            mv = c;
            mi = i;
        }
    }
    block_argmin512(mv, mi, s_v, s_i);
    if (threadIdx.x == 0) {
        out[blockIdx.x].v = mv;
        out[blockIdx.x].idx = mi;
        out[blockIdx.x].elig = 0;
    }
}

// Stand-alone pass 2 (used by the argmin test hook).
__global__ __launch_bounds__(512) void k_argmin_pass2(const TilePart *parts, int B, int *out_idx, double *out_v) {
    __shared__ double s_v[16];
    __shared__ int s_i[16];
    double v;
    int i;
    stage2_512(parts, B, v, i, s_v, s_i);
    if (threadIdx.x == 0) {
        *out_idx = i;
        *out_v = v;
    }
}

// sc1 (write-through, L1-bypassing) 8-byte accesses for the in-launch tile hand-off
// (MI355X_MICROARCH.md "Valid forms", first row: sc1 stores + one agent-scope counter add
// per storing workgroup; the last arriver, told by the add's return value, reads with sc1
// loads).  No fences needed.
__device__ __forceinline__ void store_tile_sc1(TilePart *t, double v, int idx, int elig) {
    unsigned long long *w = reinterpret_cast<unsigned long long *>(t);
    const unsigned long long lo = __double_as_longlong(v);
    const unsigned long long hi = (unsigned long long)(unsigned)idx | ((unsigned long long)(unsigned)elig << 32);
    __hip_atomic_store(w, lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(w + 1, hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void load_tile_sc1(const TilePart *t, double &v, int &idx, int &elig) {
    const unsigned long long *w = reinterpret_cast<const unsigned long long *>(t);
    const unsigned long long lo = __hip_atomic_load(const_cast<unsigned long long *>(w), __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long hi = __hip_atomic_load(const_cast<unsigned long long *>(w + 1), __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
    v = __longlong_as_double(lo);
    idx = (int)(unsigned)(hi & 0xffffffffull);
    elig = (int)(unsigned)(hi >> 32);
}

// Pass 2 of the entering argmin at the start of a phase (later pivots get it from the
// update kernel): (e_next, dmin_next) from the pass-1 partials.
__global__ __launch_bounds__(512) void k_enter_finish(const TilePart *parts, int B1, DevState *st) {
    __shared__ double s_v[16];
    __shared__ int s_i[16];
    double v;
    int i;
    stage2_512(parts, B1, v, i, s_v, s_i);
    if (threadIdx.x == 0) {
        st->e_next = i;
        st->dmin_next = v;
    }
}

// ---------------------------------------------------------------------------------------
// Deferred pivots.  T holds the tableau as of the last sweep; the q pivots
// of the current batch since then are kept as
//   U[s][j]   pivot row of slot s: the leaving row's values at that pivot (before /p),
//   F[i][s]   factor of local row i at slot s: -(a_ie / p)  (solver.cu:41),
//   recs[s]   (leaving row r, entering variable e, pivot p),
//   PM[i]     the slots where local row i was the leaving row, tagged with the batch id
//             (entries of older batches read as empty).
// The current value of an element is T[i][j] with the q pivots applied in order -- exactly
// the IEEE operations the reference applies one pivot at a time (solver.cu:34-46):
//   row r_s:  x = x / p_s             other rows:  x = fma(F[i][s], U[s][j], x)
// so every decision (entering argmin, ratio test) sees the reference's bits.  One sweep per
// batch applies all q pivots to every element: one read and one write of T per q pivots.

__device__ __forceinline__ unsigned slot_mask(int q) { return q >= 32 ? ~0u : ((1u << q) - 1u); }

__device__ __forceinline__ unsigned pend_bits(const unsigned long long *__restrict__ PM, int li, unsigned B,
                                              unsigned mask) {
    const unsigned long long w = PM[li];
    return ((unsigned)(w >> 32) == B) ? ((unsigned)w & mask) : 0u;
}

// Values of NC stored columns col[] of ONE row after its q pending pivots.  The row's
// factors sf[s] = F[row][s] and the pivots sp[s] are block-uniform (staged in LDS); the
// pivot-row values U[s][col] are loaded 8 slots at a time so their latencies overlap (slots
// >= q are read -- U has SX_KMAX rows -- but not used).
template <int NC>
__device__ __forceinline__ void cur_cols(double (&x)[NC], const int (&col)[NC], int q, unsigned bits,
                                         const double *sf, const double *sp, const double *__restrict__ U,
                                         size_t ld) {
    for (int s0 = 0; s0 < q; s0 += 8) {
        double u[8][NC];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const double *Us = U + (size_t)(s0 + k) * ld;
#pragma unroll
            for (int c = 0; c < NC; ++c) u[k][c] = Us[col[c]];
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int s = s0 + k;
            if (s < q) {
                if ((bits >> s) & 1u) {
#pragma unroll
                    for (int c = 0; c < NC; ++c) x[c] = x[c] / sp[s];
                } else {
#pragma unroll
                    for (int c = 0; c < NC; ++c) x[c] = fma(sf[s], u[k][c], x[c]);
                }
            }
        }
    }
}

__device__ __forceinline__ void cur_pair(double &xa, double &xb, int ca, int cb, int q, unsigned bits,
                                         const double *sf, const double *sp, const double *__restrict__ U,
                                         size_t ld) {
    double x[2] = {xa, xb};
    const int col[2] = {ca, cb};
    cur_cols<2>(x, col, q, bits, sf, sp, U, ld);
    xa = x[0];
    xb = x[1];
}

// Block-uniform pending data of one row (the pivot row being formed): its factors, the
// pivots, and its pivot-slot bits.  All threads of the block must call it.
__device__ __forceinline__ unsigned stage_row(const double *__restrict__ F, const PivRec *__restrict__ recs,
                                              const unsigned long long *__restrict__ PM, int rl, unsigned B, int q,
                                              double *sf, double *sp) {
    const int t = threadIdx.x;
    if (t < q) {
        sf[t] = F[sx_fidx(rl, t)];
        sp[t] = recs[t].p;
    }
    __syncthreads();
    return q > 0 ? pend_bits(PM, rl, B, slot_mask(q)) : 0u;
}

// current values of row rl, columns [0, Ns), written to out (stride over the block; Ns
// columns in pairs j, j + blockDim)
__device__ __forceinline__ void cur_row(const double *__restrict__ T, TLay tl, long long rl, int Ns, int q, unsigned bits,
                                        const double *sf, const double *sp, const double *__restrict__ U, size_t ld,
                                        double *out, int first, int stride) {
    for (int j = first; j < Ns; j += 2 * stride) {
        const int jb = j + stride < Ns ? j + stride : j;
        double xa = T[tl.idx(rl, j)], xb = T[tl.idx(rl, jb)];
        cur_pair(xa, xb, j, jb, q, bits, sf, sp, U, ld);
        out[j] = xa;
        if (j + stride < Ns) out[jb] = xb;
    }
}

// ---------------------------------------------------------------------------------------
// K2: ratio test (+ row selection on a single shard).  The entering variable and its
// reduced cost were produced by the previous pivot's k_pivot_row (or k_enter_finish).
// Every block:
//  - ends the phase if compare(dmin) >= 0 (solver.cu:88),
//  - builds the ratio vector of its 512 rows (createIndicatorsVector, reduction.cu:106-114)
//    from the current entering column and RHS, saves the entering column (the reference's
//    rowPivot copy, solver.cu:90-94) and reduces it to the tile winner + "any entry >= eps"
//    (isLessOrEqualThanZero, reduction.cu:186-201).
// With select != 0 the last block to arrive runs the pass-2 tree over the tile winners
// (minElement(knownTerms, rowPivot), solver.cu:104), declares UNBOUNDED (:96-102) or records
// the pivot: base[r] = e (:105).  With several shards the tile winners are allgathered
// first and k_select_row / k_select_gathered do that step.
__global__ __launch_bounds__(512) void k_ratio_select(const double *__restrict__ T, int rows, int row0, size_t ld, TLay tl,
                                                      TilePart *tiles_local, double *colE, DevState *st, int *base,
                                                      int select, double *slots, size_t slot_stride, Cols c,
                                                      const double *__restrict__ F, const double *__restrict__ U,
                                                      const PivRec *__restrict__ recs,
                                                      const unsigned long long *__restrict__ PM, unsigned B, int q) {
    if (st->status != SX_NOT_ENDED) return;
    const bool leader = blockIdx.x == 0 && threadIdx.x == 0;
    const long long piv = st->pivots;
    if (st->max_pivots >= 0 && piv >= st->max_pivots) {
        if (leader) st->status = SX_PIVOT_CAP;
        return;
    }
    const double v = st->dmin_next;
    const int e = st->e_next;
    if (!(cmp_eps(v, 0.0) < 0)) {
        if (leader) st->status = SX_FEASIBLE;
        return;
    }
    if (leader) {
        st->e = e;
        st->dmin = v;
    }
    const int ce = c.map(1 + e);
    const unsigned mask = slot_mask(q);
    __shared__ double s_v[16];
    __shared__ int s_i[16];
    // the pending pivot rows' RHS and entering-column entries, and the pivots (uniform)
    __shared__ double s_u0[SX_KMAX], s_ue[SX_KMAX], s_p[SX_KMAX];
    if ((int)threadIdx.x < q) {
        const double *Us = U + (size_t)threadIdx.x * ld;
        s_u0[threadIdx.x] = Us[0];
        s_ue[threadIdx.x] = Us[ce];
        s_p[threadIdx.x] = recs[threadIdx.x].p;
    }
    const int li = blockIdx.x * SX_TILE + threadIdx.x;
    double rv = DBL_MAX;
    int ri = -1;
    int elig = 0;
    double b = 0.0, a = 0.0;
    unsigned bits = 0u;
    if (li < rows) {
        b = T[tl.idx(li, 0)];
        a = T[tl.idx(li, ce)];
        if (q > 0) bits = pend_bits(PM, li, B, mask);
    }
    __syncthreads();
    if (li < rows) {
        for (int s0 = 0; s0 < q; s0 += 8) {
            double f[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) f[k] = F[sx_fidx(li, s0 + k)];  // s0 + k < SX_KMAX
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int s = s0 + k;
                if (s < q) {
                    if ((bits >> s) & 1u) {
                        b = b / s_p[s];
                        a = a / s_p[s];
                    } else {
                        b = fma(f[k], s_u0[s], b);
                        a = fma(f[k], s_ue[s], a);
                    }
                }
            }
        }
        colE[li] = a;
        elig = a >= SX_EPS;
        const double ratio = cmp_eps(a, 0.0) > 0 ? b / a : DBL_MAX;
        if (cmp_eps(ratio, rv) < 0) {
            rv = ratio;
            ri = row0 + li;
        }
    }
    const int any = __syncthreads_or(elig);
    block_argmin512(rv, ri, s_v, s_i);
    if (!select) {
        if (slots == nullptr) {
            if (threadIdx.x == 0) {
                tiles_local[blockIdx.x].v = rv;
                tiles_local[blockIdx.x].idx = ri;
                tiles_local[blockIdx.x].elig = any;
            }
            return;
        }
        // row-gather exchange: the slot carries the tile winner and that row's current
        // values, so one allgather hands every rank the pivot row whichever tile wins
        __shared__ int s_ri;
        __shared__ double s_f[SX_KMAX];
        double *slot = slots + (size_t)blockIdx.x * slot_stride;
        if (threadIdx.x == 0) {
            TilePart *h = reinterpret_cast<TilePart *>(slot);
            h->v = rv;
            h->idx = ri;
            h->elig = any;
            s_ri = ri;
        }
        __syncthreads();
        if (s_ri < 0) return;
        const int wl = s_ri - row0;
        const unsigned wbits = stage_row(F, recs, PM, wl, B, q, s_f, s_p);
        cur_row(T, tl, wl, c.Ns, q, wbits, s_f, s_p, U, ld, slot + 2, threadIdx.x, SX_TILE);
        return;
    }
    __shared__ int s_last;
    if (threadIdx.x == 0) {
        store_tile_sc1(tiles_local + blockIdx.x, rv, ri, any);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned t = __hip_atomic_fetch_add(&st->ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = (t == gridDim.x - 1);
    }
    __syncthreads();
    if (!s_last) return;
    const int B2 = gridDim.x;
    double tv = DBL_MAX;
    int ti = -1, te = 0;
    if ((int)threadIdx.x < B2) {
        double cv;
        int ci;
        load_tile_sc1(tiles_local + threadIdx.x, cv, ci, te);
        if (cmp_eps(cv, tv) < 0) {
            tv = cv;
            ti = ci;
        }
    }
    const int anyall = __syncthreads_or(SX_ELIG(te));
    if (!anyall) {
        if (threadIdx.x == 0) {
            st->ticket = 0;
            st->status = SX_UNBOUNDED;
        }
        return;
    }
    block_argmin512(tv, ti, s_v, s_i);
    if (threadIdx.x == 0) {
        st->ticket = 0;
        if (ti < 0) {
            st->status = SX_NUMERIC_FAIL;
        } else {
            base[ti] = e;
            st->r = ti;
            st->pivots = piv + 1;
            st->batch_tag = B;
            st->batch_count = q + 1;
        }
    }
}

// ---------------------------------------------------------------------------------------
// K3 (several shards): every block re-derives the leaving row from the allgathered tile
// winners, checks the unbounded condition, records the pivot, and writes its chunk of the
// current pivot row (the reference's copyColumn, solver.cu:24-32, is a contiguous row
// here).  Only the owner contributes the row; the others contribute -0.0, the exact
// additive identity, so the sum-allreduce reproduces the owner's row bit for bit.
__global__ __launch_bounds__(512) void k_select_row(const double *__restrict__ T, int rows, int row0, size_t ld, TLay tl,
                                                    int Ns, const TilePart *__restrict__ tiles_all, int B2,
                                                    double *prow_out, int *base, DevState *st,
                                                    const double *__restrict__ F, const double *__restrict__ U,
                                                    const PivRec *__restrict__ recs,
                                                    const unsigned long long *__restrict__ PM, unsigned B, int q) {
    if (st->status != SX_NOT_ENDED) return;
    const bool leader = blockIdx.x == 0 && threadIdx.x == 0;
    __shared__ double s_v[16];
    __shared__ int s_i[16];
    __shared__ int s_r;
    const int pk = ((int)threadIdx.x < B2) ? tiles_all[threadIdx.x].elig : 0;
    if (!__syncthreads_or(SX_ELIG(pk))) {
        if (leader) st->status = SX_UNBOUNDED;  // solver.cu:96-102
        return;
    }
    double v;
    int r;
    stage2_512(tiles_all, B2, v, r, s_v, s_i);
    if (threadIdx.x == 0) s_r = r;
    __syncthreads();
    r = s_r;
    if (r < 0) {
        if (leader) st->status = SX_NUMERIC_FAIL;
        return;
    }
    const long long piv = st->pivots;
    const int rl = r - row0;
    const bool own = rl >= 0 && rl < rows;
    if (own) {
        __shared__ double s_f[SX_KMAX], s_p[SX_KMAX];
        const unsigned bits = stage_row(F, recs, PM, rl, B, q, s_f, s_p);
        cur_row(T, tl, rl, Ns, q, bits, s_f, s_p, U, ld, prow_out, blockIdx.x * blockDim.x + threadIdx.x,
                gridDim.x * blockDim.x);
    } else {
        for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < Ns; j += gridDim.x * blockDim.x) prow_out[j] = -0.0;
    }
    // commit the pivot once every block has read the state above: the last block to
    // arrive does it (the next kernel sees it after the launch boundary)
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned t = __hip_atomic_fetch_add(&st->ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (t == gridDim.x - 1) {
            st->ticket = 0;
            base[r] = st->e;  // solver.cu:105
            st->r = r;
            st->pivots = piv + 1;
            st->batch_tag = B;
            st->batch_count = q + 1;
        }
    }
}

// K3 (row-gather exchange): one block picks the leaving row among the gathered tile
// winners (the reference's pass-2 tree), checks the unbounded condition and records the
// pivot; k_pivot_row then reads the pivot row from the winning slot.
__global__ __launch_bounds__(512) void k_select_gathered(const double *__restrict__ slots, size_t slot_stride, int B2,
                                                         int *base, DevState *st, unsigned B, int q) {
    if (st->status != SX_NOT_ENDED) return;
    __shared__ double s_v[16];
    __shared__ int s_i[16];
    double v = DBL_MAX;
    int r = -1, pk = 0;
    if ((int)threadIdx.x < B2) {
        const TilePart *h = reinterpret_cast<const TilePart *>(slots + (size_t)threadIdx.x * slot_stride);
        pk = h->elig;
        const double c = h->v;
        if (cmp_eps(c, v) < 0) {
            v = c;
            r = h->idx;
        }
    }
    if (!__syncthreads_or(SX_ELIG(pk))) {
        if (threadIdx.x == 0) st->status = SX_UNBOUNDED;  // solver.cu:96-102
        return;
    }
    block_argmin512(v, r, s_v, s_i);
    if (threadIdx.x == 0) {
        if (r < 0) {
            st->status = SX_NUMERIC_FAIL;
        } else {
            base[r] = st->e;  // solver.cu:105
            st->r = r;
            st->pivots += 1;
            st->batch_tag = B;
            st->batch_count = q + 1;
        }
    }
}

// ---------------------------------------------------------------------------------------
// K4: the pivot row of slot q and everything that depends only on it.
//   U[q][j]  = current row r (the reference's colPivot, solver.cu:24-32)  -- read in place
//              with the pending pivots applied on one shard, or taken from the exchanged
//              row (prow_buf) on several;
//   p        = U[q][e]  (= the entering column's entry at r; solver.cu:66);
//   d[j]     = fma(-(d_e / p), U[q][j], d[j])  (updateCostsVector, solver.cu:48-56), and pass
//              1 of the NEXT entering argmin per 512-tile (reduction.cu:51-80); the last block
//              to arrive runs pass 2 and stores (e_next, dmin_next);
//   F[i][q]  = -(a_ie / p) for the shard's rows (the factor of solver.cu:41);
//   recs[q], PM[r] |= slot q.
// Blocks [0, B1) are the objective-row tiles (512 logical columns each, 2 per thread);
// the rest compute the factor column.  Writes to recs[q] / PM[r] race with nothing: readers
// in this launch only look at slots < q.
__global__ __launch_bounds__(256) void k_pivot_row(const double *__restrict__ T, int rows, int row0, size_t ld, TLay tl, Cols c,
                                                   double *__restrict__ d, const double *__restrict__ prow_buf,
                                                   size_t prow_stride, const double *__restrict__ colE, DevState *st,
                                                   double *U, double *F, PivRec *recs, unsigned long long *PM,
                                                   TilePart *enter_parts, unsigned B, int q, int B1) {
    if (st->status != SX_NOT_ENDED) return;
    const int r = st->r, e = st->e;
    const int rl = r - row0;
    const double *prow =
        prow_buf ? (prow_stride ? prow_buf + (size_t)(r / SX_TILE) * prow_stride + 2 : prow_buf) : nullptr;
    const long long trl = prow ? 0 : rl;  // (the stored row is read only when the row is local)
    __shared__ double s_f[SX_KMAX], s_p[SX_KMAX];
    const unsigned bits = prow ? 0u : stage_row(F, recs, PM, rl, B, q, s_f, s_p);
    // current values of the pivot row at the entering column (the pivot), column 0 and this
    // thread's two objective-row columns, with all their loads in flight together
    const int L = c.N - 1;
    const int ia = blockIdx.x * SX_TILE + threadIdx.x, ib = ia + 256;
    const int col[4] = {c.map(1 + e), 0, c.map(1 + (ia < L ? ia : 0)), c.map(1 + (ib < L ? ib : 0))};
    double x[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) x[k] = prow ? prow[col[k]] : T[tl.idx(trl, col[k])];
    if (!prow) cur_cols<4>(x, col, q, bits, s_f, s_p, U, ld);
    const double p = x[0], u0 = x[1], ua = x[2], ub = x[3];
    if ((int)blockIdx.x >= B1) {
        const int i = ((int)blockIdx.x - B1) * 256 + (int)threadIdx.x;
        if (i < rows) F[sx_fidx(i, q)] = -colE[i] / p;
        if (i == rl) {
            const unsigned long long w = PM[rl];
            PM[rl] = (((unsigned)(w >> 32) == B) ? w : ((unsigned long long)B << 32)) | (1ull << q);
        }
        return;
    }
    double *Uq = U + (size_t)q * ld;
    const double fd = -st->dmin / p;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        Uq[0] = u0;
        d[0] = fma(fd, u0, d[0]);
        recs[q].r = r;
        recs[q].e = e;
        recs[q].p = p;
    }
    // ---- objective row + next entering argmin (512 reference threads on 256)
    __shared__ double s_v[16];
    __shared__ int s_i[16];
    __shared__ int s_last;
    double v0 = DBL_MAX, v1 = DBL_MAX;
    int i0 = -1, i1 = -1;
    if (ia < L) {
        const int j = 1 + ia;
        if (j < c.Ns) Uq[col[2]] = ua;  // stored position (slack compaction)
        const double x = fma(fd, ua, d[j]);
        d[j] = x;
        if (cmp_eps(x, v0) < 0) {
            v0 = x;
            i0 = ia;
        }
    }
    if (ib < L) {
        const int j = 1 + ib;
        if (j < c.Ns) Uq[col[3]] = ub;
        const double x = fma(fd, ub, d[j]);
        d[j] = x;
        if (cmp_eps(x, v1) < 0) {
            v1 = x;
            i1 = ib;
        }
    }
    half_argmin(v0, i0);  // reference warps 0..7
    half_argmin(v1, i1);  // reference warps 8..15
    const int lane = threadIdx.x & 31, h = threadIdx.x >> 5;
    if (lane == 0) {
        s_v[h] = v0;
        s_i[h] = i0;
        s_v[h + 8] = v1;
        s_i[h + 8] = i1;
    }
    __syncthreads();
    if (threadIdx.x < 32) {
        double v = (threadIdx.x < 16) ? s_v[threadIdx.x] : DBL_MAX;
        int i = (threadIdx.x < 16) ? s_i[threadIdx.x] : -1;
        half_argmin(v, i);
        if (threadIdx.x == 0) {
            store_tile_sc1(enter_parts + blockIdx.x, v, i, 0);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const unsigned t = __hip_atomic_fetch_add(&st->ticket_d, 1u, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT);
            s_last = (t == (unsigned)B1 - 1);
        }
    }
    __syncthreads();
    if (!s_last) return;
    // last objective block: pass 2 (reference pass-2 tree; B1 <= 256 here)
    double v = DBL_MAX;
    int i = -1;
    if ((int)threadIdx.x < B1) {
        double cv;
        int ci, ce;
        load_tile_sc1(enter_parts + threadIdx.x, cv, ci, ce);
        if (cmp_eps(cv, v) < 0) {
            v = cv;
            i = ci;
        }
    }
    half_argmin(v, i);
    __syncthreads();
    if (lane == 0) {
        s_v[h] = v;
        s_i[h] = i;
    }
    __syncthreads();
    if (threadIdx.x < 32) {
        v = (threadIdx.x < 8) ? s_v[threadIdx.x] : DBL_MAX;
        i = (threadIdx.x < 8) ? s_i[threadIdx.x] : -1;
        half_argmin(v, i);
        if (threadIdx.x == 0) {
            st->e_next = i;
            st->dmin_next = v;
            st->ticket_d = 0;
        }
    }
}

typedef unsigned long long u64;

__device__ __forceinline__ void drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Granule tag word: [batch id mod 2^15 | slot q (6 bits) | payload (11 bits)].  A consumer
// matches on batch and slot and ignores the payload, so a tile winner's value granules also
// carry its index (and the ratio tiles' eligibility bit): 2 granules per winner instead of 3-4.
#define SX_PAYBITS 11
#define SX_PAYMASK ((1u << SX_PAYBITS) - 1u)
#define SX_NOIDX 0x3FFu  // payload index of a tile without a candidate
__device__ __forceinline__ unsigned make_tag(unsigned B, int q) {
    return ((B & 0x7FFFu) << (6 + SX_PAYBITS)) | ((unsigned)q << SX_PAYBITS);
}

__device__ __forceinline__ void put_g(u64 *g, unsigned data, unsigned tag) {
    __hip_atomic_store(g, ((u64)tag << 32) | data, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double gd(unsigned lo, unsigned hi) {
    return __longlong_as_double((long long)(((u64)hi << 32) | lo));
}
__device__ __forceinline__ u64 ld_sc1(const u64 *p) {
    return __hip_atomic_load(const_cast<u64 *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned ld_sc1(const unsigned *p) {
    return __hip_atomic_load(const_cast<unsigned *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// k_batch's objective-tile records as its ratio blocks poll them: 4 granules per tile (the tile
// winner's d value and its pivot-row value of the pivot), at most SX_OBJ_TILES
// tiles (every wave of a ratio block polls an eighth of them: at most 2 granules per lane)
#define SX_GB4 4
#define SX_GBS 16  // their stride in memory, granules: one 128-byte line per record (no two producers share a line)
#define SX_OBJ_TILES 160

// 8-byte write-through (sc1) store / L1-bypassing load of a double
__device__ __forceinline__ void st_sc1(double *p, double v) {
    __hip_atomic_store(reinterpret_cast<u64 *>(p), (u64)__double_as_longlong(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1d(const double *p) {
    return __longlong_as_double((long long)ld_sc1(reinterpret_cast<const u64 *>(p)));
}
struct IdOff {
    __device__ __forceinline__ int operator()(int k) const { return k; }
};
// the value granules (2 per tile) of k_batch's 4-granule objective records
struct Rec4Val {
    __device__ __forceinline__ int operator()(int k) const { return (k >> 1) * SX_GBS + (k & 1); }
};
// all 4 granules of each record, from granule k0 on
struct Rec4AllFrom {
    int k0;
    __device__ __forceinline__ int operator()(int k) const { return ((k0 + k) >> 2) * SX_GBS + ((k0 + k) & 3); }
};
// all 4 granules of each record
struct Rec4All {
    __device__ __forceinline__ int operator()(int k) const { return (k >> 2) * SX_GBS + (k & 3); }
};

__device__ __forceinline__ u64 ld_sys(const u64 *p) {
    return __hip_atomic_load(const_cast<u64 *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// granules per lane of the one-wave gather (larger gathers use every thread of the block)
#define SX_GATHER_PER_LANE 8

// pause between two polls of a hand-off (one s_sleep unit, 64 clocks: longer or no pauses
// measured no different)
__device__ __forceinline__ void poll_pause() { __builtin_amdgcn_s_sleep(1); }

// Wave 0 of the block (threads 0..63) polls n <= 64 * PL granules, granule k at base[off(k)], each
// until it carries `tag`, into out[k] (LDS), all of a round's loads in flight together, no block
// barrier per poll; payf(k, payload) is called for every granule as it arrives.  Wave-uniform
// result: false when the batch was aborted (or this wait timed out, which aborts it).  Only wave 0
// may call it.
template <typename OFF, bool SYS, int PL, typename PAYF>
__device__ __forceinline__ int poll_wave_f(const u64 *base, int n, OFF off, unsigned tag, unsigned *out, unsigned *abort_w,
                           unsigned long long timeout, PAYF payf) {
    const int t = threadIdx.x & 63;
    const u64 t0 = __builtin_amdgcn_s_memrealtime();
    if (n <= 64) {
        bool have = t >= n;
        for (unsigned it = 0;; ++it) {
            if (!have) {
                const u64 w = SYS ? ld_sys(base + off(t)) : ld_sc1(base + off(t));
                if (((unsigned)(w >> 32) | SX_PAYMASK) == (tag | SX_PAYMASK)) {
                    have = true;
                    out[t] = (unsigned)w;
                    payf(t, (unsigned)(w >> 32) & SX_PAYMASK);
                }
            }
            if (__ballot(!have) == 0ull) return 1;
            if ((it & 63) == 63) {
                int stop = ld_sc1(abort_w) != 0u;
                if (!stop && __builtin_amdgcn_s_memrealtime() - t0 > timeout) {
                    __hip_atomic_store(abort_w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    stop = 1;
                }
                if (__builtin_amdgcn_readfirstlane(stop)) return 0;
            }
            poll_pause();
        }
    }
    unsigned miss = 0u;  // bit c: granule t + 64 c still missing
#pragma unroll
    for (int c = 0; c < PL; ++c)
        if (t + 64 * c < n) miss |= 1u << c;
    for (unsigned it = 0;; ++it) {
        u64 w[PL];
#pragma unroll
        for (int c = 0; c < PL; ++c)
            if ((miss >> c) & 1u) w[c] = SYS ? ld_sys(base + off(t + 64 * c)) : ld_sc1(base + off(t + 64 * c));
#pragma unroll
        for (int c = 0; c < PL; ++c) {
            const int k = t + 64 * c;
            if (((miss >> c) & 1u) && ((unsigned)(w[c] >> 32) | SX_PAYMASK) == (tag | SX_PAYMASK)) {
                miss &= ~(1u << c);
                out[k] = (unsigned)w[c];
                payf(k, (unsigned)(w[c] >> 32) & SX_PAYMASK);
            }
        }
        if (__ballot(miss != 0u) == 0ull) return 1;
        if ((it & 63) == 63) {
            int stop = ld_sc1(abort_w) != 0u;
            if (!stop && __builtin_amdgcn_s_memrealtime() - t0 > timeout) {
                __hip_atomic_store(abort_w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                stop = 1;
            }
            if (__builtin_amdgcn_readfirstlane(stop)) return 0;
        }
        poll_pause();
    }
}

// The same with the payload of every even granule k stored to pay[k / 2] (records whose value
// granules come in pairs), or dropped (pay null).
template <typename OFF, bool SYS = false>
__device__ int poll_wave(const u64 *base, int n, OFF off, unsigned tag, unsigned *out, unsigned *abort_w,
                         unsigned long long timeout, unsigned *pay) {
    return poll_wave_f<OFF, SYS, SX_GATHER_PER_LANE>(base, n, off, tag, out, abort_w, timeout,
                                                     [pay](int k, unsigned pl) {
                                                         if (pay && !(k & 1)) pay[k >> 1] = pl;
                                                     });
}

// The same poll spread over every wave of the block: wave w polls its share of the n granules (whole
// records of `rec` granules, in order; granule k at base[off(k)] into out[k], payf(k, payload) as
// it arrives), then one block barrier; block-uniform result (false: the batch was aborted or a wait
// timed out).  Every thread of the block must call it.  Eight waves with at most two granules per
// lane each hand a batch's records over faster than one wave with up to ten per lane (round 6,
// profiles/r06_poll_waves_ab.txt: the objective->ratio hop 3.18 -> 2.46 us at config 5).
template <typename OFF>
struct OffFrom {
    OFF off;
    int k0;
    __device__ __forceinline__ int operator()(int k) const { return off(k0 + k); }
};
template <typename OFF, typename PAYF>
__device__ __forceinline__ int poll_block(const u64 *base, int n, int rec, OFF off, unsigned tag, unsigned *out,
                                          unsigned *abort_w, unsigned long long timeout, PAYF payf, int *s_okw) {
    const int w = (int)threadIdx.x >> 6, nw = (int)blockDim.x >> 6;
    const int per = ((n + nw - 1) / nw + rec - 1) / rec * rec;
    const int k0 = w * per, nk = n - k0 < per ? (n - k0 > 0 ? n - k0 : 0) : per;
    int ok = 1;
    if (nk > 0)
        ok = poll_wave_f<OffFrom<OFF>, false, 2>(base, nk, OffFrom<OFF>{off, k0}, tag, out + k0, abort_w, timeout,
                                                 [&](int kl, unsigned pl) { payf(k0 + kl, pl); });
    if ((threadIdx.x & 63) == 0) s_okw[w] = ok;
    __syncthreads();
    int all = 1;
    for (int w1 = 0; w1 < nw; ++w1) all &= s_okw[w1];
    return all;
}

// Pass 2 of the reference's argmin (deviceReduceKernel<false><<<1,1024>>>, reduction.cu:239-241)
// over nt <= 256 two-granule tile records already gathered into s_g / s_pay, run by wave 0
// alone: part p (tile p's winner) sits on lane p % 64 of round p / 64, so round r's two halves
// are the reference warps 2r and 2r + 1 (half_argmin); their winners go through LDS to lanes
// 0..2R-1, padded with (DBL_MAX, -1) to the reference's 32 warps, and one more half_argmin
// combines them -- the combines of block_argmin512 on the same parts.  Result in lane 0;
// any_elig (wave-uniform): some record carries the "entry >= eps" payload bit (ratio tiles).
// (S: granules per gathered record, its value in the first two)
template <int S = 2, typename PT = unsigned>
__device__ __forceinline__ void wave_pass2(const unsigned *s_g, const PT *s_pay, int nt, double *s_v,
                                           int *s_i, double &v_out, int &i_out, int &any_elig) {
    const int lane = threadIdx.x;
    const int R = (nt + 63) >> 6;
    unsigned te = 0u;
    for (int r = 0; r < R; ++r) {
        const int p = r * 64 + lane;
        double v = DBL_MAX;
        int i = -1;
        if (p < nt) {
            const double cv = gd(s_g[S * p], s_g[S * p + 1]);
            const unsigned pl = s_pay[p];
            te |= (pl >> 10) & 1u;
            if (cmp_eps(cv, v) < 0) {
                v = cv;
                i = (pl & SX_NOIDX) == SX_NOIDX ? -1 : p * SX_TILE + (int)(pl & SX_NOIDX);
            }
        }
        half_argmin(v, i);
        if ((lane & 31) == 0) {
            s_v[2 * r + (lane >> 5)] = v;
            s_i[2 * r + (lane >> 5)] = i;
        }
    }
    double v = DBL_MAX;
    int i = -1;
    if (lane < 2 * R) {
        v = s_v[lane];
        i = s_i[lane];
    }
    half_argmin(v, i);
    any_elig = __ballot(te != 0u) != 0ull;
    v_out = v;
    i_out = i;
}

// The block reads n <= 4 * blockDim granules, granule k at base[off(k)], each until it
// carries `tag`, into out[k] (LDS): up to 64 * SX_GATHER_PER_LANE granules one wave polls
// (poll_wave); larger gathers: every thread polls its own granules (k = t, t + 512, ...), all
// of them in flight together, until the block agrees that all have arrived.  Block-uniform
// result: false when the batch was aborted (or this wait timed out, which aborts it).  Every
// thread of the block must call it.
template <typename OFF, bool SYS = false>
__device__ bool gather_tagged(const u64 *base, int n, OFF off, unsigned tag, unsigned *out, unsigned *abort_w,
                              int *s_ok, unsigned long long timeout = 20000000ull, unsigned *pay = nullptr) {
    const int t = threadIdx.x, nt = blockDim.x;
    if (n <= 64 * SX_GATHER_PER_LANE) {
        if (t < 64) {
            const int ok = poll_wave<OFF, SYS>(base, n, off, tag, out, abort_w, timeout, pay);
            if (t == 0) *s_ok = ok;
        }
        __syncthreads();
        return *s_ok != 0;
    }
    unsigned have = 0u;  // bit c: granule t + c * nt has arrived (or does not exist)
#pragma unroll
    for (int c = 0; c < 4; ++c)
        if (t + c * nt >= n) have |= 1u << c;
    const u64 t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
    for (unsigned it = 0;; ++it) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            if (!((have >> c) & 1u)) {
                const int k = t + c * nt;
                const u64 w = SYS ? ld_sys(base + off(k)) : ld_sc1(base + off(k));
                if (((unsigned)(w >> 32) | SX_PAYMASK) == (tag | SX_PAYMASK)) {
                    have |= 1u << c;
                    out[k] = (unsigned)w;
                    if (pay && !(k & 1)) pay[k >> 1] = (unsigned)(w >> 32) & SX_PAYMASK;
                }
            }
        }
        if (!__syncthreads_or(have != 0xFu)) break;
        if ((it & 63) == 63) {
            if (t == 0) {
                int stop = ld_sc1(abort_w) != 0u;
                if (!stop && __builtin_amdgcn_s_memrealtime() - t0 > timeout) {  // 100 MHz ticks
                    __hip_atomic_store(abort_w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    stop = 1;
                }
                *s_ok = !stop;
            }
            __syncthreads();
            if (!*s_ok) return false;
        }
        poll_pause();
    }
    return true;  // the vote's barrier made every thread's LDS writes visible
}

// granule layout of one tile record
// (k_batch: the RV..RF / OV..OU layouts below; k_batch_mr: v(2) pad(2) a(2) b(2) F(2 per slot) and
// v(2) pad(2) U(2 per slot) inside the same strides)
#define SX_GA_STRIDE (10 + 2 * SX_HMAX)  // ratio tile record, granules (one stage of history)
#define SX_GB_STRIDE (9 + 2 * SX_HMAX)   // objective tile record, granules
__device__ __forceinline__ int rec2_a(int k) { return (k >> 1) * SX_GA_STRIDE + (k & 1); }
// granules of all tile records
__host__ __device__ __forceinline__ size_t sx_ga_size() { return (size_t)SX_TILE * SX_GA_STRIDE; }
__host__ __device__ __forceinline__ size_t sx_gb_size() { return (size_t)SX_TILE * SX_GB_STRIDE; }
__device__ __forceinline__ int rec2_b(int k) { return (k >> 1) * SX_GB_STRIDE + (k & 1); }

// The history chains below read the block-uniform values of a slot (the entering column's
// U[s][e], the leaving row's F[r][s], the pivots) through one register per wave -- lane s holds
// slot s, read with v_readlane into scalar registers -- instead of an LDS read per slot: with
// the fused batch's register file nearly full, per-slot LDS reads were issued one at a time
// and each waited its round trip (ISA of round 3).
__device__ __forceinline__ double rdlane(double v, int l) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

// The batch's pending pivots s < q of one stage are applied, in slot order, to a ratio row's
// entering-column entry (solver.cu:34-46 on that element): a / p_s at the slots where the row itself
// left the basis, fma(F[row][s], U[s][e], a) at the others -- and to the pivot row's entry on an
// objective tile's column: u / p_s where the leaving row r left before, fma(F[r][s], U[s][j], u)
// elsewhere.  A row that left at slots in `bits` has, just before its last such slot sl, exactly the
// value the pivot row of slot sl held in this column -- U[sl][e], formed by the objective tiles with the
// same operations in the same order -- so its chain is U[sl][e] / p_sl followed by the fmas of the
// slots after sl: one division and a select per slot instead of a branch per slot.  Two stages
// (pivots SX_HMAX .. SX_KMAX - 1): the first stage's history, moved from LDS to registers at the
// switch (h1), is applied before the second stage's.  The block-uniform operands of a slot (the
// entering column's U[s][e], the leaving row's F[r][s]) come from one wave register or LDS array per
// stage, fed to each step by a DPP broadcast (below).

// 64-bit value of lane src (per-lane src; ds_bpermute)
__device__ __forceinline__ double shfl_d(double v, int src) {
    const long long b = __double_as_longlong(v);
    const int lo = __shfl((int)b, src), hi = __shfl((int)(b >> 32), src);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

// ---- history chains with the slot values as DPP broadcasts (round 6).  A chain step
// x = fma(w_s, h_s, x) took two v_readlane (lane s of the wave register holding the slot values, into
// scalar registers), an s_nop for the scalar hazard and the fma -- three VALU issues per step, the two
// waves of a SIMD sharing them.  Here the 32 slot values sit in two registers as broadcast sources --
// lane l of W.w[j] holds slot 16 j + (l & 15) -- and each step is ONE v_fmac_f64_dpp with
// row_newbcast:(s & 15), which feeds every lane of a 16-lane row from that row's lane s & 15, i.e.
// slot s.  The same fma per element in the same slot order (w_s * h_s is one exactly rounded product
// either way): the same bits.
template <int K>
__device__ __forceinline__ double fma_bc(double w, double h, double x) {
    asm("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf" : "+v"(x) : "v"(w), "v"(h), "n"(K));
    return x;
}
struct Bc2 {
    double w[2];
};
// (a VALU write of a register a DPP instruction reads needs 2 wait states: the s_nop, ordered after the
// writes by its operands, provides them once per chain)
__device__ __forceinline__ void bc2_fence(Bc2 &b) { asm volatile("s_nop 1" : "+v"(b.w[0]), "+v"(b.w[1])); }
// from a wave register holding slot s in lane s (s < 32)
__device__ __forceinline__ Bc2 bc2_from_lanes(double wv) {
    const int l = (int)threadIdx.x & 15;
    Bc2 b{{shfl_d(wv, l), shfl_d(wv, 16 + l)}};
    bc2_fence(b);
    return b;
}
// from an LDS array holding slot s at s_v[s] (s < 32)
__device__ __forceinline__ Bc2 bc2_from_lds(const double *s_v) {
    const int l = (int)threadIdx.x & 15;
    Bc2 b{{s_v[l], s_v[16 + l]}};
    bc2_fence(b);
    return b;
}
// steps S0 .. S0 + 7 of a chain on the history values h[0..8), those at slots in [from, q) applied
// (all: plain steps; SEL: y = the step, kept only where keep(slot) -- a lane-dependent select)
template <int S0>
__device__ __forceinline__ double bc_steps8(double x, const Bc2 &W, const double (&h)[8], int from, int q) {
#define SX_BCS(K)                                                                       \
    if (S0 + K >= from && S0 + K < q) x = fma_bc<(S0 + K) & 15>(W.w[(S0 + K) >> 4], h[K], x);
    SX_BCS(0) SX_BCS(1) SX_BCS(2) SX_BCS(3) SX_BCS(4) SX_BCS(5) SX_BCS(6) SX_BCS(7)
#undef SX_BCS
    return x;
}
template <int S0>
__device__ __forceinline__ double bc_steps8_after(double x, const Bc2 &W, const double (&h)[8], int q, int sl,
                                                  bool all) {
#define SX_BCS(K)                                                                          \
    if (S0 + K < q) {                                                                      \
        const double y = fma_bc<(S0 + K) & 15>(W.w[(S0 + K) >> 4], h[K], x);               \
        x = (all || S0 + K > sl) ? y : x;                                                  \
    }
    SX_BCS(0) SX_BCS(1) SX_BCS(2) SX_BCS(3) SX_BCS(4) SX_BCS(5) SX_BCS(6) SX_BCS(7)
#undef SX_BCS
    return x;
}
// the history of slots [from, q) of this thread's column / row from LDS (s_hist[s][t]), 8 slots per
// group of loads
__device__ __forceinline__ double bc_chain_lds(double x, const Bc2 &W, const double *s_hist, int from, int q) {
    const int t = threadIdx.x;
    double h[8];
#define SX_BCG(S0)                                                                     \
    if (S0 < q && S0 + 8 > from) {                                                     \
        _Pragma("unroll") for (int k = 0; k < 8; ++k) h[k] = s_hist[(S0 + k) * SX_TILE + t]; \
        x = bc_steps8<S0>(x, W, h, from, q);                                           \
    }
    SX_BCG(0) SX_BCG(8) SX_BCG(16) SX_BCG(24)
#undef SX_BCG
    return x;
}
__device__ __forceinline__ double bc_chain_lds_after(double x, const Bc2 &W, const double *s_hist, int q, int sl,
                                                     bool all) {
    const int t = threadIdx.x;
    double h[8];
#define SX_BCG(S0)                                                                     \
    if (S0 < q) {                                                                      \
        _Pragma("unroll") for (int k = 0; k < 8; ++k) h[k] = s_hist[(S0 + k) * SX_TILE + t]; \
        x = bc_steps8_after<S0>(x, W, h, q, sl, all);                                  \
    }
    SX_BCG(0) SX_BCG(8) SX_BCG(16) SX_BCG(24)
#undef SX_BCG
    return x;
}
// ... of all 32 slots of a register-held history (the first stage, h1)
__device__ __forceinline__ double bc_chain_regs(double x, const Bc2 &W, const double (&h1)[SX_HMAX], int from) {
    double h[8];
#define SX_BCG(S0)                                                                     \
    _Pragma("unroll") for (int k = 0; k < 8; ++k) h[k] = h1[S0 + k];                   \
    x = bc_steps8<S0>(x, W, h, from, SX_HMAX);
    SX_BCG(0) SX_BCG(8) SX_BCG(16) SX_BCG(24)
#undef SX_BCG
    return x;
}
__device__ __forceinline__ double bc_chain_regs_after(double x, const Bc2 &W, const double (&h1)[SX_HMAX], int sl,
                                                      bool all) {
    double h[8];
#define SX_BCG(S0)                                                                     \
    _Pragma("unroll") for (int k = 0; k < 8; ++k) h[k] = h1[S0 + k];                   \
    x = bc_steps8_after<S0>(x, W, h, SX_HMAX, sl, all);
    SX_BCG(0) SX_BCG(8) SX_BCG(16) SX_BCG(24)
#undef SX_BCG
    return x;
}

// hist_col_w / stage1_col_w / hist_row / stage1_row with the broadcast steps: the same decisions
// (the leaving-row restart from U[sl] / p_sl, then the slots after sl), the same operations
__device__ __forceinline__ double hist_col_bc(double a, int q, unsigned bits, const double *s_hist, double wu,
                                              const double *s_p) {
    const Bc2 W = bc2_from_lanes(wu);
    if (__ballot(bits != 0u) == 0ull) return bc_chain_lds(a, W, s_hist, 0, q);
    const int sl = bits ? 31 - __builtin_clz(bits) : 0;  // the row's last leaving slot
    const double usl = shfl_d(wu, sl);
    if (bits) a = usl / s_p[sl];
    return bc_chain_lds_after(a, W, s_hist, q, bits ? sl : -1, !bits);
}
__device__ __forceinline__ double stage1_col_bc(double a, const double (&h)[SX_HMAX], unsigned bits, double wu,
                                                const double *s_p) {
    const Bc2 W = bc2_from_lanes(wu);
    if (__ballot(bits != 0u) == 0ull) return bc_chain_regs(a, W, h, 0);
    const int sl = bits ? 31 - __builtin_clz(bits) : 0;
    const double usl = shfl_d(wu, sl);
    if (bits) a = usl / s_p[sl];
    return bc_chain_regs_after(a, W, h, bits ? sl : -1, !bits);
}
// The multi-rank batch keeps the round-5 form of its chains: the slot value of each step read by
// v_readlane into scalar registers (lane s of a wave register holds slot s).  Its register file is
// full: with the broadcast form (two more register pairs per chain) its chain measured 0.1-0.25 us per
// pivot slower on 2..8 virtual ranks (profiles/r06_dpp_chains_ab.txt).
__device__ __forceinline__ double hist_col_rl(double a, int q, unsigned bits, const double *s_hist, const double *s_ue,
                                              const double *s_p) {
    const int t = threadIdx.x, lane = t & 63;
    const double wu = s_ue[lane & (SX_HMAX - 1)];  // lane s: U[s][e]
    if (__ballot(bits != 0u) == 0ull) {
        int s = 0;
        for (; s + 8 <= q; s += 8) {
            double h[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) h[k] = s_hist[(s + k) * SX_TILE + t];
#pragma unroll
            for (int k = 0; k < 8; ++k) a = fma(h[k], rdlane(wu, s + k), a);
        }
        for (; s < q; ++s) a = fma(s_hist[s * SX_TILE + t], rdlane(wu, s), a);
        return a;
    }
    const int sl = bits ? 31 - __builtin_clz(bits) : -1;  // the row's last leaving slot
    if (bits) a = s_ue[sl] / s_p[sl];
    for (int s0 = 0; s0 < q; s0 += 8) {  // (slots past q read slot s0 and are not used)
        double h[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) h[k] = s_hist[(s0 + k < q ? s0 + k : s0) * SX_TILE + t];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (s0 + k < q) {
                const double y = fma(h[k], rdlane(wu, s0 + k), a);
                a = s0 + k > sl ? y : a;
            }
        }
    }
    return a;
}
__device__ __forceinline__ double stage1_col_rl(double a, const double (&h)[SX_HMAX], unsigned bits, const double *s_u,
                                                const double *s_p) {
    const int lane = threadIdx.x & 63;
    const double wu = s_u[lane & (SX_HMAX - 1)];
    if (__ballot(bits != 0u) == 0ull) {
#pragma unroll
        for (int s = 0; s < SX_HMAX; ++s) a = fma(h[s], rdlane(wu, s), a);
        return a;
    }
    const int sl = bits ? 31 - __builtin_clz(bits) : -1;
    if (bits) a = s_u[sl] / s_p[sl];
#pragma unroll
    for (int s = 0; s < SX_HMAX; ++s) {
        const double y = fma(h[s], rdlane(wu, s), a);
        a = s > sl ? y : a;
    }
    return a;
}
__device__ __forceinline__ double hist_row_rl(double u, int q, int r, const double *s_hist, const double *s_fr,
                                              const double *s_p, const int *s_r) {
    const int t = threadIdx.x, lane = t & 63;
    const double wf = s_fr[lane & (SX_HMAX - 1)];  // lane s: F[r][s]
    const unsigned long long left = __ballot(lane < q && s_r[lane < q ? lane : 0] == r);
    int s = 0;
    if (left) {
        const int sl = 63 - __builtin_clzll(left);
        u = s_hist[sl * SX_TILE + t] / s_p[sl];
        s = sl + 1;
    }
    for (; s + 8 <= q; s += 8) {
        double h[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) h[k] = s_hist[(s + k) * SX_TILE + t];
#pragma unroll
        for (int k = 0; k < 8; ++k) u = fma(rdlane(wf, s + k), h[k], u);
    }
    for (; s < q; ++s) u = fma(rdlane(wf, s), s_hist[s * SX_TILE + t], u);
    return u;
}
__device__ __forceinline__ double stage1_row_rl(double u, const double (&h)[SX_HMAX], int r, const double *s_f,
                                                const double *s_p, const int *s_r) {
    const int lane = threadIdx.x & 63;
    const double wf = s_f[lane & (SX_HMAX - 1)];
    const unsigned long long left = __ballot(lane < SX_HMAX && s_r[lane < SX_HMAX ? lane : 0] == r);
    if (left == 0ull) {
#pragma unroll
        for (int s = 0; s < SX_HMAX; ++s) u = fma(rdlane(wf, s), h[s], u);
        return u;
    }
    const int sl = 63 - __builtin_clzll(left);  // (block-uniform)
    double hs = 0.0;
#pragma unroll
    for (int s = 0; s < SX_HMAX; ++s) hs = s == sl ? h[s] : hs;
    u = hs / s_p[sl];
#pragma unroll
    for (int s = 0; s < SX_HMAX; ++s) {
        const double y = fma(rdlane(wf, s), h[s], u);
        u = s > sl ? y : u;
    }
    return u;
}
__device__ __forceinline__ double hist_row_bc(double u, int q, int r, const double *s_hist, const double *s_fr,
                                              const double *s_p, const int *s_r) {
    const int t = threadIdx.x, lane = t & 63;
    const Bc2 W = bc2_from_lds(s_fr);
    const unsigned long long left = __ballot(lane < q && s_r[lane < q ? lane : 0] == r);
    int from = 0;
    if (left) {
        const int sl = 63 - __builtin_clzll(left);
        u = s_hist[sl * SX_TILE + t] / s_p[sl];
        from = sl + 1;
    }
    return bc_chain_lds(u, W, s_hist, from, q);
}
__device__ __forceinline__ double stage1_row_bc(double u, const double (&h)[SX_HMAX], int r, const double *s_f,
                                                const double *s_p, const int *s_r) {
    const int lane = threadIdx.x & 63;
    const Bc2 W = bc2_from_lds(s_f);
    const unsigned long long left = __ballot(lane < SX_HMAX && s_r[lane < SX_HMAX ? lane : 0] == r);
    if (left == 0ull) return bc_chain_regs(u, W, h, 0);
    const int sl = 63 - __builtin_clzll(left);  // (block-uniform)
    double hs = 0.0;
#pragma unroll
    for (int s1 = 0; s1 < SX_HMAX; ++s1) hs = s1 == sl ? h[s1] : hs;
    u = hs / s_p[sl];
    return bc_chain_regs(u, W, h, sl + 1);
}

// Slack compaction's bookkeeping for one batch (what k_activate does as its own launch; here
// run by the fused batch's last block, after every other block has left): when row r leaves the
// basis and an unswept slack column is the unit vector e_r -- its own slack, untouched since the
// build, or a slack that entered at row r and was moved out of the swept block since
// (k_deact_*) -- that column (ucol[r]) is exchanged with the slack column at the first unswept
// stored position s0 + nact (also a unit vector, of row urow[.]), so the swept block
// [0, s0 + nact) grows by one.  The exchanges of the batch are
// resolved in slot order by wave 0, one list entry per lane (stored offset, slack held before
// the batch, slack held now); their net effect is then applied at once: to the pending pivot
// rows U[s] (whose entries at the two columns are the leaving rows' current values there; the
// objective blocks stored them write-through, and they are read here with sc1 loads), to T
// (zeros and ones of the unit vectors) and to perm / iperm / ucol / nact.  All threads of the
// block call it; s_rr[0..cnt) are the batch's leaving rows (local = global: one shard).
__device__ void activate_block(int *__restrict__ perm, int *__restrict__ iperm, int *__restrict__ ucol,
                               const int *__restrict__ urow,
                               int *__restrict__ nact_p, int m, double *__restrict__ T, int rows, TLay tl, int s0,
                               double *__restrict__ U, size_t ld, int nU, const int *s_rr, int cnt, int *s_pl,
                               int *s_ol, int *s_cl, int *s_src, int *s_misc, double *s_u) {
    const int t = threadIdx.x;
    if (t < 64) {
        const int na0 = *nact_p;
        int kc = -1, pr = 0, win = -1;
        if (t < cnt) {
            kc = ucol[s_rr[t]];  // the unswept slack column that is e_r, if any
            pr = kc >= 0 ? perm[kc] : 0;
            if (na0 + t < m) win = iperm[na0 + t];
        }
        int pl = -1, ol = -1, cl = -1;  // this lane's list entry
        int nl = 0, added = 0;
        for (int s = 0; s < cnt; ++s) {
            const int rs = __shfl(kc, s);  // (a slack id from here on)
            if (rs < 0) continue;  // every column of the row's basic variable is swept already
            // already moved into the window in this batch?
            if (__ballot(t < nl && cl == rs && pl >= na0 && pl < na0 + added)) continue;
            const unsigned long long hP = __ballot(t < nl && cl == rs);
            int iP;
            if (hP) {
                iP = __ffsll((long long)hP) - 1;
            } else {  // untouched in this batch: at its pre-batch offset
                iP = nl++;
                const int P = __shfl(pr, s);
                if (t == iP) {
                    pl = P;
                    ol = rs;
                    cl = rs;
                }
            }
            const int pos = na0 + added;
            const unsigned long long hW = __ballot(t < nl && pl == pos);
            int iW;
            if (hW) {
                iW = __ffsll((long long)hW) - 1;
            } else {
                iW = nl++;
                const int w = __shfl(win, added);
                if (t == iW) {
                    pl = pos;
                    ol = w;
                    cl = w;
                }
            }
            const int cP = __shfl(cl, iP), cW = __shfl(cl, iW);
            if (t == iP) cl = cW;
            if (t == iW) cl = cP;
            ++added;
        }
        if (t < nl) {
            s_pl[t] = pl;
            s_ol[t] = ol;
            s_cl[t] = cl;
        }
        if (t == 0) {
            s_misc[0] = nl;
            s_misc[1] = added;
            s_misc[2] = na0;
        }
    }
    __syncthreads();
    const int nl = s_misc[0];
    if (nl == 0) return;
    if (t < nl) {  // the entry whose pre-batch slack this position holds now
        int j = 0;
        while (s_ol[j] != s_cl[t]) ++j;
        s_src[t] = j;
    }
    __syncthreads();
    for (int k = t; k < nU * nl; k += blockDim.x) {
        const int s = k / nl, i = k - s * nl;
        s_u[k] = __longlong_as_double(
            (long long)ld_sc1(reinterpret_cast<const u64 *>(U + (size_t)s * ld + s0 + s_pl[s_src[i]])));
    }
    __syncthreads();
    for (int k = t; k < nU * nl; k += blockDim.x) {
        const int s = k / nl, i = k - s * nl;
        U[(size_t)s * ld + s0 + s_pl[i]] = s_u[k];
    }
    if (t < nl) {
        const int x = s_pl[t], o = s_ol[t], cc = s_cl[t];
        if (o != cc) {  // (both unswept unit vectors before the batch: of rows urow[o], urow[cc])
            const int ro = urow[o], rc = urow[cc];
            if (ro < rows) T[tl.idx(ro, s0 + x)] = 0.0;
            if (rc < rows) T[tl.idx(rc, s0 + x)] = 1.0;
        }
        iperm[x] = cc;
        perm[cc] = x;
        const int na0 = s_misc[2];
        if (x >= na0 && x < na0 + s_misc[1]) ucol[urow[cc]] = -1;
    }
    if (t == 0) *nact_p = s_misc[2] + s_misc[1];
}

// Tile-record layouts of the fused batch (granule offsets; each value 2 granules):
//   ratio tile q      kRV v (payload: winner index, "entry >= eps" bit) | kRD d_e of pivot q |
//                     kRA a of the winner row | kRB its RHS | kRE e of pivot q | kRS status of the
//                     ratio side (NOT_ENDED, or FEASIBLE: the phase ended) | kRF F[winner][s < q]
//   objective tile q  kOV v (payload: winner index) | kOP pivot p | kOB the pivot row's RHS | kOR
//                     leaving row r | kOS status of the objective side (NOT_ENDED, UNBOUNDED,
//                     NUMERIC_FAIL) | kOM the winner's stored column (c.map) | kOU U[s <= q][winner]
[[maybe_unused]] constexpr int kRV = 0;  // (the value granules come first: rec2_a / rec2_b index them)
constexpr int kRD = 2;
constexpr int kRA = 4;
constexpr int kRB = 6;
constexpr int kRE = 8;
constexpr int kRS = 9;
constexpr int kRF = 10;
[[maybe_unused]] constexpr int kOV = 0;
constexpr int kOP = 2;
constexpr int kOB = 4;
constexpr int kOR = 6;
constexpr int kOS = 7;
constexpr int kOM = 8;
constexpr int kOU = 9;  // (odd: a history value's low word at kOU + 2s, its high word after it)

// K6: a whole batch of pivots in ONE resident launch (one shard).  Blocks [0, NA) own the
// 512-row ratio tiles, blocks [NA, NA + NB) the 512-entry objective-row tiles.  Each block
// keeps its slice of the state on chip for the whole batch: a ratio block its rows' current
// RHS and factor history F[.][s] (LDS); an objective block its columns' d values (registers)
// and pivot-row history U[s][.] (LDS).  Per pivot q, two hand-offs, each read only by the
// blocks that need it:
//   ratio blocks      form the current entering column of their rows (T[i][e] + pending
//                     pivots), the ratio vector and the tile winner (reduction.cu:106-140), and
//                     publish it with the pivot's e and d_e;
//   objective blocks  read every ratio record and run pass 2 (the leaving row r, solver.cu:
//                     96-105), take p, the RHS and F[r][s] from the winner's record, form the
//                     current pivot row on their columns, update d and reduce it per tile
//                     (solver.cu:48-56, reduction.cu:51-80), and publish that with r, p, the RHS;
//   ratio blocks      read every objective record and run pass 2 (the entering variable of
//                     pivot q + 1), take r, p, the RHS and U[s][e] from the winner's record, and
//                     apply the pivot to their rows' RHS and factor history.
// The ratio side decides the end of the phase (compare(d_e) >= 0, solver.cu:88) and tells the
// objective side through its records; the objective side decides UNBOUNDED / NUMERIC_FAIL and
// tells the ratio side through its records.  A record is tagged 8-byte granules {32 data bits,
// 32-bit tag} (MI355X_MICROARCH.md price list: handoff-1to1), each one write-through store; a
// consumer polls (sc1 loads) until every granule it needs carries the pivot's tag.  Every wait
// is bounded: past ~0.2 s the block raises abort_w and all blocks leave (status SX_HANG).  The
// last block out writes the batch's outcome -- and, with slack compaction, does the batch's
// column activation (activate_block) -- so no launch sits between the batch and its sweep.  The
// grid is launched only when all its blocks are resident at once (sx_batch_fits).
__global__ __launch_bounds__(512) void k_batch(const double *T, int rows, size_t ld, TLay tl, Cols c,
                                               double *__restrict__ d, double *__restrict__ d_save, int *base,
                                               DevState *st, double *U, double *F, PivRec *recs,
                                               unsigned long long *PM, unsigned long long *PM2, unsigned B, int K,
                                               int NA, int NB,
                                               BatchChan *ch, u64 *ga, u64 *gb, unsigned long long *stamps,
                                               int *perm, int *iperm, int *ucol, const int *urow, int *nact, int m) {
    extern __shared__ double s_hist[];  // [stage slots][512]: F history (ratio blocks) / U history (objective blocks)
    __shared__ double s_v[16];
    __shared__ int s_i[16];
    __shared__ double s_p[SX_KMAX];                  // pivots of the batch
    __shared__ int s_r[SX_KMAX], s_e[SX_KMAX];       // leaving rows / entering variables of the batch
    __shared__ double s_fr[SX_HMAX], s_fr1[SX_HMAX];  // F[r][s] (leaving row), this stage / the first stage's slots
    __shared__ double s_a[SX_TILE], s_b[SX_TILE];    // ratio blocks: entering column, RHS (winner lookup)
    __shared__ unsigned s_g[4 * SX_TILE];            // gathered granules
    __shared__ unsigned s_pay[SX_TILE];              // their payloads (two-granule records)
    __shared__ unsigned short s_payo[3 * SX_OBJ_TILES];  // payloads of the objective records' granules 0..2
    __shared__ double s_uq;                          // the entering column's pivot-row value of this pivot
    __shared__ int s_last;
    // per-step results written by wave 0 before the step's one barrier (each step its own
    // words, so no wave still reading an earlier step's result can see them change)
    __shared__ int s_sel_ok, s_sel_r, s_sel_any, s_det_ok, s_det_e, s_det_st, s_ent_ok, s_ent_e, s_ent_m;
    __shared__ double s_det_dmin, s_ent_v, s_br, s_ent_p;
    __shared__ int s_welig[SX_TILE / 64];
    __shared__ int s_okw[SX_TILE / 64];
    const int t = threadIdx.x;
    const bool isA = (int)blockIdx.x < NA;
    // stamps (diagnostic, normally null): s_memrealtime (100 MHz) at hand-off points of ratio
    // block 0 and objective block 0, [q][8]
#define SX_STAMP(k)                                                                           \
    do {                                                                                       \
        if (stamps && t == 0) stamps[(size_t)q * 8 + (k)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
    // ... and every block's own, after the [K][8] block: [q][block][4] (ratio: compute start,
    // publish, entering seen; objective: selection seen, details in, publish)
#define SX_BSTAMP(k)                                                                                    \
    do {                                                                                                \
        if (stamps && t == 0)                                                                           \
            stamps[(size_t)K * 8 + ((size_t)q * (NA + NB) + blockIdx.x) * 4 + (k)] =                    \
                __builtin_amdgcn_s_memrealtime();                                                       \
    } while (0)
    // state at the start of the batch (written only by the last block to leave)
    const int status0 = st->status;
    const long long piv0 = st->pivots, cap = st->max_pivots;
    int e = st->e_next;
    double dmin = st->dmin_next;
    int status = SX_NOT_ENDED, cnt = 0;
    bool aborted = false;
    const unsigned inj = ch->inject_q;  // (test hook, normally 0)
    if (status0 == SX_NOT_ENDED) {
        // ratio block: its row; objective block: its logical column d[1 + ia]
        const int li = blockIdx.x * SX_TILE + t;
        const bool liveA = isA && li < rows;
        const int tb = blockIdx.x - NA;
        const int L = c.N - 1;
        const int ia = tb * SX_TILE + t;
        const bool liveB = !isA && ia < L;
        const int mj = c.map(1 + (liveB ? ia : 0));
        // (objective blocks: every column's stored position, for the record of the tile winner)
        if (!isA) reinterpret_cast<int *>(s_a)[t] = mj;
        double b = liveA ? T[tl.idx(li, 0)] : 0.0;  // current RHS of the row
        unsigned bits = 0u;                            // slots of this stage where this row left the basis
        unsigned bits1 = 0u;                           // ... of the first stage (second stage)
        double h1[SX_HMAX];                            // this thread's first-stage history (second stage)
#pragma unroll
        for (int s1 = 0; s1 < SX_HMAX; ++s1) h1[s1] = 0.0;
        int hb = 0;                                    // first slot of the current stage
        double dj = liveB ? d[1 + ia] : 0.0;
        double d0 = (!isA && tb == 0 && t == 0) ? d[0] : 0.0;
        // the objective row as the batch found it, for the host to restore when the batch is
        // aborted (SX_HANG): saved by the very thread that writes the entry at the end
        if (liveB) d_save[1 + ia] = dj;
        if (!isA && tb == 0 && t == 0) d_save[0] = d0;
        // the entering column's stored value of this row: loaded as soon as the entering
        // variable is known, so the load overlaps the wait for its pending history
        double a_pre = liveA ? T[tl.idx(li, c.map(1 + (e >= 0 ? e : 0)))] : 0.0;
        // the stage switch at slot SX_HMAX: this thread's first-stage history to registers, the
        // LDS history reused.  The block's first-stage F / U stores are written back from its L2
        // (every thread's stores acknowledged, then one agent-scope release: buffer_wbl2) before
        // any second-stage record of the block, so a block that reads one of them with sc1 loads
        // (the leaving row's F, the entering column's U) after that record sees them
        auto next_stage = [&]() {
#pragma unroll
            for (int s1 = 0; s1 < SX_HMAX; ++s1) h1[s1] = s_hist[s1 * SX_TILE + t];
            bits1 = bits;
            bits = 0u;
            drain();
            __syncthreads();
            if (t == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            __syncthreads();
            hb = SX_HMAX;
        };
        // The two roles run separate loops (the same steps per pivot), so the compiler's memory
        // counter waits on one role's path never cover the other role's loads.  Per pivot q: does
        // the phase end here (the pivot cap: the same decision in every block), the stage switch.
        if (isA) {
            // the entering column's pending pivot-row values, one register per wave (lane s: U[hb + s][e]
            // of the current stage; wu1: U[s][e] of the first stage), loaded by every wave with the
            // column's stored values (the fresh slot from the objective record)
            double wu = 0.0, wu1 = 0.0;
            for (int q = 0; q < K; ++q) {
                const unsigned tag = make_tag(B, q);
                if (cap >= 0 && piv0 + q >= cap) {
                    status = SX_PIVOT_CAP;
                    break;
                }
                if (q == SX_HMAX) next_stage();
                if (inj != 0u && blockIdx.x == 0 && (unsigned)q + 1u == inj) {  // test hook: leave, aborted
                    if (t == 0) __hip_atomic_store(&ch->abort_w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    aborted = true;
                    break;
                }
                const int qq = q - hb;  // slot within the stage
                const bool done = !(cmp_eps(dmin, 0.0) < 0);  // solver.cu:88: optimal
                // ---- ratio tile: current entering column, ratios, tile winner
                if (blockIdx.x == 0) SX_STAMP(0);
                SX_BSTAMP(0);
                double a1 = a_pre;
                if (hb && !done) a1 = stage1_col_bc(a1, h1, bits1, wu1, s_p);
                const double a = done ? 0.0 : hist_col_bc(a1, qq, bits, s_hist, wu, s_p + hb);
                double rv = DBL_MAX;
                int ri = -1, elig = 0;
                if (liveA && !done) {
                    elig = a >= SX_EPS;
                    const double ratio = cmp_eps(a, 0.0) > 0 ? b / a : DBL_MAX;  // reduction.cu:106-114
                    if (cmp_eps(ratio, rv) < 0) {
                        rv = ratio;
                        ri = li;
                    }
                }
                if (blockIdx.x == 0) SX_STAMP(2);
                s_a[t] = a;
                s_b[t] = b;
                // (every wave's F store of the previous pivot acknowledged before this pivot's record:
                // the objective side reads F[r][s < q] from memory after seeing it)
                drain();
                // pass 1 (reduction.cu:51-80): every half-wave its tree, one block barrier, then
                // wave 0 combines the 16 half winners (block_argmin512's second step) and
                // publishes the record alone
                half_argmin(rv, ri);
                const int anyw = __ballot(elig) != 0ull;
                if ((t & 31) == 0) {
                    s_v[t >> 5] = rv;
                    s_i[t >> 5] = ri;
                }
                if ((t & 63) == 0) s_welig[t >> 6] = anyw;
                __syncthreads();
                if (t < 64) {
                    double v = t < 16 ? s_v[t] : DBL_MAX;
                    int i = t < 16 ? s_i[t] : -1;
                    half_argmin(v, i);
                    int any = 0;
#pragma unroll
                    for (int w = 0; w < SX_TILE / 64; ++w) any |= s_welig[w];
                    const int wi = __builtin_amdgcn_readfirstlane(i);
                    const long long vb = __double_as_longlong(v);
                    const double wv = __longlong_as_double(
                        ((long long)__builtin_amdgcn_readfirstlane((int)(vb >> 32)) << 32) |
                        (long long)(unsigned)__builtin_amdgcn_readfirstlane((int)vb));
                    const int wl = wi >= 0 ? wi - (int)blockIdx.x * SX_TILE : 0;
                    const unsigned pl = (wi >= 0 ? (unsigned)wl : SX_NOIDX) | ((unsigned)any << 10);
                    const int nG = kRF + 2 * qq;
                    for (int k = t; k < nG; k += 64) {
                        unsigned data;
                        if (k == kRE) {
                            data = (unsigned)e;
                        } else if (k == kRS) {
                            data = (unsigned)(done ? SX_FEASIBLE : SX_NOT_ENDED);
                        } else {
                            const double val = k < kRD ? wv : k < kRA ? dmin : k < kRB ? s_a[wl] : k < kRE ? s_b[wl]
                                                                           : s_hist[((k - kRF) >> 1) * SX_TILE + wl];
                            const u64 bits64 = (u64)__double_as_longlong(val);
                            data = (k & 1) ? (unsigned)(bits64 >> 32) : (unsigned)bits64;
                        }
                        put_g(ga + (size_t)blockIdx.x * SX_GA_STRIDE + k, data, k < kRD ? (tag | pl) : tag);
                    }
                }
                if (blockIdx.x == 0) SX_STAMP(1);
                SX_BSTAMP(1);
                if (done) {
                    status = SX_FEASIBLE;
                    break;
                }
                // ---- this pivot's leaving row, from the ratio records (every ratio block runs the pass 2
                // the objective blocks run, reduction.cu:116-140, and takes p and the RHS from the
                // winner's record): the objective side answers much later, so this is off the chain
                if (t < 64) {
                    int ok = poll_wave(ga, 2 * NA, rec2_a, tag, s_g, &ch->abort_w, 20000000ull, s_pay);
                    double tv = DBL_MAX;
                    int ti = -1, any = 0;
                    if (ok) wave_pass2(s_g, s_pay, NA, s_v, s_i, tv, ti, any);
                    ti = __builtin_amdgcn_readfirstlane(ti);
                    if (ok && ti >= 0) {
                        const int wt = ti / SX_TILE;
                        ok = poll_wave(ga + (size_t)wt * SX_GA_STRIDE + kRA, 4, IdOff(), tag, s_g + 2048 - 64,
                                       &ch->abort_w, 20000000ull, (unsigned *)nullptr);
                    }
                    if (t == 0) {
                        s_sel_ok = ok;
                        s_sel_r = ti;
                        s_sel_any = any;
                        if (ok && ti >= 0) {
                            s_ent_p = gd(s_g[2048 - 64], s_g[2048 - 63]);
                            s_br = gd(s_g[2048 - 62], s_g[2048 - 61]);
                        }
                    }
                }
                __syncthreads();
                if (!s_sel_ok) {
                    aborted = true;
                    break;
                }
                if (!s_sel_any) {  // solver.cu:96-102 (the objective side decides the same)
                    status = SX_UNBOUNDED;
                    break;
                }
                const int r = s_sel_r;
                if (r < 0) {
                    status = SX_NUMERIC_FAIL;
                    break;
                }
                // ---- this pivot's factor column and the rows' new RHS (solver.cu:34-46)
                const double p = s_ent_p, br = s_br;
                if (t == 0) {
                    s_p[q] = p;
                    s_r[q] = r;
                    s_e[q] = e;
                }
                cnt = q + 1;
                const double f = -a / p;
                s_hist[qq * SX_TILE + t] = f;
                if (liveA) {
                    st_sc1(F + sx_fidx(li, q), f);  // (write-through: read by the objective side from memory)
                    if (li == r) {
                        b = b / p;
                        bits |= 1u << qq;
                        // (the row's slots of this stage are `bits`: the word is written, not
                        // read-modified, so no load waits behind the entering column's)
                        (hb ? PM2 : PM)[li] = ((u64)B << 32) | bits;
                    } else {
                        b = fma(f, br, b);
                    }
                }
                if (blockIdx.x == 0 && t == 0) {  // (base[r] = e, solver.cu:105: at the end of the batch)
                    recs[q].r = r;
                    recs[q].e = e;
                    recs[q].p = p;
                    U[(size_t)q * ld] = br;  // the pivot row's RHS entry, for the sweep
                }
                // ---- the objective side's answer: pass 2 over the objective tiles (the entering variable
                // of pivot q + 1), its stored column and its pivot-row entry of this pivot from the
                // winner's record.  Every wave polls an eighth of the records (poll_block: 3.18 -> 2.46 us
                // for this hop at config 5 against wave 0 alone, profiles/r06_poll_waves_ab.txt), then
                // wave 0 runs pass 2; two block barriers.  (The ratio records -- 2 granules per tile,
                // at most 2 per lane of one wave -- stay polled by wave 0: the second barrier cost more
                // than the split saved, config 3 ratio->objective hop 1.12 -> 1.40 us.)
                unsigned short *po = s_payo;
                const int okb = poll_block(gb, SX_GB4 * NB, SX_GB4, Rec4All(), tag, s_g, &ch->abort_w, 20000000ull,
                                           [po](int k, unsigned pl) {
                                               if ((k & 3) < 3) po[(k & 3) * SX_OBJ_TILES + (k >> 2)] = (unsigned short)pl;
                                           }, s_okw);
                if (t < 64) {
                    double ev = DBL_MAX;
                    int ei = -1, any = 0;
                    if (okb) wave_pass2<SX_GB4, unsigned short>(s_g, s_payo, NB, s_v, s_i, ev, ei, any);
                    if (t == 0) {
                        s_ent_ok = okb;
                        s_ent_e = ei;
                        s_ent_v = ev;
                        s_ent_m = 0;
                        s_uq = 0.0;
                        if (okb && ei >= 0) {
                            const int wt = ei / SX_TILE;
                            s_ent_m = (int)s_payo[SX_OBJ_TILES + wt] | ((int)s_payo[2 * SX_OBJ_TILES + wt] << SX_PAYBITS);
                            s_uq = gd(s_g[SX_GB4 * wt + 2], s_g[SX_GB4 * wt + 3]);
                        }
                    }
                }
                __syncthreads();
                if (blockIdx.x == 0) SX_STAMP(5);
                SX_BSTAMP(2);
                if (!s_ent_ok) {
                    aborted = true;
                    break;
                }
                e = s_ent_e;
                dmin = s_ent_v;
                // the next pivot's operands, issued together: this row's stored value of the entering
                // column and (every wave) the column's pending pivot-row values U[s][e] -- U[q][e] from
                // the record, the older ones from memory (write-through, acknowledged before their
                // objective records)
                {
                    const int me = s_ent_m, lane = t & 63, q1 = q + 1, hb1 = q1 >= SX_HMAX ? SX_HMAX : 0;
                    const double uq = s_uq;
                    if (liveA) a_pre = T[tl.idx(li, me)];
                    const int sa = hb1 + lane;
                    wu = lane < q1 - hb1 ? (sa == q ? uq : ld_sc1d(U + (size_t)sa * ld + me)) : 0.0;
                    if (hb1) wu1 = lane < SX_HMAX ? (lane == q ? uq : ld_sc1d(U + (size_t)lane * ld + me)) : 0.0;
                }
            }
        } else {
            for (int q = 0; q < K; ++q) {
                const unsigned tag = make_tag(B, q);
                if (cap >= 0 && piv0 + q >= cap) {
                    status = SX_PIVOT_CAP;
                    break;
                }
                if (q == SX_HMAX) next_stage();
                const int qq = q - hb;  // slot within the stage
                // ---- selection: pass 2 over the ratio tiles (wave 0 polls and runs the tree)
                if (t < 64) {
                    const int ok = poll_wave(ga, 2 * NA, rec2_a, tag, s_g, &ch->abort_w, 20000000ull, s_pay);
                    double tv = DBL_MAX;
                    int ti = -1, any = 0;
                    if (ok) wave_pass2(s_g, s_pay, NA, s_v, s_i, tv, ti, any);
                    if (t == 0) {
                        s_sel_ok = ok;
                        s_sel_r = ti;
                        s_sel_any = any;
                    }
                }
                __syncthreads();
                if (tb == 0) SX_STAMP(3);
                SX_BSTAMP(0);
                if (!s_sel_ok) {
                    aborted = true;
                    break;
                }
                const int r = s_sel_r;
                // the pivot-row load does not wait for the winner's details
                double u = liveB && r >= 0 ? T[tl.idx(r, mj)] : 0.0;
                // the winner's record (the ratio tile 0's when there is none): d_e, p, the RHS,
                // e, the ratio side's status and F[r][s < q], read by wave 0 into LDS
                if (t < 64) {
                    const int wt = r >= 0 ? r / SX_TILE : 0;
                    // second stage: the leaving row's first-stage factors F[r][s] (write-through,
                    // drained at the stage switch), loaded while the record is polled
                    u64 fr1 = 0ull;
                    if (hb && t < SX_HMAX)
                        fr1 = ld_sc1(reinterpret_cast<const u64 *>(F + sx_fidx(r >= 0 ? r : 0, t)));
                    const int ok = poll_wave(ga + (size_t)wt * SX_GA_STRIDE + kRD, (kRF - kRD) + 2 * qq,
                                             [](int k) { return k; }, tag, s_g, &ch->abort_w, 20000000ull,
                                             (unsigned *)nullptr);
                    if (hb && t < SX_HMAX) s_fr1[t] = __longlong_as_double((long long)fr1);
                    if (ok) {
                        if (t < qq) s_fr[t] = gd(s_g[kRF - kRD + 2 * t], s_g[kRF - kRD + 1 + 2 * t]);
                        if (t == 0) {
                            s_det_dmin = gd(s_g[0], s_g[1]);
                            s_p[q] = gd(s_g[kRA - kRD], s_g[kRA - kRD + 1]);
                            s_br = gd(s_g[kRB - kRD], s_g[kRB - kRD + 1]);
                            s_det_e = (int)s_g[kRE - kRD];
                            s_det_st = (int)s_g[kRS - kRD];
                            s_r[q] = r;
                            s_e[q] = (int)s_g[kRE - kRD];
                        }
                    }
                    if (t == 0) s_det_ok = ok;
                }
                __syncthreads();
                SX_BSTAMP(1);
                if (!s_det_ok) {
                    aborted = true;
                    break;
                }
                e = s_det_e;
                dmin = s_det_dmin;
                int ost = SX_NOT_ENDED;
                if (s_det_st != SX_NOT_ENDED) {  // the ratio side ended the phase (optimal)
                    status = s_det_st;
                    break;
                }
                if (!s_sel_any) {
                    ost = SX_UNBOUNDED;  // solver.cu:96-102
                } else if (r < 0) {
                    ost = SX_NUMERIC_FAIL;
                }
                const double p = s_p[q], br = s_br;
                double v = DBL_MAX;
                int i = -1;
                if (ost == SX_NOT_ENDED) {
                    cnt = q + 1;
                    // ---- objective tile: current pivot row on this column, d, tile winner
                    if (tb == 0) SX_STAMP(6);
                    if (hb) u = stage1_row_bc(u, h1, r, s_fr1, s_p, s_r);
                    u = hist_row_bc(u, qq, r, s_hist, s_fr, s_p + hb, s_r + hb);
                    s_hist[qq * SX_TILE + t] = u;
                    if (tb == 0) SX_STAMP(7);
                    const double fd = -dmin / p;  // updateCostsVector, solver.cu:48-56
                    if (tb == 0 && t == 0) d0 = fma(fd, br, d0);
                    if (liveB) {
                        dj = fma(fd, u, dj);
                        if (cmp_eps(dj, v) < 0) {
                            v = dj;
                            i = ia;
                        }
                    }
                }
                // pass 1 (reduction.cu:51-80): half-wave trees, one block barrier, wave 0 combines
                // the half winners and publishes the record alone.  (Every wave's U store of the
                // previous pivot is acknowledged first: the ratio side reads U[s < q] from memory
                // after seeing this record.)
                half_argmin(v, i);
                if ((t & 31) == 0) {
                    s_v[t >> 5] = v;
                    s_i[t >> 5] = i;
                }
                drain();
                __syncthreads();
                if (t < 64) {
                    double wv = t < 16 ? s_v[t] : DBL_MAX;
                    int wi = t < 16 ? s_i[t] : -1;
                    half_argmin(wv, wi);
                    wi = __builtin_amdgcn_readfirstlane(wi);
                    const long long vb = __double_as_longlong(wv);
                    wv = __longlong_as_double(((long long)__builtin_amdgcn_readfirstlane((int)(vb >> 32)) << 32) |
                                              (long long)(unsigned)__builtin_amdgcn_readfirstlane((int)vb));
                    const int win = wi >= 0 ? wi - tb * SX_TILE : 0;
                    // the record: the winner's d value (payload: its index in the tile) and its pivot-row
                    // value of this pivot U[q][w] (the ratio side's newest pending entry of the entering
                    // column if w enters), the winner's stored column in the payloads of granules 1, 2
                    if (t < SX_GB4) {
                        const int k = t;
                        const int mw = reinterpret_cast<const int *>(s_a)[win];
                        const double val = k < 2 ? wv : s_hist[qq * SX_TILE + win];
                        const u64 bits64 = (u64)__double_as_longlong(val);
                        const unsigned data = (k & 1) ? (unsigned)(bits64 >> 32) : (unsigned)bits64;
                        const unsigned pl = k == 0 ? (wi >= 0 ? (unsigned)win : SX_NOIDX)
                                          : k == 1 ? ((unsigned)mw & SX_PAYMASK)
                                          : k == 2 ? (((unsigned)mw >> SX_PAYBITS) & SX_PAYMASK) : 0u;
                        put_g(gb + (size_t)tb * SX_GBS + k, data, tag | pl);
                    }
                }
                // the pivot row into U[q] (the sweep's input, and the ratio side's pending entries of
                // later entering columns) behind the record, write-through
                if (ost == SX_NOT_ENDED && liveB && 1 + ia < c.Ns) st_sc1(U + (size_t)q * ld + mj, s_hist[qq * SX_TILE + t]);
                if (tb == 0) SX_STAMP(4);
                SX_BSTAMP(2);
                if (ost != SX_NOT_ENDED) {
                    status = ost;
                    break;
                }
            }
        }
        // a batch that ended without a decision of the ratio side (all K pivots ran, or the pivot
        // cap): the objective blocks learn the next entering variable, which only the ratio side
        // computed, from the last objective records
        if (!isA && !aborted && (status == SX_NOT_ENDED || status == SX_PIVOT_CAP) && cnt > 0) {
            const unsigned tag = make_tag(B, cnt - 1);
            if (t < 64) {
                const int ok = poll_wave(gb, 2 * NB, Rec4Val(), tag, s_g, &ch->abort_w, 20000000ull, s_pay);
                double ev = DBL_MAX;
                int ei = -1, any = 0;
                if (ok) wave_pass2(s_g, s_pay, NB, s_v, s_i, ev, ei, any);
                if (t == 0) {
                    s_ent_ok = ok;
                    s_ent_e = ei;
                    s_ent_v = ev;
                }
            }
            __syncthreads();
            if (!s_ent_ok) aborted = true;
            e = s_ent_e;
            dmin = s_ent_v;
        }
        if (liveB) d[1 + ia] = dj;
        if (!isA && tb == 0 && t == 0) d[0] = d0;
    }
    // leave; the last block out writes the batch's outcome into the state (every block holds
    // the same outcome) and activates the batch's slack columns (every block's U stores were
    // write-through and drained before its arrival; the last block reads them with sc1 loads)
    drain();
    __syncthreads();
    if (t == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // (the block's U stores out of its L2)
        const unsigned k = __hip_atomic_fetch_add(&ch->exit_cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = k == (unsigned)(NA + NB) - 1;
        if (s_last) {
            __hip_atomic_store(&ch->exit_cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (inj != 0u) ch->inject_q = 0u;  // (every block read it at its start)
        }
    }
    __syncthreads();
    if (!s_last || status0 != SX_NOT_ENDED) return;
    const bool hang = ld_sc1(&ch->abort_w) != 0u || aborted;
    if (!hang && perm != nullptr && cnt > 0) {
        // one stage at a time (a list entry per lane): the exchanges of the first stage's slots,
        // then of the second's from the state the first left -- the same exchanges in slot order;
        // each swaps the entries of all the batch's pending rows U[s]
        for (int s1 = 0; s1 < cnt; s1 += SX_HMAX) {
            if (s1) __syncthreads();
            activate_block(perm, iperm, ucol, urow, nact, m, const_cast<double *>(T), rows, tl, c.s0, U, ld, cnt, s_r + s1,
                           cnt - s1 < SX_HMAX ? cnt - s1 : SX_HMAX, reinterpret_cast<int *>(s_g),
                           reinterpret_cast<int *>(s_g) + 64, reinterpret_cast<int *>(s_g) + 128,
                           reinterpret_cast<int *>(s_g) + 192, reinterpret_cast<int *>(s_pay), s_hist);
        }
    }
    if (t != 0) return;
    if (hang) {
        st->status = SX_HANG;
        __hip_atomic_store(&ch->abort_w, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    // base[r] = e of every pivot, in order (solver.cu:105), only for a batch that completed
    for (int s = 0; s < cnt; ++s) base[s_r[s]] = s_e[s];
    st->status = status;
    st->pivots = piv0 + cnt;
    if (cnt > 0) {
        st->r = s_r[cnt - 1];
        st->e = s_e[cnt - 1];
        st->batch_tag = B;
        st->batch_count = cnt;
    }
    st->e_next = e;
    st->dmin_next = dmin;
#undef SX_STAMP
#undef SX_BSTAMP
}


// ---------------------------------------------------------------------------------------
// K7: the fused batch on W row-block shards (one per GPU, or virtual shards on one GPU),
// exchanging over peer memory (xGMI) inside the launch instead of RCCL calls between
// launches.  Rank k runs `slots` ratio tiles (its rows) and the objective tiles [tb0, tb1)
// of the logical row (the objective work is split across ranks; every rank still gets every
// decision).  The hand-offs are k_batch's, each read only by the blocks that need it:
//   ratio tiles       as k_batch; each tile winner (+ the winning row's factor history, the
//                     pivot's e and d_e) is written as tagged granules into EVERY rank's
//                     ga[global tile];
//   objective tiles   read all W * slots ratio records from their own ga and run pass 2, read
//                     the leaving row's stored values straight from its owner's tableau (remote
//                     loads), form the current pivot row on their columns, write it into every
//                     rank's U[q] (the sweep's input), update their d slice, and publish the
//                     tile winner (+ the winning column's pivot-row history, r, p, the RHS) into
//                     every rank's gb;
//   ratio tiles       read all objective records from their own gb and run pass 2 (the next
//                     entering variable), and apply the pivot to their rows.
// Between batches every rank keeps only its own slice of d current (Engine::gather_d).
// Replicated objective (repl): every rank runs ALL the objective tiles
// (tb0 = 0, tb1 = NBg) on its own copy of d, writes their records into its own gb and the pivot
// row into its own U only -- the ratio records and the leaving row's remote reads stay the only
// cross-rank traffic of a pivot, and every rank's d stays whole.  At the
// end of the batch a done granule per rank: a rank's last block leaves only when every rank's
// data has landed, so the sweep that follows reads complete U.  Cross-rank stores and loads are
// system-scope (sc0 sc1); the records polled across GPUs are uncached allocations.  The same
// arithmetic, trees and order as k_batch.
__device__ __forceinline__ void put_g_sys(u64 *g, unsigned data, unsigned tag) {
    __hip_atomic_store(g, ((u64)tag << 32) | data, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(double *p, double v) {
    __hip_atomic_store(reinterpret_cast<u64 *>(p), (u64)__double_as_longlong(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ double ld_sys(const double *p) {
    return __longlong_as_double((long long)ld_sys(reinterpret_cast<const u64 *>(p)));
}

__device__ __forceinline__ void batch_mr_body(int bid, unsigned nbl, const double *__restrict__ T, int rows, int row0,
                                              int rpr, size_t ld, TLay tl, Cols c, double *__restrict__ d,
                                              double *__restrict__ d_save, int *base, DevState *st, double *U, double *F,
                                              PivRec *recs, unsigned long long *PM, unsigned long long *PM2, unsigned B,
                                              int K, int slots, int W,
                                              int rank, int tb0, int tb1, int NBg, int repl, BatchChan *ch,
                                              const u64 *ga, const u64 *gb, const u64 *gdone, PeerView pv,
                                              unsigned long long timeout) {
    extern __shared__ double s_hist[];  // [K][512]: F history (ratio tiles) / U history (objective tiles)
    __shared__ double s_v[16];
    __shared__ int s_i[16];
    __shared__ double s_p[SX_KMAX];
    __shared__ int s_r[SX_KMAX], s_e[SX_KMAX];
    __shared__ double s_ue[SX_KMAX], s_fr[SX_KMAX];
    __shared__ double s_ue1[SX_HMAX], s_fr1[SX_HMAX];  // the first stage's U[s][e] / F[r][s] (second stage)
    __shared__ double s_a[SX_TILE], s_b[SX_TILE];
    __shared__ unsigned s_g[4 * SX_TILE];
    __shared__ unsigned s_pay[SX_TILE];
    __shared__ int s_ok, s_flag;
    // per-step results written by wave 0 before the step's one barrier (as in k_batch)
    __shared__ int s_sel_ok, s_sel_r, s_sel_any, s_det_ok, s_det_e, s_det_st, s_ent_ok, s_ent_e, s_ent_r, s_ent_st, s_ent_m;
    __shared__ double s_det_dmin, s_ent_v, s_br, s_ent_p;
    __shared__ int s_welig[SX_TILE / 64];
    const int t = threadIdx.x;
    const bool isA = bid < slots;
    const int NAg = W * slots;
    const int status0 = st->status;
    const long long piv0 = st->pivots, cap = st->max_pivots;
    int e = st->e_next;
    double dmin = st->dmin_next;
    int status = SX_NOT_ENDED, cnt = 0;
    bool aborted = false;
    const unsigned inj = ch->inject_q;  // (test hook, normally 0)
    auto gather_a = [](int k) { return rec2_a(k); };
    auto gather_b = [](int k) { return rec2_b(k); };
    auto ident = [](int k) { return k; };
    const int li = bid * SX_TILE + t;
    const bool liveA = isA && li < rows;
    const int gt = rank * slots + bid;  // global ratio tile of this block
    const int tb = tb0 + bid - slots;   // objective tile of this block
    const int L = c.N - 1;
    const int ia = tb * SX_TILE + t;
    const bool liveB = !isA && ia < L;
    const int mj = c.map(1 + (liveB ? ia : 0));
    if (!isA) reinterpret_cast<int *>(s_a)[t] = mj;  // (as k_batch)
    double dj = liveB ? d[1 + ia] : 0.0;
    double d0 = (!isA && tb == 0 && t == 0) ? d[0] : 0.0;
    if (status0 == SX_NOT_ENDED) {
        // this rank's slice of the objective row as the batch found it (restored by the host on
        // SX_HANG), saved by the very thread that writes the entry at the end
        if (liveB) d_save[1 + ia] = dj;
        if (!isA && tb == 0 && t == 0) d_save[0] = d0;
        double b = liveA ? T[tl.idx(li, 0)] : 0.0;
        unsigned bits = 0u;   // slots of this stage where this row left the basis
        unsigned bits1 = 0u;  // ... of the first stage (second stage)
        double h1[SX_HMAX];   // this thread's first-stage history (second stage)
#pragma unroll
        for (int s1 = 0; s1 < SX_HMAX; ++s1) h1[s1] = 0.0;
        int hb = 0;  // first slot of the current stage
        // the entering column's stored value of this row: loaded as soon as the entering
        // variable is known, so the load overlaps the wait for its pending history
        double a_pre = liveA ? T[tl.idx(li, c.map(1 + (e >= 0 ? e : 0)))] : 0.0;
        // The two roles run separate loops (the same steps per pivot, as k_batch), so neither
        // role's registers are held across the other's code.
        if (isA) {
            for (int q = 0; q < K; ++q) {
                const unsigned tag = make_tag(B, q);
                if (cap >= 0 && piv0 + q >= cap) {
                    status = SX_PIVOT_CAP;
                    break;
                }
                if (inj != 0u && isA && rank == 0 && bid == 0 && (unsigned)q + 1u == inj) {  // test hook
                    if (t == 0) __hip_atomic_store(&ch->abort_w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    aborted = true;
                    break;
                }
                if (q == SX_HMAX) {
                    // the stage switch (k_batch's, at system scope): this thread's first-stage history
                    // to registers, the LDS history reused.  Every thread's stores acknowledged -- the
                    // objective tiles' U rows (write-through into every rank), the ratio tiles' F --
                    // then one system-scope release writes this device's L2 back, before any
                    // second-stage record: a block that has seen one reads the first stage's U[s][e]
                    // (its own rank's U) and F[r][s] (the owner's F) with system-scope loads
    #pragma unroll
                    for (int s1 = 0; s1 < SX_HMAX; ++s1) h1[s1] = s_hist[s1 * SX_TILE + t];
                    bits1 = bits;
                    bits = 0u;
                    if (t < SX_HMAX) s_ue1[t] = s_ue[t];  // (U[s][e] of pivot SX_HMAX: its objective record)
                    drain();
                    __syncthreads();
                    if (t == 0) {
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
                        drain();
                    }
                    __syncthreads();
                    hb = SX_HMAX;
                }
                const int qq = q - hb;  // slot within the stage
                const bool done = !(cmp_eps(dmin, 0.0) < 0);  // solver.cu:88: optimal
                double a1 = a_pre;
                if (hb && !done) a1 = stage1_col_rl(a1, h1, bits1, s_ue1, s_p);
                const double a = done ? 0.0 : hist_col_rl(a1, qq, bits, s_hist, s_ue, s_p + hb);
                double rv = DBL_MAX;
                int ri = -1, elig = 0;
                if (liveA && !done) {
                    elig = a >= SX_EPS;
                    const double ratio = cmp_eps(a, 0.0) > 0 ? b / a : DBL_MAX;  // reduction.cu:106-114
                    if (cmp_eps(ratio, rv) < 0) {
                        rv = ratio;
                        ri = row0 + li;
                    }
                }
                s_a[t] = a;
                s_b[t] = b;
                // pass 1: half-wave trees, one block barrier, wave 0 combines and publishes (k_batch)
                half_argmin(rv, ri);
                const int anyw = __ballot(elig) != 0ull;
                if ((t & 31) == 0) {
                    s_v[t >> 5] = rv;
                    s_i[t >> 5] = ri;
                }
                if ((t & 63) == 0) s_welig[t >> 6] = anyw;
                __syncthreads();
                if (t < 64) {
                    double wv = t < 16 ? s_v[t] : DBL_MAX;
                    int wi = t < 16 ? s_i[t] : -1;
                    half_argmin(wv, wi);
                    int any = 0;
#pragma unroll
                    for (int w = 0; w < SX_TILE / 64; ++w) any |= s_welig[w];
                    wi = __builtin_amdgcn_readfirstlane(wi);
                    const long long vb = __double_as_longlong(wv);
                    wv = __longlong_as_double(((long long)__builtin_amdgcn_readfirstlane((int)(vb >> 32)) << 32) |
                                              (long long)(unsigned)__builtin_amdgcn_readfirstlane((int)vb));
                    const int wl = wi >= 0 ? wi - row0 - bid * SX_TILE : 0;
                    // the record into every rank's copy
                    const unsigned pl = (wi >= 0 ? (unsigned)(wi - gt * SX_TILE) : SX_NOIDX) | ((unsigned)any << 10);
                    // granule-major over the ranks: the value granules reach every rank first
                    const int nG = kRF + 2 * qq;
                    for (int idx = t; idx < W * nG; idx += 64) {
                        const int k = idx / W, rk = idx - k * W;
                        unsigned data;
                        if (k == kRE) {
                            data = (unsigned)e;
                        } else if (k == kRS) {
                            data = (unsigned)(done ? SX_FEASIBLE : SX_NOT_ENDED);
                        } else {
                            const double val = k < kRD ? wv : k < kRA ? dmin : k < kRB ? s_a[wl] : k < kRE ? s_b[wl]
                                                                           : s_hist[((k - kRF) >> 1) * SX_TILE + wl];
                            const u64 bits64 = (u64)__double_as_longlong(val);
                            data = (k & 1) ? (unsigned)(bits64 >> 32) : (unsigned)bits64;
                        }
                        put_g_sys(pv.ga[rk] + (size_t)gt * SX_GA_STRIDE + k, data, k < kRD ? (tag | pl) : tag);
                    }
                }
                if (done) {
                    status = SX_FEASIBLE;
                    break;
                }
                // ---- the objective side's answer (every rank's objective tiles, from this rank's gb):
                // the next entering variable, then r, p, the RHS, the status and U[s <= q][e]
                if (t < 64) {
                    int ok = poll_wave<decltype(gather_b), true>(gb, 2 * NBg, gather_b, tag, s_g, &ch->abort_w, timeout,
                                                                 s_pay);
                    double ev = DBL_MAX;
                    int ei = -1, any = 0;
                    if (ok) wave_pass2(s_g, s_pay, NBg, s_v, s_i, ev, ei, any);
                    ei = __builtin_amdgcn_readfirstlane(ei);
                    // second stage: the next entering column's first-stage pivot-row values U[s][e]
                    // from this rank's U (written through by every rank before the stage switch),
                    // loaded while the record is polled
                    u64 ue1 = 0ull;
                    if (hb && ok && ei >= 0 && t < SX_HMAX)
                        ue1 = ld_sys(reinterpret_cast<const u64 *>(U + (size_t)t * ld + c.map(1 + ei)));
                    if (ok) {
                        const int wt = ei >= 0 ? ei / SX_TILE : 0;
                        ok = poll_wave<decltype(ident), true>(gb + (size_t)wt * SX_GB_STRIDE + kOP,
                                                              (kOU - kOP) + 2 * (qq + 1), ident, tag, s_g, &ch->abort_w,
                                                              timeout, (unsigned *)nullptr);
                        if (ok && t <= qq) s_ue[t] = gd(s_g[kOU - kOP + 2 * t], s_g[kOU - kOP + 1 + 2 * t]);
                    }
                    if (hb && t < SX_HMAX) s_ue1[t] = __longlong_as_double((long long)ue1);
                    if (t == 0) {
                        s_ent_ok = ok;
                        s_ent_e = ei;
                        s_ent_v = ev;
                        if (ok) {
                            s_ent_p = gd(s_g[0], s_g[1]);
                            s_br = gd(s_g[kOB - kOP], s_g[kOB - kOP + 1]);
                            s_ent_r = (int)s_g[kOR - kOP];
                            s_ent_st = (int)s_g[kOS - kOP];
                            s_ent_m = (int)s_g[kOM - kOP];
                        }
                    }
                }
                __syncthreads();
                if (!s_ent_ok) {
                    aborted = true;
                    break;
                }
                if (s_ent_st != SX_NOT_ENDED) {
                    status = s_ent_st;
                    break;
                }
                const int enext = s_ent_e;
                const int r = s_ent_r;
                const double p = s_ent_p, br = s_br;
                if (t == 0) {
                    s_p[q] = p;
                    s_r[q] = r;
                    s_e[q] = e;
                }
                cnt = q + 1;
                const double f = -a / p;
                s_hist[qq * SX_TILE + t] = f;
                if (liveA) {
                    F[sx_fidx(li, q)] = f;
                    if (row0 + li == r) {
                        b = b / p;
                        bits |= 1u << qq;
                        (hb ? PM2 : PM)[li] = ((u64)B << 32) | bits;  // (as k_batch: written, not read-modified)
                    } else {
                        b = fma(f, br, b);
                    }
                }
                if (bid == 0 && t == 0) {  // every rank keeps the whole basis and the records
                    recs[q].r = r;         // (base[r] = e, solver.cu:105: at the end of the batch)
                    recs[q].e = e;
                    recs[q].p = p;
                    U[(size_t)q * ld] = br;
                }
                e = enext;
                dmin = s_ent_v;
                if (liveA) a_pre = T[tl.idx(li, s_ent_m)];  // (as k_batch)
                __syncthreads();
            }
        } else {
            for (int q = 0; q < K; ++q) {
                const unsigned tag = make_tag(B, q);
                if (cap >= 0 && piv0 + q >= cap) {
                    status = SX_PIVOT_CAP;
                    break;
                }
                if (inj != 0u && isA && rank == 0 && bid == 0 && (unsigned)q + 1u == inj) {  // test hook
                    if (t == 0) __hip_atomic_store(&ch->abort_w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    aborted = true;
                    break;
                }
                if (q == SX_HMAX) {
                    // the stage switch (k_batch's, at system scope): this thread's first-stage history
                    // to registers, the LDS history reused.  Every thread's stores acknowledged -- the
                    // objective tiles' U rows (write-through into every rank), the ratio tiles' F --
                    // then one system-scope release writes this device's L2 back, before any
                    // second-stage record: a block that has seen one reads the first stage's U[s][e]
                    // (its own rank's U) and F[r][s] (the owner's F) with system-scope loads
    #pragma unroll
                    for (int s1 = 0; s1 < SX_HMAX; ++s1) h1[s1] = s_hist[s1 * SX_TILE + t];
                    bits1 = bits;
                    bits = 0u;
                    if (t < SX_HMAX) s_ue1[t] = s_ue[t];  // (U[s][e] of pivot SX_HMAX: its objective record)
                    drain();
                    __syncthreads();
                    if (t == 0) {
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
                        drain();
                    }
                    __syncthreads();
                    hb = SX_HMAX;
                }
                const int qq = q - hb;  // slot within the stage
                // ---- selection: pass 2 over every rank's ratio tiles (wave 0 polls and reduces)
                if (t < 64) {
                    const int ok = poll_wave<decltype(gather_a), true>(ga, 2 * NAg, gather_a, tag, s_g, &ch->abort_w,
                                                                       timeout, s_pay);
                    double tv = DBL_MAX;
                    int ti = -1, any = 0;
                    if (ok) wave_pass2(s_g, s_pay, NAg, s_v, s_i, tv, ti, any);
                    if (t == 0) {
                        s_sel_ok = ok;
                        s_sel_r = ti;
                        s_sel_any = any;
                    }
                }
                __syncthreads();
                if (!s_sel_ok) {
                    aborted = true;
                    break;
                }
                const int r = s_sel_r;
                // the leaving row's stored values, from its owner's tableau (read-only in this launch)
                double u = 0.0;
                if (liveB && r >= 0) {
                    const int owner = r / rpr;
                    const double *src = pv.T[owner] + tl.idx(r - owner * rpr, mj);  // (every rank: the same layout)
                    u = owner == rank ? *src : ld_sys(src);
                }
                // the winner's record (ratio tile 0's when there is none): d_e, p, the RHS, e, the
                // ratio side's status and F[r][s < q] of this stage, read by wave 0 into LDS
                if (t < 64) {
                    const int wt = r >= 0 ? r / SX_TILE : 0;
                    // second stage: the leaving row's first-stage factors F[r][s] from its owner's F
                    // (written back before the stage switch), loaded while the record is polled
                    u64 fr1 = 0ull;
                    if (hb && t < SX_HMAX && r >= 0) {
                        const int owner = r / rpr;
                        fr1 = ld_sys(reinterpret_cast<const u64 *>(pv.F[owner] + sx_fidx(r - owner * rpr, t)));
                    }
                    const int ok = poll_wave<decltype(ident), true>(ga + (size_t)wt * SX_GA_STRIDE + kRD,
                                                                    (kRF - kRD) + 2 * qq, ident, tag, s_g, &ch->abort_w,
                                                                    timeout, (unsigned *)nullptr);
                    if (hb && t < SX_HMAX) s_fr1[t] = __longlong_as_double((long long)fr1);
                    if (ok) {
                        if (t < qq) s_fr[t] = gd(s_g[kRF - kRD + 2 * t], s_g[kRF - kRD + 1 + 2 * t]);
                        if (t == 0) {
                            s_det_dmin = gd(s_g[0], s_g[1]);
                            s_p[q] = gd(s_g[kRA - kRD], s_g[kRA - kRD + 1]);
                            s_br = gd(s_g[kRB - kRD], s_g[kRB - kRD + 1]);
                            s_det_e = (int)s_g[kRE - kRD];
                            s_det_st = (int)s_g[kRS - kRD];
                            s_r[q] = r;
                            s_e[q] = (int)s_g[kRE - kRD];
                        }
                    }
                    if (t == 0) s_det_ok = ok;
                }
                __syncthreads();
                if (!s_det_ok) {
                    aborted = true;
                    break;
                }
                e = s_det_e;
                dmin = s_det_dmin;
                if (s_det_st != SX_NOT_ENDED) {  // the ratio side ended the phase (optimal)
                    status = s_det_st;
                    break;
                }
                int ost = SX_NOT_ENDED;
                if (!s_sel_any) {
                    ost = SX_UNBOUNDED;  // solver.cu:96-102
                } else if (r < 0) {
                    ost = SX_NUMERIC_FAIL;
                }
                const double p = s_p[q], br = s_br;
                double v = DBL_MAX;
                int i = -1;
                if (ost == SX_NOT_ENDED) {
                    cnt = q + 1;
                    if (hb) u = stage1_row_rl(u, h1, r, s_fr1, s_p, s_r);
                    u = hist_row_rl(u, qq, r, s_hist, s_fr, s_p + hb, s_r + hb);
                    s_hist[qq * SX_TILE + t] = u;
                    const double fd = -dmin / p;  // updateCostsVector, solver.cu:48-56
                    if (tb == 0 && t == 0) d0 = fma(fd, br, d0);
                    if (liveB) {
                        dj = fma(fd, u, dj);
                        if (cmp_eps(dj, v) < 0) {
                            v = dj;
                            i = ia;
                        }
                    }
                }
                half_argmin(v, i);
                if ((t & 31) == 0) {
                    s_v[t >> 5] = v;
                    s_i[t >> 5] = i;
                }
                __syncthreads();
                if (t < 64) {  // wave 0 combines the half winners and publishes (k_batch)
                    double wv = t < 16 ? s_v[t] : DBL_MAX;
                    int wi = t < 16 ? s_i[t] : -1;
                    half_argmin(wv, wi);
                    wi = __builtin_amdgcn_readfirstlane(wi);
                    const long long vb = __double_as_longlong(wv);
                    wv = __longlong_as_double(((long long)__builtin_amdgcn_readfirstlane((int)(vb >> 32)) << 32) |
                                              (long long)(unsigned)__builtin_amdgcn_readfirstlane((int)vb));
                    const int win = wi >= 0 ? wi - tb * SX_TILE : 0;
                    const unsigned pl = wi >= 0 ? (unsigned)win : SX_NOIDX;
                    // granule-major over the ranks: the value granules reach every rank first
                    // (replicated objective, repl: every rank runs every objective tile, so the
                    // record goes to this rank's copy alone)
                    const int nG = kOU + 2 * (qq + 1), WR = repl ? 1 : W;
                    for (int idx = t; idx < WR * nG; idx += 64) {
                        const int k = idx / WR, rk = repl ? rank : idx - k * WR;
                        unsigned data;
                        if (k == kOR) {
                            data = (unsigned)r;
                        } else if (k == kOS) {
                            data = (unsigned)ost;
                        } else if (k == kOM) {
                            data = (unsigned)reinterpret_cast<const int *>(s_a)[win];
                        } else {
                            const double val = k < kOP ? wv : k < kOB ? p : k < kOR ? br
                                                                            : s_hist[((k - kOU) >> 1) * SX_TILE + win];
                            const u64 bits64 = (u64)__double_as_longlong(val);
                            data = ((k < kOU ? k : k - kOU) & 1) ? (unsigned)(bits64 >> 32) : (unsigned)bits64;
                        }
                        put_g_sys(pv.gb[rk] + (size_t)tb * SX_GB_STRIDE + k, data, k < kOP ? (tag | pl) : tag);
                    }
                }
                // the pivot row into every rank's U[q] (the sweep's input, read after the batch):
                // issued behind the record, so the W-fold stores do not delay it (repl: this
                // rank's U alone -- every rank forms the whole row)
                if (ost == SX_NOT_ENDED && liveB && 1 + ia < c.Ns) {
                    const double uq = s_hist[qq * SX_TILE + t];
                    if (repl)
                        st_sys(pv.U[rank] + (size_t)q * ld + mj, uq);
                    else
                        for (int k = 0; k < W; ++k) st_sys(pv.U[k] + (size_t)q * ld + mj, uq);
                }
                if (ost != SX_NOT_ENDED) {
                    status = ost;
                    break;
                }
            }
        }
        // a batch that ended without a decision of the ratio side: the objective tiles learn the
        // next entering variable from the last objective records (k_batch)
        if (!isA && !aborted && (status == SX_NOT_ENDED || status == SX_PIVOT_CAP) && cnt > 0) {
            const unsigned tag = make_tag(B, cnt - 1);
            if (t < 64) {
                const int ok = poll_wave<decltype(gather_b), true>(gb, 2 * NBg, gather_b, tag, s_g, &ch->abort_w,
                                                                   timeout, s_pay);
                double ev = DBL_MAX;
                int ei = -1, any = 0;
                if (ok) wave_pass2(s_g, s_pay, NBg, s_v, s_i, ev, ei, any);
                if (t == 0) {
                    s_ent_ok = ok;
                    s_ent_e = ei;
                    s_ent_v = ev;
                }
            }
            __syncthreads();
            if (!s_ent_ok) aborted = true;
            e = s_ent_e;
            dmin = s_ent_v;
        }
    }
    // this rank's slice of the objective row (its objective tiles' columns; d[0] with tile 0): between
    // fused batches each rank keeps only its own slice current -- no rank writes another's d, so an
    // aborted batch cannot overwrite a peer's restored row -- and the host gathers the whole row
    // when it is needed (Engine::gather_d)
    if (liveB) d[1 + ia] = dj;
    if (!isA && tb == 0 && t == 0) d[0] = d0;
    // leave: the last block of this rank tells every rank it is done, waits until every rank
    // is, and writes the batch's outcome into the state.  Ordering: every wave
    // drains its stores (U rows written into every rank, F, PM, its d slice), the block barrier
    // joins them, and the block's arrival on exit_cnt is a system-scope RELEASE (its L2 writes
    // back what is dirty); the last block's arrival is an acquire-release, so it observes every
    // block's stores before its own system-scope release of the done granules; a rank reads a
    // peer's done granule with system-scope loads and takes a system-scope acquire before it
    // commits the batch.  The next kernel on this rank (the sweep) reads U after that commit.
    drain();
    __syncthreads();
    if (t == 0) {
        const unsigned k = __hip_atomic_fetch_add(&ch->exit_cnt, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_SYSTEM);
        s_flag = (k == nbl - 1);
        if (s_flag) {
            __hip_atomic_store(&ch->exit_cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (inj != 0u) ch->inject_q = 0u;  // (every block of this rank read it at its start)
        }
    }
    __syncthreads();
    if (!s_flag) return;
    if (t == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        drain();  // (MI355X_MICROARCH.md: the compiler may drop the wait behind the write-back)
    }
    __syncthreads();
    const unsigned dtag = make_tag(B, 0);
    if (t < W) put_g_sys(pv.gdone[t] + rank, aborted ? 1u : 0u, dtag);
    const bool ok = gather_tagged<decltype(ident), true>(gdone, W, ident, dtag, s_g, &ch->abort_w, &s_ok, timeout);
    if (t != 0) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    bool peer_abort = false;
    for (int k = 0; ok && k < W; ++k) peer_abort |= s_g[k] != 0u;
    if (status0 != SX_NOT_ENDED) return;
    if (!ok || aborted || peer_abort || ld_sc1(&ch->abort_w) != 0u) {
        st->status = SX_HANG;
        __hip_atomic_store(&ch->abort_w, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    for (int s = 0; s < cnt; ++s) base[s_r[s]] = s_e[s];  // solver.cu:105, in pivot order
    st->status = status;
    st->pivots = piv0 + cnt;
    if (cnt > 0) {
        st->r = s_r[cnt - 1];
        st->e = s_e[cnt - 1];
        st->batch_tag = B;
        st->batch_count = cnt;
    }
    st->e_next = e;
    st->dmin_next = dmin;
}


__global__ __launch_bounds__(512) void k_batch_mr(const double *__restrict__ T, int rows, int row0, int rpr, size_t ld, TLay tl,
                                                  Cols c, double *__restrict__ d, double *__restrict__ d_save, int *base,
                                                  DevState *st, double *U, double *F, PivRec *recs,
                                                  unsigned long long *PM, unsigned long long *PM2, unsigned B, int K,
                                                  int slots, int W, int rank, int tb0, int tb1, int NBg, int repl,
                                                  BatchChan *ch, const u64 *ga, const u64 *gb, const u64 *gdone,
                                                  PeerView pv, unsigned long long timeout) {
    batch_mr_body((int)blockIdx.x, gridDim.x, T, rows, row0, rpr, ld, tl, c, d, d_save, base, st, U, F, recs, PM, PM2, B, K,
                  slots, W, rank, tb0, tb1, NBg, repl, ch, ga, gb, gdone, pv, timeout);
}

// The batches of the nloc ranks (of W) that live on one GPU in ONE launch: block b belongs to
// the local rank k with first[k] <= b < first[k + 1], as its block b - first[k].  One grid, so
// every local rank's blocks are resident together whenever the grid fits the device -- nloc
// launches on nloc streams also need nloc hardware queues that run at once, which a process
// does not control.  (Virtual shards: all W ranks on one GPU; one process driving several
// GPUs: one launch per GPU.)
struct MrRank {
    const double *T;
    int rows, row0, rank, tb0, tb1, repl;
    const int *perm;
    double *d, *d_save;
    int *base;
    DevState *st;
    double *U, *F;
    PivRec *recs;
    unsigned long long *PM, *PM2;
    BatchChan *ch;
    const u64 *ga, *gb, *gdone;
};
struct MrRanks {
    MrRank r[SX_MAXW];
    int first[SX_MAXW + 1];
};
__global__ __launch_bounds__(512) void k_batch_mr_multi(MrRanks R, int nloc, int rpr, size_t ld, TLay tl, Cols c,
                                                        unsigned B, int K, int slots, int W, int NBg, PeerView pv,
                                                        unsigned long long timeout) {
    int k = 0;
    while (k + 1 < nloc && (int)blockIdx.x >= R.first[k + 1]) ++k;
    const MrRank &x = R.r[k];
    Cols cx = c;
    cx.perm = x.perm;
    batch_mr_body((int)blockIdx.x - R.first[k], (unsigned)(R.first[k + 1] - R.first[k]), x.T, x.rows, x.row0, rpr, ld,
                  tl, cx, x.d, x.d_save, x.base, x.st, x.U, x.F, x.recs, x.PM, x.PM2, B, K, slots, W, x.rank, x.tb0, x.tb1,
                  NBg, x.repl, x.ch, x.ga, x.gb, x.gdone, pv, timeout);
}

// ---------------------------------------------------------------------------------------
// K5: the sweep -- the batch's pivots applied to every stored element of the shard
// (updateContraintsMatrix, solver.cu:34-46, for q pivots at once), in pivot order:
//   x = T[i][j];  for s < q:  x = (i == r_s) ? x / p_s : fma(F[i][s], U[s][j], x);  T[i][j] = x
// A thread owns two adjacent columns (one 16-byte load and store per row) and keeps their
// KT pivot-row values in registers for the whole sweep; the row's factors F[i][0..q) and its
// pivot-slot bits are wave-uniform (scalar loads).  A fixed set of G blocks per 512-column
// tile walks the row groups (RB rows per step).  On odd sweeps the tile and row order are
// reversed, so a sweep starts on the lines the previous one wrote last (still in the 256 MB
// Infinity Cache).  The sweep runs whatever the phase status: a batch cut short by the end
// of the phase is still materialised.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef double d4_t __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

// (batch tag, batch count, swept slack columns) of this sweep into rec[0..2] (bench sessions'
// timed sweeps; null otherwise) -- written by the sweep itself instead of two device copies
// between kernels (two dispatches, ~9 us per batch)
__device__ __forceinline__ void sweep_record(int *rec, const DevState *st, const int *nact) {
    if (rec && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
        rec[0] = (int)st->batch_tag;
        rec[1] = st->batch_count;
        if (nact) rec[2] = *nact;
    }
}

// Cache policy of the tableau traffic: non-temporal loads, write-through (sc1) stores (measured best
// of five load/store policies at both sizes, profiles/r03_sweep_policy_ab.txt).
template <int KT, int RB>
__global__ __launch_bounds__(256) void k_sweep(double *T, int rows, size_t ld, TLay tl, int Ns,
                                               const int *__restrict__ nact, int s0,
                                               const double *__restrict__ F, const double *__restrict__ U,
                                               const PivRec *__restrict__ recs,
                                               const unsigned long long *__restrict__ PM,
                                               const DevState *__restrict__ st, unsigned B, int rev,
                                               int *__restrict__ rec) {
    sweep_record(rec, st, nact);
    const int cnt = st->batch_tag == B ? st->batch_count : 0;
    if (cnt <= 0) return;
    // slack compaction: the columns past s0 + *nact are untouched unit vectors (not swept);
    // the grid's blocks are re-dealt over the active column tiles
    if (nact && s0 + *nact < Ns) Ns = s0 + *nact;
    const int cb = (Ns + 511) / 512;
    const int lin = (int)(blockIdx.y * gridDim.x + blockIdx.x);
    const int G = (int)(gridDim.x * gridDim.y) / cb;
    const int tile = lin % cb, gy = lin / cb;
    if (gy >= G) return;
    const int bx = rev ? cb - 1 - tile : tile;
    const int j = (bx * 256 + (int)threadIdx.x) * 2;
    if (j >= Ns) return;  // the thread of an odd last column moves (j, j+1): j+1 < ld is padding
    // this tile's storage region (jB is a multiple of 512: a tile lies in one region)
    const bool inB = bx * 512 >= tl.jB;
    double *const Tr = inB ? T + tl.offB : T;
    const size_t ldr = inB ? tl.ldB : tl.ldA;
    const int jr = inB ? j - tl.jB : j;
    const unsigned mask = slot_mask(cnt);
    double2 u[KT];
#pragma unroll
    for (int s = 0; s < KT; ++s)
        u[s] = s < cnt ? *reinterpret_cast<const double2 *>(U + (size_t)s * ld + j) : make_double2(0.0, 0.0);
    const int ng = (rows + RB - 1) / RB;
    // a row's buffer resource: its first element (row-major), or its first 4-column block row inside
    // the 16-row strip (blocked layout, TLay); the thread's column pair at a fixed offset from it
    const int oob = (int)(tl.blk ? ldr * 16 * 8 : ldr * 8);
    const int jo = tl.blk ? ((jr >> 2) * 64 + (jr & 3)) * 8 : jr * 8;
    auto row_base = [&](int i) {
        return tl.blk ? Tr + (size_t)(i >> 4) * 16 * ldr + (size_t)(((i & 15) >> 2) * 16 + (i & 3) * 4)
                      : Tr + (size_t)i * ldr;
    };
    for (int g = gy; g < ng; g += G) {
        const int i0 = (rev ? ng - 1 - g : g) * RB;
        double2 x[RB];
        // non-temporal loads (cache policy nt): each element is read once per sweep; measured
        // 1.5 % faster at config 5, neutral at config 3 (profiles/r01_v13_sweep_load_policy.txt)
        constexpr int LAUX = 2;
#pragma unroll
        for (int k = 0; k < RB; ++k) {
            const int i = i0 + k < rows ? i0 + k : i0;
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(row_base(i), 0, oob, 0x00020000);
            x[k] = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(rs, i0 + k < rows ? jo : oob,
                                                                                      0, LAUX));
        }
#pragma unroll
        for (int k = 0; k < RB; ++k) {
            const int i = i0 + k;
            if (i >= rows) break;
            // the row's factors: unconditional (wave-uniform, scalar) loads issued together --
            // F rows hold SX_KMAX allocated doubles; slots >= cnt are loaded but not used.
            // Only a full batch (cnt == KT) runs the unguarded chain: a partial one (the last
            // batch of a phase) takes the per-slot guarded path, about 2x slower per byte
            // (1668 vs 851 us at config 5 with 20-pivot batches, profiles/r02_sweep_partial_batch.txt).
            // Padding slots >= cnt with f = -0.0 (fma(-0, +0, y) = y exactly) instead cost every
            // full sweep 40 % (1218 vs 851 us): 32 scalar selects per row behind spilled masks.
            double f[KT];
#pragma unroll
            for (int s = 0; s < KT; ++s) f[s] = F[sx_fidx(i, s)];
            const unsigned bits = pend_bits(PM, i, B, mask);
            double2 y = x[k];
            if (bits == 0u && cnt == KT) {  // a full batch, no leaving row: no per-slot branch
#pragma unroll
                for (int s = 0; s < KT; ++s) {
                    y.x = fma(f[s], u[s].x, y.x);
                    y.y = fma(f[s], u[s].y, y.y);
                }
            } else if (bits == 0u) {
#pragma unroll
                for (int s = 0; s < KT; ++s) {
                    if (s < cnt) {
                        y.x = fma(f[s], u[s].x, y.x);
                        y.y = fma(f[s], u[s].y, y.y);
                    }
                }
            } else {
#pragma unroll
                for (int s = 0; s < KT; ++s) {
                    if (s < cnt) {
                        if ((bits >> s) & 1u) {
                            const double p = recs[s].p;
                            y.x = y.x / p;
                            y.y = y.y / p;
                        } else {
                            y.x = fma(f[s], u[s].x, y.x);
                            y.y = fma(f[s], u[s].y, y.y);
                        }
                    }
                }
            }
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(row_base(i), 0, oob, 0x00020000);
            constexpr int SAUX = 16;
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, y), rs, jo, 0, SAUX);
        }
    }
}

// A strip's matrix steps (k_msweep): acc[p][0] / acc[p][1] = tile X / Y of pair p; all four chains
// advance one 4-slot step at a time (each element's fmas stay in slot order)
template <int NKB>
__device__ __forceinline__ void msweep_steps(d4_t (&acc)[2][2], const double (&ff)[NKB], const double2 (&uf)[NKB][2],
                                             int nkb) {
    if (nkb == NKB) {
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
            for (int p = 0; p < 2; ++p) {
                acc[p][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(ff[kb], uf[kb][p].x, acc[p][0], 0, 0, 0);
                acc[p][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(ff[kb], uf[kb][p].y, acc[p][1], 0, 0, 0);
            }
    } else {
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb)
            if (kb < nkb)
#pragma unroll
                for (int p = 0; p < 2; ++p) {
                    acc[p][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(ff[kb], uf[kb][p].x, acc[p][0], 0, 0, 0);
                    acc[p][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(ff[kb], uf[kb][p].y, acc[p][1], 0, 0, 0);
                }
    }
}

// ... and its stores: the lane's column pair of rows rg + 4v, write-through; a leaving row (bit v of
// skip) and columns past Ns are not written; an odd last column's neighbour is an untouched
// column: only the even one is written
template <typename OFF>
__device__ __forceinline__ void msweep_store(const d4_t (&acc)[2][2], __amdgpu_buffer_rsrc_t rss, int c0, int jl, int Ns,
                                             unsigned skip, OFF tile_off) {
    const int OOB = 0x7fffffff;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        const int j = c0 + 32 * p + 2 * jl;
        const bool pair = j + 1 < Ns;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const int off = tile_off(p, v);
            const bool keep = j < Ns && !((skip >> v) & 1u);
            if (pair) {
                const double2 y = make_double2(acc[p][0][v], acc[p][1][v]);
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, y), rss, keep ? off : OOB, 0, 16);
            } else {
                // (built from the 64-bit integer: a bit_cast of acc[p][0][v] straight to u32x2 compiled
                // to a store of element 0 for every v -- ROCm 7.2 clang, checked in the ISA)
                const unsigned long long xb = (unsigned long long)__double_as_longlong(acc[p][0][v]);
                const u32x2 w = {(unsigned)xb, (unsigned)(xb >> 32)};
                __builtin_amdgcn_raw_buffer_store_b64(w, rss, keep ? off : OOB, 0, 16);
            }
        }
    }
}

// The rows that left the basis in a batch (k_msweep): row r_s (first slot s where it left) by
// the row slot s % G, one column per lane (the strips leave them unwritten).  The row slot's rows
// and their leaving slots come from the sweep's register list rl (lane s: the shard row that left
// at slot s) -- a shuffle and a ballot per slot, no memory access (round 6: the PM / PM2 loads were
// two dependent round trips in the sweep's tail); the column's pivot-row values of every slot are
// loaded once; each group of NR rows costs one round trip (the pivot-row value it restarts from and
// its factors; the pivots: lane s = slot s, read by v_readlane) and a branch-free chain.
template <int NKB>
__device__ __forceinline__ void msweep_fixup(const double *Tr, double *Tw, size_t ldr, int cr, int c0, int Ns, int rows,
                                             int row0, TLay tl, int gy, int G, int cnt,
                                             const double *__restrict__ F, const double *__restrict__ U, size_t ld,
                                             const PivRec *__restrict__ recs, int rl) {
    const int OOB = 0x7fffffff;
    const int l = (int)threadIdx.x & 63;
    const int j = c0 + l;
    int rk = -1;                // lane k: the row of slot gy + G k, if this is its first slot
    unsigned long long bk = 0;  // ... and its leaving slots
    for (int k = 0; gy + G * k < cnt; ++k) {  // (wave-uniform)
        const int sk = gy + G * k;
        const int r = __shfl(rl, sk);
        const unsigned long long b = __ballot(r >= 0 && rl == r);
        if (l == k && r >= 0 && (int)__builtin_ctzll(b) == sk) {
            rk = r;
            bk = b;
        }
    }
    unsigned long long todo = __ballot(rk >= 0);
    if (todo == 0ull) return;
    const double pl = l < cnt ? recs[l].p : 1.0;  // lane s: p_s
    // the column's pivot-row values of the NKB * 4 slots held (in the registers of the strips'
    // U fragments, free by now)
    constexpr int KU = NKB * 4;
    double uu[KU];
#pragma unroll
    for (int k1 = 0; k1 < KU; ++k1) uu[k1] = (k1 < cnt && j < Ns) ? U[(size_t)k1 * ld + j] : 0.0;
    // NR rows at a time (independent chains)
    constexpr int NR = NKB == SX_KMAX / 4 ? 4 : 2;
    while (todo) {
        int r[NR];
        unsigned long long bits[NR];
        bool live[NR];
#pragma unroll
        for (int q1 = 0; q1 < NR; ++q1) {
            live[q1] = todo != 0ull;
            const int k = live[q1] ? __builtin_ctzll(todo) : 0;
            if (live[q1]) todo &= todo - 1ull;
            r[q1] = __builtin_amdgcn_readlane(rk, k);
            bits[q1] = ((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(bk >> 32), k) << 32) |
                       (unsigned)__builtin_amdgcn_readlane((int)bk, k);
        }
        // A row that last left at slot sl held, just before sl, exactly the pivot row's value
        // U[sl][j] (formed by the objective tiles with the same operations in the same order,
        // DESIGN.md §3.2), so its value after the batch is U[sl][j] / p_sl followed by the fmas of
        // the slots after sl: one division, no stored value read, no per-slot branch.
        double x[NR], fl[NR];
        int sl[NR];
        int slmin = KU;
#pragma unroll
        for (int q1 = 0; q1 < NR; ++q1) {
            sl[q1] = live[q1] ? 63 - (int)__builtin_clzll(bits[q1]) : KU;
            slmin = sl[q1] < slmin ? sl[q1] : slmin;
            x[q1] = (live[q1] && j < Ns) ? U[(size_t)sl[q1] * ld + j] : 0.0;
            fl[q1] = (live[q1] && l < cnt) ? F[sx_fidx(r[q1], l)] : 0.0;  // lane s: F[r][s]
        }
#pragma unroll
        for (int q1 = 0; q1 < NR; ++q1)
            if (live[q1]) x[q1] = x[q1] / rdlane(pl, sl[q1]);
#pragma unroll
        for (int s1 = 0; s1 < KU; ++s1) {
            if (s1 < cnt && s1 > slmin) {
#pragma unroll
                for (int q1 = 0; q1 < NR; ++q1) {
                    const double t = fma(rdlane(fl[q1], s1), uu[s1], x[q1]);
                    x[q1] = s1 > sl[q1] ? t : x[q1];
                }
            }
        }
#pragma unroll
        for (int q1 = 0; q1 < NR; ++q1) {
            if (!live[q1]) continue;
            // (the row's strip through one resource: its element of column cr + l at b4 within it)
            const int rr = r[q1];
            const __amdgpu_buffer_rsrc_t rsr =
                tl.blk ? __builtin_amdgcn_make_buffer_rsrc(Tw + (size_t)(rr >> 4) * 16 * ldr, 0, (int)(ldr * 16 * 8), 0x00020000)
                       : __builtin_amdgcn_make_buffer_rsrc(Tw + (size_t)rr * ldr, 0, (int)(ldr * 8), 0x00020000);
            const int eo = tl.blk ? (int)(TLay::b4(rr & 15, cr + l, ldr) * 8) : (cr + l) * 8;
            const unsigned long long xb = (unsigned long long)__double_as_longlong(x[q1]);
            const u32x2 w = {(unsigned)xb, (unsigned)(xb >> 32)};
            __builtin_amdgcn_raw_buffer_store_b64(w, rsr, j < Ns ? eo : OOB, 0, 16);  // (write-through, as the strips)
        }
    }
}

// K5': the same sweep on the matrix cores.  v_mfma_f64_16x16x4f64 computes a 16x16 tile's
// D = A B + C as the slot-ordered chain of fused multiply-adds, bit for bit
// (experiments/mfma_f64_probe.hip: every element equals fma(a3, b3, fma(a2, b2, fma(a1, b1,
// fma(a0, b0, c)))) on MI355X), so SX_KMAX / 4 MFMAs per tile are the batch's updates in the
// reference's order (solver.cu:34-46).  Operands of step k (slots 4k .. 4k+3):
//   A (16 rows x 4 slots)     lane l = F[r0 + l % 16][4k + l / 16]   (sx_fidx: 64 consecutive doubles)
//   B (4 slots x 16 columns)  lane l = U[4k + l / 16][col(l % 16)]
//   C / D                     lane l, register v = T[r0 + l / 16 + 4v][col(l % 16)]
// Two tiles share each lane's 16-byte access (tile X the even column 2c, tile Y the odd 2c + 1),
// so every tableau access is one 16-byte load or store per lane.  A wave owns 64 columns (two
// pairs of tiles) and walks 16-row strips; its U fragments stay in registers for the whole
// sweep, the strip's F fragments are loaded per strip; a strip's tableau accesses go through
// one wave-uniform buffer resource.  A partial batch pads slots >= cnt with f = -0.0, u = +0.0
// (fma(-0, +0, x) == x for every x) and skips the 4-slot steps past cnt.
// The rows that left the basis in this batch (x / p at their slot instead of the fma; at most
// SX_KMAX of the shard's rows) are not stored by the strips: each is recomputed after the strip
// loop, by the waves of the row slot s % G, from its stored values with the vector chain (one
// column per lane).  The strips never write those rows, so the values read are the originals.
// Grid, column order, regions, compaction and cache policy as k_sweep (POL 1), with 256-column
// tiles.  In place (Tsrc == Tdst: the strips read through one pointer and write through the other).
// NKB: 4-slot steps held (SX_HMAX / 4: one stage, 3 waves per SIMD; SX_KMAX / 4: two stages,
// 2 waves per SIMD).  Both pairs' four accumulators advance one 4-slot step at a time (msweep_steps):
// four independent MFMA chains per wave, eight per SIMD -- the f64 probe needs about eight to keep
// the matrix pipe busy.  Pair by pair (two chains per wave) measured 2.5 % slower
// at config 5, same box (profiles/r05_variants_ab.txt).
template <int NKB>
__global__ __launch_bounds__(256, 2) void k_msweep(const double *Tsrc, double *Tdst, int rows, int row0, size_t ld,
                                                   TLay tl, int Ns, const int *__restrict__ nact, int s0,
                                                   const double *__restrict__ F, const double *__restrict__ U,
                                                   const PivRec *__restrict__ recs,
                                                   const unsigned long long *__restrict__ PM,
                                                   const unsigned long long *__restrict__ PM2,
                                                   const DevState *__restrict__ st, unsigned B, int rev,
                                                   int *__restrict__ rec) {
    sweep_record(rec, st, nact);
    const int cnt = st->batch_tag == B ? st->batch_count : 0;
    if (cnt <= 0) return;
    if (nact && s0 + *nact < Ns) Ns = s0 + *nact;
    const int cb = (Ns + 255) / 256;
    const int lin = (int)(blockIdx.y * gridDim.x + blockIdx.x);
    const int G = (int)(gridDim.x * gridDim.y) / cb;
    const int tile = lin % cb, gy = lin / cb;
    if (gy >= G) return;
    const int bx = rev ? cb - 1 - tile : tile;
    const int l = (int)threadIdx.x & 63, jl = l & 15, rg = l >> 4;
    const int c0 = (bx * 4 + ((int)threadIdx.x >> 6)) * 64;  // the wave's first column
    if (c0 >= Ns) return;
    // this tile's storage region (jB is a multiple of 512: a 256-column tile lies in one region)
    const bool inB = bx * 256 >= tl.jB;
    const double *const Tr = inB ? Tsrc + tl.offB : Tsrc;
    double *const Tw = inB ? Tdst + tl.offB : Tdst;
    const size_t ldr = inB ? tl.ldB : tl.ldA;
    const int cr = inB ? c0 - tl.jB : c0;
    const int nkb = (cnt + 3) >> 2;
    const int OOB = 0x7fffffff;
    // lane s: the shard row that left at slot s (-1: none here) -- the strips find their leaving
    // rows in this register instead of loading per-row bits
    const int rl = [&] {
        if (l >= cnt) return -1;
        const int r = recs[l].r - row0;
        return r >= 0 && r < rows ? r : -1;
    }();
    {
        // the lane's columns: c0 + 32p + 2jl and the next, p = 0, 1 (an odd last column's neighbour
        // is an untouched column: not written)
        double2 uf[NKB][2];
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
            for (int p = 0; p < 2; ++p) {
                const int sl = 4 * kb + rg, j = c0 + 32 * p + 2 * jl;
                uf[kb][p] = (sl < cnt && j < Ns) ? *reinterpret_cast<const double2 *>(U + (size_t)sl * ld + j)
                                                 : make_double2(0.0, 0.0);
            }
        const int nstrip = (rows + 15) >> 4;
        // a strip's tableau tiles (both pairs), through one buffer resource per strip
        // (wave-uniform) holding the strip's valid rows; rows past the end read 0 and drop their
        // stores
        auto strip_r0 = [&](int g) { return (rev ? nstrip - 1 - g : g) * 16; };
        // (blocked layout, TLay: a strip's rows past the end exist -- rows are allocated in whole
        // strips -- and hold values no row reads; row-major: they read 0 and their stores drop)
        auto strip_rsrc = [&](const double *base, int r0) {
            const int nr = tl.blk ? 16 : (rows - r0 < 16 ? rows - r0 : 16);
            return __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(base) + (size_t)r0 * ldr, 0,
                                                     (int)((size_t)nr * ldr * 8), 0x00020000);
        };
        // byte offset in the strip of the lane's column pair (c0 + 32 p + 2 jl, + 1) in row rg + 4 v
        auto tile_off = [&](int p, int v) {
            const int jr = cr + 32 * p + 2 * jl;
            return tl.blk ? (int)((size_t)((jr >> 2) * 64 + v * 16 + rg * 4 + (jr & 3)) * 8)
                          : (int)(((size_t)(rg + 4 * v) * ldr + jr) * 8);
        };
        auto load_tiles = [&](double2 (&cx)[2][4], int r0) {
            const __amdgpu_buffer_rsrc_t rsl = strip_rsrc(Tr, r0);
#pragma unroll
            for (int p = 0; p < 2; ++p)
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                    const int j = c0 + 32 * p + 2 * jl;
                    cx[p][v] = __builtin_bit_cast(
                        double2, __builtin_amdgcn_raw_buffer_load_b128(rsl, j < Ns ? tile_off(p, v) : OOB, 0, 2));
                }
        };
        for (int g = gy; g < nstrip; g += G) {
            const int r0 = strip_r0(g);
            const __amdgpu_buffer_rsrc_t rss = strip_rsrc(Tw, r0);
            // issue order: both pairs' tableau tiles, the strip's factors -- one memory round trip
            // per strip
            double2 cx[2][4];
            load_tiles(cx, r0);
            double ff[NKB];
            {
                // (lane l of step kb: F[sx_fidx(r0 + l % 16, 4 kb + l / 16)] = strip base + 64 kb + l;
                // the strip's rows past the end hold stale factors of rows that are not stored)
                const double *Fs = F + sx_fidx(r0, 0) + l;
#pragma unroll
                for (int kb = 0; kb < NKB; ++kb) ff[kb] = Fs[64 * kb];
            }
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb)
                if (4 * kb + rg >= cnt) ff[kb] = -0.0;
            // both pairs' four accumulators advance together: four independent MFMA chains per
            // wave (two chains at a time leave the matrix pipe waiting on each step's result)
            d4_t acc[2][2];
#pragma unroll
            for (int p = 0; p < 2; ++p) {
                acc[p][0] = d4_t{cx[p][0].x, cx[p][1].x, cx[p][2].x, cx[p][3].x};
                acc[p][1] = d4_t{cx[p][0].y, cx[p][1].y, cx[p][2].y, cx[p][3].y};
            }
            msweep_steps<NKB>(acc, ff, uf, nkb);
            // bit v of skip: row r0 + rg + 4v left in this batch (not stored here): the slots whose
            // row lies in this strip, from the register list (no memory access)
            unsigned skip = 0u;
            {
                unsigned long long sm = __ballot(rl >= r0 && rl < r0 + 16);
                while (sm) {
                    const int k = __builtin_ctzll(sm);
                    sm &= sm - 1ull;
                    const int rr = __builtin_amdgcn_readlane(rl, k) - r0;
                    if ((rr & 3) == rg) skip |= 1u << (rr >> 2);
                }
            }
            msweep_store(acc, rss, c0, jl, Ns, skip, tile_off);
        }
    }
    msweep_fixup<NKB>(Tr, Tw, ldr, cr, c0, Ns, rows, row0, tl, gy, G, cnt, F, U, ld, recs, rl);
}

// Slack compaction (sx_common.hpp Cols), between a batch's selections and its
// sweep.  The first time row r leaves the basis, its slack column -- still the unit vector e_r
// as built, never swept -- is exchanged with the slack column at the first untouched stored
// position s0 + nact (also a unit vector), so the swept block [0, s0 + nact) grows by one.
// The exchanges of one batch are resolved in slot order by wave 0, one list entry per lane
// (stored offset, slack held before the batch, slack held now); their net effect is then
// applied at once: to the pending pivot rows U[s] (whose entries at the two columns are
// the leaving rows' current values there), to T (zeros and ones of the unit vectors, this
// shard's rows only) and to perm / iperm / act / nact.  The shards run it alike.
// A batch of more than SX_HMAX pivots is activated in two passes (sb = 0, then sb = SX_HMAX, from
// the state the first left -- the same exchanges in slot order, as the fused batch's last block
// does): a pass lists the exchanges of the slots [sb, sb + SX_HMAX) -- at most 2 entries per slot,
// one per lane -- and swaps the entries of every pending row U[s], s < cnt.
__global__ __launch_bounds__(256) void k_activate(int *__restrict__ perm, int *__restrict__ iperm,
                                                  int *__restrict__ ucol, const int *__restrict__ urow,
                                                  int *__restrict__ nact_p, int m,
                                                  double *__restrict__ T, int rows, int row0, size_t ld, TLay tl,
                                                  int s0, double *__restrict__ U, const PivRec *__restrict__ recs,
                                                  const DevState *__restrict__ st, unsigned B, int sb) {
    const int cnt = st->batch_tag == B ? st->batch_count : 0;
    if (cnt <= sb) return;
    const int pc = cnt - sb < SX_HMAX ? cnt - sb : SX_HMAX;  // this pass's slots
    recs += sb;
    const int t = threadIdx.x;
    const int na0 = *nact_p;
    __shared__ int s_pl[64], s_ol[64], s_cl[64], s_src[64];
    __shared__ int s_nl, s_added;
    __shared__ double s_u[SX_KMAX * 64];
    if (t < 64) {
        // lane s: the unswept slack column that is the unit vector of slot s's leaving row (-1:
        // none), its stored offset, and the slack at window offset na0 + s
        int kc = -1, pr = 0, win = -1;
        if (t < pc) {
            kc = ucol[recs[t].r];
            pr = kc >= 0 ? perm[kc] : 0;
            if (na0 + t < m) win = iperm[na0 + t];
        }
        int pl = -1, ol = -1, cl = -1;  // this lane's list entry
        int nl = 0, added = 0;
        for (int s = 0; s < pc; ++s) {
            const int rs = __shfl(kc, s);  // (a slack id from here on)
            if (rs < 0) continue;  // every column of the row's basic variable is swept already
            // already moved into the window in this batch?
            if (__ballot(t < nl && cl == rs && pl >= na0 && pl < na0 + added)) continue;
            const unsigned long long hP = __ballot(t < nl && cl == rs);
            int iP;
            if (hP) {
                iP = __ffsll((long long)hP) - 1;
            } else {  // untouched in this batch: at its pre-batch offset
                iP = nl++;
                const int P = __shfl(pr, s);
                if (t == iP) {
                    pl = P;
                    ol = rs;
                    cl = rs;
                }
            }
            const int pos = na0 + added;
            const unsigned long long hW = __ballot(t < nl && pl == pos);
            int iW;
            if (hW) {
                iW = __ffsll((long long)hW) - 1;
            } else {
                iW = nl++;
                const int w = __shfl(win, added);
                if (t == iW) {
                    pl = pos;
                    ol = w;
                    cl = w;
                }
            }
            const int cP = __shfl(cl, iP), cW = __shfl(cl, iW);
            if (t == iP) cl = cW;
            if (t == iW) cl = cP;
            ++added;
        }
        if (t < nl) {
            s_pl[t] = pl;
            s_ol[t] = ol;
            s_cl[t] = cl;
        }
        if (t == 0) {
            s_nl = nl;
            s_added = added;
        }
    }
    __syncthreads();
    const int nl = s_nl;
    if (nl == 0) return;
    if (t < nl) {  // the entry whose pre-batch slack this position holds now
        int j = 0;
        while (s_ol[j] != s_cl[t]) ++j;
        s_src[t] = j;
    }
    __syncthreads();
    for (int k = t; k < cnt * nl; k += blockDim.x) {
        const int s = k / nl, i = k - s * nl;
        s_u[k] = U[(size_t)s * ld + s0 + s_pl[s_src[i]]];
    }
    __syncthreads();
    for (int k = t; k < cnt * nl; k += blockDim.x) {
        const int s = k / nl, i = k - s * nl;
        U[(size_t)s * ld + s0 + s_pl[i]] = s_u[k];
    }
    if (t < nl) {
        const int x = s_pl[t], o = s_ol[t], c = s_cl[t];
        if (o != c) {  // (both unswept unit vectors before the batch: of rows urow[o], urow[c])
            const int ro = urow[o], rc = urow[c];
            if (ro >= row0 && ro < row0 + rows) T[tl.idx(ro - row0, s0 + x)] = 0.0;
            if (rc >= row0 && rc < row0 + rows) T[tl.idx(rc - row0, s0 + x)] = 1.0;
        }
        iperm[x] = c;
        perm[c] = x;
        if (x >= na0 && x < na0 + s_added) ucol[urow[c]] = -1;
    }
    if (t == 0) *nact_p = na0 + s_added;
}

// Basic slack columns out of the sweep (one shard; after a sweep, every few batches).  When a variable
// enters at row r the reference (solver.cu:34-46) makes its pivot-row entry p / p = 1 and every other
// entry fma(-(a_k / p), p, a_k) = a_k - fl(a_k / p) p, rounded once: +0 wherever fl(a_k / p) p == a_k,
// a residual of an ulp or so elsewhere.  A column whose residuals all vanished is exactly the unit
// vector e_r, every later pivot row holds +0 there while the variable stays basic, and the updates
// leave it bit-identical (fma(f, +0, +0) = +0, fma(f, +0, 1) = 1, finite f) until row r leaves.  The
// swept slack columns whose slack is basic and whose column checks out as e_r, bit for bit, are
// therefore moved behind the swept block, like the untouched
// slacks of slack compaction: the sweep stops before them, and the batch whose leaving row is r moves
// the column back (activate_block / k_activate: ucol[r] is the unswept column that is e_r, urow[k]
// the row of unswept slack k).  Five launches per round:
//   k_deact_mark   one thread per row: a row whose basic variable is a swept slack tags that slack's
//                  stored position with (round, row);
//   k_deact_list   one block: the tagged positions in order (at most SX_DEACT_CAP; the rest wait for
//                  the next round);
//   k_deact_check  every row compares each listed column with e_r bit for bit (a column that is not
//                  -- a non-finite entry when it entered -- stays swept);
//   k_deact_plan   one block: the d checked columns keep their positions if they lie in the last d
//                  positions of the swept block, else each is exchanged with a column there that is
//                  not one of them (the j-th such candidate with the j-th such position); perm / iperm /
//                  ucol / urow / nact updated;
//   k_deact_move   the exchanges on T: the other column copied to the candidate's position, e_r
//                  written at the candidate's new one.
__device__ __forceinline__ int deact_slack(int v, int n, int m, bool alias) {
    if (v >= n && v < n + m) return v - n;
    if (alias && v >= n + m && v < n + 2 * m) return v - n - m;  // (an artificial is stored as its slack)
    return -1;
}

// exclusive prefix sum of v over a block of 1024 threads (s_w: 16 ints of LDS); *total = the sum
__device__ __forceinline__ int block_exscan1024(int v, int *s_w, int *total) {
    const int t = threadIdx.x, l = t & 63, w = t >> 6;
    int x = v;  // inclusive scan within the wave
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o);
        if (l >= o) x += y;
    }
    if (l == 63) s_w[w] = x;
    __syncthreads();
    int before = 0, all = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int c = s_w[k];
        before += k < w ? c : 0;
        all += c;
    }
    __syncthreads();  // (s_w reusable)
    *total = all;
    return before + x - v;
}

__global__ __launch_bounds__(256) void k_deact_mark(const int *__restrict__ base, const int *__restrict__ perm,
                                                    const int *__restrict__ nact_p, int n, int m, bool alias,
                                                    const int *__restrict__ fail, unsigned long long *__restrict__ tag,
                                                    unsigned epoch) {
    const int i = (int)blockIdx.x * 256 + (int)threadIdx.x;
    if (i >= m) return;
    const int k = deact_slack(base[i], n, m, alias);
    if (k < 0 || fail[k] == i + 1) return;  // (failed the check while basic in this row: keeps its residual)
    const int x = perm[k];
    if (x < *nact_p) tag[x] = ((unsigned long long)epoch << 32) | (unsigned)i;  // (a swept slack basic in row i)
}

__global__ __launch_bounds__(1024) void k_deact_list(const int *__restrict__ nact_p,
                                                     const unsigned long long *__restrict__ tag, unsigned epoch,
                                                     DeactList *L) {
    __shared__ int s_w[16];
    const int t = threadIdx.x;
    const int na = *nact_p;
    const int chunk = (na + 1023) / 1024, x0 = t * chunk, x1 = x0 + chunk < na ? x0 + chunk : na;
    // the chunk's tags, 8 loads in flight at a time; a bit per tagged position (chunk <= 64: at most
    // 65536 slacks, sx_launch_deactivate)
    unsigned long long bits = 0ull;
    for (int b = x0; b < x1; b += 8) {
        unsigned long long v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = b + q < x1 ? tag[b + q] : 0ull;
#pragma unroll
        for (int q = 0; q < 8; ++q)
            if (b + q < x1 && (unsigned)(v[q] >> 32) == epoch) bits |= 1ull << (b + q - x0);
    }
    int total;
    int o = block_exscan1024(__popcll(bits), s_w, &total);
    while (bits && o < SX_DEACT_CAP) {
        const int q = __builtin_ctzll(bits);
        bits &= bits - 1ull;
        L->x[o] = x0 + q;
        L->r[o] = (int)(unsigned)tag[x0 + q];
        L->bad[o] = 0;
        ++o;
    }
    if (t == 0) L->C = total < SX_DEACT_CAP ? total : SX_DEACT_CAP;
}

__global__ __launch_bounds__(256) void k_deact_check(const double *__restrict__ T, int rows, int row0, TLay tl,
                                                     int s0, DeactList *L) {
    __shared__ int s_x[1024 + 8], s_r[1024 + 8];  // (+8: the unrolled tail reads past nj)
    const int C = L->C;
    const int t = threadIdx.x, i = (int)blockIdx.x * 256 + t;
    for (int j0 = 0; j0 < C; j0 += 1024) {  // the list through LDS, 1024 entries at a time
        const int nj = C - j0 < 1024 ? C - j0 : 1024;
        __syncthreads();
        for (int q = t; q < nj; q += 256) {
            s_x[q] = s0 + L->x[j0 + q];
            s_r[q] = L->r[j0 + q];
        }
        __syncthreads();
        if (i >= rows) continue;
        for (int j = 0; j < nj; j += 8) {  // 8 loads in flight
            double v[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] = j + q < nj ? T[tl.idx(i, s_x[j + q])] : 0.0;
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const double want = i + row0 == s_r[j + q] ? 1.0 : 0.0;
                if (j + q < nj && __double_as_longlong(v[q]) != __double_as_longlong(want)) L->bad[j0 + j + q] = 1;
            }
        }
    }
}

__global__ __launch_bounds__(1024) void k_deact_plan(int *__restrict__ perm, int *__restrict__ iperm,
                                                     int *__restrict__ ucol, int *__restrict__ urow,
                                                     int *__restrict__ nact_p, int *__restrict__ fail, DeactList *L) {
    __shared__ int s_w[16];
    __shared__ int s_free[SX_DEACT_CAP];           // tail positions that receive a candidate
    __shared__ unsigned s_tail[SX_DEACT_CAP / 32];  // tail positions held by a candidate (bits)
    const int t = threadIdx.x;
    const int C = L->C, na = *nact_p;
    constexpr int PER = SX_DEACT_CAP / 1024;
    // candidates: list entries j = PER t .. PER t + PER - 1 that passed the check
    int ok[PER], nok = 0;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const int j = PER * t + q;
        ok[q] = j < C && L->bad[j] == 0;
        nok += ok[q];
        if (j < C && !ok[q]) fail[iperm[L->x[j]]] = L->r[j] + 1;  // (not listed again while basic there)
    }
    int d;
    const int before = block_exscan1024(nok, s_w, &d);
    (void)before;
    if (d == 0) {
        if (t == 0) L->nsw = 0;
        return;
    }
    const int nna = na - d;  // the swept block after
    for (int k = t; k < SX_DEACT_CAP / 32; k += 1024) s_tail[k] = 0u;
    __syncthreads();
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const int j = PER * t + q;
        if (ok[q] && L->x[j] >= nna) atomicOr(&s_tail[(L->x[j] - nna) >> 5], 1u << ((L->x[j] - nna) & 31));
    }
    __syncthreads();
    // free tail positions (not a candidate's), in order: the j-th receives the j-th outside candidate
    {
        const int chunk = (d + 1023) / 1024, y0 = t * chunk, y1 = y0 + chunk < d ? y0 + chunk : d;
        int c = 0;
        for (int y = y0; y < y1; ++y) c += !((s_tail[y >> 5] >> (y & 31)) & 1u);
        int tot;
        int o = block_exscan1024(c, s_w, &tot);
        for (int y = y0; y < y1; ++y)
            if (!((s_tail[y >> 5] >> (y & 31)) & 1u)) s_free[o++] = nna + y;
    }
    __syncthreads();
    // outside candidates (position < nna), in list (= position) order
    int nout = 0;
#pragma unroll
    for (int q = 0; q < PER; ++q) nout += ok[q] && L->x[PER * t + q] < nna;
    int nsw;
    int o = block_exscan1024(nout, s_w, &nsw);
    // read every slack involved before any write
    int kc[PER], ko[PER], Pq[PER], Qq[PER], jo[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const int j = PER * t + q;
        kc[q] = ok[q] ? iperm[L->x[j]] : -1;
        jo[q] = -1;
        if (ok[q] && L->x[j] < nna) {
            jo[q] = o++;
            Pq[q] = L->x[j];
            Qq[q] = s_free[jo[q]];
            ko[q] = iperm[Qq[q]];
        }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const int j = PER * t + q;
        if (kc[q] < 0) continue;
        const int r = L->r[j];
        urow[kc[q]] = r;
        ucol[r] = kc[q];
        if (jo[q] >= 0) {
            L->dst[jo[q]] = Pq[q];
            L->src[jo[q]] = Qq[q];
            L->row[jo[q]] = r;
            perm[kc[q]] = Qq[q];
            iperm[Qq[q]] = kc[q];
            perm[ko[q]] = Pq[q];
            iperm[Pq[q]] = ko[q];
        }
    }
    if (t == 0) {
        L->nsw = nsw;
        *nact_p = nna;
    }
}

__global__ __launch_bounds__(256) void k_deact_move(double *__restrict__ T, int rows, int row0, TLay tl, int s0,
                                                    const DeactList *__restrict__ L) {
    const int nsw = L->nsw;
    const int i = (int)blockIdx.x * 256 + (int)threadIdx.x;
    if (nsw <= 0 || i >= rows) return;
    for (int j = 0; j < nsw; ++j) {
        const int P = s0 + L->dst[j], Q = s0 + L->src[j];
        T[tl.idx(i, P)] = T[tl.idx(i, Q)];
        T[tl.idx(i, Q)] = i + row0 == L->row[j] ? 1.0 : 0.0;
    }
}

// Virtual-rank "allreduce": out = sum of the shards' contributions in rank order.  Exact,
// since all but one contribution are -0.0.
__global__ void k_sum_rows(double *out, const double *const *srcs, int nsrc, int N) {
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < N; j += gridDim.x * blockDim.x) {
        double s = srcs[0][j];
        for (int k = 1; k < nsrc; ++k) s = s + srcs[k][j];
        out[j] = s;
    }
}

// A rank's contribution to the objective-row gather (Engine::gather_d): its slice [j0, j1) (and
// d[0] on the rank holding tile 0), -0.0 elsewhere; the sum all-reduce of the ranks' contributions is then the
// whole row bit for bit (x + -0.0 == x).
__global__ void k_d_contrib(const double *__restrict__ d, double *__restrict__ out, int N, int j0, int j1, int with0) {
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < N; j += gridDim.x * blockDim.x)
        out[j] = ((j >= j0 && j < j1) || (j == 0 && with0)) ? d[j] : -0.0;
}

// ---------------------------------------------------------------------------------------
// Objective canonicalisation (updateObjectiveFunction, gaussian.cu:132-162):
//   coef[i] = d[1 + base[i]] (snapshot), then d[j] -= sum_i T[i][j] * coef[i].
// The reference sums with fp64 atomics in arrival order (nondeterministic).  Here the
// order is fixed: an fma chain over each 512-row block, then the block partials summed in
// block order -- identical on 1 or W shards because shard boundaries are 512-aligned.
__global__ void k_coef(const double *d, const int *base, int row0, int rows, double *coef) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < rows) coef[i] = d[1 + base[row0 + i]];
}

__global__ __launch_bounds__(256) void k_gemv_partials(const double *__restrict__ T, int rows, TLay tl, int N,
                                                       const double *__restrict__ coef, double *partials) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    const int k = blockIdx.y;
    if (j >= N) return;
    const int i1 = (k + 1) * SX_TILE < rows ? (k + 1) * SX_TILE : rows;
    double s = 0.0;
    int i = k * SX_TILE;
    for (; i + 4 <= i1; i += 4) {
        const double t0 = T[tl.idx(i, j)], t1 = T[tl.idx(i + 1, j)];
        const double t2 = T[tl.idx(i + 2, j)], t3 = T[tl.idx(i + 3, j)];
        s = fma(t0, coef[i], s);
        s = fma(t1, coef[i + 1], s);
        s = fma(t2, coef[i + 2], s);
        s = fma(t3, coef[i + 3], s);
    }
    for (; i < i1; ++i) s = fma(T[tl.idx(i, j)], coef[i], s);
    partials[(size_t)k * N + j] = s;
}

__global__ void k_gemv_apply(double *d, Cols c, const double *__restrict__ partials, int nblk) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= c.N) return;
    const int js = c.map(j);  // an artificial column's sum is its slack column's (identical columns)
    double s = partials[js];
    for (int k = 1; k < nblk; ++k) s = s + partials[(size_t)k * c.Ns + js];
    d[j] = d[j] - s;
}

// ---------------------------------------------------------------------------------------
// Tableau construction (fillTableu + checkColumns, twoPhaseMethod.cu:145-200, 86-111).
// A_local is the shard's slice of the column-major A: A_local[j*rows + i] = A(row0+i, j).
// 32x32 LDS transpose so both the read (along i) and the write (along j) are coalesced.
__global__ __launch_bounds__(256) void k_fill_structural(double *T, int rows, TLay tl, int n,
                                                         const double *__restrict__ A_local) {
    __shared__ double tile[32][33];
    const int i_base = blockIdx.x * 32, j_base = blockIdx.y * 32;
    for (int jj = threadIdx.y; jj < 32; jj += 8) {
        const int i = i_base + threadIdx.x, j = j_base + jj;
        tile[jj][threadIdx.x] = (i < rows && j < n) ? A_local[(size_t)j * rows + i] : 0.0;
    }
    __syncthreads();
    for (int ii = threadIdx.y; ii < 32; ii += 8) {
        const int i = i_base + ii, j = j_base + threadIdx.x;
        if (i < rows && j < n) T[tl.idx(i, 1 + j)] = tile[threadIdx.x][ii];
    }
}

// RHS, slack/artificial identities, and the b<0 quirk: a row with compare(b_i) < 0 is
// negated across ALL its entries, slack and artificial included.
__global__ void k_fill_rows(double *T, int rows, int row0, TLay tl, int n, int m, int Ns, const double *b_full) {
    const int i = blockIdx.y;
    if (i >= rows) return;
    const int gi = row0 + i;
    const double bi = b_full[gi];
    const bool neg = cmp_eps(bi, 0.0) < 0;
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < Ns; j += gridDim.x * blockDim.x) {
        double &el = T[tl.idx(i, j)];
        double x;
        if (j == 0)
            x = bi;
        else if (j <= n)
            x = el;
        else
            x = (j == 1 + n + gi || j == 1 + n + m + gi) ? 1.0 : 0.0;
        el = neg ? -x : x;
    }
}

// d: phase-1 costs (0 for x and slacks, 1 for artificials, twoPhaseMethod.cu:152-157);
// base[i] = n+m+i (fillBaseVector, :44-52).
__global__ void k_init_vectors(double *d, int N1, int n, int m, int *base) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < N1) d[t] = (t <= n + m) ? 0.0 : 1.0;
    if (t < m) base[t] = n + m + t;
}

// Phase-2 costs (twoPhaseMethod.cu:306-318): d[1..n] = -c, d[n+1..n+m] = 0, d[0] kept.
__global__ void k_phase2_costs(double *d, int n, int m, const double *c) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n) d[1 + t] = -c[t];
    if (t < m) d[1 + n + t] = 0.0;
}

// rows [i0, i0 + nr) of the tableau, stored columns [0, Ns), to / from a row-major buffer (the
// host's view of a blocked tableau: download, upload, and the synthetic sweep bench's column 0)
__global__ void k_rows_out(const double *__restrict__ T, TLay tl, int i0, int nr, int Ns, double *__restrict__ out) {
    const long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= (long long)nr * Ns) return;
    const int r = (int)(k / Ns), j = (int)(k % Ns);
    out[k] = T[tl.idx(i0 + r, j)];
}
__global__ void k_rows_in(double *__restrict__ T, TLay tl, int i0, int nr, int Ns, int j0, const double *__restrict__ in,
                          size_t ld_in) {
    const long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= (long long)nr * Ns) return;
    const int r = (int)(k / Ns), j = (int)(k % Ns);
    T[tl.idx(i0 + r, j0 + j)] = in[(size_t)r * ld_in + j];
}

__global__ void k_gather_rhs(const double *T, int rows, TLay tl, double *out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < rows) out[i] = T[tl.idx(i, 0)];
}

}  // namespace

// =========================== launchers ===========================

int sx_enter_blocks(int L) {
    int g = (L + SX_TILE - 1) / SX_TILE;
    if (g > 1024) g = 1024;
    if (g < 1) g = 1;
    return g;
}

void sx_launch_enter(const double *d, int L, TilePart *parts, DevState *st, hipStream_t s) {
    const int g = sx_enter_blocks(L);
    if (g > SX_TILE) SX_FATAL("entering vector too long for the 512-thread pass 2");
    k_argmin_pass1<<<g, SX_TILE, 0, s>>>(d + 1, L, parts, nullptr);
    k_enter_finish<<<1, SX_TILE, 0, s>>>(parts, g, st);
}

void sx_launch_ratio_select(const double *T, int rows, int row0, size_t ld, TLay tl, TilePart *tiles_local, double *colE,
                            DevState *st, int *base, bool select, double *slots, size_t slot_stride, Cols c,
                            const Pending &pd, hipStream_t s) {
    int g = (rows + SX_TILE - 1) / SX_TILE;
    if (g < 1) g = 1;  // a shard without rows still decides optimality for its own state
    if (select && g > SX_TILE) SX_FATAL("too many ratio tiles for the 512-thread pass 2");
    if (pd.q < 0 || pd.q >= SX_HMAX) SX_FATAL("pending slot out of range");
    k_ratio_select<<<g, SX_TILE, 0, s>>>(T, rows, row0, ld, tl, tiles_local, colE, st, base, select ? 1 : 0, slots,
                                         slot_stride, c, pd.F, pd.U, pd.recs, pd.PM, pd.batch, pd.q);
}

void sx_launch_select_gathered(const double *slots, size_t slot_stride, int B2, int *base, DevState *st,
                               const Pending &pd, hipStream_t s) {
    if (B2 > SX_TILE) SX_FATAL("too many ratio tiles for the 512-thread pass 2");
    k_select_gathered<<<1, SX_TILE, 0, s>>>(slots, slot_stride, B2, base, st, pd.batch, pd.q);
}

void sx_launch_select_row(const double *T, int rows, int row0, size_t ld, TLay tl, Cols c, const TilePart *tiles_all, int B2,
                          double *prow_out, int *base, DevState *st, const Pending &pd, hipStream_t s) {
    if (B2 > SX_TILE) SX_FATAL("too many ratio tiles for the 512-thread pass 2");
    const int N = c.Ns;
    int g = (N + 4 * SX_TILE - 1) / (4 * SX_TILE);
    if (g < 1) g = 1;
    if (g > 64) g = 64;
    k_select_row<<<g, SX_TILE, 0, s>>>(T, rows, row0, ld, tl, N, tiles_all, B2, prow_out, base, st, pd.F, pd.U, pd.recs,
                                       pd.PM, pd.batch, pd.q);
}

void sx_launch_pivot_row(const double *T, int rows, int row0, size_t ld, TLay tl, Cols c, double *d, const double *prow_buf,
                         size_t prow_stride, const double *colE, DevState *st, const Pending &pd,
                         TilePart *enter_parts, hipStream_t s) {
    const int B1 = (c.N - 1 + SX_TILE - 1) / SX_TILE;
    if (B1 > 256) SX_FATAL("entering vector too long for the pivot-row kernel's pass 2");
    if (B1 < 1) SX_FATAL("empty objective row");
    const int fb = rows > 0 ? (rows + 255) / 256 : 0;
    k_pivot_row<<<B1 + fb, 256, 0, s>>>(T, rows, row0, ld, tl, c, d, prow_buf, prow_stride, colE, st, pd.U, pd.F, pd.recs,
                                        pd.PM, enter_parts, pd.batch, pd.q, B1);
}

// record target of the next sweep launches (sx_set_sweep_record; null: none)
static int *g_sweep_rec = nullptr;
void sx_set_sweep_record(int *rec) { g_sweep_rec = rec; }

// blocks of a kernel resident on the whole device at once (cached per kernel: the template
// parameter is the kernel itself -- instantiations of one kernel template share a type)
template <auto kernel>
static int sweep_capacity() {
    static int cap = 0;
    if (cap == 0) {
        int per_cu = 0, dev = 0, cus = 0;
        SX_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, 256, 0));
        SX_HIP(hipGetDevice(&dev));
        SX_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
        cap = (per_cu > 0 ? per_cu : 1) * (cus > 0 ? cus : 1);
    }
    return cap;
}

// row slots per column tile: waves x (resident blocks) blocks in all, each walking its share
// of the row groups
static float g_sweep_waves = 1.0f;
void sx_set_update_waves(float w) { g_sweep_waves = w > 0.f ? w : 1.0f; }

static int row_slots(int capacity, int col_blocks, int rows, int rb, float waves = -1.f) {
    long long g = (long long)((waves > 0.f ? waves : g_sweep_waves) * (float)capacity) / col_blocks;
    const long long groups = rows > 0 ? (rows + rb - 1) / rb : 1;
    if (g > groups) g = groups;
    if (g < 1) g = 1;
    if (g > 65535) g = 65535;
    return (int)g;
}

template <int KT, int RB>
static void launch_sweep_t(double *T, int rows, size_t ld, TLay tl, int Ns, const int *nact, int s0, const Pending &pd,
                           const DevState *st, int rev, hipStream_t s) {
    const int cb = (Ns + 511) / 512;
    dim3 grid(cb, row_slots(sweep_capacity<k_sweep<KT, RB>>(), cb, rows, RB));
    k_sweep<KT, RB><<<grid, 256, 0, s>>>(T, rows, ld, tl, Ns, nact, s0, pd.F, pd.U, pd.recs, pd.PM, st, pd.batch, rev,
                                         g_sweep_rec);
}

// rows per step: 4 for batches of more than 16 pivots, else 2 (round 1 measurements)
template <int KT>
static void launch_sweep_k(double *T, int rows, size_t ld, TLay tl, int Ns, const int *nact, int s0, const Pending &pd,
                           const DevState *st, int rev, hipStream_t s) {
    if (KT > 16)
        launch_sweep_t<KT, 4>(T, rows, ld, tl, Ns, nact, s0, pd, st, rev, s);
    else
        launch_sweep_t<KT, 2>(T, rows, ld, tl, Ns, nact, s0, pd, st, rev, s);
}

// Row slots of the matrix-core sweeps (measured, profiles/r03_msweep_waves_ab.txt): the one-stage
// kernel with 2 of its 3 resident blocks per CU (4096 x 8192: 87-90 vs 95-100 us; the same at
// 32768 rows); the two-stage kernel with twice its resident grid when each block would walk 64
// strips or more (32768 x 9216: 974 vs 1006 us; at 4096 rows the resident grid stays best).  An
// explicit simplex_set_update_waves overrides both.
static int msweep_slots(int capacity, int cb, int rows, bool two_stage) {
    if (g_sweep_waves != 1.0f) return row_slots(capacity, cb, rows, 16);
    if (!two_stage) return row_slots(capacity, cb, rows, 16, 2.0f / 3.0f);
    const long long nstrip = (rows + 15) / 16, g0 = std::max(1, capacity / std::max(cb, 1));
    return row_slots(capacity, cb, rows, 16, nstrip / g0 >= 64 ? 2.0f : 1.0f);
}

static void launch_msweep(double *T, int rows, int row0, size_t ld, TLay tl, int Ns, const int *nact, int s0,
                          const Pending &pd, const DevState *st, int rev, SweepCfg cfg, int cb, hipStream_t s) {
    if (cfg.batch > SX_HMAX) {
        dim3 grid(cb, msweep_slots(sweep_capacity<k_msweep<SX_KMAX / 4>>(), cb, rows, true));
        k_msweep<SX_KMAX / 4><<<grid, 256, 0, s>>>(T, T, rows, row0, ld, tl, Ns, nact, s0, pd.F, pd.U, pd.recs,
                                                        pd.PM, pd.PM2, st, pd.batch, rev, g_sweep_rec);
    } else {
        dim3 grid(cb, msweep_slots(sweep_capacity<k_msweep<SX_HMAX / 4>>(), cb, rows, false));
        k_msweep<SX_HMAX / 4><<<grid, 256, 0, s>>>(T, T, rows, row0, ld, tl, Ns, nact, s0, pd.F, pd.U, pd.recs,
                                                        pd.PM, pd.PM2, st, pd.batch, rev, g_sweep_rec);
    }
}

void sx_launch_activate(int *perm, int *iperm, int *ucol, const int *urow, int *nact, int m, double *T, int rows,
                        int row0, size_t ld, TLay tl, int s0, const Pending &pd, const DevState *st, int slots,
                        hipStream_t s) {
    k_activate<<<1, 256, 0, s>>>(perm, iperm, ucol, urow, nact, m, T, rows, row0, ld, tl, s0, pd.U, pd.recs, st, pd.batch,
                                 0);
    if (slots > SX_HMAX)
        k_activate<<<1, 256, 0, s>>>(perm, iperm, ucol, urow, nact, m, T, rows, row0, ld, tl, s0, pd.U, pd.recs, st,
                                     pd.batch, SX_HMAX);
}

void sx_launch_deactivate(int *perm, int *iperm, int *ucol, int *urow, int *nact, const int *base, int n, int m,
                          bool alias, double *T, int rows, int row0, TLay tl, int s0, unsigned long long *tag,
                          unsigned epoch, bool check, int *fail, DeactList *L, hipStream_t s) {
    if (m <= 0) return;
    if (m > 65536) SX_FATAL("basic-slack deactivation: at most 65536 slacks");
    const int g = rows > 0 ? (rows + 255) / 256 : 1;
    k_deact_mark<<<(m + 255) / 256, 256, 0, s>>>(base, perm, nact, n, m, alias, fail, tag, epoch);
    k_deact_list<<<1, 1024, 0, s>>>(nact, tag, epoch, L);
    if (check && rows > 0) k_deact_check<<<g, 256, 0, s>>>(T, rows, row0, tl, s0, L);
    k_deact_plan<<<1, 1024, 0, s>>>(perm, iperm, ucol, urow, nact, fail, L);
    if (rows > 0) k_deact_move<<<g, 256, 0, s>>>(T, rows, row0, tl, s0, L);
}

void sx_launch_sweep(double *T, int rows, int row0, size_t ld, TLay tl, int Ns, const int *nact, int s0,
                     const Pending &pd, const DevState *st, int rev, SweepCfg cfg, hipStream_t s) {
    if (rows <= 0) return;
    if (cfg.mfma) {
        if (ld % 2 != 0 || tl.ldA % 2 != 0 || (tl.jB < Ns && (tl.jB % 256 != 0 || tl.ldB % 2 != 0 || tl.offB % 2 != 0)))
            SX_FATAL("matrix-core sweep: 16-byte rows and 256-aligned regions required");
        const int cb = (Ns + 255) / 256;
        launch_msweep(T, rows, row0, ld, tl, Ns, nact, s0, pd, st, rev, cfg, cb, s);
        return;
    }
    const int k = cfg.batch;  // pivots the sweep may have to apply (register slots)
    if (k <= 1)
        launch_sweep_k<1>(T, rows, ld, tl, Ns, nact, s0, pd, st, rev, s);
    else if (k <= 4)
        launch_sweep_k<4>(T, rows, ld, tl, Ns, nact, s0, pd, st, rev, s);
    else if (k <= 8)
        launch_sweep_k<8>(T, rows, ld, tl, Ns, nact, s0, pd, st, rev, s);
    else if (k <= 16)
        launch_sweep_k<16>(T, rows, ld, tl, Ns, nact, s0, pd, st, rev, s);
    else if (k <= SX_HMAX)
        launch_sweep_k<SX_HMAX>(T, rows, ld, tl, Ns, nact, s0, pd, st, rev, s);
    else
        SX_FATAL("the vector sweep holds at most SX_HMAX slots");
}

// LDS history of a fused batch of k pivots: one stage
static size_t batch_lds(int k) { return (size_t)(k < SX_HMAX ? k : SX_HMAX) * SX_TILE * sizeof(double); }

size_t sx_batch_granules_a() { return sx_ga_size(); }
size_t sx_batch_granules_b() { return sx_gb_size(); }

int sx_batch_obj_tile_limit() { return SX_OBJ_TILES; }

bool sx_batch_fits(int rows, Cols c, int k) {
    if (k < 1 || k > SX_KMAX || rows <= 0) return false;
    const int NA = (rows + SX_TILE - 1) / SX_TILE, NB = (c.N - 1 + SX_TILE - 1) / SX_TILE;
    if (NA > SX_TILE || NB > SX_OBJ_TILES || NB < 1) return false;
    static int per_cu[SX_KMAX + 1] = {0};
    static int cus = 0;
    if (per_cu[k] == 0) {
        int dev = 0;
        SX_HIP(hipGetDevice(&dev));
        SX_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
        SX_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_batch),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)batch_lds(SX_KMAX)));
        int n = 0;
        SX_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_batch, SX_TILE, batch_lds(k)));
        per_cu[k] = n > 0 ? n : -1;
    }
    // every block resident at once (the hand-offs wait on every block), 16 CUs to spare
    return per_cu[k] > 0 && (long long)(NA + NB) <= (long long)per_cu[k] * cus - 16;
}

void sx_launch_batch(const double *T, int rows, size_t ld, TLay tl, Cols c, double *d, double *d_save, int *base,
                     DevState *st, const Pending &pd, int k, BatchChan *chan, unsigned long long *ga,
                     unsigned long long *gb, unsigned long long *stamps, int *perm, int *iperm, int *ucol,
                     const int *urow, int *nact, int m, hipStream_t s) {
    if (!sx_batch_fits(rows, c, k)) SX_FATAL("fused batch grid does not fit the device");
    const int NA = (rows + SX_TILE - 1) / SX_TILE, NB = (c.N - 1 + SX_TILE - 1) / SX_TILE;
    k_batch<<<NA + NB, SX_TILE, batch_lds(k), s>>>(T, rows, ld, tl, c, d, d_save, base, st, pd.U, pd.F, pd.recs, pd.PM,
                                                   pd.PM2, pd.batch, k, NA, NB, chan, ga, gb, stamps, perm, iperm, ucol,
                                                   urow, nact, m);
}

bool sx_batch_mr_fits(int slots, int nb_local, int k, int grids) {
    if (k < 1 || k > SX_KMAX || slots < 1 || slots > SX_TILE) return false;  // (two stages at most)
    static int per_cu[SX_KMAX + 1] = {0};
    static int cus = 0;
    if (per_cu[k] == 0) {
        int dev = 0;
        SX_HIP(hipGetDevice(&dev));
        SX_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
        SX_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_batch_mr),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)batch_lds(SX_KMAX)));
        SX_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_batch_mr_multi),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)batch_lds(SX_KMAX)));
        // the kernel launched is k_batch_mr (RCCL / IPC ranks) or k_batch_mr_multi (ranks sharing
        // a process): the grid must fit with either
        int n = 0, n2 = 0;
        SX_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_batch_mr, SX_TILE, batch_lds(k)));
        SX_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&n2, k_batch_mr_multi, SX_TILE, batch_lds(k)));
        n = n < n2 ? n : n2;
        per_cu[k] = n > 0 ? n : -1;
    }
    return per_cu[k] > 0 && (long long)grids * (slots + nb_local) <= (long long)per_cu[k] * cus - 16;
}

void sx_launch_batch_mr(const double *T, int rows, int row0, int rpr, size_t ld, TLay tl, Cols c, double *d, double *d_save,
                        int *base, DevState *st, const Pending &pd, int k, int slots, int W, int rank, int tb0, int tb1,
                        int repl, BatchChan *chan, const unsigned long long *ga, const unsigned long long *gb,
                        const unsigned long long *gdone, const PeerView &pv, unsigned long long timeout,
                        hipStream_t s) {
    const int NBg = (c.N - 1 + SX_TILE - 1) / SX_TILE;
    if (W < 1 || W > SX_MAXW || W * slots > SX_TILE || NBg > SX_TILE || NBg < 1 || tb0 < 0 || tb1 > NBg || tb0 > tb1 ||
        (repl && (tb0 != 0 || tb1 != NBg)))
        SX_FATAL("multi-rank fused batch: bad shape");
    k_batch_mr<<<slots + (tb1 - tb0), SX_TILE, batch_lds(k), s>>>(T, rows, row0, rpr, ld, tl, c, d, d_save, base, st, pd.U, pd.F,
                                                                  pd.recs, pd.PM, pd.PM2, pd.batch, k, slots, W, rank, tb0,
                                                                  tb1, NBg, repl, chan, ga, gb, gdone, pv, timeout);
}

void sx_launch_batch_mr_multi(const MrLaunchRank *ranks, int nloc, int W, int rpr, size_t ld, TLay tl, Cols c, unsigned B,
                              int k, int slots, const PeerView &pv, unsigned long long timeout, hipStream_t s) {
    const int NBg = (c.N - 1 + SX_TILE - 1) / SX_TILE;
    if (W < 1 || W > SX_MAXW || nloc < 1 || nloc > W || W * slots > SX_TILE || NBg > SX_TILE || NBg < 1)
        SX_FATAL("multi-rank fused batch: bad shape");
    MrRanks R;
    R.first[0] = 0;
    for (int i = 0; i < nloc; ++i) {
        const MrLaunchRank &q = ranks[i];
        if (q.tb0 < 0 || q.tb1 > NBg || q.tb0 > q.tb1 || (q.repl && (q.tb0 != 0 || q.tb1 != NBg)) ||
            q.repl != ranks[0].repl)
            SX_FATAL("multi-rank fused batch: bad objective tiles");
        MrRank &x = R.r[i];
        x.T = q.T;
        x.rows = q.rows;
        x.row0 = q.row0;
        x.rank = q.rank;
        x.tb0 = q.tb0;
        x.tb1 = q.tb1;
        x.repl = q.repl;
        x.perm = q.perm;
        x.d = q.d;
        x.d_save = q.d_save;
        x.base = q.base;
        x.st = q.st;
        x.U = q.pd.U;
        x.F = q.pd.F;
        x.recs = q.pd.recs;
        x.PM = q.pd.PM;
        x.PM2 = q.pd.PM2;
        x.ch = q.chan;
        x.ga = q.ga;
        x.gb = q.gb;
        x.gdone = q.gdone;
        R.first[i + 1] = R.first[i] + slots + (q.tb1 - q.tb0);
    }
    for (int i = nloc + 1; i <= SX_MAXW; ++i) R.first[i] = R.first[nloc];
    k_batch_mr_multi<<<R.first[nloc], SX_TILE, batch_lds(k), s>>>(R, nloc, rpr, ld, tl, c, B, k, slots, W, NBg, pv,
                                                                  timeout);
}

// every XCD's L2 writes back its dirty lines (blocks are dealt over all XCDs; each block's
// first wave issues an agent-scope release: buffer_wbl2)
__global__ void k_l2_writeback() {
    if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
}
void sx_launch_l2_writeback(hipStream_t s) { k_l2_writeback<<<4096, 64, 0, s>>>(); }

// Diagnostic (simplex_set_check_pivot_rows): before the sweep reads them, every
// shard's copy of the batch's pending pivot rows U[q][0..Ns) must equal shard 0's bit for bit -- in
// every exchange form each rank holds the same rows (split objective: written into every rank by
// the tile owners; replicated: formed by every rank; per-pivot exchange: copied from one summed
// row).  Loads are system-scope (peer copies on other GPUs are read over xGMI).  A mismatch is
// counted in *bad and the first one printed (batch, slot, shard, column, both values' bits).
__global__ void k_check_u(PeerView pv, int W, size_t ld, int Ns, const DevState *__restrict__ st, unsigned B,
                          unsigned long long *bad) {
    const int cnt = st->batch_tag == B ? st->batch_count : 0;
    const long long total = (long long)cnt * Ns;
    for (long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x; k < total;
         k += (long long)gridDim.x * blockDim.x) {
        const int q = (int)(k / Ns), j = (int)(k - (long long)q * Ns);
        const u64 a = ld_sys(reinterpret_cast<const u64 *>(pv.U[0] + (size_t)q * ld + j));
        for (int r = 1; r < W; ++r) {
            const u64 b = ld_sys(reinterpret_cast<const u64 *>(pv.U[r] + (size_t)q * ld + j));
            if (a != b && atomicAdd(bad, 1ull) == 0ull)
                printf("simplex: pivot-row copies differ: batch %u slot %d shard %d column %d: %016llx vs shard 0 %016llx\n",
                       B, q, r, j, (unsigned long long)b, (unsigned long long)a);
        }
    }
}

void sx_launch_check_u(const PeerView &pv, int W, size_t ld, int Ns, const DevState *st, unsigned B,
                       unsigned long long *bad, hipStream_t s) {
    k_check_u<<<1024, 256, 0, s>>>(pv, W, ld, Ns, st, B, bad);
}

void sx_launch_sum_rows(double *out, const double *const *srcs, int nsrc, int N, hipStream_t s) {
    int g = (N + 255) / 256;
    if (g > 1024) g = 1024;
    k_sum_rows<<<g, 256, 0, s>>>(out, srcs, nsrc, N);
}

void sx_launch_d_contrib(const double *d, double *out, int N, int j0, int j1, int with0, hipStream_t s) {
    int g = (N + 255) / 256;
    if (g > 1024) g = 1024;
    if (g < 1) g = 1;
    k_d_contrib<<<g, 256, 0, s>>>(d, out, N, j0, j1, with0);
}

void sx_launch_coef(const double *d, const int *base, int row0, int rows, double *coef, hipStream_t s) {
    if (rows <= 0) return;
    k_coef<<<(rows + 255) / 256, 256, 0, s>>>(d, base, row0, rows, coef);
}

void sx_launch_gemv_partials(const double *T, int rows, TLay tl, int N, const double *coef, double *partials,
                             hipStream_t s) {
    const int nblk = (rows + SX_TILE - 1) / SX_TILE;
    if (nblk == 0) return;
    dim3 grid((N + 255) / 256, nblk);
    k_gemv_partials<<<grid, 256, 0, s>>>(T, rows, tl, N, coef, partials);
}

void sx_launch_gemv_apply(double *d, Cols c, const double *partials, int nblk, hipStream_t s) {
    k_gemv_apply<<<(c.N + 255) / 256, 256, 0, s>>>(d, c, partials, nblk);
}

void sx_launch_build_rows(double *T, int rows, int row0, TLay tl, int n, int m, int Ns, const double *A_local,
                          const double *b_full, hipStream_t s) {
    if (rows <= 0) return;
    dim3 tb(32, 8);
    dim3 tg((rows + 31) / 32, (n + 31) / 32);
    // A_local == nullptr: the structural columns are already in T (device generator)
    if (n > 0 && A_local != nullptr) k_fill_structural<<<tg, tb, 0, s>>>(T, rows, tl, n, A_local);
    int gx = (Ns + 255) / 256;
    if (gx > 64) gx = 64;
    dim3 rg(gx, rows);
    k_fill_rows<<<rg, 256, 0, s>>>(T, rows, row0, tl, n, m, Ns, b_full);
}

void sx_launch_init_vectors(double *d, int N1, int n, int m, int *base, hipStream_t s) {
    const int t = N1 > m ? N1 : m;
    k_init_vectors<<<(t + 255) / 256, 256, 0, s>>>(d, N1, n, m, base);
}

void sx_launch_phase2_costs(double *d, int n, int m, const double *c, hipStream_t s) {
    const int t = n > m ? n : m;
    if (t == 0) return;
    k_phase2_costs<<<(t + 255) / 256, 256, 0, s>>>(d, n, m, c);
}

void sx_launch_rows_out(const double *T, TLay tl, int i0, int nr, int Ns, double *out, hipStream_t s) {
    const long long n = (long long)nr * Ns;
    if (n <= 0) return;
    k_rows_out<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(T, tl, i0, nr, Ns, out);
}
void sx_launch_rows_in(double *T, TLay tl, int i0, int nr, int Ns, int j0, const double *in, size_t ld_in,
                       hipStream_t s) {
    const long long n = (long long)nr * Ns;
    if (n <= 0) return;
    k_rows_in<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(T, tl, i0, nr, Ns, j0, in, ld_in);
}

void sx_launch_gather_rhs(const double *T, int rows, TLay tl, double *out, hipStream_t s) {
    if (rows <= 0) return;
    k_gather_rhs<<<(rows + 255) / 256, 256, 0, s>>>(T, rows, tl, out);
}

void sx_launch_argmin_vector(const double *v, long long L, TilePart *parts, int *out_idx, double *out_v,
                             hipStream_t s) {
    const int g = sx_enter_blocks((int)L);
    if (g > SX_TILE) SX_FATAL("vector too long for the 512-thread pass 2");
    k_argmin_pass1<<<g, SX_TILE, 0, s>>>(v, (int)L, parts, nullptr);
    k_argmin_pass2<<<1, SX_TILE, 0, s>>>(parts, g, out_idx, out_v);
}
