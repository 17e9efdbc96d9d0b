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

// warpReduceMin (reduction.cu:10-22) on one 32-lane half of a wave64.
__device__ __forceinline__ void half_argmin(double &v, int &i) {
#pragma unroll
    for (int off = 16; off > 0; off >>= 1) {
        const double sv = __shfl_down(v, off, 32);
        const int si = __shfl_down(i, off, 32);
        if (cmp_eps(sv, v) < 0) {
            v = sv;
            i = si;
        }
    }
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

// The leaving row of the previous pivot is not yet written back to T: its current values
// are rnew[pivots & 1].  Source row i of a shard for the pivot being selected:
__device__ __forceinline__ const double *row_src(const double *T, size_t ld, int li, int pend,
                                                 const double *rnew_cur) {
    return li == pend ? rnew_cur : T + (size_t)li * ld;
}

// ---------------------------------------------------------------------------------------
// K2: ratio test (+ row selection on a single shard).  The entering variable and its
// reduced cost were produced by the previous update (or k_enter_finish).  Every block:
//  - ends the phase if compare(dmin) >= 0 (solver.cu:88),
//  - builds the ratio vector of its 512 rows (createIndicatorsVector, reduction.cu:106-114),
//    saves the pre-update entering column (the reference's rowPivot copy, solver.cu:90-94)
//    and reduces it to the tile winner + "any entry >= eps" (isLessOrEqualThanZero,
//    reduction.cu:186-201).
// With select != 0 the last block to arrive runs the pass-2 tree over the tile winners
// (minElement(knownTerms, rowPivot), solver.cu:104), declares UNBOUNDED (:96-102) or records
// the pivot: base[r] = e (:105).  With several shards the tile winners are allgathered
// first and k_select_row does that step.
__global__ __launch_bounds__(512) void k_ratio_select(const double *__restrict__ T, int rows, int row0, size_t ld,
                                                      TilePart *tiles_local, double *colE, DevState *st, int *base,
                                                      const double *__restrict__ rnew, size_t rnew_stride,
                                                      int select, double *slots, size_t slot_stride, Cols c,
                                                      int *rowlist, int *tile_cnt, int skip_zero) {
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
    const int pend = piv > 0 ? st->r - row0 : -1;
    const double *rcur = rnew + (size_t)(piv & 1) * rnew_stride;
    __shared__ double s_v[16];
    __shared__ int s_i[16];
    const int li = blockIdx.x * SX_TILE + threadIdx.x;
    double rv = DBL_MAX;
    int ri = -1;
    int elig = 0;
    bool listed = false, wide = false;
    if (li < rows) {
        const double *row = row_src(T, ld, li, pend, rcur);
        const double a = row[c.map(1 + e)];
        const double b = row[0];
        colE[li] = a;
        elig = a >= SX_EPS;
        // rows the update must sweep: a nonzero factor, or the pending row (its values live in
        // rnew until the update writes them back); every row when skipping is off
        listed = !skip_zero || a != 0.0 || li == pend;
        wide = listed && !(fabs(a) <= 1e299);  // |a / p| could overflow (p >= 1e-9), or a is not finite
        const double ratio = cmp_eps(a, 0.0) > 0 ? b / a : DBL_MAX;
        if (cmp_eps(ratio, rv) < 0) {
            rv = ratio;
            ri = row0 + li;
        }
    }
    // compact this tile's listed rows, in row order, to rowlist[tile*512 ...]
    __shared__ int s_wc[SX_TILE / 64];
    const unsigned long long bal = __ballot(listed);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (lane == 0) s_wc[wv] = __popcll(bal);
    int any = __syncthreads_or(elig);
    const int any_wide = __syncthreads_or(wide);
    int pos = 0, cnt = 0;
    for (int w = 0; w < SX_TILE / 64; ++w) {
        pos += w < wv ? s_wc[w] : 0;
        cnt += s_wc[w];
    }
    if (listed) rowlist[blockIdx.x * SX_TILE + pos + __popcll(bal & ((1ull << lane) - 1))] = li;
    if (threadIdx.x == 0) tile_cnt[blockIdx.x] = cnt | (any_wide ? SX_TILE_WIDE : 0);
    if (leader) st->touched_pairs = 0;  // counted by the update
    any |= cnt << 1;  // packed: SX_ELIG / SX_NNZ
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
        double *slot = slots + (size_t)blockIdx.x * slot_stride;
        if (threadIdx.x == 0) {
            TilePart *h = reinterpret_cast<TilePart *>(slot);
            h->v = rv;
            h->idx = ri;
            h->elig = any;
            s_ri = ri;
        }
        __syncthreads();
        const int wl = s_ri - row0;
        if (s_ri >= 0) {
            const double *src = row_src(T, ld, wl, pend, rcur);
            for (int j = threadIdx.x; j < c.Ns; j += SX_TILE) slot[2 + j] = src[j];
        }
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
    __shared__ int s_nnz;
    if (threadIdx.x == 0) s_nnz = 0;
    __syncthreads();
    if ((int)threadIdx.x < B2) {
        double cv;
        int ci;
        load_tile_sc1(tiles_local + threadIdx.x, cv, ci, te);
        if (cmp_eps(cv, tv) < 0) {
            tv = cv;
            ti = ci;
        }
        atomicAdd(&s_nnz, SX_NNZ(te));
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
            st->r_prev = st->r;
            st->r = ti;
            st->pivots = piv + 1;
            st->touched = s_nnz;
        }
    }
}

// ---------------------------------------------------------------------------------------
// K3 (several shards): every block re-derives the leaving row from the allgathered tile
// winners, checks the unbounded condition, records the pivot, and copies its chunk of the
// pre-update pivot row (the reference's copyColumn, solver.cu:24-32, is a contiguous row
// here).  Only the owner contributes the row; the others contribute -0.0, the exact
// additive identity, so the sum-allreduce reproduces the owner's row bit for bit.
__global__ __launch_bounds__(512) void k_select_row(const double *__restrict__ T, int rows, int row0, size_t ld,
                                                    int Ns, const TilePart *__restrict__ tiles_all, int B2,
                                                    double *prow_out, int *base, DevState *st,
                                                    const double *__restrict__ rnew, size_t rnew_stride, int tile0,
                                                    int nslots) {
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
    __shared__ int s_nnz;
    if (threadIdx.x == 0) s_nnz = 0;
    __syncthreads();
    if ((int)threadIdx.x >= tile0 && (int)threadIdx.x < tile0 + nslots) atomicAdd(&s_nnz, SX_NNZ(pk));
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
    const int pend = piv > 0 ? st->r - row0 : -1;
    const bool own = r >= row0 && r < row0 + rows;
    const double *src = own ? row_src(T, ld, r - row0, pend, rnew + (size_t)(piv & 1) * rnew_stride) : T;
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < Ns; j += gridDim.x * blockDim.x)
        prow_out[j] = own ? src[j] : -0.0;
    // commit the pivot once every block has read the state above: the last block to
    // arrive does it (the next kernel sees it after the launch boundary)
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned t = __hip_atomic_fetch_add(&st->ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (t == gridDim.x - 1) {
            st->ticket = 0;
            base[r] = st->e;  // solver.cu:105
            st->r_prev = st->r;
            st->r = r;
            st->pivots = piv + 1;
            st->touched = s_nnz;
        }
    }
}

// K3 (row-gather exchange): one block picks the leaving row among the gathered tile
// winners (the reference's pass-2 tree), checks the unbounded condition and records the
// pivot; the update then reads the pivot row from the winning slot.
__global__ __launch_bounds__(512) void k_select_gathered(const double *__restrict__ slots, size_t slot_stride, int B2,
                                                         int *base, DevState *st, int tile0, int nslots) {
    if (st->status != SX_NOT_ENDED) return;
    __shared__ double s_v[16];
    __shared__ int s_i[16];
    double v = DBL_MAX;
    int r = -1, pk = 0;
    __shared__ int s_nnz;
    if (threadIdx.x == 0) s_nnz = 0;
    __syncthreads();
    if ((int)threadIdx.x < B2) {
        const TilePart *h = reinterpret_cast<const TilePart *>(slots + (size_t)threadIdx.x * slot_stride);
        pk = h->elig;
        const double c = h->v;
        if (cmp_eps(c, v) < 0) {
            v = c;
            r = h->idx;
        }
        if ((int)threadIdx.x >= tile0 && (int)threadIdx.x < tile0 + nslots) atomicAdd(&s_nnz, SX_NNZ(pk));
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
            st->r_prev = st->r;
            st->r = r;
            st->pivots += 1;
            st->touched = s_nnz;
        }
    }
}

// ---------------------------------------------------------------------------------------
// K4: the rank-1 pivot update (updateContraintsMatrix + updateCostsVector, solver.cu:34-56)
//   row r:       rnew[q&1][j] = prow[j] / p     (q = pivot number; written back to T by the
//                                                next update, which reads it as row r_prev)
//   other rows:  T[i][j] = fma(-(a_ie / p), prow[j], T[i][j])   (factor hoisted per row:
//                the reference recomputes the same division per element, bit-identical)
//   objective:   d[j]    = fma(-(d_e / p),  prow[j], d[j])
// prow is the pre-update pivot row, read in place on one shard (nothing writes row r
// during the launch) or the allreduced copy on several.  Grid row 0 (dispatched first)
// updates d and finishes the NEXT pivot's entering argmin: pass 1 per 512-tile
// (reduction.cu:51-80), then the last block to arrive runs pass 2 and stores
// (e_next, dmin_next).  Grid rows >= 1: a thread owns 2 adjacent columns (one 16-byte
// load/store per row), a block covers 512 columns x RB rows.  With SNAKE the tile order
// is reversed on every other pivot, so a sweep starts on the lines the previous one wrote
// last -- still resident in the 256 MB Infinity Cache.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// 16-byte store of a tableau element pair: plain, or write-through (sc1) via a buffer
// resource so the line leaves the XCD L2 at once (no dirty-L2 write-back at the end of the
// launch, less L2 pollution on a once-touched stream)
template <bool SC1>
__device__ __forceinline__ void store_pair(double *p, double2 v, __amdgpu_buffer_rsrc_t rs, int byte_off) {
    if (SC1)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rs, byte_off, 0, 16);
    else
        *reinterpret_cast<double2 *>(p) = v;
}

// Objective row of the update (grid row 0 of either update kernel, dispatched first): d[j] =
// fma(-(d_e / p), prow[j], d[j]) and pass 1 of the NEXT entering argmin per 512-tile
// (reduction.cu:51-80); the last block to arrive runs pass 2 and stores (e_next, dmin_next).
// 512 reference threads on 256.
__device__ void objective_row(const double *__restrict__ prow, double p, double *__restrict__ d, DevState *st,
                              TilePart *enter_parts, Cols c) {
    // ---- objective row + next entering argmin (512 reference threads on 256)
    __shared__ double s_v[16];
    __shared__ int s_i[16];
    __shared__ int s_last;
    const int L = c.N - 1;
    const int B1 = (L + SX_TILE - 1) / SX_TILE;
    if ((int)blockIdx.x >= B1) return;
    const double fd = -st->dmin / p;
    if (blockIdx.x == 0 && threadIdx.x == 0) d[0] = fma(fd, prow[0], d[0]);
    double v0 = DBL_MAX, v1 = DBL_MAX;
    int i0 = -1, i1 = -1;
    const int ia = blockIdx.x * SX_TILE + threadIdx.x, ib = ia + 256;
    if (ia < L) {
        const double x = fma(fd, prow[c.map(1 + ia)], d[1 + ia]);
        d[1 + ia] = x;
        if (cmp_eps(x, v0) < 0) {
            v0 = x;
            i0 = ia;
        }
    }
    if (ib < L) {
        const double x = fma(fd, prow[c.map(1 + ib)], d[1 + ib]);
        d[1 + ib] = x;
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
    return;
}

// Exclusive prefix of the per-tile list lengths (n <= 512 tiles, 256 threads): s_pre[t] =
// first list position of tile t, s_pre[n] = total; wide = some tile flagged SX_TILE_WIDE.
// All threads of the block must call it.
__device__ int scan_tile_counts(const int *__restrict__ cnt, int n, int *s_pre, bool &wide) {
    __shared__ int s_w[4];
    const int t = threadIdx.x, lane = t & 63;
    const int ra = 2 * t < n ? cnt[2 * t] : 0;
    const int rb = 2 * t + 1 < n ? cnt[2 * t + 1] : 0;
    wide = __syncthreads_or((ra | rb) & SX_TILE_WIDE) != 0;
    const int a = SX_TILE_COUNT(ra), b = SX_TILE_COUNT(rb);
    int v = a + b;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(v, o, 64);
        if (lane >= o) v += y;
    }
    if (lane == 63) s_w[t >> 6] = v;
    __syncthreads();
    int off = 0;
    for (int w = 0; w < (t >> 6); ++w) off += s_w[w];
    const int excl = v + off - a - b;
    if (2 * t < n) s_pre[2 * t] = excl;
    if (2 * t + 1 < n) s_pre[2 * t + 1] = excl + a;
    if (t == 0) s_pre[n] = s_w[0] + s_w[1] + s_w[2] + s_w[3];
    __syncthreads();
    return s_pre[n];
}

// row of list position k (0 <= k < total): tile t holds positions [s_pre[t], s_pre[t+1]) at
// rowlist[t*512 ...]; the cursor t moves from the previous lookup, either direction
__device__ __forceinline__ int list_row(int k, int &t, const int *s_pre, const int *__restrict__ rowlist) {
    while (s_pre[t + 1] <= k) ++t;
    while (s_pre[t] > k) --t;
    return rowlist[t * SX_TILE + (k - s_pre[t])];
}

template <int RB, bool SNAKE, bool SC1>
__global__ __launch_bounds__(256) void k_update(double *__restrict__ T, int rows, int row0, size_t ld, Cols c,
                                                double *__restrict__ d, const double *__restrict__ prow_buf,
                                                size_t prow_stride, const double *__restrict__ colE, DevState *st,
                                                double *__restrict__ rnew, size_t rnew_stride,
                                                TilePart *enter_parts, const int *__restrict__ rowlist,
                                                const int *__restrict__ tile_cnt, int ntiles, int skip_zero) {
    if (st->status != SX_NOT_ENDED) return;
    const long long q = st->pivots;
    const int e = st->e;
    const int rl = st->r - row0;
    const int pl = (q >= 2 && st->r_prev != st->r) ? st->r_prev - row0 : -1;  // pending row, local
    const double *rprev = rnew + (size_t)((q - 1) & 1) * rnew_stride;
    double *rout = rnew + (size_t)(q & 1) * rnew_stride;
    const double *prow = prow_buf ? (prow_stride ? prow_buf + (size_t)(st->r / SX_TILE) * prow_stride + 2 : prow_buf)
                                  : ((q >= 2 && st->r_prev == st->r) ? rprev : T + (size_t)rl * ld);
    const double p = prow[c.map(1 + e)];
    if (blockIdx.y == 0) {
        objective_row(prow, p, d, st, enter_parts, c);
        return;
    }
    // ---- tableau rows: a fixed set of G blocks per 512-column tile sweeps the rows; each
    // thread holds its two pivot-row values for the whole sweep
    const int G = gridDim.y - 1;
    const int N = c.Ns;  // stored columns
    const int cb = (N + 511) / 512;
    if ((int)blockIdx.x >= cb) return;
    const bool rev = SNAKE && (q & 1);
    const int bx = rev ? cb - 1 - (int)blockIdx.x : (int)blockIdx.x;
    const int by = blockIdx.y - 1;
    const int j = (bx * 256 + threadIdx.x) * 2;
    const bool active = j < N, pair = j + 1 < N;
    double2 pr = make_double2(0.0, 0.0);
    if (active) {
        if (pair)
            pr = *reinterpret_cast<const double2 *>(prow + j);
        else
            pr.x = prow[j];
    }
    // Rows left out of the sweep (factor exactly +-0) keep their bits only when every
    // fma(+-0, p, x) == x: p finite (checked here, per column tile) and x != -0.0 (the engine
    // passes skip_zero only for tableaux without -0.0).  Otherwise the tile sweeps all rows.
    __shared__ int s_pre[SX_TILE + 1];
    const bool listed = skip_zero && __syncthreads_and(isfinite(pr.x) && isfinite(pr.y));
    bool wide = true;
    const int total = listed ? scan_tile_counts(tile_cnt, ntiles, s_pre, wide) : rows;
    // Columns whose pivot-row pair is (+-0, +-0) are left as they are, in every row but the
    // pending one (its values come from rprev): fma(f, +-0, x) == x for finite f and x != -0.0.
    // Those lanes' loads and stores carry an out-of-range buffer offset, which the hardware
    // drops -- no memory access, and no branch in the loop.
    const bool zc = active && listed && !wide && pr.x == 0.0 && pr.y == 0.0;
    {
        const int nzp = __syncthreads_count(active && !zc);
        if (by == 0 && threadIdx.x == 0) atomicAdd(&st->touched_pairs, nzp);
    }
    if (!active) return;
    const int ng = (total + RB - 1) / RB;
    if (by >= ng) return;
    int tc = rev ? ntiles - 1 : 0;  // tile cursor of the list lookups
    const double2 rp = make_double2(pr.x / p, pr.y / p);  // the new pivot row
    // The loop body is straight-line memory code (no loads or stores under branches), so
    // the compiler's wait counters can keep the next group's loads in flight across the
    // current group's stores.  Past the end of the list a group repeats its first row (same
    // thread, same value), and a fetch past the last group reads rprev.  The thread of an odd
    // last column moves the pair (j, j+1): j+1 < ld is row padding (or, in phase 2 without
    // aliasing, a dead artificial column).
    const int off_j = j * 8;
    const int oob = (int)(ld * 8);  // past the descriptor's range: the access is dropped
    auto fetch = [&](int g, int *row, double2 *x, double *f) {
        const bool live = g < ng;
        const int gg = rev ? ng - 1 - g : g;
#pragma unroll
        for (int k = 0; k < RB; ++k) {
            const int idx = gg * RB + k;
            int r = (live && idx < total) ? (listed ? list_row(idx, tc, s_pre, rowlist) : idx) : -1;
            r = __builtin_amdgcn_readfirstlane(r);
            row[k] = (k > 0 && r < 0) ? row[0] : r;
        }
#pragma unroll
        for (int k = 0; k < RB; ++k) {
            const bool from_prev = row[k] == pl;
            const double *src = (row[k] < 0 || from_prev) ? rprev : T + (size_t)row[k] * ld;
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(src), 0, oob,
                                                                               0x00020000);
            const bool skip = row[k] < 0 || row[k] == rl || (zc && !from_prev);
            x[k] = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(rs, skip ? oob : off_j, 0, 0));
            f[k] = row[k] >= 0 ? -colE[row[k]] / p : 0.0;
        }
    };
    auto update = [&](const int *row, const double2 *x, const double *f) {
#pragma unroll
        for (int k = 0; k < RB; ++k) {
            const bool is_r = row[k] == rl;
            double *dst = is_r ? rout : T + (size_t)row[k] * ld;
            double2 y;
            y.x = is_r ? rp.x : fma(f[k], pr.x, x[k].x);
            y.y = is_r ? rp.y : fma(f[k], pr.y, x[k].y);
            // a lane of a zero column keeps x only if f is finite (checked per row: uniform)
            const bool skip = zc && !is_r && row[k] != pl && isfinite(f[k]);
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(dst, 0, oob, 0x00020000);
            if (SC1)
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, y), rs, skip ? oob : off_j, 0, 16);
            else
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, y), rs, skip ? oob : off_j, 0, 0);
        }
    };
    // software pipeline, ping-pong between two register sets: the loads of group g+G are in
    // flight while group g is updated
    int ra[RB], rb_[RB];
    double2 xa[RB], xb[RB];
    double fa[RB], fb[RB];
    fetch(by, ra, xa, fa);
    for (int g = by; g < ng; g += 2 * G) {
        fetch(g + G, rb_, xb, fb);
        update(ra, xa, fa);
        if (g + G >= ng) break;
        fetch(g + 2 * G, ra, xa, fa);
        update(rb_, xb, fb);
    }
}

// One-shot variant of the update: one block per (512 columns, RB rows), the whole tableau in
// one grid -- the hardware's in-order dispatch keeps the active window of rows tight, which
// streams best when every row is swept.  Zero-factor rows are skipped per thread (same
// exactness conditions as the list sweep) but their blocks still run.
template <int RB, bool SNAKE, bool SC1>
__global__ __launch_bounds__(256) void k_update_grid(double *__restrict__ T, int rows, int row0, size_t ld, Cols c,
                                                     double *__restrict__ d, const double *__restrict__ prow_buf,
                                                     size_t prow_stride, const double *__restrict__ colE,
                                                     DevState *st, double *__restrict__ rnew, size_t rnew_stride,
                                                     TilePart *enter_parts, int skip_zero) {
    if (st->status != SX_NOT_ENDED) return;
    const long long q = st->pivots;
    const int rl = st->r - row0;
    const int pl = (q >= 2 && st->r_prev != st->r) ? st->r_prev - row0 : -1;
    const double *rprev = rnew + (size_t)((q - 1) & 1) * rnew_stride;
    double *rout = rnew + (size_t)(q & 1) * rnew_stride;
    const double *prow = prow_buf ? (prow_stride ? prow_buf + (size_t)(st->r / SX_TILE) * prow_stride + 2 : prow_buf)
                                  : ((q >= 2 && st->r_prev == st->r) ? rprev : T + (size_t)rl * ld);
    const double p = prow[c.map(1 + st->e)];
    if (blockIdx.y == 0) {
        objective_row(prow, p, d, st, enter_parts, c);
        return;
    }
    const int rg = gridDim.y - 1;
    const int N = c.Ns;
    const int cb = (N + 511) / 512;
    if ((int)blockIdx.x >= cb) return;
    int bx = blockIdx.x, by = blockIdx.y - 1;
    if (SNAKE && (q & 1)) {
        bx = cb - 1 - bx;
        by = rg - 1 - by;
    }
    __shared__ double s_f[RB];
    const int i0 = by * RB;
    if ((int)threadIdx.x < RB) {
        const int i = i0 + threadIdx.x;
        s_f[threadIdx.x] = (i < rows) ? -colE[i] / p : 0.0;
    }
    __syncthreads();
    const int j = (bx * 256 + threadIdx.x) * 2;
    if (j >= N) return;
    const int nrow = rows - i0 < RB ? rows - i0 : RB;
    // pair (j, j+1) always: j+1 < ld (see k_update)
    const double2 pr = *reinterpret_cast<const double2 *>(prow + j);
    const bool fin = skip_zero && isfinite(pr.x) && isfinite(pr.y);
    double *base = T + (size_t)i0 * ld + j;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(T + (size_t)i0 * ld, 0, (int)(RB * ld * 8), 0x00020000);
    bool skip[RB];
    double2 x[RB];
#pragma unroll
    for (int k = 0; k < RB; ++k) {
        skip[k] = k >= nrow || i0 + k == rl || (fin && s_f[k] == 0.0 && i0 + k != pl);
        if (!skip[k]) x[k] = *reinterpret_cast<const double2 *>(i0 + k == pl ? rprev + j : base + (size_t)k * ld);
    }
#pragma unroll
    for (int k = 0; k < RB; ++k) {
        if (k < nrow && i0 + k == rl)
            *reinterpret_cast<double2 *>(rout + j) = make_double2(pr.x / p, pr.y / p);
        if (skip[k]) continue;
        x[k].x = fma(s_f[k], pr.x, x[k].x);
        x[k].y = fma(s_f[k], pr.y, x[k].y);
        store_pair<SC1>(base + (size_t)k * ld, x[k], rs, (int)(((size_t)k * ld + j) * 8));
    }
}

// Phase end: write the last pivot row back from rnew[pivots & 1] (idempotent).
__global__ void k_flush_row(double *T, int rows, int row0, size_t ld, int Ns, const double *rnew, size_t rnew_stride,
                            const DevState *st) {
    const long long q = st->pivots;
    if (q <= 0) return;
    const int rl = st->r - row0;
    if (rl < 0 || rl >= rows) return;
    const double *src = rnew + (size_t)(q & 1) * rnew_stride;
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < Ns; j += gridDim.x * blockDim.x)
        T[(size_t)rl * ld + j] = src[j];
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

__global__ __launch_bounds__(256) void k_gemv_partials(const double *__restrict__ T, int rows, size_t ld, int N,
                                                       const double *__restrict__ coef, double *partials) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    const int k = blockIdx.y;
    if (j >= N) return;
    const int i1 = (k + 1) * SX_TILE < rows ? (k + 1) * SX_TILE : rows;
    double s = 0.0;
    const double *col = T + j;
    int i = k * SX_TILE;
    for (; i + 4 <= i1; i += 4) {
        const double t0 = col[(size_t)i * ld], t1 = col[(size_t)(i + 1) * ld];
        const double t2 = col[(size_t)(i + 2) * ld], t3 = col[(size_t)(i + 3) * ld];
        s = fma(t0, coef[i], s);
        s = fma(t1, coef[i + 1], s);
        s = fma(t2, coef[i + 2], s);
        s = fma(t3, coef[i + 3], s);
    }
    for (; i < i1; ++i) s = fma(col[(size_t)i * ld], coef[i], s);
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
__global__ __launch_bounds__(256) void k_fill_structural(double *T, int rows, size_t ld, int n,
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
        if (i < rows && j < n) T[(size_t)i * ld + 1 + j] = tile[threadIdx.x][ii];
    }
}

// RHS, slack/artificial identities, and the b<0 quirk: a row with compare(b_i) < 0 is
// negated across ALL its entries, slack and artificial included.
__global__ void k_fill_rows(double *T, int rows, int row0, size_t ld, int n, int m, int Ns, const double *b_full) {
    const int i = blockIdx.y;
    if (i >= rows) return;
    const int gi = row0 + i;
    const double bi = b_full[gi];
    const bool neg = cmp_eps(bi, 0.0) < 0;
    double *row = T + (size_t)i * ld;
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < Ns; j += gridDim.x * blockDim.x) {
        double x;
        if (j == 0)
            x = bi;
        else if (j <= n)
            x = row[j];
        else
            x = (j == 1 + n + gi || j == 1 + n + m + gi) ? 1.0 : 0.0;
        row[j] = neg ? -x : x;
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

__global__ void k_gather_rhs(const double *T, int rows, size_t ld, double *out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < rows) out[i] = T[(size_t)i * ld];
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

void sx_launch_ratio_select(const double *T, int rows, int row0, size_t ld, TilePart *tiles_local, double *colE,
                            DevState *st, int *base, const double *rnew, size_t rnew_stride, bool select,
                            double *slots, size_t slot_stride, Cols c, int *rowlist, int *tile_cnt, int skip_zero,
                            hipStream_t s) {
    int g = (rows + SX_TILE - 1) / SX_TILE;
    if (g < 1) g = 1;  // a shard without rows still decides optimality for its own state
    if (select && g > SX_TILE) SX_FATAL("too many ratio tiles for the 512-thread pass 2");
    k_ratio_select<<<g, SX_TILE, 0, s>>>(T, rows, row0, ld, tiles_local, colE, st, base, rnew, rnew_stride,
                                         select ? 1 : 0, slots, slot_stride, c, rowlist, tile_cnt, skip_zero);
}

void sx_launch_select_gathered(const double *slots, size_t slot_stride, int B2, int *base, DevState *st,
                               int tile0, int nslots, hipStream_t s) {
    if (B2 > SX_TILE) SX_FATAL("too many ratio tiles for the 512-thread pass 2");
    k_select_gathered<<<1, SX_TILE, 0, s>>>(slots, slot_stride, B2, base, st, tile0, nslots);
}

void sx_launch_select_row(const double *T, int rows, int row0, size_t ld, Cols c, const TilePart *tiles_all, int B2,
                          double *prow_out, int *base, DevState *st, const double *rnew, size_t rnew_stride,
                          int tile0, int nslots, hipStream_t s) {
    if (B2 > SX_TILE) SX_FATAL("too many ratio tiles for the 512-thread pass 2");
    const int N = c.Ns;
    int g = (N + 4 * SX_TILE - 1) / (4 * SX_TILE);
    if (g < 1) g = 1;
    if (g > 64) g = 64;
    k_select_row<<<g, SX_TILE, 0, s>>>(T, rows, row0, ld, N, tiles_all, B2, prow_out, base, st, rnew, rnew_stride,
                                       tile0, nslots);
}

// blocks of a kernel resident on the whole device at once
template <typename K>
static int update_capacity(K kernel) {
    static int cap = 0;  // per kernel instantiation
    if (cap == 0) {
        int per_cu = 0, dev = 0, cus = 0;
        SX_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, 256, 0));
        SX_HIP(hipGetDevice(&dev));
        SX_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
        cap = (per_cu > 0 ? per_cu : 1) * (cus > 0 ? cus : 1);
    }
    return cap;
}

// row-sweeping blocks per column tile: the whole grid (objective row + G rows of tiles)
// resident in one wave, each block looping over its share of the row groups
static float g_update_waves = 2.0f;
void sx_set_update_waves(float w) { g_update_waves = w > 0.f ? w : 2.0f; }

static int row_slots(int capacity, int col_blocks, int rows, int rb) {
    long long g = (long long)(g_update_waves * (float)capacity) / col_blocks - 1;
    const long long groups = rows > 0 ? (rows + rb - 1) / rb : 1;
    if (g > groups) g = groups;
    if (g < 1) g = 1;
    if (g > 65535 - 1) g = 65535 - 1;
    return (int)g;
}

template <int RB>
static void launch_update_rb(dim3 grid, bool snake, bool sc1, double *T, int rows, int row0, size_t ld, Cols N,
                             double *d, const double *prow_buf, size_t prow_stride, const double *colE, DevState *st,
                             double *rnew, size_t rnew_stride, TilePart *enter_parts, const int *rowlist,
                             const int *tile_cnt, int ntiles, int skip_zero, bool one_shot, hipStream_t s) {
#define SX_UPD(SN, SC)                                                                                           \
    do {                                                                                                         \
        if (one_shot) {                                                                                          \
            grid.y = 1 + (rows > 0 ? (rows + RB - 1) / RB : 0);                                                  \
            k_update_grid<RB, SN, SC><<<grid, 256, 0, s>>>(T, rows, row0, ld, N, d, prow_buf, prow_stride, colE,  \
                                                           st, rnew, rnew_stride, enter_parts, skip_zero);      \
        } else {                                                                                                 \
            grid.y = 1 + row_slots(update_capacity(k_update<RB, SN, SC>), grid.x, rows, RB);                    \
            k_update<RB, SN, SC><<<grid, 256, 0, s>>>(T, rows, row0, ld, N, d, prow_buf, prow_stride, colE, st,   \
                                                      rnew, rnew_stride, enter_parts, rowlist, tile_cnt, ntiles,  \
                                                      skip_zero);                                                \
        }                                                                                                        \
    } while (0)
    if (snake) {
        if (sc1)
            SX_UPD(true, true);
        else
            SX_UPD(true, false);
    } else {
        if (sc1)
            SX_UPD(false, true);
        else
            SX_UPD(false, false);
    }
#undef SX_UPD
}

void sx_launch_update(double *T, int rows, int row0, size_t ld, Cols N, double *d, const double *prow_buf,
                      size_t prow_stride, const double *colE, DevState *st, double *rnew, size_t rnew_stride,
                      TilePart *enter_parts, const int *rowlist, const int *tile_cnt, UpdateCfg cfg, hipStream_t s) {
    const int B1 = (N.N - 1 + SX_TILE - 1) / SX_TILE;
    if (B1 > 256) SX_FATAL("entering vector too long for the update's pass 2");
    int cols_blocks = (N.Ns + 511) / 512;
    if (cols_blocks < B1) cols_blocks = B1;
    const int ntiles = rows > 0 ? (rows + SX_TILE - 1) / SX_TILE : 1;  // k_ratio_select's grid
    if (ntiles > SX_TILE) SX_FATAL("too many row tiles for the update's list scan");
    dim3 grid(cols_blocks, 2);
    const bool sn = cfg.snake != 0, sc = cfg.sc1 != 0;
#define SX_RB(R)                                                                                             \
    launch_update_rb<R>(grid, sn, sc, T, rows, row0, ld, N, d, prow_buf, prow_stride, colE, st, rnew, rnew_stride, \
                        enter_parts, rowlist, tile_cnt, ntiles, cfg.skip_zero, cfg.one_shot != 0, s)
    switch (cfg.rows_per_block) {
    case 1: SX_RB(1); break;
    case 2: SX_RB(2); break;
    case 4: SX_RB(4); break;
    default: SX_RB(8); break;
    }
#undef SX_RB
}

void sx_launch_flush_row(double *T, int rows, int row0, size_t ld, int Ns, const double *rnew, size_t rnew_stride,
                         const DevState *st, hipStream_t s) {
    if (rows <= 0) return;
    int g = (Ns + 255) / 256;
    if (g > 256) g = 256;
    k_flush_row<<<g, 256, 0, s>>>(T, rows, row0, ld, Ns, rnew, rnew_stride, st);
}

void sx_launch_sum_rows(double *out, const double *const *srcs, int nsrc, int N, hipStream_t s) {
    int g = (N + 255) / 256;
    if (g > 1024) g = 1024;
    k_sum_rows<<<g, 256, 0, s>>>(out, srcs, nsrc, N);
}

void sx_launch_coef(const double *d, const int *base, int row0, int rows, double *coef, hipStream_t s) {
    if (rows <= 0) return;
    k_coef<<<(rows + 255) / 256, 256, 0, s>>>(d, base, row0, rows, coef);
}

void sx_launch_gemv_partials(const double *T, int rows, size_t ld, int N, const double *coef, double *partials,
                             hipStream_t s) {
    const int nblk = (rows + SX_TILE - 1) / SX_TILE;
    if (nblk == 0) return;
    dim3 grid((N + 255) / 256, nblk);
    k_gemv_partials<<<grid, 256, 0, s>>>(T, rows, ld, N, coef, partials);
}

void sx_launch_gemv_apply(double *d, Cols c, const double *partials, int nblk, hipStream_t s) {
    k_gemv_apply<<<(c.N + 255) / 256, 256, 0, s>>>(d, c, partials, nblk);
}

void sx_launch_build_rows(double *T, int rows, int row0, size_t ld, int n, int m, int Ns, const double *A_local,
                          const double *b_full, hipStream_t s) {
    if (rows <= 0) return;
    dim3 tb(32, 8);
    dim3 tg((rows + 31) / 32, (n + 31) / 32);
    // A_local == nullptr: the structural columns are already in T (device generator)
    if (n > 0 && A_local != nullptr) k_fill_structural<<<tg, tb, 0, s>>>(T, rows, ld, n, A_local);
    int gx = (Ns + 255) / 256;
    if (gx > 64) gx = 64;
    dim3 rg(gx, rows);
    k_fill_rows<<<rg, 256, 0, s>>>(T, rows, row0, ld, n, m, Ns, b_full);
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

void sx_launch_gather_rhs(const double *T, int rows, size_t ld, double *out, hipStream_t s) {
    if (rows <= 0) return;
    k_gather_rhs<<<(rows + 255) / 256, 256, 0, s>>>(T, rows, ld, out);
}

void sx_launch_argmin_vector(const double *v, long long L, TilePart *parts, int *out_idx, double *out_v,
                             hipStream_t s) {
    const int g = sx_enter_blocks((int)L);
    if (g > SX_TILE) SX_FATAL("vector too long for the 512-thread pass 2");
    k_argmin_pass1<<<g, SX_TILE, 0, s>>>(v, (int)L, parts, nullptr);
    k_argmin_pass2<<<1, SX_TILE, 0, s>>>(parts, g, out_idx, out_v);
}
