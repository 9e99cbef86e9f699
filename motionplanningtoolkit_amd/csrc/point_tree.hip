// point_tree.hip -- exact 1-NN over a tree snapshot with a packed Morton tree.
//
// Replaces FLANN_KDTreeWrapper::nearest (utilities/flannkdtreewrapper.hpp:57-89) for trees
// that do not fill the sampling box: an RRT grows from its start, so most uniform samples
// lie far from every node, and a uniform grid over the sampling box walks many empty rings
// for them.  Here the cost of a query depends on the tree's shape, not on where it lies.
//
// Build (every round, stream-ordered, no host sync; five launches + the sort): bounding box
// of the live nodes -> code plan (below) -> 30-bit interleaved code per node -> hipcub radix
// sort -> coordinates and ids gathered into code order with the leaf boxes (8 consecutive
// points) -> the 8-ary levels above them in one launch, each box the float-widened bounds over
// all state dims (a lower bound on FLANN's squared L2).
//
// Query: 8 lanes per query walk the tree with a per-group LDS stack.  At an inner node the
// lanes test its 8 children's boxes against the best distance so far and push the survivors
// nearest-last (so the nearest is popped first); at a leaf each lane computes one point's
// distance in FLANN's L2<double> order and the group merges (d2, id) by xor-shuffles.  Ties
// resolve to the lowest id (nn_better), so results equal the brute-force scan bit for bit.
#include <hipcub/hipcub.hpp>

#include "point_tree.h"
#include "grid_nn.h"

namespace mpt {

namespace {

__host__ __device__ __forceinline__ int64_t lvl_size(int64_t n, int l) {
    return (n + (int64_t(1) << (3 * l)) - 1) >> (3 * l);
}
__host__ __device__ __forceinline__ int64_t lvl_off(int64_t n_upper, int l) {
    int64_t o = 0;
    for (int k = 1; k < l; ++k) o += lvl_size(n_upper, k);
    return o;
}
__device__ __forceinline__ int64_t live_n(const PointTreeDev &T) {
    const int64_t n = *T.n_dev;
    return n < T.n_upper ? n : T.n_upper;
}

// Codes over ALL state dims with one common quantisation step h (cubic cells in raw state
// units, the units of FLANN's L2): dim j gets b_j = ceil(log2(extent_j / h)) bits, h the
// smallest step for which sum b_j <= 30, and bits interleave from the most significant level
// down, a level taking the dims still wider than it.  Widest dims are split first, as a
// kd-tree would; leaves then hold points close in every dim, so their boxes prune on the
// non-spatial dims as well.  The bounding box comes from the device (no host sync).
constexpr int kCodeBits = 30;

}  // namespace

struct CodePlan {
    double lo[kPtMaxDim], scale[kPtMaxDim];
    uint32_t qmax[kPtMaxDim];
    int32_t n;                       // code bits used
    int8_t dim[kCodeBits], bit[kCodeBits];  // MSB first
};

namespace {

__device__ __forceinline__ unsigned long long order_key_pt(double x) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(x);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double key_value_pt(unsigned long long k) {
    const unsigned long long b = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
    return __longlong_as_double((long long)b);
}

// Code plan from the box (the first wave of the last k_pt_bbox workgroup): lane k-1 sizes
// level k (h = emax / 2^k); the plan takes the finest level before the first whose bit total
// exceeds the code.  The box is reset to empty for the next build.  All threads of the
// workgroup must call it (barriers).
__device__ void pt_plan(int32_t d, unsigned long long *__restrict__ box, CodePlan *__restrict__ plan,
                        const SpreadOut &sp) {
    __shared__ double s_lo[kPtMaxDim], s_ext[kPtMaxDim];
    __shared__ int32_t s_b[kPtMaxDim];
    const int t = threadIdx.x;
    if (t == 0 && sp.host_out) {  // the engine's MPT_NN_AUTO feedback (grid_nn.h SpreadOut)
        for (int j = 0; j < 3; ++j) {
            sp.host_out[j] = j < sp.gd ? box[sp.dims[j]] : ~0ull;
            sp.host_out[3 + j] = j < sp.gd ? box[kPtMaxDim + sp.dims[j]] : 0ull;
        }
        __threadfence_system();
    }
    if (t < d) {
        const double lo = key_value_pt(box[t]), hi = key_value_pt(box[kPtMaxDim + t]);
        s_lo[t] = lo;
        s_ext[t] = hi > lo ? hi - lo : 0.0;
    }
    __syncthreads();
    if (t < kPtMaxDim) {
        box[t] = ~0ull;
        box[kPtMaxDim + t] = 0ull;
    }
    double emax = 0.0;
    for (int j = 0; j < d; ++j) emax = s_ext[j] > emax ? s_ext[j] : emax;
    bool fail = false;
    if (emax > 0.0 && t < kCodeBits) {
        const int k = t + 1;
        const double h = ldexp(emax, -k);
        int32_t tot = 0;
        for (int j = 0; j < d; ++j) {
            int32_t bj = 0;
            while (bj < k && ldexp(h, bj) < s_ext[j]) ++bj;
            tot += bj;
        }
        fail = tot > kCodeBits;
    }
    const unsigned long long fm = __ballot(fail);
    const int kstar = emax > 0.0 ? (fm ? __ffsll((long long)fm) - 1 : kCodeBits) : 0;
    if (t < d) {
        int32_t bj = 0;
        if (kstar > 0) {
            const double h = ldexp(emax, -kstar);
            while (bj < kstar && ldexp(h, bj) < s_ext[t]) ++bj;
        }
        s_b[t] = bj;
        plan->lo[t] = s_lo[t];
        plan->qmax[t] = bj > 0 ? (1u << bj) - 1 : 0u;
        plan->scale[t] = bj > 0 ? ldexp(1.0, bj) / s_ext[t] : 0.0;
    }
    __syncthreads();
    if (t != 0) return;
    int32_t bmax = 0;
    for (int j = 0; j < d; ++j) bmax = s_b[j] > bmax ? s_b[j] : bmax;
    int32_t n = 0;
    for (int b = bmax - 1; b >= 0; --b)
        for (int j = 0; j < d; ++j)
            if (s_b[j] > b) {
                plan->dim[n] = (int8_t)j;
                plan->bit[n] = (int8_t)b;
                ++n;
            }
    plan->n = n;
}

// per-dim min / max of the live points as order keys: box[0..d) min, box[kPtMaxDim..) max
// D > 0: the state dim at compile time (rows loaded whole, several points in flight); D = 0:
// the run-time d
template <int D = 0>
__device__ __forceinline__ void pt_bbox(const double *__restrict__ pts, int32_t d_rt, int64_t n_upper,
                                        const int64_t *__restrict__ n_dev, unsigned long long *__restrict__ box,
                                        unsigned int *__restrict__ ticket, CodePlan *__restrict__ plan,
                                        const SpreadOut &sp, int64_t blk, int64_t nblk) {
    const int32_t d = D > 0 ? D : d_rt;
    __shared__ unsigned long long s_min[kPtMaxDim], s_max[kPtMaxDim];
    if (threadIdx.x < kPtMaxDim) {
        s_min[threadIdx.x] = ~0ull;
        s_max[threadIdx.x] = 0ull;
    }
    __syncthreads();
    const int64_t n = *n_dev < n_upper ? *n_dev : n_upper;
    // one pass over each point's row (all dims at once: a per-dim pass re-reads every row d
    // times, which the joint build's 256 trees cannot keep in L2)
    unsigned long long mn[kPtMaxDim], mx[kPtMaxDim];
#pragma unroll
    for (int j = 0; j < kPtMaxDim; ++j) {
        mn[j] = ~0ull;
        mx[j] = 0ull;
    }
    if constexpr (D > 0) {
        // U rows loaded before any is reduced (a row past n repeats the first: min / max
        // do not change), instead of one guarded load and its wait per coordinate
        constexpr int U = D >= 15 ? 2 : 4;
        const int64_t stride = nblk * blockDim.x;
        for (int64_t i0 = blk * blockDim.x + threadIdx.x; i0 < n; i0 += U * stride) {
            double v[U][D];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t i = i0 + u * stride < n ? i0 + u * stride : i0;
#pragma unroll
                for (int j = 0; j < D; ++j) v[u][j] = pts[i * D + j];
            }
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int j = 0; j < D; ++j) {
                    const unsigned long long k = order_key_pt(v[u][j]);
                    mn[j] = k < mn[j] ? k : mn[j];
                    mx[j] = k > mx[j] ? k : mx[j];
                }
        }
    } else {
        for (int64_t i = blk * blockDim.x + threadIdx.x; i < n; i += nblk * blockDim.x) {
#pragma unroll
            for (int j = 0; j < kPtMaxDim; ++j)
                if (j < d) {
                    const unsigned long long k = order_key_pt(pts[i * d + j]);
                    mn[j] = k < mn[j] ? k : mn[j];
                    mx[j] = k > mx[j] ? k : mx[j];
                }
        }
    }
#pragma unroll
    for (int j = 0; j < kPtMaxDim; ++j) {
        if (j >= d) break;
        // one LDS atomic per wave, not per lane (256 same-address 64-bit atomics serialise)
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const unsigned long long omn = __shfl_xor(mn[j], off), omx = __shfl_xor(mx[j], off);
            mn[j] = omn < mn[j] ? omn : mn[j];
            mx[j] = omx > mx[j] ? omx : mx[j];
        }
        if ((threadIdx.x & 63) == 0) {
            atomicMin(&s_min[j], mn[j]);
            atomicMax(&s_max[j], mx[j]);
        }
    }
    __syncthreads();
    if (threadIdx.x < (unsigned)d) {
        atomicMin(box + threadIdx.x, s_min[threadIdx.x]);
        atomicMax(box + kPtMaxDim + threadIdx.x, s_max[threadIdx.x]);
    }
    if (!plan) return;  // the plan runs as its own launch (k_pt_plan)
    // the last workgroup to finish turns the box into the code plan (no separate launch)
    __shared__ bool last;
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) last = atomicAdd(ticket, 1u) == nblk - 1;
    __syncthreads();
    if (!last) return;
    __threadfence();
    if (threadIdx.x == 0) *ticket = 0u;
    pt_plan(d, box, plan, sp);
}

__global__ __launch_bounds__(256) void k_pt_bbox(const double *__restrict__ pts, int32_t d, int64_t n_upper,
                                                 const int64_t *__restrict__ n_dev, unsigned long long *__restrict__ box,
                                                 unsigned int *__restrict__ ticket, CodePlan *__restrict__ plan,
                                                 SpreadOut sp) {
    pt_bbox(pts, d, n_upper, n_dev, box, ticket, plan, sp, blockIdx.x, gridDim.x);
}

template <int D = 0>
__device__ __forceinline__ void pt_morton(const double *__restrict__ pts, int32_t d_rt, int64_t n_upper,
                                          const int64_t *__restrict__ n_dev, const CodePlan *__restrict__ plan,
                                          uint32_t *__restrict__ keys, int32_t *__restrict__ vals, int64_t blk) {
    const int64_t i = blk * blockDim.x + threadIdx.x;
    if (i >= n_upper) return;
    const int64_t n = *n_dev < n_upper ? *n_dev : n_upper;
    vals[i] = (int32_t)i;
    if (i >= n) {
        keys[i] = 0xffffffffu;  // past the live count: sorted to the end
        return;
    }
    const int32_t d = D > 0 ? D : d_rt;
    uint32_t q[kPtMaxDim];
    if constexpr (D > 0) {
        double x[D];  // the row loaded whole before any use
#pragma unroll
        for (int j = 0; j < D; ++j) x[j] = pts[i * D + j];
#pragma unroll
        for (int j = 0; j < D; ++j) {
            const double u = (x[j] - plan->lo[j]) * plan->scale[j];
            const uint32_t m = plan->qmax[j];
            q[j] = u <= 0.0 ? 0u : (u >= (double)m ? m : (uint32_t)u);
        }
    } else {
        for (int j = 0; j < d; ++j) {
            const double u = (pts[i * d + j] - plan->lo[j]) * plan->scale[j];
            const uint32_t m = plan->qmax[j];
            q[j] = u <= 0.0 ? 0u : (u >= (double)m ? m : (uint32_t)u);
        }
    }
    uint32_t code = 0;
    const int32_t nb = plan->n;
    for (int k = 0; k < nb; ++k) {
        const int32_t dk = plan->dim[k];
        uint32_t v = q[0];
        if constexpr (D > 0) {  // a select over the row instead of an indexed register read
#pragma unroll
            for (int j = 1; j < D; ++j)
                if (j == dk) v = q[j];
        } else {
            v = q[dk];
        }
        code = (code << 1) | ((v >> plan->bit[k]) & 1u);
    }
    keys[i] = code;
}

__global__ void k_pt_morton(const double *__restrict__ pts, int32_t d, int64_t n_upper, const int64_t *__restrict__ n_dev,
                            const CodePlan *__restrict__ plan, uint32_t *__restrict__ keys, int32_t *__restrict__ vals) {
    pt_morton(pts, d, n_upper, n_dev, plan, keys, vals, blockIdx.x);
}

// Coordinates and ids into code order, and the level-1 boxes with them: a leaf is 8
// consecutive sorted points, i.e. 8 consecutive lanes, so its bounds are an 8-lane reduction.
template <int D = 0>
__device__ __forceinline__ void pt_gather(const double *__restrict__ pts, int32_t d_rt, int64_t n_upper,
                                          const int64_t *__restrict__ n_dev, const int32_t *__restrict__ order,
                                          double *__restrict__ spts, int32_t *__restrict__ sids,
                                          float *__restrict__ leaf_boxes, int64_t blk) {
    const int64_t i = blk * blockDim.x + threadIdx.x;
    const int64_t n = *n_dev < n_upper ? *n_dev : n_upper;
    const bool live = i < n;  // no early exit: the leaf reduction needs all 8 lanes
    const int32_t d = D > 0 ? D : d_rt;
    const int32_t src = live ? order[i] : 0;
    if (live) sids[i] = src + 1;
    constexpr int DM = D > 0 ? D : 1;
    double row[DM];
    if constexpr (D > 0) {  // the source row loaded whole (row 0 stands in past the live count)
#pragma unroll
        for (int j = 0; j < D; ++j) row[j] = pts[(int64_t)src * D + j];
    }
#pragma unroll
    for (int j = 0; j < d; ++j) {
        const double x = D > 0 ? (live ? row[j < DM ? j : 0] : 0.0) : (live ? pts[(int64_t)src * d + j] : 0.0);
        if (live) spts[i * d + j] = x;
        double lo = live ? x : __builtin_huge_val(), hi = live ? x : -__builtin_huge_val();
#pragma unroll
        for (int off = kPtFan / 2; off > 0; off >>= 1) {
            const double olo = __shfl_xor(lo, off, kPtFan), ohi = __shfl_xor(hi, off, kPtFan);
            lo = olo < lo ? olo : lo;
            hi = ohi > hi ? ohi : hi;
        }
        if (live && (i & (kPtFan - 1)) == 0) {
            float *b = leaf_boxes + (i / kPtFan) * 2 * d;
            b[j] = widen_lo(lo);
            b[d + j] = widen_hi(hi);
        }
    }
}

__global__ __launch_bounds__(256) void k_pt_gather(const double *__restrict__ pts, int32_t d, int64_t n_upper,
                                                   const int64_t *__restrict__ n_dev, const int32_t *__restrict__ order,
                                                   double *__restrict__ spts, int32_t *__restrict__ sids,
                                                   float *__restrict__ leaf_boxes) {
    pt_gather(pts, d, n_upper, n_dev, order, spts, sids, leaf_boxes, blockIdx.x);
}

// (box j, dim k) of level l >= 2: the bounds of its (up to) 8 children at level l - 1
__device__ __forceinline__ void pt_up_box(const PointTreeDev &T, int64_t n, int l, float *__restrict__ boxes,
                                          int64_t j, int k) {
    const int d = T.d;
    const float *child = boxes + lvl_off(T.n_upper, l - 1) * 2 * d;
    float *b = boxes + (lvl_off(T.n_upper, l) + j) * 2 * d;
    const int64_t c0 = j * kPtFan, nc = lvl_size(n, l - 1), c1 = c0 + kPtFan < nc ? c0 + kPtFan : nc;
    float lo = child[c0 * 2 * d + k], hi = child[c0 * 2 * d + d + k];
#pragma unroll
    for (int c = 1; c < kPtFan; ++c) {  // independent loads; missing children repeat the first
        const int64_t cc = c0 + c < c1 ? c0 + c : c0;
        lo = fminf(lo, child[cc * 2 * d + k]);
        hi = fmaxf(hi, child[cc * 2 * d + d + k]);
    }
    b[k] = lo;
    b[d + k] = hi;
}

// Box levels 2.. in one launch (k_pt_gather writes level 1).  Workgroup g builds the subtree
// of points [g * 4096, + 4096): levels 2..4 above its 512 leaves (each level's children are its
// own writes), one thread per (box, dim); the last workgroup to finish (ticket) builds levels
// 5.. over everyone's level-4 boxes and resets the ticket for the next build.
constexpr int kPtChunkLeaves = 512;  // 8^3: levels 1..4 inside a workgroup
constexpr int kPtInBlockLevels = 4;

// levels 5.. of the tree over every group's level-4 boxes (one workgroup)
__device__ __forceinline__ void pt_top_boxes(const PointTreeDev &T, float *__restrict__ boxes) {
    const int64_t n = live_n(T);
    for (int l = kPtInBlockLevels + 1; l <= T.n_levels; ++l) {
        const int64_t nl = lvl_size(n, l);
        for (int64_t it = threadIdx.x; it < nl * T.d; it += blockDim.x)
            pt_up_box(T, n, l, boxes, it / T.d, (int)(it % T.d));
        __threadfence_block();
        __syncthreads();
    }
}

// ticket == nullptr: levels 5.. are left to a launch of their own (k_pt_top_jobs)
__device__ __forceinline__ void pt_boxes(const PointTreeDev &T, float *__restrict__ boxes,
                                         unsigned int *__restrict__ ticket, int64_t g, int64_t ngroups) {
    const int64_t n = live_n(T);
    const int top_in = T.n_levels < kPtInBlockLevels ? T.n_levels : kPtInBlockLevels;
    for (int l = 2; l <= top_in; ++l) {
        const int64_t per = (int64_t)kPtChunkLeaves >> (3 * (l - 1));
        const int64_t j0 = g * per, nl = lvl_size(n, l), j1 = j0 + per < nl ? j0 + per : nl;
        // one thread per (box, dim): short dependent chains at the small upper levels
        for (int64_t it = threadIdx.x; it < (j1 - j0) * T.d; it += blockDim.x) {
            const int64_t j = j0 + it / T.d;
            const int k = (int)(it % T.d);
            pt_up_box(T, n, l, boxes, j, k);
        }
        __threadfence_block();
        __syncthreads();
    }
    if (T.n_levels <= kPtInBlockLevels || !ticket) return;  // one workgroup: its level 4 is the root
    __shared__ bool last;
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) last = atomicAdd(ticket, 1u) == ngroups - 1;
    __syncthreads();
    if (!last) return;
    __threadfence();  // agent-scope acquire: this CU's L1 holds no stale copy of the others' boxes
    pt_top_boxes(T, boxes);
    if (threadIdx.x == 0) *ticket = 0u;
}

__global__ __launch_bounds__(256) void k_pt_boxes(PointTreeDev T, float *__restrict__ boxes,
                                                  unsigned int *__restrict__ ticket) {
    pt_boxes(T, boxes, ticket, blockIdx.x, gridDim.x);
}

// ---- incremental index (point_tree.h PtIncJob) ----

// the job table on the device (a joint build), or one job passed in the kernel arguments
struct IncJobs {
    const PtIncJob *table;
    PtIncJob one;
    __device__ __forceinline__ const PtIncJob &at(int k) const { return table ? table[k] : one; }
};

// the point's 64-bit code under the fixed plan (row loaded whole)
template <int D>
__device__ __forceinline__ uint64_t inc_code(const IncPlan *__restrict__ P, const double (&x)[D]) {
    uint32_t q[D];
#pragma unroll
    for (int j = 0; j < D; ++j) {
        const double u = (x[j] - P->lo[j]) * P->scale[j];
        const uint32_t m = P->qmax[j];
        q[j] = u <= 0.0 ? 0u : (u >= (double)m ? m : (uint32_t)u);
    }
    uint64_t c = 0;
    const int32_t nb = P->n;
    // unrolled to the code width (d <= 7), so the plan's table reads issue together instead of
    // one round trip per bit; the 15-dim select chain would not fit the registers unrolled
    if constexpr (D <= 7) {
#pragma unroll
        for (int k = 0; k < kPtIncBits; ++k) {
            if (k >= nb) break;
            const int32_t dk = P->dim[k];
            uint32_t v = q[0];
#pragma unroll
            for (int j = 1; j < D; ++j)
                if (j == dk) v = q[j];
            c = (c << 1) | (uint64_t)((v >> P->bit[k]) & 1u);
        }
    } else {
        for (int k = 0; k < nb; ++k) {
            const int32_t dk = P->dim[k];
            uint32_t v = q[0];
#pragma unroll
            for (int j = 1; j < D; ++j)
                if (j == dk) v = q[j];
            c = (c << 1) | (uint64_t)((v >> P->bit[k]) & 1u);
        }
    }
    return c;
}

// bitwise, not short-circuit: the && / || form compiled to divergent branches around every
// compare-exchange of the sorts
__device__ __forceinline__ bool inc_less(uint64_t ka, int32_t va, uint64_t kb, int32_t vb) {
    return (ka < kb) | ((ka == kb) & (va < vb));
}
// compare-exchange against a partner: keep the smaller pair (keep_min) or the larger, by
// selects.  Pairs are distinct but for padding, and swapping equal pairs changes nothing.
__device__ __forceinline__ void inc_cx(uint64_t &k, int32_t &v, uint64_t pk, int32_t pv, bool keep_min) {
    const bool sw = keep_min == inc_less(pk, pv, k, v);
    k = sw ? pk : k;
    v = sw ? pv : v;
}

// The new points' sort over many CUs: one workgroup per tree runs the 4096-element bitonic
// network on one CU (~78 stages), which leaves most of the chip idle when there are few trees.
// Instead: the codes one thread a point (k_pt_inc_ncodes); each wave sorts a chunk of 512 (8
// elements a lane: partners 8+ apart by lane shuffles, closer ones in registers; no LDS, no
// barriers); a third kernel places every element at its rank, its index in its own chunk plus,
// per other chunk, the count of smaller (code, row) pairs there (a fixed-step binary search,
// the chunks' searches interleaved).  (code, row) pairs are distinct, so the ranks are a
// permutation and the result is the one total order any sort gives.
constexpr int kIncChunk = 512;
constexpr int kIncChunks = kPtIncSeg / kIncChunk;
constexpr int kIncChunkWaves = 4;  // chunks a workgroup sorts
static_assert(kIncChunks % kIncChunkWaves == 0, "whole workgroups");

// Seed slots (point_tree.h kPtHull): lane h of a wave scores slot h over the wave's 64 points
// (staged in LDS: every lane reads the same point at once, a broadcast) and offers its best to
// the tree's slot with one 64-bit atomicMax of (score as an ordered float key << 32 | row).  Rows
// of a wave are consecutive (row0 + lane).  The float rounding of the score only decides which
// near-tie becomes the seed; any point is a valid seed.
constexpr int kHullWaves = 4;  // waves of the workgroups that score (256 threads)
template <int D>
__device__ __forceinline__ void hull_offer(const IncPlan &P, const double (&x)[D], bool live, int64_t row0,
                                           double (*s_rows)[D], unsigned long long *__restrict__ keys) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int j = 0; j < D; ++j) s_rows[lane][j] = live ? x[j] : 0.0;
    const uint64_t lm = __ballot(live);
    __builtin_amdgcn_wave_barrier();
    if (lane < P.n_hull) {
        const int kind = P.hkind[lane], dm = P.hdim[lane];
        const float u0 = P.hdir[lane][0], u1 = P.hdir[lane][1], u2 = P.hdir[lane][2];
        unsigned long long best = 0;
        for (uint64_t m = lm; m; m &= m - 1) {
            const int j = __ffsll((long long)m) - 1;
            double v;
            if (kind == 0) {
                v = (double)u0 * s_rows[j][0];
                if (D > 1) v += (double)u1 * s_rows[j][D > 1 ? 1 : 0];
                if (D > 2) v += (double)u2 * s_rows[j][D > 2 ? 2 : 0];
            } else {
                double xv = s_rows[j][0];
#pragma unroll
                for (int k = 1; k < D; ++k)
                    if (k == dm) xv = s_rows[j][k];
                v = kind == 1 ? -xv : xv;
            }
            const uint32_t b = __float_as_uint((float)v);
            const uint32_t key = (b & 0x80000000u) ? ~b : (b | 0x80000000u);
            const unsigned long long k64 = ((unsigned long long)key << 32) | (uint32_t)(row0 + j);
            best = k64 > best ? k64 : best;
        }
        if (best) atomicMax(keys + lane, best);
    }
    __builtin_amdgcn_wave_barrier();
}

// the new points' codes and rows (one thread a point) into nkeys / nvals, in row order, their
// box into ibox, and their offers to the seed slots
template <int D>
__device__ __forceinline__ void pt_inc_ncodes(const PtIncJob &J, const IncPlan &P, double (*s_rows)[D]) {
    if (J.full) return;
    const int64_t nd = *J.T.n_dev, n = nd < J.T.n_upper ? nd : J.T.n_upper;
    const int64_t base = *J.nidx;
    int64_t m = n - base;
    if (m > kPtIncSeg && blockIdx.x == 0 && threadIdx.x == 0 && J.err) atomicAdd(J.err, 1ull);  // the host's bound broke
    m = m < 0 ? 0 : (m > kPtIncSeg ? kPtIncSeg : m);
    const int i = (int)blockIdx.x * (int)blockDim.x + (int)threadIdx.x;
    if ((int64_t)blockIdx.x * blockDim.x >= m) return;  // block-uniform
    const bool live = i < m;
    unsigned long long mn[D], mx[D];
    double x[D];
    if (live) {
        const int64_t row = base + i;
        load_global<D>(J.pts + row * D, x);
        ((MPT_GLOBAL uint64_t *)J.nkeys)[i] = inc_code<D>(&P, x);
        ((MPT_GLOBAL int32_t *)J.nvals)[i] = (int32_t)row;
#pragma unroll
        for (int j = 0; j < D; ++j) mn[j] = mx[j] = order_key_pt(x[j]);
    } else {
#pragma unroll
        for (int j = 0; j < D; ++j) {
            mn[j] = ~0ull;
            mx[j] = 0ull;
        }
    }
    // the persistent box of the indexed points (MPT_NN_AUTO's spread)
#pragma unroll
    for (int j = 0; j < D; ++j) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const unsigned long long omn = __shfl_xor(mn[j], off), omx = __shfl_xor(mx[j], off);
            mn[j] = omn < mn[j] ? omn : mn[j];
            mx[j] = omx > mx[j] ? omx : mx[j];
        }
    }
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
        for (int j = 0; j < D; ++j) {
            atomicMin(J.ibox + j, mn[j]);
            atomicMax(J.ibox + kPtMaxDim + j, mx[j]);
        }
    }
    const int64_t row0 = base + (i & ~63);
    hull_offer<D>(P, x, live, row0, s_rows, J.hull_keys);
}

template <int D>
__global__ __launch_bounds__(64 * kHullWaves) void k_pt_inc_ncodes(IncJobs jobs) {
    __shared__ IncPlan s_plan;
    __shared__ double s_rows[kHullWaves][64][D];
    const PtIncJob &J = jobs.table ? jobs.table[blockIdx.y] : jobs.one;
    for (int w = threadIdx.x; w < (int)(sizeof(IncPlan) / 4); w += blockDim.x)
        reinterpret_cast<uint32_t *>(&s_plan)[w] = reinterpret_cast<const uint32_t *>(J.plan)[w];
    __syncthreads();
    if (jobs.table) pt_inc_ncodes<D>(jobs.table[blockIdx.y], s_plan, s_rows[threadIdx.x >> 6]);
    else pt_inc_ncodes<D>(jobs.one, s_plan, s_rows[threadIdx.x >> 6]);
}

// one chunk of 512 (code, row) pairs a wave: nkeys / nvals -> ckeys / cvals
__device__ __forceinline__ void pt_inc_csort(const PtIncJob &J) {
    if (J.full) return;
    const int64_t nd = *J.T.n_dev, n = nd < J.T.n_upper ? nd : J.T.n_upper;
    int64_t m = n - *J.nidx;
    m = m < 0 ? 0 : (m > kPtIncSeg ? kPtIncSeg : m);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int c0 = ((int)blockIdx.x * kIncChunkWaves + wave) * kIncChunk;
    if (c0 >= m) return;
    constexpr int E = kIncChunk / 64;
    uint64_t key[E];
    int32_t val[E];
#pragma unroll
    for (int a = 0; a < E; ++a) {
        const int i = c0 + lane * E + a;
        const bool live = i < m;
        // real codes use 63 bits: padding sorts last
        key[a] = live ? ((const MPT_GLOBAL uint64_t *)J.nkeys)[i] : ~0ull;
        val[a] = live ? ((const MPT_GLOBAL int32_t *)J.nvals)[i] : 0x7fffffff;
    }
#pragma unroll 1
    for (int k = 2; k <= kIncChunk; k <<= 1) {
#pragma unroll 1
        for (int j = k >> 1; j > 0; j >>= 1) {
            if (j >= E) {
                const int lm = j / E;
                const bool lower = (lane & lm) == 0;
#pragma unroll
                for (int a = 0; a < E; ++a) {
                    const uint64_t pk = __shfl_xor(key[a], lm);
                    const int32_t pv = __shfl_xor(val[a], lm);
                    inc_cx(key[a], val[a], pk, pv, lower == (((lane * E + a) & k) == 0));
                }
            } else {
#pragma unroll
                for (int jj = E / 2; jj > 0; jj >>= 1) {
                    if (jj != j) continue;
#pragma unroll
                    for (int a = 0; a < E; ++a) {
                        const int b = a ^ jj;
                        if (b < a) continue;
                        const bool up = ((lane * E + a) & k) == 0;
                        const bool sw = up == inc_less(key[b], val[b], key[a], val[a]);
                        const uint64_t ka = key[a], kb = key[b];
                        const int32_t va = val[a], vb = val[b];
                        key[a] = sw ? kb : ka;
                        val[a] = sw ? vb : va;
                        key[b] = sw ? ka : kb;
                        val[b] = sw ? va : vb;
                    }
                }
            }
        }
    }
    // the whole chunk, padding included (the rank search reads 512 per chunk)
#pragma unroll
    for (int a = 0; a < E; ++a) {
        ((MPT_GLOBAL uint64_t *)J.ckeys)[c0 + lane * E + a] = key[a];
        ((MPT_GLOBAL int32_t *)J.cvals)[c0 + lane * E + a] = val[a];
    }
}

__global__ __launch_bounds__(64 * kIncChunkWaves) void k_pt_inc_csort(IncJobs jobs) {
    if (jobs.table) pt_inc_csort(jobs.table[blockIdx.y]);
    else pt_inc_csort(jobs.one);
}

// NC: the chunks searched (the whole set: 16 only when more than 8 are live)
template <int NC>
__device__ __forceinline__ void pt_inc_crank_n(const PtIncJob &J, int64_t m, int e) {
    const int nch = (int)((m + kIncChunk - 1) / kIncChunk);
    const uint64_t key = J.ckeys[e];
    const int32_t val = J.cvals[e];
    // per chunk: the count of its pairs below (key, val); for the element's own chunk that is
    // its index there.  Fixed steps, the chunks' loads issued together.
    int pos[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) pos[c] = 0;
    // (every chunk's loads unconditional -- a branch per chunk made each load wait alone;
    // chunks past nch read scratch and are masked out of the sum)
    const MPT_GLOBAL uint64_t *ck = (const MPT_GLOBAL uint64_t *)J.ckeys;
    const MPT_GLOBAL int32_t *cv = (const MPT_GLOBAL int32_t *)J.cvals;
#pragma unroll
    for (int st = kIncChunk / 2; st > 0; st >>= 1) {
        uint64_t pk[NC];
        int32_t pv[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const int q = c * kIncChunk + pos[c] + st - 1;
            pk[c] = ck[q];
            pv[c] = cv[q];
        }
#pragma unroll
        for (int c = 0; c < NC; ++c) pos[c] += inc_less(pk[c], pv[c], key, val) ? st : 0;
    }
    int rank = 0;
    {
        uint64_t pk[NC];
        int32_t pv[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const int q = c * kIncChunk + pos[c];
            pk[c] = ck[q];
            pv[c] = cv[q];
        }
#pragma unroll
        for (int c = 0; c < NC; ++c)
            rank += c < nch ? pos[c] + (inc_less(pk[c], pv[c], key, val) ? 1 : 0) : 0;
    }
    J.nkeys[rank] = key;
    J.nvals[rank] = val;
}

__device__ __forceinline__ void pt_inc_crank(const PtIncJob &J) {
    if (J.full) return;
    const int64_t nd = *J.T.n_dev, n = nd < J.T.n_upper ? nd : J.T.n_upper;
    int64_t m = n - *J.nidx;
    m = m < 0 ? 0 : (m > kPtIncSeg ? kPtIncSeg : m);
    const int e = (int)blockIdx.x * (int)blockDim.x + (int)threadIdx.x;
    if (e >= m) return;
    if (m <= (int64_t)kIncChunk * (kIncChunks / 2)) pt_inc_crank_n<kIncChunks / 2>(J, m, e);
    else pt_inc_crank_n<kIncChunks>(J, m, e);
}

__global__ __launch_bounds__(256) void k_pt_inc_crank(IncJobs jobs) {
    if (jobs.table) pt_inc_crank(jobs.table[blockIdx.y]);
    else pt_inc_crank(jobs.one);
}

// number of a's among the first p elements of merge(a, b), an a before a b of the same key
template <class K>
__device__ __forceinline__ int64_t merge_split(const K *a, int64_t na, const K *b, int64_t nb, int64_t p) {
    int64_t lo = p > nb ? p - nb : 0, hi = p < na ? p : na;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (a[mid] <= b[p - 1 - mid]) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

constexpr int kIncTile = 256;  // merged outputs per workgroup (one per thread)

// Merge path: workgroup g writes outputs [g * 256, + 256) of merge(old, new): its split of
// the old / new arrays by two binary searches, the tile's keys staged in LDS, each thread's
// source by a search of its diagonal there; the row and id copied from the old sorted arrays
// or the node rows; the leaf boxes (8 consecutive outputs) by an 8-lane reduction.
template <int D>
__device__ __forceinline__ void pt_inc_merge(const PtIncJob &J) {
    __shared__ uint64_t sa[kIncTile], sb[kIncTile];
    __shared__ int64_t s_split[2];
    const int64_t nd = *J.T.n_dev, n = nd < J.T.n_upper ? nd : J.T.n_upper;
    const int64_t p0 = (int64_t)blockIdx.x * kIncTile;
    if (p0 >= n) return;
    const int64_t n_old = J.full ? 0 : *J.nidx;
    int64_t m = n - n_old;
    if (!J.full) m = m < 0 ? 0 : (m > kPtIncSeg ? kPtIncSeg : m);
    const int64_t p1 = p0 + kIncTile < n ? p0 + kIncTile : n;
    const int t = threadIdx.x;
    if (t < 2) s_split[t] = merge_split(J.okeys, n_old, J.nkeys, m, t == 0 ? p0 : p1);
    __syncthreads();
    const int64_t i0 = s_split[0], i1 = s_split[1];
    const int na = (int)(i1 - i0), nb = (int)((p1 - p0) - na);
    const int64_t j0 = p0 - i0;
    if (t < na) sa[t] = J.okeys[i0 + t];
    if (t < nb) sb[t] = J.nkeys[j0 + t];
    __syncthreads();
    const int64_t p = p0 + t;
    const bool live = p < p1;
    double row[D];
    int32_t id = 0;
    uint64_t key = 0;
    if (live) {
        const int a = (int)merge_split(sa, na, sb, nb, t), b = t - a;
        if (a < na && (b >= nb || sa[a] <= sb[b])) {
            const int64_t s = i0 + a;
            key = sa[a];
            id = J.oids[s];
#pragma unroll
            for (int j = 0; j < D; ++j) row[j] = J.opts[s * D + j];
        } else {
            const int64_t r = J.nvals[j0 + b];
            key = sb[b];
            id = (int32_t)r + 1;
#pragma unroll
            for (int j = 0; j < D; ++j) row[j] = J.pts[r * D + j];
        }
        J.keys[p] = key;
        J.ids[p] = id;
#pragma unroll
        for (int j = 0; j < D; ++j) J.spts[p * D + j] = row[j];
    }
#pragma unroll
    for (int j = 0; j < D; ++j) {
        double lo = live ? row[j] : __builtin_huge_val(), hi = live ? row[j] : -__builtin_huge_val();
#pragma unroll
        for (int off = kPtFan / 2; off > 0; off >>= 1) {
            const double olo = __shfl_xor(lo, off, kPtFan), ohi = __shfl_xor(hi, off, kPtFan);
            lo = olo < lo ? olo : lo;
            hi = ohi > hi ? ohi : hi;
        }
        if (live && (p & (kPtFan - 1)) == 0) {
            float *bx = J.boxes + (p / kPtFan) * 2 * D;
            bx[j] = widen_lo(lo);
            bx[D + j] = widen_hi(hi);
        }
    }
}

// An incremental merge with its split points precomputed: the output place of every new point
// (k_pt_inc_npos: its index among the new plus the count of old codes <= its code, old first
// on a tie as in merge_split) makes a tile's split a search of that short, cache-resident
// array, and an output's source the count of the tile's new places below it.  The merge-path
// form searched the whole old code array (17 dependent loads a workgroup, cold) and the
// tile's keys in LDS per output.  A tile is kIncPer outputs a thread.
constexpr int kIncPer = 4;
constexpr int kIncTile2 = kIncTile * kIncPer;

__device__ __forceinline__ void pt_inc_npos(const PtIncJob &J) {
    if (J.full) return;
    const int64_t nd = *J.T.n_dev, n = nd < J.T.n_upper ? nd : J.T.n_upper;
    const int64_t n_old = *J.nidx;
    int64_t m = n - n_old;
    m = m < 0 ? 0 : (m > kPtIncSeg ? kPtIncSeg : m);
    const int j = (int)blockIdx.x * (int)blockDim.x + (int)threadIdx.x;
    if (j >= m) return;
    const uint64_t key = J.nkeys[j];
    int64_t lo = 0, hi = n_old;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (J.okeys[mid] <= key) lo = mid + 1;
        else hi = mid;
    }
    J.npos[j] = (int32_t)(lo + j);
}

__global__ __launch_bounds__(256) void k_pt_inc_npos(IncJobs jobs) {
    if (jobs.table) pt_inc_npos(jobs.table[blockIdx.y]);
    else pt_inc_npos(jobs.one);
}

template <int D>
__device__ __forceinline__ void pt_inc_merge2(const PtIncJob &J) {
    __shared__ int32_t s_np[kIncTile2];
    __shared__ int32_t s_nb[2];
    const int64_t nd = *J.T.n_dev, n = nd < J.T.n_upper ? nd : J.T.n_upper;
    const int64_t p0 = (int64_t)blockIdx.x * kIncTile2;
    if (p0 >= n) return;
    const int64_t n_old = *J.nidx;
    int64_t m = n - n_old;
    m = m < 0 ? 0 : (m > kPtIncSeg ? kPtIncSeg : m);
    const int64_t p1 = p0 + kIncTile2 < n ? p0 + kIncTile2 : n;
    const int t = threadIdx.x;
    // the job's arrays through global pointers (read from the job table they are flat, and a
    // flat access counts against the LDS counter: each LDS search would wait for the loads)
    const MPT_GLOBAL int32_t *npos = (const MPT_GLOBAL int32_t *)J.npos;
    const MPT_GLOBAL uint64_t *nkeys = (const MPT_GLOBAL uint64_t *)J.nkeys, *okeys = (const MPT_GLOBAL uint64_t *)J.okeys;
    const MPT_GLOBAL int32_t *nvals = (const MPT_GLOBAL int32_t *)J.nvals, *oids = (const MPT_GLOBAL int32_t *)J.oids;
    const MPT_GLOBAL double *pts = (const MPT_GLOBAL double *)J.pts, *opts = (const MPT_GLOBAL double *)J.opts;
    MPT_GLOBAL uint64_t *keys = (MPT_GLOBAL uint64_t *)J.keys;
    MPT_GLOBAL int32_t *ids = (MPT_GLOBAL int32_t *)J.ids;
    MPT_GLOBAL double *spts = (MPT_GLOBAL double *)J.spts;
    MPT_GLOBAL float *boxes = (MPT_GLOBAL float *)J.boxes;
    if (t < 2) {  // new points placed before p0 / p1
        const int64_t target = t == 0 ? p0 : p1;
        int lo = 0, hi = (int)m;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (npos[mid] < target) lo = mid + 1;
            else hi = mid;
        }
        s_nb[t] = lo;
    }
    __syncthreads();
    const int nb0 = s_nb[0], cnt = s_nb[1] - nb0;
    for (int k = t; k < cnt; k += kIncTile) s_np[k] = npos[nb0 + k];
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kIncPer; ++u) {
        const int64_t p = p0 + u * kIncTile + t;
        const bool live = p < p1;
        double row[D];
        if (live) {
            int lo = 0, hi = cnt;  // the tile's new places below p
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (s_np[mid] < p) lo = mid + 1;
                else hi = mid;
            }
            uint64_t key;
            int32_t id;
            if (lo < cnt && s_np[lo] == p) {
                const int j = nb0 + lo;
                const int64_t r = nvals[j];
                key = nkeys[j];
                id = (int32_t)r + 1;
#pragma unroll
                for (int k = 0; k < D; ++k) row[k] = pts[r * D + k];
            } else {
                const int64_t o = p - nb0 - lo;
                key = okeys[o];
                id = oids[o];
#pragma unroll
                for (int k = 0; k < D; ++k) row[k] = opts[o * D + k];
            }
            keys[p] = key;
            ids[p] = id;
#pragma unroll
            for (int k = 0; k < D; ++k) spts[p * D + k] = row[k];
        }
#pragma unroll
        for (int k = 0; k < D; ++k) {
            double lo = live ? row[k] : __builtin_huge_val(), hi = live ? row[k] : -__builtin_huge_val();
#pragma unroll
            for (int off = kPtFan / 2; off > 0; off >>= 1) {
                const double olo = __shfl_xor(lo, off, kPtFan), ohi = __shfl_xor(hi, off, kPtFan);
                lo = olo < lo ? olo : lo;
                hi = ohi > hi ? ohi : hi;
            }
            if (live && (p & (kPtFan - 1)) == 0) {
                MPT_GLOBAL float *bx = boxes + (p / kPtFan) * 2 * D;
                bx[k] = widen_lo(lo);
                bx[D + k] = widen_hi(hi);
            }
        }
    }
}

// the placed merge for incremental jobs (a full rebuild keeps the merge-path form; its tiles
// are kIncTile outputs, so the grid is sized for those)
template <int D>
__global__ __launch_bounds__(kIncTile) void k_pt_inc_merge(IncJobs jobs) {
    const PtIncJob &J = jobs.table ? jobs.table[blockIdx.y] : jobs.one;
    if (!J.full) {
        if (jobs.table) pt_inc_merge2<D>(jobs.table[blockIdx.y]);
        else pt_inc_merge2<D>(jobs.one);
    } else {
        if (jobs.table) pt_inc_merge<D>(jobs.table[blockIdx.y]);
        else pt_inc_merge<D>(jobs.one);
    }
}

__device__ __forceinline__ void pt_inc_boxes(const PtIncJob &J) {
    if (J.T.n_levels < 2) return;
    const int64_t groups = (J.T.n_upper + kPtChunkLeaves * kPtFan - 1) / (kPtChunkLeaves * kPtFan);
    if (blockIdx.x >= groups) return;
    pt_boxes(J.T, J.boxes, nullptr, blockIdx.x, groups);
}

__global__ __launch_bounds__(256) void k_pt_inc_boxes(IncJobs jobs) {
    if (jobs.table) pt_inc_boxes(jobs.table[blockIdx.y]);
    else pt_inc_boxes(jobs.one);
}

// levels 5.. (one workgroup per tree), the seed rows of the slots' best points, then the
// indexed count and the spread feedback
__device__ __forceinline__ void pt_inc_top(const PtIncJob &J) {
    if (J.T.n_levels > kPtInBlockLevels) pt_top_boxes(J.T, J.boxes);
    const int d = J.T.d;
    for (int it = threadIdx.x; it < kPtHull * d; it += blockDim.x) {
        const int h = it / d, k = it - h * d;
        const unsigned long long key = J.hull_keys[h];
        const int64_t row = (int64_t)(uint32_t)key;
        J.hull_pts[it] = key ? J.pts[row * d + k] : 0.0;
        if (k == 0) J.hull_ids[h] = key ? (int32_t)row + 1 : 0;
    }
    if (threadIdx.x != 0) return;
    *J.nidx = live_n(J.T);
    const SpreadOut &sp = J.sp;
    if (sp.host_out) {
        for (int j = 0; j < 3; ++j) {
            sp.host_out[j] = j < sp.gd ? J.ibox[sp.dims[j]] : ~0ull;
            sp.host_out[3 + j] = j < sp.gd ? J.ibox[kPtMaxDim + sp.dims[j]] : 0ull;
        }
        __threadfence_system();
    }
}

__global__ __launch_bounds__(256) void k_pt_inc_top(IncJobs jobs) {
    if (jobs.table) pt_inc_top(jobs.table[blockIdx.x]);
    else pt_inc_top(jobs.one);
}

// full rebuild: the box of every live point (from empty)
__global__ __launch_bounds__(64) void k_pt_inc_box_reset(unsigned long long *__restrict__ box) {
    if (threadIdx.x < 2 * kPtMaxDim) box[threadIdx.x] = threadIdx.x < kPtMaxDim ? ~0ull : 0ull;
}
template <int D>
__global__ __launch_bounds__(256) void k_pt_inc_bbox(const double *__restrict__ pts, int32_t d, int64_t n_upper,
                                                     const int64_t *__restrict__ n_dev,
                                                     unsigned long long *__restrict__ box) {
    pt_bbox<D>(pts, d, n_upper, n_dev, box, nullptr, nullptr, SpreadOut{}, blockIdx.x, gridDim.x);
}

// full rebuild: every point's code (rows past the live count sort to the end) and its offers to
// the seed slots (reset before this launch)
template <int D>
__global__ __launch_bounds__(64 * kHullWaves) void k_pt_inc_codes(const double *__restrict__ pts, int64_t n_upper,
                                                                  const int64_t *__restrict__ n_dev,
                                                                  const IncPlan *__restrict__ plan,
                                                                  uint64_t *__restrict__ keys,
                                                                  int32_t *__restrict__ vals,
                                                                  unsigned long long *__restrict__ hull_keys) {
    __shared__ IncPlan s_plan;
    __shared__ double s_rows[kHullWaves][64][D];
    for (int w = threadIdx.x; w < (int)(sizeof(IncPlan) / 4); w += blockDim.x)
        reinterpret_cast<uint32_t *>(&s_plan)[w] = reinterpret_cast<const uint32_t *>(plan)[w];
    __syncthreads();
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if ((int64_t)blockIdx.x * blockDim.x >= n_upper) return;  // block-uniform
    const int64_t n = *n_dev < n_upper ? *n_dev : n_upper;
    const bool live = i < n;
    double x[D];
#pragma unroll
    for (int j = 0; j < D; ++j) x[j] = live ? pts[i * D + j] : 0.0;
    if (i < n_upper) {
        vals[i] = (int32_t)i;
        keys[i] = live ? inc_code<D>(&s_plan, x) : ~0ull;
    }
    hull_offer<D>(s_plan, x, live, i & ~(int64_t)63, s_rows[threadIdx.x >> 6], hull_keys);
}

constexpr int kPtGroupsPerBlock = 256 / kPtFan;
constexpr int kPtStack = kPtFan * kPtMaxLevels;

// A box's lower bound on FLANN's squared L2 from the query, as a float rounded down.  d <= 7:
// computed in float (a quarter of the double box test's VALU work) from the query rounded
// outward -- each gap at most (1 + u) over the exact one (u = 2^-24), its square and each
// partial sum another (1 + u), so the float sum is at most (1 + u)^(D + 3) over the exact
// bound, and the final scale by 1 - 2^-19 (itself rounded) brings it below it; d = 15: in
// double (register budget) and rounded down.  Pruning on it keeps every box the exact bound
// keeps.
constexpr float kLbF32Shrink = 1.0f - 0x1p-19f;

// The walks' point rows, ids and boxes through address-space-1 pointers: the tree comes from a
// job table, so the compiler cannot tell its pointers are global and emits flat loads, which
// also count against the LDS counter (every lane-shuffle / stack wait then waits for them).
using gdbl = const __attribute__((address_space(1))) double *;
using gflt = const __attribute__((address_space(1))) float *;
using gi32 = const __attribute__((address_space(1))) int32_t *;
template <int D>
__device__ __forceinline__ double leaf_l2(const double (&qq)[D], const PointTreeDev &T, int64_t p) {
    double row[D];
#pragma unroll
    for (int k = 0; k < D; ++k) row[k] = ((gdbl)T.pts)[p * D + k];
    return flann_l2<D>(qq, row);
}
__device__ __forceinline__ int32_t leaf_id(const PointTreeDev &T, int64_t p) { return ((gi32)T.ids)[p]; }
template <int D>
__device__ __forceinline__ void load_box(const PointTreeDev &T, int64_t box, float (&b)[2 * D]) {
#pragma unroll
    for (int k = 0; k < 2 * D; ++k) b[k] = ((gflt)T.boxes)[box * 2 * D + k];
}
template <int D>
__device__ __forceinline__ float box_lb(const float *__restrict__ b, const double (&qq)[D], const float (&qlo)[D],
                                        const float (&qhi)[D]) {
    if constexpr (D <= 7) {
        float s = 0.0f;
#pragma unroll
        for (int k = 0; k < D; ++k) {
            const float g = fmaxf(fmaxf(b[k] - qhi[k], qlo[k] - b[D + k]), 0.0f);
            s = s + g * g;
        }
        return s * kLbF32Shrink;
    } else {
        double lb2 = 0.0;
#pragma unroll
        for (int k = 0; k < D; ++k) {
            const double g = fmax(fmax((double)b[k] - qq[k], qq[k] - (double)b[D + k]), 0.0);
            lb2 += g * g;
        }
        return __double2float_rd(lb2);
    }
}

// the seeds' best (d2, id) for the query, over a group of G lanes (point_tree.h kPtHull): lane
// `sub` takes seeds sub, sub + G, ...; the group's best by xor-shuffles.  Leaves (bd, bi) at
// +inf / -1 when the tree carries no seeds.
template <int D, int G>
__device__ __forceinline__ void hull_seed(const PointTreeDev &T, const double (&qq)[D], int sub, double &bd,
                                          int32_t &bi, uint32_t &n_pts) {
    if (!T.hull_ids) return;
    for (int h = sub; h < kPtHull; h += G) {
        const int32_t id = ((gi32)T.hull_ids)[h];
        if (id <= 0) continue;
        double row[D];
#pragma unroll
        for (int k = 0; k < D; ++k) row[k] = ((gdbl)T.hull_pts)[h * D + k];
        const double dd = flann_l2<D>(qq, row);
        ++n_pts;
        if (nn_better(dd, id, bd, bi)) {
            bd = dd;
            bi = id;
        }
    }
#pragma unroll
    for (int off = G / 2; off > 0; off >>= 1) {
        const double od = __shfl_xor(bd, off, G);
        const int32_t oi = __shfl_xor(bi, off, G);
        if (nn_better(od, oi, bd, bi)) {
            bd = od;
            bi = oi;
        }
    }
}

// queries [blk * BS / 8, + BS / 8) of one tree (a workgroup's share of k_tree_nn1 / _jobs)
template <int D, int BS>
__device__ __forceinline__ void tree_nn1_block(const PointTreeDev &T, const double *__restrict__ q, int64_t nq,
                                               int32_t *__restrict__ out_ids, double *__restrict__ out_d2,
                                               int64_t blk) {
    __shared__ int32_t s_node[BS / kPtFan][kPtStack];
    // stacked lower bounds as floats rounded down (still lower bounds: pruning stays exact),
    // half the LDS of doubles, so more one-wave workgroups fit a CU
    __shared__ float s_lb[BS / kPtFan][kPtStack];
    const int64_t t = blk * BS + threadIdx.x;
    const int64_t slot = t / kPtFan;
    const int sub = (int)(t % kPtFan);
    const int grp = threadIdx.x / kPtFan;
    if (slot >= nq) return;  // whole groups leave together
    const int64_t qi = slot;
    double qq[D];
#pragma unroll
    for (int i = 0; i < D; ++i) qq[i] = q[qi * D + i];
    float qlo[D], qhi[D];  // the query rounded outward (box_lb, d <= 7)
#pragma unroll
    for (int i = 0; i < D; ++i) {
        qlo[i] = __double2float_rd(qq[i]);
        qhi[i] = __double2float_ru(qq[i]);
    }
    const int64_t n = live_n(T);
    double bd = __builtin_huge_val();
    int32_t bi = -1;
    uint32_t n_pts = 0, n_box = 0;
    if (n > 0) {
        hull_seed<D, kPtFan>(T, qq, sub, bd, bi, n_pts);
        int sp = 1;
        if (sub == 0) {
            s_node[grp][0] = T.n_levels << 27;  // the root: level n_levels, index 0
            s_lb[grp][0] = 0.0f;
        }
        __builtin_amdgcn_wave_barrier();
        while (sp > 0) {
            --sp;
            const int32_t code = s_node[grp][sp];
            const double lbs = (double)s_lb[grp][sp];
            __builtin_amdgcn_wave_barrier();
            // the 1e-12 shrink covers FLANN's summation order (as the grid kernel)
            if (lbs * (1.0 - 1e-12) > bd) continue;
            const int lev = code >> 27;
            const int64_t idx = code & ((1 << 27) - 1);
            if (lev == 1) {
                const int64_t p = idx * kPtFan + sub;
                if (p < n) {
                    const double dd = leaf_l2<D>(qq, T, p);
                    const int32_t id = leaf_id(T, p);
                    ++n_pts;
                    if (nn_better(dd, id, bd, bi)) {
                        bd = dd;
                        bi = id;
                    }
                }
#pragma unroll
                for (int off = kPtFan / 2; off > 0; off >>= 1) {
                    const double od = __shfl_xor(bd, off, kPtFan);
                    const int32_t oi = __shfl_xor(bi, off, kPtFan);
                    if (nn_better(od, oi, bd, bi)) {
                        bd = od;
                        bi = oi;
                    }
                }
            } else {
                const int64_t c = idx * kPtFan + sub;
                bool keep = false;
                float lbf = 0.0f;
                if (c < lvl_size(n, lev - 1)) {
                    float bx[2 * D];
                    load_box<D>(T, lvl_off(T.n_upper, lev - 1) + c, bx);
                    lbf = box_lb<D>(bx, qq, qlo, qhi);
                    keep = (double)lbf * (1.0 - 1e-12) <= bd;
                    ++n_box;
                }
                const int base = (threadIdx.x & 63) & ~(kPtFan - 1);
                const uint32_t gm = (uint32_t)(__ballot(keep) >> base) & 0xffu;
                int rank = 0;
#pragma unroll
                for (int j = 0; j < kPtFan; ++j) {
                    const float o = __shfl(lbf, j, kPtFan);
                    if (((gm >> j) & 1u) && (o > lbf || (o == lbf && j > sub))) ++rank;
                }
                if (keep) {
                    s_node[grp][sp + rank] = ((lev - 1) << 27) | (int32_t)c;
                    s_lb[grp][sp + rank] = lbf;
                }
                sp += __popc(gm);
                __builtin_amdgcn_wave_barrier();
            }
        }
    }
    if (T.stats) {
#pragma unroll
        for (int off = kPtFan / 2; off > 0; off >>= 1) {
            n_pts += __shfl_xor(n_pts, off, kPtFan);
            n_box += __shfl_xor(n_box, off, kPtFan);
        }
        if (sub == 0) {
            atomicAdd(T.stats + 0, (unsigned long long)n_pts);
            atomicAdd(T.stats + 1, (unsigned long long)n_box);
        }
    }
    if (sub == 0) {
        out_ids[qi] = bi;
        out_d2[qi] = bd;
    }
}

// The same exact search with two nodes expanded per step: 16 lanes per query, the stack's top
// two entries popped together, each taken by one half of the group (a leaf's 8 points or an
// inner node's 8 children); the halves' best (d2, id) merged over the 16 lanes, the children
// re-tested against the merged bound, and the second entry's survivors pushed below the top
// entry's (each half nearest-last), so the walk stays nearest-first.  Half the dependent
// steps of the one-node walk for a few more nodes visited; the result is the same exact 1-NN
// (any visiting order is: only boxes whose lower bound exceeds the best are skipped).  The
// stack holds at most ~14 entries a level (two sibling blocks of 7) + 2: 2 * 8 * 10 entries.
constexpr int64_t kPtNnWideMaxQueries = 262144;  // d = 15: the four-node walk up to this many queries a launch

// nodes a walk step by default: d = 7 (config 5, where it was measured) eight (one query a
// wave) at every launch size; d = 3 and d = 15 (its registers) four up to kPtNnWideMaxQueries
// queries, else one (the round-3 rule the eight-node walk replaced for d = 7 only)
inline int pt_nn_width(int32_t d, int64_t queries) {
    if (d == 7) return 8;
    return queries <= kPtNnWideMaxQueries ? 4 : 1;
}

// NW nodes a step (2 or 4): 8 * NW lanes per query, the stack's top NW entries popped together
template <int D, int BS, int NW>
__device__ __forceinline__ void tree_nn1_blockn(const PointTreeDev &T, const double *__restrict__ q, int64_t nq,
                                                int32_t *__restrict__ out_ids, double *__restrict__ out_d2,
                                                int64_t blk) {
    constexpr int kPtG2 = NW * kPtFan;                     // lanes per query
    constexpr int kPtStack2 = NW * kPtFan * kPtMaxLevels;  // ~NW blocks of 7 a level
    static_assert(kPtG2 <= 64, "ballot bits per group");
    __shared__ int32_t s_node[BS / kPtG2][kPtStack2];
    __shared__ float s_lb[BS / kPtG2][kPtStack2];
    const int64_t t = blk * BS + threadIdx.x;
    const int64_t slot = t / kPtG2;
    const int sub = (int)(t % kPtG2);
    const int half = sub / kPtFan;  // which popped entry: 0 the top, 1 the one below it, ...
    const int ls = sub % kPtFan;    // the child / point this lane takes
    const int grp = threadIdx.x / kPtG2;
    if (slot >= nq) return;  // whole groups leave together
    const int64_t qi = slot;
    double qq[D];
#pragma unroll
    for (int i = 0; i < D; ++i) qq[i] = q[qi * D + i];
    float qlo[D], qhi[D];  // the query rounded outward (box_lb, d <= 7)
#pragma unroll
    for (int i = 0; i < D; ++i) {
        qlo[i] = __double2float_rd(qq[i]);
        qhi[i] = __double2float_ru(qq[i]);
    }
    const int64_t n = live_n(T);
    double bd = __builtin_huge_val();
    int32_t bi = -1;
    uint32_t n_pts = 0, n_box = 0;
    if (n > 0) {
        hull_seed<D, kPtG2>(T, qq, sub, bd, bi, n_pts);
        int sp = 1;
        if (sub == 0) {
            s_node[grp][0] = T.n_levels << 27;
            s_lb[grp][0] = 0.0f;
        }
        __builtin_amdgcn_wave_barrier();
        const int base = (threadIdx.x & 63) & ~(kPtG2 - 1);
        while (sp > 0) {
            const int np = sp >= NW ? NW : sp;
            const bool have = half < np;
            int32_t code = 0;
            double lbs = 0.0;
            if (have) {
                code = s_node[grp][sp - 1 - half];
                lbs = (double)s_lb[grp][sp - 1 - half];
            }
            sp -= np;
            __builtin_amdgcn_wave_barrier();
            const bool act = have && !(lbs * (1.0 - 1e-12) > bd);
            const int lev = act ? code >> 27 : 0;
            const int64_t idx = code & ((1 << 27) - 1);
            bool keep = false, leaf = false;
            float lbf = 0.0f;
            int64_t c = 0;
            if (lev == 1) {
                const int64_t p = idx * kPtFan + ls;
                if (p < n) {
                    const double dd = leaf_l2<D>(qq, T, p);
                    const int32_t id = leaf_id(T, p);
                    ++n_pts;
                    leaf = true;
                    if (nn_better(dd, id, bd, bi)) {
                        bd = dd;
                        bi = id;
                    }
                }
            } else if (lev > 1) {
                c = idx * kPtFan + ls;
                if (c < lvl_size(n, lev - 1)) {
                    float bx[2 * D];
                    load_box<D>(T, lvl_off(T.n_upper, lev - 1) + c, bx);
                    lbf = box_lb<D>(bx, qq, qlo, qhi);
                    keep = true;
                    ++n_box;
                }
            }
            // the parts' best, then the survivors against it.  Wave-uniform skips: a group's
            // lanes already share one best unless a lane examined a point this step, and with no
            // survivor in the wave there is nothing to rank
            if (__ballot(leaf)) {
#pragma unroll
                for (int off = kPtG2 / 2; off > 0; off >>= 1) {
                    const double od = __shfl_xor(bd, off, kPtG2);
                    const int32_t oi = __shfl_xor(bi, off, kPtG2);
                    if (nn_better(od, oi, bd, bi)) {
                        bd = od;
                        bi = oi;
                    }
                }
            }
            keep = keep && (double)lbf * (1.0 - 1e-12) <= bd;
            const uint64_t wm = __ballot(keep);
            const uint64_t gm = (wm >> base) & (kPtG2 == 64 ? ~0ull : ((1ull << kPtG2) - 1));
            const uint32_t mine = (uint32_t)(gm >> (half * kPtFan)) & 0xffu;
            // deeper entries' survivors go below: positions after every later half's
            const int below = __popcll(half + 1 < NW ? gm >> ((half + 1) * kPtFan) : 0ull);
            int rank = 0;
            if (wm) {
#pragma unroll
                for (int j = 0; j < kPtFan; ++j) {
                    const float o = __shfl(lbf, half * kPtFan + j, kPtG2);
                    if (((mine >> j) & 1u) && (o > lbf || (o == lbf && j > ls))) ++rank;
                }
            }
            if (keep) {
                const int pos = sp + below + rank;
                s_node[grp][pos] = ((lev - 1) << 27) | (int32_t)c;
                s_lb[grp][pos] = lbf;
            }
            sp += __popcll(gm);
            __builtin_amdgcn_wave_barrier();
        }
    }
    if (T.stats) {
#pragma unroll
        for (int off = kPtG2 / 2; off > 0; off >>= 1) {
            n_pts += __shfl_xor(n_pts, off, kPtG2);
            n_box += __shfl_xor(n_box, off, kPtG2);
        }
        if (sub == 0) {
            atomicAdd(T.stats + 0, (unsigned long long)n_pts);
            atomicAdd(T.stats + 1, (unsigned long long)n_box);
        }
    }
    if (sub == 0) {
        out_ids[qi] = bi;
        out_d2[qi] = bd;
    }
}

template <int D, int BS, int W>
__global__ __launch_bounds__(BS) void k_tree_nn1(PointTreeDev T, const double *__restrict__ q, int64_t nq,
                                                 int32_t *__restrict__ out_ids, double *__restrict__ out_d2) {
    if constexpr (W >= 2) tree_nn1_blockn<D, BS, W>(T, q, nq, out_ids, out_d2, blockIdx.x);
    else tree_nn1_block<D, BS>(T, q, nq, out_ids, out_d2, blockIdx.x);
}

// Many trees in one launch (mpt_rrt_step_many: one engine per independent seed).  Jobs are
// dealt to XCDs: workgroup b runs on XCD b % 8, so job j takes the workgroups of XCD j % 8
// and its tree stays in that XCD's L2.
// 8 waves per SIMD for d <= 7 (56 VGPRs, no spill); d = 15 would spill at 8, so 4 (108 VGPRs)
// W = 2: the two-node walk (tree_nn1_block2, 16 lanes per query), at 7 waves per SIMD for
// d <= 7 (72 VGPRs: the 8-wave budget spilled 8 a lane and ran 9 % slower); W = 8 (the default
// eight-node walk, one query a wave) at 8 waves: 64 VGPRs with 2 spilled vs 66 at 7 waves, joint
// NN 0.964 -> 0.945 ms (32 seeds), 7.36 -> 7.28 ms (256 seeds), profiles/r19/ab_c5/w8_summary.txt
template <int D, int BS, int W>
__global__ __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(D >= 15 ? 4 : (W >= 2 && W < 8 ? 7 : 8)))) void k_tree_nn1_jobs(
    const PtJob *__restrict__ jobs, int32_t n_jobs, int64_t nq, int64_t blocks_per_job) {
    const int64_t xcd = blockIdx.x % kXcds, slot = blockIdx.x / kXcds;
    const int64_t job = xcd + kXcds * (slot / blocks_per_job);
    if (job >= n_jobs) return;
    const PtJob &J = jobs[job];
    if constexpr (W >= 2) tree_nn1_blockn<D, BS, W>(J.T, J.q, nq, J.ids, J.d2, slot % blocks_per_job);
    else tree_nn1_block<D, BS>(J.T, J.q, nq, J.ids, J.d2, slot % blocks_per_job);
}

// Radius search (FLANN_KDTreeWrapper::kNearestWithin, utilities/flannkdtreewrapper.hpp:91-117:
// points with squared L2 < r2) over the tree; below_only keeps only ids <= the query's row
// (the milestones inserted before it).  Count pass (kFill = false) writes counts[qi]; the fill
// pass writes the ids and d2 of query qi at offsets[qi] in traversal order.
template <int D, bool kFill>
__global__ __launch_bounds__(256) void k_tree_radius(PointTreeDev T, const double *__restrict__ q, int64_t nq, double r2,
                                                     int32_t below_only, int32_t *__restrict__ counts,
                                                     const int64_t *__restrict__ offsets, int32_t *__restrict__ out_ids,
                                                     double *__restrict__ out_d2) {
    __shared__ int32_t s_node[kPtGroupsPerBlock][kPtStack];
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t slot = t / kPtFan;
    const int sub = (int)(t % kPtFan);
    const int grp = threadIdx.x / kPtFan;
    if (slot >= nq) return;
    double qq[D];
#pragma unroll
    for (int i = 0; i < D; ++i) qq[i] = q[slot * D + i];
    const int64_t n = live_n(T);
    const int base = (threadIdx.x & 63) & ~(kPtFan - 1);
    int64_t cursor = kFill ? offsets[slot] : 0;
    int32_t found = 0;
    if (n > 0) {
        int sp = 1;
        if (sub == 0) s_node[grp][0] = T.n_levels << 27;
        __builtin_amdgcn_wave_barrier();
        while (sp > 0) {
            --sp;
            const int32_t code = s_node[grp][sp];
            __builtin_amdgcn_wave_barrier();
            const int lev = code >> 27;
            const int64_t idx = code & ((1 << 27) - 1);
            if (lev == 1) {
                const int64_t p = idx * kPtFan + sub;
                bool hit = false;
                double dd = 0.0;
                int32_t id = 0;
                if (p < n) {
                    dd = flann_l2<D>(qq, T.pts + p * D);
                    id = T.ids[p];
                    hit = dd < r2 && (!below_only || (int64_t)id - 1 < slot);
                }
                const uint32_t gm = (uint32_t)(__ballot(hit) >> base) & 0xffu;
                if (kFill && hit) {
                    const int64_t pos = cursor + __popc(gm & ((1u << sub) - 1));
                    out_ids[pos] = id;
                    out_d2[pos] = dd;
                }
                cursor += __popc(gm);
                found += __popc(gm);
            } else {
                const int64_t c = idx * kPtFan + sub;
                bool keep = false;
                if (c < lvl_size(n, lev - 1)) {
                    const float *b = T.boxes + (lvl_off(T.n_upper, lev - 1) + c) * 2 * D;
                    double lb2 = 0.0;
#pragma unroll
                    for (int k = 0; k < D; ++k) {
                        const double g = fmax(fmax((double)b[k] - qq[k], qq[k] - (double)b[D + k]), 0.0);
                        lb2 += g * g;
                    }
                    keep = lb2 * (1.0 - 1e-12) < r2;
                }
                const uint32_t gm = (uint32_t)(__ballot(keep) >> base) & 0xffu;
                if (keep) s_node[grp][sp + __popc(gm & ((1u << sub) - 1))] = ((lev - 1) << 27) | (int32_t)c;
                sp += __popc(gm);
                __builtin_amdgcn_wave_barrier();
            }
        }
    }
    if (!kFill && sub == 0) counts[slot] = found;
}

}  // namespace

PointTree::~PointTree() {
    for (void *p : {(void *)keys, (void *)keys_sorted, (void *)vals, (void *)vals_sorted, (void *)sids, (void *)spts,
                    (void *)boxes, temp, (void *)bbox, (void *)plan})
        if (p) (void)hipFree(p);
    for (void *p : {(void *)ikeys[0], (void *)ikeys[1], (void *)iids[0], (void *)iids[1], (void *)ipts[0],
                    (void *)ipts[1], (void *)inkeys, (void *)invals, itemp, (void *)inidx, (void *)ibox, (void *)iplan,
                    (void *)ickeys, (void *)icvals, (void *)inpos, (void *)ihull_keys, (void *)ihull_pts,
                    (void *)ihull_ids})
        if (p) (void)hipFree(p);
}

void PointTree::reserve(int64_t n_upper, int32_t d) {
    if (n_upper > cap || d != dim) {
        for (void *p : {(void *)keys, (void *)keys_sorted, (void *)vals, (void *)vals_sorted, (void *)sids, (void *)spts})
            if (p) hip_check(hipFree(p), "free");
        const int64_t c = std::max<int64_t>(n_upper, std::max<int64_t>(2 * cap, 1024));
        hip_check(hipMalloc(&keys, sizeof(uint32_t) * c), "pt keys");
        hip_check(hipMalloc(&keys_sorted, sizeof(uint32_t) * c), "pt keys");
        hip_check(hipMalloc(&vals, sizeof(int32_t) * c), "pt vals");
        hip_check(hipMalloc(&vals_sorted, sizeof(int32_t) * c), "pt vals");
        hip_check(hipMalloc(&sids, sizeof(int32_t) * c), "pt ids");
        hip_check(hipMalloc(&spts, sizeof(double) * d * c), "pt points");
        cap = c;
        dim = d;
        size_t tb = 0;
        hipcub::DoubleBuffer<uint32_t> kbuf(keys, keys_sorted);
        hipcub::DoubleBuffer<int32_t> vbuf(vals, vals_sorted);
        hip_check(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, kbuf, vbuf, (int)c), "sort size");
        if (tb > temp_bytes) {
            if (temp) hip_check(hipFree(temp), "free");
            hip_check(hipMalloc(&temp, tb), "sort temp");
            temp_bytes = tb;
        }
        box_cap = 0;
    }
    if (!bbox) {
        // [min keys][max keys] + the box-level and bbox tickets (two u32); set once here, reset
        // by the build's own kernels
        hip_check(hipMalloc(&bbox, sizeof(unsigned long long) * (2 * kPtMaxDim + 1)), "pt bbox");
        hip_check(hipMemset(bbox, 0xff, sizeof(unsigned long long) * kPtMaxDim), "bbox init");
        hip_check(hipMemset(bbox + kPtMaxDim, 0, sizeof(unsigned long long) * (kPtMaxDim + 1)), "bbox init");
        hip_check(hipDeviceSynchronize(), "bbox init sync");  // null stream vs the caller's stream
        ticket = reinterpret_cast<unsigned int *>(bbox + 2 * kPtMaxDim);
        hip_check(hipMalloc(&plan, sizeof(CodePlan)), "pt plan");
    }
    reserve_boxes(n_upper, d);
}

void PointTree::reserve_boxes(int64_t n_upper, int32_t d) {
    const int64_t nb = lvl_off(n_upper, pt_levels(n_upper) + 1);
    if (nb * 2 * d > box_cap) {
        if (boxes) hip_check(hipFree(boxes), "free");
        box_cap = std::max<int64_t>(nb * 2 * d, 2 * box_cap);
        hip_check(hipMalloc(&boxes, sizeof(float) * box_cap), "pt boxes");
    }
}

void PointTree::build(const double *pts, int64_t n_upper, const int64_t *n_dev, int32_t d, hipStream_t stream,
                      const SpreadOut *spread) {
    if (d != 3 && d != 7 && d != 15) throw Error{1, "point tree: state dim must be 3, 7 or 15"};
    if (n_upper >= (int64_t(1) << 27)) throw Error{1, "point tree: too many points"};
    reserve(n_upper, d);
    t.d = d;
    t.n_upper = n_upper;
    t.n_levels = pt_levels(n_upper);
    t.n_dev = n_dev;
    t.boxes = boxes;
    t.pts = spts;
    t.ids = sids;
    t.hull_pts = nullptr;
    t.hull_ids = nullptr;
    if (n_upper <= 0) return;
    const unsigned blocks = (unsigned)((n_upper + 255) / 256);
    // bbox starts empty (reserve) and the plan (in k_pt_bbox's last workgroup) resets it after
    // reading it
    const SpreadOut sp = spread ? *spread : SpreadOut{};
    hipLaunchKernelGGL(k_pt_bbox, dim3(64), dim3(256), 0, stream, pts, d, n_upper, n_dev, bbox, ticket + 1, plan, sp);
    hipLaunchKernelGGL(k_pt_morton, dim3(blocks), dim3(256), 0, stream, pts, d, n_upper, n_dev, plan, keys, vals);
    hip_check(hipGetLastError(), "k_pt_morton");
    size_t tb = temp_bytes;
    // double-buffered: the sort ends in whichever buffer its last pass wrote (no copy back)
    hipcub::DoubleBuffer<uint32_t> kbuf(keys, keys_sorted);
    hipcub::DoubleBuffer<int32_t> vbuf(vals, vals_sorted);
    hip_check(hipcub::DeviceRadixSort::SortPairs(temp, tb, kbuf, vbuf, (int)n_upper, 0, 32, stream), "radix sort");
    hipLaunchKernelGGL(k_pt_gather, dim3(blocks), dim3(256), 0, stream, pts, d, n_upper, n_dev, vbuf.Current(), spts,
                       sids, boxes);
    hip_check(hipGetLastError(), "k_pt_gather");
    if (t.n_levels < 2) return;  // the gather's one leaf box is the root
    const unsigned box_groups = (unsigned)((n_upper + kPtChunkLeaves * kPtFan - 1) / (kPtChunkLeaves * kPtFan));
    hipLaunchKernelGGL(k_pt_boxes, dim3(box_groups), dim3(256), 0, stream, t, boxes, ticket);
    hip_check(hipGetLastError(), "k_pt_boxes");
}

IncPlan make_inc_plan(int32_t d, const double *lo, const double *hi, int32_t spatial) {
    IncPlan P{};
    double ext[kPtMaxDim] = {}, emax = 0.0;
    for (int j = 0; j < d; ++j) {
        ext[j] = hi[j] > lo[j] ? hi[j] - lo[j] : 0.0;
        emax = std::max(emax, ext[j]);
    }
    auto bits_of = [&](int j, double h, int k) {
        int b = 0;
        while (b < k && std::ldexp(h, b) < ext[j]) ++b;
        return b;
    };
    int kstar = 0;
    for (int k = 1; emax > 0.0 && k <= 31; ++k) {
        const double h = std::ldexp(emax, -k);
        int tot = 0;
        for (int j = 0; j < d; ++j) tot += bits_of(j, h, k);
        if (tot > kPtIncBits) break;
        kstar = k;
    }
    int b[kPtMaxDim] = {}, bmax = 0;
    for (int j = 0; j < d; ++j) {
        b[j] = kstar > 0 ? bits_of(j, std::ldexp(emax, -kstar), kstar) : 0;
        bmax = std::max(bmax, b[j]);
        P.lo[j] = lo[j];
        P.qmax[j] = b[j] > 0 ? (uint32_t)((1ull << b[j]) - 1) : 0u;
        P.scale[j] = b[j] > 0 ? std::ldexp(1.0, b[j]) / ext[j] : 0.0;
    }
    int n = 0;
    for (int l = bmax - 1; l >= 0; --l)
        for (int j = 0; j < d; ++j)
            if (b[j] > l) {
                P.dim[n] = (int8_t)j;
                P.bit[n] = (int8_t)l;
                ++n;
            }
    P.n = n;
    // seed slots: every dim's minimum and maximum, then directions over the first `spatial`
    // dims spread evenly (a Fibonacci lattice on the sphere; the circle for two dims)
    int h = 0;
    for (int j = 0; j < d && h + 1 < kPtHull; ++j) {
        P.hkind[h] = 1;
        P.hdim[h++] = (int8_t)j;
        P.hkind[h] = 2;
        P.hdim[h++] = (int8_t)j;
    }
    const int sd = std::max(1, std::min<int>(spatial, std::min(d, 3)));
    const int nd = kPtHull - h;
    for (int k = 0; k < nd; ++k, ++h) {
        double u[3] = {0.0, 0.0, 0.0};
        if (sd == 3) {
            const double z = 1.0 - (2.0 * k + 1.0) / nd, r = std::sqrt(std::max(0.0, 1.0 - z * z));
            const double phi = k * 2.399963229728653;  // the golden angle
            u[0] = r * std::cos(phi);
            u[1] = r * std::sin(phi);
            u[2] = z;
        } else if (sd == 2) {
            const double a = 2.0 * M_PI * (k + 0.5) / nd;
            u[0] = std::cos(a);
            u[1] = std::sin(a);
        } else {
            u[0] = (k & 1) ? 1.0 : -1.0;
        }
        P.hkind[h] = 0;
        P.hdim[h] = 0;
        for (int j = 0; j < 3; ++j) P.hdir[h][j] = (float)u[j];
    }
    P.n_hull = h;
    return P;
}

void PointTree::inc_reserve(int64_t c, int32_t d) {
    if (c <= icap && d == idim) return;
    hip_check(hipDeviceSynchronize(), "sync");  // the old buffers may still be in use
    for (void *p : {(void *)ikeys[0], (void *)ikeys[1], (void *)iids[0], (void *)iids[1], (void *)ipts[0],
                    (void *)ipts[1], (void *)inkeys, (void *)invals, itemp, (void *)ihull_pts})
        if (p) hip_check(hipFree(p), "free");
    c = std::max<int64_t>(c, 1024);
    for (int b = 0; b < 2; ++b) {
        hip_check(hipMalloc(&ikeys[b], sizeof(uint64_t) * c), "inc keys");
        hip_check(hipMalloc(&iids[b], sizeof(int32_t) * c), "inc ids");
        hip_check(hipMalloc(&ipts[b], sizeof(double) * d * c), "inc points");
    }
    hip_check(hipMalloc(&inkeys, sizeof(uint64_t) * c), "inc new keys");
    hip_check(hipMalloc(&invals, sizeof(int32_t) * c), "inc new rows");
    hip_check(hipMalloc(&ihull_pts, sizeof(double) * kPtHull * d), "inc seed rows");
    if (!ihull_keys) {
        hip_check(hipMalloc(&ihull_keys, sizeof(unsigned long long) * kPtHull), "inc seed keys");
        hip_check(hipMalloc(&ihull_ids, sizeof(int32_t) * kPtHull), "inc seed ids");
    }
    if (!ickeys) {
        hip_check(hipMalloc(&ickeys, sizeof(uint64_t) * kPtIncSeg), "inc chunk keys");
        hip_check(hipMalloc(&icvals, sizeof(int32_t) * kPtIncSeg), "inc chunk rows");
        hip_check(hipMalloc(&inpos, sizeof(int32_t) * kPtIncSeg), "inc new places");
    }
    size_t tb = 0;
    hip_check(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, ikeys[0], inkeys, iids[0], invals, (int)c, 0,
                                                  kPtIncBits),
              "inc sort size");
    hip_check(hipMalloc(&itemp, tb), "inc sort temp");
    itemp_bytes = tb;
    if (!inidx) {
        hip_check(hipMalloc(&inidx, sizeof(int64_t)), "inc count");
        hip_check(hipMemset(inidx, 0, sizeof(int64_t)), "inc count zero");
        hip_check(hipMalloc(&ibox, sizeof(unsigned long long) * 2 * kPtMaxDim), "inc box");
        hip_check(hipMalloc(&iplan, sizeof(IncPlan)), "inc plan");
        hip_check(hipDeviceSynchronize(), "inc init sync");  // null stream vs the caller's stream
    }
    icap = c;
    idim = d;
    icur = 0;
}

PtIncJob PointTree::prepare_inc(const double *pts, int64_t n_upper, const int64_t *n_dev, int32_t d, const double *lo,
                                const double *hi, int32_t spatial, bool full, hipStream_t stream,
                                const SpreadOut *spread) {
    if (d != 3 && d != 7 && d != 15) throw Error{1, "point tree: state dim must be 3, 7 or 15"};
    if (n_upper < 1 || n_upper >= (int64_t(1) << 27)) throw Error{1, "point tree: bad point count"};
    if (n_upper > icap || d != idim) {
        inc_reserve(n_upper, d);
        full = true;
    }
    reserve_boxes(icap, d);
    bool same = iplan_set;
    for (int j = 0; j < d && same; ++j) same = iplan_lo[j] == lo[j] && iplan_hi[j] == hi[j];
    if (!same) {
        const IncPlan P = make_inc_plan(d, lo, hi, spatial);
        hip_check(hipMemcpy(iplan, &P, sizeof(P), hipMemcpyHostToDevice), "inc plan");
        for (int j = 0; j < d; ++j) {
            iplan_lo[j] = lo[j];
            iplan_hi[j] = hi[j];
        }
        iplan_set = true;
        full = true;
    }
    const int old = icur, nw = icur ^ 1;
    if (full) {
        // every point: box, codes and seed offers, one radix sort into the new-point arrays; the
        // old arrays are scratch (the merge reads no old point)
        hipLaunchKernelGGL(k_pt_inc_box_reset, dim3(1), dim3(64), 0, stream, ibox);
        hip_check(hipMemsetAsync(ihull_keys, 0, sizeof(unsigned long long) * kPtHull, stream), "seed reset");
        hipLaunchKernelGGL(d == 3 ? k_pt_inc_bbox<3> : d == 7 ? k_pt_inc_bbox<7> : k_pt_inc_bbox<15>, dim3(64),
                           dim3(256), 0, stream, pts, d, n_upper, n_dev, ibox);
        const unsigned blocks = (unsigned)((n_upper + 255) / 256);
        hipLaunchKernelGGL(d == 3 ? k_pt_inc_codes<3> : d == 7 ? k_pt_inc_codes<7> : k_pt_inc_codes<15>, dim3(blocks),
                           dim3(64 * kHullWaves), 0, stream, pts, n_upper, n_dev, (const IncPlan *)iplan, ikeys[old],
                           iids[old], ihull_keys);
        hip_check(hipGetLastError(), "k_pt_inc_codes");
        size_t tb = itemp_bytes;
        hip_check(hipcub::DeviceRadixSort::SortPairs(itemp, tb, ikeys[old], inkeys, iids[old], invals, (int)n_upper, 0,
                                                      kPtIncBits, stream),
                  "inc full sort");
    }
    t.d = d;
    t.n_upper = n_upper;
    t.n_levels = pt_levels(n_upper);
    t.n_dev = n_dev;
    t.boxes = boxes;
    t.pts = ipts[nw];
    t.ids = iids[nw];
    t.hull_pts = ihull_pts;
    t.hull_ids = ihull_ids;
    icur = nw;
    PtIncJob J{};
    J.T = t;
    J.pts = pts;
    J.plan = iplan;
    J.okeys = ikeys[old];
    J.oids = iids[old];
    J.opts = ipts[old];
    J.keys = ikeys[nw];
    J.ids = iids[nw];
    J.spts = ipts[nw];
    J.boxes = boxes;
    J.nkeys = inkeys;
    J.nvals = invals;
    J.ckeys = ickeys;
    J.cvals = icvals;
    J.npos = inpos;
    J.nidx = inidx;
    J.ibox = ibox;
    J.err = nullptr;
    J.hull_keys = ihull_keys;
    J.hull_pts = ihull_pts;
    J.hull_ids = ihull_ids;
    J.full = full ? 1 : 0;
    if (spread) J.sp = *spread;
    return J;
}

void launch_tree_inc_jobs(const PtIncJob *d_jobs, const PtIncJob *h_jobs, int32_t n, int32_t d, hipStream_t stream) {
    if (n <= 0) return;
    // one job: passed in the kernel arguments (no staged table)
    IncJobs js{n == 1 ? nullptr : d_jobs, h_jobs[0]};
    int64_t max_n = 0;
    for (int32_t j = 0; j < n; ++j) max_n = std::max(max_n, h_jobs[j].T.n_upper);
    auto by_d = [&](auto k3, auto k7, auto k15) { return d == 3 ? k3 : d == 7 ? k7 : k15; };
    if (d != 3 && d != 7 && d != 15) throw Error{1, "point tree: state dim must be 3, 7 or 15"};
    // the new points' chunked sort (config 5 builds, 32 / 64 / 256 trees: 0.366 / 0.545 / 1.759
    // ms with the former one-workgroup sort, 0.297 / 0.515 / 1.761 ms chunked): codes and seed
    // offers, 512-pair chunks a wave, ranks across chunks
    hipLaunchKernelGGL(by_d(k_pt_inc_ncodes<3>, k_pt_inc_ncodes<7>, k_pt_inc_ncodes<15>),
                       dim3(kPtIncSeg / (64 * kHullWaves), n), dim3(64 * kHullWaves), 0, stream, js);
    hip_check(hipGetLastError(), "k_pt_inc_ncodes");
    hipLaunchKernelGGL(k_pt_inc_csort, dim3(kIncChunks / kIncChunkWaves, n), dim3(64 * kIncChunkWaves), 0, stream, js);
    hip_check(hipGetLastError(), "k_pt_inc_csort");
    hipLaunchKernelGGL(k_pt_inc_crank, dim3(kPtIncSeg / 256, n), dim3(256), 0, stream, js);
    hip_check(hipGetLastError(), "k_pt_inc_crank");
    hipLaunchKernelGGL(k_pt_inc_npos, dim3(kPtIncSeg / 256, n), dim3(256), 0, stream, js);
    hip_check(hipGetLastError(), "k_pt_inc_npos");
    hipLaunchKernelGGL(by_d(k_pt_inc_merge<3>, k_pt_inc_merge<7>, k_pt_inc_merge<15>),
                       dim3((unsigned)((max_n + kIncTile - 1) / kIncTile), n), dim3(kIncTile), 0, stream, js);
    hip_check(hipGetLastError(), "k_pt_inc_merge");
    const int64_t groups = (max_n + kPtChunkLeaves * kPtFan - 1) / (kPtChunkLeaves * kPtFan);
    hipLaunchKernelGGL(k_pt_inc_boxes, dim3((unsigned)groups, n), dim3(256), 0, stream, js);
    hipLaunchKernelGGL(k_pt_inc_top, dim3(n), dim3(256), 0, stream, js);
    hip_check(hipGetLastError(), "k_pt_inc_top");
}

void launch_tree_radius(const PointTreeDev &T, const double *q, int64_t nq, double r2, bool below_only,
                        int32_t *counts, const int64_t *offsets, int32_t *ids, double *d2, hipStream_t stream) {
    if (nq <= 0) return;
    if (T.d != 3) throw Error{1, "point tree radius: keys must have 3 dims"};
    const dim3 grid((unsigned)((nq * kPtFan + 255) / 256));
    if (offsets)
        hipLaunchKernelGGL((k_tree_radius<3, true>), grid, dim3(256), 0, stream, T, q, nq, r2, (int32_t)below_only,
                           counts, offsets, ids, d2);
    else
        hipLaunchKernelGGL((k_tree_radius<3, false>), grid, dim3(256), 0, stream, T, q, nq, r2, (int32_t)below_only,
                           counts, offsets, ids, d2);
    hip_check(hipGetLastError(), "k_tree_radius launch");
}

template <int W>
static void launch_tree_nn1_w(const PointTreeDev &T, const double *q, int64_t nq, int32_t *ids, double *d2,
                              hipStream_t stream) {
    constexpr int BS = 64;  // one-wave workgroups spread an engine round's few thousand queries over all CUs
    const dim3 grid((unsigned)((nq * kPtFan * W + BS - 1) / BS));
    switch (T.d) {
        case 3: hipLaunchKernelGGL((k_tree_nn1<3, BS, W>), grid, dim3(BS), 0, stream, T, q, nq, ids, d2); break;
        case 7: hipLaunchKernelGGL((k_tree_nn1<7, BS, W>), grid, dim3(BS), 0, stream, T, q, nq, ids, d2); break;
        case 15: hipLaunchKernelGGL((k_tree_nn1<15, BS, W>), grid, dim3(BS), 0, stream, T, q, nq, ids, d2); break;
        default: throw Error{1, "point tree: state dim must be 3, 7 or 15"};
    }
    hip_check(hipGetLastError(), "k_tree_nn1 launch");
}

void launch_tree_nn1(const PointTreeDev &T, const double *q, int64_t nq, int32_t *ids, double *d2, hipStream_t stream) {
    if (nq <= 0) return;
    const int w = pt_nn_width(T.d, nq);
    if (w == 8) launch_tree_nn1_w<8>(T, q, nq, ids, d2, stream);
    else if (w == 4) launch_tree_nn1_w<4>(T, q, nq, ids, d2, stream);
    else launch_tree_nn1_w<1>(T, q, nq, ids, d2, stream);
}

template <int BS, int W>
static void launch_tree_nn1_jobs_bs(const PtJob *d_jobs, int32_t n_jobs, int32_t d, int64_t nq, hipStream_t stream) {
    const int64_t bpj = (nq * kPtFan * W + BS - 1) / BS;
    const int64_t groups = (n_jobs + kXcds - 1) / kXcds;
    const dim3 grid((unsigned)(kXcds * groups * bpj));
    switch (d) {
        case 3: hipLaunchKernelGGL((k_tree_nn1_jobs<3, BS, W>), grid, dim3(BS), 0, stream, d_jobs, n_jobs, nq, bpj); break;
        case 7: hipLaunchKernelGGL((k_tree_nn1_jobs<7, BS, W>), grid, dim3(BS), 0, stream, d_jobs, n_jobs, nq, bpj); break;
        case 15: hipLaunchKernelGGL((k_tree_nn1_jobs<15, BS, W>), grid, dim3(BS), 0, stream, d_jobs, n_jobs, nq, bpj); break;
        default: throw Error{1, "point tree: state dim must be 3, 7 or 15"};
    }
    hip_check(hipGetLastError(), "k_tree_nn1_jobs launch");
}

void launch_tree_nn1_jobs(const PtJob *d_jobs, int32_t n_jobs, int32_t d, int64_t nq, hipStream_t stream) {
    if (nq <= 0 || n_jobs <= 0) return;
    // The multi-node walk cuts a query's dependent steps (eight nodes a step: an eighth) for
    // more nodes visited.  With the parts' best merged only on steps where a lane examined a
    // point and the ranks skipped on steps without a survivor, the widest walk wins at every
    // size: config 5 round time by nodes a step (1 / 2 / 4 / 8), 32 seeds (131 072 queries)
    // - / - / 1.86 / 1.59 ms, 64 seeds - / - / 3.36 / 2.97 ms, 256 seeds (1 M queries) 12.83 /
    // 12.53 / 11.26 / 10.80 ms (round 3, before the seeds).
    const int w = pt_nn_width(d, (int64_t)n_jobs * nq);
    if (w == 2) launch_tree_nn1_jobs_bs<64, 2>(d_jobs, n_jobs, d, nq, stream);
    else if (w == 8) launch_tree_nn1_jobs_bs<64, 8>(d_jobs, n_jobs, d, nq, stream);
    else if (w == 4) launch_tree_nn1_jobs_bs<64, 4>(d_jobs, n_jobs, d, nq, stream);
    else launch_tree_nn1_jobs_bs<64, 1>(d_jobs, n_jobs, d, nq, stream);
}

}  // namespace mpt
