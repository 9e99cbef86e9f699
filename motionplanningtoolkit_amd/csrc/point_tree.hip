// point_tree.hip -- radius search over a point snapshot with a packed Morton tree (PRM).
//
// Replaces FLANN_KDTreeWrapper::kNearestWithin (utilities/flannkdtreewrapper.hpp:91-117) for
// PRM's connection step (planners/prm.hpp:330-346): every milestone's neighbours within the
// connection radius, among the milestones inserted before it.
//
// Build (stream-ordered, no host sync; four launches + the sort): bounding box of the points
// -> code plan (below) -> 30-bit interleaved code per point -> hipcub radix sort ->
// coordinates and ids gathered into code order with the leaf boxes (8 consecutive points) ->
// the 8-ary levels above them in one launch, each box the float-widened bounds (a lower bound
// on FLANN's squared L2).
//
// Query: 8 lanes per query walk the tree with a per-group LDS stack; at an inner node the
// lanes test its 8 children's boxes against the radius, at a leaf each lane tests one point in
// FLANN's L2<double> order.  A count pass sizes each query's output, a fill pass writes it.
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

constexpr int kPtGroupsPerBlock = 256 / kPtFan;
constexpr int kPtStack = kPtFan * kPtMaxLevels;

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

}  // namespace mpt
