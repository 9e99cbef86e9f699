// point_tree.hip -- exact 1-NN over a tree snapshot with a packed Morton tree.
//
// Replaces FLANN_KDTreeWrapper::nearest (utilities/flannkdtreewrapper.hpp:57-89) for trees
// that do not fill the sampling box: an RRT grows from its start, so most uniform samples
// lie far from every node, and a uniform grid over the sampling box walks many empty rings
// for them.  Here the cost of a query depends on the tree's shape, not on where it lies.
//
// Build (every round, stream-ordered, no host sync): bounding box of the live nodes ->
// code plan (below) -> 30-bit interleaved code per node -> hipcub radix sort -> coordinates
// and ids gathered into code order -> leaves of 8 consecutive points and 8-ary levels above
// them, each box the float-widened bounds over all state dims (a lower bound on FLANN's
// squared L2).
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

// per-dim min / max of the live points as order keys: box[0..d) min, box[kPtMaxDim..) max
__global__ __launch_bounds__(256) void k_pt_bbox(const double *__restrict__ pts, int32_t d, int64_t n_upper,
                                                 const int64_t *__restrict__ n_dev, unsigned long long *__restrict__ box) {
    __shared__ unsigned long long s_min[kPtMaxDim], s_max[kPtMaxDim];
    if (threadIdx.x < kPtMaxDim) {
        s_min[threadIdx.x] = ~0ull;
        s_max[threadIdx.x] = 0ull;
    }
    __syncthreads();
    const int64_t n = *n_dev < n_upper ? *n_dev : n_upper;
    for (int j = 0; j < d; ++j) {
        unsigned long long mn = ~0ull, mx = 0ull;
        for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
            const unsigned long long k = order_key_pt(pts[i * d + j]);
            mn = k < mn ? k : mn;
            mx = k > mx ? k : mx;
        }
        atomicMin(&s_min[j], mn);
        atomicMax(&s_max[j], mx);
    }
    __syncthreads();
    if (threadIdx.x < (unsigned)d) {
        atomicMin(box + threadIdx.x, s_min[threadIdx.x]);
        atomicMax(box + kPtMaxDim + threadIdx.x, s_max[threadIdx.x]);
    }
}

__global__ void k_pt_plan(int32_t d, const unsigned long long *__restrict__ box, CodePlan *__restrict__ plan,
                          SpreadOut sp) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    if (sp.host_out) {  // the engine's MPT_NN_AUTO feedback (grid_nn.h SpreadOut)
        for (int j = 0; j < 3; ++j) {
            sp.host_out[j] = j < sp.gd ? box[sp.dims[j]] : ~0ull;
            sp.host_out[3 + j] = j < sp.gd ? box[kPtMaxDim + sp.dims[j]] : 0ull;
        }
        __threadfence_system();
    }
    double lo[kPtMaxDim], ext[kPtMaxDim], emax = 0.0;
    for (int j = 0; j < d; ++j) {
        lo[j] = key_value_pt(box[j]);
        const double hi = key_value_pt(box[kPtMaxDim + j]);
        ext[j] = hi > lo[j] ? hi - lo[j] : 0.0;
        emax = ext[j] > emax ? ext[j] : emax;
    }
    int32_t b[kPtMaxDim];
    for (int j = 0; j < d; ++j) b[j] = 0;
    if (emax > 0.0) {
        // finest level k (h = emax / 2^k) whose bit total fits the code
        for (int k = 1; k <= kCodeBits; ++k) {
            const double h = ldexp(emax, -k);
            int32_t bt[kPtMaxDim], tot = 0;
            for (int j = 0; j < d; ++j) {
                int32_t bj = 0;
                while (bj < k && ldexp(h, bj) < ext[j]) ++bj;
                bt[j] = bj;
                tot += bj;
            }
            if (tot > kCodeBits) break;
            for (int j = 0; j < d; ++j) b[j] = bt[j];
        }
    }
    int32_t bmax = 0;
    for (int j = 0; j < d; ++j) {
        plan->lo[j] = lo[j];
        plan->qmax[j] = b[j] > 0 ? (1u << b[j]) - 1 : 0u;
        plan->scale[j] = b[j] > 0 ? ldexp(1.0, b[j]) / ext[j] : 0.0;
        bmax = b[j] > bmax ? b[j] : bmax;
    }
    int32_t n = 0;
    for (int t = bmax - 1; t >= 0; --t)
        for (int j = 0; j < d; ++j)
            if (b[j] > t) {
                plan->dim[n] = (int8_t)j;
                plan->bit[n] = (int8_t)t;
                ++n;
            }
    plan->n = n;
}

__global__ void k_pt_morton(const double *__restrict__ pts, int32_t d, int64_t n_upper, const int64_t *__restrict__ n_dev,
                            const CodePlan *__restrict__ plan, uint32_t *__restrict__ keys, int32_t *__restrict__ vals) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_upper) return;
    const int64_t n = *n_dev < n_upper ? *n_dev : n_upper;
    vals[i] = (int32_t)i;
    if (i >= n) {
        keys[i] = 0xffffffffu;  // past the live count: sorted to the end
        return;
    }
    uint32_t q[kPtMaxDim];
    for (int j = 0; j < d; ++j) {
        const double u = (pts[i * d + j] - plan->lo[j]) * plan->scale[j];
        const uint32_t m = plan->qmax[j];
        q[j] = u <= 0.0 ? 0u : (u >= (double)m ? m : (uint32_t)u);
    }
    uint32_t code = 0;
    const int32_t nb = plan->n;
    for (int k = 0; k < nb; ++k) code = (code << 1) | ((q[plan->dim[k]] >> plan->bit[k]) & 1u);
    keys[i] = code;
}

__global__ void k_pt_gather(const double *__restrict__ pts, int32_t d, int64_t n_upper, const int64_t *__restrict__ n_dev,
                            const int32_t *__restrict__ order, double *__restrict__ spts, int32_t *__restrict__ sids) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t n = *n_dev < n_upper ? *n_dev : n_upper;
    if (i >= n) return;
    const int32_t src = order[i];
    for (int j = 0; j < d; ++j) spts[i * d + j] = pts[(int64_t)src * d + j];
    sids[i] = src + 1;
}

// level-1 boxes: the widened bounds of 8 consecutive points over every dim
__global__ void k_pt_leaf_boxes(PointTreeDev T, const double *__restrict__ spts, float *__restrict__ boxes) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t n = live_n(T);
    if (j >= lvl_size(n, 1)) return;
    const int d = T.d;
    float *b = boxes + j * 2 * d;
    const int64_t p0 = j * kPtFan, p1 = p0 + kPtFan < n ? p0 + kPtFan : n;
    for (int k = 0; k < d; ++k) {
        double lo = spts[p0 * d + k], hi = lo;
        for (int64_t p = p0 + 1; p < p1; ++p) {
            const double x = spts[p * d + k];
            lo = x < lo ? x : lo;
            hi = x > hi ? x : hi;
        }
        b[k] = widen_lo(lo);
        b[d + k] = widen_hi(hi);
    }
}

__global__ void k_pt_up_boxes(PointTreeDev T, int l, float *__restrict__ boxes) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t n = live_n(T);
    if (j >= lvl_size(n, l)) return;
    const int d = T.d;
    const float *child = boxes + lvl_off(T.n_upper, l - 1) * 2 * d;
    float *b = boxes + (lvl_off(T.n_upper, l) + j) * 2 * d;
    const int64_t c0 = j * kPtFan, nc = lvl_size(n, l - 1), c1 = c0 + kPtFan < nc ? c0 + kPtFan : nc;
    for (int k = 0; k < d; ++k) {
        float lo = child[c0 * 2 * d + k], hi = child[c0 * 2 * d + d + k];
        for (int64_t c = c0 + 1; c < c1; ++c) {
            lo = fminf(lo, child[c * 2 * d + k]);
            hi = fmaxf(hi, child[c * 2 * d + d + k]);
        }
        b[k] = lo;
        b[d + k] = hi;
    }
}

constexpr int kPtGroupsPerBlock = 256 / kPtFan;
constexpr int kPtStack = kPtFan * kPtMaxLevels;

template <int D>
__global__ __launch_bounds__(256) void k_tree_nn1(PointTreeDev T, const double *__restrict__ q, int64_t nq,
                                                  int32_t *__restrict__ out_ids, double *__restrict__ out_d2) {
    __shared__ int32_t s_node[kPtGroupsPerBlock][kPtStack];
    __shared__ double s_lb[kPtGroupsPerBlock][kPtStack];
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t slot = t / kPtFan;
    const int sub = (int)(t % kPtFan);
    const int grp = threadIdx.x / kPtFan;
    if (slot >= nq) return;  // whole groups leave together
    double qq[D];
#pragma unroll
    for (int i = 0; i < D; ++i) qq[i] = q[slot * D + i];
    const int64_t n = live_n(T);
    double bd = __builtin_huge_val();
    int32_t bi = -1;
    uint32_t n_pts = 0, n_box = 0;
    if (n > 0) {
        int sp = 1;
        if (sub == 0) {
            s_node[grp][0] = T.n_levels << 27;  // the root: level n_levels, index 0
            s_lb[grp][0] = 0.0;
        }
        __builtin_amdgcn_wave_barrier();
        while (sp > 0) {
            --sp;
            const int32_t code = s_node[grp][sp];
            const double lbs = s_lb[grp][sp];
            __builtin_amdgcn_wave_barrier();
            // the 1e-12 shrink covers FLANN's summation order (as the grid kernel)
            if (lbs * (1.0 - 1e-12) > bd) continue;
            const int lev = code >> 27;
            const int64_t idx = code & ((1 << 27) - 1);
            if (lev == 1) {
                const int64_t p = idx * kPtFan + sub;
                if (p < n) {
                    const double dd = flann_l2<D>(qq, T.pts + p * D);
                    const int32_t id = T.ids[p];
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
                double lb2 = 0.0;
                if (c < lvl_size(n, lev - 1)) {
                    const float *b = T.boxes + (lvl_off(T.n_upper, lev - 1) + c) * 2 * D;
#pragma unroll
                    for (int k = 0; k < D; ++k) {
                        const double g = fmax(fmax((double)b[k] - qq[k], qq[k] - (double)b[D + k]), 0.0);
                        lb2 += g * g;
                    }
                    keep = lb2 * (1.0 - 1e-12) <= bd;
                    ++n_box;
                }
                const int base = (threadIdx.x & 63) & ~(kPtFan - 1);
                const uint32_t gm = (uint32_t)(__ballot(keep) >> base) & 0xffu;
                int rank = 0;
#pragma unroll
                for (int j = 0; j < kPtFan; ++j) {
                    const double o = __shfl(lb2, j, kPtFan);
                    if (((gm >> j) & 1u) && (o > lb2 || (o == lb2 && j > sub))) ++rank;
                }
                if (keep) {
                    s_node[grp][sp + rank] = ((lev - 1) << 27) | (int32_t)c;
                    s_lb[grp][sp + rank] = lb2;
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
        out_ids[slot] = bi;
        out_d2[slot] = bd;
    }
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
}

void PointTree::reserve(int64_t n_upper, int32_t d) {
    const int32_t L = pt_levels(n_upper);
    const int64_t nb = lvl_off(n_upper, L + 1);
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
        hip_check(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, keys, keys_sorted, vals, vals_sorted, (int)c),
                  "sort size");
        if (tb > temp_bytes) {
            if (temp) hip_check(hipFree(temp), "free");
            hip_check(hipMalloc(&temp, tb), "sort temp");
            temp_bytes = tb;
        }
        box_cap = 0;
    }
    if (!bbox) {
        hip_check(hipMalloc(&bbox, sizeof(unsigned long long) * 2 * kPtMaxDim), "pt bbox");
        hip_check(hipMalloc(&plan, sizeof(CodePlan)), "pt plan");
    }
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
    hip_check(hipMemsetAsync(bbox, 0xff, sizeof(unsigned long long) * kPtMaxDim, stream), "bbox memset");
    hip_check(hipMemsetAsync(bbox + kPtMaxDim, 0, sizeof(unsigned long long) * kPtMaxDim, stream), "bbox memset");
    hipLaunchKernelGGL(k_pt_bbox, dim3(64), dim3(256), 0, stream, pts, d, n_upper, n_dev, bbox);
    hipLaunchKernelGGL(k_pt_plan, dim3(1), dim3(64), 0, stream, d, bbox, plan, spread ? *spread : SpreadOut{});
    hipLaunchKernelGGL(k_pt_morton, dim3(blocks), dim3(256), 0, stream, pts, d, n_upper, n_dev, plan, keys, vals);
    hip_check(hipGetLastError(), "k_pt_morton");
    size_t tb = temp_bytes;
    hip_check(hipcub::DeviceRadixSort::SortPairs(temp, tb, keys, keys_sorted, vals, vals_sorted, (int)n_upper, 0,
                                                 32, stream),
              "radix sort");
    hipLaunchKernelGGL(k_pt_gather, dim3(blocks), dim3(256), 0, stream, pts, d, n_upper, n_dev, vals_sorted, spts,
                       sids);
    hip_check(hipGetLastError(), "k_pt_gather");
    const int64_t m1 = lvl_size(n_upper, 1);
    hipLaunchKernelGGL(k_pt_leaf_boxes, dim3((unsigned)((m1 + 255) / 256)), dim3(256), 0, stream, t, spts, boxes);
    hip_check(hipGetLastError(), "k_pt_leaf_boxes");
    for (int l = 2; l <= t.n_levels; ++l) {
        const int64_t ml = lvl_size(n_upper, l);
        hipLaunchKernelGGL(k_pt_up_boxes, dim3((unsigned)((ml + 255) / 256)), dim3(256), 0, stream, t, l, boxes);
        hip_check(hipGetLastError(), "k_pt_up_boxes");
    }
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

void launch_tree_nn1(const PointTreeDev &T, const double *q, int64_t nq, int32_t *ids, double *d2, hipStream_t stream) {
    if (nq <= 0) return;
    const dim3 grid((unsigned)((nq * kPtFan + 255) / 256));
    switch (T.d) {
        case 3: hipLaunchKernelGGL(k_tree_nn1<3>, grid, dim3(256), 0, stream, T, q, nq, ids, d2); break;
        case 7: hipLaunchKernelGGL(k_tree_nn1<7>, grid, dim3(256), 0, stream, T, q, nq, ids, d2); break;
        case 15: hipLaunchKernelGGL(k_tree_nn1<15>, grid, dim3(256), 0, stream, T, q, nq, ids, d2); break;
        default: throw Error{1, "point tree: state dim must be 3, 7 or 15"};
    }
    hip_check(hipGetLastError(), "k_tree_nn1 launch");
}

}  // namespace mpt
