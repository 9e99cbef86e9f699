// grid_nn.hip -- exact nearest-neighbour search through a uniform grid built on the device.
//
// Same contract as nn.hip (FLANN L2<double> order, 1-based ids, (d2, id) order), but each
// query visits only the grid cells that can still hold a better point:
//   * the grid covers gd <= 3 "spatial" state dims (x, y, z for the omni/blimp agents,
//     x, y for the snake) with cubic cells of side h (about `ppc` points per cell);
//   * a query walks Chebyshev rings r = 0, 1, 2, ... of cells around its own cell; after
//     ring r every unvisited point lies outside the (2r+1)^gd block, so its squared
//     distance is >= LB^2, LB = distance from the query to the block boundary along the
//     grid dims (the other dims only add non-negative terms; FLANN's sum of squares is
//     monotone in each term, so fl(d2) >= fl(LB^2) for the exact LB);
//   * the walk stops once LB_safe^2 > worst-of-k (strict: exact ties are still visited and
//     resolved by id), LB_safe = LB minus a slack far above the rounding of the cell
//     assignment, so the result equals the brute-force result bit for bit.
// Build per snapshot: cell id per point (atomic histogram) -> exclusive scan (scan.h) ->
// scatter of coordinates and ids into cell order.  The in-cell order is arbitrary, which
// cannot change any result (all ties resolve by id).
#include <algorithm>
#include <cstring>

#include <hipcub/hipcub.hpp>

#include "../../include/mpt.h"
#include "grid_nn.h"
#include "scan.h"

namespace mpt {

__device__ __forceinline__ int cell_coord(double x, double lo, double inv_h, int n) {
    double c = floor((x - lo) * inv_h);
    c = c < 0.0 ? 0.0 : c;
    c = c > (double)(n - 1) ? (double)(n - 1) : c;
    return (int)c;
}

__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_xor(v, off);
        v = o < v ? o : v;
    }
    return v;
}
__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_xor(v, off);
        v = o > v ? o : v;
    }
    return v;
}

// Block-wide fold of per-thread (min[3], max[3]) keys (blockDim.x == 256) into s_out[6],
// visible to every thread of the block on return.
__device__ __forceinline__ void block_fold_spread(unsigned long long (&mn)[3], unsigned long long (&mx)[3],
                                                  unsigned long long (*s_v)[6], unsigned long long *s_out) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        mn[j] = wave_min_u64(mn[j]);
        mx[j] = wave_max_u64(mx[j]);
    }
    if (lane == 0)
        for (int j = 0; j < 3; ++j) {
            s_v[wave][j] = mn[j];
            s_v[wave][3 + j] = mx[j];
        }
    __syncthreads();
    if (threadIdx.x < 6) {
        const int j = threadIdx.x;
        unsigned long long v = s_v[0][j];
        for (int w = 1; w < 4; ++w) v = j < 3 ? (s_v[w][j] < v ? s_v[w][j] : v) : (s_v[w][j] > v ? s_v[w][j] : v);
        s_out[j] = v;
    }
    __syncthreads();
}

// Cell of every live point + histogram.  kSpread: the same pass also reduces the points'
// spread (SpreadOut) into one partial per block (plain stores, no fence: the scatter kernel
// that follows in the stream folds them).
// One workgroup's kQueriesPerBlock queries into their buckets: an LDS histogram, then one
// device atomic per (workgroup, bucket) for the bucket's base, then each query's slot.  The
// device atomics on one bucket serialise, so a workgroup takes 256 * kQueriesPerThread
// queries (512 by default: 128 atomics per bucket for 65536 queries).
template <int kQueriesPerThread>
__device__ __forceinline__ void bucket_queries(const QueryBucketing &qb, int32_t d, int64_t first) {
    __shared__ int32_t s_cnt[kQueryBuckets], s_base[kQueryBuckets];
    const QueryOrder &o = qb.o;
    if (threadIdx.x < kQueryBuckets) s_cnt[threadIdx.x] = 0;
    __syncthreads();
    const SampleGen &gen = qb.gen;
    if (gen.out && first == 0 && threadIdx.x == 0) {
        // the round's start (what k_sample's thread 0 does): the count kernel's point blocks
        // take the pending truncation as an argument, so this write races with no reader
        if (gen.set_n >= 0) {
            gen.n_dev[0] = gen.set_n;
            gen.counters[3] = (unsigned long long)gen.set_n;
        }
        gen.n_dev[1] = gen.set_n >= 0 ? gen.set_n : gen.n_dev[0];
        if (gen.n_live) *gen.n_live = 0u;
    }
    int32_t b[kQueriesPerThread], rank[kQueriesPerThread];
#pragma unroll
    for (int h = 0; h < kQueriesPerThread; ++h) {
        const int64_t k = first + h * 256 + threadIdx.x;
        b[h] = -1;
        rank[h] = 0;
        if (k < qb.nq) {
            double x;
            if (gen.out) {
                // the engine's sample k (rrt_engine.hip k_sample: counters g * 64 + j)
                const uint64_t g = gen.ext_base + (uint64_t)k;
                x = 0.0;
                for (int j = 0; j < d; ++j) {
                    const double v = engine_uniform(gen.seed, g * 64 + j, gen.lo[j], gen.hi[j]);
                    gen.out[k * d + j] = v;
                    if (j == o.dim) x = v;
                }
            } else {
                x = qb.q[k * d + o.dim];
            }
            b[h] = query_bucket(o, x);
            rank[h] = atomicAdd(&s_cnt[b[h]], 1);
        }
    }
    __syncthreads();
    if (threadIdx.x < o.nb && s_cnt[threadIdx.x] > 0)
        s_base[threadIdx.x] = atomicAdd(o.count + threadIdx.x * kQCountStride, s_cnt[threadIdx.x]);
    __syncthreads();
#pragma unroll
    for (int h = 0; h < kQueriesPerThread; ++h)
        if (b[h] >= 0) o.list[(int64_t)b[h] * o.cap + s_base[b[h]] + rank[h]] = (int32_t)(first + h * 256 + threadIdx.x);
}

// n_pt_blocks: the workgroups that count points; q_lead: the query-bucketing workgroups (qb)
// placed before them (0: after them)
template <bool kSpread, int kQPT>
__global__ __launch_bounds__(256) void k_grid_count(GridParams g, const double *__restrict__ pts, int32_t d,
                                                    int64_t n, const int64_t *__restrict__ n_dev,
                                                    int32_t *__restrict__ cell_of, int32_t *__restrict__ counts,
                                                    SpreadOut sp, uint32_t n_pt_blocks, uint32_t q_lead,
                                                    QueryBucketing qb) {
    if (blockIdx.x < q_lead) {  // workgroup-uniform
        bucket_queries<kQPT>(qb, d, (int64_t)blockIdx.x * (256 * kQPT));
        return;
    }
    const uint32_t pb = blockIdx.x - q_lead;
    if (pb >= n_pt_blocks) {  // workgroup-uniform
        bucket_queries<kQPT>(qb, d, (int64_t)(pb - n_pt_blocks) * (256 * kQPT));
        return;
    }
    const int64_t i = (int64_t)pb * blockDim.x + threadIdx.x;
    if (qb.gen.out && qb.gen.set_n >= 0)
        n = qb.gen.set_n < n ? qb.gen.set_n : n;  // applied to n_dev by the round-start block
    else if (n_dev)
        n = *n_dev < n ? *n_dev : n;
    if (i < n) {
        // the grid dims' coordinates loaded together (clamped, unconditional), then the cell
        double x[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) x[j] = pts[i * d + g.dims[j < g.gd ? j : 0]];
        int c[3] = {0, 0, 0};
#pragma unroll
        for (int j = 0; j < 3; ++j)
            if (j < g.gd) c[j] = cell_coord(x[j], g.lo[j], g.inv_h, g.n[j]);
        const int32_t cell = (c[0] * g.n[1] + c[1]) * g.n[2] + c[2];
        // the point's rank in its cell (arbitrary order: every result resolves ties by id), so
        // the scatter places it without an atomic of its own
        const int32_t rank = atomicAdd(counts + cell, 1);
        reinterpret_cast<int2 *>(cell_of)[i] = make_int2(cell, rank);
    }
    if constexpr (kSpread) {
        __shared__ unsigned long long s_v[4][6], s_out[6];
        unsigned long long mn[3] = {~0ull, ~0ull, ~0ull}, mx[3] = {0ull, 0ull, 0ull};
        if (i < n) {
#pragma unroll
            for (int j = 0; j < 3; ++j)
                if (j < sp.gd) mn[j] = mx[j] = order_key_u64(pts[i * d + sp.dims[j]]);
        }
        block_fold_spread(mn, mx, s_v, s_out);
        if (threadIdx.x < 6) sp.partial[(int64_t)pb * 6 + threadIdx.x] = s_out[threadIdx.x];
    }
}

// Scatter into cell order.  kSpread: block 0 first folds k_grid_count's per-block spread
// partials (n_part of them, all threads) and writes the result to mapped host memory.
template <bool kSpread, int D>
__global__ __launch_bounds__(256) void k_grid_scatter(const double *__restrict__ pts, int32_t d, int64_t n,
                                                      const int64_t *__restrict__ n_dev,
                                                      const int32_t *__restrict__ cell_of,
                                                      const int32_t *__restrict__ cell_start,
                                                      double *__restrict__ spts,
                                                      int32_t *__restrict__ sids, SpreadOut sp, int32_t n_part) {
    if constexpr (kSpread) {
        if (blockIdx.x == 0) {
            __shared__ unsigned long long s_v[4][6], s_out[6];
            unsigned long long mn[3] = {~0ull, ~0ull, ~0ull}, mx[3] = {0ull, 0ull, 0ull};
            for (int b = threadIdx.x; b < n_part; b += blockDim.x) {
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                    const unsigned long long lo = sp.partial[(int64_t)b * 6 + j];
                    const unsigned long long hi = sp.partial[(int64_t)b * 6 + 3 + j];
                    mn[j] = lo < mn[j] ? lo : mn[j];
                    mx[j] = hi > mx[j] ? hi : mx[j];
                }
            }
            block_fold_spread(mn, mx, s_v, s_out);
            // fine-grained mapped memory: the stores go straight to the host; the event the
            // engine records after the build orders them before the host reads
            if (threadIdx.x < 6) sp.host_out[threadIdx.x] = s_out[threadIdx.x];
        }
    }
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (n_dev) n = *n_dev < n ? *n_dev : n;
    if (i >= n) return;
    if constexpr (D > 0) {
        // the point's row loaded alongside its (cell, rank), not after the cell start (a
        // run-time-length copy loop would wait on each load in turn)
        double v[grid_stride(D) + 1];
#pragma unroll
        for (int j = 0; j < D; ++j) v[j] = pts[i * D + j];
        v[D] = __longlong_as_double((long long)(i + 1));
        const int2 cr = reinterpret_cast<const int2 *>(cell_of)[i];
        const int64_t pos = (int64_t)cell_start[cr.x] + cr.y;
        double *rec = spts + pos * grid_stride(D);
        if constexpr (grid_stride(D) > D) {  // even-length padded record: 16-B stores
#pragma unroll
            for (int j = 0; j < grid_stride(D) / 2; ++j)
                reinterpret_cast<double2 *>(rec)[j] = make_double2(v[2 * j], v[2 * j + 1]);
        } else {
#pragma unroll
            for (int j = 0; j < D; ++j) rec[j] = v[j];
            sids[pos] = (int32_t)(i + 1);
        }
    } else {
        const int2 cr = reinterpret_cast<const int2 *>(cell_of)[i];
        const int64_t pos = (int64_t)cell_start[cr.x] + cr.y;
        // record of d + 1 doubles: the coordinates, then the 1-based id in the pad slot, so a
        // query reads a point and its id from one 32 / 64 / 128-B aligned record
        double *rec = spts + pos * grid_stride(d);
        for (int j = 0; j < d; ++j) rec[j] = pts[i * d + j];
        if (grid_stride(d) > d)
            rec[d] = __longlong_as_double((long long)(i + 1));
        else
            sids[pos] = (int32_t)(i + 1);
    }
}

// scan epilogue of the grid build: each count back to zero once scanned
struct ZeroCounts {
    uint32_t *counts;
    __device__ void operator()(int64_t i, uint32_t, uint32_t v) const {
        if (v) counts[i] = 0u;
    }
};

template <int KMAX>
__device__ __forceinline__ void grid_push(double (&bd)[KMAX], int32_t (&bi)[KMAX], int32_t k, double dd, int32_t id) {
    bool done = false;
#pragma unroll
    for (int j = KMAX - 1; j >= 0; --j) {
        if (j >= k || done) continue;
        if (j == k - 1) {
            if (!nn_better(dd, id, bd[j], bi[j])) { done = true; continue; }
            bd[j] = dd;
            bi[j] = id;
        }
        if (j > 0 && nn_better(bd[j], bi[j], bd[j - 1], bi[j - 1])) {
            const double td = bd[j]; bd[j] = bd[j - 1]; bd[j - 1] = td;
            const int32_t ti = bi[j]; bi[j] = bi[j - 1]; bi[j - 1] = ti;
        } else {
            done = true;
        }
    }
}

// Lower bound on the distance (along the grid dims) from q to any cell outside the ring-r
// block; returns -1 when no cell lies outside (every cell visited).
__device__ __forceinline__ double ring_bound(const GridParams &g, const double *qg, const int *cq, int r) {
    double lb = __builtin_huge_val();
    bool more = false;
    for (int j = 0; j < g.gd; ++j) {
        if (cq[j] - r > 0) {
            more = true;
            const double edge = g.lo[j] + (double)(cq[j] - r) * g.h;
            lb = fmin(lb, qg[j] - edge);
        }
        if (cq[j] + r + 1 < g.n[j]) {
            more = true;
            const double edge = g.lo[j] + (double)(cq[j] + r + 1) * g.h;
            lb = fmin(lb, edge - qg[j]);
        }
    }
    if (!more) return -1.0;
    lb -= g.slack;
    return lb > 0.0 ? lb : 0.0;
}

template <int D, int KMAX>
__global__ __launch_bounds__(256) void k_grid_knn(GridDev G, int32_t d, const double *__restrict__ q, int64_t nq,
                                                  int32_t k, int32_t *__restrict__ out_ids, double *__restrict__ out_d2) {
    constexpr int DD = D > 0 ? D : 16;
    const int64_t ti = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (ti >= nq) return;
    const int64_t qi = ti;
    const GridParams &g = G.g;
    const int dim = D > 0 ? D : d;
    double qq[DD];
#pragma unroll
    for (int i = 0; i < DD; ++i) qq[i] = i < dim ? q[qi * dim + i] : 0.0;
    double qg[3] = {0, 0, 0};
    int cq[3] = {0, 0, 0};
    for (int j = 0; j < g.gd; ++j) {
        const double x = q[qi * dim + g.dims[j]];
        qg[j] = x;
        cq[j] = cell_coord(x, g.lo[j], g.inv_h, g.n[j]);
    }
    double bd[KMAX];
    int32_t bi[KMAX];
#pragma unroll
    for (int i = 0; i < KMAX; ++i) { bd[i] = __builtin_huge_val(); bi[i] = -1; }
    const int n1 = g.n[1], n2 = g.n[2];
    for (int r = 0;; ++r) {
        for (int dx = -r; dx <= r; ++dx) {
            const int cx = cq[0] + dx;
            if (cx < 0 || cx >= g.n[0]) continue;
            const bool ex = dx == -r || dx == r;
            for (int dy = -r; dy <= r; ++dy) {
                const int cy = cq[1] + dy;
                if (cy < 0 || cy >= n1) continue;
                const bool ey = ex || dy == -r || dy == r;
                const int step = ey ? 1 : (r > 0 ? 2 * r : 1);
                for (int dz = -r; dz <= r; dz += step) {
                    const int cz = cq[2] + dz;
                    if (cz < 0 || cz >= n2) continue;
                    const int32_t cell = (cx * n1 + cy) * n2 + cz;
                    const int32_t s = G.cell_start[cell], e = G.cell_start[cell + 1];
                    for (int32_t p = s; p < e; ++p) {
                        const double *rec = G.pts + (int64_t)p * (D > 0 ? grid_stride(D) : G.stride);
                        const double dd = D > 0 ? flann_l2<DD>(qq, rec) : flann_l2_dyn(qq, rec, dim);
                        const int32_t id = grid_id<D>(G, rec, dim, p);
                        if (G.removed && G.removed[id - 1]) continue;
                        double kd = bd[0];
                        int32_t ki = bi[0];
#pragma unroll
                        for (int i = 0; i < KMAX; ++i)
                            if (i == k - 1) { kd = bd[i]; ki = bi[i]; }
                        if (nn_better(dd, id, kd, ki)) grid_push<KMAX>(bd, bi, k, dd, id);
                    }
                }
            }
        }
        const double lb = ring_bound(g, qg, cq, r);
        if (lb < 0.0) break;  // every cell visited
        double worst = bd[0];
#pragma unroll
        for (int i = 0; i < KMAX; ++i)
            if (i == k - 1) worst = bd[i];
        if (lb * lb > worst) break;
    }
#pragma unroll
    for (int i = 0; i < KMAX; ++i)
        if (i < k) {
            out_ids[qi * k + i] = bi[i];
            out_d2[qi * k + i] = bd[i];
        }
}

GridParams make_grid_params(int32_t d, const int32_t *dims, int32_t gd, const double *lo, const double *hi, int64_t n,
                            double ppc, double h_min) {
    GridParams g{};
    g.gd = gd;
    double vol = 1.0, span_max = 0.0;
    for (int j = 0; j < gd; ++j) {
        g.dims[j] = dims[j];
        const double span = hi[j] > lo[j] ? hi[j] - lo[j] : 1.0;
        vol *= span;
        span_max = span > span_max ? span : span_max;
        g.lo[j] = lo[j];
    }
    for (int j = gd; j < 3; ++j) {
        g.dims[j] = 0;
        g.lo[j] = 0.0;
        g.n[j] = 1;
    }
    const double cells_wanted = n > 0 ? (double)n / ppc : 1.0;
    double h = pow(vol / (cells_wanted > 1.0 ? cells_wanted : 1.0), 1.0 / gd);
    h = h > h_min ? h : h_min;
    // cap the cell count (memory, scan length): at most 4 cells per point and 2^25 total
    for (;;) {
        double cells = 1.0;
        for (int j = 0; j < gd; ++j) {
            const double span = hi[j] > lo[j] ? hi[j] - lo[j] : 1.0;
            cells *= ceil(span / h) > 1.0 ? ceil(span / h) : 1.0;
        }
        if (cells <= 4.0 * (double)(n > 1 ? n : 1) && cells <= (double)(1 << 25)) break;
        h *= 1.25;
    }
    g.h = h;
    g.inv_h = 1.0 / h;
    g.ncells = 1;
    double coord_max = 0.0;
    for (int j = 0; j < gd; ++j) {
        const double span = hi[j] > lo[j] ? hi[j] - lo[j] : 1.0;
        const double c = ceil(span / h);
        g.n[j] = c > 1.0 ? (int32_t)c : 1;
        g.ncells *= g.n[j];
        coord_max = fmax(coord_max, fabs(lo[j]) + g.n[j] * h);
    }
    // slack >> rounding of floor((x - lo) * inv_h) and of the edge coordinates
    g.slack = 1e-9 * (1.0 + coord_max);
    (void)d;
    return g;
}

void GridIndex::reserve(int64_t cap_pts, int32_t d, int64_t ncells) {
    if (cap_pts > pts_cap || d != dim) {
        if (spts) hip_check(hipFree(spts), "free");
        if (sids) hip_check(hipFree(sids), "free");
        sids = nullptr;
        if (cell_of) hip_check(hipFree(cell_of), "free");
        const int64_t c = cap_pts > 0 ? cap_pts : 1;
        hip_check(hipMalloc(&spts, sizeof(double) * c * grid_stride(d)), "grid pts");
        if (grid_stride(d) == d) hip_check(hipMalloc(&sids, sizeof(int32_t) * c), "grid ids");
        hip_check(hipMalloc(&cell_of, sizeof(int32_t) * 2 * c), "grid cell_of");  // (cell, rank) pairs
        pts_cap = c;
        dim = d;
    }
    if (ncells + 1 > cells_cap) {
        if (counts) hip_check(hipFree(counts), "free");
        if (cell_start) hip_check(hipFree(cell_start), "free");
        hip_check(hipMalloc(&counts, sizeof(int32_t) * (ncells + 1)), "grid counts");
        hip_check(hipMalloc(&cell_start, sizeof(int32_t) * (ncells + 1)), "grid starts");
        cells_cap = ncells + 1;
        // every count starts at zero and each build leaves them so (k_grid_scatter counts
        // down); a build with more cells than the last one relies on this
        hip_check(hipMemset(counts, 0, sizeof(int32_t) * (size_t)cells_cap), "grid counts zero");
        // the null-stream memset is not ordered with the build's (non-blocking) stream: wait for
        // it, or k_grid_count may add to stale counts and the scatter write past the points
        hip_check(hipDeviceSynchronize(), "grid counts zero sync");
        counts_zero = true;
        scan.reserve((ncells + 1 + 2047) / 2048);  // launch_scan_excl<8> tiles
    }
}

GridIndex::~GridIndex() {
    void *ps[] = {spts, sids, cell_of, counts, cell_start};
    for (void *p : ps)
        if (p) (void)hipFree(p);
}

void GridIndex::build(const double *pts, int64_t n_upper, const int64_t *n_dev, int32_t d, const GridParams &gp,
                      hipStream_t stream, const SpreadOut *spread, const QueryBucketing *qb) {
    if (gp.ncells >= (int64_t(1) << 31) - 1) throw Error{5, "grid too large"};
    reserve(n_upper, d, gp.ncells);
    g = gp;
    n_max = n_upper;
    if (!counts_zero) hip_check(hipMemsetAsync(counts, 0, sizeof(int32_t) * (size_t)cells_cap, stream), "grid memset");
    counts_zero = false;
    // two queries per bucketing thread, those workgroups after the points' (config 2's build
    // 28.2 us with four, 27.0 with two, 27.1 with one; leading workgroups no different; round 3)
    constexpr int kQpt = 2;
    const int qpb = 256 * kQpt;
    const unsigned qblocks = qb ? (unsigned)((qb->nq + qpb - 1) / qpb) : 0u;
    if (n_upper > 0 || qblocks > 0) {
        const unsigned blocks = (unsigned)((n_upper + 255) / 256);
        const QueryBucketing q = qb ? *qb : QueryBucketing{};
        const SpreadOut sp = spread ? *spread : SpreadOut{};
        auto go = [&](auto kern) {
            hipLaunchKernelGGL(kern, dim3(blocks + qblocks), dim3(256), 0, stream, g, pts, d, n_upper, n_dev, cell_of,
                               counts, sp, blocks, 0u, q);
        };
        if (spread) go(k_grid_count<true, kQpt>);
        else go(k_grid_count<false, kQpt>);
        hip_check(hipGetLastError(), "k_grid_count");
    }
    // the scan leaves every count zero again, so the next build needs no memset
    launch_scan_excl(scan, reinterpret_cast<const uint32_t *>(counts), reinterpret_cast<uint32_t *>(cell_start),
                     g.ncells + 1, stream, ZeroCounts{reinterpret_cast<uint32_t *>(counts)});
    if (n_upper > 0) {
        const unsigned blocks = (unsigned)((n_upper + 255) / 256);
        // the state dims the engines use get a compile-time row (the run-time copy loop waited
        // on each coordinate)
        const SpreadOut sp = spread ? *spread : SpreadOut{};
        const int32_t n_part = spread ? (int32_t)blocks : 0;
        auto go = [&](auto kern) {
            hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, stream, pts, d, n_upper, n_dev, cell_of, cell_start,
                               spts, sids, sp, n_part);
        };
        const int dd = d;
        if (spread) {
            if (dd == 3) go(k_grid_scatter<true, 3>);
            else if (dd == 7) go(k_grid_scatter<true, 7>);
            else if (dd == 15) go(k_grid_scatter<true, 15>);
            else go(k_grid_scatter<true, 0>);
        } else {
            if (dd == 3) go(k_grid_scatter<false, 3>);
            else if (dd == 7) go(k_grid_scatter<false, 7>);
            else if (dd == 15) go(k_grid_scatter<false, 15>);
            else go(k_grid_scatter<false, 0>);
        }
        hip_check(hipGetLastError(), "k_grid_scatter");
    }
    counts_zero = true;  // the scan zeroed every count it read
}

GridDev GridIndex::dev() const {
    GridDev G;
    G.g = g;
    G.cell_start = cell_start;
    G.pts = spts;
    G.ids = sids;
    G.stride = grid_stride(dim);
    G.removed = nullptr;
    G.stats = nullptr;
    return G;
}

__global__ __launch_bounds__(256) void k_bbox(const double *__restrict__ pts, int64_t n, int32_t d,
                                              double *__restrict__ out) {
    __shared__ double slo[256], shi[256];
    const int j = blockIdx.x;
    double lo = __builtin_huge_val(), hi = -__builtin_huge_val();
    for (int64_t i = threadIdx.x; i < n; i += 256) {
        const double v = pts[i * d + j];
        lo = fmin(lo, v);
        hi = fmax(hi, v);
    }
    slo[threadIdx.x] = lo;
    shi[threadIdx.x] = hi;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (threadIdx.x < s) {
            slo[threadIdx.x] = fmin(slo[threadIdx.x], slo[threadIdx.x + s]);
            shi[threadIdx.x] = fmax(shi[threadIdx.x], shi[threadIdx.x + s]);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        out[2 * j] = slo[0];
        out[2 * j + 1] = shi[0];
    }
}

void launch_bbox(const double *pts, int64_t n, int32_t d, double *d_out, hipStream_t stream) {
    hipLaunchKernelGGL(k_bbox, dim3((unsigned)d), dim3(256), 0, stream, pts, n, d, d_out);
    hip_check(hipGetLastError(), "k_bbox");
}

double expected_nn_distance(int32_t d, const double *lo, const double *hi, int64_t n) {
    double log_v = 0.0;
    int32_t de = 0;
    for (int j = 0; j < d; ++j)
        if (hi[j] > lo[j]) {
            log_v += log(hi[j] - lo[j]);
            ++de;
        }
    if (de == 0 || n < 1) return 0.0;
    const double log_ball = 0.5 * de * log(M_PI) - lgamma(0.5 * de + 1.0);  // unit de-ball volume
    return exp((log_v - log((double)n) - log_ball) / de);
}

int32_t choose_grid_dims(int32_t d, const double *lohi, int32_t dims[3]) {
    int32_t order[16];
    for (int j = 0; j < d; ++j) order[j] = j;
    auto ext = [&](int j) { return lohi[2 * j + 1] - lohi[2 * j]; };
    for (int a = 0; a < d; ++a)
        for (int b = a + 1; b < d; ++b)
            if (ext(order[b]) > ext(order[a])) std::swap(order[a], order[b]);
    const double top = ext(order[0]);
    int32_t gd = 0;
    for (int i = 0; i < d && gd < 3; ++i)
        if (ext(order[i]) >= 0.25 * top && ext(order[i]) > 0) dims[gd++] = order[i];
    if (gd == 0) dims[gd++] = 0;
    std::sort(dims, dims + gd);
    return gd;
}

// 1-NN with kGroup lanes per query: the lanes of a group split the cells of each ring (the
// (2r+1)^gd block, interior cells skipped), keep a private best, and merge it with
// (d2, id) order by xor-shuffles before the ring bound test, which is group-uniform.
// Sixteen times more waves than k_grid_knn, so the dependent cell_start -> point loads
// are hidden by occupancy instead of exposed one query per lane.
// kFirst = the ring the walk starts at: with kFirst = 1 the centre cell and ring 1 (the 3^gd
// block) are one pass, so the group spends one dependent cell -> point load chain less per
// query (ring 0 alone keeps 15 of 16 lanes idle and seldom settles the query).
// One query qi for the kGroup lanes of a group (sub = lane in the group; group-uniform call).
template <int D, int kGroup, int kFirst>
__device__ __forceinline__ void nn1_group_query(const GridDev &G, int32_t d, const double *__restrict__ q, int64_t qi,
                                                int sub, int32_t *__restrict__ out_ids, double *__restrict__ out_d2) {
    constexpr int DD = D > 0 ? D : 16;
    const GridParams &g = G.g;
    const int dim = D > 0 ? D : d;
    double qq[DD];
#pragma unroll
    for (int i = 0; i < DD; ++i) qq[i] = i < dim ? q[qi * dim + i] : 0.0;
    double qg[3] = {0, 0, 0};
    int cq[3] = {0, 0, 0};
    for (int j = 0; j < g.gd; ++j) {
        const double x = q[qi * dim + g.dims[j]];
        qg[j] = x;
        cq[j] = cell_coord(x, g.lo[j], g.inv_h, g.n[j]);
    }
    double bd = __builtin_huge_val();
    int32_t bi = -1;
    uint32_t n_pts = 0, n_cells = 0;
    for (int r = kFirst;; ++r) {
        const int side = 2 * r + 1;
        const int cube = g.gd == 3 ? side * side * side : (g.gd == 2 ? side * side : side);
        for (int c = sub; c < cube; c += kGroup) {
            int o[3] = {0, 0, 0}, rest = c;
            for (int j = g.gd - 1; j >= 0; --j) {
                o[j] = rest % side - r;
                rest /= side;
            }
            const int cheb = max(abs(o[0]), max(abs(o[1]), abs(o[2])));
            if (cheb != r && r != kFirst) continue;  // interior: visited in an earlier ring
            int cc[3];
            bool inside = true;
            for (int j = 0; j < 3; ++j) {
                cc[j] = cq[j] + o[j];
                inside = inside && cc[j] >= 0 && cc[j] < g.n[j];
            }
            if (!inside) continue;
            if (r > 0) {
                // skip a cell whose box is farther than the best so far: lb2 sums the
                // (slack-reduced) gaps along the grid dims; border cells are open outward
                double lb2 = 0.0;
                for (int j = 0; j < g.gd; ++j) {
                    const double clo = cc[j] == 0 ? -__builtin_huge_val() : g.lo[j] + (double)cc[j] * g.h;
                    const double chi = cc[j] == g.n[j] - 1 ? __builtin_huge_val() : g.lo[j] + (double)(cc[j] + 1) * g.h;
                    const double gap = fmax(fmax(clo - qg[j], qg[j] - chi), 0.0) - g.slack;
                    if (gap > 0.0) lb2 += gap * gap;
                }
                // the 1e-12 shrink covers the different summation order of FLANN's distance
                if (lb2 * (1.0 - 1e-12) > bd) continue;
            }
            const int32_t cell = (cc[0] * g.n[1] + cc[1]) * g.n[2] + cc[2];
            const int32_t s = G.cell_start[cell], e = G.cell_start[cell + 1];
            ++n_cells;
            n_pts += (uint32_t)(e - s);
            for (int32_t p = s; p < e; ++p) {
                const double *rec = G.pts + (int64_t)p * (D > 0 ? grid_stride(D) : G.stride);
                const double dd = D > 0 ? flann_l2<DD>(qq, rec) : flann_l2_dyn(qq, rec, dim);
                const int32_t id = grid_id<D>(G, rec, dim, p);
                if (G.removed && G.removed[id - 1]) continue;
                if (nn_better(dd, id, bd, bi)) {
                    bd = dd;
                    bi = id;
                }
            }
        }
#pragma unroll
        for (int off = kGroup / 2; off > 0; off >>= 1) {
            const double od = __shfl_xor(bd, off, kGroup);
            const int32_t oi = __shfl_xor(bi, off, kGroup);
            if (nn_better(od, oi, bd, bi)) {
                bd = od;
                bi = oi;
            }
        }
        const double lb = ring_bound(g, qg, cq, r);
        if (lb < 0.0) break;  // every cell visited
        if (lb * lb > bd) break;
    }
    if (G.stats) {
#pragma unroll
        for (int off = kGroup / 2; off > 0; off >>= 1) {
            n_pts += __shfl_xor(n_pts, off, kGroup);
            n_cells += __shfl_xor(n_cells, off, kGroup);
        }
        if (sub == 0) {
            atomicAdd(G.stats + 0, (unsigned long long)n_pts);
            atomicAdd(G.stats + 1, (unsigned long long)n_cells);
        }
    }
    if (sub == 0) {
        out_ids[qi] = bi;
        out_d2[qi] = bd;
    }
}

template <int D, int kGroup, int kFirst>
__global__ __launch_bounds__(256) void k_grid_nn1_group(GridDev G, int32_t d, const double *__restrict__ q,
                                                        int64_t nq, int32_t *__restrict__ out_ids,
                                                        double *__restrict__ out_d2) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t slot = t / kGroup;
    if (slot >= nq) return;  // whole groups leave together (nq is per group)
    nn1_group_query<D, kGroup, kFirst>(G, d, q, slot, (int)(t % kGroup), out_ids, out_d2);
}

// Group primitives for the run kernels: a group is kGroup aligned lanes of a wave.  A 16-lane
// group is one DPP row, so its scans and reductions are row-local DPP moves (VALU, no LDS
// round trip: row_shr for the scan, row_ror for the all-reduce); wider groups use shuffles.
template <int kGroup>
__device__ __forceinline__ int32_t grp_incl_scan(int32_t v, int sub) {
    if constexpr (kGroup == 16) {
        (void)sub;
        v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);  // row_shr:1 (0 past the row start)
        v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);  // row_shr:2
        v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);  // row_shr:4
        v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);  // row_shr:8
        return v;
    } else {
#pragma unroll
        for (int off = 1; off < kGroup; off <<= 1) {
            const int32_t o = __shfl_up(v, off, kGroup);
            if (sub >= off) v += o;
        }
        return v;
    }
}

template <int kGroup>
__device__ __forceinline__ int32_t grp_last(int32_t v) {
    if constexpr (kGroup == 16) return __builtin_amdgcn_update_dpp(0, v, 0x15F, 0xf, 0xf, false);  // row_newbcast:15
    else return __shfl(v, kGroup - 1, kGroup);
}

template <int CTRL>
__device__ __forceinline__ void dpp_merge_step(double &bd, int32_t &bi) {
    const int32_t lo = __builtin_amdgcn_update_dpp(0, __double2loint(bd), CTRL, 0xf, 0xf, false);
    const int32_t hi = __builtin_amdgcn_update_dpp(0, __double2hiint(bd), CTRL, 0xf, 0xf, false);
    const int32_t oi = __builtin_amdgcn_update_dpp(0, bi, CTRL, 0xf, 0xf, false);
    const double od = __hiloint2double(hi, lo);
    if (nn_better(od, oi, bd, bi)) {
        bd = od;
        bi = oi;
    }
}

// every lane of the group ends with the group's best (d2, id) in (d2, id) order
template <int kGroup>
__device__ __forceinline__ void grp_merge_best(double &bd, int32_t &bi) {
    if constexpr (kGroup == 16) {
        // rotations within the row: after ror 8, 4, 2, 1 each lane has seen all 16
        dpp_merge_step<0x128>(bd, bi);
        dpp_merge_step<0x124>(bd, bi);
        dpp_merge_step<0x122>(bd, bi);
        dpp_merge_step<0x121>(bd, bi);
    } else {
#pragma unroll
        for (int off = kGroup / 2; off > 0; off >>= 1) {
            const double od = __shfl_xor(bd, off, kGroup);
            const int32_t oi = __shfl_xor(bi, off, kGroup);
            if (nn_better(od, oi, bd, bi)) {
                bd = od;
                bi = oi;
            }
        }
    }
}

// small non-negative integer quotient by a run-time divisor through f32 (exact while
// a * side < 2^20: (a + 0.5) / side is at least 0.5 / side from an integer)
__device__ __forceinline__ int small_div(int a, int side, float inv_side) {
    (void)side;
    return (int)(((float)a + 0.5f) * inv_side);
}

// 1-NN over runs of cells.  Cells are laid out with the last grid dim contiguous, so the
// cells of a pass that share their other coordinates form one run whose points are one
// contiguous range [cell_start[first], cell_start[last + 1]):
//   * first pass (r = 1, the 3^GD block): 3^(GD-1) runs of 3 cells, one step of the group;
//   * ring r >= 2: border columns give a full run of 2r+1 cells, interior columns only the
//     two cells at +-r (two single-cell runs).
// Each lane of the group takes run slots, prunes a run whose box is farther than its best so
// far (not in the first pass: nothing is known yet), and loads the run's [start, end).  A scan
// of the run lengths then spreads the pass's points evenly over the group (a per-lane binary
// search over the scanned prefixes maps a flat index to its run; the lane of the group's
// longest run no longer sets every wave's time).  GD (the grid dims) is a template argument,
// so every per-dim loop is unrolled and the query's grid coordinates come from registers.
// The merge is in (d2, id) order and the stop test is the ring bound, so the result is the
// brute-force result bit for bit.
template <int D, int GD, int kGroup, int kPts, int kHeadScreen = 0>
__device__ __forceinline__ void nn1_runs_query(const GridDev &G, const double *__restrict__ q, int64_t qi, int sub,
                                               int32_t *__restrict__ out_ids, double *__restrict__ out_d2) {
    const GridParams &g = G.g;
    double qq[D];
#pragma unroll
    for (int i = 0; i < D; ++i) qq[i] = q[qi * D + i];
    double qg[3] = {0, 0, 0};
    int cq[3] = {0, 0, 0};
    constexpr int zl = GD - 1;  // the run (contiguous) dim
#pragma unroll
    for (int j = 0; j < GD; ++j) {
        double x = qq[0];
#pragma unroll
        for (int i = 1; i < D; ++i)
            if (i == g.dims[j]) x = qq[i];
        qg[j] = x;
        cq[j] = cell_coord(x, g.lo[j], g.inv_h, g.n[j]);
    }
    // the lane's base address for ds_bpermute inside its group
    const int grp_base = (int)((threadIdx.x & 63) & ~(kGroup - 1)) << 2;
    double bd = __builtin_huge_val();
    int32_t bi = -1;
    uint32_t n_pts = 0, n_cells = 0;
    // box gap of cells [c0, c1] along grid dim j (border cells open outward), minus the slack
    auto gap = [&](int j, int c0, int c1) {
        const double clo = c0 == 0 ? -__builtin_huge_val() : g.lo[j] + (double)c0 * g.h;
        const double chi = c1 == g.n[j] - 1 ? __builtin_huge_val() : g.lo[j] + (double)(c1 + 1) * g.h;
        const double v = fmax(fmax(clo - qg[j], qg[j] - chi), 0.0) - g.slack;
        return v > 0.0 ? v * v : 0.0;
    };
    for (int r = 1;; ++r) {
        const int side = 2 * r + 1;
        const float inv_side = 1.0f / (float)side, inv_in = r > 1 ? 1.0f / (float)(side - 2) : 0.f;
        const int ncol = GD == 3 ? side * side : (GD == 2 ? side : 1);
        // run slots: one per column (the full run of a border column, or of every column in
        // the first pass; an interior column's -r cell), then one per interior column for its
        // +r cell
        const int nint = r == 1 ? 0 : (GD == 3 ? (side - 2) * (side - 2) : (GD == 2 ? side - 2 : 1));
        const int nslot = ncol + nint;
        for (int base = 0; base < nslot; base += kGroup) {
            const int u = base + sub;
            int32_t s = 0, len = 0;
            if (u < nslot) {
                const int part = u >= ncol ? 1 : 0;
                int o0 = 0, o1 = 0;
                if (!part) {
                    if constexpr (GD == 3) {
                        const int a = small_div(u, side, inv_side);
                        o0 = a - r;
                        o1 = u - a * side - r;
                    } else if constexpr (GD == 2) {
                        o0 = u - r;
                    }
                } else {
                    const int v = u - ncol;  // interior column v
                    if constexpr (GD == 3) {
                        const int a = small_div(v, side - 2, inv_in);
                        o0 = a + 1 - r;
                        o1 = v - a * (side - 2) + 1 - r;
                    } else if constexpr (GD == 2) {
                        o0 = v + 1 - r;
                    }
                }
                const bool border = GD == 3 ? (abs(o0) == r || abs(o1) == r) : (GD == 2 ? abs(o0) == r : false);
                const bool full = r == 1 || border;
                int z0 = cq[zl] + (full ? -r : (part ? r : -r));
                int z1 = cq[zl] + (full ? r : (part ? r : -r));
                z0 = z0 < 0 ? 0 : z0;
                z1 = z1 > g.n[zl] - 1 ? g.n[zl] - 1 : z1;
                bool ok = z0 <= z1;
                int c0 = 0, c1 = 0;
                if constexpr (GD >= 2) {
                    c0 = cq[0] + o0;
                    ok = ok && c0 >= 0 && c0 < g.n[0];
                }
                if constexpr (GD == 3) {
                    c1 = cq[1] + o1;
                    ok = ok && c1 >= 0 && c1 < g.n[1];
                }
                if (ok && r > 1) {
                    double lb2 = gap(zl, z0, z1);
                    if constexpr (GD >= 2) lb2 += gap(0, c0, c0);
                    if constexpr (GD == 3) lb2 += gap(1, c1, c1);
                    // the 1e-12 shrink covers the different summation order of FLANN's distance
                    ok = lb2 * (1.0 - 1e-12) <= bd;
                }
                if (ok) {
                    const int32_t cell0 = GD == 3 ? (c0 * g.n[1] + c1) * g.n[2] + z0 : (GD == 2 ? c0 * g.n[1] + z0 : z0);
                    s = G.cell_start[cell0];
                    len = G.cell_start[cell0 + (z1 - z0) + 1] - s;
                    n_cells += (uint32_t)(z1 - z0 + 1);
                }
            }
            const int32_t incl = grp_incl_scan<kGroup>(len, sub);
            const int32_t total = grp_last<kGroup>(incl);
            const int32_t shift = s - (incl - len);  // point index = shift[run] + flat index
            for (int32_t t = 0; t < total; t += kPts * kGroup) {
                int32_t p[kPts];
#pragma unroll
                for (int h = 0; h < kPts; ++h) {
                    const int32_t idx = t + h * kGroup + sub;
                    // run of idx: the first lane whose inclusive prefix exceeds it
                    int lo = 0, hi = kGroup - 1;
#pragma unroll
                    for (int step = kGroup; step > 1; step >>= 1) {
                        const int mid = (lo + hi) >> 1;
                        const int32_t v = __builtin_amdgcn_ds_bpermute(grp_base + (mid << 2), incl);
                        if (v > idx) hi = mid;
                        else lo = mid + 1;
                    }
                    // every lane of the group runs the permute (a lane past the end still
                    // serves as a source: ds_bpermute reads nothing from inactive lanes)
                    const int32_t sh = __builtin_amdgcn_ds_bpermute(grp_base + (lo << 2), shift);
                    p[h] = idx < total ? sh + idx : -1;
                }
                double dd[kPts];
                int32_t id[kPts];
                bool skip[kPts];
                if constexpr (kHeadScreen > 0 && D >= 8) {
                    // long records (the snake's 120 B): each point's first four dims first, the
                    // rest and its id only when that head sum does not exceed the lane's best
                    // (the full sum is at least the head, so a skipped point cannot be better)
                    double head[kPts];
#pragma unroll
                    for (int h = 0; h < kPts; ++h) {
                        head[h] = 0.0;
                        if (p[h] >= 0) head[h] = flann_l2_head<kHeadScreen>(qq, G.pts + (int64_t)p[h] * grid_stride(D));
                    }
#pragma unroll
                    for (int h = 0; h < kPts; ++h) {
                        skip[h] = p[h] >= 0 && head[h] > bd;
                        if (p[h] >= 0 && !skip[h]) {
                            const double *rec = G.pts + (int64_t)p[h] * grid_stride(D);
                            dd[h] = flann_l2_rest<D, kHeadScreen>(qq, rec, head[h]);
                            id[h] = grid_id<D>(G, rec, D, p[h]);
                        }
                    }
                } else {
#pragma unroll
                    for (int h = 0; h < kPts; ++h) {
                        skip[h] = false;
                        if (p[h] >= 0) {
                            const double *rec = G.pts + (int64_t)p[h] * grid_stride(D);
                            dd[h] = flann_l2<D>(qq, rec);
                            id[h] = grid_id<D>(G, rec, D, p[h]);
                        }
                    }
                }
#pragma unroll
                for (int h = 0; h < kPts; ++h) {
                    if (p[h] < 0) continue;
                    ++n_pts;
                    if (skip[h]) continue;
                    if (G.removed && G.removed[id[h] - 1]) continue;
                    if (nn_better(dd[h], id[h], bd, bi)) {
                        bd = dd[h];
                        bi = id[h];
                    }
                }
            }
        }
        grp_merge_best<kGroup>(bd, bi);
        // lower bound on the distance (along the grid dims) from q to any cell outside the
        // ring-r block; stop once it exceeds the best (or every cell has been visited)
        double lb = __builtin_huge_val();
        bool more = false;
#pragma unroll
        for (int j = 0; j < GD; ++j) {
            if (cq[j] - r > 0) {
                more = true;
                lb = fmin(lb, qg[j] - (g.lo[j] + (double)(cq[j] - r) * g.h));
            }
            if (cq[j] + r + 1 < g.n[j]) {
                more = true;
                lb = fmin(lb, g.lo[j] + (double)(cq[j] + r + 1) * g.h - qg[j]);
            }
        }
        if (!more) break;  // every cell visited
        lb -= g.slack;
        lb = lb > 0.0 ? lb : 0.0;
        if (lb * lb > bd) break;
    }
    if (G.stats) {
#pragma unroll
        for (int off = kGroup / 2; off > 0; off >>= 1) {
            n_pts += __shfl_xor(n_pts, off, kGroup);
            n_cells += __shfl_xor(n_cells, off, kGroup);
        }
        if (sub == 0) {
            atomicAdd(G.stats + 0, (unsigned long long)n_pts);
            atomicAdd(G.stats + 1, (unsigned long long)n_cells);
        }
    }
    if (sub == 0) {
        out_ids[qi] = bi;
        out_d2[qi] = bd;
    }
}

// kPts: points per lane per step (loads in flight together)
template <int D, int GD, int kGroup, int kPts>
__global__ __launch_bounds__(256) void k_grid_nn1_runs(GridDev G, const double *__restrict__ q, int64_t nq,
                                                       int32_t *__restrict__ out_ids, double *__restrict__ out_d2) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t slot = t / kGroup;
    if (slot >= nq) return;  // whole groups leave together (nq is per group)
    nn1_runs_query<D, GD, kGroup, kPts, (D >= 8 ? 2 : 0)>(G, q, slot, (int)(t % kGroup), out_ids, out_d2);
}

// XCD-aware variant.  The points are in cell order, x-major, so the cells of an x-slab
// [s n0 / 8, (s + 1) n0 / 8) are one contiguous slice of the point array.  Workgroups are
// dealt round-robin over the 8 XCDs, so workgroup b and b + 8 share an XCD (and its 4 MiB
// L2): workgroup b serves slab b % 8 and scans the chunk b / 8 of kSlabChunk queries for
// the ones whose cell lies in its slab.  Each XCD's L2 then holds about an eighth of the
// tree (plus the neighbouring cells), instead of every XCD streaming the whole point array
// through its L2.  Queries whose walk leaves the slab are still exact (placement only
// changes speed).  About 3/4 of the groups have a query per chunk (the chunk holds 6 NG
// queries for NG groups; more than NG of one slab take a second turn).  The engine's
// bucket-sorted launch (k_grid_nn1_runs_sorted) replaces it when the queries come bucketed.
template <int D, int GD, int kGroup, int kPts>
__global__ __launch_bounds__(256) void k_grid_nn1_runs_xcd(GridDev G, const double *__restrict__ q, int64_t nq,
                                                           int32_t *__restrict__ out_ids,
                                                           double *__restrict__ out_d2) {
    constexpr int NG = 256 / kGroup;
    constexpr int kChunk = 6 * NG;  // <= 96 queries: two waves scan them
    __shared__ int32_t s_idx[kChunk];
    __shared__ int32_t s_cnt[2];
    const int slab = blockIdx.x & 7;
    const int64_t base = (int64_t)(blockIdx.x >> 3) * kChunk;
    const GridParams &g = G.g;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    bool mine = false;
    if (threadIdx.x < kChunk && base + threadIdx.x < nq) {
        const double x = q[(base + threadIdx.x) * D + g.dims[0]];
        const int cx = cell_coord(x, g.lo[0], g.inv_h, g.n[0]);
        mine = (cx * 8) / g.n[0] == slab;
    }
    const uint64_t m = __ballot(mine);
    if (wave < 2 && lane == 0) s_cnt[wave] = (int32_t)__popcll(m);
    __syncthreads();
    if (mine) s_idx[(wave ? s_cnt[0] : 0) + (int)__popcll(m & ((1ull << lane) - 1ull))] = (int32_t)(base + threadIdx.x);
    __syncthreads();
    const int total = s_cnt[0] + (kChunk > 64 ? s_cnt[1] : 0);
    const int grp = threadIdx.x / kGroup, sub = threadIdx.x % kGroup;
    for (int i = grp; i < total; i += NG)
        nn1_runs_query<D, GD, kGroup, kPts, (D >= 8 ? 2 : 0)>(G, q, s_idx[i], sub, out_ids, out_d2);
}

// Bucket-sorted 1-NN (QueryOrder): workgroup b runs on XCD b % 8 and takes slice b % 8,
// chunk b / 8 of the bucket-major query order; a query's index comes from its bucket's list.
template <int D, int GD, int kGroup, int kPts, int kHS>
__global__ __launch_bounds__(256) void k_grid_nn1_runs_sorted(GridDev G, const double *__restrict__ q, int64_t nq,
                                                              QueryOrder o, int32_t *__restrict__ out_ids,
                                                              double *__restrict__ out_d2) {
    __shared__ int32_t s_pre[kQueryBuckets + 1];
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        int32_t incl = lane < o.nb ? o.count[lane * kQCountStride] : 0;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int32_t v = __shfl_up(incl, off);
            if (lane >= off) incl += v;
        }
        if (lane < o.nb) s_pre[lane + 1] = incl;
        if (lane == 0) s_pre[0] = 0;
    }
    __syncthreads();
    constexpr int QPW = 256 / kGroup;  // queries per workgroup
    const int64_t per_xcd = (int64_t)(gridDim.x >> 3);  // gridDim.x is a multiple of 8
    const int64_t wg = (int64_t)(blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
    const int64_t pos = wg * QPW + threadIdx.x / kGroup;
    if (pos >= nq) return;  // whole groups leave together
    // bucket of pos: binary search over the prefix (nb <= 32: five LDS reads)
    int lo = 0, hi = o.nb - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (s_pre[mid] <= pos) lo = mid;
        else hi = mid - 1;
    }
    const int64_t qi = o.list[(int64_t)lo * o.cap + (pos - s_pre[lo])];
    nn1_runs_query<D, GD, kGroup, kPts, kHS>(G, q, qi, (int)(threadIdx.x % kGroup), out_ids, out_d2);
}

// run-kernel group shape per state dim: 16 lanes x 1 point for d <= 7 (config 2: 54.7 us vs
// 58.2 us at 32 x 2); 32 lanes x 2 points for the snake's d = 15 (0.85 ms vs 0.90 ms at 16 x 2)
template <int D>
struct RunShape {
    static constexpr int kGroup = D >= 15 ? 32 : 16, kPts = D >= 15 ? 2 : 1;
};

template <int D, int GD>
static void grid_nn1_sorted_dg(const GridDev &G, const double *q, int64_t nq, const QueryOrder &o, int32_t *ids,
                               double *d2, hipStream_t stream) {
    constexpr int GRP = RunShape<D>::kGroup, PTS = RunShape<D>::kPts;
    constexpr int QPW = 256 / GRP;
    int64_t wgs = (nq + QPW - 1) / QPW;
    wgs = (wgs + 7) / 8 * 8;
    // records of d >= 8 (the snake's 120 B) are screened by their first two groups of four dims
    // (config 3's NN: 0.617 ms unscreened, 0.566 at one group, 0.472 at two, 0.533 at three)
    if (D >= 8)
        hipLaunchKernelGGL((k_grid_nn1_runs_sorted<D, GD, GRP, PTS, 2>), dim3((unsigned)wgs), dim3(256), 0, stream,
                           G, q, nq, o, ids, d2);
    else
        hipLaunchKernelGGL((k_grid_nn1_runs_sorted<D, GD, GRP, PTS, 0>), dim3((unsigned)wgs), dim3(256), 0, stream,
                           G, q, nq, o, ids, d2);
}

template <int D>
static void grid_nn1_sorted_d(const GridDev &G, const double *q, int64_t nq, const QueryOrder &o, int32_t *ids,
                              double *d2, hipStream_t stream) {
    switch (G.g.gd) {
        case 1: grid_nn1_sorted_dg<D, 1>(G, q, nq, o, ids, d2, stream); break;
        case 2: grid_nn1_sorted_dg<D, 2>(G, q, nq, o, ids, d2, stream); break;
        default: grid_nn1_sorted_dg<D, 3>(G, q, nq, o, ids, d2, stream); break;
    }
}

void launch_grid_nn1_sorted(const GridDev &G, int32_t d, const double *q, int64_t nq, const QueryOrder &o,
                            int32_t *ids, double *d2, hipStream_t stream) {
    if (nq <= 0) return;
    if (o.nb < 1 || o.nb > kQueryBuckets || !o.count || !o.list) throw Error{MPT_ERR_INVALID, "bad query order"};
    switch (d) {
        case 3: grid_nn1_sorted_d<3>(G, q, nq, o, ids, d2, stream); break;
        case 7: grid_nn1_sorted_d<7>(G, q, nq, o, ids, d2, stream); break;
        case 15: grid_nn1_sorted_d<15>(G, q, nq, o, ids, d2, stream); break;
        default: throw Error{MPT_ERR_INVALID, "sorted 1-NN: d must be 3, 7 or 15"};
    }
    hip_check(hipGetLastError(), "k_grid_nn1_runs_sorted launch");
}

// unsorted run-kernel launch; for d = 15 the XCD-slab variant (the snake's 12 MB of points are
// three L2s' worth, NN 0.85 -> 0.72 ms; config 2's tree gains less than the idle groups cost,
// 54 -> 65 us)
template <int D, int GD>
static void grid_nn1_runs_dg(const GridDev &G, const double *q, int64_t nq, int32_t *ids, double *d2,
                             hipStream_t stream) {
    constexpr int GRP = RunShape<D>::kGroup, PTS = RunShape<D>::kPts;
    if (D >= 15)
        hipLaunchKernelGGL((k_grid_nn1_runs_xcd<D, GD, GRP, PTS>),
                           dim3((unsigned)(((nq + 6 * (256 / GRP) - 1) / (6 * (256 / GRP))) * 8)), dim3(256), 0,
                           stream, G, q, nq, ids, d2);
    else
        hipLaunchKernelGGL((k_grid_nn1_runs<D, GD, GRP, PTS>), dim3((unsigned)((nq * GRP + 255) / 256)), dim3(256), 0,
                           stream, G, q, nq, ids, d2);
}

template <int D>
static void grid_nn1_runs_d(const GridDev &G, const double *q, int64_t nq, int32_t *ids, double *d2,
                            hipStream_t stream) {
    switch (G.g.gd) {
        case 1: grid_nn1_runs_dg<D, 1>(G, q, nq, ids, d2, stream); break;
        case 2: grid_nn1_runs_dg<D, 2>(G, q, nq, ids, d2, stream); break;
        default: grid_nn1_runs_dg<D, 3>(G, q, nq, ids, d2, stream); break;
    }
}

template <int D>
static void grid_knn_d(const GridDev &G, int32_t d, const double *q, int64_t nq, int32_t k, int32_t *ids, double *d2,
                       hipStream_t stream) {
    const dim3 grid((unsigned)((nq + 255) / 256));
    if constexpr (D > 0) {
        if (k == 1) {  // the cell-run kernel for the engines' state dims
            grid_nn1_runs_d<D>(G, q, nq, ids, d2, stream);
            return;
        }
    }
    if (k == 1) {
        // any other d: 32 lanes per query and rings 0 + 1 as the first pass (the 27 cells of the
        // 3^3 block in one step): 12 % faster than 16 lanes from ring 0 on config 2
        hipLaunchKernelGGL((k_grid_nn1_group<D, 32, 1>), dim3((unsigned)((nq * 32 + 255) / 256)), dim3(256), 0, stream,
                           G, d, q, nq, ids, d2);
    } else if (k <= 16) {
        hipLaunchKernelGGL((k_grid_knn<D, 16>), grid, dim3(256), 0, stream, G, d, q, nq, k, ids, d2);
    } else {
        hipLaunchKernelGGL((k_grid_knn<D, 32>), grid, dim3(256), 0, stream, G, d, q, nq, k, ids, d2);
    }
}

void launch_grid_knn(const GridDev &G, int32_t d, const double *q, int64_t nq, int32_t k, int32_t *ids, double *d2,
                     hipStream_t stream) {
    if (nq <= 0) return;
    switch (d) {
        case 3: grid_knn_d<3>(G, d, q, nq, k, ids, d2, stream); break;
        case 7: grid_knn_d<7>(G, d, q, nq, k, ids, d2, stream); break;
        case 15: grid_knn_d<15>(G, d, q, nq, k, ids, d2, stream); break;
        default: grid_knn_d<0>(G, d, q, nq, k, ids, d2, stream); break;
    }
    hip_check(hipGetLastError(), "k_grid_knn launch");
}


}  // namespace mpt
