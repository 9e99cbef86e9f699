// grid_nn.h -- device grid index for exact NN (see grid_nn.hip).
#pragma once
#include "mpt_internal.h"

namespace mpt {

struct GridParams {
    int32_t gd;       // number of grid dims (1..3)
    int32_t dims[3];  // state dims the grid covers
    double lo[3];     // grid origin per grid dim
    double h, inv_h;  // cubic cell side
    double slack;     // subtracted from ring bounds (covers cell-assignment rounding)
    int32_t n[3];     // cells per grid dim (1 for unused dims)
    int64_t ncells;
};

struct GridDev {
    GridParams g;
    const int32_t *cell_start;  // [ncells + 1]
    const double *pts;          // [n][stride] in cell order: coordinates (then the id, if padded)
    const int32_t *ids;         // 1-based ids in cell order, or nullptr: the id is in each record's pad
    int32_t stride;             // doubles per record: d + 1 (padded, d < 8) or d
    const uint8_t *removed;     // by original row, or nullptr
    unsigned long long *stats;  // optional [2]: points examined, cells visited (1-NN kernel)
};

// Points are stored as records of d + 1 doubles with the 1-based id in the pad (32 / 64-B
// aligned: a point and its id in one line) for d < 8; the snake's d = 15 keeps 15-double
// records and an id array (its 128-B padded records measured 1.7x slower: 0.73 -> 1.22 ms).
__host__ __device__ __forceinline__ constexpr int32_t grid_stride(int32_t d) { return d < 8 ? d + 1 : d; }
// D > 0: the layout is known at compile time; D = 0: the run-time dim d decides
template <int D>
__device__ __forceinline__ int32_t grid_id(const GridDev &G, const double *rec, int d, int64_t p) {
    if constexpr (D > 0) {
        if constexpr (D < 8) return (int32_t)__double_as_longlong(rec[D]);
        else return G.ids[p];
    } else {
        return d < 8 ? (int32_t)__double_as_longlong(rec[d]) : G.ids[p];
    }
}

// Optional by-product of an index build (the engine's MPT_NN_AUTO feedback): the live
// points' min / max over up to three state dims as order-preserving 64-bit keys, written
// to host_out[0..3) (min) and host_out[3..6) (max) -- mapped pinned memory -- by the build
// itself, so no extra pass over the nodes.  Unused dims: ~0 / 0.
struct SpreadOut {
    int32_t gd = 0;
    int32_t dims[3] = {0, 0, 0};
    unsigned long long *partial = nullptr;  // [blocks][6] per-block partials (grid build), device
    unsigned long long *host_out = nullptr; // [6], device pointer of mapped host memory
};

__host__ __device__ __forceinline__ unsigned long long order_key_u64(double x) {
    unsigned long long b;
    __builtin_memcpy(&b, &x, sizeof b);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__host__ __device__ __forceinline__ double key_value_u64(unsigned long long k) {
    const unsigned long long b = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
    double x;
    __builtin_memcpy(&x, &b, sizeof x);
    return x;
}

// h chosen for about `ppc` points per cell and at least h_min, capped at 4 cells per point
// and 2^25 cells.
GridParams make_grid_params(int32_t d, const int32_t *dims, int32_t gd, const double *lo, const double *hi, int64_t n,
                            double ppc, double h_min = 0.0);

// Expected nearest-neighbour distance of n points uniform over the box [lo, hi]^d (dims of
// zero width ignored): the radius r with n * vol(ball_r) = vol(box).  When many state dims
// lie outside the grid (the snake: 13 of 15), r is far above the ppc-sized cell, and the
// walk pays per-cell overhead for cells that never prune; the engine floors h at a fraction
// of r.
double expected_nn_distance(int32_t d, const double *lo, const double *hi, int64_t n);

// Queries bucketed by their coordinate along one state dim (the grid's first dim), written by
// extra workgroups of the index build's count launch (GridIndex::build with a QueryBucketing:
// block-aggregated atomics, so the order inside a bucket is arbitrary; the work overlaps the
// point count instead of adding a dependent step to the round).  The sorted 1-NN launch deals the bucket-major query order to
// the XCDs in eight contiguous slices of equal size: each XCD then walks an x-slab of the
// points (plus the neighbouring cells) through its own L2 instead of every XCD streaming the
// whole point array, and no workgroup idles (the slices are cut by query count, not by x).
// Results are per query and exact, so the order changes only speed.
struct QueryOrder {
    int32_t *count = nullptr;  // [nb * kQCountStride] queries per bucket; zero before the producer runs
    int32_t *list = nullptr;   // [nb][cap] query indices per bucket
    int32_t nb = 0, cap = 0;
    int32_t dim = 0;           // state dim that orders the queries
    double lo = 0.0, inv_w = 0.0;  // bucket = clamp(floor((x - lo) * inv_w), 0, nb - 1)
};
constexpr int32_t kQueryBuckets = 32;
// bucket b's count lives at count[b * kQCountStride]: one 128-B line per counter, so the
// producer's device atomics on different buckets do not serialise on one line
constexpr int32_t kQCountStride = 32;

__host__ __device__ __forceinline__ int32_t query_bucket(const QueryOrder &o, double x) {
    double b = floor((x - o.lo) * o.inv_w);
    b = b < 0.0 ? 0.0 : b;
    b = b > (double)(o.nb - 1) ? (double)(o.nb - 1) : b;
    return (int32_t)b;
}

// The engine's round start, folded into the grid count launch (one launch less per round):
// the samples generated there instead of by a k_sample launch, and k_sample's bookkeeping.
constexpr int kGenMaxDim = 16;
struct SampleGen {
    double *out = nullptr;  // [nq][d] samples written here (nullptr: the queries are given)
    uint64_t seed = 0, ext_base = 0;
    double lo[kGenMaxDim] = {}, hi[kGenMaxDim] = {};
    int64_t *n_dev = nullptr;              // [0] node count, [1] the round's starting count
    int64_t set_n = -1;                    // a pending truncation (mpt_rrt_set_size), or -1
    unsigned long long *counters = nullptr;
    uint32_t *n_live = nullptr;            // the round's live-unit count, zeroed
};

// what GridIndex::build buckets alongside its point count
struct QueryBucketing {
    const double *q = nullptr;  // [nq][d] queries (state dim d, as the points)
    int64_t nq = 0;
    QueryOrder o;
    SampleGen gen;  // gen.out: generate the queries (engine samples) instead of reading q
};

class GridIndex {
public:
    ~GridIndex();
    // Index points [0, min(n_upper, *n_dev)) of pts [.][d]; stream-ordered, no host sync.
    // spread (optional): also reduce the points' spread into spread->host_out (partial needs
    // ceil(n_upper / 256) * 6 slots).
    // qb (optional): also bucket qb->nq queries into qb->o (counts zero on entry).
    void build(const double *pts, int64_t n_upper, const int64_t *n_dev, int32_t d, const GridParams &g,
               hipStream_t stream, const SpreadOut *spread = nullptr, const QueryBucketing *qb = nullptr);
    GridDev dev() const;
    const GridParams &params() const { return g; }
    // allocate for up to cap_pts points and ncells cells now (allocation synchronises the
    // device; engines reserve their capacity once so rounds on several streams overlap)
    void reserve(int64_t cap_pts, int32_t d, int64_t ncells);

private:
    GridParams g{};
    int64_t n_max = 0, pts_cap = 0, cells_cap = 0;
    bool counts_zero = false;  // counts[] is all zero (true after every complete build)
    int32_t dim = 0;
    double *spts = nullptr;  // [cap][grid_stride(d)] records
    int32_t *sids = nullptr, *cell_of = nullptr, *counts = nullptr, *cell_start = nullptr;
    ScanState scan;  // counts -> cell_start, one launch
};

void launch_grid_knn(const GridDev &G, int32_t d, const double *q, int64_t nq, int32_t k, int32_t *ids, double *d2,
                     hipStream_t stream);

// 1-NN of the nq queries listed by o (every query in exactly one bucket), results by query
// index as launch_grid_knn with k = 1.
void launch_grid_nn1_sorted(const GridDev &G, int32_t d, const double *q, int64_t nq, const QueryOrder &o,
                            int32_t *ids, double *d2, hipStream_t stream);


// Per-dim [min, max] of pts[0, n) into d_out[2*d] (lo0, hi0, lo1, hi1, ...).
void launch_bbox(const double *pts, int64_t n, int32_t d, double *d_out, hipStream_t stream);

// Grid dims: up to three dims with the largest extents, keeping only those whose extent
// is at least a quarter of the largest (others would only add empty rings).
int32_t choose_grid_dims(int32_t d, const double *lohi, int32_t dims[3]);

}  // namespace mpt
