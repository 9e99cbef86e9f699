// point_tree.h -- packed Morton tree for exact NN over a tree snapshot (see point_tree.hip).
#pragma once
#include "mpt_internal.h"
#include "grid_nn.h"  // SpreadOut

namespace mpt {

constexpr int kPtFan = 8;        // children per node, points per leaf
constexpr int kPtMaxLevels = 10; // 8^10 points
constexpr int kPtMaxDim = 16;

// Seed points of a query's search (the incremental index): the tree's extreme points in
// kPtHull directions -- the minimum and the maximum of every state dim, the rest spread over the
// spatial dims' directions.  An RRT grows from its start while samples are uniform over the
// ranges, so most queries lie far outside the tree and their nearest node sits on its hull: the
// nearest seed bounds the search from its first step, where a walk from the root finds a tight
// bound only after descending.  Any seed is an upper bound on the nearest distance, so the
// result stays exact whichever points the seeds are.
constexpr int kPtHull = 64;

struct PointTreeDev {
    int32_t d;
    int32_t n_levels;          // box levels 1..n_levels (level n_levels = the root)
    int64_t n_upper;           // layout bound: level l holds ceil(n_upper / 8^l) boxes
    const int64_t *n_dev;      // live point count (<= n_upper)
    const float *boxes;        // levels 1..n_levels back to back, each box [2d] floats: lo then hi
    const double *pts;         // [n][d], Morton order
    const int32_t *ids;        // 1-based original ids
    unsigned long long *stats; // optional [2]: points examined, boxes tested
    const double *hull_pts;    // optional [kPtHull][d]: seed points (ids in hull_ids, 0 = none)
    const int32_t *hull_ids;
};

// ---- incremental index (the engine's rounds; FLANN_KDTreeWrapper::insertPoint,
// utilities/flannkdtreewrapper.hpp:27-40, adds points to a live index instead of rebuilding it)
//
// Codes come from a plan fixed by the sampling ranges (not the live box), so a point's code
// never changes and last round's sorted order stays valid: a round sorts only its new points
// (<= kPtIncSeg, in LDS) and merges them into the sorted arrays (merge path, one pass over
// the tree), then rebuilds the boxes.  The same sort orders the round's queries by code, so
// the groups of a wave walk neighbouring paths.  A full rebuild (first round, after a
// truncation or a bulk insert, or more new points than kPtIncSeg) sorts every code with
// hipcub and runs the same merge with no old points.
constexpr int kPtIncSeg = 8192;   // new points one round merges in
constexpr int kPtIncBits = 63;    // code bits (64-bit keys)
struct IncPlan {
    double lo[kPtMaxDim], scale[kPtMaxDim];
    uint32_t qmax[kPtMaxDim];
    int32_t n;                               // code bits used
    int8_t dim[kPtIncBits], bit[kPtIncBits]; // MSB first
    // the seeds' directions: slot h keeps the point of the largest score, kind 0: hdir . (the
    // first three state dims), kind 1: -x[hdim], kind 2: +x[hdim]
    float hdir[kPtHull][3];
    int8_t hkind[kPtHull], hdim[kPtHull];
    int32_t n_hull;
    int32_t pad;
};
// the fixed plan of the ranges [lo, hi] (host): one quantisation step h for every dim, the
// smallest for which the bits sum to <= 63 (<= 31 per dim), widest dims split first; the seed
// directions over the first `spatial` dims
IncPlan make_inc_plan(int32_t d, const double *lo, const double *hi, int32_t spatial);

struct PtIncJob {
    PointTreeDev T;               // the tree after this build (T.pts / T.ids = the out arrays)
    const double *pts;            // [n_upper][d] node rows
    const IncPlan *plan;          // device
    const uint64_t *okeys;        // last build's sorted codes / ids / rows (old points)
    const int32_t *oids;
    const double *opts;
    uint64_t *keys;               // out: sorted codes, ids, rows
    int32_t *ids;
    double *spts;
    float *boxes;
    uint64_t *nkeys;              // the new points' sorted codes and rows
    int32_t *nvals;
    uint64_t *ckeys;              // scratch [kPtIncSeg]: the new points sorted by chunks of 512
    int32_t *cvals;
    int32_t *npos;                // scratch [kPtIncSeg]: the sorted new points' output places
    int64_t *nidx;                // points the last build indexed; set to n by this build
    unsigned long long *ibox;     // persistent box of the indexed points (order keys)
    unsigned long long *err;      // device error count (the engine's counters[6]): an incremental
                                  // build found more than kPtIncSeg new points (host bound broken)
    unsigned long long *hull_keys;// [kPtHull] (score key << 32 | row) of each seed slot's best point
    double *hull_pts;             // out: [kPtHull][d] the seed rows, and their ids (0: empty slot)
    int32_t *hull_ids;
    int32_t full;                 // 1: nkeys / nvals hold every point (hipcub-sorted), no old points
    SpreadOut sp;
};
// the incremental build of n trees of dim d (stream-ordered): sort, merge, box levels.
// d_jobs / h_jobs: the same table on the device and the host (n == 1: d_jobs unused)
void launch_tree_inc_jobs(const PtIncJob *d_jobs, const PtIncJob *h_jobs, int32_t n, int32_t d, hipStream_t stream);

class PointTree {
public:
    // The incremental index: the job of this round's build (launch_tree_inc_jobs), dev()
    // valid once it has run.  full: rebuild from every point (its code + sort launches are
    // issued on `stream` here); else the points past the last build's count are merged in
    // (at most kPtIncSeg of them: the caller's bound, checked on the device too).  lo / hi:
    // the sampling ranges (the code plan), spatial: the leading state dims the seed
    // directions span.
    PtIncJob prepare_inc(const double *pts, int64_t n_upper, const int64_t *n_dev, int32_t d, const double *lo,
                         const double *hi, int32_t spatial, bool full, hipStream_t stream,
                         const struct SpreadOut *spread);
    ~PointTree();
    // Index rows [0, min(n_upper, *n_dev)) of pts [.][d]: bounding box and code plan on the
    // device, 30-bit codes over all dims, radix sort, boxes bottom-up.  Stream-ordered.
    // spread (optional, grid_nn.h): also write the live points' spread over spread->dims
    // (from the build's bounding box) to spread->host_out.
    void build(const double *pts, int64_t n_upper, const int64_t *n_dev, int32_t d, hipStream_t stream,
               const struct SpreadOut *spread = nullptr);
    PointTreeDev dev() const { return t; }
    // allocate for up to n_upper points now (see GridIndex::reserve)
    void reserve(int64_t n_upper, int32_t d);
    // the same for the incremental index (prepare_inc)
    void inc_reserve(int64_t cap, int32_t d);

private:
    PointTreeDev t{};
    int64_t cap = 0, box_cap = 0;
    int32_t dim = 0;
    uint32_t *keys = nullptr, *keys_sorted = nullptr;
    int32_t *vals = nullptr, *vals_sorted = nullptr, *sids = nullptr;
    double *spts = nullptr;
    float *boxes = nullptr;
    unsigned long long *bbox = nullptr;  // [2][kPtMaxDim] order keys, then the box-build ticket
    unsigned int *ticket = nullptr;
    struct CodePlan *plan = nullptr;
    void *temp = nullptr;
    size_t temp_bytes = 0;
    void reserve_boxes(int64_t n_upper, int32_t d);
    // incremental index (prepare_inc): two sets of sorted arrays, `icur` the last build's
    int64_t icap = 0;
    int32_t idim = 0, icur = 0;
    uint64_t *ikeys[2] = {nullptr, nullptr};
    int32_t *iids[2] = {nullptr, nullptr};
    double *ipts[2] = {nullptr, nullptr};
    uint64_t *inkeys = nullptr;
    int32_t *invals = nullptr;
    unsigned long long *ihull_keys = nullptr;
    double *ihull_pts = nullptr;
    int32_t *ihull_ids = nullptr;
    uint64_t *ickeys = nullptr;
    int32_t *icvals = nullptr, *inpos = nullptr;
    int64_t *inidx = nullptr;
    unsigned long long *ibox = nullptr;
    IncPlan *iplan = nullptr;
    double iplan_lo[kPtMaxDim] = {}, iplan_hi[kPtMaxDim] = {};
    bool iplan_set = false;
    void *itemp = nullptr;
    size_t itemp_bytes = 0;
};

// box level sizes for a layout bound: level l (1-based) has ceil(n / 8^l) boxes
inline int32_t pt_levels(int64_t n) {
    int32_t L = 1;
    int64_t m = (n + kPtFan - 1) / kPtFan;
    while (m > 1) {
        m = (m + kPtFan - 1) / kPtFan;
        ++L;
    }
    return L;
}

// One 1-NN job per tree: nq queries at q, results to ids / d2 (the joint launch of many engines).
struct PtJob {
    PointTreeDev T;
    const double *q;
    int32_t *ids;
    double *d2;
};
constexpr int kXcds = 8;  // MI355X: workgroups are dealt round-robin over 8 XCDs
// jobs: a device array [n_jobs], all trees of dim d, nq queries each
void launch_tree_nn1_jobs(const PtJob *d_jobs, int32_t n_jobs, int32_t d, int64_t nq, hipStream_t stream);
void launch_tree_nn1(const PointTreeDev &T, const double *q, int64_t nq, int32_t *ids, double *d2, hipStream_t stream);
// Radius search (d2 < r2) over 3-dim keys: offsets == nullptr -> counts[qi]; else fill ids /
// d2 of query qi from offsets[qi] on (traversal order).  below_only: ids <= qi only.
void launch_tree_radius(const PointTreeDev &T, const double *q, int64_t nq, double r2, bool below_only,
                        int32_t *counts, const int64_t *offsets, int32_t *ids, double *d2, hipStream_t stream);

}  // namespace mpt
