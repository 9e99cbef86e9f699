// cell_tree.h -- the engine's incremental NN index: cell-aligned buckets in a directory, an
// 8-ary box hierarchy above the directory rebuilt each round (see cell_tree.hip).
//
// Replaces FLANN_KDTreeWrapper (utilities/flannkdtreewrapper.hpp:8-125) on the RRT path:
// insertPoint (:27-40) adds points to the live index -- here a round's new points go into the
// buckets of the code cells they fall in, and only the buckets they touch change -- and
// nearest (:57-89) is the exact 1-NN in FLANN's squared-L2 order, ties to the lowest id.
#pragma once
#include "grid_nn.h"  // SpreadOut
#include "mpt_internal.h"

namespace mpt {

constexpr int kCtCap = 8;          // points per bucket (a leaf: one lane each)
constexpr int kCtMaxDim = 16;
constexpr int kCtBits = 126;       // code bits (two 64-bit words)
constexpr int kCtSeg = 8192;       // new points one round inserts (the host bounds a round's growth)
constexpr int kCtScratch = kCtSeg * (kCtCap + 1);  // a round's split elements (new + old of touched buckets)
constexpr int kCtHull = 64;        // seed points (extreme points in fixed directions)
constexpr int kCtL1Tile = 512;     // level-1 entries a workgroup groups (k_ct_lflags / k_ct_lgroup)

// the fixed code plan over the sampling ranges and the seed directions
struct CtPlan {
    double lo[kCtMaxDim], scale[kCtMaxDim];
    uint32_t qmax[kCtMaxDim];
    int32_t n;                           // code bits used (<= kCtBits)
    int8_t dim[kCtBits], bit[kCtBits];   // MSB first
    int8_t nb[kCtMaxDim];                // bits of each dim: level l (MSB first) takes the dims with nb > l
    int32_t bmax;                        // levels (the most bits of a dim)
    // seed slot h keeps the indexed point of the largest score: kind 0: hdir . (the first three
    // state dims), kind 1: -x[hdim], kind 2: +x[hdim]
    float hdir[kCtHull][3];
    int8_t hkind[kCtHull], hdim[kCtHull];
    int32_t n_hull;
    int32_t pad;
};
static_assert(sizeof(CtPlan) % 4 == 0, "the kernels copy the plan to LDS as 4-byte words");
// one quantisation step h for every dim (cubic cells in raw state units, the units of FLANN's
// L2), the smallest for which the bits sum to <= kCtBits (<= 31 a dim), widest dims split first;
// seed directions over the first `spatial` dims
CtPlan make_ct_plan(int32_t d, const double *lo, const double *hi, int32_t spatial);

// per-tree device counters
struct CtCounts {
    int32_t n_buckets;   // buckets in use (the pool)
    int32_t n_dir;       // directory entries (buckets in code order) after this round's merge
    int32_t n_seg;       // this round's touched buckets
    int32_t n_new_dir;   // this round's new directory entries
    int32_t root;        // the hierarchy's root node
    int32_t n_l2;        // this round's level-2 / level-3 node counts (k_ct_lgroup)
    int32_t n_l3;
    int32_t n_scratch;   // this round's split elements (the split segments' old + new points)
    int64_t nidx;        // points indexed (rows [0, nidx) of the node array)
    // the walk's first entries: the root's children (the root itself when it is a leaf), so a
    // query's first step tests the root's grandchildren -- one walk step fewer (k_ct_levels)
    uint32_t top[8];
    int32_t n_top;
    // the two-stack walk's first entries: the nodes [lv_first, lv_first + lv_n) of the lowest
    // level of at most 64 nodes, their boxes tested in the seeds' step (k_ct_levels)
    int32_t lv_first;
    int32_t lv_n;
    int32_t pad;
};

// What the walk reads.  The hierarchy's nodes, level after level: level 1 = one node per
// directory entry (its bucket), each higher level groups consecutive nodes of the one below into
// maximal aligned code cells of at most 8 (as buckets group points), up to one root.  A node's
// meta (the walk's stack code): bit 31 leaf, bits 28..30 count - 1, bits 0..27 a leaf's bucket or
// an inner node's first child node (its children are contiguous).
struct CellTreeDev {
    int32_t d;
    int32_t pad;
    int64_t n_bound;           // host bound of the directory size (grid sizes)
    const int64_t *n_dev;      // live node count (0: empty tree)
    const int32_t *root;       // the root node (in the tree's CtCounts)
    const uint32_t *top;       // the walk's first entries (CtCounts top / n_top)
    const int32_t *n_top;
    const int32_t *lv;         // CtCounts lv_first, lv_n (the two-stack walk's first entries)
    const uint32_t *nmeta;     // [nodes]
    const float *nbox;         // [nodes][d][2] widened float bounds: (lo, -hi) a dim
    const double *bpts;        // [buckets][kCtCap][d]
    const int32_t *bids;       // [buckets][kCtCap] 1-based ids
    const double *hull_pts;    // [kCtHull][d] seed rows, ids in hull_ids (0: empty slot)
    const int32_t *hull_ids;
    unsigned long long *stats; // optional: [0] points examined, [1] boxes tested, [3] walk steps
};

// One tree's build of a round (the joint build of many engines: one per engine).
struct CtJob {
    CellTreeDev T;
    const double *pts;         // [n_upper][d] node rows, id = row + 1
    const CtPlan *plan;
    CtCounts *cnt;
    int32_t bcap;              // bucket / directory capacity
    int32_t mb;                // host bound of this round's new points (0 after a full rebuild)
    int32_t reset;             // 1: start from an empty index (k_ct_reset), then insert rows [0, n) as new
    int32_t pad_;
    // buckets
    double *bpts;
    int32_t *bids;
    uint64_t *bcode;           // [buckets][kCtCap][2] the slots' codes (hi, lo)
    int32_t *bcnt;
    float *bbox;               // [buckets][2d]
    // The directory is the hierarchy's level 1 (node i = entry i: its start code, its bucket's
    // meta and box), double-buffered: last round's in ocode / ometa / obox (the touched buckets'
    // records updated in place), this round's written to ndir_code and the level-1 part of
    // nmeta / nbox (T's arrays, the levels above following it)
    const uint64_t *odir_code; // [n_dir][2] interval start codes
    uint32_t *ometa;
    float *obox;
    uint64_t *ndir_code;
    uint32_t *nmeta;
    float *nbox;
    uint64_t *ucode;           // [nodes][2]
    int32_t *lflag;            // [nodes] scratch: the level's group starts
    int32_t *lcount;           // [nodes / kCtL1Tile + 1] scratch: level 1's group starts a tile
    // new points: codes / rows in row order, then sorted; chunk scratch; directory positions
    uint64_t *ncode;           // [kCtSeg][2]
    int32_t *nrow;
    uint64_t *ccode;           // [kCtSeg][2]
    int32_t *crow;
    int32_t *npos;             // [kCtSeg] directory position of sorted new point j
    int32_t *nseg;             // [kCtSeg] its segment
    int4 *seg;                 // [kCtSeg] (bucket, old count, new count, split scratch offset or -1)
    int32_t *seg_pos;          // [kCtSeg] the segment's directory position
    int32_t *seg_first;        // [kCtSeg] the segment's first sorted new point
    // split scratch [kCtScratch]: merged (code, row) of each split segment, packed
    uint64_t *scode;           // [..][2]
    int32_t *srow;
    int32_t *sseg;
    int32_t *slead;            // 1: the element starts a leaf
    int32_t *srank;            // rank of a new leaf among the round's new leaves
    // new directory entries in code order: (start, bucket, directory position of the segment)
    uint64_t *edir_code;       // [kCtScratch][2]
    int32_t *edir_bk;
    int32_t *edir_pos;
    // seeds, spread, errors
    unsigned long long *hull_keys; // [kCtHull] (score key << 32 | row)
    double *hull_pts;
    int32_t *hull_ids;
    unsigned long long *ibox;  // persistent box of the indexed points (order keys) [2][kCtMaxDim]; rounds update dims 0..2 (the spread's)
    SpreadOut sp;
    unsigned long long *err;   // the engine's counters[6]: index errors (bounds the host broke)
};

class CellTree {
public:
    // reserve for up to cap points of dim d (allocates and synchronises: call before the rounds)
    void reserve(int64_t cap, int32_t d);
    // This round's job.  full: rebuild the buckets from every point now (launches on stream);
    // a full rebuild of at most kCtSeg rows instead starts from an empty index and inserts them
    // all as the round's new points (no launches here: launch_ct_jobs resets and inserts, so a
    // joint build of many young trees is one launch per stage); else the rows [nidx, n) are
    // inserted by launch_ct_jobs (at most kCtSeg of them: the caller's bound, checked on the
    // device).  lo / hi: the sampling ranges, spatial: the
    // leading state dims the seed directions span.  dev() is valid once the jobs have run.
    // grow: nodes appended since the last build (the host's bound of the new points).
    CtJob prepare(const double *pts, int64_t n_upper, const int64_t *n_dev, int32_t d, const double *lo,
                  const double *hi, int32_t spatial, bool full, int64_t grow, hipStream_t stream,
                  const SpreadOut *spread, unsigned long long *err);
    CellTreeDev dev() const { return t; }
    // the code plan for these sampling ranges, uploaded now (synchronous) unless it is the
    // current one; true when it changed (the index must then be rebuilt).  prepare() calls it;
    // calling it beforehand (mpt_rrt_set_nn) keeps the upload out of the rounds.
    bool set_plan(const double *lo, const double *hi, int32_t spatial);
    // is the code plan the one for these ranges (set_plan would change nothing)?
    bool plan_current(const double *lo, const double *hi) const {
        bool same = plan_set;
        for (int j = 0; j < dim && same; ++j) same = plan_lo[j] == lo[j] && plan_hi[j] == hi[j];
        return same;
    }
    ~CellTree();

private:
    void release();
    CellTreeDev t{};
    int64_t cap_ = 0;
    int32_t dim = 0, cur = 0, bcap = 0;
    CtPlan *plan = nullptr;
    double plan_lo[kCtMaxDim] = {}, plan_hi[kCtMaxDim] = {};
    bool plan_set = false;
    CtCounts *cnt = nullptr;
    double *bpts = nullptr;
    int32_t *bids = nullptr, *bcnt = nullptr;
    uint64_t *bcode = nullptr, *ucode = nullptr;
    float *bbox = nullptr, *nbox[2] = {nullptr, nullptr};
    uint32_t *nmeta[2] = {nullptr, nullptr};
    int32_t *lflag = nullptr, *lcount = nullptr;
    uint64_t *dir_code[2] = {nullptr, nullptr};
    uint64_t *ncode = nullptr, *ccode = nullptr, *scode = nullptr, *edir_code = nullptr;
    int32_t *nrow = nullptr, *crow = nullptr, *npos = nullptr, *nseg = nullptr, *seg_pos = nullptr, *seg_first = nullptr,
            *srow = nullptr,
            *sseg = nullptr, *slead = nullptr, *srank = nullptr, *edir_bk = nullptr, *edir_pos = nullptr;
    int4 *seg = nullptr;
    unsigned long long *hull_keys = nullptr, *ibox = nullptr;
    double *hull_pts = nullptr;
    int32_t *hull_ids = nullptr;
    // full rebuilds: every point's code and row, sorted by hipcub (two stable 64-bit passes)
    uint64_t *fhi = nullptr, *flo = nullptr, *fk0 = nullptr, *fk1 = nullptr;
    int32_t *fv0 = nullptr, *fv1 = nullptr, *fflag = nullptr, *fleaf = nullptr;
    void *ftemp = nullptr;
    size_t ftemp_bytes = 0;
    void *slab = nullptr;  // every buffer above is carved from it
};

// the round's build of n trees of dim d (stream-ordered): insert the new points, merge the new
// directory entries, rebuild the box levels, copy the seeds.  d_jobs / h_jobs: the same table
// on the device and the host (n == 1: d_jobs unused).
void launch_ct_jobs(const CtJob *d_jobs, const CtJob *h_jobs, int32_t n, int32_t d, hipStream_t stream);

// One 1-NN job per tree: nq queries at q, results to ids / d2.
struct CtNnJob {
    CellTreeDev T;
    const double *q;
    int32_t *ids;
    double *d2;
};
// jobs: a device array [n_jobs], all trees of dim d, nq queries each
// parts: 0 = every job's workgroups dealt over all eight XCDs one by one; P > 0 = each job in P
// contiguous parts, each on one XCD (k_ct_nn1_jobs); kCtJointParts: the engine's choice
constexpr int32_t kCtJointParts = 8;
void launch_ct_nn1_jobs(const CtNnJob *d_jobs, int32_t n_jobs, int32_t d, int64_t nq, hipStream_t stream,
                        int32_t parts);
// kCtJointParts when the launch's shape allows it, else 0
int32_t ct_joint_parts(int32_t n_jobs, int32_t d, int64_t nq);
void launch_ct_nn1(const CellTreeDev &T, const double *q, int64_t nq, int32_t *ids, double *d2, hipStream_t stream);

}  // namespace mpt
