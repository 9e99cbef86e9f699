// point_tree.h -- packed Morton tree for exact NN over a tree snapshot (see point_tree.hip).
#pragma once
#include "mpt_internal.h"
#include "grid_nn.h"  // SpreadOut

namespace mpt {

constexpr int kPtFan = 8;        // children per node, points per leaf
constexpr int kPtMaxLevels = 10; // 8^10 points
constexpr int kPtMaxDim = 16;

struct PointTreeDev {
    int32_t d;
    int32_t n_levels;          // box levels 1..n_levels (level n_levels = the root)
    int64_t n_upper;           // layout bound: level l holds ceil(n_upper / 8^l) boxes
    const int64_t *n_dev;      // live point count (<= n_upper)
    const float *boxes;        // levels 1..n_levels back to back, each box [2d] floats: lo then hi
    const double *pts;         // [n][d], Morton order
    const int32_t *ids;        // 1-based original ids
    unsigned long long *stats; // optional [2]: points examined, boxes tested
};

// One tree of a joint build (mpt_rrt_step_many): the tree's own buffers, its points, and the
// offset of its keys / values in the shared sort buffers.
struct PtBuildJob {
    PointTreeDev T;            // as PointTree::dev() after the build
    const double *pts;         // [n_upper][d] input rows
    int64_t off;               // into the shared key / value buffers
    unsigned long long *bbox;  // the tree's box keys
    unsigned int *ticket;      // [2]: box-level ticket, bbox ticket
    struct CodePlan *plan;
    double *spts;
    int32_t *sids;
    float *boxes;
    SpreadOut sp;
};

// shared sort buffers of a joint build (owned by the caller; reserve_tree_build_jobs sizes
// them for the joined trees' capacities so later rounds never allocate)
struct JointTreeScratch {
    uint32_t *keys = nullptr, *keys_sorted = nullptr;
    int32_t *vals = nullptr, *vals_sorted = nullptr;
    int64_t cap = 0;
    void *temp = nullptr;
    size_t temp_bytes = 0;
};

// Build n trees of dim d in one launch per stage + one segmented sort.  d_jobs / h_jobs: the
// same table on the device and the host; d_offsets: [n + 1] segment starts (int32) on the
// device, total = its last entry.  Stream-ordered.
void launch_tree_build_jobs(const PtBuildJob *d_jobs, const PtBuildJob *h_jobs, int32_t n, int32_t d,
                            const int32_t *d_offsets, int64_t total, JointTreeScratch &S, hipStream_t stream);
// Size S for up to total_cap points in n_jobs segments (synchronises the device only when it
// grows: call it before staging a round, not inside one).
void reserve_tree_build_jobs(JointTreeScratch &S, int64_t total_cap, int32_t n_jobs);

class PointTree {
public:
    // the host part of build(): reserve, lay out the levels, and describe the device work as
    // a job of a joint build (launch_tree_build_jobs); dev() is valid once that has run
    PtBuildJob prepare(const double *pts, int64_t n_upper, const int64_t *n_dev, int32_t d, int64_t off,
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
