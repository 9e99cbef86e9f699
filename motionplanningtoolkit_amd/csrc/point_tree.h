// point_tree.h -- packed Morton tree over a point snapshot: PRM's radius search (see point_tree.hip).
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
};

class PointTree {
public:
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
    void reserve_boxes(int64_t n_upper, int32_t d);
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

// Radius search (d2 < r2) over 3-dim keys: offsets == nullptr -> counts[qi]; else fill ids /
// d2 of query qi from offsets[qi] on (traversal order).  below_only: ids <= qi only.
void launch_tree_radius(const PointTreeDev &T, const double *q, int64_t nq, double r2, bool below_only,
                        int32_t *counts, const int64_t *offsets, int32_t *ids, double *d2, hipStream_t stream);

}  // namespace mpt
