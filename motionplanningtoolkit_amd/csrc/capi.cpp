// capi.cpp -- extern "C" boundary (include/mpt.h): handles, host<->device copies, BVH
// and cluster construction for the environment and agent meshes.
#include <algorithm>
#include <atomic>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <mutex>
#include <numeric>
#include <string>
#include <vector>

#include <memory>

#include "../../include/mpt.h"
#include "grid_nn.h"
#include "mpt_internal.h"

namespace mpt {

static thread_local std::string g_last_error;
std::string &last_error_ref() { return g_last_error; }
static int g_device = -1;
static thread_local bool g_stats_enabled = false;
static thread_local unsigned long long g_last_stats[kCollideStats] = {};
static std::atomic<int32_t> g_collide_mode{MPT_COLLIDE_SPLIT};
int32_t collide_mode() { return g_collide_mode.load(std::memory_order_relaxed); }

void hip_check(hipError_t e, const char *what) {
    if (e != hipSuccess) throw Error{MPT_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e)};
}

static void require(bool ok, const char *msg) {
    if (!ok) throw Error{MPT_ERR_INVALID, msg};
}

static void ensure_device() {
    if (g_device < 0) {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) throw Error{MPT_ERR_NO_DEVICE, "no HIP device"};
        hip_check(hipGetDevice(&g_device), "hipGetDevice");
    }
}

// Growable device buffer (per-thread workspace for the host-pointer entry points).
struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    void *get(size_t bytes) {
        if (bytes > cap) {
            if (p) hip_check(hipFree(p), "hipFree");
            p = nullptr;
            size_t c = std::max<size_t>(bytes, cap * 2);
            c = std::max<size_t>(c, 256);
            hip_check(hipMalloc(&p, c), "hipMalloc workspace");
            cap = c;
        }
        return p;
    }
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};

struct Workspace {
    DevBuf poses, pose_edge, verdict, links, q, ids, d2, scratch, offsets, stats;
    CollideScratch cs;
};
static thread_local Workspace g_ws;

}  // namespace mpt

using namespace mpt;

// ---------------------------------------------------------------- handles
struct mpt_env {
    EnvDev dev{};
    EnvTri *d_tris = nullptr;
    BvhNode *d_nodes = nullptr;
    Item *d_items = nullptr;
    uint4 *d_qitems = nullptr;
    int64_t n_tris = 0, n_nodes = 0, depth = 0;
};

struct mpt_agent {
    AgentDev dev{};
    EnvTri *d_etris = nullptr;
    double *d_tris = nullptr;
    Cluster *d_clusters = nullptr;
    int64_t n_tris = 0;
};

struct mpt_nn {
    int32_t d = 0;
    int64_t cap = 0, n = 0;
    double *d_pts = nullptr;
    uint8_t *d_removed = nullptr;
    // grid index over the current points, rebuilt lazily after appends (grid_nn.hip)
    std::unique_ptr<GridIndex> grid;
    int64_t grid_n = -1;
    double *d_bbox = nullptr;
    int32_t mode = MPT_NN_AUTO;
};

// ---------------------------------------------------------------- BVH build
namespace {

struct TriRef {
    double lo[3], hi[3], c[3];
    int64_t idx;
};

// Top-down median split on the widest centroid axis; one triangle per leaf.  Nodes are
// emitted in pre-order (left child = node + 1).  Boxes come from the exact double
// vertex bounds, widened outward to float (fcl_math.h widen_*).
int64_t build_env_bvh(std::vector<TriRef> &refs, int64_t first, int64_t n, std::vector<BvhNode> &nodes,
                      std::vector<int64_t> &order, int depth, int64_t &max_depth) {
    const int64_t id = (int64_t)nodes.size();
    nodes.push_back(BvhNode{});
    max_depth = std::max<int64_t>(max_depth, depth);
    double lo[3] = {HUGE_VAL, HUGE_VAL, HUGE_VAL}, hi[3] = {-HUGE_VAL, -HUGE_VAL, -HUGE_VAL};
    double clo[3] = {HUGE_VAL, HUGE_VAL, HUGE_VAL}, chi[3] = {-HUGE_VAL, -HUGE_VAL, -HUGE_VAL};
    for (int64_t i = first; i < first + n; ++i)
        for (int k = 0; k < 3; ++k) {
            lo[k] = std::min(lo[k], refs[i].lo[k]);
            hi[k] = std::max(hi[k], refs[i].hi[k]);
            clo[k] = std::min(clo[k], refs[i].c[k]);
            chi[k] = std::max(chi[k], refs[i].c[k]);
        }
    BvhNode nd{};
    for (int k = 0; k < 3; ++k) {
        nd.lo[k] = widen_lo(lo[k]);
        nd.hi[k] = widen_hi(hi[k]);
    }
    if (n == 1) {
        nd.a = (int32_t)order.size();
        nd.b = -1;
        order.push_back(refs[first].idx);
        nodes[id] = nd;
        return id;
    }
    int ax = 0;
    for (int k = 1; k < 3; ++k)
        if (chi[k] - clo[k] > chi[ax] - clo[ax]) ax = k;
    const int64_t h = n / 2;
    std::nth_element(refs.begin() + first, refs.begin() + first + h, refs.begin() + first + n,
                     [ax](const TriRef &x, const TriRef &y) {
                         return x.c[ax] < y.c[ax] || (x.c[ax] == y.c[ax] && x.idx < y.idx);
                     });
    const int64_t l = build_env_bvh(refs, first, h, nodes, order, depth + 1, max_depth);
    const int64_t r = build_env_bvh(refs, first + h, n - h, nodes, order, depth + 1, max_depth);
    nd.a = (int32_t)l;
    nd.b = (int32_t)r;
    nodes[id] = nd;
    return id;
}

// Level (breadth-first) order: the root and the top levels form a prefix of the array.
std::vector<BvhNode> bfs_order(const std::vector<BvhNode> &in) {
    std::vector<BvhNode> out;
    out.reserve(in.size());
    std::vector<int32_t> queue;
    queue.reserve(in.size());
    queue.push_back(0);
    for (size_t h = 0; h < queue.size(); ++h) {
        const BvhNode &n = in[queue[h]];
        BvhNode m = n;
        if (n.b >= 0) {
            m.a = (int32_t)(queue.size());      // children get the next free BFS slots
            queue.push_back(n.a);
            m.b = (int32_t)(queue.size());
            queue.push_back(n.b);
        }
        out.push_back(m);
    }
    return out;
}

// Broad-phase 64-ary tree (mpt_internal.h Item) from the pre-order median-split BVH,
// whose subtrees are contiguous ranges of the leaf order.
struct Range {
    int32_t first, count;
};
Range subtree_range(const std::vector<BvhNode> &pre, int32_t id, std::vector<Range> &memo) {
    const BvhNode &n = pre[id];
    Range r = n.b < 0 ? Range{n.a, 1} : Range{0, 0};
    if (n.b >= 0) {
        const Range l = subtree_range(pre, n.a, memo), h = subtree_range(pre, n.b, memo);
        r = Range{l.first, l.count + h.count};
    }
    memo[id] = r;
    return r;
}
// Bucket size of the broad-phase tree: small buckets keep bucket boxes tight for meshes of
// large triangles (rooms), where a 64-triangle bucket spans several walls.
constexpr int32_t env_bucket_size() { return 16; }
static_assert(env_bucket_size() <= kClusterMax, "bucket size");
void collect_buckets(const std::vector<BvhNode> &pre, int32_t id, const std::vector<Range> &memo,
                     std::vector<Range> &out) {
    if (memo[id].count <= env_bucket_size()) {
        out.push_back(memo[id]);
        return;
    }
    collect_buckets(pre, pre[id].a, memo, out);
    collect_buckets(pre, pre[id].b, memo, out);
}
Item union_item(const std::vector<Item> &lvl, int32_t first, int32_t count) {
    Item it{{HUGE_VALF, HUGE_VALF, HUGE_VALF}, first, {-HUGE_VALF, -HUGE_VALF, -HUGE_VALF}, count};
    for (int32_t i = first; i < first + count; ++i)
        for (int k = 0; k < 3; ++k) {
            it.lo[k] = std::min(it.lo[k], lvl[i].lo[k]);
            it.hi[k] = std::max(it.hi[k], lvl[i].hi[k]);
        }
    return it;
}
std::vector<Item> wide_tree(const std::vector<BvhNode> &pre, int64_t n_tris, std::vector<int32_t> &lev_off) {
    std::vector<std::vector<Item>> levels(1);
    levels[0].resize((size_t)n_tris);
    for (const BvhNode &n : pre)
        if (n.b < 0) levels[0][n.a] = Item{{n.lo[0], n.lo[1], n.lo[2]}, n.a, {n.hi[0], n.hi[1], n.hi[2]}, 1};
    {  // always a bucket level (a single bucket for <= 64 triangles)
        std::vector<Range> memo(pre.size()), buckets;
        subtree_range(pre, 0, memo);
        collect_buckets(pre, 0, memo, buckets);
        std::vector<Item> l1;
        for (const Range &r : buckets) l1.push_back(union_item(levels[0], r.first, r.count));
        levels.push_back(std::move(l1));
    }
    while (levels.back().size() > (size_t)kClusterMax) {
        const std::vector<Item> &lo = levels.back();
        std::vector<Item> up;
        for (size_t f = 0; f < lo.size(); f += kClusterMax)
            up.push_back(union_item(lo, (int32_t)f, (int32_t)std::min<size_t>(kClusterMax, lo.size() - f)));
        levels.push_back(std::move(up));
    }
    if ((int)levels.size() > kMaxLevels) throw Error{MPT_ERR_INTERNAL, "env tree too deep"};
    std::vector<Item> all;
    lev_off.assign(1, 0);
    for (size_t l = 0; l < levels.size(); ++l) {
        for (Item it : levels[l]) {
            if (l > 0) it.first += lev_off[l - 1];  // children as absolute item indices
            all.push_back(it);
        }
        lev_off.push_back((int32_t)all.size());
    }
    return all;
}

// Agent clusters: the same median split, stopping at <= 64 triangles.
void build_clusters(std::vector<TriRef> &refs, int64_t first, int64_t n, std::vector<std::pair<int64_t, int64_t>> &out) {
    if (n <= kClusterMax) {
        out.emplace_back(first, n);
        return;
    }
    double clo[3] = {HUGE_VAL, HUGE_VAL, HUGE_VAL}, chi[3] = {-HUGE_VAL, -HUGE_VAL, -HUGE_VAL};
    for (int64_t i = first; i < first + n; ++i)
        for (int k = 0; k < 3; ++k) {
            clo[k] = std::min(clo[k], refs[i].c[k]);
            chi[k] = std::max(chi[k], refs[i].c[k]);
        }
    int ax = 0;
    for (int k = 1; k < 3; ++k)
        if (chi[k] - clo[k] > chi[ax] - clo[ax]) ax = k;
    // split into multiples of 64 where possible to keep clusters full
    int64_t h = ((n / 2 + kClusterMax - 1) / kClusterMax) * kClusterMax;
    if (h >= n) h = n / 2;
    std::nth_element(refs.begin() + first, refs.begin() + first + h, refs.begin() + first + n,
                     [ax](const TriRef &x, const TriRef &y) {
                         return x.c[ax] < y.c[ax] || (x.c[ax] == y.c[ax] && x.idx < y.idx);
                     });
    build_clusters(refs, first, h, out);
    build_clusters(refs, first + h, n - h, out);
}

std::vector<TriRef> make_refs(const double *tris, int64_t n) {
    std::vector<TriRef> refs((size_t)n);
    for (int64_t i = 0; i < n; ++i) {
        const double *t = tris + 9 * i;
        for (int k = 0; k < 3; ++k) {
            refs[i].lo[k] = std::min(t[k], std::min(t[3 + k], t[6 + k]));
            refs[i].hi[k] = std::max(t[k], std::max(t[3 + k], t[6 + k]));
            refs[i].c[k] = 0.5 * (refs[i].lo[k] + refs[i].hi[k]);
        }
        refs[i].idx = i;
    }
    return refs;
}

}  // namespace

// ---------------------------------------------------------------- runtime
extern "C" mpt_status mpt_init(int32_t device) {
    return guarded([&] {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) throw Error{MPT_ERR_NO_DEVICE, "no HIP device visible"};
        require(device >= 0 && device < n, "device index out of range");
        hip_check(hipSetDevice(device), "hipSetDevice");
        hipDeviceProp_t prop;
        hip_check(hipGetDeviceProperties(&prop, device), "hipGetDeviceProperties");
        if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
            throw Error{MPT_ERR_NO_DEVICE, std::string("libmpt is built for gfx950, device is ") + prop.gcnArchName};
        g_device = device;
    });
}

extern "C" const char *mpt_last_error(void) { return g_last_error.c_str(); }
extern "C" int32_t mpt_version(void) { return 100; }

extern "C" mpt_status mpt_device_synchronize(void) {
    return guarded([&] { hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize"); });
}

extern "C" mpt_status mpt_transform_from_location(const double loc7[7], double tf12[12]) {
    return guarded([&] {
        require(loc7 && tf12, "null pointer");
        quat_to_rot(loc7 + 3, tf12);
        tf12[9] = loc7[0];
        tf12[10] = loc7[1];
        tf12[11] = loc7[2];
    });
}

// ---------------------------------------------------------------- env / agent
extern "C" mpt_status mpt_env_create(const double *tris, int64_t n_tris, const double tf12[12], mpt_env **out) {
    return guarded([&] {
        require(out && tf12, "null pointer");
        require(n_tris >= 0 && (n_tris == 0 || tris), "bad triangle soup");
        require(n_tris < (int64_t(1) << 30), "too many env triangles");
        ensure_device();
        auto *env = new mpt_env();
        try {
            std::vector<BvhNode> nodes;
            std::vector<int64_t> order;
            std::vector<EnvTri> recs;
            int64_t depth = 0;
            if (n_tris > 0) {
                auto refs = make_refs(tris, n_tris);
                nodes.reserve(2 * n_tris);
                build_env_bvh(refs, 0, n_tris, nodes, order, 0, depth);
                if (depth + 1 >= kStackDepth) throw Error{MPT_ERR_INTERNAL, "env BVH too deep"};
                std::vector<int32_t> lev_off;
                const std::vector<Item> items = wide_tree(nodes, n_tris, lev_off);
                hip_check(hipMalloc(&env->d_items, sizeof(Item) * items.size()), "hipMalloc env items");
                hip_check(hipMemcpy(env->d_items, items.data(), sizeof(Item) * items.size(), hipMemcpyHostToDevice),
                          "H2D");
                env->dev.n_levels = (int32_t)lev_off.size() - 1;
                for (size_t l = 0; l < lev_off.size(); ++l) env->dev.lev_off[l] = lev_off[l];
                // quantized copies (EnvDev::qitems) over the root box (= the top level's union)
                {
                    float rlo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, rhi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
                    for (int32_t i = lev_off[lev_off.size() - 2]; i < lev_off.back(); ++i)
                        for (int k = 0; k < 3; ++k) {
                            rlo[k] = std::min(rlo[k], items[i].lo[k]);
                            rhi[k] = std::max(rhi[k], items[i].hi[k]);
                        }
                    double scale[3];
                    for (int k = 0; k < 3; ++k) {
                        const double ext = (double)rhi[k] - (double)rlo[k];
                        scale[k] = ext > 0 ? (double)kQMax / ext : 0.0;
                        env->dev.q_org[k] = rlo[k];
                        env->dev.q_scale[k] = (float)scale[k];
                    }
                    // outward: floor / ceil of the exact grid coordinate (the 1e-6 covers the
                    // double rounding of the product)
                    auto qlo = [&](float x, int k) {
                        const double v = std::floor(((double)x - (double)rlo[k]) * scale[k] - 1e-6);
                        return (uint32_t)std::min<double>(kQMax, std::max(0.0, v));
                    };
                    auto qhi = [&](float x, int k) {
                        const double v = std::ceil(((double)x - (double)rlo[k]) * scale[k] + 1e-6);
                        return (uint32_t)std::min<double>(kQMax, std::max(0.0, v));
                    };
                    std::vector<uint4> q(items.size());
                    bool packable = true;
                    for (size_t i = 0; i < items.size(); ++i) {
                        const Item &it = items[i];
                        if (it.first < 0 || it.first >= (1 << 26) || it.count < 1 || it.count > 64) packable = false;
                        q[i].x = qlo(it.lo[0], 0) | qlo(it.lo[1], 1) << 16;
                        q[i].y = qhi(it.hi[0], 0) | qhi(it.hi[1], 1) << 16;
                        q[i].z = qlo(it.lo[2], 2) | qhi(it.hi[2], 2) << 16;
                        q[i].w = (uint32_t)it.first | (uint32_t)(it.count - 1) << 26;
                    }
                    if (packable) {
                        hip_check(hipMalloc(&env->d_qitems, sizeof(uint4) * q.size()), "hipMalloc env qitems");
                        hip_check(hipMemcpy(env->d_qitems, q.data(), sizeof(uint4) * q.size(), hipMemcpyHostToDevice),
                                  "H2D");
                    }
                }
                nodes = bfs_order(nodes);  // top levels first: the prefix k_collide stages in LDS
                recs.resize(n_tris);
                for (int64_t i = 0; i < n_tris; ++i) make_env_tri(tris + 9 * order[i], recs[i]);
                hip_check(hipMalloc(&env->d_tris, sizeof(EnvTri) * n_tris), "hipMalloc env tris");
                hip_check(hipMalloc(&env->d_nodes, sizeof(BvhNode) * nodes.size()), "hipMalloc env nodes");
                hip_check(hipMemcpy(env->d_tris, recs.data(), sizeof(EnvTri) * n_tris, hipMemcpyHostToDevice), "H2D");
                hip_check(hipMemcpy(env->d_nodes, nodes.data(), sizeof(BvhNode) * nodes.size(), hipMemcpyHostToDevice),
                          "H2D");
                for (int k = 0; k < 3; ++k) {
                    env->dev.root_lo[k] = nodes[0].lo[k];
                    env->dev.root_hi[k] = nodes[0].hi[k];
                }
            }
            env->dev.items = env->d_items;
            env->dev.qitems = env->d_qitems;
            env->n_tris = n_tris;
            env->n_nodes = (int64_t)nodes.size();
            env->depth = depth;
            env->dev.tris = env->d_tris;
            env->dev.nodes = env->d_nodes;
            std::memcpy(env->dev.tf, tf12, sizeof(double) * 12);
            env->dev.n_tris = (int32_t)n_tris;
            env->dev.n_nodes = (int32_t)nodes.size();
            *out = env;
        } catch (...) {
            mpt_env_destroy(env);
            throw;
        }
    });
}

extern "C" mpt_status mpt_env_destroy(mpt_env *env) {
    return guarded([&] {
        if (!env) return;
        if (env->d_tris) (void)hipFree(env->d_tris);
        if (env->d_nodes) (void)hipFree(env->d_nodes);
        if (env->d_items) (void)hipFree(env->d_items);
        if (env->d_qitems) (void)hipFree(env->d_qitems);
        delete env;
    });
}

extern "C" mpt_status mpt_env_info(const mpt_env *env, int64_t info[3]) {
    return guarded([&] {
        require(env && info, "null pointer");
        info[0] = env->n_tris;
        info[1] = env->n_nodes;
        info[2] = env->depth;
    });
}

extern "C" mpt_status mpt_agent_create(const double *tris, int64_t n_tris, mpt_agent **out) {
    return guarded([&] {
        require(out, "null pointer");
        require(n_tris >= 0 && (n_tris == 0 || tris), "bad triangle soup");
        require(n_tris < (int64_t(1) << 30), "too many agent triangles");
        ensure_device();
        auto *ag = new mpt_agent();
        try {
            std::vector<double> sorted((size_t)n_tris * 9);
            std::vector<Cluster> cl;
            if (n_tris > 0) {
                auto refs = make_refs(tris, n_tris);
                std::vector<std::pair<int64_t, int64_t>> ranges;
                build_clusters(refs, 0, n_tris, ranges);
                for (auto &r : ranges) {
                    Cluster c{};
                    double lo[3] = {HUGE_VAL, HUGE_VAL, HUGE_VAL}, hi[3] = {-HUGE_VAL, -HUGE_VAL, -HUGE_VAL};
                    for (int64_t i = r.first; i < r.first + r.second; ++i) {
                        std::memcpy(&sorted[9 * i], tris + 9 * refs[i].idx, 9 * sizeof(double));
                        for (int k = 0; k < 3; ++k) {
                            lo[k] = std::min(lo[k], refs[i].lo[k]);
                            hi[k] = std::max(hi[k], refs[i].hi[k]);
                        }
                    }
                    for (int k = 0; k < 3; ++k) {
                        c.c[k] = 0.5 * (lo[k] + hi[k]);
                        // half-extent covering both ends after rounding of the centre
                        c.e[k] = std::max(hi[k] - c.c[k], c.c[k] - lo[k]) * (1.0 + 1e-12) + 1e-12;
                    }
                    c.first = (int32_t)r.first;
                    c.count = (int32_t)r.second;
                    cl.push_back(c);
                }
                hip_check(hipMalloc(&ag->d_tris, sizeof(double) * 9 * n_tris), "hipMalloc agent tris");
                hip_check(hipMalloc(&ag->d_clusters, sizeof(Cluster) * cl.size()), "hipMalloc clusters");
                hip_check(hipMemcpy(ag->d_tris, sorted.data(), sizeof(double) * 9 * n_tris, hipMemcpyHostToDevice),
                          "H2D");
                hip_check(hipMemcpy(ag->d_clusters, cl.data(), sizeof(Cluster) * cl.size(), hipMemcpyHostToDevice),
                          "H2D");
                // the same triangles as P-side records, for link-vs-link (self) collision
                std::vector<EnvTri> rec((size_t)n_tris);
                for (int64_t i = 0; i < n_tris; ++i) make_env_tri(&sorted[9 * i], rec[i]);
                hip_check(hipMalloc(&ag->d_etris, sizeof(EnvTri) * n_tris), "hipMalloc agent records");
                hip_check(hipMemcpy(ag->d_etris, rec.data(), sizeof(EnvTri) * n_tris, hipMemcpyHostToDevice), "H2D");
            }
            ag->dev.etris = ag->d_etris;
            ag->n_tris = n_tris;
            ag->dev.tris = ag->d_tris;
            ag->dev.clusters = ag->d_clusters;
            ag->dev.n_clusters = (int32_t)cl.size();
            ag->dev.n_tris = (int32_t)n_tris;
            // whole-link box (centre / half-extent) for the per-unit cull of the broad phase
            double lo[3] = {HUGE_VAL, HUGE_VAL, HUGE_VAL}, hi[3] = {-HUGE_VAL, -HUGE_VAL, -HUGE_VAL};
            for (int64_t i = 0; i < 3 * n_tris; ++i)
                for (int k = 0; k < 3; ++k) {
                    lo[k] = std::min(lo[k], tris[3 * i + k]);
                    hi[k] = std::max(hi[k], tris[3 * i + k]);
                }
            for (int k = 0; k < 3; ++k) {
                ag->dev.bc[k] = n_tris > 0 ? 0.5 * (lo[k] + hi[k]) : 0.0;
                ag->dev.be[k] = n_tris > 0 ? std::max(hi[k] - ag->dev.bc[k], ag->dev.bc[k] - lo[k]) * (1.0 + 1e-12) + 1e-12
                                           : 0.0;
            }
            *out = ag;
        } catch (...) {
            mpt_agent_destroy(ag);
            throw;
        }
    });
}

extern "C" mpt_status mpt_agent_destroy(mpt_agent *ag) {
    return guarded([&] {
        if (!ag) return;
        if (ag->d_tris) (void)hipFree(ag->d_tris);
        if (ag->d_clusters) (void)hipFree(ag->d_clusters);
        if (ag->d_etris) (void)hipFree(ag->d_etris);
        delete ag;
    });
}

// ---------------------------------------------------------------- collide
namespace mpt {
// used by the RRT engine as well
const EnvDev &env_dev(const mpt_env *e) { return e->dev; }
const AgentDev &agent_dev(const mpt_agent *a) { return a->dev; }
}  // namespace mpt

// The link table lives in a per-thread device buffer that is rewritten only when the
// set of links changes; the rewrite waits for in-flight work that may still read it
// and copies synchronously, so no pageable staging memory outlives the call.
static const AgentDev *link_table(const mpt_agent *const *links, int32_t L, int32_t *max_clusters) {
    static thread_local std::vector<AgentDev> cached;
    std::vector<AgentDev> lk((size_t)L);
    for (int32_t l = 0; l < L; ++l) lk[l] = links[l]->dev;
    const bool same = cached.size() == lk.size() &&
                      std::memcmp(cached.data(), lk.data(), sizeof(AgentDev) * lk.size()) == 0 && g_ws.links.p;
    auto *d_links = (AgentDev *)g_ws.links.p;
    if (!same) {
        hip_check(hipDeviceSynchronize(), "sync before link table update");
        d_links = (AgentDev *)g_ws.links.get(sizeof(AgentDev) * L);
        hip_check(hipMemcpy(d_links, lk.data(), sizeof(AgentDev) * L, hipMemcpyHostToDevice), "links H2D");
        cached = lk;
    }
    *max_clusters = 1;
    for (const AgentDev &a : lk) *max_clusters = std::max(*max_clusters, a.n_clusters);
    return d_links;
}

static void collide_common(const mpt_env *env, const mpt_agent *const *links, int32_t L, const double *d_poses,
                           const int32_t *d_pose_edge, int64_t total_poses, int64_t E, uint8_t *d_verdict,
                           hipStream_t stream) {
    int32_t max_clusters = 1;
    const AgentDev *d_links = link_table(links, L, &max_clusters);
    hip_check(hipMemsetAsync(d_verdict, 0, (size_t)E, stream), "verdict memset");
    CollideWork w{};
    w.poses = d_poses;
    w.pose_edge = d_pose_edge;
    w.pcount = nullptr;
    w.pmax = 1;
    w.L = L;
    w.n_units = total_poses * L;
    w.verdict = d_verdict;
    w.stats = nullptr;
    if (g_stats_enabled) {
        w.stats = (unsigned long long *)g_ws.stats.get(sizeof(g_last_stats));
        hip_check(hipMemsetAsync(w.stats, 0, sizeof(g_last_stats), stream), "stats memset");
    }
    if (collide_mode() == MPT_COLLIDE_FUSED) {
        launch_collide(env->dev, d_links, w, stream);
    } else {
        g_ws.cs.ensure(w.n_units, max_clusters);
        launch_collide_split(env->dev, d_links, max_clusters, w, g_ws.cs, stream);
    }
    if (w.stats) {
        hip_check(hipMemcpyAsync(g_last_stats, w.stats, sizeof(g_last_stats), hipMemcpyDeviceToHost, stream), "stats");
    }
}

static void check_links(const mpt_env *env, const mpt_agent *const *links, int32_t L) {
    require(env != nullptr, "null env");
    require(L >= 1 && links != nullptr, "need at least one link");
    for (int32_t l = 0; l < L; ++l) require(links[l] != nullptr, "null link");
}

extern "C" mpt_status mpt_collide_batch(const mpt_env *env, const mpt_agent *const *links, int32_t L,
                                        const double *poses, const int64_t *edge_pose_offsets, int64_t E,
                                        uint8_t *verdict_out, void *stream_) {
    return mpt_collide_batch_ex(env, links, L, poses, edge_pose_offsets, E, 0, verdict_out, stream_);
}

extern "C" mpt_status mpt_collide_batch_ex(const mpt_env *env, const mpt_agent *const *links, int32_t L,
                                           const double *poses, const int64_t *edge_pose_offsets, int64_t E,
                                           int32_t check_self, uint8_t *verdict_out, void *stream_) {
    return guarded([&] {
        check_links(env, links, L);
        require(E >= 0 && (E == 0 || (edge_pose_offsets && verdict_out)), "bad edge arrays");
        if (E == 0) return;
        require(edge_pose_offsets[0] == 0, "edge_pose_offsets[0] must be 0");
        for (int64_t e = 0; e < E; ++e) require(edge_pose_offsets[e + 1] >= edge_pose_offsets[e], "offsets not monotone");
        const int64_t P = edge_pose_offsets[E];
        require(P == 0 || poses, "null poses");
        require(P < (int64_t(1) << 31), "too many poses");
        hipStream_t stream = (hipStream_t)stream_;
        std::vector<int32_t> pe((size_t)P);
        for (int64_t e = 0; e < E; ++e)
            for (int64_t p = edge_pose_offsets[e]; p < edge_pose_offsets[e + 1]; ++p) pe[p] = (int32_t)e;
        auto *d_poses = (double *)g_ws.poses.get(sizeof(double) * 12 * std::max<int64_t>(P * L, 1));
        auto *d_pe = (int32_t *)g_ws.pose_edge.get(sizeof(int32_t) * std::max<int64_t>(P, 1));
        auto *d_v = (uint8_t *)g_ws.verdict.get((size_t)E);
        if (P > 0) {
            hip_check(hipMemcpyAsync(d_poses, poses, sizeof(double) * 12 * P * L, hipMemcpyHostToDevice, stream),
                      "poses H2D");
            hip_check(hipMemcpyAsync(d_pe, pe.data(), sizeof(int32_t) * P, hipMemcpyHostToDevice, stream), "pe H2D");
        }
        collide_common(env, links, L, d_poses, d_pe, P, E, d_v, stream);
        if (check_self && L > 1) {  // after the env pass, which zeroed the verdicts: OR
            int32_t mc = 1;
            const AgentDev *d_links = link_table(links, L, &mc);
            launch_self_collide(d_links, L, d_poses, d_pe, P, d_v, stream);
        }
        hip_check(hipMemcpyAsync(verdict_out, d_v, (size_t)E, hipMemcpyDeviceToHost, stream), "verdict D2H");
        hip_check(hipStreamSynchronize(stream), "collide sync");
    });
}

extern "C" mpt_status mpt_collide_batch_device(const mpt_env *env, const mpt_agent *const *links, int32_t L,
                                               const double *d_poses, const int64_t *d_edge_pose_offsets, int64_t E,
                                               int64_t total_poses, uint8_t *d_verdict_out, void *stream_) {
    return guarded([&] {
        check_links(env, links, L);
        require(E >= 0 && total_poses >= 0, "bad sizes");
        if (E == 0) return;
        require(d_edge_pose_offsets && d_verdict_out && (total_poses == 0 || d_poses), "null pointer");
        hipStream_t stream = (hipStream_t)stream_;
        auto *d_pe = (int32_t *)g_ws.pose_edge.get(sizeof(int32_t) * std::max<int64_t>(total_poses, 1));
        launch_pose_edge(d_edge_pose_offsets, E, d_pe, stream);
        collide_common(env, links, L, d_poses, d_pe, total_poses, E, d_verdict_out, stream);
    });
}

// ---------------------------------------------------------------- PRMLite edges
extern "C" mpt_status mpt_prmlite_edges(const mpt_env *env, const mpt_agent *agent, const double *vertices, int64_t V,
                                        double step, uint8_t *collides, void *stream_) {
    return guarded([&] {
        require(env && agent, "null handle");
        require(V >= 0 && (V == 0 || vertices), "bad vertices");
        require(step > 0, "step must be > 0");
        const int64_t E = V * (V - 1) / 2;
        if (E == 0) return;
        require(collides != nullptr, "null output");
        hipStream_t stream = (hipStream_t)stream_;
        int32_t mc = 1;
        const mpt_agent *links[1] = {agent};
        const AgentDev *d_link = link_table(links, 1, &mc);
        auto *d_v = (double *)g_ws.poses.get(sizeof(double) * 12 * V);
        auto *d_hit = (uint8_t *)g_ws.verdict.get((size_t)E);
        hip_check(hipMemcpyAsync(d_v, vertices, sizeof(double) * 12 * V, hipMemcpyHostToDevice, stream), "verts H2D");
        hip_check(hipMemsetAsync(d_hit, 0, (size_t)E, stream), "memset");
        launch_prmlite_edges(env->dev, d_link, mc, d_v, V, step, d_hit, nullptr, stream);
        hip_check(hipMemcpyAsync(collides, d_hit, (size_t)E, hipMemcpyDeviceToHost, stream), "D2H");
        hip_check(hipStreamSynchronize(stream), "sync");
    });
}

// ---------------------------------------------------------------- distance
static void distance_common(const mpt_env *env, const mpt_agent *const *links, int32_t L, const double *d_poses,
                            const int32_t *d_pose_edge, int64_t total_poses, int64_t E, double *d_dist,
                            hipStream_t stream) {
    DistWork w{};
    const AgentDev *d_links = link_table(links, L, &w.max_clusters);
    w.poses = d_poses;
    w.pose_edge = d_pose_edge;
    w.L = L;
    w.n_units = total_poses * L;
    w.best = reinterpret_cast<unsigned long long *>(d_dist);  // written as double bit patterns
    if (g_stats_enabled) {
        w.stats = (unsigned long long *)g_ws.stats.get(sizeof(g_last_stats));
        hip_check(hipMemsetAsync(w.stats, 0, sizeof(g_last_stats), stream), "stats memset");
    }
    launch_distance(env->dev, d_links, w, E, stream);
    if (w.stats) {
        hip_check(hipMemcpyAsync(g_last_stats, w.stats, sizeof(g_last_stats), hipMemcpyDeviceToHost, stream), "stats");
    }
}

extern "C" mpt_status mpt_distance_batch(const mpt_env *env, const mpt_agent *const *links, int32_t L,
                                         const double *poses, const int64_t *edge_pose_offsets, int64_t E,
                                         double *dist_out, void *stream_) {
    return guarded([&] {
        check_links(env, links, L);
        require(E >= 0 && (E == 0 || (edge_pose_offsets && dist_out)), "bad edge arrays");
        if (E == 0) return;
        require(edge_pose_offsets[0] == 0, "edge_pose_offsets[0] must be 0");
        for (int64_t e = 0; e < E; ++e) require(edge_pose_offsets[e + 1] >= edge_pose_offsets[e], "offsets not monotone");
        const int64_t P = edge_pose_offsets[E];
        require(P == 0 || poses, "null poses");
        require(P < (int64_t(1) << 31), "too many poses");
        hipStream_t stream = (hipStream_t)stream_;
        std::vector<int32_t> pe((size_t)P);
        for (int64_t e = 0; e < E; ++e)
            for (int64_t p = edge_pose_offsets[e]; p < edge_pose_offsets[e + 1]; ++p) pe[p] = (int32_t)e;
        auto *d_poses = (double *)g_ws.poses.get(sizeof(double) * 12 * std::max<int64_t>(P * L, 1));
        auto *d_pe = (int32_t *)g_ws.pose_edge.get(sizeof(int32_t) * std::max<int64_t>(P, 1));
        auto *d_d = (double *)g_ws.d2.get(sizeof(double) * (size_t)E);
        if (P > 0) {
            hip_check(hipMemcpyAsync(d_poses, poses, sizeof(double) * 12 * P * L, hipMemcpyHostToDevice, stream),
                      "poses H2D");
            hip_check(hipMemcpyAsync(d_pe, pe.data(), sizeof(int32_t) * P, hipMemcpyHostToDevice, stream), "pe H2D");
        }
        distance_common(env, links, L, d_poses, d_pe, P, E, d_d, stream);
        hip_check(hipMemcpyAsync(dist_out, d_d, sizeof(double) * (size_t)E, hipMemcpyDeviceToHost, stream), "dist D2H");
        hip_check(hipStreamSynchronize(stream), "distance sync");
    });
}

extern "C" mpt_status mpt_distance_batch_device(const mpt_env *env, const mpt_agent *const *links, int32_t L,
                                                const double *d_poses, const int64_t *d_edge_pose_offsets, int64_t E,
                                                int64_t total_poses, double *d_dist_out, void *stream_) {
    return guarded([&] {
        check_links(env, links, L);
        require(E >= 0 && total_poses >= 0, "bad sizes");
        if (E == 0) return;
        require(d_edge_pose_offsets && d_dist_out && (total_poses == 0 || d_poses), "null pointer");
        hipStream_t stream = (hipStream_t)stream_;
        auto *d_pe = (int32_t *)g_ws.pose_edge.get(sizeof(int32_t) * std::max<int64_t>(total_poses, 1));
        launch_pose_edge(d_edge_pose_offsets, E, d_pe, stream);
        distance_common(env, links, L, d_poses, d_pe, total_poses, E, d_dist_out, stream);
    });
}

extern "C" mpt_status mpt_set_collide_mode(int32_t mode) {
    return guarded([&] {
        require(mode == MPT_COLLIDE_SPLIT || mode == MPT_COLLIDE_FUSED, "unknown collide mode");
        g_collide_mode.store(mode, std::memory_order_relaxed);
    });
}

extern "C" mpt_status mpt_set_stats(int32_t enable) {
    return guarded([&] { g_stats_enabled = enable != 0; });
}

extern "C" mpt_status mpt_last_collide_stats(uint64_t stats[4]) {
    return guarded([&] {
        require(stats, "null pointer");
        hip_check(hipDeviceSynchronize(), "sync");
        for (int i = 0; i < 4; ++i) stats[i] = g_last_stats[i];
    });
}

// ---------------------------------------------------------------- NN
static void nn_reserve(mpt_nn *nn, int64_t need) {
    if (need <= nn->cap) return;
    int64_t cap = std::max<int64_t>(need, std::max<int64_t>(nn->cap * 2, 1024));
    double *p = nullptr;
    hip_check(hipMalloc(&p, sizeof(double) * nn->d * cap), "hipMalloc nn points");
    if (nn->d_pts) {
        hip_check(hipMemcpy(p, nn->d_pts, sizeof(double) * nn->d * nn->n, hipMemcpyDeviceToDevice), "nn grow");
        (void)hipFree(nn->d_pts);
    }
    nn->d_pts = p;
    if (nn->d_removed) {
        uint8_t *r = nullptr;
        hip_check(hipMalloc(&r, (size_t)cap), "hipMalloc removed");
        hip_check(hipMemset(r, 0, (size_t)cap), "memset");
        hip_check(hipMemcpy(r, nn->d_removed, (size_t)nn->n, hipMemcpyDeviceToDevice), "grow removed");
        (void)hipFree(nn->d_removed);
        nn->d_removed = r;
    }
    nn->cap = cap;
}

extern "C" mpt_status mpt_nn_create(int32_t dim, int64_t capacity, mpt_nn **out) {
    return guarded([&] {
        require(out, "null pointer");
        require(dim >= 1 && dim <= 16, "dim must be in [1, 16]");
        require(capacity >= 0, "bad capacity");
        ensure_device();
        auto *nn = new mpt_nn();
        nn->d = dim;
        try {
            nn_reserve(nn, std::max<int64_t>(capacity, 1));
        } catch (...) {
            delete nn;
            throw;
        }
        *out = nn;
    });
}

extern "C" mpt_status mpt_nn_destroy(mpt_nn *nn) {
    return guarded([&] {
        if (!nn) return;
        if (nn->d_pts) (void)hipFree(nn->d_pts);
        if (nn->d_removed) (void)hipFree(nn->d_removed);
        if (nn->d_bbox) (void)hipFree(nn->d_bbox);
        delete nn;
    });
}

extern "C" mpt_status mpt_nn_append(mpt_nn *nn, const double *pts, int64_t n, int32_t *ids_out) {
    return guarded([&] {
        require(nn && n >= 0 && (n == 0 || pts), "bad arguments");
        require(nn->n + n < (int64_t(1) << 31) - 1, "id space exhausted");
        nn_reserve(nn, nn->n + n);
        if (n > 0)
            hip_check(hipMemcpy(nn->d_pts + nn->n * nn->d, pts, sizeof(double) * nn->d * n, hipMemcpyHostToDevice),
                      "nn append");
        if (ids_out)
            for (int64_t i = 0; i < n; ++i) ids_out[i] = (int32_t)(nn->n + i + 1);
        nn->n += n;
    });
}

extern "C" mpt_status mpt_nn_append_device(mpt_nn *nn, const double *d_pts, int64_t n, void *stream) {
    return guarded([&] {
        require(nn && n >= 0 && (n == 0 || d_pts), "bad arguments");
        nn_reserve(nn, nn->n + n);
        if (n > 0)
            hip_check(hipMemcpyAsync(nn->d_pts + nn->n * nn->d, d_pts, sizeof(double) * nn->d * n,
                                     hipMemcpyDeviceToDevice, (hipStream_t)stream),
                      "nn append device");
        nn->n += n;
    });
}

extern "C" mpt_status mpt_nn_remove(mpt_nn *nn, int32_t id) {
    return guarded([&] {
        require(nn, "null nn");
        require(id >= 1 && id <= nn->n, "id out of range");
        if (!nn->d_removed) {
            hip_check(hipMalloc(&nn->d_removed, (size_t)nn->cap), "hipMalloc removed");
            hip_check(hipMemset(nn->d_removed, 0, (size_t)nn->cap), "memset removed");
        }
        const uint8_t one = 1;
        hip_check(hipMemcpy(nn->d_removed + (id - 1), &one, 1, hipMemcpyHostToDevice), "remove");
    });
}

extern "C" mpt_status mpt_nn_size(const mpt_nn *nn, int64_t *n_out) {
    return guarded([&] {
        require(nn && n_out, "null pointer");
        *n_out = nn->n;
    });
}

extern "C" mpt_status mpt_nn_points_device(const mpt_nn *nn, const double **d_pts) {
    return guarded([&] {
        require(nn && d_pts, "null pointer");
        *d_pts = nn->d_pts;
    });
}

static NNWork nn_work(const mpt_nn *nn, const double *d_q, int64_t nq) {
    NNWork w{};
    w.pts = nn->d_pts;
    w.removed = nn->d_removed;
    w.n = nn->n;
    w.d = nn->d;
    w.q = d_q;
    w.nq = nq;
    return w;
}

// Grid index when it pays (enough points and queries), brute force otherwise; both are exact
// and return identical results.  A stale grid is rebuilt first (bbox D2H: synchronises).
static void nn_query(mpt_nn *nn, const double *d_q, int64_t nq, int32_t k, int32_t *d_ids, double *d_d2,
                     hipStream_t stream) {
    const bool use_grid = nn->mode == MPT_NN_GRID || (nn->mode == MPT_NN_AUTO && nn->n >= 4096 && nq >= 32);
    if (!use_grid || nn->n == 0) {
        const NNWork w = nn_work(nn, d_q, nq);
        void *scratch = g_ws.scratch.get(nn_knn_scratch_bytes(nq, std::max<int64_t>(nn->n, 1), k));
        launch_knn(w, k, d_ids, d_d2, scratch, stream);
        return;
    }
    if (!nn->grid) nn->grid.reset(new GridIndex());
    if (nn->grid_n != nn->n) {
        if (!nn->d_bbox) hip_check(hipMalloc(&nn->d_bbox, sizeof(double) * 2 * 16), "bbox alloc");
        launch_bbox(nn->d_pts, nn->n, nn->d, nn->d_bbox, stream);
        double lohi[32];
        hip_check(hipMemcpyAsync(lohi, nn->d_bbox, sizeof(double) * 2 * nn->d, hipMemcpyDeviceToHost, stream), "bbox");
        hip_check(hipStreamSynchronize(stream), "bbox sync");
        int32_t dims[3];
        const int32_t gd = choose_grid_dims(nn->d, lohi, dims);
        double lo[3], hi[3];
        for (int j = 0; j < gd; ++j) {
            lo[j] = lohi[2 * dims[j]];
            hi[j] = lohi[2 * dims[j] + 1];
        }
        const GridParams g = make_grid_params(nn->d, dims, gd, lo, hi, nn->n, 2.0);
        nn->grid->build(nn->d_pts, nn->n, nullptr, nn->d, g, stream);
        nn->grid_n = nn->n;
    }
    GridDev G = nn->grid->dev();
    G.removed = nn->d_removed;
    launch_grid_knn(G, nn->d, d_q, nq, k, d_ids, d_d2, stream);
}

extern "C" mpt_status mpt_nn_set_index(mpt_nn *nn, int32_t mode) {
    return guarded([&] {
        require(nn && mode >= MPT_NN_AUTO && mode <= MPT_NN_GRID, "bad arguments");
        nn->mode = mode;
    });
}

extern "C" mpt_status mpt_nn_knn_device(mpt_nn *nn, const double *d_q, int64_t nq, int32_t k, int32_t *d_ids,
                                        double *d_d2, void *stream) {
    return guarded([&] {
        require(nn && nq >= 0, "bad arguments");
        require(k >= 1 && k <= 32, "k must be in [1, 32]");
        if (nq == 0) return;
        require(d_q && d_ids && d_d2, "null pointer");
        nn_query(nn, d_q, nq, k, d_ids, d_d2, (hipStream_t)stream);
    });
}

extern "C" mpt_status mpt_nn_knn(mpt_nn *nn, const double *q, int64_t nq, int32_t k, int32_t *ids, double *d2,
                                 void *stream_) {
    return guarded([&] {
        require(nn && nq >= 0, "bad arguments");
        require(k >= 1 && k <= 32, "k must be in [1, 32]");
        if (nq == 0) return;
        require(q && ids && d2, "null pointer");
        hipStream_t stream = (hipStream_t)stream_;
        auto *d_q = (double *)g_ws.q.get(sizeof(double) * nn->d * nq);
        auto *d_ids = (int32_t *)g_ws.ids.get(sizeof(int32_t) * nq * k);
        auto *d_d2 = (double *)g_ws.d2.get(sizeof(double) * nq * k);
        hip_check(hipMemcpyAsync(d_q, q, sizeof(double) * nn->d * nq, hipMemcpyHostToDevice, stream), "q H2D");
        nn_query(nn, d_q, nq, k, d_ids, d_d2, stream);
        hip_check(hipMemcpyAsync(ids, d_ids, sizeof(int32_t) * nq * k, hipMemcpyDeviceToHost, stream), "ids D2H");
        hip_check(hipMemcpyAsync(d2, d_d2, sizeof(double) * nq * k, hipMemcpyDeviceToHost, stream), "d2 D2H");
        hip_check(hipStreamSynchronize(stream), "knn sync");
    });
}

extern "C" mpt_status mpt_nn_radius(mpt_nn *nn, const double *q, int64_t nq, double r2, int32_t max_nb,
                                    int64_t *offsets, int32_t *ids, double *d2, int64_t cap, void *stream_) {
    return guarded([&] {
        require(nn && nq >= 0 && offsets, "bad arguments");
        require(cap >= 0 && (cap == 0 || (ids && d2)), "bad output arrays");
        hipStream_t stream = (hipStream_t)stream_;
        if (nq == 0) {
            offsets[0] = 0;
            return;
        }
        require(q, "null queries");
        auto *d_q = (double *)g_ws.q.get(sizeof(double) * nn->d * nq);
        auto *d_off = (int64_t *)g_ws.offsets.get(sizeof(int64_t) * (nq + 1));
        auto *d_ids = (int32_t *)g_ws.ids.get(sizeof(int32_t) * std::max<int64_t>(cap, 1));
        auto *d_d2 = (double *)g_ws.d2.get(sizeof(double) * std::max<int64_t>(cap, 1));
        hip_check(hipMemcpyAsync(d_q, q, sizeof(double) * nn->d * nq, hipMemcpyHostToDevice, stream), "q H2D");
        const NNWork w = nn_work(nn, d_q, nq);
        const int64_t total = launch_radius(w, r2, max_nb, d_off, d_ids, d_d2, cap, nullptr, 0, stream);
        hip_check(hipMemcpyAsync(offsets, d_off, sizeof(int64_t) * (nq + 1), hipMemcpyDeviceToHost, stream), "off");
        const int64_t m = std::min(total, cap);
        if (m > 0) {
            hip_check(hipMemcpyAsync(ids, d_ids, sizeof(int32_t) * m, hipMemcpyDeviceToHost, stream), "ids D2H");
            hip_check(hipMemcpyAsync(d2, d_d2, sizeof(double) * m, hipMemcpyDeviceToHost, stream), "d2 D2H");
        }
        hip_check(hipStreamSynchronize(stream), "radius sync");
    });
}
