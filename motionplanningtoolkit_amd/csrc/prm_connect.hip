// prm_connect.hip -- PRM roadmap edges on the device (BASELINE config 4).
//
// PRM::addMilestone (planners/prm/prm.hpp:334-387) per milestone: neighbours from the NN,
// steer(src, tgt, 1000), Map3D::safeEdge, add_edge + union_set.  Config 4 asks for radius
// neighbours (FLANN_KDTreeWrapper::kNearestWithin, utilities/flannkdtreewrapper.hpp:91-117:
// squared L2 < radius) in place of the approximate kNN(10).  With radius neighbours the
// roadmap does not depend on the insertion batching: milestone i connects to every earlier j
// within the radius.  So all milestones go through one pipeline:
//   keys (first three state variables, prm.hpp:155) -> point tree (point_tree.hip) ->
//   radius count -> scan -> radius fill (j < i) -> per-query sort by j -> per edge
//   Omnidirectional::steer(i, j, 1000) and getPoses at cc_dt -> pose scan -> poses ->
//   batched collision (sweep.hip: one wave per (edge, agent cluster)) -> verdicts; components
//   on the host.
// Edge poses translate along the key segment (Omnidirectional::getPoses); a blimp mesh keeps
// the yaw of milestone i (Blimp::stateToFCLTransform's R, cos/sin from the host's libm so the
// rotation is bit-identical to the oracle's).
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "../../include/mpt.h"
#include "mpt_internal.h"
#include "point_tree.h"
#include "prm_edges.h"

namespace mpt {
const EnvDev &env_dev(const mpt_env *e);
const AgentDev &agent_dev(const mpt_agent *a);
int32_t collide_mode();
}  // namespace mpt

using namespace mpt;

namespace {

__global__ void k_widen(const int32_t *__restrict__ c, int64_t n, int64_t *__restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = c[i];
    if (i == n) out[i] = 0;
}

// each query's neighbours by id (ascending), and the edge -> source milestone map
__global__ void k_sort_segments(const int64_t *__restrict__ off, int64_t nq, int32_t *__restrict__ ids,
                                int32_t *__restrict__ src) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nq) return;
    const int64_t a = off[q], b = off[q + 1];
    for (int64_t i = a + 1; i < b; ++i) {
        const int32_t v = ids[i];
        int64_t k = i - 1;
        while (k >= a && ids[k] > v) {
            ids[k + 1] = ids[k];
            --k;
        }
        ids[k + 1] = v;
    }
    for (int64_t i = a; i < b; ++i) src[i] = (int32_t)q;
}

__global__ void k_edge_pose_count(PrmEdges P, int64_t E, int64_t *__restrict__ pc) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e > E) return;
    if (e == E) {
        pc[e] = 0;
        return;
    }
    const PrmEdge g = prm_edge(P, e);
    pc[e] = g.it < 1 ? 2 : (int64_t)g.it + (g.tail ? 1 : 0);
}

// the pose array (mpt_set_collide_mode FUSED: the per-pose walk reads it; the sweep generates
// the same poses in-kernel instead, sweep.hip PrmEdge)
__global__ void k_edge_poses(PrmEdges P, int64_t E, const int64_t *__restrict__ poff, double *__restrict__ poses,
                             int32_t *__restrict__ pose_edge) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    const PrmEdge g = prm_edge(P, e);
    int64_t p = poff[e];
    g.each([&](const double *t) {
        double *o = poses + 12 * p;
#pragma unroll
        for (int k = 0; k < 9; ++k) o[k] = g.R[k];
        o[9] = t[0];
        o[10] = t[1];
        o[11] = t[2];
        pose_edge[p++] = (int32_t)e;
        return false;
    });
}

template <class T>
struct DBuf {
    T *p = nullptr;
    int64_t cap = 0;
    T *get(int64_t n) {
        if (n > cap) {
            if (p) hip_check(hipFree(p), "free");
            cap = std::max<int64_t>(n, 2 * cap);
            hip_check(hipMalloc(&p, sizeof(T) * (size_t)std::max<int64_t>(cap, 1)), "prm buffer");
        }
        return p;
    }
    ~DBuf() {
        if (p) (void)hipFree(p);
    }
};

// a pinned host buffer that grows (the milestones' keys and yaw go up from it asynchronously)
struct PinnedBuf {
    double *p = nullptr;
    size_t cap = 0;
    double *get(size_t n) {
        if (n > cap) {
            if (p) hip_check(hipHostFree(p), "free");
            p = nullptr;
            hip_check(hipHostMalloc(&p, sizeof(double) * std::max<size_t>(n, 1)), "pinned staging");
            cap = n;
        }
        return p;
    }
    ~PinnedBuf() {
        if (p) (void)hipHostFree(p);
    }
};

struct PrmScratch {
    PointTree tree;
    PinnedBuf hkeys, hrot;
    CollideScratch cs;
    DBuf<double> keys, rot, d2, poses;
    DBuf<int32_t> counts, nbr, src, pose_edge;
    DBuf<int64_t> off, poff, n_dev;
    DBuf<uint8_t> verdict;
    DBuf<AgentDev> link;
    DBuf<char> temp;
};

int64_t scan_total(int64_t *d_in_out, int64_t n_plus_1, DBuf<char> &temp, hipStream_t stream) {
    size_t tb = 0;
    hip_check(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, d_in_out, d_in_out, (int)n_plus_1), "scan size");
    void *t = temp.get((int64_t)tb + 1);
    hip_check(hipcub::DeviceScan::ExclusiveSum(t, tb, d_in_out, d_in_out, (int)n_plus_1, stream), "scan");
    int64_t total = 0;
    hip_check(hipMemcpyAsync(&total, d_in_out + n_plus_1 - 1, sizeof(int64_t), hipMemcpyDeviceToHost, stream), "total");
    hip_check(hipStreamSynchronize(stream), "scan sync");
    return total;
}

// mpt_prm_stats: the sweep's work counters for the next mpt_prm_connect calls (one
// same-address atomic per wave: diagnostics only, never in a timed call)
thread_local bool g_prm_stats_on = false;
thread_local uint64_t g_prm_stats[8] = {};

int32_t uf_find(std::vector<int32_t> &p, int32_t x) {
    while (p[x] != x) {
        p[x] = p[p[x]];
        x = p[x];
    }
    return x;
}

}  // namespace

extern "C" mpt_status mpt_prm_stats(int32_t enable, uint64_t *out, int32_t count) {
    return guarded([&] {
        if (out)
            for (int i = 0; i < 8 && i < count; ++i) out[i] = g_prm_stats[i];
        g_prm_stats_on = enable != 0;
    });
}

extern "C" mpt_status mpt_prm_deferred_edges(int32_t *out, int64_t cap, int64_t *n) {
    return guarded([&] {
        if (!n) throw Error{MPT_ERR_INVALID, "mpt_prm_deferred_edges: n is NULL"};
        *n = (int64_t)last_sweep_deferred.size();
        if (out)
            for (int64_t i = 0; i < *n && i < cap; ++i) out[i] = last_sweep_deferred[(size_t)i];
    });
}

extern "C" mpt_status mpt_set_sweep_queue_cap(int64_t max_candidates) {
    return guarded([&] {
        if (max_candidates < 0) throw Error{MPT_ERR_INVALID, "mpt_set_sweep_queue_cap: negative"};
        sweep_queue_cap_limit = max_candidates;
    });
}

extern "C" mpt_status mpt_prm_connect(const mpt_env *env, const mpt_agent *agent, int32_t agent_kind,
                                      const double *states, int64_t n, int32_t dim, double radius2, double cc_dt,
                                      int64_t cap, int32_t *edges, uint8_t *verdict, int64_t *n_edges, int32_t *comp,
                                      float ms[4]) {
    return guarded([&] {
        if (!env || !agent || !n_edges || n < 0 || (n > 0 && !states)) throw Error{MPT_ERR_INVALID, "bad arguments"};
        if (!(agent_kind == MPT_AGENT_OMNI && dim == 3) && !(agent_kind == MPT_AGENT_BLIMP && dim == 7))
            throw Error{MPT_ERR_INVALID, "mpt_prm_connect: omnidirectional (dim 3) or blimp (dim 7) milestones"};
        if (!(cc_dt > 0) || !(radius2 >= 0)) throw Error{MPT_ERR_INVALID, "bad radius / dt"};
        if (n >= (int64_t(1) << 27)) throw Error{MPT_ERR_INVALID, "too many milestones"};
        static thread_local PrmScratch S;
        hipStream_t stream = nullptr;
        hipEvent_t ev[5];
        for (auto &e : ev) hip_check(hipEventCreate(&e), "event");
        struct EvGuard {
            hipEvent_t *e;
            ~EvGuard() {
                for (int i = 0; i < 5; ++i) (void)hipEventDestroy(e[i]);
            }
        } guard{ev};
        hip_check(hipEventRecord(ev[0], stream), "event");
        // keys and yaw on the host (libm cos/sin, as the oracle), over up to 16 threads: one
        // thread took ~2 ms of the 100 000-milestone call with the device idle
        double *hk = S.hkeys.get((size_t)n * 3), *hr = S.hrot.get((size_t)n * 2);
        auto fill = [&](int64_t i0, int64_t i1) {
            for (int64_t i = i0; i < i1; ++i) {
                for (int k = 0; k < 3; ++k) hk[i * 3 + k] = states[i * dim + k];
                hr[i * 2] = dim == 7 ? std::cos(states[i * dim + 3]) : 1.0;
                hr[i * 2 + 1] = dim == 7 ? std::sin(states[i * dim + 3]) : 0.0;
            }
        };
        {
            const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
            const int64_t nt = std::min<int64_t>(hw, (n + 8191) / 8192);
            std::vector<std::thread> pool;
            for (int64_t t = 1; t < nt; ++t) pool.emplace_back(fill, n * t / nt, n * (t + 1) / nt);
            fill(0, nt > 1 ? n / nt : n);
            for (auto &th : pool) th.join();
        }
        double *d_keys = S.keys.get(n * 3), *d_rot = S.rot.get(n * 2);
        int64_t *d_n = S.n_dev.get(1);
        hip_check(hipMemcpyAsync(d_keys, hk, sizeof(double) * n * 3, hipMemcpyHostToDevice, stream), "keys");
        hip_check(hipMemcpyAsync(d_rot, hr, sizeof(double) * n * 2, hipMemcpyHostToDevice, stream), "rot");
        hip_check(hipMemcpy(d_n, &n, sizeof(int64_t), hipMemcpyHostToDevice), "n");
        // neighbours: j < i with squared key distance < radius2, sorted by j
        int64_t E = 0;
        int32_t *d_cnt = S.counts.get(n + 1);
        int64_t *d_off = S.off.get(n + 1);
        if (n > 0) {
            S.tree.build(d_keys, n, d_n, 3, stream);
            const PointTreeDev T = S.tree.dev();
            launch_tree_radius(T, d_keys, n, radius2, true, d_cnt, nullptr, nullptr, nullptr, stream);
            hipLaunchKernelGGL(k_widen, dim3((unsigned)((n + 1 + 255) / 256)), dim3(256), 0, stream, d_cnt, n, d_off);
            E = scan_total(d_off, n + 1, S.temp, stream);
        }
        if (E >= (int64_t(1) << 31)) throw Error{MPT_ERR_CAPACITY, "too many roadmap edges"};
        int32_t *d_nbr = S.nbr.get(E), *d_src = S.src.get(E);
        double *d_d2 = S.d2.get(E);
        if (E > 0) {
            launch_tree_radius(S.tree.dev(), d_keys, n, radius2, true, d_cnt, d_off, d_nbr, d_d2, stream);
            hipLaunchKernelGGL(k_sort_segments, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, d_off, n, d_nbr,
                               d_src);
            hip_check(hipGetLastError(), "k_sort_segments");
        }
        hip_check(hipEventRecord(ev[1], stream), "event");
        // the edges' poses: the sweep generates them where it tests them (no pose array); the
        // fused per-pose walk (mpt_set_collide_mode FUSED) and the work counters (the pose
        // count) need the count scan, the fused walk the array
        const bool sweep = collide_mode() != MPT_COLLIDE_FUSED;
        const PrmEdges PE{d_keys, d_rot, d_src, d_nbr, cc_dt};
        int64_t P = 0;
        int64_t *d_poff = nullptr;
        double *d_poses = nullptr;
        int32_t *d_pe = nullptr;
        if (E > 0 && (!sweep || g_prm_stats_on)) {
            d_poff = S.poff.get(E + 1);
            hipLaunchKernelGGL(k_edge_pose_count, dim3((unsigned)((E + 1 + 255) / 256)), dim3(256), 0, stream, PE, E,
                               d_poff);
            P = scan_total(d_poff, E + 1, S.temp, stream);
            if (P >= (int64_t(1) << 31)) throw Error{MPT_ERR_CAPACITY, "too many edge poses"};
        }
        if (E > 0 && !sweep) {
            d_poses = S.poses.get(P * 12);
            d_pe = S.pose_edge.get(P);
            hipLaunchKernelGGL(k_edge_poses, dim3((unsigned)((E + 255) / 256)), dim3(256), 0, stream, PE, E, d_poff,
                               d_poses, d_pe);
        }
        hip_check(hipEventRecord(ev[2], stream), "event");
        // collision verdicts (the sweep path; mpt_set_collide_mode FUSED: the per-pose fused walk)
        uint8_t *d_v = S.verdict.get(E);
        if (E > 0) {
            hip_check(hipMemsetAsync(d_v, 0, (size_t)E, stream), "verdict memset");
            AgentDev *d_link = S.link.get(1);
            const AgentDev ag = agent_dev(agent);
            hip_check(hipMemcpy(d_link, &ag, sizeof(AgentDev), hipMemcpyHostToDevice), "link");
            const int32_t mc = std::max(1, ag.n_clusters);
            if (sweep) {
                unsigned long long *st = nullptr;
                if (g_prm_stats_on) {
                    st = reinterpret_cast<unsigned long long *>(S.temp.get(64));
                    hip_check(hipMemsetAsync(st, 0, sizeof(unsigned long long) * 4, stream), "stats zero");
                }
                launch_collide_sweep_prm(env_dev(env), d_link, mc, PE, E, d_v, st, stream);
                if (st) {
                    unsigned long long h[4];
                    hip_check(hipMemcpyAsync(h, st, sizeof(h), hipMemcpyDeviceToHost, stream), "stats");
                    hip_check(hipStreamSynchronize(stream), "stats sync");
                    for (int i = 0; i < 4; ++i) g_prm_stats[i] = h[i];
                    g_prm_stats[4] = (uint64_t)E;
                    g_prm_stats[5] = (uint64_t)P;
                    g_prm_stats[6] = last_sweep_counts[0];
                    g_prm_stats[7] = last_sweep_counts[1];
                }
            } else {
                CollideWork w{};
                w.poses = d_poses;
                w.pose_edge = d_pe;
                w.pmax = 1;
                w.L = 1;
                w.n_units = P;
                w.verdict = d_v;
                launch_collide(env_dev(env), d_link, w, stream);
            }
        }
        hip_check(hipEventRecord(ev[3], stream), "event");
        std::vector<int32_t> h_src((size_t)E), h_nbr((size_t)E);
        std::vector<uint8_t> h_v((size_t)E);
        if (E > 0) {
            hip_check(hipMemcpyAsync(h_src.data(), d_src, sizeof(int32_t) * E, hipMemcpyDeviceToHost, stream), "src");
            hip_check(hipMemcpyAsync(h_nbr.data(), d_nbr, sizeof(int32_t) * E, hipMemcpyDeviceToHost, stream), "nbr");
            hip_check(hipMemcpyAsync(h_v.data(), d_v, (size_t)E, hipMemcpyDeviceToHost, stream), "verdict");
        }
        hip_check(hipStreamSynchronize(stream), "prm sync");
        // union-find over the collision-free edges (disjoint_sets, prm.hpp:346,376)
        std::vector<int32_t> parent((size_t)n);
        for (int64_t i = 0; i < n; ++i) parent[i] = (int32_t)i;
        for (int64_t e = 0; e < E; ++e) {
            if (h_v[e]) continue;
            const int32_t a = uf_find(parent, h_src[e]), b = uf_find(parent, h_nbr[e] - 1);
            if (a != b) parent[std::max(a, b)] = std::min(a, b);
        }
        hip_check(hipEventRecord(ev[4], stream), "event");
        hip_check(hipEventSynchronize(ev[4]), "event sync");
        *n_edges = E;
        const int64_t m = std::min(E, cap);
        for (int64_t e = 0; e < m; ++e) {
            if (edges) {
                edges[2 * e] = h_src[e];
                edges[2 * e + 1] = h_nbr[e] - 1;
            }
            if (verdict) verdict[e] = h_v[e];
        }
        if (comp)
            for (int64_t i = 0; i < n; ++i) comp[i] = uf_find(parent, (int32_t)i);
        if (ms) {
            hip_check(hipEventElapsedTime(&ms[0], ev[0], ev[1]), "elapsed");
            hip_check(hipEventElapsedTime(&ms[1], ev[1], ev[2]), "elapsed");
            hip_check(hipEventElapsedTime(&ms[2], ev[2], ev[3]), "elapsed");
            hip_check(hipEventElapsedTime(&ms[3], ev[0], ev[4]), "elapsed");
        }
    });
}
