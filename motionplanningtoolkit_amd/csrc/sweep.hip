// sweep.hip -- collision of straight-line edges whose poses share one rotation.
//
// Same verdicts as the two-phase and fused paths (verdict[e] = some pose p of edge e, agent
// triangle a and env triangle t with tri_gate and intersect_Triangle true), organised around
// the edge instead of the pose.  PRM edges (prm_connect.hip: Omnidirectional::getPoses along
// the key segment, one yaw per edge) have ~40 poses 0.1 apart that overlap nearly the same env
// triangles, so per-pose broad phases redo the same work ~40 times.  Here one wave handles one
// (edge, agent cluster):
//   1. R, T of the first and last pose (fcl::relativeTransform, uniform); the cluster's box at
//      both ends -> swept box (every pose's translation lies on the segment between them; the
//      widened float boxes cover the rounding of the interpolated translations);
//   2. lanes = the cluster's triangles: R Q once (the rotated vertices; each pose only adds
//      its T, exactly as xform() orders the operations), swept triangle box;
//   3. the wave walks the 64-ary env tree against the swept cluster box (lanes = a node's
//      children, LDS stack); at a bucket, each env triangle whose box meets the swept cluster
//      box is tested by the lanes whose swept triangle box meets it, over the edge's poses:
//      Q'_p = R Q + T_p, exact tri_gate, intersect_Triangle; a hit sets verdict[e] and every
//      wave of the edge stops.
#include "collide_common.h"
#include "prm_edges.h"
#include "wave_ops.h"

namespace mpt {

constexpr int kSweepWaves = 4;
constexpr int kSweepStack = kMaxLevels * kWave;

struct SweepCounters {
    uint32_t waves = 0, items = 0, pair_poses = 0, sat = 0;
};

// fcl::relativeTransform's T for a world translation t (R1^T (t - T1), relative_transform()'s order)
__device__ __forceinline__ void env_rel_t(const EnvDev &env, const double *t, double Tp[3]) {
    const double d0 = t[0] - env.tf[9], d1 = t[1] - env.tf[10], d2 = t[2] - env.tf[11];
#pragma unroll
    for (int i = 0; i < 3; ++i) Tp[i] = env.tf[0 * 3 + i] * d0 + env.tf[1 * 3 + i] * d1 + env.tf[2 * 3 + i] * d2;
}

// One (edge, cluster): Rw = the edge's world rotation, tf / tl = world translations of its
// first and last pose, gen(f, RQ, E, env) calls f(world translation) for each pose in order
// whose gate with env triangle E may pass (every pose, or a superset of those) and stops when f
// returns true (a contact).
template <class Gen>
__device__ __forceinline__ void sweep_core(const EnvDev &env, const AgentDev &ag, int32_t cl, const double *Rw,
                                           const double *tf, const double *tl, Gen gen, uint8_t *flag, int lane,
                                           int32_t *stk, SweepCounters &cnt) {
    ++cnt.waves;
    double R[9], T0[3], TN[3];
    relative_transform(env.tf, env.tf + 9, Rw, tf, R, T0);
    env_rel_t(env, tl, TN);
#pragma unroll
    for (int i = 0; i < 9; ++i) R[i] = uniform_d(R[i]);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        T0[i] = uniform_d(T0[i]);
        TN[i] = uniform_d(TN[i]);
    }
    const Cluster c = ag.clusters[cl];
    float clo[3], chi[3];
    {
        float alo[3], ahi[3], blo[3], bhi[3];
        local_box(c.c, c.e, R, T0, alo, ahi);
        local_box(c.c, c.e, R, TN, blo, bhi);
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            clo[k] = fminf(alo[k], blo[k]);
            chi[k] = fmaxf(ahi[k], bhi[k]);
        }
    }
    // the lane's triangle rotated once (R Q, xform's products and sums before the + T)
    const bool act = lane < c.count;
    v3 RQ[3] = {mk(0, 0, 0), mk(0, 0, 0), mk(0, 0, 0)};
    float tlo[3] = {0, 0, 0}, thi[3] = {0, 0, 0};
    if (act) {
        const double *t = ag.tris + (int64_t)(c.first + lane) * 9;
#pragma unroll
        for (int v = 0; v < 3; ++v) {
            const double x = t[3 * v], y = t[3 * v + 1], z = t[3 * v + 2];
            RQ[v] = mk(R[0] * x + R[1] * y + R[2] * z, R[3] * x + R[4] * y + R[5] * z, R[6] * x + R[7] * y + R[8] * z);
        }
        // swept box of the triangle: its boxes at both ends (translation only in between)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const double a0 = (&RQ[0].x)[k], a1 = (&RQ[1].x)[k], a2 = (&RQ[2].x)[k];
            const double mn = dmin(a0, dmin(a1, a2)), mx = dmax(a0, dmax(a1, a2));
            tlo[k] = widen_lo(dmin(mn + T0[k], mn + TN[k]));
            thi[k] = widen_hi(dmax(mx + T0[k], mx + TN[k]));
        }
    }
    int sp = 0;
    int lev = env.n_levels - 1;
    int32_t first = env.lev_off[lev];
    int32_t count = env.lev_off[lev + 1] - first;
    for (;;) {
        bool keep = false;
        int32_t cf = 0, cc = 0;
        if (lane < count) {
            const Item it = env.items[first + lane];
            keep = box_overlap(clo, chi, it.lo, it.hi);
            cf = it.first;
            cc = it.count;
        }
        cnt.items += (uint32_t)count;
        uint64_t m = __ballot(keep);
        if (lev == 0) {
            // env triangles: lanes whose swept box meets one run its poses
            while (m) {
                const int j = __ffsll((unsigned long long)m) - 1;
                m &= m - 1;
                const int32_t t = first + j;
                const Item ti = env.items[t];  // level 0: item index = triangle index
                const bool near = act && box_overlap(tlo, thi, ti.lo, ti.hi);
                if (!__ballot(near)) continue;
                if (load_flag(flag)) return;
                const EnvTri &E = env.tris[t];
                bool hit = false;
                if (near) {
                    gen([&](const double *tw) {
                        double Tp[3];
                        env_rel_t(env, tw, Tp);
                        const v3 Q1 = mk(RQ[0].x + Tp[0], RQ[0].y + Tp[1], RQ[0].z + Tp[2]);
                        const v3 Q2 = mk(RQ[1].x + Tp[0], RQ[1].y + Tp[1], RQ[1].z + Tp[2]);
                        const v3 Q3 = mk(RQ[2].x + Tp[0], RQ[2].y + Tp[1], RQ[2].z + Tp[2]);
                        ++cnt.pair_poses;
                        if (!tri_gate(E.lo, E.hi, Q1, Q2, Q3)) return false;
                        ++cnt.sat;
                        hit = tri_intersect(E, Q1, Q2, Q3);
                        return hit;
                    }, RQ, E, env);
                }
                if (__ballot(hit)) {
                    if (lane == 0) __hip_atomic_store(flag, (uint8_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    return;
                }
            }
        } else if (m) {
            // enter the first overlapping child, push the rest
            const int j = __ffsll((unsigned long long)m) - 1;
            const uint64_t rest = m & (m - 1);
            if (keep && lane != j) {
                const int pos = sp + (int)__popcll(rest & ((1ull << lane) - 1));
                stk[pos] = ((lev - 1) << 27) | cf;  // the child range: level, first
                stk[kSweepStack + pos] = cc;
            }
            sp += (int)__popcll(rest);
            first = __builtin_amdgcn_readlane(cf, j);  // j is uniform (a ballot's bit)
            count = __builtin_amdgcn_readlane(cc, j);
            lev -= 1;
            continue;
        }
        if (sp == 0) return;
        --sp;
        const int32_t code = __builtin_amdgcn_readfirstlane(stk[sp]);
        count = __builtin_amdgcn_readfirstlane(stk[kSweepStack + sp]);
        lev = code >> 27;
        first = code & ((1 << 27) - 1);
    }
}

// Where an edge's poses come from.  A source's edge(e, core) calls core(Rw, tf, tl, gen) with
// the edge's world rotation, its first and last pose's translation and the pose generator
// (gen(f, RQ, E, env): f(world translation) for each pose in order until f returns true --
// every pose whose translated triangle RQ + T may meet env triangle E's box), or returns
// without calling it when the edge has no poses.
// A PRM roadmap edge (prm_edges.h): the poses generated from the two milestones' keys with the
// pose stage's operations -- no pose array (config 4: ~20-115 M poses a roadmap) -- and, for a
// (triangle, env triangle) pair, only those whose gate can pass (PrmEdge::each_near)
struct PrmSrc {
    PrmEdges P;
    template <class Core>
    __device__ __forceinline__ void edge(int64_t e, Core &&core) const {
        PrmEdge g = prm_edge(P, e);
        // one edge a wave: every field is wave-uniform -- scalar registers, not ~40 VGPRs held
        // across the walk and the SAT
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            g.s[k] = uniform_d(g.s[k]);
            g.end[k] = uniform_d(g.end[k]);
            g.dx[k] = uniform_d(g.dx[k]);
        }
#pragma unroll
        for (int k = 0; k < 9; ++k) g.R[k] = uniform_d(g.R[k]);
        g.step = uniform_d(g.step);
        g.it = __builtin_amdgcn_readfirstlane(g.it);
        g.tail = __builtin_amdgcn_readfirstlane((int)g.tail) != 0;
        double tf[3], tl[3];
        g.first(tf);
        g.last(tl);
        core(g.R, tf, tl, [&](auto &&f, const v3 *RQ, const EnvTri &E, const EnvDev &env) {
            g.each_near(f, RQ, E.lo, E.hi, env.tf);
        });
    }
};

// one wave an (edge, cluster) (agents of more than 64 clusters)
template <class Src>
__global__ __launch_bounds__(kSweepWaves * 64) void k_sweep(EnvDev env, const AgentDev *__restrict__ link, Src src,
                                                            int64_t E, int32_t n_clusters, uint8_t *verdict,
                                                            unsigned long long *stats) {
    __shared__ int32_t s_stk[kSweepWaves][2 * kSweepStack];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int64_t g = (int64_t)blockIdx.x * kSweepWaves + wave;
    const int64_t e = g / n_clusters;
    const int32_t cl = (int32_t)(g % n_clusters);
    SweepCounters cnt;
    if (e < E && !load_flag(verdict + e))
        src.edge(e, [&](const double *Rw, const double *tf, const double *tl, auto &&gen) {
            sweep_core(env, link[0], cl, Rw, tf, tl, gen, verdict + e, lane, s_stk[wave], cnt);
        });
    if (stats && lane == 0 && cnt.waves) {
        atomicAdd(stats + 0, (unsigned long long)cnt.waves);
        atomicAdd(stats + 1, (unsigned long long)cnt.items);
        atomicAdd(stats + 2, (unsigned long long)cnt.pair_poses);
        atomicAdd(stats + 3, (unsigned long long)cnt.sat);
    }
}

// PRMLite::generateEdges (discretizations/workspace/prmlite.hpp:128-164, interpolate :181-203):
// pair e = (i, j), i < j row-major; steps = (unsigned)(|t_i - t_j| / step) poses, each one
// vecStep = (t_j - t_i) / steps further (accumulated, as setTransform(q1, T + vecStep)), all
// with vertex i's rotation; no poses = safe.
__global__ __launch_bounds__(kSweepWaves * 64) void k_sweep_lite(EnvDev env, const AgentDev *__restrict__ link,
                                                                 const double *__restrict__ verts, int64_t V,
                                                                 double step, int64_t E, int32_t n_clusters,
                                                                 uint8_t *hit, unsigned long long *stats) {
    __shared__ int32_t s_stk[kSweepWaves][2 * kSweepStack];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int64_t g = (int64_t)blockIdx.x * kSweepWaves + wave;
    const int64_t e = g / n_clusters;
    const int32_t cl = (int32_t)(g % n_clusters);
    SweepCounters cnt;
    if (e < E && !load_flag(hit + e)) {
        // pair index -> (i, j): row i holds V - 1 - i pairs
        const double b = 2.0 * (double)V - 1.0;
        int64_t i = (int64_t)((b - sqrt(b * b - 8.0 * (double)e)) * 0.5);
        if (i < 0) i = 0;
        while (i > 0 && i * (2 * V - i - 1) / 2 > e) --i;
        while ((i + 1) * (2 * V - i - 2) / 2 <= e) ++i;
        const int64_t j = e - i * (2 * V - i - 1) / 2 + i + 1;
        const double *ti = verts + i * 12, *tj = verts + j * 12;
        const double *v1 = ti + 9, *v2 = tj + 9;
        const double df[3] = {v1[0] - v2[0], v1[1] - v2[1], v1[2] - v2[2]};
        const double dist = sqrt(df[0] * df[0] + df[1] * df[1] + df[2] * df[2]);
        const double q = dist / step;
        const unsigned steps = (q >= 4294967296.0 || !(q >= 0)) ? 0u : (unsigned)q;
        if (steps > 0) {
            const double vs[3] = {(v2[0] - v1[0]) / (double)steps, (v2[1] - v1[1]) / (double)steps,
                                  (v2[2] - v1[2]) / (double)steps};
            double tf[3] = {v1[0] + vs[0], v1[1] + vs[1], v1[2] + vs[2]}, tl[3] = {v1[0], v1[1], v1[2]};
            for (unsigned s = 0; s < steps; ++s)
                for (int k = 0; k < 3; ++k) tl[k] = tl[k] + vs[k];
            sweep_core(env, link[0], cl, ti, tf, tl,
                       [&](auto &&f, const v3 *, const EnvTri &, const EnvDev &) {
                           double t[3] = {v1[0], v1[1], v1[2]};
                           for (unsigned s = 0; s < steps; ++s) {
                               for (int k = 0; k < 3; ++k) t[k] = t[k] + vs[k];
                               if (f(t)) return;
                           }
                       },
                       hit + e, lane, s_stk[wave], cnt);
        }
    }
    if (stats && lane == 0 && cnt.waves) {
        atomicAdd(stats + 0, (unsigned long long)cnt.waves);
        atomicAdd(stats + 1, (unsigned long long)cnt.items);
        atomicAdd(stats + 2, (unsigned long long)cnt.pair_poses);
        atomicAdd(stats + 3, (unsigned long long)cnt.sat);
    }
}

// ---- PRM edges (mpt_prm_connect's sweep path), four launches over the roadmap:
//  0. k_sweep_prm over every edge, each (triangle, env triangle) pair at its middle pose only
//     (kSweepCoarse): one wave an edge walks the env tree (prm_walk), the gate-passing triples
//     go through the SAT 64 at a time, the edge ending at its first contact -- a contact with a
//     wall lasts many poses, so this decides nearly every colliding edge (config 4 at --bounds
//     rooms: 44 % of the edges collide);
//  1. k_sweep_cands over the undecided edges: the walk again, (edge, agent triangle, env
//     triangle, pose range) candidates, at most kSweepEdgeCands an edge: an edge that reaches
//     the cap stops and is listed;
//  2. k_sweep_sat: the gate + SAT over each candidate's poses, one candidate a lane (full waves
//     at full occupancy): the free edges, ~430 k candidates a roadmap;
//  3. k_sweep_prm over the listed edges (~5 000): the poses step 0 skipped.
// Verdicts are the same set: every (edge, agent triangle, env triangle, pose) the reference
// tests either is in some candidate or in one of k_sweep_prm's two pose sets (same fan-out, same
// box tests, the same pose interval), each with the same operations, and a contact found
// anywhere is a contact.

struct SweepCand {
    int32_t e, atri, etri;
    uint32_t q0, q1t;  // poses [q0, q1) of the edge's sequence, then its tail pose when bit 31 of q1t is set
};
constexpr int kSweepStage = 128;  // a wave's candidates staged in LDS before one atomic reserves their slots
constexpr int kSweepChunk = 8;    // poses a candidate covers at most

struct SweepQueue {
    SweepCand *c;
    uint32_t *n;  // [0] candidates written (may pass cap), [1] edges a full queue stopped
    uint32_t cap;
    int32_t *fused;       // [E] edges a full queue stopped (k_sweep_prm decides them)
    const int32_t *in_e;  // this pass's edges (null: every edge) and their resume indices
    const uint32_t *in_r;
    const uint32_t *n_in;
    int32_t *out_e;  // the edges this pass capped: the next pass resumes them
    uint32_t *out_r;
    uint32_t *n_out;
    uint32_t edge_cap;  // candidates an edge emits at most in this pass
};
// The passes: each emits an edge's candidates from where its previous pass stopped (its resume
// index: candidates are numbered in the walk's order, which is the same every pass) up to the
// pass's per-edge cap, then the SAT launch decides what it can; an edge still undecided at the
// cap goes to the next pass with a larger cap; after the last pass k_sweep_prm takes the edges
// still undecided.  Emitting every candidate of an edge at once (config 4 at --bounds rooms:
// some edges emit thousands) cost a second a roadmap.  Config 4 at --bounds rooms, collision ms
// by the number of passes (first cap 64, x4 a pass, as far as the queue holds; the tail then in
// the round's first single-kernel sweep): 1: 47.5, 2: 52.0, 3: 52.9, 4: 60.2 -- an edge a pass
// leaves undecided mostly stays so over hundreds more candidates, whose SATs a pass runs in
// parallel where the walk kernels stop at the edge's first contact; caps 512 / 2048 in one
// pass: 53 / 53.
constexpr int kSweepEdgeCands = 64;  // the first pass's cap; x4 a pass
constexpr int kSweepPasses = 1;      // then k_sweep_prm takes what is left
// k_sweep_prm's first pose stride, its poses centred on each pair's interval: 1024 exceeds
// nearly every interval, so the first pass tests each pair's middle pose (config 4 at --bounds
// rooms, collision ms on one box: stride 8: 14.8, 16: 14.3, 1024: 14.1; with the first pose at
// the interval's start instead of its middle: no coarse pass 30.8, stride 4: 19.1, 8: 17.9, 16:
// 23.9; the coarse pass over every edge before the candidates instead: 20.0, and over every
// edge with no candidates at all: 21.2).  The middle-pose pass then went first, over every edge
// (step 0 above): 13.9 -> 10.3 ms (without the candidate pass after it: 10.45)
constexpr unsigned kSweepCoarse = 1024;

// false when the queue is full: the wave's edge is then deferred (the candidates that did fit
// are tested all the same, which is harmless: a contact among them is a contact)
__device__ __forceinline__ bool sweep_flush(SweepCand *buf, int nb, const SweepQueue &Q, int lane) {
    if (nb <= 0) return true;
    // a queue already full takes no more reservations, so the counter stays within cap plus
    // one stage a running wave (no u32 wrap however many edges are deferred)
    uint32_t base = 0;
    if (lane == 0) {
        base = __hip_atomic_load(Q.n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (base < Q.cap) base = atomicAdd(Q.n, (uint32_t)nb);
    }
    base = __builtin_amdgcn_readfirstlane(base);
    if (base >= Q.cap) return false;
    for (int i = lane; i < nb; i += kWave)
        if ((uint64_t)base + (uint64_t)i < Q.cap) Q.c[base + i] = buf[i];
    return (uint64_t)base + (uint64_t)nb <= Q.cap;
}

// A PRM edge for one wave: every field wave-uniform (scalar registers), and the env-relative
// rotation R and translations T0 / TN of its first and last pose
__device__ __forceinline__ PrmEdge prm_edge_uniform(const PrmEdges &P, int64_t e) {
    PrmEdge g = prm_edge(P, e);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        g.s[k] = uniform_d(g.s[k]);
        g.end[k] = uniform_d(g.end[k]);
        g.dx[k] = uniform_d(g.dx[k]);
    }
#pragma unroll
    for (int k = 0; k < 9; ++k) g.R[k] = uniform_d(g.R[k]);
    g.step = uniform_d(g.step);
    g.it = __builtin_amdgcn_readfirstlane(g.it);
    g.tail = __builtin_amdgcn_readfirstlane((int)g.tail) != 0;
    return g;
}

__device__ __forceinline__ void prm_edge_frame(const EnvDev &env, const PrmEdge &g, double R[9], double T0[3],
                                               double TN[3]) {
    double tf[3], tl[3];
    g.first(tf);
    g.last(tl);
    relative_transform(env.tf, env.tf + 9, g.R, tf, R, T0);
    env_rel_t(env, tl, TN);
#pragma unroll
    for (int i = 0; i < 9; ++i) R[i] = uniform_d(R[i]);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        T0[i] = uniform_d(T0[i]);
        TN[i] = uniform_d(TN[i]);
    }
}

// the agent triangle a rotated (R Q, xform's products and sums before the + T)
__device__ __forceinline__ void rotate_tri(const AgentDev &ag, int32_t a, const double *R, v3 RQ[3]) {
    const double *tr = ag.tris + (int64_t)a * 9;
#pragma unroll
    for (int v = 0; v < 3; ++v) {
        const double x = tr[3 * v], y = tr[3 * v + 1], z = tr[3 * v + 2];
        RQ[v] = mk(R[0] * x + R[1] * y + R[2] * z, R[3] * x + R[4] * y + R[5] * z, R[6] * x + R[7] * y + R[8] * z);
    }
}

// One wave an edge, every agent cluster (at most 64: lane c holds cluster c): the wave walks the
// env tree once against the union of the clusters' swept boxes and fans out to the clusters only
// at the env triangles that meet it, each cluster rotated once a bucket.  visit(c, t, act, RQ, elo, ehi)
// runs for each (cluster c, env triangle t) with a lane (act: one of c's triangles, rotated in
// RQ) whose swept triangle box meets t's item box elo / ehi (near); a true from it (wave-uniform)
// ends the walk.
template <class Visit>
__device__ __forceinline__ void prm_walk(const EnvDev &env, const AgentDev &ag, const double *R, const double *T0,
                                         const double *TN, int lane, int32_t *stk, SweepCounters &cnt, double *rq_lds,
                                         Visit &&visit) {
    const int ncl = ag.n_clusters;
    float clo[3] = {__builtin_huge_valf(), __builtin_huge_valf(), __builtin_huge_valf()};
    float chi[3] = {-__builtin_huge_valf(), -__builtin_huge_valf(), -__builtin_huge_valf()};
    if (lane < ncl) {  // lane c: cluster c's box swept along the edge
        const Cluster c = ag.clusters[lane];
        float alo[3], ahi[3], blo[3], bhi[3];
        local_box(c.c, c.e, R, T0, alo, ahi);
        local_box(c.c, c.e, R, TN, blo, bhi);
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            clo[k] = fminf(alo[k], blo[k]);
            chi[k] = fmaxf(ahi[k], bhi[k]);
        }
    }
    float ulo[3], uhi[3];  // their union (uniform; DPP / permlane levels, wave_ops.h)
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        ulo[k] = wave_min_dpp(clo[k]);
        uhi[k] = wave_max_dpp(chi[k]);
    }
    bool stop = false;
    int sp = 0;
    int lev = env.n_levels - 1;
    int32_t first = env.lev_off[lev];
    int32_t count = env.lev_off[lev + 1] - first;
    for (;;) {
        bool keep = false;
        int32_t cf = 0, cc = 0;
        float ilo[3] = {0, 0, 0}, ihi[3] = {0, 0, 0};
        if (lane < count) {
            const Item it = env.items[first + lane];
            keep = box_overlap(ulo, uhi, it.lo, it.hi);
            cf = it.first;
            cc = it.count;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                ilo[k] = it.lo[k];
                ihi[k] = it.hi[k];
            }
        }
        cnt.items += (uint32_t)count;
        uint64_t m = __ballot(keep);
        if (lev == 0) {
            uint64_t Tm = 0;  // lane c: the bucket's triangles cluster c's swept box meets
            for (uint64_t mm = m; mm; mm &= mm - 1) {
                const int j = __ffsll((unsigned long long)mm) - 1;
                const float elo[3] = {lane_f(ilo[0], j), lane_f(ilo[1], j), lane_f(ilo[2], j)};
                const float ehi[3] = {lane_f(ihi[0], j), lane_f(ihi[1], j), lane_f(ihi[2], j)};
                if (lane < ncl && box_overlap(clo, chi, elo, ehi)) Tm |= 1ull << j;
            }
            for (uint64_t C = __ballot(Tm != 0); C && !stop; C &= C - 1) {
                const int ci = __ffsll((unsigned long long)C) - 1;
                const uint32_t Th = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(Tm >> 32), ci);
                uint64_t Tc = ((uint64_t)Th << 32) | (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)Tm, ci);
                const Cluster c = ag.clusters[ci];
                const bool act = lane < c.count;
                v3 RQ[3] = {mk(0, 0, 0), mk(0, 0, 0), mk(0, 0, 0)};
                float tlo[3] = {0, 0, 0}, thi[3] = {0, 0, 0};
                if (act) {
                    rotate_tri(ag, c.first + lane, R, RQ);
#pragma unroll
                    for (int k = 0; k < 3; ++k) {  // its box swept along the edge
                        const double a0 = (&RQ[0].x)[k], a1 = (&RQ[1].x)[k], a2 = (&RQ[2].x)[k];
                        const double mn = dmin(a0, dmin(a1, a2)), mx = dmax(a0, dmax(a1, a2));
                        tlo[k] = widen_lo(dmin(mn + T0[k], mn + TN[k]));
                        thi[k] = widen_hi(dmax(mx + T0[k], mx + TN[k]));
                    }
                    if (rq_lds) {  // the visitor reads it where it needs it (not held across its SATs)
#pragma unroll
                        for (int v = 0; v < 3; ++v) {
                            rq_lds[lane * 9 + 3 * v] = RQ[v].x;
                            rq_lds[lane * 9 + 3 * v + 1] = RQ[v].y;
                            rq_lds[lane * 9 + 3 * v + 2] = RQ[v].z;
                        }
                    }
                }
                __builtin_amdgcn_wave_barrier();
                for (; Tc && !stop; Tc &= Tc - 1) {
                    const int j = __ffsll((unsigned long long)Tc) - 1;
                    const float elo[3] = {lane_f(ilo[0], j), lane_f(ilo[1], j), lane_f(ilo[2], j)};
                    const float ehi[3] = {lane_f(ihi[0], j), lane_f(ihi[1], j), lane_f(ihi[2], j)};
                    const bool near = act && box_overlap(tlo, thi, elo, ehi);
                    if (!__ballot(near)) continue;
                    stop = visit(c, first + j, near, RQ, elo, ehi);  // level 0: item index = triangle index
                }
            }
        } else if (m) {
            const int j = __ffsll((unsigned long long)m) - 1;
            const uint64_t rest = m & (m - 1);
            if (keep && lane != j) {
                const int pos = sp + (int)__popcll(rest & ((1ull << lane) - 1));
                stk[pos] = ((lev - 1) << 27) | cf;
                stk[kSweepStack + pos] = cc;
            }
            sp += (int)__popcll(rest);
            first = __builtin_amdgcn_readlane(cf, j);  // j is uniform (a ballot's bit)
            count = __builtin_amdgcn_readlane(cc, j);
            lev -= 1;
            continue;
        }
        if (sp == 0 || stop) return;
        --sp;
        const int32_t code = __builtin_amdgcn_readfirstlane(stk[sp]);
        count = __builtin_amdgcn_readfirstlane(stk[kSweepStack + sp]);
        lev = code >> 27;
        first = code & ((1 << 27) - 1);
    }
}

// One wave an edge: prm_walk, a candidate per near lane whose pose interval is not empty
__global__ __launch_bounds__(kSweepWaves * 64) void k_sweep_cands(EnvDev env, const AgentDev *__restrict__ link,
                                                                  PrmEdges P, int64_t E, const uint8_t *verdict,
                                                                  SweepQueue Q, unsigned long long *stats) {
    __shared__ int32_t s_stk[kSweepWaves][2 * kSweepStack];
    __shared__ SweepCand s_buf[kSweepWaves][kSweepStage];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    SweepCounters cnt;
    SweepCand *buf = s_buf[wave];
    const int64_t n_list = Q.in_e ? (int64_t)*Q.n_in : E;
    for (int64_t i = (int64_t)blockIdx.x * kSweepWaves + wave; i < n_list; i += (int64_t)gridDim.x * kSweepWaves) {
        const int64_t e = Q.in_e ? Q.in_e[i] : i;
        const uint32_t skip = Q.in_e ? __builtin_amdgcn_readfirstlane(Q.in_r[i]) : 0u;
        const uint32_t upto = skip + Q.edge_cap;
        uint32_t n_edge = 0;  // candidates numbered so far (those below skip were emitted by an earlier pass)
        int nb = 0;
        bool stop = false, full = false;
        if (!load_flag(verdict + e)) {
            const PrmEdge g = prm_edge_uniform(P, e);
            ++cnt.waves;
            double R[9], T0[3], TN[3];
            prm_edge_frame(env, g, R, T0, TN);
            prm_walk(env, link[0], R, T0, TN, lane, s_stk[wave], cnt, nullptr,
                     [&](const Cluster &c, int32_t t, bool near, const v3 *RQ, const float *elo, const float *ehi) {
                         unsigned q0 = 0, q1 = 0;
                         bool tail_too = false, emit = false;
                         if (near) {
                             // the item box (widened floats) holds the triangle's exact box: its
                             // interval holds the exact gate's poses
                             const double elod[3] = {elo[0], elo[1], elo[2]}, ehid[3] = {ehi[0], ehi[1], ehi[2]};
                             g.near_range(RQ, elod, ehid, env.tf, q0, q1, tail_too);
                             emit = q1 > q0 || tail_too;
                         }
                         // a lane's poses go out in chunks of at most kSweepChunk (the tail pose
                         // with the last): the SAT launch then runs equal short loops a lane
                         // instead of each wave waiting for its longest interval
                         for (uint64_t em = __ballot(emit); em && !stop; em = __ballot(emit)) {
                             const int ne = __popcll(em);
                             const bool fresh = n_edge >= skip;  // a step boundary: all or none of it
                             if (fresh && nb + ne > kSweepStage) {
                                 if (!sweep_flush(buf, nb, Q, lane)) stop = full = true;
                                 nb = 0;
                                 if (stop) break;
                             }
                             if (emit) {
                                 const int rank = __popcll(em & ((1ull << lane) - 1ull));
                                 const bool last = q1 - q0 <= (unsigned)kSweepChunk;
                                 const unsigned qe = last ? q1 : q0 + kSweepChunk;
                                 if (fresh)
                                     buf[nb + rank] = SweepCand{(int32_t)e, c.first + lane, t, q0,
                                                                qe | (last && tail_too ? 0x80000000u : 0u)};
                                 q0 = qe;
                                 emit = !last;
                             }
                             if (fresh) nb += ne;
                             n_edge += (uint32_t)ne;
                             if (n_edge >= upto) stop = true;  // wave-uniform: the next pass resumes here
                             __builtin_amdgcn_wave_barrier();
                         }
                         return stop;
                     });
        }
        __builtin_amdgcn_wave_barrier();
        if (!full && !sweep_flush(buf, nb, Q, lane)) stop = full = true;
        if (lane == 0 && full) {
            Q.fused[atomicAdd(Q.n + 1, 1u)] = (int32_t)e;
        } else if (lane == 0 && stop) {
            const uint32_t k = atomicAdd(Q.n_out, 1u);
            Q.out_e[k] = (int32_t)e;
            Q.out_r[k] = n_edge;
        }
        __builtin_amdgcn_wave_barrier();
    }
    if (stats && lane == 0 && cnt.waves) {
        atomicAdd(stats + 0, (unsigned long long)cnt.waves);
        atomicAdd(stats + 1, (unsigned long long)cnt.items);
    }
}

// ---- k_sweep_prm: prm_walk, then for each near lane the poses of its interval in step over the
// wave (every stride-th, or the ones a coarse pass at that stride skipped plus the tail), each
// pose's exact gate; the (triangle, env triangle, pose) triples that pass go to a per-wave LDS
// list, and each 64 of them run the SAT one a lane.  The round-5 single-kernel sweep (removed)
// ran a SAT wherever any lane's gate passed: ~2.5 us of FP64 a wave for a lane or two, and at
// config 4 --bounds rooms a colliding edge took up to 7000 of them before its contact (its tail
// of ~105 k edges: 38 ms; batched: 24 ms; coarse poses first: 12 ms).  The edge stops at the
// batch holding its first contact.  Same verdicts: every (pair, pose) whose gate passes is
// tested, with the reference's operations (R Q recomputed from the triangle by the walk's
// expression, the pose by PrmEdge::pose).
struct SatTriple {
    int32_t atri, etri;
    uint32_t q;
};
constexpr int kSatBatch = 64;

// the SATs of list[0, n) (n <= 64), one a lane; true: a contact
__device__ __forceinline__ bool prm_sat_batch(const EnvDev &env, const AgentDev &ag, const PrmEdge &g, const double *R,
                                              const SatTriple *list, int n, int lane) {
    bool hit = false;
    if (lane < n) {
        const SatTriple s = list[lane];
        v3 RQ[3];
        rotate_tri(ag, s.atri, R, RQ);
        double t[3], Tp[3];
        g.pose(s.q, t);
        env_rel_t(env, t, Tp);
        const v3 Q1 = mk(RQ[0].x + Tp[0], RQ[0].y + Tp[1], RQ[0].z + Tp[2]);
        const v3 Q2 = mk(RQ[1].x + Tp[0], RQ[1].y + Tp[1], RQ[1].z + Tp[2]);
        const v3 Q3 = mk(RQ[2].x + Tp[0], RQ[2].y + Tp[1], RQ[2].z + Tp[2]);
        hit = tri_intersect(env.tris[s.etri], Q1, Q2, Q3);
    }
    return __ballot(hit) != 0;
}

// 3 waves a SIMD: the lanes' rotated triangles live in LDS (prm_walk's copy, re-read each pose
// step), 211 -> 164 VGPRs, no VGPR spill (config 4 at --bounds rooms: collision 17.9 -> 16.0 ms;
// at 4 waves 24 VGPRs spill: 15.9 ms)
template <unsigned stride>
__global__ __launch_bounds__(kSweepWaves * 64) __attribute__((amdgpu_waves_per_eu(3))) void k_sweep_prm(EnvDev env, const AgentDev *__restrict__ link,
                                                                PrmEdges P, const int32_t *__restrict__ list,
                                                                const uint32_t *__restrict__ n_list, int64_t E,
                                                                bool rest, uint32_t *next, uint8_t *verdict,
                                                                unsigned long long *stats) {
    __shared__ int32_t s_stk[kSweepWaves][2 * kSweepStack];
    __shared__ SatTriple s_sat[kSweepWaves][2 * kSatBatch];
    __shared__ double s_rq[kSweepWaves][kWave * 9];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    SweepCounters cnt;
    SatTriple *sat = s_sat[wave];
    const AgentDev &ag = link[0];
    const int64_t n = list ? (int64_t)*n_list : E;
    // edges taken one at a time from a shared counter (an edge's cost runs from a walk with no
    // pair to thousands of gates: a fixed stride left waves with a run of costly ones last)
    for (;;) {
        uint32_t ni = 0;
        if (lane == 0) ni = atomicAdd(next, 1u);
        const int64_t i = (int64_t)__builtin_amdgcn_readfirstlane((int)ni);
        if (i >= n) break;
        const int64_t e = list ? list[i] : i;
        if (load_flag(verdict + e)) continue;
        const PrmEdge g = prm_edge_uniform(P, e);
        ++cnt.waves;
        double R[9], T0[3], TN[3];
        prm_edge_frame(env, g, R, T0, TN);
        int ns = 0;  // triples listed
        bool hit = false;
        double *rq = s_rq[wave];
        prm_walk(env, ag, R, T0, TN, lane, s_stk[wave], cnt, rq,
                 [&](const Cluster &c, int32_t t, bool near, const v3 *, const float *, const float *) {
                     const EnvTri &Et = env.tris[t];
                     double elo[3], ehi[3];
#pragma unroll
                     for (int k = 0; k < 3; ++k) {
                         elo[k] = uniform_d(Et.lo[k]);
                         ehi[k] = uniform_d(Et.hi[k]);
                     }
                     // the lane's rotated triangle from LDS (prm_walk's copy): read again in each
                     // pose step, so no register holds it across the SAT batches
                     auto rq_of = [&](v3 *RQ) {
#pragma unroll
                         for (int v = 0; v < 3; ++v)
                             RQ[v] = mk(rq[lane * 9 + 3 * v], rq[lane * 9 + 3 * v + 1], rq[lane * 9 + 3 * v + 2]);
                     };
                     unsigned q0 = 0, q1 = 0;
                     bool tail_too = false;
                     if (near) {
                         v3 RQ[3];
                         rq_of(RQ);
                         g.near_range(RQ, elo, ehi, env.tf, q0, q1, tail_too);
                     }
                     // coarse (stride > 1): every stride-th pose of the run, its middle among them
                     // (the run is the box-overlap interval widened a pose or two each side: with
                     // q0 first, a run shorter than the stride tested only a widened end); then
                     // the rest (rest: the poses a coarse pass at that stride skipped, and the tail)
                     const unsigned run = q1 - q0, off = (run / 2) % stride;
                     const unsigned coarse = run > off ? (run - off + stride - 1) / stride : 0u;
                     const unsigned nmain = rest ? run - coarse : coarse;
                     const unsigned np = near ? nmain + (tail_too && (rest || stride == 1) ? 1u : 0u) : 0u;
                     for (unsigned j = 0;; ++j) {
                         const bool more = j < np;
                         const uint64_t mm = __ballot(more);
                         if (!mm) break;
                         cnt.pair_poses += (uint32_t)__popcll(mm);
                         bool pass = false;
                         const unsigned jb = stride > 1 ? j / (stride - 1) : 0u, jo = j - jb * (stride - 1);
                         const unsigned jr = rest ? jb * stride + (jo < off ? jo : jo + 1) : off + j * stride;
                         const unsigned q = j < nmain ? q0 + jr : g.it;  // past the run: the tail
                         if (more) {
                             double tw[3], Tp[3];
                             v3 RQ[3];
                             asm volatile("" ::: "memory");  // the LDS copy is read here, every step
                             rq_of(RQ);
                             g.pose(q, tw);
                             env_rel_t(env, tw, Tp);
                             const v3 Q1 = mk(RQ[0].x + Tp[0], RQ[0].y + Tp[1], RQ[0].z + Tp[2]);
                             const v3 Q2 = mk(RQ[1].x + Tp[0], RQ[1].y + Tp[1], RQ[1].z + Tp[2]);
                             const v3 Q3 = mk(RQ[2].x + Tp[0], RQ[2].y + Tp[1], RQ[2].z + Tp[2]);
                             pass = tri_gate(elo, ehi, Q1, Q2, Q3);
                         }
                         const uint64_t pm = __ballot(pass);
                         if (!pm) continue;
                         if (pass) sat[ns + __popcll(pm & ((1ull << lane) - 1ull))] = SatTriple{c.first + lane, t, q};
                         ns += __popcll(pm);
                         if (ns >= kSatBatch) {
                             __builtin_amdgcn_wave_barrier();
                             cnt.sat += kSatBatch;
                             if (prm_sat_batch(env, ag, g, R, sat, kSatBatch, lane)) {
                                 hit = true;
                                 return true;
                             }
                             ns -= kSatBatch;  // < 64 left past the batch: to the front
                             SatTriple rest{};
                             if (lane < ns) rest = sat[kSatBatch + lane];
                             __builtin_amdgcn_wave_barrier();
                             if (lane < ns) sat[lane] = rest;
                             __builtin_amdgcn_wave_barrier();
                         }
                     }
                     return false;
                 });
        if (!hit && ns > 0) {
            __builtin_amdgcn_wave_barrier();
            cnt.sat += (uint32_t)ns;
            hit = prm_sat_batch(env, ag, g, R, sat, ns, lane);
        }
        if (hit && lane == 0) __hip_atomic_store(verdict + e, (uint8_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_wave_barrier();
    }
    if (stats && lane == 0 && cnt.waves) {
        atomicAdd(stats + 0, (unsigned long long)cnt.waves);
        atomicAdd(stats + 1, (unsigned long long)cnt.items);
        atomicAdd(stats + 2, (unsigned long long)cnt.pair_poses);
        atomicAdd(stats + 3, (unsigned long long)cnt.sat);
    }
}

// One candidate a lane (a resident grid striding over them): the edge's rotation and its
// poses regenerated (prm_edge: the same operations as the walk's), the agent triangle rotated
// (R Q) and, over the candidate's poses, Q' = R Q + T', the exact gate and intersect_Triangle
__global__ __launch_bounds__(256) void k_sweep_sat(EnvDev env, const AgentDev *__restrict__ link, PrmEdges P,
                                                   SweepQueue Q, uint8_t *verdict, unsigned long long *stats) {
    const uint32_t n = *Q.n < Q.cap ? *Q.n : Q.cap;
    uint32_t n_gate = 0, n_sat = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const SweepCand cd = Q.c[i];
        if (load_flag(verdict + cd.e)) continue;
        const PrmEdge g = prm_edge(P, cd.e);
        double tf[3], R[9], T0[3];
        g.first(tf);
        relative_transform(env.tf, env.tf + 9, g.R, tf, R, T0);
        const double *tr = link[0].tris + (int64_t)cd.atri * 9;
        v3 RQ[3];
#pragma unroll
        for (int v = 0; v < 3; ++v) {
            const double x = tr[3 * v], y = tr[3 * v + 1], z = tr[3 * v + 2];
            RQ[v] = mk(R[0] * x + R[1] * y + R[2] * z, R[3] * x + R[4] * y + R[5] * z, R[6] * x + R[7] * y + R[8] * z);
        }
        const EnvTri &E = env.tris[cd.etri];
        const unsigned q1 = cd.q1t & 0x7fffffffu;
        const unsigned np = (q1 - cd.q0) + (cd.q1t >> 31);
        for (unsigned j = 0; j < np; ++j) {
            double t[3], Tp[3];
            if (j > 0 && load_flag(verdict + cd.e)) break;  // another lane found the edge's contact
            g.pose(cd.q0 + j < q1 ? cd.q0 + j : g.it, t);
            env_rel_t(env, t, Tp);
            const v3 Q1 = mk(RQ[0].x + Tp[0], RQ[0].y + Tp[1], RQ[0].z + Tp[2]);
            const v3 Q2 = mk(RQ[1].x + Tp[0], RQ[1].y + Tp[1], RQ[1].z + Tp[2]);
            const v3 Q3 = mk(RQ[2].x + Tp[0], RQ[2].y + Tp[1], RQ[2].z + Tp[2]);
            ++n_gate;
            if (!tri_gate(E.lo, E.hi, Q1, Q2, Q3)) continue;
            ++n_sat;
            if (tri_intersect(E, Q1, Q2, Q3)) {
                __hip_atomic_store(verdict + cd.e, (uint8_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
    }
    if (stats) {
        uint32_t a = n_gate, b = n_sat;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            a += __shfl_xor(a, off);
            b += __shfl_xor(b, off);
        }
        if ((threadIdx.x & 63) == 0 && (a | b)) {
            atomicAdd(stats + 2, (unsigned long long)a);
            atomicAdd(stats + 3, (unsigned long long)b);
        }
    }
}

void launch_prmlite_edges(const EnvDev &env, const AgentDev *d_link, int32_t n_clusters, const double *verts, int64_t V,
                          double step, uint8_t *hit, unsigned long long *stats, hipStream_t stream) {
    const int64_t E = V * (V - 1) / 2;
    if (E <= 0 || env.n_tris <= 0) return;
    const int64_t blocks = (E * n_clusters + kSweepWaves - 1) / kSweepWaves;
    if (blocks > 0x7fffffff) throw Error{5, "PRMLite batch too large"};
    hipLaunchKernelGGL(k_sweep_lite, dim3((unsigned)blocks), dim3(kSweepWaves * 64), 0, stream, env, d_link, verts, V,
                       step, E, n_clusters, hit, stats);
    hip_check(hipGetLastError(), "k_sweep_lite launch");
}

template <class Src>
static void launch_sweep_src(const EnvDev &env, const AgentDev *d_link, int32_t n_clusters, const Src &src, int64_t E,
                             uint8_t *verdict, unsigned long long *stats, hipStream_t stream) {
    if (E <= 0 || env.n_tris <= 0) return;
    if (env.n_tris >= (1 << 27)) throw Error{5, "env too large for the sweep path"};
    const int64_t waves = E * n_clusters;
    const int64_t blocks = (waves + kSweepWaves - 1) / kSweepWaves;
    if (blocks > 0x7fffffff) throw Error{5, "sweep batch too large"};
    hipLaunchKernelGGL(k_sweep<Src>, dim3((unsigned)blocks), dim3(kSweepWaves * 64), 0, stream, env, d_link, src, E,
                       n_clusters, verdict, stats);
    hip_check(hipGetLastError(), "k_sweep launch");
}

thread_local uint64_t last_sweep_counts[2] = {0, 0};
thread_local std::vector<int32_t> last_sweep_deferred;  // with counters on: the edges k_sweep_prm took
int64_t sweep_queue_cap_limit = 0;  // mpt_set_sweep_queue_cap: a test hook (0: the sized queue)

void launch_collide_sweep_prm(const EnvDev &env, const AgentDev *d_link, int32_t n_clusters, const PrmEdges &edges,
                              int64_t E, uint8_t *verdict, unsigned long long *stats, hipStream_t stream) {
    if (E <= 0 || env.n_tris <= 0) return;
    if (n_clusters > 64 || env.n_tris >= (1 << 27)) {
        launch_sweep_src(env, d_link, n_clusters, PrmSrc{edges}, E, verdict, stats, stream);
        return;
    }
    // the candidate queue and the pass lists, one set per thread of the caller's process
    // (mpt_prm_connect is per thread)
    struct Q {
        SweepCand *c = nullptr;
        int32_t *fused = nullptr, *le[2] = {nullptr, nullptr};
        uint32_t *lr[2] = {nullptr, nullptr};
        uint32_t *n = nullptr, *h = nullptr, *next = nullptr;
        int64_t cap = 0, ecap = 0;
        ~Q() {
            for (void *p : {(void *)c, (void *)fused, (void *)le[0], (void *)le[1], (void *)lr[0], (void *)lr[1],
                            (void *)n, (void *)next})
                if (p) (void)hipFree(p);
            if (h) (void)hipHostFree(h);
        }
    };
    static thread_local Q q;
    // 16 candidates an edge, at least 4 M (after step 0 the candidate pass sees the free edges:
    // config 4 at --bounds rooms queues ~1 an edge; an edge that finds the queue full goes to
    // k_sweep_prm's full pass instead, so the size decides speed only); later passes size their
    // caps to it
    const int64_t want = std::min<int64_t>(std::max<int64_t>(int64_t(1) << 22, 16 * E), int64_t(1) << 31);
    if (want > q.cap || E > q.ecap) {
        hip_check(hipStreamSynchronize(stream), "sync");
        for (void *p : {(void *)q.c, (void *)q.fused, (void *)q.le[0], (void *)q.le[1], (void *)q.lr[0],
                        (void *)q.lr[1]})
            if (p) hip_check(hipFree(p), "free");
        hip_check(hipMalloc(&q.c, sizeof(SweepCand) * (size_t)want), "sweep candidates");
        hip_check(hipMalloc(&q.fused, sizeof(int32_t) * (size_t)E), "sweep edge lists");
        for (int k = 0; k < 2; ++k) {
            hip_check(hipMalloc(&q.le[k], sizeof(int32_t) * (size_t)E), "sweep edge lists");
            hip_check(hipMalloc(&q.lr[k], sizeof(uint32_t) * (size_t)E), "sweep edge lists");
        }
        if (!q.n) hip_check(hipMalloc(&q.n, sizeof(uint32_t) * 4), "sweep counts");
        if (!q.next) hip_check(hipMalloc(&q.next, sizeof(uint32_t) * 8), "sweep edge counters");
        if (!q.h) hip_check(hipHostMalloc(&q.h, sizeof(uint32_t) * 4), "sweep counts");
        q.cap = want;
        q.ecap = E;
    }
    // the queue's capacity this call (a test shrinks it to drive the full-queue path)
    const int64_t qcap = sweep_queue_cap_limit > 0 ? std::min<int64_t>(q.cap, sweep_queue_cap_limit) : q.cap;
    int pass_no = 0;
    auto prm_pass = [&](const int32_t *list, const uint32_t *n_list, unsigned stride, bool rest) {
        uint32_t *next = q.next + (pass_no++ & 7);  // a counter a launch (zeroed below, once a call)
        if (stride == kSweepCoarse)
            hipLaunchKernelGGL(k_sweep_prm<kSweepCoarse>, dim3(4096), dim3(kSweepWaves * 64), 0, stream, env, d_link,
                               edges, list, n_list, E, rest, next, verdict, stats);
        else
            hipLaunchKernelGGL(k_sweep_prm<1>, dim3(4096), dim3(kSweepWaves * 64), 0, stream, env, d_link, edges, list,
                               n_list, E, false, next, verdict, stats);
        hip_check(hipGetLastError(), "k_sweep_prm launch");
    };
    hip_check(hipMemsetAsync(q.next, 0, sizeof(uint32_t) * 8, stream), "sweep counters zero");
    // 0. every edge's pairs at their middle poses (k_sweep_prm): decides nearly every colliding
    //    edge (a contact with a wall lasts many poses) before any candidate is queued
    prm_pass(nullptr, nullptr, kSweepCoarse, false);
    // n: [0] queue, [1] fused list, [2 + k] list k
    hip_check(hipMemsetAsync(q.n, 0, sizeof(uint32_t) * 4, stream), "sweep counts zero");
    uint64_t emitted = 0;
    int64_t n_in = E;
    uint32_t edge_cap = kSweepEdgeCands;
    int last = -1;  // the list the last pass wrote
    for (int pass = 0; pass < kSweepPasses && n_in > 0; ++pass) {
        const int o = pass & 1;
        if (pass > 0) hip_check(hipMemsetAsync(q.n, 0, sizeof(uint32_t), stream), "sweep counts zero");
        hip_check(hipMemsetAsync(q.n + 2 + o, 0, sizeof(uint32_t), stream), "sweep counts zero");
        SweepQueue Qd{q.c, q.n, (uint32_t)std::min<int64_t>(qcap, 0xffffffffLL), q.fused,
                      pass ? q.le[1 - o] : nullptr, pass ? q.lr[1 - o] : nullptr, q.n + 2 + (1 - o),
                      q.le[o], q.lr[o], q.n + 2 + o, edge_cap};
        const int64_t blocks = pass ? std::min<int64_t>(4096, (n_in + kSweepWaves - 1) / kSweepWaves)
                                    : (E + kSweepWaves - 1) / kSweepWaves;
        if (blocks > 0x7fffffff) throw Error{5, "sweep batch too large"};
        hipLaunchKernelGGL(k_sweep_cands, dim3((unsigned)blocks), dim3(kSweepWaves * 64), 0, stream, env, d_link,
                           edges, E, verdict, Qd, stats);
        hip_check(hipGetLastError(), "k_sweep_cands launch");
        hipLaunchKernelGGL(k_sweep_sat, dim3(4096), dim3(256), 0, stream, env, d_link, edges, Qd, verdict, stats);
        hip_check(hipGetLastError(), "k_sweep_sat launch");
        hip_check(hipMemcpyAsync(q.h, q.n, sizeof(uint32_t) * 4, hipMemcpyDeviceToHost, stream), "sweep counts");
        hip_check(hipStreamSynchronize(stream), "sweep sync");
        emitted += q.h[0];
        n_in = q.h[2 + o];  // capped edges (some now decided: the next pass skips those)
        last = o;
        // the next cap: x4, as far as the queue holds every capped edge's share
        const int64_t fit = n_in > 0 ? qcap / n_in - kWave : 0;
        edge_cap = (uint32_t)std::max<int64_t>(kSweepEdgeCands, std::min<int64_t>(int64_t(edge_cap) * 4, fit));
    }
    // what the passes left (capped at the last pass, or stopped by a full queue): k_sweep_prm,
    // which skips the edges already decided -- the coarse poses, then the rest
    uint64_t to_fused = q.h[1];
    if (n_in > 0 && last >= 0) {
        prm_pass(q.le[last], q.n + 2 + last, kSweepCoarse, true);  // their middle poses were step 0's
        to_fused += (uint64_t)n_in;
    }
    if (q.h[1] > 0) prm_pass(q.fused, q.n + 1, 1u, false);
    last_sweep_deferred.clear();
    if (stats) {
        // diagnostics (mpt_prm_deferred_edges): the capped edges, then the full queue's
        const size_t a = (n_in > 0 && last >= 0) ? (size_t)n_in : 0, b = q.h[1];
        last_sweep_deferred.resize(a + b);
        if (a) hip_check(hipMemcpyAsync(last_sweep_deferred.data(), q.le[last], sizeof(int32_t) * a,
                                        hipMemcpyDeviceToHost, stream), "deferred edges");
        if (b) hip_check(hipMemcpyAsync(last_sweep_deferred.data() + a, q.fused, sizeof(int32_t) * b,
                                        hipMemcpyDeviceToHost, stream), "deferred edges");
    }
    hip_check(hipStreamSynchronize(stream), "sweep sync");
    last_sweep_counts[0] = emitted;    // candidates emitted over the passes
    last_sweep_counts[1] = to_fused;  // edges left to k_sweep_prm
}

}  // namespace mpt
