// collide_common.h -- device helpers shared by the fused (collide.hip) and the two-phase
// (broad.hip) collision paths.
#pragma once
#include "mpt_internal.h"

namespace mpt {

__device__ __forceinline__ uint8_t load_flag(const uint8_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// unit -> (link, pose slot, edge); false for a padding slot past the edge's pose count
__device__ __forceinline__ bool decode_unit(const CollideWork &w, int64_t unit, int32_t &link, int64_t &slot,
                                            int64_t &edge) {
    link = (int32_t)(unit % w.L);
    slot = unit / w.L;
    if (w.pose_edge) {
        edge = w.pose_edge[slot];
        return true;
    }
    edge = slot / w.pmax;
    return (int32_t)(slot % w.pmax) < w.pcount[edge];
}

// A wave-uniform double moved to SGPRs (FP64 VALU ops take one SGPR operand each).
__device__ __forceinline__ double uniform_d(double x) {
    const uint64_t b = (uint64_t)__double_as_longlong(x);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// R, T = fcl::relativeTransform(env tf, pose of the unit) (FCL's frame: env = o1).
__device__ __forceinline__ void unit_transform(const EnvDev &env, const double *__restrict__ pose, double R[9],
                                               double T[3]) {
    double R2[9], T2[3];
#pragma unroll
    for (int i = 0; i < 9; ++i) R2[i] = pose[i];
#pragma unroll
    for (int i = 0; i < 3; ++i) T2[i] = pose[9 + i];
    relative_transform(env.tf, env.tf + 9, R2, T2, R, T);
}

// The unit's relative transform: precomputed (w.unit_rt: bitwise unit_transform's result) or
// computed from its pose.
__device__ __forceinline__ void unit_rt(const EnvDev &env, const CollideWork &w, int64_t slot, int32_t link,
                                        double R[9], double T[3]) {
    const int64_t o = (slot * w.L + link) * 12;
    if (w.unit_rt) {
#pragma unroll
        for (int i = 0; i < 9; ++i) R[i] = w.unit_rt[o + i];
#pragma unroll
        for (int i = 0; i < 3; ++i) T[i] = w.unit_rt[o + 9 + i];
    } else {
        unit_transform(env, w.poses + o, R, T);
    }
}

// Agent triangle mapped exactly as FCL does (Q' = R Q + T) and its widened float box.
__device__ __forceinline__ void agent_tri_box(const double *__restrict__ t, const double R[9], const double T[3],
                                              float blo[3], float bhi[3]) {
    const v3 Q1 = xform(R, T, mk(t[0], t[1], t[2]));
    const v3 Q2 = xform(R, T, mk(t[3], t[4], t[5]));
    const v3 Q3 = xform(R, T, mk(t[6], t[7], t[8]));
    blo[0] = widen_lo(dmin(Q1.x, dmin(Q2.x, Q3.x)));
    blo[1] = widen_lo(dmin(Q1.y, dmin(Q2.y, Q3.y)));
    blo[2] = widen_lo(dmin(Q1.z, dmin(Q2.z, Q3.z)));
    bhi[0] = widen_hi(dmax(Q1.x, dmax(Q2.x, Q3.x)));
    bhi[1] = widen_hi(dmax(Q1.y, dmax(Q2.y, Q3.y)));
    bhi[2] = widen_hi(dmax(Q1.z, dmax(Q2.z, Q3.z)));
}

// Widened float box of a local box (centre c, half-extent e) under R, T.
__device__ __forceinline__ void local_box(const double c[3], const double e[3], const double R[9], const double T[3],
                                          float lo[3], float hi[3]) {
    const v3 cc = xform(R, T, mk(c[0], c[1], c[2]));
    const double ccv[3] = {cc.x, cc.y, cc.z};
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const double ex = fabs(R[i * 3 + 0]) * e[0] + fabs(R[i * 3 + 1]) * e[1] + fabs(R[i * 3 + 2]) * e[2];
        lo[i] = widen_lo(ccv[i] - ex);
        hi[i] = widen_hi(ccv[i] + ex);
    }
}

// lane j's float, uniform
__device__ __forceinline__ float lane_f(float v, int j) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), j));
}

__device__ __forceinline__ bool box_overlap(const float alo[3], const float ahi[3], const float *blo,
                                            const float *bhi) {
    return alo[0] <= bhi[0] && blo[0] <= ahi[0] && alo[1] <= bhi[1] && blo[1] <= ahi[1] && alo[2] <= bhi[2] &&
           blo[2] <= ahi[2];
}

// Quantized boxes (EnvDev::qitems): 15-bit coordinates over the env root box, rounded outward
// on the host; a query box quantized outward with a margin of 0.02 quanta beyond its float
// rounding (see broad.hip walk_two_q), so an overlap test on them keeps every pair the float
// test keeps.
struct QBox {
    uint32_t lxy, hxy, lz, hz;  // query: lo.x | lo.y << 16, hi.x | hi.y << 16, lo.z, hi.z
};
__device__ __forceinline__ QBox quantize_box(const EnvDev &env, const float lo[3], const float hi[3]) {
    uint32_t l[3], h[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float vl = floorf((lo[k] - env.q_org[k]) * env.q_scale[k] - 0.02f);
        const float vh = ceilf((hi[k] - env.q_org[k]) * env.q_scale[k] + 0.02f);
        l[k] = (uint32_t)fminf(fmaxf(vl, 0.0f), (float)kQMax);
        h[k] = (uint32_t)fminf(fmaxf(vh, 0.0f), (float)kQMax);
    }
    return QBox{l[0] | l[1] << 16, h[0] | h[1] << 16, l[2], h[2]};
}
__device__ __forceinline__ bool qbox_overlap(const QBox &q, uint4 it) {
    constexpr uint32_t H = 0x80008000u;
    const uint32_t t1 = (q.hxy | H) - it.x;  // query hi >= item lo (x, y)
    const uint32_t t2 = (it.y | H) - q.lxy;  // item hi >= query lo (x, y)
    const uint32_t A = (it.z & 0xffff0000u) | q.hz, B = (it.z & 0x0000ffffu) | (q.lz << 16);
    const uint32_t t3 = (A | H) - B;         // query hi.z >= item lo.z, item hi.z >= query lo.z
    return (t1 & t2 & t3 & H) == H;
}

// The top-level items of a two-level quantized env tree (at most 64) that a box may meet: bit i
// for item i -- k_steer's per-unit link-box mask, which k_pairs' cluster threads of the unit
// start from instead of all top-level items (every cluster box lies inside its link's box)
__device__ __forceinline__ uint64_t top_item_mask(const EnvDev &env, const float lo[3], const float hi[3]) {
    const QBox q = quantize_box(env, lo, hi);
    const int32_t top = env.n_levels - 1;
    const int32_t first = env.lev_off[top], n = env.lev_off[top + 1] - first;
    uint64_t M = 0;
    for (int32_t i0 = 0; i0 < n; i0 += 8) {
        uint4 b[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) b[j] = env.qitems[first + (i0 + j < n ? i0 + j : n - 1)];
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (i0 + j < n && qbox_overlap(q, b[j])) M |= 1ull << (i0 + j);
    }
    return M;
}

// --- the fused per-unit walk (collide.hip k_collide; broad.hip k_narrow's overflow re-run) ---
// Uniform walk of the env BVH by one wave per (pose, link) unit; s_nodes is an LDS prefix of
// env.nodes (or env.nodes itself with n_lds = n_nodes), the stack kStackDepth ints per wave.
__device__ __forceinline__ bool box_hit(const float lo[3], const float hi[3], const BvhNode &n) {
    return lo[0] <= n.hi[0] && n.lo[0] <= hi[0] && lo[1] <= n.hi[1] && n.lo[1] <= hi[1] &&
           lo[2] <= n.hi[2] && n.lo[2] <= hi[2];
}

// Uniform walk of the env BVH for one cluster.  Returns true on a contact.
__device__ inline bool walk_env(const BvhNode *__restrict__ s_nodes, int32_t n_lds, const BvhNode *__restrict__ nodes,
                         const EnvTri *__restrict__ etris, int32_t *stk, bool act, v3 Q1, v3 Q2, v3 Q3,
                         const float blo[3], const float bhi[3], uint32_t &n_nodes, uint32_t &n_sat) {
    int sp = 0;
    int32_t node = 0;
    for (;;) {
        // node is wave-uniform (SGPR): LDS prefix via ds_read, the rest via global loads
        BvhNode nd;
        if (node < n_lds) {
            nd = s_nodes[node];
        } else {
            typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
            const u32x4 *g = reinterpret_cast<const u32x4 *>(nodes + node);
            const u32x4 a = __builtin_nontemporal_load(g), b = __builtin_nontemporal_load(g + 1);
            nd.lo[0] = __uint_as_float(a.x); nd.lo[1] = __uint_as_float(a.y); nd.lo[2] = __uint_as_float(a.z);
            nd.a = (int32_t)a.w;
            nd.hi[0] = __uint_as_float(b.x); nd.hi[1] = __uint_as_float(b.y); nd.hi[2] = __uint_as_float(b.z);
            nd.b = (int32_t)b.w;
        }
        ++n_nodes;
        const bool ov = act && box_hit(blo, bhi, nd);
        const uint64_t m = __ballot(ov);
        if (m) {
            if (nd.b < 0) {
                const EnvTri &E = etris[nd.a];
                bool hit = false;
                if (ov) hit = tri_gate(E.lo, E.hi, Q1, Q2, Q3) && tri_intersect(E, Q1, Q2, Q3);
                n_sat += __popcll(m);
                if (__ballot(hit)) return true;
            } else {
                if (sp < kStackDepth) stk[sp] = nd.b;
                ++sp;
                node = __builtin_amdgcn_readfirstlane(nd.a);
                continue;
            }
        }
        if (sp == 0) return false;
        --sp;
        node = __builtin_amdgcn_readfirstlane(stk[sp]);
    }
}

__device__ inline void collide_unit(const EnvDev &env, const BvhNode *s_nodes, int32_t n_lds,
                             const AgentDev *__restrict__ links, const CollideWork &w, int64_t unit, int32_t *stk,
                             int lane, bool shared_edges, uint32_t &n_clusters, uint32_t &n_nodes,
                             uint32_t &n_sat, uint32_t &n_units) {
    int32_t link;
    int64_t slot, edge;
    if (!decode_unit(w, unit, link, slot, edge)) return;
    const int32_t L = w.L;
    if (shared_edges && load_flag(w.verdict + edge)) return;
    ++n_units;

    const double *pose = w.poses + (slot * L + link) * 12;
    double R2[9], T2[3], R[9], T[3];
#pragma unroll
    for (int i = 0; i < 9; ++i) R2[i] = pose[i];
#pragma unroll
    for (int i = 0; i < 3; ++i) T2[i] = pose[9 + i];
    relative_transform(env.tf, env.tf + 9, R2, T2, R, T);

    const AgentDev ag = links[link];
    const BvhNode root = s_nodes[0];

    for (int32_t cbase = 0; cbase < ag.n_clusters; cbase += kWave) {
        const int32_t ci = cbase + lane;
        bool ok = false;
        if (ci < ag.n_clusters) {
            const Cluster c = ag.clusters[ci];
            const v3 cc = xform(R, T, mk(c.c[0], c.c[1], c.c[2]));
            const double ccv[3] = {cc.x, cc.y, cc.z};
            float lo[3], hi[3];
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                const double ex = fabs(R[i * 3 + 0]) * c.e[0] + fabs(R[i * 3 + 1]) * c.e[1] +
                                  fabs(R[i * 3 + 2]) * c.e[2];
                lo[i] = widen_lo(ccv[i] - ex);
                hi[i] = widen_hi(ccv[i] + ex);
            }
            ok = box_hit(lo, hi, root);
        }
        uint64_t m = __ballot(ok);
        while (m) {
            const int j = __ffsll((unsigned long long)m) - 1;
            m &= m - 1;
            // another unit of this edge may already have found the contact
            if (shared_edges && load_flag(w.verdict + edge)) return;
            ++n_clusters;
            const Cluster c = ag.clusters[cbase + j];
            const bool act = lane < c.count;
            v3 Q1 = mk(0, 0, 0), Q2 = Q1, Q3 = Q1;
            float blo[3] = {0, 0, 0}, bhi[3] = {0, 0, 0};
            if (act) {
                const double *t = ag.tris + (int64_t)(c.first + lane) * 9;
                Q1 = xform(R, T, mk(t[0], t[1], t[2]));
                Q2 = xform(R, T, mk(t[3], t[4], t[5]));
                Q3 = xform(R, T, mk(t[6], t[7], t[8]));
                blo[0] = widen_lo(dmin(Q1.x, dmin(Q2.x, Q3.x)));
                blo[1] = widen_lo(dmin(Q1.y, dmin(Q2.y, Q3.y)));
                blo[2] = widen_lo(dmin(Q1.z, dmin(Q2.z, Q3.z)));
                bhi[0] = widen_hi(dmax(Q1.x, dmax(Q2.x, Q3.x)));
                bhi[1] = widen_hi(dmax(Q1.y, dmax(Q2.y, Q3.y)));
                bhi[2] = widen_hi(dmax(Q1.z, dmax(Q2.z, Q3.z)));
            }
            if (walk_env(s_nodes, n_lds, env.nodes, env.tris, stk, act, Q1, Q2, Q3, blo, bhi, n_nodes, n_sat)) {
                if (lane == 0)
                    __hip_atomic_store(w.verdict + edge, (uint8_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                return;
            }
        }
    }
}

}  // namespace mpt
