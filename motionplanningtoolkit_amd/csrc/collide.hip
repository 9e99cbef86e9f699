// collide.hip -- batched mesh-vs-mesh collision verdicts on gfx950.
//
// Replaces MeshHandler::isInCollision (utilities/meshhandler.hpp:187-243) and the FCL
// 0.3.2 path behind it (DynamicAABBTreeCollisionManager broadphase + OBBRSS traversal
// + Intersect::intersect_Triangle).  Verdict per edge = exists (pose, link, env tri,
// agent tri) with intersect_Triangle true, i.e. the all-pairs definition; every box
// test below only prunes, with margins (fcl_math.h widen_*) that keep it conservative.
//
// Mapping: one wavefront per (pose, link) unit.  The agent link mesh is stored in
// clusters of <= 64 triangles (one triangle per lane).  Per unit:
//   1. R, T = fcl::relativeTransform(env tf, pose)                      (uniform)
//   2. lanes over clusters: transformed cluster box vs env root box -> ballot mask
//   3. per surviving cluster: each lane maps its triangle Q_i' = R Q_i + T exactly as
//      FCL does and takes its float box; the wave then walks the env BVH UNIFORMLY
//      (one node at a time, stack in LDS, node index in an SGPR so node / triangle
//      records arrive by scalar loads); at each node the lanes' boxes are tested and
//      a ballot decides descent, so there is no traversal divergence;
//   4. at a leaf, lanes whose box overlaps the env triangle run the 17-axis test;
//      any hit -> verdict[edge] = 1 and the wave (and later units of that edge) stop.
#include "mpt_internal.h"

namespace mpt {

__device__ __forceinline__ bool box_hit(const float lo[3], const float hi[3], const BvhNode &n) {
    return lo[0] <= n.hi[0] && n.lo[0] <= hi[0] && lo[1] <= n.hi[1] && n.lo[1] <= hi[1] &&
           lo[2] <= n.hi[2] && n.lo[2] <= hi[2];
}

__device__ __forceinline__ uint8_t load_flag(const uint8_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Uniform walk of the env BVH for one cluster.  Returns true on a contact.
__device__ bool walk_env(const BvhNode *__restrict__ nodes, const EnvTri *__restrict__ etris,
                         int32_t *stk, bool act, v3 Q1, v3 Q2, v3 Q3, const float blo[3],
                         const float bhi[3], uint32_t &n_nodes, uint32_t &n_sat) {
    int sp = 0;
    int32_t node = 0;
    for (;;) {
        const BvhNode nd = nodes[node];
        ++n_nodes;
        const bool ov = act && box_hit(blo, bhi, nd);
        if (__ballot(ov)) {
            if (nd.b < 0) {
                const EnvTri E = etris[nd.a];
                bool hit = false;
                if (ov) {
                    hit = tri_intersect(E, Q1, Q2, Q3);
                }
                n_sat += __popcll(__ballot(ov));
                if (__ballot(hit)) return true;
            } else {
                if (sp < kStackDepth) stk[sp] = nd.b;
                ++sp;
                node = nd.a;
                continue;
            }
        }
        if (sp == 0) return false;
        --sp;
        node = __builtin_amdgcn_readfirstlane(stk[sp]);
    }
}

__global__ __launch_bounds__(256) void k_collide(EnvDev env, const AgentDev *__restrict__ links,
                                                 CollideWork w) {
    __shared__ int32_t s_stack[4][kStackDepth];
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int64_t unit = (int64_t)blockIdx.x * 4 + wave;
    if (unit >= w.n_units) return;

    const int32_t L = w.L;
    const int32_t link = (int32_t)(unit % L);
    const int64_t slot = unit / L;
    int64_t edge;
    if (w.pose_edge) {
        edge = w.pose_edge[slot];
    } else {
        edge = slot / w.pmax;
        if ((int32_t)(slot % w.pmax) >= w.pcount[edge]) return;
    }
    if (load_flag(w.verdict + edge)) return;

    const double *pose = w.poses + (slot * L + link) * 12;
    double R2[9], T2[3], R[9], T[3];
#pragma unroll
    for (int i = 0; i < 9; ++i) R2[i] = pose[i];
#pragma unroll
    for (int i = 0; i < 3; ++i) T2[i] = pose[9 + i];
    relative_transform(env.tf, env.tf + 9, R2, T2, R, T);

    const AgentDev ag = links[link];
    const BvhNode root = env.nodes[0];
    uint32_t n_clusters = 0, n_nodes = 0, n_sat = 0;
    bool contact = false;

    for (int32_t cbase = 0; cbase < ag.n_clusters && !contact; cbase += kWave) {
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
            if (load_flag(w.verdict + edge)) {
                m = 0;
                contact = true;  // another unit of this edge already hit
                break;
            }
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
            if (walk_env(env.nodes, env.tris, s_stack[wave], act, Q1, Q2, Q3, blo, bhi, n_nodes,
                         n_sat)) {
                if (lane == 0)
                    __hip_atomic_store(w.verdict + edge, (uint8_t)1, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                contact = true;
                break;
            }
        }
    }
    if (w.stats && lane == 0) {
        atomicAdd(w.stats + 0, 1ull);
        atomicAdd(w.stats + 1, (unsigned long long)n_clusters);
        atomicAdd(w.stats + 2, (unsigned long long)n_nodes);
        atomicAdd(w.stats + 3, (unsigned long long)n_sat);
    }
}

__global__ void k_pose_edge(const int64_t *__restrict__ off, int64_t E, int32_t *__restrict__ pe) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    for (int64_t p = off[e]; p < off[e + 1]; ++p) pe[p] = (int32_t)e;
}

void launch_collide(const EnvDev &env, const AgentDev *d_links, const CollideWork &w,
                    hipStream_t stream) {
    if (w.n_units <= 0 || env.n_tris <= 0) return;
    const int64_t blocks = (w.n_units + 3) / 4;
    hipLaunchKernelGGL(k_collide, dim3((unsigned)blocks), dim3(256), 0, stream, env, d_links, w);
    hip_check(hipGetLastError(), "k_collide launch");
}

void launch_pose_edge(const int64_t *d_offsets, int64_t E, int32_t *d_pose_edge, hipStream_t stream) {
    if (E <= 0) return;
    hipLaunchKernelGGL(k_pose_edge, dim3((unsigned)((E + 255) / 256)), dim3(256), 0, stream, d_offsets, E,
                       d_pose_edge);
    hip_check(hipGetLastError(), "k_pose_edge launch");
}

}  // namespace mpt
