// self.hip -- self-collision of multi-link agents.
//
// MeshHandler::isInCollision with checkSelfCollision (utilities/meshhandler.hpp:205-219): the
// link objects of one pose go into a DynamicAABBTreeCollisionManager whose self-collide calls
// fcl::collide on every pair of distinct link objects (defaultCollisionFunction,
// fcl_helpers.hpp:52-65).  The verdict of a pair is the one of the env case with link j as o1
// (intersect_Triangle's P side, its precomputed records AgentDev::etris) and link k > j as o2:
// R, T = relativeTransform(pose_j, pose_k), Q' = R Q + T, some (a, b) with tri_gate and
// intersect_Triangle true.  FCL orders a pair by its tree layout; the build fixes o1 = the
// lower link index.
//
// One wave per (pose, link pair): link-box cull, then per cluster of link k (one triangle per
// lane) the cluster box against link j's box, and each triangle of link j (uniform loop, its
// box against the cluster box) against the lanes' triangles.
#include "collide_common.h"

namespace mpt {

constexpr int kSelfWaves = 4;

__global__ __launch_bounds__(kSelfWaves * 64) void k_self(const AgentDev *__restrict__ links, int32_t L, int32_t npairs,
                                                          const double *__restrict__ poses,
                                                          const int32_t *__restrict__ pose_edge, int64_t n_units,
                                                          uint8_t *verdict) {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int64_t unit = (int64_t)blockIdx.x * kSelfWaves + wave;
    if (unit >= n_units) return;
    const int64_t slot = unit / npairs;
    int32_t pr = (int32_t)(unit % npairs), j = 0;
    while (pr >= L - 1 - j) {  // pair index -> (j, k), j < k, row-major
        pr -= L - 1 - j;
        ++j;
    }
    const int32_t k = j + 1 + pr;
    const int64_t edge = pose_edge[slot];
    if (load_flag(verdict + edge)) return;
    const double *pj = poses + (slot * L + j) * 12, *pk = poses + (slot * L + k) * 12;
    double R[9], T[3];
    relative_transform(pj, pj + 9, pk, pk + 9, R, T);
#pragma unroll
    for (int i = 0; i < 9; ++i) R[i] = uniform_d(R[i]);
#pragma unroll
    for (int i = 0; i < 3; ++i) T[i] = uniform_d(T[i]);
    const AgentDev A = links[j], B = links[k];
    float alo[3], ahi[3], blo[3], bhi[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        alo[i] = widen_lo(A.bc[i] - A.be[i]);
        ahi[i] = widen_hi(A.bc[i] + A.be[i]);
    }
    local_box(B.bc, B.be, R, T, blo, bhi);
    if (!box_overlap(alo, ahi, blo, bhi)) return;
    for (int32_t cb = 0; cb < B.n_clusters; ++cb) {
        const Cluster c = B.clusters[cb];
        float clo[3], chi[3];
        local_box(c.c, c.e, R, T, clo, chi);
        if (!box_overlap(alo, ahi, clo, chi)) continue;
        const bool act = lane < c.count;
        v3 Q1 = mk(0, 0, 0), Q2 = Q1, Q3 = Q1;
        float tlo[3] = {0, 0, 0}, thi[3] = {0, 0, 0};
        if (act) {
            const double *t = B.tris + (int64_t)(c.first + lane) * 9;
            Q1 = xform(R, T, mk(t[0], t[1], t[2]));
            Q2 = xform(R, T, mk(t[3], t[4], t[5]));
            Q3 = xform(R, T, mk(t[6], t[7], t[8]));
            tlo[0] = widen_lo(dmin(Q1.x, dmin(Q2.x, Q3.x)));
            tlo[1] = widen_lo(dmin(Q1.y, dmin(Q2.y, Q3.y)));
            tlo[2] = widen_lo(dmin(Q1.z, dmin(Q2.z, Q3.z)));
            thi[0] = widen_hi(dmax(Q1.x, dmax(Q2.x, Q3.x)));
            thi[1] = widen_hi(dmax(Q1.y, dmax(Q2.y, Q3.y)));
            thi[2] = widen_hi(dmax(Q1.z, dmax(Q2.z, Q3.z)));
        }
        for (int32_t a = 0; a < A.n_tris; ++a) {
            const EnvTri &E = A.etris[a];
            const float elo[3] = {widen_lo(E.lo[0]), widen_lo(E.lo[1]), widen_lo(E.lo[2])};
            const float ehi[3] = {widen_hi(E.hi[0]), widen_hi(E.hi[1]), widen_hi(E.hi[2])};
            if (!box_overlap(clo, chi, elo, ehi)) continue;
            const bool hit = act && box_overlap(tlo, thi, elo, ehi) && tri_gate(E.lo, E.hi, Q1, Q2, Q3) &&
                             tri_intersect(E, Q1, Q2, Q3);
            if (__ballot(hit)) {
                if (lane == 0) __hip_atomic_store(verdict + edge, (uint8_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                return;
            }
        }
    }
}

void launch_self_collide(const AgentDev *d_links, int32_t L, const double *poses, const int32_t *pose_edge,
                         int64_t n_poses, uint8_t *verdict, hipStream_t stream) {
    if (L < 2 || n_poses <= 0) return;
    const int32_t npairs = L * (L - 1) / 2;
    const int64_t units = n_poses * npairs;
    const int64_t blocks = (units + kSelfWaves - 1) / kSelfWaves;
    if (blocks > 0x7fffffff) throw Error{5, "self-collision batch too large"};
    hipLaunchKernelGGL(k_self, dim3((unsigned)blocks), dim3(kSelfWaves * 64), 0, stream, d_links, L, npairs, poses,
                       pose_edge, units, verdict);
    hip_check(hipGetLastError(), "k_self launch");
}

}  // namespace mpt
