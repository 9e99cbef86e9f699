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

__device__ __forceinline__ bool box_overlap(const float alo[3], const float ahi[3], const float *blo,
                                            const float *bhi) {
    return alo[0] <= bhi[0] && blo[0] <= ahi[0] && alo[1] <= bhi[1] && blo[1] <= ahi[1] && alo[2] <= bhi[2] &&
           blo[2] <= ahi[2];
}

}  // namespace mpt
