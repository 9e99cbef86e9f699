// prm_edges.h -- a PRM roadmap edge's poses, generated where they are used.
//
// PRM::addMilestone (planners/prm/prm.hpp:356-382): Omnidirectional::steer(src, tgt, 1000)
// (agents/omnidirectional.hpp:186-198) then getPoses at cc_dt (omnidirectional.hpp:202-247)
// along the key segment; a blimp mesh keeps milestone src's yaw (its cos / sin from the host's
// libm).  prm_connect.hip's pose stage and sweep.hip's fused sweep both use these functions,
// so the translations the sweep tests are bit for bit the ones the pose array held.
#pragma once
#include "mpt_internal.h"

namespace mpt {

// Omnidirectional::steer(start, goal, 1000)
__device__ __forceinline__ void prm_steer_end(const double *s, const double *g, double *e) {
    const double dx = g[0] - s[0], dy = g[1] - s[1], dz = g[2] - s[2];
    const double dist = sqrt(dx * dx + dy * dy + dz * dz);
    double fraction = 1000.0 / dist;
    if (fraction > 1) fraction = 1;
    e[0] = s[0] + dx * fraction;
    e[1] = s[1] + dy * fraction;
    e[2] = s[2] + dz * fraction;
}

// Omnidirectional::getPoses count: it = (unsigned)(dist / dt) poses at step * i, the end pose
// when it * dt < dist; fewer than one step: the start and the end
__device__ __forceinline__ int64_t prm_pose_count(const double *s, const double *e, double dt, double &dist,
                                                  unsigned &it) {
    const double dx = e[0] - s[0], dy = e[1] - s[1], dz = e[2] - s[2];
    dist = sqrt(dx * dx + dy * dy + dz * dz);
    const double q = dist / dt;
    it = (q >= 4294967296.0 || !(q >= 0)) ? 0u : (unsigned)q;
    if (it < 1) return 2;
    return (int64_t)it + (((double)it * dt < dist) ? 1 : 0);
}

// The roadmap's edges as the device holds them: edge e from milestone src[e] (0-based) to
// nbr[e] - 1, keys [n][3], yaw [n][2] (cos, sin)
struct PrmEdges {
    const double *keys;
    const double *rot;
    const int32_t *src;
    const int32_t *nbr;
    double dt;
};

// one edge's pose sequence: translation i (i < it) = s + (step * i) * (end - s), then the end
// (tail); it == 0: the start and the end
struct PrmEdge {
    double s[3], end[3], dx[3], step;
    double R[9];  // the world rotation of every pose (yaw about z)
    unsigned it;
    bool tail;
    __device__ __forceinline__ void at(unsigned i, double *t) const {
        const double st = step * (double)i;
        t[0] = s[0] + st * dx[0];
        t[1] = s[1] + st * dx[1];
        t[2] = s[2] + st * dx[2];
    }
    __device__ __forceinline__ void first(double *t) const {
        if (it < 1) {
            t[0] = s[0];
            t[1] = s[1];
            t[2] = s[2];
        } else {
            at(0, t);
        }
    }
    __device__ __forceinline__ void last(double *t) const {
        if (it < 1 || tail) {
            t[0] = end[0];
            t[1] = end[1];
            t[2] = end[2];
        } else {
            at(it - 1, t);
        }
    }
    // f(world translation) for each pose in order until f returns true
    template <class F>
    __device__ __forceinline__ void each(F &&f) const {
        if (it < 1) {
            if (f(s)) return;
            f(end);
            return;
        }
        for (unsigned i = 0; i < it; ++i) {
            double t[3];
            at(i, t);
            if (f(t)) return;
        }
        if (tail) f(end);
    }
};

__device__ __forceinline__ PrmEdge prm_edge(const PrmEdges &P, int64_t e) {
    PrmEdge g;
    const int32_t a = P.src[e];
    const double *s = P.keys + (int64_t)a * 3;
    const double c = P.rot[(int64_t)a * 2], sn = P.rot[(int64_t)a * 2 + 1];
    g.s[0] = s[0];
    g.s[1] = s[1];
    g.s[2] = s[2];
    prm_steer_end(g.s, P.keys + (int64_t)(P.nbr[e] - 1) * 3, g.end);
    double dist;
    (void)prm_pose_count(g.s, g.end, P.dt, dist, g.it);
    g.dx[0] = g.end[0] - g.s[0];
    g.dx[1] = g.end[1] - g.s[1];
    g.dx[2] = g.end[2] - g.s[2];
    g.step = P.dt / dist;
    g.tail = g.it >= 1 && (double)g.it * P.dt < dist;
    g.R[0] = c;
    g.R[1] = sn;
    g.R[2] = 0.0;
    g.R[3] = -sn;
    g.R[4] = c;
    g.R[5] = 0.0;
    g.R[6] = 0.0;
    g.R[7] = 0.0;
    g.R[8] = 1.0;
    return g;
}

}  // namespace mpt
