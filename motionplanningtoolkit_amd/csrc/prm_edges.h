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
    // translation of pose q of the sequence: it < 1: the start then the end; else pose q of
    // the main run, then the end (tail)
    __device__ __forceinline__ void pose(unsigned q, double *t) const {
        if (it >= 1 && q < it) {
            at(q, t);
        } else {
            const double *src = (it < 1 && q == 0) ? s : end;
            t[0] = src[0];
            t[1] = src[1];
            t[2] = src[2];
        }
    }
    __device__ __forceinline__ unsigned count() const { return it < 1 ? 2u : it + (tail ? 1u : 0u); }

    // f(world translation) for each pose in order until f returns true (one call site of f:
    // the SAT it carries is inlined once)
    template <class F>
    __device__ __forceinline__ void each(F &&f) const {
        const unsigned n = count();
        for (unsigned q = 0; q < n; ++q) {
            double t[3];
            pose(q, t);
            if (f(t)) return;
        }
    }

    // The poses of the sequence [q0, q1), then the tail pose (index it) when tail_too, whose
    // gate with env triangle box elo / ehi can pass for agent triangle RQ (see each_near)
    template <class V>
    __device__ __forceinline__ void near_range(const V *RQ, const double *elo, const double *ehi, const double *env_tf,
                                               unsigned &q0, unsigned &q1, bool &tail_too) const {
        q0 = 0;
        q1 = count();
        tail_too = false;
        if (it < 2) return;
        const float d0 = (float)(s[0] - env_tf[9]), d1 = (float)(s[1] - env_tf[10]), d2 = (float)(s[2] - env_tf[11]);
        // T0 and Dk below are float sums of rotated terms: their rounding follows the terms'
        // magnitudes (|d|, step * it * |dx|), not the (possibly cancelled) sums, so eps carries
        // both (|R| <= 1 entrywise bounds each term by them)
        const float mag = fabsf(d0) + fabsf(d1) + fabsf(d2) +
                          (float)step * (float)it * (float)(fabs(dx[0]) + fabs(dx[1]) + fabs(dx[2]));
        float lo = 0.0f, hi = (float)(it - 1);
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const float rk0 = (float)env_tf[k], rk1 = (float)env_tf[3 + k], rk2 = (float)env_tf[6 + k];
            const float T0 = rk0 * d0 + rk1 * d1 + rk2 * d2;
            const float Dk = (float)step * (rk0 * (float)dx[0] + rk1 * (float)dx[1] + rk2 * (float)dx[2]);
            const float a0 = (float)(&RQ[0].x)[k], a1 = (float)(&RQ[1].x)[k], a2 = (float)(&RQ[2].x)[k];
            const float a = fminf(a0, fminf(a1, a2)), b = fmaxf(a0, fmaxf(a1, a2));
            const float el = (float)elo[k], eh = (float)ehi[k];
            const float eps = 1e-5f * (1.0f + mag + fabsf(T0) + fabsf(Dk) * (float)it + fabsf(a) + fabsf(b) +
                                       fabsf(el) + fabsf(eh) + fabsf((float)env_tf[9 + k]) + fabsf(rk0) +
                                       fabsf(rk1) + fabsf(rk2));
            const float u = eh - a - T0 + eps;  // i * D'_k <= u
            const float l = el - b - T0 - eps;  // i * D'_k >= l
            if (Dk > 0.0f) {
                lo = fmaxf(lo, l / Dk);
                hi = fminf(hi, u / Dk);
            } else if (Dk < 0.0f) {
                lo = fmaxf(lo, u / Dk);
                hi = fminf(hi, l / Dk);
            } else if (l > 0.0f || u < 0.0f) {
                hi = -4.0f;  // this dim never overlaps
            }
        }
        q0 = hi >= lo - 2.0f ? (unsigned)fmaxf(0.0f, floorf(lo) - 1.0f) : it;
        q1 = hi >= lo - 2.0f ? (unsigned)fminf((float)it, ceilf(hi) + 2.0f) : it;
        if (q1 < q0) q1 = q0;
        tail_too = tail;
    }

    // The same for the poses whose gate with an env triangle can pass.  RQ: the agent triangle
    // rotated (R Q, before + T); elo / ehi: the env triangle's exact box; env_tf: the env
    // transform (R rows | T).  Pose i's env-relative translation is T'(i) = envT(s + (step * i)
    // * dx), which in real arithmetic is T'(0) + i D', D' = step * R_env^T dx: the gate's box
    // test along dim k then bounds i * D'_k between two numbers, an interval of i.  The interval
    // is computed in float, widened by eps (1e-5 of the magnitudes involved: ~30x the rounding
    // of the float and double terms) and by one index either side, so every pose outside it
    // fails the exact gate; the poses inside run the exact test as before (bit-identical
    // verdicts).  The per-pose loop over all ~260 poses of a config-4 edge (--bounds rooms: 1.1 G
    // gate tests a roadmap) becomes a loop over the few poses that cross the env triangle's box.
    template <class F, class V>
    __device__ __forceinline__ void each_near(F &&f, const V *RQ, const double *elo, const double *ehi,
                                              const double *env_tf) const {
        unsigned q0, q1;
        bool tail_too;
        near_range(RQ, elo, ehi, env_tf, q0, q1, tail_too);
        const unsigned n = (q1 - q0) + (tail_too ? 1u : 0u);
        // in step over the lanes that called it: the loop ends for all of them at the first
        // lane's true (a contact decides the edge; a lane looping on past it only held the wave:
        // config 4 at --bounds rooms, the colliding edges the sweep took ~180 iterations a lane,
        // up to 7000)
        bool done = false;
        for (unsigned j = 0;; ++j) {
            const bool more = j < n;
            if (!__ballot(more)) return;
            if (more) {
                double t[3];
                pose(q0 + j < q1 ? q0 + j : it, t);  // past the run: the tail (index it)
                done = f(t);
            }
            if (__ballot(done)) return;
        }
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
