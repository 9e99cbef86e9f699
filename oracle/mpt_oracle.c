/*
 * mpt_oracle.c -- TEST INFRASTRUCTURE ONLY (see mpt_oracle.h header).
 *
 * CPU restatement of the reference's hot path.  Every function cites the
 * reference call site it follows (paths relative to the reference root) and,
 * where the arithmetic lives in FCL 0.3.2 / FLANN 1.8.4 (not vendored, not in
 * the container), the upstream routine it restates, marked [upstream].
 *
 * Build: gcc -O2 -std=c99 -fPIC -ffp-contract=off -fno-fast-math (oracle/Makefile).
 * FMA contraction must stay off: FCL/FLANN were built for x86-64 SSE2 without FMA.
 */
#define _GNU_SOURCE
#include "mpt_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

/* ======================================================================
 * FCL 0.3.2 math [upstream]: fcl/math/vec_3f.h, matrix_3f.h, transform.cpp
 * ====================================================================== */

static inline double dot3(const double a[3], const double b[3]) {
    /* Vec3Data::dot: x*x' + y*y' + z*z' */
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}
static inline void cross3(const double a[3], const double b[3], double o[3]) {
    /* Vec3Data::cross */
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}
static inline void sub3(const double a[3], const double b[3], double o[3]) {
    o[0] = a[0] - b[0];
    o[1] = a[1] - b[1];
    o[2] = a[2] - b[2];
}

/* Quaternion3f::toRotation [upstream]; used by fcl_helpers::parseTransform
 * (utilities/fcl_helpers.hpp:16-25) through Transform3f(quaternion, vector). */
void orc_quat_to_rot(const double q[4], double R[9]) {
    const double w = q[0], x = q[1], y = q[2], z = q[3];
    const double twoX = 2.0 * x, twoY = 2.0 * y, twoZ = 2.0 * z;
    const double twoWX = twoX * w, twoWY = twoY * w, twoWZ = twoZ * w;
    const double twoXX = twoX * x, twoXY = twoY * x, twoXZ = twoZ * x;
    const double twoYY = twoY * y, twoYZ = twoZ * y, twoZZ = twoZ * z;
    R[0] = 1.0 - (twoYY + twoZZ); R[1] = twoXY - twoWZ;         R[2] = twoXZ + twoWY;
    R[3] = twoXY + twoWZ;         R[4] = 1.0 - (twoXX + twoZZ); R[5] = twoYZ - twoWX;
    R[6] = twoXZ - twoWY;         R[7] = twoYZ + twoWX;         R[8] = 1.0 - (twoXX + twoYY);
}

/* fcl::relativeTransform [upstream], called by setupMeshCollisionOrientedNode with
 * (tf1 = env object, tf2 = agent object) -- the callback order of
 * envManager->collide(agentManager) at utilities/meshhandler.hpp:229. */
void orc_relative_transform(const double R1[9], const double T1[3],
                            const double R2[9], const double T2[3],
                            double R[9], double T[3]) {
    /* Matrix3Data::transposeTimes: (R1^T R2)(i,j) = sum_k R1(k,i) R2(k,j), k ascending */
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            R[i * 3 + j] = R1[0 * 3 + i] * R2[0 * 3 + j] + R1[1 * 3 + i] * R2[1 * 3 + j] +
                           R1[2 * 3 + i] * R2[2 * 3 + j];
    double d[3];
    sub3(T2, T1, d);
    for (int i = 0; i < 3; ++i) T[i] = R1[0 * 3 + i] * d[0] + R1[1 * 3 + i] * d[1] + R1[2 * 3 + i] * d[2];
}

/* Matrix3f * Vec3f (dotX/dotY/dotZ) followed by + T. */
void orc_transform_point(const double R[9], const double T[3], const double q[3], double out[3]) {
    for (int i = 0; i < 3; ++i) {
        const double r = R[i * 3 + 0] * q[0] + R[i * 3 + 1] * q[1] + R[i * 3 + 2] * q[2];
        out[i] = r + T[i];
    }
}

/* Intersect::project6 [upstream]: 0 = separated along ax. */
static inline int project6(const double ax[3], const double p1[3], const double p2[3],
                           const double p3[3], const double q1[3], const double q2[3],
                           const double q3[3]) {
    const double P1 = dot3(ax, p1), P2 = dot3(ax, p2), P3 = dot3(ax, p3);
    const double Q1 = dot3(ax, q1), Q2 = dot3(ax, q2), Q3 = dot3(ax, q3);
    const double mx1 = fmax(P1, fmax(P2, P3)), mn1 = fmin(P1, fmin(P2, P3));
    const double mx2 = fmax(Q1, fmax(Q2, Q3)), mn2 = fmin(Q1, fmin(Q2, Q3));
    if (mn1 > mx2) return 0;
    if (mn2 > mx1) return 0;
    return 1;
}

/* Intersect::intersect_Triangle(P1,P2,P3,Q1,Q2,Q3) [upstream, FCL 0.3.2 intersect.cpp]:
 * 17 separating-axis tests (n1, m1, e_i x f_j, e_i x n1, f_j x m1) in the frame
 * translated to P1.  Touching counts as intersection (strict '>' in project6). */
int orc_tri_intersect(const double P[9], const double Q[9]) {
    const double *P1 = P, *P2 = P + 3, *P3 = P + 6;
    const double *Q1 = Q, *Q2 = Q + 3, *Q3 = Q + 6;
    double p1[3], p2[3], p3[3], q1[3], q2[3], q3[3];
    sub3(P1, P1, p1); sub3(P2, P1, p2); sub3(P3, P1, p3);
    sub3(Q1, P1, q1); sub3(Q2, P1, q2); sub3(Q3, P1, q3);
    double e1[3], e2[3], e3[3], f1[3], f2[3], f3[3];
    sub3(p2, p1, e1); sub3(p3, p2, e2); sub3(p1, p3, e3);
    sub3(q2, q1, f1); sub3(q3, q2, f2); sub3(q1, q3, f3);
    double n1[3], m1[3], ax[3];
    cross3(e1, e2, n1);
    if (!project6(n1, p1, p2, p3, q1, q2, q3)) return 0;
    cross3(f1, f2, m1);
    if (!project6(m1, p1, p2, p3, q1, q2, q3)) return 0;
    const double *E[3] = {e1, e2, e3}, *F[3] = {f1, f2, f3};
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            cross3(E[i], F[j], ax);
            if (!project6(ax, p1, p2, p3, q1, q2, q3)) return 0;
        }
    for (int i = 0; i < 3; ++i) {
        cross3(E[i], n1, ax);
        if (!project6(ax, p1, p2, p3, q1, q2, q3)) return 0;
    }
    for (int j = 0; j < 3; ++j) {
        cross3(F[j], m1, ax);
        if (!project6(ax, p1, p2, p3, q1, q2, q3)) return 0;
    }
    return 1;
}

static inline void map_tri(const double R[9], const double T[3], const double *Q, double *out) {
    orc_transform_point(R, T, Q, out);
    orc_transform_point(R, T, Q + 3, out + 3);
    orc_transform_point(R, T, Q + 6, out + 6);
}

/* Intersect::intersect_Triangle(P1..3, Q1..3, R, T) [upstream]: Q_i' = R Q_i + T. */
int orc_tri_intersect_RT(const double P[9], const double Q[9], const double R[9], const double T[3]) {
    double Qp[9];
    map_tri(R, T, Q, Qp);
    return orc_tri_intersect(P, Qp);
}

/* ======================================================================
 * Collision: MeshHandler::isInCollision (utilities/meshhandler.hpp:187-243) +
 * fcl_helpers::defaultCollisionFunction (utilities/fcl_helpers.hpp:52-65).
 * Verdict = exists (env tri, agent tri) pair whose exact vertex AABBs overlap (closed)
 * and that intersect_Triangle does not separate.  FCL 0.3.2 only calls
 * intersect_Triangle on pairs whose leaf bounding volumes overlap
 * (MeshCollisionTraversalNode::BVTesting before leafTesting); the AABB gate is that
 * precondition.  Without it, a degenerate (collinear) triangle "intersects" any
 * parallel one at any distance, since all 17 axes vanish; with it the all-pairs loop
 * below is the definition and every BVH in this repo only prunes.
 * ====================================================================== */

static int tri_gate(const double *P, const double *Qp) {
    for (int k = 0; k < 3; ++k) {
        const double plo = fmin(P[k], fmin(P[3 + k], P[6 + k])), phi = fmax(P[k], fmax(P[3 + k], P[6 + k]));
        const double qlo = fmin(Qp[k], fmin(Qp[3 + k], Qp[6 + k])), qhi = fmax(Qp[k], fmax(Qp[3 + k], Qp[6 + k]));
        if (plo > qhi || qlo > phi) return 0;
    }
    return 1;
}

static void unit_RT(const double env_tf[12], const double pose[12], double R[9], double T[3]) {
    orc_relative_transform(env_tf, env_tf + 9, pose, pose + 9, R, T);
}

int orc_collide_unit(const double *env_tris, int64_t Te, const double env_tf[12],
                     const double *agent_tris, int64_t Ta, const double pose[12]) {
    double R[9], T[3], Qp[9];
    unit_RT(env_tf, pose, R, T);
    for (int64_t b = 0; b < Ta; ++b) {
        map_tri(R, T, agent_tris + 9 * b, Qp);
        for (int64_t a = 0; a < Te; ++a)
            if (tri_gate(env_tris + 9 * a, Qp) && orc_tri_intersect(env_tris + 9 * a, Qp)) return 1;
    }
    return 0;
}

void orc_collide_batch(const double *env_tris, int64_t Te, const double env_tf[12],
                       const double *agent_tris, const int64_t *link_tri_off, int32_t L,
                       const double *poses, const int64_t *edge_pose_offsets, int64_t E,
                       uint8_t *verdict) {
    for (int64_t e = 0; e < E; ++e) {
        int hit = 0;
        for (int64_t p = edge_pose_offsets[e]; p < edge_pose_offsets[e + 1] && !hit; ++p)
            for (int32_t l = 0; l < L && !hit; ++l)
                hit = orc_collide_unit(env_tris, Te, env_tf, agent_tris + 9 * link_tri_off[l],
                                       link_tri_off[l + 1] - link_tri_off[l],
                                       poses + 12 * (p * L + l));
        verdict[e] = (uint8_t)hit;
    }
}

/* ---------------- AABB tree (speed only; conservative margins) ---------------- */
struct orc_bvh {
    int64_t T, nn;
    double *tris;   /* [T][9], reordered copy */
    double *lo, *hi; /* [nn][3] */
    int64_t *left;  /* child index or -1 - first tri for leaf */
    int64_t *cnt;   /* leaf triangle count, 0 for inner */
};

/* margin applied to every box comparison: far above the rounding error of the
 * 17-axis test, so pruning never removes a pair the all-pairs loop would report. */
static inline double bmargin(double a, double b) { return 1e-9 * (1.0 + fabs(a) + fabs(b)); }
static inline int box_overlap(const double *alo, const double *ahi, const double *blo, const double *bhi) {
    for (int k = 0; k < 3; ++k) {
        if (alo[k] > bhi[k] + bmargin(alo[k], bhi[k])) return 0;
        if (blo[k] > ahi[k] + bmargin(blo[k], ahi[k])) return 0;
    }
    return 1;
}
static void tri_box(const double *t, double lo[3], double hi[3]) {
    for (int k = 0; k < 3; ++k) {
        lo[k] = fmin(t[k], fmin(t[3 + k], t[6 + k]));
        hi[k] = fmax(t[k], fmax(t[3 + k], t[6 + k]));
    }
}

typedef struct { double c[3]; int64_t idx; } cent_t;
static int g_axis;
static int cent_cmp(const void *a, const void *b) {
    const cent_t *x = (const cent_t *)a, *y = (const cent_t *)b;
    if (x->c[g_axis] < y->c[g_axis]) return -1;
    if (x->c[g_axis] > y->c[g_axis]) return 1;
    return (x->idx < y->idx) ? -1 : (x->idx > y->idx);
}

static int64_t bvh_rec(orc_bvh *b, cent_t *c, int64_t first, int64_t n, const double *src) {
    const int64_t node = b->nn++;
    double lo[3] = {DBL_MAX, DBL_MAX, DBL_MAX}, hi[3] = {-DBL_MAX, -DBL_MAX, -DBL_MAX};
    double clo[3] = {DBL_MAX, DBL_MAX, DBL_MAX}, chi[3] = {-DBL_MAX, -DBL_MAX, -DBL_MAX};
    for (int64_t i = first; i < first + n; ++i) {
        double tl[3], th[3];
        tri_box(src + 9 * c[i].idx, tl, th);
        for (int k = 0; k < 3; ++k) {
            lo[k] = fmin(lo[k], tl[k]); hi[k] = fmax(hi[k], th[k]);
            clo[k] = fmin(clo[k], c[i].c[k]); chi[k] = fmax(chi[k], c[i].c[k]);
        }
    }
    memcpy(b->lo + 3 * node, lo, sizeof lo);
    memcpy(b->hi + 3 * node, hi, sizeof hi);
    if (n <= 2) {
        b->left[node] = first;
        b->cnt[node] = n;
        return node;
    }
    int ax = 0;
    for (int k = 1; k < 3; ++k)
        if (chi[k] - clo[k] > chi[ax] - clo[ax]) ax = k;
    g_axis = ax;
    qsort(c + first, (size_t)n, sizeof(cent_t), cent_cmp);
    const int64_t h = n / 2;
    b->cnt[node] = 0;
    const int64_t l = bvh_rec(b, c, first, h, src);
    (void)l;
    const int64_t r = bvh_rec(b, c, first + h, n - h, src);
    b->left[node] = r; /* left child is node + 1, store the right one */
    return node;
}

orc_bvh *orc_bvh_build(const double *tris, int64_t T) {
    orc_bvh *b = (orc_bvh *)calloc(1, sizeof *b);
    b->T = T;
    const int64_t cap = 2 * (T > 0 ? T : 1);
    b->tris = (double *)malloc(sizeof(double) * 9 * (size_t)(T > 0 ? T : 1));
    b->lo = (double *)malloc(sizeof(double) * 3 * (size_t)cap);
    b->hi = (double *)malloc(sizeof(double) * 3 * (size_t)cap);
    b->left = (int64_t *)malloc(sizeof(int64_t) * (size_t)cap);
    b->cnt = (int64_t *)malloc(sizeof(int64_t) * (size_t)cap);
    if (T == 0) return b;
    cent_t *c = (cent_t *)malloc(sizeof(cent_t) * (size_t)T);
    for (int64_t i = 0; i < T; ++i) {
        for (int k = 0; k < 3; ++k) c[i].c[k] = (tris[9 * i + k] + tris[9 * i + 3 + k] + tris[9 * i + 6 + k]) / 3.0;
        c[i].idx = i;
    }
    bvh_rec(b, c, 0, T, tris);
    for (int64_t i = 0; i < T; ++i) memcpy(b->tris + 9 * i, tris + 9 * c[i].idx, 9 * sizeof(double));
    free(c);
    return b;
}

void orc_bvh_free(orc_bvh *b) {
    if (!b) return;
    free(b->tris); free(b->lo); free(b->hi); free(b->left); free(b->cnt);
    free(b);
}

int orc_collide_unit_bvh(const orc_bvh *env, const double env_tf[12],
                         const double *agent_tris, int64_t Ta, const double pose[12],
                         int64_t *n_tri_tests) {
    if (env->T == 0) return 0;
    double R[9], T[3], Qp[9], qlo[3], qhi[3];
    int64_t stack[128];
    unit_RT(env_tf, pose, R, T);
    int64_t tests = 0;
    for (int64_t b = 0; b < Ta; ++b) {
        map_tri(R, T, agent_tris + 9 * b, Qp);
        tri_box(Qp, qlo, qhi);
        int sp = 0;
        stack[sp++] = 0;
        while (sp) {
            const int64_t nd = stack[--sp];
            if (!box_overlap(qlo, qhi, env->lo + 3 * nd, env->hi + 3 * nd)) continue;
            if (env->cnt[nd]) {
                for (int64_t i = env->left[nd]; i < env->left[nd] + env->cnt[nd]; ++i) {
                    if (!tri_gate(env->tris + 9 * i, Qp)) continue;
                    ++tests;
                    if (orc_tri_intersect(env->tris + 9 * i, Qp)) {
                        if (n_tri_tests) *n_tri_tests += tests;
                        return 1;
                    }
                }
            } else {
                stack[sp++] = env->left[nd];
                stack[sp++] = nd + 1;
            }
        }
    }
    if (n_tri_tests) *n_tri_tests += tests;
    return 0;
}

void orc_collide_batch_bvh(const orc_bvh *env, const double env_tf[12],
                           const double *agent_tris, const int64_t *link_tri_off, int32_t L,
                           const double *poses, const int64_t *edge_pose_offsets, int64_t E,
                           uint8_t *verdict, int nthreads) {
#ifdef _OPENMP
    if (nthreads < 1) nthreads = 1;
#pragma omp parallel for schedule(dynamic, 16) num_threads(nthreads)
#endif
    for (int64_t e = 0; e < E; ++e) {
        int hit = 0;
        for (int64_t p = edge_pose_offsets[e]; p < edge_pose_offsets[e + 1] && !hit; ++p)
            for (int32_t l = 0; l < L && !hit; ++l)
                hit = orc_collide_unit_bvh(env, env_tf, agent_tris + 9 * link_tri_off[l],
                                           link_tri_off[l + 1] - link_tri_off[l],
                                           poses + 12 * (p * L + l), NULL);
        verdict[e] = (uint8_t)hit;
    }
    (void)nthreads;
}

/* ======================================================================
 * FLANN 1.8.4 [upstream]: flann/algorithms/dist.h L2<double>::operator(),
 * used by FLANN_KDTreeWrapper (utilities/flannkdtreewrapper.hpp:57-117).
 * ====================================================================== */

double orc_l2(const double *a, const double *b, int32_t d) {
    double result = 0.0;
    int32_t i = 0;
    /* while (a < lastgroup), lastgroup = last - 3: groups of 4 */
    for (; i + 3 < d; i += 4) {
        const double d0 = a[i] - b[i], d1 = a[i + 1] - b[i + 1];
        const double d2 = a[i + 2] - b[i + 2], d3 = a[i + 3] - b[i + 3];
        result += d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3;
    }
    for (; i < d; ++i) {
        const double d0 = a[i] - b[i];
        result += d0 * d0;
    }
    return result;
}

/* (d2, id) lexicographic: the canonical order of every NN result in this build
 * (FLANN's own tie order is traversal order; exact ties are canonicalised to the
 * lowest id). */
static inline int better(double da, int32_t ia, double db, int32_t ib) {
    return da < db || (da == db && ia < ib);
}

static void topk_insert(double *bd, int32_t *bi, int32_t k, double dd, int32_t id) {
    if (!better(dd, id, bd[k - 1], bi[k - 1])) return;
    int32_t j = k - 1;
    while (j > 0 && better(dd, id, bd[j - 1], bi[j - 1])) {
        bd[j] = bd[j - 1];
        bi[j] = bi[j - 1];
        --j;
    }
    bd[j] = dd;
    bi[j] = id;
}

void orc_knn(const double *pts, const uint8_t *removed, int64_t n, int32_t d,
             const double *q, int64_t nq, int32_t k, int32_t *ids, double *d2) {
    for (int64_t s = 0; s < nq; ++s) {
        double *bd = d2 + s * k;
        int32_t *bi = ids + s * k;
        for (int32_t j = 0; j < k; ++j) { bd[j] = INFINITY; bi[j] = -1; }
        for (int64_t i = 0; i < n; ++i) {
            if (removed && removed[i]) continue;
            topk_insert(bd, bi, k, orc_l2(q + s * d, pts + i * d, d), (int32_t)(i + 1));
        }
    }
}

typedef struct { double d; int32_t id; } did_t;
static int did_cmp(const void *a, const void *b) {
    const did_t *x = (const did_t *)a, *y = (const did_t *)b;
    if (better(x->d, x->id, y->d, y->id)) return -1;
    if (better(y->d, y->id, x->d, x->id)) return 1;
    return 0;
}

int64_t orc_radius(const double *pts, const uint8_t *removed, int64_t n, int32_t d,
                   const double *q, int64_t nq, double r2, int32_t max_nb,
                   int64_t *offsets, int32_t *ids, double *d2, int64_t cap) {
    did_t *buf = (did_t *)malloc(sizeof(did_t) * (size_t)(n > 0 ? n : 1));
    int64_t total = 0;
    for (int64_t s = 0; s < nq; ++s) {
        int64_t m = 0;
        for (int64_t i = 0; i < n; ++i) {
            if (removed && removed[i]) continue;
            const double dd = orc_l2(q + s * d, pts + i * d, d);
            if (dd < r2) { buf[m].d = dd; buf[m].id = (int32_t)(i + 1); ++m; }
        }
        qsort(buf, (size_t)m, sizeof(did_t), did_cmp);
        if (max_nb > 0 && m > max_nb) m = max_nb;
        if (offsets) offsets[s] = total;
        for (int64_t j = 0; j < m; ++j, ++total)
            if (total < cap) { ids[total] = buf[j].id; d2[total] = buf[j].d; }
    }
    if (offsets) offsets[nq] = total;
    free(buf);
    return total;
}

/* ---------------- kd-tree (CPU baseline, KDTreeSingleIndex-like) ---------------- */
struct orc_kdtree {
    int64_t n;
    int32_t d;
    double *pts;     /* reordered [n][d] */
    int32_t *ids;    /* 1-based ids in reordered order */
    int64_t nn;
    int32_t *dim;    /* split dim, -1 leaf */
    double *split;
    int64_t *a, *b; /* inner: left,right ; leaf: first,count */
};

/* (value along dim, index) total order of two points */
static inline int kd_less(const double *src, int32_t d, int32_t dim, int64_t i, int64_t j) {
    const double a = src[i * d + dim], b = src[j * d + dim];
    return a < b || (a == b && i < j);
}

/* Quickselect: idx[first, first + n) reordered so that position h holds the h-th smallest
 * point in (value, index) order, smaller ones before it, larger ones after (the median split
 * in O(n), as FLANN's KDTreeSingleIndex::divideTree partitions instead of sorting). */
static void kd_select(int64_t *idx, int64_t first, int64_t n, int64_t h, const double *src, int32_t d, int32_t dim) {
    int64_t lo = first, hi = first + n - 1;
    const int64_t k = first + h;
    while (hi > lo) {
        /* median of three as the pivot */
        const int64_t mid = lo + (hi - lo) / 2;
        if (kd_less(src, d, dim, idx[mid], idx[lo])) { int64_t s = idx[mid]; idx[mid] = idx[lo]; idx[lo] = s; }
        if (kd_less(src, d, dim, idx[hi], idx[lo])) { int64_t s = idx[hi]; idx[hi] = idx[lo]; idx[lo] = s; }
        if (kd_less(src, d, dim, idx[hi], idx[mid])) { int64_t s = idx[hi]; idx[hi] = idx[mid]; idx[mid] = s; }
        const int64_t pv = idx[mid];
        int64_t i = lo, j = hi;
        while (i <= j) {
            while (kd_less(src, d, dim, idx[i], pv)) ++i;
            while (kd_less(src, d, dim, pv, idx[j])) --j;
            if (i <= j) {
                const int64_t s = idx[i]; idx[i] = idx[j]; idx[j] = s;
                ++i; --j;
            }
        }
        if (k <= j) hi = j;
        else if (k >= i) lo = i;
        else return;
    }
}

static int64_t kd_rec(orc_kdtree *t, int64_t *idx, int64_t first, int64_t n, const double *src) {
    const int64_t node = t->nn++;
    if (n <= 8) {
        t->dim[node] = -1;
        t->a[node] = first;
        t->b[node] = n;
        return node;
    }
    int32_t best = 0;
    double bw = -1;
    for (int32_t k = 0; k < t->d; ++k) {
        double lo = DBL_MAX, hi = -DBL_MAX;
        for (int64_t i = first; i < first + n; ++i) {
            const double v = src[idx[i] * t->d + k];
            lo = fmin(lo, v); hi = fmax(hi, v);
        }
        if (hi - lo > bw) { bw = hi - lo; best = k; }
    }
    const int64_t h = n / 2;
    kd_select(idx, first, n, h, src, t->d, best);
    t->dim[node] = best;
    t->split[node] = src[idx[first + h] * t->d + best];
    t->a[node] = kd_rec(t, idx, first, h, src);
    t->b[node] = kd_rec(t, idx, first + h, n - h, src);
    return node;
}

orc_kdtree *orc_kdtree_build(const double *pts, int64_t n, int32_t d) {
    orc_kdtree *t = (orc_kdtree *)calloc(1, sizeof *t);
    t->n = n; t->d = d;
    const int64_t cap = 2 * (n / 4 + 2);
    t->pts = (double *)malloc(sizeof(double) * (size_t)(n * d + 1));
    t->ids = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n + 1));
    t->dim = (int32_t *)malloc(sizeof(int32_t) * (size_t)cap);
    t->split = (double *)malloc(sizeof(double) * (size_t)cap);
    t->a = (int64_t *)malloc(sizeof(int64_t) * (size_t)cap);
    t->b = (int64_t *)malloc(sizeof(int64_t) * (size_t)cap);
    int64_t *idx = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n + 1));
    for (int64_t i = 0; i < n; ++i) idx[i] = i;
    if (n > 0) kd_rec(t, idx, 0, n, pts);
    for (int64_t i = 0; i < n; ++i) {
        memcpy(t->pts + i * d, pts + idx[i] * d, sizeof(double) * (size_t)d);
        t->ids[i] = (int32_t)(idx[i] + 1);
    }
    free(idx);
    return t;
}

void orc_kdtree_free(orc_kdtree *t) {
    if (!t) return;
    free(t->pts); free(t->ids); free(t->dim); free(t->split); free(t->a); free(t->b);
    free(t);
}

static void kd_search(const orc_kdtree *t, int64_t node, const double *q, int32_t k, double *bd, int32_t *bi) {
    if (t->dim[node] < 0) {
        for (int64_t i = t->a[node]; i < t->a[node] + t->b[node]; ++i)
            topk_insert(bd, bi, k, orc_l2(q, t->pts + i * t->d, t->d), t->ids[i]);
        return;
    }
    const int32_t dm = t->dim[node];
    const double diff = q[dm] - t->split[node];
    const int64_t nearc = diff < 0 ? t->a[node] : t->b[node];
    const int64_t farc = diff < 0 ? t->b[node] : t->a[node];
    kd_search(t, nearc, q, k, bd, bi);
    /* Exact pruning: every far-side point p has |q-p|_dm >= |diff| and FLANN's sum of
     * non-negative terms is monotone, so fl(d2(p)) >= fl(diff*diff).  Strict '>'
     * keeps exact ties, which the (d2, id) order then resolves. */
    if (diff * diff > bd[k - 1]) return;
    kd_search(t, farc, q, k, bd, bi);
}

void orc_kdtree_knn(const orc_kdtree *t, const double *q, int64_t nq, int32_t k,
                    int32_t *ids, double *d2, int nthreads) {
#ifdef _OPENMP
    if (nthreads < 1) nthreads = 1;
#pragma omp parallel for schedule(static) num_threads(nthreads)
#endif
    for (int64_t s = 0; s < nq; ++s) {
        double *bd = d2 + s * k;
        int32_t *bi = ids + s * k;
        for (int32_t j = 0; j < k; ++j) { bd[j] = INFINITY; bi[j] = -1; }
        if (t->n > 0) kd_search(t, 0, q + s * t->d, k, bd, bi);
    }
    (void)nthreads;
}

/* ======================================================================
 * RNG restatements
 * ====================================================================== */

/* glibc stdlib/random_r.c TYPE_3 (x**31 + x**3 + 1), srandom_r + random_r. */
void orc_glibc_srand(orc_glibc_rand *s, uint32_t seed) {
    int32_t *r = s->r;
    (void)r;
    int32_t state[31];
    if (seed == 0) seed = 1;
    state[0] = (int32_t)seed;
    int32_t word = (int32_t)seed;
    for (int i = 1; i < 31; ++i) {
        /* word = 16807 * hi/lo (Schrage), as srandom_r */
        const long hi = word / 127773;
        const long lo = word % 127773;
        word = (int32_t)(16807 * lo - 2836 * hi);
        if (word < 0) word += 2147483647;
        state[i] = word;
    }
    memcpy(s->r, state, sizeof state);
    s->f = 3;   /* fptr = &state[SEP_3] */
    s->b = 0;   /* rptr = &state[0] */
    for (int i = 0; i < 310; ++i) (void)orc_glibc_rand_next(s);
}

int32_t orc_glibc_rand_next(orc_glibc_rand *s) {
    uint32_t *st = (uint32_t *)s->r;
    const uint32_t val = (st[s->f] += st[s->b]);
    const int32_t result = (int32_t)(val >> 1);
    if (++s->f >= 31) { s->f = 0; ++s->b; }
    else if (++s->b >= 31) s->b = 0;
    return result;
}

/* std::linear_congruential_engine<uint_fast32_t, 16807, 0, 2147483647> */
void orc_minstd_seed(orc_minstd *g, uint64_t seed) {
    uint64_t x = seed % 2147483647ULL;
    g->x = x == 0 ? 1 : x;
}
uint64_t orc_minstd_next(orc_minstd *g) {
    g->x = (g->x * 16807ULL) % 2147483647ULL;
    return g->x;
}

/* libstdc++ (GCC 11) std::generate_canonical<double, 53>(minstd_rand0):
 * R = max - min + 1 = 2147483646, log2R = floor(log2(R)) = 30, m = 2 draws. */
static double generate_canonical_minstd(orc_minstd *g) {
    const long double r = 2147483646.0L;
    double sum = 0.0, tmp = 1.0;
    for (int k = 2; k != 0; --k) {
        sum += (double)(orc_minstd_next(g) - 1ULL) * tmp;
        tmp = (double)((long double)tmp * r);
    }
    double ret = sum / tmp;
    if (ret >= 1.0) ret = nextafter(1.0, 0.0);
    return ret;
}

/* uniform_real_distribution<double>::operator(): (canonical * (b - a)) + a */
double orc_uniform_real(orc_minstd *g, double a, double b) {
    return generate_canonical_minstd(g) * (b - a) + a;
}

/* Device engine RNG (the build's, not the reference's): splitmix64 finaliser of
 * seed ^ golden*counter, top 53 bits -> [0,1), then (u * (b - a)) + a. */
static inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
double orc_engine_uniform(uint64_t seed, uint64_t counter, double a, double b) {
    const uint64_t z = mix64(seed + 0x9E3779B97F4A7C15ULL * (counter + 1ULL));
    const double u = (double)(z >> 11) * (1.0 / 9007199254740992.0);
    return u * (b - a) + a;
}

/* ======================================================================
 * Agents
 * ====================================================================== */

static void identity_pose(const double t[3], double *pose) {
    static const double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    memcpy(pose, I, sizeof I);
    pose[9] = t[0]; pose[10] = t[1]; pose[11] = t[2];
}

/* Omnidirectional::randomSteer, agents/omnidirectional.hpp:168-184 */
static double omni_steer_from(const double r[3], const double start[3], double end[3]) {
    const double dist = sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
    end[0] = start[0] + r[0] / dist;
    end[1] = start[1] + r[1] / dist;
    end[2] = start[2] + r[2] / dist;
    return dist;
}
double orc_omni_random_steer(orc_glibc_rand *rng, const double start[3], double end[3]) {
    const double RM = 2147483647.0; /* RAND_MAX */
    double r[3];
    for (int i = 0; i < 3; ++i) r[i] = ((double)orc_glibc_rand_next(rng) - (RM / 2)) / (RM / 2);
    return omni_steer_from(r, start, end);
}

/* Omnidirectional::getPoses, agents/omnidirectional.hpp:202-247 */
int32_t orc_omni_get_poses(const double start[3], const double end[3], double dt,
                           double *poses_out, int32_t maxP) {
    const double dx = end[0] - start[0], dy = end[1] - start[1], dz = end[2] - start[2];
    const double dist = sqrt(dx * dx + dy * dy + dz * dz);
    const double q = dist / dt;
    const unsigned int iterations = (q >= 4294967296.0 || !(q >= 0)) ? 0u : (unsigned int)q;
    int32_t P = 0;
    if (iterations < 1) {
        if (P < maxP) identity_pose(start, poses_out + 12 * P);
        ++P;
        if (P < maxP) identity_pose(end, poses_out + 12 * P);
        ++P;
    } else {
        const double step = dt / dist;
        for (unsigned int i = 0; i < iterations; ++i) {
            const double stepSize = step * (double)i;
            const double t[3] = {start[0] + stepSize * dx, start[1] + stepSize * dy,
                                 start[2] + stepSize * dz};
            if (P < maxP) identity_pose(t, poses_out + 12 * P);
            ++P;
        }
        if ((double)iterations * dt < dist) {
            if (P < maxP) identity_pose(end, poses_out + 12 * P);
            ++P;
        }
    }
    return P;
}

/* ======================================================================
 * Correctly rounded sin / cos / tan: the trigonometry contract of the batched engine round
 * (orc_engine_step; the device's fcl_math.h cr_sin / cr_cos / cr_tan follow the same
 * definition).  The reference calls std::sin / cos / tan, i.e. the host's libm; glibc 2.35's
 * are not correctly rounded (about 0.15 % of sin / cos and 0.23 % of tan arguments in
 * [-7, 7] / [-0.8, 0.8] are 1 ulp off, tests/test_oracle.py against libquadmath) and differ
 * between its FMA and SSE2 variants, so no device code can be bitwise "libm"; the engine
 * instead uses the one implementation-independent definition, the correctly rounded value.
 * The sequential loops (orc_rrt_run, the K = 1 replay) keep the host libm, as the reference.
 *
 * Method: x = k pi/2 + r with pi/2 split into four parts (P1..P3 of 33 bits, so k * Pi is
 * exact for |k| < 2^20), r in double-double; sin r and cos r by Horner over r^2 in
 * double-double (Taylor series to r^29 / r^28, |r| <= pi/4 + 2^-30: truncation < 2^-110; the
 * eight leading terms in double-double, the tail in double);
 * tan = sin / cos in double-double.  The double-double result (relative error below
 * 2^-100) rounded to double is the correctly rounded value unless the exact value lies
 * within 2^-100 of a rounding boundary.  Coefficients: exact 1/n! split hi + lo.
 * ====================================================================== */
typedef struct { double h, l; } orc_dd;
static inline orc_dd dd_two_sum(double a, double b) {
    const double s = a + b, bb = s - a;
    const orc_dd r = {s, (a - (s - bb)) + (b - bb)};
    return r;
}
static inline orc_dd dd_fast(double a, double b) {  /* |a| >= |b| (or a == 0) */
    const double s = a + b;
    const orc_dd r = {s, b - (s - a)};
    return r;
}
static inline orc_dd dd_prod(double a, double b) {
    const double p = a * b;
    const orc_dd r = {p, fma(a, b, -p)};
    return r;
}
static inline orc_dd dd_add(orc_dd a, orc_dd b) {
    const orc_dd s = dd_two_sum(a.h, b.h);
    return dd_fast(s.h, s.l + (a.l + b.l));
}
static inline orc_dd dd_mul(orc_dd a, orc_dd b) {
    const orc_dd p = dd_prod(a.h, b.h);
    return dd_fast(p.h, p.l + (a.h * b.l + a.l * b.h));
}

static const double CR_SIN[15][2] = {
    {0x1p+0, 0x0p+0}, {-0x1.5555555555555p-3, -0x1.5555555555555p-57},
    {0x1.1111111111111p-7, 0x1.1111111111111p-63}, {-0x1.a01a01a01a01ap-13, -0x1.a01a01a01a01ap-73},
    {0x1.71de3a556c734p-19, -0x1.c154f8ddc6c00p-73}, {-0x1.ae64567f544e4p-26, 0x1.c062e06d1f209p-80},
    {0x1.6124613a86d09p-33, 0x1.f28e0cc748ebep-87}, {-0x1.ae7f3e733b81fp-41, -0x1.1d8656b0ee8cbp-97},
    {0x1.952c77030ad4ap-49, 0x1.ac981465ddc6cp-103}, {-0x1.2f49b46814157p-57, -0x1.2650f61dbdcb4p-112},
    {0x1.71b8ef6dcf572p-66, -0x1.d043ae40c4647p-120}, {-0x1.761b41316381ap-75, 0x1.3423c7d91404fp-130},
    {0x1.3f3ccdd165fa9p-84, -0x1.58ddadf344487p-139}, {-0x1.d1ab1c2dccea3p-94, -0x1.054d0c78aea14p-149},
    {0x1.259f98b4358adp-103, 0x1.eaf8c39dd9bc5p-157}};
static const double CR_COS[15][2] = {
    {0x1p+0, 0x0p+0}, {-0x1p-1, 0x0p+0},
    {0x1.5555555555555p-5, 0x1.5555555555555p-59}, {-0x1.6c16c16c16c17p-10, 0x1.f49f49f49f49fp-65},
    {0x1.a01a01a01a01ap-16, 0x1.a01a01a01a01ap-76}, {-0x1.27e4fb7789f5cp-22, -0x1.cbbc05b4fa99ap-76},
    {0x1.1eed8eff8d898p-29, -0x1.2aec959e14c06p-83}, {-0x1.93974a8c07c9dp-37, -0x1.05d6f8a2efd1fp-92},
    {0x1.ae7f3e733b81fp-45, 0x1.1d8656b0ee8cbp-101}, {-0x1.6827863b97d97p-53, -0x1.eec01221a8b0bp-107},
    {0x1.e542ba4020225p-62, 0x1.ea72b4afe3c2fp-120}, {-0x1.0ce396db7f853p-70, 0x1.aebcdbd20331cp-124},
    {0x1.f2cf01972f578p-80, -0x1.9ada5fcc1ab14p-135}, {-0x1.88e85fc6a4e5ap-89, 0x1.71c37ebd16540p-143},
    {0x1.0a18a2635085dp-98, 0x1.b9e2e28e1aa54p-153}};

/* r = x - k pi/2 in double-double; returns k mod 4 */
static int cr_reduce(double x, orc_dd *r) {
    const double k = nearbyint(x * 0x1.45f306dc9c883p-1);
    const double t = x - k * 0x1.921fb54400000p+0;  /* exact for |k| < 2^20 */
    orc_dd a = dd_two_sum(t, -(k * 0x1.0b4611a600000p-34));
    a = dd_add(a, dd_prod(-k, 0x1.3198a2e000000p-69));
    a = dd_add(a, dd_prod(-k, 0x1.b839a252049c1p-104));
    *r = a;
    return (int)((int64_t)k & 3);
}
/* terms 14..8 (at most 2^-53 of the sum for |r| <= pi/4 + 2^-30) in double over z.h, their
 * rounding below 2^-105 of the result; terms 7..0 in double-double */
static orc_dd cr_poly(const double c[15][2], orc_dd z) {
    double t = c[14][0];
    for (int n = 13; n >= 8; --n) t = t * z.h + c[n][0];
    orc_dd acc = {t, 0.0};
    for (int n = 7; n >= 0; --n) {
        const orc_dd cn = {c[n][0], c[n][1]};
        acc = dd_add(dd_mul(acc, z), cn);
    }
    return acc;
}
/* sin r and cos r of the reduced argument */
static void cr_sincos_r(orc_dd r, orc_dd *s, orc_dd *c) {
    const orc_dd z = dd_mul(r, r);
    *s = dd_mul(r, cr_poly(CR_SIN, z));
    *c = cr_poly(CR_COS, z);
}
/* domain |x| <= 2^20 (the reduction is exact for |k| < 2^20): NaN beyond it, as fcl_math.h */
#define ORC_CR_MAX_ARG 0x1p20
double orc_cr_sin(double x) {
    if (x == 0.0 || !isfinite(x)) return x == 0.0 ? x : x - x;
    if (fabs(x) > ORC_CR_MAX_ARG) return NAN;
    orc_dd r, s, c;
    const int q = cr_reduce(x, &r);
    cr_sincos_r(r, &s, &c);
    const double v = (q & 1) ? c.h : s.h;
    return (q & 2) ? -v : v;
}
double orc_cr_cos(double x) {
    if (!isfinite(x)) return x - x;
    if (fabs(x) > ORC_CR_MAX_ARG) return NAN;
    orc_dd r, s, c;
    const int q = cr_reduce(x, &r);
    cr_sincos_r(r, &s, &c);
    const double v = (q & 1) ? s.h : c.h;
    return ((q + 1) & 2) ? -v : v;
}
double orc_cr_tan(double x) {
    if (x == 0.0 || !isfinite(x)) return x == 0.0 ? x : x - x;
    if (fabs(x) > ORC_CR_MAX_ARG) return NAN;
    orc_dd r, s, c;
    const int q = cr_reduce(x, &r);
    cr_sincos_r(r, &s, &c);
    orc_dd n = s, d = c;  /* tan = sin / cos, or -cos / sin in odd quadrants */
    if (q & 1) {
        n.h = -c.h; n.l = -c.l;
        d = s;
    }
    const double q1 = n.h / d.h;
    const orc_dd p = dd_prod(q1, d.h);
    const double rem = (((n.h - p.h) - p.l) + n.l) - q1 * d.l;
    return dd_fast(q1, rem / d.h).h;
}

/* the trigonometry a steering routine uses: the host libm (the reference's std::sin / cos /
 * tan; the sequential loops) or the correctly rounded one (the batched engine round) */
typedef struct { double (*sin)(double); double (*cos)(double); double (*tan)(double); } orc_trig;
static const orc_trig TRIG_LIBM = {sin, cos, tan};
static const orc_trig TRIG_CR = {orc_cr_sin, orc_cr_cos, orc_cr_tan};

static double normalize_theta(double t) {
    /* Blimp/SnakeTrailers::normalizeTheta */
    return t - 2 * M_PI * floor((t + M_PI) / (2 * M_PI));
}

/* Blimp::doStep, agents/blimp.hpp:293-317 (theta update omits dt, as written) */
static void blimp_do_step_t(const orc_trig *tr, const double prm[7], const double s[7], double a, double w,
                            double z, double dt, double out[7]) {
    const double L = prm[0], vmin = prm[1], vmax = prm[2], pmin = prm[3], pmax = prm[4];
    const double zmin = prm[5], zmax = prm[6];
    double n[7];
    n[0] = s[0] + tr->cos(s[3]) * s[4] * dt;
    n[1] = s[1] + tr->sin(s[3]) * s[4] * dt;
    n[3] = normalize_theta(s[3] + s[4] * tr->tan(s[5]) / L);
    n[2] = s[2] + s[6] * dt;
    n[4] = s[4] + a * dt;
    n[5] = s[5] + w * dt;
    n[6] = s[6] + z * dt;
    if (n[4] > vmax) n[4] = vmax; else if (n[4] < vmin) n[4] = vmin;
    if (n[5] > pmax) n[5] = pmax; else if (n[5] < pmin) n[5] = pmin;
    if (n[6] > zmax) n[6] = zmax; else if (n[6] < zmin) n[6] = zmin;
    memcpy(out, n, sizeof n);
}
void orc_blimp_do_step(const double prm[7], const double s[7], double a, double w, double z,
                       double dt, double out[7]) {
    blimp_do_step_t(&TRIG_LIBM, prm, s, a, w, z, dt, out);
}
void orc_blimp_do_step_cr(const double prm[7], const double s[7], double a, double w, double z,
                          double dt, double out[7]) {
    blimp_do_step_t(&TRIG_CR, prm, s, a, w, z, dt, out);
}

/* Blimp::randomSteer, agents/blimp.hpp:179-187: draws a, w, z in that order from
 * uniform(-1,1), uniform(-0.1745,0.1745), uniform(-1,1) on one default engine. */
void orc_blimp_random_steer(const double prm[7], orc_minstd *g, const double start[7],
                            double dt, double end[7], double awz[3]) {
    awz[0] = orc_uniform_real(g, -1, 1);
    awz[1] = orc_uniform_real(g, -0.1745, 0.1745);
    awz[2] = orc_uniform_real(g, -1, 1);
    orc_blimp_do_step(prm, start, awz[0], awz[1], awz[2], dt, end);
}

/* Blimp::stateToFCLTransform, agents/blimp.hpp:339-356 */
static void blimp_pose(const orc_trig *tr, const double s[7], double *pose) {
    const double sv = tr->sin(s[3]), cv = tr->cos(s[3]);
    const double R[9] = {cv, sv, 0, -sv, cv, 0, 0, 0, 1};
    memcpy(pose, R, sizeof R);
    pose[9] = s[0]; pose[10] = s[1]; pose[11] = s[2];
}

/* Build-defined Blimp::getPoses (the reference's agents/blimp.hpp:219-223 returns one
 * empty pose list, i.e. never checks): the states after each of the
 * max(1, floor(edge_dt / dt)) doStep(dt) increments, end state included. */
static int32_t blimp_get_poses_t(const orc_trig *tr, const double prm[7], const double start[7],
                                 const double awz[3], double edge_dt, double dt, double *poses_out, int32_t maxP) {
    const double q = edge_dt / dt;
    unsigned int steps = (q >= 4294967296.0 || !(q >= 0)) ? 0u : (unsigned int)q;
    if (steps == 0) steps = 1;
    double s[7];
    memcpy(s, start, sizeof s);
    for (unsigned int i = 0; i < steps; ++i) {
        blimp_do_step_t(tr, prm, s, awz[0], awz[1], awz[2], dt, s);
        if ((int32_t)i < maxP) blimp_pose(tr, s, poses_out + 12 * i);
    }
    return (int32_t)steps;
}
int32_t orc_blimp_get_poses(const double prm[7], const double start[7], const double awz[3],
                            double edge_dt, double dt, double *poses_out, int32_t maxP) {
    return blimp_get_poses_t(&TRIG_LIBM, prm, start, awz, edge_dt, dt, poses_out, maxP);
}
int32_t orc_blimp_get_poses_cr(const double prm[7], const double start[7], const double awz[3],
                               double edge_dt, double dt, double *poses_out, int32_t maxP) {
    return blimp_get_poses_t(&TRIG_CR, prm, start, awz, edge_dt, dt, poses_out, maxP);
}

/* SnakeTrailers::doStep, agents/snake_trailers.hpp:341-369 */
static void snake_do_step_t(const orc_trig *tr, const double prm[7], const double *s, double a, double w,
                            double dt, double *out) {
    const int T = (int)prm[0];
    const double Lt = prm[1], Lh = prm[2], vmin = prm[3], vmax = prm[4], pmin = prm[5], pmax = prm[6];
    enum { X = 0, Y = 1, V = 2, PSI = 3, THETA = 4 };
    double n[64];
    n[X] = s[X] + tr->cos(s[THETA]) * s[V] * dt;
    n[Y] = s[Y] + tr->sin(s[THETA]) * s[V] * dt;
    n[THETA] = normalize_theta(s[THETA] + s[V] * tr->tan(s[PSI]) / Lt * dt);
    n[V] = s[V] + a * dt;
    n[PSI] = s[PSI] + w * dt;
    if (n[V] > vmax) n[V] = vmax; else if (n[V] < vmin) n[V] = vmin;
    if (n[PSI] > pmax) n[PSI] = pmax; else if (n[PSI] < pmin) n[PSI] = pmin;
    double coeff = s[V] / (Lt + Lh);
    double prev = s[THETA];
    for (int i = 1; i < T + 1; ++i) {
        n[THETA + i] = normalize_theta(s[THETA + i] + coeff * tr->sin(prev - s[THETA + i]) * dt);
        coeff *= tr->cos(prev - s[THETA + i]);
        prev = s[THETA + i];
    }
    memcpy(out, n, sizeof(double) * (size_t)(5 + T));
}
void orc_snake_do_step(const double prm[7], const double *s, double a, double w, double dt,
                       double *out) {
    snake_do_step_t(&TRIG_LIBM, prm, s, a, w, dt, out);
}
void orc_snake_do_step_cr(const double prm[7], const double *s, double a, double w, double dt,
                          double *out) {
    snake_do_step_t(&TRIG_CR, prm, s, a, w, dt, out);
}

/* SnakeTrailers::randomSteer, agents/snake_trailers.hpp:206-213: a ~ U(-0.1, 1),
 * w ~ U(-pi/18, pi/18) from the agent's default engine. */
void orc_snake_random_steer(const double prm[7], orc_minstd *g, const double *start, double dt,
                            double *end, double aw[2]) {
    aw[0] = orc_uniform_real(g, -0.1, 1);
    aw[1] = orc_uniform_real(g, -M_PI / 18., M_PI / 18.);
    orc_snake_do_step(prm, start, aw[0], aw[1], dt, end);
}

/* SnakeTrailers::stateToFCLTransforms, agents/snake_trailers.hpp:411-459, verbatim:
 * trailer translations are (-(Lt+Lh), Y, 0), not chained. */
static void snake_poses(const orc_trig *tr, const double prm[7], const double *s, double *poses /*[L][12]*/) {
    const int T = (int)prm[0];
    const double Lt = prm[1], Lh = prm[2];
    enum { X = 0, Y = 1, THETA = 4 };
    double pose_t[3] = {s[X], s[Y], 0};
    double R[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    double sv = tr->sin(s[THETA]), cv = tr->cos(s[THETA]);
    R[0] = cv; R[3] = -sv; R[1] = sv; R[4] = cv;
    memcpy(poses, R, sizeof R);
    memcpy(poses + 9, pose_t, sizeof pose_t);
    for (int i = 1; i < T + 1; ++i) {
        pose_t[0] = -(Lt + Lh);
        const double t = s[THETA + i] - s[THETA + i - 1];
        sv = tr->sin(t); cv = tr->cos(t);
        R[0] = cv; R[3] = -sv; R[1] = sv; R[4] = cv;
        /* rotation = rotation * identity: Matrix3Data::operator* sums x*1 + y*0 + z*0 */
        double M[9];
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) {
                const double I0 = (c == 0), I1 = (c == 1), I2 = (c == 2);
                M[r * 3 + c] = R[r * 3 + 0] * I0 + R[r * 3 + 1] * I1 + R[r * 3 + 2] * I2;
            }
        memcpy(R, M, sizeof M);
        memcpy(poses + 12 * i, R, sizeof R);
        memcpy(poses + 12 * i + 9, pose_t, sizeof pose_t);
    }
}

/* SnakeTrailers::getPoses, agents/snake_trailers.hpp:246-268 */
static int32_t snake_get_poses_t(const orc_trig *tr, const double prm[7], const double *start, const double aw[2],
                                 double edge_dt, double dt, double *poses_out, int32_t maxP) {
    const int T = (int)prm[0];
    const int L = T + 1;
    const double q = edge_dt / dt;
    unsigned int steps = (q >= 4294967296.0 || !(q >= 0)) ? 0u : (unsigned int)q;
    if (steps == 0) steps = 1;
    double s[64];
    memcpy(s, start, sizeof(double) * (size_t)(5 + T));
    for (unsigned int i = 0; i < steps; ++i) {
        if ((int32_t)i < maxP) snake_poses(tr, prm, s, poses_out + (size_t)12 * L * i);
        snake_do_step_t(tr, prm, s, aw[0], aw[1], dt, s);
    }
    return (int32_t)steps;
}
int32_t orc_snake_get_poses(const double prm[7], const double *start, const double aw[2],
                            double edge_dt, double dt, double *poses_out, int32_t maxP) {
    return snake_get_poses_t(&TRIG_LIBM, prm, start, aw, edge_dt, dt, poses_out, maxP);
}
int32_t orc_snake_get_poses_cr(const double prm[7], const double *start, const double aw[2],
                               double edge_dt, double dt, double *poses_out, int32_t maxP) {
    return snake_get_poses_t(&TRIG_CR, prm, start, aw, edge_dt, dt, poses_out, maxP);
}

/* ======================================================================
 * Sequential RRT: planners/rrt.hpp:21-94 with UniformSampler
 * (samplers/uniformsampler.hpp:20-35), TreeInterface (tree_interfaces/treeinterface.hpp),
 * FLANN_KDTreeWrapper ids (utilities/flannkdtreewrapper.hpp:21-40) and Map3D::safeEdge
 * (workspaces/map3d.hpp:33-37).
 * ====================================================================== */

static int is_goal(int kind, const double *s, const double *g, const double *thr) {
    if (kind == 2) return fabs(s[0] - g[0]) < thr[0] && fabs(s[1] - g[1]) < thr[1];
    return fabs(s[0] - g[0]) < thr[0] && fabs(s[1] - g[1]) < thr[1] && fabs(s[2] - g[2]) < thr[2];
}

#define ORC_MAXP 4096

int64_t orc_rrt_run(int32_t agent_kind, const double *prm, int32_t d, const double *ranges,
                    const double *start, const double *goal, const double *goal_thr,
                    double steer_dt, double cc_dt,
                    const double *env_tris, int64_t Te, const double env_tf[12],
                    const double *agent_tris, int64_t Ta,
                    int64_t iterations_at_a_time, int64_t max_nodes,
                    double *nodes, int32_t *parents, int64_t *solved, int64_t *iters_out) {
    *solved = -1;
    *iters_out = 0;
    /* rrt.hpp:27-30: goal test before anything is inserted */
    if (is_goal(agent_kind, start, goal, goal_thr)) { *solved = -2; return 0; }
    orc_minstd sampler;     /* UniformSampler::generator (uniformsampler.hpp:43) */
    orc_minstd agent_gen;   /* Blimp/SnakeTrailers::generator */
    orc_glibc_rand crand;   /* glibc rand() for Omnidirectional (never seeded: srand(1)) */
    orc_minstd_seed(&sampler, 1);
    orc_minstd_seed(&agent_gen, 1);
    orc_glibc_srand(&crand, 1);
    orc_bvh *env = orc_bvh_build(env_tris, Te);
    const int L = agent_kind == 2 ? (int)prm[0] + 1 : 1;
    double *poses = (double *)malloc(sizeof(double) * 12 * (size_t)ORC_MAXP * (size_t)L);
    /* rrt.hpp:32-35: root = Edge(start), inserted first (FLANN id 1) */
    memcpy(nodes, start, sizeof(double) * (size_t)d);
    parents[0] = 0;
    int64_t n = 1;
    double sample[64], end[64], ctrl[3];
    unsigned int iterations = 0;
    const int64_t iat = iterations_at_a_time;
    int64_t pass;
    for (pass = 0; pass < 100000000; ++pass) {
        for (int32_t j = 0; j < d; ++j) sample[j] = orc_uniform_real(&sampler, ranges[2 * j], ranges[2 * j + 1]);
        /* nearest: exact 1-NN, lowest id on exact ties */
        int64_t best = 0;
        double bd = INFINITY;
        for (int64_t i = 0; i < n; ++i) {
            const double dd = orc_l2(sample, nodes + i * d, d);
            if (dd < bd) { bd = dd; best = i; }
        }
        const double *from = nodes + best * d;
        int32_t P;
        const double edge_dt = steer_dt;  /* Blimp/Snake Edge::dt = cost = steering dt */
        if (agent_kind == 0) {
            (void)orc_omni_random_steer(&crand, from, end);
            P = orc_omni_get_poses(from, end, cc_dt, poses, ORC_MAXP);
        } else if (agent_kind == 1) {
            orc_blimp_random_steer(prm, &agent_gen, from, steer_dt, end, ctrl);
            P = orc_blimp_get_poses(prm, from, ctrl, edge_dt, cc_dt, poses, ORC_MAXP);
        } else {
            orc_snake_random_steer(prm, &agent_gen, from, steer_dt, end, ctrl);
            P = orc_snake_get_poses(prm, from, ctrl, edge_dt, cc_dt, poses, ORC_MAXP);
        }
        if (P > ORC_MAXP) P = ORC_MAXP;
        int hit = 0;
        for (int32_t p = 0; p < P && !hit; ++p)
            for (int l = 0; l < L && !hit; ++l)
                hit = orc_collide_unit_bvh(env, env_tf, agent_tris, Ta, poses + 12 * ((size_t)p * L + l), NULL);
        if (hit) {  /* rrt.hpp:50-56 (iterations counted twice, as written) */
            ++iterations;
            if (iat > 0 && ++iterations > (unsigned int)iat) break;
            continue;
        }
        if (is_goal(agent_kind, end, goal, goal_thr)) { *solved = pass; break; }
        if (n >= max_nodes) break;
        memcpy(nodes + n * d, end, sizeof(double) * (size_t)d);
        parents[n] = (int32_t)(best + 1);
        ++n;
        if (iat > 0 && ++iterations > (unsigned int)iat) break;
    }
    *iters_out = pass;
    free(poses);
    orc_bvh_free(env);
    return n;
}

/* ======================================================================
 * Batched device-engine step (the build's throughput mode; see
 * motionplanningtoolkit_amd/csrc/rrt_engine.hip): K extensions against the tree
 * snapshot, collision-free edges appended in extension order.
 * Counter layout per extension g: dims use counter g*64 + j, controls g*64 + 32 + j.
 * ====================================================================== */

int64_t orc_engine_step(int32_t agent_kind, const double *prm, int32_t d, const double *ranges,
                        double steer_dt, double cc_dt, uint64_t seed, uint64_t ext_base,
                        int32_t K, const orc_bvh *env, const double env_tf[12],
                        const double *agent_tris, int64_t Ta,
                        double *nodes, int32_t *parents, int64_t n_nodes, int64_t capacity,
                        int32_t *nn_out, uint8_t *verdict_out, int nthreads, int use_kdtree) {
    const int L = agent_kind == 2 ? (int)prm[0] + 1 : 1;
    double *samples = (double *)malloc(sizeof(double) * (size_t)K * (size_t)d);
    double *ends = (double *)malloc(sizeof(double) * (size_t)K * (size_t)d);
    int32_t *ids = nn_out;
    double *d2 = (double *)malloc(sizeof(double) * (size_t)K);
    for (int32_t k = 0; k < K; ++k) {
        const uint64_t g = ext_base + (uint64_t)k;
        for (int32_t j = 0; j < d; ++j)
            samples[k * d + j] = orc_engine_uniform(seed, g * 64 + j, ranges[2 * j], ranges[2 * j + 1]);
    }
    if (use_kdtree) {
        orc_kdtree *t = orc_kdtree_build(nodes, n_nodes, d);
        orc_kdtree_knn(t, samples, K, 1, ids, d2, nthreads);
        orc_kdtree_free(t);
    } else {
        orc_knn(nodes, NULL, n_nodes, d, samples, K, 1, ids, d2);
    }
#ifdef _OPENMP
    if (nthreads < 1) nthreads = 1;
#pragma omp parallel for schedule(dynamic, 16) num_threads(nthreads)
#endif
    for (int32_t k = 0; k < K; ++k) {
        const uint64_t g = ext_base + (uint64_t)k;
        const double *from = nodes + (int64_t)(ids[k] - 1) * d;
        double *end = ends + (size_t)k * d;
        double poses[12 * 64];
        int32_t P;
        if (agent_kind == 0) {
            double r[3];
            for (int j = 0; j < 3; ++j) r[j] = orc_engine_uniform(seed, g * 64 + 32 + j, -1.0, 1.0);
            omni_steer_from(r, from, end);
            P = orc_omni_get_poses(from, end, cc_dt, poses, 64);
        } else if (agent_kind == 1) {
            double awz[3];
            awz[0] = orc_engine_uniform(seed, g * 64 + 32, -1, 1);
            awz[1] = orc_engine_uniform(seed, g * 64 + 33, -0.1745, 0.1745);
            awz[2] = orc_engine_uniform(seed, g * 64 + 34, -1, 1);
            orc_blimp_do_step_cr(prm, from, awz[0], awz[1], awz[2], steer_dt, end);
            P = orc_blimp_get_poses_cr(prm, from, awz, steer_dt, cc_dt, poses, 64);
        } else {
            double aw[2];
            aw[0] = orc_engine_uniform(seed, g * 64 + 32, -0.1, 1);
            aw[1] = orc_engine_uniform(seed, g * 64 + 33, -M_PI / 18., M_PI / 18.);
            orc_snake_do_step_cr(prm, from, aw[0], aw[1], steer_dt, end);
            P = orc_snake_get_poses_cr(prm, from, aw, steer_dt, cc_dt, poses, 64 / L);
        }
        if (P > 64 / L) P = 64 / L;
        int hit = 0;
        for (int32_t p = 0; p < P && !hit; ++p)
            for (int l = 0; l < L && !hit; ++l)
                hit = orc_collide_unit_bvh(env, env_tf, agent_tris, Ta, poses + 12 * ((size_t)p * L + l), NULL);
        verdict_out[k] = (uint8_t)hit;
    }
    int64_t n = n_nodes;
    for (int32_t k = 0; k < K; ++k) {
        if (verdict_out[k]) continue;
        if (n >= capacity) break;
        memcpy(nodes + n * d, ends + (size_t)k * d, sizeof(double) * (size_t)d);
        parents[n] = ids[k];
        ++n;
    }
    free(samples); free(ends); free(d2);
    return n;
}

/* ======================================================================
 * The reference's own sequential loop at a given tree size (CPU baseline leg): RRT::query
 * (planners/rrt.hpp:42-94) one extension at a time against the current tree, with
 * FLANN_KDTreeWrapper::insertPoint (utilities/flannkdtreewrapper.hpp:27-40) calling
 * addPoints(point, 2) -> [upstream FLANN 1.8.4] KDTreeSingleIndex::buildIndex() over every point
 * after each insertion.  Samples and controls come from the engine's counter-based streams
 * (extension g = ext_base + i), so the first extensions equal the batched round's when no
 * earlier one was inserted.  Stops after max_ext extensions or time_budget seconds.
 * ====================================================================== */
static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

int64_t orc_rrt_seq_rebuild(int32_t agent_kind, const double *prm, int32_t d, const double *ranges,
                            double steer_dt, double cc_dt, uint64_t seed, uint64_t ext_base, int64_t max_ext,
                            double time_budget, const orc_bvh *env, const double env_tf[12],
                            const double *agent_tris, int64_t Ta, double *nodes, int32_t *parents,
                            int64_t n_nodes, int64_t capacity, int64_t *ext_done, double *seconds) {
    const int L = agent_kind == 2 ? (int)prm[0] + 1 : 1;
    double sample[64], end[64], poses[12 * 64];
    int64_t n = n_nodes, valid = 0, i = 0;
    const double t0 = now_s();
    orc_kdtree *t = orc_kdtree_build(nodes, n, d);
    for (; i < max_ext && n < capacity; ++i) {
        if (now_s() - t0 > time_budget) break;
        const uint64_t g = ext_base + (uint64_t)i;
        for (int32_t j = 0; j < d; ++j) sample[j] = orc_engine_uniform(seed, g * 64 + j, ranges[2 * j], ranges[2 * j + 1]);
        int32_t id;
        double d2;
        orc_kdtree_knn(t, sample, 1, 1, &id, &d2, 1);
        const double *from = nodes + (int64_t)(id - 1) * d;
        int32_t P;
        if (agent_kind == 0) {
            double r[3];
            for (int j = 0; j < 3; ++j) r[j] = orc_engine_uniform(seed, g * 64 + 32 + j, -1.0, 1.0);
            omni_steer_from(r, from, end);
            P = orc_omni_get_poses(from, end, cc_dt, poses, 64);
        } else if (agent_kind == 1) {
            double awz[3];
            awz[0] = orc_engine_uniform(seed, g * 64 + 32, -1, 1);
            awz[1] = orc_engine_uniform(seed, g * 64 + 33, -0.1745, 0.1745);
            awz[2] = orc_engine_uniform(seed, g * 64 + 34, -1, 1);
            orc_blimp_do_step_cr(prm, from, awz[0], awz[1], awz[2], steer_dt, end);
            P = orc_blimp_get_poses_cr(prm, from, awz, steer_dt, cc_dt, poses, 64);
        } else {
            double aw[2];
            aw[0] = orc_engine_uniform(seed, g * 64 + 32, -0.1, 1);
            aw[1] = orc_engine_uniform(seed, g * 64 + 33, -M_PI / 18., M_PI / 18.);
            orc_snake_do_step_cr(prm, from, aw[0], aw[1], steer_dt, end);
            P = orc_snake_get_poses_cr(prm, from, aw, steer_dt, cc_dt, poses, 64 / L);
        }
        if (P > 64 / L) P = 64 / L;
        int hit = 0;
        for (int32_t p = 0; p < P && !hit; ++p)
            for (int l = 0; l < L && !hit; ++l)
                hit = orc_collide_unit_bvh(env, env_tf, agent_tris, Ta, poses + 12 * ((size_t)p * L + l), NULL);
        if (hit) continue;
        memcpy(nodes + n * d, end, sizeof(double) * (size_t)d);
        parents[n] = id;
        ++n;
        ++valid;
        /* insertPoint -> addPoints -> buildIndex over all n points */
        orc_kdtree_free(t);
        t = orc_kdtree_build(nodes, n, d);
    }
    orc_kdtree_free(t);
    *ext_done = i;
    *seconds = now_s() - t0;
    return valid;
}

/* ======================================================================
 * PRM construction: planners/prm/prm.hpp:334-387 (addMilestone), omnidirectional agent.
 * Milestones are added in order, `batch` at a time (1 = the reference's sequence); each is
 * connected to its k nearest earlier milestones (exact kNN over the first 3 state vars,
 * prm.hpp:155 KDTree(..., 3, 0) and :350 kNearest(.., 10); milestones of one batch do not
 * see each other) through Omnidirectional::steer(s, t, 1000) (omnidirectional.hpp:144-162:
 * end = s + (t - s) * min(1, 1000 / |t - s|), cost = |t - s|) and Map3D::safeEdge over
 * Omnidirectional::getPoses(edge, dt).  A safe edge is recorded as (target, source) with
 * its cost and unites the two components (prm.hpp:372-376).
 * ====================================================================== */
static int32_t uf_find(int32_t *p, int32_t x) {
    while (p[x] != x) {
        p[x] = p[p[x]];
        x = p[x];
    }
    return x;
}

int64_t orc_prm_build(const orc_bvh *env, const double env_tf[12], const double *agent_tris, int64_t Ta,
                      const double *states, int64_t n, int32_t k, int32_t batch, double cc_dt,
                      int32_t *edges, double *costs, int64_t cap, int32_t *comp) {
    if (batch < 1) batch = 1;
    double *keys = (double *)malloc(sizeof(double) * 3 * (size_t)(n > 0 ? n : 1));
    int32_t *parent = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
    int32_t *ids = (int32_t *)malloc(sizeof(int32_t) * (size_t)k);
    double *d2 = (double *)malloc(sizeof(double) * (size_t)k);
    int32_t maxP = 1 << 20;
    double *poses = (double *)malloc(sizeof(double) * 12 * (size_t)maxP);
    int64_t ne = 0;
    for (int64_t i = 0; i < n; ++i) {
        memcpy(keys + 3 * i, states + 3 * i, 3 * sizeof(double));
        parent[i] = (int32_t)i;
    }
    for (int64_t b0 = 0; b0 < n; b0 += batch) {
        const int64_t b1 = b0 + batch < n ? b0 + batch : n;
        for (int64_t i = b0; i < b1; ++i) {
            orc_knn(keys, NULL, b0, 3, keys + 3 * i, 1, k, ids, d2);
            const double *s = states + 3 * i;
            for (int32_t j = 0; j < k; ++j) {
                if (ids[j] < 0) break;
                const int32_t tgt = ids[j] - 1;
                const double *t = states + 3 * tgt;
                const double dx = t[0] - s[0], dy = t[1] - s[1], dz = t[2] - s[2];
                const double dist = sqrt(dx * dx + dy * dy + dz * dz);
                double fraction = 1000.0 / dist;
                if (fraction > 1) fraction = 1;
                const double end[3] = {s[0] + dx * fraction, s[1] + dy * fraction, s[2] + dz * fraction};
                const int32_t P = orc_omni_get_poses(s, end, cc_dt, poses, maxP);
                int hit = 0;
                for (int32_t p = 0; p < P && p < maxP && !hit; ++p)
                    hit = orc_collide_unit_bvh(env, env_tf, agent_tris, Ta, poses + 12 * p, NULL);
                if (hit) continue;
                if (ne < cap) {
                    edges[2 * ne] = tgt;
                    edges[2 * ne + 1] = (int32_t)i;
                    costs[ne] = dist;
                }
                ++ne;
                const int32_t ra = uf_find(parent, tgt), rb = uf_find(parent, (int32_t)i);
                if (ra != rb) parent[ra > rb ? ra : rb] = ra < rb ? ra : rb;
            }
        }
    }
    /* component label = smallest milestone of the component (roots are minimal by construction) */
    for (int64_t i = 0; i < n; ++i) comp[i] = uf_find(parent, (int32_t)i);
    free(keys);
    free(parent);
    free(ids);
    free(d2);
    free(poses);
    return ne <= cap ? ne : -1;
}

/* ======================================================================
 * Mesh-vs-mesh distance: FCL 0.3.2 TriangleDistance [upstream] (a port of PQP's
 * TriDist.cpp), called by MeshDistanceTraversalNode leaf tests under fcl::distance, which
 * utilities/fcl_helpers.hpp:67-84 (defaultDistanceFunction) drives over the broadphase.
 * ====================================================================== */

static void seg_pts(const double P[3], const double A[3], const double Q[3], const double B[3],
                    double VEC[3], double X[3], double Y[3]) {
    double T[3], TMP[3], W[3];
    int k;
    sub3(Q, P, T);
    const double AA = dot3(A, A), BB = dot3(B, B), AB = dot3(A, B), AT = dot3(A, T), BT = dot3(B, T);
    const double denom = AA * BB - AB * AB;
    double t = (AT * BB - BT * AB) / denom;
    if ((t < 0) || isnan(t)) t = 0;
    else if (t > 1) t = 1;
    double u = (t * AB - BT) / BB;
    if ((u <= 0) || isnan(u)) {
        for (k = 0; k < 3; ++k) Y[k] = Q[k];
        t = AT / AA;
        if ((t <= 0) || isnan(t)) {
            for (k = 0; k < 3; ++k) X[k] = P[k];
            sub3(Q, P, VEC);
        } else if (t >= 1) {
            for (k = 0; k < 3; ++k) X[k] = P[k] + A[k];
            sub3(Q, X, VEC);
        } else {
            for (k = 0; k < 3; ++k) X[k] = P[k] + A[k] * t;
            cross3(T, A, TMP);
            cross3(A, TMP, VEC);
        }
    } else if (u >= 1) {
        for (k = 0; k < 3; ++k) Y[k] = Q[k] + B[k];
        t = (AB + AT) / AA;
        if ((t <= 0) || isnan(t)) {
            for (k = 0; k < 3; ++k) X[k] = P[k];
            sub3(Y, P, VEC);
        } else if (t >= 1) {
            for (k = 0; k < 3; ++k) X[k] = P[k] + A[k];
            sub3(Y, X, VEC);
        } else {
            for (k = 0; k < 3; ++k) X[k] = P[k] + A[k] * t;
            sub3(Y, P, W);
            cross3(W, A, TMP);
            cross3(A, TMP, VEC);
        }
    } else {
        for (k = 0; k < 3; ++k) Y[k] = Q[k] + B[k] * u;
        if ((t <= 0) || isnan(t)) {
            for (k = 0; k < 3; ++k) X[k] = P[k];
            cross3(T, B, TMP);
            cross3(B, TMP, VEC);
        } else if (t >= 1) {
            for (k = 0; k < 3; ++k) X[k] = P[k] + A[k];
            sub3(Q, X, W);
            cross3(W, B, TMP);
            cross3(B, TMP, VEC);
        } else {
            for (k = 0; k < 3; ++k) X[k] = P[k] + A[k] * t;
            cross3(A, B, VEC);
            if (dot3(VEC, T) < 0)
                for (k = 0; k < 3; ++k) VEC[k] = VEC[k] * -1.0;
        }
    }
}

double orc_tri_distance(const double S_[9], const double T_[9]) {
    const double *S[3] = {S_, S_ + 3, S_ + 6}, *T[3] = {T_, T_ + 3, T_ + 6};
    double Sv[3][3], Tv[3][3], VEC[3], P[3], Q[3], V[3], Z[3];
    int i, j, k, shown_disjoint = 0;
    for (i = 0; i < 3; ++i) {
        sub3(S[(i + 1) % 3], S[i], Sv[i]);
        sub3(T[(i + 1) % 3], T[i], Tv[i]);
    }
    sub3(S[0], T[0], V);
    double mindd = dot3(V, V) + 1; /* first minimum safely high */
    for (i = 0; i < 3; ++i)
        for (j = 0; j < 3; ++j) {
            seg_pts(S[i], Sv[i], T[j], Tv[j], VEC, P, Q);
            sub3(Q, P, V);
            const double dd = dot3(V, V);
            if (dd <= mindd) {
                mindd = dd;
                sub3(S[(i + 2) % 3], P, Z);
                double a = dot3(Z, VEC);
                sub3(T[(j + 2) % 3], Q, Z);
                double b = dot3(Z, VEC);
                if ((a <= 0) && (b >= 0)) return sqrt(dd);
                const double p = dot3(V, VEC);
                if (a < 0) a = 0;
                if (b > 0) b = 0;
                if ((p - a + b) > 0) shown_disjoint = 1;
            }
        }
    /* case 1: a vertex of one triangle over the face of the other; first T over S */
    for (int side = 0; side < 2; ++side) {
        const double *const *A = side == 0 ? S : T, *const *B = side == 0 ? T : S;
        double (*Av)[3] = side == 0 ? Sv : Tv;
        double N[3];
        cross3(Av[0], Av[1], N);
        const double Nl = dot3(N, N);
        if (!(Nl > 1e-15)) continue;
        double Bp[3];
        for (k = 0; k < 3; ++k) {
            sub3(A[0], B[k], V);
            Bp[k] = dot3(V, N);
        }
        int point = -1;
        if ((Bp[0] > 0) && (Bp[1] > 0) && (Bp[2] > 0)) {
            point = (Bp[0] < Bp[1]) ? 0 : 1;
            if (Bp[2] < Bp[point]) point = 2;
        } else if ((Bp[0] < 0) && (Bp[1] < 0) && (Bp[2] < 0)) {
            point = (Bp[0] > Bp[1]) ? 0 : 1;
            if (Bp[2] > Bp[point]) point = 2;
        }
        if (point < 0) continue;
        shown_disjoint = 1;
        int inside = 1;
        for (k = 0; k < 3 && inside; ++k) {
            sub3(B[point], A[k], V);
            cross3(N, Av[k], Z);
            inside = dot3(V, Z) > 0;
        }
        if (!inside) continue;
        double F[3];
        for (k = 0; k < 3; ++k) F[k] = B[point][k] + N[k] * (Bp[point] / Nl);
        sub3(F, B[point], V);
        return sqrt(dot3(V, V));
    }
    if (shown_disjoint) return sqrt(mindd); /* FCL also returns minP / minQ as the points */
    /* overlap answer, gated on the exact boxes (the build's definition) */
    return tri_gate(S_, T_) ? 0.0 : sqrt(mindd);
}

/* exact box gap between two triangles, a lower bound on any distance between them */
static double tri_gap2(const double *A, const double *B) {
    double alo[3], ahi[3], blo[3], bhi[3], s = 0;
    tri_box(A, alo, ahi);
    tri_box(B, blo, bhi);
    for (int k = 0; k < 3; ++k) {
        double g = fmax(fmax(alo[k] - bhi[k], blo[k] - ahi[k]), 0.0);
        s += g * g;
    }
    return s;
}

double orc_distance_unit(const double *env_tris, int64_t Te, const double env_tf[12],
                         const double *agent_tris, int64_t Ta, const double pose[12]) {
    double R[9], T[3], Qp[9];
    double best = DBL_MAX;
    unit_RT(env_tf, pose, R, T);
    for (int64_t b = 0; b < Ta && best > 0; ++b) {
        map_tri(R, T, agent_tris + 9 * b, Qp);
        for (int64_t a = 0; a < Te && best > 0; ++a) {
            /* the gap is a lower bound on the computed distance up to rounding; the slack
             * keeps every pair that could reach the minimum */
            const double thr = best * (1 + 1e-9) + 1e-9;
            if (tri_gap2(env_tris + 9 * a, Qp) > thr * thr) continue;
            const double d = orc_tri_distance(env_tris + 9 * a, Qp);
            if (d < best) best = d;
        }
    }
    return best;
}

void orc_distance_batch(const double *env_tris, int64_t Te, const double env_tf[12],
                        const double *agent_tris, const int64_t *link_tri_off, int32_t L,
                        const double *poses, const int64_t *edge_pose_offsets, int64_t E,
                        double *dist, int nthreads) {
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1)
#endif
    for (int64_t e = 0; e < E; ++e) {
        double best = DBL_MAX;
        for (int64_t p = edge_pose_offsets[e]; p < edge_pose_offsets[e + 1] && best > 0; ++p)
            for (int32_t l = 0; l < L && best > 0; ++l) {
                const double d = orc_distance_unit(env_tris, Te, env_tf, agent_tris + 9 * link_tri_off[l],
                                                   link_tri_off[l + 1] - link_tri_off[l], poses + 12 * (p * L + l));
                if (d < best) best = d;
            }
        dist[e] = best;
    }
    (void)nthreads;
}

/* ======================================================================
 * PRM with radius neighbours (config 4): planners/prm/prm.hpp:334-387 (addMilestone) with
 * FLANN_KDTreeWrapper::kNearestWithin (utilities/flannkdtreewrapper.hpp:91-117) as the NN.
 * ====================================================================== */
int64_t orc_prm_radius(const orc_bvh *env, const double env_tf[12], const double *agent_tris, int64_t Ta,
                       const double *states, int64_t n, int32_t dim, double r2, double cc_dt,
                       int32_t *edges, uint8_t *verdict, int64_t cap, int32_t *comp, int nthreads) {
    /* neighbours of each milestone among the earlier ones, in (i, j) order */
    int64_t E = 0, ecap = 1024;
    int32_t *ei = (int32_t *)malloc(sizeof(int32_t) * 2 * (size_t)ecap);
    for (int64_t i = 0; i < n; ++i) {
        double ki[3];
        memcpy(ki, states + i * dim, sizeof ki);
        for (int64_t j = 0; j < i; ++j) {
            double kj[3];
            memcpy(kj, states + j * dim, sizeof kj);
            if (!(orc_l2(ki, kj, 3) < r2)) continue;
            if (E == ecap) {
                ecap *= 2;
                ei = (int32_t *)realloc(ei, sizeof(int32_t) * 2 * (size_t)ecap);
            }
            ei[2 * E] = (int32_t)i;
            ei[2 * E + 1] = (int32_t)j;
            ++E;
        }
    }
    uint8_t *v = (uint8_t *)calloc((size_t)(E > 0 ? E : 1), 1);
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 16) num_threads(nthreads > 0 ? nthreads : 1)
#endif
    for (int64_t e = 0; e < E; ++e) {
        const double *s = states + (int64_t)ei[2 * e] * dim, *g = states + (int64_t)ei[2 * e + 1] * dim;
        /* Omnidirectional::steer(start, goal, 1000) */
        const double dx = g[0] - s[0], dy = g[1] - s[1], dz = g[2] - s[2];
        const double dist = sqrt(dx * dx + dy * dy + dz * dz);
        double fraction = 1000.0 / dist;
        if (fraction > 1) fraction = 1;
        const double end[3] = {s[0] + dx * fraction, s[1] + dy * fraction, s[2] + dz * fraction};
        const int32_t P = orc_omni_get_poses(s, end, cc_dt, NULL, 0);
        double *poses = (double *)malloc(sizeof(double) * 12 * (size_t)(P > 0 ? P : 1));
        orc_omni_get_poses(s, end, cc_dt, poses, P);
        if (dim == 7) { /* Blimp::stateToFCLTransform's R from milestone i's yaw */
            const double c = cos(s[3]), sn = sin(s[3]);
            for (int32_t p = 0; p < P; ++p) {
                double *R = poses + 12 * p;
                R[0] = c; R[1] = sn; R[2] = 0; R[3] = -sn; R[4] = c; R[5] = 0; R[6] = 0; R[7] = 0; R[8] = 1;
            }
        }
        int hit = 0;
        for (int32_t p = 0; p < P && !hit; ++p) hit = orc_collide_unit_bvh(env, env_tf, agent_tris, Ta, poses + 12 * p, NULL);
        v[e] = (uint8_t)hit;
        free(poses);
    }
    (void)nthreads;
    int32_t *parent = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
    for (int64_t i = 0; i < n; ++i) parent[i] = (int32_t)i;
    for (int64_t e = 0; e < E; ++e) {
        if (v[e]) continue;
        const int32_t a = uf_find(parent, ei[2 * e]), b = uf_find(parent, ei[2 * e + 1]);
        if (a != b) parent[a > b ? a : b] = a < b ? a : b;
    }
    for (int64_t e = 0; e < E && e < cap; ++e) {
        edges[2 * e] = ei[2 * e];
        edges[2 * e + 1] = ei[2 * e + 1];
        verdict[e] = v[e];
    }
    if (comp)
        for (int64_t i = 0; i < n; ++i) comp[i] = uf_find(parent, (int32_t)i);
    free(ei);
    free(v);
    free(parent);
    return E;
}

/* ======================================================================
 * Self-collision: MeshHandler::isInCollision's checkSelfCollision branch
 * (utilities/meshhandler.hpp:205-219): every pair of distinct link objects of a pose.
 * ====================================================================== */
static int self_collide_pose(const double *agent_tris, const int64_t *off, int32_t L, const double *pose) {
    for (int32_t j = 0; j < L; ++j)
        for (int32_t k = j + 1; k < L; ++k) {
            const double *pj = pose + 12 * j, *pk = pose + 12 * k;
            double R[9], T[3], Qp[9];
            orc_relative_transform(pj, pj + 9, pk, pk + 9, R, T);
            for (int64_t b = off[k]; b < off[k + 1]; ++b) {
                map_tri(R, T, agent_tris + 9 * b, Qp);
                for (int64_t a = off[j]; a < off[j + 1]; ++a)
                    if (tri_gate(agent_tris + 9 * a, Qp) && orc_tri_intersect(agent_tris + 9 * a, Qp)) return 1;
            }
        }
    return 0;
}

void orc_self_collide_batch(const double *agent_tris, const int64_t *link_tri_off, int32_t L, const double *poses,
                            const int64_t *edge_pose_offsets, int64_t E, uint8_t *verdict) {
    for (int64_t e = 0; e < E; ++e) {
        int hit = 0;
        for (int64_t p = edge_pose_offsets[e]; p < edge_pose_offsets[e + 1] && !hit; ++p)
            hit = self_collide_pose(agent_tris, link_tri_off, L, poses + 12 * L * p);
        verdict[e] = (uint8_t)hit;
    }
}

/* ======================================================================
 * PRMLite::generateEdges (discretizations/workspace/prmlite.hpp:128-164) with
 * PRMLite::interpolate (:181-203): translation steps accumulated from vertex i toward j, the
 * rotation of vertex i, endpoints excluded; no steps = an edge without poses (kept).
 * ====================================================================== */
void orc_prmlite_edges(const orc_bvh *env, const double env_tf[12], const double *agent_tris, int64_t Ta,
                       const double *verts, int64_t V, double step, uint8_t *collides, int nthreads) {
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 4) num_threads(nthreads > 0 ? nthreads : 1)
#endif
    for (int64_t i = 0; i < V; ++i) {
        const int64_t row = i * (2 * V - i - 1) / 2;
        double pose[12];
        memcpy(pose, verts + 12 * i, 9 * sizeof(double));
        for (int64_t j = i + 1; j < V; ++j) {
            const double *v1 = verts + 12 * i + 9, *v2 = verts + 12 * j + 9;
            double diff[3];
            sub3(v1, v2, diff);
            const double dist = sqrt(dot3(diff, diff));
            const double q = dist / step;
            const unsigned int steps = (q >= 4294967296.0 || !(q >= 0)) ? 0u : (unsigned int)q;
            int hit = 0;
            if (steps > 0) {
                const double vs[3] = {(v2[0] - v1[0]) / (double)steps, (v2[1] - v1[1]) / (double)steps,
                                      (v2[2] - v1[2]) / (double)steps};
                pose[9] = v1[0]; pose[10] = v1[1]; pose[11] = v1[2];
                for (unsigned int s = 0; s < steps && !hit; ++s) {
                    for (int k = 0; k < 3; ++k) pose[9 + k] = pose[9 + k] + vs[k];
                    hit = orc_collide_unit_bvh(env, env_tf, agent_tris, Ta, pose, NULL);
                }
            }
            collides[row + (j - i - 1)] = (uint8_t)hit;
        }
    }
    (void)nthreads;
}

/* ======================================================================
 * GridDiscretization (discretizations/workspace/griddiscretization.hpp:9-36, getGridCenter
 * :111-124 as written) with getRepresentivePosesForLocation (agents/omnidirectional.hpp:191-200,
 * blimp.hpp:194-217, snake_trailers.hpp:220-244).
 * ====================================================================== */
int64_t orc_grid_discretization(const orc_bvh *env, const double env_tf[12], const double *agent_tris, int64_t Ta,
                                const double bounds[6], const double sizes[3], int32_t n_rot, uint8_t *free_out,
                                int64_t cap) {
    unsigned int dims[3], cells = 1;
    for (int i = 0; i < 3; ++i) {
        const double range = fabs(bounds[2 * i] - bounds[2 * i + 1]);
        dims[i] = range == 0 ? 1u : (unsigned int)ceil(range / sizes[i]);
        cells *= dims[i];
    }
    for (unsigned int n = 0; n < cells && (int64_t)n < cap; ++n) {
        double c[3];
        c[0] = bounds[0] + (double)(n % dims[0]) * sizes[0] + sizes[0] * 0.5;
        unsigned int prev = 1;
        for (int i = 1; i < 3; ++i) {
            prev *= dims[i];
            c[i] = bounds[2 * i] + (double)(n / prev % dims[i]) * sizes[i] + sizes[1] * 0.5;
        }
        int hit = 0;
        const double increment = M_PI / ((double)4 * 2.);
        for (int r = 0; r < n_rot && !hit; ++r) {
            double pose[12] = {1, 0, 0, 0, 1, 0, 0, 0, 1, c[0], c[1], c[2]};
            if (n_rot > 1) {
                const double cs = cos((double)r * increment), sn = sin((double)r * increment);
                pose[0] = cs; pose[1] = sn; pose[3] = -sn; pose[4] = cs;
            }
            hit = orc_collide_unit_bvh(env, env_tf, agent_tris, Ta, pose, NULL);
        }
        free_out[n] = (uint8_t)!hit;
    }
    return (int64_t)cells;
}
