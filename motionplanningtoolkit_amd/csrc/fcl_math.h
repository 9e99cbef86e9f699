// fcl_math.h -- FP64 geometry in FCL 0.3.2 operation order, shared by the HIP kernels
// and the host-side precomputation of environment triangle records.
//
// Bit-exactness contract: every expression below is written in the order FCL 0.3.2
// evaluates it ([upstream] fcl/math/vec_3f.h, matrix_3f.h, intersect.cpp) and the
// whole library is compiled with -ffp-contract=off, so no a*b+c is fused on either
// the host (x86-64) or the device (gfx950).  The verdict of tri_intersect() is the
// AND of the 17 project6() tests, so the tests may run in any order.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#pragma clang fp contract(off)

#define MPT_HD __host__ __device__ __forceinline__

namespace mpt {

struct v3 {
    double x, y, z;
};

MPT_HD v3 mk(double x, double y, double z) { return v3{x, y, z}; }
MPT_HD v3 sub(v3 a, v3 b) { return v3{a.x - b.x, a.y - b.y, a.z - b.z}; }
// Vec3Data::dot: x*x' + y*y' + z*z' evaluated left to right
MPT_HD double dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
// Vec3Data::cross
MPT_HD v3 cross(v3 a, v3 b) {
    return v3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
MPT_HD double dmax(double a, double b) { return a < b ? b : a; }  // std::max
MPT_HD double dmin(double a, double b) { return b < a ? b : a; }  // std::min

// Matrix3f * Vec3f + T (dotX/dotY/dotZ, then the translation add).
MPT_HD v3 xform(const double R[9], const double T[3], v3 q) {
    const double r0 = R[0] * q.x + R[1] * q.y + R[2] * q.z;
    const double r1 = R[3] * q.x + R[4] * q.y + R[5] * q.z;
    const double r2 = R[6] * q.x + R[7] * q.y + R[8] * q.z;
    return v3{r0 + T[0], r1 + T[1], r2 + T[2]};
}

// fcl::relativeTransform(R1, T1, R2, T2): R = R1^T R2, T = R1^T (T2 - T1).
MPT_HD void relative_transform(const double R1[9], const double T1[3], const double R2[9],
                               const double T2[3], double R[9], double T[3]) {
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
            R[i * 3 + j] = R1[0 * 3 + i] * R2[0 * 3 + j] + R1[1 * 3 + i] * R2[1 * 3 + j] +
                           R1[2 * 3 + i] * R2[2 * 3 + j];
    const double d0 = T2[0] - T1[0], d1 = T2[1] - T1[1], d2 = T2[2] - T1[2];
#pragma unroll
    for (int i = 0; i < 3; ++i) T[i] = R1[0 * 3 + i] * d0 + R1[1 * 3 + i] * d1 + R1[2 * 3 + i] * d2;
}

// Quaternion3f::toRotation, q = {w, x, y, z}.
MPT_HD void quat_to_rot(const double q[4], double R[9]) {
    const double w = q[0], x = q[1], y = q[2], z = q[3];
    const double twoX = 2.0 * x, twoY = 2.0 * y, twoZ = 2.0 * z;
    const double twoWX = twoX * w, twoWY = twoY * w, twoWZ = twoZ * w;
    const double twoXX = twoX * x, twoXY = twoY * x, twoXZ = twoZ * x;
    const double twoYY = twoY * y, twoYZ = twoZ * y, twoZZ = twoZ * z;
    R[0] = 1.0 - (twoYY + twoZZ); R[1] = twoXY - twoWZ;         R[2] = twoXZ + twoWY;
    R[3] = twoXY + twoWZ;         R[4] = 1.0 - (twoXX + twoZZ); R[5] = twoYZ - twoWX;
    R[6] = twoXZ - twoWY;         R[7] = twoYZ + twoWX;         R[8] = 1.0 - (twoXX + twoYY);
}

// Conservative float bounds: the margin (1e-6 absolute + 4e-7 relative) exceeds both
// the double->float rounding (<= 6e-8 relative) and the rounding error of the 17-axis
// test by many orders, so box pruning never removes a pair the all-pairs loop reports.
MPT_HD float widen_lo(double x) { return (float)(x - (1e-6 + 4e-7 * fabs(x))); }
MPT_HD float widen_hi(double x) { return (float)(x + (1e-6 + 4e-7 * fabs(x))); }

// Environment triangle record: everything intersect_Triangle derives from P alone,
// precomputed on the host with the same operations (so bit-identical), plus the exact
// vertex box of P that gates the test (see tri_gate), 48 doubles.
struct EnvTri {
    double P1[3];   // q_i = Q_i' - P1
    double p2[3];   // p2 = P2 - P1 (= e1, since p1 = P1 - P1 = 0)
    double p3[3];   // p3 = P3 - P1
    double e2[3];   // p3 - p2
    double e3[3];   // p1 - p3
    double n1[3];   // e1 x e2
    double g[3][3]; // e_i x n1
    double nP[2];   // min/max of {p1,p2,p3}.n1 (p1 term is +-0)
    double gP[3][2];// min/max of {p1,p2,p3}.g_i
    double lo[3];   // min over P1,P2,P3 (env-local, exact)
    double hi[3];   // max over P1,P2,P3
    double P2[3];   // the other two vertices as given (triangle distance)
    double P3[3];
    double pad[1];
};
static_assert(sizeof(EnvTri) == 48 * 8, "EnvTri layout");

inline void make_env_tri(const double *t, EnvTri &r) {
    const v3 P1 = mk(t[0], t[1], t[2]), P2 = mk(t[3], t[4], t[5]), P3 = mk(t[6], t[7], t[8]);
    const v3 p1 = sub(P1, P1), p2 = sub(P2, P1), p3 = sub(P3, P1);
    const v3 e1 = sub(p2, p1), e2 = sub(p3, p2), e3 = sub(p1, p3);
    const v3 n1 = cross(e1, e2);
    const v3 g[3] = {cross(e1, n1), cross(e2, n1), cross(e3, n1)};
    r.P1[0] = P1.x; r.P1[1] = P1.y; r.P1[2] = P1.z;
    r.p2[0] = e1.x; r.p2[1] = e1.y; r.p2[2] = e1.z;
    r.p3[0] = p3.x; r.p3[1] = p3.y; r.p3[2] = p3.z;
    r.e2[0] = e2.x; r.e2[1] = e2.y; r.e2[2] = e2.z;
    r.e3[0] = e3.x; r.e3[1] = e3.y; r.e3[2] = e3.z;
    r.n1[0] = n1.x; r.n1[1] = n1.y; r.n1[2] = n1.z;
    auto proj = [&](v3 ax, double *mnmx) {
        const double a = dot(ax, p1), b = dot(ax, p2), c = dot(ax, p3);
        mnmx[0] = dmin(a, dmin(b, c));
        mnmx[1] = dmax(a, dmax(b, c));
    };
    proj(n1, r.nP);
    for (int i = 0; i < 3; ++i) {
        r.g[i][0] = g[i].x; r.g[i][1] = g[i].y; r.g[i][2] = g[i].z;
        proj(g[i], r.gP[i]);
    }
    const double *v[3] = {t, t + 3, t + 6};
    for (int k = 0; k < 3; ++k) {
        r.lo[k] = dmin(v[0][k], dmin(v[1][k], v[2][k]));
        r.hi[k] = dmax(v[0][k], dmax(v[1][k], v[2][k]));
        r.P2[k] = t[3 + k];
        r.P3[k] = t[6 + k];
    }
    r.pad[0] = 0.0;
}

// FCL only runs intersect_Triangle on pairs whose leaf bounding volumes overlap
// (BVHCollisionTraversalNode: BVTesting before leafTesting); the exact closed AABB
// overlap of P and Q' is that gate here.  It matters for degenerate (collinear / point)
// triangles, for which intersect_Triangle finds no separating axis against any parallel
// counterpart however far away.  Every float box test in the kernels is a widened
// superset of this one, so pruning never changes a verdict.
MPT_HD bool tri_gate(const double lo[3], const double hi[3], v3 Q1, v3 Q2, v3 Q3) {
    const double qlo[3] = {dmin(Q1.x, dmin(Q2.x, Q3.x)), dmin(Q1.y, dmin(Q2.y, Q3.y)), dmin(Q1.z, dmin(Q2.z, Q3.z))};
    const double qhi[3] = {dmax(Q1.x, dmax(Q2.x, Q3.x)), dmax(Q1.y, dmax(Q2.y, Q3.y)), dmax(Q1.z, dmax(Q2.z, Q3.z))};
    return lo[0] <= qhi[0] && qlo[0] <= hi[0] && lo[1] <= qhi[1] && qlo[1] <= hi[1] && lo[2] <= qhi[2] &&
           qlo[2] <= hi[2];
}

// project6 with the P-side interval known: 0 = separated.
MPT_HD bool overlap_q(v3 ax, double mn1, double mx1, v3 q1, v3 q2, v3 q3) {
    const double Q1 = dot(ax, q1), Q2 = dot(ax, q2), Q3 = dot(ax, q3);
    const double mx2 = dmax(Q1, dmax(Q2, Q3));
    const double mn2 = dmin(Q1, dmin(Q2, Q3));
    if (mn1 > mx2) return false;
    if (mn2 > mx1) return false;
    return true;
}

// project6 for an axis depending on Q: P-side = {ax.p1 (= +-0), ax.p2, ax.p3}.
MPT_HD bool project6_p(v3 ax, v3 p2, v3 p3, v3 q1, v3 q2, v3 q3) {
    const double P1 = 0.0, P2 = dot(ax, p2), P3 = dot(ax, p3);
    const double mx1 = dmax(P1, dmax(P2, P3));
    const double mn1 = dmin(P1, dmin(P2, P3));
    return overlap_q(ax, mn1, mx1, q1, q2, q3);
}

// Intersect::intersect_Triangle(P1,P2,P3, Q1',Q2',Q3') with Q' already in the env frame.
// Returns true when no axis separates (touching counts as intersecting).
template <class ETri>
MPT_HD bool tri_intersect(const ETri &E, v3 Q1, v3 Q2, v3 Q3) {
    const v3 P1 = mk(E.P1[0], E.P1[1], E.P1[2]);
    const v3 q1 = sub(Q1, P1), q2 = sub(Q2, P1), q3 = sub(Q3, P1);
    const v3 n1 = mk(E.n1[0], E.n1[1], E.n1[2]);
    if (!overlap_q(n1, E.nP[0], E.nP[1], q1, q2, q3)) return false;
    const v3 p2 = mk(E.p2[0], E.p2[1], E.p2[2]);
    const v3 p3 = mk(E.p3[0], E.p3[1], E.p3[2]);
    const v3 f1 = sub(q2, q1), f2 = sub(q3, q2), f3 = sub(q1, q3);
    const v3 m1 = cross(f1, f2);
    if (!project6_p(m1, p2, p3, q1, q2, q3)) return false;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const v3 gi = mk(E.g[i][0], E.g[i][1], E.g[i][2]);
        if (!overlap_q(gi, E.gP[i][0], E.gP[i][1], q1, q2, q3)) return false;
    }
    const v3 e1 = p2;
    const v3 e2 = mk(E.e2[0], E.e2[1], E.e2[2]);
    const v3 e3 = mk(E.e3[0], E.e3[1], E.e3[2]);
    if (!project6_p(cross(e1, f1), p2, p3, q1, q2, q3)) return false;
    if (!project6_p(cross(e1, f2), p2, p3, q1, q2, q3)) return false;
    if (!project6_p(cross(e1, f3), p2, p3, q1, q2, q3)) return false;
    if (!project6_p(cross(e2, f1), p2, p3, q1, q2, q3)) return false;
    if (!project6_p(cross(e2, f2), p2, p3, q1, q2, q3)) return false;
    if (!project6_p(cross(e2, f3), p2, p3, q1, q2, q3)) return false;
    if (!project6_p(cross(e3, f1), p2, p3, q1, q2, q3)) return false;
    if (!project6_p(cross(e3, f2), p2, p3, q1, q2, q3)) return false;
    if (!project6_p(cross(e3, f3), p2, p3, q1, q2, q3)) return false;
    if (!project6_p(cross(f1, m1), p2, p3, q1, q2, q3)) return false;
    if (!project6_p(cross(f2, m1), p2, p3, q1, q2, q3)) return false;
    if (!project6_p(cross(f3, m1), p2, p3, q1, q2, q3)) return false;
    return true;
}

// tri_gate + tri_intersect from the env triangle's three vertices t[9] alone: every P-side
// quantity is recomputed with exactly make_env_tri's operations (so bitwise the record's
// fields) at its point of use, so a kernel can keep only the 72-B vertices on chip (LDS)
// and spend FP64 instead of dependent loads of the 384-B record.
// the env triangle's exact vertex box from its vertices t[9] (make_env_tri's lo / hi)
MPT_HD void tri_box_verts(const double *t, double lo[3], double hi[3]) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        lo[k] = dmin(t[k], dmin(t[3 + k], t[6 + k]));
        hi[k] = dmax(t[k], dmax(t[3 + k], t[6 + k]));
    }
}
MPT_HD bool tri_sat_verts(const double *t, v3 Q1, v3 Q2, v3 Q3);
MPT_HD bool tri_collide_verts(const double *t, v3 Q1, v3 Q2, v3 Q3) {
    double lo[3], hi[3];
    tri_box_verts(t, lo, hi);
    if (!tri_gate(lo, hi, Q1, Q2, Q3)) return false;
    return tri_sat_verts(t, Q1, Q2, Q3);
}
// intersect_Triangle from the env triangle's vertices (the P-side fields recomputed as
// make_env_tri does), without the box gate
MPT_HD bool tri_sat_verts(const double *t, v3 Q1, v3 Q2, v3 Q3) {
    const v3 P1 = mk(t[0], t[1], t[2]), P2 = mk(t[3], t[4], t[5]), P3 = mk(t[6], t[7], t[8]);
    const v3 p1 = sub(P1, P1), p2 = sub(P2, P1), p3 = sub(P3, P1);
    const v3 e1 = sub(p2, p1), e2 = sub(p3, p2), e3 = sub(p1, p3);
    // make_env_tri's proj(): min / max of {p1, p2, p3} . ax
    auto proj_overlap = [&](v3 ax, v3 q1, v3 q2, v3 q3) {
        const double a = dot(ax, p1), b = dot(ax, p2), c = dot(ax, p3);
        return overlap_q(ax, dmin(a, dmin(b, c)), dmax(a, dmax(b, c)), q1, q2, q3);
    };
    const v3 q1 = sub(Q1, P1), q2 = sub(Q2, P1), q3 = sub(Q3, P1);
    const v3 n1 = cross(e1, e2);
    if (!proj_overlap(n1, q1, q2, q3)) return false;
    const v3 f1 = sub(q2, q1), f2 = sub(q3, q2), f3 = sub(q1, q3);
    const v3 m1 = cross(f1, f2);
    // the record's p2 field holds e1 (make_env_tri); tri_intersect passes it as project6_p's p2
    if (!project6_p(m1, e1, p3, q1, q2, q3)) return false;
    if (!proj_overlap(cross(e1, n1), q1, q2, q3)) return false;
    if (!proj_overlap(cross(e2, n1), q1, q2, q3)) return false;
    if (!proj_overlap(cross(e3, n1), q1, q2, q3)) return false;
    if (!project6_p(cross(e1, f1), e1, p3, q1, q2, q3)) return false;
    if (!project6_p(cross(e1, f2), e1, p3, q1, q2, q3)) return false;
    if (!project6_p(cross(e1, f3), e1, p3, q1, q2, q3)) return false;
    if (!project6_p(cross(e2, f1), e1, p3, q1, q2, q3)) return false;
    if (!project6_p(cross(e2, f2), e1, p3, q1, q2, q3)) return false;
    if (!project6_p(cross(e2, f3), e1, p3, q1, q2, q3)) return false;
    if (!project6_p(cross(e3, f1), e1, p3, q1, q2, q3)) return false;
    if (!project6_p(cross(e3, f2), e1, p3, q1, q2, q3)) return false;
    if (!project6_p(cross(e3, f3), e1, p3, q1, q2, q3)) return false;
    if (!project6_p(cross(f1, m1), e1, p3, q1, q2, q3)) return false;
    if (!project6_p(cross(f2, m1), e1, p3, q1, q2, q3)) return false;
    if (!project6_p(cross(f3, m1), e1, p3, q1, q2, q3)) return false;
    return true;
}

MPT_HD v3 add(v3 a, v3 b) { return v3{a.x + b.x, a.y + b.y, a.z + b.z}; }
MPT_HD v3 scale(v3 a, double s) { return v3{a.x * s, a.y * s, a.z * s}; }

// TriangleDistance::segPoints ([upstream] FCL 0.3.2 intersect.cpp, PQP's SegPoints):
// closest points X on P + t A and Y on Q + u B, and VEC, the direction the caller tests
// the off-edge vertices against.
MPT_HD void seg_points(v3 P, v3 A, v3 Q, v3 B, v3 &VEC, v3 &X, v3 &Y) {
    const v3 T = sub(Q, P);
    const double AA = dot(A, A), BB = dot(B, B), AB = dot(A, B), AT = dot(A, T), BT = dot(B, T);
    const double denom = AA * BB - AB * AB;
    double t = (AT * BB - BT * AB) / denom;
    if (t < 0 || isnan(t)) t = 0;
    else if (t > 1) t = 1;
    const double u = (t * AB - BT) / BB;
    if (u <= 0 || isnan(u)) {
        Y = Q;
        t = AT / AA;
        if (t <= 0 || isnan(t)) {
            X = P;
            VEC = sub(Q, P);
        } else if (t >= 1) {
            X = add(P, A);
            VEC = sub(Q, X);
        } else {
            X = add(P, scale(A, t));
            VEC = cross(A, cross(T, A));
        }
    } else if (u >= 1) {
        Y = add(Q, B);
        t = (AB + AT) / AA;
        if (t <= 0 || isnan(t)) {
            X = P;
            VEC = sub(Y, P);
        } else if (t >= 1) {
            X = add(P, A);
            VEC = sub(Y, X);
        } else {
            X = add(P, scale(A, t));
            VEC = cross(A, cross(sub(Y, P), A));
        }
    } else {
        Y = add(Q, scale(B, u));
        if (t <= 0 || isnan(t)) {
            X = P;
            VEC = cross(B, cross(T, B));
        } else if (t >= 1) {
            X = add(P, A);
            VEC = cross(B, cross(sub(Q, X), B));
        } else {
            X = add(P, scale(A, t));
            VEC = cross(A, B);
            if (dot(VEC, T) < 0) VEC = scale(VEC, -1.0);
        }
    }
}

// seg_points without branches (the same values: each case's result is computed by the same
// operations and selected).  In a wave each lane takes its own case of the nested branches,
// so the branchy form runs the cases one after another; this form runs every lane through
// one straight path (three divisions and three cross-product chains).
MPT_HD v3 sel3(bool c, v3 a, v3 b) { return v3{c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z}; }
MPT_HD void seg_points_sel(v3 P, v3 A, v3 Q, v3 B, v3 &VEC, v3 &X, v3 &Y) {
    const v3 T = sub(Q, P);
    const double AA = dot(A, A), BB = dot(B, B), AB = dot(A, B), AT = dot(A, T), BT = dot(B, T);
    const double denom = AA * BB - AB * AB;
    double t = (AT * BB - BT * AB) / denom;
    if (t < 0 || isnan(t)) t = 0;
    else if (t > 1) t = 1;
    const double u = (t * AB - BT) / BB;
    const bool u0 = u <= 0 || isnan(u), u1 = !u0 && u >= 1, ue = u0 || u1;
    // u0 / u1: Y = Q or Q + B and t again from AT / AA or (AB + AT) / AA
    const double tt = (u0 ? AT : AB + AT) / AA;
    const v3 QB = add(Q, B), QBu = add(Q, scale(B, u));
    Y = u0 ? Q : (u1 ? QB : QBu);
    const double s = ue ? tt : t;  // the parameter X is placed at
    const bool c0 = s <= 0 || isnan(s), c1 = !c0 && s >= 1;
    const v3 PA = add(P, A), PAs = add(P, scale(A, s));
    X = c0 ? P : (c1 ? PA : PAs);
    // u0 / u1: Y - P, Y - X or A x ((Y - P) x A) (for u0, Y - P is T's subtraction);
    // interior u: B x ((Q - X) x B) at t = 0 or 1 (Q - P is T's), else +-(A x B)
    const v3 YP = sub(Y, P), YX = sub(Y, X), QX = sub(Q, X);
    const v3 D = ue ? A : B, W = ue ? YP : QX;
    const v3 VC = cross(D, cross(W, D));
    v3 VAB = cross(A, B);
    if (dot(VAB, T) < 0) VAB = scale(VAB, -1.0);
    VEC = ue ? (c0 ? YP : (c1 ? YX : VC)) : ((c0 || c1) ? VC : VAB);
}

// One triangle's vertex projected onto the other's plane, if it lies inside that face
// (the "case 1" test of TriangleDistance::triDistance).  Sn = normal of S, Snl = |Sn|^2,
// Sv = S's edge vectors; Tp[i] = (S0 - T_i).Sn.  Returns true and the distance if found;
// sets shown_disjoint when Sn separates.
MPT_HD bool face_vertex(const v3 S[3], const v3 Sv[3], v3 Sn, double Snl, const v3 T[3], bool s_first,
                        int &shown_disjoint, double &d) {
    const double Tp[3] = {dot(sub(S[0], T[0]), Sn), dot(sub(S[0], T[1]), Sn), dot(sub(S[0], T[2]), Sn)};
    int point = -1;
    if (Tp[0] > 0 && Tp[1] > 0 && Tp[2] > 0) {
        point = Tp[0] < Tp[1] ? 0 : 1;
        if (Tp[2] < Tp[point]) point = 2;
    } else if (Tp[0] < 0 && Tp[1] < 0 && Tp[2] < 0) {
        point = Tp[0] > Tp[1] ? 0 : 1;
        if (Tp[2] > Tp[point]) point = 2;
    }
    if (point < 0) return false;
    shown_disjoint = 1;
    // selects, not T[point] / Tp[point]: a dynamic index would put the arrays in scratch
    const v3 Tq = point == 0 ? T[0] : (point == 1 ? T[1] : T[2]);
    const double Tpp = point == 0 ? Tp[0] : (point == 1 ? Tp[1] : Tp[2]);
    if (!(dot(sub(Tq, S[0]), cross(Sn, Sv[0])) > 0)) return false;
    if (!(dot(sub(Tq, S[1]), cross(Sn, Sv[1])) > 0)) return false;
    if (!(dot(sub(Tq, S[2]), cross(Sn, Sv[2])) > 0)) return false;
    const v3 proj = add(Tq, scale(Sn, Tpp / Snl));
    // (P - Q).length() with P on S's face, Q the vertex of T
    const v3 V = s_first ? sub(proj, Tq) : sub(Tq, proj);
    d = sqrt(dot(V, V));
    return true;
}

// TriangleDistance::triDistance(S1..S3, T1..T3) ([upstream] FCL 0.3.2 intersect.cpp, PQP's
// TriDist) on T already mapped into S's frame (Q' = R Q + T, as for tri_intersect).
// Build-defined gate, the distance counterpart of tri_gate: the final "no edge pair or face
// vertex explains the minimum, so the triangles overlap -> 0" answer is given only when the
// exact boxes of S and T overlap; otherwise the edge-pair minimum is returned.  For
// non-degenerate triangles the two agree (overlapping triangles have overlapping boxes);
// for collinear ones FCL's answer is 0 at any distance.
// kUnroll = 1: rolled loops (about 100 fewer VGPRs); 3: fully unrolled (the rotations become
// register renames).  The same operations in the same order either way.
template <int kUnroll = 3, bool kSel = false>
MPT_HD double tri_distance(const v3 S[3], const double slo[3], const double shi[3], const v3 T[3]) {
    // The 9 edge pairs in triDistance's order (i over S's edges, j over T's), as rolled loops:
    // the triangles are rotated one vertex per step, so edge i / j is always vertex 0 -> 1 of
    // the rotated triple and the off-edge vertex is vertex 2 (S[(i+2)%3], T[(j+2)%3]); edge
    // vectors are recomputed from the vertices by the same subtraction.  Unrolled, the nine
    // segPoints kept ~220 VGPRs live (2 waves per SIMD); the values and their order of
    // operations are unchanged, so results are bitwise those of the unrolled form.
    const v3 D0 = sub(S[0], T[0]);
    double mindd = dot(D0, D0) + 1;
    int shown_disjoint = 0;
    // the rotating copies are the only vertex registers: three rotations bring each triple
    // back, so after the loops they are S and T again (S / T themselves are not kept live)
    v3 s0 = S[0], s1 = S[1], s2 = S[2];
    v3 t0 = T[0], t1 = T[1], t2 = T[2];
#pragma unroll kUnroll
    for (int i = 0; i < 3; ++i) {
        const v3 sv = sub(s1, s0);
#pragma unroll kUnroll
        for (int j = 0; j < 3; ++j) {
            const v3 tv = sub(t1, t0);
            v3 VEC, P, Q;
            if constexpr (kSel) seg_points_sel(s0, sv, t0, tv, VEC, P, Q);
            else seg_points(s0, sv, t0, tv, VEC, P, Q);
            const v3 V = sub(Q, P);
            const double dd = dot(V, V);
            if (dd <= mindd) {
                mindd = dd;
                double a = dot(sub(s2, P), VEC);
                double b = dot(sub(t2, Q), VEC);
                if (a <= 0 && b >= 0) return sqrt(dd);
                const double p = dot(V, VEC);
                if (a < 0) a = 0;
                if (b > 0) b = 0;
                if (p - a + b > 0) shown_disjoint = 1;
            }
            const v3 tt = t0;
            t0 = t1;
            t1 = t2;
            t2 = tt;
        }
        const v3 ss = s0;
        s0 = s1;
        s1 = s2;
        s2 = ss;
    }
    double d;
    const v3 Sx[3] = {s0, s1, s2}, Tx[3] = {t0, t1, t2};
    {
        const v3 Sv[3] = {sub(Sx[1], Sx[0]), sub(Sx[2], Sx[1]), sub(Sx[0], Sx[2])};
        const v3 Sn = cross(Sv[0], Sv[1]);
        const double Snl = dot(Sn, Sn);
        if (Snl > 1e-15 && face_vertex(Sx, Sv, Sn, Snl, Tx, true, shown_disjoint, d)) return d;
    }
    {
        const v3 Tv[3] = {sub(Tx[1], Tx[0]), sub(Tx[2], Tx[1]), sub(Tx[0], Tx[2])};
        const v3 Tn = cross(Tv[0], Tv[1]);
        const double Tnl = dot(Tn, Tn);
        if (Tnl > 1e-15 && face_vertex(Tx, Tv, Tn, Tnl, Sx, false, shown_disjoint, d)) return d;
    }
    if (shown_disjoint) return sqrt(mindd);
    const double tlo[3] = {dmin(Tx[0].x, dmin(Tx[1].x, Tx[2].x)), dmin(Tx[0].y, dmin(Tx[1].y, Tx[2].y)),
                           dmin(Tx[0].z, dmin(Tx[1].z, Tx[2].z))};
    const double thi[3] = {dmax(Tx[0].x, dmax(Tx[1].x, Tx[2].x)), dmax(Tx[0].y, dmax(Tx[1].y, Tx[2].y)),
                           dmax(Tx[0].z, dmax(Tx[1].z, Tx[2].z))};
    const bool boxes = slo[0] <= thi[0] && tlo[0] <= shi[0] && slo[1] <= thi[1] && tlo[1] <= shi[1] &&
                       slo[2] <= thi[2] && tlo[2] <= shi[2];
    return boxes ? 0.0 : sqrt(mindd);
}

// ---------------------------------------------------------------------------------------
// Correctly rounded sin / cos / tan: the trigonometry of the batched engine's steering (blimp
// doStep, snake doStep, their stateToFCLTransform rotations).  The reference calls std::sin /
// cos / tan, i.e. the host libm; glibc's are not correctly rounded (about 0.15 % of sin / cos
// and 0.23 % of tan arguments come out 1 ulp off) and differ between its FMA and SSE2
// variants, so the engine uses the implementation-independent definition, the correctly
// rounded value, which the oracle's engine round (orc_cr_sin / cos / tan) computes the same
// way: engine trees are bitwise the oracle's.  x = k pi/2 + r with pi/2 in four parts (the
// first three of 33 bits: k * P_i exact for |k| < 2^20), r in double-double, sin r / cos r by
// Horner over r^2 (Taylor to r^29 / r^28; the eight leading terms in double-double, the tail
// in double), tan = sin / cos in double-double;
// the double-double value (relative error < 2^-100) rounded to double.  The contract is this
// deterministic implementation, shared bit for bit with the oracle and correctly rounded on the
// pinned argument set (tests/test_oracle.py, against libquadmath) -- not a proof of correct
// rounding for every double.  Domain: |x| <= 2^20 (the reduction's k * P_i products are exact
// for |k| < 2^20); beyond it the result is NaN, loudly, instead of a silently inexact value (the
// engine's angles are normalised to [-pi, pi) and its tan arguments are clamped turn rates).
constexpr double kCrMaxArg = 0x1p20;
struct DD {
    double h, l;
};
MPT_HD DD dd_two_sum(double a, double b) {
    const double s = a + b, bb = s - a;
    return DD{s, (a - (s - bb)) + (b - bb)};
}
MPT_HD DD dd_fast(double a, double b) {  // |a| >= |b| (or a == 0)
    const double s = a + b;
    return DD{s, b - (s - a)};
}
MPT_HD DD dd_prod(double a, double b) {
    const double p = a * b;
    return DD{p, fma(a, b, -p)};
}
MPT_HD DD dd_add(DD a, DD b) {
    const DD s = dd_two_sum(a.h, b.h);
    return dd_fast(s.h, s.l + (a.l + b.l));
}
MPT_HD DD dd_mul(DD a, DD b) {
    const DD p = dd_prod(a.h, b.h);
    return dd_fast(p.h, p.l + (a.h * b.l + a.l * b.h));
}
// exact 1/n! split hi + lo: sin r = r sum_n (-1)^n r^2n / (2n+1)!, cos r = sum_n (-1)^n r^2n / (2n)!
#define MPT_CR_SIN_COEFFS                                                                                  \
    {{0x1p+0, 0x0p+0}, {-0x1.5555555555555p-3, -0x1.5555555555555p-57},                                \
     {0x1.1111111111111p-7, 0x1.1111111111111p-63}, {-0x1.a01a01a01a01ap-13, -0x1.a01a01a01a01ap-73},     \
     {0x1.71de3a556c734p-19, -0x1.c154f8ddc6c00p-73}, {-0x1.ae64567f544e4p-26, 0x1.c062e06d1f209p-80},    \
     {0x1.6124613a86d09p-33, 0x1.f28e0cc748ebep-87}, {-0x1.ae7f3e733b81fp-41, -0x1.1d8656b0ee8cbp-97},    \
     {0x1.952c77030ad4ap-49, 0x1.ac981465ddc6cp-103}, {-0x1.2f49b46814157p-57, -0x1.2650f61dbdcb4p-112},  \
     {0x1.71b8ef6dcf572p-66, -0x1.d043ae40c4647p-120}, {-0x1.761b41316381ap-75, 0x1.3423c7d91404fp-130},  \
     {0x1.3f3ccdd165fa9p-84, -0x1.58ddadf344487p-139}, {-0x1.d1ab1c2dccea3p-94, -0x1.054d0c78aea14p-149}, \
     {0x1.259f98b4358adp-103, 0x1.eaf8c39dd9bc5p-157}}
#define MPT_CR_COS_COEFFS                                                                                  \
    {{0x1p+0, 0x0p+0}, {-0x1p-1, 0x0p+0},                                                                \
     {0x1.5555555555555p-5, 0x1.5555555555555p-59}, {-0x1.6c16c16c16c17p-10, 0x1.f49f49f49f49fp-65},      \
     {0x1.a01a01a01a01ap-16, 0x1.a01a01a01a01ap-76}, {-0x1.27e4fb7789f5cp-22, -0x1.cbbc05b4fa99ap-76},    \
     {0x1.1eed8eff8d898p-29, -0x1.2aec959e14c06p-83}, {-0x1.93974a8c07c9dp-37, -0x1.05d6f8a2efd1fp-92},   \
     {0x1.ae7f3e733b81fp-45, 0x1.1d8656b0ee8cbp-101}, {-0x1.6827863b97d97p-53, -0x1.eec01221a8b0bp-107},  \
     {0x1.e542ba4020225p-62, 0x1.ea72b4afe3c2fp-120}, {-0x1.0ce396db7f853p-70, 0x1.aebcdbd20331cp-124},   \
     {0x1.f2cf01972f578p-80, -0x1.9ada5fcc1ab14p-135}, {-0x1.88e85fc6a4e5ap-89, 0x1.71c37ebd16540p-143},  \
     {0x1.0a18a2635085dp-98, 0x1.b9e2e28e1aa54p-153}}

// r = x - k pi/2 (double-double); returns k mod 4
MPT_HD int cr_reduce(double x, DD &r) {
    const double k = rint(x * 0x1.45f306dc9c883p-1);
    const double t = x - k * 0x1.921fb54400000p+0;  // exact for |k| < 2^20
    DD a = dd_two_sum(t, -(k * 0x1.0b4611a600000p-34));
    a = dd_add(a, dd_prod(-k, 0x1.3198a2e000000p-69));
    a = dd_add(a, dd_prod(-k, 0x1.b839a252049c1p-104));
    r = a;
    return (int)((long long)k & 3);
}
// sin r and cos r of a reduced argument
MPT_HD void cr_sincos_r(DD r, DD &s, DD &c) {
    constexpr double cs[15][2] = MPT_CR_SIN_COEFFS;
    constexpr double cc[15][2] = MPT_CR_COS_COEFFS;
    const DD z = dd_mul(r, r);
    // terms 14..8 (at most 2^-53 of the sum for |r| <= pi/4 + 2^-30) in plain double over z.h:
    // their rounding stays below 2^-105 of the result; terms 7..0 in double-double
    double ts = cs[14][0], tc = cc[14][0];
#pragma unroll
    for (int n = 13; n >= 8; --n) {
        ts = ts * z.h + cs[n][0];
        tc = tc * z.h + cc[n][0];
    }
    DD ps{ts, 0.0}, pc{tc, 0.0};
#pragma unroll
    for (int n = 7; n >= 0; --n) {
        ps = dd_add(dd_mul(ps, z), DD{cs[n][0], cs[n][1]});
        pc = dd_add(dd_mul(pc, z), DD{cc[n][0], cc[n][1]});
    }
    s = dd_mul(r, ps);
    c = pc;
}
MPT_HD double cr_sin(double x) {
    if (x == 0.0 || !isfinite(x)) return x == 0.0 ? x : x - x;
    if (fabs(x) > kCrMaxArg) return __builtin_nan("");
    DD r, s, c;
    const int q = cr_reduce(x, r);
    cr_sincos_r(r, s, c);
    const double v = (q & 1) ? c.h : s.h;
    return (q & 2) ? -v : v;
}
MPT_HD double cr_cos(double x) {
    if (!isfinite(x)) return x - x;
    if (fabs(x) > kCrMaxArg) return __builtin_nan("");
    DD r, s, c;
    const int q = cr_reduce(x, r);
    cr_sincos_r(r, s, c);
    const double v = (q & 1) ? s.h : c.h;
    return ((q + 1) & 2) ? -v : v;
}
// both at once (one reduction): the pose rotations need sin and cos of the same angle
MPT_HD void cr_sincos(double x, double &sv, double &cv) {
    if (!isfinite(x) || fabs(x) > kCrMaxArg) {
        sv = cv = isfinite(x) ? __builtin_nan("") : x - x;
        return;
    }
    DD r, s, c;
    const int q = cr_reduce(x, r);
    cr_sincos_r(r, s, c);
    const double vs = (q & 1) ? c.h : s.h, vc = (q & 1) ? s.h : c.h;
    sv = x == 0.0 ? x : ((q & 2) ? -vs : vs);
    cv = ((q + 1) & 2) ? -vc : vc;
}
MPT_HD double cr_tan(double x) {
    if (x == 0.0 || !isfinite(x)) return x == 0.0 ? x : x - x;
    if (fabs(x) > kCrMaxArg) return __builtin_nan("");
    DD r, s, c;
    const int q = cr_reduce(x, r);
    cr_sincos_r(r, s, c);
    DD n = s, d = c;  // tan = sin / cos, or -cos / sin in odd quadrants
    if (q & 1) {
        n = DD{-c.h, -c.l};
        d = s;
    }
    const double q1 = n.h / d.h;
    const DD p = dd_prod(q1, d.h);
    const double rem = (((n.h - p.h) - p.l) + n.l) - q1 * d.l;
    return dd_fast(q1, rem / d.h).h;
}

// FLANN 1.8.4 L2<double>::operator() accumulation order: groups of four
// result += ((d0*d0 + d1*d1) + d2*d2) + d3*d3, then the tail one at a time.
// The first group is stored instead of added to 0.0 (0.0 + t == t bit for bit, t >= 0).
template <int D>
MPT_HD double flann_l2(const double *a, const double *b) {
    double result = 0.0;
    int i = 0;
#pragma unroll
    for (; i + 3 < D; i += 4) {
        const double d0 = a[i] - b[i], d1 = a[i + 1] - b[i + 1];
        const double d2 = a[i + 2] - b[i + 2], d3 = a[i + 3] - b[i + 3];
        const double t = d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3;
        result = (i == 0) ? t : result + t;
    }
#pragma unroll
    for (; i < D; ++i) {
        const double d0 = a[i] - b[i];
        result += d0 * d0;
    }
    return result;
}

// flann_l2's first NG groups of four dims alone, and the sum continued from them:
// flann_l2_rest<D, NG>(a, b, flann_l2_head<NG>(a, b)) == flann_l2<D>(a, b) bit for bit, and the
// head never exceeds the full sum (every later term is non-negative, rounding is monotone)
template <int NG>
MPT_HD double flann_l2_head(const double *a, const double *b) {
    double result = 0.0;
#pragma unroll
    for (int i = 0; i < 4 * NG; i += 4) {
        const double d0 = a[i] - b[i], d1 = a[i + 1] - b[i + 1];
        const double d2 = a[i + 2] - b[i + 2], d3 = a[i + 3] - b[i + 3];
        const double t = d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3;
        result = (i == 0) ? t : result + t;
    }
    return result;
}
template <int D, int NG>
MPT_HD double flann_l2_rest(const double *a, const double *b, double head) {
    static_assert(D >= 4 * NG, "the head is whole groups of four");
    double result = head;
    int i = 4 * NG;
#pragma unroll
    for (; i + 3 < D; i += 4) {
        const double d0 = a[i] - b[i], d1 = a[i + 1] - b[i + 1];
        const double d2 = a[i + 2] - b[i + 2], d3 = a[i + 3] - b[i + 3];
        result = result + (d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3);
    }
#pragma unroll
    for (; i < D; ++i) {
        const double d0 = a[i] - b[i];
        result += d0 * d0;
    }
    return result;
}

MPT_HD double flann_l2_dyn(const double *a, const double *b, int d) {
    double result = 0.0;
    int i = 0;
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

// (d2, id) lexicographic order of all NN results.
MPT_HD bool nn_better(double da, int32_t ia, double db, int32_t ib) {
    return da < db || (da == db && ia < ib);
}

// Counter-based RNG of the batched engine: splitmix64 finaliser of
// seed + golden * (counter + 1); top 53 bits -> [0, 1); (u * (b - a)) + a.
MPT_HD uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
MPT_HD double engine_uniform(uint64_t seed, uint64_t counter, double a, double b) {
    const uint64_t z = mix64(seed + 0x9E3779B97F4A7C15ULL * (counter + 1ULL));
    const double u = (double)(z >> 11) * (1.0 / 9007199254740992.0);
    return u * (b - a) + a;
}

}  // namespace mpt
