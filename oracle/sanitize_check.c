/*
 * sanitize_check.c -- TEST INFRASTRUCTURE ONLY: drives every oracle entry point on small
 * inputs under AddressSanitizer + UndefinedBehaviorSanitizer (oracle/Makefile `sanitize`,
 * run by tests/test_sanitize_cpu.py).  Exits non-zero on a sanitizer report (the build uses
 * -fno-sanitize-recover) or when two restatements that must agree disagree (kd-tree vs
 * brute-force kNN, AABB-tree vs all-pairs collision).
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mpt_oracle.h"

static uint64_t g_rng = 88172645463325252ull;
static double urand(double a, double b) {
    g_rng ^= g_rng << 13;
    g_rng ^= g_rng >> 7;
    g_rng ^= g_rng << 17;
    return a + (b - a) * (double)(g_rng >> 11) * (1.0 / 9007199254740992.0);
}

/* 12 triangles of the box centre c, half-extent h */
static void box_tris(const double c[3], double h, double *out) {
    static const int F[12][3] = {{0, 1, 3}, {0, 3, 2}, {4, 6, 7}, {4, 7, 5}, {0, 4, 5}, {0, 5, 1},
                                 {2, 3, 7}, {2, 7, 6}, {0, 2, 6}, {0, 6, 4}, {1, 5, 7}, {1, 7, 3}};
    double v[8][3];
    for (int i = 0; i < 8; ++i) {
        v[i][0] = c[0] + ((i >> 2) & 1 ? h : -h);
        v[i][1] = c[1] + ((i >> 1) & 1 ? h : -h);
        v[i][2] = c[2] + (i & 1 ? h : -h);
    }
    for (int f = 0; f < 12; ++f)
        for (int k = 0; k < 3; ++k) memcpy(out + 9 * f + 3 * k, v[F[f][k]], sizeof(double) * 3);
}

#define CHECK(c, msg)                              \
    do {                                           \
        if (!(c)) {                                \
            fprintf(stderr, "FAILED: %s\n", msg);  \
            return 1;                              \
        }                                          \
    } while (0)

int main(void) {
    const double I12[12] = {1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0};
    /* env: 20 boxes (240 triangles); agent: one unit box */
    enum { NB = 20, TE = NB * 12, TA = 12 };
    double *env = malloc(sizeof(double) * 9 * TE), agent[9 * TA];
    for (int b = 0; b < NB; ++b) {
        const double c[3] = {urand(-8, 8), urand(-8, 8), urand(-2, 2)};
        box_tris(c, urand(0.3, 1.5), env + 9 * 12 * b);
    }
    const double c0[3] = {0, 0, 0};
    box_tris(c0, 0.5, agent);
    orc_bvh *bvh = orc_bvh_build(env, TE);

    /* collision: all-pairs vs AABB tree, random poses */
    enum { P = 400 };
    double *poses = malloc(sizeof(double) * 12 * P);
    int64_t off[P + 1];
    for (int p = 0; p < P; ++p) {
        double q[4] = {urand(-1, 1), urand(-1, 1), urand(-1, 1), urand(-1, 1)};
        const double nq = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
        for (int k = 0; k < 4; ++k) q[k] /= nq;
        orc_quat_to_rot(q, poses + 12 * p);
        for (int k = 0; k < 3; ++k) poses[12 * p + 9 + k] = urand(-9, 9);
        off[p] = p;
    }
    off[P] = P;
    const int64_t link_off[2] = {0, TA};
    uint8_t v1[P], v2[P];
    orc_collide_batch(env, TE, I12, agent, link_off, 1, poses, off, P, v1);
    orc_collide_batch_bvh(bvh, I12, agent, link_off, 1, poses, off, P, v2, 1);
    int hits = 0;
    for (int p = 0; p < P; ++p) {
        CHECK(v1[p] == v2[p], "AABB-tree collision differs from all-pairs");
        hits += v1[p];
    }
    CHECK(hits > 0 && hits < P, "degenerate collision sample");

    /* distance and self-collision */
    double dist[8];
    orc_distance_batch(env, TE, I12, agent, link_off, 1, poses, off, 8, dist, 1);
    for (int e = 0; e < 8; ++e) CHECK(dist[e] >= 0 && (dist[e] == 0) == (v1[e] != 0), "distance / verdict mismatch");
    const int64_t two_links[3] = {0, TA, 2 * TA};
    double agent2[2 * 9 * TA];
    memcpy(agent2, agent, sizeof agent);
    memcpy(agent2 + 9 * TA, agent, sizeof agent);
    uint8_t sv[4];
    orc_self_collide_batch(agent2, two_links, 2, poses, off, 4, sv);

    /* NN: brute force vs kd-tree, d = 7, with exact ties */
    enum { N = 3000, Q = 300, D = 7, K = 5 };
    double *pts = malloc(sizeof(double) * N * D), *qs = malloc(sizeof(double) * Q * D);
    for (int i = 0; i < N * D; ++i) pts[i] = floor(urand(0, 20));  /* integer grid: many ties */
    for (int i = 0; i < Q * D; ++i) qs[i] = floor(urand(0, 20));
    int32_t id1[Q * K], id2[Q * K];
    double d1[Q * K], d2[Q * K];
    orc_knn(pts, NULL, N, D, qs, Q, K, id1, d1);
    orc_kdtree *kd = orc_kdtree_build(pts, N, D);
    orc_kdtree_knn(kd, qs, Q, K, id2, d2, 1);
    orc_kdtree_free(kd);
    for (int i = 0; i < Q * K; ++i) CHECK(id1[i] == id2[i] && d1[i] == d2[i], "kd-tree kNN differs from brute force");
    int64_t roff[Q + 1];
    const int64_t total = orc_radius(pts, NULL, N, D, qs, Q, 30.0, -1, roff, NULL, NULL, 0);
    int32_t *rid = malloc(sizeof(int32_t) * (size_t)(total + 1));
    double *rd = malloc(sizeof(double) * (size_t)(total + 1));
    CHECK(orc_radius(pts, NULL, N, D, qs, Q, 30.0, -1, roff, rid, rd, total) == total, "radius total");
    for (int64_t i = 0; i < total; ++i) CHECK(rd[i] < 30.0, "radius bound");

    /* RNG restatements, agents, sequential RRT, engine round, rebuild loop */
    orc_glibc_rand gr;
    orc_glibc_srand(&gr, 1);
    CHECK(orc_glibc_rand_next(&gr) == 1804289383, "glibc rand() first value");
    orc_minstd ms;
    orc_minstd_seed(&ms, 1);
    CHECK(orc_minstd_next(&ms) == 16807, "minstd_rand0 first value");
    const double ranges3[6] = {-10, 10, -10, 10, -10, 10};
    const double start[3] = {-9, -9, 0}, goal[3] = {9, 9, 0}, thr[3] = {1, 1, 1};
    double *nodes = malloc(sizeof(double) * 3 * 4000);
    int32_t *par = malloc(sizeof(int32_t) * 4000);
    int64_t solved = 0, iters = 0;
    const double prm0[7] = {0};
    const int64_t n = orc_rrt_run(0, prm0, 3, ranges3, start, goal, thr, 0.1, 0.1, env, TE, I12, agent, TA, 300, 4000,
                                  nodes, par, &solved, &iters);
    CHECK(n > 1, "sequential RRT grew nothing");
    int32_t nn[256];
    uint8_t vd[256];
    const int64_t n2 = orc_engine_step(0, prm0, 3, ranges3, 0.1, 0.1, 7, 0, 256, bvh, I12, agent, TA, nodes, par, n,
                                       4000, nn, vd, 1, 1);
    CHECK(n2 >= n && n2 <= n + 256, "engine round");
    int64_t done = 0;
    double secs = 0;
    const int64_t ok = orc_rrt_seq_rebuild(0, prm0, 3, ranges3, 0.1, 0.1, 7, 256, 200, 5.0, bvh, I12, agent, TA, nodes,
                                           par, n2, 4000, &done, &secs);
    CHECK(ok >= 0 && ok <= done && done <= 200, "rebuild loop");
    const double bprm[7] = {10.0, -1.0, 5.0, -0.785398, 0.785398, -5.0, 5.0};
    const double s7[7] = {0, 0, 0, 0.3, 1.0, 0.1, 0.2};
    double e7[7], awz[3] = {0.5, 0.1, -0.2}, bp[12 * 4];
    orc_blimp_do_step(bprm, s7, awz[0], awz[1], awz[2], 0.1, e7);
    CHECK(orc_blimp_get_poses(bprm, s7, awz, 0.4, 0.1, bp, 4) == 4, "blimp poses");
    const double sprm[7] = {3, 1.0, 0.25, -1.0, 5.0, -0.785398, 0.785398};
    double s8[8] = {0, 0, 1, 0.1, 0.2, 0.3, 0.4, 0.5}, e8[8], aw[2] = {0.5, 0.05}, sp[12 * 4 * 2];
    orc_snake_do_step(sprm, s8, aw[0], aw[1], 0.25, e8);
    CHECK(orc_snake_get_poses(sprm, s8, aw, 0.25, 1.0, sp, 2) == 1, "snake poses");

    /* PRM (kNN and radius), PRMLite, grid discretisation */
    enum { M = 150 };
    double ms3[M * 3];
    for (int i = 0; i < M * 3; ++i) ms3[i] = urand(-9, 9);
    int32_t edges[M * 10 * 2], comp[M];
    double costs[M * 10];
    CHECK(orc_prm_build(bvh, I12, agent, TA, ms3, M, 10, 7, 0.1, edges, costs, M * 10, comp) >= 0, "prm build");
    int32_t redges[M * M];
    uint8_t rv[M * M / 2];
    CHECK(orc_prm_radius(bvh, I12, agent, TA, ms3, M, 3, 9.0, 0.1, redges, rv, M * M / 2, comp, 1) >= 0, "prm radius");
    double verts[12 * 20];
    for (int i = 0; i < 20; ++i) {
        memcpy(verts + 12 * i, I12, sizeof(double) * 9);
        for (int k = 0; k < 3; ++k) verts[12 * i + 9 + k] = urand(-9, 9);
    }
    uint8_t lite[20 * 19 / 2];
    orc_prmlite_edges(bvh, I12, agent, TA, verts, 20, 0.1, lite, 1);
    const double bounds[6] = {-10, 10, -10, 10, -3, 3}, sizes[3] = {1.0, 1.0, 1.0};
    uint8_t freec[20 * 20 * 6];
    CHECK(orc_grid_discretization(bvh, I12, agent, TA, bounds, sizes, 4, freec, 20 * 20 * 6) == 20 * 20 * 6,
          "grid cells");

    orc_bvh_free(bvh);
    free(env); free(poses); free(pts); free(qs); free(rid); free(rd); free(nodes); free(par);
    printf("sanitize_check ok: %d/%d poses in collision, %lld radius hits, RRT %lld nodes\n", hits, P,
           (long long)total, (long long)n);
    return 0;
}
