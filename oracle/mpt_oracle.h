/*
 * mpt_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C99, gcc, -ffp-contract=off) of the arithmetic that the
 * reference's RRT/PRM inner loop runs through FCL 0.3.2 and FLANN 1.8.4.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library; the product (motionplanningtoolkit_amd/) never links or calls it.
 *
 * Parity status: the reference ships no tests, no golden vectors and cannot be
 * compiled here (FCL/FLANN/Boost/Assimp absent), so this oracle is pinned by
 *   (1) analytic known-answer tests (box/box, triangle/triangle),
 *   (2) scipy.spatial.cKDTree for NN indices on tie-free inputs,
 *   (3) glibc rand() / libstdc++ minstd_rand0 for the RNG restatements.
 * The FCL/FLANN op orders restated here are [upstream] (their sources are not in
 * the container).  See DESIGN.md "Oracle".
 */
#ifndef MPT_ORACLE_H
#define MPT_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------- FCL 0.3.2 math (upstream, restated) ---------------- */
/* Quaternion3f::toRotation, q = {w,x,y,z}; R row-major. */
void orc_quat_to_rot(const double q[4], double R[9]);
/* fcl::relativeTransform: R = R1^T R2, T = R1^T (T2 - T1). */
void orc_relative_transform(const double R1[9], const double T1[3],
                            const double R2[9], const double T2[3],
                            double R[9], double T[3]);
/* Matrix3f * Vec3f + Vec3f, FCL op order. */
void orc_transform_point(const double R[9], const double T[3], const double q[3], double out[3]);
/* Intersect::intersect_Triangle(P1..3, Q1..3): 1 = not separated on all 17 axes. */
int orc_tri_intersect(const double P[9], const double Q[9]);
/* Intersect::intersect_Triangle(P1..3, Q1..3, R, T): Q mapped by R,T first. */
int orc_tri_intersect_RT(const double P[9], const double Q[9], const double R[9], const double T[3]);

/* ---------------- collision (MeshHandler::isInCollision semantics) ---------------- */
/* One (pose, link) unit, all-pairs definition of the FCL verdict.
 * env_tris [Te][9] in env-local frame; env_tf = R1 (9, row-major) + T1 (3);
 * agent_tris [Ta][9] in agent-local frame; pose = R2 (9) + T2 (3). */
int orc_collide_unit(const double *env_tris, int64_t Te, const double env_tf[12],
                     const double *agent_tris, int64_t Ta, const double pose[12]);
/* Batch: link l has agent_tris + link_tri_off[l] .. link_tri_off[l+1] (in triangles).
 * poses [sum P][L][12]; edge_pose_offsets [E+1] (in poses); verdict[e] = 1 if in collision. */
void orc_collide_batch(const double *env_tris, int64_t Te, const double env_tf[12],
                       const double *agent_tris, const int64_t *link_tri_off, int32_t L,
                       const double *poses, const int64_t *edge_pose_offsets, int64_t E,
                       uint8_t *verdict);
/* Same verdicts, AABB-tree broadphase (CPU baseline / speed only).  env_bvh built
 * by orc_bvh_build. */
typedef struct orc_bvh orc_bvh;
orc_bvh *orc_bvh_build(const double *tris, int64_t T);
void orc_bvh_free(orc_bvh *b);
int orc_collide_unit_bvh(const orc_bvh *env, const double env_tf[12],
                         const double *agent_tris, int64_t Ta, const double pose[12],
                         int64_t *n_tri_tests);
void orc_collide_batch_bvh(const orc_bvh *env, const double env_tf[12],
                           const double *agent_tris, const int64_t *link_tri_off, int32_t L,
                           const double *poses, const int64_t *edge_pose_offsets, int64_t E,
                           uint8_t *verdict, int nthreads);

/* ---------------- FLANN 1.8.4 L2<double> (upstream, restated) ---------------- */
double orc_l2(const double *a, const double *b, int32_t d);
/* Exact kNN, ids are 1-based insertion order (FLANN_KDTreeWrapper ids), sorted by
 * (d2, id); removed[i] != 0 skips point i (may be NULL).  Missing slots: id -1, d2 +inf. */
void orc_knn(const double *pts, const uint8_t *removed, int64_t n, int32_t d,
             const double *q, int64_t nq, int32_t k, int32_t *ids, double *d2);
/* Radius search: d2 < r2 (FLANN leaf test `dist < worst_dist`); results per query
 * sorted by (d2, id), truncated to max_nb if max_nb > 0.  offsets [nq+1];
 * returns total count (writes only while <= cap). */
int64_t orc_radius(const double *pts, const uint8_t *removed, int64_t n, int32_t d,
                   const double *q, int64_t nq, double r2, int32_t max_nb,
                   int64_t *offsets, int32_t *ids, double *d2, int64_t cap);
/* kd-tree (CPU baseline): exact 1-NN/kNN with the same contract as orc_knn. */
typedef struct orc_kdtree orc_kdtree;
orc_kdtree *orc_kdtree_build(const double *pts, int64_t n, int32_t d);
void orc_kdtree_free(orc_kdtree *t);
void orc_kdtree_knn(const orc_kdtree *t, const double *q, int64_t nq, int32_t k,
                    int32_t *ids, double *d2, int nthreads);

/* ---------------- RNG restatements ---------------- */
/* glibc random_r TYPE_3 (srand(seed); rand()). */
typedef struct { int32_t r[34]; int32_t f, b; } orc_glibc_rand;
void orc_glibc_srand(orc_glibc_rand *s, uint32_t seed);
int32_t orc_glibc_rand_next(orc_glibc_rand *s);
/* libstdc++ std::default_random_engine == minstd_rand0, default seed 1. */
typedef struct { uint64_t x; } orc_minstd;
void orc_minstd_seed(orc_minstd *g, uint64_t seed);
uint64_t orc_minstd_next(orc_minstd *g);
/* uniform_real_distribution<double>(a,b)(g) via generate_canonical<double,53>. */
double orc_uniform_real(orc_minstd *g, double a, double b);
/* Counter-based generator of the batched device engine (splitmix64 finaliser). */
double orc_engine_uniform(uint64_t seed, uint64_t counter, double a, double b);

/* ---------------- agents ---------------- */
/* Omnidirectional (agents/omnidirectional.hpp). */
double orc_omni_random_steer(orc_glibc_rand *rng, const double start[3], double end[3]);
/* poses_out [maxP][12]; returns P (may exceed maxP: then only maxP written). */
int32_t orc_omni_get_poses(const double start[3], const double end[3], double dt,
                           double *poses_out, int32_t maxP);
/* Blimp (agents/blimp.hpp): prm = {length, vmin, vmax, psimin, psimax, vzmin, vzmax}. */
void orc_blimp_do_step(const double prm[7], const double s[7], double a, double w, double z,
                       double dt, double out[7]);
void orc_blimp_random_steer(const double prm[7], orc_minstd *g, const double start[7],
                            double dt, double end[7], double awz[3]);
/* Build-defined pose sampling (reference stub returns no poses): P = max(1, floor(edge_dt/dt))
 * poses after each doStep of dt; R from theta as Blimp::stateToFCLTransform. */
int32_t orc_blimp_get_poses(const double prm[7], const double start[7], const double awz[3],
                            double edge_dt, double dt, double *poses_out, int32_t maxP);
/* SnakeTrailers (agents/snake_trailers.hpp): prm = {trailerCount, trailerLength, hitchLength,
 * vmin, vmax, psimin, psimax}; state dim 5 + trailerCount. */
void orc_snake_do_step(const double prm[7], const double *s, double a, double w, double dt,
                       double *out);
void orc_snake_random_steer(const double prm[7], orc_minstd *g, const double *start, double dt,
                            double *end, double aw[2]);
/* poses_out [P][L][12], L = trailerCount + 1; returns P. */
int32_t orc_snake_get_poses(const double prm[7], const double *start, const double aw[2],
                            double edge_dt, double dt, double *poses_out, int32_t maxP);

/* The batched engine round's trigonometry: correctly rounded sin / cos / tan (mpt_oracle.c
 * explains why not the host libm), and the blimp / snake steering with it (the plain
 * functions above use the host libm, as the reference's sequential loop). */
double orc_cr_sin(double x);
double orc_cr_cos(double x);
double orc_cr_tan(double x);
void orc_blimp_do_step_cr(const double prm[7], const double s[7], double a, double w, double z,
                          double dt, double out[7]);
int32_t orc_blimp_get_poses_cr(const double prm[7], const double start[7], const double awz[3],
                               double edge_dt, double dt, double *poses_out, int32_t maxP);
void orc_snake_do_step_cr(const double prm[7], const double *s, double a, double w, double dt,
                          double *out);
int32_t orc_snake_get_poses_cr(const double prm[7], const double *start, const double aw[2],
                               double edge_dt, double dt, double *poses_out, int32_t maxP);

/* ---------------- sequential RRT (planners/rrt.hpp, K = 1 replay) ---------------- */
/* agent_kind: 0 omni, 1 blimp, 2 snake.  ranges [d][2] = getStateVarRanges(bounds).
 * iterations_at_a_time: RRT::query's argument (<= 0: run until solved or max_nodes).
 * Outputs: node states [max_nodes][d], parent ids (1-based FLANN ids; root 0).
 * Returns number of nodes; *solved = loop pass at which the goal was hit, -1 if not,
 * -2 if start is already a goal (nothing inserted). */
int64_t orc_rrt_run(int32_t agent_kind, const double *prm, int32_t d, const double *ranges,
                    const double *start, const double *goal, const double *goal_thr,
                    double steer_dt, double cc_dt,
                    const double *env_tris, int64_t Te, const double env_tf[12],
                    const double *agent_tris, int64_t Ta,
                    int64_t iterations_at_a_time, int64_t max_nodes,
                    double *nodes, int32_t *parents, int64_t *solved, int64_t *iters_out);

/* ---------------- batched device-engine step restatement ---------------- */
/* One round of the device RRT engine (motionplanningtoolkit_amd/csrc/rrt_engine.hip):
 * samples from orc_engine_uniform, 1-NN over nodes[0..n), steer, poses, collision,
 * ordered append of the collision-free edges.  Used as the checker and cpu_baseline. */
int64_t orc_engine_step(int32_t agent_kind, const double *prm, int32_t d, const double *ranges,
                        double steer_dt, double cc_dt, uint64_t seed, uint64_t ext_base,
                        int32_t K, const orc_bvh *env, const double env_tf[12],
                        const double *agent_tris, int64_t Ta,
                        double *nodes, int32_t *parents, int64_t n_nodes, int64_t capacity,
                        int32_t *nn_out, uint8_t *verdict_out, int nthreads, int use_kdtree);

/* The reference's sequential loop at a tree size (CPU baseline leg): extensions one at a time
 * on the engine's RNG streams (extension ext_base + i), kd-tree NN, collision, and after every
 * insertion a full kd-tree rebuild, as FLANN 1.8.4's addPoints -> buildIndex
 * (utilities/flannkdtreewrapper.hpp:35).  Stops after max_ext extensions or time_budget
 * seconds; returns the extensions inserted, *ext_done = tried, *seconds = elapsed. */
int64_t orc_rrt_seq_rebuild(int32_t agent_kind, const double *prm, int32_t d, const double *ranges,
                            double steer_dt, double cc_dt, uint64_t seed, uint64_t ext_base, int64_t max_ext,
                            double time_budget, const orc_bvh *env, const double env_tf[12],
                            const double *agent_tris, int64_t Ta, double *nodes, int32_t *parents,
                            int64_t n_nodes, int64_t capacity, int64_t *ext_done, double *seconds);

/* PRM construction (planners/prm/prm.hpp:334-387) for the omnidirectional agent over
 * explicit milestones states[n][3]: edges[E][2] = (target, source), costs[E], comp[n] =
 * smallest milestone of each component.  Returns E, or -1 if E > cap. */
int64_t orc_prm_build(const orc_bvh *env, const double env_tf[12], const double *agent_tris, int64_t Ta,
                      const double *states, int64_t n, int32_t k, int32_t batch, double cc_dt,
                      int32_t *edges, double *costs, int64_t cap, int32_t *comp);

/* Mesh-vs-mesh distance (utilities/fcl_helpers.hpp:67-84 defaultDistanceFunction over the
 * isInCollision object sets, meshhandler.hpp:187-243): FCL 0.3.2 TriangleDistance::triDistance
 * [upstream] with the build's box gate on the overlap answer.  T is already in
 * S's frame.  orc_distance_unit = min over all (env, agent) triangle pairs (exact pruning by
 * box gaps); orc_distance_batch = per edge, min over its poses and links (DBL_MAX if none). */
double orc_tri_distance(const double S[9], const double T[9]);
double orc_distance_unit(const double *env_tris, int64_t Te, const double env_tf[12],
                         const double *agent_tris, int64_t Ta, const double pose[12]);
void orc_distance_batch(const double *env_tris, int64_t Te, const double env_tf[12],
                        const double *agent_tris, const int64_t *link_tri_off, int32_t L,
                        const double *poses, const int64_t *edge_pose_offsets, int64_t E,
                        double *dist, int nthreads);

/* Self-collision (utilities/meshhandler.hpp:205-219, checkSelfCollision): verdict[e] = 1 when
 * two distinct links j < k of one of edge e's poses touch (link j = FCL's o1, all triangle
 * pairs, tri_gate + intersect_Triangle).  poses [sumP][L][12]. */
void orc_self_collide_batch(const double *agent_tris, const int64_t *link_tri_off, int32_t L, const double *poses,
                            const int64_t *edge_pose_offsets, int64_t E, uint8_t *verdict);

/* GridDiscretization (discretizations/workspace/griddiscretization.hpp:9-36): cells over
 * bounds [3][2] (lo, hi) of the given sizes; a cell is free when none of its representative
 * poses collides: n_rot = 1 -> identity (Omnidirectional), 4 -> yaw i*pi/8 (Blimp, Snake head).
 * Centres per getGridCenter as written.  Returns the cell count (free written up to cap). */
int64_t orc_grid_discretization(const orc_bvh *env, const double env_tf[12], const double *agent_tris, int64_t Ta,
                                const double bounds[6], const double sizes[3], int32_t n_rot, uint8_t *free_out,
                                int64_t cap);

/* PRMLite::generateEdges (discretizations/workspace/prmlite.hpp:128-164): collides[e] for all
 * vertex pairs i < j (row-major), verts [V][12] = R | T, poses per PRMLite::interpolate. */
void orc_prmlite_edges(const orc_bvh *env, const double env_tf[12], const double *agent_tris, int64_t Ta,
                       const double *verts, int64_t V, double step, uint8_t *collides, int nthreads);

/* PRM roadmap with radius neighbours (config 4; prm.hpp:334-387 with kNearestWithin):
 * edges (i, j), j < i, squared L2 of the first three state variables < r2, sorted by (i, j);
 * verdict per edge over Omnidirectional::steer(key_i, key_j, 1000) + getPoses(cc_dt) with the
 * blimp yaw of milestone i (dim 7) or identity (dim 3); comp = smallest milestone of each
 * component over the free edges.  Returns E (arrays written up to cap). */
int64_t orc_prm_radius(const orc_bvh *env, const double env_tf[12], const double *agent_tris, int64_t Ta,
                       const double *states, int64_t n, int32_t dim, double r2, double cc_dt,
                       int32_t *edges, uint8_t *verdict, int64_t cap, int32_t *comp, int nthreads);

#ifdef __cplusplus
}
#endif
#endif
