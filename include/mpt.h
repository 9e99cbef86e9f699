/*
 * mpt.h -- C ABI of libmpt.so, the MI355X (gfx950) hot path of the RRT/PRM inner loop.
 *
 * Drop-in boundary: the reference composes its planner from header-only templates
 * (main.cpp:38-76) and reaches native code through three seams.  Each entry point
 * below replaces one of them:
 *
 *   collision  MeshHandler::isInCollision            utilities/meshhandler.hpp:187-243
 *              (via Map3D::safeEdge                  workspaces/map3d.hpp:33-37,
 *               fcl_helpers::defaultCollisionFunction utilities/fcl_helpers.hpp:52-65)
 *              StaticEnvironmentMeshHandler ctor     utilities/meshhandler.hpp:18-55
 *              SimpleAgentMeshHandler ctor           utilities/meshhandler.hpp:114-135
 *   NN         FLANN_KDTreeWrapper ctor/insertPoint  utilities/flannkdtreewrapper.hpp:21-40
 *              removePoint                           utilities/flannkdtreewrapper.hpp:42-50
 *              nearest/kNearest                      utilities/flannkdtreewrapper.hpp:57-89
 *              kNearestWithin                        utilities/flannkdtreewrapper.hpp:91-117
 *   RRT loop   RRT::query hot loop                   planners/rrt.hpp:42-94 (batched engine)
 *
 * Conventions
 *   - Plain C types only; `stream` is a hipStream_t passed as void* (NULL = default stream).
 *   - Functions without a `_device` suffix take HOST pointers, copy in/out and return
 *     when the results are in host memory.  `_device` variants take DEVICE pointers and
 *     are asynchronous on `stream` (graph-capturable unless stated otherwise).
 *   - Every function returns mpt_status (0 = OK); the message of the last failure on the
 *     calling thread is mpt_last_error().  Nothing throws or exits across the ABI (the
 *     reference exit()s on bad meshes/keys: meshhandler.hpp:22, instancefilemap.hpp:47).
 *   - Transforms are 12 doubles: R (3x3 row-major, fcl::Matrix3f(i,j) = R[3i+j]) then T.
 *   - Triangle soups are [n][9] doubles (three vertices) in the mesh-local frame.
 *   - NN ids are 1-based in insertion order (FLANN_KDTreeWrapper::currentPointIndex
 *     starts at 1); squared L2 distances in FLANN L2<double> accumulation order.
 *
 * Threading: one handle per host thread; calls on a handle are stream-ordered.
 */
#ifndef MPT_H
#define MPT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int32_t mpt_status;
enum {
    MPT_OK = 0,
    MPT_ERR_INVALID = 1,   /* bad argument / shape */
    MPT_ERR_HIP = 2,       /* HIP runtime error */
    MPT_ERR_NO_DEVICE = 3, /* no gfx950 device / extension not usable */
    MPT_ERR_CAPACITY = 4,  /* capacity exceeded */
    MPT_ERR_INTERNAL = 5
};

typedef struct mpt_env mpt_env;
typedef struct mpt_agent mpt_agent;
typedef struct mpt_nn mpt_nn;
typedef struct mpt_rrt mpt_rrt;

/* ---- runtime ---- */
mpt_status mpt_init(int32_t device);
const char *mpt_last_error(void);
/* ABI version (major*100 + minor). */
int32_t mpt_version(void);
mpt_status mpt_device_synchronize(void);

/* ---- collision: StaticEnvironmentMeshHandler / SimpleAgentMeshHandler / isInCollision ---- */
/* Environment soup (all submeshes concatenated: they share one transform, meshhandler.hpp:27-49).
 * tf12 = parseTransform("x y z qw qx qy qz") as R|T (mpt_transform_from_location). */
mpt_status mpt_env_create(const double *tris, int64_t n_tris, const double tf12[12], mpt_env **out);
mpt_status mpt_env_destroy(mpt_env *env);
/* env statistics: [n_tris, n_bvh_nodes, bvh_depth] */
mpt_status mpt_env_info(const mpt_env *env, int64_t info[3]);
/* Agent link mesh in its local frame (SimpleAgentMeshHandler keeps ONE submesh). */
mpt_status mpt_agent_create(const double *tris, int64_t n_tris, mpt_agent **out);
mpt_status mpt_agent_destroy(mpt_agent *agent);
/* fcl_helpers::parseTransform: loc7 = {x, y, z, qw, qx, qy, qz} -> tf12 (Quaternion3f::toRotation). */
mpt_status mpt_transform_from_location(const double loc7[7], double tf12[12]);

/* Batched Map3D::safeEdge / MeshHandler::isInCollision(env, links, poses):
 *   links[L]            agent mesh of each link (Agent::getMeshes())
 *   poses               [sum_P][L][12]   (Agent::getPoses(edge, dt) for every edge, concatenated)
 *   edge_pose_offsets   [E+1]            poses of edge e are [off[e], off[e+1])
 *   verdict_out         [E]              1 = in collision (safeEdge == false), 0 = safe
 * An edge with no poses is safe (the reference Blimp case, agents/blimp.hpp:219-223). */
mpt_status mpt_collide_batch(const mpt_env *env, const mpt_agent *const *links, int32_t L,
                             const double *poses, const int64_t *edge_pose_offsets, int64_t E,
                             uint8_t *verdict_out, void *stream);
/* MeshHandler::isInCollision(env, agent, poses, checkSelfCollision) (meshhandler.hpp:187-243):
 * as mpt_collide_batch, and with check_self != 0 an edge is also in collision when two
 * distinct links of one of its poses touch (the self-collision branch, :205-219; each link
 * pair (j < k) is tested with link j as FCL's o1). */
mpt_status mpt_collide_batch_ex(const mpt_env *env, const mpt_agent *const *links, int32_t L, const double *poses,
                                const int64_t *edge_pose_offsets, int64_t E, int32_t check_self,
                                uint8_t *verdict_out, void *stream);
/* Device-pointer variant: poses, edge_pose_offsets, verdict_out in device memory;
 * total_poses = edge_pose_offsets[E] (passed so no device->host read is needed). */
mpt_status mpt_collide_batch_device(const mpt_env *env, const mpt_agent *const *links, int32_t L,
                                    const double *d_poses, const int64_t *d_edge_pose_offsets, int64_t E,
                                    int64_t total_poses, uint8_t *d_verdict_out, void *stream);
/* Collision statistics of the last collide call on this thread (synchronises):
 * [units, clusters, bvh node visits, triangle-pair tests]; enabled by mpt_set_stats(1). */
mpt_status mpt_set_stats(int32_t enable);
mpt_status mpt_last_collide_stats(uint64_t stats[4]);
/* Collision kernel structure (process-wide, both for mpt_collide_batch* and the RRT
 * engine): MPT_COLLIDE_SPLIT (default) = broad-phase box traversal writing candidate
 * triangle pairs, then one exact triangle test per candidate; MPT_COLLIDE_FUSED = one
 * kernel walking the BVH and testing at the leaves with per-edge early exit.
 * Verdicts are identical; the choice only changes speed. */
enum { MPT_COLLIDE_SPLIT = 0, MPT_COLLIDE_FUSED = 1 };
mpt_status mpt_set_collide_mode(int32_t mode);

/* ---- distance: fcl::distance through fcl_helpers::defaultDistanceFunction ----
 * (utilities/fcl_helpers.hpp:67-84, DistanceData :35-42; no caller in the reference) over
 * the same object sets as mpt_collide_batch: dist_out[e] = minimum over the edge's poses,
 * links and (env, agent) triangle pairs of FCL's TriangleDistance::triDistance; 0 = in
 * contact (the callback's dist <= 0 stop); DBL_MAX (the initial DistanceResult) for an edge
 * without poses.  Same arguments as mpt_collide_batch[_device].  mpt_last_collide_stats
 * then reports [agent clusters walked, env box tests, triangle-distance calls, pair box tests]. */
mpt_status mpt_distance_batch(const mpt_env *env, const mpt_agent *const *links, int32_t L, const double *poses,
                              const int64_t *edge_pose_offsets, int64_t E, double *dist_out, void *stream);
mpt_status mpt_distance_batch_device(const mpt_env *env, const mpt_agent *const *links, int32_t L,
                                     const double *d_poses, const int64_t *d_edge_pose_offsets, int64_t E,
                                     int64_t total_poses, double *d_dist_out, void *stream);

/* ---- PRM roadmap edges (BASELINE config 4): PRM::addMilestone, planners/prm/prm.hpp:334-387,
 * with radius neighbours (FLANN_KDTreeWrapper::kNearestWithin, flannkdtreewrapper.hpp:91-117)
 * in place of the approximate kNN(10).  Milestone i connects to every earlier milestone j < i
 * whose first three state variables (prm.hpp:155, the NN key) lie at squared L2 < radius2;
 * the edge is Omnidirectional::steer(key_i, key_j, 1000) checked at getPoses(edge, cc_dt)
 * poses (translation along the key segment; a blimp mesh keeps milestone i's yaw, R of
 * Blimp::stateToFCLTransform).  agent_kind / dim: MPT_AGENT_OMNI / 3 or MPT_AGENT_BLIMP / 7.
 * Out: edges[E][2] = (i, j) sorted by i then j, verdict[E] (1 = in collision), both written
 * up to cap; *n_edges = E; comp[n] = smallest milestone of each component over the free
 * edges (may be NULL); ms[4] (may be NULL) = device ms of [neighbours, poses, collision, all].
 * Synchronous. */
mpt_status mpt_prm_connect(const mpt_env *env, const mpt_agent *agent, int32_t agent_kind, const double *states,
                           int64_t n, int32_t dim, double radius2, double cc_dt, int64_t cap, int32_t *edges,
                           uint8_t *verdict, int64_t *n_edges, int32_t *comp, float ms[4]);
/* Diagnostics: out (may be NULL) = the edge sweep's work counters of the calling thread's last
 * mpt_prm_connect made with counters on: waves, env item box tests, (pair, pose) gate tests,
 * exact triangle tests, edges, poses, (edge, triangle, triangle, pose range) candidates emitted,
 * edges the candidate pass capped (decided by k_sweep_prm); the first min(count, 8) of them are
 * written (count: out's length; 8 since round 5, 6 before); enable switches the counters on for
 * its later calls (one same-address atomic per wave: not for timed calls). */
mpt_status mpt_prm_stats(int32_t enable, uint64_t *out, int32_t count);
/* Diagnostics: the edges (indices into that call's edge list) the sweep of the calling thread's
 * last mpt_prm_connect made with counters on sent to its per-edge pass (k_sweep_prm): first those
 * its candidate pass capped, then those a full candidate queue deferred.  *n = their number, the
 * first min(*n, cap) written to out (may be NULL). */
mpt_status mpt_prm_deferred_edges(int32_t *out, int64_t cap, int64_t *n);
/* Test hook: caps the PRM sweep's candidate queue at max_candidates (0 restores the sized
 * queue, at least 4 M entries) so that a small roadmap drives the full-queue path (edges
 * deferred to the per-edge sweep).  Process-wide; verdicts are unchanged by it. */
mpt_status mpt_set_sweep_queue_cap(int64_t max_candidates);

/* ---- workspace discretisation: PRMLite::generateEdges (discretizations/workspace/prmlite.hpp:128-164)
 * All vertex pairs i < j, pair index e = row-major over i < j (E = V(V-1)/2).  vertices [V][12] =
 * R | T with R = Quaternion3f::toRotation of the vertex's quaternion.  The edge's poses are
 * PRMLite::interpolate (:181-203): steps = (unsigned)(|t_i - t_j| / step), each pose
 * (t_j - t_i) / steps further than the previous one (accumulated), rotation of vertex i; an
 * edge without poses is safe.  collides[e] = 1 when a pose is in collision (edge dropped). */
mpt_status mpt_prmlite_edges(const mpt_env *env, const mpt_agent *agent, const double *vertices, int64_t V,
                             double step, uint8_t *collides, void *stream);

/* ---- NN: FLANN_KDTreeWrapper ---- */
mpt_status mpt_nn_create(int32_t dim, int64_t capacity, mpt_nn **out);
mpt_status mpt_nn_destroy(mpt_nn *nn);
/* insertPoint for n points [n][dim]; ids_out[i] = assigned 1-based id (may be NULL). */
mpt_status mpt_nn_append(mpt_nn *nn, const double *pts, int64_t n, int32_t *ids_out);
mpt_status mpt_nn_append_device(mpt_nn *nn, const double *d_pts, int64_t n, void *stream);
/* flann::Index::removePoint(id - 1) for a 1-based id: the point is skipped by queries. */
mpt_status mpt_nn_remove(mpt_nn *nn, int32_t id);
mpt_status mpt_nn_size(const mpt_nn *nn, int64_t *n_out);
/* Device pointer of the [capacity][dim] point array (for zero-copy engines / tests). */
mpt_status mpt_nn_points_device(const mpt_nn *nn, const double **d_pts);
/* Search structure: AUTO (grid when n >= 4096 and nq >= 32), BRUTE (tiled scan), GRID
 * (device-built uniform grid over the widest <= 3 dims, rebuilt after appends).  All modes
 * are exact and return identical results; GRID/AUTO rebuilds synchronise once. */
enum { MPT_NN_AUTO = 0, MPT_NN_BRUTE = 1, MPT_NN_GRID = 2, MPT_NN_TREE = 3 };
mpt_status mpt_nn_set_index(mpt_nn *nn, int32_t mode);
/* kNearest / nearest (k = 1): ids [nq][k] (-1 when fewer than k points), d2 [nq][k] (+inf). */
mpt_status mpt_nn_knn(mpt_nn *nn, const double *q, int64_t nq, int32_t k, int32_t *ids, double *d2,
                      void *stream);
mpt_status mpt_nn_knn_device(mpt_nn *nn, const double *d_q, int64_t nq, int32_t k, int32_t *d_ids,
                             double *d_d2, void *stream);
/* kNearestWithin: points with d2 < r2 (note: the reference passes `radius` straight to a
 * squared-distance index, so its argument IS r2), at most max_nb (> 0) nearest per query,
 * each list sorted by (d2, id).  offsets [nq+1]; ids/d2 written up to cap entries; the
 * total is offsets[nq].  Synchronises (list sizes are data dependent). */
mpt_status mpt_nn_radius(mpt_nn *nn, const double *q, int64_t nq, double r2, int32_t max_nb,
                         int64_t *offsets, int32_t *ids, double *d2, int64_t cap, void *stream);

/* ---- batched RRT engine (planners/rrt.hpp:42-94, K extensions per round) ---- */
enum { MPT_AGENT_OMNI = 0, MPT_AGENT_BLIMP = 1, MPT_AGENT_SNAKE = 2 };
/* prm (7 doubles): blimp {length, vmin, vmax, psimin, psimax, vzmin, vzmax};
 *                  snake {trailerCount, trailerLength, hitchLength, vmin, vmax, psimin, psimax};
 *                  omni  ignored.
 * ranges [dim][2] = Agent::getStateVarRanges(Map3D::getBounds()).
 * The engine holds one tree of up to `capacity` nodes on the device. */
mpt_status mpt_rrt_create(const mpt_env *env, const mpt_agent *agent, int32_t agent_kind, const double prm[7],
                          const double *ranges, int32_t dim, double steer_dt, double cc_dt, int64_t capacity,
                          uint64_t seed, mpt_rrt **out);
mpt_status mpt_rrt_destroy(mpt_rrt *rrt);
/* Append n tree nodes [n][dim] with parent ids (NULL = 0). */
mpt_status mpt_rrt_add_nodes(mpt_rrt *rrt, const double *states, const int32_t *parents, int64_t n);
/* Set the node count (truncate) without a host sync: applied by the next round on its own
 * stream (`stream` is unused) or before mpt_rrt_counters / mpt_rrt_add_nodes read the count. */
mpt_status mpt_rrt_set_size(mpt_rrt *rrt, int64_t n, void *stream);
/* One batched round: K uniform samples -> exact 1-NN -> randomSteer -> getPoses ->
 * collision -> ordered append of the collision-free edges.  Asynchronous. */
mpt_status mpt_rrt_step(mpt_rrt *rrt, int32_t K, void *stream);
/* One round of n independent engines (BASELINE config 5: one engine per seed), engine i on
 * streams[i].  Identical results to mpt_rrt_step per engine.  When every engine's round uses
 * the Morton-tree NN and the engines share the env, the agent and every parameter but the
 * seed (and K is a multiple of 16), the whole round is a joint round on joint_stream: one
 * launch per stage (sample, incremental index build, NN, steer, collide, append) for all
 * engines, after the engines' streams and before their next work (a joint round indexes trees
 * of any size, so engines grown from their start states are joint from their first round); an engine's last-round
 * buffers (mpt_rrt_last_round / _last_poses) are then the joint state's, valid until the next
 * call on that joint stream (those two calls fail with MPT_ERR_INVALID once mpt_rrt_joint_release
 * or a larger joint round has freed the buffers; stage times of a joint round come from
 * mpt_rrt_joint_stage_times, and mpt_rrt_kernel_times fails after one).  Otherwise the engines whose round uses the Morton tree share
 * one index build and one query launch on joint_stream, and the rest of each round runs on
 * the engine's own stream.  The job tables and buffers of the joint launches belong to
 * joint_stream: calls with different joint streams (from one or several host threads) may
 * overlap; calls on one joint stream are serialised.  Asynchronous. */
mpt_status mpt_rrt_step_many(mpt_rrt *const *rrts, int32_t n, int32_t K, void *const *streams, void *joint_stream);
/* Duration (ms, hipEvents) of the most recent timed joint NN launch on the joint stream of the
 * calling thread's last timed mpt_rrt_step_many (joint state is per joint stream: if other
 * threads share that stream, their later launch is the one reported; mpt_rrt_joint_times
 * names the stream explicitly).  Synchronises on it. */
mpt_status mpt_rrt_joint_nn_ms(float *ms);
/* Release the joint state of joint_stream (job-table staging ring, events, shared sort
 * buffers), after synchronising on it.  Call before destroying or recycling a stream handle
 * that mpt_rrt_step_many used as its joint stream: a recycled handle would otherwise inherit
 * the old state.  No-op for a stream that holds none.  Must not run at the same time as an
 * mpt_rrt_step_many on the same joint stream (another host thread's mpt_rrt_last_round /
 * _last_poses hold the state's lock through their copies and are safe). */
mpt_status mpt_rrt_joint_release(void *joint_stream);
/* Diagnostics: launch joint_stream's last joint NN launch again on that stream (same job table,
 * queries and index; its outputs are rewritten with the same values), e.g. alone after an L2
 * flush under rocprofv3 counters.  parts: how the launch maps trees to the 8 XCDs -- 0 = each
 * tree's workgroups dealt over all eight; P > 0 = each tree cut into P contiguous runs of its
 * queries, each run on one XCD (trees * P a multiple of 8; P = 1: whole trees per XCD).
 * Asynchronous. */
mpt_status mpt_rrt_joint_replay_nn(void *joint_stream, int32_t parts);
/* The last timed mpt_rrt_step_many on joint_stream: ms[0] = the joint tree build, ms[1] = the
 * joint NN launch (hipEvents on joint_stream).  Synchronises on it. */
mpt_status mpt_rrt_joint_times(void *joint_stream, float ms[2]);
/* The last mpt_rrt_step_many on joint_stream if it was a timed joint round (an engine with
 * timing on): ms = sample, index build, NN, steer, collide, append (hipEvents on
 * joint_stream).  Synchronises on it. */
mpt_status mpt_rrt_joint_stage_times(void *joint_stream, float ms[6]);
/* counters [8]: rounds, extensions checked, extensions valid, nodes, capacity drops,
 * pose overflow, index errors (an incremental tree build handed more new points than it
 * merges: an internal bound broken; mpt_rrt_counters then fails with MPT_ERR_INTERNAL), reserved.
 * Synchronises. */
mpt_status mpt_rrt_counters(mpt_rrt *rrt, uint64_t counters[8]);
/* Copy out the first n nodes and parents (1-based parent ids, 0 for roots). Synchronises. */
mpt_status mpt_rrt_read_tree(mpt_rrt *rrt, double *states, int32_t *parents, int64_t n);
/* Intermediates of the last round for verification (host copies, synchronises):
 * samples [K][dim], nn ids [K], ends [K][dim], verdicts [K]; any pointer may be NULL. */
mpt_status mpt_rrt_last_round(mpt_rrt *rrt, double *samples, int32_t *nn_ids, double *ends, uint8_t *verdicts);
/* Pose slots of the last round: poses [K][pmax][L][12], pose counts [K]; pmax/L via info. */
mpt_status mpt_rrt_last_poses(mpt_rrt *rrt, double *poses, int32_t *pose_counts);
/* [dim, links L, pose slots per edge pmax, capacity] */
mpt_status mpt_rrt_info(const mpt_rrt *rrt, int64_t info[4]);
/* Per-kernel device times (ms) of the last round, recorded with hipEvents on the launch
 * stream when timing is enabled: [sample, nn_build, nn_query, steer, collide, append]
 * (nn_build = grid index build, 0 in brute-force mode; nn_query includes the merge). */
mpt_status mpt_rrt_enable_timing(mpt_rrt *rrt, int32_t enable);
/* NN structure of the rounds: MPT_NN_AUTO / _BRUTE / _GRID / _TREE (the incremental cell
 * tree, for trees that do not fill the sampling box), grid occupancy target (points per cell,
 * <= 0: the default, 2 points per cell with the cell side floored at 0.3x the expected NN
 * distance over all state dims; for 15-dim states 3 points per cell, no floor).  Results are
 * identical.  When the engine's rounds will use
 * the tree (MPT_NN_TREE, or MPT_NN_AUTO after mpt_rrt_add_nodes' first nodes chose it), the
 * tree's memory for the engine's capacity is reserved here (allocates, synchronises). */
mpt_status mpt_rrt_set_nn(mpt_rrt *rrt, int32_t mode, double points_per_cell);
/* NN structure the last round used (MPT_NN_BRUTE / _GRID / _TREE; what MPT_NN_AUTO chose),
 * -1 before the first round. */
mpt_status mpt_rrt_last_nn(const mpt_rrt *rrt, int32_t *mode);
/* Collision work counters accumulated since the previous call (synchronises), then reset;
 * enable = 1 keeps counting in later rounds (atomics: off for timed runs).
 * out [16] (may be NULL): [0] (pose, link) units, [1] agent clusters past the root cull,
 * [2] env tree node tests, [3] exact triangle tests, [4] (cluster, env triangle) pair tests,
 * [5] units re-run by the fused kernel, [6] agent cluster transforms, [7] broad-phase
 * candidates, [8] NN points examined, [9] NN cells visited (grid) / boxes tested (tree), [10]
 * (unit, cluster) broad-phase threads, [11] tree NN walk steps (all queries), [12..15] reserved. */
mpt_status mpt_rrt_collide_stats(mpt_rrt *rrt, int32_t enable, uint64_t out[16]);
/* hipEvent times (ms) of the last round's stages, after mpt_rrt_enable_timing(1):
 * [sample, nn_build, nn_query, steer, collide_pairs, collide_cands, collide_narrow,
 *  collide_rest (memsets, fused re-run; the whole collide stage in fused mode), append]. */
mpt_status mpt_rrt_kernel_times(mpt_rrt *rrt, float ms[9]);
/* The same stages summed over every round recorded since the previous call, and the number
 * of rounds (then reset).  Rounds record into a ring of 64 event sets, so timing a sequence
 * of rounds needs no host synchronisation between them. */
mpt_status mpt_rrt_kernel_times_sum(mpt_rrt *rrt, double ms[9], int64_t *rounds);

#ifdef __cplusplus
}
#endif
#endif /* MPT_H */
