/*
 * mpt_host.h -- C entry points into the C++ host planner of libmpt.so (the reference's
 * Agent / Sampler / TreeInterface / RRT composition driven by a `.inst` file, main.cpp:192-212).
 * The compute path underneath is include/mpt.h.
 */
#ifndef MPT_HOST_H
#define MPT_HOST_H
#include <stdint.h>

#include "mpt.h"

#ifdef __cplusplus
extern "C" {
#endif

const char *mpt_host_last_error(void);

/* AssimpMeshLoader replacement (utilities/assimp_mesh_loader.hpp): which = 0 all submeshes
 * concatenated (environment), 1 = last non-empty submesh (SimpleAgentMeshHandler).
 * Writes min(cap, n) triangles [n][9]. */
mpt_status mpt_host_load_mesh(const char *path, int32_t which, double *tris, int64_t cap, int64_t *n_tris,
                              int32_t *n_submeshes);

/* Planner <file.inst> (main.cpp) with RRT::query(start, goal, iterations_at_a_time) on the GPU
 * collision + NN path.  Outputs the tree edges in insertion order (root first):
 * starts/ends [n][dim], each a buffer of state_cap doubles, written up to min(cap, state_cap / dim)
 * edges (dim is an output: size the buffers for the largest agent, 16 doubles a state). */
mpt_status mpt_host_rrt_inst(const char *inst_path, int32_t iterations_at_a_time, int64_t cap, int64_t state_cap,
                             double *starts, double *ends, int64_t *n_edges, int32_t *dim, int32_t *solved);

/* Batched throughput mode of Planner <file.inst>: the file sets `Batch Size ? K` (and optionally
 * `Seed`, `Seed Count`, `Rounds`, `Max Tree Size`, `NN Index`; motionplanningtoolkit_amd/csrc/host/
 * compose.hpp run_batched); Seed Count trees grow from `Agent Start Location` on the device engine
 * (mpt_rrt_step / mpt_rrt_step_many).  out[4] = {rounds, extensions checked, extensions valid,
 * trees with a goal node}; *seconds = device wall time of the rounds; tree 0's parents [n] are
 * written up to cap nodes and its states [n][dim] up to the min(cap, state_cap / dim) rows a
 * buffer of state_cap doubles holds (either may be NULL), *tree0_nodes = n. */
mpt_status mpt_host_rrt_batched(const char *inst_path, int64_t out[4], double *seconds, int64_t cap, int64_t state_cap,
                                double *tree0_states, int32_t *tree0_parents, int64_t *tree0_nodes, int32_t *dim);

/* PRM (planners/prm/prm.hpp) with the .inst's agent and workspace.
 * states != NULL: addMilestone for states[n][dim] in order, `batch` at a time (1 = the
 *   reference's sequence), and nothing else.
 * states == NULL: PRM::query(start, goal) repeated (100 sampled milestones per call,
 *   prm.hpp:207-213) until solved or max_queries calls; then *solved / *cost are set.
 * Roadmap out: edges[E][2] = (target, source) vertex ids (milestones 0-based in insertion
 * order), costs[E], comp[n_milestones] = smallest milestone of each component; arrays are
 * written up to cap edges / comp_cap milestones. */
mpt_status mpt_host_prm(const char *inst_path, const double *states, int64_t n, int32_t batch, int32_t max_queries,
                        int64_t cap, int32_t *edges, double *costs, int64_t *n_edges, int64_t comp_cap,
                        int32_t *comp, int64_t *n_milestones, int32_t *solved, double *cost);

/* GridDiscretization (discretizations/workspace/griddiscretization.hpp:6-189) over the .inst's
 * workspace and agent: a cell is free when none of getRepresentivePosesForLocation(centre)
 * collides.  free_out[cells], centers[cells][3] written up to cap. */
mpt_status mpt_host_grid_discretization(const char *inst_path, const double sizes[3], int64_t cap, uint8_t *free_out,
                                        double *centers, int64_t *n_cells);

/* PRMLite (discretizations/workspace/prmlite.hpp:8-263): n_vertices collision-free random
 * vertices (the reference's RNG stream), then every pair connected unless an interpolated pose
 * collides (mpt_prmlite_edges).  verts[n_vertices][12] = R | T; edges[E][2] = (i, j), i < j,
 * sorted; written up to cap. */
mpt_status mpt_host_prmlite(const char *inst_path, int32_t n_vertices, double step, double *verts, int64_t cap,
                            int32_t *edges, int64_t *n_edges);

#ifdef __cplusplus
}
#endif
#endif
