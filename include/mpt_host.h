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
 * starts/ends [n][dim] (written up to cap edges). */
mpt_status mpt_host_rrt_inst(const char *inst_path, int32_t iterations_at_a_time, int64_t cap, double *starts,
                             double *ends, int64_t *n_edges, int32_t *dim, int32_t *solved);

#ifdef __cplusplus
}
#endif
#endif
