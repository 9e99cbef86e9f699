// host_capi.cpp -- C entry points into the C++ host planner (for ctypes tests, the
// Python package and other FFI callers).  Declared in include/mpt_host.h.
#include <cstring>
#include <stdexcept>
#include <string>

#include "../../../include/mpt_host.h"
#include "compose.hpp"

namespace {
thread_local std::string g_host_err;

template <class F>
mpt_status hguard(F &&f) {
    try {
        f();
        return MPT_OK;
    } catch (const std::exception &e) {
        g_host_err = e.what();
        return MPT_ERR_INVALID;
    } catch (...) {
        g_host_err = "unknown error";
        return MPT_ERR_INTERNAL;
    }
}
}  // namespace

extern "C" const char *mpt_host_last_error(void) { return g_host_err.c_str(); }

extern "C" mpt_status mpt_host_load_mesh(const char *path, int32_t which, double *tris, int64_t cap,
                                         int64_t *n_tris, int32_t *n_submeshes) {
    return hguard([&] {
        if (!path || !n_tris) throw std::invalid_argument("null pointer");
        const auto m = mpt_host::load_mesh(path);
        if (m.error) throw std::runtime_error(m.message);
        const std::vector<double> t = which == 1 ? m.last_nonempty() : m.soup();
        *n_tris = (int64_t)(t.size() / 9);
        if (n_submeshes) *n_submeshes = (int32_t)m.submeshes.size();
        if (tris && cap > 0) std::memcpy(tris, t.data(), sizeof(double) * 9 * std::min<int64_t>(cap, *n_tris));
    });
}

extern "C" mpt_status mpt_host_rrt_inst(const char *inst_path, int32_t iterations_at_a_time, int64_t cap,
                                        int64_t state_cap, double *starts, double *ends, int64_t *n_edges,
                                        int32_t *dim, int32_t *solved) {
    return hguard([&] {
        if (!inst_path || !n_edges) throw std::invalid_argument("null pointer");
        const auto r = mpt_host::run_inst(inst_path, iterations_at_a_time);
        const int64_t n = r.dim ? (int64_t)(r.ends.size() / r.dim) : 0;
        *n_edges = n;
        if (dim) *dim = r.dim;
        if (solved) *solved = r.solved ? 1 : 0;
        // rows that fit both the edge cap and the state buffers (state_cap doubles each)
        const int64_t m = std::min<int64_t>(n, std::min<int64_t>(cap, r.dim ? state_cap / r.dim : 0));
        if (starts && m > 0) std::memcpy(starts, r.starts.data(), sizeof(double) * r.dim * m);
        if (ends && m > 0) std::memcpy(ends, r.ends.data(), sizeof(double) * r.dim * m);
    });
}

extern "C" mpt_status mpt_host_rrt_batched(const char *inst_path, int64_t out[4], double *seconds, int64_t cap,
                                           int64_t state_cap, double *tree0_states, int32_t *tree0_parents,
                                           int64_t *tree0_nodes, int32_t *dim) {
    return hguard([&] {
        if (!inst_path || !out) throw std::invalid_argument("null pointer");
        const auto r = mpt_host::run_batched_inst(inst_path);
        int64_t solved = 0;
        for (int32_t s : r.solved) solved += s;
        out[0] = r.rounds;
        out[1] = r.checked;
        out[2] = r.valid;
        out[3] = solved;
        if (seconds) *seconds = r.seconds;
        if (dim) *dim = r.dim;
        const int64_t n = r.nodes.empty() ? 0 : r.nodes[0];
        if (tree0_nodes) *tree0_nodes = n;
        // parents: up to cap nodes; states: up to the rows state_cap doubles hold
        const int64_t m = std::min<int64_t>(n, cap);
        const int64_t ms = std::min<int64_t>(m, r.dim ? state_cap / r.dim : 0);
        if (tree0_states && ms > 0) std::memcpy(tree0_states, r.first.data(), sizeof(double) * r.dim * ms);
        if (tree0_parents && m > 0) std::memcpy(tree0_parents, r.first_parents.data(), sizeof(int32_t) * m);
    });
}

extern "C" mpt_status mpt_host_prm(const char *inst_path, const double *states, int64_t n, int32_t batch,
                                   int32_t max_queries, int64_t cap, int32_t *edges, double *costs, int64_t *n_edges,
                                   int64_t comp_cap, int32_t *comp, int64_t *n_milestones, int32_t *solved,
                                   double *cost) {
    return hguard([&] {
        if (!inst_path || !n_edges || !n_milestones) throw std::invalid_argument("null pointer");
        if (states && n < 0) throw std::invalid_argument("n < 0");
        const auto r = mpt_host::run_prm_inst(inst_path, states, n, batch, max_queries);
        const int64_t ne = (int64_t)r.costs.size();
        *n_edges = ne;
        *n_milestones = r.milestones;
        if (solved) *solved = r.solved ? 1 : 0;
        if (cost) *cost = r.cost;
        const int64_t m = std::min<int64_t>(ne, cap);
        if (edges && m > 0) std::memcpy(edges, r.edges.data(), sizeof(int32_t) * 2 * m);
        if (costs && m > 0) std::memcpy(costs, r.costs.data(), sizeof(double) * m);
        const int64_t mc = std::min<int64_t>(r.milestones, comp_cap);
        if (comp && mc > 0) std::memcpy(comp, r.comp.data(), sizeof(int32_t) * mc);
    });
}

extern "C" mpt_status mpt_host_grid_discretization(const char *inst_path, const double sizes[3], int64_t cap,
                                                   uint8_t *free_out, double *centers, int64_t *n_cells) {
    return hguard([&] {
        if (!inst_path || !sizes || !n_cells) throw std::invalid_argument("null pointer");
        const auto r = mpt_host::run_grid_inst(inst_path, std::vector<double>(sizes, sizes + 3));
        const int64_t n = (int64_t)r.free.size();
        *n_cells = n;
        const int64_t m = std::min<int64_t>(n, cap);
        if (free_out && m > 0) std::memcpy(free_out, r.free.data(), (size_t)m);
        if (centers && m > 0) std::memcpy(centers, r.centers.data(), sizeof(double) * 3 * m);
    });
}

extern "C" mpt_status mpt_host_prmlite(const char *inst_path, int32_t n_vertices, double step, double *verts,
                                       int64_t cap, int32_t *edges, int64_t *n_edges) {
    return hguard([&] {
        if (!inst_path || !n_edges || n_vertices < 0) throw std::invalid_argument("bad arguments");
        const auto r = mpt_host::run_prmlite_inst(inst_path, n_vertices, step);
        if (verts) std::memcpy(verts, r.verts.data(), sizeof(double) * std::min<size_t>(r.verts.size(), (size_t)n_vertices * 12));
        const int64_t ne = (int64_t)r.edges.size() / 2;
        *n_edges = ne;
        const int64_t m = std::min<int64_t>(ne, cap);
        if (edges && m > 0) std::memcpy(edges, r.edges.data(), sizeof(int32_t) * 2 * m);
    });
}
