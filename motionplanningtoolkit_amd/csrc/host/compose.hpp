// compose.hpp -- composition root for `.inst` planning runs, main.cpp:38-76 (omnidirectional)
// extended to the Blimp and Snake agents whose dispatch is commented out in the
// reference (main.cpp:78-190, 202-207).  The typedef stack is the reference's with
// FLANN_KDTreeWrapper replaced by GpuNN and Map3D/MeshHandler running on the GPU.
#pragma once
#include <cstdlib>
#include <string>
#include <vector>

#include "agents.hpp"
#include "planning.hpp"
#include "discretizations.hpp"
#include "prm.hpp"

namespace mpt_host {

struct RunResult {
    int dim = 0;
    bool solved = false;
    std::vector<double> starts, ends;  // per inserted edge (root: start == end)
};

template <class Agent>
RunResult run_rrt(const InstanceFileMap &args, int iterationsAtATime) {
    typedef Map3D<Agent> Workspace;
    typedef GpuNN<typename Agent::Edge> KDTree;
    typedef UniformSampler<Workspace, Agent, KDTree> Sampler;
    typedef TreeInterface<Agent, KDTree, Sampler> TreeIface;
    typedef RRT<Workspace, Agent, TreeIface> Planner;

    Agent agent(args);
    Workspace workspace(args);
    typename Agent::State start(parse_doubles(args.value("Agent Start Location")));
    typename Agent::State goal(parse_doubles(args.value("Agent Goal Location")));
    KDTree kdtree(agent.getTreeStateSize());
    Sampler sampler(workspace, agent, kdtree);
    TreeIface treeInterface(kdtree, sampler);
    Planner planner(workspace, agent, treeInterface, args);
    planner.query(start, goal, iterationsAtATime, true);

    RunResult r;
    r.dim = (int)agent.getTreeStateSize();
    r.solved = planner.isSolved();
    for (const auto &e : planner.tree()) {
        const auto &s = e->start.getStateVars();
        const auto &t = e->getTreeStateVars();
        r.starts.insert(r.starts.end(), s.begin(), s.begin() + r.dim);
        r.ends.insert(r.ends.end(), t.begin(), t.begin() + r.dim);
    }
    return r;
}

// PRM roadmap over explicit milestone states (tests / FFI): the .inst's agent, workspace and
// step sizes, milestones added in order `batch` at a time.
struct PrmResult {
    std::vector<int32_t> edges;  // [E][2] (target, source)
    std::vector<double> costs;   // [E]
    std::vector<int32_t> comp;   // [n] smallest milestone of each component
    bool solved = false;
    double cost = -1;
    int64_t milestones = 0, queries = 0;
};

template <class Agent>
PrmResult run_prm(const InstanceFileMap &args, const double *states, int64_t n, int32_t batch, int32_t max_queries) {
    typedef Map3D<Agent> Workspace;
    typedef GpuNN<typename Agent::Edge> KDTree;
    typedef UniformSampler<Workspace, Agent, KDTree> Sampler;
    typedef PRM<Workspace, Agent, Sampler> Planner;

    Agent agent(args);
    Workspace workspace(args);
    KDTree kdtree(agent.getTreeStateSize());
    Sampler sampler(workspace, agent, kdtree);
    Planner prm(workspace, agent, sampler, args, batch);
    PrmResult r;
    const unsigned d = agent.getTreeStateSize();
    if (states) {
        std::vector<typename Agent::State> ms;
        for (int64_t i = 0; i < n; ++i) ms.push_back(agent.buildState(StateVars(states + i * d, states + (i + 1) * d)));
        prm.addMilestones(ms);
    } else {
        typename Agent::State start(parse_doubles(args.value("Agent Start Location")));
        typename Agent::State goal(parse_doubles(args.value("Agent Goal Location")));
        bool first = true;
        while (r.queries < max_queries && !prm.query(start, goal, -1, first)) {
            first = false;
            ++r.queries;
        }
        r.solved = prm.isSolved();
        r.cost = prm.getSolutionCost();
    }
    for (const auto &e : prm.edges()) {
        r.edges.push_back(e.target);
        r.edges.push_back(e.source);
        r.costs.push_back(e.cost);
    }
    r.milestones = (int64_t)prm.milestoneCount();
    for (int64_t v = 0; v < r.milestones; ++v) r.comp.push_back(prm.component((int)v));
    return r;
}

inline PrmResult run_prm_inst(const std::string &path, const double *states, int64_t n, int32_t batch,
                              int32_t max_queries) {
    InstanceFileMap args(path);
    srand(1);
    const std::string type = args.value("Agent Type");
    if (type == "Omnidirectional") return run_prm<Omnidirectional>(args, states, n, batch, max_queries);
    if (type == "Blimp") return run_prm<Blimp>(args, states, n, batch, max_queries);
    if (type == "Snake") return run_prm<SnakeTrailers>(args, states, n, batch, max_queries);
    throw std::runtime_error("unrecognized Agent Type: " + type);
}

// Workspace discretisations over the .inst's workspace and agent (discretizations/workspace/).
struct GridResult {
    std::vector<uint8_t> free;
    std::vector<double> centers;  // [cells][3]
};
template <class Agent>
GridResult run_grid(const InstanceFileMap &args, const std::vector<double> &sizes) {
    Agent agent(args);
    Map3D<Agent> workspace(args);
    GridDiscretization<Map3D<Agent>, Agent> grid(workspace, agent, sizes);
    GridResult r;
    for (unsigned int c = 0; c < grid.getCellCount(); ++c) {
        r.free.push_back(grid.isFree(c) ? 1 : 0);
        const auto p = grid.getGridCenter(c);
        r.centers.insert(r.centers.end(), p.begin(), p.end());
    }
    return r;
}

struct LiteResult {
    std::vector<double> verts;   // [V][12]
    std::vector<int32_t> edges;  // [E][2], i < j, row-major order
};
template <class Agent>
LiteResult run_prmlite(const InstanceFileMap &args, int32_t n_vertices, double step) {
    Agent agent(args);
    Map3D<Agent> workspace(args);
    PRMLite<Map3D<Agent>, Agent> lite(workspace, agent, (unsigned)n_vertices, step);
    LiteResult r;
    for (const auto &v : lite.getVertices()) {
        r.verts.insert(r.verts.end(), v.transform.R.begin(), v.transform.R.end());
        r.verts.insert(r.verts.end(), v.transform.T.begin(), v.transform.T.end());
    }
    for (unsigned i = 0; i < lite.getCellCount(); ++i) {
        auto nb = lite.getNeighboringCells(i);
        std::sort(nb.begin(), nb.end());
        for (unsigned j : nb)
            if (j > i) {
                r.edges.push_back((int32_t)i);
                r.edges.push_back((int32_t)j);
            }
    }
    return r;
}

inline GridResult run_grid_inst(const std::string &path, const std::vector<double> &sizes) {
    InstanceFileMap args(path);
    const std::string type = args.value("Agent Type");
    if (type == "Omnidirectional") return run_grid<Omnidirectional>(args, sizes);
    if (type == "Blimp") return run_grid<Blimp>(args, sizes);
    if (type == "Snake") return run_grid<SnakeTrailers>(args, sizes);
    throw std::runtime_error("unrecognized Agent Type: " + type);
}

inline LiteResult run_prmlite_inst(const std::string &path, int32_t n_vertices, double step) {
    InstanceFileMap args(path);
    const std::string type = args.value("Agent Type");
    if (type == "Omnidirectional") return run_prmlite<Omnidirectional>(args, n_vertices, step);
    if (type == "Blimp") return run_prmlite<Blimp>(args, n_vertices, step);
    if (type == "Snake") return run_prmlite<SnakeTrailers>(args, n_vertices, step);
    throw std::runtime_error("unrecognized Agent Type: " + type);
}

// main.cpp:192-212 dispatch on "Agent Type".  The reference never seeds rand() or the
// default engines; a fresh process starts from srand(1), which is re-established here so
// repeated runs in one process replay identically.
inline RunResult run_inst(const std::string &path, int iterationsAtATime) {
    InstanceFileMap args(path);
    srand(1);
    const std::string type = args.value("Agent Type");
    if (type == "Omnidirectional") return run_rrt<Omnidirectional>(args, iterationsAtATime);
    if (type == "Blimp") return run_rrt<Blimp>(args, iterationsAtATime);
    if (type == "Snake") return run_rrt<SnakeTrailers>(args, iterationsAtATime);
    throw std::runtime_error("unrecognized Agent Type: " + type);
}

}  // namespace mpt_host
