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
