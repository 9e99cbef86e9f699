// compose.hpp -- composition root for `.inst` planning runs, main.cpp:38-76 (omnidirectional)
// extended to the Blimp and Snake agents whose dispatch is commented out in the
// reference (main.cpp:78-190, 202-207).  The typedef stack is the reference's with
// FLANN_KDTreeWrapper replaced by GpuNN and Map3D/MeshHandler running on the GPU.
#pragma once
#include <chrono>
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
    // main.cpp:39-55 with FLANN_KDTreeWrapper<KDTreeType, flann::L2<double>, Edge> -> GpuNN<Edge>
    typedef Map3D<Agent> Workspace;
    typedef flann::KDTreeSingleIndexParams KDTreeType;
    typedef GpuNN<typename Agent::Edge> KDTree;
    typedef UniformSampler<Workspace, Agent, KDTree> Sampler;
    typedef TreeInterface<Agent, KDTree, Sampler> TreeIface;
    typedef RRT<Workspace, Agent, TreeIface> Planner;

    Agent agent(args);
    Workspace workspace(args);
    typename Agent::State start(parse_doubles(args.value("Agent Start Location")));
    typename Agent::State goal(parse_doubles(args.value("Agent Goal Location")));
    KDTreeType kdtreeType;
    KDTree kdtree(kdtreeType, agent.getTreeStateSize());
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

// Batched throughput mode of the `.inst` entry point (SURVEY §5 config keys): when the file
// names `Batch Size ? K`, the planner runs the device engine (include/mpt.h mpt_rrt_*) instead
// of the one-extension-at-a-time RRT::query:
//   Batch Size ? K          extensions per round (per tree)
//   Seed ? s                engine seed of the first tree (default 0)
//   Seed Count ? n          independent trees, seeds s .. s + n - 1 (default 1), one
//                           mpt_rrt_step_many round for all of them
//   Rounds ? R              rounds to run (default: until every tree holds Max Tree Size
//                           nodes, checked every 8 rounds; a check window in which no tree
//                           grew ends the run too, so a fully blocked start terminates)
//   Max Tree Size ? N       nodes per tree (default 1 + R * K; 100 000 without Rounds)
//   NN Index ? auto|brute|grid|tree   (default auto)
// Every tree grows from `Agent Start Location`; a tree is solved when one of its nodes is a
// goal (Agent::isGoal against `Agent Goal Location`).
struct BatchedResult {
    int dim = 0;
    int64_t rounds = 0, checked = 0, valid = 0;
    double seconds = 0;
    std::vector<int64_t> nodes;  // per tree
    std::vector<int32_t> solved; // per tree: 1 when a node is a goal
    std::vector<double> first;   // tree 0's states [nodes[0]][dim]
    std::vector<int32_t> first_parents;
};

template <class Agent>
BatchedResult run_batched(const InstanceFileMap &args) {
    Agent agent(args);
    Map3D<Agent> workspace(args);
    typename Agent::State start(parse_doubles(args.value("Agent Start Location")));
    typename Agent::State goal(parse_doubles(args.value("Agent Goal Location")));
    const int32_t K = std::stoi(args.value("Batch Size"));
    const uint64_t seed = std::stoull(args.value_or("Seed", "0"));
    const int32_t n = std::stoi(args.value_or("Seed Count", "1"));
    const int64_t R = std::stoll(args.value_or("Rounds", "-1"));
    const int64_t cap = std::stoll(args.value_or("Max Tree Size", R > 0 ? std::to_string(1 + R * (int64_t)K) : "100000"));
    const std::string nn = args.value_or("NN Index", "auto");
    const int32_t nn_mode = nn == "brute" ? MPT_NN_BRUTE : nn == "grid" ? MPT_NN_GRID : nn == "tree" ? MPT_NN_TREE
                                                                                                     : MPT_NN_AUTO;
    if (K < 1 || n < 1 || cap < 1) throw std::runtime_error("Batch Size, Seed Count and Max Tree Size must be >= 1");
    const unsigned d = agent.getTreeStateSize();
    std::vector<double> ranges;
    for (const auto &r : agent.getStateVarRanges(workspace.getBounds())) {
        ranges.push_back(r.first);
        ranges.push_back(r.second);
    }
    double prm[7];
    agent.params(prm);
    const double steer_dt = std::stod(args.value("Steering Delta t"));
    const double cc_dt = std::stod(args.value("Collision Check Delta t"));
    std::vector<mpt_rrt *> rs((size_t)n, nullptr);
    struct Guard {
        std::vector<mpt_rrt *> &rs;
        ~Guard() {
            for (mpt_rrt *r : rs)
                if (r) mpt_rrt_destroy(r);
        }
    } guard{rs};
    const std::vector<double> &sv = start.getStateVars();
    for (int32_t i = 0; i < n; ++i) {
        mpt_throw(mpt_rrt_create(workspace.environment().handle(), agent.agentMesh().handle(), Agent::kEngineKind, prm,
                                 ranges.data(), (int32_t)d, steer_dt, cc_dt, cap, seed + (uint64_t)i, &rs[i]),
                  "mpt_rrt_create");
        mpt_throw(mpt_rrt_add_nodes(rs[i], sv.data(), nullptr, 1), "mpt_rrt_add_nodes");
        mpt_throw(mpt_rrt_set_nn(rs[i], nn_mode, 0.0), "mpt_rrt_set_nn");
    }
    std::vector<void *> streams((size_t)n, nullptr);
    BatchedResult r;
    r.dim = (int)d;
    const auto t0 = std::chrono::steady_clock::now();
    constexpr int64_t kCheckEvery = 8;
    uint64_t last_total = 0;
    for (int64_t round = 0; R > 0 ? round < R : true; ++round) {
        if (n == 1)
            mpt_throw(mpt_rrt_step(rs[0], K, nullptr), "mpt_rrt_step");
        else
            mpt_throw(mpt_rrt_step_many(rs.data(), n, K, streams.data(), nullptr), "mpt_rrt_step_many");
        ++r.rounds;
        if (R <= 0 && (round + 1) % kCheckEvery == 0) {  // until Max Tree Size (a sync per check)
            uint64_t total = 0;
            bool full = true;
            for (int32_t i = 0; i < n; ++i) {
                uint64_t c[8];
                mpt_throw(mpt_rrt_counters(rs[i], c), "mpt_rrt_counters");
                total += c[3];
                full = full && (int64_t)c[3] >= cap;
            }
            if (full || total == last_total) break;
            last_total = total;
        }
    }
    mpt_throw(mpt_device_synchronize(), "mpt_device_synchronize");
    r.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    for (int32_t i = 0; i < n; ++i) {
        uint64_t c[8];
        mpt_throw(mpt_rrt_counters(rs[i], c), "mpt_rrt_counters");
        r.checked += (int64_t)c[1];
        r.valid += (int64_t)c[2];
        r.nodes.push_back((int64_t)c[3]);
        std::vector<double> st((size_t)c[3] * d);
        std::vector<int32_t> par((size_t)c[3]);
        mpt_throw(mpt_rrt_read_tree(rs[i], st.data(), par.data(), (int64_t)c[3]), "mpt_rrt_read_tree");
        int32_t solved = 0;
        for (uint64_t k = 0; k < c[3] && !solved; ++k)
            solved = agent.isGoal(agent.buildState(StateVars(st.begin() + k * d, st.begin() + (k + 1) * d)), goal) ? 1 : 0;
        r.solved.push_back(solved);
        if (i == 0) {
            r.first = std::move(st);
            r.first_parents = std::move(par);
        }
    }
    return r;
}

inline BatchedResult run_batched_inst(const std::string &path) {
    InstanceFileMap args(path);
    const std::string type = args.value("Agent Type");
    if (type == "Omnidirectional") return run_batched<Omnidirectional>(args);
    if (type == "Blimp") return run_batched<Blimp>(args);
    if (type == "Snake") return run_batched<SnakeTrailers>(args);
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
