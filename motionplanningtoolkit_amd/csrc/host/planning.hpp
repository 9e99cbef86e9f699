// planning.hpp -- Workspace, NN, Sampler, TreeInterface and RRT with the reference's
// plugin surface, over the GPU hot path:
//   Map3D                 workspaces/map3d.hpp:11-50
//   GpuNN (drop-in for)   FLANN_KDTreeWrapper, utilities/flannkdtreewrapper.hpp:8-125
//   UniformSampler        samplers/uniformsampler.hpp:6-43
//   TreeInterface         tree_interfaces/treeinterface.hpp:1-19
//   RRT                   planners/rrt.hpp:10-143
// Template composition is the plugin system, exactly as main.cpp:39-45 composes it.
#pragma once
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <memory>
#include <random>
#include <stdexcept>
#include <unordered_map>
#include <vector>

#include "../../../include/mpt.h"
#include "agents.hpp"
#include "instance_file_map.hpp"
#include "mesh_handler.hpp"

namespace mpt_host {

// ------------------------------------------------------------------ Map3D
template <class Agent>
class Map3D {
public:
    typedef typename Agent::Edge Edge;

    explicit Map3D(const InstanceFileMap &args)
        : mesh(args.resolve(args.value("Environment Mesh")), args.value("Environment Location")), bounds(3) {
        const auto b = parse_doubles(args.value("Environment Bounding Box"));
        if (b.size() < 6) throw std::runtime_error("Environment Bounding Box needs 6 numbers");
        for (int i = 0; i < 3; ++i) bounds[i] = {b[2 * i], b[2 * i + 1]};
    }

    const WorkspaceBounds &getBounds() const { return bounds; }

    bool safeEdge(const Agent &agent, const Edge &edge, double dt, bool checkSelfCollision = false) const {
        return !MeshHandler::isInCollision(mesh, agent.getMeshes(), agent.getPoses(edge, dt), checkSelfCollision);
    }

    // safeEdge over many edges in one device call (the batched form PRM construction uses).
    std::vector<bool> safeEdges(const Agent &agent, const std::vector<Edge> &edges, double dt,
                                bool checkSelfCollision = false) const {
        std::vector<std::vector<std::vector<Transform3f>>> poses;
        poses.reserve(edges.size());
        for (const Edge &e : edges) poses.push_back(agent.getPoses(e, dt));
        const std::vector<uint8_t> v = MeshHandler::collideEdges(mesh, agent.getMeshes(), poses, checkSelfCollision);
        std::vector<bool> ok(v.size());
        for (size_t i = 0; i < v.size(); ++i) ok[i] = v[i] == 0;
        return ok;
    }

    // Map3D::safePoses (map3d.hpp:39-42) as the reference evidently meant it: one pose
    // list per configuration.
    bool safePoses(const Agent &agent, const std::vector<std::vector<Transform3f>> &poses) const {
        return !MeshHandler::isInCollision(mesh, agent.getMeshes(), poses);
    }

    const StaticEnvironmentMeshHandler &environment() const { return mesh; }

private:
    StaticEnvironmentMeshHandler mesh;
    WorkspaceBounds bounds;
};

// ------------------------------------------------------------------ GpuNN
// FLANN's index-parameter types as the reference's composition names them (main.cpp:41,
// prm.hpp:145): tags only -- the device search is exact whichever is chosen, as FLANN's
// KDTreeSingleIndex is with eps = 0 (KDTreeIndex's randomized approximation is not modelled,
// DESIGN.md §2).
namespace flann {
struct KDTreeSingleIndexParams {
    explicit KDTreeSingleIndexParams(int leaf_max_size = 10) : leaf_max_size(leaf_max_size) {}
    int leaf_max_size;
};
struct KDTreeIndexParams {
    explicit KDTreeIndexParams(int trees = 4) : trees(trees) {}
    int trees;
};
template <class T>
struct L2 {
    typedef T ElementType;
    typedef T ResultType;
};
}  // namespace flann

// Same method set and result conventions as FLANN_KDTreeWrapper<KDTreeType, L2<double>, Element>:
// ids start at 1, distances are squared L2, kNearestWithin's `radius` is compared with
// squared distances (as the reference passes it straight to an L2<double> index).
template <class Element>
class GpuNN {
public:
    struct KNNResult {
        std::vector<Element *> elements;
        std::vector<double> distances;
    };

    explicit GpuNN(unsigned int dim, int64_t capacity_hint = 1024) : dim_(dim) {
        mpt_nn *nn = nullptr;
        mpt_throw(mpt_nn_create((int32_t)dim, capacity_hint, &nn), "mpt_nn_create");
        nn_.reset(nn, [](mpt_nn *p) { mpt_nn_destroy(p); });
    }

    // FLANN_KDTreeWrapper(const KDTreeType &type, unsigned int dim, double epsilon = 0)
    // (utilities/flannkdtreewrapper.hpp:21), so main.cpp:54-55's `KDTree kdtree(kdtreeType,
    // agent.getTreeStateSize())` compiles unchanged; the search is exact (epsilon 0).
    template <class KDTreeType>
    GpuNN(const KDTreeType & /*type*/, unsigned int dim, double epsilon = 0) : GpuNN(dim) {
        if (epsilon != 0) throw std::invalid_argument("GpuNN: approximate search (epsilon != 0) is not supported");
    }

    void insertPoint(Element *elem) {
        const std::vector<double> &v = elem->getTreeStateVars();
        int32_t id = 0;
        mpt_throw(mpt_nn_append(nn_.get(), v.data(), 1, &id), "mpt_nn_append");
        elem->setPointIndex(id);
        lookup_[id] = elem;
    }

    // Verbatim flannkdtreewrapper.hpp:42-50: FLANN removePoint(index - 1), i.e. the point
    // inserted just before this one (the reference's off-by-one; no caller uses it).
    void removePoint(Element *elem) {
        const int index = elem->getPointIndex();
        if (index == 0) return;
        if (index - 1 >= 1) mpt_throw(mpt_nn_remove(nn_.get(), index - 1), "mpt_nn_remove");
        elem->setPointIndex(0);
        lookup_.erase(index);
    }

    KNNResult nearest(const Element *elem) { return kNearest(elem, 1); }

    KNNResult kNearest(const Element *elem, unsigned int k) {
        if (k == 0 || elem == nullptr) throw std::invalid_argument("kNearest: k > 0 and elem != NULL");
        const std::vector<double> v = elem->getTreeStateVars();
        std::vector<int32_t> ids(k);
        std::vector<double> d2(k);
        mpt_throw(mpt_nn_knn(nn_.get(), v.data(), 1, (int32_t)k, ids.data(), d2.data(), nullptr), "mpt_nn_knn");
        KNNResult r;
        for (unsigned i = 0; i < k; ++i) {
            if (ids[i] < 0) break;
            r.elements.push_back(lookup_.at(ids[i]));
            r.distances.push_back(d2[i]);
        }
        return r;
    }

    // kNearest for many query elements in one device call.
    std::vector<KNNResult> kNearestBatch(const std::vector<const Element *> &elems, unsigned int k) {
        if (k == 0) throw std::invalid_argument("kNearestBatch: k > 0");
        const int64_t nq = (int64_t)elems.size();
        std::vector<KNNResult> out((size_t)nq);
        if (nq == 0) return out;
        std::vector<double> q;
        q.reserve((size_t)nq * dim_);
        for (const Element *e : elems) {
            const std::vector<double> &v = e->getTreeStateVars();
            q.insert(q.end(), v.begin(), v.begin() + dim_);
        }
        std::vector<int32_t> ids((size_t)nq * k);
        std::vector<double> d2((size_t)nq * k);
        mpt_throw(mpt_nn_knn(nn_.get(), q.data(), nq, (int32_t)k, ids.data(), d2.data(), nullptr), "mpt_nn_knn");
        for (int64_t i = 0; i < nq; ++i)
            for (unsigned j = 0; j < k; ++j) {
                const int32_t id = ids[i * k + j];
                if (id < 0) break;
                out[i].elements.push_back(lookup_.at(id));
                out[i].distances.push_back(d2[i * k + j]);
            }
        return out;
    }

    KNNResult kNearestWithin(const Element *elem, double radius, int max_neighbors = -1) const {
        const std::vector<double> v = elem->getTreeStateVars();
        int64_t off[2] = {0, 0};
        mpt_throw(mpt_nn_radius(nn_.get(), v.data(), 1, radius, max_neighbors, off, nullptr, nullptr, 0, nullptr),
                  "mpt_nn_radius");
        std::vector<int32_t> ids((size_t)off[1] + 1);
        std::vector<double> d2((size_t)off[1] + 1);
        mpt_throw(mpt_nn_radius(nn_.get(), v.data(), 1, radius, max_neighbors, off, ids.data(), d2.data(), off[1],
                                nullptr),
                  "mpt_nn_radius");
        KNNResult r;
        for (int64_t i = 0; i < off[1]; ++i) {
            r.elements.push_back(lookup_.at(ids[i]));
            r.distances.push_back(d2[i]);
        }
        return r;
    }

    int64_t size() const {
        int64_t n = 0;
        mpt_nn_size(nn_.get(), &n);
        return n;
    }
    mpt_nn *handle() { return nn_.get(); }

private:
    unsigned int dim_;
    std::shared_ptr<mpt_nn> nn_;
    std::unordered_map<int, Element *> lookup_;
};

// ------------------------------------------------------------------ UniformSampler
template <class Workspace, class Agent, class NN>
class UniformSampler {
    typedef typename Agent::State State;
    typedef typename Agent::Edge Edge;

public:
    UniformSampler(const Workspace &workspace, const Agent &agent, NN &nn) : workspace(workspace), agent(agent), nn(nn) {
        stateVarDomains = agent.getStateVarRanges(workspace.getBounds());
        for (auto range : stateVarDomains) distributions.emplace_back(range.first, range.second);
    }

    State getTreeSample() const {
        auto sample = sampleConfiguration();
        auto sampleEdge = Edge(sample);
        typename NN::KNNResult result = nn.nearest(&sampleEdge);
        return result.elements[0]->end;
    }

    // private in the reference (uniformsampler.hpp:28); public here so PRM can use it
    // (prm.hpp:223 calls it and would not compile against the reference sampler).
    State sampleConfiguration() const {
        StateVars vars;
        for (auto distribution : distributions) vars.push_back(distribution(generator));
        return agent.buildState(vars);
    }

private:
    const Workspace &workspace;
    const Agent &agent;
    NN &nn;
    StateVarRanges stateVarDomains;
    std::vector<std::uniform_real_distribution<double>> distributions;
    mutable std::default_random_engine generator;
};

// ------------------------------------------------------------------ TreeInterface
template <class Agent, class InsertionInterface, class QueryInterface>
class TreeInterface {
    typedef typename Agent::State State;
    typedef typename Agent::Edge Edge;

public:
    TreeInterface(InsertionInterface &ins, QueryInterface &q) : insertionInterface(ins), queryInterface(q) {}
    State getTreeSample() { return queryInterface.getTreeSample(); }
    void insertIntoTree(Edge *edge) { insertionInterface.insertPoint(edge); }

private:
    InsertionInterface &insertionInterface;
    QueryInterface &queryInterface;
};

// ------------------------------------------------------------------ RRT
template <class Workspace, class Agent, class TreeInterfaceT>
class RRT {
public:
    typedef typename Agent::State State;
    typedef typename Agent::Edge Edge;

    RRT(const Workspace &workspace, const Agent &agent, TreeInterfaceT &treeInterface, const InstanceFileMap &args)
        : workspace(workspace), agent(agent), treeInterface(treeInterface) {
        steeringDT = std::stod(args.value("Steering Delta t"));
        collisionCheckDT = std::stod(args.value("Collision Check Delta t"));
        trace = std::getenv("MPT_RRT_TRACE") != nullptr;
    }

    // planners/rrt.hpp:21-131 (graphics / V-REP branches out of scope).
    void query(const State &start, const State &goal, int iterationsAtATime = -1, bool firstInvocation = true) {
        if (agent.isGoal(start, goal)) {
            fprintf(stderr, "found goal\n");
            return;
        }
        if (firstInvocation) {
            pool.emplace_back(new Edge(start));
            treeInterface.insertIntoTree(pool.back().get());
        }
        unsigned int iterations = 0;
        const auto t0 = std::chrono::steady_clock::now();
        while (!solved) {
            State treeSample = treeInterface.getTreeSample();
            auto edge = agent.randomSteer(treeSample, steeringDT);
            if (trace) std::fputs("RRT iter 2.1\n", stderr);  // rrt.hpp:48, opt-in here
            if (!workspace.safeEdge(agent, edge, collisionCheckDT)) {
                ++iterations;
                if (iterationsAtATime > 0 && (int)++iterations > iterationsAtATime) break;
                continue;
            }
            if (agent.isGoal(edge.end, goal)) {
                const auto ms =
                    std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0);
                fprintf(stdout, "RRT solved in %d[ms]\n", (int)ms.count());
                fprintf(stderr, "found goal\n");
                solved = true;
                goalEdge.reset(new Edge(edge));
                break;
            }
            pool.emplace_back(new Edge(edge));
            treeInterface.insertIntoTree(pool.back().get());
            if (iterationsAtATime > 0 && (int)++iterations > iterationsAtATime) break;
        }
    }

    bool isSolved() const { return solved; }
    const std::deque<std::unique_ptr<Edge>> &tree() const { return pool; }
    const Edge *solutionEdge() const { return goalEdge.get(); }

private:
    const Workspace &workspace;
    const Agent &agent;
    TreeInterfaceT &treeInterface;
    std::deque<std::unique_ptr<Edge>> pool;  // boost::object_pool<Edge> (rrt.hpp:136)
    std::unique_ptr<Edge> goalEdge;
    double steeringDT = 0, collisionCheckDT = 0;
    bool solved = false;
    bool trace = false;
};

}  // namespace mpt_host
