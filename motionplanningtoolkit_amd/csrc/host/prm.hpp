// prm.hpp -- PRM (planners/prm/prm.hpp:47-387) with the reference's plugin surface, over the
// GPU hot path: milestone kNN through GpuNN (device), edge validation through
// Map3D::safeEdges (one device collision call per batch).  The roadmap graph, the
// connected components and Dijkstra stay on the host, as in the reference (BGL there).
//
// addMilestones(batch) is the batched form of addMilestone (prm.hpp:334-387): each new
// milestone connects to its k nearest milestones inserted before the batch; with a batch of
// one this is the reference's sequence exactly.  The reference indexes milestones by their
// first three state variables (prm.hpp:155, KDTree(KDTreeType(), 3, 0)); its
// KDTreeIndexParams index is approximate, the build's kNN is exact.
#pragma once
#include <algorithm>
#include <cstdio>
#include <functional>
#include <limits>
#include <memory>
#include <queue>
#include <stdexcept>
#include <vector>

#include "instance_file_map.hpp"
#include "planning.hpp"

namespace mpt_host {

template <class Workspace, class Agent, class Sampler>
class PRM {
public:
    typedef typename Agent::State AgentState;
    typedef typename Agent::Edge AgentEdge;
    typedef int Vertex;

    // VertexWrapper (prm.hpp:110-141): what the NN stores per milestone.
    struct Milestone {
        std::vector<double> key;  // first three state variables
        Vertex vertex;
        int index = 0;
        const std::vector<double> &getTreeStateVars() const { return key; }
        int getPointIndex() const { return index; }
        void setPointIndex(int v) { index = v; }
    };

    struct RoadmapEdge {
        Vertex target, source;  // boost::add_edge(targetVertex, sourceVertex, ...) order, prm.hpp:373
        double cost;
        std::shared_ptr<AgentEdge> edge;
    };

    PRM(const Workspace &workspace, const Agent &agent, Sampler &sampler, const InstanceFileMap &args,
        int batch = 1, unsigned int k = 10)
        : workspace(workspace), agent(agent), sampler(sampler), nn(3), batch(batch < 1 ? 1 : batch), k(k) {
        steeringDT = std::stod(args.value("Steering Delta t"));
        collisionCheckDT = std::stod(args.value("Collision Check Delta t"));
    }

    // prm.hpp:184-219: start/goal milestones on the first call, then 100 sampled milestones
    // per call until start and goal share a component; then Dijkstra and the path.
    bool query(const AgentState &start, const AgentState &goal, int /*iterationsAtATime*/ = -1,
               bool firstInvocation = true) {
        if (solutionFound) return true;
        if (firstInvocation && agent.isGoal(start, goal)) return true;
        if (firstInvocation) {
            startVertex = addMilestone(start);
            goalVertex = addMilestone(goal);
        }
        if (prmBuilt) {
            constructSolution();
            solutionFound = true;
            return true;
        }
        std::vector<AgentState> samples;
        samples.reserve(100);
        for (int i = 0; i < 100; i++) samples.push_back(sampler.sampleConfiguration());
        addMilestones(samples);
        prmBuilt = sameComponent(startVertex, goalVertex);
        return false;
    }

    Vertex addMilestone(const AgentState &s) { return addMilestones(std::vector<AgentState>{s}).front(); }

    std::vector<Vertex> addMilestones(const std::vector<AgentState> &states) {
        std::vector<Vertex> out;
        out.reserve(states.size());
        for (size_t b0 = 0; b0 < states.size(); b0 += (size_t)batch) {
            const size_t b1 = std::min(states.size(), b0 + (size_t)batch);
            std::vector<const Milestone *> queries;
            for (size_t i = b0; i < b1; ++i) {
                const Vertex v = newVertex(states[i]);
                out.push_back(v);
                queries.push_back(milestones[v].get());
            }
            // kNN of the whole batch against the milestones inserted before it
            std::vector<typename GpuNN<Milestone>::KNNResult> near;
            if (nn.size() > 0) near = nn.kNearestBatch(queries, k);
            else near.resize(queries.size());
            std::vector<AgentEdge> edges;
            std::vector<std::pair<Vertex, Vertex>> ends;
            for (size_t q = 0; q < queries.size(); ++q) {
                const Vertex src = queries[q]->vertex;
                for (const Milestone *m : near[q].elements) {
                    const Vertex tgt = m->vertex;
                    ++totalAttempts[src];
                    ++totalAttempts[tgt];
                    edges.push_back(agent.steer(stateOf[src], stateOf[tgt], 1000));
                    ends.emplace_back(tgt, src);
                }
            }
            const std::vector<bool> ok = workspace.safeEdges(agent, edges, collisionCheckDT);
            for (size_t e = 0; e < edges.size(); ++e) {
                if (!ok[e]) continue;
                const Vertex tgt = ends[e].first, src = ends[e].second;
                ++successfulAttempts[src];
                ++successfulAttempts[tgt];
                roadmap.push_back(RoadmapEdge{tgt, src, edges[e].cost, std::make_shared<AgentEdge>(edges[e])});
                adjacency[tgt].push_back((int)roadmap.size() - 1);
                adjacency[src].push_back((int)roadmap.size() - 1);
                uniteComponents(tgt, src);
            }
            for (const Milestone *m : queries) nn.insertPoint(const_cast<Milestone *>(m));
        }
        return out;
    }

    // prm.hpp:221-272: Dijkstra from the goal over edge costs, then the predecessor chain
    // from the start.  Ties between equal tentative distances resolve by vertex id.
    bool constructSolution() {
        const size_t n = stateOf.size();
        std::vector<double> dist(n, std::numeric_limits<double>::infinity());
        std::vector<int> pred(n);
        for (size_t i = 0; i < n; ++i) pred[i] = (int)i;
        typedef std::pair<double, int> QE;
        std::priority_queue<QE, std::vector<QE>, std::greater<QE>> pq;
        dist[goalVertex] = 0;
        pq.push({0.0, goalVertex});
        while (!pq.empty()) {
            const QE top = pq.top();
            pq.pop();
            if (top.first > dist[top.second]) continue;
            for (int ei : adjacency[top.second]) {
                const RoadmapEdge &e = roadmap[ei];
                const int w = e.target == top.second ? e.source : e.target;
                const double nd = top.first + e.cost;
                if (nd < dist[w]) {
                    dist[w] = nd;
                    pred[w] = top.second;
                    pq.push({nd, w});
                }
            }
        }
        goalDistance = dist;
        solution.clear();
        solutionCost = 0;
        if (!(dist[startVertex] < std::numeric_limits<double>::infinity())) return false;
        for (Vertex v = startVertex; v != goalVertex; v = pred[v]) {
            const Vertex nxt = pred[v];
            for (int ei : adjacency[v]) {
                const RoadmapEdge &e = roadmap[ei];
                if ((e.target == v && e.source == nxt) || (e.source == v && e.target == nxt)) {
                    solution.push_back(e.edge.get());
                    solutionCost += e.cost;
                    break;
                }
            }
        }
        return false;
    }

    bool sameComponent(Vertex a, Vertex b) { return find(a) == find(b); }
    unsigned long milestoneCount() const { return stateOf.size(); }
    unsigned long edgeCount() const { return roadmap.size(); }
    const std::vector<RoadmapEdge> &edges() const { return roadmap; }
    // component label: the smallest milestone of the component
    Vertex component(Vertex v) {
        const Vertex r = find(v);
        return minOf[r];
    }
    bool isSolved() const { return solutionFound; }
    double getSolutionCost() const { return solutionCost; }
    const std::vector<AgentEdge *> &getSolution() const { return solution; }

private:
    Vertex newVertex(const AgentState &s) {
        const Vertex v = (Vertex)stateOf.size();
        stateOf.push_back(s);
        auto m = std::make_unique<Milestone>();
        const auto &sv = s.getStateVars();
        m->key.assign(sv.begin(), sv.begin() + 3);
        m->vertex = v;
        milestones.push_back(std::move(m));
        totalAttempts.push_back(1);  // prm.hpp:343
        successfulAttempts.push_back(0);
        adjacency.emplace_back();
        parent.push_back(v);  // disjointSets.make_set, prm.hpp:346
        rank.push_back(0);
        minOf.push_back(v);
        return v;
    }

    Vertex find(Vertex x) {
        while (parent[x] != x) {
            parent[x] = parent[parent[x]];
            x = parent[x];
        }
        return x;
    }

    // disjoint_sets::union_set: link by rank
    void uniteComponents(Vertex a, Vertex b) {
        a = find(a);
        b = find(b);
        if (a == b) return;
        if (rank[a] < rank[b]) std::swap(a, b);
        parent[b] = a;
        minOf[a] = std::min(minOf[a], minOf[b]);
        if (rank[a] == rank[b]) ++rank[a];
    }

    const Workspace &workspace;
    const Agent &agent;
    Sampler &sampler;
    GpuNN<Milestone> nn;
    int batch;
    unsigned int k;
    double steeringDT = 0, collisionCheckDT = 0;
    std::vector<AgentState> stateOf;
    std::vector<std::unique_ptr<Milestone>> milestones;
    std::vector<unsigned long> totalAttempts, successfulAttempts;
    std::vector<std::vector<int>> adjacency;
    std::vector<RoadmapEdge> roadmap;
    std::vector<Vertex> parent, minOf;
    std::vector<int> rank;
    std::vector<double> goalDistance;
    std::vector<AgentEdge *> solution;
    Vertex startVertex = 0, goalVertex = 0;
    bool solutionFound = false, prmBuilt = false;
    double solutionCost = -1;
};

}  // namespace mpt_host
