// discretizations.hpp -- the workspace discretisations (discretizations/workspace/) over the
// GPU collision path.  Both are batched collision workloads: every grid cell's representative
// poses go to the device in one mpt_collide_batch call, and all PRMLite vertex pairs in one
// mpt_prmlite_edges call (sweep.hip: the pose interpolation runs on the device).
#pragma once
#include <cmath>
#include <random>
#include <stdexcept>
#include <unordered_map>
#include <vector>

#include "planning.hpp"

namespace mpt_host {

// GridDiscretization (griddiscretization.hpp:6-189).  getGridCenter / getGridCoordinates are
// reproduced as written, including their index arithmetic for dims >= 1 (the divisor
// multiplies dimensions[i] rather than dimensions[i-1], and the half-cell offset uses
// discretizationSizes[1] for every dim >= 1).
template <class Workspace, class Agent>
class GridDiscretization {
public:
    GridDiscretization(const Workspace &workspace, const Agent &agent, const std::vector<double> &discretizationSizes)
        : discretizationSizes(discretizationSizes) {
        bounds = workspace.getBounds();
        if (bounds.size() != discretizationSizes.size()) throw std::runtime_error("bounds / sizes mismatch");
        unsigned int cellCount = 1;
        for (unsigned int i = 0; i < discretizationSizes.size(); i++) {
            const double range = std::fabs(bounds[i].first - bounds[i].second);
            dimensions.push_back(range == 0 ? 1u : (unsigned int)std::ceil(range / discretizationSizes[i]));
            cellCount *= dimensions.back();
        }
        // every cell's representative poses in one device call (:26-33 checks them one cell at a time)
        std::vector<std::vector<std::vector<Transform3f>>> cells(cellCount);
        size_t links = 1;
        for (unsigned int i = 0; i < cellCount; i++) {
            cells[i] = agent.getRepresentivePosesForLocation(getGridCenter(i));
            for (const auto &p : cells[i]) links = std::max(links, p.size());
        }
        // isInCollision uses the first pose.size() meshes of the agent (meshhandler.hpp:197-201)
        const auto meshes = agent.getMeshes();
        const std::vector<const SimpleAgentMeshHandler *> used(meshes.begin(), meshes.begin() + links);
        const std::vector<uint8_t> hit = MeshHandler::collideEdges(workspace.environment(), used, cells);
        grid.resize(cellCount);
        for (unsigned int i = 0; i < cellCount; i++) grid[i] = hit[i] == 0;
        populateGridNeighborOffsets();
    }

    unsigned int getContainingCellId(const std::vector<double> &point) const { return getIndex(point); }
    unsigned int getCellCount() const { return (unsigned int)grid.size(); }
    bool isFree(unsigned int cell) const { return grid[cell]; }

    double getCostBetweenCells(unsigned int c1, unsigned int c2) const {
        double sum = 0;
        const auto c1Vec = getGridCoordinates(c1), c2Vec = getGridCoordinates(c2);
        for (unsigned int i = 0; i < discretizationSizes.size(); ++i) {
            const double delta = std::fabs((double)c1Vec[i] - (double)c2Vec[i]) * discretizationSizes[i];
            sum += delta * delta;
        }
        return std::sqrt(sum);
    }

    // :58-71: the box is centre +- the full cell size, as written
    std::vector<std::vector<double>> getCellBoundingHyperRect(unsigned int n) const {
        std::vector<std::vector<double>> out(dimensions.size());
        const auto center = getGridCenter(n);
        for (unsigned int i = 0; i < center.size(); ++i) {
            out[i].push_back(center[i] - discretizationSizes[i]);
            out[i].push_back(center[i] + discretizationSizes[i]);
        }
        return out;
    }

    std::vector<unsigned int> getNeighbors(unsigned int n) const {
        std::vector<unsigned int> neighbors;
        const auto coordinate = getGridCoordinates(n);
        for (const std::vector<int> &offsets : gridNeighborOffsets) {
            std::vector<unsigned int> neighbor(offsets.size());
            bool valid = true;
            for (unsigned int i = 0; i < neighbor.size(); ++i) {
                const int coord = (int)coordinate[i] + offsets[i];
                if (coord < 0 || coord >= (int)dimensions[i]) valid = false;
                neighbor[i] = (unsigned int)coord;
            }
            if (!valid) continue;
            const unsigned int index = getIndex(neighbor);
            if (index < grid.size() && grid[index]) neighbors.push_back(index);
        }
        return neighbors;
    }

    std::vector<double> getGridCenter(unsigned int n) const {
        std::vector<double> point;
        point.push_back(bounds[0].first + (double)(n % dimensions[0]) * discretizationSizes[0] +
                        discretizationSizes[0] * 0.5);
        unsigned int previousDimSizes = 1;
        for (unsigned int i = 1; i < dimensions.size(); i++) {
            previousDimSizes *= dimensions[i];
            point.push_back(bounds[i].first + (double)(n / previousDimSizes % dimensions[i]) * discretizationSizes[i] +
                            discretizationSizes[1] * 0.5);
        }
        return point;
    }

private:
    std::vector<unsigned int> getGridCoordinates(unsigned int n) const {
        std::vector<unsigned int> coordinate;
        coordinate.push_back(n % dimensions[0]);
        unsigned int previousDimSizes = 1;
        for (unsigned int i = 1; i < dimensions.size(); i++) {
            previousDimSizes *= dimensions[i];
            coordinate.push_back(n / previousDimSizes % dimensions[i]);
        }
        return coordinate;
    }

    unsigned int getIndex(const std::vector<double> &point) const {
        unsigned int index = 0;
        for (unsigned int i = 0; i < discretizationSizes.size(); i++) {
            const unsigned int which = (unsigned int)std::floor((point[i] - bounds[i].first) / discretizationSizes[i]);
            double offset = 1;
            for (unsigned int j = 0; j < i; j++) offset *= dimensions[j];
            index += (unsigned int)(which * offset);
        }
        return index;
    }

    unsigned int getIndex(const std::vector<unsigned int> &gridCoordinate) const {
        unsigned int index = 0;
        for (unsigned int i = 0; i < dimensions.size(); i++) {
            double offset = 1;
            for (unsigned int j = 0; j < i; j++) offset *= dimensions[j];
            index += (unsigned int)(gridCoordinate[i] * offset);
        }
        return index;
    }

    void populateGridNeighborOffsets() {
        std::vector<int> neighbor(dimensions.size());
        populateHelper(0, neighbor);
    }
    void populateHelper(unsigned int coord, std::vector<int> &neighbor) {
        if (coord >= dimensions.size()) {
            for (int v : neighbor)
                if (v != 0) {
                    gridNeighborOffsets.push_back(neighbor);
                    return;
                }
            return;
        }
        for (int i = -1; i < 2; ++i) {
            neighbor[coord] = i;
            populateHelper(coord + 1, neighbor);
        }
    }

    std::vector<std::pair<double, double>> bounds;
    std::vector<bool> grid;
    std::vector<double> discretizationSizes;
    std::vector<unsigned int> dimensions;
    std::vector<std::vector<int>> gridNeighborOffsets;
};

// PRMLite (prmlite.hpp:8-263): random collision-free vertices (translation ~ U(bounds),
// uniform random quaternion; the reference's default_random_engine stream), then every vertex
// pair i < j connected unless a pose of PRMLite::interpolate collides.  Vertex candidates are
// checked in batches on the device and the engine is rewound to just after the last
// accepted candidate, so the RNG stream is the reference's.
template <class Workspace, class Agent>
class PRMLite {
public:
    struct Vertex {
        Transform3f transform;
        unsigned int id;
        std::vector<double> treeStateVars;  // tx, ty, tz, qx, qy, qz, qw (:12-24)
        int index = 0;
        const std::vector<double> &getTreeStateVars() const { return treeStateVars; }
        int getPointIndex() const { return index; }
        void setPointIndex(int v) { index = v; }
    };
    struct Edge {
        unsigned int endpoint;
        double weight;
    };

    PRMLite(const Workspace &workspace, const Agent &agent, unsigned int numVertices, double collisionCheckDT = 0.1)
        : kdtree(7) {
        generateVertices(workspace, agent, numVertices);
        generateEdges(workspace, agent, collisionCheckDT);
    }

    unsigned int getCellCount() const { return (unsigned int)vertices.size(); }
    const std::vector<Vertex> &getVertices() const { return vertices; }
    double getEdgeCostBetweenCells(unsigned int c1, unsigned int c2) const { return edges.at(c1).at(c2).weight; }
    std::vector<unsigned int> getNeighboringCells(unsigned int index) const {
        std::vector<unsigned int> ids;
        auto it = edges.find(index);
        if (it == edges.end()) return ids;
        for (const auto &e : it->second) ids.push_back(e.second.endpoint);
        return ids;
    }
    // :96-101 getCellId: the vertex nearest to a transform (7-D key) on the device NN
    unsigned int getCellId(const Transform3f &t, const double quat_wxyz[4]) {
        Vertex v{t, 0, {t.T[0], t.T[1], t.T[2], quat_wxyz[1], quat_wxyz[2], quat_wxyz[3], quat_wxyz[0]}};
        auto res = kdtree.nearest(&v);
        if (res.elements.empty()) throw std::runtime_error("PRMLite: empty roadmap");
        return res.elements[0]->id;
    }

private:
    double zero_to_one() { return zeroToOne(generator); }

    void generateVertices(const Workspace &workspace, const Agent &agent, unsigned int numVertices) {
        const auto bounds = workspace.getBounds();
        std::vector<std::uniform_real_distribution<double>> linear;
        for (const auto &r : bounds) linear.emplace_back(r.first, r.second);
        const auto meshes = agent.getMeshes();
        const std::vector<const SimpleAgentMeshHandler *> head(meshes.begin(), meshes.begin() + 1);
        vertices.reserve(numVertices);
        while (vertices.size() < numVertices) {
            const size_t want = numVertices - vertices.size();
            const size_t batch = std::max<size_t>(64, 2 * want);
            std::vector<Vertex> cand;
            std::vector<std::default_random_engine> after;  // engine state after each candidate
            std::vector<std::vector<std::vector<Transform3f>>> poses;
            for (size_t k = 0; k < batch; ++k) {
                double tr[3];
                for (unsigned int i = 0; i < 3 && i < linear.size(); ++i) tr[i] = linear[i](generator);
                // getRandomQuaternion (:240-249): Quaternion3f(w, x, y, z) arguments in this order
                const double u1 = zero_to_one(), u2 = zero_to_one(), u3 = zero_to_one();
                const double q[4] = {std::sqrt(1 - u1) * std::sin(2 * M_PI * u2), std::sqrt(1 - u1) * std::cos(2 * M_PI * u2),
                                     std::sqrt(u1) * std::sin(2 * M_PI * u3), std::sqrt(u1) * std::cos(2 * M_PI * u3)};
                const double loc[7] = {tr[0], tr[1], tr[2], q[0], q[1], q[2], q[3]};
                double tf[12];
                mpt_throw(mpt_transform_from_location(loc, tf), "quaternion");
                Transform3f t({{tf[0], tf[1], tf[2], tf[3], tf[4], tf[5], tf[6], tf[7], tf[8]}}, {{tr[0], tr[1], tr[2]}});
                cand.push_back(Vertex{t, 0, {tr[0], tr[1], tr[2], q[1], q[2], q[3], q[0]}});
                poses.push_back({{t}});
                after.push_back(generator);
            }
            const std::vector<uint8_t> hit = MeshHandler::collideEdges(workspace.environment(), head, poses);
            for (size_t k = 0; k < cand.size() && vertices.size() < numVertices; ++k) {
                if (hit[k]) continue;
                cand[k].id = (unsigned int)vertices.size();
                vertices.push_back(cand[k]);
                if (vertices.size() == numVertices) generator = after[k];  // as if generation stopped here
            }
        }
        for (auto &v : vertices) kdtree.insertPoint(&v);
    }

    void generateEdges(const Workspace &workspace, const Agent &agent, double collisionCheckDT) {
        const int64_t V = (int64_t)vertices.size();
        std::vector<double> tf((size_t)V * 12);
        for (int64_t i = 0; i < V; ++i) {
            std::copy(vertices[i].transform.R.begin(), vertices[i].transform.R.end(), tf.begin() + i * 12);
            std::copy(vertices[i].transform.T.begin(), vertices[i].transform.T.end(), tf.begin() + i * 12 + 9);
        }
        std::vector<uint8_t> collides((size_t)(V * (V - 1) / 2));
        if (!collides.empty())
            mpt_throw(mpt_prmlite_edges(workspace.environment().handle(), agent.getMeshes()[0]->handle(), tf.data(), V,
                                        collisionCheckDT, collides.data(), nullptr),
                      "mpt_prmlite_edges");
        int64_t e = 0;
        for (int64_t i = 0; i < V; ++i)
            for (int64_t j = i + 1; j < V; ++j, ++e) {
                if (collides[e]) continue;
                const auto &p1 = vertices[i].transform.T, &p2 = vertices[j].transform.T;
                const double dx = p1[0] - p2[0], dy = p1[1] - p2[1], dz = p1[2] - p2[2];
                const double cost = std::sqrt(dx * dx + dy * dy + dz * dz);
                edges[(unsigned)i][(unsigned)j] = Edge{(unsigned)j, cost};
                edges[(unsigned)j][(unsigned)i] = Edge{(unsigned)i, cost};
            }
    }

    std::vector<Vertex> vertices;
    std::unordered_map<unsigned int, std::unordered_map<unsigned int, Edge>> edges;
    GpuNN<Vertex> kdtree;
    std::default_random_engine generator;
    std::uniform_real_distribution<double> zeroToOne;
};

}  // namespace mpt_host
