// mesh_handler.hpp -- GPU-backed StaticEnvironmentMeshHandler / SimpleAgentMeshHandler /
// MeshHandler (utilities/meshhandler.hpp:16-243) and fcl_helpers::parseTransform
// (utilities/fcl_helpers.hpp:16-25).  The FCL BVHModel<OBBRSS> + DynamicAABBTree managers
// are replaced by device-resident meshes behind the C ABI (include/mpt.h); isInCollision
// becomes one mpt_collide_batch_ex call for the whole pose list (checkSelfCollision included).
#pragma once
#include <array>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../../include/mpt.h"
#include "mesh_loader.hpp"

namespace mpt_host {

// fcl::Transform3f as R (row-major 3x3) + T.
struct Transform3f {
    std::array<double, 9> R{{1, 0, 0, 0, 1, 0, 0, 0, 1}};
    std::array<double, 3> T{{0, 0, 0}};
    Transform3f() = default;
    explicit Transform3f(const std::array<double, 3> &t) : T(t) {}
    Transform3f(const std::array<double, 9> &r, const std::array<double, 3> &t) : R(r), T(t) {}
};

inline void mpt_throw(mpt_status st, const char *what) {
    if (st != MPT_OK) throw std::runtime_error(std::string(what) + ": " + mpt_last_error());
}

// fcl_helpers::parseTransform("x y z qw qx qy qz") -> Transform3f(Quaternion3f, Vec3f)
inline Transform3f parseTransform(const std::string &s) {
    std::istringstream in(s);
    double loc[7];
    for (double &v : loc)
        if (!(in >> v)) throw std::runtime_error("bad transform: " + s);
    double tf[12];
    mpt_throw(mpt_transform_from_location(loc, tf), "parseTransform");
    Transform3f t;
    for (int i = 0; i < 9; ++i) t.R[i] = tf[i];
    for (int i = 0; i < 3; ++i) t.T[i] = tf[9 + i];
    return t;
}

class StaticEnvironmentMeshHandler {
public:
    StaticEnvironmentMeshHandler(const std::string &filename, const std::string &pose)
        : StaticEnvironmentMeshHandler(load_or_throw(filename).soup(), parseTransform(pose)) {}

    StaticEnvironmentMeshHandler(const std::vector<double> &soup, const Transform3f &tf) : tf_(tf), soup_(soup) {
        double t12[12];
        for (int i = 0; i < 9; ++i) t12[i] = tf.R[i];
        for (int i = 0; i < 3; ++i) t12[9 + i] = tf.T[i];
        mpt_env *e = nullptr;
        mpt_throw(mpt_env_create(soup.data(), (int64_t)(soup.size() / 9), t12, &e), "mpt_env_create");
        env_.reset(e, [](mpt_env *p) { mpt_env_destroy(p); });
    }

    const mpt_env *handle() const { return env_.get(); }
    const Transform3f &transform() const { return tf_; }
    const std::vector<double> &triangles() const { return soup_; }

    static MeshFile load_or_throw(const std::string &f) {
        MeshFile m = load_mesh(f);
        if (m.error) throw std::runtime_error(m.message);
        return m;
    }

private:
    Transform3f tf_;
    std::vector<double> soup_;
    std::shared_ptr<mpt_env> env_;
};

class SimpleAgentMeshHandler {
public:
    // keep_all = false reproduces the reference (last non-empty submesh only).
    explicit SimpleAgentMeshHandler(const std::string &filename, bool keep_all = false) {
        const MeshFile m = StaticEnvironmentMeshHandler::load_or_throw(filename);
        init(keep_all ? m.soup() : m.last_nonempty());
    }
    explicit SimpleAgentMeshHandler(const std::vector<double> &soup) { init(soup); }

    const mpt_agent *handle() const { return agent_.get(); }
    const std::vector<double> &triangles() const { return soup_; }

private:
    void init(const std::vector<double> &soup) {
        soup_ = soup;
        mpt_agent *a = nullptr;
        mpt_throw(mpt_agent_create(soup.data(), (int64_t)(soup.size() / 9), &a), "mpt_agent_create");
        agent_.reset(a, [](mpt_agent *p) { mpt_agent_destroy(p); });
    }
    std::vector<double> soup_;
    std::shared_ptr<mpt_agent> agent_;
};

class MeshHandler {
public:
    // MeshHandler::isInCollision(environment, agent meshes, poses[P][L]) -> any contact.
    static bool isInCollision(const StaticEnvironmentMeshHandler &environment,
                              const std::vector<const SimpleAgentMeshHandler *> &agent,
                              const std::vector<std::vector<Transform3f>> &poses, bool checkSelfCollision = false) {
        const int32_t L = (int32_t)agent.size();
        if (L == 0 || poses.empty()) return false;
        std::vector<double> buf;
        buf.reserve(poses.size() * L * 12);
        int64_t P = 0;
        for (const auto &pose : poses) {
            if (pose.empty()) continue;  // Blimp's reference stub: an empty pose list
            if ((int32_t)pose.size() != L) throw std::runtime_error("pose/link count mismatch");
            for (const auto &t : pose) {
                buf.insert(buf.end(), t.R.begin(), t.R.end());
                buf.insert(buf.end(), t.T.begin(), t.T.end());
            }
            ++P;
        }
        if (P == 0) return false;
        std::vector<const mpt_agent *> links(L);
        for (int32_t l = 0; l < L; ++l) links[l] = agent[l]->handle();
        const int64_t off[2] = {0, P};
        uint8_t verdict = 0;
        mpt_throw(mpt_collide_batch_ex(environment.handle(), links.data(), L, buf.data(), off, 1,
                                       checkSelfCollision ? 1 : 0, &verdict, nullptr),
                  "mpt_collide_batch_ex");
        return verdict != 0;
    }

    // isInCollision for many edges in one device call: edges[e] = poses[P_e][L];
    // returns one verdict per edge (1 = contact).
    static std::vector<uint8_t> collideEdges(const StaticEnvironmentMeshHandler &environment,
                                             const std::vector<const SimpleAgentMeshHandler *> &agent,
                                             const std::vector<std::vector<std::vector<Transform3f>>> &edges,
                                             bool checkSelfCollision = false) {
        const int32_t L = (int32_t)agent.size();
        std::vector<uint8_t> verdict(edges.size(), 0);
        if (L == 0 || edges.empty()) return verdict;
        std::vector<double> buf;
        std::vector<int64_t> off(edges.size() + 1, 0);
        for (size_t e = 0; e < edges.size(); ++e) {
            int64_t P = 0;
            for (const auto &pose : edges[e]) {
                if (pose.empty()) continue;
                if ((int32_t)pose.size() != L) throw std::runtime_error("pose/link count mismatch");
                for (const auto &t : pose) {
                    buf.insert(buf.end(), t.R.begin(), t.R.end());
                    buf.insert(buf.end(), t.T.begin(), t.T.end());
                }
                ++P;
            }
            off[e + 1] = off[e] + P;
        }
        std::vector<const mpt_agent *> links(L);
        for (int32_t l = 0; l < L; ++l) links[l] = agent[l]->handle();
        mpt_throw(mpt_collide_batch_ex(environment.handle(), links.data(), L, buf.data(), off.data(),
                                       (int64_t)edges.size(), checkSelfCollision ? 1 : 0, verdict.data(), nullptr),
                  "mpt_collide_batch_ex");
        return verdict;
    }
};

}  // namespace mpt_host
