// agents.hpp -- the Agent plugin surface (State, Edge, steer, randomSteer, getPoses, ...)
// for the three agents the BASELINE configs use:
//   Omnidirectional  agents/omnidirectional.hpp:10-287
//   Blimp            agents/blimp.hpp:11-373
//   SnakeTrailers    agents/snake_trailers.hpp:11-496
// Arithmetic, RNG engines and draw order are the reference's (glibc rand() for the
// omni agent, a default-seeded std::default_random_engine member for blimp/snake).
// The OpenGL/V-REP members are out of scope.  One build-defined extension:
// Blimp::getPoses, a stub in the reference (blimp.hpp:219-223, no poses => never
// checked), samples max(1, floor(edge.dt / dt)) states along doStep (end state
// included) with R from theta as Blimp::stateToFCLTransform (blimp.hpp:339-356);
// `Blimp Poses ? reference` in the .inst restores the stub.
#pragma once
#include <cmath>
#include <cstdlib>
#include <limits>
#include <random>
#include <string>
#include <vector>

#include "instance_file_map.hpp"
#include "mesh_handler.hpp"

namespace mpt_host {

typedef std::vector<std::pair<double, double>> WorkspaceBounds;

// getRepresentivePosesForLocation of the blimp and the snake (agents/blimp.hpp:194-217,
// snake_trailers.hpp:220-244): 4 yaw rotations i * pi/8 at loc, rotation(0,0) = cos,
// (0,1) = sin, (1,0) = -sin, (1,1) = cos; one single-link pose each.
inline std::vector<std::vector<Transform3f>> rotated_location_poses(const std::vector<double> &loc) {
    std::vector<std::vector<Transform3f>> ret;
    const unsigned rotations = 4;
    const double increment = M_PI / ((double)rotations * 2.);
    for (unsigned i = 0; i < rotations; ++i) {
        const double c = std::cos((double)i * increment), s = std::sin((double)i * increment);
        ret.push_back({Transform3f({{c, s, 0, -s, c, 0, 0, 0, 1}}, {{loc[0], loc[1], loc[2]}})});
    }
    return ret;
}
typedef std::vector<std::pair<double, double>> StateVarRanges;
typedef std::vector<double> StateVars;

inline double normalizeTheta(double t) { return t - 2 * M_PI * std::floor((t + M_PI) / (2 * M_PI)); }

inline unsigned int to_unsigned(double q) {  // C++ double -> unsigned conversion, range-guarded
    return (q >= 4294967296.0 || !(q >= 0)) ? 0u : (unsigned int)q;
}

inline std::vector<double> parse_doubles(const std::string &s) {
    std::vector<double> out;
    size_t i = 0;
    while (i < s.size()) {
        while (i < s.size() && s[i] == ' ') ++i;
        size_t j = i;
        while (j < s.size() && s[j] != ' ') ++j;
        if (j > i) out.push_back(std::stod(s.substr(i, j - i)));
        i = j;
    }
    return out;
}

inline bool keep_all_submeshes(const InstanceFileMap &args) {
    return args.value_or("Agent Mesh Submeshes", "last") == "all";
}

// ------------------------------------------------------------------ Omnidirectional
class Omnidirectional {
public:
    class State {
    public:
        State() : stateVars(3, 0.0), treeIndex(0) {}
        State(double x, double y, double z = 0) : stateVars{x, y, z}, treeIndex(0) {}
        State(const StateVars &vars) : stateVars(vars.begin(), vars.begin() + 3), treeIndex(0) {}
        bool equals(const State &s) const {
            return std::fabs(stateVars[0] - s.stateVars[0]) <= 0.000001 &&
                   std::fabs(stateVars[1] - s.stateVars[1]) <= 0.000001 &&
                   std::fabs(stateVars[2] - s.stateVars[2]) <= 0.000001;
        }
        double x() const { return stateVars[0]; }
        double y() const { return stateVars[1]; }
        double z() const { return stateVars[2]; }
        const StateVars &getStateVars() const { return stateVars; }
        int getPointIndex() const { return treeIndex; }
        void setPointIndex(int i) { treeIndex = i; }

    private:
        StateVars stateVars;
        int treeIndex;
    };

    class Edge {
    public:
        Edge(const State &s) : start(s), end(s), cost(0), treeIndex(0) {}
        Edge(const State &s, const State &e, double c) : start(s), end(e), cost(c), treeIndex(0) {}
        const StateVars &getTreeStateVars() const { return end.getStateVars(); }
        int getPointIndex() const { return treeIndex; }
        void setPointIndex(int i) { treeIndex = i; }
        const State start, end;
        double cost;
        int treeIndex;
    };

    explicit Omnidirectional(const InstanceFileMap &args)
        : mesh(args.resolve(args.value("Agent Mesh")), keep_all_submeshes(args)),
          goalThresholds(parse_doubles(args.value("Goal Thresholds"))) {}

    unsigned int getTreeStateSize() const { return 3; }
    StateVarRanges getStateVarRanges(const WorkspaceBounds &bounds) const { return bounds; }
    State buildState(const StateVars &v) const { return State(v); }

    bool isGoal(const State &s, const State &g) const {
        return std::fabs(s.x() - g.x()) < goalThresholds[0] && std::fabs(s.y() - g.y()) < goalThresholds[1] &&
               std::fabs(s.z() - g.z()) < goalThresholds[2];
    }

    Edge steer(const State &start, const State &goal, double dt) const {
        const double dx = goal.x() - start.x(), dy = goal.y() - start.y(), dz = goal.z() - start.z();
        const double dist = std::sqrt(dx * dx + dy * dy + dz * dz);
        double fraction = dt / dist;
        if (fraction > 1) fraction = 1;
        State st(start.x() + dx * fraction, start.y() + dy * fraction, start.z() + dz * fraction);
        return Edge(start, st, dist);
    }
    Edge steer(const State &start, const State &goal) const {
        return steer(start, goal, std::numeric_limits<double>::infinity());
    }

    Edge randomSteer(const State &start, double /*dt*/) const {
        const double randX = ((double)rand() - ((double)RAND_MAX / 2)) / ((double)RAND_MAX / 2);
        const double randY = ((double)rand() - ((double)RAND_MAX / 2)) / ((double)RAND_MAX / 2);
        const double randZ = ((double)rand() - ((double)RAND_MAX / 2)) / ((double)RAND_MAX / 2);
        const double dist = std::sqrt(randX * randX + randY * randY + randZ * randZ);
        State st(start.x() + randX / dist, start.y() + randY / dist, start.z() + randZ / dist);
        return Edge(start, st, dist);
    }

    std::vector<const SimpleAgentMeshHandler *> getMeshes() const { return {&mesh}; }

    // agents/omnidirectional.hpp:191-200: one pose, translation only
    std::vector<std::vector<Transform3f>> getRepresentivePosesForLocation(const std::vector<double> &loc) const {
        return {{Transform3f({{loc[0], loc[1], loc[2]}})}};
    }

    std::vector<std::vector<Transform3f>> getPoses(const Edge &edge, double dt) const {
        std::vector<std::vector<Transform3f>> ret;
        const double sx = edge.start.x(), sy = edge.start.y(), sz = edge.start.z();
        const double ex = edge.end.x(), ey = edge.end.y(), ez = edge.end.z();
        const double dx = ex - sx, dy = ey - sy, dz = ez - sz;
        const double dist = std::sqrt(dx * dx + dy * dy + dz * dz);
        const unsigned int iterations = to_unsigned(dist / dt);
        if (iterations < 1) {
            ret.push_back({Transform3f({sx, sy, sz})});
            ret.push_back({Transform3f({ex, ey, ez})});
        } else {
            const double step = dt / dist;
            for (unsigned int i = 0; i < iterations; ++i) {
                const double st = step * (double)i;
                ret.push_back({Transform3f({sx + st * dx, sy + st * dy, sz + st * dz})});
            }
            if ((double)iterations * dt < dist) ret.push_back({Transform3f({ex, ey, ez})});
        }
        return ret;
    }

    // the batched engine's view of the agent (include/mpt.h mpt_rrt_create)
    static constexpr int32_t kEngineKind = MPT_AGENT_OMNI;
    const double *params(double out[7]) const {
        for (int i = 0; i < 7; ++i) out[i] = 0.0;
        return out;
    }
    const SimpleAgentMeshHandler &agentMesh() const { return mesh; }

private:
    SimpleAgentMeshHandler mesh;
    std::vector<double> goalThresholds;
};

// ------------------------------------------------------------------ Blimp
class Blimp {
    enum { X = 0, Y = 1, Z = 2, THETA = 3, V = 4, PSI = 5, VZ = 6 };

public:
    class State {
    public:
        State() : stateVars(7, 0.0) {}
        State(const StateVars &vars) : stateVars(vars.begin(), vars.end()) {}
        const StateVars &getStateVars() const { return stateVars; }
        int getPointIndex() const { return treeIndex; }
        void setPointIndex(int i) { treeIndex = i; }

    private:
        StateVars stateVars;
        int treeIndex = 0;
    };

    class Edge {
    public:
        Edge(const State &s) : start(s), end(s), cost(0), dt(0), a(0), w(0), z(0), treeIndex(0) {}
        Edge(const State &s, const State &e, double c, double a_, double w_, double z_)
            : start(s), end(e), cost(c), dt(c), a(a_), w(w_), z(z_), treeIndex(0) {}
        const StateVars &getTreeStateVars() const { return end.getStateVars(); }
        int getPointIndex() const { return treeIndex; }
        void setPointIndex(int i) { treeIndex = i; }
        const State start, end;
        double cost, dt, a, w, z;
        int treeIndex;
    };

    explicit Blimp(const InstanceFileMap &args)
        : mesh(args.resolve(args.value("Agent Mesh")), keep_all_submeshes(args)), linearAccelerations(-1, 1),
          zLinearAccelerations(-1, 1), angularAccelerations(-0.1745, 0.1745) {
        blimpLength = std::stod(args.value("Blimp Length"));
        minimumVelocity = std::stod(args.value("Minimum Velocity"));
        maximumVelocity = std::stod(args.value("Maximum Velocity"));
        minimumTurning = std::stod(args.value("Minimum Turning"));
        maximumTurning = std::stod(args.value("Maximum Turning"));
        minimumVelocityZ = std::stod(args.value("Minimum Velocity Z"));
        maximumVelocityZ = std::stod(args.value("Maximum Velocity Z"));
        goalThresholds = parse_doubles(args.value("Goal Thresholds"));
        referencePoses = args.value_or("Blimp Poses", "sampled") == "reference";
    }

    unsigned int getTreeStateSize() const { return 7; }

    StateVarRanges getStateVarRanges(const WorkspaceBounds &b) const {
        StateVarRanges r(b.begin(), b.end());
        r.emplace_back(0, 2 * M_PI);
        r.emplace_back(minimumVelocity, maximumVelocity);
        r.emplace_back(minimumTurning, maximumTurning);
        r.emplace_back(minimumVelocityZ, maximumVelocityZ);
        return r;
    }

    State buildState(const StateVars &v) const { return State(v); }

    bool isGoal(const State &state, const State &goal) const {
        const StateVars &s = state.getStateVars(), &g = goal.getStateVars();
        return std::fabs(s[X] - g[X]) < goalThresholds[X] && std::fabs(s[Y] - g[Y]) < goalThresholds[Y] &&
               std::fabs(s[Z] - g[Z]) < goalThresholds[Z];
    }

    Edge steer(const State &start, const State & /*goal*/, double dt) const { return randomSteer(start, dt); }

    Edge randomSteer(const State &start, double dt) const {
        const double a = linearAccelerations(generator);
        const double w = angularAccelerations(generator);
        const double z = zLinearAccelerations(generator);
        State end = doStep(start, a, w, z, dt);
        return Edge(start, end, dt, a, w, z);
    }

    std::vector<const SimpleAgentMeshHandler *> getMeshes() const { return {&mesh}; }

    // agents/blimp.hpp:194-217 returns the 4 transforms as one list; each is a pose here
    std::vector<std::vector<Transform3f>> getRepresentivePosesForLocation(const std::vector<double> &loc) const {
        return rotated_location_poses(loc);
    }

    std::vector<std::vector<Transform3f>> getPoses(const Edge &edge, double dt) const {
        std::vector<std::vector<Transform3f>> ret;
        if (referencePoses) {
            ret.resize(1);  // agents/blimp.hpp:219-223
            return ret;
        }
        unsigned int steps = to_unsigned(edge.dt / dt);
        if (steps == 0) steps = 1;
        State s = edge.start;
        for (unsigned int i = 0; i < steps; ++i) {
            s = doStep(s, edge.a, edge.w, edge.z, dt);
            ret.push_back({stateToFCLTransform(s)});
        }
        return ret;
    }

    State doStep(const State &st, double a, double w, double z, double dt) const {
        const StateVars &v = st.getStateVars();
        StateVars n(7);
        n[X] = v[X] + std::cos(v[THETA]) * v[V] * dt;
        n[Y] = v[Y] + std::sin(v[THETA]) * v[V] * dt;
        n[THETA] = normalizeTheta(v[THETA] + v[V] * std::tan(v[PSI]) / blimpLength);
        n[Z] = v[Z] + v[VZ] * dt;
        n[V] = v[V] + a * dt;
        n[PSI] = v[PSI] + w * dt;
        n[VZ] = v[VZ] + z * dt;
        if (n[V] > maximumVelocity) n[V] = maximumVelocity;
        else if (n[V] < minimumVelocity) n[V] = minimumVelocity;
        if (n[PSI] > maximumTurning) n[PSI] = maximumTurning;
        else if (n[PSI] < minimumTurning) n[PSI] = minimumTurning;
        if (n[VZ] > maximumVelocityZ) n[VZ] = maximumVelocityZ;
        else if (n[VZ] < minimumVelocityZ) n[VZ] = minimumVelocityZ;
        return State(n);
    }

    Transform3f stateToFCLTransform(const State &st) const {
        const StateVars &v = st.getStateVars();
        const double s = std::sin(v[THETA]), c = std::cos(v[THETA]);
        return Transform3f({c, s, 0, -s, c, 0, 0, 0, 1}, {v[X], v[Y], v[Z]});
    }

    const double *params(double out[7]) const {
        out[0] = blimpLength; out[1] = minimumVelocity; out[2] = maximumVelocity; out[3] = minimumTurning;
        out[4] = maximumTurning; out[5] = minimumVelocityZ; out[6] = maximumVelocityZ;
        return out;
    }
    const SimpleAgentMeshHandler &agentMesh() const { return mesh; }
    static constexpr int32_t kEngineKind = MPT_AGENT_BLIMP;

private:
    SimpleAgentMeshHandler mesh;
    double blimpLength, minimumVelocity, maximumVelocity, minimumTurning, maximumTurning, minimumVelocityZ,
        maximumVelocityZ;
    mutable std::uniform_real_distribution<double> linearAccelerations, zLinearAccelerations, angularAccelerations;
    mutable std::default_random_engine generator;
    std::vector<double> goalThresholds;
    bool referencePoses = false;
};

// ------------------------------------------------------------------ SnakeTrailers
class SnakeTrailers {
    enum { X = 0, Y = 1, V = 2, PSI = 3, THETA = 4 };

public:
    class State {
    public:
        State() : stateVars(5 + trailerCount, 0.0) {}
        State(const StateVars &vars) : stateVars(vars.begin(), vars.end()) { stateVars.resize(5 + trailerCount); }
        const StateVars &getStateVars() const { return stateVars; }
        int getPointIndex() const { return treeIndex; }
        void setPointIndex(int i) { treeIndex = i; }
        static unsigned int trailerCount;

    private:
        StateVars stateVars;
        int treeIndex = 0;
    };

    class Edge {
    public:
        Edge(const State &s) : start(s), end(s), cost(0), dt(0), a(0), w(0), treeIndex(0) {}
        Edge(const State &s, const State &e, double c, double a_, double w_)
            : start(s), end(e), cost(c), dt(c), a(a_), w(w_), treeIndex(0) {}
        const StateVars &getTreeStateVars() const { return end.getStateVars(); }
        int getPointIndex() const { return treeIndex; }
        void setPointIndex(int i) { treeIndex = i; }
        const State start, end;
        double cost, dt, a, w;
        int treeIndex;
    };

    explicit SnakeTrailers(const InstanceFileMap &args)
        : mesh(args.resolve(args.value("Agent Mesh")), keep_all_submeshes(args)), linearAccelerations(-0.1, 1),
          angularAccelerations(-M_PI / 18., M_PI / 18.) {
        trailerCount = State::trailerCount = (unsigned)std::stoi(args.value("Trailer Count"));
        trailerLength = std::stod(args.value("Trailer Length"));
        hitchLength = std::stod(args.value("Hitch Length"));
        minimumVelocity = std::stod(args.value("Minimum Velocity"));
        maximumVelocity = std::stod(args.value("Maximum Velocity"));
        minimumTurning = std::stod(args.value("Minimum Turning"));
        maximumTurning = std::stod(args.value("Maximum Turning"));
        goalThresholds = parse_doubles(args.value("Goal Thresholds"));
    }

    StateVarRanges getStateVarRanges(const WorkspaceBounds &b) const {
        StateVarRanges r(b.begin(), b.begin() + 2);
        r.emplace_back(minimumVelocity, maximumVelocity);
        r.emplace_back(minimumTurning, maximumTurning);
        for (unsigned i = 0; i < trailerCount + 1; ++i) r.emplace_back(0, 2 * M_PI);
        return r;
    }

    unsigned int getTreeStateSize() const { return 5 + trailerCount; }
    State buildState(const StateVars &v) const { return State(v); }

    bool isGoal(const State &state, const State &goal) const {
        const StateVars &s = state.getStateVars(), &g = goal.getStateVars();
        return std::fabs(s[X] - g[X]) < goalThresholds[X] && std::fabs(s[Y] - g[Y]) < goalThresholds[Y];
    }

    Edge steer(const State &start, const State & /*goal*/, double dt) const {
        const double a = linearAccelerations(generator);
        const double w = angularAccelerations(generator);
        return Edge(start, doStep(start, a, w, dt), dt, a, w);
    }

    Edge randomSteer(const State &start, double dt) const {
        const double a = linearAccelerations(generator);
        const double w = angularAccelerations(generator);
        return Edge(start, doStep(start, a, w, dt), dt, a, w);
    }

    std::vector<const SimpleAgentMeshHandler *> getMeshes() const {
        return std::vector<const SimpleAgentMeshHandler *>(trailerCount + 1, &mesh);
    }

    // snake_trailers.hpp:220-244: 4 poses of one transform (the head link)
    std::vector<std::vector<Transform3f>> getRepresentivePosesForLocation(const std::vector<double> &loc) const {
        return rotated_location_poses(loc);
    }

    std::vector<std::vector<Transform3f>> getPoses(const Edge &edge, double dt) const {
        std::vector<std::vector<Transform3f>> poses;
        unsigned int steps = to_unsigned(edge.dt / dt);
        if (steps == 0) steps = 1;
        State state = edge.start;
        for (unsigned int step = 0; step < steps; ++step) {
            poses.push_back(stateToFCLTransforms(state));
            state = doStep(state, edge.a, edge.w, dt);
        }
        return poses;
    }

    State doStep(const State &st, double a, double w, double dt) const {
        const StateVars &v = st.getStateVars();
        StateVars n(5 + trailerCount);
        n[X] = v[X] + std::cos(v[THETA]) * v[V] * dt;
        n[Y] = v[Y] + std::sin(v[THETA]) * v[V] * dt;
        n[THETA] = normalizeTheta(v[THETA] + v[V] * std::tan(v[PSI]) / trailerLength * dt);
        n[V] = v[V] + a * dt;
        n[PSI] = v[PSI] + w * dt;
        if (n[V] > maximumVelocity) n[V] = maximumVelocity;
        else if (n[V] < minimumVelocity) n[V] = minimumVelocity;
        if (n[PSI] > maximumTurning) n[PSI] = maximumTurning;
        else if (n[PSI] < minimumTurning) n[PSI] = minimumTurning;
        double coeff = v[V] / (trailerLength + hitchLength);
        double prev = v[THETA];
        for (unsigned int i = 1; i < trailerCount + 1; ++i) {
            n[THETA + i] = normalizeTheta(v[THETA + i] + coeff * std::sin(prev - v[THETA + i]) * dt);
            coeff *= std::cos(prev - v[THETA + i]);
            prev = v[THETA + i];
        }
        return State(n);
    }

    // verbatim (snake_trailers.hpp:411-459): trailers at (-(Lt+Lh), Y, 0), not chained
    std::vector<Transform3f> stateToFCLTransforms(const State &st) const {
        std::vector<Transform3f> out;
        const StateVars &v = st.getStateVars();
        std::array<double, 3> pose{{v[X], v[Y], 0}};
        std::array<double, 9> R{{1, 0, 0, 0, 1, 0, 0, 0, 1}};
        double s = std::sin(v[THETA]), c = std::cos(v[THETA]);
        R[0] = c; R[3] = -s; R[1] = s; R[4] = c;
        out.emplace_back(R, pose);
        for (unsigned int i = 1; i < trailerCount + 1; ++i) {
            pose[0] = -(trailerLength + hitchLength);
            const double t = v[THETA + i] - v[THETA + i - 1];
            s = std::sin(t);
            c = std::cos(t);
            R[0] = c; R[3] = -s; R[1] = s; R[4] = c;
            std::array<double, 9> M;
            for (int r = 0; r < 3; ++r)
                for (int cc = 0; cc < 3; ++cc)
                    M[r * 3 + cc] = R[r * 3 + 0] * (cc == 0 ? 1.0 : 0.0) + R[r * 3 + 1] * (cc == 1 ? 1.0 : 0.0) +
                                    R[r * 3 + 2] * (cc == 2 ? 1.0 : 0.0);
            R = M;
            out.emplace_back(R, pose);
        }
        return out;
    }

    const double *params(double out[7]) const {
        out[0] = trailerCount; out[1] = trailerLength; out[2] = hitchLength; out[3] = minimumVelocity;
        out[4] = maximumVelocity; out[5] = minimumTurning; out[6] = maximumTurning;
        return out;
    }
    const SimpleAgentMeshHandler &agentMesh() const { return mesh; }
    static constexpr int32_t kEngineKind = MPT_AGENT_SNAKE;

private:
    SimpleAgentMeshHandler mesh;
    unsigned int trailerCount;
    double trailerLength, hitchLength, minimumVelocity, maximumVelocity, minimumTurning, maximumTurning;
    mutable std::uniform_real_distribution<double> linearAccelerations, angularAccelerations;
    mutable std::default_random_engine generator;
    std::vector<double> goalThresholds;
};

inline unsigned int SnakeTrailers::State::trailerCount = 0;

}  // namespace mpt_host
