// rrt_engine.hip -- device-resident batched RRT rounds (throughput mode of planners/rrt.hpp:42-94).
//
// The reference loop does one extension per iteration:
//   sample (UniformSampler::getTreeSample, samplers/uniformsampler.hpp:20-35)
//   -> nearest (FLANN_KDTreeWrapper::nearest, utilities/flannkdtreewrapper.hpp:57-89)
//   -> Agent::randomSteer -> Map3D::safeEdge (Agent::getPoses + MeshHandler::isInCollision)
//   -> TreeInterface::insertIntoTree.
// A round here performs K such extensions against the tree snapshot taken at the start
// of the round (new nodes become visible to the next round), entirely on the device:
//   k_sample -> NN index build + query -> k_steer -> collision -> k_append_commit
// No host synchronisation inside a round; the node count lives in device memory.
// The per-extension randomness comes from a counter-based generator (fcl_math.h
// engine_uniform): extension g uses counters g*64 + j (sample dims) and g*64 + 32 + j
// (controls), so results are independent of the launch geometry and of the GPU count.
// K = 1 reference replay with the reference's own RNG streams is the host planner's job
// (host/rrt.hpp over the same kernels).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

#include "../../include/mpt.h"
#include "grid_nn.h"
#include "cell_tree.h"
#include "mpt_internal.h"
#include "collide_common.h"

namespace mpt {
const EnvDev &env_dev(const mpt_env *e);
int32_t collide_mode();
const AgentDev &agent_dev(const mpt_agent *a);
}  // namespace mpt

using namespace mpt;

namespace {

constexpr int kMaxDim = 16;

// grid cell floor = kGridHminK x the expected NN distance (make_grid_params h_min)
constexpr double kGridHminK = 0.3;
// MPT_NN_AUTO re-reads the nodes' spread at most every kSpreadEvery rounds
constexpr int kSpreadEvery = 8;
// MPT_NN_AUTO: the tree index when the nodes' spatial box covers less than this fraction of
// the sampling box (most samples then lie far from every node, where the grid walks empty
// rings and the tree does not)
constexpr double kAutoTreeFrac = 0.25;

struct EngineParams {
    int32_t kind, d, L, pmax;
    double prm[7];
    double lo[kMaxDim], hi[kMaxDim];
    double steer_dt, cc_dt;
    uint64_t seed;
};

__device__ __forceinline__ double normalize_theta(double t) {
    return t - 2 * M_PI * floor((t + M_PI) / (2 * M_PI));
}

// Blimp::doStep (agents/blimp.hpp:293-317), theta update without dt as written.
__device__ void blimp_step(const double *prm, const double *s, double a, double w, double z, double dt,
                           double *out) {
    double n[7];
    double sv, cv;
    cr_sincos(s[3], sv, cv);  // correctly rounded (fcl_math.h): bitwise the oracle's engine round
    n[0] = s[0] + cv * s[4] * dt;
    n[1] = s[1] + sv * s[4] * dt;
    n[3] = normalize_theta(s[3] + s[4] * cr_tan(s[5]) / prm[0]);
    n[2] = s[2] + s[6] * dt;
    n[4] = s[4] + a * dt;
    n[5] = s[5] + w * dt;
    n[6] = s[6] + z * dt;
    if (n[4] > prm[2]) n[4] = prm[2]; else if (n[4] < prm[1]) n[4] = prm[1];
    if (n[5] > prm[4]) n[5] = prm[4]; else if (n[5] < prm[3]) n[5] = prm[3];
    if (n[6] > prm[6]) n[6] = prm[6]; else if (n[6] < prm[5]) n[6] = prm[5];
#pragma unroll
    for (int i = 0; i < 7; ++i) out[i] = n[i];
}

// SnakeTrailers::doStep (agents/snake_trailers.hpp:341-369).
__device__ void snake_step(const double *prm, int T, const double *s, double a, double w, double dt, double *out) {
    const double Lt = prm[1], Lh = prm[2];
    double n[kMaxDim];
    double sv, cv;
    cr_sincos(s[4], sv, cv);
    n[0] = s[0] + cv * s[2] * dt;
    n[1] = s[1] + sv * s[2] * dt;
    n[4] = normalize_theta(s[4] + s[2] * cr_tan(s[3]) / Lt * dt);
    n[2] = s[2] + a * dt;
    n[3] = s[3] + w * dt;
    if (n[2] > prm[4]) n[2] = prm[4]; else if (n[2] < prm[3]) n[2] = prm[3];
    if (n[3] > prm[6]) n[3] = prm[6]; else if (n[3] < prm[5]) n[3] = prm[5];
    double coeff = s[2] / (Lt + Lh);
    double prev = s[4];
    for (int i = 1; i < T + 1; ++i) {
        double sd, cd;
        cr_sincos(prev - s[4 + i], sd, cd);
        n[4 + i] = normalize_theta(s[4 + i] + coeff * sd * dt);
        coeff *= cd;
        prev = s[4 + i];
    }
    for (int i = 0; i < 5 + T; ++i) out[i] = n[i];
}

__device__ __forceinline__ void put_pose(double *p, const double R[9], double x, double y, double z) {
#pragma unroll
    for (int i = 0; i < 9; ++i) p[i] = R[i];
    p[9] = x;
    p[10] = y;
    p[11] = z;
}

// SnakeTrailers::stateToFCLTransforms (agents/snake_trailers.hpp:411-459), verbatim:
// trailers at (-(Lt + Lh), Y, 0), rotation = rotation * identity (x*1 + y*0 + z*0).
__device__ void snake_poses(const double *prm, int T, const double *s, double *out /*[L][12]*/) {
    double R[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    double sv, cv;
    cr_sincos(s[4], sv, cv);
    R[0] = cv; R[3] = -sv; R[1] = sv; R[4] = cv;
    put_pose(out, R, s[0], s[1], 0.0);
    const double px = -(prm[1] + prm[2]);
    for (int i = 1; i < T + 1; ++i) {
        const double t = s[4 + i] - s[4 + i - 1];
        cr_sincos(t, sv, cv);
        R[0] = cv; R[3] = -sv; R[1] = sv; R[4] = cv;
        double M[9];
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int c = 0; c < 3; ++c)
                M[r * 3 + c] = R[r * 3 + 0] * (c == 0 ? 1.0 : 0.0) + R[r * 3 + 1] * (c == 1 ? 1.0 : 0.0) +
                               R[r * 3 + 2] * (c == 2 ? 1.0 : 0.0);
#pragma unroll
        for (int j = 0; j < 9; ++j) R[j] = M[j];
        put_pose(out + 12 * i, R, px, s[1], 0.0);
    }
}

// n_dev[1] = n_dev[0]: the round's starting node count, read by k_append_commit (which
// overwrites n_dev[0] in the same launch)
// set_n >= 0: a truncation left by mpt_rrt_set_size, applied first (k_set_n folded into the
// round's first launch)
__global__ void k_sample(EngineParams p, uint64_t ext_base, int32_t K, double *__restrict__ samples,
                         int64_t *__restrict__ n_dev, uint32_t *__restrict__ n_live, int64_t set_n,
                         unsigned long long *__restrict__ counters) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k == 0) {
        if (set_n >= 0) {
            n_dev[0] = set_n;
            counters[3] = (unsigned long long)set_n;
        }
        n_dev[1] = n_dev[0];
        if (n_live) *n_live = 0u;  // k_steer's live-unit list of this round
    }
    if (k >= K) return;
    const uint64_t g = ext_base + (uint64_t)k;
    for (int j = 0; j < p.d; ++j) samples[k * p.d + j] = engine_uniform(p.seed, g * 64 + j, p.lo[j], p.hi[j]);
}

// randomSteer + getPoses per extension.  Writes the end state, the pose slots
// [k*pmax + i][L][12] and pcount[k].  KIND fixes the state dim of the omnidirectional (3)
// and blimp (7) agents at compile time, so their states stay in registers (the snake's
// 5 + T is a run-time value).
template <int KIND>
__device__ __forceinline__ int32_t steer_one(const EngineParams &p, uint64_t ext_base, int64_t k,
                                             const double *__restrict__ nodes, const int32_t *__restrict__ nn,
                                             double *__restrict__ ends, double *__restrict__ poses,
                                             int32_t *__restrict__ pcount, uint8_t *__restrict__ verdict,
                                             unsigned long long *__restrict__ counters) {
    verdict[k] = 0;  // the collision stage only ever sets verdicts
    const uint64_t g = ext_base + (uint64_t)k;
    constexpr int DD = KIND == MPT_AGENT_OMNI ? 3 : (KIND == MPT_AGENT_BLIMP ? 7 : kMaxDim);
    const int d = KIND == MPT_AGENT_SNAKE ? p.d : DD;
    double from[DD], end[DD];
    const int64_t src = nn[k] - 1;  // nn ids are 1-based
    if constexpr (KIND == MPT_AGENT_SNAKE) {
        // run-time d: the row loaded whole (clamped, unconditional), not one load at a time
#pragma unroll
        for (int j = 0; j < DD; ++j) from[j] = nodes[src * d + (j < d ? j : d - 1)];
    } else {
#pragma unroll
        for (int j = 0; j < DD; ++j) from[j] = nodes[src * DD + j];
    }
    double *ps = poses + (int64_t)k * p.pmax * p.L * 12;
    int32_t P = 0;
    if constexpr (KIND == MPT_AGENT_OMNI) {
        // Omnidirectional::randomSteer (agents/omnidirectional.hpp:168-184)
        const double rx = engine_uniform(p.seed, g * 64 + 32, -1.0, 1.0);
        const double ry = engine_uniform(p.seed, g * 64 + 33, -1.0, 1.0);
        const double rz = engine_uniform(p.seed, g * 64 + 34, -1.0, 1.0);
        const double dist = sqrt(rx * rx + ry * ry + rz * rz);
        end[0] = from[0] + rx / dist;
        end[1] = from[1] + ry / dist;
        end[2] = from[2] + rz / dist;
        // Omnidirectional::getPoses (agents/omnidirectional.hpp:202-247)
        const double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
        const double dx = end[0] - from[0], dy = end[1] - from[1], dz = end[2] - from[2];
        const double dd = sqrt(dx * dx + dy * dy + dz * dz);
        const double qq = dd / p.cc_dt;
        const unsigned it = (qq >= 4294967296.0 || !(qq >= 0)) ? 0u : (unsigned)qq;
        if (it < 1) {
            if (P < p.pmax) put_pose(ps + 12 * P, I, from[0], from[1], from[2]);
            ++P;
            if (P < p.pmax) put_pose(ps + 12 * P, I, end[0], end[1], end[2]);
            ++P;
        } else {
            const double step = p.cc_dt / dd;
            for (unsigned i = 0; i < it; ++i) {
                const double st = step * (double)i;
                if (P < p.pmax) put_pose(ps + 12 * P, I, from[0] + st * dx, from[1] + st * dy, from[2] + st * dz);
                ++P;
            }
            if ((double)it * p.cc_dt < dd) {
                if (P < p.pmax) put_pose(ps + 12 * P, I, end[0], end[1], end[2]);
                ++P;
            }
        }
    } else if constexpr (KIND == MPT_AGENT_BLIMP) {
        const double a = engine_uniform(p.seed, g * 64 + 32, -1.0, 1.0);
        const double w = engine_uniform(p.seed, g * 64 + 33, -0.1745, 0.1745);
        const double z = engine_uniform(p.seed, g * 64 + 34, -1.0, 1.0);
        blimp_step(p.prm, from, a, w, z, p.steer_dt, end);
        // build-defined Blimp::getPoses (reference stub agents/blimp.hpp:219-223 checks nothing):
        // states after each of max(1, floor(steer_dt / cc_dt)) doStep(cc_dt), end included;
        // R from theta as Blimp::stateToFCLTransform (agents/blimp.hpp:339-356).
        const double qq = p.steer_dt / p.cc_dt;
        unsigned steps = (qq >= 4294967296.0 || !(qq >= 0)) ? 0u : (unsigned)qq;
        if (steps == 0) steps = 1;
        double s[7];
        for (int j = 0; j < 7; ++j) s[j] = from[j];
        // one step of cc_dt == steer_dt is the end state itself (same inputs, same operations):
        // reuse it instead of recomputing its cos / sin / tan
        const bool same = steps == 1 && p.cc_dt == p.steer_dt;
        for (unsigned i = 0; i < steps; ++i) {
            if (same) {
                for (int j = 0; j < 7; ++j) s[j] = end[j];
            } else {
                blimp_step(p.prm, s, a, w, z, p.cc_dt, s);
            }
            double sv, cv;
            cr_sincos(s[3], sv, cv);
            const double R[9] = {cv, sv, 0, -sv, cv, 0, 0, 0, 1};
            if (P < p.pmax) put_pose(ps + 12 * P, R, s[0], s[1], s[2]);
            ++P;
        }
    } else {
        const int T = (int)p.prm[0];
        const double a = engine_uniform(p.seed, g * 64 + 32, -0.1, 1.0);
        const double w = engine_uniform(p.seed, g * 64 + 33, -M_PI / 18., M_PI / 18.);
        snake_step(p.prm, T, from, a, w, p.steer_dt, end);
        // SnakeTrailers::getPoses (agents/snake_trailers.hpp:246-268)
        const double qq = p.steer_dt / p.cc_dt;
        unsigned steps = (qq >= 4294967296.0 || !(qq >= 0)) ? 0u : (unsigned)qq;
        if (steps == 0) steps = 1;
        double s[kMaxDim];
        for (int j = 0; j < d; ++j) s[j] = from[j];
        for (unsigned i = 0; i < steps; ++i) {
            if (P < p.pmax) snake_poses(p.prm, T, s, ps + (int64_t)12 * p.L * P);
            ++P;
            snake_step(p.prm, T, s, a, w, p.cc_dt, s);
        }
    }
    if (P > p.pmax) {
        atomicAdd(counters + 5, 1ull);
        P = p.pmax;
    }
    pcount[k] = P;
    for (int j = 0; j < d; ++j) ends[k * d + j] = end[j];
    return P;
}

// The round's units whose whole-link box (AgentDev bc / be) under the pose meets the env
// root box -- FCL's object-level AABB test before any BVH work; every cluster box lies inside
// its link's box, so the units left out could only be culled by k_pairs' root test anyway.
struct LiveOut {
    int32_t *list;       // [K * pmax * L], or nullptr: no list this round
    uint32_t *n_live;    // zeroed by k_sample
    const AgentDev *links;
    EnvDev env;
    int32_t *q_count;    // the round's QueryOrder counts (read by the NN launch): zeroed here
    int32_t q_nb;
    double *unit_rt;     // [K * pmax * L][12]: each unit's relative transform (CollideWork::unit_rt)
    uint64_t *tmask;     // [K * pmax * L]: each unit's top-level item mask (CollideWork::unit_tmask), or nullptr
};

// the per-unit top-level masks apply: a two-level quantized env tree of at most 64 top items
// (k_pairs' quantized LDS walk)
inline bool tmask_applies(const EnvDev &env) {
    return env.qitems != nullptr && env.n_levels <= 2 && env.lev_off[env.n_levels] - env.lev_off[env.n_levels - 1] <= 64;
}

// randomSteer + getPoses, then the extension's live units appended to the round's list
// (one device atomic per workgroup; the list order does not matter to any verdict).
template <int KIND>
__global__ __launch_bounds__(256) void k_steer(EngineParams p, uint64_t ext_base, int32_t K,
                                               const double *__restrict__ nodes, const int32_t *__restrict__ nn,
                                               double *__restrict__ ends, double *__restrict__ poses,
                                               int32_t *__restrict__ pcount, uint8_t *__restrict__ verdict,
                                               unsigned long long *__restrict__ counters, LiveOut lv) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int32_t P = 0;
    if (k < K) P = steer_one<KIND>(p, ext_base, k, nodes, nn, ends, poses, pcount, verdict, counters);
    if (lv.q_count && k < lv.q_nb) lv.q_count[k * kQCountStride] = 0;  // the NN launch has run: next round's k_sample counts
    if (!lv.list) return;  // kernel argument: uniform
    const int32_t units = p.pmax * p.L;  // <= 64 (the launcher checks)
    uint64_t mask = 0;
    const double *ps = poses + k * units * 12;
    for (int32_t i = 0; i < P; ++i)
        for (int32_t l = 0; l < p.L; ++l) {
            double R[9], T[3];
            unit_transform(lv.env, ps + (i * p.L + l) * 12, R, T);
            double *rt = lv.unit_rt + (k * units + i * p.L + l) * 12;
#pragma unroll
            for (int j = 0; j < 9; ++j) rt[j] = R[j];
#pragma unroll
            for (int j = 0; j < 3; ++j) rt[9 + j] = T[j];
            float blo[3], bhi[3];
            local_box(lv.links[l].bc, lv.links[l].be, R, T, blo, bhi);
            const bool ov = box_overlap(blo, bhi, lv.env.root_lo, lv.env.root_hi);
            if (ov) mask |= 1ull << (i * p.L + l);
            // every unit's mask (a chunked collide walks units off the list too; a unit that
            // misses the root box has no top-level item to meet)
            if (lv.tmask) lv.tmask[k * units + i * p.L + l] = ov ? top_item_mask(lv.env, blo, bhi) : 0ull;
        }
    __shared__ uint32_t s_wave[4];
    __shared__ uint32_t s_base;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t c = (uint32_t)__popcll(mask);
    uint32_t incl = c;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t o = __shfl_up(incl, off);
        if (lane >= off) incl += o;
    }
    if (lane == 63) s_wave[wave] = incl;
    __syncthreads();
    if (threadIdx.x == 0) s_base = atomicAdd(lv.n_live, s_wave[0] + s_wave[1] + s_wave[2] + s_wave[3]);
    __syncthreads();
    uint32_t pos = s_base + incl - c;
    for (int w = 0; w < wave; ++w) pos += s_wave[w];
    while (mask) {
        const int b = __ffsll((unsigned long long)mask) - 1;
        mask &= mask - 1;
        lv.list[pos++] = (int32_t)(k * units + b);
    }
}

// Ordered append and commit in one launch: extension k lands at n0 + (number of valid
// extensions before k).  Each block counts the valid extensions before it straight from the
// verdict bytes (0 / 1, so 16 minus the popcount of every 16-byte load), so no block waits
// on another; the last block also commits n and the counters.  n0 = n_dev[1] (k_sample).
//
// ov (two-phase collide, one chunk): the round's overflowed units (none in practice) are re-run
// here first with the fused walk (k_overflow's work, one wave per unit).  Then no block may
// read a verdict before every re-run has stored its own, and no block may wait for another
// (a spinning block could hold the slot another needs): the blocks take a ticket, all but the
// last one leave, and the last one appends every extension in order itself.  The usual empty
// case costs one load; the k_overflow launch it replaces cost ~5 us a round.
__device__ __forceinline__ void append_commit_tail(int64_t before_block, int32_t blk_ones, const uint8_t *verdict,
                                                   int64_t k0, int32_t K, int32_t d, const double *ends,
                                                   const int32_t *nn, int64_t n0, int64_t cap, double *nodes,
                                                   int32_t *parents, int32_t (&s_wave)[4], int64_t *tot_out) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t k = k0 + tid;
    const bool ok = k < K && verdict[k] == 0;
    const uint64_t m = __ballot(ok);
    if (lane == 0) s_wave[wave] = __popcll(m);
    __syncthreads();
    int wbase = 0;
    for (int w = 0; w < wave; ++w) wbase += s_wave[w];
    if (ok) {
        const int64_t idx = n0 + before_block + wbase + __popcll(m & ((1ull << lane) - 1ull));
        if (idx < cap) {
            // the row loaded whole before any store (clamped, unconditional: one round trip; a
            // run-time-length copy loop waits on each load in turn)
            double v[kMaxDim];
#pragma unroll
            for (int j = 0; j < kMaxDim; ++j) v[j] = ends[k * d + (j < d ? j : d - 1)];
#pragma unroll
            for (int j = 0; j < kMaxDim; ++j)
                if (j < d) nodes[idx * d + j] = v[j];
            parents[idx] = nn[k];
        }
    }
    *tot_out = before_block + s_wave[0] + s_wave[1] + s_wave[2] + s_wave[3];
    (void)blk_ones;
}

__device__ __forceinline__ void append_commit_counters(int64_t tot, int64_t n0, int64_t cap, int32_t K,
                                                       int64_t *n_dev, unsigned long long *counters) {
    const int64_t room = cap - n0 > 0 ? cap - n0 : 0;
    const int64_t add = tot < room ? tot : room;
    n_dev[0] = n0 + add;
    counters[0] += 1;
    counters[1] += (unsigned long long)K;
    counters[2] += (unsigned long long)add;
    counters[3] = (unsigned long long)(n0 + add);
    counters[4] += (unsigned long long)(tot - add);
}

__global__ __launch_bounds__(256) void k_append_commit(const uint8_t *__restrict__ verdict, int32_t K, int32_t d,
                                                       const double *__restrict__ ends,
                                                       const int32_t *__restrict__ nn, int64_t *__restrict__ n_dev,
                                                       int64_t cap, double *__restrict__ nodes,
                                                       int32_t *__restrict__ parents,
                                                       unsigned long long *__restrict__ counters, OvfDefer ov,
                                                       uint32_t *__restrict__ ticket) {
    __shared__ int32_t s_wave[4], s_ones[4];
    __shared__ int32_t s_last;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (ov.n_ovf) {
        const uint32_t n_ovf = __hip_atomic_load(ov.n_ovf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (n_ovf > 0) {  // grid-uniform
            __shared__ int32_t s_stk[4][kStackDepth];
            const bool shared_edges = ov.w.pose_edge != nullptr || ov.w.L > 1 || ov.w.pmax > 1;
            uint32_t nu = 0, nc = 0, nnod = 0, ns = 0;
            const uint32_t nw = gridDim.x * 4;
            for (uint32_t i = blockIdx.x * 4 + wave; i < n_ovf; i += nw)
                collide_unit(ov.env, ov.env.nodes, ov.env.n_nodes, ov.links, ov.w, ov.ovf_list[i], s_stk[wave], lane,
                             shared_edges, nc, nnod, ns, nu);
            __threadfence();
            __syncthreads();
            if (tid == 0) s_last = atomicAdd(ticket, 1u) == gridDim.x - 1;
            __syncthreads();
            if (!s_last) return;  // block-uniform
            __threadfence();
            // the last block: every extension, in order, with a running count
            const int64_t n0 = n_dev[1];
            int64_t before = 0;
            for (int64_t k0 = 0; k0 < K; k0 += 256) {
                int64_t tot;
                append_commit_tail(before, 0, verdict, k0, K, d, ends, nn, n0, cap, nodes, parents, s_wave, &tot);
                before = tot;
                __syncthreads();  // s_wave is reused
            }
            if (tid == 0) {
                append_commit_counters(before, n0, cap, K, n_dev, counters);
                *ticket = 0u;  // for the next round's launch (stream-ordered)
            }
            return;
        }
    }
    const uint4 *v4 = reinterpret_cast<const uint4 *>(verdict);
    const int64_t nv4 = (int64_t)blockIdx.x * 16;  // 256 verdicts per block before this one
    int32_t ones = 0;
    // eight 16-B loads in flight per thread (clamped, unconditional), not one round trip each
    for (int64_t i0 = tid; i0 < nv4; i0 += 256 * 8) {
        uint4 x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int64_t i = i0 + u * 256;
            x[u] = v4[i < nv4 ? i : 0];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (i0 + u * 256 < nv4) ones += __popc(x[u].x) + __popc(x[u].y) + __popc(x[u].z) + __popc(x[u].w);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) ones += __shfl_xor(ones, off);
    if (lane == 0) s_ones[wave] = ones;
    __syncthreads();
    const int64_t before_block = nv4 * 16 - (int64_t)(s_ones[0] + s_ones[1] + s_ones[2] + s_ones[3]);
    const int64_t n0 = n_dev[1];
    int64_t tot;
    append_commit_tail(before_block, 0, verdict, (int64_t)blockIdx.x * 256, K, d, ends, nn, n0, cap, nodes, parents,
                       s_wave, &tot);
    if (blockIdx.x == gridDim.x - 1 && tid == 0) append_commit_counters(tot, n0, cap, K, n_dev, counters);
}

__global__ void k_set_n(int64_t *n_dev, int64_t n, unsigned long long *counters) {
    *n_dev = n;
    counters[3] = (unsigned long long)n;
}

// ---- joint rounds (mpt_rrt_step_many): every engine's round in one launch per stage ----
//
// Engines that share the env, the agent links, the agent kind and the pose layout, and whose
// rounds all use the Morton tree, run a round as one launch per stage on the joint stream:
// sample -> incremental tree build -> NN -> steer -> collide (over every engine's units) ->
// ordered append, each launch's blockIdx.y (or its unit range) naming the engine.  The round
// buffers (samples, ends, poses, verdicts, live units) are the joint state's, engine j at
// offset j * K.  An engine's randomness, NN, steering and append are its own (per-engine
// seed, extension counter, nodes, count), so every tree equals the one the engine grows alone.
struct EngineJob {
    uint64_t seed, ext_base;
    int64_t set_n;  // a pending mpt_rrt_set_size, or -1
    int64_t cap;
    double *nodes;
    int32_t *parents;
    int64_t *n_dev;
    unsigned long long *counters;
};

__global__ void k_sample_jobs(EngineParams p, const EngineJob *__restrict__ jobs, int32_t K,
                              double *__restrict__ samples, uint32_t *__restrict__ n_live, int32_t n_sub) {
    const int job = blockIdx.y;
    const EngineJob &J = jobs[job];
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k == 0) {
        if (J.set_n >= 0) {
            J.n_dev[0] = J.set_n;
            J.counters[3] = (unsigned long long)J.set_n;
        }
        J.n_dev[1] = J.n_dev[0];
        if (job == 0)
            for (int b = 0; b < n_sub; ++b) n_live[b] = 0u;  // the live-unit lists of this round
    }
    if (k >= K) return;
    const uint64_t g = J.ext_base + (uint64_t)k;
    double *out = samples + ((int64_t)job * K + k) * p.d;
    for (int j = 0; j < p.d; ++j) out[j] = engine_uniform(J.seed, g * 64 + j, p.lo[j], p.hi[j]);
}

// k_steer for engine blockIdx.y: its extensions are joint edges job * K + k; the live units go
// to the list of the engine's collide sub-batch (engines [b * per_sub, + per_sub)), indexed
// from that sub-batch's first unit
template <int KIND>
__global__ __launch_bounds__(256) void k_steer_jobs(EngineParams p, const EngineJob *__restrict__ jobs, int32_t K,
                                                    const int32_t *__restrict__ nn, double *__restrict__ ends,
                                                    double *__restrict__ poses, int32_t *__restrict__ pcount,
                                                    uint8_t *__restrict__ verdict, LiveOut lv, int32_t per_sub) {
    const int job = blockIdx.y;
    const EngineJob &J = jobs[job];
    p.seed = J.seed;
    const int32_t units = p.pmax * p.L;  // <= 64 (the launcher checks)
    const int64_t e0 = (int64_t)job * K;  // this engine's first joint edge
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int32_t P = 0;
    if (k < K)
        P = steer_one<KIND>(p, J.ext_base, k, J.nodes, nn + e0, ends + e0 * p.d, poses + e0 * units * 12, pcount + e0,
                            verdict + e0, J.counters);
    const int sub = job / per_sub;
    const int64_t sub_e0 = (int64_t)sub * per_sub * K;  // the sub-batch's first edge
    int32_t *list = lv.list + sub_e0 * units;
    uint64_t mask = 0;
    const int64_t ge = e0 + k;  // joint edge
    const double *ps = poses + ge * units * 12;
    for (int32_t i = 0; i < P; ++i)
        for (int32_t l = 0; l < p.L; ++l) {
            double R[9], T[3];
            unit_transform(lv.env, ps + (i * p.L + l) * 12, R, T);
            double *rt = lv.unit_rt + (ge * units + i * p.L + l) * 12;
#pragma unroll
            for (int j = 0; j < 9; ++j) rt[j] = R[j];
#pragma unroll
            for (int j = 0; j < 3; ++j) rt[9 + j] = T[j];
            float blo[3], bhi[3];
            local_box(lv.links[l].bc, lv.links[l].be, R, T, blo, bhi);
            const bool ov = box_overlap(blo, bhi, lv.env.root_lo, lv.env.root_hi);
            if (ov) mask |= 1ull << (i * p.L + l);
            // every unit's mask (a chunked collide walks units off the list too; a unit that
            // misses the root box has no top-level item to meet)
            if (lv.tmask) lv.tmask[ge * units + i * p.L + l] = ov ? top_item_mask(lv.env, blo, bhi) : 0ull;
        }
    __shared__ uint32_t s_wave[4];
    __shared__ uint32_t s_base;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t c = (uint32_t)__popcll(mask);
    uint32_t incl = c;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t o = __shfl_up(incl, off);
        if (lane >= off) incl += o;
    }
    if (lane == 63) s_wave[wave] = incl;
    __syncthreads();
    if (threadIdx.x == 0) s_base = atomicAdd(lv.n_live + sub, s_wave[0] + s_wave[1] + s_wave[2] + s_wave[3]);
    __syncthreads();
    uint32_t pos = s_base + incl - c;
    for (int w = 0; w < wave; ++w) pos += s_wave[w];
    const int64_t local_u0 = (ge - sub_e0) * units;
    while (mask) {
        const int b = __ffsll((unsigned long long)mask) - 1;
        mask &= mask - 1;
        list[pos++] = (int32_t)(local_u0 + b);
    }
}

// k_append_commit for engine blockIdx.y over its K joint verdicts
// kOvf: ov / ticket carry the joint collide's deferred overflow re-run, as k_append_commit
// takes it (the last block then appends every engine's extensions in order).  The fused walk's
// registers cost the kernel its occupancy (a 256-seed round's append 49 -> 63 us), so only
// small joint rounds, whose append is a few latency-bound waves, take it (the launch it saves
// is ~5 us); larger ones keep the k_overflow launch.
template <bool kOvf>
__global__ __launch_bounds__(256) void k_append_jobs(const EngineJob *__restrict__ jobs,
                                                     const uint8_t *__restrict__ verdict, int32_t K, int32_t d,
                                                     const double *__restrict__ ends, const int32_t *__restrict__ nn,
                                                     OvfDefer ov, uint32_t *__restrict__ ticket) {
    __shared__ int32_t s_wave[4], s_ones[4];
    __shared__ int32_t s_last;
    const int job = blockIdx.y;
    const EngineJob &J = jobs[job];
    const int64_t e0 = (int64_t)job * K;
    const uint8_t *vj = verdict + e0;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (kOvf && ov.n_ovf) {
        const uint32_t n_ovf = __hip_atomic_load(ov.n_ovf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (n_ovf > 0) {  // grid-uniform
            __shared__ int32_t s_stk[4][kStackDepth];
            const bool shared_edges = ov.w.pose_edge != nullptr || ov.w.L > 1 || ov.w.pmax > 1;
            uint32_t nu = 0, nc = 0, nnod = 0, ns = 0;
            const uint32_t nblk = gridDim.x * gridDim.y, blk = blockIdx.y * gridDim.x + blockIdx.x;
            for (uint32_t i = blk * 4 + wave; i < n_ovf; i += nblk * 4)
                collide_unit(ov.env, ov.env.nodes, ov.env.n_nodes, ov.links, ov.w, ov.ovf_list[i], s_stk[wave], lane,
                             shared_edges, nc, nnod, ns, nu);
            __threadfence();
            __syncthreads();
            if (tid == 0) s_last = atomicAdd(ticket, 1u) == nblk - 1;
            __syncthreads();
            if (!s_last) return;  // block-uniform
            __threadfence();
            for (int32_t j = 0; j < (int32_t)gridDim.y; ++j) {  // every engine, every extension, in order
                const EngineJob &Jj = jobs[j];
                const int64_t n0 = Jj.n_dev[1];
                int64_t before = 0;
                for (int64_t k0 = 0; k0 < K; k0 += 256) {
                    int64_t tot;
                    append_commit_tail(before, 0, verdict + (int64_t)j * K, k0, K, d, ends + (int64_t)j * K * d,
                                       nn + (int64_t)j * K, n0, Jj.cap, Jj.nodes, Jj.parents, s_wave, &tot);
                    before = tot;
                    __syncthreads();  // s_wave is reused
                }
                if (tid == 0) append_commit_counters(before, n0, Jj.cap, K, Jj.n_dev, Jj.counters);
            }
            if (tid == 0) *ticket = 0u;  // for the next round's launch (stream-ordered)
            return;
        }
    }
    // the engine's valid extensions before this block (K is a multiple of 16: the launcher checks)
    const uint4 *v4 = reinterpret_cast<const uint4 *>(vj);
    const int64_t nv4 = (int64_t)blockIdx.x * 16;
    int32_t ones = 0;
    for (int64_t i0 = tid; i0 < nv4; i0 += 256 * 8) {
        uint4 x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int64_t i = i0 + u * 256;
            x[u] = v4[i < nv4 ? i : 0];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (i0 + u * 256 < nv4) ones += __popc(x[u].x) + __popc(x[u].y) + __popc(x[u].z) + __popc(x[u].w);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) ones += __shfl_xor(ones, off);
    if (lane == 0) s_ones[wave] = ones;
    __syncthreads();
    const int64_t before_block = nv4 * 16 - (int64_t)(s_ones[0] + s_ones[1] + s_ones[2] + s_ones[3]);
    const int64_t n0 = J.n_dev[1];
    int64_t tot;
    append_commit_tail(before_block, 0, vj, (int64_t)blockIdx.x * 256, K, d, ends + e0 * d, nn + e0, n0, J.cap,
                       J.nodes, J.parents, s_wave, &tot);
    if (blockIdx.x == gridDim.x - 1 && tid == 0) append_commit_counters(tot, n0, J.cap, K, J.n_dev, J.counters);
}

}  // namespace

struct mpt_rrt {
    EngineParams p{};
    EnvDev env{};
    AgentDev *d_links = nullptr;
    int64_t cap = 0;
    int64_t n_upper = 0;  // host-side upper bound of the device node count
    double *d_nodes = nullptr;
    int32_t *d_parents = nullptr;
    int64_t *d_n = nullptr;
    unsigned long long *d_counters = nullptr;
    int32_t kcap = 0;
    double *d_samples = nullptr, *d_ends = nullptr, *d_poses = nullptr, *d_nnd2 = nullptr;
    int32_t *d_nn = nullptr, *d_pcount = nullptr;
    int32_t *d_live = nullptr;     // k_steer's live-unit list [K * pmax * L] (two-phase collide)
    uint64_t *d_tmask = nullptr;   // k_steer's per-unit top-level item masks [K * pmax * L]
    double *d_rt = nullptr;        // k_steer's unit relative transforms [K * pmax * L][12] (two-phase)
    uint32_t *d_nlive = nullptr;   // its length
    uint8_t *d_verdict = nullptr;
    uint32_t *d_bar = nullptr;  // k_append_commit's ticket (overflow re-run)
    void *d_scratch = nullptr;
    size_t scratch_bytes = 0;
    uint64_t ext_base = 0;
    int32_t last_K = 0;
    bool timing = false;
    // stage timing: a ring of per-round event sets, so timed rounds need no host sync; the
    // oldest set is folded into acc_ms only when the ring wraps (it completed long before)
    std::vector<hipEvent_t> ring;  // [kTimingRing][10]
    int64_t ring_next = 0, ring_done = 0, acc_rounds = 0;
    double acc_ms[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    float last_ms[6] = {0, 0, 0, 0, 0, 0};
    // NN structure over the round's snapshot (grid_nn.hip), rebuilt every round
    int32_t nn_mode = MPT_NN_AUTO;
    std::unique_ptr<GridIndex> grid;
    std::unique_ptr<CellTree> ctree;  // MPT_NN_TREE (cell_tree.hip)
    int32_t grid_gd = 0, grid_dims[3] = {0, 0, 0};
    double ppc = 0.0;  // grid points per cell; <= 0: 2, floored by the expected NN distance
    // MPT_NN_AUTO feedback: the live nodes' spatial spread, a by-product of the round's index
    // build (SpreadOut, grid_nn.h) written to mapped host memory and read at a later round once
    // its event has completed (never waited for; the NN choice changes only speed, results
    // are identical).  d_spread: the grid build's per-block partials.
    unsigned long long *d_spread = nullptr, *h_spread = nullptr, *h_spread_dev = nullptr;
    hipEvent_t ev_spread = nullptr;
    bool spread_pending = false, auto_tree = false, spread_seen = false;
    int32_t rounds_since_spread = 0;
    int32_t last_nn = -1;  // structure the last round used (mpt_rrt_last_nn)
    // optional collision work counters (k_collide atomics): units, clusters, node visits, tri tests
    bool stats_on = false;
    CollideScratch cscratch;
    int32_t max_clusters = 1;
    unsigned long long *d_cstats = nullptr;
    // grid rounds: the samples bucketed along the grid's first dim (QueryOrder, grid_nn.h)
    int32_t *d_qcount = nullptr, *d_qlist = nullptr;
    int32_t q_cap = 0;
    // mpt_rrt_set_size's node count, applied by the next round's k_sample (or by flush_size
    // before the host reads the count); -1: none
    int64_t pending_n = -1;
    // incremental Morton tree (point_tree.h prepare_inc): valid while nodes are only appended
    // since its last build; pt_grow bounds the nodes appended since then (the K of each round)
    bool pt_inc_ok = false;
    int64_t pt_grow = 0;
    const mpt_agent *agent = nullptr;
    // the last round ran in a joint round of mpt_rrt_step_many: its round buffers are the
    // joint state's slices (valid until the next step_many on that joint stream)
    bool last_joint = false;
    struct {
        const double *samples = nullptr, *ends = nullptr, *poses = nullptr;
        const int32_t *nn = nullptr, *pcount = nullptr;
        const uint8_t *verdict = nullptr;
    } jv;
    // the joint stream and the id of its round buffers the slices point into (a release or a
    // reallocation of those buffers changes the id: last_round / last_poses then refuse)
    hipStream_t jv_stream = nullptr;
    uint64_t jv_id = 0;
};

namespace {
// Mapped pinned slots for the engines' spread words (6 u64 each), carved from shared chunks:
// one hipHostMalloc per 1024 engines instead of one per engine (config 5 starts 256 engines in
// its first round; each pinned allocation costs far more than a round of kernels)
struct PinnedSlots {
    std::mutex mu;
    std::vector<unsigned long long *> free_slots;
    static constexpr int kSlotWords = 8, kSlots = 1024;
    void take(unsigned long long **host, unsigned long long **dev) {
        std::lock_guard<std::mutex> lk(mu);
        if (free_slots.empty()) {
            unsigned long long *chunk = nullptr;
            hip_check(hipHostMalloc(&chunk, sizeof(unsigned long long) * kSlotWords * kSlots,
                                    hipHostMallocMapped | hipHostMallocCoherent), "alloc spread slots");
            for (int i = kSlots - 1; i >= 0; --i) free_slots.push_back(chunk + (size_t)i * kSlotWords);
        }
        *host = free_slots.back();
        free_slots.pop_back();
        hip_check(hipHostGetDevicePointer(reinterpret_cast<void **>(dev), *host, 0), "spread device pointer");
    }
    void give(unsigned long long *host) {
        std::lock_guard<std::mutex> lk(mu);
        free_slots.push_back(host);
    }
};
PinnedSlots &pinned_slots() {
    static PinnedSlots *p = new PinnedSlots();  // never freed: engines may outlive static destruction order
    return *p;
}

}  // namespace

namespace {
void rfree(mpt_rrt *r) {
    void *ps[] = {r->d_links, r->d_nodes,   r->d_parents, r->d_n,       r->d_counters, r->d_samples,
                  r->d_ends,  r->d_poses,   r->d_nnd2,    r->d_nn,      r->d_pcount,
                  r->d_verdict, r->d_scratch, r->d_cstats, r->d_live, r->d_nlive, r->d_rt, r->d_bar, r->d_tmask};
    for (void *p : ps)
        if (p) (void)hipFree(p);
    for (auto &e : r->ring)
        if (e) (void)hipEventDestroy(e);
    if (r->d_spread) (void)hipFree(r->d_spread);
    if (r->d_qcount) (void)hipFree(r->d_qcount);
    if (r->d_qlist) (void)hipFree(r->d_qlist);
    if (r->h_spread) pinned_slots().give(r->h_spread);
    if (r->ev_spread) (void)hipEventDestroy(r->ev_spread);
}

constexpr int kTimingRing = 64;

// fold the oldest recorded round's stage times into acc_ms
void timing_fold_one(mpt_rrt *r) {
    hipEvent_t *e = r->ring.data() + (r->ring_done % kTimingRing) * 10;
    hip_check(hipEventSynchronize(e[9]), "event sync");
    for (int i = 0; i < 9; ++i) {
        float ms = 0.f;
        hip_check(hipEventElapsedTime(&ms, e[i], e[i + 1]), "elapsed");
        r->acc_ms[i] += ms;
    }
    ++r->acc_rounds;
    ++r->ring_done;
}

void ensure_round_buffers(mpt_rrt *r, int32_t K) {
    const size_t need_scratch = nn_knn_scratch_bytes(K, std::max<int64_t>(r->cap, 1), 1);
    if (K > r->kcap) {
        void *ps[] = {r->d_samples, r->d_ends, r->d_poses, r->d_nnd2, r->d_nn, r->d_pcount, r->d_verdict, r->d_live,
                      r->d_rt, r->d_tmask};
        for (void *p : ps)
            if (p) hip_check(hipFree(p), "hipFree");
        const int64_t d = r->p.d;
        hip_check(hipMalloc(&r->d_samples, sizeof(double) * K * d), "alloc samples");
        hip_check(hipMalloc(&r->d_ends, sizeof(double) * K * d), "alloc ends");
        hip_check(hipMalloc(&r->d_poses, sizeof(double) * 12 * (int64_t)K * r->p.pmax * r->p.L), "alloc poses");
        hip_check(hipMalloc(&r->d_nnd2, sizeof(double) * K), "alloc nnd2");
        hip_check(hipMalloc(&r->d_nn, sizeof(int32_t) * K), "alloc nn");
        hip_check(hipMalloc(&r->d_pcount, sizeof(int32_t) * K), "alloc pcount");
        hip_check(hipMalloc(&r->d_verdict, (size_t)K), "alloc verdict");
        hip_check(hipMalloc(&r->d_live, sizeof(int32_t) * (int64_t)K * r->p.pmax * r->p.L), "alloc live units");
        hip_check(hipMalloc(&r->d_rt, sizeof(double) * 12 * (int64_t)K * r->p.pmax * r->p.L), "alloc unit transforms");
        hip_check(hipMalloc(&r->d_tmask, sizeof(uint64_t) * (int64_t)K * r->p.pmax * r->p.L), "alloc unit masks");
        if (!r->d_nlive) hip_check(hipMalloc(&r->d_nlive, sizeof(uint32_t)), "alloc live count");
        r->kcap = K;
        r->cscratch.ensure((int64_t)K * r->p.pmax * r->p.L, r->max_clusters);
    }
    // the split count depends on n, so size the NN scratch for the capacity bound
    if (need_scratch > r->scratch_bytes) {
        if (r->d_scratch) hip_check(hipFree(r->d_scratch), "hipFree");
        hip_check(hipMalloc(&r->d_scratch, need_scratch), "alloc nn scratch");
        r->scratch_bytes = need_scratch;
    }
}
}  // namespace

extern "C" mpt_status mpt_rrt_create(const mpt_env *env, const mpt_agent *agent, int32_t agent_kind,
                                     const double prm[7], const double *ranges, int32_t dim, double steer_dt,
                                     double cc_dt, int64_t capacity, uint64_t seed, mpt_rrt **out) {
    return guarded([&] {
        if (!env || !agent || !out || !ranges) throw Error{MPT_ERR_INVALID, "null pointer"};
        if (agent_kind < 0 || agent_kind > 2) throw Error{MPT_ERR_INVALID, "unknown agent kind"};
        if (capacity < 1 || capacity >= (int64_t(1) << 31) - 1) throw Error{MPT_ERR_INVALID, "bad capacity"};
        if (!(cc_dt > 0) || !(steer_dt > 0)) throw Error{MPT_ERR_INVALID, "dt must be > 0"};
        auto *r = new mpt_rrt();
        try {
            EngineParams &p = r->p;
            p.kind = agent_kind;
            p.d = dim;
            p.seed = seed;
            p.steer_dt = steer_dt;
            p.cc_dt = cc_dt;
            if (prm) std::memcpy(p.prm, prm, sizeof(p.prm));
            int expect = 3;
            if (agent_kind == MPT_AGENT_BLIMP) expect = 7;
            if (agent_kind == MPT_AGENT_SNAKE) {
                if (!prm || prm[0] < 0 || prm[0] > kMaxDim - 5) throw Error{MPT_ERR_INVALID, "bad trailer count"};
                expect = 5 + (int)prm[0];
            }
            if (dim != expect) throw Error{MPT_ERR_INVALID, "dim does not match the agent's tree state size"};
            for (int j = 0; j < dim; ++j) {
                p.lo[j] = ranges[2 * j];
                p.hi[j] = ranges[2 * j + 1];
            }
            p.L = agent_kind == MPT_AGENT_SNAKE ? (int)prm[0] + 1 : 1;
            if (agent_kind == MPT_AGENT_OMNI) {
                // |end - start| = 1 up to rounding: floor(1/dt) poses + the end pose (+1 slack)
                p.pmax = (int32_t)(1.0 / cc_dt) + 3;
            } else {
                const double qq = steer_dt / cc_dt;
                p.pmax = qq >= 1 ? (int32_t)qq : 1;
            }
            if ((int64_t)p.pmax * p.L > 4096) throw Error{MPT_ERR_INVALID, "too many poses per edge"};
            r->env = env_dev(env);
            r->agent = agent;
            std::vector<AgentDev> links(p.L, agent_dev(agent));
            r->max_clusters = std::max(1, agent_dev(agent).n_clusters);
            hip_check(hipMalloc(&r->d_links, sizeof(AgentDev) * p.L), "alloc links");
            hip_check(hipMemcpy(r->d_links, links.data(), sizeof(AgentDev) * p.L, hipMemcpyHostToDevice), "links");
            r->cap = capacity;
            hip_check(hipMalloc(&r->d_nodes, sizeof(double) * dim * capacity), "alloc nodes");
            hip_check(hipMalloc(&r->d_parents, sizeof(int32_t) * capacity), "alloc parents");
            hip_check(hipMalloc(&r->d_n, 2 * sizeof(int64_t)), "alloc n");  // [0] n, [1] round start
            hip_check(hipMemset(r->d_n, 0, 2 * sizeof(int64_t)), "memset n");
            hip_check(hipMalloc(&r->d_counters, sizeof(unsigned long long) * 8), "alloc counters");
            hip_check(hipMemset(r->d_counters, 0, sizeof(unsigned long long) * 8), "memset counters");
            r->grid.reset(new GridIndex());
            r->ctree.reset(new CellTree());
            r->grid_gd = agent_kind == MPT_AGENT_SNAKE ? 2 : 3;
            for (int j = 0; j < 3; ++j) r->grid_dims[j] = j;
        } catch (...) {
            rfree(r);
            delete r;
            throw;
        }
        *out = r;
    });
}

extern "C" mpt_status mpt_rrt_destroy(mpt_rrt *r) {
    return guarded([&] {
        if (!r) return;
        (void)hipDeviceSynchronize();
        rfree(r);
        delete r;
    });
}

namespace {
// apply a pending mpt_rrt_set_size before the host reads the node count or the counters
void flush_size(mpt_rrt *r) {
    hip_check(hipDeviceSynchronize(), "sync");
    if (r->pending_n >= 0) {
        hipLaunchKernelGGL(k_set_n, dim3(1), dim3(1), 0, 0, r->d_n, r->pending_n, r->d_counters);
        hip_check(hipGetLastError(), "k_set_n");
        hip_check(hipDeviceSynchronize(), "sync");
        r->pending_n = -1;
    }
}
}  // namespace

extern "C" mpt_status mpt_rrt_add_nodes(mpt_rrt *r, const double *states, const int32_t *parents, int64_t n) {
    return guarded([&] {
        if (!r || n < 0 || (n > 0 && !states)) throw Error{MPT_ERR_INVALID, "bad arguments"};
        flush_size(r);
        int64_t cur = 0;
        hip_check(hipMemcpy(&cur, r->d_n, sizeof(int64_t), hipMemcpyDeviceToHost), "n D2H");
        if (cur + n > r->cap) throw Error{MPT_ERR_CAPACITY, "tree capacity exceeded"};
        const int d = r->p.d;
        if (n > 0) {
            hip_check(hipMemcpy(r->d_nodes + cur * d, states, sizeof(double) * d * n, hipMemcpyHostToDevice), "nodes");
            std::vector<int32_t> par(n, 0);
            if (parents) std::memcpy(par.data(), parents, sizeof(int32_t) * n);
            hip_check(hipMemcpy(r->d_parents + cur, par.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice), "par");
        }
        const int64_t nn = cur + n;
        hipLaunchKernelGGL(k_set_n, dim3(1), dim3(1), 0, 0, r->d_n, nn, r->d_counters);
        hip_check(hipGetLastError(), "k_set_n");
        hip_check(hipDeviceSynchronize(), "sync");
        r->n_upper = nn;
        r->pt_inc_ok = false;
        if (cur == 0 && n > 0) {
            // the first nodes: MPT_NN_AUTO's spread from the host copy, so the first indexed
            // round already uses the right structure (a tree grown from one root would
            // otherwise run one grid round over a clustered tree with samples over the whole
            // box before the device spread came back)
            double frac = 1.0;
            for (int j = 0; j < r->grid_gd; ++j) {
                const int dj = r->grid_dims[j];
                double lo = states[dj], hi = states[dj];
                for (int64_t i = 1; i < n; ++i) {
                    lo = std::min(lo, states[i * d + dj]);
                    hi = std::max(hi, states[i * d + dj]);
                }
                const double range = r->p.hi[dj] - r->p.lo[dj];
                frac *= range > 0 ? std::min(1.0, std::max(0.0, (hi - lo) / range)) : 1.0;
            }
            r->auto_tree = frac < kAutoTreeFrac;
            r->spread_seen = true;
            r->spread_pending = false;
            r->rounds_since_spread = 0;
        } else {
            r->spread_seen = false;  // bulk nodes: re-read the spread at the next index build
        }
    });
}

extern "C" mpt_status mpt_rrt_set_size(mpt_rrt *r, int64_t n, void *stream) {
    return guarded([&] {
        if (!r || n < 0 || n > r->cap) throw Error{MPT_ERR_INVALID, "bad size"};
        if (n > r->n_upper) throw Error{MPT_ERR_INVALID, "set_size can only truncate"};
        // applied by the next round's k_sample on its stream (no launch of its own: a round
        // trip of one small kernel per reset in the bench's timed loop), or by flush_size
        (void)stream;
        r->pending_n = n;
        r->n_upper = n;
        r->pt_inc_ok = false;  // the index may hold truncated nodes
    });
}

namespace {

// One round is three phases so that many engines can share the NN launch (mpt_rrt_step_many):
// head = sample + NN index build, nn = the NN query, tail = steer, collide, append.
struct StepCtx {
    hipEvent_t *ev = nullptr;  // this round's timing events (engine timing on) or null
    unsigned kb = 0;
    bool use_tree = false, use_grid = false, live_list = false;
    bool defer_tree = false, want_spread = false;  // tree build left to the caller (step_many)
    SpreadOut spread{};
    QueryOrder qo{};  // qo.list: this round's samples are bucketed (sorted grid 1-NN)
    void mark(int i, hipStream_t stream) const {
        if (ev) hip_check(hipEventRecord(ev[i], stream), "event record");
    }
};

// this round's incremental tree build (a full rebuild when the index is stale or more nodes
// were appended since its last build than one round's merge takes: the host's bound, which the
// build's first kernel checks on the device into counters[6])
// does this round's tree_inc_job launch a full rebuild (CellTree::prepare: a full build, or a
// new code plan, of more than kCtSeg rows; fewer restart the index inside launch_ct_jobs)?
bool tree_inc_launches(const mpt_rrt *r) {
    const bool full = !r->pt_inc_ok || r->pt_grow > kCtSeg || !r->ctree->plan_current(r->p.lo, r->p.hi);
    return full && r->n_upper > kCtSeg;
}

CtJob tree_inc_job(mpt_rrt *r, hipStream_t stream, const SpreadOut *spread) {
    const bool full = !r->pt_inc_ok || r->pt_grow > kCtSeg;
    CtJob J = r->ctree->prepare(r->d_nodes, r->n_upper, r->d_n, r->p.d, r->p.lo, r->p.hi, r->grid_gd, full,
                                r->pt_grow, stream, spread, r->d_counters + 6);
    r->pt_inc_ok = true;
    r->pt_grow = 0;
    return J;
}

// MPT_NN_AUTO: take up the spread a past round's index build left (never waited for)
void refresh_auto(mpt_rrt *r) {
    const EngineParams &p = r->p;
    if (r->nn_mode == MPT_NN_AUTO && r->spread_pending && hipEventQuery(r->ev_spread) == hipSuccess) {
        // the tree fills less than a quarter of the sampling box: most samples are far
        // from every node, where the grid walks empty rings and the Morton tree does not
        double frac = 1.0;
        for (int j = 0; j < r->grid_gd; ++j) {
            const int dj = r->grid_dims[j];
            const double ext = key_value_u64(r->h_spread[3 + j]) - key_value_u64(r->h_spread[j]);
            const double range = p.hi[dj] - p.lo[dj];
            frac *= range > 0 ? std::min(1.0, std::max(0.0, ext / range)) : 1.0;
        }
        r->auto_tree = frac < kAutoTreeFrac;
        r->spread_pending = false;
        r->spread_seen = true;
    }
}

bool round_uses_tree(const mpt_rrt *r) {
    const bool big = r->n_upper >= 4096;
    return r->nn_mode == MPT_NN_TREE || (r->nn_mode == MPT_NN_AUTO && big && r->auto_tree);
}

// a joint round indexes every engine's tree in the cell tree whatever its size: a young tree
// (<= kCtSeg nodes) starts from an empty index inside the joint build, so a planner run from
// its start states is joint from its first round (no per-engine brute-force rounds, no
// per-engine scratch, no per-seed full rebuilds)
bool joint_uses_tree(const mpt_rrt *r) {
    return r->nn_mode == MPT_NN_TREE || (r->nn_mode == MPT_NN_AUTO && r->auto_tree);
}

// the spread feedback rides on this round's index build when none is in flight; true when
// this round's build should write it (spread filled in)
bool spread_request(mpt_rrt *r, bool indexed, SpreadOut &spread) {
    const bool want = r->nn_mode == MPT_NN_AUTO && !r->spread_pending && indexed &&
                      (!r->spread_seen || r->rounds_since_spread >= kSpreadEvery);
    ++r->rounds_since_spread;
    if (!want) return false;
    if (!r->h_spread) {
        pinned_slots().take(&r->h_spread, &r->h_spread_dev);
        hip_check(hipEventCreateWithFlags(&r->ev_spread, hipEventDisableTiming), "event");
    }
    spread.gd = r->grid_gd;
    for (int j = 0; j < 3; ++j) spread.dims[j] = r->grid_dims[j];
    spread.partial = r->d_spread;  // the grid build's per-block partials (step_head allocates them)
    spread.host_out = r->h_spread_dev;
    return true;
}

StepCtx step_head(mpt_rrt *r, int32_t K, hipStream_t stream, bool defer_tree = false) {
    StepCtx c;
    if (r->n_upper < 1) throw Error{MPT_ERR_INVALID, "tree is empty: add a root first"};
    ensure_round_buffers(r, K);
    r->last_joint = false;
    const EngineParams &p = r->p;
    const unsigned kb = (unsigned)((K + 255) / 256);
    hipEvent_t *ev = nullptr;
    if (r->timing) {
        if (r->ring_next - r->ring_done >= kTimingRing) timing_fold_one(r);
        ev = r->ring.data() + (r->ring_next % kTimingRing) * 10;
        ++r->ring_next;
    }
    c.ev = ev;
    c.kb = kb;
    refresh_auto(r);
    const bool big = r->n_upper >= 4096;
    const bool use_tree = round_uses_tree(r);
    const bool use_grid = !use_tree && (r->nn_mode == MPT_NN_GRID || (r->nn_mode == MPT_NN_AUTO && big));
    r->last_nn = use_tree ? MPT_NN_TREE : (use_grid ? MPT_NN_GRID : MPT_NN_BRUTE);
    c.mark(0, stream);
    // k_steer lists the live units for the two-phase collide (FCL's object-level AABB test)
    const bool live_list = collide_mode() != MPT_COLLIDE_FUSED && p.pmax * p.L <= 64;
    // grid rounds: the index build also buckets the samples along the grid's first dim, so the
    // 1-NN launch can deal them to the XCDs by x-slab
    if (use_grid && (p.d == 3 || p.d == 7 || p.d == 15)) {
        if (r->q_cap < K) {
            if (r->d_qlist) hip_check(hipFree(r->d_qlist), "hipFree");
            hip_check(hipMalloc(&r->d_qlist, sizeof(int32_t) * (size_t)kQueryBuckets * K), "alloc query lists");
            r->q_cap = K;
        }
        if (!r->d_qcount) {
            const size_t qc_bytes = sizeof(int32_t) * kQueryBuckets * kQCountStride;
            hip_check(hipMalloc(&r->d_qcount, qc_bytes), "alloc query counts");
            hip_check(hipMemset(r->d_qcount, 0, qc_bytes), "zero query counts");
            // the null-stream memset is not ordered with the engine's stream
            hip_check(hipDeviceSynchronize(), "query counts zero sync");
        }
        const int dj = r->grid_dims[0];
        const double span = p.hi[dj] - p.lo[dj];
        c.qo.count = r->d_qcount;
        c.qo.list = r->d_qlist;
        c.qo.nb = kQueryBuckets;
        c.qo.cap = r->q_cap;
        c.qo.dim = dj;
        c.qo.lo = p.lo[dj];
        c.qo.inv_w = span > 0 ? (double)kQueryBuckets / span : 0.0;
    }
    // grid rounds with bucketed samples generate them in the grid count launch (its extra
    // workgroups, with k_sample's bookkeeping): one launch less per round
    const bool fuse_sample = c.qo.list != nullptr;
    const int64_t set_n = r->pending_n;
    r->pending_n = -1;
    if (!fuse_sample) {
        hipLaunchKernelGGL(k_sample, dim3(kb), dim3(256), 0, stream, p, r->ext_base, K, r->d_samples, r->d_n,
                           live_list ? r->d_nlive : nullptr, set_n, r->d_counters);
        hip_check(hipGetLastError(), "k_sample");
    }
    c.mark(1, stream);
    SpreadOut spread;
    const bool want_spread = spread_request(r, use_tree || use_grid, spread);
    if (use_tree) {
        r->ctree->reserve(r->cap, p.d);  // once: no allocation (device sync) in later rounds
        if (defer_tree) {
            c.defer_tree = true;
            c.want_spread = want_spread;
            c.spread = spread;
        } else {
            CtJob J = tree_inc_job(r, stream, want_spread ? &spread : nullptr);
            launch_ct_jobs(nullptr, &J, 1, p.d, stream);
        }
    } else if (use_grid) {
        // spatial dims of the agent's tree state: x, y, z (omni, blimp) or x, y (snake);
        // the grid spans the sampling ranges, nodes outside fall into the border cells
        double lo[3], hi[3];
        for (int j = 0; j < r->grid_gd; ++j) {
            lo[j] = p.lo[r->grid_dims[j]];
            hi[j] = p.hi[r->grid_dims[j]];
        }
        // cells of ~2 points, but not much finer than the expected NN distance over all
        // state dims (kGridHminK: the fraction).  A state of 15 dims (the snake: the grid
        // spans x, y of them) takes cells of ~3 points with no floor: the floor from the
        // 15-dim NN distance made cells so coarse that a query examined 1.51x the points any
        // x, y index must (scripts/snake_floor.py: 1 100.6 vs 731.0); at 3 points a cell 1.29x
        // (945.3), the round within its run-to-run spread (config 3 54.87 M before, 54.65 / 53.78
        // M in two runs after; 2 points a cell: 1.26x but 51.1 M, the cells' overhead)
        const double hk = kGridHminK;
        const bool wide = p.d >= 15;
        const double ppc = r->ppc > 0 ? r->ppc : (wide ? 3.0 : 2.0);
        const bool floor_h = r->ppc <= 0 && !wide;
        const double hmin_n = floor_h ? hk * expected_nn_distance(p.d, p.lo, p.hi, r->n_upper) : 0.0;
        const double hmin_c = floor_h ? hk * expected_nn_distance(p.d, p.lo, p.hi, r->cap) : 0.0;
        const GridParams g = make_grid_params(p.d, r->grid_dims, r->grid_gd, lo, hi, r->n_upper, ppc, hmin_n);
        const GridParams gcap = make_grid_params(p.d, r->grid_dims, r->grid_gd, lo, hi, r->cap, ppc, hmin_c);
        r->grid->reserve(r->cap, p.d, std::max(g.ncells, gcap.ncells));  // once, as for the tree
        QueryBucketing qb;
        qb.q = r->d_samples;
        qb.nq = K;
        qb.o = c.qo;
        if (fuse_sample) {
            SampleGen &gen = qb.gen;
            gen.out = r->d_samples;
            gen.seed = p.seed;
            gen.ext_base = r->ext_base;
            for (int j = 0; j < p.d && j < kGenMaxDim; ++j) {
                gen.lo[j] = p.lo[j];
                gen.hi[j] = p.hi[j];
            }
            gen.n_dev = r->d_n;
            gen.set_n = set_n;
            gen.counters = r->d_counters;
            gen.n_live = live_list ? r->d_nlive : nullptr;
        }
        if (want_spread && !r->d_spread) {
            // the grid build's per-block partials [ceil(cap / 256)][6]
            const int64_t blocks = (r->cap + 255) / 256;
            hip_check(hipMalloc(&r->d_spread, sizeof(unsigned long long) * blocks * 6), "alloc spread");
            spread.partial = r->d_spread;
        }
        r->grid->build(r->d_nodes, r->n_upper, r->d_n, p.d, g, stream, want_spread ? &spread : nullptr,
                       c.qo.list ? &qb : nullptr);
    }
    if (want_spread) {
        if (!c.defer_tree) hip_check(hipEventRecord(r->ev_spread, stream), "spread event");
        r->spread_pending = true;
        r->rounds_since_spread = 0;
    }
    // a deferred build is marked where it runs (build_deferred, or after the joint build)
    if (!c.defer_tree) c.mark(2, stream);
    c.use_tree = use_tree;
    c.use_grid = use_grid;
    c.live_list = live_list;
    return c;
}

// a deferred tree build that did not join a joint build: run it on the engine's stream
void build_deferred(mpt_rrt *r, hipStream_t stream, const StepCtx &c) {
    {
        CtJob J = tree_inc_job(r, stream, c.want_spread ? &c.spread : nullptr);
        launch_ct_jobs(nullptr, &J, 1, r->p.d, stream);
    }
    if (c.want_spread) hip_check(hipEventRecord(r->ev_spread, stream), "spread event");
    c.mark(2, stream);
}

void step_nn(mpt_rrt *r, int32_t K, hipStream_t stream, const StepCtx &c) {
    const EngineParams &p = r->p;
    const bool use_tree = c.use_tree, use_grid = c.use_grid;
    if (use_tree) {
        CellTreeDev T = r->ctree->dev();
        T.stats = r->stats_on ? r->d_cstats + 8 : nullptr;
        launch_ct_nn1(T, r->d_samples, K, r->d_nn, r->d_nnd2, stream);
    } else if (use_grid) {
        GridDev G = r->grid->dev();
        G.stats = r->stats_on ? r->d_cstats + 8 : nullptr;
        if (c.qo.list)
            launch_grid_nn1_sorted(G, p.d, r->d_samples, K, c.qo, r->d_nn, r->d_nnd2, stream);
        else
            launch_grid_knn(G, p.d, r->d_samples, K, 1, r->d_nn, r->d_nnd2, stream);
    } else {
        NNWork w{};
        w.pts = r->d_nodes;
        w.removed = nullptr;
        w.n = r->n_upper;
        w.d = p.d;
        w.q = r->d_samples;
        w.nq = K;
        w.n_dev = r->d_n;
        launch_knn(w, 1, r->d_nn, r->d_nnd2, r->d_scratch, stream);
    }
    c.mark(3, stream);
}

void step_tail(mpt_rrt *r, int32_t K, hipStream_t stream, const StepCtx &c) {
    const EngineParams &p = r->p;
    const unsigned kb = c.kb;
    const bool live_list = c.live_list;
    hipEvent_t *ev = c.ev;
    auto steer = p.kind == MPT_AGENT_OMNI ? k_steer<MPT_AGENT_OMNI>
                 : (p.kind == MPT_AGENT_BLIMP ? k_steer<MPT_AGENT_BLIMP> : k_steer<MPT_AGENT_SNAKE>);
    uint64_t *tm = live_list && tmask_applies(r->env) ? r->d_tmask : nullptr;
    LiveOut lv{live_list ? r->d_live : nullptr, r->d_nlive, r->d_links, r->env, c.qo.count, c.qo.nb, r->d_rt, tm};
    hipLaunchKernelGGL(steer, dim3(kb), dim3(256), 0, stream, p, r->ext_base, K, r->d_nodes, r->d_nn, r->d_ends,
                       r->d_poses, r->d_pcount, r->d_verdict, r->d_counters, lv);
    hip_check(hipGetLastError(), "k_steer");
    c.mark(4, stream);
    CollideWork cw{};
    cw.poses = r->d_poses;
    cw.pose_edge = nullptr;
    cw.pcount = r->d_pcount;
    cw.pmax = p.pmax;
    cw.L = p.L;
    cw.n_units = (int64_t)K * p.pmax * p.L;
    cw.verdict = r->d_verdict;
    cw.stats = r->stats_on ? r->d_cstats : nullptr;
    cw.live_units = live_list ? r->d_live : nullptr;
    cw.unit_rt = live_list ? r->d_rt : nullptr;  // k_steer writes them with the live list
    cw.unit_tmask = tm;
    cw.n_live = live_list ? r->d_nlive : nullptr;
    OvfDefer ovf{};
    if (collide_mode() == MPT_COLLIDE_FUSED) {
        launch_collide(r->env, r->d_links, cw, stream);
        c.mark(5, stream);
        c.mark(6, stream);
        c.mark(7, stream);
    } else {
        // the overflow re-run moves into the append launch (no k_overflow launch of its own)
        if (!r->d_bar) {
            hip_check(hipMalloc(&r->d_bar, sizeof(uint32_t)), "alloc append ticket");
            hip_check(hipMemset(r->d_bar, 0, sizeof(uint32_t)), "zero append ticket");
            hip_check(hipDeviceSynchronize(), "append ticket zero sync");  // null stream vs the engine's
        }
        launch_collide_split(r->env, r->d_links, r->max_clusters, cw, r->cscratch, stream, ev ? ev + 5 : nullptr,
                             &ovf);
    }
    c.mark(8, stream);
    hipLaunchKernelGGL(k_append_commit, dim3(kb), dim3(256), 0, stream, r->d_verdict, K, p.d, r->d_ends, r->d_nn,
                       r->d_n, r->cap, r->d_nodes, r->d_parents, r->d_counters, ovf, r->d_bar);
    hip_check(hipGetLastError(), "append");
    c.mark(9, stream);
    r->ext_base += (uint64_t)K;
    r->n_upper = std::min<int64_t>(r->cap, r->n_upper + K);
    r->pt_grow += K;
    r->last_K = K;
}

}  // namespace

extern "C" mpt_status mpt_rrt_step(mpt_rrt *r, int32_t K, void *stream_) {
    return guarded([&] {
        if (!r || K < 1) throw Error{MPT_ERR_INVALID, "bad arguments"};
        hipStream_t stream = (hipStream_t)stream_;
        const StepCtx c = step_head(r, K, stream);
        step_nn(r, K, stream, c);
        step_tail(r, K, stream, c);
    });
}

namespace {

// Host-side state of the joint build + NN launch, one per joint stream: the device job table
// (d_stage) and the build's sort buffers are read by kernels on that stream, so only work
// ordered on the same stream may overwrite them.  (Round 1 kept one per host thread: two
// step_many groups on different joint streams then overwrote each other's job table and
// sort keys while the other group's kernels still read them.)  The table is staged through
// a ring of pinned buffers, so filling one never waits for a copy still in flight.
constexpr int kJobRing = 16;
struct JointNN {
    std::mutex mu;  // one step_many at a time per joint stream (the ring and the tables)
    char *d_stage = nullptr;
    char *h_stage[kJobRing] = {};
    const char *hd_stage[kJobRing] = {};  // the same pinned buffers' device addresses
    hipEvent_t copied[kJobRing] = {};
    size_t cap = 0;
    int32_t next = 0;
    std::vector<hipEvent_t> joins;
    hipEvent_t done = nullptr, built = nullptr;
    // engine timing on: b0 -> t0 = the joint tree build, t0 -> t1 = the joint NN launch
    hipEvent_t b0 = nullptr, t0 = nullptr, t1 = nullptr;
    bool timed = false;
    // joint rounds (joint_round): the engines' round buffers, engine j at edge offset j * K
    int64_t r_edges = 0, r_units = 0;
    int32_t r_dim = 0, r_subs = 0;
    double *j_samples = nullptr, *j_ends = nullptr, *j_poses = nullptr, *j_nnd2 = nullptr, *j_rt = nullptr;
    uint64_t *j_tmask = nullptr;
    int32_t *j_nn = nullptr, *j_pcount = nullptr, *j_live = nullptr;
    uint8_t *j_verdict = nullptr;
    uint32_t *j_nlive = nullptr;
    uint64_t buf_id = 0;  // id of the round buffers above (0: none); engines' jv slices carry it
    CollideScratch cs;
    uint32_t *d_bar = nullptr;  // k_append_jobs' ticket (the deferred overflow re-run)
    // timed joint round: start, sample, build, NN, steer, collide, append
    hipEvent_t st[7] = {};
    bool round_timed = false;
    // the last joint NN launch (mpt_rrt_joint_replay_nn): its device job table and shape
    const CtNnJob *nn_jobs = nullptr;
    int32_t nn_n = 0, nn_d = 0;
    int64_t nn_q = 0;
};
std::mutex g_joints_mu;
std::map<hipStream_t, std::shared_ptr<JointNN>> g_joints;
std::atomic<uint64_t> g_joint_buf_ids{0};
thread_local JointNN *g_last_timed = nullptr;  // mpt_rrt_joint_nn_ms: this thread's last timed call

JointNN &joint_state(hipStream_t s) {
    std::lock_guard<std::mutex> lk(g_joints_mu);
    std::shared_ptr<JointNN> &p = g_joints[s];
    if (!p) p.reset(new JointNN());
    return *p;
}

JointNN *joint_find(hipStream_t s) {
    std::lock_guard<std::mutex> lk(g_joints_mu);
    const auto it = g_joints.find(s);
    return it == g_joints.end() ? nullptr : it->second.get();
}

std::shared_ptr<JointNN> joint_find_shared(hipStream_t s) {
    std::lock_guard<std::mutex> lk(g_joints_mu);
    const auto it = g_joints.find(s);
    return it == g_joints.end() ? nullptr : it->second;
}

// The job tables go up by a kernel that reads the pinned ring over PCIe (a few KB), ordered on
// the joint stream like any launch.  hipMemcpyAsync's DMA copy left the compute queue idle ~23 us
// a round between k_sample_jobs and the build (config 5 at 32 seeds, kernel trace: the only
// gap of the round besides ~6 us before the engine-table copy).
__global__ void k_stage_copy(uint64_t *__restrict__ dst, const uint64_t *__restrict__ src, int64_t words) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += (int64_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}
void stage_copy(JointNN &g, int slot, size_t off, size_t bytes, hipStream_t s) {
    if (bytes == 0) return;
    if (off % 8 || bytes % 8) throw Error{MPT_ERR_INTERNAL, "job tables: 8-byte records expected"};
    const int64_t words = (int64_t)(bytes / 8);
    const unsigned blocks = (unsigned)std::min<int64_t>(16, (words + 255) / 256);
    hipLaunchKernelGGL(k_stage_copy, dim3(blocks), dim3(256), 0, s, reinterpret_cast<uint64_t *>(g.d_stage + off),
                       reinterpret_cast<const uint64_t *>(g.hd_stage[slot] + off), words);
    hip_check(hipGetLastError(), "k_stage_copy");
}

// a pinned staging buffer of at least `bytes` whose previous copy has completed
char *joint_stage(JointNN &g, size_t bytes, int *slot) {
    if (bytes > g.cap) {
        hip_check(hipDeviceSynchronize(), "sync");  // buffers may still be in use
        if (g.d_stage) hip_check(hipFree(g.d_stage), "free");
        if (g.h_stage[0]) hip_check(hipHostFree(g.h_stage[0]), "free");  // the ring's one allocation
        const size_t c = std::max(bytes, 2 * g.cap);
        hip_check(hipMalloc(&g.d_stage, c), "stage");
        // the ring's buffers carved from one pinned allocation (one hipHostMalloc, not kJobRing),
        // mapped and coherent explicitly: k_stage_copy reads it through its device address
        // (as PinnedSlots), independent of the runtime's default host-allocation flags
        char *ring = nullptr;
        hip_check(hipHostMalloc(&ring, c * kJobRing, hipHostMallocMapped | hipHostMallocCoherent), "stage pinned");
        char *dring = nullptr;
        hip_check(hipHostGetDevicePointer((void **)&dring, ring, 0), "stage pinned device address");
        for (int i = 0; i < kJobRing; ++i) {
            g.h_stage[i] = ring + (size_t)i * c;
            g.hd_stage[i] = dring + (size_t)i * c;
            if (!g.copied[i]) hip_check(hipEventCreateWithFlags(&g.copied[i], hipEventDisableTiming), "event");
        }
        if (!g.done) hip_check(hipEventCreateWithFlags(&g.done, hipEventDisableTiming), "event");
        if (!g.built) hip_check(hipEventCreateWithFlags(&g.built, hipEventDisableTiming), "event");
        g.cap = c;
    }
    *slot = g.next;
    g.next = (g.next + 1) % kJobRing;
    // the copy that last read this staging buffer was kJobRing calls ago
    hip_check(hipEventSynchronize(g.copied[*slot]), "jobs staging");
    return g.h_stage[*slot];
}

void joint_free_round(JointNN &g) {
    for (void *p : {(void *)g.j_samples, (void *)g.j_ends, (void *)g.j_poses, (void *)g.j_nnd2, (void *)g.j_rt,
                    (void *)g.j_nn, (void *)g.j_pcount, (void *)g.j_live, (void *)g.j_verdict, (void *)g.j_nlive,
                    (void *)g.j_tmask})
        if (p) hip_check(hipFree(p), "free");
    g.j_samples = g.j_ends = g.j_poses = g.j_nnd2 = g.j_rt = nullptr;
    g.j_tmask = nullptr;
    g.j_nn = g.j_pcount = g.j_live = nullptr;
    g.j_verdict = nullptr;
    g.j_nlive = nullptr;
    g.r_edges = g.r_units = 0;
    g.buf_id = 0;
}

// Engines whose rounds can run as one joint round (see EngineJob): every round on the Morton
// tree (incremental index), the same env, agent and engine parameters but the seed, the
// two-phase collide with the live-unit list, no work counters, K a multiple of 16 (the
// append's 16-byte verdict loads).
bool joint_round_ok(mpt_rrt *const *rs, int32_t n, int32_t K) {
    if (n < 2 || K < 16 || K % 16 != 0 || collide_mode() == MPT_COLLIDE_FUSED)
        return false;
    const mpt_rrt *a = rs[0];
    const EngineParams &p = a->p;
    const int64_t units = (int64_t)p.pmax * p.L;
    if (units > 64 || (int64_t)K * units > collide_chunk_units(a->max_clusters)) return false;
    for (int32_t i = 0; i < n; ++i) {
        mpt_rrt *r = rs[i];
        if (r->stats_on || r->agent != a->agent || r->env.tris != a->env.tris || r->n_upper < 1) return false;
        const EngineParams &q = r->p;
        if (q.kind != p.kind || q.d != p.d || q.L != p.L || q.pmax != p.pmax || q.steer_dt != p.steer_dt ||
            q.cc_dt != p.cc_dt || std::memcmp(q.prm, p.prm, sizeof(p.prm)) != 0 ||
            std::memcmp(q.lo, p.lo, sizeof(p.lo)) != 0 || std::memcmp(q.hi, p.hi, sizeof(p.hi)) != 0)
            return false;
        refresh_auto(r);
        if (!joint_uses_tree(r)) return false;
    }
    return true;
}

void joint_round(mpt_rrt *const *rs, int32_t n, int32_t K, void *const *streams_, hipStream_t joint) {
    JointNN &g = joint_state(joint);
    std::lock_guard<std::mutex> lk(g.mu);
    const mpt_rrt *a = rs[0];
    const EngineParams &p = a->p;
    const int32_t d = p.d;
    const int64_t units = (int64_t)p.pmax * p.L;
    // collide sub-batches: as many engines as one two-phase launch takes with the live list
    const int32_t per_sub = (int32_t)std::max<int64_t>(1, collide_chunk_units(a->max_clusters) / ((int64_t)K * units));
    const int32_t n_sub = (n + per_sub - 1) / per_sub;
    const int64_t edges = (int64_t)n * K;
    if (edges > g.r_edges || d != g.r_dim || units * edges > g.r_units || n_sub > g.r_subs) {
        hip_check(hipDeviceSynchronize(), "sync");  // the old buffers may still be in use
        joint_free_round(g);
        hip_check(hipMalloc(&g.j_samples, sizeof(double) * edges * d), "joint samples");
        hip_check(hipMalloc(&g.j_ends, sizeof(double) * edges * d), "joint ends");
        hip_check(hipMalloc(&g.j_poses, sizeof(double) * 12 * edges * units), "joint poses");
        hip_check(hipMalloc(&g.j_rt, sizeof(double) * 12 * edges * units), "joint unit transforms");
        hip_check(hipMalloc(&g.j_tmask, sizeof(uint64_t) * edges * units), "joint unit masks");
        hip_check(hipMalloc(&g.j_nnd2, sizeof(double) * edges), "joint nn d2");
        hip_check(hipMalloc(&g.j_nn, sizeof(int32_t) * edges), "joint nn");
        hip_check(hipMalloc(&g.j_pcount, sizeof(int32_t) * edges), "joint pose counts");
        hip_check(hipMalloc(&g.j_live, sizeof(int32_t) * edges * units), "joint live units");
        hip_check(hipMalloc(&g.j_verdict, (size_t)edges), "joint verdicts");
        hip_check(hipMalloc(&g.j_nlive, sizeof(uint32_t) * std::max(n_sub, 64)), "joint live counts");
        g.r_edges = edges;
        g.r_units = edges * units;
        g.r_dim = d;
        g.r_subs = std::max(n_sub, 64);
        g.buf_id = ++g_joint_buf_ids;
    }
    g.cs.ensure((int64_t)std::min(per_sub, n) * K * units, a->max_clusters);
    // the engines' host bookkeeping and their job table
    const size_t b_eng = sizeof(EngineJob) * n, b_inc = sizeof(CtJob) * n, b_nn = sizeof(CtNnJob) * n;
    int slot = 0;
    char *h = joint_stage(g, b_eng + b_inc + b_nn, &slot);
    EngineJob *he = reinterpret_cast<EngineJob *>(h);
    CtJob *hi = reinterpret_cast<CtJob *>(h + b_eng);
    CtNnJob *hn = reinterpret_cast<CtNnJob *>(h + b_eng + b_inc);
    const EngineJob *de = reinterpret_cast<const EngineJob *>(g.d_stage);
    const CtJob *di = reinterpret_cast<const CtJob *>(g.d_stage + b_eng);
    const CtNnJob *dn = reinterpret_cast<const CtNnJob *>(g.d_stage + b_eng + b_inc);
    std::vector<SpreadOut> spreads(n);
    std::vector<char> want(n, 0);
    bool timed = false;
    for (int32_t i = 0; i < n; ++i) {
        mpt_rrt *r = rs[i];
        he[i] = EngineJob{r->p.seed, r->ext_base, r->pending_n, r->cap, r->d_nodes, r->d_parents, r->d_n,
                          r->d_counters};
        r->pending_n = -1;
        r->ctree->reserve(r->cap, d);  // once: no allocation in later rounds
        want[i] = spread_request(r, true, spreads[i]) ? 1 : 0;
        timed = timed || r->timing;
    }
    // the joint stream waits for every engine stream's earlier work, the engines' streams
    // for the joint round
    std::vector<hipStream_t> uniq;
    for (int32_t i = 0; i < n; ++i) {
        const hipStream_t s = (hipStream_t)streams_[i];
        if (s != joint && std::find(uniq.begin(), uniq.end(), s) == uniq.end()) uniq.push_back(s);
    }
    while (g.joins.size() < uniq.size()) {
        hipEvent_t e;
        hip_check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "event");
        g.joins.push_back(e);
    }
    for (size_t u = 0; u < uniq.size(); ++u) {
        hip_check(hipEventRecord(g.joins[u], uniq[u]), "join record");
        hip_check(hipStreamWaitEvent(joint, g.joins[u], 0), "join wait");
    }
    if (timed && !g.st[0]) {
        for (hipEvent_t &e : g.st) hip_check(hipEventCreate(&e), "event");
        if (!g.b0) {
            hip_check(hipEventCreate(&g.b0), "event");
            hip_check(hipEventCreate(&g.t0), "event");
            hip_check(hipEventCreate(&g.t1), "event");
        }
    }
    auto mark = [&](int i) {
        if (timed) hip_check(hipEventRecord(g.st[i], joint), "joint stage event");
    };
    // the index builds' jobs (a full rebuild issues its code and sort launches in
    // tree_inc_job: those go after the samples' launch, which applies any truncation) and the
    // NN jobs.  A round with no full rebuild fills them first and stages all three tables in
    // one copy (one launch fewer a round).
    bool rebuilds = false;
    for (int32_t i = 0; i < n; ++i) rebuilds = rebuilds || tree_inc_launches(rs[i]);
    auto fill_tree_jobs = [&]() {
        for (int32_t i = 0; i < n; ++i) {
            mpt_rrt *r = rs[i];
            hi[i] = tree_inc_job(r, joint, want[i] ? &spreads[i] : nullptr);
            CellTreeDev T = r->ctree->dev();
            T.stats = nullptr;
            hn[i] = CtNnJob{T, g.j_samples + (int64_t)i * K * d, g.j_nn + (int64_t)i * K, g.j_nnd2 + (int64_t)i * K};
        }
    };
    if (!rebuilds) fill_tree_jobs();
    mark(0);
    stage_copy(g, slot, 0, rebuilds ? b_eng : b_eng + b_inc + b_nn, joint);
    const unsigned kb = (unsigned)((K + 255) / 256);
    hipLaunchKernelGGL(k_sample_jobs, dim3(kb, n), dim3(256), 0, joint, p, de, K, g.j_samples, g.j_nlive, n_sub);
    hip_check(hipGetLastError(), "k_sample_jobs");
    mark(1);
    if (timed) hip_check(hipEventRecord(g.b0, joint), "joint b0");
    if (rebuilds) {
        fill_tree_jobs();
        stage_copy(g, slot, b_eng, b_inc + b_nn, joint);
    }
    hip_check(hipEventRecord(g.copied[slot], joint), "jobs copied");
    launch_ct_jobs(di, hi, n, d, joint);
    for (int32_t i = 0; i < n; ++i)
        if (want[i]) {
            hip_check(hipEventRecord(rs[i]->ev_spread, joint), "spread event");
            rs[i]->spread_pending = true;
            rs[i]->rounds_since_spread = 0;
        }
    mark(2);
    if (timed) hip_check(hipEventRecord(g.t0, joint), "joint t0");
    launch_ct_nn1_jobs(dn, n, d, K, joint, ct_joint_parts(n, d, K));
    g.nn_jobs = dn;
    g.nn_n = n;
    g.nn_d = d;
    g.nn_q = K;
    mark(3);
    if (timed) hip_check(hipEventRecord(g.t1, joint), "joint t1");
    auto steer = p.kind == MPT_AGENT_OMNI ? k_steer_jobs<MPT_AGENT_OMNI>
                 : (p.kind == MPT_AGENT_BLIMP ? k_steer_jobs<MPT_AGENT_BLIMP> : k_steer_jobs<MPT_AGENT_SNAKE>);
    uint64_t *tm = tmask_applies(a->env) ? g.j_tmask : nullptr;
    LiveOut lv{g.j_live, g.j_nlive, a->d_links, a->env, nullptr, 0, g.j_rt, tm};
    hipLaunchKernelGGL(steer, dim3(kb, n), dim3(256), 0, joint, p, de, K, g.j_nn, g.j_ends, g.j_poses, g.j_pcount,
                       g.j_verdict, lv, per_sub);
    hip_check(hipGetLastError(), "k_steer_jobs");
    mark(4);
    OvfDefer ovf{};
    const bool fold_ovf = (int64_t)kb * n <= 1024;  // k_append_jobs<true>'s case (its comment)
    if (fold_ovf && !g.d_bar) {
        hip_check(hipMalloc(&g.d_bar, sizeof(uint32_t)), "alloc append ticket");
        hip_check(hipMemsetAsync(g.d_bar, 0, sizeof(uint32_t), joint), "zero append ticket");
    }
    for (int32_t b = 0; b < n_sub; ++b) {
        const int64_t e0 = (int64_t)b * per_sub * K;
        const int32_t ne = std::min(per_sub, n - b * per_sub);
        CollideWork cw{};
        cw.poses = g.j_poses + e0 * units * 12;
        cw.pose_edge = nullptr;
        cw.pcount = g.j_pcount + e0;
        cw.pmax = p.pmax;
        cw.L = p.L;
        cw.n_units = (int64_t)ne * K * units;
        cw.verdict = g.j_verdict + e0;
        cw.stats = nullptr;
        cw.live_units = g.j_live + e0 * units;
        cw.n_live = g.j_nlive + b;
        cw.unit_rt = g.j_rt + e0 * units * 12;
        cw.unit_tmask = tm ? tm + e0 * units : nullptr;
        // a small round's last batch moves its overflow re-run into the append launch (when it
        // ran in one chunk)
        launch_collide_split(a->env, a->d_links, a->max_clusters, cw, g.cs, joint, nullptr,
                             b == n_sub - 1 && fold_ovf ? &ovf : nullptr);
    }
    mark(5);
    hipLaunchKernelGGL(fold_ovf ? k_append_jobs<true> : k_append_jobs<false>, dim3(kb, n), dim3(256), 0, joint, de,
                       g.j_verdict, K, d, g.j_ends, g.j_nn, ovf, g.d_bar);
    hip_check(hipGetLastError(), "k_append_jobs");
    mark(6);
    g.timed = timed;
    g.round_timed = timed;
    if (timed) g_last_timed = &g;
    if (!g.done) hip_check(hipEventCreateWithFlags(&g.done, hipEventDisableTiming), "event");
    hip_check(hipEventRecord(g.done, joint), "joint done");
    for (hipStream_t s : uniq) hip_check(hipStreamWaitEvent(s, g.done, 0), "joint wait");
    for (int32_t i = 0; i < n; ++i) {
        mpt_rrt *r = rs[i];
        r->ext_base += (uint64_t)K;
        r->n_upper = std::min<int64_t>(r->cap, r->n_upper + K);
        r->pt_grow += K;
        r->last_K = K;
        r->last_nn = MPT_NN_TREE;
        r->last_joint = true;
        r->jv_stream = joint;
        r->jv_id = g.buf_id;
        const int64_t e0 = (int64_t)i * K;
        r->jv.samples = g.j_samples + e0 * d;
        r->jv.ends = g.j_ends + e0 * d;
        r->jv.poses = g.j_poses + e0 * units * 12;
        r->jv.nn = g.j_nn + e0;
        r->jv.pcount = g.j_pcount + e0;
        r->jv.verdict = g.j_verdict + e0;
    }
}

}  // namespace

extern "C" mpt_status mpt_rrt_step_many(mpt_rrt *const *rs, int32_t n, int32_t K, void *const *streams_,
                                        void *joint_stream_) {
    return guarded([&] {
        if (!rs || n < 1 || K < 1 || !streams_) throw Error{MPT_ERR_INVALID, "bad arguments"};
        for (int32_t i = 0; i < n; ++i)
            if (!rs[i]) throw Error{MPT_ERR_INVALID, "null engine"};
        auto stream_of = [&](int32_t i) { return (hipStream_t)streams_[i]; };
        const hipStream_t joint = (hipStream_t)joint_stream_;
        if (joint_round_ok(rs, n, K)) {
            joint_round(rs, n, K, streams_, joint);
            return;
        }
        std::vector<StepCtx> cs(n);
        for (int32_t i = 0; i < n; ++i) cs[i] = step_head(rs[i], K, stream_of(i), true);
        // engines whose round uses the Morton tree (and the first such engine's state dim)
        // share one index build (a launch per stage + one segmented sort) and one NN launch;
        // the rest query their own index on their own stream
        std::vector<int32_t> J;
        for (int32_t i = 0; i < n; ++i)
            if (cs[i].use_tree && (J.empty() || rs[i]->p.d == rs[J[0]]->p.d)) J.push_back(i);
        if (J.size() < 2) J.clear();
        std::vector<char> joined(n, 0);
        for (int32_t i : J) joined[i] = 1;
        for (int32_t i = 0; i < n; ++i)
            if (cs[i].defer_tree && !joined[i]) build_deferred(rs[i], stream_of(i), cs[i]);
        if (!J.empty()) {
            JointNN &g = joint_state(joint);
            std::lock_guard<std::mutex> lk(g.mu);
            const int32_t nj = (int32_t)J.size();
            const size_t b_build = sizeof(CtJob) * nj, b_nn = sizeof(CtNnJob) * nj;
            int slot = 0;
            char *h = joint_stage(g, b_build + b_nn, &slot);
            CtJob *hi = reinterpret_cast<CtJob *>(h);
            CtNnJob *hn = reinterpret_cast<CtNnJob *>(h + b_build);
            // the joint stream waits for every engine stream's heads, the engines' tails for it
            // (before the builds: a full incremental rebuild issues its launches here)
            std::vector<hipStream_t> uniq;
            for (int32_t i : J)
                if (std::find(uniq.begin(), uniq.end(), stream_of(i)) == uniq.end()) uniq.push_back(stream_of(i));
            while (g.joins.size() < uniq.size()) {
                hipEvent_t e;
                hip_check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "event");
                g.joins.push_back(e);
            }
            for (size_t u = 0; u < uniq.size(); ++u) {
                hip_check(hipEventRecord(g.joins[u], uniq[u]), "join record");
                hip_check(hipStreamWaitEvent(joint, g.joins[u], 0), "join wait");
            }
            bool timed = false;
            for (int32_t i : J) timed = timed || rs[i]->timing;
            if (timed) {
                if (!g.t0) {
                    hip_check(hipEventCreate(&g.b0), "event");
                    hip_check(hipEventCreate(&g.t0), "event");
                    hip_check(hipEventCreate(&g.t1), "event");
                }
                hip_check(hipEventRecord(g.b0, joint), "joint b0");
            }
            for (int32_t k = 0; k < nj; ++k) {
                mpt_rrt *r = rs[J[k]];
                const StepCtx &c = cs[J[k]];
                hi[k] = tree_inc_job(r, joint, c.want_spread ? &c.spread : nullptr);
                CellTreeDev T = r->ctree->dev();
                T.stats = r->stats_on ? r->d_cstats + 8 : nullptr;
                hn[k] = CtNnJob{T, r->d_samples, r->d_nn, r->d_nnd2};
            }
            stage_copy(g, slot, 0, b_build + b_nn, joint);
            hip_check(hipEventRecord(g.copied[slot], joint), "jobs copied");
            const CtJob *di = reinterpret_cast<const CtJob *>(g.d_stage);
            const CtNnJob *dn = reinterpret_cast<const CtNnJob *>(g.d_stage + b_build);
            launch_ct_jobs(di, hi, nj, rs[J[0]]->p.d, joint);
            for (int32_t i : J)
                if (cs[i].want_spread) hip_check(hipEventRecord(rs[i]->ev_spread, joint), "spread event");
            if (timed) {
                hip_check(hipEventRecord(g.t0, joint), "joint t0");
                // the engines' nn_build stage ends with the joint build
                hip_check(hipEventRecord(g.built, joint), "joint built");
                for (hipStream_t s : uniq) hip_check(hipStreamWaitEvent(s, g.built, 0), "built wait");
                for (int32_t i : J) cs[i].mark(2, stream_of(i));
            }
            launch_ct_nn1_jobs(dn, nj, rs[J[0]]->p.d, K, joint, ct_joint_parts(nj, rs[J[0]]->p.d, K));
            g.nn_jobs = dn;
            g.nn_n = nj;
            g.nn_d = rs[J[0]]->p.d;
            g.nn_q = K;
            if (timed) {
                hip_check(hipEventRecord(g.t1, joint), "joint t1");
                g_last_timed = &g;
            }
            g.timed = timed;
            g.round_timed = false;
            hip_check(hipEventRecord(g.done, joint), "joint done");
            for (hipStream_t s : uniq) hip_check(hipStreamWaitEvent(s, g.done, 0), "joint wait");
            for (int32_t i : J) cs[i].mark(3, stream_of(i));
        }
        for (int32_t i = 0; i < n; ++i)
            if (!joined[i]) step_nn(rs[i], K, stream_of(i), cs[i]);
        for (int32_t i = 0; i < n; ++i) step_tail(rs[i], K, stream_of(i), cs[i]);
    });
}

namespace {
// an engine's last joint round slices are still the joint state's live buffers: the joint
// state's lock, held by the caller through its copies (a step_many that reallocates the round
// buffers or a joint_release on another host thread waits for it; the state itself stays alive
// through the shared pointer)
struct JointSlices {
    std::shared_ptr<JointNN> g;
    std::unique_lock<std::mutex> lk;
};
JointSlices joint_slices_lock(const mpt_rrt *r) {
    JointSlices js;
    js.g = joint_find_shared(r->jv_stream);
    if (js.g) js.lk = std::unique_lock<std::mutex>(js.g->mu);
    if (!js.g || js.g->buf_id == 0 || js.g->buf_id != r->jv_id)
        throw Error{MPT_ERR_INVALID, "the joint round's buffers were released or reallocated since this engine's "
                                     "last round"};
    return js;
}
}  // namespace

extern "C" mpt_status mpt_rrt_joint_nn_ms(float *ms) {
    return guarded([&] {
        if (!ms) throw Error{MPT_ERR_INVALID, "null pointer"};
        JointNN *g = g_last_timed;
        if (!g) throw Error{MPT_ERR_INVALID, "no timed joint NN launch on this thread"};
        std::lock_guard<std::mutex> lk(g->mu);
        hip_check(hipEventSynchronize(g->t1), "event sync");
        hip_check(hipEventElapsedTime(ms, g->t0, g->t1), "elapsed");
    });
}

extern "C" mpt_status mpt_rrt_joint_times(void *joint_stream, float ms[2]) {
    return guarded([&] {
        if (!ms) throw Error{MPT_ERR_INVALID, "null pointer"};
        JointNN *g = joint_find((hipStream_t)joint_stream);
        if (!g) throw Error{MPT_ERR_INVALID, "no joint launch on this stream"};
        std::lock_guard<std::mutex> lk(g->mu);
        if (!g->timed) throw Error{MPT_ERR_INVALID, "the last joint launch on this stream was not timed"};
        hip_check(hipEventSynchronize(g->t1), "event sync");
        hip_check(hipEventElapsedTime(&ms[0], g->b0, g->t0), "elapsed");
        hip_check(hipEventElapsedTime(&ms[1], g->t0, g->t1), "elapsed");
    });
}

extern "C" mpt_status mpt_rrt_joint_stage_times(void *joint_stream, float ms[6]) {
    return guarded([&] {
        if (!ms) throw Error{MPT_ERR_INVALID, "null pointer"};
        JointNN *g = joint_find((hipStream_t)joint_stream);
        if (!g) throw Error{MPT_ERR_INVALID, "no joint launch on this stream"};
        std::lock_guard<std::mutex> lk(g->mu);
        if (!g->round_timed) throw Error{MPT_ERR_INVALID, "the last step_many on this stream was not a timed joint round"};
        hip_check(hipEventSynchronize(g->st[6]), "event sync");
        for (int i = 0; i < 6; ++i) hip_check(hipEventElapsedTime(&ms[i], g->st[i], g->st[i + 1]), "elapsed");
    });
}

// Diagnostics: the joint stream's last NN launch again, on that stream, over the same job table
// (its queries, its trees' index as that round's build left it, its output slots: the results are
// rewritten with the same values) -- the NN alone for rocprofv3 counters, e.g. after an L2 flush.
extern "C" mpt_status mpt_rrt_joint_replay_nn(void *joint_stream, int32_t parts) {
    return guarded([&] {
        std::shared_ptr<JointNN> g = joint_find_shared((hipStream_t)joint_stream);
        if (!g || !g->nn_jobs) throw Error{MPT_ERR_INVALID, "no joint NN launch on this stream"};
        std::lock_guard<std::mutex> lk(g->mu);
        launch_ct_nn1_jobs(g->nn_jobs, g->nn_n, g->nn_d, g->nn_q, (hipStream_t)joint_stream, parts);
    });
}

extern "C" mpt_status mpt_rrt_joint_release(void *joint_stream) {
    return guarded([&] {
        std::shared_ptr<JointNN> g;
        {
            std::lock_guard<std::mutex> lk(g_joints_mu);
            const auto it = g_joints.find((hipStream_t)joint_stream);
            if (it == g_joints.end()) return;
            g = std::move(it->second);
            g_joints.erase(it);
        }
        std::lock_guard<std::mutex> lk(g->mu);  // no step_many of this stream is staging
        hip_check(hipStreamSynchronize((hipStream_t)joint_stream), "joint stream sync");
        if (g_last_timed == g.get()) g_last_timed = nullptr;
        if (g->d_stage) hip_check(hipFree(g->d_stage), "free");
        if (g->h_stage[0]) hip_check(hipHostFree(g->h_stage[0]), "free");  // the ring's one allocation
        for (int i = 0; i < kJobRing; ++i)
            if (g->copied[i]) hip_check(hipEventDestroy(g->copied[i]), "event");
        for (hipEvent_t e : g->joins) hip_check(hipEventDestroy(e), "event");
        for (hipEvent_t e : {g->done, g->built, g->b0, g->t0, g->t1})
            if (e) hip_check(hipEventDestroy(e), "event");
        joint_free_round(*g);
        for (hipEvent_t e : g->st)
            if (e) hip_check(hipEventDestroy(e), "event");
    });
}

extern "C" mpt_status mpt_rrt_counters(mpt_rrt *r, uint64_t c[8]) {
    return guarded([&] {
        if (!r || !c) throw Error{MPT_ERR_INVALID, "null pointer"};
        flush_size(r);
        unsigned long long h[8];
        hip_check(hipMemcpy(h, r->d_counters, sizeof(h), hipMemcpyDeviceToHost), "counters");
        for (int i = 0; i < 8; ++i) c[i] = h[i];
        if (h[6]) throw Error{MPT_ERR_INTERNAL, "incremental tree index: a build found more new points than it merges"};
    });
}

extern "C" mpt_status mpt_rrt_read_tree(mpt_rrt *r, double *states, int32_t *parents, int64_t n) {
    return guarded([&] {
        if (!r || n < 0 || n > r->cap) throw Error{MPT_ERR_INVALID, "bad arguments"};
        hip_check(hipDeviceSynchronize(), "sync");
        if (states && n) hip_check(hipMemcpy(states, r->d_nodes, sizeof(double) * r->p.d * n, hipMemcpyDeviceToHost), "");
        if (parents && n) hip_check(hipMemcpy(parents, r->d_parents, sizeof(int32_t) * n, hipMemcpyDeviceToHost), "");
    });
}

extern "C" mpt_status mpt_rrt_last_round(mpt_rrt *r, double *samples, int32_t *nn_ids, double *ends,
                                         uint8_t *verdicts) {
    return guarded([&] {
        if (!r) throw Error{MPT_ERR_INVALID, "null pointer"};
        hip_check(hipDeviceSynchronize(), "sync");
        const int64_t K = r->last_K, d = r->p.d;
        if (K == 0) return;
        // a joint round's buffers are the joint state's slices (valid until its next step_many)
        const bool j = r->last_joint;
        JointSlices lock;
        if (j) lock = joint_slices_lock(r);
        const double *s = j ? r->jv.samples : r->d_samples, *e = j ? r->jv.ends : r->d_ends;
        const int32_t *nn = j ? r->jv.nn : r->d_nn;
        const uint8_t *v = j ? r->jv.verdict : r->d_verdict;
        if (samples) hip_check(hipMemcpy(samples, s, sizeof(double) * K * d, hipMemcpyDeviceToHost), "");
        if (nn_ids) hip_check(hipMemcpy(nn_ids, nn, sizeof(int32_t) * K, hipMemcpyDeviceToHost), "");
        if (ends) hip_check(hipMemcpy(ends, e, sizeof(double) * K * d, hipMemcpyDeviceToHost), "");
        if (verdicts) hip_check(hipMemcpy(verdicts, v, (size_t)K, hipMemcpyDeviceToHost), "");
    });
}

extern "C" mpt_status mpt_rrt_last_poses(mpt_rrt *r, double *poses, int32_t *pose_counts) {
    return guarded([&] {
        if (!r) throw Error{MPT_ERR_INVALID, "null pointer"};
        hip_check(hipDeviceSynchronize(), "sync");
        const int64_t K = r->last_K;
        if (K == 0) return;
        const bool j = r->last_joint;
        JointSlices lock;
        if (j) lock = joint_slices_lock(r);
        if (poses)
            hip_check(hipMemcpy(poses, j ? r->jv.poses : r->d_poses, sizeof(double) * 12 * K * r->p.pmax * r->p.L,
                                hipMemcpyDeviceToHost),
                      "poses D2H");
        if (pose_counts)
            hip_check(hipMemcpy(pose_counts, j ? r->jv.pcount : r->d_pcount, sizeof(int32_t) * K, hipMemcpyDeviceToHost),
                      "pcount D2H");
    });
}

extern "C" mpt_status mpt_rrt_last_nn(const mpt_rrt *r, int32_t *mode) {
    return guarded([&] {
        if (!r || !mode) throw Error{MPT_ERR_INVALID, "null pointer"};
        *mode = r->last_nn;
    });
}

extern "C" mpt_status mpt_rrt_info(const mpt_rrt *r, int64_t info[4]) {
    return guarded([&] {
        if (!r || !info) throw Error{MPT_ERR_INVALID, "null pointer"};
        info[0] = r->p.d;
        info[1] = r->p.L;
        info[2] = r->p.pmax;
        info[3] = r->cap;
    });
}

extern "C" mpt_status mpt_rrt_collide_stats(mpt_rrt *r, int32_t enable, uint64_t out[kCollideStats]) {
    return guarded([&] {
        if (!r) throw Error{MPT_ERR_INVALID, "null pointer"};
        hip_check(hipDeviceSynchronize(), "sync");
        if (!r->d_cstats) {
            hip_check(hipMalloc(&r->d_cstats, sizeof(unsigned long long) * kCollideStats), "alloc stats");
            hip_check(hipMemset(r->d_cstats, 0, sizeof(unsigned long long) * kCollideStats), "memset stats");
        }
        if (out) {
            unsigned long long h[kCollideStats];
            hip_check(hipMemcpy(h, r->d_cstats, sizeof(h), hipMemcpyDeviceToHost), "stats D2H");
            for (int i = 0; i < kCollideStats; ++i) out[i] = h[i];
        }
        hip_check(hipMemset(r->d_cstats, 0, sizeof(unsigned long long) * kCollideStats), "memset stats");
        hip_check(hipDeviceSynchronize(), "memset stats sync");  // null stream vs the engine's stream
        r->stats_on = enable != 0;
    });
}

extern "C" mpt_status mpt_rrt_set_nn(mpt_rrt *r, int32_t mode, double points_per_cell) {
    return guarded([&] {
        if (!r || mode < MPT_NN_AUTO || mode > MPT_NN_TREE) throw Error{MPT_ERR_INVALID, "bad arguments"};
        r->nn_mode = mode;
        r->ppc = points_per_cell > 0 ? points_per_cell : 0.0;
        // the cell tree's memory for the engine's capacity, now rather than in a round (it
        // allocates and synchronises the device): when its rounds will use the tree -- MPT_NN_TREE,
        // or MPT_NN_AUTO once the first nodes' spread chose it (mpt_rrt_add_nodes)
        if (mode == MPT_NN_TREE || (mode == MPT_NN_AUTO && r->spread_seen && r->auto_tree)) {
            r->ctree->reserve(r->cap, r->p.d);
            (void)r->ctree->set_plan(r->p.lo, r->p.hi, r->grid_gd);  // the first build then starts from it
        }
    });
}

extern "C" mpt_status mpt_rrt_enable_timing(mpt_rrt *r, int32_t enable) {
    return guarded([&] {
        if (!r) throw Error{MPT_ERR_INVALID, "null pointer"};
        r->timing = enable != 0;
        if (r->timing && r->ring.empty()) {
            r->ring.assign((size_t)kTimingRing * 10, nullptr);
            for (auto &e : r->ring) hip_check(hipEventCreate(&e), "event");
        }
    });
}

extern "C" mpt_status mpt_rrt_kernel_times(mpt_rrt *r, float ms[9]) {
    return guarded([&] {
        if (!r || !ms) throw Error{MPT_ERR_INVALID, "null pointer"};
        if (!r->timing || r->ring_next == 0) throw Error{MPT_ERR_INVALID, "timing not enabled or no round yet"};
        if (r->last_joint)
            throw Error{MPT_ERR_INVALID, "the last round ran in a joint round (mpt_rrt_step_many), which times its "
                                         "stages on the joint stream: use mpt_rrt_joint_stage_times"};
        hipEvent_t *e = r->ring.data() + ((r->ring_next - 1) % kTimingRing) * 10;
        hip_check(hipEventSynchronize(e[9]), "event sync");
        // [sample, nn_build, nn_query, steer, collide_pairs, collide_cands, collide_narrow,
        //  collide_rest, append]: consecutive event pairs
        for (int i = 0; i < 9; ++i) hip_check(hipEventElapsedTime(&ms[i], e[i], e[i + 1]), "elapsed");
    });
}

extern "C" mpt_status mpt_rrt_kernel_times_sum(mpt_rrt *r, double ms[9], int64_t *rounds) {
    return guarded([&] {
        if (!r || !ms || !rounds) throw Error{MPT_ERR_INVALID, "null pointer"};
        while (r->ring_done < r->ring_next) timing_fold_one(r);
        for (int i = 0; i < 9; ++i) {
            ms[i] = r->acc_ms[i];
            r->acc_ms[i] = 0.0;
        }
        *rounds = r->acc_rounds;
        r->acc_rounds = 0;
    });
}
