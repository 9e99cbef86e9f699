// collide.hip -- batched mesh-vs-mesh collision verdicts on gfx950.
//
// Replaces MeshHandler::isInCollision (utilities/meshhandler.hpp:187-243) and the FCL
// 0.3.2 path behind it (DynamicAABBTreeCollisionManager broadphase + OBBRSS traversal
// + Intersect::intersect_Triangle).  Verdict per edge = exists (pose, link, env tri,
// agent tri) whose exact AABBs overlap (fcl_math.h tri_gate: FCL's BV test before the
// leaf test) and with intersect_Triangle true, i.e. the gated all-pairs definition;
// every float box test below only prunes, with margins (fcl_math.h widen_*) that keep
// it conservative.
//
// Two structures, same verdicts (mpt_set_collide_mode):
//  * split (default): k_broad -> k_narrow below, the fused kernel only for overflow;
//  * fused: k_collide, described here.
// Fused mapping: one wavefront per (pose, link) unit, waves stride over the units (a bounded
// grid, so the per-workgroup LDS staging below is amortised).  The agent link mesh is
// stored in clusters of <= 64 triangles (one triangle per lane).  Per unit:
//   1. R, T = fcl::relativeTransform(env tf, pose)                      (uniform)
//   2. lanes over clusters: transformed cluster box vs env root box -> ballot mask
//   3. per surviving cluster: each lane maps its triangle Q_i' = R Q_i + T exactly as
//      FCL does and takes its float box; the wave walks the env BVH UNIFORMLY (one node
//      at a time, node index in an SGPR, stack in LDS); the top of the BVH (breadth-first
//      prefix, up to kLdsNodes nodes -- all of it for the benchmark rooms) is staged in LDS
//      once per workgroup, deeper nodes come from global memory; at each node a ballot
//      of the lanes' box tests decides descent, so traversal never diverges;
//   4. at a leaf, lanes whose box overlaps the env triangle run the 17-axis test;
//      any hit -> verdict[edge] = 1 and the wave (and later units of that edge) stop.
#include "collide_common.h"

namespace mpt {

constexpr int kCollideWaves = 4;     // waves per workgroup
constexpr int kLdsNodes = 1024;      // 32 KiB of BVH nodes per workgroup

__global__ __launch_bounds__(kCollideWaves * 64) void k_collide(EnvDev env, const AgentDev *__restrict__ links,
                                                                 CollideWork w) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    // list mode (overflow re-run of the two-phase path): usually empty, leave at once
    const int64_t n_work = w.unit_list ? (int64_t)*w.unit_list_n : w.n_units;
    if ((int64_t)blockIdx.x * kCollideWaves >= n_work) return;
    BvhNode *s_nodes = reinterpret_cast<BvhNode *>(smem);
    const int32_t n_lds = env.n_nodes < kLdsNodes ? env.n_nodes : kLdsNodes;
    int32_t *s_stack = reinterpret_cast<int32_t *>(smem + sizeof(BvhNode) * n_lds);
    // stage the breadth-first prefix of the BVH (16-B pieces, all lanes of the workgroup)
    {
        const uint4 *src = reinterpret_cast<const uint4 *>(env.nodes);
        uint4 *dst = reinterpret_cast<uint4 *>(s_nodes);
        for (int i = threadIdx.x; i < n_lds * 2; i += blockDim.x) dst[i] = src[i];
    }
    __syncthreads();

    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform for the compiler
    const int lane = threadIdx.x & 63;
    int32_t *stk = s_stack + wave * kStackDepth;
    // several units per edge (links, poses, or host-given pose lists): share early exits
    const bool shared_edges = w.pose_edge != nullptr || w.L > 1 || w.pmax > 1;
    uint32_t n_units = 0, n_clusters = 0, n_nodes = 0, n_sat = 0;
    const int64_t stride = (int64_t)gridDim.x * kCollideWaves;
    for (int64_t i = (int64_t)blockIdx.x * kCollideWaves + wave; i < n_work; i += stride) {
        const int64_t unit = w.unit_list ? (int64_t)w.unit_list[i] : i;
        collide_unit(env, s_nodes, n_lds, links, w, unit, stk, lane, shared_edges, n_clusters, n_nodes, n_sat,
                     n_units);
    }
    if (w.stats && lane == 0) {
        atomicAdd(w.stats + 0, (unsigned long long)n_units);
        atomicAdd(w.stats + 1, (unsigned long long)n_clusters);
        atomicAdd(w.stats + 2, (unsigned long long)n_nodes);
        atomicAdd(w.stats + 3, (unsigned long long)n_sat);
    }
}

__global__ void k_pose_edge(const int64_t *__restrict__ off, int64_t E, int32_t *__restrict__ pe) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    for (int64_t p = off[e]; p < off[e + 1]; ++p) pe[p] = (int32_t)e;
}

void launch_collide(const EnvDev &env, const AgentDev *d_links, const CollideWork &w, hipStream_t stream,
                    int cap_blocks) {
    if (w.n_units <= 0 || env.n_tris <= 0) return;
    // computed once (thread-safe static init: engines may step from several host threads)
    static const int max_blocks = [] {
        int dev = 0, cus = 256;
        if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        const int per_cu = 6;  // ~2 workgroups per CU resident (VGPR-limited) x 3 rounds
        return cus * per_cu;
    }();
    const int32_t n_lds = env.n_nodes < kLdsNodes ? env.n_nodes : kLdsNodes;
    const size_t lds = sizeof(BvhNode) * n_lds + sizeof(int32_t) * kStackDepth * kCollideWaves;
    int64_t blocks = (w.n_units + kCollideWaves - 1) / kCollideWaves;
    if (blocks > max_blocks) blocks = max_blocks;
    if (cap_blocks > 0 && blocks > cap_blocks) blocks = cap_blocks;
    hipLaunchKernelGGL(k_collide, dim3((unsigned)blocks), dim3(kCollideWaves * 64), lds, stream, env, d_links, w);
    hip_check(hipGetLastError(), "k_collide launch");
}

void launch_pose_edge(const int64_t *d_offsets, int64_t E, int32_t *d_pose_edge, hipStream_t stream) {
    if (E <= 0) return;
    hipLaunchKernelGGL(k_pose_edge, dim3((unsigned)((E + 255) / 256)), dim3(256), 0, stream, d_offsets, E,
                       d_pose_edge);
    hip_check(hipGetLastError(), "k_pose_edge launch");
}

}  // namespace mpt
