// mpt_internal.h -- device data layout in HBM and the internal launch interfaces.
//
// Environment (StaticEnvironmentMeshHandler, utilities/meshhandler.hpp:18-55): all
// submeshes share one transform, so they are merged into one triangle soup, stored
//   tris  [T] EnvTri (320 B, env-local frame, BVH leaf order)
//   nodes [2T-1] BvhNode (32 B: float AABB widened outward + children / leaf index)
// Agent link mesh (SimpleAgentMeshHandler, meshhandler.hpp:112-135):
//   tris     [T][9] doubles, agent-local frame, grouped in clusters of <= 64
//   clusters [C] Cluster (local box centre/half-extent + first/count)
// Tree nodes (FLANN_KDTreeWrapper, utilities/flannkdtreewrapper.hpp): [capacity][d] FP64,
// id = row + 1 (FLANN ids start at 1, the ctor's dummy point 0 is removed).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <exception>
#include <string>
#include <vector>

#include "fcl_math.h"

namespace mpt {

constexpr int kWave = 64;
constexpr int kCollideStats = 16;  // collide work counters (mpt_rrt_collide_stats)
constexpr int kClusterMax = 64;
constexpr int kStackDepth = 64;

struct BvhNode {
    float lo[3];
    int32_t a;   // inner: left child   | leaf: triangle index
    float hi[3];
    int32_t b;   // inner: right child  | leaf: -1
};
static_assert(sizeof(BvhNode) == 32, "BvhNode layout");

struct Cluster {
    double c[3];   // local box centre
    double e[3];   // local half-extent
    int32_t first; // first triangle
    int32_t count; // <= 64
};

// a pointer qualifier for global memory (address space 1)
#define MPT_GLOBAL __attribute__((address_space(1)))

// N doubles from p, which points to global memory, with global instructions: pointers read
// from memory (job tables, AgentDev records) are otherwise accessed with flat instructions,
// which also count against the LDS counter
template <int N>
__device__ __forceinline__ void load_global(const double *p, double (&out)[N]) {
    const MPT_GLOBAL double *g = (const MPT_GLOBAL double *)p;
#pragma unroll
    for (int k = 0; k < N; ++k) out[k] = g[k];
}

struct AgentDev {
    const double *tris;       // [T][9]
    const Cluster *clusters;  // [C]
    int32_t n_clusters;
    int32_t n_tris;
    double bc[3], be[3];      // whole-link local box centre / half-extent
    const EnvTri *etris;      // [T] the triangles as intersect_Triangle's P side (self-collision)
};

// Broad-phase env tree, 64 children per node so one wave tests a node's children with one
// lane each.  Level 0 = one item per triangle (leaf order, box = the triangle's widened
// box); level 1 = buckets, the maximal median-split subtrees with <= 64 triangles; each
// higher level groups <= 64 consecutive items of the level below, up to a top level of
// <= 64 items (the children of a virtual root).  first/count = children in the level below.
struct Item {
    float lo[3];
    int32_t first;
    float hi[3];
    int32_t count;
};
static_assert(sizeof(Item) == 32, "Item layout");
constexpr int kMaxLevels = 8;

// An Item's box quantized to 15 bits per coordinate over the env root box, rounded outward
// (a superset of the float box, so a test on it never drops a pair the float test keeps), and
// its children packed: 16 B instead of 32, one LDS read per box (k_pairs' two-level walk).
//   x = lo.x | lo.y << 16, y = hi.x | hi.y << 16, z = lo.z | hi.z << 16,
//   w = first | (count - 1) << 26
constexpr uint32_t kQMax = 32767u;
struct EnvDev {
    const EnvTri *tris;
    const BvhNode *nodes;
    const Item *items;    // all levels, level l at [lev_off[l], lev_off[l+1])
    const uint4 *qitems;  // the same items quantized (see kQMax), or nullptr
    float q_org[3], q_scale[3];  // quantization frame: q = (x - q_org) * q_scale
    double tf[12];        // R1 (row-major) + T1: parseTransform of "Environment Location"
    float root_lo[3], root_hi[3];  // root box (float, widened)
    int32_t n_tris;
    int32_t n_nodes;
    int32_t n_levels;
    int32_t lev_off[kMaxLevels + 1];
};

// Work description for one collide launch.  Units are (pose, link) pairs.
//  mode A (host API): pose_edge[p] gives the edge of pose p; units = n_poses * L.
//  mode B (engine):   edge e owns pose slots [e*pmax, e*pmax + pcount[e]);
//                     units = n_edges * pmax * L, slots past pcount are skipped.
struct CollideWork {
    const double *poses;      // [slots][L][12]
    const int32_t *pose_edge; // mode A, else nullptr
    const int32_t *pcount;    // mode B
    int32_t pmax;             // mode B
    int32_t L;
    int64_t n_units;
    uint8_t *verdict;         // [E], 0-initialised by the launcher, set to 1 on contact
    // optional [8]: units run, clusters visited, node visits, SAT tests, max node visits of
    // one unit, max / sum wave lifetime (s_memtime), broad-phase candidates
    unsigned long long *stats;
    // fused kernel only: run just the units listed here (count read on the device)
    const int32_t *unit_list;
    const uint32_t *unit_list_n;
    // two-phase path, optional: the units whose whole-link box meets the env root box
    // (FCL's object-level AABB test, done by the producer of the poses); k_pairs then runs
    // (live unit, cluster) threads only.  Any order; n_live read on the device.
    const int32_t *live_units;
    const uint32_t *n_live;
    // two-phase path, optional: each unit's FCL relative transform [slots][L][12] (R row-major,
    // then T), computed by the producer of the poses exactly as unit_transform does, so the
    // stages load it instead of recomputing it per (unit, cluster), header and candidate
    const double *unit_rt;
    // two-phase path, optional (with live_units, two-level quantized env trees): each unit's
    // mask of the top-level items its whole-link box meets (top_item_mask), by unit index
    const uint64_t *unit_tmask;
};

// Broad-phase candidate: (unit, agent triangle, env triangle) whose float boxes overlap.
struct Cand {
    int32_t unit;
    int32_t atri;
    int32_t etri;
};

// (unit, agent cluster) whose box overlaps n env triangles' boxes; the triangle indices
// are pairs[p0, p0 + n) of the same wave segment.
// Pairs are packed (lane << 26 | env triangle) words in the k_pairs wave's segment, in
// append order; a header names its lane.
struct PairHdr {
    int32_t unit;
    int32_t cluster;
    int32_t seg;     // k_pairs wave segment holding the pairs
    int32_t n;       // pairs of this (unit, cluster)
    int32_t tfirst;  // the cluster's agent triangles
    int32_t tcount;
    int32_t lane;    // k_pairs lane that made them
    int32_t pad;
};
constexpr int kPairTriBits = 26;  // env triangles per env < 2^26 on the split path

void hip_check(hipError_t e, const char *what);
// Device state of a single-launch decoupled-look-back scan (scan.h): per-tile status words
// (epoch-tagged, never reset) and a monotone tile ticket.
struct ScanState {
    unsigned long long *status = nullptr;  // [cap_tiles]
    unsigned long long *ticket = nullptr;  // [1], monotone
    int64_t cap_tiles = 0;
    uint32_t epoch = 0;      // of the last launch (1..2^30-1)
    uint64_t launched = 0;   // tickets handed out by earlier launches
    ScanState() = default;
    ScanState(const ScanState &) = delete;
    ScanState &operator=(const ScanState &) = delete;
    ~ScanState() {
        if (status) (void)hipFree(status);
        if (ticket) (void)hipFree(ticket);
    }
    // allocation-time zeroing is followed by a device sync (the null stream does not order
    // with the caller's non-blocking stream)
    void reserve(int64_t tiles) {
        if (!ticket) {
            hip_check(hipMalloc(&ticket, sizeof(unsigned long long)), "scan ticket");
            hip_check(hipMemset(ticket, 0, sizeof(unsigned long long)), "scan ticket zero");
            hip_check(hipDeviceSynchronize(), "scan ticket sync");
            launched = 0;
        }
        if (tiles > cap_tiles) {
            if (status) hip_check(hipFree(status), "free");
            cap_tiles = (tiles > 2 * cap_tiles ? tiles : 2 * cap_tiles);
            hip_check(hipMalloc(&status, sizeof(unsigned long long) * cap_tiles), "scan status");
            hip_check(hipMemset(status, 0, sizeof(unsigned long long) * cap_tiles), "scan status zero");
            hip_check(hipDeviceSynchronize(), "scan status sync");
            epoch = 0;
        }
    }
};

// Device scratch of the two-phase collide path (broad.hip).  Every stage writes to fixed
// per-wave segments (no device-wide atomics on the hot path); what does not fit goes to
// the shared spill list, and units that overflow even that are re-run by the fused kernel.
struct CollideScratch {
    int32_t *pairs = nullptr;       // [n_seg][pair_cap]   env triangle per (unit, cluster) pair
    PairHdr *hdr = nullptr;         // [n_seg][64]
    uint32_t *hdr_count = nullptr;  // [n_seg + 1], exclusive-scanned into hdr_off
    uint32_t *pair_count = nullptr; // [n_seg] pairs written per segment
    uint32_t *hdr_off = nullptr;    // [n_seg + 1]
    int32_t *hdr_dense = nullptr;   // [n_seg * 64] header slots in dense order
    ScanState hdr_scan;             // header counts -> hdr_off + hdr_dense (one launch)
    Cand *cand = nullptr;           // [n_cwaves][cand_cap]
    uint32_t *cand_count = nullptr; // [n_cwaves]
    Cand *spill = nullptr;          // [spill_cap] shared overflow of full candidate segments
    uint32_t *ctl = nullptr;        // 2 x [4]: [1] overflow units, [2] spill count (double-buffered)
    int32_t ctl_par = 0;            // the half the next launch uses
    int32_t *ovf_list = nullptr;    // [ovf_cap]
    int64_t ovf_cap = 0, n_seg = 0;
    int32_t pair_cap = 0, cand_cap = 0, spill_cap = 0, n_cwaves = 0;
    CollideScratch() = default;
    CollideScratch(const CollideScratch &) = delete;
    CollideScratch &operator=(const CollideScratch &) = delete;
    ~CollideScratch();
    // allocates on first use / growth (not stream-ordered); max_clusters over the links
    void ensure(int64_t n_units, int32_t max_clusters);
};

// Fused single-kernel path (one wave per unit, BVH walk + SAT at the leaves).
// max_blocks > 0 caps the grid (list mode re-runs, usually empty).
void launch_collide(const EnvDev &env, const AgentDev *d_links, const CollideWork &w,
                    hipStream_t stream, int max_blocks = 0);
// Two-phase path (broad.hip): k_pairs -> k_cands -> k_narrow -> fused kernel over
// overflowed units.  s.ensure(w.n_units, max_clusters) must have run with the same value.
// marks (optional, 3 events): recorded after the pair, candidate and exact-test stages.
// What the last stage of the two-phase path (the fused re-run of overflowed units, k_overflow)
// needs, for a caller that runs it inside its own next launch instead (the engine's append:
// one launch less per round; see rrt_engine.hip k_append_commit).
struct OvfDefer {
    EnvDev env{};
    const AgentDev *links = nullptr;
    CollideWork w{};
    const uint32_t *n_ovf = nullptr;  // nullptr: nothing deferred
    const int32_t *ovf_list = nullptr;
};
// defer (optional): filled instead of launching k_overflow when the batch runs in one chunk
// (otherwise defer->n_ovf stays nullptr and k_overflow runs as usual).
// units one launch of the two-phase path takes (larger batches run in chunks, without the
// live-unit list)
int64_t collide_chunk_units(int32_t max_clusters);
void launch_collide_split(const EnvDev &env, const AgentDev *d_links, int32_t max_clusters, const CollideWork &w,
                          CollideScratch &s, hipStream_t stream, hipEvent_t *marks = nullptr,
                          OvfDefer *defer = nullptr);
void launch_pose_edge(const int64_t *d_offsets, int64_t E, int32_t *d_pose_edge, hipStream_t stream);

// Edges whose poses share one rotation and translate along a segment (sweep.hip): PRM roadmap
// edges, their poses generated in-kernel from the milestones' keys (prm_edges.h PrmEdges; no
// pose array); one wave an edge (one an (edge, cluster) beyond 64 clusters) of the single link
// d_link[0]; verdict[E] must be zeroed.  stats (optional [4]): waves, env item tests, (pair,
// pose) gate tests, SAT tests.
struct PrmEdges;
// the calling thread's last two-phase sweep: candidates emitted, edges deferred
extern thread_local uint64_t last_sweep_counts[2];
extern thread_local std::vector<int32_t> last_sweep_deferred;
extern int64_t sweep_queue_cap_limit;  // mpt_set_sweep_queue_cap (0: the sized queue)
void launch_collide_sweep_prm(const EnvDev &env, const AgentDev *d_link, int32_t n_clusters, const PrmEdges &edges,
                              int64_t E, uint8_t *verdict, unsigned long long *stats, hipStream_t stream);

// Self-collision (self.hip, MeshHandler::isInCollision's checkSelfCollision branch): units
// are (pose, link pair j < k); verdict[pose_edge[p]] = 1 when links j and k of pose p touch.
void launch_self_collide(const AgentDev *d_links, int32_t L, const double *poses, const int32_t *pose_edge,
                         int64_t n_poses, uint8_t *verdict, hipStream_t stream);

// PRMLite edges (sweep.hip): all pairs i < j of verts [V][12] (R|T), hit[V(V-1)/2] zeroed.
void launch_prmlite_edges(const EnvDev &env, const AgentDev *d_link, int32_t n_clusters, const double *verts, int64_t V,
                          double step, uint8_t *hit, unsigned long long *stats, hipStream_t stream);

// ---------------- distance (distance.hip) ----------------
// Units are (pose, link) pairs as for collide mode A; best[E] receives the per-edge minimum
// distance as the bit pattern of a double (DBL_MAX when the edge has no poses).
struct DistWork {
    const double *poses;       // [P][L][12]
    const int32_t *pose_edge;  // [P]
    int32_t L;
    int32_t max_clusters;      // over the links
    int64_t n_units;           // P * L
    unsigned long long *best;  // [E]
    // optional [4]: agent clusters walked, env item box tests, triDistance calls, pair box tests
    unsigned long long *stats;
};
void launch_distance(const EnvDev &env, const AgentDev *d_links, const DistWork &w, int64_t E, hipStream_t stream);

// ---------------- NN ----------------
struct NNWork {
    const double *pts;       // [n][d]
    const uint8_t *removed;  // [n] or nullptr
    int64_t n;
    int32_t d;
    const double *q;         // [nq][d]
    int64_t nq;
    const int64_t *n_dev;    // optional device-resident point count (<= n); n is then an upper bound
};
// 1-NN / kNN (k <= 32): ids [nq][k] 1-based (-1 empty), d2 [nq][k] (+inf empty).
// scratch must hold nn_knn_scratch_bytes(nq, n, k) bytes.
size_t nn_knn_scratch_bytes(int64_t nq, int64_t n, int32_t k);
void launch_knn(const NNWork &w, int32_t k, int32_t *ids, double *d2, void *scratch,
                hipStream_t stream);
// radius: counts pass then fill pass; offsets [nq+1] device.  Results per query are
// sorted by (d2, id) and truncated to max_nb (> 0).  Needs the host to read the total
// between passes; returns the total.
int64_t launch_radius(const NNWork &w, double r2, int32_t max_nb, int64_t *d_offsets,
                      int32_t *d_ids, double *d2, int64_t cap, void *scratch, size_t scratch_bytes,
                      hipStream_t stream);

// ---------------- error helpers ----------------
struct Error {
    int code;
    std::string msg;
};

void hip_check(hipError_t e, const char *what);

// per-thread message returned by mpt_last_error()
std::string &last_error_ref();

// Run f(), translating exceptions into an mpt_status + last_error message.
template <class F>
int32_t guarded(F &&f) {
    try {
        f();
        return 0;
    } catch (const Error &e) {
        last_error_ref() = e.msg;
        return e.code;
    } catch (const std::exception &e) {
        last_error_ref() = e.what();
        return 5;
    } catch (...) {
        last_error_ref() = "unknown error";
        return 5;
    }
}

}  // namespace mpt
