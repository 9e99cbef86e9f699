// distance.hip -- batched mesh-vs-mesh minimum distance on gfx950.
//
// The "distance" half of the reference's FCL layer: fcl::distance between the env objects
// and the agent's (pose, link) objects, driven by the broadphase callback
// fcl_helpers::defaultDistanceFunction (utilities/fcl_helpers.hpp:67-84, DistanceData :35-42)
// over the same object sets as MeshHandler::isInCollision (meshhandler.hpp:187-243).  FCL's
// MeshDistanceTraversalNode only prunes BV pairs whose lower bound is not below the running
// minimum, so its answer is the minimum of TriangleDistance::triDistance over all triangle
// pairs (fcl_math.h tri_distance, with the box-gated overlap answer).  Per edge:
//   dist[e] = min over its poses, links and (env, agent) triangle pairs; DBL_MAX (FCL's
//   initial DistanceResult::min_distance) for an edge without poses; 0 = in contact.
//
// Mapping: one wavefront per (unit, agent cluster), one agent triangle per lane (mapped
// Q' = R Q + T exactly as for collision).  The wave walks the 64-ary env tree (EnvDev
// items) depth first: at each node the lanes test its <= 64 children's float boxes against
// the cluster's box, the nearest surviving child is entered at once and the others are
// pushed (with their lower bound) on a per-wave LDS stack; a popped entry is re-tested
// against the current bound.  At a bucket the lanes run triDistance against each of its
// env triangles, skipping pairs whose exact box gap exceeds the bound.  The running bound
// U of the edge is shared by every wave of the edge through a 64-bit atomicMin on the
// double's bit pattern (non-negative doubles order like their bits); it only prunes, so
// the result is the exact minimum whatever the interleaving.
#include <float.h>
#include <string.h>

#include "../../include/mpt.h"
#include "collide_common.h"
#include "wave_ops.h"

namespace mpt {

constexpr int kDistWaves = 4;
// Tuning constants (measured in round 3 with the run-time knobs since removed).  Queued pairs
// are evaluated when 64 wait, at a pass's end and at the seed; round 3 also flushed a bucket's
// pairs at its end once 32 waited (1 = after every bucket: 4 % slower), which with the queue
// carried over clusters costs more than it gains (blimp vs room: 16 / 32 / 48 / never: 5.96 /
// 5.72 / 5.67 / 5.57 ms, profiles/r23/ab/distance_carried_queue.json).
// the first pass's bound scale (1 = one pass).  Blimp vs room, 65 536 poses, alpha 1 / 0.7 /
// 0.5 / 0.3: 8.04 / 7.68 / 7.65 / 7.89 ms (triDistance calls 65.2 / 37.0 / 35.7 / 37.3 M); the
// reference's last submesh 3.81 / 2.43 / 2.38 / 2.55 ms.  Any value in (0, 1] is exact: see
// flush_pairs for the one invariant the second pass relies on.
constexpr double c_dist_alpha = 0.5;
// clusters the first pass walks at most: the nearest one sets the bound nearly as well as all
// of them, without their second walk (blimp: 1 / 2 / 4 / all: 6.45 / 6.54 / 6.65 / 7.65 ms,
// calls 36.4 / 36.4 / 36.3 / 35.7 M)
constexpr int32_t c_dist_passa = 1;
constexpr int kDistStack = kMaxLevels * kWave;

__device__ __forceinline__ double read_best(const unsigned long long *p) {
    return __longlong_as_double((long long)__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// Squared float bound for the widened-box tests: the boxes are widened beyond float
// rounding (fcl_math.h widen_*), the factor covers the rounding of the float sum.
__device__ __forceinline__ float prune2(double U) {
    const float u = (float)(U * (1.0 + 1e-5) + 1e-6);  // DBL_MAX -> inf
    return u * u;
}

__device__ __forceinline__ float gap2f(const float alo[3], const float ahi[3], const float *blo, const float *bhi) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float g = fmaxf(fmaxf(alo[k] - bhi[k], blo[k] - ahi[k]), 0.f);
        s += g * g;
    }
    return s;
}

// the wave reductions below run on DPP / permlane exchanges (wave_ops.h): __shfl_xor's
// ds_bpermute put an LDS round trip at each of their 6 levels, in the walk's hottest loops
__device__ __forceinline__ double wave_min_d(double v) { return wave_min_f64_dpp(v); }

struct DistCounters {
    uint32_t clusters = 0, items = 0, tri_calls = 0, pair_tests = 0;
};

// Per-wave LDS: the unit's transform, the pair queue and the DFS stack (5 KiB a wave).  The
// queue holds (env, agent) triangle indices, not a cluster's mapped triangles, so its pairs
// carry over from one cluster's walk to the next and a flush waits for 64 of them over the
// clusters (blimp vs room: 10.6 flushes a pose instead of 11.9, one part-full at the end of each
// cluster's walk; 5.77 vs 5.95 ms, profiles/r23/ab/distance_carried_queue.json); a flush maps
// its agent triangles again (27 FMAs a lane beside triDistance's ~2000 instructions).
struct DistLds {
    double rt[12];             // the unit's R (row-major) and T
    int32_t queue[2 * kWave];  // pending pairs: env triangle
    int32_t qag[2 * kWave];    // and agent triangle (index into the link's triangles)
    float qgap[2 * kWave];     // their squared box gaps, rounded down (re-tested at the flush)
    int32_t stk_il[kDistStack];  // item << 3 | level (kMaxLevels <= 8)
    float stk_b[kDistStack];
};
static_assert(kMaxLevels <= 8, "stack entries pack the level in 3 bits");

// Exact triangle distances of the queued pairs, one pair per lane; returns the new bound.
template <int kOcc, bool kSel>
__device__ __forceinline__ double flush_pairs(const EnvDev &env, const double *atris, DistLds &s, int n, int lane,
                                              double U, unsigned long long *bp, DistCounters &cnt) {
    double d = DBL_MAX;
    // a pair queued against an older bound is re-tested against the current one (its gap
    // rounded down: never drops a pair the exact test keeps).  This threshold must stay the
    // full bound U, never alpha * U: the second pass (distance_unit) skips the first pass's
    // pairs with a gap <= alpha * U_A on the grounds that the first pass evaluated every one of
    // them, and a pair dropped here against alpha * U would then be lost.
    const double Un = uniform_d(dmin(U, read_best(bp)));
    const double thr = Un * (1.0 + 1e-9) + 1e-9;
    const bool ev = lane < n && (double)s.qgap[lane] <= thr * thr;
    if (ev) {
        const EnvTri &E = env.tris[s.queue[lane]];
        const double *q = atris + (int64_t)s.qag[lane] * 9;
        // Q' = R Q + T exactly as the walk mapped the triangle (and as FCL does)
        const double *R = s.rt, *T = s.rt + 9;
        const v3 Q[3] = {xform(R, T, mk(q[0], q[1], q[2])), xform(R, T, mk(q[3], q[4], q[5])),
                         xform(R, T, mk(q[6], q[7], q[8]))};
        const v3 S[3] = {mk(E.P1[0], E.P1[1], E.P1[2]), mk(E.P2[0], E.P2[1], E.P2[2]), mk(E.P3[0], E.P3[1], E.P3[2])};
        // at 4 waves per SIMD the rolled form (128 VGPRs); else the unrolled one
        d = tri_distance<kOcc >= 4 ? 1 : 3, kSel>(S, E.lo, E.hi, Q);
    }
    cnt.tri_calls += (uint32_t)__popcll(__ballot(ev));
    const double wb = wave_min_d(d);
    if (wb < U) {
        if (lane == 0) atomicMin(bp, (unsigned long long)__double_as_longlong(wb));
        U = wb;
    }
    return uniform_d(dmin(U, read_best(bp)));
}

// Depth-first walk of the env tree for one agent cluster (box cblo/cbhi, lane's agent
// triangle ai with box qlo/qhi), nearest child first; pairs that survive the exact box-gap
// test are queued (qn pending, left for the next cluster's walk or the pass's end) and
// evaluated 64 at a time.  Returns the updated bound.
template <int kOcc, bool kSel>
__device__ double walk_cluster(const EnvDev &env, const double *atris, DistLds &s, int &qn, const float cblo[3],
                               const float cbhi[3], bool act, int32_t ai, const double qlo[3], const double qhi[3],
                               const double xlo[3], const double xhi[3], int lane, double U, unsigned long long *bp,
                               DistCounters &cnt, double alpha, double lo2) {
    int sp = 0;
    int lev = env.n_levels - 1;
    int32_t first = env.lev_off[lev];
    int32_t count = env.lev_off[lev + 1] - first;
    for (;;) {
        const float Uf2 = prune2(alpha * U);
        float lb = __builtin_huge_valf();
        int32_t cf = 0, cc = 0;
        bool keep = false;
        if (lane < count) {
            const Item it = env.items[first + lane];
            lb = gap2f(cblo, cbhi, it.lo, it.hi);
            keep = lb <= Uf2;
            cf = it.first;
            cc = it.count;
        }
        cnt.items += (uint32_t)count;
        uint64_t m = __ballot(keep);
        if (lev == 1) {
            while (m) {
                const int j = __ffsll((unsigned long long)m) - 1;
                m &= m - 1;
                if (lane_f(lb, j) > prune2(alpha * U)) continue;
                const int32_t bf = __builtin_amdgcn_readlane(cf, j);
                const int32_t bc = __builtin_amdgcn_readlane(cc, j);
                int32_t seed_t = -1;
                if (U == DBL_MAX) {
                    // first bucket of the edge: bound from one pair per agent triangle, its
                    // env triangle of smallest box gap, before the gap test can prune anything
                    double best_g2 = DBL_MAX;
                    for (int32_t t = bf; t < bf + bc; ++t) {
                        const EnvTri &E = env.tris[t];
                        double g2 = 0.0;
#pragma unroll
                        for (int k = 0; k < 3; ++k) {
                            const double g = dmax(dmax(E.lo[k] - qhi[k], qlo[k] - E.hi[k]), 0.0);
                            g2 += g * g;
                        }
                        if (g2 < best_g2) {
                            best_g2 = g2;
                            seed_t = t;
                        }
                    }
                    if (!act) seed_t = -1;
                    const uint64_t pm = __ballot(act);
                    if (act) {
                        const int pos = (int)__popcll(pm & ((1ull << lane) - 1));
                        s.queue[pos] = seed_t;
                        s.qag[pos] = ai;
                        s.qgap[pos] = 0.0f;
                    }
                    U = flush_pairs<kOcc, kSel>(env, atris, s, (int)__popcll(pm), lane, U, bp, cnt);
                    if (U == 0.0) return U;
                }
                // the bucket's env triangles whose exact box is within the bound of the cluster's
                // exact box (xlo / xhi: the union of the lanes' triangle boxes), one per lane; a
                // pair of any other triangle has a box gap above the bound (no lane would pass)
                uint64_t tm;
                {
                    const double thr = alpha * U * (1.0 + 1e-9) + 1e-9;
                    bool near = false;
                    if (lane < bc) {
                        const EnvTri &E = env.tris[bf + lane];
                        double g2 = 0.0;
#pragma unroll
                        for (int k = 0; k < 3; ++k) {
                            const double g = dmax(dmax(E.lo[k] - xhi[k], xlo[k] - E.hi[k]), 0.0);
                            g2 += g * g;
                        }
                        near = g2 <= thr * thr;
                    }
                    tm = __ballot(near);
                }
                while (tm) {
                    const int32_t t = bf + __ffsll((unsigned long long)tm) - 1;
                    tm &= tm - 1;
                    const EnvTri &E = env.tris[t];
                    const double thr = alpha * U * (1.0 + 1e-9) + 1e-9;
                    double g2 = 0.0;
#pragma unroll
                    for (int k = 0; k < 3; ++k) {
                        const double g = dmax(dmax(E.lo[k] - qhi[k], qlo[k] - E.hi[k]), 0.0);
                        g2 += g * g;
                    }
                    const bool pass = act && t != seed_t && g2 <= thr * thr && g2 > lo2;
                    const uint64_t pm = __ballot(pass);
                    if (pass) {
                        const int pos = qn + (int)__popcll(pm & ((1ull << lane) - 1));
                        s.queue[pos] = t;
                        s.qag[pos] = ai;
                        s.qgap[pos] = __double2float_rd(g2);
                    }
                    qn += (int)__popcll(pm);
                    cnt.pair_tests += (uint32_t)__popcll(__ballot(act));
                    if (qn >= kWave) {
                        U = flush_pairs<kOcc, kSel>(env, atris, s, kWave, lane, U, bp, cnt);
                        qn -= kWave;
                        if (lane < qn) {
                            s.queue[lane] = s.queue[kWave + lane];
                            s.qag[lane] = s.qag[kWave + lane];
                            s.qgap[lane] = s.qgap[kWave + lane];
                        }
                        if (U == 0.0) return U;
                    }
                }
            }
        } else if (m) {
            // enter the nearest surviving child now, push the others
            float v = keep ? lb : __builtin_huge_valf();
            int idx = lane;
            wave_argmin_f32_dpp(v, idx);
            const int j = __builtin_amdgcn_readfirstlane(idx);
            const uint64_t rest = m & ~(1ull << j);
            if (keep && lane != j) {
                const int pos = sp + (int)__popcll(rest & ((1ull << lane) - 1));
                s.stk_il[pos] = ((first + lane) << 3) | lev;
                s.stk_b[pos] = lb;
            }
            sp += (int)__popcll(rest);
            first = __builtin_amdgcn_readlane(cf, j);
            count = __builtin_amdgcn_readlane(cc, j);
            lev -= 1;
            continue;
        }
        // pop the next pending subtree that can still hold the minimum
        const float Uf2p = prune2(alpha * U);
        bool found = false;
        while (sp > 0) {
            --sp;
            if (s.stk_b[sp] <= Uf2p) {
                const int32_t il = s.stk_il[sp];
                const Item it = env.items[il >> 3];
                first = __builtin_amdgcn_readfirstlane(it.first);
                count = __builtin_amdgcn_readfirstlane(it.count);
                lev = __builtin_amdgcn_readfirstlane((il & 7) - 1);
                found = true;
                break;
            }
        }
        if (!found) return U;  // the pending pairs wait for the next cluster's
    }
}

// One wave per (pose, link) unit: clusters in increasing order of their lower bound over
// the env tree's top level, each walked with the bound the earlier ones left.
template <int kOcc, bool kSel>
__device__ void distance_unit(const EnvDev &env, const AgentDev *__restrict__ links, const DistWork &w, int64_t unit,
                              int lane, DistLds &s, DistCounters &cnt) {
    const int32_t L = w.L;
    const int32_t link = (int32_t)(unit % L);
    const int64_t slot = unit / L;
    const int64_t edge = w.pose_edge[slot];
    const AgentDev ag = links[link];
    unsigned long long *bp = w.best + edge;
    double U = uniform_d(read_best(bp));
    if (U == 0.0) return;  // defaultDistanceFunction stops at dist <= 0

    {
        double R[9], T[3];
        unit_transform(env, w.poses + (slot * L + link) * 12, R, T);
        if (lane == 0) {
#pragma unroll
            for (int i = 0; i < 9; ++i) s.rt[i] = R[i];
#pragma unroll
            for (int i = 0; i < 3; ++i) s.rt[9 + i] = T[i];
        }
        __builtin_amdgcn_wave_barrier();  // lane 0's stores before every lane's reads (one wave's LDS)
    }
    const double *R = s.rt, *T = s.rt + 9;
    const double *atris = ag.tris;
    int qn = 0;  // pending pairs, carried from one cluster's walk to the next
    const int top = env.n_levels - 1;
    const int32_t tfirst = env.lev_off[top], tcount = env.lev_off[top + 1] - tfirst;

    for (int32_t cbase = 0; cbase < ag.n_clusters; cbase += kWave) {
        const int32_t ci = cbase + lane;
        float clo[3] = {0, 0, 0}, chi[3] = {0, 0, 0};
        float clb = __builtin_huge_valf();
        if (ci < ag.n_clusters) {
            const Cluster c = ag.clusters[ci];
            local_box(c.c, c.e, R, T, clo, chi);
            for (int32_t i = 0; i < tcount; ++i) {
                const Item it = env.items[tfirst + i];
                clb = fminf(clb, gap2f(clo, chi, it.lo, it.hi));
            }
        }
        // Two passes (c_dist_alpha < 1): the first walks the nearest cluster(s) against alpha * U (its
        // nodes pruned and its pairs queued on that tighter bound), so the pairs nearest to the
        // unit are evaluated first and the bound falls to near its final value; the second walks
        // against U for the pairs the first left, those with a gap above alpha * U_A (U_A the
        // bound after the first; every pair the first queued had a gap at most alpha * U(t)
        // with U(t) >= U_A, so none is skipped).  One pass evaluated ~5x the pairs whose gap is
        // within the final distance, most of them against a bound still far from it.
        const int npass = c_dist_alpha < 1.0 ? 2 : 1;
        double lo2 = -1.0;
        uint64_t first_walked = 0;  // the clusters the first pass walked (only their pairs are excluded)
        for (int pass = 0; pass < npass; ++pass) {
        const double alpha = pass == 0 && npass == 2 ? c_dist_alpha : 1.0;
        uint64_t rem = __ballot(ci < ag.n_clusters);
        int32_t walked = 0;
        while (rem) {
            if (pass == 0 && npass == 2 && walked >= c_dist_passa) break;
            ++walked;
            // nearest remaining cluster first
            float v = (rem >> lane) & 1 ? clb : __builtin_huge_valf();
            int idx = lane;
            wave_argmin_f32_dpp(v, idx);
            const int j = __builtin_amdgcn_readfirstlane(idx);
            rem &= ~(1ull << j);
            if (lane_f(clb, j) > prune2(alpha * U)) break;  // the rest are farther still
            if (pass == 0) first_walked |= 1ull << j;
            ++cnt.clusters;
            float cblo[3], cbhi[3];
#pragma unroll
            for (int k = 0; k < 3; ++k) {  // wave-uniform: scalar registers
                cblo[k] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(clo[k]), j));
                cbhi[k] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(chi[k]), j));
            }
            const Cluster c = ag.clusters[cbase + j];
            const bool act = lane < c.count;
            const int32_t ai = c.first + lane;
            double qlo[3] = {0, 0, 0}, qhi[3] = {0, 0, 0};
            if (act) {
                const double *t = ag.tris + (int64_t)ai * 9;
                v3 Q[3];
#pragma unroll
                for (int k = 0; k < 3; ++k) Q[k] = xform(R, T, mk(t[3 * k], t[3 * k + 1], t[3 * k + 2]));
                qlo[0] = dmin(Q[0].x, dmin(Q[1].x, Q[2].x));
                qlo[1] = dmin(Q[0].y, dmin(Q[1].y, Q[2].y));
                qlo[2] = dmin(Q[0].z, dmin(Q[1].z, Q[2].z));
                qhi[0] = dmax(Q[0].x, dmax(Q[1].x, Q[2].x));
                qhi[1] = dmax(Q[0].y, dmax(Q[1].y, Q[2].y));
                qhi[2] = dmax(Q[0].z, dmax(Q[1].z, Q[2].z));
            }
            // the cluster's exact box: the union of its lanes' triangle boxes
            double xlo[3], xhi[3];
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                xlo[k] = uniform_d(wave_min_f64_dpp(act ? qlo[k] : DBL_MAX));
                xhi[k] = uniform_d(wave_max_f64_dpp(act ? qhi[k] : -DBL_MAX));
            }
            U = walk_cluster<kOcc, kSel>(env, atris, s, qn, cblo, cbhi, act, ai, qlo, qhi, xlo, xhi, lane, U, bp, cnt,
                                         alpha, pass == 1 && ((first_walked >> j) & 1) ? lo2 : -1.0);
            if (U == 0.0) return;
        }
        // every pair of the pass evaluated before the next (the second pass's lo2 relies on it)
        if (qn > 0) {
            U = flush_pairs<kOcc, kSel>(env, atris, s, qn, lane, U, bp, cnt);
            qn = 0;
            if (U == 0.0) return;
        }
        if (pass == 0 && npass == 2) {
            const double ua = c_dist_alpha * U;
            lo2 = ua * ua * (1.0 - 1e-12);  // below every first-pass threshold (rounding margin)
        }
        }
    }
}

// kOcc workgroups per CU.  3 (the one instantiated): the
// unrolled triDistance under 168 VGPRs, 3 waves per SIMD (5 dwords spilled): blimp in the room
// 10.4 -> 7.8 ms against 2 (the unconstrained allocation, 178 VGPRs since triDistance no longer
// holds S and T beside their rotating copies).  4: the rolled triDistance under 128 VGPRs
// spills ~100 dwords and 51 scalars (the walk's state is ~55 VGPRs beside triDistance's 112):
// 9.3 ms.
template <int kOcc, bool kSel>
__global__ __launch_bounds__(kDistWaves * 64, kOcc) void k_distance(EnvDev env, const AgentDev *__restrict__ links,
                                                                 DistWork w) {
    __shared__ DistLds s_lds[kDistWaves];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int64_t unit = (int64_t)blockIdx.x * kDistWaves + wave;
    DistCounters cnt;
    if (unit < w.n_units) distance_unit<kOcc, kSel>(env, links, w, unit, lane, s_lds[wave], cnt);
    if (w.stats && lane == 0 && unit < w.n_units) {
        atomicAdd(w.stats + 0, (unsigned long long)cnt.clusters);
        atomicAdd(w.stats + 1, (unsigned long long)cnt.items);
        atomicAdd(w.stats + 2, (unsigned long long)cnt.tri_calls);
        atomicAdd(w.stats + 3, (unsigned long long)cnt.pair_tests);
    }
}

__global__ void k_fill_u64(unsigned long long *p, int64_t n, unsigned long long v) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}

void launch_distance(const EnvDev &env, const AgentDev *d_links, const DistWork &w, int64_t E, hipStream_t stream) {
    if (E <= 0) return;
    const double dmax_v = DBL_MAX;
    unsigned long long inf_bits;
    memcpy(&inf_bits, &dmax_v, sizeof inf_bits);
    hipLaunchKernelGGL(k_fill_u64, dim3((unsigned)((E + 255) / 256)), dim3(256), 0, stream, w.best, E, inf_bits);
    hip_check(hipGetLastError(), "k_fill_u64 launch");
    if (w.n_units <= 0 || env.n_tris <= 0) return;
    const int64_t blocks = (w.n_units + kDistWaves - 1) / kDistWaves;
    if (blocks > 0x7fffffff) throw Error{MPT_ERR_INVALID, "distance batch too large"};
    // 3 workgroups per CU and the branch-free segPoints (seg_points_sel: the same values as the
    // branchy form; blimp vs room 12.4 -> 10.1 ms)
    hipLaunchKernelGGL((k_distance<3, true>), dim3((unsigned)blocks), dim3(kDistWaves * 64), 0, stream, env, d_links, w);
    hip_check(hipGetLastError(), "k_distance launch");
}

}  // namespace mpt
