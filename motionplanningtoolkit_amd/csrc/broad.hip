// broad.hip -- the two-phase collision path (default structure, mpt_set_collide_mode).
//
// Same verdicts as the fused kernel (collide.hip): exists (pose, link, env tri, agent tri)
// with overlapping exact boxes (tri_gate) and intersect_Triangle true.  Work is split so
// that neither phase carries the other's registers:
//
// k_broad  one wave per (pose, link) unit (static first chunk per wave, then an atomic
//          work queue).  Lanes = agent clusters: each lane maps its cluster's local box
//          (FP64, R T from fcl::relativeTransform) to a widened float box, culled against
//          the env root box.  For each surviving cluster the wave walks the 64-ary env
//          tree (mpt_internal.h Item) with that box: at a node, lane i tests child i, the
//          ballot is the set of children to enter; the walk state (mask, base, level) is a
//          few SGPRs with the pending levels in lane-indexed VGPRs.  When a bucket's
//          triangles overlap the cluster box, lanes = the cluster's agent triangles, each
//          mapped exactly and boxed once per cluster (lazily), and every (lane, env tri)
//          box overlap is written as a candidate to the wave's own segment.
// k_narrow one 64-lane workgroup per segment, one candidate per lane: the exact transform of
//          the agent triangle, tri_gate, intersect_Triangle; verdict[edge] = 1 on contact.
// Units whose candidates do not fit their segment are listed and re-run by the fused kernel.
#include "collide_common.h"

namespace mpt {

constexpr int kBroadWaves = 8;     // waves per workgroup
constexpr int kChunk = 4;          // units per queue grab (one pre-pass lane each)
constexpr int kSegCap = 1024;      // candidates per wave segment
constexpr int kLdsItems = 2048;    // whole env tree staged in LDS (64 KiB) when it fits

constexpr int kSpillCap = 1 << 22;  // shared spill list (48 MiB)
constexpr int kSpillBlocks = 256;   // k_narrow workgroups over the spill list

struct BroadArgs {
    Cand *cand;
    uint32_t *seg_count;
    Cand *spill;
    uint32_t *ctl;
    int32_t *ovf_list;
    int32_t seg_cap;
    int32_t n_waves;
    int32_t spill_cap;
};

// Append the lanes of h (ballot m) as candidates: to the wave's segment, or once that is
// full to the shared spill list; false if both are full.  Called with all lanes active.
__device__ __forceinline__ bool emit(bool h, uint64_t m, int32_t unit, int32_t atri, int32_t etri, Cand *seg,
                                     uint32_t &cnt, uint32_t cap, const BroadArgs &b) {
    const uint32_t n = (uint32_t)__popcll(m);
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    if (cnt + n <= cap) {
        if (h) seg[cnt + rank] = Cand{unit, atri, etri};
        cnt += n;
        return true;
    }
    uint32_t base = 0;
    if ((threadIdx.x & 63) == 0) base = atomicAdd(b.ctl + 2, n);
    base = __builtin_amdgcn_readfirstlane(base);
    if (base + n > (uint32_t)b.spill_cap) return false;
    if (h) b.spill[base + rank] = Cand{unit, atri, etri};
    return true;
}

// Children [first, first + count) of a node (absolute item indices): lane i tests child i
// against the query box; returns the ballot, the lane keeps its child's box in `mine`.
template <bool kLds>
__device__ __forceinline__ uint64_t visit(const Item *s_items, const Item *__restrict__ items, int32_t first,
                                          int32_t count, const float qlo[3], const float qhi[3], int lane,
                                          Item &mine) {
    bool h = false;
    if (lane < count) {
        mine = kLds ? s_items[first + lane] : items[first + lane];
        h = box_overlap(qlo, qhi, mine.lo, mine.hi);
    }
    return __ballot(h);
}

// (first, count) of one item, wave-uniform index.
template <bool kLds>
__device__ __forceinline__ void item_range(const Item *s_items, const Item *__restrict__ items, int32_t idx,
                                           int32_t &first, int32_t &count) {
    if (kLds) {
        first = __builtin_amdgcn_readfirstlane(s_items[idx].first);
        count = __builtin_amdgcn_readfirstlane(s_items[idx].count);
    } else {
#if defined(__HIP_DEVICE_COMPILE__)
        typedef __attribute__((address_space(4))) const Item *cptr;  // scalar cache, s_load
        const Item *g = items;
        first = ((cptr)g)[idx].first;
        count = ((cptr)g)[idx].count;
#else
        first = items[idx].first;
        count = items[idx].count;
#endif
    }
}

// One item, wave-uniform index (LDS broadcast read, or the scalar cache).
template <bool kLds>
__device__ __forceinline__ Item load_item_u(const Item *s_items, const Item *__restrict__ items, int32_t idx) {
    if (kLds) return s_items[idx];
#if defined(__HIP_DEVICE_COMPILE__)
    typedef __attribute__((address_space(4))) const Item *cptr;
    const Item *g = items;
    return ((cptr)g)[idx];
#else
    return items[idx];
#endif
}

__device__ __forceinline__ float lane_f(float v, int j) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), j));
}

__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = fminf(v, __shfl_xor(v, off));
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off));
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}

// One unit whose whole-link box passed the root cull; R, T wave-uniform.  False on
// candidate overflow (the unit is then re-run by the fused kernel).
template <bool kLds>
__device__ bool broad_unit(const EnvDev &env, const Item *s_items, const AgentDev &ag, const double R[9],
                           const double T[3], const BroadArgs &b, int32_t unit, int lane, Cand *seg,
                           uint32_t &cnt, uint32_t cap, uint32_t &n_clusters, uint32_t &n_nodes,
                           uint32_t &n_pairs, uint32_t &n_xf) {
    const int32_t top = env.n_levels - 1;
    const int32_t top_off = env.lev_off[top];
    const int32_t n_top = env.lev_off[top + 1] - top_off;
    for (int32_t cbase = 0; cbase < ag.n_clusters; cbase += kWave) {
        float clo[3] = {0, 0, 0}, chi[3] = {0, 0, 0};
        bool ok = false;
        int32_t cf = 0, cc = 0;
        if (cbase + lane < ag.n_clusters) {
            const Cluster &c = ag.clusters[cbase + lane];
            local_box(c.c, c.e, R, T, clo, chi);
            ok = box_overlap(clo, chi, env.root_lo, env.root_hi);
            cf = c.first;
            cc = c.count;
        }
        uint64_t cm = __ballot(ok);
        if (!cm) continue;
        if (top == 1) {
            // Two-level tree (top items = buckets of triangles): lanes = clusters test every
            // bucket box in one pass (lane keeps a bucket bitmask), then cluster by cluster
            // the overlapping buckets' triangles, lanes = triangles.
            uint64_t bm = 0;
            for (int32_t i = 0; i < n_top; ++i) {
                const Item t = load_item_u<kLds>(s_items, env.items, top_off + i);
                bm |= (uint64_t)(ok && box_overlap(clo, chi, t.lo, t.hi)) << i;
            }
            n_nodes += (uint32_t)n_top;
            uint64_t cm2 = __ballot(bm != 0);
            while (cm2) {
                const int j = __ffsll((unsigned long long)cm2) - 1;
                cm2 &= cm2 - 1;
                ++n_clusters;
                uint64_t B = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int32_t)(uint32_t)(bm >> 32), j) << 32) |
                             (uint32_t)__builtin_amdgcn_readlane((int32_t)(uint32_t)bm, j);
                const float qlo[3] = {lane_f(clo[0], j), lane_f(clo[1], j), lane_f(clo[2], j)};
                const float qhi[3] = {lane_f(chi[0], j), lane_f(chi[1], j), lane_f(chi[2], j)};
                const int32_t tfirst = __builtin_amdgcn_readlane(cf, j);
                const int32_t tcount = __builtin_amdgcn_readlane(cc, j);
                const bool act = lane < tcount;
                bool have = false;
                float blo[3] = {0, 0, 0}, bhi[3] = {0, 0, 0}, tlo[3] = {0, 0, 0}, thi[3] = {0, 0, 0};
                while (B) {
                    const int i = __ffsll((unsigned long long)B) - 1;
                    B &= B - 1;
                    int32_t first, count;
                    item_range<kLds>(s_items, env.items, top_off + i, first, count);
                    Item mine{};
                    uint64_t M = visit<kLds>(s_items, env.items, first, count, qlo, qhi, lane, mine);
                    ++n_nodes;
                    if (!M) continue;
                    if (!have) {
                        if (act) agent_tri_box(ag.tris + (int64_t)(tfirst + lane) * 9, R, T, blo, bhi);
                        have = true;
                        ++n_xf;
#pragma unroll
                        for (int k = 0; k < 3; ++k) {
                            tlo[k] = wave_min(act ? blo[k] : __builtin_huge_valf());
                            thi[k] = wave_max(act ? bhi[k] : -__builtin_huge_valf());
                        }
                    }
                    M &= __ballot(box_overlap(tlo, thi, mine.lo, mine.hi));
                    n_pairs += (uint32_t)__popcll(M);
                    while (M) {
                        const int t = __ffsll((unsigned long long)M) - 1;
                        M &= M - 1;
                        const float elo[3] = {lane_f(mine.lo[0], t), lane_f(mine.lo[1], t), lane_f(mine.lo[2], t)};
                        const float ehi[3] = {lane_f(mine.hi[0], t), lane_f(mine.hi[1], t), lane_f(mine.hi[2], t)};
                        const bool h = act && box_overlap(blo, bhi, elo, ehi);
                        const uint64_t m = __ballot(h);
                        if (m && !emit(h, m, unit, tfirst + lane, first + t, seg, cnt, cap, b)) return false;
                    }
                }
            }
            continue;
        }
        while (cm) {
            const int j = __ffsll((unsigned long long)cm) - 1;
            cm &= cm - 1;
            ++n_clusters;
            const float qlo[3] = {lane_f(clo[0], j), lane_f(clo[1], j), lane_f(clo[2], j)};
            const float qhi[3] = {lane_f(chi[0], j), lane_f(chi[1], j), lane_f(chi[2], j)};
            const int32_t tfirst = __builtin_amdgcn_readfirstlane(ag.clusters[cbase + j].first);
            const int32_t tcount = __builtin_amdgcn_readfirstlane(ag.clusters[cbase + j].count);
            const bool act = lane < tcount;
            bool have = false;  // agent triangle boxes of this cluster computed
            float blo[3] = {0, 0, 0}, bhi[3] = {0, 0, 0};
            float tlo[3] = {0, 0, 0}, thi[3] = {0, 0, 0};  // their union (tighter than the cluster box)

            Item mine{};
            int32_t lv = top, base = top_off;
            uint64_t M = visit<kLds>(s_items, env.items, top_off, n_top, qlo, qhi, lane, mine);
            ++n_nodes;
            int32_t sp = 0, st_mlo = 0, st_mhi = 0, st_base = 0, st_lv = 0;  // lane k = pending entry k
            for (;;) {
                if (lv == 0) {
                    // M = env triangles base + bit overlapping the cluster box
                    if (M && !have) {
                        if (act) agent_tri_box(ag.tris + (int64_t)(tfirst + lane) * 9, R, T, blo, bhi);
                        have = true;
                        ++n_xf;
#pragma unroll
                        for (int k = 0; k < 3; ++k) {
                            tlo[k] = wave_min(act ? blo[k] : __builtin_huge_valf());
                            thi[k] = wave_max(act ? bhi[k] : -__builtin_huge_valf());
                        }
                    }
                    // lanes of the last visit hold these triangles' boxes: drop those that miss
                    // the union of the agent triangle boxes
                    if (M) M &= __ballot(box_overlap(tlo, thi, mine.lo, mine.hi));
                    n_pairs += (uint32_t)__popcll(M);
                    while (M) {
                        const int t = __ffsll((unsigned long long)M) - 1;
                        M &= M - 1;
                        const float elo[3] = {lane_f(mine.lo[0], t), lane_f(mine.lo[1], t), lane_f(mine.lo[2], t)};
                        const float ehi[3] = {lane_f(mine.hi[0], t), lane_f(mine.hi[1], t), lane_f(mine.hi[2], t)};
                        const bool h = act && box_overlap(blo, bhi, elo, ehi);
                        const uint64_t m = __ballot(h);
                        if (m && !emit(h, m, unit, tfirst + lane, base + t, seg, cnt, cap, b)) return false;
                    }
                }
                if (!M) {
                    if (sp == 0) break;
                    --sp;
                    M = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(st_mhi, sp) << 32) |
                        (uint32_t)__builtin_amdgcn_readlane(st_mlo, sp);
                    base = __builtin_amdgcn_readlane(st_base, sp);
                    lv = __builtin_amdgcn_readlane(st_lv, sp);
                    continue;
                }
                const int c = __ffsll((unsigned long long)M) - 1;
                M &= M - 1;
                int32_t cfirst, ccount;
                item_range<kLds>(s_items, env.items, base + c, cfirst, ccount);
                if (M) {  // keep the rest of this node for later
                    st_mlo = lane == sp ? (int32_t)(uint32_t)M : st_mlo;
                    st_mhi = lane == sp ? (int32_t)(uint32_t)(M >> 32) : st_mhi;
                    st_base = lane == sp ? base : st_base;
                    st_lv = lane == sp ? lv : st_lv;
                    ++sp;
                }
                --lv;
                base = cfirst;
                M = visit<kLds>(s_items, env.items, cfirst, ccount, qlo, qhi, lane, mine);
                ++n_nodes;
            }
        }
    }
    return true;
}

template <bool kLds>
__global__ __launch_bounds__(kBroadWaves * 64) void k_broad(EnvDev env, const AgentDev *__restrict__ links,
                                                             CollideWork w, BroadArgs b) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    Item *s_items = reinterpret_cast<Item *>(smem);
    if (kLds) {
        const int32_t n = env.lev_off[env.n_levels];
        const uint4 *src = reinterpret_cast<const uint4 *>(env.items);
        uint4 *dst = reinterpret_cast<uint4 *>(s_items);
        for (int i = threadIdx.x; i < n * 2; i += blockDim.x) dst[i] = src[i];
        __syncthreads();
    }
    __shared__ double s_rt[kBroadWaves][kChunk][12];  // R, T of the chunk's surviving units
    __shared__ int32_t s_link[kBroadWaves][kChunk];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform for the compiler
    const int lane = threadIdx.x & 63;
    const int32_t gw = (int32_t)blockIdx.x * kBroadWaves + wave;
    Cand *seg = b.cand + (int64_t)gw * b.seg_cap;
    const uint32_t cap = (uint32_t)b.seg_cap;
    uint32_t cnt = 0, n_units = 0, n_clusters = 0, n_nodes = 0, n_pairs = 0, n_xf = 0;
    const int64_t n_static = (int64_t)b.n_waves * kChunk;
    int64_t base = (int64_t)gw * kChunk;
    while (base < w.n_units) {
        const int64_t end = base + kChunk < w.n_units ? base + kChunk : w.n_units;
        // lane-parallel pre-pass, one lane per unit of the chunk: decode, FCL relative
        // transform, whole-link box against the env root box
        bool live = false, ok = false;
        if (lane < end - base) {
            int32_t link;
            int64_t slot, edge;
            live = decode_unit(w, base + lane, link, slot, edge);
            if (live) {
                double R[9], T[3];
                unit_transform(env, w.poses + (slot * w.L + link) * 12, R, T);
                float lo[3], hi[3];
                local_box(links[link].bc, links[link].be, R, T, lo, hi);
                ok = box_overlap(lo, hi, env.root_lo, env.root_hi);
#pragma unroll
                for (int i = 0; i < 9; ++i) s_rt[wave][lane][i] = R[i];
#pragma unroll
                for (int i = 0; i < 3; ++i) s_rt[wave][lane][9 + i] = T[i];
                s_link[wave][lane] = link;
            }
        }
        n_units += (uint32_t)__popcll(__ballot(live));
        uint64_t um = __ballot(ok);
        __builtin_amdgcn_wave_barrier();
        while (um) {
            const int j = __ffsll((unsigned long long)um) - 1;
            um &= um - 1;
            double R[9], T[3];
#pragma unroll
            for (int i = 0; i < 9; ++i) R[i] = uniform_d(s_rt[wave][j][i]);
#pragma unroll
            for (int i = 0; i < 3; ++i) T[i] = uniform_d(s_rt[wave][j][9 + i]);
            const int32_t link = __builtin_amdgcn_readfirstlane(s_link[wave][j]);
            const int32_t u = (int32_t)(base + j);
            if (!broad_unit<kLds>(env, s_items, links[link], R, T, b, u, lane, seg, cnt, cap, n_clusters, n_nodes,
                                  n_pairs, n_xf)) {
                if (lane == 0) b.ovf_list[atomicAdd(b.ctl + 1, 1u)] = u;
            }
        }
        __builtin_amdgcn_wave_barrier();
        if (n_static >= w.n_units) break;
        uint32_t nb = 0;
        if (lane == 0) nb = atomicAdd(b.ctl, 1u);
        nb = __builtin_amdgcn_readfirstlane(nb);
        base = n_static + (int64_t)nb * kChunk;
    }
    if (lane == 0) b.seg_count[gw] = cnt;
    if (w.stats && lane == 0) {
        atomicAdd(w.stats + 0, (unsigned long long)n_units);
        atomicAdd(w.stats + 1, (unsigned long long)n_clusters);
        atomicAdd(w.stats + 2, (unsigned long long)n_nodes);
        atomicAdd(w.stats + 4, (unsigned long long)n_pairs);
        atomicAdd(w.stats + 6, (unsigned long long)n_xf);
        atomicAdd(w.stats + 7, (unsigned long long)cnt);
    }
}

__device__ __forceinline__ void narrow_one(const EnvDev &env, const AgentDev *__restrict__ links,
                                           const CollideWork &w, const Cand cd, uint32_t &n_sat) {
    int32_t link;
    int64_t slot, edge;
    decode_unit(w, cd.unit, link, slot, edge);
    if (load_flag(w.verdict + edge)) return;
    double R[9], T[3];
    unit_transform(env, w.poses + (slot * w.L + link) * 12, R, T);
    const double *t = links[link].tris + (int64_t)cd.atri * 9;
    const v3 Q1 = xform(R, T, mk(t[0], t[1], t[2]));
    const v3 Q2 = xform(R, T, mk(t[3], t[4], t[5]));
    const v3 Q3 = xform(R, T, mk(t[6], t[7], t[8]));
    const EnvTri &E = env.tris[cd.etri];
    if (!tri_gate(E.lo, E.hi, Q1, Q2, Q3)) return;
    ++n_sat;
    if (tri_intersect(E, Q1, Q2, Q3))
        __hip_atomic_store(w.verdict + edge, (uint8_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Workgroups [0, n_waves): one broad segment each; the next kSpillBlocks: the spill list.
__global__ __launch_bounds__(64) void k_narrow(EnvDev env, const AgentDev *__restrict__ links, CollideWork w,
                                               BroadArgs b) {
    const int32_t gw = blockIdx.x;
    uint32_t n_sat = 0;
    if (gw < b.n_waves) {
        const uint32_t cnt = b.seg_count[gw];
        const Cand *seg = b.cand + (int64_t)gw * b.seg_cap;
        for (uint32_t i = threadIdx.x; i < cnt; i += 64) narrow_one(env, links, w, seg[i], n_sat);
    } else {
        const uint32_t n = b.ctl[2] < (uint32_t)b.spill_cap ? b.ctl[2] : (uint32_t)b.spill_cap;
        for (uint32_t i = (uint32_t)(gw - b.n_waves) * 64 + threadIdx.x; i < n; i += kSpillBlocks * 64)
            narrow_one(env, links, w, b.spill[i], n_sat);
    }
    if (w.stats && n_sat) atomicAdd(w.stats + 3, (unsigned long long)n_sat);
    if (w.stats && gw == 0 && threadIdx.x == 0) {
        atomicAdd(w.stats + 5, (unsigned long long)b.ctl[1]);
        atomicAdd(w.stats + 7, (unsigned long long)b.ctl[2]);
    }
}

CollideScratch::~CollideScratch() {
    void *ps[] = {cand, seg_count, spill, ctl, ovf_list};
    for (void *p : ps)
        if (p) (void)hipFree(p);
}

void CollideScratch::ensure(int64_t n_units) {
    if (!cand) {
        int dev = 0, cus = 256;
        if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        n_blocks = cus * 4;  // 4 x 8 waves per CU: full occupancy if registers allow
        n_waves = n_blocks * kBroadWaves;
        seg_cap = kSegCap;
        hip_check(hipMalloc(&cand, sizeof(Cand) * (size_t)n_waves * seg_cap), "alloc candidates");
        hip_check(hipMalloc(&seg_count, sizeof(uint32_t) * n_waves), "alloc seg counts");
        spill_cap = kSpillCap;
        hip_check(hipMalloc(&spill, sizeof(Cand) * (size_t)spill_cap), "alloc spill");
        hip_check(hipMalloc(&ctl, sizeof(uint32_t) * 4), "alloc collide ctl");
    }
    if (n_units > ovf_cap) {
        if (ovf_list) hip_check(hipFree(ovf_list), "hipFree");
        ovf_list = nullptr;
        hip_check(hipMalloc(&ovf_list, sizeof(int32_t) * (size_t)n_units), "alloc overflow list");
        ovf_cap = n_units;
    }
}

void launch_collide_split(const EnvDev &env, const AgentDev *d_links, const CollideWork &w, CollideScratch &s,
                          hipStream_t stream) {
    if (w.n_units <= 0 || env.n_tris <= 0) return;
    if (w.n_units >= (int64_t(1) << 31) || w.n_units > s.ovf_cap || !s.cand)
        throw Error{5, "collide scratch not sized for this launch"};
    BroadArgs b{s.cand, s.seg_count, s.spill, s.ctl, s.ovf_list, s.seg_cap, s.n_waves, s.spill_cap};
    hip_check(hipMemsetAsync(s.ctl, 0, sizeof(uint32_t) * 4, stream), "collide ctl memset");
    const int32_t n_items = env.lev_off[env.n_levels];
    static const bool force_global = getenv("MPT_BROAD_GLOBAL") != nullptr;  // experiment knob
    if (n_items <= kLdsItems && !force_global)
        hipLaunchKernelGGL(k_broad<true>, dim3((unsigned)s.n_blocks), dim3(kBroadWaves * 64),
                           sizeof(Item) * n_items, stream, env, d_links, w, b);
    else
        hipLaunchKernelGGL(k_broad<false>, dim3((unsigned)s.n_blocks), dim3(kBroadWaves * 64), 0, stream, env,
                           d_links, w, b);
    hip_check(hipGetLastError(), "k_broad launch");
    hipLaunchKernelGGL(k_narrow, dim3((unsigned)(s.n_waves + kSpillBlocks)), dim3(64), 0, stream, env, d_links, w,
                       b);
    hip_check(hipGetLastError(), "k_narrow launch");
    // units whose candidates overflowed segment and spill list (none in practice): fused
    // path, list read on the device, a small grid so the usual empty launch costs little
    CollideWork f = w;
    f.unit_list = s.ovf_list;
    f.unit_list_n = s.ctl + 1;
    f.stats = nullptr;
    launch_collide(env, d_links, f, stream, 64);
}

}  // namespace mpt
