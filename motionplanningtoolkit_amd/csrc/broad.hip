// broad.hip -- the two-phase collision path (default structure, mpt_set_collide_mode).
//
// Same verdicts as the fused kernel (collide.hip): exists (pose, link, env tri, agent tri)
// with overlapping exact boxes (tri_gate) and intersect_Triangle true.  The work is done
// breadth-first, every stage a flat parallel loop over its own items, so no wave carries a
// long chain of dependent memory accesses (what limits the fused kernel):
//
// k_pairs   one thread per (unit, agent cluster).  FCL relative transform of the unit's pose
//           (FP64), the cluster's local box mapped to a widened float box, culled by the env
//           root box, then walked down the 64-ary env tree (mpt_internal.h Item, staged in
//           LDS when it fits): every env triangle whose box overlaps the cluster box makes a
//           (unit, cluster, triangle) pair.  Two passes (count, then write) give each thread
//           a contiguous run of its wave's pair segment and one header; the reservations are
//           LDS atomics.
// scan      exclusive sum of the per-segment header counts whose epilogue writes the header
//           slots densely (scan.h, one launch).
// k_cands   one wave per header (grid-stride over the dense list): lanes = the cluster's
//           agent triangles, mapped exactly (FP64) and boxed; lanes also fetch the header's
//           env triangle boxes, which are then tested from registers; overlaps become
//           candidates in the wave's segment (or the spill list).
// k_narrow  one workgroup per four candidate segments taken as one list (plus the spill
//           list), one candidate per lane: exact transform, tri_gate, intersect_Triangle;
//           verdict[edge] = 1.
// k_overflow  units whose pairs overflowed a segment are re-run with the fused kernel's
//           per-unit walk (collide_common.h collide_unit).
#include <hipcub/hipcub.hpp>
#include <cstdio>
#include <type_traits>
#include <vector>

#include "collide_common.h"
#include "scan.h"

namespace mpt {

constexpr int kPairThreads = 256;   // k_pairs workgroup (4 waves)
constexpr int kPairCap = 512;       // env triangles per k_pairs wave segment (256: the room overflowed units into k_overflow, 17-27 us a round)
constexpr int kHdrCap = 64;         // headers per segment (one per lane at most)
constexpr int kCandCap = 8192;      // candidates per k_cands wave (then the spill list)
// (unit, cluster) threads per launch of the two-phase path: a whole config-5 round of 256 blimp
// seeds (1 M units x 22 clusters) in one chunk; its scratch (pair words, headers, candidates:
// ~2 GiB) is small beside 288 GB of HBM, and one launch per kernel has one tail, not six
constexpr int64_t kSplitChunkThreads = int64_t(1) << 25;
constexpr int kSpillCap = 1 << 23;  // shared spill list (96 MiB)
constexpr int kLdsItems = 2048;     // env tree staged in LDS by k_pairs up to this size (64 KiB)
constexpr int kCandsLdsItems = 1024;  // env triangle items staged in LDS by k_cands up to this count
constexpr int kStack = kMaxLevels;  // per-thread walk stack (general trees)

struct SplitArgs {
    int32_t *pairs;
    PairHdr *hdr;
    uint32_t *hdr_count;
    uint32_t *pair_count;
    const uint32_t *hdr_off;
    int32_t *hdr_dense;
    Cand *cand;
    uint32_t *cand_count;
    Cand *spill;
    uint32_t *ctl;       // this launch's counters: [1] overflow units, [2] spill count
    uint32_t *ctl_next;  // the other half, zeroed by k_pairs for the next launch
    int32_t *ovf_list;
    int64_t n_seg;
    int32_t pair_cap, cand_cap, spill_cap, n_clusters, n_cwaves;
};

// wave-uniform item load through the scalar cache (items are read-only in these kernels)
__device__ __forceinline__ Item load_item_u(const Item *__restrict__ items, int64_t idx) {
#if defined(__HIP_DEVICE_COMPILE__)
    typedef __attribute__((address_space(4))) const Item *cptr;
    const Item *g = items;
    return ((cptr)g)[idx];
#else
    return items[idx];
#endif
}

// Per-thread walk of the env tree (items from LDS or global) with box (lo, hi);
// sink(tri) for every overlapping triangle box; returns the number of item tests.
// Two-level trees (top = buckets of triangles) need no stack; deeper ones keep one
// (mask, base, level) entry per level in LDS.
template <bool kTwo, class Sink>
__device__ __forceinline__ uint32_t walk_tree(const EnvDev &env, const Item *__restrict__ items, const float lo[3],
                                              const float hi[3], uint4 *stk, Sink &&sink) {
    const int32_t top = env.n_levels - 1;
    const int32_t top_off = env.lev_off[top];
    const int32_t n_top = env.lev_off[top + 1] - top_off;
    uint32_t tests = (uint32_t)n_top;
    // boxes of items [first, first + count) that overlap (lo, hi) as a bit mask; eight
    // independent loads in flight per step (a one-at-a-time loop is a chain of dependent
    // LDS round trips, which is what bounded the walk)
    // (batches of 8, then of 4 for the remainder: a 10-triangle bucket reads 12 boxes, not 16)
    auto overlap_batch = [&](auto kB, int32_t first, int32_t count, int32_t i0, uint64_t &M) {
        constexpr int B = decltype(kB)::value;
        float bl[B][3], bh[B][3];
#pragma unroll
        for (int j = 0; j < B; ++j) {
            const Item b = items[first + (i0 + j < count ? i0 + j : count - 1)];
#pragma unroll
            for (int x = 0; x < 3; ++x) {
                bl[j][x] = b.lo[x];
                bh[j][x] = b.hi[x];
            }
        }
#pragma unroll
        for (int j = 0; j < B; ++j)
            if (i0 + j < count && box_overlap(lo, hi, bl[j], bh[j])) M |= 1ull << (i0 + j);
    };
    auto overlap_mask = [&](int32_t first, int32_t count) {
        uint64_t M = 0;
        int32_t i0 = 0;
        for (; i0 + 8 <= count; i0 += 8) overlap_batch(std::integral_constant<int, 8>{}, first, count, i0, M);
        for (; i0 < count; i0 += 4) overlap_batch(std::integral_constant<int, 4>{}, first, count, i0, M);
        return M;
    };
    auto tri_run = [&](int32_t first, int32_t count) {
        uint64_t M = overlap_mask(first, count);
        while (M) {
            const int j = __ffsll((unsigned long long)M) - 1;
            M &= M - 1;
            sink(first + j);
        }
    };
    if (kTwo) {
        uint64_t M = overlap_mask(top_off, n_top);
        while (M) {
            const int i = __ffsll((unsigned long long)M) - 1;
            M &= M - 1;
            const Item b = items[top_off + i];
            tests += (uint32_t)b.count;
            tri_run(b.first, b.count);
        }
        return tests;
    }
    // general: DFS over (level, base, remaining-children mask)
    uint64_t M = overlap_mask(top_off, n_top);
    int32_t lv = top, base = top_off, sp = 0;
    for (;;) {
        if (!M) {
            if (sp == 0) break;
            --sp;
            const uint4 e = stk[sp];
            M = ((uint64_t)e.y << 32) | e.x;
            base = (int32_t)e.z;
            lv = (int32_t)e.w;
            continue;
        }
        const int j = __ffsll((unsigned long long)M) - 1;
        M &= M - 1;
        const Item it = items[base + j];
        tests += (uint32_t)it.count;
        if (lv == 1) {  // children are triangles
            tri_run(it.first, it.count);
            continue;
        }
        const uint64_t Mc = overlap_mask(it.first, it.count);
        if (!Mc) continue;
        if (M) stk[sp++] = make_uint4((uint32_t)M, (uint32_t)(M >> 32), (uint32_t)base, (uint32_t)lv);
        M = Mc;
        base = it.first;
        --lv;
    }
    return tests;
}

// The two-level walk on quantized boxes (EnvDev::qitems, staged in LDS): one 16-B read per
// box instead of two 12-B ones, and the overlap test as 15-bit SWAR on 32-bit words (bit 15 of
// each half of (a | 0x8000) - b is set iff a >= b).  The items were quantized outward on the
// host, the query box is here with a margin of 0.02 quanta beyond the float rounding of its
// grid coordinate (<= 0.01 quanta: two roundings of ~0.004 and the float scale's 0.002), so
// every pair the float walk keeps is kept (a superset: k_cands tests the exact float boxes
// again).  The walk is LDS-bandwidth bound: per-workgroup phase times (a round-2 timer since
// removed) showed the cull + staging ~4 us and the walk ~16 us of a ~20-us lifetime; with these boxes
// the walk takes ~11 us (config 2's k_pairs 31 -> 25 us, the room's 115 -> 90 us).
// sel: the top-level items to test (the unit's link-box mask, top_item_mask; all ones: every
// one) -- the others cannot meet the cluster's box, which lies inside the link's
template <class Sink>
__device__ __forceinline__ uint32_t walk_two_q(const EnvDev &env, const uint4 *__restrict__ qi, const QBox &q,
                                               uint64_t sel, Sink &&sink) {
    const int32_t top = env.n_levels - 1;
    const int32_t top_off = env.lev_off[top];
    const int32_t n_top = env.lev_off[top + 1] - top_off;
    uint32_t tests = 0;
    auto batch = [&](auto kB, int32_t first, int32_t count, int32_t i0, uint64_t &M) {
        constexpr int B = decltype(kB)::value;
        uint4 b[B];
#pragma unroll
        for (int j = 0; j < B; ++j) b[j] = qi[first + (i0 + j < count ? i0 + j : count - 1)];
#pragma unroll
        for (int j = 0; j < B; ++j)
            if (i0 + j < count && qbox_overlap(q, b[j])) M |= 1ull << (i0 + j);
    };
    auto mask = [&](int32_t first, int32_t count) {
        uint64_t M = 0;
        int32_t i0 = 0;
        for (; i0 + 8 <= count; i0 += 8) batch(std::integral_constant<int, 8>{}, first, count, i0, M);
        for (; i0 < count; i0 += 4) batch(std::integral_constant<int, 4>{}, first, count, i0, M);
        return M;
    };
    uint64_t M = 0;
    if (n_top > 64 || sel == ~0ull) {
        M = mask(top_off, n_top);
        tests = (uint32_t)n_top;
    } else {
        // the selected items, eight loads in flight a batch
        for (uint64_t rem = sel & (n_top == 64 ? ~0ull : ((1ull << n_top) - 1)); rem;) {
            int idx[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                idx[j] = rem ? __ffsll((unsigned long long)rem) - 1 : -1;
                rem &= rem - 1;
            }
            uint4 b[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) b[j] = qi[top_off + (idx[j] >= 0 ? idx[j] : idx[0])];
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (idx[j] >= 0) {
                    ++tests;
                    if (qbox_overlap(q, b[j])) M |= 1ull << idx[j];
                }
        }
    }
    while (M) {
        const int i = __ffsll((unsigned long long)M) - 1;
        M &= M - 1;
        const uint32_t w = qi[top_off + i].w;
        const int32_t first = (int32_t)(w & ((1u << 26) - 1u)), count = (int32_t)(w >> 26) + 1;
        tests += (uint32_t)count;
        uint64_t Mt = mask(first, count);
        while (Mt) {
            const int j = __ffsll((unsigned long long)Mt) - 1;
            Mt &= Mt - 1;
            sink(first + j);
        }
    }
    return tests;
}

// Per-(pose, cluster) record of a thread that survived the root cull, compacted in LDS so
// the tree walks run on as few waves as possible (most clusters are culled at the root).
struct PairRec {
    float lo[3], hi[3];
    int32_t unit, c, tfirst, tcount;
    uint64_t tmask;  // the unit's top-level item mask (CollideWork::unit_tmask), or all ones
};

template <bool kTwo, bool kLds>
__global__ __launch_bounds__(kPairThreads) void k_pairs(EnvDev env, const AgentDev *__restrict__ links,
                                                       CollideWork w, SplitArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ uint32_t s_pc[kPairThreads / 64], s_hc[kPairThreads / 64], s_live[kPairThreads / 64];
    __shared__ uint4 s_stk[kTwo ? 1 : kPairThreads * kStack];
    __shared__ PairRec s_rec[kPairThreads];
    if (blockIdx.x == 0) {  // stream-ordered resets instead of memset launches
        if (threadIdx.x < 4) a.ctl_next[threadIdx.x] = 0u;
        if (threadIdx.x == 0) a.hdr_count[a.n_seg] = 0u;  // the header scan's sentinel slot
    }
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int64_t t = (int64_t)blockIdx.x * kPairThreads + threadIdx.x;
    const int64_t seg = t >> 6;
    // 0. with a live-unit list, threads map to (live unit, cluster); workgroups past the list
    //    only zero their segments' counts
    const int64_t n_thr = w.live_units ? (int64_t)*w.n_live * a.n_clusters : w.n_units * a.n_clusters;
    // 1. thread per (pose, cluster): FCL relative transform, cluster box, root cull
    {
        const int64_t unit = t < n_thr ? (w.live_units ? (int64_t)w.live_units[t / a.n_clusters] : t / a.n_clusters)
                                       : w.n_units;
        const int32_t c = (int32_t)(t % a.n_clusters);
        bool live = unit < w.n_units;
        int32_t link = 0;
        int64_t slot = 0, edge = 0;
        if (live) live = decode_unit(w, unit, link, slot, edge);
        if (live) live = c < links[link].n_clusters;
        const bool decoded = live;
        PairRec r;
        if (live) {
            double R[9], T[3];
            unit_rt(env, w, slot, link, R, T);
            const Cluster &cl = links[link].clusters[c];
            local_box(cl.c, cl.e, R, T, r.lo, r.hi);
            r.unit = (int32_t)unit;
            r.c = c;
            r.tfirst = cl.first;
            r.tcount = cl.count;
            r.tmask = w.unit_tmask ? w.unit_tmask[unit] : ~0ull;
            live = box_overlap(r.lo, r.hi, env.root_lo, env.root_hi);
        }
        const uint64_t m = __ballot(live);
        if (lane == 0) {
            s_live[wave] = (uint32_t)__popcll(m);
            s_pc[wave] = 0;
            s_hc[wave] = 0;
        }
        if (w.stats) {
            const uint64_t dm = __ballot(decoded);
            if (lane == 0) {
                atomicAdd(w.stats + 1, (unsigned long long)__popcll(m));
                atomicAdd(w.stats + 10, (unsigned long long)__popcll(dm));
            }
        }
        __syncthreads();
        if (live) {
            uint32_t base = 0;
            for (int v = 0; v < wave; ++v) base += s_live[v];
            s_rec[base + (uint32_t)__popcll(m & ((1ull << lane) - 1))] = r;
        }
    }
    uint32_t total = 0;
    for (int v = 0; v < kPairThreads / 64; ++v) total += s_live[v];
    if (total == 0) {  // block-uniform: nothing reaches the env tree
        if (lane == 0 && seg < a.n_seg) {
            a.hdr_count[seg] = 0;
            a.pair_count[seg] = 0;
        }
        return;
    }
    // the walk's items: in LDS (kLds) or global, decided at compile time -- a pointer that may
    // be either compiles to flat instructions, slower for LDS and counted against the LDS
    // counter for global
    const Item *items = kLds ? reinterpret_cast<const Item *>(smem) : env.items;
    // two-level trees in LDS walk the quantized boxes (env.qitems; 16 B an item)
    const bool quant = kTwo && kLds && env.qitems != nullptr;
    const uint4 *qitems = reinterpret_cast<const uint4 *>(smem);
    if (kLds) {
        const int32_t n = env.lev_off[env.n_levels];
        uint4 *dst = reinterpret_cast<uint4 *>(smem);
        if (quant) {
            for (int i = threadIdx.x; i < n; i += blockDim.x) dst[i] = env.qitems[i];
        } else {
            const uint4 *src = reinterpret_cast<const uint4 *>(env.items);
            for (int i = threadIdx.x; i < n * 2; i += blockDim.x) dst[i] = src[i];
        }
    }
    __syncthreads();
    // 2. the surviving records, packed onto the first waves: walk the env tree; the pair
    //    words and headers carry the (segment, lane) of the thread that walked
    const bool live = threadIdx.x < total;
    PairRec r;
    if (live) r = s_rec[threadIdx.x];
    uint4 *stk = s_stk + (kTwo ? 0 : threadIdx.x * kStack);
    uint32_t np = 0, tests = 0;
    bool ovf = false;
    int32_t *out = a.pairs + seg * a.pair_cap;
    // one pass: each pair takes the next slot of the wave's segment (LDS atomic) as a
    // (lane, triangle) word; k_cands picks a header's pairs out by lane
    auto emit_pair = [&](int32_t tri) {
        const uint32_t pos = atomicAdd(&s_pc[wave], 1u);
        if (pos < (uint32_t)a.pair_cap)
            out[pos] = (int32_t)(((uint32_t)lane << kPairTriBits) | (uint32_t)tri);
        else
            ovf = true;
        ++np;
    };
    if (live) {
        if (quant) tests = walk_two_q(env, qitems, quantize_box(env, r.lo, r.hi), r.tmask, emit_pair);
        else tests = walk_tree<kTwo>(env, items, r.lo, r.hi, stk, emit_pair);
    }
    if (np > 0 && !ovf) {
        const uint32_t h = atomicAdd(&s_hc[wave], 1u);
        a.hdr[seg * kHdrCap + h] = PairHdr{r.unit, r.c, (int32_t)seg, (int32_t)np, r.tfirst, r.tcount, lane, 0};
    }
    if (ovf) a.ovf_list[atomicAdd(a.ctl + 1, 1u)] = r.unit;  // rare: fused re-run
    __builtin_amdgcn_wave_barrier();
    if (lane == 0 && seg < a.n_seg) {
        a.hdr_count[seg] = s_hc[wave];
        a.pair_count[seg] = s_pc[wave] < (uint32_t)a.pair_cap ? s_pc[wave] : (uint32_t)a.pair_cap;
    }
    if (w.stats) {
        uint32_t sum_tests = tests, sum_pairs = np;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            sum_tests += __shfl_xor(sum_tests, off);
            sum_pairs += __shfl_xor(sum_pairs, off);
        }
        if (lane == 0) {
            atomicAdd(w.stats + 2, (unsigned long long)sum_tests);
            atomicAdd(w.stats + 4, (unsigned long long)sum_pairs);
        }
    }
}

// scan epilogue: header slots in dense order, dense[off[seg] + h] = seg * kHdrCap + h
struct ExpandHeaders {
    int32_t *dense;
    int64_t n_seg;
    __device__ void operator()(int64_t seg, uint32_t off, uint32_t n) const {
        if (seg >= n_seg) return;  // the sentinel slot
        for (uint32_t h = 0; h < n; ++h) dense[off + h] = (int32_t)(seg * kHdrCap + h);
    }
};

// Append the lanes of h (ballot m) as candidates: to the wave's segment, or once that is
// full to the shared spill list; false if both are full.  Called with all lanes active.
__device__ __forceinline__ bool emit(bool h, uint64_t m, int32_t unit, int32_t atri, int32_t etri, Cand *seg,
                                     uint32_t &cnt, const SplitArgs &a) {
    const uint32_t n = (uint32_t)__popcll(m);
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    if (cnt + n <= (uint32_t)a.cand_cap) {
        if (h) seg[cnt + rank] = Cand{unit, atri, etri};
        cnt += n;
        return true;
    }
    uint32_t base = 0;
    if ((threadIdx.x & 63) == 0) base = atomicAdd(a.ctl + 2, n);
    base = __builtin_amdgcn_readfirstlane(base);
    if (base + n > (uint32_t)a.spill_cap) return false;
    if (h) a.spill[base + rank] = Cand{unit, atri, etri};
    return true;
}

// lds_items: the env's triangle items [0, n_tris) staged in LDS (small envs), else read
// through the caches.  A header's chain of dependent loads is dense slot -> header -> {pose,
// agent triangles, pair words} -> env items; the next header's dense slot is fetched ahead.
// kLds: the items in LDS, a compile-time choice (a pointer that may be LDS or global compiles
// to flat instructions).  Round 5, measured and not kept: the workgroup's headers claimed from
// an LDS counter instead of each wave's fixed stride (k_narrow's pooling, for the headers):
// config 2 ~385 M, the room 126 vs 127 M, 32 seeds 131.2 vs 132.3 M -- no gain.
template <bool kLds>
__global__ __launch_bounds__(256) void k_cands(EnvDev env, const AgentDev *__restrict__ links, CollideWork w,
                                               SplitArgs a, int32_t lds_items) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int32_t cw = (int32_t)blockIdx.x * 4 + wave;
    const uint32_t total = __builtin_amdgcn_readfirstlane(a.hdr_off[a.n_seg]);
    const Item *items = kLds ? reinterpret_cast<const Item *>(smem) : env.items;
    if (kLds) {
        const uint4 *src = reinterpret_cast<const uint4 *>(env.items);
        uint4 *dst = reinterpret_cast<uint4 *>(smem);
        for (int i = threadIdx.x; i < lds_items * 2; i += blockDim.x) dst[i] = src[i];
        __syncthreads();
    }
    Cand *cseg = a.cand + (int64_t)cw * a.cand_cap;
    uint32_t cnt = 0, n_xf = 0;
    int32_t slot_next = (uint32_t)cw < total ? __builtin_amdgcn_readfirstlane(a.hdr_dense[cw]) : 0;
    for (uint32_t g = (uint32_t)cw; g < total; g += (uint32_t)a.n_cwaves) {
        const int32_t slot_h = slot_next;
        const PairHdr H = a.hdr[slot_h];
        if (g + (uint32_t)a.n_cwaves < total)
            slot_next = __builtin_amdgcn_readfirstlane(a.hdr_dense[g + (uint32_t)a.n_cwaves]);
        const int32_t unit = __builtin_amdgcn_readfirstlane(H.unit);
        const int32_t hseg = __builtin_amdgcn_readfirstlane(H.seg);
        const int32_t hlane = __builtin_amdgcn_readfirstlane(H.lane);
        const int32_t hn = __builtin_amdgcn_readfirstlane(H.n);  // this header's pair words
        const int32_t tfirst = __builtin_amdgcn_readfirstlane(H.tfirst);
        const int32_t tcount = __builtin_amdgcn_readfirstlane(H.tcount);
        const int32_t *spairs = a.pairs + (int64_t)hseg * a.pair_cap;
        int32_t link;
        int64_t slot, edge;
        decode_unit(w, unit, link, slot, edge);
        const bool act = lane < tcount;
        double tri[9];  // global loads (the agent's pointers are read from memory: flat otherwise)
        load_global<9>(links[link].tris + (int64_t)(tfirst + (act ? lane : 0)) * 9, tri);
        double R[9], T[3];
        unit_rt(env, w, slot, link, R, T);
#pragma unroll
        for (int i = 0; i < 9; ++i) R[i] = uniform_d(R[i]);
#pragma unroll
        for (int i = 0; i < 3; ++i) T[i] = uniform_d(T[i]);
        float blo[3] = {0, 0, 0}, bhi[3] = {0, 0, 0}, tlo[3], thi[3];
        if (act) agent_tri_box(tri, R, T, blo, bhi);
        ++n_xf;
#pragma unroll
        // (ds_bpermute levels: the DPP / permlane form, wave_ops.h, measured slower here -- room
        // k_cands 0.149-0.153 vs 0.145-0.146 ms, A/B on one box: its selects cost more VALU issue
        // than the LDS round trips it saves in this kernel)
        for (int k = 0; k < 3; ++k) {
            float lo = act ? blo[k] : __builtin_huge_valf(), hi = act ? bhi[k] : -__builtin_huge_valf();
            for (int off = 32; off > 0; off >>= 1) {
                lo = fminf(lo, __shfl_xor(lo, off));
                hi = fmaxf(hi, __shfl_xor(hi, off));
            }
            tlo[k] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(lo)));
            thi[k] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(hi)));
        }
        // lanes scan the segment 64 words at a time; this header's words are those of its lane,
        // all hn of them in the segment (a thread whose pairs overflowed wrote no header), so
        // the scan stops once it has seen hn: no read of the segment's count, and never a word
        // past the last one written this round
        for (int32_t k0 = 0, found = 0; found < hn && k0 < a.pair_cap; k0 += 64) {
            bool mine = false;
            int32_t etri = 0;
            Item e{};
            if (k0 + lane < a.pair_cap) {
                const uint32_t word = (uint32_t)spairs[k0 + lane];
                mine = (int32_t)(word >> kPairTriBits) == hlane;
                etri = (int32_t)(word & ((1u << kPairTriBits) - 1u));
            }
            found += (int32_t)__popcll(__ballot(mine));
            // words past this header's last one may be stale (earlier rounds): keep only the
            // first hn - (found before this block) of this block's matches
            if (found > hn) {
                const uint64_t mm = __ballot(mine);
                const int keep = hn - (found - (int32_t)__popcll(mm));
                const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(mm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mm, 0u));
                if (mine && (int)rank >= keep) mine = false;
                found = hn;
            }
            if (mine) e = items[etri];
            // env triangles that miss the union of the agent triangle boxes are dropped
            uint64_t M = __ballot(mine && box_overlap(tlo, thi, e.lo, e.hi));
            bool ok = true;
            while (M && ok) {
                const int j = __ffsll((unsigned long long)M) - 1;
                M &= M - 1;
                const float elo[3] = {lane_f(e.lo[0], j), lane_f(e.lo[1], j), lane_f(e.lo[2], j)};
                const float ehi[3] = {lane_f(e.hi[0], j), lane_f(e.hi[1], j), lane_f(e.hi[2], j)};
                const int32_t et = __builtin_amdgcn_readlane(etri, j);
                const bool hh = act && box_overlap(blo, bhi, elo, ehi);
                const uint64_t m = __ballot(hh);
                if (m) ok = emit(hh, m, unit, tfirst + lane, et, cseg, cnt, a);
            }
            if (!ok && lane == 0) a.ovf_list[atomicAdd(a.ctl + 1, 1u)] = unit;  // spill full: fused re-run
        }
    }
    if (lane == 0 && cw < a.n_cwaves) a.cand_count[cw] = cnt;
    if (w.stats && lane == 0) {
        atomicAdd(w.stats + 6, (unsigned long long)n_xf);
        atomicAdd(w.stats + 7, (unsigned long long)cnt);
    }
}

// One candidate per lane.  Every load a candidate needs (its edge's verdict flag, the pose, the
// agent triangle and the env triangle) is issued before any of them is tested, so a
// candidate costs one dependent round trip after its record instead of three; the next
// record is fetched while this one computes.  kLds: the env triangles' vertices sit in LDS
// and the P-side of intersect_Triangle is recomputed from them (tri_collide_verts, bitwise
// make_env_tri's fields); otherwise the precomputed 384-B records are read (large envs).
template <bool kLds, class Get>
__device__ __forceinline__ void narrow_range(const EnvDev &env, const AgentDev *__restrict__ links,
                                             const CollideWork &w, Get cand_at, uint32_t i0, uint32_t n,
                                             uint32_t stride, const double *__restrict__ s_verts, uint32_t &n_sat) {
    Cand next{};
    if (i0 < n) next = cand_at(i0);
    for (uint32_t i = i0; i < n; i += stride) {
        const Cand cd = next;
        if (i + stride < n) next = cand_at(i + stride);
        int32_t link;
        int64_t slot, edge;
        decode_unit(w, cd.unit, link, slot, edge);
        const uint8_t decided = load_flag(w.verdict + edge);
        // the unit's relative transform (precomputed) or its pose
        const double *pose = (w.unit_rt ? w.unit_rt : w.poses) + (slot * w.L + link) * 12;
        double P[12];
#pragma unroll
        for (int k = 0; k < 12; ++k) P[k] = pose[k];
        double A[9];
        load_global<9>(links[link].tris + (int64_t)cd.atri * 9, A);
        if (decided) continue;  // another candidate of this edge already found the contact
        double R[9], T[3];
        if (w.unit_rt) {
#pragma unroll
            for (int k = 0; k < 9; ++k) R[k] = P[k];
#pragma unroll
            for (int k = 0; k < 3; ++k) T[k] = P[9 + k];
        } else {
            relative_transform(env.tf, env.tf + 9, P, P + 9, R, T);
        }
        const v3 Q1 = xform(R, T, mk(A[0], A[1], A[2]));
        const v3 Q2 = xform(R, T, mk(A[3], A[4], A[5]));
        const v3 Q3 = xform(R, T, mk(A[6], A[7], A[8]));
        bool hit;
        if constexpr (kLds) {
            hit = tri_collide_verts(s_verts + (int64_t)cd.etri * 9, Q1, Q2, Q3);
        } else {
            const EnvTri &E = env.tris[cd.etri];
            hit = tri_gate(E.lo, E.hi, Q1, Q2, Q3) && tri_intersect(E, Q1, Q2, Q3);
        }
        if (w.stats) {
            // SAT tests (the gate passed): recount with the cheap gate alone (stats runs only)
            const double *tv = kLds ? s_verts + (int64_t)cd.etri * 9 : nullptr;
            double lo[3], hi[3];
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                lo[k] = kLds ? dmin(tv[k], dmin(tv[3 + k], tv[6 + k])) : env.tris[cd.etri].lo[k];
                hi[k] = kLds ? dmax(tv[k], dmax(tv[3 + k], tv[6 + k])) : env.tris[cd.etri].hi[k];
            }
            if (tri_gate(lo, hi, Q1, Q2, Q3)) ++n_sat;
        }
        if (hit) __hip_atomic_store(w.verdict + edge, (uint8_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// 256-thread workgroups over the candidate segments, 4 a workgroup pooled into one list (one
// wave a segment before: k_narrow 54.7 -> 46.7 us at 32 seeds, 181 -> 161 us at 256, the room
// 112 -> 124 M valid ext/s; 8 segments in 512-thread workgroups: config 2 385 -> 374 M, the
// rest unchanged); the next kSpillWaves waves stride the spill list.  A workgroup whose segments hold at least
// 4 * n_tris candidates (lds_ok: the env fits) first stages the env triangles' vertices
// (72 B each) in LDS and recomputes their SAT fields -- below that the staging and the
// recompute cost more than the 384-B records they save (A/B: blimp.inst, 2.1 candidates
// per env tri per workgroup, 34 us global vs 36 us staged; blimp-room, 16: 174 vs 162 us).  The overflow re-run lives in
// k_overflow: the fused walk's registers in this kernel cost a wave per SIMD (158 VGPRs).
// Not kept: a gate-first pass queueing survivors in LDS and running the SAT on full waves of
// them (reloaded and re-transformed) -- room narrow 169 -> 181 us, config 2 33 -> 34 us.
constexpr int kNarrowWaves = 4;    // k_narrow's workgroup: its 4 segments pooled
constexpr int kOvfBlockWaves = 4;  // k_overflow's workgroup
constexpr int kSpillWaves = 256;
constexpr int kOvfWaves = 64;
constexpr int kNarrowLdsTris = 1024;  // env triangles staged in LDS up to this count (72 KiB)

__global__ __launch_bounds__(kNarrowWaves * 64, 4) void k_narrow(EnvDev env, const AgentDev *__restrict__ links,
                                                                 CollideWork w, SplitArgs a, int32_t lds_ok) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ uint32_t s_cnt[kNarrowWaves];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int32_t gw = (int32_t)blockIdx.x * kNarrowWaves + wave;
    double *s_verts = reinterpret_cast<double *>(smem);
    const uint32_t n_spill = a.ctl[2] < (uint32_t)a.spill_cap ? a.ctl[2] : (uint32_t)a.spill_cap;
    const uint32_t cnt = gw < a.n_cwaves ? a.cand_count[gw] : 0;
    bool lds = false;
    if (lds_ok) {
        if (lane == 0) s_cnt[wave] = gw < a.n_cwaves ? cnt : n_spill / kSpillWaves;
        __syncthreads();
        uint32_t tot = 0;
#pragma unroll
        for (int i = 0; i < kNarrowWaves; ++i) tot += s_cnt[i];
        lds = tot >= (uint32_t)env.n_tris * 4u;
        if (lds) {
            // the vertices P1, P2, P3 of each EnvTri record, as given (fcl_math.h EnvTri)
            for (int32_t i = threadIdx.x; i < env.n_tris * 9; i += blockDim.x) {
                const int32_t tri = i / 9, k = i % 9;
                const double *r = reinterpret_cast<const double *>(env.tris + tri);
                s_verts[i] = k < 3 ? r[k] : (k < 6 ? r[41 + (k - 3)] : r[44 + (k - 6)]);
            }
            __syncthreads();
        }
    }
    uint32_t n_sat = 0;
    const int32_t gw0 = (int32_t)blockIdx.x * kNarrowWaves;  // (n_cwaves is a multiple of kNarrowWaves)
    if (gw0 < a.n_cwaves) {
        // the workgroup's kNarrowWaves segments as one list, strided over its threads: a
        // segment's count follows the headers its k_cands wave happened to take, so at small
        // batches one long segment held its wave (and the launch) long after the others
        uint32_t pre[kNarrowWaves + 1];
        pre[0] = 0;
#pragma unroll
        for (int i = 0; i < kNarrowWaves; ++i) pre[i + 1] = pre[i] + __builtin_amdgcn_readfirstlane(a.cand_count[gw0 + i]);
        const Cand *seg0 = a.cand + (int64_t)gw0 * a.cand_cap;
        const int64_t cap = a.cand_cap;
        auto cand_at = [&](uint32_t i) {
            int sgi = 0;
#pragma unroll
            for (int k = 1; k < kNarrowWaves; ++k) sgi += i >= pre[k] ? 1 : 0;
            return seg0[sgi * cap + (i - pre[sgi])];
        };
        if (lds)
            narrow_range<true>(env, links, w, cand_at, threadIdx.x, pre[kNarrowWaves], kNarrowWaves * 64, s_verts, n_sat);
        else
            narrow_range<false>(env, links, w, cand_at, threadIdx.x, pre[kNarrowWaves], kNarrowWaves * 64, s_verts, n_sat);
    } else {
        const Cand *cands = a.spill;
        auto cand_at = [&](uint32_t i) { return cands[i]; };
        const uint32_t i0 = (uint32_t)(gw - a.n_cwaves) * 64 + lane, stride = (uint32_t)kSpillWaves * 64u;
        if (lds)
            narrow_range<true>(env, links, w, cand_at, i0, n_spill, stride, s_verts, n_sat);
        else
            narrow_range<false>(env, links, w, cand_at, i0, n_spill, stride, s_verts, n_sat);
    }
    if (w.stats && n_sat) atomicAdd(w.stats + 3, (unsigned long long)n_sat);
    if (w.stats && gw == 0 && lane == 0) {
        atomicAdd(w.stats + 5, (unsigned long long)a.ctl[1]);
        atomicAdd(w.stats + 7, (unsigned long long)n_spill);
    }
}

// Units that overflowed a pair segment or the spill list (none in practice) are re-run whole
// with the fused walk (one wave per unit, BVH from global memory).  Launched unconditionally:
// the usual empty case is one read of the overflow count.
__global__ __launch_bounds__(kOvfBlockWaves * 64) void k_overflow(EnvDev env, const AgentDev *__restrict__ links,
                                                                CollideWork w, SplitArgs a) {
    __shared__ int32_t s_stk[kOvfBlockWaves][kStackDepth];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int32_t gw = (int32_t)blockIdx.x * kOvfBlockWaves + wave;
    const uint32_t n_ovf = __hip_atomic_load(a.ctl + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool shared_edges = w.pose_edge != nullptr || w.L > 1 || w.pmax > 1;
    uint32_t nu = 0, nc = 0, nn = 0, ns = 0;
    for (uint32_t i = (uint32_t)gw; i < n_ovf; i += kOvfWaves)
        collide_unit(env, env.nodes, env.n_nodes, links, w, a.ovf_list[i], s_stk[wave], lane, shared_edges, nc, nn, ns,
                     nu);
}

// units decoded (stats only; the other stages count their own work)
__global__ void k_count_units(CollideWork w) {
    const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int32_t link;
    int64_t slot, edge;
    const bool live = u < w.n_units && decode_unit(w, u, link, slot, edge);
    const uint64_t m = __ballot(live);
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(w.stats + 0, (unsigned long long)__popcll(m));
}

CollideScratch::~CollideScratch() {
    void *ps[] = {pairs, hdr, hdr_count, pair_count, hdr_off, hdr_dense, cand, cand_count, spill, ctl, ovf_list};
    for (void *p : ps)
        if (p) (void)hipFree(p);
}

// units per chunk of the two-phase path: kSplitChunkThreads (unit, cluster) threads, so the
// per-launch segments hold a chunk's pairs and candidates (the 11-link snake, one cluster per
// link, runs a whole 720k-unit round in one launch; the 22-cluster blimp 190k units)
static int64_t split_chunk_units(int32_t max_clusters) {
    return kSplitChunkThreads / (max_clusters > 0 ? max_clusters : 1);
}
int64_t collide_chunk_units(int32_t max_clusters) { return split_chunk_units(max_clusters); }

void CollideScratch::ensure(int64_t n_units, int32_t max_clusters) {
    n_units = std::min<int64_t>(n_units, split_chunk_units(max_clusters));  // launch_collide_split runs chunks
    const int64_t threads = n_units * (int64_t)(max_clusters > 0 ? max_clusters : 1);
    if (!ctl) {
        int dev = 0, cus = 256;
        if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        // k_cands: a resident grid striding over the headers; each header is a chain of
        // dependent loads, so more waves in flight hide more of it (8 / 24 a CU measured slower
        // than 16 at the round-3 head)
        const int per_cu = 16;
        n_cwaves = cus * per_cu;
        hip_check(hipMalloc(&cand_count, sizeof(uint32_t) * (size_t)n_cwaves), "alloc candidate counts");
        hip_check(hipMalloc(&ctl, sizeof(uint32_t) * 8), "alloc collide ctl");
        hip_check(hipMemset(ctl, 0, sizeof(uint32_t) * 8), "zero collide ctl");
        // the null-stream memset is not ordered with the caller's (non-blocking) stream: wait
        // for it, or the first k_narrow / fused re-run may read stale overflow and spill counts
        hip_check(hipDeviceSynchronize(), "zero collide ctl sync");
        ctl_par = 0;
    }
    // Candidate segments and the spill list sized by the launch's (unit, cluster) threads: ~16
    // candidates a thread of a k_cands wave's share (config 2 and the room: ~350 threads a wave,
    // 154 / 1214 candidates on average), at most kCandCap; the spill list 2 a thread, at most
    // kSpillCap.  An engine's own K = 4096 round then takes ~25 MiB instead of ~480 (config 5's
    // per-engine rounds); what overflows still reaches the fused re-run, so sizes change speed only.
    const int64_t per_wave = (threads + n_cwaves - 1) / n_cwaves;
    int64_t want_cand = 512, want_spill = int64_t(1) << 18;
    while (want_cand < 16 * per_wave && want_cand < kCandCap) want_cand <<= 1;
    while (want_spill < 2 * threads && want_spill < kSpillCap) want_spill <<= 1;
    if (want_cand > cand_cap || want_spill > spill_cap) {
        hip_check(hipDeviceSynchronize(), "sync");  // the old segments may still be in use
        if (want_cand > cand_cap) {
            if (cand) hip_check(hipFree(cand), "hipFree");
            cand_cap = (int32_t)want_cand;
            hip_check(hipMalloc(&cand, sizeof(Cand) * (size_t)n_cwaves * cand_cap), "alloc candidates");
        }
        if (want_spill > spill_cap) {
            if (spill) hip_check(hipFree(spill), "hipFree");
            spill_cap = (int32_t)want_spill;
            hip_check(hipMalloc(&spill, sizeof(Cand) * (size_t)spill_cap), "alloc spill");
        }
    }
    const int64_t segs = (n_units * (int64_t)(max_clusters > 0 ? max_clusters : 1) + 63) / 64;
    if (segs > n_seg) {
        if (segs * kHdrCap >= (int64_t(1) << 31)) throw Error{5, "collide batch too large"};
        void *ps[] = {pairs, hdr, hdr_count, pair_count, hdr_off, hdr_dense};
        for (void *p : ps)
            if (p) hip_check(hipFree(p), "hipFree");
        pair_cap = kPairCap;  // pair words per k_pairs wave segment
        // Not kept: each thread's pairs as one contiguous run (staged in LDS, placed after a
        // wave scan) so a k_cands header reads only its own words -- room k_pairs 119 -> 140 us
        // (LDS staging, occupancy), k_cands unchanged (its pair scan was not what bounds it).
        hip_check(hipMalloc(&pairs, sizeof(int32_t) * (size_t)segs * pair_cap), "alloc pairs");
        hip_check(hipMalloc(&hdr, sizeof(PairHdr) * (size_t)segs * kHdrCap), "alloc headers");
        hip_check(hipMalloc(&hdr_count, sizeof(uint32_t) * (size_t)(segs + 1)), "alloc header counts");
        hip_check(hipMalloc(&pair_count, sizeof(uint32_t) * (size_t)segs), "alloc pair counts");
        hip_check(hipMalloc(&hdr_off, sizeof(uint32_t) * (size_t)(segs + 1)), "alloc header offsets");
        hip_check(hipMalloc(&hdr_dense, sizeof(int32_t) * (size_t)segs * kHdrCap), "alloc dense headers");
        hip_check(hipMemset(hdr_count, 0, sizeof(uint32_t) * (size_t)(segs + 1)), "memset header counts");
        hip_check(hipDeviceSynchronize(), "memset header counts sync");  // see ctl above
        hdr_scan.reserve((segs + 1 + 255) / 256);
        n_seg = segs;
    }
    if (n_units > ovf_cap) {
        if (ovf_list) hip_check(hipFree(ovf_list), "hipFree");
        ovf_list = nullptr;
        // a unit can be listed once per cluster (k_pairs) plus once per header (k_cands)
        hip_check(hipMalloc(&ovf_list, sizeof(int32_t) * (size_t)n_units * (2 * max_clusters + 1)),
                  "alloc overflow list");
        ovf_cap = n_units;
    }
}

static void collide_split_chunk(const EnvDev &env, const AgentDev *d_links, int32_t max_clusters,
                                const CollideWork &w, CollideScratch &s, hipStream_t stream, hipEvent_t *marks,
                                OvfDefer *defer) {
    auto mark = [&](int i) {
        if (marks) hip_check(hipEventRecord(marks[i], stream), "event record");
    };
    if (w.n_units <= 0 || env.n_tris <= 0) {
        for (int i = 0; i < 3; ++i) mark(i);
        return;
    }
    const int32_t C = max_clusters > 0 ? max_clusters : 1;
    const int64_t threads = w.n_units * C;
    const int64_t segs = (threads + 63) / 64;
    if (threads >= (int64_t(1) << 31) || w.n_units > s.ovf_cap || segs > s.n_seg || !s.pairs)
        throw Error{5, "collide scratch not sized for this launch"};
    if (env.n_tris >= (1 << kPairTriBits)) throw Error{5, "env too large for the split collide path"};
    // ctl is double-buffered: this launch's half was zeroed by the previous launch's k_pairs
    // (or at allocation), and this k_pairs zeroes the other half for the next launch
    uint32_t *ctl = s.ctl + 4 * s.ctl_par, *ctl_next = s.ctl + 4 * (1 - s.ctl_par);
    s.ctl_par ^= 1;
    SplitArgs a{s.pairs,  s.hdr,      s.hdr_count, s.pair_count, s.hdr_off, s.hdr_dense, s.cand,    s.cand_count,
                s.spill,  ctl,        ctl_next,    s.ovf_list,   segs,      s.pair_cap,  s.cand_cap, s.spill_cap,
                C,        s.n_cwaves};
    const unsigned pblocks = (unsigned)((threads + kPairThreads - 1) / kPairThreads);
    const int32_t n_items = env.lev_off[env.n_levels];
    const bool lds = n_items <= kLdsItems;  // the env's tree items staged in LDS when they fit
    const size_t lds_bytes = lds ? sizeof(Item) * n_items : 0;
    if (env.n_levels <= 2) {
        if (lds)
            hipLaunchKernelGGL((k_pairs<true, true>), dim3(pblocks), dim3(kPairThreads), lds_bytes, stream, env,
                               d_links, w, a);
        else
            hipLaunchKernelGGL((k_pairs<true, false>), dim3(pblocks), dim3(kPairThreads), 0, stream, env, d_links, w,
                               a);
    } else {
        if (lds)
            hipLaunchKernelGGL((k_pairs<false, true>), dim3(pblocks), dim3(kPairThreads), lds_bytes, stream, env,
                               d_links, w, a);
        else
            hipLaunchKernelGGL((k_pairs<false, false>), dim3(pblocks), dim3(kPairThreads), 0, stream, env, d_links,
                               w, a);
    }
    hip_check(hipGetLastError(), "k_pairs launch");
    mark(0);
    // count slot `segs` is the scan's sentinel (a larger earlier launch may have used it): k_pairs zeroed it
    // one segment per thread: the epilogue writes up to 64 header slots per segment
    launch_scan_excl<1>(s.hdr_scan, s.hdr_count, s.hdr_off, segs + 1, stream, ExpandHeaders{s.hdr_dense, segs});
    // the env's triangle items in LDS when they fit in 32 KiB (four workgroups per CU)
    const int32_t cl_items = env.n_tris <= kCandsLdsItems ? env.n_tris : 0;
    if (cl_items > 0)
        hipLaunchKernelGGL(k_cands<true>, dim3((unsigned)((s.n_cwaves + 3) / 4)), dim3(256),
                           sizeof(Item) * (size_t)cl_items, stream, env, d_links, w, a, cl_items);
    else
        hipLaunchKernelGGL(k_cands<false>, dim3((unsigned)((s.n_cwaves + 3) / 4)), dim3(256), 0, stream, env, d_links, w,
                           a, 0);
    hip_check(hipGetLastError(), "k_cands launch");
    mark(1);
    const unsigned nblocks = (unsigned)((s.n_cwaves + kSpillWaves + kNarrowWaves - 1) / kNarrowWaves);
    const int32_t lds_ok = env.n_tris <= kNarrowLdsTris;  // k_narrow may stage the env's vertices in LDS
    hipLaunchKernelGGL(k_narrow, dim3(nblocks), dim3(kNarrowWaves * 64), lds_ok ? sizeof(double) * 9 * env.n_tris : 0,
                       stream, env, d_links, w, a, lds_ok);
    hip_check(hipGetLastError(), "k_narrow launch");
    if (defer) {
        defer->env = env;
        defer->links = d_links;
        defer->w = w;
        defer->n_ovf = a.ctl + 1;
        defer->ovf_list = a.ovf_list;
    } else {
        hipLaunchKernelGGL(k_overflow, dim3(kOvfWaves / kOvfBlockWaves), dim3(kOvfBlockWaves * 64), 0, stream, env, d_links,
                           w, a);
        hip_check(hipGetLastError(), "k_overflow launch");
    }
    mark(2);
    if (w.stats) {
        hipLaunchKernelGGL(k_count_units, dim3((unsigned)((w.n_units + 255) / 256)), dim3(256), 0, stream, w);
        hip_check(hipGetLastError(), "k_count_units launch");
    }
}

// Large batches run in chunks of whole edges (mode A: whole poses) of about split_chunk_units
// units, by offsetting the pointers: the per-launch candidate segments and spill list then
// hold a chunk's candidates instead of overflowing to the fused kernel (config 4's 21 M
// poses overflowed 8 M units).  The scratch is sized for one chunk.
void launch_collide_split(const EnvDev &env, const AgentDev *d_links, int32_t max_clusters, const CollideWork &w,
                          CollideScratch &s, hipStream_t stream, hipEvent_t *marks, OvfDefer *defer) {
    if (defer) defer->n_ovf = nullptr;
    const int64_t g = w.pose_edge ? (int64_t)w.L : (int64_t)w.pmax * w.L;
    const int64_t per = std::max<int64_t>(g, (split_chunk_units(max_clusters) / g) * g);
    if (w.n_units <= per) {
        collide_split_chunk(env, d_links, max_clusters, w, s, stream, marks, defer);
        return;
    }
    for (int64_t u0 = 0; u0 < w.n_units; u0 += per) {
        CollideWork c = w;
        c.live_units = nullptr;  // absolute unit indices: not per chunk
        c.n_live = nullptr;
        if (w.unit_tmask) c.unit_tmask = w.unit_tmask + u0;  // chunks hold whole edges: unit u0 first
        c.n_units = std::min(per, w.n_units - u0);
        if (w.pose_edge) {
            const int64_t p0 = u0 / w.L;
            c.poses = w.poses + p0 * w.L * 12;
            if (w.unit_rt) c.unit_rt = w.unit_rt + p0 * w.L * 12;
            c.pose_edge = w.pose_edge + p0;
        } else {
            const int64_t e0 = u0 / g;
            c.poses = w.poses + e0 * g * 12;
            if (w.unit_rt) c.unit_rt = w.unit_rt + e0 * g * 12;
            c.pcount = w.pcount + e0;
            c.verdict = w.verdict + e0;
        }
        collide_split_chunk(env, d_links, max_clusters, c, s, stream, u0 + per >= w.n_units ? marks : nullptr,
                            nullptr);
    }
}

}  // namespace mpt
