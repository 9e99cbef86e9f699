// cell_tree.hip -- the engine's incremental exact 1-NN index (cell_tree.h).
//
// FLANN_KDTreeWrapper (utilities/flannkdtreewrapper.hpp:27-40) inserts each point into a live
// kd-tree and FLANN 1.8.4 rebuilds it on every insert; a batched round here inserts its K new
// points at once and touches only what they fall in.
//
// Codes.  A point's code interleaves its state dims quantised with one step h over the
// sampling ranges (126 bits: the step is fine enough that distinct states get distinct codes,
// where 63 bits left ~4 RRT nodes a cell), so a code never changes and code order is a fixed
// space-filling order.
//
// Buckets.  The indexed points live in buckets of at most 8 (one lane each in the walk), each
// the points of one interval [start, next start) of code space; the directory lists the
// buckets by start.  A round sorts its new points by code, finds each one's bucket by a
// binary search of the directory, and either appends them (the bucket still holds at most 8)
// or splits the bucket: its old and new points, merged in code order, are cut into maximal
// aligned code cells of at most 8 points -- points i - 1 and i share a bucket iff the smallest
// cell holding both holds at most 8 of them -- and every bucket after the first gets a new
// directory entry starting at the cell boundary.  Buckets are therefore cells of the code
// space's binary trie, as a radix tree's leaves, and a round's work is its new points and the
// buckets they touch.
//
// Boxes.  Above the directory an implicit 8-ary hierarchy (level 1 = each directory entry's
// bucket box, level l = 8 consecutive level-(l - 1) boxes) is rebuilt each round from the
// bucket boxes (~1/5 of a float box a point).  The walk is the Morton tree's (point_tree.hip):
// 8 nodes a step, one query a wave, seeded by the tree's extreme points.
//
// Every result is exact whatever the buckets and boxes are (only boxes whose float lower bound
// exceeds the best are skipped), so the layout decides speed only.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <type_traits>
#include <cmath>

#include "cell_tree.h"

namespace mpt {

namespace {

// ---- 128-bit codes as (hi, lo) ----

// (code, row) total order
__device__ __forceinline__ bool cr_lt(uint64_t ah, uint64_t al, int32_t ar, uint64_t bh, uint64_t bl, int32_t br) {
    return (ah < bh) | ((ah == bh) & ((al < bl) | ((al == bl) & (ar < br))));
}
// common prefix length of two codes (128: equal)
__device__ __forceinline__ int c_cpl(uint64_t ah, uint64_t al, uint64_t bh, uint64_t bl) {
    const uint64_t xh = ah ^ bh, xl = al ^ bl;
    return xh ? __clzll((long long)xh) : (xl ? 64 + __clzll((long long)xl) : 128);
}
// the aligned cell boundary between two codes a < b: b with every bit below its first
// difference from a cleared (the start of the cell of b's side)
__device__ __forceinline__ void c_boundary(uint64_t ah, uint64_t al, uint64_t &bh, uint64_t &bl) {
    const int k = c_cpl(ah, al, bh, bl);
    if (k >= 127) return;     // equal, or differ in the last bit only: b itself
    const int keep = k + 1;   // the common prefix and the differing bit
    if (keep <= 64) {
        bh &= keep == 64 ? ~0ull : ~(~0ull >> keep);
        bl = 0;
    } else {
        bl &= ~(~0ull >> (keep - 64));
    }
}

__device__ __forceinline__ unsigned long long okey(double x) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(x);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

template <int D>
__device__ __forceinline__ void ct_code(const CtPlan &P, const double (&x)[D], uint64_t &h, uint64_t &l) {
    uint32_t q[D];
#pragma unroll
    for (int j = 0; j < D; ++j) {
        const double u = (x[j] - P.lo[j]) * P.scale[j];
        const uint32_t m = P.qmax[j];
        q[j] = u <= 0.0 ? 0u : (u >= (double)m ? m : (uint32_t)u);
    }
    // level by level (MSB first): the level's bits of the dims that have one, gathered into a
    // word and shifted in together (the plan's dim / bit order).  The plan is the same for
    // every lane: its bit counts go to scalar registers, so which dims a level takes and the
    // shift amounts are scalar work, and the vector work is the bits themselves.
    int nb[D];
#pragma unroll
    for (int j = 0; j < D; ++j) nb[j] = __builtin_amdgcn_readfirstlane(P.nb[j]);
    const int bmax = __builtin_amdgcn_readfirstlane(P.bmax);
    h = 0;
    l = 0;
    for (int lev = bmax - 1; lev >= 0; --lev) {
        uint32_t w = 0;
        int c = 0;
#pragma unroll
        for (int j = 0; j < D; ++j)
            if (nb[j] > lev) {
                w = (w << 1) | ((q[j] >> lev) & 1u);
                ++c;
            }
        h = (h << c) | (l >> (64 - c));  // 1 <= c <= D: the widest dim has a bit at every level
        l = (l << c) | w;
    }
}

// Seed slots (cell_tree.h kCtHull): lane h of a wave scores slot h over the wave's 64 points
// (staged in LDS: every lane reads the same point at once) and offers its best to
// the tree's slot with one 64-bit atomicMax of (score as an ordered float key << 32 | row).
// Rows of a wave are consecutive (row0 + lane).  The float rounding of the score only decides
// which near-tie becomes the seed; any point is a valid seed.
constexpr int kCtWaves = 4;  // waves of the workgroups that stage rows (256 threads)
template <int D>
__device__ __forceinline__ void hull_offer(const CtPlan &P, const double (&x)[D], bool live, int64_t row0,
                                           double (*s_rows)[D], unsigned long long *__restrict__ keys) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int j = 0; j < D; ++j) s_rows[lane][j] = live ? x[j] : 0.0;
    const uint64_t lm = __ballot(live);
    __builtin_amdgcn_wave_barrier();
    if (lane < P.n_hull) {
        // one form for every kind (no divergence between the lanes' kinds): c0 x[i0] + c1 x[i1]
        // + c2 x[i2]; kind 1 / 2 is -1 / +1 times x[hdim] (the other terms 0 x[hdim])
        const int kind = P.hkind[lane], dm = P.hdim[lane];
        const bool dir = kind == 0;
        const int i0 = dir ? 0 : dm, i1 = dir ? (D > 1 ? 1 : 0) : dm, i2 = dir ? (D > 2 ? 2 : 0) : dm;
        const double c0 = dir ? (double)P.hdir[lane][0] : (kind == 1 ? -1.0 : 1.0);
        const double c1 = dir && D > 1 ? (double)P.hdir[lane][1] : 0.0;
        const double c2 = dir && D > 2 ? (double)P.hdir[lane][2] : 0.0;
        unsigned long long best = 0;
        // every point of the wave, unrolled by 8 so the LDS reads overlap (a loop over the live
        // mask's bits waited out each point's reads); dead points score key 0
#pragma unroll 8
        for (int j = 0; j < 64; ++j) {
            const double v = c0 * s_rows[j][i0] + c1 * s_rows[j][i1] + c2 * s_rows[j][i2];
            const uint32_t b = __float_as_uint((float)v);
            const uint32_t key = (b & 0x80000000u) ? ~b : (b | 0x80000000u);
            const unsigned long long k64 = ((unsigned long long)key << 32) | (uint32_t)(row0 + j);
            best = ((lm >> j) & 1) && k64 > best ? k64 : best;
        }
        if (best) atomicMax(keys + lane, best);
    }
    __builtin_amdgcn_wave_barrier();
}

// the box of rows (widened float bounds over every dim).  A box is D (lo, -hi) float pairs,
// dim by dim: pair k is one 8-byte word, so the walk's lower bound takes dim k's two gaps in
// one packed addition (ct_box_lb), and a union of boxes is a minimum of both halves (an empty
// box: (+inf, +inf))
template <int D>
__device__ __forceinline__ void write_box(float *__restrict__ b, const double (&lo)[D], const double (&hi)[D]) {
#pragma unroll
    for (int k = 0; k < D; ++k) {
        b[2 * k] = widen_lo(lo[k]);
        b[2 * k + 1] = -widen_hi(hi[k]);
    }
}

// the job table on the device (a joint build), or one job in the kernel arguments
struct CtJobs {
    const CtJob *table;
    CtJob one;
};
#define CT_JOB(js) ((js).table ? (js).table[blockIdx.y] : (js).one)

// this round's new points: the rows past the indexed count, at most the host's bound mb (the
// grids are sized by it; a device count beyond it -- a host bound broken, reported by
// k_ct_ncodes into counters[6] -- leaves the rest for the next round instead of indexing rows
// no kernel coded)
__device__ __forceinline__ int64_t ct_new_count(const CtJob &J) {
    const int64_t m = *J.T.n_dev - J.cnt->nidx, cap = J.mb < kCtSeg ? J.mb : kCtSeg;
    return m < 0 ? 0 : (m > cap ? cap : m);
}

constexpr uint32_t kCtLeafBit = 0x80000000u;
__device__ __forceinline__ uint32_t leaf_code(int32_t bucket, int32_t count) {
    return kCtLeafBit | ((uint32_t)(count - 1) << 28) | (uint32_t)bucket;
}
__device__ __forceinline__ uint32_t inner_code(int64_t first, int32_t count) {
    return ((uint32_t)(count - 1) << 28) | (uint32_t)first;
}

// ---- a round's new points ----

// codes and rows of the new points [nidx, n) in row order, their box into ibox, their offers
// to the seed slots
template <int D>
__global__ __launch_bounds__(64 * kCtWaves) void k_ct_ncodes(CtJobs js) {
    __shared__ CtPlan s_plan;
    __shared__ double s_rows[kCtWaves][64][D];
    __shared__ unsigned long long s_keys[kCtHull], s_ibox[6];  // the workgroup's offers, then one global atomic each
    const CtJob J = CT_JOB(js);  // by value: the fields stay in registers across the stores
    // the plan's loads in flight with the counts' (a workgroup past the new points still exits
    // before its first barrier)
    for (int w = threadIdx.x; w < (int)(sizeof(CtPlan) / 4); w += blockDim.x)
        reinterpret_cast<uint32_t *>(&s_plan)[w] = reinterpret_cast<const uint32_t *>(J.plan)[w];
    if (threadIdx.x < kCtHull) s_keys[threadIdx.x] = 0ull;
    if (threadIdx.x < 6) s_ibox[threadIdx.x] = threadIdx.x < 3 ? ~0ull : 0ull;
    const int64_t base = J.cnt->nidx, mraw = *J.T.n_dev - base;
    if ((mraw > kCtSeg || mraw > J.mb) && blockIdx.x == 0 && threadIdx.x == 0 && J.err)
        atomicAdd(J.err, 1ull);  // the host's bound broken
    const int64_t m = ct_new_count(J);
    const int i = (int)blockIdx.x * (int)blockDim.x + (int)threadIdx.x;
    if ((int64_t)blockIdx.x * blockDim.x >= m) return;  // block-uniform
    __syncthreads();
    const bool live = i < m;
    double x[D];
    if (live) {
        const int64_t row = base + i;
        load_global<D>(J.pts + row * D, x);
        uint64_t h, l;
        ct_code<D>(s_plan, x, h, l);
        J.ncode[2 * i] = h;
        J.ncode[2 * i + 1] = l;
        J.nrow[i] = (int32_t)row;
    } else {
#pragma unroll
        for (int j = 0; j < D; ++j) x[j] = 0.0;
    }
    // the persistent box over dims 0..2 only: its one reader is k_ct_levels' copy for the
    // engine's MPT_NN_AUTO spread, whose dims are the first two or three (rrt_engine grid_dims)
#pragma unroll
    for (int j = 0; j < (D < 3 ? D : 3); ++j) {
        unsigned long long mn = live ? okey(x[j]) : ~0ull, mx = live ? okey(x[j]) : 0ull;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const unsigned long long omn = __shfl_xor(mn, off), omx = __shfl_xor(mx, off);
            mn = omn < mn ? omn : mn;
            mx = omx > mx ? omx : mx;
        }
        if ((threadIdx.x & 63) == 0) {
            atomicMin(s_ibox + j, mn);
            atomicMax(s_ibox + 3 + j, mx);
        }
    }
    hull_offer<D>(s_plan, x, live, base + (i & ~63), s_rows[threadIdx.x >> 6], s_keys);
    // one global atomic a slot a workgroup (not one a wave: the tree's offers to a slot are
    // serialised at one address)
    __syncthreads();
    if (threadIdx.x < kCtHull && s_keys[threadIdx.x]) atomicMax(J.hull_keys + threadIdx.x, s_keys[threadIdx.x]);
    if (threadIdx.x < (D < 3 ? D : 3)) {
        atomicMin(J.ibox + threadIdx.x, s_ibox[threadIdx.x]);
        atomicMax(J.ibox + kCtMaxDim + threadIdx.x, s_ibox[3 + threadIdx.x]);
    }
}

// (code, row) compare-exchange by selects (no divergent branches)
__device__ __forceinline__ void cx3(uint64_t &h, uint64_t &l, int32_t &r, uint64_t ph, uint64_t pl, int32_t pr,
                                    bool keep_min) {
    const bool sw = keep_min == cr_lt(ph, pl, pr, h, l, r);
    h = sw ? ph : h;
    l = sw ? pl : l;
    r = sw ? pr : r;
}

// The new points' sort over many CUs: a 256-thread workgroup sorts a chunk of 512 (code, row)
// pairs, 2 a thread (bitonic: the partner 1 apart in registers, 2..64 apart by lane shuffles in
// the wave, 128+ apart through LDS); then every element's rank = its index in its chunk + the
// count of smaller pairs in each other chunk (fixed-step binary searches).  (One wave a chunk,
// 8 pairs a lane, ran 36 us at 32 seeds: one wave a SIMD and a long serial chain each.)
constexpr int kCtChunk = 512;
constexpr int kCtChunks = kCtSeg / kCtChunk;
constexpr int kCtSortThreads = kCtChunk / 2;

__global__ __launch_bounds__(kCtSortThreads) void k_ct_csort(CtJobs js) {
    const CtJob J = CT_JOB(js);  // by value: the fields stay in registers across the stores
    __shared__ uint64_t s_h[kCtChunk], s_l[kCtChunk];
    __shared__ int32_t s_r[kCtChunk];
    const int64_t m = ct_new_count(J);
    const int c0 = (int)blockIdx.x * kCtChunk;
    if (c0 >= m) return;  // block-uniform
    const int t = threadIdx.x;
    uint64_t kh[2], kl[2];
    int32_t kr[2];
#pragma unroll
    for (int a = 0; a < 2; ++a) {
        const int i = c0 + 2 * t + a;
        const bool live = i < m;
        kh[a] = live ? J.ncode[2 * i] : ~0ull;  // padding sorts last (codes use 126 bits)
        kl[a] = live ? J.ncode[2 * i + 1] : ~0ull;
        kr[a] = live ? J.nrow[i] : 0x7fffffff;
    }
#pragma unroll 1
    for (int k = 2; k <= kCtChunk; k <<= 1) {
#pragma unroll 1
        for (int j = k >> 1; j > 0; j >>= 1) {
            const bool up = ((2 * t) & k) == 0;  // this thread's pairs sort ascending
            if (j == 1) {
                const bool sw = up == cr_lt(kh[1], kl[1], kr[1], kh[0], kl[0], kr[0]);
                const uint64_t h0 = kh[0], l0 = kl[0];
                const int32_t r0 = kr[0];
                kh[0] = sw ? kh[1] : h0;
                kl[0] = sw ? kl[1] : l0;
                kr[0] = sw ? kr[1] : r0;
                kh[1] = sw ? h0 : kh[1];
                kl[1] = sw ? l0 : kl[1];
                kr[1] = sw ? r0 : kr[1];
            } else if (j < 128) {  // partner thread t ^ (j / 2), in this wave
                const int lm = j >> 1;
                const bool lower = (t & lm) == 0;
#pragma unroll
                for (int a = 0; a < 2; ++a) {
                    const uint64_t ph = __shfl_xor(kh[a], lm), pl = __shfl_xor(kl[a], lm);
                    const int32_t pr = __shfl_xor(kr[a], lm);
                    cx3(kh[a], kl[a], kr[a], ph, pl, pr, lower == up);
                }
            } else {  // partner thread t ^ (j / 2) in another wave: through LDS
                const bool lower = (t & (j >> 1)) == 0;
                __syncthreads();
#pragma unroll
                for (int a = 0; a < 2; ++a) {
                    s_h[2 * t + a] = kh[a];
                    s_l[2 * t + a] = kl[a];
                    s_r[2 * t + a] = kr[a];
                }
                __syncthreads();
#pragma unroll
                for (int a = 0; a < 2; ++a) {
                    const int p = (2 * t + a) ^ j;
                    cx3(kh[a], kl[a], kr[a], s_h[p], s_l[p], s_r[p], lower == up);
                }
            }
        }
    }
#pragma unroll
    for (int a = 0; a < 2; ++a) {
        const int i = c0 + 2 * t + a;
        J.ccode[2 * i] = kh[a];
        J.ccode[2 * i + 1] = kl[a];
        J.crow[i] = kr[a];
    }
}

// Every 8th element of each chunk (the last of each group of 8) is staged in LDS: the binary
// search's steps of 256 .. 8 probe exactly those, so they run in LDS and only the steps of 4, 2
// and 1 and the last probe read global memory (4 dependent loads, not 10).
constexpr int kCtRankGroup = 8;
constexpr int kCtRankSamples = kCtChunk / kCtRankGroup;  // 64 a chunk
template <int NC>
__device__ __forceinline__ void ct_crank_n(const CtJob &J, int64_t m, int e, const uint64_t *s_h, const uint64_t *s_l,
                                           const int32_t *s_r) {
    const int nch = (int)((m + kCtChunk - 1) / kCtChunk);
    const uint64_t h = J.ccode[2 * e], l = J.ccode[2 * e + 1];
    const int32_t r = J.crow[e];
    int pos[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) pos[c] = 0;
#pragma unroll
    for (int st = kCtChunk / 2; st >= kCtRankGroup; st >>= 1) {
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const int q = c * kCtRankSamples + (pos[c] + st) / kCtRankGroup - 1;  // element pos + st - 1
            pos[c] += cr_lt(s_h[q], s_l[q], s_r[q], h, l, r) ? st : 0;
        }
    }
#pragma unroll
    for (int st = kCtRankGroup / 2; st > 0; st >>= 1) {
        uint64_t ph[NC], pl[NC];
        int32_t pr[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const int q = c * kCtChunk + pos[c] + st - 1;
            ph[c] = J.ccode[2 * q];
            pl[c] = J.ccode[2 * q + 1];
            pr[c] = J.crow[q];
        }
#pragma unroll
        for (int c = 0; c < NC; ++c) pos[c] += cr_lt(ph[c], pl[c], pr[c], h, l, r) ? st : 0;
    }
    int rank = 0;
    {
        uint64_t ph[NC], pl[NC];
        int32_t pr[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const int q = c * kCtChunk + pos[c];
            ph[c] = J.ccode[2 * q];
            pl[c] = J.ccode[2 * q + 1];
            pr[c] = J.crow[q];
        }
#pragma unroll
        for (int c = 0; c < NC; ++c) rank += c < nch ? pos[c] + (cr_lt(ph[c], pl[c], pr[c], h, l, r) ? 1 : 0) : 0;
    }
    J.ncode[2 * rank] = h;
    J.ncode[2 * rank + 1] = l;
    J.nrow[rank] = r;
}

__global__ __launch_bounds__(256) void k_ct_crank(CtJobs js) {
    const CtJob J = CT_JOB(js);  // by value: the fields stay in registers across the stores
    __shared__ uint64_t s_h[kCtChunks * kCtRankSamples], s_l[kCtChunks * kCtRankSamples];
    __shared__ int32_t s_r[kCtChunks * kCtRankSamples];
    const int64_t m = ct_new_count(J);
    if ((int64_t)blockIdx.x * blockDim.x >= m) return;  // block-uniform
    const int nch = (int)((m + kCtChunk - 1) / kCtChunk);
    const int NCs = m <= (int64_t)kCtChunk * 4 ? 4 : m <= (int64_t)kCtChunk * 8 ? 8 : kCtChunks;
    for (int v = threadIdx.x; v < NCs * kCtRankSamples; v += blockDim.x) {
        const int c = v / kCtRankSamples;
        const int q = c * kCtChunk + (v - c * kCtRankSamples) * kCtRankGroup + kCtRankGroup - 1;
        const bool in = c < nch;  // chunks past the last are never counted (their probes only steer)
        s_h[v] = in ? J.ccode[2 * q] : ~0ull;
        s_l[v] = in ? J.ccode[2 * q + 1] : ~0ull;
        s_r[v] = in ? J.crow[q] : 0x7fffffff;
    }
    __syncthreads();
    const int e = (int)blockIdx.x * (int)blockDim.x + (int)threadIdx.x;
    if (e >= m) return;
    if (NCs == 4) ct_crank_n<4>(J, m, e, s_h, s_l, s_r);
    else if (NCs == 8) ct_crank_n<8>(J, m, e, s_h, s_l, s_r);  // a round's K = 4096: 8 chunks
    else ct_crank_n<kCtChunks>(J, m, e, s_h, s_l, s_r);
}

// each sorted new point's directory position: the last entry whose start is <= its code
__global__ __launch_bounds__(256) void k_ct_locate(CtJobs js) {
    const CtJob J = CT_JOB(js);  // by value: the fields stay in registers across the stores
    const int64_t m = ct_new_count(J);
    const int j = (int)blockIdx.x * (int)blockDim.x + (int)threadIdx.x;
    if (j >= m) return;
    const uint64_t h = J.ncode[2 * j], l = J.ncode[2 * j + 1];
    int lo = 0, hi = J.cnt->n_dir;  // entry 0 starts at code 0: the answer is in [0, n_dir)
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        const uint64_t sh = J.odir_code[2 * mid], sl = J.odir_code[2 * mid + 1];
        if (sh < h || (sh == h && sl <= l)) lo = mid;
        else hi = mid;
    }
    J.npos[j] = lo;
}

// The segments' records (k_ct_segments, after its head scan): segment s =
// (bucket, old count c, new count k, scratch offset), its directory position and first point.
// Only split segments (c + k > kCtCap) take scratch -- their c + k merged elements, packed in
// segment order -- so the split kernels visit live elements only.
template <int PER, int T>
__device__ __forceinline__ void ct_write_segments(const CtJob &J, int m, const int32_t (&pos)[PER],
                                                  const int (&head)[PER], int s0, int s_total,
                                                  const int32_t *s_first, int32_t *s_sum) {
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    int32_t b[PER], c[PER], k[PER];
    int sz = 0, sg = s0;
    // the heads' buckets, then their counts: each pass's loads all in flight together
#pragma unroll
    for (int a = 0; a < PER; ++a) {
        const bool h = t * PER + a < m && head[a];
        b[a] = h ? (int32_t)(J.ometa[pos[a]] & 0x0fffffffu) : 0;
    }
#pragma unroll
    for (int a = 0; a < PER; ++a) {
        const bool h = t * PER + a < m && head[a];
        c[a] = h ? J.bcnt[b[a]] : 0;
    }
#pragma unroll
    for (int a = 0; a < PER; ++a) {
        const int j = t * PER + a;
        k[a] = 0;
        if (j >= m) continue;
        sg += head[a];
        if (!head[a]) continue;
        k[a] = s_first[sg + 1] - j;
        sz += c[a] + k[a] > kCtCap ? c[a] + k[a] : 0;
    }
    int incl = sz;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int o = __shfl_up(incl, off);
        if (lane >= off) incl += o;
    }
    __syncthreads();
    if (lane == 63) s_sum[wave] = incl;
    __syncthreads();
    int before = 0, tot = 0;
    for (int w = 0; w < T / 64; ++w) {
        before += w < wave ? s_sum[w] : 0;
        tot += s_sum[w];
    }
    int off = before + incl - sz;
    sg = s0;
#pragma unroll
    for (int a = 0; a < PER; ++a) {
        const int j = t * PER + a;
        if (j >= m) break;
        sg += head[a];
        if (!head[a]) continue;
        const bool split = c[a] + k[a] > kCtCap;
        J.seg[sg] = make_int4(b[a], c[a], k[a], split ? off : -1);
        J.seg_pos[sg] = pos[a];
        J.seg_first[sg] = j;
        off += split ? c[a] + k[a] : 0;
    }
    if (t == 0) {
        J.cnt->n_seg = s_total;
        J.cnt->n_scratch = tot;
    }
}

// One workgroup a tree: the runs of equal directory positions (the touched buckets) become the
// round's segments (ct_write_segments).
constexpr int kCtSegThreads = 1024;
constexpr int kCtSegPer = kCtSeg / kCtSegThreads;

__global__ __launch_bounds__(kCtSegThreads) void k_ct_segments(CtJobs js) {
    const CtJob J = CT_JOB(js);  // by value: the fields stay in registers across the stores
    __shared__ int32_t s_sum[kCtSegThreads / 64];
    __shared__ int32_t s_total;
    __shared__ int32_t s_first[kCtSeg + 1];  // each segment's first new point
    const int64_t m = ct_new_count(J);
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    int32_t pos[kCtSegPer];
    int head[kCtSegPer];
    int cnt = 0;
#pragma unroll
    for (int a = 0; a < kCtSegPer; ++a) {
        const int j = t * kCtSegPer + a;
        pos[a] = j < m ? J.npos[j] : -1;
    }
    const int32_t prev = (t * kCtSegPer > 0 && t * kCtSegPer - 1 < m) ? J.npos[t * kCtSegPer - 1] : -2;
#pragma unroll
    for (int a = 0; a < kCtSegPer; ++a) {
        const int j = t * kCtSegPer + a;
        const int32_t pv = a == 0 ? prev : pos[a - 1];
        head[a] = (j < m && (j == 0 || pos[a] != pv)) ? 1 : 0;
        cnt += head[a];
    }
    // block exclusive scan of the head counts
    int incl = cnt;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int o = __shfl_up(incl, off);
        if (lane >= off) incl += o;
    }
    if (lane == 63) s_sum[wave] = incl;
    __syncthreads();
    if (t == 0) {
        int acc = 0;
        for (int w = 0; w < kCtSegThreads / 64; ++w) {
            const int v = s_sum[w];
            s_sum[w] = acc;
            acc += v;
        }
        s_total = acc;
        s_first[acc] = (int32_t)m;
    }
    __syncthreads();
    const int s0 = s_sum[wave] + incl - cnt - 1;  // segment of the element before this thread's first
    int s = s0;
#pragma unroll
    for (int a = 0; a < kCtSegPer; ++a) {
        const int j = t * kCtSegPer + a;
        if (j >= m) break;
        s += head[a];
        J.nseg[j] = s;
        if (head[a]) s_first[s] = j;
    }
    __syncthreads();
    ct_write_segments<kCtSegPer, kCtSegThreads>(J, (int)m, pos, head, s0, s_total, s_first, s_sum);
}

// Per sorted new point: appended to its bucket, or placed in its split segment's merged list
// with the old points just below it (on append, the segment's first point sets the bucket's
// count and box).
template <int D>
__global__ __launch_bounds__(256) void k_ct_apply(CtJobs js) {
    const CtJob J = CT_JOB(js);  // by value: the fields stay in registers across the stores
    const int64_t m = ct_new_count(J);
    const int j = (int)blockIdx.x * (int)blockDim.x + (int)threadIdx.x;
    if (j >= m) return;
    const int s = J.nseg[j];
    const int4 g = J.seg[s];
    const int32_t b = g.x, c = g.y, k = g.z, off = g.w;
    const int32_t j0 = J.seg_first[s];
    const uint64_t h = J.ncode[2 * j], l = J.ncode[2 * j + 1];
    const int32_t row = J.nrow[j];
    if (c + k <= kCtCap) {
        const int64_t slot = (int64_t)b * kCtCap + c + (j - j0);
        double x[D];
        load_global<D>(J.pts + (int64_t)row * D, x);
#pragma unroll
        for (int q = 0; q < D; ++q) J.bpts[slot * D + q] = x[q];
        J.bids[slot] = row + 1;
        J.bcode[2 * slot] = h;
        J.bcode[2 * slot + 1] = l;
        if (j == j0) {
            double lo[D], hi[D];
            if (c > 0) {
                const float *ob = J.bbox + (int64_t)b * 2 * D;
#pragma unroll
                for (int q = 0; q < D; ++q) {
                    lo[q] = (double)ob[2 * q];  // widened already: widening again only loosens it
                    hi[q] = -(double)ob[2 * q + 1];
                }
            } else {
#pragma unroll
                for (int q = 0; q < D; ++q) {
                    lo[q] = __builtin_huge_val();
                    hi[q] = -__builtin_huge_val();
                }
            }
            // the segment's k <= 8 rows, then their points: unconditional loads (slots past k
            // repeat its last point), so each pass's loads are in flight together -- a loop over
            // k waited out two dependent loads a point
            int32_t rs[kCtCap];
#pragma unroll
            for (int u = 0; u < kCtCap; ++u) rs[u] = J.nrow[j0 + (u < k ? u : k - 1)];
#pragma unroll
            for (int u = 0; u < kCtCap; ++u) {
                double y[D];
                load_global<D>(J.pts + (int64_t)rs[u] * D, y);
#pragma unroll
                for (int q = 0; q < D; ++q) {
                    lo[q] = y[q] < lo[q] ? y[q] : lo[q];
                    hi[q] = y[q] > hi[q] ? y[q] : hi[q];
                }
            }
            write_box<D>(J.bbox + (int64_t)b * 2 * D, lo, hi);
            J.bcnt[b] = c + k;
            const int64_t dp = J.seg_pos[s];  // the bucket's record in last round's directory
            write_box<D>(J.obox + dp * 2 * D, lo, hi);
            J.ometa[dp] = leaf_code(b, c + k);
        }
        return;
    }
    // split: this point's place in the merged list = its index among the new + the old points
    // below it.  The bucket's old (code, row) pairs into registers first (independent loads).
    uint64_t oh[kCtCap], ol[kCtCap];
    int32_t orw[kCtCap];
#pragma unroll
    for (int o = 0; o < kCtCap; ++o) {
        const int64_t os = (int64_t)b * kCtCap + (o < c ? o : 0);
        oh[o] = J.bcode[2 * os];
        ol[o] = J.bcode[2 * os + 1];
        orw[o] = J.bids[os] - 1;
    }
    // and the previous new point's (the segment's points are sorted, so `below` never falls)
    const int jp = j > j0 ? j - 1 : j;
    const uint64_t ph = J.ncode[2 * jp], pl = J.ncode[2 * jp + 1];
    const int32_t pr = J.nrow[jp];
    int below = 0, below_prev = 0;
#pragma unroll
    for (int o = 0; o < kCtCap; ++o) {
        below += (o < c && cr_lt(oh[o], ol[o], orw[o], h, l, row)) ? 1 : 0;
        below_prev += (o < c && cr_lt(oh[o], ol[o], orw[o], ph, pl, pr)) ? 1 : 0;
    }
    if (j == j0) below_prev = 0;
    const int32_t e = off + (j - j0) + below;
    J.scode[2 * e] = h;
    J.scode[2 * e + 1] = l;
    J.srow[e] = row;
    J.sseg[e] = s;
    // The old points of ranks [below_prev, below) lie between the previous new point and this
    // one: j - j0 new points below them.  The segment's last point also places the old points
    // above it (k new points below them).  Every old point is placed once, by the new point
    // after it, with no searches (a segment's first point searching for all of them waited out
    // up to 8 dependent binary searches).
    const int r_hi = j == j0 + k - 1 ? c : below;
    if (below_prev >= r_hi) return;
#pragma unroll
    for (int o = 0; o < kCtCap; ++o) {
        if (o >= c) break;
        int ob = 0;  // old point o's rank among the old points
#pragma unroll
        for (int o2 = 0; o2 < kCtCap; ++o2) ob += (o2 < c && cr_lt(oh[o2], ol[o2], orw[o2], oh[o], ol[o], orw[o])) ? 1 : 0;
        if (ob < below_prev || ob >= r_hi) continue;
        const int32_t eo = off + ob + (ob < below ? j - j0 : k);
        J.scode[2 * eo] = oh[o];
        J.scode[2 * eo + 1] = ol[o];
        J.srow[eo] = orw[o];
        J.sseg[eo] = s;
    }
}

// Do elements i - 1 and i of a sorted run [lo, hi) share a bucket?  Yes iff the smallest code
// cell holding both holds at most 8 of the run's elements (a contiguous range around them);
// equal codes that are more than 8 are grouped by row / 8 instead.  Leaves formed this way
// hold at most 8: a leaf lies inside the largest of its pairs' cells.
__device__ __forceinline__ bool ct_same(const uint64_t *__restrict__ code, const int32_t *__restrict__ row,
                                        int64_t lo, int64_t hi, int64_t i) {
    const uint64_t ah = code[2 * (i - 1)], al = code[2 * (i - 1) + 1];
    const uint64_t bh = code[2 * i], bl = code[2 * i + 1];
    const int k = c_cpl(ah, al, bh, bl);
    int cnt = 2;
    for (int64_t u = i - 2; u >= lo && cnt <= kCtCap; --u) {
        if (c_cpl(code[2 * u], code[2 * u + 1], bh, bl) < k) break;
        ++cnt;
    }
    for (int64_t u = i + 1; u < hi && cnt <= kCtCap; ++u) {
        if (c_cpl(code[2 * u], code[2 * u + 1], bh, bl) < k) break;
        ++cnt;
    }
    if (cnt <= kCtCap) return true;
    if (k < 128) return false;
    return row ? (row[i] >> 3) == (row[i - 1] >> 3) : ((i - lo) >> 3) == ((i - 1 - lo) >> 3);
}

// ct_same over adjacent prefix lengths a[u] = c_cpl(code u - 1, code u) (a window of them in
// LDS): the cell of elements i - 1, i at prefix length k = a[i] extends left over u while
// a[u] >= k and right likewise; equal codes (k = 128) that are more than 8 go by index / 8.
__device__ __forceinline__ bool ct_same_a(const uint8_t *__restrict__ a, int64_t lo, int64_t hi, int64_t i) {
    const int k = a[i];
    int cnt = 2;
    for (int64_t u = i - 1; u > lo && cnt <= kCtCap; --u) {
        if (a[u] < k) break;
        ++cnt;
    }
    for (int64_t u = i + 1; u < hi && cnt <= kCtCap; ++u) {
        if (a[u] < k) break;
        ++cnt;
    }
    if (cnt <= kCtCap) return true;
    if (k < 128) return false;
    return ((i - lo) >> 3) == ((i - 1 - lo) >> 3);
}

__device__ __forceinline__ int64_t ct_scratch_total(const CtJob &J) { return J.cnt->n_scratch; }

// leaf starts of the split segments: 1 the segment's first leaf (keeps the bucket), 2 a new leaf
// (ct_same over the adjacent prefix lengths of 256 elements and kCtCap either side, staged in
// LDS by one coalesced pass: ct_same's neighbour loads waited out each other, up to 14 in a row)
__global__ __launch_bounds__(256) void k_ct_split_flags(CtJobs js) {
    const CtJob J = CT_JOB(js);  // by value: the fields stay in registers across the stores
    __shared__ uint8_t s_a[256 + 2 * kCtCap];  // s_a[v] = c_cpl(element u - 1, element u), u = c0 - kCtCap + v
    const int64_t total = ct_scratch_total(J);
    for (int64_t c0 = (int64_t)blockIdx.x * 256; c0 < total; c0 += (int64_t)gridDim.x * 256) {
        for (int v = threadIdx.x; v < 256 + 2 * kCtCap; v += 256) {
            const int64_t u = c0 - kCtCap + v;
            int cp = 0;
            if (u >= 1 && u < total)
                cp = c_cpl(J.scode[2 * (u - 1)], J.scode[2 * (u - 1) + 1], J.scode[2 * u], J.scode[2 * u + 1]);
            s_a[v] = (uint8_t)cp;
        }
        __syncthreads();
        const int64_t e = c0 + threadIdx.x;
        if (e < total) {
            const int s = J.sseg[e];
            int flag = 0;
            if (s >= 0) {
                const int4 g = J.seg[s];
                const int64_t off = g.w, L = (int64_t)g.y + g.z;
                if (e == off) {
                    flag = 1;
                } else {
                    // ct_same (row rule for equal codes) over the segment [off, off + L)
                    const int i = (int)threadIdx.x + kCtCap;
                    const int k = s_a[i];
                    const int64_t lo = off - (c0 - kCtCap), hi = off + L - (c0 - kCtCap);
                    int cnt = 2;
                    for (int u = i - 1; u > lo && cnt <= kCtCap; --u) {
                        if (s_a[u] < k) break;
                        ++cnt;
                    }
                    for (int u = i + 1; u < hi && cnt <= kCtCap; ++u) {
                        if (s_a[u] < k) break;
                        ++cnt;
                    }
                    const bool same = cnt <= kCtCap ? true
                                      : k < 128     ? false
                                                    : (J.srow[e] >> 3) == (J.srow[e - 1] >> 3);
                    flag = same ? 0 : 2;
                }
            }
            J.slead[e] = flag;
        }
        __syncthreads();  // s_a reused by the next chunk
    }
}

// one workgroup a tree: each new leaf's rank among the round's new leaves (code order)
constexpr int kCtScanThreads = 1024;
__global__ __launch_bounds__(kCtScanThreads) void k_ct_split_scan(CtJobs js) {
    const CtJob J = CT_JOB(js);  // by value: the fields stay in registers across the stores
    __shared__ int32_t s_sum[kCtScanThreads / 64];
    const int64_t total = ct_scratch_total(J);
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int64_t per = (total + kCtScanThreads - 1) / kCtScanThreads;
    const int64_t e0 = t * per, e1 = e0 + per < total ? e0 + per : total;
    int cnt = 0;
    for (int64_t e = e0; e < e1; ++e) cnt += J.slead[e] == 2 ? 1 : 0;
    int incl = cnt;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int o = __shfl_up(incl, off);
        if (lane >= off) incl += o;
    }
    if (lane == 63) s_sum[wave] = incl;
    __syncthreads();
    if (t == 0) {
        int acc = 0;
        for (int w = 0; w < kCtScanThreads / 64; ++w) {
            const int v = s_sum[w];
            s_sum[w] = acc;
            acc += v;
        }
        J.cnt->n_new_dir = acc;
    }
    __syncthreads();
    int r = s_sum[wave] + incl - cnt;
    for (int64_t e = e0; e < e1; ++e) {
        J.srank[e] = r;
        r += J.slead[e] == 2 ? 1 : 0;
    }
}

// A split leaf's bucket: the segment's first leaf keeps the split bucket, a new leaf takes the
// next free bucket by its rank among the round's new leaves.
__device__ __forceinline__ int32_t ct_leaf_bucket(const CtJob &J, int64_t st, int flag, const int4 &g) {
    return flag == 1 ? g.x : J.cnt->n_buckets + J.srank[st];
}

// the leaf starting at split element e closes its bucket: count, box (from the rows), and the
// directory (a new leaf: its entry; the split bucket: its record updated in place)
template <int D>
__device__ __forceinline__ void ct_leaf_close(const CtJob &J, int64_t e, int flag, int s, int32_t b, int len,
                                              const double (*s_x)[D] = nullptr) {
    if (b >= J.bcap || len > kCtCap) {
        if (J.err) atomicAdd(J.err, 1ull);
        return;
    }
    if (flag == 2) {
        const int32_t r = J.srank[e];
        uint64_t bh = J.scode[2 * e], bl = J.scode[2 * e + 1];
        c_boundary(J.scode[2 * (e - 1)], J.scode[2 * (e - 1) + 1], bh, bl);
        J.edir_code[2 * r] = bh;
        J.edir_code[2 * r + 1] = bl;
        J.edir_bk[r] = b;
        J.edir_pos[r] = J.seg_pos[s];
    }
    double lo[D], hi[D];
#pragma unroll
    for (int q = 0; q < D; ++q) {
        lo[q] = __builtin_huge_val();
        hi[q] = -__builtin_huge_val();
    }
#pragma unroll
    for (int u = 0; u < kCtCap; ++u) {  // unrolled: the rows' loads are all in flight together
        if (u < len) {
            double x[D];
            if (s_x) {  // the leaf's rows as its elements' threads loaded them (LDS)
#pragma unroll
                for (int q = 0; q < D; ++q) x[q] = s_x[u][q];
            } else {
                load_global<D>(J.pts + (int64_t)J.srow[e + u] * D, x);
            }
#pragma unroll
            for (int q = 0; q < D; ++q) {
                lo[q] = x[q] < lo[q] ? x[q] : lo[q];
                hi[q] = x[q] > hi[q] ? x[q] : hi[q];
            }
        }
    }
    write_box<D>(J.bbox + (int64_t)b * 2 * D, lo, hi);
    J.bcnt[b] = len;
    if (flag == 1) {
        const int64_t dp = J.seg_pos[s];
        write_box<D>(J.obox + dp * 2 * D, lo, hi);
        J.ometa[dp] = leaf_code(b, len);
    }
}

// every split element copies its row into its leaf's bucket slot; each leaf's first element
// also closes the leaf (ct_leaf_close).  A workgroup takes 256 consecutive elements, their
// leaf flags and kCtCap either side staged in LDS for the walks to the leaf's ends.
template <int D>
__global__ __launch_bounds__(256) void k_ct_split_fill(CtJobs js) {
    const CtJob J = CT_JOB(js);  // by value: the fields stay in registers across the stores
    __shared__ int8_t s_f[256 + 2 * kCtCap];  // flag of element c0 - kCtCap + v; -1 past the ends
    __shared__ double s_x[256][D];             // the chunk's rows: a leaf inside it boxes from LDS
    const int64_t total = ct_scratch_total(J);
    for (int64_t c0 = (int64_t)blockIdx.x * 256; c0 < total; c0 += (int64_t)gridDim.x * 256) {
    // the element's own loads first, in flight with the flags' staging
    const int64_t e = c0 + threadIdx.x;
    const bool live = e < total;
    const int s = live ? J.sseg[e] : -1;
    const int32_t row = live ? J.srow[e] : 0;
    const uint64_t eh = live ? J.scode[2 * e] : 0, el = live ? J.scode[2 * e + 1] : 0;
    for (int v = threadIdx.x; v < 256 + 2 * kCtCap; v += 256) {
        const int64_t x = c0 - kCtCap + v;
        s_f[v] = (int8_t)(x >= 0 && x < total ? J.slead[x] : -1);
    }
    __syncthreads();
    const int ve = threadIdx.x + kCtCap;
    int flag = 0, len = 0;
    int32_t b = 0;
    if (s >= 0) {
        double x[D];
        load_global<D>(J.pts + (int64_t)row * D, x);  // (its bucket is not needed to load it)
        int vs = ve;  // the leaf's first element (a segment's first element starts a leaf)
        while (vs > 0 && s_f[vs] == 0) --vs;
        int64_t st = c0 - kCtCap + vs;
        if (s_f[vs] <= 0) {  // beyond the staged flags (a leaf longer than kCtCap: an index error)
            st = st < 0 ? 0 : st;
            while (st > 0 && J.slead[st] == 0) --st;
            flag = J.slead[st];
        } else {
            flag = s_f[vs];
        }
        const int4 g = J.seg[s];
        b = ct_leaf_bucket(J, st, flag, g);
        const int64_t u = e - st;
        if (b < J.bcap && u < kCtCap) {
            const int64_t slot = (int64_t)b * kCtCap + u;
#pragma unroll
            for (int q = 0; q < D; ++q) {
                J.bpts[slot * D + q] = x[q];
                s_x[threadIdx.x][q] = x[q];
            }
            J.bids[slot] = row + 1;
            J.bcode[2 * slot] = eh;
            J.bcode[2 * slot + 1] = el;
        }
        if (e == st) {
            const int64_t end = (int64_t)g.w + g.y + g.z;
            len = 1;
            while (e + len < end && len <= kCtCap && s_f[ve + len] == 0) ++len;
        }
    }
    __syncthreads();  // s_x complete
    if (len > 0) {  // this thread starts a leaf: close it
        const bool in_chunk = threadIdx.x + len <= 256 && len <= kCtCap;
        ct_leaf_close<D>(J, e, flag, s, b, len, in_chunk ? s_x + threadIdx.x : nullptr);
    }
    __syncthreads();  // s_f, s_x reused by the next chunk
    }
}

// The first index of a sorted a[0, n) whose value is >= key, by one wave: 64 probes a step
// (a 64-ary search: 2 dependent loads for n <= 4096 where a binary search by one lane waits
// out 12).  Every lane of the wave calls it and gets the answer.
__device__ __forceinline__ int32_t wave_lower_bound(const int32_t *__restrict__ a, int32_t n, int64_t key) {
    const int lane = threadIdx.x & 63;
    int32_t lo = 0, hi = n;  // the answer is in [lo, hi]
    while (lo < hi) {
        const int32_t step = (hi - lo + 63) / 64;
        const int32_t p = lo + (lane + 1) * step - 1;  // probe: is the answer past p?
        const bool less = p < hi && a[p] < key;
        const int32_t c = __popcll(__ballot(less));    // probes below key: lanes 0 .. c - 1
        const int32_t nlo = lo + c * step, nhi = lo + (c + 1) * step - 1;
        lo = nlo < hi ? nlo : hi;
        hi = nhi < hi ? nhi : hi;
    }
    return lo;
}

// The new directory: old entry p goes to p + (new entries of segments before p), new entry r
// (of the segment at directory position q) to q + 1 + r; with each entry its level-1 node (the
// bucket's box and meta: a stream of last round's records, the new entries' from their
// buckets).  A workgroup takes 256 consecutive old entries: two threads find the new entries
// bounding them, which are staged in LDS for the threads' searches; the boxes then move as
// 8-byte words, consecutive threads on consecutive words (coalesced both ways).
template <int D>
__global__ __launch_bounds__(256) void k_ct_dmerge(CtJobs js) {
    const CtJob J = CT_JOB(js);  // by value: the fields stay in registers across the stores
    __shared__ int32_t s_pos[256];
    __shared__ int32_t s_lo[2];
    __shared__ int32_t s_shift[256];
    const int64_t n_old = J.cnt->n_dir, n_new = J.cnt->n_new_dir;
    for (int64_t c0 = (int64_t)blockIdx.x * 256; c0 < n_old; c0 += (int64_t)gridDim.x * 256) {
        const int64_t t = c0 + threadIdx.x;
        if (threadIdx.x < 128) {  // new entries whose segment lies before c0 / before the chunk's end
            const int wv = threadIdx.x >> 6;  // wave 0: c0, wave 1: the chunk's end
            const int64_t key = wv == 0 ? c0 : (c0 + 256 < n_old ? c0 + 256 : n_old);
            const int32_t lo = wave_lower_bound(J.edir_pos, (int32_t)n_new, key);
            if ((threadIdx.x & 63) == 0) s_lo[wv] = lo;
        }
        __syncthreads();
        const int32_t lo_a = s_lo[0], lo_b = s_lo[1];
        const bool staged = lo_b - lo_a <= 256;
        if (staged && threadIdx.x < lo_b - lo_a) s_pos[threadIdx.x] = J.edir_pos[lo_a + threadIdx.x];
        __syncthreads();
        if (t < n_old) {
            int32_t lo = lo_a, hi = lo_b;
            while (lo < hi) {
                const int32_t mid = (lo + hi) >> 1;
                if ((staged ? s_pos[mid - lo_a] : J.edir_pos[mid]) < t) lo = mid + 1;
                else hi = mid;
            }
            const int64_t out = t + lo;
            s_shift[threadIdx.x] = lo;
            J.ndir_code[2 * out] = J.odir_code[2 * t];
            J.ndir_code[2 * out + 1] = J.odir_code[2 * t + 1];
            J.nmeta[out] = J.ometa[t];
        }
        __syncthreads();
        const int ne = (int)(n_old - c0 < 256 ? n_old - c0 : 256);
        const uint2 *src = reinterpret_cast<const uint2 *>(J.obox) + c0 * D;  // a box = D words of 8 bytes
        uint2 *dst = reinterpret_cast<uint2 *>(J.nbox);
        for (int w = threadIdx.x; w < ne * D; w += 256) {
            const int e = w / D;
            dst[(c0 + e + s_shift[e]) * D + (w - e * D)] = src[w];
        }
        __syncthreads();  // s_lo / s_pos / s_shift reused by the next chunk
    }
    for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < n_new; r += (int64_t)gridDim.x * 256) {
        const int64_t out = J.edir_pos[r] + 1 + r;
        const int32_t b = J.edir_bk[r];
        J.ndir_code[2 * out] = J.edir_code[2 * r];
        J.ndir_code[2 * out + 1] = J.edir_code[2 * r + 1];
        J.nmeta[out] = leaf_code(b, J.bcnt[b]);
#pragma unroll
        for (int q = 0; q < 2 * D; ++q) J.nbox[out * 2 * D + q] = J.bbox[(int64_t)b * 2 * D + q];
    }
}

// The hierarchy above the directory.  Levels 1 and 2 (the directory, the big one, and the one
// above it) are grouped over many workgroups (k_ct_lflags, k_ct_lgroup): consecutive nodes into
// maximal aligned code cells of at most 8 (ct_same over the nodes' codes: a node's code is its
// first directory entry's start), or, when that would leave more than half as many groups as
// nodes or more levels than the walk's stack allows, runs of 8.  Above level 3 one workgroup a
// tree (k_ct_levels) groups runs of 8, then copies the seeds and closes the round's counts.
constexpr int kCtMaxLevels = 10;  // the walk's stack bound (ct_walk kStack); runs of 8 reach it below 8^9 entries
constexpr int kCtL1Per = kCtL1Tile / 256;  // level-1 entries a thread of k_ct_lflags / k_ct_lgroup

// the levels a tree needs when level `lev` has G groups and runs of 8 follow
__device__ __forceinline__ bool ct_fixed(int64_t n, int64_t G, int lev) {
    int need = lev + 1;
    for (int64_t m = G; m > 1; m = (m + 7) / 8) ++need;
    return G > n / 2 || need > kCtMaxLevels;
}

__device__ __forceinline__ int ct_block_scan(int v, int32_t *s_w, int nthreads, int &total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int incl = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int o = __shfl_up(incl, off);
        if (lane >= off) incl += o;
    }
    __syncthreads();
    if (lane == 63) s_w[wave] = incl;
    __syncthreads();
    int before = 0, tot = 0;
    for (int w = 0; w < nthreads / 64; ++w) {
        before += w < wave ? s_w[w] : 0;
        tot += s_w[w];
    }
    total = tot;
    return before + incl - v;  // exclusive
}

// Level LEV (1: the directory, 2: the level above it) as the multi-workgroup kernels see it:
// its nodes [base, base + n), their codes, where its tiles' counts go.
template <int LEV>
struct CtLevel {
    int64_t base, n;
    const uint64_t *code;
    int32_t *lcount;
};
template <int LEV>
__device__ __forceinline__ CtLevel<LEV> ct_level(const CtJob &J) {
    const int64_t n1 = (int64_t)J.cnt->n_dir + J.cnt->n_new_dir;
    if constexpr (LEV == 1) return {0, n1, J.ndir_code, J.lcount};
    else return {n1, n1 > 1 ? (int64_t)J.cnt->n_l2 : 0, J.ucode + 2 * n1, J.lcount + J.bcap / kCtL1Tile + 1};
}

// a level's group starts, kCtL1Per consecutive nodes a thread; the tile's count.  The
// adjacent prefix lengths of the tile and 8 entries either side go to LDS first (one coalesced
// pass over the codes).
constexpr int kCtHalo = kCtCap;
template <int LEV>
__global__ __launch_bounds__(256) void k_ct_lflags(CtJobs js) {
    const CtJob J = CT_JOB(js);  // by value: the fields stay in registers across the stores
    __shared__ int32_t s_w[4];
    __shared__ uint8_t s_a[kCtL1Tile + 2 * kCtHalo];
    const CtLevel<LEV> V = ct_level<LEV>(J);
    const int64_t n = V.n;
    const uint64_t *__restrict__ code = V.code;
    if (n <= 1) return;  // block-uniform
    // tiles over a grid sized by the level's typical size (a grid for the host's bound of it
    // dispatched mostly empty workgroups)
    for (int64_t tile = blockIdx.x; tile * kCtL1Tile < n; tile += gridDim.x) {
    const int64_t t0 = tile * kCtL1Tile;
    const int64_t a0 = t0 - kCtHalo;  // s_a[v] = a[a0 + v]
    for (int v = threadIdx.x; v < kCtL1Tile + 2 * kCtHalo; v += 256) {
        const int64_t u = a0 + v;
        int cp = 0;
        if (u >= 1 && u < n)
            cp = c_cpl(code[2 * (u - 1)], code[2 * (u - 1) + 1], code[2 * u], code[2 * u + 1]);
        s_a[v] = (uint8_t)cp;
    }
    __syncthreads();
    // ct_same_a's window in tile coordinates: [max(0, a0), n) shifted by a0
    const int64_t wlo = (a0 < 0 ? 0 : a0) - a0, whi = (n < a0 + kCtL1Tile + 2 * kCtHalo ? n : a0 + kCtL1Tile + 2 * kCtHalo) - a0;
    int c = 0;
#pragma unroll
    for (int q = 0; q < kCtL1Per; ++q) {
        const int64_t i = t0 + threadIdx.x * kCtL1Per + q;
        if (i < n) {
            // the index / 8 rule counts from the run start 0: shift lo so (i - lo) keeps i's phase
            const int f = i == 0 || !ct_same_a(s_a, wlo, whi, i - a0);
            J.lflag[V.base + i] = f;
            c += f;
        }
    }
    int tot;
    (void)ct_block_scan(c, s_w, 256, tot);
    if (threadIdx.x == 0) V.lcount[tile] = tot;
    __syncthreads();  // s_a, s_w reused by the next tile
    }
}

// level 2: each tile's groups, numbered after the tiles before it.  The tile's boxes and flags
// (and the 7 entries after it, where its last groups end) are staged in LDS with coalesced loads.
template <int D, int LEV>
__global__ __launch_bounds__(256) void k_ct_lgroup(CtJobs js) {
    const CtJob J = CT_JOB(js);  // by value: the fields stay in registers across the stores
    constexpr int kSpan = kCtL1Tile + kCtCap - 1;
    __shared__ int32_t s_w[4];
    __shared__ int64_t s_sum[2];
    __shared__ uint2 s_box[kSpan * D];  // box e of the span: words [e * D, e * D + D)
    __shared__ uint8_t s_f[kSpan];
    const CtLevel<LEV> V = ct_level<LEV>(J);
    const int64_t n = V.n, base = V.base;
    if (n <= 1) return;  // block-uniform
    const int64_t tiles = (n + kCtL1Tile - 1) / kCtL1Tile;
    for (int64_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) {  // (k_ct_lflags' grid)
    const int64_t t0 = tile * kCtL1Tile;
    if (threadIdx.x < 64) {  // the groups of all tiles and of the tiles before this one
        int64_t all = 0, before = 0;
        for (int64_t b = threadIdx.x; b < tiles; b += 64) {
            const int32_t v = V.lcount[b];
            all += v;
            before += b < tile ? v : 0;
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            all += __shfl_xor(all, off);
            before += __shfl_xor(before, off);
        }
        if (threadIdx.x == 0) {
            s_sum[0] = all;
            s_sum[1] = before;
        }
    }
    const int span = (int)(n - t0 < kSpan ? n - t0 : kSpan);
    const uint2 *src = reinterpret_cast<const uint2 *>(J.nbox) + (base + t0) * D;
    for (int w = threadIdx.x; w < span * D; w += 256) s_box[w] = src[w];
    for (int e = threadIdx.x; e < span; e += 256) s_f[e] = (uint8_t)J.lflag[base + t0 + e];
    __syncthreads();
    const int64_t G = s_sum[0];
    const bool fixed = ct_fixed(n, G, LEV);
    if (tile == 0 && threadIdx.x == 0) (LEV == 1 ? J.cnt->n_l2 : J.cnt->n_l3) = (int32_t)(fixed ? (n + 7) / 8 : G);
    const int e0 = threadIdx.x * kCtL1Per;  // this thread's entries [e0, e0 + kCtL1Per) of the tile
    int f[kCtL1Per], c = 0;
#pragma unroll
    for (int a = 0; a < kCtL1Per; ++a) {
        const int e = e0 + a;
        f[a] = t0 + e < n && (fixed ? ((t0 + e) & 7) == 0 : s_f[e] != 0);
        c += f[a];
    }
    int tot;
    const int64_t ex = ct_block_scan(c, s_w, 256, tot);
    int64_t g = fixed ? 0 : s_sum[1] + ex;
#pragma unroll
    for (int a = 0; a < kCtL1Per; ++a) {
        if (!f[a]) continue;
        const int e = e0 + a;
        const int64_t i = t0 + e;
        int len = 1;
        if (fixed) {
            len = n - i < 8 ? (int)(n - i) : 8;
            g = i / 8;
        } else {
            while (i + len < n && len < kCtCap && !s_f[e + len]) ++len;
        }
        float lo[D], nhi[D];  // the union: (lo, -hi) pairs, a minimum of both
        const float *b0 = reinterpret_cast<const float *>(s_box + e * D);
#pragma unroll
        for (int q = 0; q < D; ++q) {
            lo[q] = b0[2 * q];
            nhi[q] = b0[2 * q + 1];
        }
        for (int u = 1; u < len; ++u) {
            const float *bu = reinterpret_cast<const float *>(s_box + (e + u) * D);
#pragma unroll
            for (int q = 0; q < D; ++q) {
                lo[q] = fminf(lo[q], bu[2 * q]);
                nhi[q] = fminf(nhi[q], bu[2 * q + 1]);
            }
        }
        const int64_t P = base + n + g;
#pragma unroll
        for (int q = 0; q < D; ++q) {
            J.nbox[P * 2 * D + 2 * q] = lo[q];
            J.nbox[P * 2 * D + 2 * q + 1] = nhi[q];
        }
        J.nmeta[P] = inner_code(base + i, len);
        J.ucode[2 * P] = V.code[2 * i];
        J.ucode[2 * P + 1] = V.code[2 * i + 1];
        ++g;
    }
    __syncthreads();  // s_sum, s_box, s_f reused by the next tile
    }
}

// one workgroup a tree: the levels above level 3, then the counts, the seed rows, the indexed
// count and the spread.  Round 5, measured and not kept: the upper levels' boxes in LDS (14.4
// us a round at 32 seeds either way); this work run by the last of k_ct_lgroup<2>'s workgroups
// to finish a tree (a ticket: one launch less), which made k_ct_lgroup<2> 12.7 -> 58 us at 32
// seeds and 39 -> 449 us at 256 (every workgroup then fences at device scope before its
// ticket: with one L2 an XCD, the likely cost).
constexpr int kCtLevelThreads = 1024;
template <int D>
__global__ __launch_bounds__(kCtLevelThreads) void k_ct_levels(CtJobs js) {
    constexpr int NT = kCtLevelThreads;
    const CtJob J = CT_JOB(js);  // by value: the fields stay in registers across the stores
    const int t = threadIdx.x;
    // the seed rows first: independent of the levels, so their loads overlap the levels' work
    for (int it = t; it < kCtHull * D; it += NT) {
        const int h = it / D, k = it - h * D;
        const unsigned long long key = J.hull_keys[h];
        const int64_t row = (int64_t)(uint32_t)key;
        J.hull_pts[it] = key ? J.pts[row * D + k] : 0.0;
        if (k == 0) J.hull_ids[h] = key ? (int32_t)row + 1 : 0;
    }
    const int64_t n1 = (int64_t)J.cnt->n_dir + J.cnt->n_new_dir;
    // levels 1 and 2 were grouped by k_ct_lflags / k_ct_lgroup into levels 2 and 3
    int64_t ls = 0, n = n1;
    for (int k = 0; k < 2 && n > 1; ++k) {
        ls += n;
        n = k == 0 ? J.cnt->n_l2 : J.cnt->n_l3;
    }
    // above level 3: runs of 8 (boxes high in the tree prune little; what counts is how few
    // levels a walk descends)
    while (n > 1) {
        const int64_t nG = (n + 7) / 8;
        for (int64_t g = t; g < nG; g += NT) {
            const int64_t first = ls + 8 * g;
            const int len = n - 8 * g < 8 ? (int)(n - 8 * g) : 8;
            float lo[D], nhi[D];  // (lo, -hi) pairs: the union is a minimum of both
#pragma unroll
            for (int q = 0; q < D; ++q) {
                lo[q] = J.nbox[first * 2 * D + 2 * q];
                nhi[q] = J.nbox[first * 2 * D + 2 * q + 1];
            }
            for (int u = 1; u < len; ++u)
#pragma unroll
                for (int q = 0; q < D; ++q) {
                    lo[q] = fminf(lo[q], J.nbox[(first + u) * 2 * D + 2 * q]);
                    nhi[q] = fminf(nhi[q], J.nbox[(first + u) * 2 * D + 2 * q + 1]);
                }
            const int64_t P = ls + n + g;
#pragma unroll
            for (int q = 0; q < D; ++q) {
                J.nbox[P * 2 * D + 2 * q] = lo[q];
                J.nbox[P * 2 * D + 2 * q + 1] = nhi[q];
            }
            J.nmeta[P] = inner_code(first, len);
        }
        __threadfence_block();
        __syncthreads();
        ls += n;
        n = nG;
    }
    __syncthreads();
    if (t < 8) {  // the walk's first entries: the root's children, or the root when it is a leaf
        const uint32_t rm = J.nmeta[ls];
        const int nc = (rm & kCtLeafBit) ? 1 : (int)((rm >> 28) & 7u) + 1;
        if (t < nc) J.cnt->top[t] = (rm & kCtLeafBit) ? rm : J.nmeta[(int64_t)(rm & 0x0fffffffu) + t];
        if (t == 0) J.cnt->n_top = nc;
    }
    if (t != 0) return;
    CtCounts *c = J.cnt;
    {
        // the lowest level of at most 64 nodes (levels are contiguous: 1 = the directory, then
        // levels 2 and 3 as k_ct_lgroup counted them, then runs of 8)
        int64_t s = 0, m = n1;
        for (int k = 0; m > 64; ++k) {
            const int64_t next = k == 0 ? c->n_l2 : (k == 1 ? c->n_l3 : (m + 7) / 8);
            s += m;
            m = next;
        }
        c->lv_first = (int32_t)s;
        c->lv_n = (int32_t)m;
    }
    const int32_t nn = c->n_new_dir;
    c->root = (int32_t)ls;
    c->n_dir += nn;
    c->n_buckets += nn;
    c->n_new_dir = 0;
    c->n_seg = 0;
    c->n_scratch = 0;
    c->nidx = c->nidx + ct_new_count(J);
    const SpreadOut &sp = J.sp;
    if (sp.host_out) {
        for (int j = 0; j < 3; ++j) {
            sp.host_out[j] = j < sp.gd ? J.ibox[sp.dims[j]] : ~0ull;
            sp.host_out[3 + j] = j < sp.gd ? J.ibox[kCtMaxDim + sp.dims[j]] : 0ull;
        }
        __threadfence_system();
    }
}

// An empty index (one empty bucket at code 0, as k_ct_bulk_fill makes for an empty tree), the
// seeds and the persistent box cleared: the round then inserts rows [0, n) as new points.
// One workgroup a job; jobs without the reset flag return.
__global__ __launch_bounds__(64) void k_ct_reset(CtJobs js) {
    const CtJob J = CT_JOB(js);
    if (!J.reset) return;
    const int t = threadIdx.x;
    const int d = J.T.d;
    J.hull_keys[t] = 0ull;  // kCtHull = 64 slots
    if (t < 2 * kCtMaxDim) J.ibox[t] = t < kCtMaxDim ? ~0ull : 0ull;
    if (t < 2 * d) {
        const float v = __builtin_huge_valf();  // the empty box: (lo, -hi) = (+inf, +inf)
        J.bbox[t] = v;
        J.obox[t] = v;
    }
    if (t == 0) {
        J.bcnt[0] = 0;
        uint64_t *dc = const_cast<uint64_t *>(J.odir_code);
        dc[0] = 0;
        dc[1] = 0;
        J.ometa[0] = leaf_code(0, 1);  // the bucket's count is 0: the first round appends or splits it
        CtCounts *c = J.cnt;
        c->n_dir = c->n_buckets = 1;
        c->n_seg = c->n_new_dir = c->n_scratch = 0;
        c->root = 0;
        c->nidx = 0;
    }
}

// ---- full rebuild (prepare, full): every point sorted by (code, row), then cut into buckets ----

template <int D>
__global__ __launch_bounds__(64 * kCtWaves) void k_ct_codes_all(const double *__restrict__ pts, int64_t n_upper,
                                                                const int64_t *__restrict__ n_dev,
                                                                const CtPlan *__restrict__ plan,
                                                                uint64_t *__restrict__ hi_out, uint64_t *__restrict__ lo_out,
                                                                int32_t *__restrict__ rows,
                                                                unsigned long long *__restrict__ hull_keys,
                                                                unsigned long long *__restrict__ ibox) {
    __shared__ CtPlan s_plan;
    __shared__ double s_rows[kCtWaves][64][D];
    for (int w = threadIdx.x; w < (int)(sizeof(CtPlan) / 4); w += blockDim.x)
        reinterpret_cast<uint32_t *>(&s_plan)[w] = reinterpret_cast<const uint32_t *>(plan)[w];
    __syncthreads();
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if ((int64_t)blockIdx.x * blockDim.x >= n_upper) return;  // block-uniform
    const int64_t n = *n_dev < n_upper ? *n_dev : n_upper;
    const bool live = i < n;
    double x[D];
#pragma unroll
    for (int j = 0; j < D; ++j) x[j] = live ? pts[i * D + j] : 0.0;
    if (i < n_upper) {
        uint64_t h = ~0ull, l = ~0ull;  // rows past the live count sort last
        if (live) ct_code<D>(s_plan, x, h, l);
        hi_out[i] = h;
        lo_out[i] = l;
        rows[i] = (int32_t)i;
    }
    unsigned long long mn[D], mx[D];
#pragma unroll
    for (int j = 0; j < D; ++j) {
        mn[j] = live ? okey(x[j]) : ~0ull;
        mx[j] = live ? okey(x[j]) : 0ull;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const unsigned long long omn = __shfl_xor(mn[j], off), omx = __shfl_xor(mx[j], off);
            mn[j] = omn < mn[j] ? omn : mn[j];
            mx[j] = omx > mx[j] ? omx : mx[j];
        }
    }
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
        for (int j = 0; j < D; ++j) {
            atomicMin(ibox + j, mn[j]);
            atomicMax(ibox + kCtMaxDim + j, mx[j]);
        }
    }
    hull_offer<D>(s_plan, x, live, i & ~(int64_t)63, s_rows[threadIdx.x >> 6], hull_keys);
}

// after the first (low-word) pass: the high words in that order, for the second pass
__global__ void k_ct_gather_hi(const uint64_t *__restrict__ hi, const int32_t *__restrict__ order, int64_t n,
                               uint64_t *__restrict__ out) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < n) out[j] = hi[order[j]];
}

// the sorted codes as (hi, lo) pairs (lo gathered by row) for the leaf rule
__global__ void k_ct_pack(const uint64_t *__restrict__ hi_sorted, const uint64_t *__restrict__ lo_by_row,
                          const int32_t *__restrict__ rows, int64_t n_upper, const int64_t *__restrict__ n_dev,
                          uint64_t *__restrict__ code) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t n = *n_dev < n_upper ? *n_dev : n_upper;
    if (j >= n) return;
    code[2 * j] = hi_sorted[j];
    code[2 * j + 1] = lo_by_row[rows[j]];
}

__global__ void k_ct_bulk_flags(const uint64_t *__restrict__ code, const int32_t *__restrict__ rows, int64_t n_upper,
                                const int64_t *__restrict__ n_dev, int32_t *__restrict__ flag) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n_upper) return;
    const int64_t n = *n_dev < n_upper ? *n_dev : n_upper;
    flag[j] = j < n && (j == 0 || !ct_same(code, rows, 0, n, j)) ? 1 : 0;
}

// leaf starts fill bucket r = their rank and directory entry r; an empty tree gets one empty
// bucket (its box empty) starting at code 0
template <int D>
__global__ void k_ct_bulk_fill(const double *__restrict__ pts, const uint64_t *__restrict__ code,
                               const int32_t *__restrict__ rows, const int32_t *__restrict__ flag,
                               const int32_t *__restrict__ leaf, int64_t n_upper, const int64_t *__restrict__ n_dev,
                               double *__restrict__ bpts, int32_t *__restrict__ bids, uint64_t *__restrict__ bcode,
                               int32_t *__restrict__ bcnt, float *__restrict__ bbox, uint64_t *__restrict__ dir_code,
                               uint32_t *__restrict__ dir_meta, float *__restrict__ dir_box, CtCounts *__restrict__ cnt) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t n = *n_dev < n_upper ? *n_dev : n_upper;
    if (n == 0) {
        if (j == 0) {
            bcnt[0] = 0;
            for (int q = 0; q < 2 * D; ++q) bbox[q] = __builtin_huge_valf();  // empty: (+inf, +inf) pairs
            dir_code[0] = 0;
            dir_code[1] = 0;
            dir_meta[0] = leaf_code(0, 1);  // never walked: the walk skips an empty tree
            for (int q = 0; q < 2 * D; ++q) dir_box[q] = __builtin_huge_valf();
            cnt->n_dir = cnt->n_buckets = 1;
            cnt->n_seg = cnt->n_new_dir = cnt->n_scratch = 0;
            cnt->nidx = 0;
        }
        return;
    }
    if (j >= n) return;
    if (j == n - 1) {
        const int32_t nb = leaf[j] + flag[j];
        cnt->n_dir = cnt->n_buckets = nb;
        cnt->n_seg = cnt->n_new_dir = cnt->n_scratch = 0;
        cnt->nidx = n;
    }
    if (!flag[j]) return;
    const int32_t r = leaf[j];
    int len = 1;
    while (j + len < n && !flag[j + len]) ++len;
    uint64_t sh = 0, sl = 0;
    if (j > 0) {
        sh = code[2 * j];
        sl = code[2 * j + 1];
        c_boundary(code[2 * (j - 1)], code[2 * (j - 1) + 1], sh, sl);
    }
    dir_code[2 * r] = sh;
    dir_code[2 * r + 1] = sl;
    double lo[D], hi[D];
#pragma unroll
    for (int q = 0; q < D; ++q) {
        lo[q] = __builtin_huge_val();
        hi[q] = -__builtin_huge_val();
    }
    for (int u = 0; u < len && u < kCtCap; ++u) {
        const int32_t row = rows[j + u];
        const int64_t slot = (int64_t)r * kCtCap + u;
#pragma unroll
        for (int q = 0; q < D; ++q) {
            const double x = pts[(int64_t)row * D + q];
            bpts[slot * D + q] = x;
            lo[q] = x < lo[q] ? x : lo[q];
            hi[q] = x > hi[q] ? x : hi[q];
        }
        bids[slot] = row + 1;
        bcode[2 * slot] = code[2 * (j + u)];
        bcode[2 * slot + 1] = code[2 * (j + u) + 1];
    }
    write_box<D>(bbox + (int64_t)r * 2 * D, lo, hi);
    write_box<D>(dir_box + (int64_t)r * 2 * D, lo, hi);
    bcnt[r] = len < kCtCap ? len : kCtCap;
    dir_meta[r] = leaf_code(r, len < kCtCap ? len : kCtCap);
}

__global__ __launch_bounds__(64) void k_ct_box_reset(unsigned long long *__restrict__ box) {
    if (threadIdx.x < 2 * kCtMaxDim) box[threadIdx.x] = threadIdx.x < kCtMaxDim ? ~0ull : 0ull;
}

// ---- the walk (point_tree.hip tree_nn1_blockn over the bucket hierarchy) ----

using gdbl = const __attribute__((address_space(1))) double *;
using gflt = const __attribute__((address_space(1))) float *;
using gi32 = const __attribute__((address_space(1))) int32_t *;
using gu32 = const __attribute__((address_space(1))) uint32_t *;

// A box's lower bound on FLANN's squared L2 from the query, as a float rounded down (see
// point_tree.hip box_lb: d <= 7 in float from the query rounded outward and scaled below the
// exact bound, d = 15 in double rounded down).  Pruning on it keeps every box the exact bound
// keeps.
constexpr float kCtLbShrink = 1.0f - 0x1p-19f;
template <int D>
__device__ __forceinline__ float ct_box_lb(const float *__restrict__ b, const double (&qq)[D], const float (&qlo)[D],
                                           const float (&qhi)[D]) {
    if constexpr (D <= 7) {
        // dim k's two gaps (lo - qhi, qlo - hi) as one packed addition of the box's (lo, -hi)
        // word and the query's (-qhi, qlo); then one max3 and one fused multiply-add: 3
        // instructions a dim (4 unpacked).  One rounding a term, still far inside the shrink
        // (each gap and each step at most (1 + 2^-24) above the exact value: (1 + 2^-24)^9)
        typedef float f2 __attribute__((ext_vector_type(2)));
        float s = 0.0f;
#pragma unroll
        for (int k = 0; k < D; ++k) {
            const f2 box = {b[2 * k], b[2 * k + 1]};
            const f2 qry = {-qhi[k], qlo[k]};
            const f2 gap = box + qry;
            const float g = fmaxf(fmaxf(gap.x, gap.y), 0.0f);
            s = __builtin_fmaf(g, g, s);
        }
        return s * kCtLbShrink;
    } else {
        double lb2 = 0.0;
#pragma unroll
        for (int k = 0; k < D; ++k) {
            const double g = fmax(fmax((double)b[2 * k] - qq[k], qq[k] + (double)b[2 * k + 1]), 0.0);
            lb2 += g * g;
        }
        return __double2float_rd(lb2);
    }
}

// ---- lane exchanges of the walk (DPP lane permutations and the gfx950 row / half swaps: no
// LDS traffic, unlike ds_bpermute) ----
constexpr int kDppXor1 = 0xB1;   // quad_perm [1,0,3,2]: lane i ^ 1
constexpr int kDppXor2 = 0x4E;   // quad_perm [2,3,0,1]: lane i ^ 2
constexpr int kDppRev8 = 0x141;  // row_half_mirror: lane i ^ 7 within 8
constexpr int kDppRev16 = 0x140; // row_mirror: lane i ^ 15 within 16
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xf, 0xf, true);  // every source lane is in range
}
// level L of a group reduction: each lane gets a lane of the other half of its 2L-lane block
// (after the levels below L that half's lanes hold one value)
template <int L>
__device__ __forceinline__ uint32_t xchg(uint32_t v) {
    if constexpr (L == 1) return dpp_u<kDppXor1>(v);
    else if constexpr (L == 2) return dpp_u<kDppXor2>(v);
    else if constexpr (L == 4) return dpp_u<kDppRev8>(v);
    else if constexpr (L == 8) return dpp_u<kDppRev16>(v);
    else if constexpr (L == 16) {  // rows 0 <-> 1, 2 <-> 3
        const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        return (threadIdx.x & 16) ? r[0] : r[1];
    } else {  // lanes 0..31 <-> 32..63
        static_assert(L == 32, "xchg level");
        const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        return (threadIdx.x & 32) ? r[0] : r[1];
    }
}
template <int L>
__device__ __forceinline__ double xchg_d(double x) {
    const uint32_t lo = (uint32_t)__double2loint(x), hi = (uint32_t)__double2hiint(x);
    return __hiloint2double((int)xchg<L>(hi), (int)xchg<L>(lo));
}
template <int L, class F>
__device__ __forceinline__ void each_level(F &&f) {
    if constexpr (L >= 1) f(std::integral_constant<int, 1>{});
    if constexpr (L >= 2) f(std::integral_constant<int, 2>{});
    if constexpr (L >= 4) f(std::integral_constant<int, 4>{});
    if constexpr (L >= 8) f(std::integral_constant<int, 8>{});
    if constexpr (L >= 16) f(std::integral_constant<int, 16>{});
    if constexpr (L >= 32) f(std::integral_constant<int, 32>{});
}
// (d2, id) take-better without branches (nn_better)
__device__ __forceinline__ void nn_take(double &bd, int32_t &bi, double od, int32_t oi) {
    const bool t = (od < bd) | ((od == bd) & (oi < bi));
    bd = t ? od : bd;
    bi = t ? oi : bi;
}
// The least u32 of the wave, uniform: the row butterflies (DPP), then rows 0 -> 1 and 2 -> 3
// (row_bcast:15) and rows 0..1 -> 2..3 (row_bcast:31), so lane 63 holds it (7 instructions, no
// LDS)
constexpr int kDppBcast15 = 0x142;
constexpr int kDppBcast31 = 0x143;
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
    v = min(v, dpp_u<kDppXor1>(v));
    v = min(v, dpp_u<kDppXor2>(v));
    v = min(v, dpp_u<kDppRev8>(v));
    v = min(v, dpp_u<kDppRev16>(v));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, kDppBcast15, 0xa, 0xf, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, kDppBcast31, 0xc, 0xf, false));
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// The best (d2, id) of each G-lane group, in every lane of it (nn_better's order): the least
// d2 first, then the least id among the lanes holding it -- read from the one such lane of a
// 64-lane group when it is alone (the common case), else reduced.  A 64-lane group compares
// the d2 bit patterns (non-negative doubles order as their bits): the least high word, then
// the least low word among the lanes holding it, as two wave minimums of u32.
template <int G>
__device__ __forceinline__ void best_group(double &bd, int32_t &bi) {
    if constexpr (G == 64) {
        const uint32_t hi = (uint32_t)__double2hiint(bd), lo = (uint32_t)__double2loint(bd);
        const uint32_t mh = wave_min_u32(hi);
        const uint32_t ml = wave_min_u32(hi == mh ? lo : 0xffffffffu);
        const bool win = (hi == mh) & (lo == ml);
        bd = __hiloint2double((int)mh, (int)ml);
        const uint64_t wm = __ballot(win);
        if (__popcll(wm) == 1) {
            bi = __builtin_amdgcn_readlane(bi, __ffsll((long long)wm) - 1);
        } else {
            const uint32_t c = win ? (uint32_t)bi ^ 0x80000000u : 0xffffffffu;  // signed order as u32
            bi = (int32_t)(wave_min_u32(c) ^ 0x80000000u);
        }
        return;
    }
    double m = bd;
    each_level<G / 2>([&](auto L) {
        const double o = xchg_d<decltype(L)::value>(m);
        m = o < m ? o : m;
    });
    const bool win = bd == m;
    bd = m;
    int32_t c = win ? bi : 0x7fffffff;
    each_level<G / 2>([&](auto L) {
        const int32_t o = (int32_t)xchg<decltype(L)::value>((uint32_t)c);
        c = o < c ? o : c;
    });
    bi = c;
}
// x rounded down / up to float (the largest float <= x, the smallest >= x) for finite x: the
// nearest float, stepped one ulp when it lies on the wrong side -- 7 instructions where the
// __double2float_rd / _ru library forms took ~14 each (14 conversions a query)
__device__ __forceinline__ float f32_dn(double x) {
    const float f = (float)x;
    const uint32_t b = __float_as_uint(f);
    const uint32_t nb = f > 0.0f ? b - 1u : (f < 0.0f ? b + 1u : 0x80000001u);
    return (double)f > x ? __uint_as_float(nb) : f;
}
__device__ __forceinline__ float f32_up_any(double x) {
    const float f = (float)x;
    const uint32_t b = __float_as_uint(f);
    const uint32_t nb = f > 0.0f ? b + 1u : (f < 0.0f ? b - 1u : 0x00000001u);
    return (double)f < x ? __uint_as_float(nb) : f;
}

// the smallest float >= x (x >= 0): the walk's pruning threshold in float (any box whose
// lower bound is <= the best squared distance is <= it too)
__device__ __forceinline__ float f32_up(double x) {
    const float f = (float)x;
    return (double)f < x ? __uint_as_float(__float_as_uint(f) + 1u) : f;
}

// the seeds' best (d2, id) over a group of G lanes: lane `sub` takes seeds sub, sub + G, ...
template <int D, int G>
__device__ __forceinline__ void ct_seed(const CellTreeDev &T, const double (&qq)[D], int sub, double &bd, int32_t &bi,
                                        uint32_t &n_pts) {
    for (int h = sub; h < kCtHull; h += G) {
        const int32_t id = ((gi32)T.hull_ids)[h];
        if (id <= 0) continue;
        double row[D];
#pragma unroll
        for (int k = 0; k < D; ++k) row[k] = ((gdbl)T.hull_pts)[h * D + k];
        const double dd = flann_l2<D>(qq, row);
        ++n_pts;
        nn_take(bd, bi, dd, id);
    }
    best_group<G>(bd, bi);
}

// One query a wave (8 entries a step, 8 lanes an entry) over two stacks in the one LDS array:
// inner entries growing up from slot 0, buckets growing down from the last slot.  A step pops
// from one stack only -- buckets when 8 wait or no inner entry is left, else inner entries --
// so every step runs one kind's code: a bucket step the points' exact distances (no push), an
// inner step the children's float lower bounds and their pushes (no merge).  The one-stack walk
// popped the top 8 entries whatever their kinds and ran both paths in most steps (SQ counters
// at the config-5 shape: the walk issue-bound, ACTIVE_INST_VALU x 8 waves ~1.06 of a SIMD).
// Bounds: an inner step pops <= 8 and pushes <= 64 inner children, so the inner stack holds
// <= 8 + 56 a level over <= 9 inner levels (512); buckets are popped whenever 8 wait, so the
// bucket stack holds < 8 + 64: together <= 584 of the 640 slots.  Which entries a step takes
// changes the order of the walk only: every box whose float lower bound exceeds the shared bound
// (f32_up of the best so far, an upper bound of the final best) is skipped, every other bucket's
// points are examined, and the exact (d2, id) merge of the lanes' bests runs once at the end.
constexpr int kCtSplitStack = 8 * 8 * kCtMaxLevels;
constexpr bool kCtSplitWalk = true;  // ct_walk's 8-entry form (the one-stack walk otherwise)
template <int D, int BS>
__device__ __forceinline__ void ct_walk_split(const CellTreeDev &T, const double *__restrict__ q, int64_t nq,
                                              int32_t *__restrict__ out_ids, double *__restrict__ out_d2,
                                              int64_t blk) {
    constexpr int G = 64;
    constexpr int kStack = kCtSplitStack;
    __shared__ uint2 s_stk[BS / G][kStack];  // (code, lower bound's bits)
    const int64_t t = blk * BS + threadIdx.x;
    const int64_t qi = t / G;
    const int sub = (int)(t % G);
    const int part = sub / 8;
    const int ls = sub % 8;
    const int grp = threadIdx.x / G;
    if (qi >= nq) return;  // whole waves leave together
    double qq[D];
#pragma unroll
    for (int i = 0; i < D; ++i) qq[i] = q[qi * D + i];
    float qlo[D], qhi[D];
#pragma unroll
    for (int i = 0; i < D; ++i) {
        qlo[i] = f32_dn(qq[i]);
        qhi[i] = f32_up_any(qq[i]);
    }
    double bd = __builtin_huge_val();
    int32_t bi = -1;
    uint32_t n_pts = 0, n_box = 0, n_steps = 1;  // the seeds' step
    uint2 *stk = s_stk[grp];
    const uint64_t below_me = (1ull << sub) - 1ull;
    if (*T.n_dev > 0) {
        // the first entries: the nodes of the lowest level of at most 64 (lane sub: node
        // lv_first + sub), their boxes loaded with the seeds and tested against the seeds' best
        // -- no walk step for the narrow levels above it
        const int lv_first = ((gi32)T.lv)[0], lv_n = ((gi32)T.lv)[1];
        const bool in = sub < lv_n;
        uint32_t code0 = 0;
        float lb0 = 0.0f;
        if (in) {
            const int64_t e = (int64_t)lv_first + sub;
            double row[D];
#pragma unroll
            for (int k = 0; k < D; ++k) row[k] = ((gdbl)(const void *)T.nbox)[e * D + k];
            code0 = ((gu32)T.nmeta)[e];
            float bx[2 * D];
#pragma unroll
            for (int k = 0; k < D; ++k) {
                bx[2 * k] = __int_as_float(__double2loint(row[k]));
                bx[2 * k + 1] = __int_as_float(__double2hiint(row[k]));
            }
            lb0 = ct_box_lb<D>(bx, qq, qlo, qhi);
            ++n_box;
        }
        ct_seed<D, G>(T, qq, sub, bd, bi, n_pts);
        float bdf = f32_up(bd);
        int isp = 0, lsp = 0;  // inner entries [0, isp), buckets [kStack - lsp, kStack)
        {
            const bool keep = in && lb0 <= bdf;
            const bool lf = keep && (code0 & kCtLeafBit);
            const uint64_t ml = __ballot(lf), mi = __ballot(keep && !lf);
            if (lf) stk[kStack - 1 - __popcll(ml & below_me)] = make_uint2(code0, __float_as_uint(lb0));
            if (keep && !lf) stk[__popcll(mi & below_me)] = make_uint2(code0, __float_as_uint(lb0));
            lsp = __popcll(ml);
            isp = __popcll(mi);
        }
        __builtin_amdgcn_wave_barrier();
        while (isp + lsp > 0) {
            const bool leaves = lsp >= 8 || isp == 0;  // wave-uniform
            const int avail = leaves ? lsp : isp;
            const int np = avail >= 8 ? 8 : avail;
            const bool have = part < np;
            uint32_t code = 0;
            float lbs = 0.0f;
            if (have) {
                const uint2 en = leaves ? stk[kStack - lsp + part] : stk[isp - 1 - part];
                code = en.x;
                lbs = __uint_as_float(en.y);
            }
            if (leaves) lsp -= np;
            else isp -= np;
            ++n_steps;
            __builtin_amdgcn_wave_barrier();
            const bool act = have && !(lbs > bdf) && ls < (int)((code >> 28) & 7u) + 1;
            if (leaves) {
                bool better = false;
                if (act) {
                    const int64_t e = (int64_t)(code & 0x0fffffffu) * kCtCap + ls;
                    double row[D];
#pragma unroll
                    for (int k = 0; k < D; ++k) row[k] = ((gdbl)T.bpts)[e * D + k];
                    const int32_t id = (int32_t)((gu32)(const void *)T.bids)[e];
                    const double dd = flann_l2<D>(qq, row);
                    ++n_pts;
                    better = ((dd < bd) | ((dd == bd) & (id < bi))) && dd <= (double)bdf;
                    nn_take(bd, bi, dd, id);
                }
                if (__ballot(better)) bdf = __uint_as_float(wave_min_u32(__float_as_uint(f32_up(bd))));
            } else {
                bool keep = false;
                uint32_t child = 0;
                float lbf = 0.0f;
                if (act) {
                    const int64_t e = (int64_t)(code & 0x0fffffffu) + ls;
                    double row[D];
#pragma unroll
                    for (int k = 0; k < D; ++k) row[k] = ((gdbl)(const void *)T.nbox)[e * D + k];
                    child = ((gu32)T.nmeta)[e];
                    float bx[2 * D];
#pragma unroll
                    for (int k = 0; k < D; ++k) {
                        bx[2 * k] = __int_as_float(__double2loint(row[k]));
                        bx[2 * k + 1] = __int_as_float(__double2hiint(row[k]));
                    }
                    lbf = ct_box_lb<D>(bx, qq, qlo, qhi);
                    keep = lbf <= bdf;
                    ++n_box;
                }
                const bool kl = keep && (child & kCtLeafBit), ki = keep && !(child & kCtLeafBit);
                const uint64_t ml = __ballot(kl), mi = __ballot(ki);
                if (kl) stk[kStack - 1 - (lsp + __popcll(ml & below_me))] = make_uint2(child, __float_as_uint(lbf));
                if (ki) stk[isp + __popcll(mi & below_me)] = make_uint2(child, __float_as_uint(lbf));
                lsp += __popcll(ml);
                isp += __popcll(mi);
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
    if (T.stats) {
#pragma unroll
        for (int off = G / 2; off > 0; off >>= 1) {
            n_pts += __shfl_xor(n_pts, off, G);
            n_box += __shfl_xor(n_box, off, G);
        }
        if (sub == 0) {
            atomicAdd(T.stats + 0, (unsigned long long)n_pts);
            atomicAdd(T.stats + 1, (unsigned long long)n_box);
            atomicAdd(T.stats + 3, (unsigned long long)n_steps);
        }
    }
    best_group<G>(bd, bi);  // the lanes' own bests
    if (sub == 0) {
        out_ids[qi] = bi;
        out_d2[qi] = bd;
    }
}

// NW nodes a step: 8 * NW lanes per query, the stack's top NW entries popped together (each
// taken by 8 lanes: a bucket's points or an inner box's 8 children); the parts' best merged,
// the children re-tested against it, deeper entries' survivors pushed below the top's (each
// part's in child order: the next step pops the top NW entries together, so ranking them by
// lower bound bought nothing -- sorting each part by a DPP network cost 4 % of the walk at 256
// seeds).  The stack holds at most ~NW blocks of 7 a level.
template <int D, int BS, int NW>
__device__ __forceinline__ void ct_walk(const CellTreeDev &T, const double *__restrict__ q, int64_t nq,
                                        int32_t *__restrict__ out_ids, double *__restrict__ out_d2, int64_t blk) {
    if constexpr (NW == 8 && D <= 7 && kCtSplitWalk) {
        ct_walk_split<D, BS>(T, q, nq, out_ids, out_d2, blk);
        return;
    }
    constexpr int G = NW * 8;        // lanes per query
    constexpr int kStack = NW * 8 * kCtMaxLevels;  // ~NW blocks of 7 a level, <= 10 levels (k_ct_levels): 5 KiB for NW = 8
    static_assert(G <= 64, "ballot bits per group");
    __shared__ uint2 s_stk[BS / G][kStack];  // (meta, lower bound's bits): one 8-byte access
    const int64_t t = blk * BS + threadIdx.x;
    const int64_t qi = t / G;
    const int sub = (int)(t % G);
    const int part = sub / 8;  // which popped entry: 0 the top, 1 the one below it, ...
    const int ls = sub % 8;    // the child / point this lane takes
    const int grp = threadIdx.x / G;
    if (qi >= nq) return;  // whole groups leave together
    double qq[D];
#pragma unroll
    for (int i = 0; i < D; ++i) qq[i] = q[qi * D + i];
    float qlo[D], qhi[D];
#pragma unroll
    for (int i = 0; i < D; ++i) {
        qlo[i] = f32_dn(qq[i]);
        qhi[i] = f32_up_any(qq[i]);
    }
    double bd = __builtin_huge_val();
    int32_t bi = -1;
    uint32_t n_pts = 0, n_box = 0, n_steps = 1;  // the seeds' step
    if (*T.n_dev > 0) {
        // the first entries (the root's children) loaded with the seeds: no dependent load
        const int n_top = *(const __attribute__((address_space(1))) int32_t *)T.n_top;
        const uint32_t top = sub < 8 ? ((gu32)T.top)[sub] : 0u;
        ct_seed<D, G>(T, qq, sub, bd, bi, n_pts);
        float bdf = f32_up(bd);
        int sp = n_top;
        if (sub < n_top) s_stk[grp][n_top - 1 - sub] = make_uint2(top, 0u);  // child 0 on top
        __builtin_amdgcn_wave_barrier();
        const int base = (threadIdx.x & 63) & ~(G - 1);
        while (sp > 0) {
            const int np = sp >= NW ? NW : sp;
            const bool have = part < np;
            uint32_t code = 0;
            float lbs = 0.0f;
            if (have) {
                const uint2 en = s_stk[grp][sp - 1 - part];
                code = en.x;
                lbs = __uint_as_float(en.y);
            }
            sp -= np;
            ++n_steps;
            __builtin_amdgcn_wave_barrier();
            const bool act = have && !(lbs > bdf);
            bool keep = false, better = false;
            float lbf = 0.0f;
            uint32_t child = 0;
            const int cnt = (int)((code >> 28) & 7u) + 1;
            if (act && ls < cnt) {
                // one load for either kind: a bucket's point (D doubles, its id) and an inner
                // node's child box (2D floats, its record) are the same 8D + 4 bytes, so a step
                // whose entries mix buckets and inner nodes waits on memory once
                const bool leaf = code & kCtLeafBit;
                const int64_t e = leaf ? (int64_t)(code & 0x0fffffffu) * kCtCap + ls
                                       : (int64_t)(code & 0x0fffffffu) + ls;
                const gdbl src = leaf ? (gdbl)T.bpts : (gdbl)(const void *)T.nbox;
                const gu32 msrc = leaf ? (gu32)(const void *)T.bids : (gu32)T.nmeta;
                double row[D];
#pragma unroll
                for (int k = 0; k < D; ++k) row[k] = src[e * D + k];
                const uint32_t meta = msrc[e];
                if (leaf) {
                    const double dd = flann_l2<D>(qq, row);
                    const int32_t id = (int32_t)meta;
                    ++n_pts;
                    better = (dd < bd) | ((dd == bd) & (id < bi));
                    // G = 64: the lane's own best may trail the wave's; only a point within the
                    // shared bound can move it
                    if constexpr (G == 64) better = better && dd <= (double)bdf;
                    nn_take(bd, bi, dd, id);
                } else {
                    float bx[2 * D];
#pragma unroll
                    for (int k = 0; k < D; ++k) {
                        bx[2 * k] = __int_as_float(__double2loint(row[k]));
                        bx[2 * k + 1] = __int_as_float(__double2hiint(row[k]));
                    }
                    child = meta;
                    lbf = ct_box_lb<D>(bx, qq, qlo, qhi);
                    keep = true;
                    ++n_box;
                }
            }
            // the parts' best, then the survivors against it.  Wave-uniform skips: a group's
            // lanes already share one best unless a lane found a better point this step, and
            // with no survivor in the wave there is nothing to rank
            if (__ballot(better)) {
                if constexpr (G == 64) {
                    // one query a wave: each lane keeps its own exact best (bd, bi) and only the
                    // pruning bound is shared -- the least of the lanes' bests rounded up to float,
                    // which is f32_up of the wave's best (f32_up is monotone), the bound the full
                    // (d2, id) merge gave: the same boxes are pruned, the same points examined,
                    // and the exact merge runs once, after the walk (one wave minimum a step that
                    // improves, where best_group took two plus the id's)
                    bdf = __uint_as_float(wave_min_u32(__float_as_uint(f32_up(bd))));
                } else {
                    best_group<G>(bd, bi);
                    bdf = f32_up(bd);
                }
            }
            keep = keep && lbf <= bdf;
            const uint64_t wm = __ballot(keep);
            const uint64_t gm = (wm >> base) & (G == 64 ? ~0ull : ((1ull << G) - 1));
            const int c = __popc((uint32_t)(gm >> (part * 8)) & 0xffu);
            const int below = __popcll(part + 1 < NW ? gm >> ((part + 1) * 8) : 0ull);
            if (keep) {  // in child order (the top NW entries are popped together)
                const uint32_t pm = (uint32_t)(gm >> (part * 8)) & 0xffu;
                const int r = __popc(pm & ((1u << ls) - 1u));
                const int pos = sp + below + (c - 1 - r);
                s_stk[grp][pos] = make_uint2(child, __float_as_uint(lbf));
            }
            sp += __popcll(gm);
            __builtin_amdgcn_wave_barrier();
        }
    }
    if (T.stats) {
#pragma unroll
        for (int off = G / 2; off > 0; off >>= 1) {
            n_pts += __shfl_xor(n_pts, off, G);
            n_box += __shfl_xor(n_box, off, G);
        }
        if (sub == 0) {
            atomicAdd(T.stats + 0, (unsigned long long)n_pts);
            atomicAdd(T.stats + 1, (unsigned long long)n_box);
            atomicAdd(T.stats + 3, (unsigned long long)n_steps);  // (+ 2: the collide counters' [10])
        }
    }
    if constexpr (G == 64) best_group<G>(bd, bi);  // the lanes' own bests (see the walk's merge)
    if (sub == 0) {
        out_ids[qi] = bi;
        out_d2[qi] = bd;
    }
}

template <int D, int BS, int W>
__global__ __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(D >= 15 ? 4 : 8))) void k_ct_nn1(
    CellTreeDev T, const double *__restrict__ q, int64_t nq, int32_t *__restrict__ out_ids, double *__restrict__ out_d2) {
    ct_walk<D, BS, W>(T, q, nq, out_ids, out_d2, blockIdx.x);
}

// Many trees in one launch (mpt_rrt_step_many: one engine per independent seed): job j takes
// workgroups [j * bpj, (j + 1) * bpj) (one query a workgroup), and workgroup b runs on XCD b % 8.
// parts = 0: consecutive workgroups of a job on the 8 XCDs in turn -- every XCD an equal share of
// every tree, but each 64-B line of a job's queries and of its results touched by up to eight
// XCDs' L2s.  parts = P > 0: job j cut into P contiguous runs of its workgroups, run r being part
// v = j * P + r, part v's workgroups all on XCD v % 8: a tree then lives in P XCDs' L2s, its
// queries' and results' lines in one (n_jobs * P a multiple of 8, bpj a multiple of P).  The
// engine runs P = 8 (kCtJointParts): each XCD a contiguous eighth of every tree's queries.
// Measured at the config-5 shape (scripts/nn_traffic.py: the last round's launch replayed alone,
// 256 trees, 28.3 M points indexed, 1 M queries; kernel trace / HBM bytes 2 FETCH + WRITE):
//   P = 0: 2.33 ms, 1271 MB (WRITE 68 MB for 12.6 MB of results);  P = 1 (round 4's whole
//   trees per XCD): 2.27 ms, 267 MB;  P = 2: 2.22 ms, 409 MB;  P = 4: 2.16 ms, 651 MB;
//   P = 8: 2.12 ms, 1078 MB (WRITE 13.4 MB)
// -- what costs time is balance and the split lines, not the bytes (the trees' lines come
// from the MALL).  Also measured (rounds 4-5) and not kept: P = 1 at 32 seeds (0.337 vs 0.284
// ms: with 4 trees an XCD the costliest set the end), and a 64-bit form of the index math that
// spilled the 64-VGPR walk.
template <int D, int BS, int W>
__global__ __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(D >= 15 ? 4 : 8))) void k_ct_nn1_jobs(
    const CtNnJob *__restrict__ jobs, int32_t n_jobs, int64_t nq, int32_t blocks_per_job, int32_t parts) {
    uint32_t job = blockIdx.x / (uint32_t)blocks_per_job, blk = blockIdx.x % (uint32_t)blocks_per_job;
    if (parts > 0) {
        const uint32_t bpp = (uint32_t)blocks_per_job / (uint32_t)parts;  // workgroups a part
        const uint32_t k = blockIdx.x / 8u;                                // this XCD's k-th workgroup
        const uint32_t v = blockIdx.x % 8u + 8u * (k / bpp);               // its part
        job = v / (uint32_t)parts;
        blk = (v % (uint32_t)parts) * bpp + k % bpp;
    }
    if (job >= (uint32_t)n_jobs) return;
    const CtNnJob J = jobs[job];  // by value: the tree's pointers stay in SGPRs across the walk
    ct_walk<D, BS, W>(J.T, J.q, nq, J.ids, J.d2, blk);
}

}  // namespace

// ---- host ----

CtPlan make_ct_plan(int32_t d, const double *lo, const double *hi, int32_t spatial) {
    CtPlan P{};
    double ext[kCtMaxDim] = {}, emax = 0.0;
    for (int j = 0; j < d; ++j) {
        ext[j] = hi[j] > lo[j] ? hi[j] - lo[j] : 0.0;
        emax = std::max(emax, ext[j]);
    }
    auto bits_of = [&](int j, double h, int k) {
        int b = 0;
        while (b < k && std::ldexp(h, b) < ext[j]) ++b;
        return b;
    };
    int kstar = 0;
    for (int k = 1; emax > 0.0 && k <= 31; ++k) {
        const double h = std::ldexp(emax, -k);
        int tot = 0;
        for (int j = 0; j < d; ++j) tot += bits_of(j, h, k);
        if (tot > kCtBits) break;
        kstar = k;
    }
    int b[kCtMaxDim] = {}, bmax = 0;
    for (int j = 0; j < d; ++j) {
        b[j] = kstar > 0 ? bits_of(j, std::ldexp(emax, -kstar), kstar) : 0;
        bmax = std::max(bmax, b[j]);
        P.lo[j] = lo[j];
        P.nb[j] = (int8_t)b[j];
        P.qmax[j] = b[j] > 0 ? (uint32_t)((1ull << b[j]) - 1) : 0u;
        P.scale[j] = b[j] > 0 ? std::ldexp(1.0, b[j]) / ext[j] : 0.0;
    }
    int n = 0;
    for (int l = bmax - 1; l >= 0; --l)
        for (int j = 0; j < d; ++j)
            if (b[j] > l) {
                P.dim[n] = (int8_t)j;
                P.bit[n] = (int8_t)l;
                ++n;
            }
    P.n = n;
    P.bmax = bmax;
    // seed slots: every dim's minimum and maximum, then directions over the first `spatial`
    // dims spread evenly (a Fibonacci lattice on the sphere; the circle for two dims)
    int h = 0;
    for (int j = 0; j < d && h + 1 < kCtHull; ++j) {
        P.hkind[h] = 1;
        P.hdim[h++] = (int8_t)j;
        P.hkind[h] = 2;
        P.hdim[h++] = (int8_t)j;
    }
    const int sd = std::max(1, std::min<int>(spatial, std::min(d, 3)));
    const int nd = kCtHull - h;
    for (int k = 0; k < nd; ++k, ++h) {
        double u[3] = {0.0, 0.0, 0.0};
        if (sd == 3) {
            const double z = 1.0 - (2.0 * k + 1.0) / nd, r = std::sqrt(std::max(0.0, 1.0 - z * z));
            const double phi = k * 2.399963229728653;  // the golden angle
            u[0] = r * std::cos(phi);
            u[1] = r * std::sin(phi);
            u[2] = z;
        } else if (sd == 2) {
            const double a = 2.0 * M_PI * (k + 0.5) / nd;
            u[0] = std::cos(a);
            u[1] = std::sin(a);
        } else {
            u[0] = (k & 1) ? 1.0 : -1.0;
        }
        P.hkind[h] = 0;
        P.hdim[h] = 0;
        for (int j = 0; j < 3; ++j) P.hdir[h][j] = (float)u[j];
    }
    P.n_hull = h;
    return P;
}

void CellTree::release() {
    if (slab) (void)hipFree(slab);
    slab = nullptr;
}

CellTree::~CellTree() { release(); }

void CellTree::reserve(int64_t c, int32_t d) {
    if (c <= cap_ && d == dim) return;
    if (d != 3 && d != 7 && d != 15) throw Error{1, "cell tree: state dim must be 3, 7 or 15"};
    if (c >= (int64_t(1) << 26)) throw Error{1, "cell tree: capacity too large"};  // node indices < 2^28
    hip_check(hipDeviceSynchronize(), "sync");  // the old buffers may still be in use
    release();
    *this = CellTree();
    c = std::max<int64_t>(c, 64);
    cap_ = c;
    dim = d;
    bcap = (int32_t)(c + 1);  // every bucket holds at least one point, an empty tree one bucket
    const int64_t nodes = 2 * (int64_t)bcap + 64;  // each level at most half the one below, or runs of 8
    // every buffer carved from one allocation (one hipMalloc an engine, not ~45: config 5
    // reserves 256 trees in its first round)
    std::vector<std::pair<void **, size_t>> bufs;
    auto al = [&](void **p, size_t bytes, const char *) { bufs.emplace_back(p, std::max<size_t>(bytes, 16)); };
    al((void **)&plan, sizeof(CtPlan), "ct plan");
    al((void **)&cnt, sizeof(CtCounts), "ct counts");
    al((void **)&bpts, sizeof(double) * bcap * kCtCap * d, "ct bucket rows");
    al((void **)&bids, sizeof(int32_t) * bcap * kCtCap, "ct bucket ids");
    al((void **)&bcode, sizeof(uint64_t) * 2 * bcap * kCtCap, "ct bucket codes");
    al((void **)&bcnt, sizeof(int32_t) * bcap, "ct bucket counts");
    al((void **)&bbox, sizeof(float) * 2 * d * bcap, "ct bucket boxes");
    for (int k = 0; k < 2; ++k) {
        al((void **)&nbox[k], sizeof(float) * 2 * d * nodes, "ct node boxes");
        al((void **)&nmeta[k], sizeof(uint32_t) * nodes, "ct node codes");
    }
    al((void **)&ucode, sizeof(uint64_t) * 2 * nodes, "ct node cell codes");
    al((void **)&lflag, sizeof(int32_t) * nodes, "ct level scratch");
    al((void **)&lcount, sizeof(int32_t) * (bcap / kCtL1Tile + bcap / (2 * kCtL1Tile) + 2), "ct level scratch");
    for (int k = 0; k < 2; ++k) {
        al((void **)&dir_code[k], sizeof(uint64_t) * 2 * bcap, "ct directory");
    }
    al((void **)&ncode, sizeof(uint64_t) * 2 * kCtSeg, "ct new codes");
    al((void **)&ccode, sizeof(uint64_t) * 2 * kCtSeg, "ct chunk codes");
    al((void **)&nrow, sizeof(int32_t) * kCtSeg, "ct new rows");
    al((void **)&crow, sizeof(int32_t) * kCtSeg, "ct chunk rows");
    al((void **)&npos, sizeof(int32_t) * kCtSeg, "ct positions");
    al((void **)&nseg, sizeof(int32_t) * kCtSeg, "ct segments");
    al((void **)&seg, sizeof(int4) * kCtSeg, "ct segments");
    al((void **)&seg_pos, sizeof(int32_t) * kCtSeg, "ct segments");
    al((void **)&seg_first, sizeof(int32_t) * kCtSeg, "ct segments");
    al((void **)&scode, sizeof(uint64_t) * 2 * kCtScratch, "ct scratch");
    al((void **)&srow, sizeof(int32_t) * kCtScratch, "ct scratch");
    al((void **)&sseg, sizeof(int32_t) * kCtScratch, "ct scratch");
    al((void **)&slead, sizeof(int32_t) * kCtScratch, "ct scratch");
    al((void **)&srank, sizeof(int32_t) * kCtScratch, "ct scratch");
    al((void **)&edir_code, sizeof(uint64_t) * 2 * kCtScratch, "ct new entries");
    al((void **)&edir_bk, sizeof(int32_t) * kCtScratch, "ct new entries");
    al((void **)&edir_pos, sizeof(int32_t) * kCtScratch, "ct new entries");
    al((void **)&hull_keys, sizeof(unsigned long long) * kCtHull, "ct seeds");
    al((void **)&hull_pts, sizeof(double) * kCtHull * d, "ct seeds");
    al((void **)&hull_ids, sizeof(int32_t) * kCtHull, "ct seeds");
    al((void **)&ibox, sizeof(unsigned long long) * 2 * kCtMaxDim, "ct box");
    for (uint64_t **p : {&fhi, &flo, &fk0, &fk1}) al((void **)p, sizeof(uint64_t) * 2 * c, "ct full sort");
    for (int32_t **p : {&fv0, &fv1, &fflag, &fleaf}) al((void **)p, sizeof(int32_t) * c, "ct full sort");
    size_t tb = 0, tb2 = 0;
    hip_check(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, flo, fk0, fv0, fv1, (int)c, 0, 64), "ct sort size");
    hip_check(hipcub::DeviceScan::ExclusiveSum(nullptr, tb2, fflag, fleaf, (int)c), "ct scan size");
    ftemp_bytes = std::max(tb, tb2);
    al(&ftemp, ftemp_bytes, "ct sort temp");
    size_t total = 0;
    for (auto &b : bufs) total += (b.second + 255) & ~size_t(255);
    hip_check(hipMalloc(&slab, total), "ct index");
    char *at = static_cast<char *>(slab);
    for (auto &b : bufs) {
        *b.first = at;
        at += (b.second + 255) & ~size_t(255);
    }
    hip_check(hipMemset(cnt, 0, sizeof(CtCounts)), "ct counts zero");
    hip_check(hipDeviceSynchronize(), "ct init sync");  // the null stream vs the caller's stream
}

bool CellTree::set_plan(const double *lo, const double *hi, int32_t spatial) {
    if (!plan) throw Error{1, "cell tree: not reserved"};
    bool same = plan_set;
    for (int j = 0; j < dim && same; ++j) same = plan_lo[j] == lo[j] && plan_hi[j] == hi[j];
    if (same) return false;
    const CtPlan P = make_ct_plan(dim, lo, hi, spatial);
    hip_check(hipMemcpy(plan, &P, sizeof(P), hipMemcpyHostToDevice), "ct plan");
    for (int j = 0; j < dim; ++j) {
        plan_lo[j] = lo[j];
        plan_hi[j] = hi[j];
    }
    plan_set = true;
    return true;
}

CtJob CellTree::prepare(const double *pts, int64_t n_upper, const int64_t *n_dev, int32_t d, const double *lo,
                        const double *hi, int32_t spatial, bool full, int64_t grow, hipStream_t stream,
                        const SpreadOut *spread, unsigned long long *err) {
    if (d != dim || n_upper > cap_) throw Error{1, "cell tree: not reserved for this size"};
    if (n_upper < 1) throw Error{1, "cell tree: empty layout"};
    if (set_plan(lo, hi, spatial)) full = true;
    const int old = cur, nw = cur ^ 1;
    const bool reset = full && n_upper <= kCtSeg;
    if (reset) {
        full = false;
        grow = n_upper;
    }
    if (full) {
        // every point: box, codes and seed offers, a two-pass stable sort by (code, row), the
        // leaf rule, the leaves' ranks, buckets and directory (into the round's old directory)
        hipLaunchKernelGGL(k_ct_box_reset, dim3(1), dim3(64), 0, stream, ibox);
        hip_check(hipMemsetAsync(hull_keys, 0, sizeof(unsigned long long) * kCtHull, stream), "seed reset");
        const unsigned blocks = (unsigned)((n_upper + 255) / 256);
        hipLaunchKernelGGL(d == 3 ? k_ct_codes_all<3> : d == 7 ? k_ct_codes_all<7> : k_ct_codes_all<15>, dim3(blocks),
                           dim3(64 * kCtWaves), 0, stream, pts, n_upper, n_dev, (const CtPlan *)plan, fhi, flo, fv0,
                           hull_keys, ibox);
        hip_check(hipGetLastError(), "k_ct_codes_all");
        size_t tb = ftemp_bytes;
        hip_check(hipcub::DeviceRadixSort::SortPairs(ftemp, tb, flo, fk0, fv0, fv1, (int)n_upper, 0, 64, stream),
                  "ct sort low");
        hipLaunchKernelGGL(k_ct_gather_hi, dim3(blocks), dim3(256), 0, stream, fhi, fv1, n_upper, fk1);
        tb = ftemp_bytes;
        hip_check(hipcub::DeviceRadixSort::SortPairs(ftemp, tb, fk1, fk0, fv1, fv0, (int)n_upper, 0, 64, stream),
                  "ct sort high");
        // (hi, lo) pairs of the sorted order into fk1 (n_upper * 2 words: fk1 is sized 2c)
        hipLaunchKernelGGL(k_ct_pack, dim3(blocks), dim3(256), 0, stream, fk0, flo, fv0, n_upper, n_dev, fk1);
        hipLaunchKernelGGL(k_ct_bulk_flags, dim3(blocks), dim3(256), 0, stream, fk1, fv0, n_upper, n_dev, fflag);
        tb = ftemp_bytes;
        hip_check(hipcub::DeviceScan::ExclusiveSum(ftemp, tb, fflag, fleaf, (int)n_upper, stream), "ct leaf scan");
        hipLaunchKernelGGL(d == 3 ? k_ct_bulk_fill<3> : d == 7 ? k_ct_bulk_fill<7> : k_ct_bulk_fill<15>, dim3(blocks),
                           dim3(256), 0, stream, pts, fk1, fv0, fflag, fleaf, n_upper, n_dev, bpts, bids, bcode, bcnt,
                           bbox, dir_code[old], nmeta[old], nbox[old], cnt);
        hip_check(hipGetLastError(), "k_ct_bulk_fill");
    }
    t.d = d;
    t.n_bound = std::max<int64_t>(std::min<int64_t>(n_upper, bcap), 1);
    t.n_dev = n_dev;
    t.root = &cnt->root;
    t.top = cnt->top;
    t.n_top = &cnt->n_top;
    t.lv = &cnt->lv_first;
    t.nmeta = nmeta[nw];
    t.nbox = nbox[nw];
    t.bpts = bpts;
    t.bids = bids;
    t.hull_pts = hull_pts;
    t.hull_ids = hull_ids;
    t.stats = nullptr;
    cur = nw;
    CtJob J{};
    J.T = t;
    J.pts = pts;
    J.plan = plan;
    J.cnt = cnt;
    J.bcap = bcap;
    J.mb = full ? 0 : (int32_t)std::min<int64_t>(std::max<int64_t>(grow, 0), kCtSeg);
    J.reset = reset ? 1 : 0;
    J.bpts = bpts;
    J.bids = bids;
    J.bcode = bcode;
    J.bcnt = bcnt;
    J.bbox = bbox;
    J.odir_code = dir_code[old];
    J.ometa = nmeta[old];
    J.obox = nbox[old];
    J.ndir_code = dir_code[nw];
    J.nmeta = nmeta[nw];
    J.nbox = nbox[nw];
    J.ucode = ucode;
    J.lflag = lflag;
    J.lcount = lcount;
    J.ncode = ncode;
    J.nrow = nrow;
    J.ccode = ccode;
    J.crow = crow;
    J.npos = npos;
    J.nseg = nseg;
    J.seg = seg;
    J.seg_pos = seg_pos;
    J.seg_first = seg_first;
    J.scode = scode;
    J.srow = srow;
    J.sseg = sseg;
    J.slead = slead;
    J.srank = srank;
    J.edir_code = edir_code;
    J.edir_bk = edir_bk;
    J.edir_pos = edir_pos;
    J.hull_keys = hull_keys;
    J.hull_pts = hull_pts;
    J.hull_ids = hull_ids;
    J.ibox = ibox;
    if (spread) J.sp = *spread;
    J.err = err;
    return J;
}

void launch_ct_jobs(const CtJob *d_jobs, const CtJob *h_jobs, int32_t n, int32_t d, hipStream_t stream) {
    if (n <= 0) return;
    if (d != 3 && d != 7 && d != 15) throw Error{1, "cell tree: state dim must be 3, 7 or 15"};
    CtJobs js{n == 1 ? nullptr : d_jobs, h_jobs[0]};
    // grids from the host's bounds (a workgroup that only learns on the device that it has
    // nothing to do still pays its dependent count loads: sized by the real work, not the caps)
    int64_t max_n = 0, mb = 0;
    for (int32_t j = 0; j < n; ++j) {
        max_n = std::max(max_n, h_jobs[j].T.n_bound);
        mb = std::max<int64_t>(mb, h_jobs[j].mb);
    }
    auto by_d = [&](auto k3, auto k7, auto k15) { return d == 3 ? k3 : d == 7 ? k7 : k15; };
    const unsigned yn = (unsigned)n;
    bool any_reset = false;
    for (int32_t j = 0; j < n; ++j) any_reset = any_reset || h_jobs[j].reset;
    if (any_reset) {
        hipLaunchKernelGGL(k_ct_reset, dim3(1, yn), dim3(64), 0, stream, js);
        hip_check(hipGetLastError(), "k_ct_reset");
    }
    if (mb > 0) {
        const unsigned b256 = (unsigned)((mb + 255) / 256);
        // (round 4: these four fused into one workgroup a tree ran 0.30-0.40 ms a round at 256
        // seeds and 0.28-0.36 at 32, against 0.27 and 0.15 as separate launches: the codes and
        // seed offers need the waves of many workgroups)
        hipLaunchKernelGGL(by_d(k_ct_ncodes<3>, k_ct_ncodes<7>, k_ct_ncodes<15>), dim3(b256, yn), dim3(64 * kCtWaves), 0,
                           stream, js);
        hip_check(hipGetLastError(), "k_ct_ncodes");
        // the sort over many CUs: chunks of 512 sorted by a workgroup each, then every pair's
        // rank across the chunks (round 4: one workgroup a tree sorting in LDS took 0.12 ms a
        // round at 256 seeds and 0.11 at 32 -- at 32 trees most CUs idle).  Round 5, measured and
        // not kept: the codes computed inside the sort's workgroups (one launch less: 36 -> 47 us
        // at 32 seeds, half the threads coding; equal at 256), and the directory search folded
        // into the rank kernel (23 -> 22 us at 32 seeds, 102 -> 129 us at 256: the searches in
        // chunk order lose the sorted order's cache locality)
        const unsigned chunks = (unsigned)((mb + kCtChunk - 1) / kCtChunk);
        hipLaunchKernelGGL(k_ct_csort, dim3(chunks, yn), dim3(kCtSortThreads), 0, stream, js);
        hipLaunchKernelGGL(k_ct_crank, dim3(b256, yn), dim3(256), 0, stream, js);
        hipLaunchKernelGGL(k_ct_locate, dim3(b256, yn), dim3(256), 0, stream, js);
        hipLaunchKernelGGL(k_ct_segments, dim3(1, yn), dim3(kCtSegThreads), 0, stream, js);
        hipLaunchKernelGGL(by_d(k_ct_apply<3>, k_ct_apply<7>, k_ct_apply<15>), dim3(b256, yn), dim3(256), 0, stream, js);
        hip_check(hipGetLastError(), "k_ct_apply");
        // the split elements: at most 9 a new point, a thread each, in chunks of 256 strided
        // over a grid of twice the new points' (a grid for the bound of 9 a point dispatched
        // workgroups that found no chunk; with the other round-5 build changes, split_fill
        // 23.8 -> 21.7 us a round at 32 seeds)
        const unsigned bsplit = (unsigned)std::min<int64_t>((mb * (kCtCap + 1) + 255) / 256, 2 * (int64_t)b256);
        hipLaunchKernelGGL(k_ct_split_flags, dim3(b256, yn), dim3(256), 0, stream, js);
        hipLaunchKernelGGL(k_ct_split_scan, dim3(1, yn), dim3(kCtScanThreads), 0, stream, js);
        hipLaunchKernelGGL(by_d(k_ct_split_fill<3>, k_ct_split_fill<7>, k_ct_split_fill<15>), dim3(bsplit, yn),
                           dim3(256), 0, stream, js);
        hip_check(hipGetLastError(), "k_ct_split_fill");
    }
    // the directory (at most the indexed points' count of entries, ~1/5 of them in practice)
    // (a workgroup a chunk of 256 entries when a tree has ~1/4 as many entries as points)
    hipLaunchKernelGGL(by_d(k_ct_dmerge<3>, k_ct_dmerge<7>, k_ct_dmerge<15>),
                       dim3((unsigned)std::max<int64_t>(1, (max_n + 1023) / 1024), yn), dim3(256), 0, stream, js);
    hip_check(hipGetLastError(), "k_ct_dmerge");
    // levels 1 and 2 over many workgroups, tiles in a grid-stride loop over a grid for a
    // quarter of the host's bound (a tree has ~1/5 as many directory entries as points, level 2
    // ~1/5 of those: the bound's grids dispatched ~5x as many workgroups as had a tile)
    const unsigned tiles = (unsigned)std::max<int64_t>(1, (max_n / 4 + kCtL1Tile - 1) / kCtL1Tile);
    hipLaunchKernelGGL(k_ct_lflags<1>, dim3(tiles, yn), dim3(256), 0, stream, js);
    hipLaunchKernelGGL(by_d(k_ct_lgroup<3, 1>, k_ct_lgroup<7, 1>, k_ct_lgroup<15, 1>), dim3(tiles, yn), dim3(256), 0,
                       stream, js);
    const unsigned tiles2 = (tiles + 3) / 4;
    hipLaunchKernelGGL(k_ct_lflags<2>, dim3(tiles2, yn), dim3(256), 0, stream, js);
    hipLaunchKernelGGL(by_d(k_ct_lgroup<3, 2>, k_ct_lgroup<7, 2>, k_ct_lgroup<15, 2>), dim3(tiles2, yn), dim3(256), 0,
                       stream, js);
    hipLaunchKernelGGL(by_d(k_ct_levels<3>, k_ct_levels<7>, k_ct_levels<15>), dim3(1, yn), dim3(kCtLevelThreads), 0,
                       stream, js);
    hip_check(hipGetLastError(), "k_ct_levels");
}

template <int W>
static void launch_ct_nn1_w(const CellTreeDev &T, const double *q, int64_t nq, int32_t *ids, double *d2,
                            hipStream_t stream) {
    constexpr int BS = 64;
    const dim3 grid((unsigned)((nq * 8 * W + BS - 1) / BS));
    switch (T.d) {
        case 3: hipLaunchKernelGGL((k_ct_nn1<3, BS, W>), grid, dim3(BS), 0, stream, T, q, nq, ids, d2); break;
        case 7: hipLaunchKernelGGL((k_ct_nn1<7, BS, W>), grid, dim3(BS), 0, stream, T, q, nq, ids, d2); break;
        case 15: hipLaunchKernelGGL((k_ct_nn1<15, BS, W>), grid, dim3(BS), 0, stream, T, q, nq, ids, d2); break;
        default: throw Error{1, "cell tree: state dim must be 3, 7 or 15"};
    }
    hip_check(hipGetLastError(), "k_ct_nn1 launch");
}

// nodes a walk step: eight (one query a wave) for d <= 7, four for d = 15 (its registers)
// (round 4, config 5: four nodes a step with two queries a wave took 3.42 vs 2.62 ms at 256
// seeds, 0.52 vs 0.42 ms at 32 -- more steps a query, 19.8 vs 13.4, and a wave waits for both)
static int ct_width(int32_t d) { return d <= 7 ? 8 : 4; }

void launch_ct_nn1(const CellTreeDev &T, const double *q, int64_t nq, int32_t *ids, double *d2, hipStream_t stream) {
    if (nq <= 0) return;
    if (ct_width(T.d) == 8) launch_ct_nn1_w<8>(T, q, nq, ids, d2, stream);
    else launch_ct_nn1_w<4>(T, q, nq, ids, d2, stream);
}

template <int W>
static void launch_ct_nn1_jobs_w(const CtNnJob *d_jobs, int32_t n_jobs, int32_t d, int64_t nq, hipStream_t stream,
                                 int32_t parts) {
    constexpr int BS = 64;
    const int64_t bpj = (nq * 8 * W + BS - 1) / BS;
    if (bpj * n_jobs > 0x7fffffffLL) throw Error{1, "cell tree: joint NN launch too large"};
    const dim3 grid((unsigned)(bpj * n_jobs));
    const int32_t b = (int32_t)bpj;
    switch (d) {
        case 3: hipLaunchKernelGGL((k_ct_nn1_jobs<3, BS, W>), grid, dim3(BS), 0, stream, d_jobs, n_jobs, nq, b, parts); break;
        case 7: hipLaunchKernelGGL((k_ct_nn1_jobs<7, BS, W>), grid, dim3(BS), 0, stream, d_jobs, n_jobs, nq, b, parts); break;
        case 15: hipLaunchKernelGGL((k_ct_nn1_jobs<15, BS, W>), grid, dim3(BS), 0, stream, d_jobs, n_jobs, nq, b, parts); break;
        default: throw Error{1, "cell tree: state dim must be 3, 7 or 15"};
    }
    hip_check(hipGetLastError(), "k_ct_nn1_jobs launch");
}

int32_t ct_joint_parts(int32_t n_jobs, int32_t d, int64_t nq) {
    const int64_t bpj = (nq * 8 * ct_width(d) + 63) / 64;
    return ((int64_t)n_jobs * kCtJointParts % 8 == 0 && bpj % kCtJointParts == 0) ? kCtJointParts : 0;
}

void launch_ct_nn1_jobs(const CtNnJob *d_jobs, int32_t n_jobs, int32_t d, int64_t nq, hipStream_t stream,
                        int32_t parts) {
    if (nq <= 0 || n_jobs <= 0) return;
    if (parts < 0 || parts > 64) throw Error{1, "cell tree: joint NN parts out of range"};
    if (parts > 0) {
        const int64_t bpj = (nq * 8 * ct_width(d) + 63) / 64;  // launch_ct_nn1_jobs_w's BS = 64
        if ((int64_t)n_jobs * parts % 8 != 0 || bpj % parts != 0)
            throw Error{1, "cell tree: joint NN parts need jobs * parts % 8 == 0 and a whole number of workgroups a part"};
    }
    if (ct_width(d) == 8) launch_ct_nn1_jobs_w<8>(d_jobs, n_jobs, d, nq, stream, parts);
    else launch_ct_nn1_jobs_w<4>(d_jobs, n_jobs, d, nq, stream, parts);
}

}  // namespace mpt
