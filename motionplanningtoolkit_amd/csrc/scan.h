// scan.h -- single-launch exclusive scan of uint32 counts (decoupled look-back), with an
// optional per-element epilogue, for the two scans of an engine round (the grid's cell
// counts -> cell_start, the collide path's header counts -> header offsets + dense slots).
// hipcub's scan is two launches (look-back state init + scan) and the header scan needed a
// third (k_expand); here each is one.
//
// Tile = 256 threads x kItems counts.  A workgroup takes a tile index from a monotone ticket
// (so tiles are claimed in dispatch order and a tile only ever waits on tiles already
// running or done), publishes its aggregate, walks back over its predecessors' words until
// it meets an inclusive prefix, then publishes its own inclusive prefix.  Each status word
// packs (epoch, kind, value) into one 64-bit agent-scope atomic, so a reader sees the flag and
// the value together without a fence; words of earlier launches (older epochs) read as "not
// yet".  Nothing is reset between launches: the host advances the epoch and the ticket base.
#pragma once
#include "mpt_internal.h"

namespace mpt {

constexpr int kScanThreads = 256;

struct NoEpilogue {
    __device__ void operator()(int64_t, uint32_t, uint32_t) const {}
};

__device__ __forceinline__ unsigned long long scan_word(uint32_t epoch, uint32_t kind, uint32_t v) {
    return ((unsigned long long)epoch << 34) | ((unsigned long long)kind << 32) | v;
}

// out[i] = sum of in[0, i) for i < n; epi(i, out[i], in[i]) for every i < n.  kItems counts
// per thread (a tile of 256 kItems); an epilogue with work per element wants kItems = 1.
template <class Epi, int kItems>
__global__ __launch_bounds__(kScanThreads) void k_scan_excl(const uint32_t *__restrict__ in, uint32_t *__restrict__ out,
                                                            int64_t n, unsigned long long *__restrict__ status,
                                                            unsigned long long *__restrict__ ticket, uint64_t base,
                                                            uint32_t epoch, Epi epi) {
    __shared__ uint32_t s_wave[kScanThreads / 64];
    __shared__ uint32_t s_prefix;
    __shared__ int64_t s_tile;
    if (threadIdx.x == 0) s_tile = (int64_t)(atomicAdd(ticket, 1ull) - base);
    __syncthreads();
    const int64_t tile = s_tile;
    const int64_t i0 = tile * (kScanThreads * kItems) + (int64_t)threadIdx.x * kItems;
    uint32_t v[kItems], sum = 0;
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
        v[k] = i0 + k < n ? in[i0 + k] : 0u;
        sum += v[k];
    }
    // exclusive scan of the per-thread sums over the workgroup
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t incl = sum;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t o = __shfl_up(incl, off);
        if (lane >= off) incl += o;
    }
    if (lane == 63) s_wave[wave] = incl;
    __syncthreads();
    uint32_t wbase = 0, total = 0;
#pragma unroll
    for (int w = 0; w < kScanThreads / 64; ++w) {
        wbase += w < wave ? s_wave[w] : 0u;
        total += s_wave[w];
    }
    if (wave == 0) {
        // wave 0 looks back 64 predecessors at a time (lane l reads tile - 1 - l - 64 k): the
        // window is complete once every lane up to the nearest inclusive prefix has published,
        // so a tile costs one round trip per 64 predecessors instead of one per predecessor
        uint32_t pre = 0;
        if (tile == 0) {
            if (lane == 0)
                __hip_atomic_store(status, scan_word(epoch, 2u, total), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            if (lane == 0)
                __hip_atomic_store(status + tile, scan_word(epoch, 1u, total), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            for (int64_t end = tile;;) {
                const int64_t j = end - 1 - lane;
                const unsigned long long wd =
                    j >= 0 ? __hip_atomic_load(status + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                           : scan_word(epoch, 2u, 0u);
                const bool ready = (uint32_t)(wd >> 34) == epoch;
                const uint64_t pmask = __ballot(ready && ((wd >> 32) & 3u) == 2u);
                const uint64_t rmask = __ballot(ready);
                const int first_p = pmask ? __ffsll((unsigned long long)pmask) - 1 : 64;
                const uint64_t need = first_p >= 63 ? ~0ull : ((1ull << (first_p + 1)) - 1ull);
                if ((rmask & need) != need) {
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                uint32_t val = lane <= first_p ? (uint32_t)wd : 0u;
#pragma unroll
                for (int off = 32; off > 0; off >>= 1) val += __shfl_xor(val, off);
                pre += val;
                if (first_p < 64) break;
                end -= 64;
            }
            if (lane == 0)
                __hip_atomic_store(status + tile, scan_word(epoch, 2u, pre + total), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
        if (lane == 0) s_prefix = pre;
    }
    __syncthreads();
    uint32_t run = s_prefix + wbase + (incl - sum);
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
        if (i0 + k < n) {
            out[i0 + k] = run;
            epi(i0 + k, run, v[k]);
        }
        run += v[k];
    }
}

template <int kItems = 8, class Epi>
inline void launch_scan_excl(ScanState &s, const uint32_t *in, uint32_t *out, int64_t n, hipStream_t stream, Epi epi) {
    if (n <= 0) return;
    const int64_t tiles = (n + kScanThreads * kItems - 1) / (kScanThreads * kItems);
    s.reserve(tiles);
    s.epoch = s.epoch + 1 < (1u << 30) ? s.epoch + 1 : 1u;
    hipLaunchKernelGGL((k_scan_excl<Epi, kItems>), dim3((unsigned)tiles), dim3(kScanThreads), 0, stream, in, out, n,
                       s.status, s.ticket, (uint64_t)s.launched, s.epoch, epi);
    hip_check(hipGetLastError(), "k_scan_excl launch");
    s.launched += (uint64_t)tiles;
}

}  // namespace mpt
