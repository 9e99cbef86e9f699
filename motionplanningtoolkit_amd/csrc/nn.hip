// nn.hip -- exact nearest-neighbour queries over the device-resident tree/roadmap.
//
// Replaces FLANN_KDTreeWrapper::{nearest,kNearest,kNearestWithin}
// (utilities/flannkdtreewrapper.hpp:57-117) and the FLANN 1.8.4 index behind it.
// Contract (DESIGN.md "NN"): exact search, squared L2 accumulated in FLANN's L2<double>
// order (fcl_math.h flann_l2), ids 1-based in insertion order, results ordered by
// (d2, id); radius search keeps d2 < r2 (FLANN's leaf test `dist < worst_dist`).
//
// Mapping (brute force, FP64-VALU bound): one lane per query, the node stream is
// wave-uniform so node coordinates arrive through scalar loads (SGPR operands, no LDS
// round trip); blockIdx.y splits the node range so small query batches still fill
// the 256 CUs; a merge kernel reduces the per-split partials in (d2, id) order.
#include <vector>

#include "mpt_internal.h"

namespace mpt {

constexpr int kNNBlock = 256;
constexpr double kInf = __builtin_huge_val();

template <int KMAX>
__device__ __forceinline__ void topk_push(double (&bd)[KMAX], int32_t (&bi)[KMAX], int32_t k,
                                          double dd, int32_t id) {
    // place (dd, id) in slot k-1 if it beats it, then bubble it towards slot 0;
    // every array index is a compile-time constant (no scratch spill).
    bool done = false;
#pragma unroll
    for (int j = KMAX - 1; j >= 0; --j) {
        if (j >= k || done) continue;
        if (j == k - 1) {
            if (!nn_better(dd, id, bd[j], bi[j])) { done = true; continue; }
            bd[j] = dd;
            bi[j] = id;
        }
        if (j > 0 && nn_better(bd[j], bi[j], bd[j - 1], bi[j - 1])) {
            const double td = bd[j]; bd[j] = bd[j - 1]; bd[j - 1] = td;
            const int32_t ti = bi[j]; bi[j] = bi[j - 1]; bi[j - 1] = ti;
        } else {
            done = true;
        }
    }
}

// Partial 1-NN over node range [beg, end) of split blockIdx.y.
template <int D>
__global__ __launch_bounds__(kNNBlock) void k_knn1(const double *__restrict__ pts,
                                                   const uint8_t *__restrict__ removed, int64_t n,
                                                   int32_t d, const double *__restrict__ q, int64_t nq,
                                                   int64_t chunk, const int64_t *__restrict__ n_dev,
                                                   double *__restrict__ pd2, int32_t *__restrict__ pid) {
    constexpr int DD = D > 0 ? D : 16;
    const int64_t qi = (int64_t)blockIdx.x * kNNBlock + threadIdx.x;
    const int64_t s = blockIdx.y;
    if (n_dev) n = *n_dev < n ? *n_dev : n;
    const int64_t beg = s * chunk;
    const int64_t end = beg + chunk < n ? beg + chunk : n;
    const int dim = D > 0 ? D : d;
    double qq[DD];
    const int64_t qs = qi < nq ? qi : nq - 1;
#pragma unroll
    for (int i = 0; i < DD; ++i) qq[i] = i < dim ? q[qs * dim + i] : 0.0;
    double best = kInf;
    int32_t bid = -1;
    if (removed == nullptr) {
#pragma unroll 4
        for (int64_t j = beg; j < end; ++j) {
            const double dd = D > 0 ? flann_l2<DD>(qq, pts + j * DD) : flann_l2_dyn(qq, pts + j * dim, dim);
            if (dd < best) { best = dd; bid = (int32_t)(j + 1); }
        }
    } else {
        for (int64_t j = beg; j < end; ++j) {
            if (removed[j]) continue;
            const double dd = D > 0 ? flann_l2<DD>(qq, pts + j * DD) : flann_l2_dyn(qq, pts + j * dim, dim);
            if (dd < best) { best = dd; bid = (int32_t)(j + 1); }
        }
    }
    if (qi < nq) {
        pd2[s * nq + qi] = best;
        pid[s * nq + qi] = bid;
    }
}

template <int D, int KMAX>
__global__ __launch_bounds__(kNNBlock) void k_knnk(const double *__restrict__ pts,
                                                   const uint8_t *__restrict__ removed, int64_t n,
                                                   int32_t d, const double *__restrict__ q, int64_t nq,
                                                   int64_t chunk, const int64_t *__restrict__ n_dev, int32_t k,
                                                   double *__restrict__ pd2, int32_t *__restrict__ pid) {
    constexpr int DD = D > 0 ? D : 16;
    const int64_t qi = (int64_t)blockIdx.x * kNNBlock + threadIdx.x;
    const int64_t s = blockIdx.y;
    if (n_dev) n = *n_dev < n ? *n_dev : n;
    const int64_t beg = s * chunk;
    const int64_t end = beg + chunk < n ? beg + chunk : n;
    const int dim = D > 0 ? D : d;
    double qq[DD];
    const int64_t qs = qi < nq ? qi : nq - 1;
#pragma unroll
    for (int i = 0; i < DD; ++i) qq[i] = i < dim ? q[qs * dim + i] : 0.0;
    double bd[KMAX];
    int32_t bi[KMAX];
#pragma unroll
    for (int i = 0; i < KMAX; ++i) { bd[i] = kInf; bi[i] = -1; }
    for (int64_t j = beg; j < end; ++j) {
        if (removed && removed[j]) continue;
        const double dd = D > 0 ? flann_l2<DD>(qq, pts + j * DD) : flann_l2_dyn(qq, pts + j * dim, dim);
        const int32_t id = (int32_t)(j + 1);
        // cheap reject against the current k-th best before the insertion network
        double kd = bd[0];
        int32_t ki = bi[0];
#pragma unroll
        for (int i = 0; i < KMAX; ++i)
            if (i == k - 1) { kd = bd[i]; ki = bi[i]; }
        if (nn_better(dd, id, kd, ki)) topk_push<KMAX>(bd, bi, k, dd, id);
    }
    if (qi < nq) {
        double *od = pd2 + (s * nq + qi) * k;
        int32_t *oi = pid + (s * nq + qi) * k;
#pragma unroll
        for (int i = 0; i < KMAX; ++i)
            if (i < k) { od[i] = bd[i]; oi[i] = bi[i]; }
    }
}

// Merge S partial sorted lists per query into the final k.
__global__ void k_knn_merge(const double *__restrict__ pd2, const int32_t *__restrict__ pid, int64_t S,
                            int64_t nq, int32_t k, int32_t *__restrict__ ids, double *__restrict__ d2) {
    const int64_t qi = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (qi >= nq) return;
    constexpr int KMAX = 32;
    double bd[KMAX];
    int32_t bi[KMAX];
#pragma unroll
    for (int i = 0; i < KMAX; ++i) { bd[i] = kInf; bi[i] = -1; }
    for (int64_t s = 0; s < S; ++s)
        for (int32_t i = 0; i < k; ++i) {
            const double dd = pd2[(s * nq + qi) * k + i];
            const int32_t id = pid[(s * nq + qi) * k + i];
            if (id < 0) break;
            topk_push<KMAX>(bd, bi, k, dd, id);
        }
#pragma unroll
    for (int i = 0; i < KMAX; ++i)
        if (i < k) { ids[qi * k + i] = bi[i]; d2[qi * k + i] = bd[i]; }
}

static int64_t pick_splits(int64_t nq, int64_t n) {
    const int64_t qblocks = (nq + kNNBlock - 1) / kNNBlock;
    int64_t S = (2048 + qblocks - 1) / qblocks;      // aim for >= 2048 workgroups
    const int64_t maxS = (n + 511) / 512;             // keep >= 512 nodes per split
    if (S > maxS) S = maxS;
    if (S < 1) S = 1;
    if (S > 65535) S = 65535;
    return S;
}

size_t nn_knn_scratch_bytes(int64_t nq, int64_t n, int32_t k) {
    const int64_t S = pick_splits(nq, n);
    return (size_t)S * (size_t)nq * (size_t)k * (sizeof(double) + sizeof(int32_t)) + 256;
}

template <int D>
static void launch_knn_d(const NNWork &w, int32_t k, dim3 grid, int64_t chunk, double *pd2, int32_t *pid,
                         hipStream_t stream) {
    if (k == 1)
        hipLaunchKernelGGL((k_knn1<D>), grid, dim3(kNNBlock), 0, stream, w.pts, w.removed, w.n, w.d, w.q, w.nq,
                           chunk, w.n_dev, pd2, pid);
    else if (k <= 16)
        hipLaunchKernelGGL((k_knnk<D, 16>), grid, dim3(kNNBlock), 0, stream, w.pts, w.removed, w.n, w.d, w.q,
                           w.nq, chunk, w.n_dev, k, pd2, pid);
    else
        hipLaunchKernelGGL((k_knnk<D, 32>), grid, dim3(kNNBlock), 0, stream, w.pts, w.removed, w.n, w.d, w.q,
                           w.nq, chunk, w.n_dev, k, pd2, pid);
}

void launch_knn(const NNWork &w, int32_t k, int32_t *ids, double *d2, void *scratch, hipStream_t stream) {
    if (w.nq <= 0) return;
    const int64_t S = pick_splits(w.nq, w.n > 0 ? w.n : 1);
    const int64_t chunk = (w.n + S - 1) / S;
    double *pd2 = reinterpret_cast<double *>(scratch);
    int32_t *pid = reinterpret_cast<int32_t *>(pd2 + S * w.nq * k);
    const dim3 grid((unsigned)((w.nq + kNNBlock - 1) / kNNBlock), (unsigned)S);
    switch (w.d) {
        case 3: launch_knn_d<3>(w, k, grid, chunk, pd2, pid, stream); break;
        case 7: launch_knn_d<7>(w, k, grid, chunk, pd2, pid, stream); break;
        case 15: launch_knn_d<15>(w, k, grid, chunk, pd2, pid, stream); break;
        default: launch_knn_d<0>(w, k, grid, chunk, pd2, pid, stream); break;
    }
    hip_check(hipGetLastError(), "k_knn launch");
    hipLaunchKernelGGL(k_knn_merge, dim3((unsigned)((w.nq + 255) / 256)), dim3(256), 0, stream, pd2, pid, S,
                       w.nq, k, ids, d2);
    hip_check(hipGetLastError(), "k_knn_merge launch");
}

// ---------------- radius ----------------
__global__ __launch_bounds__(kNNBlock) void k_radius_count(const double *__restrict__ pts,
                                                           const uint8_t *__restrict__ removed, int64_t n,
                                                           int32_t d, const double *__restrict__ q,
                                                           int64_t nq, int64_t chunk, double r2,
                                                           int32_t *__restrict__ counts) {
    const int64_t qi = (int64_t)blockIdx.x * kNNBlock + threadIdx.x;
    const int64_t s = blockIdx.y;
    const int64_t beg = s * chunk;
    const int64_t end = beg + chunk < n ? beg + chunk : n;
    double qq[16];
    const int64_t qs = qi < nq ? qi : nq - 1;
    for (int i = 0; i < d; ++i) qq[i] = q[qs * d + i];
    int32_t c = 0;
    for (int64_t j = beg; j < end; ++j) {
        if (removed && removed[j]) continue;
        if (flann_l2_dyn(qq, pts + j * d, d) < r2) ++c;
    }
    if (qi < nq) counts[s * nq + qi] = c;
}

__global__ __launch_bounds__(kNNBlock) void k_radius_fill(const double *__restrict__ pts,
                                                          const uint8_t *__restrict__ removed, int64_t n,
                                                          int32_t d, const double *__restrict__ q,
                                                          int64_t nq, int64_t chunk, double r2,
                                                          const int64_t *__restrict__ soff,
                                                          int32_t *__restrict__ fid, double *__restrict__ fd2) {
    const int64_t qi = (int64_t)blockIdx.x * kNNBlock + threadIdx.x;
    const int64_t s = blockIdx.y;
    const int64_t beg = s * chunk;
    const int64_t end = beg + chunk < n ? beg + chunk : n;
    double qq[16];
    const int64_t qs = qi < nq ? qi : nq - 1;
    for (int i = 0; i < d; ++i) qq[i] = q[qs * d + i];
    if (qi >= nq) return;
    int64_t o = soff[s * nq + qi];
    for (int64_t j = beg; j < end; ++j) {
        if (removed && removed[j]) continue;
        const double dd = flann_l2_dyn(qq, pts + j * d, d);
        if (dd < r2) { fid[o] = (int32_t)(j + 1); fd2[o] = dd; ++o; }
    }
}

// Per query: sort its full segment by (d2, id), write the first min(count, max_nb).
__global__ void k_radius_sort(const int64_t *__restrict__ foff, const int64_t *__restrict__ ooff, int64_t nq,
                              int32_t *__restrict__ fid, double *__restrict__ fd2, int32_t *__restrict__ ids,
                              double *__restrict__ d2, int64_t cap) {
    const int64_t qi = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (qi >= nq) return;
    const int64_t b = foff[qi], e = foff[qi + 1];
    for (int64_t i = b + 1; i < e; ++i) {  // insertion sort (segments are short)
        const double kd = fd2[i];
        const int32_t ki = fid[i];
        int64_t j = i - 1;
        while (j >= b && nn_better(kd, ki, fd2[j], fid[j])) {
            fd2[j + 1] = fd2[j];
            fid[j + 1] = fid[j];
            --j;
        }
        fd2[j + 1] = kd;
        fid[j + 1] = ki;
    }
    const int64_t ob = ooff[qi], oe = ooff[qi + 1];
    for (int64_t i = 0; i < oe - ob; ++i)
        if (ob + i < cap) { ids[ob + i] = fid[b + i]; d2[ob + i] = fd2[b + i]; }
}

// Device allocations freed at scope exit (radius search only: it is synchronous).
struct TmpAllocs {
    std::vector<void *> p;
    ~TmpAllocs() {
        for (void *x : p) (void)hipFree(x);
    }
    template <class T>
    T *alloc(size_t n) {
        void *x = nullptr;
        hip_check(hipMalloc(&x, sizeof(T) * (n > 0 ? n : 1)), "radius alloc");
        p.push_back(x);
        return (T *)x;
    }
};

int64_t launch_radius(const NNWork &w, double r2, int32_t max_nb, int64_t *d_offsets, int32_t *d_ids,
                      double *d_d2, int64_t cap, void *scratch, size_t scratch_bytes, hipStream_t stream) {
    // Synchronous by contract (list sizes are data dependent): plain allocations and
    // blocking copies, so no pageable host staging outlives a copy.
    if (w.d > 16) throw Error{1, "radius search supports d <= 16"};
    const int64_t nq = w.nq;
    std::vector<int64_t> h_off(nq + 1, 0);
    hip_check(hipStreamSynchronize(stream), "radius sync");
    if (nq <= 0) {
        hip_check(hipMemcpy(d_offsets, h_off.data(), sizeof(int64_t), hipMemcpyHostToDevice), "radius offsets");
        return 0;
    }
    const int64_t S = pick_splits(nq, w.n > 0 ? w.n : 1);
    const int64_t chunk = (w.n + S - 1) / S;
    const dim3 grid((unsigned)((nq + kNNBlock - 1) / kNNBlock), (unsigned)S);
    TmpAllocs tmp;
    int32_t *counts = tmp.alloc<int32_t>(S * nq);
    hipLaunchKernelGGL(k_radius_count, grid, dim3(kNNBlock), 0, stream, w.pts, w.removed, w.n, w.d, w.q, nq,
                       chunk, r2, counts);
    hip_check(hipGetLastError(), "k_radius_count");
    hip_check(hipStreamSynchronize(stream), "radius sync");
    std::vector<int32_t> h_counts(S * nq);
    hip_check(hipMemcpy(h_counts.data(), counts, sizeof(int32_t) * S * nq, hipMemcpyDeviceToHost), "counts D2H");
    std::vector<int64_t> soff(S * nq), foff(nq + 1);
    int64_t tot = 0;
    for (int64_t qi = 0; qi < nq; ++qi) {
        foff[qi] = tot;
        for (int64_t s = 0; s < S; ++s) {
            soff[s * nq + qi] = tot;
            tot += h_counts[s * nq + qi];
        }
        const int64_t full = tot - foff[qi];
        const int64_t kept = (max_nb > 0 && full > max_nb) ? max_nb : full;
        h_off[qi + 1] = h_off[qi] + kept;
    }
    foff[nq] = tot;
    int64_t *d_soff = tmp.alloc<int64_t>(S * nq);
    int64_t *d_foff = tmp.alloc<int64_t>(nq + 1);
    int32_t *fid = tmp.alloc<int32_t>(tot + 1);
    double *fd2 = tmp.alloc<double>(tot + 1);
    hip_check(hipMemcpy(d_soff, soff.data(), sizeof(int64_t) * S * nq, hipMemcpyHostToDevice), "soff");
    hip_check(hipMemcpy(d_foff, foff.data(), sizeof(int64_t) * (nq + 1), hipMemcpyHostToDevice), "foff");
    hip_check(hipMemcpy(d_offsets, h_off.data(), sizeof(int64_t) * (nq + 1), hipMemcpyHostToDevice), "offsets");
    hipLaunchKernelGGL(k_radius_fill, grid, dim3(kNNBlock), 0, stream, w.pts, w.removed, w.n, w.d, w.q, nq, chunk,
                       r2, d_soff, fid, fd2);
    hip_check(hipGetLastError(), "k_radius_fill");
    hipLaunchKernelGGL(k_radius_sort, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, stream, d_foff, d_offsets,
                       nq, fid, fd2, d_ids, d_d2, cap);
    hip_check(hipGetLastError(), "k_radius_sort");
    hip_check(hipStreamSynchronize(stream), "radius sync");
    (void)scratch;
    (void)scratch_bytes;
    return h_off[nq];
}

}  // namespace mpt
