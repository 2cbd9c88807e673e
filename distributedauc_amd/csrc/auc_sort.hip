// Exact AUC by sorting: LSD radix sort of the negatives' order-preserving keys,
// then two binary searches per positive. O(N + P log N) work instead of the
// pair count's O(P*N); the counts are the same integers (W, T).
//
// Reference: imagenet/main.py:79-81 -> sklearn roc_curve/auc, whose
// _binary_clf_curve (sklearn/metrics/_ranking.py:826-908) also sorts the scores
// (a stable mergesort on the CPU, :886). SURVEY §8f row 1.
//
// Keys: an fp32 score maps to a uint32 that orders like the float, with -0 and
// +0 on one key (fp32 equality semantics): k = bits ^ (sign ? 0xffffffff : 0x80000000).
//
// Sort (per 8-bit digit, 4 passes, keys only):
//   hist    : one block per 4096-key tile, 256-bin LDS histogram -> hist[digit][tile]
//   scan    : exclusive scan over the digit-major hist array (decoupled 3-step scan)
//   scatter : each tile re-reads its keys in 16 chunks of 256; a key's rank among the
//             tile's keys with the same digit comes from 8 wave ballots (wave multisplit)
//             plus per-digit wave/chunk offsets in LDS, so the scatter is STABLE (LSD
//             correctness needs it); writes to out[offset[digit][tile] + rank].
// Search: each thread takes one positive key, lower_bound / upper_bound over the sorted
//   negatives; W += lb, T += ub - lb, reduced per block, one 64-bit atomic per block.

#include "dauc_internal.h"

namespace dauc {
namespace {

constexpr int kSortThreads = 256;
constexpr int kPerThread = 16;
constexpr int kTile = kSortThreads * kPerThread;  // 4096 keys
constexpr int kRadix = 256;
constexpr int kScanBlock = 1024;

__device__ __forceinline__ unsigned key_of(float f) {
    if (f == 0.0f) f = 0.0f;  // -0 -> +0
    const unsigned u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

int64_t tiles_for(int64_t n) { return (n + kTile - 1) / kTile; }

// ---- pass kernels -------------------------------------------------------------------

// FROM_FLOAT: the first pass reads fp32 scores and converts them to keys on the fly.
template <bool FROM_FLOAT>
__global__ __launch_bounds__(kSortThreads) void radix_hist_kernel(const void* __restrict__ in, int64_t n,
                                                                  int shift, unsigned* __restrict__ hist,
                                                                  int64_t ntiles) {
    __shared__ unsigned h[kRadix];
    h[threadIdx.x] = 0;
    __syncthreads();
    const int64_t t0 = int64_t(blockIdx.x) * kTile;
    for (int k = 0; k < kPerThread; ++k) {
        const int64_t i = t0 + int64_t(k) * kSortThreads + threadIdx.x;
        if (i < n) {
            const unsigned key = FROM_FLOAT ? key_of(static_cast<const float*>(in)[i])
                                            : static_cast<const unsigned*>(in)[i];
            atomicAdd(&h[(key >> shift) & 0xffu], 1u);
        }
    }
    __syncthreads();
    hist[int64_t(threadIdx.x) * ntiles + blockIdx.x] = h[threadIdx.x];  // digit-major
}

// exclusive scan of m counts, in place: 3 steps (block sums, scan of block sums, add back)
__global__ __launch_bounds__(kScanBlock) void scan_blocks_kernel(unsigned* __restrict__ a, int64_t m,
                                                                 unsigned* __restrict__ block_sums) {
    __shared__ unsigned s[kScanBlock];
    const int64_t i = int64_t(blockIdx.x) * kScanBlock + threadIdx.x;
    const unsigned v = i < m ? a[i] : 0u;
    s[threadIdx.x] = v;
    __syncthreads();
    for (int d = 1; d < kScanBlock; d <<= 1) {
        const unsigned t = threadIdx.x >= d ? s[threadIdx.x - d] : 0u;
        __syncthreads();
        s[threadIdx.x] += t;
        __syncthreads();
    }
    if (i < m) a[i] = s[threadIdx.x] - v;  // exclusive within the block
    if (threadIdx.x == kScanBlock - 1) block_sums[blockIdx.x] = s[threadIdx.x];
}

__global__ __launch_bounds__(kScanBlock) void scan_sums_kernel(unsigned* __restrict__ sums, int64_t nb) {
    // one block: exclusive scan of nb block sums (nb <= kScanBlock * per-thread run)
    __shared__ unsigned s[kScanBlock];
    const int64_t per = (nb + kScanBlock - 1) / kScanBlock;
    const int64_t b0 = int64_t(threadIdx.x) * per;
    const int64_t b1 = (b0 + per < nb) ? b0 + per : nb;
    unsigned local = 0;
    for (int64_t b = b0; b < b1; ++b) local += sums[b];
    s[threadIdx.x] = local;
    __syncthreads();
    for (int d = 1; d < kScanBlock; d <<= 1) {
        const unsigned t = threadIdx.x >= d ? s[threadIdx.x - d] : 0u;
        __syncthreads();
        s[threadIdx.x] += t;
        __syncthreads();
    }
    unsigned run = s[threadIdx.x] - local;
    for (int64_t b = b0; b < b1; ++b) {
        const unsigned v = sums[b];
        sums[b] = run;
        run += v;
    }
}

__global__ __launch_bounds__(kScanBlock) void scan_add_kernel(unsigned* __restrict__ a, int64_t m,
                                                              const unsigned* __restrict__ sums) {
    const int64_t i = int64_t(blockIdx.x) * kScanBlock + threadIdx.x;
    if (i < m) a[i] += sums[blockIdx.x];
}

template <bool FROM_FLOAT>
__global__ __launch_bounds__(kSortThreads) void radix_scatter_kernel(const void* __restrict__ in, int64_t n,
                                                                     int shift,
                                                                     const unsigned* __restrict__ offs,
                                                                     int64_t ntiles,
                                                                     unsigned* __restrict__ out) {
    __shared__ unsigned base[kRadix];                       // running output position per digit
    __shared__ unsigned wcnt[kSortThreads / kWave][kRadix];  // per-wave digit counts of a chunk
    const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
    base[threadIdx.x] = offs[int64_t(threadIdx.x) * ntiles + blockIdx.x];
    const unsigned long long lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    const int64_t t0 = int64_t(blockIdx.x) * kTile;
    for (int k = 0; k < kPerThread; ++k) {
        const int64_t i = t0 + int64_t(k) * kSortThreads + threadIdx.x;
        const bool valid = i < n;
        unsigned key = 0;
        if (valid)
            key = FROM_FLOAT ? key_of(static_cast<const float*>(in)[i]) : static_cast<const unsigned*>(in)[i];
        const unsigned d = (key >> shift) & 0xffu;
        // lanes of this wave holding the same digit (wave multisplit)
        unsigned long long same = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const unsigned long long m = __ballot((d >> b) & 1u);
            same &= ((d >> b) & 1u) ? m : ~m;
        }
        // clear this chunk's wave counts, then publish each digit's count from its first lane
#pragma unroll
        for (int w = 0; w < kSortThreads / kWave; ++w) wcnt[w][threadIdx.x] = 0;
        __syncthreads();
        const unsigned rank_in_wave = __popcll(same & lt);
        if (valid && rank_in_wave == 0) wcnt[wid][d] = __popcll(same);
        __syncthreads();
        if (valid) {
            unsigned before = 0;
            for (int w = 0; w < wid; ++w) before += wcnt[w][d];
            out[base[d] + before + rank_in_wave] = key;
        }
        __syncthreads();
        // advance the running base of every digit by this chunk's count
        unsigned tot = 0;
#pragma unroll
        for (int w = 0; w < kSortThreads / kWave; ++w) tot += wcnt[w][threadIdx.x];
        base[threadIdx.x] += tot;
        __syncthreads();
    }
}

// ---- search ---------------------------------------------------------------------------

__device__ __forceinline__ int64_t lower_bound_u32(const unsigned* __restrict__ a, int64_t n, unsigned k) {
    int64_t lo = 0, len = n;
    while (len > 0) {
        const int64_t half = len >> 1;
        if (a[lo + half] < k) {
            lo += half + 1;
            len -= half + 1;
        } else {
            len = half;
        }
    }
    return lo;
}

__device__ __forceinline__ int64_t upper_bound_u32(const unsigned* __restrict__ a, int64_t n, unsigned k) {
    int64_t lo = 0, len = n;
    while (len > 0) {
        const int64_t half = len >> 1;
        if (a[lo + half] <= k) {
            lo += half + 1;
            len -= half + 1;
        } else {
            len = half;
        }
    }
    return lo;
}

__global__ __launch_bounds__(kSortThreads) void search_count_kernel(const float* __restrict__ pos, int64_t P,
                                                                    const unsigned* __restrict__ sorted,
                                                                    int64_t N,
                                                                    unsigned long long* __restrict__ out) {
    __shared__ unsigned long long red[2][kSortThreads / kWave];
    unsigned long long w = 0, t = 0;
    for (int64_t i = int64_t(blockIdx.x) * kSortThreads + threadIdx.x; i < P;
         i += int64_t(gridDim.x) * kSortThreads) {
        const unsigned k = key_of(pos[i]);
        const int64_t lb = lower_bound_u32(sorted, N, k);
        // ties: the run of equal keys starts at lb; search only the tail
        const int64_t ub = lb + upper_bound_u32(sorted + lb, N - lb, k);
        w += static_cast<unsigned long long>(lb);
        t += static_cast<unsigned long long>(ub - lb);
    }
    w = wave_sum(w);
    t = wave_sum(t);
    const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
    if (lane == 0) {
        red[0][wid] = w;
        red[1][wid] = t;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long bw = 0, bt = 0;
        for (int i = 0; i < kSortThreads / kWave; ++i) {
            bw += red[0][i];
            bt += red[1][i];
        }
        if (bw) atomicAdd(out + 0, bw);
        if (bt) atomicAdd(out + 1, bt);
    }
}

struct SortWs {
    unsigned* keys_a;
    unsigned* keys_b;
    unsigned* hist;
    unsigned* sums;
    int64_t ntiles, m, nsum;
};

SortWs carve(void* ws, int64_t n) {
    SortWs w;
    w.ntiles = tiles_for(n);
    w.m = int64_t(kRadix) * w.ntiles;
    w.nsum = (w.m + kScanBlock - 1) / kScanBlock;
    auto* p = static_cast<unsigned char*>(ws);
    auto take = [&](int64_t count) {
        unsigned* r = reinterpret_cast<unsigned*>(p);
        p += ((count * 4 + 255) / 256) * 256;
        return r;
    };
    w.keys_a = take(n);
    w.keys_b = take(n);
    w.hist = take(w.m);
    w.sums = take(w.nsum);
    return w;
}

size_t sort_ws_bytes(int64_t n) {
    const int64_t nt = tiles_for(n), m = int64_t(kRadix) * nt, ns = (m + kScanBlock - 1) / kScanBlock;
    auto rnd = [](int64_t c) { return ((c * 4 + 255) / 256) * 256; };
    return static_cast<size_t>(rnd(n) * 2 + rnd(m) + rnd(ns));
}

// Sorts the keys of neg[0..N) into the workspace; returns the sorted array.
int radix_sort_keys(const float* neg, int64_t N, const SortWs& w, hipStream_t st, const unsigned** sorted) {
    const unsigned* src = nullptr;
    unsigned* dst = w.keys_a;
    for (int pass = 0; pass < 4; ++pass) {
        const int shift = 8 * pass;
        if (pass == 0)
            hipLaunchKernelGGL(radix_hist_kernel<true>, dim3(w.ntiles), dim3(kSortThreads), 0, st,
                               static_cast<const void*>(neg), N, shift, w.hist, w.ntiles);
        else
            hipLaunchKernelGGL(radix_hist_kernel<false>, dim3(w.ntiles), dim3(kSortThreads), 0, st,
                               static_cast<const void*>(src), N, shift, w.hist, w.ntiles);
        hipLaunchKernelGGL(scan_blocks_kernel, dim3(w.nsum), dim3(kScanBlock), 0, st, w.hist, w.m, w.sums);
        hipLaunchKernelGGL(scan_sums_kernel, dim3(1), dim3(kScanBlock), 0, st, w.sums, w.nsum);
        hipLaunchKernelGGL(scan_add_kernel, dim3(w.nsum), dim3(kScanBlock), 0, st, w.hist, w.m, w.sums);
        if (pass == 0)
            hipLaunchKernelGGL(radix_scatter_kernel<true>, dim3(w.ntiles), dim3(kSortThreads), 0, st,
                               static_cast<const void*>(neg), N, shift, w.hist, w.ntiles, dst);
        else
            hipLaunchKernelGGL(radix_scatter_kernel<false>, dim3(w.ntiles), dim3(kSortThreads), 0, st,
                               static_cast<const void*>(src), N, shift, w.hist, w.ntiles, dst);
        const int rc = launch_status();
        if (rc) return rc;
        src = dst;
        dst = (dst == w.keys_a) ? w.keys_b : w.keys_a;
    }
    *sorted = src;
    return DAUC_OK;
}

}  // namespace
}  // namespace dauc

using namespace dauc;

extern "C" {

size_t dauc_sort_workspace_size(int64_t N) { return sort_ws_bytes(N < 1 ? 1 : N); }

int dauc_sort_keys(const float* scores, int64_t n, unsigned* keys_out, void* workspace,
                   size_t workspace_bytes, dauc_stream_t stream) {
    if (n <= 0 || scores == nullptr || keys_out == nullptr || workspace == nullptr ||
        workspace_bytes < sort_ws_bytes(n) || n > 0xffffffffLL)
        return DAUC_EINVAL;
    SortWs w = carve(workspace, n);
    const unsigned* sorted = nullptr;
    hipStream_t st = as_hip(stream);
    int rc = radix_sort_keys(scores, n, w, st, &sorted);
    if (rc) return rc;
    return -static_cast<int>(hipMemcpyAsync(keys_out, sorted, size_t(n) * 4, hipMemcpyDeviceToDevice, st));
}

int dauc_auc_counts_sorted(const float* pos, int64_t P, const float* neg, int64_t N,
                           unsigned long long* wins_ties, void* workspace, size_t workspace_bytes,
                           dauc_stream_t stream) {
    if (P < 0 || N < 0 || wins_ties == nullptr || (P > 0 && pos == nullptr) ||
        (N > 0 && neg == nullptr))
        return DAUC_EINVAL;
    if (P == 0 || N == 0) return DAUC_OK;
    if (workspace == nullptr || workspace_bytes < sort_ws_bytes(N) || N > 0xffffffffLL) return DAUC_EINVAL;
    hipStream_t st = as_hip(stream);
    SortWs w = carve(workspace, N);
    const unsigned* sorted = nullptr;
    int rc = radix_sort_keys(neg, N, w, st, &sorted);
    if (rc) return rc;
    int64_t grid = (P + kSortThreads - 1) / kSortThreads;
    if (grid > 4096) grid = 4096;
    hipLaunchKernelGGL(search_count_kernel, dim3(grid), dim3(kSortThreads), 0, st, pos, P, sorted, N,
                       wins_ties);
    return launch_status();
}

}  // extern "C"
