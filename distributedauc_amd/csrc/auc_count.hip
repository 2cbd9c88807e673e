// Exact AUC: stable positive/negative split and the LDS-tiled pairwise count.
//
// Reference: imagenet/main.py:79-81 (AUC = sklearn roc_curve + auc, pos_label=1)
// and sklearn/metrics/_ranking.py:826-908 (_binary_clf_curve). sklearn's area
// is (2W + T) / (2PN) with W = #{pos > neg}, T = #{pos == neg}; this file
// computes W and T as exact integers, with no sort and no host round trip.
//
// Pair count: the kernel is VALU compare-issue bound, not HBM bound. Each
// workgroup keeps 256*RP positives in registers (RP per lane) and streams a
// slice of the negatives through LDS in 8 KB tiles; every lane compares its
// RP positives against each staged negative, which all 64 lanes read from one
// LDS address (a broadcast, conflict-free ds_read_b128). Out-of-range slots are
// NaN-padded: ordered compares with NaN are false, so padding counts nothing
// and the inner loop has no bounds checks.

#include <math.h>

#include "dauc_internal.h"

namespace dauc {
namespace {

// ============================ stable split ====================================

constexpr int kSplitThreads = 256;
constexpr int kSplitPerThread = 16;
constexpr int kSplitTile = kSplitThreads * kSplitPerThread;  // 4096 scores per block
constexpr int kScanThreads = 1024;

int64_t split_blocks(int64_t n) { return (n + kSplitTile - 1) / kSplitTile; }

template <typename LT>
__device__ __forceinline__ bool is_pos(const LT* __restrict__ lab, int64_t i) {
    return lab[i] == LT(1);
}

// pass 1: per-block positive count, non-finite scores, labels outside {-1, 1}
template <typename LT>
__global__ __launch_bounds__(kSplitThreads) void split_count_kernel(
    const float* __restrict__ s, const LT* __restrict__ lab, int64_t n, int* __restrict__ blk) {
    __shared__ int part[3][kSplitThreads / kWave];
    const int64_t base = int64_t(blockIdx.x) * kSplitTile;
    int np = 0, nf = 0, no = 0;
    for (int k = 0; k < kSplitPerThread; ++k) {
        const int64_t i = base + int64_t(k) * kSplitThreads + threadIdx.x;
        if (i < n) {
            const LT l = lab[i];
            np += (l == LT(1));
            no += (l != LT(1) && l != LT(-1));
            nf += !isfinite(s[i]);
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        np += __shfl_xor(np, off, kWave);
        nf += __shfl_xor(nf, off, kWave);
        no += __shfl_xor(no, off, kWave);
    }
    const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
    if (lane == 0) {
        part[0][wid] = np;
        part[1][wid] = nf;
        part[2][wid] = no;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int t0 = 0, t1 = 0, t2 = 0;
        for (int w = 0; w < kSplitThreads / kWave; ++w) {
            t0 += part[0][w];
            t1 += part[1][w];
            t2 += part[2][w];
        }
        blk[3 * blockIdx.x + 0] = t0;
        blk[3 * blockIdx.x + 1] = t1;
        blk[3 * blockIdx.x + 2] = t2;
    }
}

// pass 2 (one block): exclusive scan of the per-block positive counts
__global__ __launch_bounds__(kScanThreads) void split_scan_kernel(const int* __restrict__ blk,
                                                                  int64_t nblk, int64_t n,
                                                                  int64_t* __restrict__ pos_base,
                                                                  int64_t* __restrict__ stats) {
    __shared__ int64_t sums[kScanThreads];
    __shared__ int64_t other[2][kScanThreads / kWave];
    const int64_t per = (nblk + kScanThreads - 1) / kScanThreads;
    const int64_t b0 = int64_t(threadIdx.x) * per;
    const int64_t b1 = (b0 + per < nblk) ? b0 + per : nblk;
    int64_t local = 0, nf = 0, no = 0;
    for (int64_t b = b0; b < b1; ++b) {
        local += blk[3 * b];
        nf += blk[3 * b + 1];
        no += blk[3 * b + 2];
    }
    sums[threadIdx.x] = local;
    for (int off = 32; off > 0; off >>= 1) {
        nf += __shfl_xor(nf, off, kWave);
        no += __shfl_xor(no, off, kWave);
    }
    if ((threadIdx.x & (kWave - 1)) == 0) {
        other[0][threadIdx.x / kWave] = nf;
        other[1][threadIdx.x / kWave] = no;
    }
    __syncthreads();
    // Hillis-Steele inclusive scan over the 1024 thread sums
    for (int d = 1; d < kScanThreads; d <<= 1) {
        const int64_t v = threadIdx.x >= d ? sums[threadIdx.x - d] : 0;
        __syncthreads();
        sums[threadIdx.x] += v;
        __syncthreads();
    }
    int64_t run = sums[threadIdx.x] - local;  // exclusive prefix
    for (int64_t b = b0; b < b1; ++b) {
        pos_base[b] = run;
        run += blk[3 * b];
    }
    if (threadIdx.x == 0) {
        const int64_t P = sums[kScanThreads - 1];
        int64_t tf = 0, to = 0;
        for (int w = 0; w < kScanThreads / kWave; ++w) {
            tf += other[0][w];
            to += other[1][w];
        }
        stats[0] = P;
        stats[1] = n - P;
        stats[2] = tf;
        stats[3] = to;
    }
}

// pass 3: order-preserving scatter, 256 scores at a time per block
template <typename LT>
__global__ __launch_bounds__(kSplitThreads) void split_write_kernel(
    const float* __restrict__ s, const LT* __restrict__ lab, int64_t n,
    const int64_t* __restrict__ pos_base, float* __restrict__ pos_out,
    float* __restrict__ neg_out) {
    __shared__ int wave_cnt[kSplitThreads / kWave];
    const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
    const int64_t tile0 = int64_t(blockIdx.x) * kSplitTile;
    const int64_t pbase = pos_base[blockIdx.x];
    const int64_t nbase = tile0 - pbase;
    const unsigned long long lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    int64_t run_pos = 0;  // positives already written by this block
    for (int k = 0; k < kSplitPerThread; ++k) {
        const int64_t t = int64_t(k) * kSplitThreads + threadIdx.x;  // index inside the tile
        const int64_t i = tile0 + t;
        const bool valid = i < n;
        const bool p = valid && is_pos(lab, i);
        const unsigned long long m = __ballot(p);
        if (lane == 0) wave_cnt[wid] = __popcll(m);
        __syncthreads();
        int before = 0, chunk = 0;
        for (int w = 0; w < kSplitThreads / kWave; ++w) {
            const int c = wave_cnt[w];
            before += (w < wid) ? c : 0;
            chunk += c;
        }
        const int64_t pos_rank = run_pos + before + __popcll(m & lt_mask);
        if (valid) {
            const float v = s[i];
            if (p) pos_out[pbase + pos_rank] = v;
            else neg_out[nbase + (t - pos_rank)] = v;
        }
        run_pos += chunk;
        __syncthreads();
    }
}

template <typename LT>
int launch_split(const float* s, const LT* lab, int64_t n, float* pos_out, float* neg_out,
                 int64_t* stats, void* ws, hipStream_t st) {
    const int64_t nblk = split_blocks(n);
    int64_t* pos_base = static_cast<int64_t*>(ws);
    int* blk = reinterpret_cast<int*>(pos_base + nblk);
    hipLaunchKernelGGL(split_count_kernel<LT>, dim3(nblk), dim3(kSplitThreads), 0, st, s, lab, n,
                       blk);
    int rc = launch_status();
    if (rc) return rc;
    hipLaunchKernelGGL(split_scan_kernel, dim3(1), dim3(kScanThreads), 0, st, blk, nblk, n,
                       pos_base, stats);
    rc = launch_status();
    if (rc) return rc;
    hipLaunchKernelGGL(split_write_kernel<LT>, dim3(nblk), dim3(kSplitThreads), 0, st, s, lab, n,
                       pos_base, pos_out, neg_out);
    return launch_status();
}

// ============================ pair count ======================================

constexpr int kPcThreads = 256;
constexpr int kNegTile = 2048;  // negatives per LDS tile (8 KB)
constexpr int64_t kTargetBlocks = 8192;

__device__ __forceinline__ float nan_f() { return __builtin_nanf(""); }

// MODE selects how a compare result is accumulated:
//   0: per-lane VGPR counters (v_cmp + v_cndmask/v_addc on the VALU)
//   1: wave ballot + popcount on the scalar unit (v_cmp -> SGPR mask, s_bcnt1, s_add)
//   2: mixed: '>' through the scalar unit, '>=' through VGPR counters
template <int RP, int MODE>
__global__ __launch_bounds__(kPcThreads) void pair_count_kernel(
    const float* __restrict__ pos, int64_t P, const float* __restrict__ neg, int64_t N,
    int64_t neg_per_block, int neg_aligned, unsigned long long* __restrict__ out) {
    __shared__ float4 tile[kNegTile / 4];
    __shared__ unsigned long long red[2][kPcThreads / kWave];

    float p[RP];
    const int64_t pb = int64_t(blockIdx.x) * (int64_t(kPcThreads) * RP);
#pragma unroll
    for (int r = 0; r < RP; ++r) {
        const int64_t i = pb + int64_t(r) * kPcThreads + threadIdx.x;
        p[r] = i < P ? pos[i] : nan_f();
    }
    unsigned gt[RP], ge[RP];
#pragma unroll
    for (int r = 0; r < RP; ++r) gt[r] = ge[r] = 0u;
    unsigned long long sgt = 0, sge = 0;  // wave-uniform counters (MODE 1, 2)

    const int64_t n0 = int64_t(blockIdx.y) * neg_per_block;
    const int64_t n1 = (n0 + neg_per_block < N) ? n0 + neg_per_block : N;
    for (int64_t t0 = n0; t0 < n1; t0 += kNegTile) {
#pragma unroll
        for (int k = 0; k < kNegTile / 4 / kPcThreads; ++k) {
            const int v = k * kPcThreads + threadIdx.x;
            const int64_t i = t0 + int64_t(v) * 4;
            float4 x;
            if (neg_aligned && i + 3 < n1) {
                x = *reinterpret_cast<const float4*>(neg + i);
            } else {
                x.x = i + 0 < n1 ? neg[i + 0] : nan_f();
                x.y = i + 1 < n1 ? neg[i + 1] : nan_f();
                x.z = i + 2 < n1 ? neg[i + 2] : nan_f();
                x.w = i + 3 < n1 ? neg[i + 3] : nan_f();
            }
            tile[v] = x;
        }
        __syncthreads();
#pragma unroll 2
        for (int j = 0; j < kNegTile / 4; ++j) {
            const float4 q = tile[j];  // same address in every lane: LDS broadcast
#pragma unroll
            for (int r = 0; r < RP; ++r) {
                if constexpr (MODE == 0) {
                    gt[r] += (p[r] > q.x);
                    ge[r] += (p[r] >= q.x);
                    gt[r] += (p[r] > q.y);
                    ge[r] += (p[r] >= q.y);
                    gt[r] += (p[r] > q.z);
                    ge[r] += (p[r] >= q.z);
                    gt[r] += (p[r] > q.w);
                    ge[r] += (p[r] >= q.w);
                } else if constexpr (MODE == 1) {
                    sgt += __popcll(__ballot(p[r] > q.x)) + __popcll(__ballot(p[r] > q.y)) +
                           __popcll(__ballot(p[r] > q.z)) + __popcll(__ballot(p[r] > q.w));
                    sge += __popcll(__ballot(p[r] >= q.x)) + __popcll(__ballot(p[r] >= q.y)) +
                           __popcll(__ballot(p[r] >= q.z)) + __popcll(__ballot(p[r] >= q.w));
                } else {
                    sgt += __popcll(__ballot(p[r] > q.x)) + __popcll(__ballot(p[r] > q.y)) +
                           __popcll(__ballot(p[r] > q.z)) + __popcll(__ballot(p[r] > q.w));
                    ge[r] += (p[r] >= q.x);
                    ge[r] += (p[r] >= q.y);
                    ge[r] += (p[r] >= q.z);
                    ge[r] += (p[r] >= q.w);
                }
            }
        }
        __syncthreads();
    }

    const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
    unsigned long long tg = 0, te = 0;
#pragma unroll
    for (int r = 0; r < RP; ++r) {
        tg += gt[r];
        te += ge[r];
    }
    tg = wave_sum(tg);
    te = wave_sum(te);
    if (MODE >= 1) tg = sgt;  // already a per-wave total
    if (MODE == 1) te = sge;
    if (lane == 0) {
        red[0][wid] = tg;
        red[1][wid] = te;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long bg = 0, be = 0;
        for (int w = 0; w < kPcThreads / kWave; ++w) {
            bg += red[0][w];
            be += red[1][w];
        }
        if (bg) atomicAdd(out + 0, bg);
        if (be - bg) atomicAdd(out + 1, be - bg);
    }
}

}  // namespace
}  // namespace dauc

using namespace dauc;

extern "C" {

size_t dauc_split_workspace_size(int64_t n) {
    const int64_t nblk = split_blocks(n < 0 ? 0 : n);
    return static_cast<size_t>(nblk) * (sizeof(int64_t) + 3 * sizeof(int)) + 64;
}

int dauc_split_scores(const float* scores, const void* labels, int label_dtype, int64_t n,
                      float* pos_out, float* neg_out, int64_t* stats, void* workspace,
                      size_t workspace_bytes, dauc_stream_t stream) {
    if (n <= 0 || scores == nullptr || labels == nullptr || pos_out == nullptr ||
        neg_out == nullptr || stats == nullptr || workspace == nullptr ||
        workspace_bytes < dauc_split_workspace_size(n) ||
        (reinterpret_cast<uintptr_t>(workspace) & 7u))
        return DAUC_EINVAL;
    hipStream_t st = as_hip(stream);
    switch (label_dtype) {
        case DAUC_LABEL_I8:
            return launch_split(scores, static_cast<const int8_t*>(labels), n, pos_out, neg_out,
                                stats, workspace, st);
        case DAUC_LABEL_I32:
            return launch_split(scores, static_cast<const int32_t*>(labels), n, pos_out, neg_out,
                                stats, workspace, st);
        case DAUC_LABEL_I64:
            return launch_split(scores, static_cast<const int64_t*>(labels), n, pos_out, neg_out,
                                stats, workspace, st);
        default:
            return DAUC_EINVAL;
    }
}

int dauc_pair_count(const float* pos, int64_t P, const float* neg, int64_t N,
                    unsigned long long* wins_ties, dauc_stream_t stream) {
    return dauc_pair_count_variant(pos, P, neg, N, wins_ties, 0, stream);
}

int dauc_pair_count_variant(const float* pos, int64_t P, const float* neg, int64_t N,
                            unsigned long long* wins_ties, int variant, dauc_stream_t stream) {
    if (P < 0 || N < 0 || wins_ties == nullptr || (P > 0 && pos == nullptr) ||
        (N > 0 && neg == nullptr))
        return DAUC_EINVAL;
    if (P == 0 || N == 0) return DAUC_OK;
    // variant = mode + 3 * rp_index; mode: accumulation scheme, rp: positives per lane {8, 4, 16}
    if (variant < 0 || variant >= 9) return DAUC_EINVAL;
    const int mode = variant % 3;
    const int rp = variant / 3 == 0 ? 8 : (variant / 3 == 1 ? 4 : 16);
    const int64_t pos_per_block = int64_t(kPcThreads) * rp;
    const int64_t gx = (P + pos_per_block - 1) / pos_per_block;
    if (gx > 0x7fffffffLL) return DAUC_EINVAL;
    const int64_t tiles = (N + kNegTile - 1) / kNegTile;
    int64_t gy = (kTargetBlocks + gx - 1) / gx;
    if (gy > tiles) gy = tiles;
    // per-lane counters are 32-bit: keep each block's negative slice below 2^27 (x RP <= 16 per lane)
    const int64_t cap = int64_t(1) << 27;
    const int64_t min_gy = (N + cap - 1) / cap;
    if (gy < min_gy) gy = min_gy;
    if (gy > 65535) gy = 65535;
    int64_t per = (N + gy - 1) / gy;
    per = (per + kNegTile - 1) / kNegTile * kNegTile;
    gy = (N + per - 1) / per;
    if (per > cap + kNegTile) return DAUC_EINVAL;
    const int aligned = (reinterpret_cast<uintptr_t>(neg) & 15u) == 0;
    const dim3 grid(static_cast<unsigned>(gx), static_cast<unsigned>(gy));
    hipStream_t st = as_hip(stream);
#define DAUC_PC_LAUNCH(RPV, MV)                                                                    \
    hipLaunchKernelGGL((pair_count_kernel<RPV, MV>), grid, dim3(kPcThreads), 0, st, pos, P, neg, N, \
                       per, aligned, wins_ties)
    switch (variant) {
        case 0: DAUC_PC_LAUNCH(8, 0); break;
        case 1: DAUC_PC_LAUNCH(8, 1); break;
        case 2: DAUC_PC_LAUNCH(8, 2); break;
        case 3: DAUC_PC_LAUNCH(4, 0); break;
        case 4: DAUC_PC_LAUNCH(4, 1); break;
        case 5: DAUC_PC_LAUNCH(4, 2); break;
        case 6: DAUC_PC_LAUNCH(16, 0); break;
        case 7: DAUC_PC_LAUNCH(16, 1); break;
        case 8: DAUC_PC_LAUNCH(16, 2); break;
    }
#undef DAUC_PC_LAUNCH
    (void)mode;
    (void)rp;
    return launch_status();
}

}  // extern "C"
