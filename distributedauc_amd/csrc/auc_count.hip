// Exact AUC: stable positive/negative split and the LDS-tiled pairwise count.
//
// Reference: imagenet/main.py:79-81 (AUC = sklearn roc_curve + auc, pos_label=1)
// and sklearn/metrics/_ranking.py:826-908 (_binary_clf_curve). sklearn's area
// is (2W + T) / (2PN) with W = #{pos > neg}, T = #{pos == neg}; this file
// computes W and T as exact integers, with no sort and no host round trip.
//
// Pair count: the kernel is VALU-issue bound, not HBM bound. Each workgroup
// keeps 256*RP positives in registers (RP per lane) and streams a slice of the
// negatives through LDS in 8 KB tiles; every lane counts its RP positives
// against each staged negative, which all 64 lanes read from one LDS address
// (a broadcast, conflict-free ds_read_b128). The default counting step is a
// packed-fp32 difference + clamped fma (3 v_pk instructions per 2 pairs, see
// pk_clamp_fma); tiles holding infinities or tiny subnormal-range scores fall
// back to exact compares. Out-of-range slots are NaN-padded: ordered compares
// with NaN are false and clamp(NaN) = 0, so padding counts nothing and the
// inner loop has no bounds checks.

#include <math.h>

#include <type_traits>

#include "count_index.h"

namespace dauc {
namespace {

// ============================ stable split ====================================
//
// Tiles of 8192 scores per workgroup; a thread handles kSlots float4 slots, slot k of thread t
// covering scores tile0 + (k*256 + t)*4 + [0, 4) (every load instruction of a wave reads 1 KB
// contiguous). Tile order = k-major, then thread, then the 4 lanes of the float4.

constexpr int kSplitThreads = 256;
constexpr int kSlots = 8;
constexpr int kSplitTile = kSplitThreads * 4 * kSlots;  // 8192 scores per block
constexpr int kScanThreads = 1024;

int64_t split_blocks(int64_t n) { return (n + kSplitTile - 1) / kSplitTile; }

// label class of 4 consecutive scores: 1 (positive), -1 (negative), 2 (other), 0 (past n)
template <typename LT>
__device__ __forceinline__ void load_labels4(const LT* __restrict__ lab, int64_t i, int64_t n, bool full,
                                             int (&l)[4]) {
    if (full && sizeof(LT) == 1) {
        const char4 c = *reinterpret_cast<const char4*>(lab + i);
        const int r[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) l[q] = r[q] == 1 ? 1 : (r[q] == -1 ? -1 : 2);
    } else if (full && sizeof(LT) == 4) {
        const int4 c = *reinterpret_cast<const int4*>(lab + i);
        const int r[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) l[q] = r[q] == 1 ? 1 : (r[q] == -1 ? -1 : 2);
    } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (i + q < n) {
                const LT v = lab[i + q];
                l[q] = v == LT(1) ? 1 : (v == LT(-1) ? -1 : 2);
            } else {
                l[q] = 0;
            }
        }
    }
}

__device__ __forceinline__ void load_scores4(const float* __restrict__ s, int64_t i, int64_t n, bool full,
                                             float (&v)[4]) {
    if (full) {
        const f32x4 x = *reinterpret_cast<const f32x4*>(s + i);
        v[0] = x.x;
        v[1] = x.y;
        v[2] = x.z;
        v[3] = x.w;
    } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = i + q < n ? s[i + q] : 0.0f;
    }
}

// pass 1: per-block positive count, non-finite scores, labels outside {-1, 1}
template <typename LT>
__global__ __launch_bounds__(kSplitThreads) void split_count_kernel(
    const float* __restrict__ s, const LT* __restrict__ lab, int64_t n, int vec, int* __restrict__ blk) {
    __shared__ int part[3][kSplitThreads / kWave];
    const int64_t base = int64_t(blockIdx.x) * kSplitTile;
    int np = 0, nf = 0, no = 0;
    float v[kSlots][4];
    int l[kSlots][4];
#pragma unroll
    for (int k = 0; k < kSlots; ++k) {
        const int64_t i = base + (int64_t(k) * kSplitThreads + threadIdx.x) * 4;
        const bool full = vec && i + 4 <= n;
        load_scores4(s, i, n, full, v[k]);
        load_labels4(lab, i, n, full, l[k]);
    }
#pragma unroll
    for (int k = 0; k < kSlots; ++k) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            np += l[k][q] == 1;
            no += l[k][q] == 2;
            nf += l[k][q] != 0 && !isfinite(v[k][q]);
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

// pass 3: order-preserving scatter of one tile. Each wave ballots its positives per slot and
// float4 lane, one barrier publishes the per-(slot, wave) counts, and every score's rank among
// the tile's positives (a negative's: its tile position minus that rank) follows from the
// counts before it in tile order plus the ballot bits of the lower lanes.
template <typename LT>
__global__ __launch_bounds__(kSplitThreads) void split_write_kernel(
    const float* __restrict__ s, const LT* __restrict__ lab, int64_t n, int vec,
    const int64_t* __restrict__ pos_base, float* __restrict__ pos_out, float* __restrict__ neg_out) {
    constexpr int kW = kSplitThreads / kWave;
    __shared__ int cnt[kSlots * kW];
    const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
    const int64_t tile0 = int64_t(blockIdx.x) * kSplitTile;
    const int64_t pbase = pos_base[blockIdx.x];
    const int64_t nbase = tile0 - pbase;
    const unsigned long long lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    float v[kSlots][4];
    int l[kSlots][4];
#pragma unroll
    for (int k = 0; k < kSlots; ++k) {
        const int64_t i = tile0 + (int64_t(k) * kSplitThreads + threadIdx.x) * 4;
        const bool full = vec && i + 4 <= n;
        load_scores4(s, i, n, full, v[k]);
        load_labels4(lab, i, n, full, l[k]);
    }
    int below[kSlots];  // positives of this wave's lower lanes in slot k
#pragma unroll
    for (int k = 0; k < kSlots; ++k) {
        int tot = 0, low = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const unsigned long long m = __ballot(l[k][q] == 1);
            tot += __popcll(m);
            low += __popcll(m & lt_mask);
        }
        below[k] = low;
        if (lane == 0) cnt[k * kW + wid] = tot;
    }
    __syncthreads();
    int run = 0;  // positives of the tile before slot k
#pragma unroll
    for (int k = 0; k < kSlots; ++k) {
        int before = run;
#pragma unroll
        for (int w = 0; w < kW; ++w) {
            const int c = cnt[k * kW + w];
            before += w < wid ? c : 0;
            run += c;
        }
        int r = before + below[k];  // rank of this thread's first score of slot k
        const int64_t t = (int64_t(k) * kSplitThreads + threadIdx.x) * 4;  // position in the tile
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (l[k][q] == 1) {
                pos_out[pbase + r] = v[k][q];
                ++r;
            } else if (l[k][q] != 0 && neg_out != nullptr) {  // neg_out == NULL: positives only
                neg_out[nbase + (t + q - r)] = v[k][q];
            }
        }
    }
}

template <typename LT>
int launch_split(const float* s, const LT* lab, int64_t n, float* pos_out, float* neg_out,
                 int64_t* stats, void* ws, hipStream_t st) {
    const int64_t nblk = split_blocks(n);
    int64_t* pos_base = static_cast<int64_t*>(ws);
    int* blk = reinterpret_cast<int*>(pos_base + nblk);
    const int vec = (reinterpret_cast<uintptr_t>(s) & 15u) == 0 &&
                    (reinterpret_cast<uintptr_t>(lab) & (4 * sizeof(LT) - 1)) == 0;
    hipLaunchKernelGGL(split_count_kernel<LT>, dim3(nblk), dim3(kSplitThreads), 0, st, s, lab, n, vec,
                       blk);
    int rc = launch_status();
    if (rc) return rc;
    hipLaunchKernelGGL(split_scan_kernel, dim3(1), dim3(kScanThreads), 0, st, blk, nblk, n,
                       pos_base, stats);
    rc = launch_status();
    if (rc) return rc;
    hipLaunchKernelGGL(split_write_kernel<LT>, dim3(nblk), dim3(kSplitThreads), 0, st, s, lab, n, vec,
                       pos_base, pos_out, neg_out);
    return launch_status();
}

// ============================ positive compaction =============================
//
// The sort method only needs the positives as a table (every negative is read in place by the
// query kernel, which also checks it is finite), so this pass reads the LABELS of every score
// (1 B each at int8) and the SCORE of each positive only: at 2^27 scores with 0.1 % positives it
// moves 134 MB of labels instead of the stable split's 2 x 671 MB of scores + labels. The
// output keeps the original order (a stable compaction), so every rank that compacts the same
// vector gets the same list.
//
// Block tile: 256 threads x kCmpSlots groups of 16 labels; group k of thread t covers labels
// tile0 + (k * 256 + t) * 16 + [0, 16) (each wave load instruction reads 1 KB contiguous at int8).

constexpr int kCmpThreads = 256;
constexpr int kCmpSlots = 8;
constexpr int kCmpTile = kCmpThreads * 16 * kCmpSlots;  // 32768 labels per block

int64_t compact_blocks(int64_t n) { return (n + kCmpTile - 1) / kCmpTile; }

// per tile: positives, labels outside {-1, 1}
// then the positive bit masks of every tile (1 bit per label: 4 KB per 32768-label tile)
inline size_t compact_masks_offset(int64_t n) { return (64 + static_cast<size_t>(compact_blocks(n)) * 2 * sizeof(int) + 255) / 256 * 256; }
inline size_t compact_ws_bytes(int64_t n) { return compact_masks_offset(n) + static_cast<size_t>(compact_blocks(n)) * kCmpThreads * 16; }

// bytes == 0 -> 0x80 in that byte, 0 elsewhere (exact, no carries between bytes)
__device__ __forceinline__ unsigned zero_bytes(unsigned v) {
    return ~(((v & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | v | 0x7F7F7F7Fu);
}

// the 4 byte flags (0x80 per byte) of zero_bytes() as a 4-bit mask
__device__ __forceinline__ unsigned byte_flags4(unsigned f) { return (((f >> 7) * 0x00204081u) >> 21) & 0xFu; }

// 16 labels from i: bit j of pos = (label[i + j] == 1); nother += #labels not in {-1, 1}
template <typename LT>
__device__ __forceinline__ unsigned label_masks16(const LT* __restrict__ lab, int64_t i, int64_t n, bool vec,
                                                  int& nother) {
    unsigned pos = 0;
    if (vec && i + 16 <= n) {
        if constexpr (sizeof(LT) == 1) {
            const int4 v = *reinterpret_cast<const int4*>(lab + i);
            const unsigned w[4] = {unsigned(v.x), unsigned(v.y), unsigned(v.z), unsigned(v.w)};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const unsigned p = zero_bytes(w[q] ^ 0x01010101u), m = zero_bytes(~w[q]);
                pos |= byte_flags4(p) << (4 * q);
                nother += 4 - __popc(p | m);
            }
        } else {
#pragma unroll
            for (int q = 0; q < 16; q += 16 / sizeof(LT)) {
                LT c[16 / sizeof(LT)];
                *reinterpret_cast<int4*>(c) = *reinterpret_cast<const int4*>(lab + i + q);
#pragma unroll
                for (int j = 0; j < int(16 / sizeof(LT)); ++j) {
                    pos |= unsigned(c[j] == LT(1)) << (q + j);
                    nother += c[j] != LT(1) && c[j] != LT(-1);
                }
            }
        }
    } else {
        for (int j = 0; j < 16; ++j) {
            if (i + j < n) {
                const LT c = lab[i + j];
                pos |= unsigned(c == LT(1)) << j;
                nother += c != LT(1) && c != LT(-1);
            }
        }
    }
    return pos;
}

// the compactions load a tile's labels this many 16-B loads at a time (round 2's form, one group
// per bounds-checked branch, waited out one memory latency per group; 4 and 16 measured equal / slower)
constexpr int kCompactBatch = 8;

// the positive mask and the labels outside {-1, 1} of 16 labels already in registers (the bounds-
// and alignment-checked case of label_masks16)
template <typename LT>
__device__ __forceinline__ unsigned masks16_of(const int4 (&v)[sizeof(LT)], int& nother) {
    unsigned pos = 0;
    if constexpr (sizeof(LT) == 1) {
        const unsigned w[4] = {unsigned(v[0].x), unsigned(v[0].y), unsigned(v[0].z), unsigned(v[0].w)};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const unsigned p = zero_bytes(w[q] ^ 0x01010101u), m = zero_bytes(~w[q]);
            pos |= byte_flags4(p) << (4 * q);
            nother += 4 - __popc(p | m);
        }
    } else {
        constexpr int kPer = 16 / sizeof(LT);  // labels per int4
#pragma unroll
        for (int q = 0; q < int(sizeof(LT)); ++q) {
            LT c[kPer];
            *reinterpret_cast<int4*>(c) = v[q];
#pragma unroll
            for (int j = 0; j < kPer; ++j) {
                pos |= unsigned(c[j] == LT(1)) << (q * kPer + j);
                nother += c[j] != LT(1) && c[j] != LT(-1);
            }
        }
    }
    return pos;
}

// Two launches. (1) count: per tile, its positives and its labels outside {-1, 1}, and the
// positive bit masks (1 bit per label, one 16-B store per thread). (2) write: every tile first
// sums the positive counts of the tiles before it (its 256 threads read them strided from L2 and
// reduce: no scan launch, no inter-workgroup wait), then reads its masks — not the labels again:
// 1/8 of the bytes at int8 — and writes its positives' scores at that offset in tile order; the
// last tile also sums every tile's counts into stats[].
// A single-launch decoupled look-back was built and measured: with ~1 µs of work per tile and
// ~2 µs per cross-XCD round trip its prefix frontier advances one 64-tile window per round trip
// (2^27 labels: 298 µs against this form's count + write).
template <typename LT>
__global__ __launch_bounds__(kCmpThreads) void compact_count_kernel(const LT* __restrict__ lab, int64_t n,
                                                                    int vec, int* __restrict__ blk,
                                                                    uint4* __restrict__ masks,
                                                                    int64_t* __restrict__ stats,
                                                                    unsigned long long* __restrict__ zero3,
                                                                    unsigned* __restrict__ zero_w, int nzero_w) {
    static_assert(kCmpSlots == 8, "8 16-bit group masks = one uint4 per thread");
    __shared__ int part[2][kCmpThreads / kWave];
    const int64_t base = int64_t(blockIdx.x) * kCmpTile;
    if (blockIdx.x == 0 && threadIdx.x < 4) {
        if (threadIdx.x == 0) stats[2] = 0;  // the write pass adds the non-finite positives
        else if (zero3 != nullptr) zero3[threadIdx.x - 1] = 0;  // a later stage's counters (dauc_auc_eval_counts)
    }
    if (blockIdx.x == 0)  // a later stage's histogram (the eval's direct count-index build)
        for (int i = threadIdx.x; i < nzero_w; i += kCmpThreads) zero_w[i] = 0u;
    int np = 0, no = 0;
    unsigned m[kCmpSlots];
    if (vec && base + kCmpTile <= n) {
        // a tile wholly in range and aligned (uniform): every group's loads in straight-line code,
        // not one bounds-checked branch (and so one memory latency) per group
        constexpr int kPer = int(sizeof(LT));
        int4 v[kCmpSlots][kPer];
#pragma unroll
        for (int k = 0; k < kCmpSlots; ++k) {
            const int4* src = reinterpret_cast<const int4*>(lab + base + (int64_t(k) * kCmpThreads + threadIdx.x) * 16);
#pragma unroll
            for (int q = 0; q < kPer; ++q) v[k][q] = src[q];
        }
#pragma unroll
        for (int k = 0; k < kCmpSlots; ++k) m[k] = masks16_of<LT>(v[k], no);
    } else {
#pragma unroll
        for (int k = 0; k < kCmpSlots; ++k)
            m[k] = label_masks16(lab, base + (int64_t(k) * kCmpThreads + threadIdx.x) * 16, n, vec, no);
    }
#pragma unroll
    for (int k = 0; k < kCmpSlots; ++k) np += __popc(m[k]);
    masks[int64_t(blockIdx.x) * kCmpThreads + threadIdx.x] =
        uint4{m[0] | (m[1] << 16), m[2] | (m[3] << 16), m[4] | (m[5] << 16), m[6] | (m[7] << 16)};
    for (int off = 32; off > 0; off >>= 1) {
        np += __shfl_xor(np, off, kWave);
        no += __shfl_xor(no, off, kWave);
    }
    const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
    if (lane == 0) {
        part[0][wid] = np;
        part[1][wid] = no;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int t0 = 0, t1 = 0;
        for (int w = 0; w < kCmpThreads / kWave; ++w) {
            t0 += part[0][w];
            t1 += part[1][w];
        }
        blk[blockIdx.x] = t0;
        blk[gridDim.x + blockIdx.x] = t1;
    }
}

// sum of v[0..count) over the block (every thread gets it); count <= 2^31 entries of <= 2^15
__device__ __forceinline__ long long block_sum_ints(const int* __restrict__ v, int64_t count, long long* red) {
    long long acc = 0;
    int64_t i0 = 0;
    if ((reinterpret_cast<uintptr_t>(v) & 15u) == 0) {
        // int4 loads, 4 in flight per thread per round: 4096 counts in one round
        const int4* v4 = reinterpret_cast<const int4*>(v);
        const int64_t nv = count / 4;
        for (int64_t j = threadIdx.x; j < nv; j += 4 * kCmpThreads) {
            int4 q[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int64_t jj = j + u * kCmpThreads;
                q[u] = jj < nv ? v4[jj] : make_int4(0, 0, 0, 0);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) acc += (long long)q[u].x + q[u].y + q[u].z + q[u].w;
        }
        i0 = nv * 4;
    }
    for (int64_t i = i0 + threadIdx.x; i < count; i += kCmpThreads) acc += v[i];
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, kWave);
    const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
    if (lane == 0) red[wid] = acc;
    __syncthreads();
    long long t = 0;
#pragma unroll
    for (int w = 0; w < kCmpThreads / kWave; ++w) t += red[w];
    __syncthreads();
    return t;
}

// every positive's score goes to pos_out[(positives of earlier tiles) + its rank in the tile]; rank
// order = group k, then thread, then the 16 labels of the group (original order)
__global__ __launch_bounds__(kCmpThreads) void compact_write_kernel(
    const float* __restrict__ s, int64_t n, const int* __restrict__ blk, const uint4* __restrict__ masks,
    float* __restrict__ pos_out, int64_t* __restrict__ stats) {
    constexpr int kW = kCmpThreads / kWave;
    __shared__ int cnt[kCmpSlots][kW];
    __shared__ long long red[kW];
    const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
    const int64_t nblk = gridDim.x;
    const int64_t base = int64_t(blockIdx.x) * kCmpTile;
    const uint4 mq = masks[int64_t(blockIdx.x) * kCmpThreads + threadIdx.x];
    const unsigned m[kCmpSlots] = {mq.x & 0xffffu, mq.x >> 16, mq.y & 0xffffu, mq.y >> 16,
                                   mq.z & 0xffffu, mq.z >> 16, mq.w & 0xffffu, mq.w >> 16};
    const int64_t pbase = block_sum_ints(blk, blockIdx.x, red);
    int excl[kCmpSlots];
#pragma unroll
    for (int k = 0; k < kCmpSlots; ++k) {
        const int c = __popc(m[k]);
        int incl = c;  // inclusive scan over the wave's lanes
#pragma unroll
        for (int off = 1; off < kWave; off <<= 1) {
            const int v = __shfl_up(incl, off, kWave);
            if (lane >= off) incl += v;
        }
        excl[k] = incl - c;
        if (lane == kWave - 1) cnt[k][wid] = incl;
    }
    __syncthreads();
    int run = 0, nf = 0;
#pragma unroll
    for (int k = 0; k < kCmpSlots; ++k) {
        int before = run;
#pragma unroll
        for (int w = 0; w < kW; ++w) {
            const int c = cnt[k][w];
            before += w < wid ? c : 0;
            run += c;
        }
        int64_t r = pbase + before + excl[k];
        const int64_t i = base + (int64_t(k) * kCmpThreads + threadIdx.x) * 16;
        for (unsigned b = m[k]; b != 0u; b &= b - 1u) {
            const float v = s[i + __ffs(b) - 1];
            nf += !isfinite(v);
            pos_out[r++] = v;
        }
    }
    if (nf) atomicAdd(reinterpret_cast<unsigned long long*>(stats + 2), static_cast<unsigned long long>(nf));
    if (blockIdx.x == nblk - 1) {
        // P = the positives before this tile + its own; the other-label total over every tile
        const long long other = block_sum_ints(blk + nblk, nblk, red);
        if (threadIdx.x == 0) {
            stats[0] = pbase + run;
            stats[1] = n - (pbase + run);
            stats[3] = other;
        }
    }
}

// The one-call evaluation's compaction, in ONE pass and without order: the positives' scores are
// only ever counted against (the direct count-index build scatters them into cells by atomics
// anyway), so a tile reserves its range of pos_out with one returning atomic instead of waiting
// for the earlier tiles' counts (no mask pass, no second launch). stats[0] (positives, the
// reservation counter), stats[2] (non-finite positives) and stats[3] (labels outside {-1, 1})
// must be zero on entry; stats[1] is not written (N = n - P). Block 0 zeroes `zero_next` (the
// next call's stats) and zero3[0..3); the grid zeroes the first `nzero_w` words of `zero_w`.
// SLOTS groups of 16 labels per thread: 8 (a 32768-label tile) for small inputs; 32 (131072) for
// large ones, where the reservation atomics of 4096 tiles on one address serialise (2^27 labels:
// 65 us at 8 slots). HIST: hist_out += the top-bucket histogram of the positives' keys (an LDS
// histogram per tile, its used buckets added once). Block 0 writes put_val to *put (nullable: the
// two-step evaluation's slot header length word). fill_w (nullable): the grid also fills nfill16
// 16-byte words there with all-ones (the two-step's slotted table: +inf keys), by extra workgroups
// past the tiles (blockIdx.x >= ntiles), which do only that and the zeroing.
#ifdef DAUC_TUNING
// tuning builds: DAUC_CMP_ABL = 1, a timing ablation of the tiles' reservation (WRONG output): every
// tile writes from position 0 without its returning atomic on the one counter
__device__ int g_cmp_abl = 0;
#endif
template <typename LT, int SLOTS, int THREADS = kCmpThreads, bool HIST = false>
__global__ __launch_bounds__(THREADS) void compact_unordered_kernel(
    const float* __restrict__ s, const LT* __restrict__ lab, int64_t n, int vec, float* __restrict__ pos_out,
    unsigned long long* __restrict__ stats, unsigned long long tag, unsigned long long* __restrict__ zero_next,
    unsigned long long next_tag, unsigned long long* __restrict__ zero3, unsigned* __restrict__ zero_w,
    int nzero_w, int64_t cap, unsigned* __restrict__ hist_out, unsigned long long* __restrict__ put,
    unsigned long long put_val, uint4* __restrict__ fill_w, int64_t nfill16, int64_t ntiles) {
    constexpr int kW = THREADS / kWave;
    constexpr int64_t kTileU = int64_t(THREADS) * 16 * SLOTS;
    __shared__ int wtot[2][kW];
    __shared__ unsigned long long base_s;
    __shared__ unsigned hs[HIST ? kCiTop : 1];
    if constexpr (HIST)
        for (int i = threadIdx.x; i < kCiTop; i += THREADS) hs[i] = 0u;
    if (blockIdx.x == 0) {
        if (threadIdx.x < 4) zero_next[threadIdx.x] = threadIdx.x == 1 ? next_tag : 0ull;
        else if (threadIdx.x < 7 && zero3 != nullptr) zero3[threadIdx.x - 4] = 0ull;
        else if (threadIdx.x == 7 && put != nullptr) *put = put_val;
    }
    for (int64_t i = int64_t(blockIdx.x) * THREADS + threadIdx.x; i < nzero_w; i += int64_t(gridDim.x) * THREADS)
        zero_w[i] = 0u;  // spread over the grid (a later stage's counters: up to 147 k words)
    for (int64_t i = int64_t(blockIdx.x) * THREADS + threadIdx.x; i < nfill16; i += int64_t(gridDim.x) * THREADS)
        fill_w[i] = uint4{~0u, ~0u, ~0u, ~0u};
    if (blockIdx.x >= ntiles) return;  // a fill-only workgroup (uniform)
    // the slot's tag (written with the zeroes by the previous call): a workspace whose slot was
    // not left by this thread's previous call holds stale counters, so no tile reserves from it
    // (the caller sees the tag and starts over with zeroed slots)
    const unsigned long long seen = stats[1];
    const int64_t base = int64_t(blockIdx.x) * kTileU;
    int no = 0;
    int np = 0;
    // label_masks16's bounds check is a branch per group, and a load consumed inside a branch is
    // waited for at once (vmcnt(0)): the groups' loads went out one memory latency apart. A tile
    // wholly in range and aligned (uniform) issues them kCompactBatch at a time in straight-
    // line code; the masks wait in LDS (16 bits per group) for the write phase, so no batch's
    // registers stay live across the next (a rolled loop: nothing hoisted past it)
    __shared__ unsigned short msk[SLOTS][THREADS];
    if (vec && base + kTileU <= n) {
        constexpr int kPer = int(sizeof(LT));  // 16-B loads per group
        constexpr int kB = kCompactBatch / kPer > 0 ? kCompactBatch / kPer : 1;
        constexpr int kBatch = kB < SLOTS ? kB : SLOTS;
        static_assert(SLOTS % kBatch == 0, "whole batches");
        const char* tb = reinterpret_cast<const char*>(lab + base);  // uniform
        const unsigned lane_off = threadIdx.x * 16u * unsigned(sizeof(LT));
        constexpr unsigned kSlotBytes = unsigned(THREADS) * 16u * unsigned(sizeof(LT));
#pragma unroll 1
        for (int k0 = 0; k0 < SLOTS; k0 += kBatch) {
            int4 v[kBatch][kPer];
#pragma unroll
            for (int j = 0; j < kBatch; ++j) {
                const int4* src = reinterpret_cast<const int4*>(tb + (lane_off + unsigned(k0 + j) * kSlotBytes));
#pragma unroll
                for (int q = 0; q < kPer; ++q) v[j][q] = src[q];
            }
#pragma unroll
            for (int j = 0; j < kBatch; ++j) {
                const unsigned mm = masks16_of<LT>(v[j], no);
                np += __popc(mm);
                msk[k0 + j][threadIdx.x] = static_cast<unsigned short>(mm);
            }
        }
    } else {
#pragma unroll 1
        for (int k = 0; k < SLOTS; ++k) {
            const unsigned mm = label_masks16(lab, base + (int64_t(k) * THREADS + threadIdx.x) * 16, n, vec, no);
            np += __popc(mm);
            msk[k][threadIdx.x] = static_cast<unsigned short>(mm);
        }
    }
    const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
    int incl = np;  // inclusive scan of the positives over the wave's lanes
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
        const int v = __shfl_up(incl, off, kWave);
        if (lane >= off) incl += v;
    }
    for (int off = 32; off > 0; off >>= 1) no += __shfl_xor(no, off, kWave);
    if (lane == kWave - 1) wtot[0][wid] = incl;
    if (lane == 0) wtot[1][wid] = no;
    __syncthreads();
    int before = 0, tile = 0;
#pragma unroll
    for (int w = 0; w < kW; ++w) {
        before += w < wid ? wtot[0][w] : 0;
        tile += wtot[0][w];
    }
    if (seen != tag) return;  // uniform across the workgroup
    int nf = 0;
    if (threadIdx.x == 0) {
        int other = 0;
#pragma unroll
        for (int w = 0; w < kW; ++w) other += wtot[1][w];
        if (other) atomicAdd(stats + 3, static_cast<unsigned long long>(other));
#ifdef DAUC_TUNING
        if (g_cmp_abl == 1) base_s = 0ull;
        else
#endif
        base_s = tile ? atomicAdd(stats + 0, static_cast<unsigned long long>(tile)) : 0ull;
    }
    __syncthreads();
    if (tile == 0) return;
    int64_t r = int64_t(base_s) + before + incl - np;
#pragma unroll 1
    for (int k = 0; k < SLOTS; ++k) {
        const int64_t i = base + (int64_t(k) * THREADS + threadIdx.x) * 16;
        const unsigned mk = msk[k][threadIdx.x];  // this thread's own word: no barrier needed
        for (unsigned b = mk; b != 0u; b &= b - 1u) {
            const float v = s[i + __ffs(b) - 1];
            nf += !isfinite(v);
            if (r < cap) pos_out[r] = v;  // past `cap`: counted in stats[0], not stored (the caller's overflow)
            ++r;
            if constexpr (HIST) atomicAdd(&hs[key_fast(v) >> kCiLowBits], 1u);
        }
    }
    if (nf) atomicAdd(stats + 2, static_cast<unsigned long long>(nf));
    if constexpr (HIST) {
        __syncthreads();
        for (int i = threadIdx.x; i < kCiTop; i += THREADS)
            if (hs[i]) atomicAdd(hist_out + i, hs[i]);
    }
}

template <typename LT>
int launch_compact(const float* s, const LT* lab, int64_t n, float* pos_out, int64_t* stats, void* ws,
                   hipStream_t st, unsigned long long* zero3 = nullptr, unsigned* zero_w = nullptr,
                   int nzero_w = 0) {
    const int64_t nblk = compact_blocks(n);
    if (nblk > 0x7fffffffLL) return DAUC_EINVAL;
    int* blk = static_cast<int*>(ws);
    auto* masks = reinterpret_cast<uint4*>(static_cast<char*>(ws) + compact_masks_offset(n));
    const int vec = (reinterpret_cast<uintptr_t>(lab) & 15u) == 0;
    hipLaunchKernelGGL(compact_count_kernel<LT>, dim3(static_cast<unsigned>(nblk)), dim3(kCmpThreads), 0, st, lab, n,
                       vec, blk, masks, stats, zero3, zero_w, nzero_w);
    int rc = launch_status();
    if (rc) return rc;
    hipLaunchKernelGGL(compact_write_kernel, dim3(static_cast<unsigned>(nblk)), dim3(kCmpThreads), 0, st, s, n, blk,
                       masks, pos_out, stats);
    return launch_status();
}

// ============================ pair count ======================================

constexpr int kPcThreads = 256;
constexpr int kNegTile = 2048;  // negatives per LDS tile (8 KB)
constexpr int64_t kTargetBlocks = 8192;

__device__ __forceinline__ float nan_f() { return __builtin_nanf(""); }

typedef float f32x2 __attribute__((ext_vector_type(2)));

// Packed count step for two positives (p0, p1) against one negative q:
//   u = (p0 - q, p1 - q)                     v_pk_add_f32 (q broadcast by op_sel)
//   g = clamp(u * 2^127 + 2^-12, 0, 1)        v_pk_fma_f32 ... clamp
// g is exactly 1 for a win, 2^-12 for a tie and 0 for a loss (or a NaN pad:
// clamp maps NaN to 0, dx10_clamp) PROVIDED every nonzero difference is at
// least 2^-126 in magnitude, so that u * 2^127 >= 2 -- see tile_safe(). The
// accumulator sum W + T * 2^-12 is exact in fp32 for up to 2048 negatives
// (W + T <= 2048 < 2^11, a multiple of 2^-12), so it is decoded per LDS tile.
__device__ __forceinline__ f32x2 pk_clamp_fma(f32x2 u, f32x2 s, f32x2 c) {
    f32x2 g;
    asm("v_pk_fma_f32 %0, %1, %2, %3 clamp" : "=v"(g) : "v"(u), "s"(s), "v"(c));
    return g;
}

// A score is safe for the packed step when it is NaN, +-0, or finite with
// |v| >= 2^-103: all such values are integer multiples of 2^-126, so a nonzero
// difference of two of them is >= 2^-126 (it may overflow to +-inf, which is
// fine). Unsafe: +-inf (inf - inf = NaN would drop a tie) and |v| in
// (0, 2^-103). A block that sees an unsafe value uses the exact compare loop.
__device__ __forceinline__ bool unsafe_score(float v) {
    const unsigned b = __float_as_uint(v) & 0x7fffffffu;
    return (b - 1u) < (0x0C000000u - 1u) || b == 0x7f800000u;
}

// MODE selects how a (pos, neg) pair is counted:
//   0: packed fp32 difference + clamp (1.5 VALU instructions per pair), with a
//      per-tile fallback to mode 1 for tiles holding unsafe scores (default)
//   1: per-lane VGPR counters (v_cmp + v_cndmask/v_addc: ~4 instructions per pair)
//   2: wave ballot + popcount on the scalar unit (v_cmp -> SGPR mask, s_bcnt1, s_add)
//   3: mixed: '>' through the scalar unit, '>=' through VGPR counters
template <int RP, int MODE>
__global__ __launch_bounds__(kPcThreads) void pair_count_kernel(
    const float* __restrict__ pos, int64_t P, const float* __restrict__ neg, int64_t N,
    int64_t neg_per_block, int neg_aligned, unsigned long long* __restrict__ out) {
    static_assert(RP % 2 == 0, "positives are processed in pairs");
    __shared__ float4 tile[kNegTile / 4];
    __shared__ unsigned long long red[2][kPcThreads / kWave];

    float p[RP];
    const int64_t pb = int64_t(blockIdx.x) * (int64_t(kPcThreads) * RP);
    bool bad = false;
#pragma unroll
    for (int r = 0; r < RP; ++r) {
        const int64_t i = pb + int64_t(r) * kPcThreads + threadIdx.x;
        p[r] = i < P ? pos[i] : nan_f();
        bad |= unsafe_score(p[r]);
    }
    const bool pos_bad = MODE == 0 ? __syncthreads_or(bad) != 0 : true;
    f32x2 pp[RP / 2];
#pragma unroll
    for (int k = 0; k < RP / 2; ++k) pp[k] = f32x2{p[2 * k], p[2 * k + 1]};
    const f32x2 kScale = {0x1p127f, 0x1p127f}, kTie = {0x1p-12f, 0x1p-12f};

    unsigned gt[RP], ge[RP];
#pragma unroll
    for (int r = 0; r < RP; ++r) gt[r] = ge[r] = 0u;
    unsigned long long sgt = 0, sge = 0;  // wave-uniform counters (MODE 2, 3)

    const int64_t n0 = int64_t(blockIdx.y) * neg_per_block;
    const int64_t n1 = (n0 + neg_per_block < N) ? n0 + neg_per_block : N;
    for (int64_t t0 = n0; t0 < n1; t0 += kNegTile) {
        bool tbad = false;
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
            if constexpr (MODE == 0)
                tbad |= unsafe_score(x.x) | unsafe_score(x.y) | unsafe_score(x.z) | unsafe_score(x.w);
            tile[v] = x;
        }
        bool packed = false;
        if constexpr (MODE == 0) {
            // the barrier must run in every case (no short-circuit): it publishes the tile
            const int any_bad = __syncthreads_or(tbad);
            packed = !pos_bad && any_bad == 0;  // block-uniform
        } else {
            __syncthreads();
        }
        if (packed) {
            f32x2 acc[RP / 2];
#pragma unroll
            for (int k = 0; k < RP / 2; ++k) acc[k] = f32x2{0.f, 0.f};
#pragma unroll 2
            for (int j = 0; j < kNegTile / 4; ++j) {
                const float4 q = tile[j];  // same address in every lane: LDS broadcast
#pragma unroll
                for (int k = 0; k < RP / 2; ++k) {
                    acc[k] += pk_clamp_fma(pp[k] - f32x2{q.x, q.x}, kScale, kTie);
                    acc[k] += pk_clamp_fma(pp[k] - f32x2{q.y, q.y}, kScale, kTie);
                    acc[k] += pk_clamp_fma(pp[k] - f32x2{q.z, q.z}, kScale, kTie);
                    acc[k] += pk_clamp_fma(pp[k] - f32x2{q.w, q.w}, kScale, kTie);
                }
            }
#pragma unroll
            for (int k = 0; k < RP / 2; ++k) {
                const f32x2 x = acc[k] * 4096.f;  // W * 4096 + T, exact, < 2^24
                const unsigned a0 = static_cast<unsigned>(x.x), a1 = static_cast<unsigned>(x.y);
                gt[2 * k] += a0 >> 12;
                ge[2 * k] += (a0 >> 12) + (a0 & 4095u);
                gt[2 * k + 1] += a1 >> 12;
                ge[2 * k + 1] += (a1 >> 12) + (a1 & 4095u);
            }
        } else {
#pragma unroll 2
            for (int j = 0; j < kNegTile / 4; ++j) {
                const float4 q = tile[j];
#pragma unroll
                for (int r = 0; r < RP; ++r) {
                    if constexpr (MODE <= 1) {
                        gt[r] += (p[r] > q.x);
                        ge[r] += (p[r] >= q.x);
                        gt[r] += (p[r] > q.y);
                        ge[r] += (p[r] >= q.y);
                        gt[r] += (p[r] > q.z);
                        ge[r] += (p[r] >= q.z);
                        gt[r] += (p[r] > q.w);
                        ge[r] += (p[r] >= q.w);
                    } else if constexpr (MODE == 2) {
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
    if (MODE >= 2) tg = sgt;  // already a per-wave total
    if (MODE == 2) te = sge;
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
        stats == nullptr || workspace == nullptr ||
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

size_t dauc_compact_workspace_size(int64_t n) { return compact_ws_bytes(n < 0 ? 0 : n); }

}  // extern "C"

namespace dauc {
// dauc_compact_positives that also zeroes 3 counters and nzero_w words of later stages in its
// first launch
int compact_positives_zeroing(const float* scores, const void* labels, int label_dtype, int64_t n, float* pos_out,
                              int64_t* stats, void* workspace, size_t workspace_bytes, unsigned long long* zero3,
                              hipStream_t st, unsigned* zero_w, int nzero_w) {
    if (n <= 0 || scores == nullptr || labels == nullptr || pos_out == nullptr || stats == nullptr ||
        workspace == nullptr || workspace_bytes < dauc_compact_workspace_size(n) ||
        (reinterpret_cast<uintptr_t>(workspace) & 15u) || (reinterpret_cast<uintptr_t>(stats) & 7u))
        return DAUC_EINVAL;
    switch (label_dtype) {
        case DAUC_LABEL_I8:
            return launch_compact(scores, static_cast<const int8_t*>(labels), n, pos_out, stats, workspace, st, zero3,
                                  zero_w, nzero_w);
        case DAUC_LABEL_I32:
            return launch_compact(scores, static_cast<const int32_t*>(labels), n, pos_out, stats, workspace, st, zero3,
                                  zero_w, nzero_w);
        case DAUC_LABEL_I64:
            return launch_compact(scores, static_cast<const int64_t*>(labels), n, pos_out, stats, workspace, st, zero3,
                                  zero_w, nzero_w);
        default:
            return DAUC_EINVAL;
    }
}

int compact_unordered(const float* scores, const void* labels, int label_dtype, int64_t n, float* pos_out,
                      unsigned long long* stats, unsigned long long tag, unsigned long long* zero_next,
                      unsigned long long next_tag, unsigned long long* zero3, unsigned* zero_w, int nzero_w,
                      hipStream_t st, int64_t cap, unsigned* hist_out, unsigned long long* put,
                      unsigned long long put_val, unsigned* fill_w, int64_t nfill16) {
    if (n <= 0 || scores == nullptr || labels == nullptr || pos_out == nullptr || stats == nullptr ||
        zero_next == nullptr)
        return DAUC_EINVAL;
    const bool wide = n >= (int64_t(1) << 25);
    // wide inputs: 1024-thread workgroups of 32 label groups per thread (524,288-label tiles: 256
    // reservations at 2^27 instead of 1024 on the one counter address) -- 256
    constexpr int kWideThreads = 256;
    int slots = wide ? 32 : kCmpSlots;
#ifdef DAUC_TUNING
    // tuning builds: DAUC_CMP_SLOTS (8, 16, 32, 64) = label groups per thread whatever n
    if (const char* e = getenv("DAUC_CMP_SLOTS");
        e && (atoi(e) == 8 || atoi(e) == 16 || atoi(e) == 32 || atoi(e) == 64))
        slots = atoi(e);
#endif
    // round 6: 512-thread tiles (8 groups per thread, the histogram form) from 2^23 labels below the
    // wide shape: half the tiles, so half the reservations on the one counter, which serialise
    // (the two-step's 2^24-label slice: 512 -> 256 tiles, step 1 17.9 -> 14.9 us; the one-call
    // evaluation of 2^24 labels 114.9 -> 110.1 us; the 2^21-label slice keeps 256: 12.2 vs 12.8 us)
    constexpr int kMidThreads = 512;
    const bool mid_ok = !wide && hist_out != nullptr && slots == kCmpSlots;
    int threads = wide ? kWideThreads : mid_ok && n >= (int64_t(1) << 23) ? kMidThreads : kCmpThreads;
#ifdef DAUC_TUNING
    // tuning builds: DAUC_CMP_THREADS (256, 512, 1024) = threads per tile of that form whatever n
    if (const char* e = getenv("DAUC_CMP_THREADS");
        mid_ok && e && (atoi(e) == 256 || atoi(e) == 512 || atoi(e) == 1024))
        threads = atoi(e);
#endif
#ifdef DAUC_TUNING
    {
        static int abl = -1;
        if (abl < 0) {
            const char* e = getenv("DAUC_CMP_ABL");
            abl = e ? atoi(e) : 0;
            if (hipMemcpyToSymbol(HIP_SYMBOL(g_cmp_abl), &abl, sizeof(int)) != hipSuccess) return DAUC_EINVAL;
        }
    }
#endif
    const int64_t tile = int64_t(threads) * 16 * slots;
    const int64_t nblk = (n + tile - 1) / tile;
    if (nblk > 0x7fffffffLL) return DAUC_EINVAL;
    const int vec = (reinterpret_cast<uintptr_t>(labels) & 15u) == 0;
    // fill-only workgroups past the tiles: `per` 16-byte stores per thread (the tiles' CUs stay theirs)
#ifdef DAUC_TUNING
    static int per = 0;  // tuning builds: DAUC_FILL_PER_THREAD
    if (per == 0) {
        const char* e = getenv("DAUC_FILL_PER_THREAD");
        per = e ? atoi(e) : 4;
        if (per < 1 || per > 4096) per = 4;
    }
#else
    constexpr int per = 4;
#endif
    const int64_t nfill = fill_w != nullptr ? nfill16 : 0;
    const int64_t extra = (nfill + int64_t(threads) * per - 1) / (int64_t(threads) * per);
    if (nblk + extra > 0x7fffffffLL) return DAUC_EINVAL;
    const dim3 grid(static_cast<unsigned>(nblk + extra)), block(threads);
    uint4* fw = reinterpret_cast<uint4*>(fill_w);
    auto go = [&](auto* lab) {
        using LT = std::remove_const_t<std::remove_pointer_t<decltype(lab)>>;
        if (mid_ok && threads == kMidThreads) {
            hipLaunchKernelGGL((compact_unordered_kernel<LT, kCmpSlots, kMidThreads, true>), grid, block, 0, st, scores,
                               lab, n, vec, pos_out, stats, tag, zero_next, next_tag, zero3, zero_w, nzero_w, cap,
                               hist_out, put, put_val, fw, nfill, nblk);
            return launch_status();
        }
#ifdef DAUC_TUNING
        if (mid_ok && threads == 1024) {
            hipLaunchKernelGGL((compact_unordered_kernel<LT, kCmpSlots, 1024, true>), grid, block, 0, st, scores, lab,
                               n, vec, pos_out, stats, tag, zero_next, next_tag, zero3, zero_w, nzero_w, cap, hist_out,
                               put, put_val, fw, nfill, nblk);
            return launch_status();
        }
        if (slots == 64) {
            if (hist_out != nullptr)
                hipLaunchKernelGGL((compact_unordered_kernel<LT, 64, kCmpThreads, true>), grid, block, 0, st, scores,
                                   lab, n, vec, pos_out, stats, tag, zero_next, next_tag, zero3, zero_w, nzero_w, cap,
                                   hist_out, put, put_val, fw, nfill, nblk);
            else
                hipLaunchKernelGGL((compact_unordered_kernel<LT, 64, kCmpThreads>), grid, block, 0, st, scores, lab, n,
                                   vec, pos_out, stats, tag, zero_next, next_tag, zero3, zero_w, nzero_w, cap, hist_out,
                                   put, put_val, fw, nfill, nblk);
            return launch_status();
        }
        if (slots == 16) {
            if (hist_out != nullptr)
                hipLaunchKernelGGL((compact_unordered_kernel<LT, 16, kCmpThreads, true>), grid, block, 0, st, scores,
                                   lab, n, vec, pos_out, stats, tag, zero_next, next_tag, zero3, zero_w, nzero_w, cap,
                                   hist_out, put, put_val, fw, nfill, nblk);
            else
                hipLaunchKernelGGL((compact_unordered_kernel<LT, 16, kCmpThreads>), grid, block, 0, st, scores, lab, n,
                                   vec, pos_out, stats, tag, zero_next, next_tag, zero3, zero_w, nzero_w, cap, hist_out,
                                   put, put_val, fw, nfill, nblk);
            return launch_status();
        }
        if ((slots == 32) != wide) {  // the other of the two product shapes
            if (slots == 32 && hist_out != nullptr)
                hipLaunchKernelGGL((compact_unordered_kernel<LT, 32, kWideThreads, true>), grid, block, 0, st, scores,
                                   lab, n, vec, pos_out, stats, tag, zero_next, next_tag, zero3, zero_w, nzero_w, cap,
                                   hist_out, put, put_val, fw, nfill, nblk);
            else if (slots == 32)
                hipLaunchKernelGGL((compact_unordered_kernel<LT, 32, kWideThreads>), grid, block, 0, st, scores, lab, n,
                                   vec, pos_out, stats, tag, zero_next, next_tag, zero3, zero_w, nzero_w, cap, hist_out,
                                   put, put_val, fw, nfill, nblk);
            else if (hist_out != nullptr)
                hipLaunchKernelGGL((compact_unordered_kernel<LT, kCmpSlots, kCmpThreads, true>), grid, block, 0, st,
                                   scores, lab, n, vec, pos_out, stats, tag, zero_next, next_tag, zero3, zero_w, nzero_w,
                                   cap, hist_out, put, put_val, fw, nfill, nblk);
            else
                hipLaunchKernelGGL((compact_unordered_kernel<LT, kCmpSlots>), grid, block, 0, st, scores, lab, n, vec,
                                   pos_out, stats, tag, zero_next, next_tag, zero3, zero_w, nzero_w, cap, hist_out, put,
                                   put_val, fw, nfill, nblk);
            return launch_status();
        }
#endif
        if (wide && hist_out != nullptr)
            hipLaunchKernelGGL((compact_unordered_kernel<LT, 32, kWideThreads, true>), grid, block, 0, st, scores, lab,
                               n, vec, pos_out, stats, tag, zero_next, next_tag, zero3, zero_w, nzero_w, cap, hist_out, put, put_val, fw,
                               nfill, nblk);
        else if (wide)
            hipLaunchKernelGGL((compact_unordered_kernel<LT, 32, kWideThreads>), grid, block, 0, st, scores, lab, n, vec,
                               pos_out, stats, tag, zero_next, next_tag, zero3, zero_w, nzero_w, cap, hist_out, put, put_val, fw,
                               nfill, nblk);
        else if (hist_out != nullptr)
            hipLaunchKernelGGL((compact_unordered_kernel<LT, kCmpSlots, kCmpThreads, true>), grid, block, 0, st, scores,
                               lab, n, vec, pos_out, stats, tag, zero_next, next_tag, zero3, zero_w, nzero_w, cap,
                               hist_out, put, put_val, fw, nfill, nblk);
        else
            hipLaunchKernelGGL((compact_unordered_kernel<LT, kCmpSlots>), grid, block, 0, st, scores, lab, n, vec,
                               pos_out, stats, tag, zero_next, next_tag, zero3, zero_w, nzero_w, cap, hist_out, put, put_val, fw,
                               nfill, nblk);
        return launch_status();
    };
    switch (label_dtype) {
        case DAUC_LABEL_I8: return go(static_cast<const int8_t*>(labels));
        case DAUC_LABEL_I32: return go(static_cast<const int32_t*>(labels));
        case DAUC_LABEL_I64: return go(static_cast<const int64_t*>(labels));
        default: return DAUC_EINVAL;
    }
}
}  // namespace dauc

extern "C" {

int dauc_compact_positives(const float* scores, const void* labels, int label_dtype, int64_t n,
                           float* pos_out, int64_t* stats, void* workspace, size_t workspace_bytes,
                           dauc_stream_t stream) {
    return compact_positives_zeroing(scores, labels, label_dtype, n, pos_out, stats, workspace, workspace_bytes,
                                     nullptr, as_hip(stream));
}

static int pair_count_impl(const float* pos, int64_t P, const float* neg, int64_t N,
                           unsigned long long* wins_ties, int variant, dauc_stream_t stream);

int dauc_pair_count(const float* pos, int64_t P, const float* neg, int64_t N,
                    unsigned long long* wins_ties, dauc_stream_t stream) {
    return pair_count_impl(pos, P, neg, N, wins_ties, 0, stream);
}

#ifdef DAUC_TUNING
int dauc_pair_count_variant(const float* pos, int64_t P, const float* neg, int64_t N,
                            unsigned long long* wins_ties, int variant, dauc_stream_t stream) {
    return pair_count_impl(pos, P, neg, N, wins_ties, variant, stream);
}
#endif

static int pair_count_impl(const float* pos, int64_t P, const float* neg, int64_t N,
                           unsigned long long* wins_ties, int variant, dauc_stream_t stream) {
    if (P < 0 || N < 0 || wins_ties == nullptr || (P > 0 && pos == nullptr) ||
        (N > 0 && neg == nullptr))
        return DAUC_EINVAL;
    if (P == 0 || N == 0) return DAUC_OK;
    // variant = mode + 4 * rp_index; mode: counting scheme, rp: positives per lane {8, 4, 16}
    if (variant < 0 || variant >= 12) return DAUC_EINVAL;
    const int rp = variant / 4 == 0 ? 8 : (variant / 4 == 1 ? 4 : 16);
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
#ifdef DAUC_TUNING
        case 1: DAUC_PC_LAUNCH(8, 1); break;
        case 2: DAUC_PC_LAUNCH(8, 2); break;
        case 3: DAUC_PC_LAUNCH(8, 3); break;
        case 4: DAUC_PC_LAUNCH(4, 0); break;
        case 5: DAUC_PC_LAUNCH(4, 1); break;
        case 6: DAUC_PC_LAUNCH(4, 2); break;
        case 7: DAUC_PC_LAUNCH(4, 3); break;
        case 8: DAUC_PC_LAUNCH(16, 0); break;
        case 9: DAUC_PC_LAUNCH(16, 1); break;
        case 10: DAUC_PC_LAUNCH(16, 2); break;
        case 11: DAUC_PC_LAUNCH(16, 3); break;
#endif
        default: return DAUC_EINVAL;
    }
#undef DAUC_PC_LAUNCH
    return launch_status();
}

}  // extern "C"
