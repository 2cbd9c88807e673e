// Fused BatchNorm (batch statistics) + optional residual add + optional ReLU for
// channels-last activations, forward and backward, for the CoDA backbone step.
//
// Reference: the ResNet blocks of imagenet/resnet.py (BasicBlock.forward 47-64,
// Bottleneck.forward 87-108, ResNet stem 203-206): conv -> bn -> relu, and
// bn -> (+ identity) -> relu at the end of each block, in training mode
// (main.py:280 net.train()). torch runs each of bn / add / relu as its own pass
// over HBM (MIOpen's 3-kernel BN plus two elementwise kernels, forward and
// backward); here a BN layer costs, in HBM passes over its [M, C] activation
// (M = N*H*W rows, C channels, C contiguous):
//   forward : stats (read x)  + apply (read x [+ residual], write y)
//   backward: reduce (read dy, y, x [, write dz]) + dx (read dy, y | dz, x; write dx)
// with two tiny per-channel finalize launches in between. Statistics are
// accumulated in fp32 per thread (shifted by a sample of the channel), combined in
// fp64 in a fixed order: results are bitwise reproducible run to run.
//
// ReLU mask (round 5): a forward with ReLU can also write one bit per element, y > 0 as stored
// (one byte per 16-byte vector), and the backward then reads that bit instead of the whole y for the
// ReLU's gradient mask: 0.125 B instead of 2 (bf16) per element in both backward passes -- the BN
// backward is HBM-bound, so this is ~2 B less traffic per element and pass.
//
// Geometry: a thread owns one 16-byte vector of channels (8 bf16 or 4 fp32) of
// a channel tile of CT channels; TPR = CT / vec threads cover a row, RPB = 256 /
// TPR rows are in flight per pass, and a workgroup walks a contiguous block of
// rows with kUnroll passes' loads issued before any math.

#include <hip/hip_bf16.h>

#include <stdlib.h>

#include <initializer_list>
#include <type_traits>

#include "dauc_internal.h"

namespace dauc {
namespace {

constexpr int kBnThreads = 256;
constexpr int kDefaultPartThreads = 512;  // profiles/r01/ab_bn_threads.jsonl
constexpr int kMaxRowBlocks = 2048;  // partial rows per channel (workspace bound)
constexpr int kFinThreads = 1024;    // finalize: 64 row subsets x 16 channel quads
constexpr int kFinSubsets = kFinThreads / 16;

// target row blocks per launch (tuning knob DAUC_BN_ROWBLOCKS; 256 measured best on MI355X:
// 256 and 512 tie on the ResNet-50 step, 1024 / 2048 lose to the longer finalize)
int row_block_target() {
    static int v = 0;
    if (v == 0) {
        const char* e = getenv("DAUC_BN_ROWBLOCKS");
        int t = e ? atoi(e) : 256;
        v = (t >= 1 && t <= kMaxRowBlocks) ? t : 256;
    }
    return v;
}
// threads per workgroup of the partial-sum passes (DAUC_BN_PART_THREADS: 256 | 512 | 1024). With
// ~256 row blocks the grid is about one workgroup per CU, so the workgroup size sets the bytes
// in flight per CU.
int part_threads() {
    static int v = 0;
    if (v == 0) {
        const char* e = getenv("DAUC_BN_PART_THREADS");
        const int t = e ? atoi(e) : kDefaultPartThreads;
        v = (t == 256 || t == 512 || t == 1024) ? t : kDefaultPartThreads;
    }
    return v;
}
constexpr int kUnroll = 8;          // row passes whose loads are in flight together
constexpr int kApplyVecs = 4;       // 16-byte vectors per thread in the elementwise kernels

template <typename T>
struct VecT;
template <>
struct VecT<__hip_bfloat16> {
    static constexpr int N = 8;
};
template <>
struct VecT<float> {
    static constexpr int N = 4;
};

// 16-byte raw vectors: loads are issued as raw words, converted to fp32 when used
template <typename T>
using RawT = typename std::conditional<sizeof(T) == 2, uint4, f32x4>::type;

template <typename T>
__device__ __forceinline__ RawT<T> load_raw(const T* p) {
    return *reinterpret_cast<const RawT<T>*>(p);
}

__device__ __forceinline__ void cvt(const uint4& u, float (&v)[8]) {
    const unsigned w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        v[2 * i] = __uint_as_float(w[i] << 16);
        v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
}

__device__ __forceinline__ void cvt(const f32x4& u, float (&v)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = u[i];
}

template <typename T, int N>
__device__ __forceinline__ void load_vec(const T* p, float (&v)[N]) {
    cvt(load_raw(p), v);
}

// fp32 -> bf16, round to nearest even (NaN stays NaN)
__device__ __forceinline__ unsigned bf16_bits(float f) {
    const unsigned b = __float_as_uint(f);
    if ((b & 0x7fffffffu) > 0x7f800000u) return (b >> 16) | 0x40u;
    return (b + 0x7fffu + ((b >> 16) & 1u)) >> 16;
}

__device__ __forceinline__ void store_vec(__hip_bfloat16* p, const float (&v)[8]) {
    uint4 u;
    u.x = bf16_bits(v[0]) | (bf16_bits(v[1]) << 16);
    u.y = bf16_bits(v[2]) | (bf16_bits(v[3]) << 16);
    u.z = bf16_bits(v[4]) | (bf16_bits(v[5]) << 16);
    u.w = bf16_bits(v[6]) | (bf16_bits(v[7]) << 16);
    *reinterpret_cast<uint4*>(p) = u;
}

__device__ __forceinline__ void store_vec(float* p, const float (&v)[4]) {
    f32x4 u;
#pragma unroll
    for (int i = 0; i < 4; ++i) u[i] = v[i];
    *reinterpret_cast<f32x4*>(p) = u;
}

// store_vec + the ReLU mask of what was stored: bit i = (stored element i > 0), i.e. exactly the
// backward's `y > 0` on the stored y (positive nonzero, +inf included, NaN excluded)
__device__ __forceinline__ unsigned store_vec_mask(__hip_bfloat16* p, const float (&v)[8]) {
    unsigned b[8], m = 0u;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        b[i] = bf16_bits(v[i]);
        m |= unsigned(b[i] - 1u < 0x7f80u) << i;  // 1 .. 0x7f80: +denormal .. +inf
    }
    uint4 u;
    u.x = b[0] | (b[1] << 16);
    u.y = b[2] | (b[3] << 16);
    u.z = b[4] | (b[5] << 16);
    u.w = b[6] | (b[7] << 16);
    *reinterpret_cast<uint4*>(p) = u;
    return m;
}

__device__ __forceinline__ unsigned store_vec_mask(float* p, const float (&v)[4]) {
    unsigned m = 0u;
#pragma unroll
    for (int i = 0; i < 4; ++i) m |= unsigned(__float_as_uint(v[i]) - 1u < 0x7f800000u) << i;
    store_vec(p, v);
    return m;
}

struct Geometry {
    int N;        // elements per 16-byte vector
    int CT;       // channels per tile
    int TPR;      // threads per row
    int RPB;      // rows per pass
    int ctiles;   // channel tiles
    int nrb;      // row blocks per channel tile
    int64_t rows; // rows per row block
};

int make_geometry(int64_t M, int C, int elem_bytes, Geometry& g, int threads = kBnThreads) {
    g.N = 16 / elem_bytes;
    if (M <= 0 || C <= 0 || C % g.N != 0) return DAUC_EINVAL;
    const int CV = C / g.N;
    g.TPR = CV <= kBnThreads ? CV : kBnThreads;
    if (kBnThreads % g.TPR != 0 || CV % g.TPR != 0) return DAUC_EINVAL;  // power-of-two vector counts
    g.CT = g.TPR * g.N;
    g.ctiles = C / g.CT;
    g.RPB = threads / g.TPR;
    int64_t target = (row_block_target() + g.ctiles - 1) / g.ctiles;
    const int64_t passes = (M + g.RPB - 1) / g.RPB;
    if (target > passes) target = passes;
    if (target < 1) target = 1;
    int64_t rows = (M + target - 1) / target;
    rows = (rows + g.RPB - 1) / g.RPB * g.RPB;
    g.rows = rows;
    g.nrb = static_cast<int>((M + rows - 1) / rows);
    return DAUC_OK;
}

// ---- per-channel partial sums over a block of rows ---------------------------------
// Forward (STATS): s1 = sum (x - k), s2 = sum (x - k)^2 with k = the block's first row (a
// sample of the channel, so the one-pass variance stays well conditioned: the cancellation
// factor is (mean - k)^2 / var = O(1)); k is written as a third partial row.
// Backward: g = dy * [y > 0] (RELU) or dy; s1 = sum g, s2 = sum g * (x - mean); g is
// written to dz (the residual branch's gradient) when dz != nullptr.
// MASK (backward with RELU): the ReLU mask comes from `mask` (one byte per 16-byte vector) instead
// of y.
template <typename T, bool STATS, bool RELU, int TH, bool MASK = false>
__global__ __launch_bounds__(TH) void bn_partial_kernel(
    const T* __restrict__ x, const T* __restrict__ dy, const T* __restrict__ y, T* __restrict__ dz, int64_t M,
    int C, int CT, int64_t rows_per_block, const float* __restrict__ center, float* __restrict__ partials,
    const unsigned char* __restrict__ mask) {
    constexpr int N = VecT<T>::N;
    __shared__ float red[2 * TH * N];
    const int TPR = CT / N;
    const int RPB = TH / TPR;
    const int cl = (threadIdx.x % TPR) * N;  // channel offset within the tile
    const int c0 = blockIdx.y * CT + cl;
    const int r0 = threadIdx.x / TPR;
    const int64_t rs = int64_t(blockIdx.x) * rows_per_block;
    const int64_t re = (rs + rows_per_block < M) ? rs + rows_per_block : M;
    constexpr int NP = STATS ? 3 : 2;  // partial rows per block: s1, s2 (, k)

    float k[N], s1[N], s2[N];
    if (STATS) load_vec(x + rs * C + c0, k);
#pragma unroll
    for (int i = 0; i < N; ++i) {
        if (!STATS) k[i] = center[c0 + i];
        s1[i] = 0.f;
        s2[i] = 0.f;
    }
    auto visit = [&](int64_t r) {
        const int64_t off = r * C + c0;
        float xv[N];
        load_vec(x + off, xv);
        if (STATS) {
#pragma unroll
            for (int i = 0; i < N; ++i) {
                const float d = xv[i] - k[i];
                s1[i] += d;
                s2[i] += d * d;
            }
        } else {
            float gv[N];
            load_vec(dy + off, gv);
            if (RELU && MASK) {
                const unsigned m = mask[off / N];
#pragma unroll
                for (int i = 0; i < N; ++i) gv[i] = (m >> i) & 1u ? gv[i] : 0.f;
            } else if (RELU) {
                float yv[N];
                load_vec(y + off, yv);
#pragma unroll
                for (int i = 0; i < N; ++i) gv[i] = yv[i] > 0.f ? gv[i] : 0.f;
            }
            if (dz) store_vec(dz + off, gv);
#pragma unroll
            for (int i = 0; i < N; ++i) {
                s1[i] += gv[i];
                s2[i] += gv[i] * (xv[i] - k[i]);
            }
        }
    };
    // full groups of U passes: every load of the group is issued before any math
    constexpr int U = STATS ? kUnroll : kUnroll / 2;
    int64_t r = rs + r0;
    const int64_t step = int64_t(RPB) * U;
    for (; r + step - RPB < re; r += step) {
        RawT<T> xr[U], gr[U], yr[U];
        unsigned mr[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t off = (r + int64_t(u) * RPB) * C + c0;
            xr[u] = load_raw(x + off);
            if (!STATS) gr[u] = load_raw(dy + off);
            if (!STATS && RELU && MASK) mr[u] = mask[off / N];
            else if (!STATS && RELU) yr[u] = load_raw(y + off);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            float xv[N];
            cvt(xr[u], xv);
            if (STATS) {
#pragma unroll
                for (int i = 0; i < N; ++i) {
                    const float d = xv[i] - k[i];
                    s1[i] += d;
                    s2[i] += d * d;
                }
            } else {
                float gv[N];
                cvt(gr[u], gv);
                if (RELU && MASK) {
#pragma unroll
                    for (int i = 0; i < N; ++i) gv[i] = (mr[u] >> i) & 1u ? gv[i] : 0.f;
                } else if (RELU) {
                    float yv[N];
                    cvt(yr[u], yv);
#pragma unroll
                    for (int i = 0; i < N; ++i) gv[i] = yv[i] > 0.f ? gv[i] : 0.f;
                }
                if (dz) store_vec(dz + (r + int64_t(u) * RPB) * C + c0, gv);
#pragma unroll
                for (int i = 0; i < N; ++i) {
                    s1[i] += gv[i];
                    s2[i] += gv[i] * (xv[i] - k[i]);
                }
            }
        }
    }
    for (; r < re; r += RPB) visit(r);

    // fixed-order reduction over the RPB rows of the pass
    float* r1 = red;
    float* r2 = red + TH * N;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        r1[r0 * CT + cl + i] = s1[i];
        r2[r0 * CT + cl + i] = s2[i];
    }
    __syncthreads();
    for (int j = threadIdx.x; j < 2 * CT; j += TH) {
        const int stat = j / CT, c = j % CT;
        const float* src = stat ? r2 : r1;
        float acc = 0.f;
        for (int q = 0; q < RPB; ++q) acc += src[q * CT + c];
        partials[(int64_t(blockIdx.x) * NP + stat) * C + blockIdx.y * CT + c] = acc;
    }
    if (STATS && r0 == 0) {
#pragma unroll
        for (int i = 0; i < N; ++i) partials[(int64_t(blockIdx.x) * NP + 2) * C + c0 + i] = k[i];
    }
}

// ---- per-channel finalize: fp64 sum of the partial rows in a fixed order -------------
// kFinSubsets row subsets x 16 channel quads per workgroup = 64 channels.
// STATS rows are (s1, s2, k) over n_b rows; they fold into sum x and sum x^2 in fp64:
//   sum x = s1 + n_b k,  sum x^2 = s2 + 2 k s1 + n_b k^2.
template <bool STATS>
__device__ __forceinline__ void sum_partials(const float* __restrict__ partials, int nrb, int64_t M, int64_t rows,
                                             int C, int cbase, double (*red)[kFinSubsets][64], double& t1,
                                             double& t2) {
    constexpr int NP = STATS ? 3 : 2;
    constexpr int FU = 4;  // row subsets' loads in flight per thread before any fold
    const int cq = threadIdx.x % 16, j = threadIdx.x / 16;
    const int c = cbase + cq * 4;
    double a1[4] = {0, 0, 0, 0}, a2[4] = {0, 0, 0, 0};
    auto fold = [&](int rb, const f32x4& p1, const f32x4& p2, const f32x4& pk) {
        if (STATS) {
            const int64_t r0 = int64_t(rb) * rows;
            const double nb = double((M - r0) < rows ? (M - r0) : rows);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const double k = pk[i], s1 = p1[i];
                a1[i] += s1 + nb * k;
                a2[i] += double(p2[i]) + 2.0 * k * s1 + nb * k * k;
            }
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                a1[i] += p1[i];
                a2[i] += p2[i];
            }
        }
    };
    auto ld = [&](int rb, int q) {
        return *reinterpret_cast<const f32x4*>(partials + (int64_t(rb) * NP + q) * C + c);
    };
    if (c < C) {
        // rows rb = j, j + S, j + 2S, ... folded in that order; FU rows' loads issued together
        int rb = j;
        for (; rb + (FU - 1) * kFinSubsets < nrb; rb += FU * kFinSubsets) {
            f32x4 p1[FU], p2[FU], pk[FU];
#pragma unroll
            for (int u = 0; u < FU; ++u) {
                p1[u] = ld(rb + u * kFinSubsets, 0);
                p2[u] = ld(rb + u * kFinSubsets, 1);
                if (STATS) pk[u] = ld(rb + u * kFinSubsets, 2);
            }
#pragma unroll
            for (int u = 0; u < FU; ++u) fold(rb + u * kFinSubsets, p1[u], p2[u], pk[u]);
        }
        for (; rb < nrb; rb += kFinSubsets) {
            const f32x4 p1 = ld(rb, 0), p2 = ld(rb, 1);
            f32x4 pk;
            if (STATS) pk = ld(rb, 2);
            fold(rb, p1, p2, pk);
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        red[0][j][cq * 4 + i] = a1[i];
        red[1][j][cq * 4 + i] = a2[i];
    }
    __syncthreads();
    // pairwise tree over the row subsets (a fixed order: bitwise reproducible)
#pragma unroll
    for (int s = kFinSubsets / 2; s >= 1; s >>= 1) {
        if (j < s) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                red[0][j][cq * 4 + i] += red[0][j + s][cq * 4 + i];
                red[1][j][cq * 4 + i] += red[1][j + s][cq * 4 + i];
            }
        }
        __syncthreads();
    }
    t1 = 0.0;
    t2 = 0.0;
    if (threadIdx.x < 64) {
        t1 = red[0][0][threadIdx.x];
        t2 = red[1][0][threadIdx.x];
    }
}

__global__ __launch_bounds__(kFinThreads) void bn_fwd_finalize_kernel(
    const float* __restrict__ partials, int nrb, int64_t rows, int64_t M, int C, const float* __restrict__ gamma,
    const float* __restrict__ beta, float* __restrict__ running_mean, float* __restrict__ running_var,
    float momentum, float eps, float* __restrict__ save_mean, float* __restrict__ save_invstd,
    float* __restrict__ scale, float* __restrict__ beta_out, float* __restrict__ mean_out) {
    __shared__ double red[2][kFinSubsets][64];
    double sx, sxx;
    sum_partials<true>(partials, nrb, M, rows, C, blockIdx.x * 64, red, sx, sxx);
    const int c = blockIdx.x * 64 + threadIdx.x;
    if (threadIdx.x >= 64 || c >= C) return;
    const double mean = sx / double(M);
    double var = sxx / double(M) - mean * mean;
    if (var < 0.0) var = 0.0;
    const double invstd = 1.0 / sqrt(var + double(eps));
    save_mean[c] = static_cast<float>(mean);
    save_invstd[c] = static_cast<float>(invstd);
    const double g = gamma ? gamma[c] : 1.0, b = beta ? beta[c] : 0.0;
    // applied as y = (x - mean) * scale + beta (no large-magnitude cancellation when |mean| >> std)
    scale[c] = static_cast<float>(g * invstd);
    beta_out[c] = static_cast<float>(b);
    mean_out[c] = static_cast<float>(mean);
    if (running_mean) {
        // torch: running = (1 - momentum) * running + momentum * batch (unbiased variance)
        const double unbiased = M > 1 ? var * double(M) / double(M - 1) : var;
        running_mean[c] = static_cast<float>((1.0 - momentum) * running_mean[c] + momentum * mean);
        running_var[c] = static_cast<float>((1.0 - momentum) * running_var[c] + momentum * unbiased);
    }
}

// backward: dx = a*g + b*(x - mean) + c per channel; dgamma = invstd * sum g(x-mean); dbeta = sum g
__global__ __launch_bounds__(kFinThreads) void bn_bwd_finalize_kernel(
    const float* __restrict__ partials, int nrb, int64_t M, int C, const float* __restrict__ gamma,
    const float* __restrict__ save_mean, const float* __restrict__ save_invstd, float* __restrict__ dgamma,
    float* __restrict__ dbeta, float* __restrict__ ca, float* __restrict__ cb, float* __restrict__ cc,
    float* __restrict__ cm) {
    __shared__ double red[2][kFinSubsets][64];
    double sg, sgx;
    sum_partials<false>(partials, nrb, M, 0, C, blockIdx.x * 64, red, sg, sgx);
    const int c = blockIdx.x * 64 + threadIdx.x;
    if (threadIdx.x >= 64 || c >= C) return;
    const double inv = save_invstd[c], mean = save_mean[c];
    const double g = gamma ? gamma[c] : 1.0;
    if (dgamma) dgamma[c] = static_cast<float>(sgx * inv);
    if (dbeta) dbeta[c] = static_cast<float>(sg);
    const double a = g * inv;
    const double b = -g * inv * inv * inv * sgx / double(M);
    ca[c] = static_cast<float>(a);
    cb[c] = static_cast<float>(b);
    cc[c] = static_cast<float>(-a * sg / double(M));
    cm[c] = save_mean[c];
}

// ---- elementwise passes over [M, C] -------------------------------------------------
// Forward apply: y = act((x - mean) * scale + beta [+ res]). Backward: dx = a*g + b*(x - mean) + c,
// g = dz (GMODE 2), dy * [y > 0] (GMODE 1) or dy (GMODE 0).
// HOIST: the vector count per row divides 256, so a thread's channels never change.
// MASK: forward with RELU writes the ReLU mask byte of every vector; backward GMODE 1 reads it
// instead of y (aux).
template <typename T, bool BWD, int GMODE, bool RELU, bool RES, bool HOIST, bool MASK = false>
__global__ __launch_bounds__(kBnThreads) void bn_elementwise_kernel(
    const T* __restrict__ x, const T* __restrict__ g_in, const T* __restrict__ aux, T* __restrict__ out,
    int64_t nvec, int CV, const float* __restrict__ p0, const float* __restrict__ p1, const float* __restrict__ p2,
    const float* __restrict__ p3, unsigned char* __restrict__ mask) {
    constexpr int N = VecT<T>::N;
    // forward: p0 = scale, p1 = beta, aux = residual. backward: p0..p2 = a, b, c, aux = y. p3 = mean
    auto body = [&](int64_t v, const float* P0, const float* P1, const float* P2, const float* P3) {
        const int64_t off = v * N;
        float xv[N];
        load_vec(x + off, xv);
        float o[N];
        if (!BWD) {
            float rv[N];
            if (RES) load_vec(aux + off, rv);
#pragma unroll
            for (int i = 0; i < N; ++i) {
                float t = (xv[i] - P3[i]) * P0[i] + P1[i];
                if (RES) t += rv[i];
                o[i] = (RELU && t < 0.f) ? 0.f : t;  // NaN propagates, as torch.relu
            }
        } else {
            float gv[N];
            load_vec(g_in + off, gv);
            if (GMODE == 1 && MASK) {
                const unsigned m = mask[v];
#pragma unroll
                for (int i = 0; i < N; ++i) gv[i] = (m >> i) & 1u ? gv[i] : 0.f;
            } else if (GMODE == 1) {
                float yv[N];
                load_vec(aux + off, yv);
#pragma unroll
                for (int i = 0; i < N; ++i) gv[i] = yv[i] > 0.f ? gv[i] : 0.f;
            }
#pragma unroll
            for (int i = 0; i < N; ++i) o[i] = P0[i] * gv[i] + P1[i] * (xv[i] - P3[i]) + P2[i];
        }
        if constexpr (!BWD && RELU && MASK)
            mask[v] = static_cast<unsigned char>(store_vec_mask(out + off, o));
        else
            store_vec(out + off, o);
    };
    auto params = [&](int cv, float (&q0)[N], float (&q1)[N], float (&q2)[N], float (&q3)[N]) {
#pragma unroll
        for (int i = 0; i < N; ++i) {
            q0[i] = p0[cv * N + i];
            q1[i] = p1[cv * N + i];
            q2[i] = BWD ? p2[cv * N + i] : 0.f;
            q3[i] = p3[cv * N + i];
        }
    };
    const int64_t base = int64_t(blockIdx.x) * kApplyVecs * kBnThreads + threadIdx.x;
    float q0[N], q1[N], q2[N], q3[N];
    if (HOIST) params(threadIdx.x % CV, q0, q1, q2, q3);
    if (int64_t(blockIdx.x + 1) * kApplyVecs * kBnThreads <= nvec) {
        // interior block: no guards (loads of all kApplyVecs vectors issue together)
#pragma unroll
        for (int u = 0; u < kApplyVecs; ++u) {
            const int64_t v = base + int64_t(u) * kBnThreads;
            if (!HOIST) params(static_cast<int>(v % CV), q0, q1, q2, q3);
            body(v, q0, q1, q2, q3);
        }
    } else {
        for (int u = 0; u < kApplyVecs; ++u) {
            const int64_t v = base + int64_t(u) * kBnThreads;
            if (v >= nvec) break;
            if (!HOIST) params(static_cast<int>(v % CV), q0, q1, q2, q3);
            body(v, q0, q1, q2, q3);
        }
    }
}

struct BnWs {
    float* partials;  // [kMaxRowBlocks][3][C]
    float* c0;        // [C] scale | a
    float* c1;        // [C] shift | b
    float* c2;        // [C] c
    float* c3;        // [C] mean
};

size_t ws_bytes_for(int C) {
    return (size_t(kMaxRowBlocks) * 3 + 4) * size_t(C) * sizeof(float) + 256;
}

BnWs carve(void* ws, int C) {
    char* p = static_cast<char*>(ws);
    BnWs w;
    w.partials = reinterpret_cast<float*>(p);
    w.c0 = w.partials + size_t(kMaxRowBlocks) * 3 * C;
    w.c1 = w.c0 + C;
    w.c2 = w.c1 + C;
    w.c3 = w.c2 + C;
    return w;
}

bool aligned16p(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

template <typename T, bool BWD, int GMODE, bool RELU, bool RES, bool MASK = false>
int launch_elementwise(const T* x, const T* g_in, const T* aux, T* out, int64_t M, int C, const float* p0,
                       const float* p1, const float* p2, const float* p3, hipStream_t st,
                       unsigned char* mask = nullptr) {
    constexpr int N = VecT<T>::N;
    const int CV = C / N;
    const int64_t nvec = M * CV;
    const int64_t per_block = int64_t(kApplyVecs) * kBnThreads;
    const int64_t grid = (nvec + per_block - 1) / per_block;
    if (grid > 0x7fffffffLL) return DAUC_EINVAL;
    if (kBnThreads % CV == 0)
        hipLaunchKernelGGL((bn_elementwise_kernel<T, BWD, GMODE, RELU, RES, true, MASK>), dim3(unsigned(grid)),
                           dim3(kBnThreads), 0, st, x, g_in, aux, out, nvec, CV, p0, p1, p2, p3, mask);
    else
        hipLaunchKernelGGL((bn_elementwise_kernel<T, BWD, GMODE, RELU, RES, false, MASK>), dim3(unsigned(grid)),
                           dim3(kBnThreads), 0, st, x, g_in, aux, out, nvec, CV, p0, p1, p2, p3, mask);
    return launch_status();
}

template <typename T, bool STATS, bool RELU, bool MASK = false>
void launch_partial(int th, const Geometry& g, const T* x, const T* dy, const T* y, T* dz, int64_t M, int C,
                    const float* center, float* partials, hipStream_t st, const unsigned char* mask = nullptr) {
    const dim3 grid(g.nrb, g.ctiles);
    if (th == 1024)
        hipLaunchKernelGGL((bn_partial_kernel<T, STATS, RELU, 1024, MASK>), grid, dim3(1024), 0, st, x, dy, y, dz, M,
                           C, g.CT, g.rows, center, partials, mask);
    else if (th == 512)
        hipLaunchKernelGGL((bn_partial_kernel<T, STATS, RELU, 512, MASK>), grid, dim3(512), 0, st, x, dy, y, dz, M,
                           C, g.CT, g.rows, center, partials, mask);
    else
        hipLaunchKernelGGL((bn_partial_kernel<T, STATS, RELU, 256, MASK>), grid, dim3(256), 0, st, x, dy, y, dz, M,
                           C, g.CT, g.rows, center, partials, mask);
}

template <typename T>
int bn_forward_t(const T* x, int64_t M, int C, const T* res, int relu, const float* gamma, const float* beta,
                 float* running_mean, float* running_var, float momentum, float eps, T* y, unsigned char* mask,
                 float* save_mean, float* save_invstd, void* ws, size_t ws_bytes, hipStream_t st) {
    Geometry g;
    const int th = part_threads();
    if (make_geometry(M, C, sizeof(T), g, th) != DAUC_OK) return DAUC_EINVAL;
    if (ws == nullptr || ws_bytes < ws_bytes_for(C) || !aligned16p(ws)) return DAUC_EINVAL;
    if ((running_mean == nullptr) != (running_var == nullptr)) return DAUC_EINVAL;
    const BnWs w = carve(ws, C);
    launch_partial<T, true, false>(th, g, x, nullptr, nullptr, nullptr, M, C, nullptr, w.partials, st);
    hipLaunchKernelGGL(bn_fwd_finalize_kernel, dim3((C + 63) / 64), dim3(kFinThreads), 0, st, w.partials, g.nrb,
                       g.rows, M, C, gamma, beta, running_mean, running_var, momentum, eps, save_mean, save_invstd, w.c0, w.c1, w.c3);
    int rc = launch_status();
    if (rc != DAUC_OK) return rc;
    if (relu && mask && res)
        return launch_elementwise<T, false, 0, true, true, true>(x, nullptr, res, y, M, C, w.c0, w.c1, nullptr, w.c3, st,
                                                                mask);
    if (relu && mask)
        return launch_elementwise<T, false, 0, true, false, true>(x, nullptr, nullptr, y, M, C, w.c0, w.c1, nullptr,
                                                                 w.c3, st, mask);
    if (relu && res)
        return launch_elementwise<T, false, 0, true, true>(x, nullptr, res, y, M, C, w.c0, w.c1, nullptr, w.c3, st);
    if (relu) return launch_elementwise<T, false, 0, true, false>(x, nullptr, nullptr, y, M, C, w.c0, w.c1, nullptr, w.c3, st);
    if (res) return launch_elementwise<T, false, 0, false, true>(x, nullptr, res, y, M, C, w.c0, w.c1, nullptr, w.c3, st);
    return launch_elementwise<T, false, 0, false, false>(x, nullptr, nullptr, y, M, C, w.c0, w.c1, nullptr, w.c3, st);
}

template <typename T>
int bn_backward_t(const T* dy, const T* y, const unsigned char* mask, const T* x, int64_t M, int C, int relu,
                  const float* gamma, const float* save_mean, const float* save_invstd, T* dres, T* dx, float* dgamma,
                  float* dbeta, void* ws, size_t ws_bytes, hipStream_t st) {
    Geometry g;
    const int th = part_threads();
    if (make_geometry(M, C, sizeof(T), g, th) != DAUC_OK) return DAUC_EINVAL;
    if (ws == nullptr || ws_bytes < ws_bytes_for(C) || !aligned16p(ws)) return DAUC_EINVAL;
    if (relu && y == nullptr && mask == nullptr) return DAUC_EINVAL;
    const BnWs w = carve(ws, C);
    if (relu && mask)
        launch_partial<T, false, true, true>(th, g, x, dy, nullptr, dres, M, C, save_mean, w.partials, st, mask);
    else if (relu)
        launch_partial<T, false, true>(th, g, x, dy, y, dres, M, C, save_mean, w.partials, st);
    else
        launch_partial<T, false, false>(th, g, x, dy, nullptr, dres, M, C, save_mean, w.partials, st);
    hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 63) / 64), dim3(kFinThreads), 0, st, w.partials, g.nrb, M, C,
                       gamma, save_mean, save_invstd, dgamma, dbeta, w.c0, w.c1, w.c2, w.c3);
    int rc = launch_status();
    if (rc != DAUC_OK) return rc;
    if (dres)  // the masked gradient was written once; read it back instead of dy and y
        return launch_elementwise<T, true, 2, false, false>(x, dres, nullptr, dx, M, C, w.c0, w.c1, w.c2, w.c3, st);
    if (relu && mask)
        return launch_elementwise<T, true, 1, false, false, true>(x, dy, nullptr, dx, M, C, w.c0, w.c1, w.c2, w.c3, st,
                                                                 const_cast<unsigned char*>(mask));
    if (relu) return launch_elementwise<T, true, 1, false, false>(x, dy, y, dx, M, C, w.c0, w.c1, w.c2, w.c3, st);
    return launch_elementwise<T, true, 0, false, false>(x, dy, nullptr, dx, M, C, w.c0, w.c1, w.c2, w.c3, st);
}

bool all_aligned(std::initializer_list<const void*> ps) {
    for (const void* p : ps)
        if (p != nullptr && !aligned16p(p)) return false;
    return true;
}

}  // namespace
}  // namespace dauc

using namespace dauc;

extern "C" {

size_t dauc_bn_workspace_size(int64_t M, int C) {
    (void)M;
    return C > 0 ? ws_bytes_for(C) : 0;
}

int dauc_bn_act_forward(const void* x, int dtype, int64_t M, int C, const void* residual, int relu,
                        const float* gamma, const float* beta, float* running_mean, float* running_var,
                        float momentum, float eps, void* y, uint8_t* relu_mask, float* save_mean, float* save_invstd,
                        void* workspace, size_t workspace_bytes, dauc_stream_t stream) {
    if (x == nullptr || y == nullptr || save_mean == nullptr || save_invstd == nullptr) return DAUC_EINVAL;
    if (!all_aligned({x, residual, y})) return DAUC_EINVAL;
    if (relu_mask != nullptr && !relu) return DAUC_EINVAL;
    hipStream_t st = as_hip(stream);
    if (dtype == DAUC_DTYPE_BF16)
        return bn_forward_t(static_cast<const __hip_bfloat16*>(x), M, C, static_cast<const __hip_bfloat16*>(residual),
                            relu, gamma, beta, running_mean, running_var, momentum, eps,
                            static_cast<__hip_bfloat16*>(y), relu_mask, save_mean, save_invstd, workspace,
                            workspace_bytes, st);
    if (dtype == DAUC_DTYPE_F32)
        return bn_forward_t(static_cast<const float*>(x), M, C, static_cast<const float*>(residual), relu, gamma,
                            beta, running_mean, running_var, momentum, eps, static_cast<float*>(y), relu_mask,
                            save_mean, save_invstd, workspace, workspace_bytes, st);
    return DAUC_EINVAL;
}

int dauc_bn_act_backward(const void* dy, const void* y, const uint8_t* relu_mask, const void* x, int dtype, int64_t M,
                         int C, int relu, const float* gamma, const float* save_mean, const float* save_invstd,
                         void* dres, void* dx, float* dgamma, float* dbeta, void* workspace, size_t workspace_bytes,
                         dauc_stream_t stream) {
    if (dy == nullptr || x == nullptr || dx == nullptr || save_mean == nullptr || save_invstd == nullptr)
        return DAUC_EINVAL;
    if (!all_aligned({dy, y, x, dres, dx})) return DAUC_EINVAL;
    hipStream_t st = as_hip(stream);
    if (dtype == DAUC_DTYPE_BF16)
        return bn_backward_t(static_cast<const __hip_bfloat16*>(dy), static_cast<const __hip_bfloat16*>(y), relu_mask,
                             static_cast<const __hip_bfloat16*>(x), M, C, relu, gamma, save_mean, save_invstd,
                             static_cast<__hip_bfloat16*>(dres), static_cast<__hip_bfloat16*>(dx), dgamma, dbeta,
                             workspace, workspace_bytes, st);
    if (dtype == DAUC_DTYPE_F32)
        return bn_backward_t(static_cast<const float*>(dy), static_cast<const float*>(y), relu_mask,
                             static_cast<const float*>(x), M, C, relu, gamma, save_mean, save_invstd,
                             static_cast<float*>(dres), static_cast<float*>(dx), dgamma, dbeta, workspace,
                             workspace_bytes, st);
    return DAUC_EINVAL;
}

}  // extern "C"
