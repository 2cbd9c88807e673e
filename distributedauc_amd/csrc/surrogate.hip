// Fused min-max square-loss AUC surrogate (forward + backward in one pass),
// the per-batch label map / p_hat, and the stage-start class sums.
//
// Reference: imagenet/main.py:303-317 (label map, counts, p_hat, inline loss),
// main.py:326 (its autograd backward) and main.py:166-197 (alpha estimate).
//
// HBM layout: h is read with an element stride (2 when it is column 1 of the
// [B,2] softmax output), labels are int8 (+1/-1) on the fast path, dF/dh is
// written once. Algorithmic traffic: 4 (h) + 1 (int8 y) + 4 (dh) = 9 B/element.
// Per 4-element slot the fp32 partials of sum(h-a), sum(h-b), sum((h-a)^2),
// sum((h-b)^2) are folded into fp64; with the two class counts they are reduced
// wave -> block -> grid in a fixed order, so results are bitwise reproducible.
//
// Two geometries: unit-stride batches >= 2^22 (the streaming size) take ONE launch of
// surrogate_tail_kernel — one 4096-element chunk per workgroup, rows handed to the last 64
// workgroups as data-as-flag words, which reduce them (see the comment at that kernel); smaller
// or strided batches (training, B = 256) take the persistent kernel with one last-arriver
// ticket. The other kernels below are tuning variants kept measurable through
// dauc_surrogate_fwdbwd_variant (include/dauc.h).

#include <hip/hip_bf16.h>

#include "dauc_internal.h"

namespace dauc {
namespace {

constexpr int kThreads = 256;
constexpr int kVec = 4;                                // elements per float4 slot
// Geometry from the MI355X sweep (scripts/gpu_sweep_sur.sh, profiles/r01): 8 float4
// slots per thread and 2 resident blocks per CU stream best (a narrow, deep window;
// more resident blocks lose DRAM locality).
#ifndef DAUC_SURROGATE_SLOTS
#define DAUC_SURROGATE_SLOTS 8
#endif
#ifndef DAUC_SURROGATE_BPC
#define DAUC_SURROGATE_BPC 2
#endif
constexpr int kSlots = DAUC_SURROGATE_SLOTS;           // float4 slots per thread per iteration
#ifndef DAUC_SURROGATE_NTSTORE
#define DAUC_SURROGATE_NTSTORE 1
#endif
constexpr int kMaxBlocks = 2048;                       // partial slots in the workspace
constexpr int kPerBlockIter = kThreads * kVec * kSlots;  // 8192 elements
constexpr int kNumAcc = 6;                             // fp64 partials per thread / block
constexpr size_t kCounterBytes = 256;                  // counter padded to its own lines

// Accumulators. H_pos / H_neg are not accumulated: H = S + a * n (exact in fp64
// to ~1e-16 relative), reconstructed once in finalize().
//   S_POS = sum_pos (h - a)      Q_POS = sum_pos (h - a)^2     N_POS = #pos
//   S_NEG = sum_neg (h - b)      Q_NEG = sum_neg (h - b)^2     N_NEG = #neg
enum { S_POS = 0, S_NEG, Q_POS, Q_NEG, N_POS, N_NEG };

// Resident-block capacity of the device for the surrogate kernel (queried once, cached):
// a grid of exactly that many blocks has no partially filled last wave.
int resident_blocks();

// grid of the one-element-per-thread logits kernel (never smaller than grid_for)
int grid_scalar(int64_t B) {
    int64_t g = (B + kThreads - 1) / kThreads;
    const int64_t cap = resident_blocks();
    if (g > cap) g = cap;
    if (g < 1) g = 1;
    if (g > kMaxBlocks) g = kMaxBlocks;
    return static_cast<int>(g);
}

int grid_for(int64_t B) {
    int64_t g = (B + kPerBlockIter - 1) / kPerBlockIter;
    const int64_t cap = resident_blocks();
    if (g > cap) g = cap;
    if (g < 1) g = 1;
    if (g > kMaxBlocks) g = kMaxBlocks;
    return static_cast<int>(g);
}

template <typename YT>
__device__ __forceinline__ int load_label(const YT* __restrict__ y, int64_t i) {
    return static_cast<int>(y[i]);
}

struct SurrogateScalars {
    double a, b, alpha, p;
    float af, bf;          // fp32 copies for the per-element differences
    float c_pos, k_pos;    // dF/dh = c_pos * (h - k_pos) for y = +1
    float c_neg, k_neg;    // dF/dh = c_neg * (h - k_neg) for y = -1
};

__device__ __forceinline__ SurrogateScalars make_scalars_v(float a, float b, float alpha, float p, double invB) {
    SurrogateScalars s;
    s.af = a;
    s.bf = b;
    s.a = s.af;
    s.b = s.bf;
    s.alpha = alpha;
    s.p = p;
    s.c_pos = static_cast<float>(2.0 * (1.0 - s.p) * invB);
    s.k_pos = static_cast<float>(s.a + 1.0 + s.alpha);
    s.c_neg = static_cast<float>(2.0 * s.p * invB);
    s.k_neg = static_cast<float>(s.b - 1.0 - s.alpha);
    return s;
}

__device__ __forceinline__ SurrogateScalars make_scalars(const float* abalpha, const float* p_hat, double invB) {
    return make_scalars_v(abalpha[0], abalpha[1], abalpha[2], p_hat[0], invB);
}

// Per-thread state: fp32 partials over one float4 slot, folded into fp64 per slot.
struct Acc {
    double s_pos = 0.0, s_neg = 0.0, q_pos = 0.0, q_neg = 0.0;
    int n_pos = 0, n_neg = 0;
};

// One float4 slot: accumulate and return dF/dh for its four elements.
template <bool CLASS_ONLY>
__device__ __forceinline__ f32x4 visit4(f32x4 h, const int (&yv)[4], const SurrogateScalars& s,
                                        Acc& acc) {
    float sp = 0.f, sn = 0.f, qp = 0.f, qn = 0.f;
    f32x4 g;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const bool pos = (yv[c] == 1);
        const bool neg = (yv[c] == -1);
        const float dp = pos ? h[c] - s.af : 0.f;
        const float dn = neg ? h[c] - s.bf : 0.f;
        sp += dp;
        sn += dn;
        if (!CLASS_ONLY) {
            qp += dp * dp;
            qn += dn * dn;
        }
        acc.n_pos += pos;
        acc.n_neg += neg;
        if (!CLASS_ONLY) {
            const float cc = pos ? s.c_pos : (neg ? s.c_neg : 0.f);
            const float kk = pos ? s.k_pos : s.k_neg;
            g[c] = cc * (h[c] - kk);
        }
    }
    acc.s_pos += sp;
    acc.s_neg += sn;
    if (!CLASS_ONLY) {
        acc.q_pos += qp;
        acc.q_neg += qn;
    }
    return g;
}

// Final scalars from the grid totals (one thread).
__device__ void finalize(const double (&t)[kNumAcc], const SurrogateScalars& s, double invB,
                         double* out64, float* grad3, float* loss) {
    const double p = s.p, q = 1.0 - s.p;
    const double h_pos = t[S_POS] + s.a * t[N_POS];
    const double h_neg = t[S_NEG] + s.b * t[N_NEG];
    const double cross = p * h_neg - q * h_pos;  // sum(p h [neg] - (1-p) h [pos])
    const double F = q * t[Q_POS] * invB + p * t[Q_NEG] * invB +
                     2.0 * (1.0 + s.alpha) * cross * invB - p * q * s.alpha * s.alpha;
    const double dA = -2.0 * q * t[S_POS] * invB;
    const double dB = -2.0 * p * t[S_NEG] * invB;
    const double dAl = 2.0 * cross * invB - 2.0 * p * q * s.alpha;
    if (out64) {
        out64[0] = F;
        out64[1] = dA;
        out64[2] = dB;
        out64[3] = dAl;
        out64[4] = t[N_POS];
        out64[5] = t[N_NEG];
    }
    if (grad3) {
        grad3[0] = static_cast<float>(dA);
        grad3[1] = static_cast<float>(dB);
        grad3[2] = static_cast<float>(dAl);
    }
    if (loss) loss[0] = static_cast<float>(F);
}

// class sums (a = b = 0 there, so S_* are the plain score sums)
__device__ void emit_class_sums(const double (&t)[kNumAcc], double* sums4, int accumulate) {
    const double v[4] = {t[S_NEG], t[N_NEG], t[S_POS], t[N_POS]};
    for (int k = 0; k < 4; ++k) sums4[k] = accumulate ? sums4[k] + v[k] : v[k];
}

template <typename YT>
__device__ __forceinline__ void load_labels4(const YT* __restrict__ y, int64_t base, int (&yv)[4]) {
    if constexpr (sizeof(YT) == 1) {
        const char4 c = *reinterpret_cast<const char4*>(y + base);
        yv[0] = c.x;
        yv[1] = c.y;
        yv[2] = c.z;
        yv[3] = c.w;
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) yv[j] = load_label(y, base + j);
    }
}

// Block reduction, then the grid reduction by the last-arriving block, then the
// final scalars. Every block of the grid calls this exactly once.
template <bool CLASS_ONLY>
__device__ __forceinline__ void reduce_and_finalize(const Acc& acc, const SurrogateScalars& s, double invB,
                                                    double* __restrict__ partials,
                                                    unsigned* __restrict__ counter,
                                                    double* __restrict__ out64, float* __restrict__ grad3,
                                                    float* __restrict__ loss, double* __restrict__ sums4,
                                                    int accumulate) {
    __shared__ double scratch[kNumAcc * (kThreads / kWave)];
    __shared__ int last_flag;
    double tot[kNumAcc] = {acc.s_pos, acc.s_neg, acc.q_pos, acc.q_neg,
                           static_cast<double>(acc.n_pos), static_cast<double>(acc.n_neg)};
    block_sum<kNumAcc>(tot, scratch);

    if (gridDim.x == 1) {
        if (threadIdx.x == 0) {
            if (CLASS_ONLY) emit_class_sums(tot, sums4, accumulate);
            else finalize(tot, s, invB, out64, grad3, loss);
        }
        return;
    }

    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < kNumAcc; ++k) store_sc1(&partials[blockIdx.x * kNumAcc + k], tot[k]);
    }
    if (!arrive_last(counter, gridDim.x, &last_flag)) return;

    // Last block: reduce all partials in a fixed order.
#pragma unroll
    for (int k = 0; k < kNumAcc; ++k) tot[k] = 0.0;
    for (int b = threadIdx.x; b < static_cast<int>(gridDim.x); b += kThreads) {
#pragma unroll
        for (int k = 0; k < kNumAcc; ++k) {
            tot[k] += load_sc1(&partials[b * kNumAcc + k]);
            partials[b * kNumAcc + k] = 0.0;  // the workspace is left zeroed (dauc.h)
        }
    }
    block_sum<kNumAcc>(tot, scratch);
    if (threadIdx.x == 0) {
        if (CLASS_ONLY) emit_class_sums(tot, sums4, accumulate);
        else finalize(tot, s, invB, out64, grad3, loss);
    }
}

// One element: accumulate its contribution (per-element fp64 folding) and return dF/dh.
template <bool CLASS_ONLY>
__device__ __forceinline__ float visit1(float hv, int yv, const SurrogateScalars& s, Acc& acc) {
    const bool pos = (yv == 1), neg = (yv == -1);
    const float dp = pos ? hv - s.af : 0.f;
    const float dn = neg ? hv - s.bf : 0.f;
    acc.s_pos += dp;
    acc.s_neg += dn;
    if (!CLASS_ONLY) {
        acc.q_pos += dp * dp;
        acc.q_neg += dn * dn;
    }
    acc.n_pos += pos;
    acc.n_neg += neg;
    if (CLASS_ONLY) return 0.f;
    const float cc = pos ? s.c_pos : (neg ? s.c_neg : 0.f);
    const float kk = pos ? s.k_pos : s.k_neg;
    return cc * (hv - kk);
}

__device__ __forceinline__ float to_f32(float v) { return v; }
__device__ __forceinline__ float to_f32(__hip_bfloat16 v) { return __bfloat162float(v); }
template <typename ZT>
__device__ __forceinline__ ZT from_f32(float v);
template <>
__device__ __forceinline__ float from_f32<float>(float v) { return v; }
template <>
__device__ __forceinline__ __hip_bfloat16 from_f32<__hip_bfloat16>(float v) { return __float2bfloat16(v); }

// the loss straight from the 2-way logits z [B, 2] (row stride ldz):
// h = softmax(z)[:, 1] = 1 / (1 + exp(z0 - z1)) in fp32, and the backward through the
// softmax column is fused: dF/dz1 = dF/dh * h * (1 - h), dF/dz0 = -dF/dz1 (resnet.py:218).
// h_out (nullable) receives h in fp32.
template <typename ZT, typename YT, bool CLASS_ONLY>
__global__ __launch_bounds__(kThreads) void surrogate_logits_kernel(
    const ZT* __restrict__ z, int64_t ldz, const YT* __restrict__ y, int64_t B, double invB,
    const float* __restrict__ abalpha, const float* __restrict__ p_hat, ZT* __restrict__ dz, int64_t lddz,
    float* __restrict__ h_out, double* __restrict__ partials, unsigned* __restrict__ counter,
    double* __restrict__ out64, float* __restrict__ grad3, float* __restrict__ loss,
    double* __restrict__ sums4, int accumulate) {
    SurrogateScalars s;
    if (CLASS_ONLY) s = SurrogateScalars{};
    else s = make_scalars(abalpha, p_hat, invB);
    Acc acc;
    for (int64_t i = int64_t(blockIdx.x) * kThreads + threadIdx.x; i < B; i += int64_t(gridDim.x) * kThreads) {
        const float z0 = to_f32(z[i * ldz]);
        const float z1 = to_f32(z[i * ldz + 1]);
        const float h = 1.0f / (1.0f + expf(z0 - z1));
        if (h_out) h_out[i] = h;
        const float g = visit1<CLASS_ONLY>(h, load_label(y, i), s, acc);
        if (!CLASS_ONLY && dz) {
            const float gz = g * h * (1.0f - h);
            dz[i * lddz] = from_f32<ZT>(-gz);
            dz[i * lddz + 1] = from_f32<ZT>(gz);
        }
    }
    reduce_and_finalize<CLASS_ONLY>(acc, s, invB, partials, counter, out64, grad3, loss, sums4, accumulate);
}

// UNIT: h, y and dh are unit-stride and 4-element aligned (vector loads/stores).
template <typename YT, bool CLASS_ONLY, bool UNIT>
__global__ __launch_bounds__(kThreads) void surrogate_kernel(
    const float* __restrict__ h, int64_t hs, const YT* __restrict__ y, int64_t B, double invB,
    const float* __restrict__ abalpha, const float* __restrict__ p_hat, float* __restrict__ dh,
    int64_t dhs, double* __restrict__ partials, unsigned* __restrict__ counter,
    double* __restrict__ out64, float* __restrict__ grad3, float* __restrict__ loss,
    double* __restrict__ sums4, int accumulate) {
    SurrogateScalars s;
    if (CLASS_ONLY) {
        s = SurrogateScalars{};
    } else {
        s = make_scalars(abalpha, p_hat, invB);
    }
    Acc acc;
    const bool write_dh = !CLASS_ONLY && dh != nullptr;

    // 1) vector path: whole block-iterations of kPerBlockIter elements, every slot in range
    int64_t done = 0;
    if (UNIT) {
        const int64_t n_iter = B / kPerBlockIter;
        for (int64_t it = blockIdx.x; it < n_iter; it += gridDim.x) {
            const int64_t base = it * kPerBlockIter + threadIdx.x * kVec;
            f32x4 hv[kSlots];
            int yv[kSlots][4];
#pragma unroll
            for (int k = 0; k < kSlots; ++k) {
                const int64_t b = base + int64_t(k) * kThreads * kVec;
                hv[k] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(h + b));
                load_labels4(y, b, yv[k]);
            }
#pragma unroll
            for (int k = 0; k < kSlots; ++k) {
                const f32x4 g = visit4<CLASS_ONLY>(hv[k], yv[k], s, acc);
                if (write_dh) {
                    f32x4* dst = reinterpret_cast<f32x4*>(dh + base + int64_t(k) * kThreads * kVec);
                    if (DAUC_SURROGATE_NTSTORE) __builtin_nontemporal_store(g, dst);
                    else *dst = g;
                }
            }
        }
        done = n_iter * kPerBlockIter;
    }
    // 2) scalar path: the tail of a unit-stride batch, or all of a strided one (training
    //    batches: column 1 of the [B,2] softmax). One element per thread per step.
    {
        for (int64_t i = done + int64_t(blockIdx.x) * kThreads + threadIdx.x; i < B;
             i += int64_t(gridDim.x) * kThreads) {
            const float g = visit1<CLASS_ONLY>(h[i * hs], load_label(y, i), s, acc);
            if (write_dh) dh[i * dhs] = g;
        }
    }

    reduce_and_finalize<CLASS_ONLY>(acc, s, invB, partials, counter, out64, grad3, loss, sums4, accumulate);
}

// ---- large unit-stride batches: one chunk per workgroup + a separate row reduction -------
//
// A grid-stride (persistent) loop walks the batch with a large stride, so concurrently open
// DRAM pages are far apart (measured: 6.2 TB/s for this 5:4 read:write mix vs 6.5 TB/s for
// one chunk per workgroup, scripts/probe_stream.hip). Here every workgroup takes ONE
// contiguous chunk of 256 x 4 x S elements (the dispatcher hands chunks out roughly in
// address order, like the update kernel's one-shot grid) and issues all of its loads
// before any math.
//
// No workgroup of the streaming launch waits for anything: every WAVE reduces its 6
// partials with DPP (no barrier, no LDS) and its lane 63 stores them as one 48-B row with
// plain 16-B stores, then the wave stores dF/dh and exits. A second, small launch reduces
// the rows (the kernel boundary publishes them). Measured on MI355X at B = 2^26: any
// in-launch hand-off stalls the stream -- a per-workgroup ticket (barrier + row drain +
// returning atomic) cost ~18 % (110 us), last-arriver spinners polling rows ~35 % (128 us),
// because under a full streaming load every round trip to memory queues behind ~70 MB of
// loads in flight (10-20 us per hop, scripts/probe_sur_timeline.py); the wait-free stream
// runs at the streaming ceiling of this access mix (93 us). Fixed summation orders
// everywhere: bitwise reproducible.
constexpr int kWaves = kThreads / kWave;          // waves per workgroup
// 1: one row per wave (no barrier in the stream kernel), 0: one row per workgroup
#ifndef DAUC_SURROGATE_WAVE_ROWS
#define DAUC_SURROGATE_WAVE_ROWS 0
#endif
constexpr int64_t kRowsPerChunk = DAUC_SURROGATE_WAVE_ROWS ? kWaves : 1;
constexpr int kRowWords = 6;                      // s_pos, s_neg, q_pos, q_neg, n_pos, n_neg (fp64)
#ifndef DAUC_SURROGATE_REDUCE_ROWS
#define DAUC_SURROGATE_REDUCE_ROWS 512
#endif
constexpr int kRowsPerReduceBlock = DAUC_SURROGATE_REDUCE_ROWS;  // rows one workgroup of the reduce kernel sums
static_assert(kRowsPerReduceBlock % 256 == 0, "whole rows per thread");

__host__ __device__ constexpr int64_t chunk_elems(int S) { return int64_t(kThreads) * kVec * S; }

inline int64_t reduce_blocks(int64_t nrows) { return (nrows + kRowsPerReduceBlock - 1) / kRowsPerReduceBlock; }

// Workspace layout: [persistent kernel: ticket + kMaxBlocks rows][chunk rows][reduce hand-off words].
constexpr size_t kPersistentBytes = kCounterBytes + size_t(kMaxBlocks) * kNumAcc * sizeof(double);

inline size_t chunk_ws_bytes(int64_t nblocks) {
    const int64_t nrows = nblocks * kRowsPerChunk;
    return kPersistentBytes + static_cast<size_t>(nrows + reduce_blocks(nrows)) * kRowWords * sizeof(double);
}

struct ChunkWs {
    double* rows;      // [nblocks * kRowsPerChunk][kRowWords]
    double* brows;     // [reduce blocks][kRowWords] encoded hand-off words (zero between calls)
};

inline ChunkWs chunk_ws(void* ws, int64_t nblocks) {
    ChunkWs w;
    w.rows = reinterpret_cast<double*>(static_cast<char*>(ws) + kPersistentBytes);
    w.brows = w.rows + nblocks * kRowsPerChunk * kRowWords;
    return w;
}

// One DPP step: the value of the source lane selected by CTRL (0 where ROWMASK disables the row).
template <int CTRL, int ROWMASK>
__device__ __forceinline__ double dpp_f64(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, static_cast<int>(b), CTRL, ROWMASK, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, static_cast<int>(b >> 32), CTRL, ROWMASK, 0xF, false);
    return __longlong_as_double((static_cast<long long>(hi) << 32) | static_cast<unsigned>(lo));
}

template <int CTRL, int ROWMASK>
__device__ __forceinline__ int dpp_i32(int v) {
    return __builtin_amdgcn_update_dpp(0, v, CTRL, ROWMASK, 0xF, false);
}

// Wave sum in a fixed order; the total is valid in lane 63:
// quad_perm[1,0,3,2], quad_perm[2,3,0,1], row_half_mirror, row_mirror (16-lane row sums in
// every lane), row_bcast:15 into rows 1 and 3, row_bcast:31 into rows 2 and 3.
__device__ __forceinline__ double wave_total_dpp(double v) {
    v += dpp_f64<0xB1, 0xF>(v);
    v += dpp_f64<0x4E, 0xF>(v);
    v += dpp_f64<0x141, 0xF>(v);
    v += dpp_f64<0x140, 0xF>(v);
    v += dpp_f64<0x142, 0xA>(v);
    v += dpp_f64<0x143, 0xC>(v);
    return v;
}

__device__ __forceinline__ int wave_total_dpp(int v) {
    v += dpp_i32<0xB1, 0xF>(v);
    v += dpp_i32<0x4E, 0xF>(v);
    v += dpp_i32<0x141, 0xF>(v);
    v += dpp_i32<0x140, 0xF>(v);
    v += dpp_i32<0x142, 0xA>(v);
    v += dpp_i32<0x143, 0xC>(v);
    return v;
}

template <typename YT, bool CLASS_ONLY, int S, bool NT_LOAD, bool NT_STORE>
__global__ __launch_bounds__(kThreads) void surrogate_chunk_kernel(
    const float* __restrict__ h, const YT* __restrict__ y, int64_t B, double invB,
    const float* __restrict__ abalpha, const float* __restrict__ p_hat, float* __restrict__ dh,
    double* __restrict__ rows) {
    SurrogateScalars s;
    if (CLASS_ONLY) s = SurrogateScalars{};
    else s = make_scalars(abalpha, p_hat, invB);
    Acc acc;
    const bool write_dh = !CLASS_ONLY && dh != nullptr;
    const int64_t base = int64_t(blockIdx.x) * chunk_elems(S);
    const bool full = base + chunk_elems(S) <= B;

    f32x4 hv[S];
    if (full) {
        int yv[S][4];
#pragma unroll
        for (int k = 0; k < S; ++k) {
            const int64_t b = base + (int64_t(k) * kThreads + threadIdx.x) * kVec;
            if (NT_LOAD) hv[k] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(h + b));
            else hv[k] = *reinterpret_cast<const f32x4*>(h + b);
            load_labels4(y, b, yv[k]);
        }
#pragma unroll
        for (int k = 0; k < S; ++k) hv[k] = visit4<CLASS_ONLY>(hv[k], yv[k], s, acc);
    } else {
        // the ragged last chunk: one element per thread per step
        for (int64_t i = base + threadIdx.x; i < B; i += kThreads) {
            const float g = visit1<CLASS_ONLY>(h[i], load_label(y, i), s, acc);
            if (write_dh) dh[i] = g;
        }
    }

    // Wave totals by DPP (lane 63), then the dF/dh stores, then ONE row per workgroup: the
    // barrier comes after every store of the chunk has been issued, so no wave holds its
    // stores back for it (stores need not complete before a barrier).
    const double sp = wave_total_dpp(acc.s_pos), sn = wave_total_dpp(acc.s_neg);
    const double qp = wave_total_dpp(acc.q_pos), qn = wave_total_dpp(acc.q_neg);
    const int np = wave_total_dpp(acc.n_pos), nn = wave_total_dpp(acc.n_neg);
#if DAUC_SURROGATE_WAVE_ROWS
    if ((threadIdx.x & (kWave - 1)) == kWave - 1) {
        typedef double f64x2 __attribute__((ext_vector_type(2)));
        f64x2* row = reinterpret_cast<f64x2*>(rows + (int64_t(blockIdx.x) * kWaves + threadIdx.x / kWave) * kRowWords);
        row[0] = f64x2{sp, sn};
        row[1] = f64x2{qp, qn};
        row[2] = f64x2{static_cast<double>(np), static_cast<double>(nn)};
    }
#endif
    if (full && write_dh) {
#pragma unroll
        for (int k = 0; k < S; ++k) {
            f32x4* dst = reinterpret_cast<f32x4*>(dh + base + (int64_t(k) * kThreads + threadIdx.x) * kVec);
            if (NT_STORE) __builtin_nontemporal_store(hv[k], dst);
            else *dst = hv[k];
        }
    }
#if !DAUC_SURROGATE_WAVE_ROWS
    __shared__ double wrow[kWaves][kRowWords];
    const int wid = threadIdx.x / kWave;
    if ((threadIdx.x & (kWave - 1)) == kWave - 1) {
        wrow[wid][0] = sp;
        wrow[wid][1] = sn;
        wrow[wid][2] = qp;
        wrow[wid][3] = qn;
        wrow[wid][4] = static_cast<double>(np);
        wrow[wid][5] = static_cast<double>(nn);
    }
    __syncthreads();
    if (threadIdx.x < kRowWords) {
        const int k = threadIdx.x;
        rows[int64_t(blockIdx.x) * kRowWords + k] = ((wrow[0][k] + wrow[1][k]) + wrow[2][k]) + wrow[3][k];
    }
#endif
}

// The same stream with SPAN consecutive chunks per workgroup (one contiguous span of
// SPAN x 4096 elements): the chunk after the current one is loaded while the current one is
// reduced and stored (two chunks of loads in flight per thread), and the launch writes SPAN
// times fewer rows, so the row reduce shrinks to one workgroup (<= 512 rows) with no hand-off.
// Only whole spans; the ragged tail (< SPAN chunks) is handled element-wise by the last
// workgroup.
template <typename YT, bool CLASS_ONLY, int S, int SPAN>
__global__ __launch_bounds__(kThreads) void surrogate_span_kernel(
    const float* __restrict__ h, const YT* __restrict__ y, int64_t B, double invB,
    const float* __restrict__ abalpha, const float* __restrict__ p_hat, float* __restrict__ dh,
    double* __restrict__ rows) {
    SurrogateScalars s;
    if (CLASS_ONLY) s = SurrogateScalars{};
    else s = make_scalars(abalpha, p_hat, invB);
    Acc acc;
    const bool write_dh = !CLASS_ONLY && dh != nullptr;
    constexpr int64_t kChunk = chunk_elems(S);
    const int64_t base = int64_t(blockIdx.x) * SPAN * kChunk;
    const int64_t whole = B / (SPAN * kChunk);  // workgroups with a full span
    if (int64_t(blockIdx.x) < whole) {
        f32x4 cur[S], nxt[S];
        int ycur[S][4], ynxt[S][4];
#pragma unroll
        for (int k = 0; k < S; ++k) {
            const int64_t b = base + (int64_t(k) * kThreads + threadIdx.x) * kVec;
            cur[k] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(h + b));
            load_labels4(y, b, ycur[k]);
        }
        for (int c = 0; c < SPAN; ++c) {
            const int64_t cb = base + c * kChunk;
            if (c + 1 < SPAN) {
#pragma unroll
                for (int k = 0; k < S; ++k) {
                    const int64_t b = cb + kChunk + (int64_t(k) * kThreads + threadIdx.x) * kVec;
                    nxt[k] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(h + b));
                    load_labels4(y, b, ynxt[k]);
                }
            }
#pragma unroll
            for (int k = 0; k < S; ++k) {
                const f32x4 g = visit4<CLASS_ONLY>(cur[k], ycur[k], s, acc);
                if (write_dh)
                    __builtin_nontemporal_store(
                        g, reinterpret_cast<f32x4*>(dh + cb + (int64_t(k) * kThreads + threadIdx.x) * kVec));
            }
#pragma unroll
            for (int k = 0; k < S; ++k) {
                cur[k] = nxt[k];
#pragma unroll
                for (int q = 0; q < 4; ++q) ycur[k][q] = ynxt[k][q];
            }
        }
    } else {
        // after the whole spans: one chunk per workgroup (vector path), the ragged last chunk
        // element-wise
        const int64_t cb = whole * SPAN * kChunk + (int64_t(blockIdx.x) - whole) * kChunk;
        if (cb + kChunk <= B) {
#pragma unroll
            for (int k = 0; k < S; ++k) {
                const int64_t b = cb + (int64_t(k) * kThreads + threadIdx.x) * kVec;
                int yv[4];
                load_labels4(y, b, yv);
                const f32x4 g = visit4<CLASS_ONLY>(
                    __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(h + b)), yv, s, acc);
                if (write_dh) __builtin_nontemporal_store(g, reinterpret_cast<f32x4*>(dh + b));
            }
        } else {
            for (int64_t i = cb + threadIdx.x; i < B; i += kThreads) {
                const float g = visit1<CLASS_ONLY>(h[i], load_label(y, i), s, acc);
                if (write_dh) dh[i] = g;
            }
        }
    }
    const double sp = wave_total_dpp(acc.s_pos), sn = wave_total_dpp(acc.s_neg);
    const double qp = wave_total_dpp(acc.q_pos), qn = wave_total_dpp(acc.q_neg);
    const int np = wave_total_dpp(acc.n_pos), nn = wave_total_dpp(acc.n_neg);
    __shared__ double wrow[kWaves][kRowWords];
    const int wid = threadIdx.x / kWave;
    if ((threadIdx.x & (kWave - 1)) == kWave - 1) {
        wrow[wid][0] = sp;
        wrow[wid][1] = sn;
        wrow[wid][2] = qp;
        wrow[wid][3] = qn;
        wrow[wid][4] = static_cast<double>(np);
        wrow[wid][5] = static_cast<double>(nn);
    }
    __syncthreads();
    if (threadIdx.x < kRowWords) {
        const int k = threadIdx.x;
        rows[int64_t(blockIdx.x) * kRowWords + k] = ((wrow[0][k] + wrow[1][k]) + wrow[2][k]) + wrow[3][k];
    }
}

// Reduce the streaming launch's rows (the kernel boundary published them): workgroup b sums
// rows [512 b, 512 (b + 1)) in a fixed order (thread t: rows t, t + 256). Workgroups b > 0
// hand their 6 totals to workgroup 0 as encoded 8-B words stored write-through (sc1): a word
// is bits ^ kEmptyKey, a signalling-NaN pattern no arithmetic result or count can equal, so a
// zero word means "not written yet" (cdna_hip_programming.md Guideline 16, R2: the data is
// the flag, no drain, no ticket). Workgroup 0 polls those words with sc1 loads (bounded; a
// timeout yields NaN outputs), sums them in a fixed order, zeroes them again for the next
// call, and writes the scalars. The grid is small (<= 64 workgroups up to B = 2^27) and
// workgroup 0 is the only one that waits, so every workgroup it waits for can run.
constexpr unsigned long long kEmptyKey = 0x7FF4DEADBEEF0001ull;  // signalling NaN
constexpr int kMaxPolls = 1 << 22;

__device__ __forceinline__ unsigned long long enc_word(double v) {
    return static_cast<unsigned long long>(__double_as_longlong(v)) ^ kEmptyKey;
}

template <bool CLASS_ONLY>
__global__ __launch_bounds__(kThreads) void surrogate_rows_reduce_kernel(
    double* __restrict__ rows, int64_t nrows, ChunkWs ws, double invB, const float* __restrict__ abalpha,
    const float* __restrict__ p_hat, double* __restrict__ out64, float* __restrict__ grad3, float* __restrict__ loss,
    double* __restrict__ sums4, int accumulate) {
    __shared__ double scratch[kNumAcc * kWaves];
    // Workgroup 0's scalar inputs are read up front: after the hand-off they would be one more
    // dependent round trip to memory at the very end of the call.
    __shared__ int bad;
    if (threadIdx.x == 0) bad = 0;  // ordered before any write by block_sum's barriers
    float sc[4] = {0.f, 0.f, 0.f, 0.f};
    if (!CLASS_ONLY && blockIdx.x == 0) {
        sc[0] = abalpha[0];
        sc[1] = abalpha[1];
        sc[2] = abalpha[2];
        sc[3] = p_hat[0];
    }
    double tot[kNumAcc];
#pragma unroll
    for (int k = 0; k < kNumAcc; ++k) tot[k] = 0.0;
    const int64_t r0 = int64_t(blockIdx.x) * kRowsPerReduceBlock;
    const int64_t r1 = (r0 + kRowsPerReduceBlock < nrows) ? r0 + kRowsPerReduceBlock : nrows;
    // all of a thread's rows in flight at once (rows t, t + 256, ...: a fixed order)
    typedef double f64x2 __attribute__((ext_vector_type(2)));
    constexpr int kPer = kRowsPerReduceBlock / kThreads;
    f64x2 v[kPer][3];
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
        const int64_t r = r0 + threadIdx.x + int64_t(j) * kThreads;
#pragma unroll
        for (int q = 0; q < 3; ++q)
            v[j][q] = r < r1 ? reinterpret_cast<const f64x2*>(rows + r * kRowWords)[q] : f64x2{0.0, 0.0};
    }
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            tot[2 * q] += v[j][q].x;
            tot[2 * q + 1] += v[j][q].y;
        }
    }
    block_sum<kNumAcc>(tot, scratch);
    // The rows are zeroed again for the next call only after the totals are on their way:
    // stores count in vmcnt, so zeroing before the sums would put their write acks on the
    // critical path.
    auto zero_rows = [&]() {
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
            const int64_t r = r0 + threadIdx.x + int64_t(j) * kThreads;
            if (r < r1) {
#pragma unroll
                for (int q = 0; q < 3; ++q) reinterpret_cast<f64x2*>(rows + r * kRowWords)[q] = f64x2{0.0, 0.0};
            }
        }
    };
    unsigned long long* words = reinterpret_cast<unsigned long long*>(ws.brows);
    if (blockIdx.x > 0) {
        if (threadIdx.x == 0) {
#pragma unroll
            for (int k = 0; k < kNumAcc; ++k)
                __hip_atomic_store((gu64*)(words + int64_t(blockIdx.x) * kRowWords + k), enc_word(tot[k]),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        zero_rows();
        return;
    }
    zero_rows();
    bool ok = true;
    if (gridDim.x > 1) {
        double rest[kNumAcc];
#pragma unroll
        for (int k = 0; k < kNumAcc; ++k) rest[k] = 0.0;
        for (int b = 1 + threadIdx.x; b < static_cast<int>(gridDim.x); b += kThreads) {
            unsigned long long* row = words + int64_t(b) * kRowWords;
            unsigned long long w[kRowWords];
#pragma unroll
            for (int k = 0; k < kRowWords; ++k)
                w[k] = __hip_atomic_load((gu64*)(row + k), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            for (int polls = 0;; ++polls) {
                bool missing = false;
#pragma unroll
                for (int k = 0; k < kRowWords; ++k) missing |= (w[k] == 0ull);
                if (!missing) break;
                if (polls >= kMaxPolls) {
                    ok = false;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
#pragma unroll
                for (int k = 0; k < kRowWords; ++k)
                    if (w[k] == 0ull)
                        w[k] = __hip_atomic_load((gu64*)(row + k), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
#pragma unroll
            for (int k = 0; k < kRowWords; ++k) {
                rest[k] += __longlong_as_double(static_cast<long long>(w[k] ^ kEmptyKey));
                __hip_atomic_store((gu64*)(row + k), 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        // a timed-out poll in any thread: an LDS flag (block_sum's barriers order it) instead of
        // __syncthreads_or, whose block-size read would be one more memory trip at the end
        if (!ok) bad = 1;
        block_sum<kNumAcc>(rest, scratch);
        ok = bad == 0;
#pragma unroll
        for (int k = 0; k < kNumAcc; ++k) tot[k] += rest[k];
    }
    if (threadIdx.x == 0) {
        if (!ok) {
#pragma unroll
            for (int k = 0; k < kNumAcc; ++k) tot[k] = __builtin_nan("");
        }
        if (CLASS_ONLY) {
            emit_class_sums(tot, sums4, accumulate);
        } else {
            const SurrogateScalars s = make_scalars_v(sc[0], sc[1], sc[2], sc[3], invB);
            finalize(tot, s, invB, out64, grad3, loss);
        }
    }
}

// ---- the same stream in ONE launch: start-order tickets ------------------------------------
//
// Workgroups are grouped by blockIdx (kTicketGroup consecutive chunks). A workgroup's FIRST
// instruction is a returning ticket add on its group's counter; the reply travels while the
// chunk's loads are in flight, so nobody waits for it. The workgroup that draws its group's
// last ticket is the last one of the group to START: every other member is already resident
// and waits for nothing, so it may poll their rows (data-as-flag words, as above) after its
// own chunk without any risk of waiting for a workgroup that cannot run. It sums the group's
// rows in blockIdx order, zeroes them, publishes the group total as data-as-flag words and
// draws a ticket on the final counter; the group reducer that draws the last of those (every
// other group reducer has already published) sums the group totals in group order and writes
// the scalars. Only ngroups + 1 workgroups ever wait, each near the end of its own life, and
// the summation order is fixed by blockIdx: bitwise reproducible, same as the two-launch form.
constexpr int kTicketGroupMin = 64;            // smallest group of any variant (sizes the workspace)
constexpr int kCtrStrideMax = 16384;           // widest counter spacing of any variant (64 KB)

__host__ __device__ inline int64_t ticket_groups(int64_t nblocks, int G = kTicketGroupMin) { return (nblocks + G - 1) / G; }

struct TicketWs {
    unsigned* ctr;                 // [ngroups + 1] * kCtrStride; [ngroups * kCtrStride] is the final counter
    unsigned long long* rows;      // [nblocks][kRowWords] encoded
    unsigned long long* gwords;    // [ngroups][kRowWords] encoded
};

inline size_t align256(size_t b) { return (b + 255) / 256 * 256; }

// sized for the smallest group and the widest counter spacing of any variant
inline size_t ticket_ws_bytes(int64_t nblocks) {
    const int64_t ng = ticket_groups(nblocks);
    return kPersistentBytes + align256(size_t(ng + 1) * kCtrStrideMax * 4) +
           align256(size_t(nblocks) * kRowWords * 8) + size_t(ng) * kRowWords * 8;
}

inline TicketWs ticket_ws(void* ws, int64_t nblocks) {
    const int64_t ng = ticket_groups(nblocks);
    char* p = static_cast<char*>(ws) + kPersistentBytes;
    TicketWs w;
    w.ctr = reinterpret_cast<unsigned*>(p);
    p += align256(size_t(ng + 1) * kCtrStrideMax * 4);
    w.rows = reinterpret_cast<unsigned long long*>(p);
    p += align256(size_t(nblocks) * kRowWords * 8);
    w.gwords = reinterpret_cast<unsigned long long*>(p);
    return w;
}

// Take nrows encoded rows (thread t: rows t, t + 256, then the next 512, ...): every word of a
// pass is loaded before any is examined, only the missing ones are polled again (bounded; a
// timeout leaves NaN), each is re-zeroed, and tot[] sums them in that fixed order.
__device__ __forceinline__ void take_rows(unsigned long long* words, int64_t nrows, double (&tot)[kNumAcc],
                                          bool& ok) {
    for (int64_t r0 = threadIdx.x; r0 < nrows; r0 += 2 * kThreads) {
        const int64_t r1 = r0 + kThreads;
        const bool two = r1 < nrows;
        unsigned long long w[2][kRowWords];
#pragma unroll
        for (int k = 0; k < kRowWords; ++k) {
            w[0][k] = __hip_atomic_load((gu64*)(words + r0 * kRowWords + k), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            w[1][k] = two ? __hip_atomic_load((gu64*)(words + r1 * kRowWords + k), __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT)
                          : ~0ull;
        }
        for (int polls = 0;; ++polls) {
            bool missing = false;
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int k = 0; k < kRowWords; ++k) missing |= (w[j][k] == 0ull);
            if (!missing) break;
            if (polls >= kMaxPolls) {
                ok = false;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int k = 0; k < kRowWords; ++k)
                    if (w[j][k] == 0ull)
                        w[j][k] = __hip_atomic_load((gu64*)(words + (j ? r1 : r0) * kRowWords + k), __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            if (j == 1 && !two) break;
#pragma unroll
            for (int k = 0; k < kRowWords; ++k) {
                tot[k] += __longlong_as_double(static_cast<long long>(w[j][k] ^ kEmptyKey));
                __hip_atomic_store((gu64*)(words + (j ? r1 : r0) * kRowWords + k), 0ull, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
}

// take_rows with one row per thread per pass: 12 fewer live VGPRs, which keeps a kernel that
// also streams (surrogate_tail_kernel) at the stream's own occupancy
__device__ __forceinline__ void take_rows_narrow(unsigned long long* words, int64_t nrows, double (&tot)[kNumAcc],
                                                 bool& ok) {
    for (int64_t r0 = threadIdx.x; r0 < nrows; r0 += kThreads) {
        unsigned long long w[kRowWords];
#pragma unroll
        for (int k = 0; k < kRowWords; ++k)
            w[k] = __hip_atomic_load((gu64*)(words + r0 * kRowWords + k), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (int polls = 0;; ++polls) {
            bool missing = false;
#pragma unroll
            for (int k = 0; k < kRowWords; ++k) missing |= (w[k] == 0ull);
            if (!missing) break;
            if (polls >= kMaxPolls) {
                ok = false;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
#pragma unroll
            for (int k = 0; k < kRowWords; ++k)
                if (w[k] == 0ull)
                    w[k] = __hip_atomic_load((gu64*)(words + r0 * kRowWords + k), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
        }
#pragma unroll
        for (int k = 0; k < kRowWords; ++k) {
            tot[k] += __longlong_as_double(static_cast<long long>(w[k] ^ kEmptyKey));
            __hip_atomic_store((gu64*)(words + r0 * kRowWords + k), 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

template <typename YT, bool CLASS_ONLY, int S, int kTicketGroup, int kCtrStride, bool TICKET_FIRST>
__global__ __launch_bounds__(kThreads) void surrogate_ticket_kernel(
    const float* __restrict__ h, const YT* __restrict__ y, int64_t B, double invB,
    const float* __restrict__ abalpha, const float* __restrict__ p_hat, float* __restrict__ dh, TicketWs ws,
    double* __restrict__ out64, float* __restrict__ grad3, float* __restrict__ loss, double* __restrict__ sums4,
    int accumulate) {
    const int64_t nblocks = gridDim.x;
    const int64_t ngroups = ticket_groups(nblocks, kTicketGroup);
    const int64_t grp = blockIdx.x / kTicketGroup;
    const int64_t g0 = grp * kTicketGroup;
    const int64_t gsize = (nblocks - g0 < kTicketGroup) ? nblocks - g0 : kTicketGroup;
    unsigned ticket = 0;
    // an opaque per-lane zero keeps the address divergent, so the atomic optimizer does not
    // rewrite the add into a wave-aggregated form that waits for the reply right away
    auto draw = [&]() {
        if (threadIdx.x == 0) {
            int zero;
            asm volatile("v_mov_b32 %0, 0" : "=v"(zero));
            ticket = __hip_atomic_fetch_add((gu32*)(ws.ctr + grp * kCtrStride + zero), 1u, __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT);
        }
    };
    if (TICKET_FIRST) draw();

    SurrogateScalars s;
    if (CLASS_ONLY) s = SurrogateScalars{};
    else s = make_scalars(abalpha, p_hat, invB);
    Acc acc;
    const bool write_dh = !CLASS_ONLY && dh != nullptr;
    const int64_t base = int64_t(blockIdx.x) * chunk_elems(S);
    const bool full = base + chunk_elems(S) <= B;
    f32x4 hv[S];
    if (full) {
        int yv[S][4];
#pragma unroll
        for (int k = 0; k < S; ++k) {
            const int64_t b = base + (int64_t(k) * kThreads + threadIdx.x) * kVec;
            hv[k] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(h + b));
            load_labels4(y, b, yv[k]);
        }
        if (!TICKET_FIRST) draw();  // issued behind the loads: waiting for them does not wait for it
#pragma unroll
        for (int k = 0; k < S; ++k) hv[k] = visit4<CLASS_ONLY>(hv[k], yv[k], s, acc);
    } else {
        if (!TICKET_FIRST) draw();
        for (int64_t i = base + threadIdx.x; i < B; i += kThreads) {
            const float g = visit1<CLASS_ONLY>(h[i], load_label(y, i), s, acc);
            if (write_dh) dh[i] = g;
        }
    }
    const double sp = wave_total_dpp(acc.s_pos), sn = wave_total_dpp(acc.s_neg);
    const double qp = wave_total_dpp(acc.q_pos), qn = wave_total_dpp(acc.q_neg);
    const int np = wave_total_dpp(acc.n_pos), nn = wave_total_dpp(acc.n_neg);
    if (full && write_dh) {
#pragma unroll
        for (int k = 0; k < S; ++k)
            __builtin_nontemporal_store(hv[k], reinterpret_cast<f32x4*>(dh + base + (int64_t(k) * kThreads + threadIdx.x) * kVec));
    }
    __shared__ double wrow[kWaves][kRowWords];
    __shared__ int role;  // 0: done, 1: group reducer
    const int wid = threadIdx.x / kWave;
    if ((threadIdx.x & (kWave - 1)) == kWave - 1) {
        wrow[wid][0] = sp;
        wrow[wid][1] = sn;
        wrow[wid][2] = qp;
        wrow[wid][3] = qn;
        wrow[wid][4] = static_cast<double>(np);
        wrow[wid][5] = static_cast<double>(nn);
    }
    if (threadIdx.x == 0) role = (ticket == gsize - 1);
    __syncthreads();
    if (threadIdx.x < kRowWords) {
        const int k = threadIdx.x;
        const double v = ((wrow[0][k] + wrow[1][k]) + wrow[2][k]) + wrow[3][k];
        __hip_atomic_store((gu64*)(ws.rows + int64_t(blockIdx.x) * kRowWords + k), enc_word(v), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    if (!role) return;

    // group reducer: rows g0 .. g0 + gsize in blockIdx order
    __shared__ double scratch[kNumAcc * kWaves];
    __shared__ int fin;
    bool ok = true;
    double tot[kNumAcc];
#pragma unroll
    for (int k = 0; k < kNumAcc; ++k) tot[k] = 0.0;
    take_rows(ws.rows + g0 * kRowWords, gsize, tot, ok);
    block_sum<kNumAcc>(tot, scratch);
    if (threadIdx.x < kRowWords) {
        double v = tot[0];
#pragma unroll
        for (int k = 1; k < kNumAcc; ++k)
            if (threadIdx.x == k) v = tot[k];
        __hip_atomic_store((gu64*)(ws.gwords + grp * kRowWords + threadIdx.x), enc_word(v), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    if (threadIdx.x == 0) {
        // every ticket of this group has been drawn: leave the counter zeroed for the next call
        __hip_atomic_store((gu32*)(ws.ctr + grp * kCtrStride), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned f = __hip_atomic_fetch_add((gu32*)(ws.ctr + ngroups * kCtrStride), 1u, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
        fin = (f == ngroups - 1);
        if (fin)
            __hip_atomic_store((gu32*)(ws.ctr + ngroups * kCtrStride), 0u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
    ok = __syncthreads_or(!ok) == 0;
    if (!fin) return;

    // final reducer: the group totals in group order
#pragma unroll
    for (int k = 0; k < kNumAcc; ++k) tot[k] = 0.0;
    take_rows(ws.gwords, ngroups, tot, ok);
    block_sum<kNumAcc>(tot, scratch);
    ok = __syncthreads_or(!ok) == 0;
    if (threadIdx.x == 0) {
        if (!ok) {
#pragma unroll
            for (int k = 0; k < kNumAcc; ++k) tot[k] = __builtin_nan("");
        }
        if (CLASS_ONLY) emit_class_sums(tot, sums4, accumulate);
        else finalize(tot, s, invB, out64, grad3, loss);
    }
}

// ---- the stream with its row reduce in the same launch: the LAST R workgroups reduce ---------
//
// Every workgroup streams its chunk (as surrogate_chunk_kernel) and stores its 48-B row as
// data-as-flag words (bits ^ kEmptyKey, agent-scope stores; no drain, no ticket). The last R
// workgroups by blockIdx are the reducers: reducer r, after its own chunk and row, takes the rows
// of group r (a contiguous range of ceil(nblocks / R) rows; take_rows: polls only words still
// zero, bounded, re-zeroes what it consumed, fixed summation order), and publishes the group total
// the same way; reducer R-1 takes the other R-1 group totals (in group order, then its own) and
// writes the scalars.
// Nothing waits on a workgroup that waits: the rows every reducer needs come from workgroups that
// never wait (and from the reducers' own rows, stored before they reduce), and at most R of the
// grid's resident slots are ever held by waiting workgroups. Bitwise reproducible.
// EXTRA: the R reducers are R extra workgroups after the nstream streaming ones (they stream
// nothing; a streaming workgroup never waits) instead of the last R streaming workgroups.
template <typename YT, int S, int R, bool EXTRA, bool NO_REDUCE = false>
__global__ __launch_bounds__(kThreads) void surrogate_tail_kernel(
    const float* __restrict__ h, const YT* __restrict__ y, int64_t B, double invB,
    const float* __restrict__ abalpha, const float* __restrict__ p_hat, float* __restrict__ dh,
    unsigned long long* __restrict__ rows, unsigned long long* __restrict__ gwords,
    double* __restrict__ out64, float* __restrict__ grad3, float* __restrict__ loss, int64_t nstream) {
    const SurrogateScalars s = make_scalars(abalpha, p_hat, invB);
    if (!EXTRA || int64_t(blockIdx.x) < nstream) {
    Acc acc;
    const bool write_dh = dh != nullptr;
    const int64_t base = int64_t(blockIdx.x) * chunk_elems(S);
    const bool full = base + chunk_elems(S) <= B;
    f32x4 hv[S];
    if (full) {
        int yv[S][4];
#pragma unroll
        for (int k = 0; k < S; ++k) {
            const int64_t b = base + (int64_t(k) * kThreads + threadIdx.x) * kVec;
            hv[k] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(h + b));
            load_labels4(y, b, yv[k]);
        }
#pragma unroll
        for (int k = 0; k < S; ++k) hv[k] = visit4<false>(hv[k], yv[k], s, acc);
    } else {
        for (int64_t i = base + threadIdx.x; i < B; i += kThreads) {
            const float g = visit1<false>(h[i], load_label(y, i), s, acc);
            if (write_dh) dh[i] = g;
        }
    }
    const double sp = wave_total_dpp(acc.s_pos), sn = wave_total_dpp(acc.s_neg);
    const double qp = wave_total_dpp(acc.q_pos), qn = wave_total_dpp(acc.q_neg);
    const int np = wave_total_dpp(acc.n_pos), nn = wave_total_dpp(acc.n_neg);
    if (full && write_dh) {
#pragma unroll
        for (int k = 0; k < S; ++k)
            __builtin_nontemporal_store(hv[k], reinterpret_cast<f32x4*>(dh + base + (int64_t(k) * kThreads + threadIdx.x) * kVec));
    }
    __shared__ double wrow[kWaves][kRowWords];
    const int wid = threadIdx.x / kWave;
    if ((threadIdx.x & (kWave - 1)) == kWave - 1) {
        wrow[wid][0] = sp;
        wrow[wid][1] = sn;
        wrow[wid][2] = qp;
        wrow[wid][3] = qn;
        wrow[wid][4] = static_cast<double>(np);
        wrow[wid][5] = static_cast<double>(nn);
    }
    __syncthreads();
    if (threadIdx.x < kRowWords) {
        const int k = threadIdx.x;
        const double v = ((wrow[0][k] + wrow[1][k]) + wrow[2][k]) + wrow[3][k];
        __hip_atomic_store((gu64*)(rows + int64_t(blockIdx.x) * kRowWords + k), enc_word(v), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    }
    const int64_t nblocks = EXTRA ? nstream : int64_t(gridDim.x);  // rows
    const int64_t nred = nblocks < R ? nblocks : R;
    const int64_t r = EXTRA ? int64_t(blockIdx.x) - nstream : int64_t(blockIdx.x) - (nblocks - nred);
    if (r < 0 || r >= nred || NO_REDUCE) return;

    // reducer r: the rows of group r; reducer nred - 1 (whose group holds the grid's last rows)
    // also takes the other group totals, loaded before its own group so that their trip overlaps
    // its wait, and adds its own total from registers: one memory trip after the last row lands
    __shared__ double scratch[kNumAcc * kWaves];
    const int64_t G = (nblocks + nred - 1) / nred;
    const int64_t g0 = r * G, g1 = (g0 + G < nblocks) ? g0 + G : nblocks;
    const bool final_red = r == nred - 1;
    const bool holds = final_red && threadIdx.x < nred - 1;  // thread t: group total t
    unsigned long long gw[kRowWords];
    if (holds) {
#pragma unroll
        for (int k = 0; k < kRowWords; ++k)
            gw[k] = __hip_atomic_load((gu64*)(gwords + threadIdx.x * kRowWords + k), __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT);
    }
    bool ok = true;
    double tot[kNumAcc];
#pragma unroll
    for (int k = 0; k < kNumAcc; ++k) tot[k] = 0.0;
    if (g1 > g0) take_rows_narrow(rows + g0 * kRowWords, g1 - g0, tot, ok);
    block_sum<kNumAcc>(tot, scratch);
    if (!final_red) {
        if (threadIdx.x < kRowWords) {
            double v = tot[0];
#pragma unroll
            for (int k = 1; k < kNumAcc; ++k)
                if (threadIdx.x == k) v = tot[k];
            __hip_atomic_store((gu64*)(gwords + r * kRowWords + threadIdx.x), enc_word(v), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        return;
    }
    double rest[kNumAcc];
#pragma unroll
    for (int k = 0; k < kNumAcc; ++k) rest[k] = 0.0;
    if (holds) {
        for (int polls = 0;; ++polls) {
            bool missing = false;
#pragma unroll
            for (int k = 0; k < kRowWords; ++k) missing |= (gw[k] == 0ull);
            if (!missing) break;
            if (polls >= kMaxPolls) {
                ok = false;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
#pragma unroll
            for (int k = 0; k < kRowWords; ++k)
                if (gw[k] == 0ull)
                    gw[k] = __hip_atomic_load((gu64*)(gwords + threadIdx.x * kRowWords + k), __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
        }
#pragma unroll
        for (int k = 0; k < kRowWords; ++k) {
            rest[k] = __longlong_as_double(static_cast<long long>(gw[k] ^ kEmptyKey));
            __hip_atomic_store((gu64*)(gwords + threadIdx.x * kRowWords + k), 0ull, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    block_sum<kNumAcc>(rest, scratch);
    ok = __syncthreads_or(!ok) == 0;
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < kNumAcc; ++k) tot[k] = ok ? rest[k] + tot[k] : __builtin_nan("");
        finalize(tot, s, invB, out64, grad3, loss);
    }
}

template <typename YT, int S, int R, bool EXTRA = false, bool NO_REDUCE = false>
int launch_tail(const float* h, const YT* y, int64_t B, const float* abalpha, const float* p_hat, float* dh,
                double* out64, float* grad3, float* loss, void* ws, size_t ws_bytes, hipStream_t st) {
    const int64_t nblocks = (B + chunk_elems(S) - 1) / chunk_elems(S);
    if (nblocks + R > 0x7fffffffLL) return DAUC_EINVAL;
    const size_t need = kPersistentBytes + static_cast<size_t>(nblocks + R) * kRowWords * 8;
    if (ws == nullptr || ws_bytes < need) return DAUC_EINVAL;
    auto* rows = reinterpret_cast<unsigned long long*>(static_cast<char*>(ws) + kPersistentBytes);
    const int64_t grid = EXTRA ? nblocks + R : nblocks;
    hipLaunchKernelGGL((surrogate_tail_kernel<YT, S, R, EXTRA, NO_REDUCE>), dim3(static_cast<unsigned>(grid)), dim3(kThreads), 0,
                       st, h, y, B, 1.0 / static_cast<double>(B), abalpha, p_hat, dh, rows, rows + nblocks * kRowWords,
                       out64, grad3, loss, nblocks);
    return launch_status();
}

// Default chunk geometry (variant sweep: scripts/micro_kernels.py --which surrogate).
#ifndef DAUC_SURROGATE_CHUNK_SLOTS
#define DAUC_SURROGATE_CHUNK_SLOTS 4
#endif
constexpr int kChunkSlots = DAUC_SURROGATE_CHUNK_SLOTS;
// reducers of the one-launch loss (variants 20-24 measured at B = 2^26: 16 / 32 / 64 / 128 / 256;
// profiles/r02/surrogate_ab.jsonl)
#ifndef DAUC_SURROGATE_TAIL_REDUCERS
#define DAUC_SURROGATE_TAIL_REDUCERS 64
#endif
constexpr int kTailReducers = DAUC_SURROGATE_TAIL_REDUCERS;
// Unit-stride batches at least this large take the chunked kernel; smaller ones are
// latency-bound and stay on the single-ticket persistent kernel.
constexpr int64_t kChunkMinB = int64_t(1) << 22;

int resident_blocks() {
    static int cached = 0;
    if (cached == 0) {
        int dev = 0, cus = 0, per_cu = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(
                &per_cu, reinterpret_cast<const void*>(&surrogate_kernel<int8_t, false, true>), kThreads,
                0) != hipSuccess ||
            cus <= 0 || per_cu <= 0) {
            (void)hipGetLastError();
            cached = kMaxBlocks;  // no device (e.g. size queries on a build host): upper bound
        } else {
            per_cu = per_cu < DAUC_SURROGATE_BPC ? per_cu : DAUC_SURROGATE_BPC;
            cached = cus * per_cu;
        }
    }
    return cached;
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

template <typename YT, bool CLASS_ONLY, int S, bool NTL, bool NTS>
int launch_chunk(const float* h, const YT* y, int64_t B, const float* abalpha, const float* p_hat, float* dh,
                 double* out64, float* grad3, float* loss, double* sums4, int accumulate, void* ws,
                 size_t ws_bytes, hipStream_t st) {
    const int64_t nblocks = (B + chunk_elems(S) - 1) / chunk_elems(S);
    if (nblocks > 0x7fffffffLL) return DAUC_EINVAL;
    if (ws == nullptr || ws_bytes < chunk_ws_bytes(nblocks)) return DAUC_EINVAL;
    const ChunkWs w = chunk_ws(ws, nblocks);
    const double invB = 1.0 / static_cast<double>(B);
    hipLaunchKernelGGL((surrogate_chunk_kernel<YT, CLASS_ONLY, S, NTL, NTS>), dim3(static_cast<unsigned>(nblocks)),
                       dim3(kThreads), 0, st, h, y, B, invB, abalpha, p_hat, dh, w.rows);
    int rc = launch_status();
    if (rc) return rc;
    const int64_t nrows = nblocks * kRowsPerChunk;
    hipLaunchKernelGGL((surrogate_rows_reduce_kernel<CLASS_ONLY>), dim3(static_cast<unsigned>(reduce_blocks(nrows))),
                       dim3(kThreads), 0, st, w.rows, nrows, w, invB, abalpha, p_hat, out64, grad3, loss, sums4,
                       accumulate);
    return launch_status();
}

template <typename YT, bool CLASS_ONLY, int S, int SPAN>
int launch_span(const float* h, const YT* y, int64_t B, const float* abalpha, const float* p_hat, float* dh,
                double* out64, float* grad3, float* loss, double* sums4, int accumulate, void* ws, size_t ws_bytes,
                hipStream_t st) {
    constexpr int64_t kChunk = chunk_elems(S);
    const int64_t whole = B / (SPAN * kChunk);
    const int64_t nblocks = whole + (B - whole * SPAN * kChunk + kChunk - 1) / kChunk;
    if (nblocks > 0x7fffffffLL) return DAUC_EINVAL;
    if (ws == nullptr || ws_bytes < chunk_ws_bytes(nblocks)) return DAUC_EINVAL;
    const ChunkWs w = chunk_ws(ws, nblocks);
    const double invB = 1.0 / static_cast<double>(B);
    hipLaunchKernelGGL((surrogate_span_kernel<YT, CLASS_ONLY, S, SPAN>), dim3(static_cast<unsigned>(nblocks)),
                       dim3(kThreads), 0, st, h, y, B, invB, abalpha, p_hat, dh, w.rows);
    int rc = launch_status();
    if (rc) return rc;
    hipLaunchKernelGGL((surrogate_rows_reduce_kernel<CLASS_ONLY>), dim3(static_cast<unsigned>(reduce_blocks(nblocks))),
                       dim3(kThreads), 0, st, w.rows, nblocks, w, invB, abalpha, p_hat, out64, grad3, loss, sums4,
                       accumulate);
    return launch_status();
}

template <typename YT, bool CLASS_ONLY, int S, int G, int CS, bool TF>
int launch_ticket(const float* h, const YT* y, int64_t B, const float* abalpha, const float* p_hat, float* dh,
                  double* out64, float* grad3, float* loss, double* sums4, int accumulate, void* ws, size_t ws_bytes,
                  hipStream_t st) {
    const int64_t nblocks = (B + chunk_elems(S) - 1) / chunk_elems(S);
    if (nblocks > 0x7fffffffLL) return DAUC_EINVAL;
    if (ws == nullptr || ws_bytes < ticket_ws_bytes(nblocks)) return DAUC_EINVAL;
    hipLaunchKernelGGL((surrogate_ticket_kernel<YT, CLASS_ONLY, S, G, CS, TF>), dim3(static_cast<unsigned>(nblocks)),
                       dim3(kThreads), 0, st, h, y, B, 1.0 / static_cast<double>(B), abalpha, p_hat, dh,
                       ticket_ws(ws, nblocks), out64, grad3, loss, sums4, accumulate);
    return launch_status();
}

// variant: 0 = default dispatch, 1 = persistent kernel, 2..7 = chunk kernel geometries,
// 8..14 = single-launch ticket kernel (slots, group size, counter spacing, ticket order)
// (tuning; only for int8 labels with a loss, i.e. the micro-benchmark's configuration).
template <bool CLASS_ONLY, typename YT>
int launch_surrogate(const float* h, int64_t hs, const YT* y, int64_t B, const float* abalpha,
                     const float* p_hat, float* dh, int64_t dhs, double* out64, float* grad3,
                     float* loss, double* sums4, int accumulate, void* ws, size_t ws_bytes,
                     hipStream_t st, int variant = 0) {
    const bool unit = hs == 1 && aligned16(h) &&
                      (reinterpret_cast<uintptr_t>(y) % (kVec * sizeof(YT))) == 0 &&
                      (CLASS_ONLY || dh == nullptr || (dhs == 1 && aligned16(dh)));
    if (unit && variant >= 2) {
        if constexpr (!CLASS_ONLY && sizeof(YT) == 1) {
            switch (variant) {
                case 2: return launch_chunk<YT, false, 4, true, true>(h, y, B, abalpha, p_hat, dh, out64, grad3, loss, sums4, accumulate, ws, ws_bytes, st);
                case 3: return launch_chunk<YT, false, 8, true, true>(h, y, B, abalpha, p_hat, dh, out64, grad3, loss, sums4, accumulate, ws, ws_bytes, st);
                case 4: return launch_chunk<YT, false, 16, true, true>(h, y, B, abalpha, p_hat, dh, out64, grad3, loss, sums4, accumulate, ws, ws_bytes, st);
                case 5: return launch_chunk<YT, false, 8, false, true>(h, y, B, abalpha, p_hat, dh, out64, grad3, loss, sums4, accumulate, ws, ws_bytes, st);
                case 6: return launch_chunk<YT, false, 8, true, false>(h, y, B, abalpha, p_hat, dh, out64, grad3, loss, sums4, accumulate, ws, ws_bytes, st);
                case 7: return launch_chunk<YT, false, 2, true, true>(h, y, B, abalpha, p_hat, dh, out64, grad3, loss, sums4, accumulate, ws, ws_bytes, st);
#define DAUC_TV(S, G, CS, TF) return launch_ticket<YT, false, S, G, CS, TF>(h, y, B, abalpha, p_hat, dh, out64, grad3, loss, sums4, accumulate, ws, ws_bytes, st)
                case 8: DAUC_TV(4, 512, 1024, true);
                case 9: DAUC_TV(4, 64, 1024, true);
                case 10: DAUC_TV(4, 128, 1024, true);
                case 11: DAUC_TV(4, 256, 1024, true);
                case 12: DAUC_TV(4, 64, 1024, false);
                case 13: DAUC_TV(8, 64, 1024, true);
                case 14: DAUC_TV(8, 256, 1024, true);
#undef DAUC_TV
                case 15: {
                    // the default streaming kernel alone (no row reduce, no scalars): timing only. It
                    // leaves its rows in the workspace, so it must not share one with the other variants.
                    const int64_t nblocks = (B + chunk_elems(kChunkSlots) - 1) / chunk_elems(kChunkSlots);
                    if (ws == nullptr || ws_bytes < chunk_ws_bytes(nblocks)) return DAUC_EINVAL;
                    hipLaunchKernelGGL((surrogate_chunk_kernel<YT, false, kChunkSlots, true, true>),
                                       dim3(static_cast<unsigned>(nblocks)), dim3(kThreads), 0, st, h, y, B,
                                       1.0 / static_cast<double>(B), abalpha, p_hat, dh, chunk_ws(ws, nblocks).rows);
                    return launch_status();
                }
                case 16: return launch_span<YT, false, 4, 4>(h, y, B, abalpha, p_hat, dh, out64, grad3, loss, sums4, accumulate, ws, ws_bytes, st);
                case 17: return launch_span<YT, false, 4, 8>(h, y, B, abalpha, p_hat, dh, out64, grad3, loss, sums4, accumulate, ws, ws_bytes, st);
                case 18: return launch_span<YT, false, 4, 16>(h, y, B, abalpha, p_hat, dh, out64, grad3, loss, sums4, accumulate, ws, ws_bytes, st);
                case 19: return launch_span<YT, false, 4, 32>(h, y, B, abalpha, p_hat, dh, out64, grad3, loss, sums4, accumulate, ws, ws_bytes, st);
                case 20: return launch_tail<YT, 4, 32>(h, y, B, abalpha, p_hat, dh, out64, grad3, loss, ws, ws_bytes, st);
                case 21: return launch_tail<YT, 4, 16>(h, y, B, abalpha, p_hat, dh, out64, grad3, loss, ws, ws_bytes, st);
                case 22: return launch_tail<YT, 4, 64>(h, y, B, abalpha, p_hat, dh, out64, grad3, loss, ws, ws_bytes, st);
                case 23: return launch_tail<YT, 4, 128>(h, y, B, abalpha, p_hat, dh, out64, grad3, loss, ws, ws_bytes, st);
                case 24: return launch_tail<YT, 4, 256>(h, y, B, abalpha, p_hat, dh, out64, grad3, loss, ws, ws_bytes, st);
                case 25: return launch_chunk<YT, false, kChunkSlots, true, true>(h, y, B, abalpha, p_hat, dh, out64, grad3, loss, sums4, accumulate, ws, ws_bytes, st);
                case 26: return launch_tail<YT, 4, 64, true>(h, y, B, abalpha, p_hat, dh, out64, grad3, loss, ws, ws_bytes, st);
                case 27: return launch_tail<YT, 4, 32, true>(h, y, B, abalpha, p_hat, dh, out64, grad3, loss, ws, ws_bytes, st);
                case 28: return launch_tail<YT, 4, 128, true>(h, y, B, abalpha, p_hat, dh, out64, grad3, loss, ws, ws_bytes, st);
                // timing only: the one-launch stream with its data-as-flag row stores, nobody reducing
                // (rows are left in the workspace: give it one of its own, like variant 15)
                case 29: return launch_tail<YT, 4, 64, false, true>(h, y, B, abalpha, p_hat, dh, out64, grad3, loss, ws, ws_bytes, st);
                default: return DAUC_EINVAL;
            }
        }
        return DAUC_EINVAL;
    }
    if (unit && variant == 0 && B >= kChunkMinB) {
        // the loss: the stream with its row reduce done by its last kTailReducers workgroups (one
        // launch); the class sums keep the two-launch form
        if constexpr (!CLASS_ONLY)
            return launch_tail<YT, kChunkSlots, kTailReducers>(h, y, B, abalpha, p_hat, dh, out64, grad3, loss, ws,
                                                               ws_bytes, st);
        else
            return launch_chunk<YT, CLASS_ONLY, kChunkSlots, true, true>(h, y, B, abalpha, p_hat, dh, out64, grad3,
                                                                          loss, sums4, accumulate, ws, ws_bytes, st);
    }
    const int grid = grid_for(B);
    unsigned* counter = nullptr;
    double* partials = nullptr;
    if (grid > 1) {
        if (ws == nullptr || ws_bytes < kCounterBytes + static_cast<size_t>(grid) * kNumAcc * sizeof(double))
            return DAUC_EINVAL;
        counter = static_cast<unsigned*>(ws);
        partials = reinterpret_cast<double*>(static_cast<char*>(ws) + kCounterBytes);
    }
    if (unit) {
        hipLaunchKernelGGL((surrogate_kernel<YT, CLASS_ONLY, true>), dim3(grid), dim3(kThreads), 0,
                           st, h, hs, y, B, 1.0 / static_cast<double>(B), abalpha, p_hat, dh, dhs,
                           partials, counter, out64, grad3, loss, sums4, accumulate);
    } else {
        hipLaunchKernelGGL((surrogate_kernel<YT, CLASS_ONLY, false>), dim3(grid), dim3(kThreads),
                           0, st, h, hs, y, B, 1.0 / static_cast<double>(B), abalpha, p_hat, dh,
                           dhs, partials, counter, out64, grad3, loss, sums4, accumulate);
    }
    return launch_status();
}

template <bool CLASS_ONLY>
int dispatch_labels(const float* h, int64_t hs, const void* y, int yt, int64_t B,
                    const float* abalpha, const float* p_hat, float* dh, int64_t dhs,
                    double* out64, float* grad3, float* loss, double* sums4, int accumulate,
                    void* ws, size_t ws_bytes, hipStream_t st, int variant = 0) {
    if (variant != 0 && yt != DAUC_LABEL_I8) return DAUC_EINVAL;
    switch (yt) {
        case DAUC_LABEL_I8:
            return launch_surrogate<CLASS_ONLY>(h, hs, static_cast<const int8_t*>(y), B, abalpha,
                                                p_hat, dh, dhs, out64, grad3, loss, sums4,
                                                accumulate, ws, ws_bytes, st, variant);
        case DAUC_LABEL_I32:
            return launch_surrogate<CLASS_ONLY>(h, hs, static_cast<const int32_t*>(y), B, abalpha,
                                                p_hat, dh, dhs, out64, grad3, loss, sums4,
                                                accumulate, ws, ws_bytes, st);
        case DAUC_LABEL_I64:
            return launch_surrogate<CLASS_ONLY>(h, hs, static_cast<const int64_t*>(y), B, abalpha,
                                                p_hat, dh, dhs, out64, grad3, loss, sums4,
                                                accumulate, ws, ws_bytes, st);
        default:
            return DAUC_EINVAL;
    }
}

template <bool CLASS_ONLY, typename ZT, typename YT>
int launch_logits_t(const ZT* z, int64_t ldz, const YT* y, int64_t B, const float* abalpha, const float* p_hat,
                    ZT* dz, int64_t lddz, float* h_out, double* out64, float* grad3, float* loss, double* sums4,
                    int accumulate, void* ws, size_t ws_bytes, hipStream_t st) {
    const int grid = grid_scalar(B);
    unsigned* counter = nullptr;
    double* partials = nullptr;
    if (grid > 1) {
        if (ws == nullptr || ws_bytes < dauc_surrogate_workspace_size(B)) return DAUC_EINVAL;
        counter = static_cast<unsigned*>(ws);
        partials = reinterpret_cast<double*>(static_cast<char*>(ws) + kCounterBytes);
    }
    hipLaunchKernelGGL((surrogate_logits_kernel<ZT, YT, CLASS_ONLY>), dim3(grid), dim3(kThreads), 0, st, z, ldz,
                       y, B, 1.0 / static_cast<double>(B), abalpha, p_hat, dz, lddz, h_out, partials, counter,
                       out64, grad3, loss, sums4, accumulate);
    return launch_status();
}

template <bool CLASS_ONLY, typename ZT>
int launch_logits_y(const ZT* z, int64_t ldz, const void* y, int yt, int64_t B, const float* abalpha,
                    const float* p_hat, ZT* dz, int64_t lddz, float* h_out, double* out64, float* grad3,
                    float* loss, double* sums4, int accumulate, void* ws, size_t ws_bytes, hipStream_t st) {
    switch (yt) {
        case DAUC_LABEL_I8:
            return launch_logits_t<CLASS_ONLY>(z, ldz, static_cast<const int8_t*>(y), B, abalpha, p_hat, dz, lddz,
                                               h_out, out64, grad3, loss, sums4, accumulate, ws, ws_bytes, st);
        case DAUC_LABEL_I32:
            return launch_logits_t<CLASS_ONLY>(z, ldz, static_cast<const int32_t*>(y), B, abalpha, p_hat, dz,
                                               lddz, h_out, out64, grad3, loss, sums4, accumulate, ws, ws_bytes,
                                               st);
        case DAUC_LABEL_I64:
            return launch_logits_t<CLASS_ONLY>(z, ldz, static_cast<const int64_t*>(y), B, abalpha, p_hat, dz,
                                               lddz, h_out, out64, grad3, loss, sums4, accumulate, ws, ws_bytes,
                                               st);
        default:
            return DAUC_EINVAL;
    }
}

template <bool CLASS_ONLY>
int launch_logits(const void* z, int zt, int64_t ldz, const void* y, int yt, int64_t B, const float* abalpha,
                  const float* p_hat, void* dz, int64_t lddz, float* h_out, double* out64, float* grad3,
                  float* loss, double* sums4, int accumulate, void* ws, size_t ws_bytes, hipStream_t st) {
    if (zt == DAUC_DTYPE_F32)
        return launch_logits_y<CLASS_ONLY>(static_cast<const float*>(z), ldz, y, yt, B, abalpha, p_hat,
                                           static_cast<float*>(dz), lddz, h_out, out64, grad3, loss, sums4,
                                           accumulate, ws, ws_bytes, st);
    if (zt == DAUC_DTYPE_BF16)
        return launch_logits_y<CLASS_ONLY>(static_cast<const __hip_bfloat16*>(z), ldz, y, yt, B, abalpha, p_hat,
                                           static_cast<__hip_bfloat16*>(dz), lddz, h_out, out64, grad3, loss,
                                           sums4, accumulate, ws, ws_bytes, st);
    return DAUC_EINVAL;
}

// ---- a1: label map + class counts + p_hat (one block; B is a training batch) ----
__global__ __launch_bounds__(kThreads) void label_map_phat_kernel(
    const int64_t* __restrict__ labels, int64_t B, int64_t split, int8_t* __restrict__ y_out,
    float* __restrict__ lcounts, const float* __restrict__ gcounts, float* __restrict__ p_hat) {
    __shared__ unsigned long long part[2][kThreads / kWave];
    unsigned long long npos = 0, nneg = 0;
    for (int64_t i = threadIdx.x; i < B; i += kThreads) {
        const int8_t v = labels[i] <= split ? int8_t(-1) : int8_t(1);
        if (y_out) y_out[i] = v;
        npos += (v == 1);
        nneg += (v == -1);
    }
    npos = wave_sum(npos);
    nneg = wave_sum(nneg);
    const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
    if (lane == 0) {
        part[0][wid] = npos;
        part[1][wid] = nneg;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long tp = 0, tn = 0;
        for (int w = 0; w < kThreads / kWave; ++w) {
            tp += part[0][w];
            tn += part[1][w];
        }
        // main.py:307-308: lpos/lneg accumulate (fp32, exact below 2^24)
        const float lpos = __fadd_rn(lcounts[0], static_cast<float>(tp));
        const float lneg = __fadd_rn(lcounts[1], static_cast<float>(tn));
        lcounts[0] = lpos;
        lcounts[1] = lneg;
        // main.py:309-310: fp32 tensor sums, float() to double, double divide, fp32 store
        const float gpos = gcounts[0], gneg = gcounts[1];
        const float num = __fadd_rn(gpos, lpos);
        const float den = __fadd_rn(__fadd_rn(num, gneg), lneg);
        p_hat[0] = static_cast<float>(static_cast<double>(num) / static_cast<double>(den));
    }
}

__global__ void alpha_from_sums_kernel(const double* __restrict__ s, float* __restrict__ alpha) {
    // main.py:197 computes this from fp32 sums; fp64 here, rounded once.
    alpha[0] = static_cast<float>(s[0] / s[1] - s[2] / s[3]);
}

}  // namespace
}  // namespace dauc

using namespace dauc;

extern "C" {

size_t dauc_surrogate_workspace_size(int64_t B) {
    if (B < 0) B = 0;
    const int g = grid_scalar(B);  // >= grid_for(B): covers the persistent kernels
    const size_t persistent = kCounterBytes + static_cast<size_t>(g) * kNumAcc * sizeof(double);
    // the chunk kernels (smallest chunk of any variant: S = 2)
    const int64_t nb2 = (B + chunk_elems(2) - 1) / chunk_elems(2);
    const size_t chunked = chunk_ws_bytes(nb2), ticketed = ticket_ws_bytes(nb2);
    const size_t big = chunked > ticketed ? chunked : ticketed;
    return persistent > big ? persistent : big;
}

int dauc_surrogate_fwdbwd(const float* h, int64_t h_stride, const void* y, int y_dtype, int64_t B,
                          const float* abalpha, const float* p_hat, float* dh, int64_t dh_stride,
                          double* out64, float* grad3, float* loss, void* workspace,
                          size_t workspace_bytes, dauc_stream_t stream) {
    if (B <= 0 || h == nullptr || y == nullptr || abalpha == nullptr || p_hat == nullptr ||
        h_stride <= 0 || (dh != nullptr && dh_stride <= 0))
        return DAUC_EINVAL;
    return dispatch_labels<false>(h, h_stride, y, y_dtype, B, abalpha, p_hat, dh, dh_stride, out64,
                                  grad3, loss, nullptr, 0, workspace, workspace_bytes,
                                  as_hip(stream));
}

int dauc_surrogate_fwdbwd_variant(const float* h, int64_t h_stride, const void* y, int y_dtype, int64_t B,
                                  const float* abalpha, const float* p_hat, float* dh, int64_t dh_stride,
                                  double* out64, float* grad3, float* loss, void* workspace,
                                  size_t workspace_bytes, int variant, dauc_stream_t stream) {
    if (B <= 0 || h == nullptr || y == nullptr || abalpha == nullptr || p_hat == nullptr ||
        h_stride <= 0 || (dh != nullptr && dh_stride <= 0) || variant < 0 || variant > 29)
        return DAUC_EINVAL;
    return dispatch_labels<false>(h, h_stride, y, y_dtype, B, abalpha, p_hat, dh, dh_stride, out64,
                                  grad3, loss, nullptr, 0, workspace, workspace_bytes,
                                  as_hip(stream), variant);
}

int dauc_class_sums(const float* h, int64_t h_stride, const void* y, int y_dtype, int64_t B,
                    double* sums4, int accumulate, void* workspace, size_t workspace_bytes,
                    dauc_stream_t stream) {
    if (B <= 0 || h == nullptr || y == nullptr || sums4 == nullptr || h_stride <= 0)
        return DAUC_EINVAL;
    return dispatch_labels<true>(h, h_stride, y, y_dtype, B, nullptr, nullptr, nullptr, 1, nullptr,
                                 nullptr, nullptr, sums4, accumulate, workspace, workspace_bytes,
                                 as_hip(stream));
}

int dauc_surrogate_logits_fwdbwd(const void* z, int z_dtype, int64_t ldz, const void* y, int y_dtype,
                                 int64_t B, const float* abalpha, const float* p_hat, void* dz, int64_t lddz,
                                 float* h_out, double* out64, float* grad3, float* loss, void* workspace,
                                 size_t workspace_bytes, dauc_stream_t stream) {
    if (B <= 0 || z == nullptr || y == nullptr || abalpha == nullptr || p_hat == nullptr || ldz < 2 ||
        (dz != nullptr && lddz < 2))
        return DAUC_EINVAL;
    return launch_logits<false>(z, z_dtype, ldz, y, y_dtype, B, abalpha, p_hat, dz, lddz, h_out, out64, grad3,
                                loss, nullptr, 0, workspace, workspace_bytes, as_hip(stream));
}

int dauc_class_sums_logits(const void* z, int z_dtype, int64_t ldz, const void* y, int y_dtype, int64_t B,
                           float* h_out, double* sums4, int accumulate, void* workspace, size_t workspace_bytes,
                           dauc_stream_t stream) {
    if (B <= 0 || z == nullptr || y == nullptr || sums4 == nullptr || ldz < 2) return DAUC_EINVAL;
    return launch_logits<true>(z, z_dtype, ldz, y, y_dtype, B, nullptr, nullptr, nullptr, 2, h_out, nullptr,
                               nullptr, nullptr, sums4, accumulate, workspace, workspace_bytes, as_hip(stream));
}

int dauc_alpha_from_sums(const double* sums4, float* alpha, dauc_stream_t stream) {
    if (sums4 == nullptr || alpha == nullptr) return DAUC_EINVAL;
    hipLaunchKernelGGL(alpha_from_sums_kernel, dim3(1), dim3(1), 0, as_hip(stream), sums4, alpha);
    return launch_status();
}

int dauc_label_map_phat(const int64_t* labels, int64_t B, int64_t split_index, int8_t* y_out,
                        float* lcounts, const float* gcounts, float* p_hat, dauc_stream_t stream) {
    if (B <= 0 || labels == nullptr || lcounts == nullptr || gcounts == nullptr || p_hat == nullptr)
        return DAUC_EINVAL;
    hipLaunchKernelGGL(label_map_phat_kernel, dim3(1), dim3(kThreads), 0, as_hip(stream), labels, B,
                       split_index, y_out, lcounts, gcounts, p_hat);
    return launch_status();
}

}  // extern "C"
