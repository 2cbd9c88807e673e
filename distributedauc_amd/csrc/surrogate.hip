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
// surrogate_tail_kernel -- one 4096-element chunk per workgroup, rows handed to the last 64
// workgroups as epoch-tagged granules, which reduce them (see the comment at that kernel); smaller
// or strided batches (training, B = 256) take the persistent kernel with one last-arriver
// ticket. Tuning builds (-DDAUC_TUNING, build.py) add dauc_surrogate_fwdbwd_variant: the
// persistent kernel at any size, the two-launch form, the stream alone, and a stamped tail.

#include <hip/hip_bf16.h>

#include "dauc_internal.h"

namespace dauc {
namespace {

constexpr int kThreads = 256;
constexpr int kVec = 4;                                // elements per float4 slot
// Geometry from the MI355X sweep (scripts/gpu_sweep_sur.sh, profiles/r01): 8 float4
// slots per thread and 2 resident blocks per CU stream best (a narrow, deep window;
// more resident blocks lose DRAM locality).
constexpr int kSlots = 8;           // float4 slots per thread per iteration
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
    f32x4 g = {0.f, 0.f, 0.f, 0.f};
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
                    __builtin_nontemporal_store(g, dst);
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

// ---- large unit-stride batches: one chunk per workgroup -------------------------------------
//
// A grid-stride (persistent) loop walks the batch with a large stride, so concurrently open
// DRAM pages are far apart (measured: 6.2 TB/s for this 5:4 read:write mix vs 6.5 TB/s for
// one chunk per workgroup, scripts/probe_stream.hip). Here every workgroup takes ONE
// contiguous chunk of 256 x 4 x S elements (the dispatcher hands chunks out roughly in
// address order, like the update kernel's one-shot grid) and issues all of its loads
// before any math; every WAVE reduces its 6 partials with DPP (no barrier, no LDS), the dF/dh
// stores are issued, and ONE barrier combines the 4 wave totals into the workgroup's row.
// Fixed summation orders everywhere: bitwise reproducible.
constexpr int kWaves = kThreads / kWave;          // waves per workgroup
constexpr int kRowWords = 6;                      // s_pos, s_neg, q_pos, q_neg, n_pos, n_neg (fp64)
constexpr int kRowsPerReduceBlock = 512;          // rows one workgroup of the two-launch reduce sums
constexpr size_t kPersistentBytes = kCounterBytes + size_t(kMaxBlocks) * kNumAcc * sizeof(double);

__host__ __device__ constexpr int64_t chunk_elems(int S) { return int64_t(kThreads) * kVec * S; }

inline int64_t reduce_blocks(int64_t nrows) { return (nrows + kRowsPerReduceBlock - 1) / kRowsPerReduceBlock; }

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

// The chunk of workgroup blockIdx.x: loads, dF/dh stores, and the workgroup's row total j
// (0..5: s_pos, s_neg, q_pos, q_neg, n_pos, n_neg; the counts as exact doubles) for each thread's
// own j. Every thread calls it.
template <typename YT, bool CLASS_ONLY, int S>
__device__ __forceinline__ double stream_chunk(const float* __restrict__ h, const YT* __restrict__ y, int64_t B,
                                               const SurrogateScalars& s, float* __restrict__ dh, int j) {
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
#pragma unroll
        for (int k = 0; k < S; ++k) hv[k] = visit4<CLASS_ONLY>(hv[k], yv[k], s, acc);
    } else {
        // the ragged last chunk: one element per thread per step
        for (int64_t i = base + threadIdx.x; i < B; i += kThreads) {
            const float g = visit1<CLASS_ONLY>(h[i], load_label(y, i), s, acc);
            if (write_dh) dh[i] = g;
        }
    }
    // wave totals by DPP (lane 63), then the dF/dh stores, then ONE barrier: it comes after every
    // store of the chunk has been issued, so no wave holds its stores back for it
    const double sp = wave_total_dpp(acc.s_pos), sn = wave_total_dpp(acc.s_neg);
    const double qp = wave_total_dpp(acc.q_pos), qn = wave_total_dpp(acc.q_neg);
    const int np = wave_total_dpp(acc.n_pos), nn = wave_total_dpp(acc.n_neg);
    if (full && write_dh) {
#pragma unroll
        for (int k = 0; k < S; ++k)
            __builtin_nontemporal_store(hv[k],
                                        reinterpret_cast<f32x4*>(dh + base + (int64_t(k) * kThreads + threadIdx.x) * kVec));
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
    return ((wrow[0][j] + wrow[1][j]) + wrow[2][j]) + wrow[3][j];
}

// ---- the two-launch form: plain rows, then a small reduce launch -----------------------------
// The stage-start class sums at large B take it (a few calls per stage); the loss takes the
// one-launch tail kernel below. The kernel boundary publishes the rows.
template <typename YT, bool CLASS_ONLY, int S>
__global__ __launch_bounds__(kThreads) void surrogate_chunk_kernel(
    const float* __restrict__ h, const YT* __restrict__ y, int64_t B, double invB,
    const float* __restrict__ abalpha, const float* __restrict__ p_hat, float* __restrict__ dh,
    double* __restrict__ rows) {
    SurrogateScalars s;
    if (CLASS_ONLY) s = SurrogateScalars{};
    else s = make_scalars(abalpha, p_hat, invB);
    const int j = threadIdx.x < kRowWords ? threadIdx.x : 0;
    const double v = stream_chunk<YT, CLASS_ONLY, S>(h, y, B, s, dh, j);
    if (threadIdx.x < kRowWords) rows[int64_t(blockIdx.x) * kRowWords + threadIdx.x] = v;
}

// Workgroup b sums rows [512 b, 512 (b + 1)) in a fixed order (thread t: rows t, t + 256); the
// partial totals go to a slot per workgroup and the last arriver (ticket) sums the slots in
// workgroup order and writes the scalars.
template <bool CLASS_ONLY>
__global__ __launch_bounds__(kThreads) void surrogate_rows_reduce_kernel(
    double* __restrict__ rows, int64_t nrows, double* __restrict__ partials, unsigned* __restrict__ counter,
    double invB, const float* __restrict__ abalpha, const float* __restrict__ p_hat, double* __restrict__ out64,
    float* __restrict__ grad3, float* __restrict__ loss, double* __restrict__ sums4, int accumulate) {
    __shared__ double scratch[kNumAcc * kWaves];
    __shared__ int last_flag;
    double tot[kNumAcc];
#pragma unroll
    for (int k = 0; k < kNumAcc; ++k) tot[k] = 0.0;
    const int64_t r0 = int64_t(blockIdx.x) * kRowsPerReduceBlock;
    const int64_t r1 = (r0 + kRowsPerReduceBlock < nrows) ? r0 + kRowsPerReduceBlock : nrows;
    for (int64_t r = r0 + threadIdx.x; r < r1; r += kThreads) {
#pragma unroll
        for (int k = 0; k < kNumAcc; ++k) tot[k] += rows[r * kRowWords + k];
    }
    block_sum<kNumAcc>(tot, scratch);
    if (gridDim.x > 1) {
        if (threadIdx.x == 0) {
#pragma unroll
            for (int k = 0; k < kNumAcc; ++k) store_sc1(&partials[blockIdx.x * kNumAcc + k], tot[k]);
        }
        if (!arrive_last(counter, gridDim.x, &last_flag)) return;
#pragma unroll
        for (int k = 0; k < kNumAcc; ++k) tot[k] = 0.0;
        for (int b = threadIdx.x; b < static_cast<int>(gridDim.x); b += kThreads) {
#pragma unroll
            for (int k = 0; k < kNumAcc; ++k) tot[k] += load_sc1(&partials[b * kNumAcc + k]);
        }
        block_sum<kNumAcc>(tot, scratch);
    }
    if (threadIdx.x == 0) {
        if (CLASS_ONLY) {
            emit_class_sums(tot, sums4, accumulate);
        } else {
            const SurrogateScalars s = make_scalars(abalpha, p_hat, invB);
            finalize(tot, s, invB, out64, grad3, loss);
        }
    }
}

// ---- the loss in ONE launch: tagged row granules, reduced in-launch -------------------------
//
// Every streaming workgroup publishes its row as tagged 8-byte granules (Guideline 16, R2: the
// data is the flag; ONE write-through store per granule, no drain, no ticket): granule = {tag (32
// bits), payload (32 bits)}, a row = the hi and lo halves of its 4 fp64 sums and its 2 counts = 10
// granules. The tag is the call's epoch: every workgroup reads the epoch word (a fixed word of the
// workspace) at its start, and the final reducer advances it as its very last action (when every
// row of the call has arrived, so every workgroup has read it). A granule left over from an earlier
// call -- even one written after that call gave up waiting for it -- carries an older tag and is
// never taken for a current one, and nothing is re-zeroed between calls (tag = epoch | 2^31, so a
// zeroed workspace holds no valid granule either). A poll that times out makes the outputs NaN (a
// group reducer then publishes NaN totals) and sets bit 0 of the workspace's sticky status word
// (dauc_surrogate_status reads it), and the epoch still advances. Nothing waits on a workgroup
// that waits: every row a reducer needs comes from a workgroup that never waits.
// Fixed summation order: bitwise reproducible.
constexpr int kGran = 10;                   // granules per row / group total
constexpr int kMaxPolls = 1 << 22;

struct TailWs {
    unsigned* epoch;               // the workspace's epoch word (kEpochOffset, the same for every B)
    unsigned* status;              // the sticky status word (kStatusOffset): bit 0 = a poll timed out
    unsigned long long* rows;      // [nblocks][kGran]
    unsigned long long* gtot;      // [R][kGran]
};

constexpr size_t kTailHeader = 256;

inline size_t tail_ws_bytes(int64_t nblocks, int R) {
    return kTailHeader + size_t(nblocks + R) * kGran * 8;
}

// The epoch word sits at a FIXED offset of the workspace (in the persistent kernel's counter line,
// whose other words nothing else uses), not in the B-dependent tail region: a stream alternating
// two batch sizes then still advances one epoch, and the epoch a call reads is never a word some
// other B's rows or two-launch region last held.
constexpr size_t kEpochOffset = 128;
static_assert(kEpochOffset + sizeof(unsigned) <= kCounterBytes, "the epoch word lives in the counter line");
// the sticky status word, next to it: set by a reducer that gave up waiting, cleared only by the
// caller (dauc_surrogate_status)
constexpr size_t kStatusOffset = 132;
constexpr unsigned kStatusTimeout = 1u;
static_assert(kStatusOffset + sizeof(unsigned) <= kCounterBytes, "the status word lives in the counter line");

// ws = the whole workspace; the rows start at `offset` (tail_offset(nblocks) + kTailHeader)
inline TailWs tail_ws(void* ws, size_t offset, int64_t nblocks) {
    char* p = static_cast<char*>(ws) + offset;
    TailWs w;
    w.epoch = reinterpret_cast<unsigned*>(static_cast<char*>(ws) + kEpochOffset);
    w.status = reinterpret_cast<unsigned*>(static_cast<char*>(ws) + kStatusOffset);
    w.rows = reinterpret_cast<unsigned long long*>(p + kTailHeader);
    w.gtot = w.rows + nblocks * kGran;
    return w;
}

__device__ __forceinline__ unsigned long long gran(unsigned tag, unsigned payload) {
    return (static_cast<unsigned long long>(tag) << 32) | payload;
}

// Granule k of a row: k = 0..3 the hi halves, 4..7 the lo halves of sums 0..3, 8..9 the counts.
// The total granule k carries:
__device__ __forceinline__ int gran_total(int k) { return k < 8 ? (k & 3) : k - 4; }

// thread k < kGran stores granule k of a row; v = the thread's total gran_total(k)
__device__ __forceinline__ void publish_granule(unsigned long long* row, unsigned tag, double v) {
    const int k = threadIdx.x;
    if (k >= kGran) return;
    const unsigned long long b = static_cast<unsigned long long>(__double_as_longlong(v));
    // counts: exact integers < 2^32
    const unsigned payload = k < 4 ? static_cast<unsigned>(b >> 32) : (k < 8 ? static_cast<unsigned>(b) : static_cast<unsigned>(v));
    __hip_atomic_store((gu64*)(row + k), gran(tag, payload), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// a row's 10 payloads (tags already checked) added to its 6 totals
__device__ __forceinline__ void add_row(const unsigned (&p)[kGran], double (&t)[kRowWords]) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
        t[k] += __longlong_as_double(static_cast<long long>((static_cast<unsigned long long>(p[k]) << 32) | p[k + 4]));
    t[4] += static_cast<double>(p[8]);
    t[5] += static_cast<double>(p[9]);
}

// All granules of one row, loaded together (every load in flight before any is examined): their
// payloads, and a bit per granule that does not carry `tag` yet.
__device__ __forceinline__ unsigned poll_row(const unsigned long long* row, unsigned tag, unsigned (&p)[kGran]) {
    unsigned long long g[kGran];
#pragma unroll
    for (int k = 0; k < kGran; ++k)
        g[k] = __hip_atomic_load((gu64*)(row + k), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned missing = 0u;
#pragma unroll
    for (int k = 0; k < kGran; ++k) {
        p[k] = static_cast<unsigned>(g[k]);
        missing |= unsigned(static_cast<unsigned>(g[k] >> 32) != tag) << k;
    }
    return missing;
}

// Poll until every granule of `row` carries `tag` (bounded; the whole row is re-read each time);
// false on timeout.
__device__ __forceinline__ bool wait_row(const unsigned long long* row, unsigned tag, unsigned missing,
                                         unsigned (&p)[kGran]) {
    for (int polls = 0; missing; ++polls) {
        if (polls >= kMaxPolls) return false;
        __builtin_amdgcn_s_sleep(2);
        missing = poll_row(row, tag, p);
    }
    return true;
}

// ---- the one-launch loss with R EXTRA reducer workgroups that stream nothing (the product) ---
//
// The grid is nblocks + R: the R reducers come after every streaming workgroup and stream nothing,
// so they are polling as soon as the last streaming workgroups are dispatched (round 2's form, in
// which the last 64 STREAMING workgroups reduced, put 6.3-6.6 us after the last row store: every
// group total waited for its reducer's own chunk). Reducer r < R - 1 sums a contiguous group of the
// rows [0, nblocks - K) (one row per thread, only granules not yet current are polled, bounded) and
// publishes the group total the same way; the final reducer (the grid's last workgroup) takes the
// last K rows itself (K / 256 per thread) and the R - 1 group totals, which complete K rows'
// streaming time (~K / 190 us at 2^26) before the last row: after the last row lands one hop is
// left. PLAIN: the epoch is read with a plain load (every read of it precedes the final's store; a
// later call reads it across the kernel boundary). REDUCE = false: the stream with its row stores
// and nobody reducing (a timing variant; its rows carry a tag no call expects, bit 30 set). FAULT
// (tuning builds' variant 23, a test of the timeout path): streaming workgroup nblocks / 2 does not
// publish its row.
template <typename YT, int S, int R, int K, bool PLAIN, int WAVES = 1, bool REDUCE = true, bool FAULT = false>
__global__ __launch_bounds__(kThreads, WAVES) void surrogate_tail_x_kernel(
    const float* __restrict__ h, const YT* __restrict__ y, int64_t B, int64_t nblocks, double invB,
    const float* __restrict__ abalpha, const float* __restrict__ p_hat, float* __restrict__ dh, TailWs ws,
    double* __restrict__ out64, float* __restrict__ grad3, float* __restrict__ loss) {
    static_assert(K % kThreads == 0 && R <= kThreads, "final reducer: K / 256 rows and one group total per thread");
    const unsigned epoch = __builtin_amdgcn_readfirstlane(
        PLAIN ? *ws.epoch : __hip_atomic_load((gu32*)ws.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    // a variant that reduces nothing never advances the epoch: its rows carry a tag no call
    // expects (bit 30 set), so a later call cannot take them for its own
    const unsigned tag = (epoch | 0x80000000u) ^ (REDUCE ? 0u : 0x40000000u);
    const float sa = abalpha[0], sb = abalpha[1], sal = abalpha[2], sp = p_hat[0];
    const int64_t b = blockIdx.x;
    if (b < nblocks) {
        const SurrogateScalars s = make_scalars_v(sa, sb, sal, sp, invB);
        const double v = stream_chunk<YT, false, S>(h, y, B, s, dh, gran_total(threadIdx.x < kGran ? threadIdx.x : 0));
        if (FAULT && b == nblocks / 2) return;
        publish_granule(ws.rows + b * kGran, tag, v);
        return;
    }
    if (!REDUCE) return;  // a timing variant: the stream with its row stores, nobody reducing
    const int64_t r = b - nblocks;
    const bool final_red = r == R - 1;
    // the final's direct rows: [k0, nblocks); groups split [0, k0) into R - 1 contiguous ranges
    const int64_t k0 = nblocks > K ? nblocks - K : 0;
    const int64_t G = (k0 + R - 2) / (R - 1);
    __shared__ double scratch[kNumAcc * kWaves];
    __shared__ int bad;
    if (threadIdx.x == 0) bad = 0;
    bool ok = true;
    double tot[kNumAcc];
#pragma unroll
    for (int k = 0; k < kNumAcc; ++k) tot[k] = 0.0;
    if (!final_red) {
        const int64_t g0 = r * G < k0 ? r * G : k0, g1 = g0 + G < k0 ? g0 + G : k0;
        for (int64_t i = g0 + threadIdx.x; i < g1; i += kThreads) {
            unsigned p[kGran];
            const unsigned miss = poll_row(ws.rows + i * kGran, tag, p);
            if (!wait_row(ws.rows + i * kGran, tag, miss, p)) {
                ok = false;
                break;
            }
            add_row(p, tot);
        }
    } else {
        // every poll of the thread in flight before any wait: its K / 256 rows and group total t
        constexpr int KR = K / kThreads;
        unsigned p[KR + 1][kGran], miss[KR + 1];
#pragma unroll
        for (int j = 0; j < KR; ++j) {
            const int64_t i = k0 + int64_t(j) * kThreads + threadIdx.x;
            miss[j] = i < nblocks ? poll_row(ws.rows + i * kGran, tag, p[j]) : 0u;
            if (i >= nblocks) {
#pragma unroll
                for (int k = 0; k < kGran; ++k) p[j][k] = 0u;
            }
        }
        const bool holds = threadIdx.x < R - 1;
        miss[KR] = holds ? poll_row(ws.gtot + threadIdx.x * kGran, tag, p[KR]) : 0u;
        if (!holds) {
#pragma unroll
            for (int k = 0; k < kGran; ++k) p[KR][k] = 0u;
        }
#pragma unroll
        for (int j = 0; j < KR; ++j) {
            const int64_t i = k0 + int64_t(j) * kThreads + threadIdx.x;
            if (i < nblocks && !wait_row(ws.rows + i * kGran, tag, miss[j], p[j])) ok = false;
        }
        if (holds && !wait_row(ws.gtot + threadIdx.x * kGran, tag, miss[KR], p[KR])) ok = false;
        // fixed order per thread: its rows by index, then its group total
#pragma unroll
        for (int j = 0; j <= KR; ++j) add_row(p[j], tot);
    }
    __syncthreads();  // orders bad = 0 before any thread's bad = 1
    if (!ok) bad = 1;
    block_sum<kNumAcc>(tot, scratch);  // its barriers order the flag
    ok = bad == 0;
    if (!ok) {
#pragma unroll
        for (int k = 0; k < kNumAcc; ++k) tot[k] = __builtin_nan("");
        // reported, not only NaN: the caller tells a timed-out reduction from a diverged loss
        if (threadIdx.x == 0) atomicOr(ws.status, kStatusTimeout);
    }
    if (!final_red) {
        double v = tot[0];
#pragma unroll
        for (int k = 1; k < kNumAcc; ++k)
            if (threadIdx.x < kGran && gran_total(threadIdx.x) == k) v = tot[k];
        publish_granule(ws.gtot + r * kGran, tag, v);
        return;
    }
    if (threadIdx.x == 0) {
        finalize(tot, make_scalars_v(sa, sb, sal, sp, invB), invB, out64, grad3, loss);
        // the call's last action: every workgroup has read the epoch (its row or total has arrived)
        __hip_atomic_store((gu32*)ws.epoch, epoch + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Default chunk geometry (scripts/micro_kernels.py --which surrogate, profiles/r01-r02).
constexpr int kChunkSlots = 4;
// the one-launch loss's extra-reducer tail (surrogate_tail_x_kernel): 128 reducer workgroups, the
// final one taking the grid's last 512 rows itself; at B = 2^26 (profiles/r03/a): 92.3 us vs 94.4 for
// round 2's 64 streaming reducers and 88.2 for the stream with its row stores alone (32 / 64 / 256
// reducers, 256 / 1024 / 1536 final rows, plain or atomic epoch loads and round 3's early-reducer
// form were measured there too, and removed in round 4)
constexpr int kTailXReducers = 128;
constexpr int kTailFinalRows = 512;
// Unit-stride batches at least this large take the chunked kernels; smaller ones are
// latency-bound and stay on the single-ticket persistent kernel.
constexpr int64_t kChunkMinB = int64_t(1) << 22;

inline int64_t chunk_blocks(int64_t B) { return (B + chunk_elems(kChunkSlots) - 1) / chunk_elems(kChunkSlots); }

// workspace regions after the persistent kernel's: the two-launch form's rows + reduce slots, then
// the tail kernel's header and granule rows
inline size_t chunk_region_bytes(int64_t nblocks) {
    return size_t(nblocks) * kRowWords * 8 + kCounterBytes + size_t(reduce_blocks(nblocks)) * kNumAcc * 8;
}

inline size_t tail_offset(int64_t nblocks) {
    return kPersistentBytes + (chunk_region_bytes(nblocks) + 255) / 256 * 256;
}

template <typename YT, int R, int K, bool PLAIN, int WAVES = 1, bool REDUCE = true, bool FAULT = false>
int launch_tail_x(const float* h, const YT* y, int64_t B, const float* abalpha, const float* p_hat, float* dh,
                  double* out64, float* grad3, float* loss, void* ws, size_t ws_bytes, hipStream_t st) {
    const int64_t nblocks = chunk_blocks(B);
    if (nblocks + R > 0x7fffffffLL) return DAUC_EINVAL;
    if (ws == nullptr || ws_bytes < tail_offset(nblocks) + tail_ws_bytes(nblocks, R)) return DAUC_EINVAL;
    const TailWs w = tail_ws(ws, tail_offset(nblocks), nblocks);
    hipLaunchKernelGGL((surrogate_tail_x_kernel<YT, kChunkSlots, R, K, PLAIN, WAVES, REDUCE, FAULT>),
                       dim3(static_cast<unsigned>(nblocks + R)), dim3(kThreads), 0, st, h, y, B, nblocks,
                       1.0 / static_cast<double>(B), abalpha, p_hat, dh, w, out64, grad3, loss);
    return launch_status();
}

template <typename YT, bool CLASS_ONLY>
int launch_chunk(const float* h, const YT* y, int64_t B, const float* abalpha, const float* p_hat, float* dh,
                 double* out64, float* grad3, float* loss, double* sums4, int accumulate, void* ws, size_t ws_bytes,
                 hipStream_t st, bool reduce = true) {
    const int64_t nblocks = chunk_blocks(B);
    if (nblocks > 0x7fffffffLL) return DAUC_EINVAL;
    if (ws == nullptr || ws_bytes < kPersistentBytes + chunk_region_bytes(nblocks)) return DAUC_EINVAL;
    double* rows = reinterpret_cast<double*>(static_cast<char*>(ws) + kPersistentBytes);
    unsigned* counter = reinterpret_cast<unsigned*>(rows + nblocks * kRowWords);
    double* partials = reinterpret_cast<double*>(reinterpret_cast<char*>(counter) + kCounterBytes);
    const double invB = 1.0 / static_cast<double>(B);
    hipLaunchKernelGGL((surrogate_chunk_kernel<YT, CLASS_ONLY, kChunkSlots>), dim3(static_cast<unsigned>(nblocks)),
                       dim3(kThreads), 0, st, h, y, B, invB, abalpha, p_hat, dh, rows);
    int rc = launch_status();
    if (rc || !reduce) return rc;
    hipLaunchKernelGGL((surrogate_rows_reduce_kernel<CLASS_ONLY>), dim3(static_cast<unsigned>(reduce_blocks(nblocks))),
                       dim3(kThreads), 0, st, rows, nblocks, partials, counter, invB, abalpha, p_hat, out64, grad3,
                       loss, sums4, accumulate);
    return launch_status();
}

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
            per_cu = per_cu < 2 ? per_cu : 2;
            cached = cus * per_cu;
        }
    }
    return cached;
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// variant (tuning builds only; int8 labels with a loss): 0 = default dispatch, 1 = the persistent
// kernel at any B, 2 = the two-launch form (stream + row-reduce launch), 3 = the streaming kernel
// alone (no reduce, no scalars), 20 = the product's one-launch kernel at any unit-stride B, 22 =
// its stream with the tagged row stores and nobody reducing (the hand-off's cost, by difference)
template <bool CLASS_ONLY, typename YT>
int launch_surrogate(const float* h, int64_t hs, const YT* y, int64_t B, const float* abalpha,
                     const float* p_hat, float* dh, int64_t dhs, double* out64, float* grad3,
                     float* loss, double* sums4, int accumulate, void* ws, size_t ws_bytes,
                     hipStream_t st, int variant = 0) {
    const bool unit = hs == 1 && aligned16(h) &&
                      (reinterpret_cast<uintptr_t>(y) % (kVec * sizeof(YT))) == 0 &&
                      (CLASS_ONLY || dh == nullptr || (dhs == 1 && aligned16(dh)));
#ifdef DAUC_TUNING
    if (unit && variant >= 2) {
        if constexpr (!CLASS_ONLY && sizeof(YT) == 1) {
            switch (variant) {
                case 2: return launch_chunk<YT, false>(h, y, B, abalpha, p_hat, dh, out64, grad3, loss, sums4, accumulate, ws, ws_bytes, st);
                case 3: return launch_chunk<YT, false>(h, y, B, abalpha, p_hat, dh, out64, grad3, loss, sums4, accumulate, ws, ws_bytes, st, false);
                case 20: return launch_tail_x<YT, kTailXReducers, kTailFinalRows, true, 8>(h, y, B, abalpha, p_hat, dh, out64, grad3, loss, ws, ws_bytes, st);
                case 22: return launch_tail_x<YT, kTailXReducers, kTailFinalRows, true, 8, false>(h, y, B, abalpha, p_hat, dh, out64, grad3, loss, ws, ws_bytes, st);
                case 23: return launch_tail_x<YT, kTailXReducers, kTailFinalRows, true, 8, true, true>(h, y, B, abalpha, p_hat, dh, out64, grad3, loss, ws, ws_bytes, st);
                default: return DAUC_EINVAL;
            }
        }
        return DAUC_EINVAL;
    }
#else
    (void)variant;
#endif
    if (unit && variant == 0 && B >= kChunkMinB) {
        // the loss: the stream with its row reduce done by kTailXReducers extra workgroups that
        // stream nothing (one launch); the class sums keep the two-launch form
        if constexpr (!CLASS_ONLY)
            // int8 labels: the register bound of 8 waves per SIMD costs no spill (wider labels would spill)
            return launch_tail_x<YT, kTailXReducers, kTailFinalRows, true, sizeof(YT) == 1 ? 8 : 1>(
                h, y, B, abalpha, p_hat, dh, out64, grad3, loss, ws, ws_bytes, st);
        else
            return launch_chunk<YT, true>(h, y, B, abalpha, p_hat, dh, out64, grad3, loss, sums4, accumulate, ws,
                                          ws_bytes, st);
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
    // the chunked kernels: the two-launch form's region, then the tail kernel's
    const int64_t nb = chunk_blocks(B);
    const size_t chunked = tail_offset(nb) + tail_ws_bytes(nb, kTailXReducers);
    return persistent > chunked ? persistent : chunked;
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

#ifdef DAUC_TUNING
int dauc_surrogate_fwdbwd_variant(const float* h, int64_t h_stride, const void* y, int y_dtype, int64_t B,
                                  const float* abalpha, const float* p_hat, float* dh, int64_t dh_stride,
                                  double* out64, float* grad3, float* loss, void* workspace,
                                  size_t workspace_bytes, int variant, dauc_stream_t stream) {
    if (B <= 0 || h == nullptr || y == nullptr || abalpha == nullptr || p_hat == nullptr ||
        h_stride <= 0 || (dh != nullptr && dh_stride <= 0) || variant < 0 || variant > 23)
        return DAUC_EINVAL;
    return dispatch_labels<false>(h, h_stride, y, y_dtype, B, abalpha, p_hat, dh, dh_stride, out64,
                                  grad3, loss, nullptr, 0, workspace, workspace_bytes,
                                  as_hip(stream), variant);
}
#endif

int dauc_surrogate_status(void* workspace, size_t workspace_bytes, unsigned* status_out, int clear,
                          dauc_stream_t stream) {
    if (workspace == nullptr || status_out == nullptr || workspace_bytes < kStatusOffset + sizeof(unsigned))
        return DAUC_EINVAL;
    hipStream_t st = as_hip(stream);
    unsigned* word = reinterpret_cast<unsigned*>(static_cast<char*>(workspace) + kStatusOffset);
    hipError_t e;
    if ((e = hipMemcpyAsync(status_out, word, sizeof(unsigned), hipMemcpyDeviceToHost, st)) != hipSuccess ||
        (e = hipStreamSynchronize(st)) != hipSuccess)
        return -static_cast<int>(e);
    if (clear && *status_out != 0u && (e = hipMemsetAsync(word, 0, sizeof(unsigned), st)) != hipSuccess)
        return -static_cast<int>(e);
    return DAUC_OK;
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
