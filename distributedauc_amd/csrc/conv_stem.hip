// The backbone stem: the 7x7 / stride 2 / pad 3 convolution of the 3-channel image into 64
// channels, forward and weight gradient, channels-last bf16 on MFMA with fp32 accumulation.
//
// Reference: imagenet/resnet.py:145 (conv1 = Conv2d(3, 64, kernel_size=7, stride=2, padding=3)),
// trained by main.py:311-326. torch under bf16 autocast runs MIOpen's implicit-GEMM kernels for it:
// ResNet-50 b256, forward ~360 us and backward-weights ~350 us (+ a zero-fill and two casts) for
// 60 GFLOP each, because a 3-channel, 147-deep reduction fits neither kernel's tiling. Both are
// bound here by HBM (the 411 MB activation written / read once), not by the MFMA.
//
// Layout: x [N][H][W][3], y / dy [N][Ho][Wo][64], weight [64][7][7][3] (the channels-last memory
// order of [64, 3, 7, 7]). For output pixel (n, oh, ow) and kernel row kh, the 21 inputs
// (kw, ci) are CONTIGUOUS in x: x[n][2oh - 3 + kh][2ow - 3 + kw][ci] = row_kh[6 ow + 3 kw + ci]
// of the staged input row. So the reduction index is k' = 24 kh + j (j = 3 kw + ci < 21; 21..23
// and kh = 7 carry zero weights): K' = 192 = 6 MFMA k-steps, and a lane's 8 consecutive k' of one
// pixel are 8 consecutive bf16 of one staged row (read as 5 aligned words and realigned).
//
// A task is one output row segment (n, oh, ow0 .. ow0 + 127): its 7 input rows (+ a zero row)
// are staged into LDS (zeros outside the image), then
//   forward: D[co][px] = W'[co][k'] * P[k'][px]: the weights as A fragments in registers (loaded
//            once per workgroup), the patches as B fragments read straight from the rows; the
//            64 x 128 bf16 result goes through an LDS tile to 16-byte coalesced stores.
//   wgrad:   D[co][k'] = dy^T[co][px] * P[px][k']: dy's [px][co] tile read with the transposing
//            LDS read (ds_read_b64_tr_b16), the patches gathered 2 bytes per pixel; each
//            workgroup accumulates its tasks in registers and writes one fp32 slab, summed in
//            workgroup order by dauc_slab_sum: bitwise reproducible.
// Workgroups are persistent (a fixed grid striding over the tasks); the next task's input rows
// (and dy tile) are loaded into registers while the current one computes.

#include <hip/hip_bf16.h>

#include "dauc_internal.h"

namespace dauc {
namespace {

typedef short v4s __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) short lds_short;
typedef __attribute__((address_space(3))) v4s lds_v4s;
typedef __attribute__((address_space(3))) unsigned lds_u32;
typedef __attribute__((address_space(3))) u32x4 lds_u32x4;

constexpr int kThreads = 256;             // 4 waves
constexpr int kSeg = 128;                 // output pixels per task
constexpr int kInRow = 800;               // staged input row, bf16 elements (>= 3 * (2 * 127 + 7) = 783 and
                                          // >= 6 * 127 + 23 + 1 read by the last pixel's last k-step)
constexpr int kInElems = 8 * kInRow;      // 7 kernel rows + a zero row
constexpr int kChunks = kInElems / 8;    // 16-byte chunks per staged task (100 per row)
constexpr int kChunkPer = (kChunks + kThreads - 1) / kThreads;  // 4 per thread
constexpr int kKp = 192;                  // padded reduction length of the forward
constexpr int kOutRow = 72;               // forward output tile row (64 channels + 8)
constexpr int kDyRow = 80;                // wgrad dy tile row (64 channels + 16: conflict-free transposing reads)
constexpr int kWElems = 64 * 147;         // weight / gradient elements
static_assert(kInElems % kThreads == 0, "input staging");

struct StemGeom {
    int N, H, W, Ho, Wo;
    int segs;     // ceil(Wo / kSeg)
    int tasks;    // N * Ho * segs
    int sgroups;  // wgrad: slab groups of the two-level slab sum (1: one level)
};

// this workgroup's tasks t = first, first + step, ... < end. Workgroups go to the 8 XCDs round
// robin (blockIdx.x % 8), each with its own L2: XCD x takes the x-th eighth of the tasks, so the
// tasks running at once on one XCD are consecutive output rows and share their input rows in that
// L2 (a grid-stride order spread them over all 8: ~3.5 fetches of every input row from beyond L2)
__device__ __forceinline__ void task_range(const StemGeom& g, int& first, int& end, int& step) {
    const int G = static_cast<int>(gridDim.x), b = static_cast<int>(blockIdx.x);
    if (G % 8 != 0) {
        first = b;
        end = g.tasks;
        step = G;
        return;
    }
    const int xcd = b % 8, per = G / 8;
    const int lo = static_cast<int>(int64_t(g.tasks) * xcd / 8), hi = static_cast<int>(int64_t(g.tasks) * (xcd + 1) / 8);
    first = lo + b / 8;
    end = hi;
    step = per;
}

__device__ __forceinline__ void task_coords(const StemGeom& g, int t, int& n, int& oh, int& ow0) {
    const int row = t / g.segs;
    ow0 = (t - row * g.segs) * kSeg;
    n = row / g.Ho;
    oh = row - n * g.Ho;
}

// Staged row kh holds input row ih = 2 oh - 3 + kh from the 16-byte-aligned chunk at or below the
// run's first element g0 = (n H + ih) 3W + 3 (2 ow0 - 3): position p of the LDS row is element
// (g0 & ~7) + p of x, so the run starts at position sh(kh) = g0 & 7 and every chunk lands whole
// (one 16-byte load, one 16-byte LDS store; x 16-byte aligned). Elements outside the image row are
// zeroed at the store. A chunk holding a valid element cannot leave x's allocation (an aligned
// 16-byte block around a valid byte); a chunk with none is not used (its load reads chunk 0).
__device__ __forceinline__ int row_shift(const StemGeom& g, int n, int oh, int ow0, int kh) {
    return ((n * g.H + 2 * oh - 3 + kh) * 3 * g.W + 3 * (2 * ow0 - 3)) & 7;
}

struct RowStage {
    u32x4 c[kChunkPer];
    unsigned lohi;  // per chunk u, bits 8u .. 8u + 7: the valid element range [lo, hi) (4 bits each)
};

// this thread's chunks u: chunk index q = tid + 256 u of the task's [8 rows][100 chunks]. The loads
// are unconditional and their validity goes to `lohi`, applied when the chunks are stored to LDS: a
// select right after a load would make the wave wait for it here instead of across the MFMAs.
__device__ __forceinline__ void load_rows(RowStage& st, const unsigned short* __restrict__ x, const StemGeom& g,
                                          int t) {
    int n, oh, ow0;
    task_coords(g, t, n, oh, ow0);
    const int rowlen = 3 * g.W;
    unsigned lohi = 0u;
#pragma unroll
    for (int u = 0; u < kChunkPer; ++u) {
        const int q = threadIdx.x + kThreads * u;
        const int kh = q / (kInRow / 8), k = q - kh * (kInRow / 8);
        const int ih = 2 * oh - 3 + kh;
        const int rs = (n * g.H + ih) * rowlen;                      // element of (n, ih, 0, 0)
        const int cb = ((rs + 3 * (2 * ow0 - 3)) & ~7) + 8 * k;        // this chunk's first element
        const bool row_ok = (q < kChunks) & (kh < 7) & (ih >= 0) & (ih < g.H);
        const int lo = min(max(rs - cb, 0), 8), hi = min(max(rs + rowlen - cb, 0), 8);
        const bool any = row_ok & (lo < hi);
        st.c[u] = *reinterpret_cast<const u32x4*>(x + (any ? cb : 0));
        lohi |= static_cast<unsigned>(any ? (lo | (hi << 4)) : 0) << (8 * u);
    }
    st.lohi = lohi;
}

// FAST: skip the masks when every lane's chunk lies wholly inside the image (a wave-uniform test;
// the weight-gradient kernel: 181.5 -> 177.4 us; the forward measured slower with it)
template <bool FAST>
__device__ __forceinline__ void store_rows(const RowStage& st, lds_short* in) {
#pragma unroll
    for (int u = 0; u < kChunkPer; ++u) {
        const int q = threadIdx.x + kThreads * u;
        if (q >= kChunks) break;
        const unsigned lh = (st.lohi >> (8 * u)) & 0xff;
        u32x4 v = st.c[u];
        if (!FAST || !__all(lh == 0x80u)) {  // some lane's chunk is not wholly inside the image
            const int lo = lh & 15, hi = lh >> 4;
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                const unsigned m = (((2 * d >= lo) & (2 * d < hi)) ? 0x0000ffffu : 0u) |
                                   (((2 * d + 1 >= lo) & (2 * d + 1 < hi)) ? 0xffff0000u : 0u);
                v[d] &= m;
            }
        }
        const int kh = q / (kInRow / 8), k = q - kh * (kInRow / 8);
        *(lds_u32x4*)(in + (kh * kInRow + 8 * k)) = v;
    }
}

// ------------------------------------------------------------------------------------------------
// forward

__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(2))) void stem_fwd_kernel(const unsigned short* __restrict__ x,
                                                            const unsigned short* __restrict__ w, StemGeom g,
                                                            unsigned short* __restrict__ y) {
    __shared__ short in_s[kInElems];
    __shared__ short out_s[kSeg * kOutRow];
    __shared__ short w_s[64 * kKp];
    lds_short* in = (lds_short*)in_s;
    lds_short* out = (lds_short*)out_s;
    lds_short* wl = (lds_short*)w_s;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int grp = lane >> 4, col = lane & 15;

    // the padded weight W'[co][k'] (zeros at j >= 21 and kh = 7), once per workgroup
    for (int i = tid; i < 64 * kKp; i += kThreads) {
        const int co = i / kKp, kp = i - co * kKp;
        const int kh = kp / 24, j = kp - kh * 24;
        wl[i] = (kh < 7 && j < 21) ? static_cast<short>(w[co * 147 + kh * 21 + j]) : short(0);
    }
    int t, t_end, t_step;
    task_range(g, t, t_end, t_step);
    RowStage st;
    if (t < t_end) load_rows(st, x, g, t);
    __syncthreads();
    // A fragments: lane (grp, col) holds W'[16 ct + col][32 s + 8 grp .. + 7]
    bf16x8 wa[4][6];
#pragma unroll
    for (int ct = 0; ct < 4; ++ct)
#pragma unroll
        for (int s = 0; s < 6; ++s)
            wa[ct][s] = __builtin_bit_cast(bf16x8, *(const lds_u32x4*)(wl + ((16 * ct + col) * kKp + 32 * s + 8 * grp)));
    // this lane's k' offset into the staged rows per k-step: row kh, element j0 of the pixel's run
    // (+ the row's shift, per task)
    int koff[6];
    // bit s: this lane's 8 k' of k-step s are j = 16 .. 23 of a row, whose last three (j >= 21) are
    // the input column just right of the 7-wide window. Their weights are zero, but 0 x Inf is NaN:
    // those B elements are zeroed so a non-finite neighbour cannot reach the output (torch's 7x7
    // conv never reads it)
    unsigned jtail = 0u;
#pragma unroll
    for (int s = 0; s < 6; ++s) {
        const int kp0 = 32 * s + 8 * grp;
        koff[s] = (kp0 / 24) * kInRow + kp0 % 24;
        jtail |= (kp0 % 24 == 16 ? 1u : 0u) << s;
    }

    for (; t < t_end; t += t_step) {
        int n, oh, ow0;
        task_coords(g, t, n, oh, ow0);
        const int count = g.Wo - ow0 < kSeg ? g.Wo - ow0 : kSeg;
        int kofs[6];
#pragma unroll
        for (int s = 0; s < 6; ++s) kofs[s] = koff[s] + row_shift(g, n, oh, ow0, (32 * s + 8 * grp) / 24);
        __syncthreads();  // the previous task's reads of in / out are done
        store_rows<false>(st, in);
        __syncthreads();
        if (t + t_step < t_end) load_rows(st, x, g, t + t_step);  // in flight meanwhile
#pragma unroll
        for (int pi = 0; pi < 2; ++pi) {
            const int pt = wave + 4 * pi;  // pixel tile (wave-uniform)
            if (16 * pt >= count) break;
            const int px = 16 * pt + col;
            f32x4v acc[4];
#pragma unroll
            for (int ct = 0; ct < 4; ++ct) acc[ct] = f32x4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < 6; ++s) {
                // 8 bf16 at any 2-byte offset: 5 aligned words, realigned by 0 or 2 bytes
                const int e = kofs[s] + 6 * px;
                const lds_u32* p = (const lds_u32*)(in + (e & ~1));
                const unsigned sb = (e & 1) * 16;
                const unsigned w0 = p[0], w1 = p[1], w2 = p[2], w3 = p[3], w4 = p[4];
                const bool tail = (jtail >> s) & 1u;
                const u32x4 v = {__builtin_amdgcn_alignbit(w1, w0, sb), __builtin_amdgcn_alignbit(w2, w1, sb),
                                 __builtin_amdgcn_alignbit(w3, w2, sb) & (tail ? 0x0000ffffu : 0xffffffffu),
                                 tail ? 0u : __builtin_amdgcn_alignbit(w4, w3, sb)};
                const bf16x8 b = __builtin_bit_cast(bf16x8, v);
#pragma unroll
                for (int ct = 0; ct < 4; ++ct) acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[ct][s], b, acc[ct], 0, 0, 0);
            }
            // D[co = 16 ct + 4 grp + i][px = col] -> bf16 (round to nearest even), 8 bytes per lane
#pragma unroll
            for (int ct = 0; ct < 4; ++ct) {
                v4s o;
#pragma unroll
                for (int i = 0; i < 4; ++i) o[i] = __bfloat16_as_short(__float2bfloat16(acc[ct][i]));
                *(lds_v4s*)(out + (px * kOutRow + 16 * ct + 4 * grp)) = o;
            }
        }
        __syncthreads();
        // the segment's [count][64] bf16 rows are contiguous in y: 16-byte stores
        unsigned short* yrow = y + (static_cast<int64_t>(n * g.Ho + oh) * g.Wo + ow0) * 64;
#pragma unroll
        for (int u = 0; u < kSeg * 8 / kThreads; ++u) {
            const int q = tid + kThreads * u, p = q >> 3, v = q & 7;
            if (p < count)
                *reinterpret_cast<u32x4*>(yrow + (p * 64 + 8 * v)) = *(const lds_u32x4*)(out + (p * kOutRow + 8 * v));
        }
    }
}

// ------------------------------------------------------------------------------------------------
// weight gradient

__device__ __forceinline__ v4s tr_at(const lds_short* p) { return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)p); }

// this thread's 4 16-byte vectors of task t's dy tile [128 px][64 co] (bit u of the result: vector u
// lies before the row's end; the others are stored as zeros)
__device__ __forceinline__ unsigned load_dy(u32x4 (&d)[4], const unsigned short* __restrict__ dy, const StemGeom& g,
                                            int t) {
    int n, oh, ow0;
    task_coords(g, t, n, oh, ow0);
    const int count = g.Wo - ow0 < kSeg ? g.Wo - ow0 : kSeg;
    const unsigned short* row = dy + (static_cast<int64_t>(n * g.Ho + oh) * g.Wo + ow0) * 64;
    unsigned okm = 0u;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int q = threadIdx.x + kThreads * u, p = q >> 3, v = q & 7;
        const bool ok = p < count;
        d[u] = *reinterpret_cast<const u32x4*>(row + ((ok ? p : 0) * 64 + 8 * v));
        okm |= ok ? (1u << u) : 0u;
    }
    return okm;
}

__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(2))) void stem_wgrad_kernel(const unsigned short* __restrict__ x,
                                                              const unsigned short* __restrict__ dy, StemGeom g,
                                                              float* __restrict__ slabs) {
    __shared__ short in_s[kInElems];
    __shared__ short dy_s[kSeg * kDyRow];
    lds_short* in = (lds_short*)in_s;
    lds_short* dyl = (lds_short*)dy_s;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int grp = lane >> 4, col = lane & 15;

    // pixel order of a k-step (any order sums the same products): lane group grp's 8 values are
    // pixels 4 grp + 0..3 (transposing read h = 0) and 16 + 4 grp + 0..3 (h = 1)
    int aoff[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) aoff[h] = (16 * h + 4 * grp + ((lane & 15) >> 2)) * kDyRow + 4 * (lane & 3);
    // this wave's k' tiles nt = wave, wave + 4, wave + 8 (< 11: k' < 176 covers kh <= 6), lane column k'
    int boff[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const int kp = 16 * (wave + 4 * i) + col;
        boff[i] = (kp / 24) * kInRow + kp % 24 + 6 * 4 * grp;
    }
    const int ntiles = wave + 8 < 11 ? 3 : 2;

    f32x4v acc[4][3];
#pragma unroll
    for (int ct = 0; ct < 4; ++ct)
#pragma unroll
        for (int i = 0; i < 3; ++i) acc[ct][i] = f32x4v{0.f, 0.f, 0.f, 0.f};

    int t, t_end, t_step;
    task_range(g, t, t_end, t_step);
    RowStage st;
    u32x4 d[4];
    unsigned dm = 0u;
    if (t < t_end) {
        load_rows(st, x, g, t);
        dm = load_dy(d, dy, g, t);
    }
    for (; t < t_end; t += t_step) {
        int n, oh, ow0;
        task_coords(g, t, n, oh, ow0);
        const int count = g.Wo - ow0 < kSeg ? g.Wo - ow0 : kSeg;
        int bofs[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) bofs[i] = boff[i] + row_shift(g, n, oh, ow0, (16 * (wave + 4 * i) + col) / 24);
        __syncthreads();
        store_rows<true>(st, in);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int q = tid + kThreads * u;
            const unsigned m = ((dm >> u) & 1u) ? ~0u : 0u;
            *(lds_u32x4*)(dyl + ((q >> 3) * kDyRow + 8 * (q & 7))) = u32x4{d[u][0] & m, d[u][1] & m, d[u][2] & m, d[u][3] & m};
        }
        __syncthreads();
        if (t + t_step < t_end) {
            load_rows(st, x, g, t + t_step);
            dm = load_dy(d, dy, g, t + t_step);
        }
        for (int s = 0; 32 * s < count; ++s) {
            bf16x8 fa[4];
#pragma unroll
            for (int ct = 0; ct < 4; ++ct) {
                const v4s f2[2] = {tr_at(dyl + (aoff[0] + 32 * s * kDyRow + 16 * ct)),
                                   tr_at(dyl + (aoff[1] + 32 * s * kDyRow + 16 * ct))};
                fa[ct] = *reinterpret_cast<const bf16x8*>(f2);
            }
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                if (i == 2 && ntiles == 2) break;
                // B[px][k']: pixels 32 s + {4 grp + 0..3, 16 + 4 grp + 0..3}, 6 elements apart
                const lds_short* p = in + (bofs[i] + 6 * 32 * s);
                s16x8 b;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    b[j] = p[6 * j];
                    b[4 + j] = p[6 * (16 + j)];
                }
                const bf16x8 fb = __builtin_bit_cast(bf16x8, b);
#pragma unroll
                for (int ct = 0; ct < 4; ++ct)
                    acc[ct][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[ct], fb, acc[ct][i], 0, 0, 0);
            }
        }
    }
    // D[co = 16 ct + 4 grp + e][k' = 16 nt + col] -> this workgroup's slab [co][kh][kw][ci]
    // two-level sum: workgroup b's slab is row b % G1 of group b / G1, stored [G1][groups] so the
    // first level is one slab sum of G1 slabs of groups x 9,408 floats (a wide grid)
    const int b = blockIdx.x, groups = static_cast<int>(gridDim.x) / g.sgroups;
    const int slot = g.sgroups > 1 ? (b % g.sgroups) * groups + b / g.sgroups : b;
    float* slab = slabs + static_cast<int64_t>(slot) * kWElems;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        if (i == 2 && ntiles == 2) break;
        const int kp = 16 * (wave + 4 * i) + col;
        const int kh = kp / 24, j = kp - kh * 24;
        if (kh < 7 && j < 21) {
#pragma unroll
            for (int ct = 0; ct < 4; ++ct)
#pragma unroll
                for (int e = 0; e < 4; ++e) slab[(16 * ct + 4 * grp + e) * 147 + kh * 21 + j] = acc[ct][i][e];
        }
    }
}

bool stem_geom(int64_t N, int H, int W, int Ho, int Wo, StemGeom& g) {
    if (N < 1 || H < 1 || W < 1 || Ho != (H - 1) / 2 + 1 || Wo != (W - 1) / 2 + 1) return false;
    // 32-bit element offsets: N * H * W * 3 and N * Ho * Wo * 64 (+ a segment) < 2^31
    if (N * H * int64_t(W) * 3 >= (int64_t(1) << 31) || (N * Ho * int64_t(Wo) + kSeg) * 64 >= (int64_t(1) << 31))
        return false;
    g.N = static_cast<int>(N);
    g.H = H;
    g.W = W;
    g.Ho = Ho;
    g.Wo = Wo;
    g.segs = (Wo + kSeg - 1) / kSeg;
    const int64_t tasks = N * Ho * int64_t(g.segs);
    if (tasks >= (int64_t(1) << 31)) return false;
    g.tasks = static_cast<int>(tasks);
    g.sgroups = 1;
    return true;
}

// persistent grids: workgroups per CU as registers allow (forward 196 VGPRs: 2; wgrad 155: 3)
constexpr int kFwdGrid = 512;
constexpr int kWgradGrid = 768;
constexpr int kSlabGroups = 32;  // first level of the weight-gradient slab sum: 32 slabs of 24 x 9,408 floats

}  // namespace
}  // namespace dauc

using namespace dauc;

extern "C" {

int dauc_conv7x7s2_stem_forward(const void* x, const void* w, int dtype, int64_t N, int H, int W, int Ho, int Wo,
                                void* y, dauc_stream_t stream) {
    if (x == nullptr || w == nullptr || y == nullptr || dtype != DAUC_DTYPE_BF16) return DAUC_EINVAL;
    if (((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y)) & 15u) || (reinterpret_cast<uintptr_t>(w) & 1u))
        return DAUC_EINVAL;
    StemGeom g;
    if (!stem_geom(N, H, W, Ho, Wo, g)) return DAUC_EINVAL;
    const int grid = g.tasks < kFwdGrid ? g.tasks : kFwdGrid;
    hipLaunchKernelGGL(stem_fwd_kernel, dim3(grid), dim3(kThreads), 0, as_hip(stream),
                       static_cast<const unsigned short*>(x), static_cast<const unsigned short*>(w), g,
                       static_cast<unsigned short*>(y));
    return launch_status();
}

size_t dauc_conv7x7s2_stem_wgrad_workspace_size(int64_t N, int Ho, int Wo) {
    if (N < 1 || Ho < 1 || Wo < 1) return 0;
    const int64_t tasks = N * Ho * ((Wo + kSeg - 1) / kSeg);
    const int64_t grid = tasks < kWgradGrid ? tasks : kWgradGrid;
    const int64_t second = grid == kWgradGrid ? grid / kSlabGroups : 0;  // the first level's output
    return grid > 1 ? size_t(grid + second) * kWElems * sizeof(float) : 0;
}

int dauc_conv7x7s2_stem_wgrad(const void* x, const void* dy, int dtype, int64_t N, int H, int W, int Ho, int Wo,
                              float* dw, void* workspace, size_t workspace_bytes, dauc_stream_t stream) {
    if (x == nullptr || dy == nullptr || dw == nullptr || dtype != DAUC_DTYPE_BF16) return DAUC_EINVAL;
    if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(dy) | reinterpret_cast<uintptr_t>(dw)) & 15u)
        return DAUC_EINVAL;
    StemGeom g;
    if (!stem_geom(N, H, W, Ho, Wo, g)) return DAUC_EINVAL;
    const int grid = g.tasks < kWgradGrid ? g.tasks : kWgradGrid;
    const size_t need = dauc_conv7x7s2_stem_wgrad_workspace_size(N, Ho, Wo);
    if (need && (workspace == nullptr || workspace_bytes < need || (reinterpret_cast<uintptr_t>(workspace) & 15u)))
        return DAUC_EINVAL;
    g.sgroups = grid == kWgradGrid ? kSlabGroups : 1;
    float* target = grid > 1 ? static_cast<float*>(workspace) : dw;
    hipLaunchKernelGGL(stem_wgrad_kernel, dim3(grid), dim3(kThreads), 0, as_hip(stream),
                       static_cast<const unsigned short*>(x), static_cast<const unsigned short*>(dy), g, target);
    int rc = launch_status();
    if (rc != DAUC_OK || grid == 1) return rc;
    if (g.sgroups == 1) return dauc_slab_sum(target, grid, kWElems, dw, stream);
    const int groups = grid / g.sgroups;
    float* level1 = target + int64_t(grid) * kWElems;
    rc = dauc_slab_sum(target, g.sgroups, int64_t(groups) * kWElems, level1, stream);
    if (rc != DAUC_OK) return rc;
    return dauc_slab_sum(level1, groups, kWElems, dw, stream);
}

}  // extern "C"
