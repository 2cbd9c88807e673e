// Weight gradient of the backbone's 3x3 convolutions (pad 1, stride 1 or 2), channels-last bf16,
// as a split-K MFMA implicit GEMM with an fp32 result.
//
// Reference: the ResNet blocks' 3x3 convolutions (imagenet/resnet.py:72-85 conv3x3, Bottleneck.conv2
// resnet.py:87-108) trained by main.py:326 (loss.backward). torch under bf16 autocast runs MIOpen's
// backward-weights kernel, which zero-fills an fp32 workspace, accumulates into it with atomics,
// casts the result to bf16, and autograd then casts it back to the fp32 master weight's dtype:
// ResNet-50 b256, 16 launches of 115-160 us at ~15 % of the bf16 MFMA peak, plus a zero-fill and
// two casts each, and a bf16-rounded gradient.
//
//   dW[co][kh][kw][ci] = sum over output pixels q = (n, ho, wo) of
//                        dy[q][co] * x[n][ho*s - 1 + kh][wo*s - 1 + kw][ci]   (0 outside the image)
//
// is a GEMM C[M = Co][N = 9 * Ci] = A[M][K] * B[K][N] with K = the N*Ho*Wo output pixels. Both
// operands are stored K-major (pixel rows of channels), so they are staged into LDS as loaded (one
// 16-byte vector per thread and row) and read with gfx950's transposing LDS read
// (ds_read_b64_tr_b16: 4 pixel rows x 16 channels -> each lane gets one channel's 4 consecutive
// pixels), which is exactly the k-run the 16x16x32 bf16 MFMA fragments take.
//
// A workgroup (8 waves) owns a 64-output-channel x (9 taps x 64 input-channel) tile of C and a
// contiguous range of 64-pixel K chunks (split-K); per chunk it stages dy's 64 x 64 tile and the 9
// taps' 64 x 64 gathers of x (halo rows -> zeros), then every wave runs 18 MFMAs per 32-pixel k-step
// (2 output-channel tiles x 9 (tap, input-channel) tiles of 16 x 16). The next chunk's global loads
// are issued before the current chunk's MFMAs (register double buffering). Each split writes its
// fp32 partial C to a slab; dauc_slab_sum adds the slabs in split order (no atomics): bitwise
// reproducible, one fp32 rounding per product sum instead of MIOpen's bf16 rounding.

#include <hip/hip_bf16.h>

#include "dauc_internal.h"

namespace dauc {
namespace {

typedef short v4s __attribute__((ext_vector_type(4)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

constexpr int kWgThreads = 512;  // 8 waves
constexpr int kBM = 64;          // output channels per tile
constexpr int kBC = 64;          // input channels per tile (per tap)
constexpr int kKT = 64;          // output pixels per K chunk
constexpr int kRow = 72;         // LDS row stride in bf16 elements (64 + 8: 144-byte rows)
constexpr int kTaps = 9;
constexpr int kTile = kKT * kRow;  // one staged [pixel][channel] tile, elements

struct WgradGeom {
    int N, H, W, Ci, Ho, Wo, Co, stride;
    int64_t P;        // output pixels N * Ho * Wo
    int64_t chunks;   // ceil(P / kKT)
    int64_t cps;      // chunks per split
    int ctiles;       // Ci / kBC
};

// one lane's half fragment: rows r0 .. r0 + 3 of a staged [pixel][channel] tile, channels
// c0 .. c0 + 15 across the lane's 16-lane group -> 4 consecutive pixels of channel c0 + (lane & 15)
__device__ __forceinline__ v4s tr_read(const short* tile, int r0, int c0, int lane) {
    const int i = lane & 15;
    const short* p = tile + (r0 + (i >> 2)) * kRow + c0 + 4 * (i & 3);
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)p);
}

// the 16x16x32 operand fragment of k-step ks (32 pixels) for channel block c0: lane group
// g = lane >> 4 holds pixels 32 ks + 8 g + (0 .. 7)
__device__ __forceinline__ bf16x8 frag(const short* tile, int ks, int c0, int lane) {
    const int r0 = 32 * ks + 8 * (lane >> 4);
    const v4s lo = tr_read(tile, r0, c0, lane);
    const v4s hi = tr_read(tile, r0 + 4, c0, lane);
    const v4s f[2] = {lo, hi};
    return *reinterpret_cast<const bf16x8*>(f);
}

// one thread's share of a chunk's staging: the dy vector and the 9 taps' x vectors of one pixel row,
// with the in-image bits (bit t: tap t's pixel exists; bit 9: the output pixel exists)
struct Staging {
    uint4 a, b[kTaps];
    unsigned ok;
};

// every load is issued unconditionally (a clamped in-bounds address; out-of-range rows are zeroed
// when staged, after the loads have long landed): a branch or select right behind each load would
// make the compiler wait for each one in turn
__device__ __forceinline__ void load_chunk(Staging& s, const __hip_bfloat16* __restrict__ x,
                                           const __hip_bfloat16* __restrict__ dy, const WgradGeom& g,
                                           int64_t chunk, int pr, int v, int co0, int ci0) {
    const int64_t q0 = chunk * kKT + pr;
    const bool qok = q0 < g.P;
    const unsigned q = static_cast<unsigned>(qok ? q0 : g.P - 1);  // P < 2^31 (host check)
    s.a = *reinterpret_cast<const uint4*>(dy + int64_t(q) * g.Co + co0 + 8 * v);
    const unsigned hw = static_cast<unsigned>(g.Ho * g.Wo);
    const unsigned n = q / hw, r = q - n * hw;
    const int ho = static_cast<int>(r / static_cast<unsigned>(g.Wo));
    const int wo = static_cast<int>(r) - ho * g.Wo;
    const int ih0 = ho * g.stride - 1, iw0 = wo * g.stride - 1;
    const __hip_bfloat16* xn = x + int64_t(n) * g.H * g.W * g.Ci + ci0 + 8 * v;
    unsigned m = qok ? (1u << kTaps) : 0u;
#pragma unroll
    for (int t = 0; t < kTaps; ++t) {
        const int ih = ih0 + t / 3, iw = iw0 + t % 3;
        const bool in = qok & (ih >= 0) & (ih < g.H) & (iw >= 0) & (iw < g.W);
        m |= in ? (1u << t) : 0u;
        const int ihc = min(max(ih, 0), g.H - 1), iwc = min(max(iw, 0), g.W - 1);
        s.b[t] = *reinterpret_cast<const uint4*>(xn + (int64_t(ihc) * g.W + iwc) * g.Ci);
    }
    s.ok = m;
}

// the in-image bit as an AND mask (a select of the two values would become a select of their
// addresses, i.e. the staging registers spilled to scratch)
__device__ __forceinline__ uint4 masked(uint4 u, unsigned ok, int bit) {
    const unsigned m = 0u - ((ok >> bit) & 1u);
    u.x &= m;
    u.y &= m;
    u.z &= m;
    u.w &= m;
    return u;
}

__device__ __forceinline__ void stage_chunk(const Staging& s, short* lds, int pr, int v) {
    *reinterpret_cast<uint4*>(lds + pr * kRow + 8 * v) = masked(s.a, s.ok, kTaps);
#pragma unroll
    for (int t = 0; t < kTaps; ++t)
        *reinterpret_cast<uint4*>(lds + (1 + t) * kTile + pr * kRow + 8 * v) = masked(s.b[t], s.ok, t);
}

__global__ __launch_bounds__(kWgThreads) void wgrad3x3_kernel(const __hip_bfloat16* __restrict__ x,
                                                              const __hip_bfloat16* __restrict__ dy,
                                                              WgradGeom g, float* __restrict__ out) {
    __shared__ short lds[(1 + kTaps) * kTile];  // A tile, then the 9 taps' B tiles
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int co0 = (blockIdx.x / g.ctiles) * kBM, ci0 = (blockIdx.x % g.ctiles) * kBC;
    const int64_t c_begin = int64_t(blockIdx.y) * g.cps;
    const int64_t c_end = c_begin + g.cps < g.chunks ? c_begin + g.cps : g.chunks;

    // staging: thread -> (pixel row pr, 16-byte vector v) of every tile
    const int pr = tid >> 3, v = tid & 7;
    Staging cur;
    load_chunk(cur, x, dy, g, c_begin, pr, v, co0, ci0);

    // wave tiles: output-channel tiles 2 (wave & 1) + a, a < 2; (tap, input-channel) tiles
    // 9 (wave >> 1) + b, b < 9 -> tap = tile >> 2, channel block 16 (tile & 3)
    f32x4v acc[2][9];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 9; ++b) acc[a][b] = f32x4v{0.f, 0.f, 0.f, 0.f};
    const int mt0 = 2 * (wave & 1), nt0 = 9 * (wave >> 1);

    // every split owns >= 1 chunk (host); the loads are unconditional (the last chunk's "next" is
    // itself again): a branch around them would force the loaded registers through copies that
    // wait for each load
    for (int64_t c = c_begin; c < c_end; ++c) {
        __syncthreads();  // the previous chunk's fragment reads are done
        stage_chunk(cur, lds, pr, v);
        __syncthreads();
        load_chunk(cur, x, dy, g, c + 1 < c_end ? c + 1 : c, pr, v, co0, ci0);  // in flight during the MFMAs
        __builtin_amdgcn_sched_barrier(0);  // keep the loads ahead of the MFMAs (the scheduler sinks them)
#pragma unroll
        for (int ks = 0; ks < kKT / 32; ++ks) {
            bf16x8 fa[2];
#pragma unroll
            for (int a = 0; a < 2; ++a) fa[a] = frag(lds, ks, 16 * (mt0 + a), lane);
#pragma unroll
            for (int b = 0; b < 9; ++b) {
                const int t = nt0 + b;
                const bf16x8 fb = frag(lds + (1 + (t >> 2)) * kTile, ks, 16 * (t & 3), lane);
#pragma unroll
                for (int a = 0; a < 2; ++a) acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[a], fb, acc[a][b], 0, 0, 0);
            }
        }
    }
    // C[row = output channel][col = (tap, input channel)]: col = lane & 15, row = 4 (lane >> 4) + r
    float* o = out + int64_t(blockIdx.y) * int64_t(g.Co) * kTaps * g.Ci;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 9; ++b) {
            const int t = nt0 + b, tap = t >> 2;
            const int ci = ci0 + 16 * (t & 3) + (lane & 15);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int co = co0 + 16 * (mt0 + a) + 4 * (lane >> 4) + r;
                o[(int64_t(co) * kTaps + tap) * g.Ci + ci] = acc[a][b][r];
            }
        }
}

// ---- the window form (every ResNet-50 3x3 shape: Wo <= 64) ----------------------------------
// The 9 taps' B tiles above are 9 gathers of mostly the same x pixels: 80 KB of L2 traffic per
// 64-pixel chunk, which bounds that kernel (0.21 of the MFMA peak at 110 us a launch). Here a chunk
// is R whole output rows (R = 64 / Wo, KP = R * Wo <= 64 pixels) and the workgroup stages, per
// output row, the 3 input rows its taps read, W + 2 positions wide with the zero halo: R * 3 *
// (W + 2) positions of 64 channels (ResNet-50: 174 - 432 positions, 22 - 54 KB instead of 72 KB),
// and every tap's B fragment reads the window in place -- the transposing read takes a per-lane
// row address, so lane (q, p) of a group points at pixel k's window position + kh (W + 2) + kw.
// The pixel -> position map is the same for every chunk, so each lane computes its 4 positions
// once. Two LDS buffers: the next chunk is staged while this one is multiplied, one barrier per
// chunk. Pixels k >= KP (a chunk's padding) have zero dy rows (A), so their B values (pixel 0's)
// add nothing.
constexpr int kMaxWinVec = 8;  // window vectors per thread: <= 512 positions of 8 vectors
constexpr int kWinVecFast = 8;  // window vectors per thread that fit beside the accumulators unspilled
// LDS row strides (bf16 elements) of the window kernel. A transposing read serves 32 lanes per
// pass, 8 rows of 8 bytes; the k order below puts 8 consecutive pixels in one pass, so 80-element
// (40-bank) rows land them on 8 disjoint bank octets: conflict-free for the dy tile and a stride-1
// window, where 72 (36 banks) conflicts 2-way. (A stride-2 window steps 2 rows per pixel, 2-way at
// 80; it keeps 80 so that every tap's offset is one compile-time multiple of the row.)
constexpr int kARow = 80;

// (tile, split) of this workgroup. Workgroups go to the 8 XCDs round robin by linear id, each XCD
// with its own L2; the tiles of one split read the same dy rows (same output-channel tile) or the
// same input window (same input-channel tile), so when the split count allows, a split's tiles are
// placed on one XCD (XCD x runs splits x, x + 8, ...) and share those reads in its L2.
__device__ __forceinline__ void tile_split(int& tile, int& split) {
    const int tiles = static_cast<int>(gridDim.x), splits = static_cast<int>(gridDim.y);
    tile = static_cast<int>(blockIdx.x);
    split = static_cast<int>(blockIdx.y);
    if (tiles > 1 && splits % 8 == 0) {
        const int b = tile + tiles * split, k = b / 8;
        tile = k % tiles;
        split = (k / tiles) * 8 + b % 8;
    }
}

struct WinGeom {
    int N, H, W, Ci, Ho, Wo, Co, stride;
    int KT;    // pixel rows of the staged dy tile: 64 or 128 (2 or 4 k-steps per chunk)
    int wrow;  // LDS row stride of the window (kARow: fixed, so every tap's offset is an immediate)
    int R, Wd, npos, KP, nvec;
    // shared rows (R | Ho or Ho | R): the chunk's output rows read overlapping input rows, so its
    // window is the stride R + 3 - stride input rows they span (per image: IR = stride Ho + 3 -
    // stride) instead of 3 per output row; window slot s is image n0 + s / IR, input row
    // stride ho0 - 1 + s % IR
    int shared;
    int64_t GR;      // output rows N * Ho
    int64_t chunks;  // ceil(GR / R)
    int64_t cps;
    int ctiles;
};

inline size_t win_lds_bytes(const struct WinGeom& g);

template <int NV, int KS>
struct WinStaging {
    v4u a[KS / 2], w[NV];  // zeros where the vector lies outside the image / past the chunk's rows
};

// Buffer descriptors of x and dy: the range check returns zeros for an offset past the buffer, so
// a vector outside the image or past the last output row is loaded from offset `bytes` and arrives
// as zeros -- no validity bits, no masking at the LDS store, 32-bit offsets (no 64-bit address math)
struct WinSrc {
    __amdgpu_buffer_rsrc_t x, dy;
    unsigned xbytes, dybytes;
};

__device__ __forceinline__ v4u load16(__amdgpu_buffer_rsrc_t r, unsigned off) {
    return __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(r, static_cast<int>(off), 0, 0));
}

// 32-bit element offsets throughout (host: N * H * W * Ci and N * Ho * Wo * Co < 2^31): 64-bit
// address arithmetic per load was most of the loop's VALU work. What does not change from chunk to
// chunk is decoded once per thread (apk / wpos); per chunk one division finds the chunk's first
// output row (n0, ho0), and each vector's row follows by at most a few wrap steps, not a division.
template <int NV, int KS>
__device__ __forceinline__ void load_win(WinStaging<NV, KS>& s, const WinSrc& src, const WinGeom& g, int chunk,
                                         const int (&apk)[KS / 2], const int (&wpos)[kMaxWinVec], int v, int co0,
                                         int ci0) {
    const int gr0 = chunk * g.R;
    const int GR = static_cast<int>(g.GR);
    const int n0 = gr0 / g.Ho, ho0 = gr0 - n0 * g.Ho;
#pragma unroll
    for (int i = 0; i < KS / 2; ++i) {  // dy: pixel k = pr + 64 i of the chunk (rr | wo << 8, bit 31: k < KP)
        const int rr = apk[i] & 0xff, wo = (apk[i] >> 8) & 0x7fffff;
        const int gr = gr0 + rr;
        const bool ok = (apk[i] < 0) & (gr < GR);
        const unsigned off = 2u * static_cast<unsigned>((gr * g.Wo + wo) * g.Co + co0 + 8 * v);
        s.a[i] = load16(src.dy, ok ? off : src.dybytes);
    }
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        // rr | kh << 8 | iwc << 10 (the clamped input column), or with shared rows sg | u << 8 |
        // iwc << 16 (slot sg IR + u); bit 31: a window position in the image's columns
        const int pk = wpos[j];
        int n, ih, iwc;
        bool ok;
        if (g.shared) {  // image n0 + sg, input row stride ho0 - 1 + u (a wave-uniform branch)
            const int sg = pk & 0xff, u = (pk >> 8) & 0xff;
            iwc = (pk >> 16) & 0x7fff;
            n = n0 + sg;
            ih = ho0 * g.stride - 1 + u;
            ok = (pk < 0) & (n < g.N) & (ih >= 0) & (ih < g.H);
        } else {
            const int rr = pk & 0xff, kh = (pk >> 8) & 3;
            iwc = (pk >> 10) & 0x1fffff;
            const int gr = gr0 + rr;
            int ho = ho0 + rr;
            n = n0;
            while (ho >= g.Ho) {  // rr < R: a few steps at most for the shapes the window form takes
                ho -= g.Ho;
                ++n;
            }
            ih = ho * g.stride - 1 + kh;
            ok = (pk < 0) & (gr < GR) & (ih >= 0) & (ih < g.H);
        }
        const unsigned off = 2u * static_cast<unsigned>(((n * g.H + ih) * g.W + iwc) * g.Ci + ci0 + 8 * v);
        s.w[j] = load16(src.x, ok ? off : src.xbytes);
    }
}

typedef __attribute__((address_space(3))) short lds_short;
typedef __attribute__((address_space(3))) v4u lds_v4u;

__device__ __forceinline__ void st_lds(lds_short* p, const v4u& u) { *(lds_v4u*)p = u; }

template <int NV, int KS>
__device__ __forceinline__ void stage_win(const WinStaging<NV, KS>& s, lds_short* buf, const WinGeom& g, int pr,
                                          int v) {
#pragma unroll
    for (int i = 0; i < KS / 2; ++i) st_lds(buf + ((pr + 64 * i) * kARow + 8 * v), s.a[i]);
    lds_short* win = buf + 32 * KS * kARow;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const int idx = threadIdx.x + kWgThreads * j;
        const int pos = idx >> 3;
        if (pos < g.npos)
            st_lds(win + (pos * g.wrow + 8 * (idx & 7)), s.w[j]);
    }
}

inline size_t win_lds_bytes(const WinGeom& g) {
    return size_t(2) * (size_t(g.KT) * kARow + size_t(g.npos) * g.wrow) * sizeof(short);
}

__device__ __forceinline__ v4s tr_at(const lds_short* p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)p);
}

// one wave's 72 MFMAs of a chunk staged at `cur` (A rows, then the window): its 2 output-channel
// tiles x the 9 taps of its 16-input-channel block. aoff / boff: this lane's element offsets of its
// A rows / window positions (k-step, half), the wave's channel blocks included; wd_row: one window
// row (Wd positions). Each k-step reads tap (kh, kw) at boff + kh wd_row + kw kARow: two adds per
// (k-step, half), the rest immediate offsets.
template <int KS>
__device__ __forceinline__ void win_multiply(f32x4v (&acc)[2][9], const lds_short* cur, const int (&aoff)[KS][2],
                                             const int (&boff)[KS][2], int wd_row) {
    const lds_short* win = cur + 32 * KS * kARow;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
        bf16x8 fa[2];
#pragma unroll
        for (int a = 0; a < 2; ++a) {
            const v4s f2[2] = {tr_at(cur + (aoff[ks][0] + 16 * a)), tr_at(cur + (aoff[ks][1] + 16 * a))};
            fa[a] = *reinterpret_cast<const bf16x8*>(f2);
        }
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) {
            const lds_short* r0 = win + (boff[ks][0] + kh * wd_row);
            const lds_short* r1 = win + (boff[ks][1] + kh * wd_row);
#pragma unroll
            for (int kw = 0; kw < 3; ++kw) {
                const v4s f2[2] = {tr_at(r0 + kw * kARow), tr_at(r1 + kw * kARow)};
                const bf16x8 fb = *reinterpret_cast<const bf16x8*>(f2);
#pragma unroll
                for (int a = 0; a < 2; ++a)
                    acc[a][3 * kh + kw] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[a], fb, acc[a][3 * kh + kw], 0, 0, 0);
            }
        }
    }
}

template <int NV, int KS>
__global__ __launch_bounds__(kWgThreads) void wgrad3x3_win_kernel(const __hip_bfloat16* __restrict__ x,
                                                                  const __hip_bfloat16* __restrict__ dy,
                                                                  WinGeom g, float* __restrict__ out) {
    extern __shared__ short lds_dyn[];
    lds_short* L = (lds_short*)lds_dyn;
    const int buf_elems = 32 * KS * kARow + g.npos * g.wrow;
    WinSrc src;  // host: both buffers hold < 2^31 - 64 elements, so bytes + 16 < 2^32
    src.xbytes = static_cast<unsigned>(int64_t(g.N) * g.H * g.W * g.Ci * 2);
    src.dybytes = static_cast<unsigned>(g.GR * g.Wo * g.Co * 2);
    src.x = __builtin_amdgcn_make_buffer_rsrc(const_cast<__hip_bfloat16*>(x), 0, static_cast<int>(src.xbytes), 0x00020000);
    src.dy = __builtin_amdgcn_make_buffer_rsrc(const_cast<__hip_bfloat16*>(dy), 0, static_cast<int>(src.dybytes), 0x00020000);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int tile, split;
    tile_split(tile, split);
    const int co0 = (tile / g.ctiles) * kBM, ci0 = (tile % g.ctiles) * kBC;
    const int c_begin = static_cast<int>(split * g.cps);
    const int c_end = static_cast<int>(c_begin + g.cps < g.chunks ? c_begin + g.cps : g.chunks);
    const int pr = tid >> 3, v = tid & 7;
    const int mt0 = 2 * (wave & 1), cb = wave >> 1;  // this wave's output-channel tiles, input-channel block

    // this thread's window vectors (the same positions in every chunk; the vector's channel block
    // is v = tid & 7 for every j) and dy rows
    int wpos[kMaxWinVec];
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const int pos = (tid + kWgThreads * j) >> 3;
        if (g.shared) {
            const int ir = g.stride * g.Ho + 3 - g.stride;  // input rows per image
            const int sl = pos / g.Wd, wc = pos - sl * g.Wd;
            const int sg = sl / ir, u = sl - sg * ir;
            const int iw = wc - 1;
            const bool ok = (pos < g.npos) & (iw >= 0) & (iw < g.W);
            wpos[j] = (ok ? int(0x80000000u) : 0) | sg | (u << 8) | (min(max(iw, 0), g.W - 1) << 16);
        } else {
            const int per_row = 3 * g.Wd;
            const int rr = pos / per_row, rem = pos - rr * per_row;
            const int kh = rem / g.Wd, wc = rem - kh * g.Wd;
            const int iw = wc - 1;
            const bool ok = (pos < g.npos) & (iw >= 0) & (iw < g.W);
            wpos[j] = (ok ? int(0x80000000u) : 0) | rr | (kh << 8) | (min(max(iw, 0), g.W - 1) << 10);
        }
    }
    int apk[KS / 2];
#pragma unroll
    for (int i = 0; i < KS / 2; ++i) {
        const int k = pr + 64 * i;
        const int rr = k / g.Wo, wo = k - rr * g.Wo;
        apk[i] = (k < g.KP ? int(0x80000000u) : 0) | (k < g.KP ? rr | (wo << 8) : 0);
    }
    // this lane's fragment rows: pixel k = 32 ks + 16 h + 4 (lane >> 4) + ((lane & 15) >> 2) (any
    // order of the 32 pixels of a k-step sums the same products; this one gives each 32-lane pass
    // of read h 8 consecutive pixels); A row k, window position of k for tap (0, 0); + the lane's 4
    // channels 4 (lane & 3)
    int aoff[KS][2], boff[KS][2];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int k = 32 * ks + 16 * h + 4 * (lane >> 4) + ((lane & 15) >> 2);
            const int rr = k / g.Wo, cc = k - rr * g.Wo;
            // the window position of pixel k's tap (0, 0): its output row's first window row
            const int row0 = g.shared ? g.stride * rr + (3 - g.stride) * (rr / g.Ho) : 3 * rr;
            const int pos = k < g.KP ? row0 * g.Wd + cc * g.stride : 0;
            // the wave's tiles: output channels 16 (mt0 + a), input channel block cb, all 9 taps
            aoff[ks][h] = k * kARow + 4 * (lane & 3) + 16 * mt0;
            boff[ks][h] = pos * kARow + 4 * (lane & 3) + 16 * cb;
        }
    const int wd_row = g.Wd * kARow;

    f32x4v acc[2][9];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 9; ++b) acc[a][b] = f32x4v{0.f, 0.f, 0.f, 0.f};

    WinStaging<NV, KS> st;
    load_win<NV, KS>(st, src, g, c_begin, apk, wpos, v, co0, ci0);
    stage_win<NV, KS>(st, L, g, pr, v);
    load_win<NV, KS>(st, src, g, c_begin + 1 < c_end ? c_begin + 1 : c_begin, apk, wpos, v, co0, ci0);
    __syncthreads();
    for (int c = c_begin; c < c_end; ++c) {
        const int b = (c - c_begin) & 1;
        // chunk c + 1 into the other buffer (read last by chunk c - 1, before the barrier below
        // ended that iteration); on the last chunk this stages a clamped copy nobody reads
        stage_win<NV, KS>(st, L + (b ^ 1) * buf_elems, g, pr, v);
        load_win<NV, KS>(st, src, g, c + 2 < c_end ? c + 2 : c_end - 1, apk, wpos, v, co0, ci0);
        __builtin_amdgcn_sched_barrier(0);  // the loads ahead of the MFMAs
        win_multiply<KS>(acc, L + b * buf_elems, aoff, boff, wd_row);
        __syncthreads();
    }
    float* o = out + int64_t(split) * int64_t(g.Co) * kTaps * g.Ci;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
            const int ci = ci0 + 16 * cb + (lane & 15);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int co = co0 + 16 * (mt0 + a) + 4 * (lane >> 4) + r;
                o[(int64_t(co) * kTaps + tap) * g.Ci + ci] = acc[a][tap][r];
            }
        }
}

#ifdef DAUC_TUNING
// the transposing LDS read's lane map, for the tests: LDS holds element value = row * 64 + col of a
// [16][64] tile (row stride kRow); lane l reads frag(tile, 0, c0 = 16 * (l >> 6 ... 0), l)
__global__ void probe_tr16_kernel(short* out) {
    __shared__ short t[32 * kRow];
    for (int i = threadIdx.x; i < 32 * kRow; i += 64) t[i] = static_cast<short>((i / kRow) * 64 + i % kRow);
    __syncthreads();
    const bf16x8 f = frag(t, 0, 16, threadIdx.x);
    const short* s = reinterpret_cast<const short*>(&f);
    for (int j = 0; j < 8; ++j) out[threadIdx.x * 8 + j] = s[j];
}
#endif

}  // namespace
}  // namespace dauc

using namespace dauc;

extern "C" {

namespace {
// the window form's geometry (returns false when the shape needs the gather form)
// one chunk layout: R whole output rows of a KT-row dy tile and their windows (false: does not fit)
bool win_layout(int W, int Wo, int KT, bool shared, WinGeom& g) {
    if (Wo > KT) return false;
    if (shared && W >= (1 << 15)) return false;
    g.KT = KT;
    g.shared = shared ? 1 : 0;
    g.wrow = kARow;
    g.Wd = W + 2;
    // as many whole output rows as fit the tile (fewer if the window needs more vectors per thread
    // than kWinVecFast or more LDS than a CU has; with shared rows, R divides Ho or Ho divides R,
    // so no chunk holds part of an image beside another image's rows)
    for (g.R = KT / Wo; g.R >= 1; --g.R) {
        if (shared) {
            if (g.Ho % g.R != 0 && g.R % g.Ho != 0) continue;
            const int s = g.stride;
            const int images = g.R >= g.Ho ? g.R / g.Ho : 1;
            const int rows = (g.R >= g.Ho ? s * g.Ho : s * g.R) + 3 - s;
            if (images > 255 || rows > 255) continue;  // packed in 8 bits each
            g.npos = images * rows * g.Wd;
        } else {
            g.npos = g.R * 3 * g.Wd;
        }
        g.nvec = (g.npos * 8 + kWgThreads - 1) / kWgThreads;
        if (g.nvec <= kWinVecFast && win_lds_bytes(g) <= 160 * 1024) break;
    }
    if (g.R < 1) return false;
    g.KP = g.R * Wo;
    return true;
}

// relative cost of a layout: per chunk, its k-steps' MFMAs (a SIMD's 2 waves x 18 x 16 cycles per
// k-step), the staging of its window (about 4.4 SIMD cycles per position: 8 vectors' loads,
// address VALU and LDS stores) and a fixed ~1,000 cycles (barrier, exposed load latency), times
// the chunk count. Measured at ResNet-50 b256 (profiles/r05/wgrad3x3_shared/): it picks shared rows
// with 128-pixel chunks for every stride-1 shape, the fastest of the four layouts there.
double win_cost(const WinGeom& g) {
    const double chunks = double((g.GR + g.R - 1) / g.R);
    return chunks * (576.0 * (g.KT / 32) + 4.4 * g.npos + 1000.0);
}

#ifdef DAUC_TUNING
int g_wgrad_form = 0;  // dauc_set_wgrad_form: 0 automatic, 1 gather, 2 / 3 window KT 64 / 128, 4 / 5 shared rows
#endif

bool win_geom(int64_t N, int H, int W, int Ci, int Ho, int Wo, int Co, int stride, WinGeom& g) {
    // the window kernel reads x and dy through buffer descriptors with 32-bit byte offsets (an
    // offset of `bytes` returns zeros, so bytes + 16 must not wrap) and packs a column in 21 bits
    if (N * H * int64_t(W) * Ci >= (int64_t(1) << 31) - 64 || N * Ho * int64_t(Wo) * Co >= (int64_t(1) << 31) - 64)
        return false;
    if (W >= (1 << 21)) return false;
    int form = 0;
#ifdef DAUC_TUNING
    form = g_wgrad_form;
    if (form == 1) return false;
#endif
    // stride 2: the gather form unless a shared-row window fits with its rows filling at least half
    // of the chunk (ResNet-50 b256: layer2.0 gather 123 us, shared 118; layer4.0 119 / 117;
    // layer3.0's shared layout fills 28 of 64 pixels: 177 against the gather form's 120;
    // profiles/r05/wgrad3x3_shared)
    const bool s2_shared_only = form == 0 && stride != 1;
    g.N = static_cast<int>(N);
    g.H = H;
    g.W = W;
    g.Ci = Ci;
    g.Ho = Ho;
    g.Wo = Wo;
    g.Co = Co;
    g.stride = stride;
    g.GR = N * Ho;
    // 64- or 128-pixel chunks (2 or 4 k-steps per barrier and staging wait), per-output-row or
    // shared window rows: the layout of least estimated cost (tuning forms 2 / 3: per-row windows
    // with 64 / 128-pixel chunks; 4 / 5: shared rows with 64 / 128-pixel chunks)
    WinGeom cand[4] = {g, g, g, g};
    bool ok[4];
    for (int i = 0; i < 4; ++i) ok[i] = win_layout(W, Wo, (i & 1) ? 128 : 64, i >= 2, cand[i]);
    int pick = -1;
    if (form >= 2 && form <= 5) {
        pick = form - 2;
    } else {
        for (int i = s2_shared_only ? 2 : 0; i < 4; ++i)
            if (ok[i] && !(s2_shared_only && 2 * cand[i].KP < cand[i].KT) &&
                (pick < 0 || win_cost(cand[i]) < win_cost(cand[pick])))
                pick = i;
    }
    if (pick < 0 || !ok[pick]) return false;
    g = cand[pick];
    g.chunks = (g.GR + g.R - 1) / g.R;
    g.ctiles = Ci / kBC;
    return true;
}

int64_t split_count(int64_t tiles, int64_t chunks) {
    int64_t S = (256 + tiles - 1) / tiles;
    return S > chunks ? chunks : S;
}
}  // namespace

size_t dauc_conv3x3_wgrad_workspace_size(int64_t N, int Ho, int Wo, int Ci, int Co) {
    if (N < 1 || Ho < 1 || Wo < 1 || Ci < kBC || Co < kBM || Ci % kBC || Co % kBM) return 0;
    const int64_t tiles = int64_t(Co / kBM) * (Ci / kBC);
    // the larger of the two forms' chunk counts bounds the splits of either
    const int64_t chunks = (N * Ho * Wo + kKT - 1) / kKT;
    const int64_t S = split_count(tiles, chunks > N * Ho ? chunks : N * Ho);
    if (S <= 1) return 0;
    return size_t(S) * size_t(Co) * kTaps * size_t(Ci) * sizeof(float);
}

int dauc_conv3x3_wgrad(const void* x, const void* dy, int dtype, int64_t N, int H, int W, int Ci, int Ho, int Wo,
                       int Co, int stride, float* dw, void* workspace, size_t workspace_bytes, dauc_stream_t stream) {
    if (x == nullptr || dy == nullptr || dw == nullptr || dtype != DAUC_DTYPE_BF16) return DAUC_EINVAL;
    if (N < 1 || H < 1 || W < 1 || Ho < 1 || Wo < 1 || Ci < kBC || Co < kBM || Ci % kBC || Co % kBM) return DAUC_EINVAL;
    if (stride != 1 && stride != 2) return DAUC_EINVAL;
    if (Ho != (H + 2 - 3) / stride + 1 || Wo != (W + 2 - 3) / stride + 1) return DAUC_EINVAL;  // pad 1
    if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(dy) | reinterpret_cast<uintptr_t>(dw)) & 15u)
        return DAUC_EINVAL;
    if (N * int64_t(H) * W > (int64_t(1) << 31) || N * int64_t(Ho) * Wo > (int64_t(1) << 31)) return DAUC_EINVAL;
    const int64_t tiles = int64_t(Co / kBM) * (Ci / kBC);
    const size_t need = dauc_conv3x3_wgrad_workspace_size(N, Ho, Wo, Ci, Co);
    const int64_t Smax = need ? int64_t(need / (size_t(Co) * kTaps * size_t(Ci) * sizeof(float))) : 1;
    if (need && (workspace == nullptr || workspace_bytes < need || (reinterpret_cast<uintptr_t>(workspace) & 15u)))
        return DAUC_EINVAL;
    if (tiles > 0x7fffffffLL) return DAUC_EINVAL;
    hipStream_t st = as_hip(stream);
    WinGeom wg;
    int64_t splits;
    float* target;
    if (win_geom(N, H, W, Ci, Ho, Wo, Co, stride, wg)) {
        const int64_t S = split_count(tiles, wg.chunks) < Smax ? split_count(tiles, wg.chunks) : Smax;
        wg.cps = (wg.chunks + S - 1) / S;
        splits = (wg.chunks + wg.cps - 1) / wg.cps;  // every split owns at least one chunk
        if (splits > 65535) return DAUC_EINVAL;
        target = splits > 1 ? static_cast<float*>(workspace) : dw;
        const dim3 grid(static_cast<unsigned>(tiles), static_cast<unsigned>(splits));
        const size_t lds = win_lds_bytes(wg);
        const __hip_bfloat16* xb = static_cast<const __hip_bfloat16*>(x);
        const __hip_bfloat16* db = static_cast<const __hip_bfloat16*>(dy);
        switch (wg.nvec * 8 + wg.KT / 32) {
#define DAUC_WIN_CASE(NV, KS) \
    case NV * 8 + KS:         \
        hipLaunchKernelGGL((wgrad3x3_win_kernel<NV, KS>), grid, dim3(kWgThreads), lds, st, xb, db, wg, target); break;
            DAUC_WIN_CASE(1, 2)
            DAUC_WIN_CASE(2, 2)
            DAUC_WIN_CASE(3, 2)
            DAUC_WIN_CASE(4, 2)
            DAUC_WIN_CASE(5, 2)
            DAUC_WIN_CASE(6, 2)
            DAUC_WIN_CASE(7, 2)
            DAUC_WIN_CASE(8, 2)
            DAUC_WIN_CASE(1, 4)
            DAUC_WIN_CASE(2, 4)
            DAUC_WIN_CASE(3, 4)
            DAUC_WIN_CASE(4, 4)
            DAUC_WIN_CASE(5, 4)
            DAUC_WIN_CASE(6, 4)
            DAUC_WIN_CASE(7, 4)
            DAUC_WIN_CASE(8, 4)
#undef DAUC_WIN_CASE
            default: return DAUC_EINVAL;
        }
    } else {
        WgradGeom g;
        g.N = static_cast<int>(N);
        g.H = H;
        g.W = W;
        g.Ci = Ci;
        g.Ho = Ho;
        g.Wo = Wo;
        g.Co = Co;
        g.stride = stride;
        g.P = N * Ho * Wo;
        g.chunks = (g.P + kKT - 1) / kKT;
        g.ctiles = Ci / kBC;
        const int64_t S = split_count(tiles, g.chunks) < Smax ? split_count(tiles, g.chunks) : Smax;
        g.cps = (g.chunks + S - 1) / S;
        splits = (g.chunks + g.cps - 1) / g.cps;
        if (splits > 65535) return DAUC_EINVAL;
        target = splits > 1 ? static_cast<float*>(workspace) : dw;
        hipLaunchKernelGGL(wgrad3x3_kernel, dim3(static_cast<unsigned>(tiles), static_cast<unsigned>(splits)),
                           dim3(kWgThreads), 0, st, static_cast<const __hip_bfloat16*>(x),
                           static_cast<const __hip_bfloat16*>(dy), g, target);
    }
    int rc = launch_status();
    if (rc != DAUC_OK || splits == 1) return rc;
    return dauc_slab_sum(target, splits, int64_t(Co) * kTaps * Ci, dw, stream);
}

#ifdef DAUC_TUNING
int dauc_set_wgrad_form(int form) {
    if (form < 0 || form > 5) return DAUC_EINVAL;
    g_wgrad_form = form;
    return DAUC_OK;
}

int dauc_probe_tr16(short* out, dauc_stream_t stream) {
    if (out == nullptr) return DAUC_EINVAL;
    hipLaunchKernelGGL(probe_tr16_kernel, dim3(1), dim3(64), 0, as_hip(stream), out);
    return launch_status();
}
#endif

}  // extern "C"
