// Max pooling (the ResNet stem's 3x3 / stride 2 / pad 1 max-pool) over channels-last
// activations, forward and backward, for the CoDA backbone step.
//
// Reference: imagenet/resnet.py:203-206 (conv1 -> bn1 -> relu -> maxpool) in training
// mode. torch's NHWC max-pool saves an int64 index per output element (8 B: for the
// ResNet-50 b256 stem 411 MB written forward and read again backward, more than the
// activation itself); here the saved index is one int8 per element, the position of
// the maximum inside its k x k window (-1 = torch's "no element compared greater"
// case, which it records as the absolute index 0).
//
// Semantics follow torch's max_pool_forward_nhwc / max_pool_backward_nhwc exactly:
//   forward : per channel, scan the clipped window row by row; an element replaces
//             the running maximum (initial -inf, index 0) when it compares greater
//             or is NaN; output = that element (bf16 NaN canonicalised to 0x7FC0 as
//             c10's float -> bf16 conversion does).
//   backward: per input element, visit the windows that contain it (output rows
//             then columns, ascending), add dy in fp32 where the window's index
//             names this element, round once to the output dtype.
// Same comparisons, same summation order: bit-identical to torch.
//
// Geometry: a thread owns one 16-byte vector of channels (8 bf16 / 4 fp32) of one
// output pixel (forward) or one input pixel (backward); neighbouring windows
// overlap, so the re-reads are L2 hits and HBM sees x once.

#include <hip/hip_bf16.h>

#include "dauc_internal.h"

namespace dauc {
namespace {

constexpr int kPoolThreads = 256;

template <typename T>
struct PoolVec;
template <>
struct PoolVec<__hip_bfloat16> {
    static constexpr int N = 8;
    typedef uint4 Raw;
    typedef uint2 Idx;  // 8 int8 indices
};
template <>
struct PoolVec<float> {
    static constexpr int N = 4;
    typedef f32x4 Raw;
    typedef unsigned Idx;  // 4 int8 indices
};

__device__ __forceinline__ void unpack(const uint4& u, float (&v)[8]) {
    const unsigned w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        v[2 * i] = __uint_as_float(w[i] << 16);
        v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
}

__device__ __forceinline__ void unpack(const f32x4& u, float (&v)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = u[i];
}

// c10::BFloat16(float): NaN -> 0x7FC0, otherwise round to nearest even
__device__ __forceinline__ unsigned to_bf16(float f) {
    const unsigned u = __float_as_uint(f);
    if (f != f) return 0x7FC0u;
    return (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
}

__device__ __forceinline__ uint4 pack(const float (&v)[8]) {
    uint4 u;
    u.x = to_bf16(v[0]) | (to_bf16(v[1]) << 16);
    u.y = to_bf16(v[2]) | (to_bf16(v[3]) << 16);
    u.z = to_bf16(v[4]) | (to_bf16(v[5]) << 16);
    u.w = to_bf16(v[6]) | (to_bf16(v[7]) << 16);
    return u;
}

__device__ __forceinline__ f32x4 pack(const float (&v)[4]) { return f32x4{v[0], v[1], v[2], v[3]}; }

__device__ __forceinline__ uint2 pack_idx(const int (&id)[8]) {
    uint2 r;
    r.x = (id[0] & 0xff) | ((id[1] & 0xff) << 8) | ((id[2] & 0xff) << 16) | ((unsigned)(id[3] & 0xff) << 24);
    r.y = (id[4] & 0xff) | ((id[5] & 0xff) << 8) | ((id[6] & 0xff) << 16) | ((unsigned)(id[7] & 0xff) << 24);
    return r;
}

__device__ __forceinline__ unsigned pack_idx(const int (&id)[4]) {
    return (id[0] & 0xff) | ((id[1] & 0xff) << 8) | ((id[2] & 0xff) << 16) | ((unsigned)(id[3] & 0xff) << 24);
}

__device__ __forceinline__ void unpack_idx(const uint2& r, int (&id)[8]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        id[i] = static_cast<int8_t>((r.x >> (8 * i)) & 0xff);
        id[4 + i] = static_cast<int8_t>((r.y >> (8 * i)) & 0xff);
    }
}

__device__ __forceinline__ void unpack_idx(const unsigned& r, int (&id)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) id[i] = static_cast<int8_t>((r >> (8 * i)) & 0xff);
}

struct PoolGeom {
    int64_t N;
    int H, W, C, k, s, p, Ho, Wo;
};

template <typename T>
__global__ __launch_bounds__(kPoolThreads) void maxpool_fwd_kernel(const T* __restrict__ x, PoolGeom g,
                                                                   T* __restrict__ y, int8_t* __restrict__ idx) {
    constexpr int V = PoolVec<T>::N;
    typedef typename PoolVec<T>::Raw Raw;
    typedef typename PoolVec<T>::Idx Idx;
    // blockIdx.y = image: 32-bit index arithmetic within one image (checked on the host)
    const int cv = g.C / V;
    const int t = blockIdx.x * kPoolThreads + threadIdx.x;
    if (t >= g.Ho * g.Wo * cv) return;
    const int c = (t % cv) * V;
    const int q = t / cv;  // output pixel (oh, ow) of image n
    const int ow = q % g.Wo;
    const int oh = q / g.Wo;
    const int64_t n = blockIdx.y;
    const int64_t pix = n * g.Ho * g.Wo + q;
    const int hs = oh * g.s - g.p, ws = ow * g.s - g.p;
    const int h0 = hs > 0 ? hs : 0, w0 = ws > 0 ? ws : 0;
    const int h1 = hs + g.k < g.H ? hs + g.k : g.H, w1 = ws + g.k < g.W ? ws + g.k : g.W;
    float m[V];
    int id[V];
#pragma unroll
    for (int v = 0; v < V; ++v) {
        m[v] = -__builtin_huge_valf();
        id[v] = -1;
    }
    const T* __restrict__ xn = x + n * g.H * g.W * g.C + c;
    for (int ih = h0; ih < h1; ++ih) {
        for (int iw = w0; iw < w1; ++iw) {
            float val[V];
            unpack(*reinterpret_cast<const Raw*>(xn + (int64_t(ih) * g.W + iw) * g.C), val);
            const int rel = (ih - hs) * g.k + (iw - ws);
#pragma unroll
            for (int v = 0; v < V; ++v) {
                if (val[v] > m[v] || val[v] != val[v]) {
                    m[v] = val[v];
                    id[v] = rel;
                }
            }
        }
    }
    *reinterpret_cast<Raw*>(y + pix * g.C + c) = pack(m);
    *reinterpret_cast<Idx*>(idx + pix * g.C + c) = pack_idx(id);
}

template <typename T>
__global__ __launch_bounds__(kPoolThreads) void maxpool_bwd_kernel(const T* __restrict__ dy,
                                                                   const int8_t* __restrict__ idx, PoolGeom g,
                                                                   T* __restrict__ dx) {
    constexpr int V = PoolVec<T>::N;
    typedef typename PoolVec<T>::Raw Raw;
    typedef typename PoolVec<T>::Idx Idx;
    const int cv = g.C / V;
    const int t = blockIdx.x * kPoolThreads + threadIdx.x;
    if (t >= g.H * g.W * cv) return;
    const int c = (t % cv) * V;
    const int q = t / cv;  // input pixel (ih, iw) of image n
    const int iw = q % g.W;
    const int ih = q / g.W;
    const int64_t n = blockIdx.y;
    const int64_t pix = n * g.H * g.W + q;
    // torch's p_start / p_end (dilation 1)
    const int ph0 = (ih + g.p < g.k) ? 0 : (ih + g.p - g.k) / g.s + 1;
    const int pw0 = (iw + g.p < g.k) ? 0 : (iw + g.p - g.k) / g.s + 1;
    const int ph1 = (ih + g.p) / g.s + 1 < g.Ho ? (ih + g.p) / g.s + 1 : g.Ho;
    const int pw1 = (iw + g.p) / g.s + 1 < g.Wo ? (iw + g.p) / g.s + 1 : g.Wo;
    const bool origin = (ih == 0 && iw == 0);  // torch's index 0, also the "never replaced" mark
    float acc[V];
#pragma unroll
    for (int v = 0; v < V; ++v) acc[v] = 0.0f;
    const int64_t obase = n * g.Ho * g.Wo;
    for (int oh = ph0; oh < ph1; ++oh) {
        for (int ow = pw0; ow < pw1; ++ow) {
            const int rel = (ih - (oh * g.s - g.p)) * g.k + (iw - (ow * g.s - g.p));
            const int64_t o = (obase + int64_t(oh) * g.Wo + ow) * g.C + c;
            int id[V];
            unpack_idx(*reinterpret_cast<const Idx*>(idx + o), id);
            float d[V];
            unpack(*reinterpret_cast<const Raw*>(dy + o), d);
#pragma unroll
            for (int v = 0; v < V; ++v)
                if (id[v] == rel || (origin && id[v] == -1)) acc[v] += d[v];
        }
    }
    *reinterpret_cast<Raw*>(dx + pix * g.C + c) = pack(acc);
}

// ---- the ResNet stem's shape (k = 3): every load of a window issued before any compare ------
// Forward: the 9 window loads of the generic kernel sit in a clipped loop (one load latency per
// element); here they are unrolled with per-element predicates (same comparisons, same order).
template <typename T>
__global__ __launch_bounds__(kPoolThreads) void maxpool_fwd_k3_kernel(const T* __restrict__ x, PoolGeom g,
                                                                      T* __restrict__ y, int8_t* __restrict__ idx) {
    constexpr int V = PoolVec<T>::N;
    typedef typename PoolVec<T>::Raw Raw;
    typedef typename PoolVec<T>::Idx Idx;
    const int cv = g.C / V;
    const int t = blockIdx.x * kPoolThreads + threadIdx.x;
    if (t >= g.Ho * g.Wo * cv) return;
    const int c = (t % cv) * V;
    const int q = t / cv;
    const int ow = q % g.Wo;
    const int oh = q / g.Wo;
    const int64_t n = blockIdx.y;
    const int64_t pix = n * g.Ho * g.Wo + q;
    const int hs = oh * g.s - g.p, ws = ow * g.s - g.p;
    const T* __restrict__ xn = x + n * g.H * g.W * g.C + c;
    Raw r[9];
    bool in[9];
#pragma unroll
    for (int e = 0; e < 9; ++e) {
        const int ih = hs + e / 3, iw = ws + e % 3;
        in[e] = ih >= 0 && ih < g.H && iw >= 0 && iw < g.W;
        if (in[e]) r[e] = *reinterpret_cast<const Raw*>(xn + (int64_t(ih) * g.W + iw) * g.C);
    }
    float m[V];
    int id[V];
#pragma unroll
    for (int v = 0; v < V; ++v) {
        m[v] = -__builtin_huge_valf();
        id[v] = -1;
    }
#pragma unroll
    for (int e = 0; e < 9; ++e) {
        if (!in[e]) continue;
        float val[V];
        unpack(r[e], val);
#pragma unroll
        for (int v = 0; v < V; ++v) {
            if (val[v] > m[v] || val[v] != val[v]) {
                m[v] = val[v];
                id[v] = e;
            }
        }
    }
    *reinterpret_cast<Raw*>(y + pix * g.C + c) = pack(m);
    *reinterpret_cast<Idx*>(idx + pix * g.C + c) = pack_idx(id);
}

// Backward for k = 3, s = 2, p = 1: a thread owns the 2 x 2 input pixels (2a + di, 2b + dj) of one
// channel vector. Their windows are exactly (a + i, b + j), i, j in {0, 1} (row 2a lies only in
// window row a, row 2a + 1 in rows a and a + 1; columns alike), so the thread loads those four
// windows' dy and indices once, all before any add -- every dy / index element is read by one
// thread (the generic kernel reads each 2.25 times on average, one window after another). Each
// input element adds the windows naming it in torch's order (window rows, then columns,
// ascending) in fp32 and rounds once: bit-identical to the generic kernel.
template <typename T>
__global__ __launch_bounds__(kPoolThreads) void maxpool_bwd_k3s2_kernel(const T* __restrict__ dy,
                                                                        const int8_t* __restrict__ idx, PoolGeom g,
                                                                        T* __restrict__ dx) {
    constexpr int V = PoolVec<T>::N;
    typedef typename PoolVec<T>::Raw Raw;
    typedef typename PoolVec<T>::Idx Idx;
    const int cv = g.C / V;
    const int Hb = (g.H + 1) / 2, Wb = (g.W + 1) / 2;
    const int t = blockIdx.x * kPoolThreads + threadIdx.x;
    if (t >= Hb * Wb * cv) return;
    const int c = (t % cv) * V;
    const int q = t / cv;
    const int b = q % Wb;
    const int a = q / Wb;
    const int64_t n = blockIdx.y;
    const int64_t obase = n * g.Ho * g.Wo;
    Raw d[2][2];
    Idx ix[2][2];
    bool win[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            win[i][j] = a + i < g.Ho && b + j < g.Wo;
            if (win[i][j]) {
                const int64_t o = (obase + int64_t(a + i) * g.Wo + (b + j)) * g.C + c;
                ix[i][j] = *reinterpret_cast<const Idx*>(idx + o);
                d[i][j] = *reinterpret_cast<const Raw*>(dy + o);
            }
        }
#pragma unroll
    for (int di = 0; di < 2; ++di) {
        const int ih = 2 * a + di;
        if (ih >= g.H) continue;
#pragma unroll
        for (int dj = 0; dj < 2; ++dj) {
            const int iw = 2 * b + dj;
            if (iw >= g.W) continue;
            const bool origin = (ih == 0 && iw == 0);
            float acc[V];
#pragma unroll
            for (int v = 0; v < V; ++v) acc[v] = 0.0f;
            // window (a + i, b + j) covers this pixel when i <= di and j <= dj; the pixel's
            // position in it: row di + 1 - 2i, column dj + 1 - 2j
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                if (i > di) continue;
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    if (j > dj || !win[i][j]) continue;
                    const int rel = (di + 1 - 2 * i) * 3 + (dj + 1 - 2 * j);
                    int id[V];
                    unpack_idx(ix[i][j], id);
                    float dv[V];
                    unpack(d[i][j], dv);
#pragma unroll
                    for (int v = 0; v < V; ++v)
                        if (id[v] == rel || (origin && id[v] == -1)) acc[v] += dv[v];
                }
            }
            *reinterpret_cast<Raw*>(dx + ((n * g.H + ih) * int64_t(g.W) + iw) * g.C + c) = pack(acc);
        }
    }
}

bool pool_args_ok(const void* a, const void* b, const void* c, int dtype, int64_t N, int H, int W, int C, int k,
                  int s, int p, int Ho, int Wo) {
    if (a == nullptr || b == nullptr || c == nullptr) return false;
    if (dtype != DAUC_DTYPE_BF16 && dtype != DAUC_DTYPE_F32) return false;
    const int V = dtype == DAUC_DTYPE_BF16 ? 8 : 4;
    if (N < 1 || H < 1 || W < 1 || C < V || C % V) return false;
    if (k < 1 || k * k > 127 || s < 1 || p < 0 || 2 * p > k) return false;
    if (Ho != (H + 2 * p - k) / s + 1 || Wo != (W + 2 * p - k) / s + 1 || Ho < 1 || Wo < 1) return false;
    // every vector access is 16-byte (values) / 4- or 8-byte (indices) aligned
    if ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(c)) & 15u) return false;
    if (reinterpret_cast<uintptr_t>(b) & 7u) return false;
    return true;
}

// grid: x covers one image's (pixel, vector) pairs, y the images
int pool_grid(int64_t per_image, int64_t N, dim3* grid) {
    if (per_image < 1 || per_image > 0x7fffffffLL - kPoolThreads || N < 1 || N > 65535) return DAUC_EINVAL;
    *grid = dim3(static_cast<unsigned>((per_image + kPoolThreads - 1) / kPoolThreads), static_cast<unsigned>(N));
    return DAUC_OK;
}

}  // namespace
}  // namespace dauc

using namespace dauc;

extern "C" {

int dauc_maxpool2d_forward(const void* x, int dtype, int64_t N, int H, int W, int C, int kernel, int stride,
                           int pad, void* y, int8_t* argmax, int Ho, int Wo, dauc_stream_t stream) {
    if (!pool_args_ok(x, argmax, y, dtype, N, H, W, C, kernel, stride, pad, Ho, Wo)) return DAUC_EINVAL;
    const PoolGeom g{N, H, W, C, kernel, stride, pad, Ho, Wo};
    const int V = dtype == DAUC_DTYPE_BF16 ? 8 : 4;
    dim3 grid;
    if (pool_grid(int64_t(Ho) * Wo * (C / V), N, &grid)) return DAUC_EINVAL;
    hipStream_t st = as_hip(stream);
    if (kernel == 3) {
        if (dtype == DAUC_DTYPE_BF16)
            hipLaunchKernelGGL(maxpool_fwd_k3_kernel<__hip_bfloat16>, grid, dim3(kPoolThreads), 0, st,
                               static_cast<const __hip_bfloat16*>(x), g, static_cast<__hip_bfloat16*>(y), argmax);
        else
            hipLaunchKernelGGL(maxpool_fwd_k3_kernel<float>, grid, dim3(kPoolThreads), 0, st,
                               static_cast<const float*>(x), g, static_cast<float*>(y), argmax);
        return launch_status();
    }
    if (dtype == DAUC_DTYPE_BF16)
        hipLaunchKernelGGL(maxpool_fwd_kernel<__hip_bfloat16>, grid, dim3(kPoolThreads), 0, st,
                           static_cast<const __hip_bfloat16*>(x), g, static_cast<__hip_bfloat16*>(y), argmax);
    else
        hipLaunchKernelGGL(maxpool_fwd_kernel<float>, grid, dim3(kPoolThreads), 0, st,
                           static_cast<const float*>(x), g, static_cast<float*>(y), argmax);
    return launch_status();
}

int dauc_maxpool2d_backward(const void* dy, const int8_t* argmax, int dtype, int64_t N, int H, int W, int C,
                            int kernel, int stride, int pad, int Ho, int Wo, void* dx, dauc_stream_t stream) {
    if (!pool_args_ok(dy, argmax, dx, dtype, N, H, W, C, kernel, stride, pad, Ho, Wo)) return DAUC_EINVAL;
    const PoolGeom g{N, H, W, C, kernel, stride, pad, Ho, Wo};
    const int V = dtype == DAUC_DTYPE_BF16 ? 8 : 4;
    dim3 grid;
    hipStream_t st = as_hip(stream);
    if (kernel == 3 && stride == 2 && pad == 1) {
        if (pool_grid(int64_t((H + 1) / 2) * ((W + 1) / 2) * (C / V), N, &grid)) return DAUC_EINVAL;
        if (dtype == DAUC_DTYPE_BF16)
            hipLaunchKernelGGL(maxpool_bwd_k3s2_kernel<__hip_bfloat16>, grid, dim3(kPoolThreads), 0, st,
                               static_cast<const __hip_bfloat16*>(dy), argmax, g, static_cast<__hip_bfloat16*>(dx));
        else
            hipLaunchKernelGGL(maxpool_bwd_k3s2_kernel<float>, grid, dim3(kPoolThreads), 0, st,
                               static_cast<const float*>(dy), argmax, g, static_cast<float*>(dx));
        return launch_status();
    }
    if (pool_grid(int64_t(H) * W * (C / V), N, &grid)) return DAUC_EINVAL;
    if (dtype == DAUC_DTYPE_BF16)
        hipLaunchKernelGGL(maxpool_bwd_kernel<__hip_bfloat16>, grid, dim3(kPoolThreads), 0, st,
                           static_cast<const __hip_bfloat16*>(dy), argmax, g, static_cast<__hip_bfloat16*>(dx));
    else
        hipLaunchKernelGGL(maxpool_bwd_kernel<float>, grid, dim3(kPoolThreads), 0, st,
                           static_cast<const float*>(dy), argmax, g, static_cast<float*>(dx));
    return launch_status();
}

}  // extern "C"
