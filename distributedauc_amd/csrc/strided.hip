// Channels-last bf16 copies of the backbone's strided 1x1 downsample and global-average-pool
// gradients, at HBM rate (16-byte vectors; one output row, or one image, per workgroup).
//
// Reference: the bottleneck downsample (imagenet/resnet.py:87-108, conv1x1 stride 2) and the
// average pool (resnet.py:214) of the ResNet trained by main.py:311-326. conv1x1.py runs the
// downsample's backward as GEMMs on xs = x[:, :, ::s, ::s] and adds its input gradient into the
// strided positions of dx; backbone._GlobalAvgPoolCL writes the pooled gradient broadcast over
// H x W. torch's strided / broadcast elementwise kernels move those bytes at 2.9-3.5 TB/s
// (ResNet-50 b256: 243 us per step for the six strided copies and adds, 37 us for the broadcast).
//
//   pick:      out[n][i][j][:]      = x[n][s i][s j][:]                       (Ho = ceil(H / s))
//   add:       dx[n][s i][s j][:]  += src[n][i][j][:]   (fp32 sum rounded to bf16, as torch's add_)
//   broadcast: out[n][p][:]         = g[n][:]            (p < HW)

#include <hip/hip_bf16.h>

#include "dauc_internal.h"

namespace dauc {
namespace {

constexpr int kStThreads = 256;

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned add_bf16x2(unsigned a, unsigned b) {
    const float lo = __uint_as_float(a << 16) + __uint_as_float(b << 16);
    const float hi = __uint_as_float(a & 0xffff0000u) + __uint_as_float(b & 0xffff0000u);
    const unsigned short l = __bfloat16_as_ushort(__float2bfloat16(lo));
    const unsigned short h = __bfloat16_as_ushort(__float2bfloat16(hi));
    return unsigned(l) | (unsigned(h) << 16);
}

// one output row (n, i) per workgroup (blockIdx.x = n Ho + i); its Wo x CV vectors strided by the
// workgroup: vector e = j CV + cv
template <bool ADD>
__global__ __launch_bounds__(kStThreads) void strided_kernel(u32x4* __restrict__ big, u32x4* __restrict__ small, int H,
                                                             int W, int Ho, int Wo, int CV, int s) {
    const int row = blockIdx.x;
    const int n = row / Ho, i = row - n * Ho;
    const int64_t brow = (int64_t(n) * H + int64_t(s) * i) * W * CV;  // (n, s i, 0, 0) of the full tensor
    const int64_t srow = int64_t(row) * Wo * CV;
    const int nv = Wo * CV;
    for (int e = threadIdx.x; e < nv; e += kStThreads) {
        const int j = e / CV, cv = e - j * CV;
        const int64_t b = brow + int64_t(s) * j * CV + cv;
        if (ADD) {
            const u32x4 d = big[b], a = small[srow + e];
            big[b] = u32x4{add_bf16x2(d[0], a[0]), add_bf16x2(d[1], a[1]), add_bf16x2(d[2], a[2]), add_bf16x2(d[3], a[3])};
        } else {
            small[srow + e] = big[b];
        }
    }
}

// blockIdx.x = n: the image's HW x CV vectors, vector e = p CV + cv
__global__ __launch_bounds__(kStThreads) void broadcast_kernel(const u32x4* __restrict__ g, u32x4* __restrict__ out,
                                                               int HW, int CV) {
    const int n = blockIdx.x;
    const u32x4* gn = g + int64_t(n) * CV;
    u32x4* on = out + int64_t(n) * HW * CV;
    const int nv = HW * CV;
    for (int e = threadIdx.x; e < nv; e += kStThreads) on[e] = gn[e % CV];
}

bool args_ok(const void* a, const void* b, int64_t N, int H, int W, int C, int s) {
    return a != nullptr && b != nullptr && N >= 1 && H >= 1 && W >= 1 && C >= 8 && C % 8 == 0 && s >= 1 &&
           ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b)) & 15u) == 0;
}

}  // namespace
}  // namespace dauc

using namespace dauc;

extern "C" {

int dauc_strided_pick(const void* x, int dtype, int64_t N, int H, int W, int C, int stride, void* out,
                      dauc_stream_t stream) {
    if (dtype != DAUC_DTYPE_BF16 || !args_ok(x, out, N, H, W, C, stride)) return DAUC_EINVAL;
    const int Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
    if (N * Ho > 0x7fffffffLL || int64_t(Wo) * (C / 8) > 0x7fffffffLL) return DAUC_EINVAL;
    hipLaunchKernelGGL(strided_kernel<false>, dim3(static_cast<unsigned>(N * Ho)), dim3(kStThreads), 0,
                       as_hip(stream), const_cast<u32x4*>(static_cast<const u32x4*>(x)), static_cast<u32x4*>(out), H,
                       W, Ho, Wo, C / 8, stride);
    return launch_status();
}

int dauc_strided_add(void* dx, int dtype, int64_t N, int H, int W, int C, int stride, const void* src,
                     dauc_stream_t stream) {
    if (dtype != DAUC_DTYPE_BF16 || !args_ok(dx, src, N, H, W, C, stride)) return DAUC_EINVAL;
    const int Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
    if (N * Ho > 0x7fffffffLL || int64_t(Wo) * (C / 8) > 0x7fffffffLL) return DAUC_EINVAL;
    hipLaunchKernelGGL(strided_kernel<true>, dim3(static_cast<unsigned>(N * Ho)), dim3(kStThreads), 0,
                       as_hip(stream), static_cast<u32x4*>(dx), const_cast<u32x4*>(static_cast<const u32x4*>(src)), H,
                       W, Ho, Wo, C / 8, stride);
    return launch_status();
}

int dauc_broadcast_hw(const void* g, int dtype, int64_t N, int64_t HW, int C, void* out, dauc_stream_t stream) {
    if (dtype != DAUC_DTYPE_BF16 || g == nullptr || out == nullptr || N < 1 || HW < 1 || C < 8 || C % 8) return DAUC_EINVAL;
    if ((reinterpret_cast<uintptr_t>(g) | reinterpret_cast<uintptr_t>(out)) & 15u) return DAUC_EINVAL;
    if (N > 0x7fffffffLL || HW * (C / 8) > 0x7fffffffLL) return DAUC_EINVAL;
    hipLaunchKernelGGL(broadcast_kernel, dim3(static_cast<unsigned>(N)), dim3(kStThreads), 0, as_hip(stream),
                       static_cast<const u32x4*>(g), static_cast<u32x4*>(out), static_cast<int>(HW), C / 8);
    return launch_status();
}

}  // extern "C"
