// Sum of S equal-sized fp32 slabs: out[i] = sum_s part[s * n + i], s ascending (n % 4 == 0).
//
// The split-K weight gradients of the backbone's 1x1 convolutions (conv1x1.py: dW = dy^T x
// with K = N*H*W rows split into S slabs by one batched GEMM, fp32 partials) end with this
// reduction; torch's generic reduce over the outer dimension ran it at ~11 us a launch for
// 0.1-2 MB. Here a thread owns one float4 column and walks the slabs with all loads of a
// group of 8 slabs in flight: the slabs are read once, coalesced, and the fixed slab order
// makes the result bitwise reproducible.

#include "dauc_internal.h"

namespace dauc {
namespace {

constexpr int kSlabThreads = 256;
constexpr int kSlabGroup = 8;

__global__ __launch_bounds__(kSlabThreads) void slab_sum_kernel(const float* __restrict__ part, int64_t S,
                                                                int64_t nv, float* __restrict__ out) {
    const int64_t v = int64_t(blockIdx.x) * kSlabThreads + threadIdx.x;  // float4 column
    if (v >= nv) return;
    const f32x4* __restrict__ p = reinterpret_cast<const f32x4*>(part) + v;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    int64_t s = 0;
    for (; s + kSlabGroup <= S; s += kSlabGroup) {
        f32x4 x[kSlabGroup];
#pragma unroll
        for (int g = 0; g < kSlabGroup; ++g) x[g] = __builtin_nontemporal_load(p + (s + g) * nv);
#pragma unroll
        for (int g = 0; g < kSlabGroup; ++g) acc += x[g];
    }
    for (; s < S; ++s) acc += p[s * nv];
    reinterpret_cast<f32x4*>(out)[v] = acc;
}

}  // namespace
}  // namespace dauc

using namespace dauc;

extern "C" {

int dauc_slab_sum(const float* part, int64_t S, int64_t n, float* out, dauc_stream_t stream) {
    if (part == nullptr || out == nullptr || S < 1 || n < 4 || n % 4) return DAUC_EINVAL;
    if ((reinterpret_cast<uintptr_t>(part) | reinterpret_cast<uintptr_t>(out)) & 15u) return DAUC_EINVAL;
    const int64_t nv = n / 4;
    const int64_t grid = (nv + kSlabThreads - 1) / kSlabThreads;
    if (grid > 0x7fffffffLL) return DAUC_EINVAL;
    hipLaunchKernelGGL(slab_sum_kernel, dim3(static_cast<unsigned>(grid)), dim3(kSlabThreads), 0, as_hip(stream),
                       part, S, nv, out);
    return launch_status();
}

}  // extern "C"
