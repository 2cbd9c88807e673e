// Streaming-ceiling probe for the surrogate's access mix (tuning only, not product code).
//
// The surrogate reads h (fp32, 4 B) + y (int8, 1 B) and writes dh (fp32, 4 B) per element.
// These kernels do the same traffic with trivial math (and optionally the per-lane
// accumulators), so the surrogate kernel can be priced against what this chip streams for
// a 5:4 read:write mix, not against a copy measured by someone else.
//
// Built by scripts/probe_stream.py with hipcc --offload-arch=gfx950 -O3.

#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace {

constexpr int kT = 256;

template <bool NT>
__device__ __forceinline__ f32x4 ld4(const f32x4* p) {
    if (NT) return __builtin_nontemporal_load(p);
    return *p;
}
template <bool NT>
__device__ __forceinline__ int ld1(const int* p) {
    if (NT) return __builtin_nontemporal_load(p);
    return *p;
}
template <bool NT>
__device__ __forceinline__ void st4(f32x4 v, f32x4* p) {
    if (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

__device__ __forceinline__ float sel(int lab, float h) {
    // dF/dh = c * (h - k), (c, k) chosen by the label byte: the surrogate's per-element math
    const bool pos = (lab & 0xff) == 1;
    return (pos ? 0.0018f : 0.0003f) * (h - (pos ? 1.2f : -0.7f));
}

// chunk per block: S float4 slots per thread, one contiguous chunk of 1024*S elements
template <int S, bool NTL, bool NTS, bool COPY>
__global__ __launch_bounds__(kT) void chunk_kernel(const float* __restrict__ h, const int8_t* __restrict__ y,
                                                   float* __restrict__ dh, int64_t n, float* sink) {
    const int64_t base = int64_t(blockIdx.x) * (kT * 4 * S);
    if (base + kT * 4 * S > n) return;
    f32x4 hv[S];
    int yv[S];
#pragma unroll
    for (int k = 0; k < S; ++k) {
        const int64_t b = base + (int64_t(k) * kT + threadIdx.x) * 4;
        hv[k] = ld4<NTL>(reinterpret_cast<const f32x4*>(h + b));
        if (!COPY) yv[k] = ld1<NTL>(reinterpret_cast<const int*>(y + b));
    }
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < S; ++k) {
        const int64_t b = base + (int64_t(k) * kT + threadIdx.x) * 4;
        f32x4 g = hv[k];
        if (!COPY) {
            g.x = sel(yv[k], g.x);
            g.y = sel(yv[k] >> 8, g.y);
            g.z = sel(yv[k] >> 16, g.z);
            g.w = sel(yv[k] >> 24, g.w);
            acc += g.x + g.y + g.z + g.w;
        }
        st4<NTS>(g, reinterpret_cast<f32x4*>(dh + b));
    }
    if (acc == 12345.678f) sink[0] = acc;  // keep the math alive, never true in practice
}

// persistent grid-stride: grid = blocks, each iteration S slots per thread
template <int S, bool NTL, bool NTS>
__global__ __launch_bounds__(kT) void stride_kernel(const float* __restrict__ h, const int8_t* __restrict__ y,
                                                    float* __restrict__ dh, int64_t n, float* sink) {
    const int64_t step = int64_t(gridDim.x) * (kT * 4 * S);
    float acc = 0.f;
    for (int64_t base = int64_t(blockIdx.x) * (kT * 4 * S); base + kT * 4 * S <= n; base += step) {
        f32x4 hv[S];
        int yv[S];
#pragma unroll
        for (int k = 0; k < S; ++k) {
            const int64_t b = base + (int64_t(k) * kT + threadIdx.x) * 4;
            hv[k] = ld4<NTL>(reinterpret_cast<const f32x4*>(h + b));
            yv[k] = ld1<NTL>(reinterpret_cast<const int*>(y + b));
        }
#pragma unroll
        for (int k = 0; k < S; ++k) {
            const int64_t b = base + (int64_t(k) * kT + threadIdx.x) * 4;
            f32x4 g = hv[k];
            g.x = sel(yv[k], g.x);
            g.y = sel(yv[k] >> 8, g.y);
            g.z = sel(yv[k] >> 16, g.z);
            g.w = sel(yv[k] >> 24, g.w);
            acc += g.x + g.y + g.z + g.w;
            st4<NTS>(g, reinterpret_cast<f32x4*>(dh + b));
        }
    }
    if (acc == 12345.678f) sink[0] = acc;
}

// wide labels: a lane owns 16 consecutive elements per slot (one 16-B label load, four
// float4 h loads that together cover 64 B per lane)
template <int S, bool NTL, bool NTS>
__global__ __launch_bounds__(kT) void wide_kernel(const float* __restrict__ h, const int8_t* __restrict__ y,
                                                  float* __restrict__ dh, int64_t n, float* sink) {
    const int64_t base = int64_t(blockIdx.x) * (kT * 16 * S);
    if (base + kT * 16 * S > n) return;
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < S; ++k) {
        const int64_t b = base + (int64_t(k) * kT + threadIdx.x) * 16;
        typedef int i32x4 __attribute__((ext_vector_type(4)));
        i32x4 yl;
        if (NTL) yl = __builtin_nontemporal_load(reinterpret_cast<const i32x4*>(y + b));
        else yl = *reinterpret_cast<const i32x4*>(y + b);
        f32x4 hv[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) hv[q] = ld4<NTL>(reinterpret_cast<const f32x4*>(h + b) + q);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int l = yl[q];
            f32x4 g = hv[q];
            g.x = sel(l, g.x);
            g.y = sel(l >> 8, g.y);
            g.z = sel(l >> 16, g.z);
            g.w = sel(l >> 24, g.w);
            acc += g.x + g.y + g.z + g.w;
            st4<NTS>(g, reinterpret_cast<f32x4*>(dh + b) + q);
        }
    }
    if (acc == 12345.678f) sink[0] = acc;
}


// persistent, software-pipelined: the next chunk's loads are issued before the current
// chunk's math and stores. CONTIG: block b walks its own contiguous region; else grid-stride.
// QUEUE: chunks are claimed in address order from an atomic counter (claim prefetched).
template <int S, bool CONTIG, bool QUEUE>
__global__ __launch_bounds__(kT) void pipe_kernel(const float* __restrict__ h, const int8_t* __restrict__ y,
                                                  float* __restrict__ dh, int64_t n, float* sink,
                                                  unsigned* counter) {
    constexpr int64_t C = int64_t(kT) * 4 * S;
    const int64_t nchunks = n / C;
    const int64_t per = (nchunks + gridDim.x - 1) / gridDim.x;
    __shared__ int64_t next_claim;
    auto first = [&]() -> int64_t {
        if (QUEUE) {
            if (threadIdx.x == 0) next_claim = atomicAdd(counter, 1u);
            __syncthreads();
            return next_claim;
        }
        return CONTIG ? int64_t(blockIdx.x) * per : int64_t(blockIdx.x);
    };
    int64_t c = first();
    const int64_t cend = CONTIG ? ((int64_t(blockIdx.x) + 1) * per < nchunks ? (int64_t(blockIdx.x) + 1) * per : nchunks)
                                : nchunks;
    f32x4 hv[S];
    int yv[S];
    auto load = [&](int64_t cc) {
#pragma unroll
        for (int k = 0; k < S; ++k) {
            const int64_t b = cc * C + (int64_t(k) * kT + threadIdx.x) * 4;
            hv[k] = ld4<true>(reinterpret_cast<const f32x4*>(h + b));
            yv[k] = ld1<true>(reinterpret_cast<const int*>(y + b));
        }
    };
    float acc = 0.f;
    if (c < cend) load(c);
    while (c < cend) {
        int64_t nc;
        if (QUEUE) {
            __syncthreads();
            if (threadIdx.x == 0) next_claim = atomicAdd(counter, 1u);
            __syncthreads();
            nc = next_claim;
        } else {
            nc = CONTIG ? c + 1 : c + gridDim.x;
        }
        f32x4 cur[S];
        int cy[S];
#pragma unroll
        for (int k = 0; k < S; ++k) { cur[k] = hv[k]; cy[k] = yv[k]; }
        if (nc < cend) load(nc);
#pragma unroll
        for (int k = 0; k < S; ++k) {
            const int64_t b = c * C + (int64_t(k) * kT + threadIdx.x) * 4;
            f32x4 g = cur[k];
            g.x = sel(cy[k], g.x);
            g.y = sel(cy[k] >> 8, g.y);
            g.z = sel(cy[k] >> 16, g.z);
            g.w = sel(cy[k] >> 24, g.w);
            acc += g.x + g.y + g.z + g.w;
            st4<true>(g, reinterpret_cast<f32x4*>(dh + b));
        }
        c = nc;
    }
    if (acc == 12345.678f) sink[0] = acc;
}

}  // namespace

extern "C" {

// kind: 0 copy (S=8), 1 chunk S=8 nt/nt, 2 chunk S=16 nt/nt, 3 chunk S=8 plain, 4 chunk S=8 ntload only,
//       5 stride S=4 2 blocks/CU, 6 stride S=8 1 block/CU, 7 wide S=2, 8 wide S=4, 9 chunk S=4 nt/nt,
//       10 stride S=8 4 blocks/CU, 11 copy S=16
// returns average ms per launch over reps (hip events on the null stream), or -1 on error
float probe_run(int kind, const float* h, const int8_t* y, float* dh, int64_t n, float* sink, int reps) {
    unsigned* counter = reinterpret_cast<unsigned*>(sink + 2);
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return -1.f;
    int dev = 0, cus = 256;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    auto launch = [&]() {
        switch (kind) {
            case 0: chunk_kernel<8, true, true, true><<<n / (kT * 32), kT>>>(h, y, dh, n, sink); break;
            case 1: chunk_kernel<8, true, true, false><<<n / (kT * 32), kT>>>(h, y, dh, n, sink); break;
            case 2: chunk_kernel<16, true, true, false><<<n / (kT * 64), kT>>>(h, y, dh, n, sink); break;
            case 3: chunk_kernel<8, false, false, false><<<n / (kT * 32), kT>>>(h, y, dh, n, sink); break;
            case 4: chunk_kernel<8, true, false, false><<<n / (kT * 32), kT>>>(h, y, dh, n, sink); break;
            case 5: stride_kernel<4, true, true><<<cus * 2, kT>>>(h, y, dh, n, sink); break;
            case 6: stride_kernel<8, true, true><<<cus, kT>>>(h, y, dh, n, sink); break;
            case 7: wide_kernel<2, true, true><<<n / (kT * 32), kT>>>(h, y, dh, n, sink); break;
            case 8: wide_kernel<4, true, true><<<n / (kT * 64), kT>>>(h, y, dh, n, sink); break;
            case 9: chunk_kernel<4, true, true, false><<<n / (kT * 16), kT>>>(h, y, dh, n, sink); break;
            case 10: stride_kernel<8, true, true><<<cus * 4, kT>>>(h, y, dh, n, sink); break;
            case 11: chunk_kernel<16, true, true, true><<<n / (kT * 64), kT>>>(h, y, dh, n, sink); break;
            case 12: pipe_kernel<8, true, false><<<cus * 2, kT>>>(h, y, dh, n, sink, counter); break;
            case 13: pipe_kernel<8, true, false><<<cus * 4, kT>>>(h, y, dh, n, sink, counter); break;
            case 14: pipe_kernel<8, false, false><<<cus * 2, kT>>>(h, y, dh, n, sink, counter); break;
            case 15: pipe_kernel<8, false, false><<<cus * 4, kT>>>(h, y, dh, n, sink, counter); break;
            case 16: pipe_kernel<4, false, false><<<cus * 4, kT>>>(h, y, dh, n, sink, counter); break;
            case 17: (void)hipMemsetAsync(counter, 0, 4, 0);
                     pipe_kernel<8, false, true><<<cus * 2, kT>>>(h, y, dh, n, sink, counter); break;
            case 18: (void)hipMemsetAsync(counter, 0, 4, 0);
                     pipe_kernel<8, false, true><<<cus * 4, kT>>>(h, y, dh, n, sink, counter); break;
            case 19: (void)hipMemsetAsync(counter, 0, 4, 0);
                     pipe_kernel<4, false, true><<<cus * 4, kT>>>(h, y, dh, n, sink, counter); break;
            default: break;
        }
    };
    launch();
    launch();
    hipEventRecord(e0, 0);
    for (int r = 0; r < reps; ++r) launch();
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    if (hipGetLastError() != hipSuccess) return -1.f;
    return ms / reps;
}

}  // extern "C"
