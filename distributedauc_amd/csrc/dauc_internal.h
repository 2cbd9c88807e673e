// Internal helpers shared by the libdauc.so translation units (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dauc.h"

namespace dauc {

constexpr int kWave = 64;  // CDNA wavefront width

// native 16-byte vector (one dwordx4 per lane); usable with the nontemporal builtins
typedef float f32x4 __attribute__((ext_vector_type(4)));

inline hipStream_t as_hip(dauc_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

// Launch-status helper: a failed launch is reported as -(hipError_t).
inline int launch_status() {
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? DAUC_OK : -static_cast<int>(e);
}

// ---- wavefront / block reductions (64-lane waves) ----------------------------

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
    return v;
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
    return v;
}

// Sum K doubles across the block. Every thread gets the block totals in v[].
// `scratch` must hold K * (blockDim.x / 64) doubles. The order of additions is
// fixed by the thread layout, so the result is bitwise reproducible.
template <int K>
__device__ __forceinline__ void block_sum(double (&v)[K], double* scratch) {
    const int lane = threadIdx.x & (kWave - 1);
    const int wid = threadIdx.x / kWave;
    const int nw = blockDim.x / kWave;
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = wave_sum(v[k]);
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k) scratch[k * nw + wid] = v[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < K; ++k) {
        double s = 0.0;
        for (int w = 0; w < nw; ++w) s += scratch[k * nw + w];
        v[k] = s;
    }
    __syncthreads();
}

// ---- inter-workgroup "last arriver" ticket ------------------------------------
// Producer side of the agent-scope release/acquire hand-off (cdna_hip_programming
// §6 Guideline 16): the calling block has stored its partial with plain stores
// from thread 0 only. Returns true in every thread of the block that arrived last;
// that block may then read every other block's partial with plain loads.
__device__ __forceinline__ bool arrive_last(unsigned* counter, unsigned nblocks, int* lds_flag) {
    if (threadIdx.x == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        unsigned t = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int last = (t == nblocks - 1);
        if (last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            // leave the workspace zeroed for the next call on this stream
            __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        *lds_flag = last;
    }
    __syncthreads();
    return *lds_flag != 0;
}

}  // namespace dauc
