// Proximal primal-dual SGD update over the flat parameter buffer, fused with
// the per-step running average; CoDA round finalisation; stage-end division.
//
// Reference: imagenet/main.py:56-64 (dppd_sg), main.py:333-334 (running
// average), main.py:33-54 + 297-301 (average_all / count folding),
// main.py:338-339 (stage-end division).
//
// HBM traffic per parameter: read w, g, w0 (12 B) + write w (4 B) = 16 B, plus
// read+write of the running average (8 B) = 24 B when fused. Every element is
// touched exactly once, 16 B per lane per access (float4), one launch for all
// parameter tensors: the gradients stay where autograd left them and are found
// through a segment table passed in the kernel arguments.
//
// Numerics: the fp32 operation order of main.py:61 with every operation
// rounded separately (no FMA contraction), so the result is bit-identical to
// the reference's torch fp32 ops: w' = w - lr*(g + (1/gamma)*(w - w0)).

#include "dauc_internal.h"

namespace dauc {
namespace {

constexpr int kThreads = 256;
constexpr int kMaxSeg = 176;  // segments per launch (kernel-argument table, < 4 KB)
constexpr int kSearchSlots = 192;  // blk_start entries: kMaxSeg + 1 rounded up to whole waves

// Geometry: VPT float4 per thread -> 256*4*VPT elements per block. The default
// (variant 0) is VPT = 2 with non-temporal g/w0 loads: fastest on MI355X
// (scripts/micro_kernels.py sweep, 82 us for ResNet-50's 23.5M parameters).

constexpr int64_t elems_per_block(int vpt) { return int64_t(kThreads) * 4 * vpt; }

struct SegTable {
    int nseg;
    int blk_start[kSearchSlots];  // first block of each segment; blk_start[nseg] = grid; INT_MAX after
    const float* grad[kMaxSeg];
    int offset[kMaxSeg];         // element offsets / counts fit 31 bits (checked on the host)
    int numel[kMaxSeg];
};
static_assert(sizeof(SegTable) < 4000, "kernel-argument table must stay below 4 KB");

__device__ __forceinline__ float pd_step(float w, float g, float w0, float lr, float invg) {
    const float d = __fsub_rn(w, w0);       // (param.data - model0[name])
    const float t = __fmul_rn(invg, d);     // 1/gamma * (...)
    const float gp = __fadd_rn(g, t);       // param.grad.data + ...
    const float u = __fmul_rn(lr, gp);      // lr * (...)
    return __fsub_rn(w, u);                 // param.data - ...
}

__device__ void scalar_update(float* s, const float* g3, const float* a3, float lr, float invg,
                              int mode) {
    const float a = s[0], b = s[1], al = s[2];
    const float a_new = pd_step(a, g3[0], a3[0], lr, invg);   // main.py:58
    float b_new, al_new;
    if (mode == DAUC_MODE_PAPER) {
        b_new = pd_step(b, g3[1], a3[1], lr, invg);           // intended (b - b0)
        al_new = __fadd_rn(al, __fmul_rn(lr, g3[2]));         // dual ascent
    } else {
        // main.py:59 uses the UPDATED a in b's proximal term; main.py:64 only
        // rebinds a local name, so alpha is left unchanged.
        const float t = __fmul_rn(invg, __fsub_rn(a_new, a3[0]));
        b_new = __fsub_rn(b, __fmul_rn(lr, __fadd_rn(g3[1], t)));
        al_new = al;
    }
    s[0] = a_new;
    s[1] = b_new;
    s[2] = al_new;
}

template <bool AVG, int VPT, bool NT, bool NTALL = false>
__global__ __launch_bounds__(kThreads) void pd_update_kernel(
    float* __restrict__ w, const float* __restrict__ w0, float* __restrict__ wavg, SegTable tab,
    float lr, float invg, float* __restrict__ scalars, const float* __restrict__ grad3,
    const float* __restrict__ anchor3, int mode) {
    const int bid = blockIdx.x;
    if (scalars != nullptr && bid == 0 && threadIdx.x == 0)
        scalar_update(scalars, grad3, anchor3, lr, invg, mode);

    // segment owning this block: every lane tests a few segment starts at once (independent
    // loads from the kernel-argument table), the count of starts <= bid is the segment + 1.
    // (A binary search is ~8 dependent scalar loads, ~0.7 us at every block's start.)
    int lo;
    {
        const int lane = threadIdx.x & (kWave - 1);
        int cnt = 0;
#pragma unroll
        for (int base = 0; base < kSearchSlots; base += kWave) {
            const int start = tab.blk_start[base + lane];  // unconditional: all loads in flight together
            cnt += __popcll(__ballot(start <= bid));
        }
        lo = __builtin_amdgcn_readfirstlane(cnt - 1);
    }
    const float* __restrict__ g = tab.grad[lo];
    const int64_t off = tab.offset[lo];
    const int64_t n = tab.numel[lo];
    constexpr int64_t kElemsPerBlock = elems_per_block(VPT);
    const int64_t e0 = int64_t(bid - tab.blk_start[lo]) * kElemsPerBlock;
    float* __restrict__ ws = w + off;
    const float* __restrict__ w0s = w0 + off;
    float* __restrict__ as = AVG ? wavg + off : nullptr;

    const bool vec_ok = ((off & 3) == 0) && ((reinterpret_cast<uintptr_t>(g) & 15u) == 0);
    if (vec_ok) {
        // VPT independent float4 slots per thread, all loads issued before any math.
        // A segment's last block guards each slot; only its final n % 4 elements go scalar.
        f32x4 wv[VPT], gv[VPT], zv[VPT], av[VPT];
        bool full[VPT];
#pragma unroll
        for (int v = 0; v < VPT; ++v) {
            const int64_t i = e0 + (int64_t(v) * kThreads + threadIdx.x) * 4;
            full[v] = i + 4 <= n;
            if (full[v]) {
                if (NTALL) wv[v] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(ws + i));
                else wv[v] = *reinterpret_cast<const f32x4*>(ws + i);
                if (NT) {
                    gv[v] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(g + i));
                    zv[v] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(w0s + i));
                } else {
                    gv[v] = *reinterpret_cast<const f32x4*>(g + i);
                    zv[v] = *reinterpret_cast<const f32x4*>(w0s + i);
                }
                if (AVG) {
                    if (NTALL) av[v] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(as + i));
                    else av[v] = *reinterpret_cast<const f32x4*>(as + i);
                }
            }
        }
#pragma unroll
        for (int v = 0; v < VPT; ++v) {
            const int64_t i = e0 + (int64_t(v) * kThreads + threadIdx.x) * 4;
            if (full[v]) {
                f32x4 r;
#pragma unroll
                for (int c = 0; c < 4; ++c) r[c] = pd_step(wv[v][c], gv[v][c], zv[v][c], lr, invg);
                if (NTALL) __builtin_nontemporal_store(r, reinterpret_cast<f32x4*>(ws + i));
                else *reinterpret_cast<f32x4*>(ws + i) = r;
                if (AVG) {
                    f32x4 a;
#pragma unroll
                    for (int c = 0; c < 4; ++c) a[c] = __fadd_rn(av[v][c], r[c]);
                    if (NTALL) __builtin_nontemporal_store(a, reinterpret_cast<f32x4*>(as + i));
                    else *reinterpret_cast<f32x4*>(as + i) = a;
                }
            } else {
                for (int64_t j = i; j < n && j < i + 4; ++j) {
                    const float r = pd_step(ws[j], g[j], w0s[j], lr, invg);
                    ws[j] = r;
                    if (AVG) as[j] = __fadd_rn(as[j], r);
                }
            }
        }
        return;
    }
    // unaligned gradient: scalar loop over this block's element range
    const int64_t e1 = (e0 + kElemsPerBlock < n) ? e0 + kElemsPerBlock : n;
    for (int64_t i = e0 + threadIdx.x; i < e1; i += kThreads) {
        const float r = pd_step(ws[i], g[i], w0s[i], lr, invg);
        ws[i] = r;
        if (AVG) as[i] = __fadd_rn(as[i], r);
    }
}

// scalars-only launch (used when the tensor list is empty)
__global__ void scalar_update_kernel(float* s, const float* g3, const float* a3, float lr,
                                     float invg, int mode) {
    scalar_update(s, g3, a3, lr, invg, mode);
}

template <int VPT, bool NT, bool NTALL = false>
int launch_table_t(float* w, const float* w0, float* wavg, const SegTable& tab, float lr, float invg,
                   float* scalars, const float* grad3, const float* anchor3, int mode, hipStream_t st) {
    const int grid = tab.blk_start[tab.nseg];
    if (grid <= 0) return DAUC_OK;
    if (wavg)
        hipLaunchKernelGGL((pd_update_kernel<true, VPT, NT, NTALL>), dim3(grid), dim3(kThreads), 0, st, w, w0, wavg,
                           tab, lr, invg, scalars, grad3, anchor3, mode);
    else
        hipLaunchKernelGGL((pd_update_kernel<false, VPT, NT, NTALL>), dim3(grid), dim3(kThreads), 0, st, w, w0,
                           wavg, tab, lr, invg, scalars, grad3, anchor3, mode);
    return launch_status();
}

// variant = vpt_index + 4 * k: vpt in {2, 1, 4, 3}; k = 0: non-temporal g/w0 loads, 1: all plain,
// 2: every load and store non-temporal
int launch_table(int variant, float* w, const float* w0, float* wavg, const SegTable& tab, float lr,
                 float invg, float* scalars, const float* grad3, const float* anchor3, int mode,
                 hipStream_t st) {
    switch (variant) {
        case 0: return launch_table_t<2, true>(w, w0, wavg, tab, lr, invg, scalars, grad3, anchor3, mode, st);
#ifdef DAUC_TUNING
        case 1: return launch_table_t<1, true>(w, w0, wavg, tab, lr, invg, scalars, grad3, anchor3, mode, st);
        case 2: return launch_table_t<4, true>(w, w0, wavg, tab, lr, invg, scalars, grad3, anchor3, mode, st);
        case 3: return launch_table_t<3, true>(w, w0, wavg, tab, lr, invg, scalars, grad3, anchor3, mode, st);
        case 4: return launch_table_t<2, false>(w, w0, wavg, tab, lr, invg, scalars, grad3, anchor3, mode, st);
        case 5: return launch_table_t<1, false>(w, w0, wavg, tab, lr, invg, scalars, grad3, anchor3, mode, st);
        case 6: return launch_table_t<4, false>(w, w0, wavg, tab, lr, invg, scalars, grad3, anchor3, mode, st);
        case 7: return launch_table_t<3, false>(w, w0, wavg, tab, lr, invg, scalars, grad3, anchor3, mode, st);
        case 8: return launch_table_t<2, true, true>(w, w0, wavg, tab, lr, invg, scalars, grad3, anchor3, mode, st);
        case 9: return launch_table_t<1, true, true>(w, w0, wavg, tab, lr, invg, scalars, grad3, anchor3, mode, st);
        case 10: return launch_table_t<4, true, true>(w, w0, wavg, tab, lr, invg, scalars, grad3, anchor3, mode, st);
        case 11: return launch_table_t<3, true, true>(w, w0, wavg, tab, lr, invg, scalars, grad3, anchor3, mode, st);
#endif
        default: return DAUC_EINVAL;
    }
}

int variant_vpt(int variant) {
    static const int vpt[4] = {2, 1, 4, 3};
    return vpt[variant & 3];
}

// ---- CoDA finalisation and stage-end division ---------------------------------

template <bool DIV_ONLY>
__global__ __launch_bounds__(kThreads) void div_kernel(float* __restrict__ x, int64_t n, float d,
                                                       float* __restrict__ lcounts,
                                                       float* __restrict__ gcounts) {
    if (!DIV_ONLY && blockIdx.x == 0 && threadIdx.x == 0) {
        // main.py:46-50 + 300-301: counts were summed by the all-reduce; fold them
        // into the fp32 global accumulators and restart the local ones.
        gcounts[0] = __fadd_rn(gcounts[0], lcounts[0]);
        gcounts[1] = __fadd_rn(gcounts[1], lcounts[1]);
        lcounts[0] = 0.0f;
        lcounts[1] = 0.0f;
    }
    const int64_t nvec = (reinterpret_cast<uintptr_t>(x) & 15u) ? 0 : n / 4;
    const int64_t stride = int64_t(gridDim.x) * kThreads;
    for (int64_t v = int64_t(blockIdx.x) * kThreads + threadIdx.x; v < nvec; v += stride) {
        float4 a = reinterpret_cast<float4*>(x)[v];
        a.x = __fdiv_rn(a.x, d);
        a.y = __fdiv_rn(a.y, d);
        a.z = __fdiv_rn(a.z, d);
        a.w = __fdiv_rn(a.w, d);
        reinterpret_cast<float4*>(x)[v] = a;
    }
    for (int64_t i = nvec * 4 + int64_t(blockIdx.x) * kThreads + threadIdx.x; i < n; i += stride)
        x[i] = __fdiv_rn(x[i], d);
}

int div_grid(int64_t n) {
    int64_t g = (n / 4 + kThreads - 1) / kThreads;
    if (g < 1) g = 1;
    if (g > 2048) g = 2048;
    return static_cast<int>(g);
}

}  // namespace
}  // namespace dauc

using namespace dauc;

extern "C" {

static int pd_update_impl(float* w, const float* w0, float* w_avg, const dauc_grad_seg* segs, int nseg,
                          float* scalars, const float* grad3, const float* anchor3, float lr,
                          float inv_gamma, int mode, int variant, dauc_stream_t stream) {
    if (w == nullptr || w0 == nullptr || nseg < 0 || (nseg > 0 && segs == nullptr))
        return DAUC_EINVAL;
    if (scalars != nullptr && (grad3 == nullptr || anchor3 == nullptr)) return DAUC_EINVAL;
    if (mode != DAUC_MODE_REFERENCE && mode != DAUC_MODE_PAPER) return DAUC_EINVAL;
    if (variant < 0 || variant >= 12) return DAUC_EINVAL;
    for (int i = 0; i < nseg; ++i)
        if (segs[i].numel < 0 || segs[i].offset < 0 || (segs[i].numel > 0 && !segs[i].grad) ||
            segs[i].offset + segs[i].numel > 0x7fffffffLL)
            return DAUC_EINVAL;
    hipStream_t st = as_hip(stream);
    const int64_t epb = elems_per_block(variant_vpt(variant));
    SegTable tab;
    int i = 0;
    bool first = true;
    while (i < nseg) {
        tab.nseg = 0;
        int64_t blocks = 0;
        while (i < nseg && tab.nseg < kMaxSeg) {
            const dauc_grad_seg& s = segs[i++];
            if (s.numel == 0) continue;
            const int64_t nb = (s.numel + epb - 1) / epb;
            if (blocks + nb > 0x7fffffffLL) return DAUC_EINVAL;
            tab.blk_start[tab.nseg] = static_cast<int>(blocks);
            tab.grad[tab.nseg] = s.grad;
            tab.offset[tab.nseg] = static_cast<int>(s.offset);
            tab.numel[tab.nseg] = static_cast<int>(s.numel);
            blocks += nb;
            ++tab.nseg;
        }
        tab.blk_start[tab.nseg] = static_cast<int>(blocks);
        for (int j = tab.nseg + 1; j < kSearchSlots; ++j) tab.blk_start[j] = 0x7fffffff;  // never <= a block id
        if (tab.nseg == 0) continue;
        // the scalar part rides in the first launch only
        const int rc = launch_table(variant, w, w0, w_avg, tab, lr, inv_gamma, first ? scalars : nullptr,
                                    grad3, anchor3, mode, st);
        if (rc != DAUC_OK) return rc;
        first = false;
    }
    if (first && scalars != nullptr) {  // no non-empty segment: scalars only
        hipLaunchKernelGGL(scalar_update_kernel, dim3(1), dim3(1), 0, st, scalars, grad3, anchor3, lr,
                           inv_gamma, mode);
        return launch_status();
    }
    return DAUC_OK;
}

int dauc_pd_update(float* w, const float* w0, float* w_avg, const dauc_grad_seg* segs, int nseg,
                   float* scalars, const float* grad3, const float* anchor3, float lr,
                   float inv_gamma, int mode, dauc_stream_t stream) {
    return pd_update_impl(w, w0, w_avg, segs, nseg, scalars, grad3, anchor3, lr, inv_gamma, mode, 0,
                          stream);
}

static int pd_update_dense_impl(float* w, const float* g, const float* w0, float* w_avg, int64_t n, float lr,
                                float inv_gamma, int variant, dauc_stream_t stream) {
    if (w == nullptr || g == nullptr || w0 == nullptr || n < 0) return DAUC_EINVAL;
    if (n == 0) return DAUC_OK;
    dauc_grad_seg seg{g, 0, n};
    return pd_update_impl(w, w0, w_avg, &seg, 1, nullptr, nullptr, nullptr, lr, inv_gamma,
                          DAUC_MODE_REFERENCE, variant, stream);
}

#ifdef DAUC_TUNING
int dauc_pd_update_dense_variant(float* w, const float* g, const float* w0, float* w_avg, int64_t n,
                                 float lr, float inv_gamma, int variant, dauc_stream_t stream) {
    return pd_update_dense_impl(w, g, w0, w_avg, n, lr, inv_gamma, variant, stream);
}
#endif

int dauc_pd_update_dense(float* w, const float* g, const float* w0, float* w_avg, int64_t n,
                         float lr, float inv_gamma, dauc_stream_t stream) {
    return pd_update_dense_impl(w, g, w0, w_avg, n, lr, inv_gamma, 0, stream);
}

int dauc_coda_finalize(float* flat, int64_t n_avg, int world, float* lcounts, float* gcounts,
                       dauc_stream_t stream) {
    if (flat == nullptr || n_avg < 0 || world < 1 || lcounts == nullptr || gcounts == nullptr)
        return DAUC_EINVAL;
    hipStream_t st = as_hip(stream);
    // world == 1: the reference skips averaging (main.py:297-299) and only folds counts
    const int64_t n = world == 1 ? 0 : n_avg;
    hipLaunchKernelGGL(div_kernel<false>, dim3(div_grid(n)), dim3(kThreads), 0, st, flat, n,
                       static_cast<float>(world), lcounts, gcounts);
    return launch_status();
}

int dauc_scale_div(float* x, int64_t n, float divisor, dauc_stream_t stream) {
    if (x == nullptr || n < 0) return DAUC_EINVAL;
    if (n == 0) return DAUC_OK;
    hipLaunchKernelGGL(div_kernel<true>, dim3(div_grid(n)), dim3(kThreads), 0, as_hip(stream), x,
                       n, divisor, nullptr, nullptr);
    return launch_status();
}

}  // extern "C"
