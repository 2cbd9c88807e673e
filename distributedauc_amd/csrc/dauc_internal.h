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
// The write-through form of the agent-scope hand-off (cdna_hip_programming §6
// Guideline 16, R1): the payload (one workgroup's fp64 partial row) is stored by
// thread 0 with sc1 (write-through, agent-scope atomic) stores, drained with
// s_waitcnt vmcnt(0), and signalled by a relaxed agent-scope ticket add. The last
// arriver reads every row with sc1 loads (load_sc1), so neither a release fence
// (an L2 write-back that every workgroup would pay behind its streamed stores) nor
// an acquire is needed. Tickets start at zero and the last arriver resets them.
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned gu32;

__device__ __forceinline__ void store_sc1(double* p, double v) {
    __hip_atomic_store((gu64*)p, static_cast<unsigned long long>(__double_as_longlong(v)), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ double load_sc1(const double* p) {
    return __longlong_as_double(static_cast<long long>(
        __hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)));
}

// Called by every thread of the block after thread 0 stored its row with store_sc1.
// Returns true in every thread of the block that arrived last.
__device__ __forceinline__ bool arrive_last(unsigned* counter, unsigned nblocks, int* lds_flag) {
    if (threadIdx.x == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned t = __hip_atomic_fetch_add((gu32*)counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = (t == nblocks - 1);
        // leave the workspace zeroed for the next call on this stream
        if (last) __hip_atomic_store((gu32*)counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *lds_flag = last;
    }
    __syncthreads();
    // no instruction: keeps the compiler from hoisting the sc1 row loads above the ticket
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    return *lds_flag != 0;
}

// auc_count.hip: dauc_compact_positives that also zeroes zero3[0..3) and zero_w[0..nzero_w)
// (used by auc_eval.hip)
int compact_positives_zeroing(const float* scores, const void* labels, int label_dtype, int64_t n, float* pos_out,
                              int64_t* stats, void* workspace, size_t workspace_bytes, unsigned long long* zero3,
                              hipStream_t st, unsigned* zero_w = nullptr, int nzero_w = 0);

// auc_count.hip: the one-call evaluation's single-pass, unordered positive compaction. stats[0]
// (P), stats[2] (non-finite positives), stats[3] (labels outside {-1, 1}) must be zero on entry
// and stats[1] must hold `tag` (else no tile reserves or writes anything); block 0 zeroes
// zero_next[0, 2, 3], sets zero_next[1] = next_tag, and zeroes zero3[0..3) (nullable); the grid
// zeroes zero_w[0..nzero_w). At most `cap` positives are stored (stats[0] still counts them all).
// hist_out (nullable; kCiTop words, zero on entry) += the top-bucket histogram of the positives'
// keys (count_index.h), so a build from them can skip its histogram pass. *put = put_val (put
// nullable; block 0).
int compact_unordered(const float* scores, const void* labels, int label_dtype, int64_t n, float* pos_out,
                      unsigned long long* stats, unsigned long long tag, unsigned long long* zero_next,
                      unsigned long long next_tag, unsigned long long* zero3, unsigned* zero_w, int nzero_w,
                      hipStream_t st, int64_t cap = INT64_MAX, unsigned* hist_out = nullptr,
                      unsigned long long* put = nullptr, unsigned long long put_val = 0ull,
                      unsigned* fill_w = nullptr, int64_t nfill16 = 0);

// auc_sort.hip: the count index built straight from the unsorted positives (no radix sort, no
// tree) and the labeled query pass over scores [begin, end); the table is ordered by cell only.
// The table size M is read from the device (*Mp, the compaction's count), so nothing waits for the
// host; the workspace is carved for Mcap = direct_capacity(n) keys. Without a ready histogram
// the build's own `hist` (kCiTop words at direct_hist_offset(Mcap)) must be zero on entry; with
// one (the table's top-bucket histogram, whose total is the table size), the per-cell counters
// (direct_cnt_ptr) must be. *verdict (device) = 1 when the count index held the table, 2 when the
// caller must run the sorted path (M > Mcap, or a skewed table).
bool direct_enabled();  // the search mode is automatic (always, except in a tuning build's mode 1 / 2)
int64_t direct_capacity(int64_t n);
int64_t direct_hist_offset(int64_t Mcap);  // byte offset of `hist` in the sort workspace
// the per-cell counters the count pass adds into (zeroed by the histogram pass, or by the caller
// when it hands over a ready histogram)
unsigned* direct_cnt_ptr(void* workspace, int64_t Mcap);
int64_t direct_cnt_words();
struct DirectIndex;  // count_index.h
// the direct build alone (4 launches; 3 with a ready histogram: `ready_hist` (kCiTop words, or
// nullptr) already holds the table's top-bucket histogram and the per-cell counters are zero):
// fills *ix with the index's device pointers
int build_direct_index(const float* pos, const unsigned long long* Mp, int64_t Mcap, void* workspace,
                       size_t workspace_bytes, hipStream_t st, DirectIndex* ix, const unsigned* ready_hist = nullptr);
// check (nullable, one u32; the two-step evaluation's consistency word): += #queried scores
// (labels != 1) over [begin, end), mod 2^32 -- counted by the query pass whether or not the index
// held the table.
int counts_labeled_direct(const float* pos, const unsigned long long* Mp, int64_t Mcap, const float* scores,
                          const void* labels, int label_dtype, int64_t begin, int64_t end,
                          unsigned long long* wins_ties, unsigned long long* nonfinite, unsigned* verdict,
                          void* workspace, size_t workspace_bytes, hipStream_t st,
                          const unsigned* ready_hist = nullptr, unsigned* check = nullptr);

// the two-step evaluation's build + query straight from the gathered slots (no gather copy):
// the count pass reads the slots in place (and writes the part's record header, count_index.h
// SlotSource), then blocks, scatter and the labeled query over [begin, end) as above. The per-cell
// counters must be zero on entry (dauc_auc_eval_compact_part zeroes them; a build leaves them
// zero again).
struct SlotSource;
int counts_labeled_direct_slots(const SlotSource& src, float* pos, int64_t Mcap, const float* scores,
                                const void* labels, int label_dtype, int64_t begin, int64_t end,
                                unsigned long long* wins_ties, unsigned long long* nonfinite, unsigned* verdict,
                                void* workspace, size_t workspace_bytes, hipStream_t st, unsigned* check);

// the cell-slotted form of the same (round 6; the two-step evaluation's default): one count pass
// inserts every key into its cell's 8-word slot of `stab` (filled with +inf, and the packed byte
// counters and meta's skew word zeroed, by the compaction of step 1), then the query pass, which
// builds the block words from the byte counts itself: two launches instead of four.
int64_t slotted_cells(int64_t Mcap);
size_t slotted_table_bytes(int64_t Mcap);   // primary + secondary + tertiary regions (count_index.h)
size_t slotted_fill_bytes(int64_t Mcap);    // the +inf part: primary + secondary
int64_t slotted_cnt_words();                // the packed byte counters (words) the compaction zeroes
unsigned* slotted_meta_ptr(void* workspace, int64_t Mcap);
// the one-call evaluation's slotted form: the same insertion from the compacted positives `pos`
// (P on the device at *Mp, the top-bucket histogram ready), then the query pass (two launches
// instead of three after the compaction)
int counts_labeled_direct_slotted(const float* pos, const unsigned long long* Mp, int64_t Mcap, unsigned* stab,
                                  const float* scores, const void* labels, int label_dtype, int64_t begin,
                                  int64_t end, unsigned long long* wins_ties, unsigned long long* nonfinite,
                                  unsigned* verdict, void* workspace, size_t workspace_bytes, hipStream_t st,
                                  const unsigned* ready_hist);
int counts_labeled_slotted(const SlotSource& src, unsigned* stab, int64_t Mcap, const float* scores,
                           const void* labels, int label_dtype, int64_t begin, int64_t end,
                           unsigned long long* wins_ties, unsigned long long* nonfinite, unsigned* verdict,
                           void* workspace, size_t workspace_bytes, hipStream_t st, unsigned* check);
// dauc_auc_counts_sorted_labeled with the count index optional: the evaluation's sorted path runs
// only after the count index refused the table (verdict 2), and the sorted table has the same keys
// and the same plan, so it skips that build (count_index = false) and goes to the distinct-key
// index or the tree at once
int counts_sorted_labeled(const float* pos, int64_t P, const float* scores, const void* labels, int label_dtype,
                          int64_t begin, int64_t end, unsigned long long* wins_ties, unsigned long long* nonfinite,
                          void* workspace, size_t workspace_bytes, hipStream_t st, bool count_index);

}  // namespace dauc
