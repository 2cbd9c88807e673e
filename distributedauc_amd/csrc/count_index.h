// The count index of the positive table (auc_sort.hip builds it and counts the queries through
// it). gfx950 only.
//
// Keys: an fp32 score maps to a uint32 that orders like the float, with -0 and +0 on one key
// (fp32 equality semantics). The table's keys are split into CELLS by arithmetic on the key:
//   * the key's top 11 bits pick a top bucket t (sign, exponent, 2 mantissa bits); its n_t table
//     keys get C_t = ceil(n_t * R) cells that split its 2^21 low key values evenly
//     (cell = off_t + mulhi(low21 << 11, C_t)), R = cells per table key (<= 2: at most 1.5 keys
//     per cell on average, or the index is not used);
//   * l1[t] = {off_t, C_t} (2048 x 8 B); per block of 8 cells one word {the table keys before the
//     block (within its group of 256 blocks when built directly), the 8 cells' key counts as
//     nibbles}: 1 B per cell;
//   * rank_lo(x) = #(table keys in cells before x's cell) and cnt = the cell's count, so the cell's
//     keys are table[rank_lo, rank_lo + cnt) of the cell-ordered table: keys of earlier cells are
//     < x, of later cells > x, and only the cell's own keys need comparing.
// A table whose cells would hold more than 1.5 keys on average, or any cell 15 or more keys (a
// nibble), is not indexed (clustered / tie-heavy positives): the caller takes the sorted path.
#pragma once

#include "dauc_internal.h"

namespace dauc {

constexpr unsigned kPadKey = 0xffffffffu;  // above every finite score's key (max 0xff7fffff)

// the order-preserving key (-0 -> +0 by adding +0)
__device__ __forceinline__ unsigned key_fast(float f) {
    const unsigned u = __float_as_uint(f + 0.0f);
    return u ^ (static_cast<unsigned>(static_cast<int>(u) >> 31) | 0x80000000u);
}

constexpr int kCiTopBits = 11;
constexpr int kCiTop = 1 << kCiTopBits;
constexpr int kCiLowBits = 32 - kCiTopBits;
constexpr int kCiBlock = 8;                               // cells per block word
constexpr int kCiMaxBlocks = 18320;                       // 16 KB + 8 B per block + 384 B < 160 KB of LDS
constexpr int kCiMaxCells = kCiMaxBlocks * kCiBlock - 1;  // + the virtual cell past the last
// The slotted table (the two-step evaluation, round 6), for `cells` cells: a cell's keys by rank,
// 0-3 in its PRIMARY window (4 words at 4c), 4-7 in its SECONDARY window (4 (cells + 1) + 4c), 8-14
// in its TERTIARY run (8 (cells + 1) + 8c); the primary and secondary regions are +inf filled
// (windows past a cell's count read +inf) and primary slot `cells` is the all-+inf pad window. The
// primary region (16 B per cell, 2.3 MB at most) is the one nearly every query gathers from.
__host__ __device__ __forceinline__ unsigned slot_sec(unsigned cells, unsigned c) { return 4u * (cells + 1u) + 4u * c; }
__host__ __device__ __forceinline__ unsigned slot_ter(unsigned cells, unsigned c) { return 8u * (cells + 1u) + 8u * c; }
constexpr unsigned kSlotMaxKeys = 14;  // the nibble's bound: a cell of 15+ keys marks the table skewed
// meta words: [8] usable, [9] cells, [10] blocks, [11] skewed (or inconsistent: never use),
// [13] the slotted build's state was consumed by a query pass (a second step 2 without a new step 1)
constexpr int kCiOk = 8, kCiCells = 9, kCiBlocks = 10, kCiSkew = 11, kCiConsumed = 13;

__device__ __forceinline__ unsigned ci_cell(unsigned key, uint2 e) { return e.x + __umulhi(key << kCiTopBits, e.y); }

__device__ __forceinline__ bool count_index_in_use(const unsigned* __restrict__ meta) {
    return meta[kCiOk] != 0u && meta[kCiSkew] == 0u;
}

// rank_lo and cnt of cell c from its block word b (nibbles of the cells before c summed by SAD)
__device__ __forceinline__ void ci_decode(unsigned c, uint2 b, unsigned& rl, unsigned& cnt) {
    const unsigned sh = 4u * (c % kCiBlock);
    const unsigned below = __builtin_amdgcn_ubfe(b.y, 0u, sh);
    const unsigned bytes = (below & 0x0f0f0f0fu) + ((below >> 4) & 0x0f0f0f0fu);
    rl = b.x + __builtin_amdgcn_sad_u8(bytes, 0u, 0u);
    cnt = __builtin_amdgcn_ubfe(b.y, sh, 4u);
}

// the direct build: workgroup size, and groups of 256 block words whose prefixes the consumers
// add (group_prefix)
constexpr int kDirectThreads = 256;
constexpr int kDirectGroup = 256;
constexpr int kDirectMaxGroups = (kCiMaxBlocks + kDirectGroup - 1) / kDirectGroup;  // 72
static_assert(kDirectMaxGroups <= 2 * kWave, "group_prefix handles up to 128 groups");

// wave 0 of the calling workgroup: pre[g] = sum of grp[0 .. g) for g < kDirectMaxGroups
// (groups >= ng count nothing)
__device__ __forceinline__ void group_prefix(const unsigned* __restrict__ grp, int ng, unsigned* pre) {
    if (threadIdx.x >= kWave) return;
    const int lane = threadIdx.x;
    const unsigned v0 = lane < ng ? grp[lane] : 0u, v1 = lane + kWave < ng ? grp[lane + kWave] : 0u;
    unsigned i0 = v0, i1 = v1;
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
        const unsigned t0 = __shfl_up(i0, off, kWave), t1 = __shfl_up(i1, off, kWave);
        if (lane >= off) {
            i0 += t0;
            i1 += t1;
        }
    }
    const unsigned tot0 = __shfl(i0, kWave - 1, kWave);
    if (lane < kDirectMaxGroups) pre[lane] = i0 - v0;
    if (lane + kWave < kDirectMaxGroups) pre[lane + kWave] = tot0 + i1 - v1;
}

// inclusive scan over the threads of a workgroup of up to 1024 threads (wave shuffles, one
// barrier for the wave totals); op is min or +, v the thread's value
template <bool MIN>
__device__ __forceinline__ unsigned block_incl_scan1024(unsigned v, unsigned* wtot) {
    const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
    unsigned incl = v;
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
        const unsigned t = __shfl_up(incl, off, kWave);
        if (lane >= off) incl = MIN ? (t < incl ? t : incl) : incl + t;
    }
    if (lane == kWave - 1) wtot[wid] = incl;
    __syncthreads();
    unsigned before = MIN ? ~0u : 0u;
    for (int w = 0; w < wid; ++w) before = MIN ? (wtot[w] < before ? wtot[w] : before) : before + wtot[w];
    __syncthreads();
    return MIN ? (before < incl ? before : incl) : before + incl;
}

// One float4 slot's 4 labels as loaded (int8: ONE 32-bit word, unpacked where used)
template <typename LT>
struct LabelWords {
    LT v[4];
    __device__ __forceinline__ void load(const LT* p) {
        if constexpr (sizeof(LT) == 4) {
            const int4 c = *reinterpret_cast<const int4*>(p);
            v[0] = c.x;
            v[1] = c.y;
            v[2] = c.z;
            v[3] = c.w;
        } else {
            const longlong2 c0 = reinterpret_cast<const longlong2*>(p)[0];
            const longlong2 c1 = reinterpret_cast<const longlong2*>(p)[1];
            v[0] = c0.x;
            v[1] = c0.y;
            v[2] = c1.x;
            v[3] = c1.y;
        }
    }
    __device__ __forceinline__ void set_positive() { v[0] = v[1] = v[2] = v[3] = LT(1); }
    __device__ __forceinline__ bool not_positive(int q) const { return v[q] != LT(1); }
};
template <>
struct LabelWords<int8_t> {
    unsigned w;
    __device__ __forceinline__ void load(const int8_t* p) { w = *reinterpret_cast<const unsigned*>(p); }
    __device__ __forceinline__ void set_positive() { w = 0x01010101u; }
    __device__ __forceinline__ bool not_positive(int q) const { return ((w >> (8 * q)) & 0xffu) != 1u; }
};

// The two-step sharded evaluation's gathered slots (auc_eval.hip), read in place by the direct
// build (auc_sort.hip, direct_count_slots_kernel): slot r at slots + r * sbytes holds a header of
// u64 words {P_r, 0, #non-finite positives, #labels outside {-1, 1}, n}, the
// top-bucket histogram of its positives (kCiTop u32) at hist_off and at most cap scores at
// data_off. The build's first workgroup also writes the record of the part it serves.
struct SlotSource {
    const unsigned char* slots;
    size_t sbytes, hist_off, data_off;
    int parts, part;
    int64_t cap, n, qlen;              // qlen: the part's query range length (the check word)
    unsigned long long* wt;            // record words 0..2: zeroed
    unsigned long long* stats;         // record words 3..6: P, the check word, #non-finite, #other
    unsigned long long* verdict;       // record word 7: zeroed (the query pass writes it)
    unsigned long long* m_eff;         // the table size the scatter and the query read
};
constexpr int kMaxSlotParts = 1024;

// The count index built straight from the unsorted positives (auc_sort.hip, build_direct_index):
// device pointers into the caller's sort workspace.
struct DirectIndex {
    const unsigned* table;  // [M + 16] cell-ordered keys, +inf padded
    const uint2* l1;        // [kCiTop]
    const uint2* blk;       // [kCiMaxBlocks] block words (ranks within the block's group)
    const unsigned* grp;    // [kDirectMaxGroups] group totals
    unsigned* meta;         // [16] kCiOk, kCiCells, kCiBlocks, kCiSkew
};

}  // namespace dauc
