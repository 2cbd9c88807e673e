// Exact AUC counts of the labeled queries with no per-query gather: the RANGE-SLOT index.
//
// Reference: imagenet/main.py:79-81 -> sklearn roc_curve + auc (sklearn/metrics/_ranking.py:826-908):
// W = #{(positive, negative) : s_pos > s_neg}, T = #{s_pos == s_neg}. Every score whose label is
// not +1 is a query x against the positives' table: W += M - ub(x), T += ub(x) - lb(x), with
// lb / ub = #(table keys < x) / #(table keys <= x).
//
// Round 3's query pass (auc_sort.hip, query_ci_kernel) located every query in an LDS count index
// and gathered its cell's keys from the L2-resident table: per query a chain stream -> LDS -> LDS
// -> L2 gather, 81 M scattered L2 lines per 134 M queries, the vector-memory pipe 92 % busy. Here
// the queries are first SPLIT by the range of the table they fall in, so that the count pass of a
// range holds that range's whole index -- a 16-byte SLOT per cell -- in LDS, and a query costs one
// broadcast-friendly LDS read (its top bucket) and one slot read, never a global gather:
//
//   cells    the count index's cell map (count_index.h: top 11 key bits -> C_t cells splitting the
//            bucket's 2^21 low key values, cell = off_t + mulhi(low21 << 11, C_t)) with ~2 cells per
//            table key; RANGE g = cells [8192 g, 8192 (g + 1)) (128 KB of slots), at most 128;
//   slot     per cell {rank of the cell's first key within its range | count << 28, its first
//            three keys (+inf past the count)}: the cell's rank_lo, count and -- for the ~99.8 % of
//            cells of at most 3 keys -- every key, so the count is 3 + 3 compares; a cell of 4..15
//            keys reads the rest from the cell-ordered table, 16+ keys mark the table skewed;
//   build    top-bucket histogram, per-cell counts (the plan recomputed by every workgroup in LDS),
//            per-range scans that write the slots' ranks and counts, and a scatter that puts every
//            key into its cell's place in the table and into its cell's slot (ranks within a cell
//            from the counters counted back down; every index checked before it is used: an
//            inconsistency marks the table unusable = verdict 2, never an out-of-bounds store);
//   split    (persistent, one 1024-thread workgroup per CU) scores + labels streamed once; every
//            query's key -> top bucket (LDS) -> cell -> range; the tile's 16384 queries ranked
//            within their range by LDS counters per wave, staged in LDS grouped by range, and
//            written out contiguously (no atomics outside LDS, no cross-tile scan); per tile the
//            runs' offsets, per range the runs' lengths; the non-finite queries are counted;
//   prefix   (1 / range) the exclusive prefix of a range's run lengths over the tiles -> its
//            chunks of ~64 k queries;
//   count    (1 / chunk) the chunk's range's slots and the top-bucket table go to LDS; each query
//            of the chunk's runs: top bucket -> cell -> slot -> counts.
// Traffic per query: 5 B read + 4 B written (split) + 4 B read (count); the index (~2 cells x 16 B
// per table key) and the run tables are a few % of that.

// A MEASURED AND REJECTED alternative (round 4): compiled into the tuning build only
// (tuning/libdauc_tuning.so, -DDAUC_TUNING; selected by dauc_set_query_path(2)). At configs[4]
// (2^27 @ 0.1 %) the evaluation took 0.86 ms against 0.58 for the count index with gathers, at
// configs[3] 0.47 vs 0.15 ms (profiles/r04/slots/): the split alone (276 us) moves 9 B per query and
// the count pass waits on one dependent offset read per 200-250-query run. DESIGN §3.
#ifdef DAUC_TUNING

#include "count_index.h"

namespace dauc {
namespace {

constexpr int kSlCellBits = 13;
constexpr int kSlCells = 1 << kSlCellBits;              // cells per range: 8192 x 16 B = 128 KB of LDS
constexpr int kSlMaxRanges = 128;
constexpr int64_t kSlMaxCells = int64_t(kSlMaxRanges) * kSlCells;  // 1,048,576
constexpr int kSlBuildThreads = 256;
constexpr int kSlThreads = 1024;
constexpr int kSlWaves = kSlThreads / kWave;             // 16
constexpr int kSlSlots = 2;                              // float4 slots per thread per split tile
constexpr int kSlPer = 4 * kSlSlots;                     // queries per thread per tile
constexpr int kSlTile = kSlThreads * kSlPer;             // 8192 scores per tile
constexpr int64_t kSlChunk = 65536;                      // queries per count workgroup (whole runs)
constexpr int kSlOffStride = kSlMaxRanges + 1;           // per tile: the runs' starts and the tile's total
constexpr unsigned kSlRankMask = (1u << 28) - 1u;
// meta words: usable, cells, ranges, inconsistent / skewed (never use)
constexpr int kSmOk = 0, kSmCells = 1, kSmRanges = 2, kSmBad = 3;

__device__ __forceinline__ bool sl_usable(const unsigned* __restrict__ meta) {
    return meta[kSmOk] != 0u && meta[kSmBad] == 0u;
}

// wave 0: pre[g] = rtot[0] + ... + rtot[g - 1] for g < kSlMaxRanges (two ranges per lane)
__device__ __forceinline__ void range_prefix(const unsigned* __restrict__ rtot, int G, unsigned* pre) {
    static_assert(kSlMaxRanges == 2 * kWave, "two ranges per lane");
    if (threadIdx.x >= kWave) return;
    const int lane = threadIdx.x;
    const unsigned v0 = 2 * lane < G ? rtot[2 * lane] : 0u, v1 = 2 * lane + 1 < G ? rtot[2 * lane + 1] : 0u;
    unsigned incl = v0 + v1;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        const unsigned t = __shfl_up(incl, o, kWave);
        if (lane >= o) incl += t;
    }
    const unsigned before = incl - v0 - v1;
    pre[2 * lane] = before;
    pre[2 * lane + 1] = before + v0;
}

// ---- build ------------------------------------------------------------------------------------

// top-bucket histogram of the table (LDS, then one global add per used bucket; `hist` zeroed by
// the caller); also zeroes the per-cell counters the count pass adds into
__global__ __launch_bounds__(kSlBuildThreads) void sl_hist_kernel(const float* __restrict__ pos,
                                                                  const unsigned long long* __restrict__ Mp,
                                                                  unsigned* __restrict__ hist,
                                                                  unsigned* __restrict__ cnt) {
    const int64_t M = static_cast<int64_t>(*Mp);
    __shared__ unsigned h[kCiTop];
    for (int i = threadIdx.x; i < kCiTop; i += kSlBuildThreads) h[i] = 0u;
    __syncthreads();
    const int64_t gid = int64_t(blockIdx.x) * kSlBuildThreads + threadIdx.x, stride = int64_t(gridDim.x) * kSlBuildThreads;
    for (int64_t i = gid; i < kSlMaxCells / 4; i += stride) reinterpret_cast<uint4*>(cnt)[i] = uint4{0u, 0u, 0u, 0u};
    for (int64_t i = gid; i < M; i += stride) atomicAdd(&h[key_fast(pos[i]) >> kCiLowBits], 1u);
    __syncthreads();
    for (int i = threadIdx.x; i < kCiTop; i += kSlBuildThreads)
        if (h[i]) atomicAdd(hist + i, h[i]);
}

// The plan from the bucket sizes, computed by EVERY workgroup in LDS (8 buckets per thread): C_t =
// ceil(n_t * num / M) cells per used bucket, num = min(cells left after one per used bucket, 2 M),
// the first cell of every bucket (ascending). Workgroup 0 writes the plan and the meta words.
// Then every key's cell and the per-cell counts (a wave whose keys all fall in one cell adds once).
__global__ __launch_bounds__(kSlBuildThreads) void sl_count_kernel(const float* __restrict__ pos, int64_t mcap,
                                                                   const unsigned* __restrict__ hist,
                                                                   uint2* __restrict__ l1g,
                                                                   unsigned* __restrict__ meta,
                                                                   unsigned* __restrict__ cnt,
                                                                   unsigned* __restrict__ cell) {
    static_assert(kCiTop == 8 * kSlBuildThreads, "eight top buckets per thread");
    __shared__ uint2 l1[kCiTop];
    __shared__ unsigned wtot[kSlBuildThreads / kWave];
    __shared__ unsigned totals[3];
    const uint4 h0 = reinterpret_cast<const uint4*>(hist)[2 * threadIdx.x];
    const uint4 h1 = reinterpret_cast<const uint4*>(hist)[2 * threadIdx.x + 1];
    const unsigned n[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
    unsigned used = 0u, keys = 0u;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        used += n[j] != 0u;
        keys += n[j];
    }
    used = block_incl_scan1024<false>(used, wtot);
    if (threadIdx.x == kSlBuildThreads - 1) totals[0] = used;
    keys = block_incl_scan1024<false>(keys, wtot);  // M = the histogram's total (< 2^32: M <= n / 2)
    if (threadIdx.x == kSlBuildThreads - 1) totals[2] = keys;
    __syncthreads();
    const int64_t M = totals[2];
    const int64_t avail = kSlMaxCells - int64_t(totals[0]);
    const int64_t num = avail < 2 * M ? avail : 2 * M;
    unsigned C[8], csum = 0u;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        C[j] = n[j] ? static_cast<unsigned>((int64_t(n[j]) * num + M - 1) / M) : 0u;
        csum += C[j];
    }
    const unsigned incl = block_incl_scan1024<false>(csum, wtot);
    if (threadIdx.x == kSlBuildThreads - 1) totals[1] = incl;
    unsigned run = incl - csum;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        l1[8 * threadIdx.x + j] = uint2{run, C[j]};
        run += C[j];
    }
    __syncthreads();
    const unsigned total = totals[1];
    // usable: at most 1.5 keys per cell on average, every cell in a range, the table in the
    // workspace (M <= mcap) and its ranks in 28 bits
    const bool ok = num > 0 && 3 * num >= 2 * M && total <= static_cast<unsigned>(kSlMaxCells) && M <= mcap &&
                    M <= int64_t(kSlRankMask);
    if (blockIdx.x == 0) {
        for (int t = threadIdx.x; t < kCiTop; t += kSlBuildThreads) l1g[t] = l1[t];
        if (threadIdx.x == 0) {
            meta[kSmOk] = ok ? 1u : 0u;
            meta[kSmCells] = total;
            meta[kSmRanges] = (total + kSlCells - 1) / kSlCells;
            meta[kSmBad] = 0u;
        }
    }
    if (!ok) return;
    const int lane = threadIdx.x & (kWave - 1);
    for (int64_t i0 = int64_t(blockIdx.x) * kSlBuildThreads; i0 < M; i0 += int64_t(gridDim.x) * kSlBuildThreads) {
        const int64_t i = i0 + threadIdx.x;
        const bool live = i < M;
        unsigned c = 0u;
        if (live) {
            const unsigned x = key_fast(pos[i]);
            c = ci_cell(x, l1[x >> kCiLowBits]);
            cell[i] = c;  // the scatter's cell, so it does not walk pos -> key -> plan again
        }
        const unsigned long long act = __ballot(live);
        if (act == 0ull) continue;
        const int first = __ffsll(static_cast<long long>(act)) - 1;
        const unsigned cf = __shfl(c, first, kWave);
        if (__ballot(live && c == cf) == act) {
            if (lane == first) atomicAdd(cnt + cf, static_cast<unsigned>(__popcll(act)));
        } else if (live) {
            atomicAdd(cnt + c, 1u);
        }
    }
}

// One workgroup per range, 8 cells per thread: the exclusive scan of the range's cell counts; slot
// = {rank of the cell's first key within the range | count << 28, +inf, +inf, +inf} (the scatter
// fills in the keys) and rtot[g] = the range's keys. A count of 16 or more marks the table skewed.
__global__ __launch_bounds__(kSlThreads) void sl_scan_kernel(unsigned* __restrict__ meta,
                                                             const unsigned* __restrict__ cnt,
                                                             unsigned* __restrict__ rtot, uint4* __restrict__ slots) {
    static_assert(kSlCells == 8 * kSlThreads, "eight cells per thread");
    __shared__ unsigned wtot[kSlThreads / kWave];
    if (meta[kSmOk] == 0u || blockIdx.x >= meta[kSmRanges]) return;
    const int64_t c0 = int64_t(blockIdx.x) * kSlCells + 8 * threadIdx.x;
    const uint4 a = reinterpret_cast<const uint4*>(cnt + c0)[0], b = reinterpret_cast<const uint4*>(cnt + c0)[1];
    const unsigned v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    unsigned sum = 0u;
    bool skew = false;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        sum += v[j];
        skew |= v[j] >= 16u;
    }
    const unsigned incl = block_incl_scan1024<false>(sum, wtot);
    unsigned r = incl - sum;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        slots[c0 + j] = uint4{(r & kSlRankMask) | ((v[j] < 16u ? v[j] : 15u) << 28), kPadKey, kPadKey, kPadKey};
        r += v[j];
    }
    if (threadIdx.x == kSlThreads - 1) rtot[blockIdx.x] = incl;
    if (__ballot(skew) != 0ull && (threadIdx.x & (kWave - 1)) == 0) atomicOr(meta + kSmBad, 1u);
}

// Every key into its cell's place in the table (the range prefix + its slot's rank + its rank in
// the cell, from the counter counted back down) and, for the cell's first three, into its slot.
// Every index is checked before it is used: a failed check marks the table unusable (verdict 2).
// The table's tail is padded with +inf keys.
__global__ __launch_bounds__(kSlBuildThreads) void sl_scatter_kernel(const float* __restrict__ pos,
                                                                     const unsigned long long* __restrict__ Mp,
                                                                     unsigned* __restrict__ meta,
                                                                     const unsigned* __restrict__ rtot,
                                                                     unsigned* __restrict__ cnt,
                                                                     const unsigned* __restrict__ cell,
                                                                     uint4* __restrict__ slots,
                                                                     unsigned* __restrict__ table) {
    if (!sl_usable(meta)) return;
    const int64_t M = static_cast<int64_t>(*Mp);
    const unsigned ncells = meta[kSmCells];
    const int G = static_cast<int>(meta[kSmRanges]);
    __shared__ unsigned pre[kSlMaxRanges];
    range_prefix(rtot, G, pre);
    __syncthreads();
    const int64_t gid = int64_t(blockIdx.x) * kSlBuildThreads + threadIdx.x;
    if (gid < 16) table[M + gid] = kPadKey;
    bool bad = false;
    for (int64_t i = gid; i < M; i += int64_t(gridDim.x) * kSlBuildThreads) {
        const unsigned x = key_fast(pos[i]);
        const unsigned c = cell[i];
        if (c >= ncells) {
            bad = true;
            continue;
        }
        const unsigned sx = slots[c].x;
        const unsigned cc = sx >> 28;
        const unsigned left = atomicSub(cnt + c, 1u);  // the cell's slots not yet taken, before this one
        if (left == 0u || left > cc) {
            bad = true;
            continue;
        }
        const unsigned k = left - 1u;
        const int64_t p = int64_t(pre[c >> kSlCellBits]) + (sx & kSlRankMask) + k;
        if (p >= M) {
            bad = true;
            continue;
        }
        table[p] = x;
        if (k < 3u) reinterpret_cast<unsigned*>(slots + c)[1 + k] = x;
    }
    if (__ballot(bad) != 0ull && (threadIdx.x & (kWave - 1)) == 0) atomicOr(meta + kSmBad, 1u);
}

// ---- split ------------------------------------------------------------------------------------

// A workgroup barrier that orders LDS only: the split's global stores are never waited for
// inside the loop (a full __syncthreads() would wait for every store in flight, every tile).
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

template <typename LT>
struct SlTile {
    f32x4 f[kSlSlots];
    LabelWords<LT> l[kSlSlots];
};

// The tile's queries grouped by range into out[t * kSlTile, ...): every query takes its rank
// within its range from a returning LDS add on the range's counter (the order inside a run is
// immaterial: the counts are sums), one wave turns the counters into the runs' starts, the keys go
// to an LDS stage at their places and the stage is written out with 16-byte stores. off[t][g] = the
// start of range g's run in the tile (off[t][G] = the tile's query count: the runs' lengths are the
// differences; one contiguous row per tile).
// Software-pipelined: the next tile's loads are issued before this tile is processed, and the
// tile's barriers order LDS only, so the stores of a tile are never waited for.
template <typename LT, bool VEC>
__global__ __launch_bounds__(kSlThreads) void sl_split_kernel(
    const float* __restrict__ s, const LT* __restrict__ lab, int64_t a0, int64_t begin, int64_t end, int64_t vmax,
    int64_t ntiles, const uint2* __restrict__ l1g, const unsigned* __restrict__ meta,
    const unsigned long long* __restrict__ Mp, unsigned* __restrict__ out, unsigned* __restrict__ off,
    unsigned long long* __restrict__ nonfinite) {
    // no index: nothing to split, except that with no positives at all (M = 0) the queries are
    // still checked for finiteness (sklearn raises on a non-finite score before its one-class
    // warning, _ranking.py:868-869 / 1191)
    const bool count_only = !sl_usable(meta);
    if (count_only && *Mp != 0ull) return;
    const int G = count_only ? 0 : static_cast<int>(meta[kSmRanges]);
    __shared__ uint2 l1[kCiTop];
    __shared__ __attribute__((aligned(16))) unsigned stage[kSlTile];
    __shared__ unsigned hist[kSlMaxRanges];  // the tile's counts per range, then the runs' starts
    __shared__ unsigned tile_n;
    {
        constexpr int kL1Per = kCiTop / kSlThreads;
        uint2 a[kL1Per];
#pragma unroll
        for (int j = 0; j < kL1Per; ++j) a[j] = l1g[j * kSlThreads + threadIdx.x];
#pragma unroll
        for (int j = 0; j < kL1Per; ++j) l1[j * kSlThreads + threadIdx.x] = a[j];
        if (threadIdx.x < kSlMaxRanges) hist[threadIdx.x] = 0u;
    }
    const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
    unsigned nf = 0;
    // loads of tile t: unconditional (a slot past the last full one re-reads it and is fixed up
    // from scalars; a tile past the end re-reads the last tile), so they are all in flight together
    auto load = [&](SlTile<LT>& x, int64_t t) {
        if constexpr (VEC) {
            const int64_t tt = t < ntiles ? t : ntiles - 1;
#pragma unroll
            for (int j = 0; j < kSlSlots; ++j) {
                const int64_t idx = a0 + tt * kSlTile + (int64_t(j) * kSlThreads + threadIdx.x) * 4;
                const int64_t ic = idx <= vmax ? idx : vmax;
                x.f[j] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(s + ic));
                x.l[j].load(lab + ic);
            }
        }
    };
    auto step = [&](SlTile<LT>& cur, SlTile<LT>& nxt, int64_t t) {
        load(nxt, t + gridDim.x);
        const int64_t i0 = a0 + t * kSlTile;
        // the first and the last tile hold scores outside [begin, end) (and the tail slot, or every
        // slot of unaligned arrays, takes scalar loads); every other tile is wholly inside
        const bool edge = !VEC || i0 < begin || i0 + kSlTile > end;
        unsigned key[kSlPer], rk[kSlPer];  // rk: range | rank in the range << 8; 0xff = not a query
#pragma unroll
        for (int j = 0; j < kSlSlots; ++j) {
            const float f4[4] = {cur.f[j].x, cur.f[j].y, cur.f[j].z, cur.f[j].w};
            const int64_t idx = i0 + (int64_t(j) * kSlThreads + threadIdx.x) * 4;
            const bool scalar = !VEC || idx > vmax;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float v = f4[e];
                bool valid = cur.l[j].not_positive(e);
                if (edge) {
                    const bool in = idx + e >= begin && idx + e < end;
                    if (scalar) {
                        v = in ? s[idx + e] : 0.0f;
                        valid = in && lab[idx + e] != LT(1);
                    } else {
                        valid = valid && in;
                    }
                }
                nf += valid && !isfinite(v);
                key[4 * j + e] = key_fast(v);
                rk[4 * j + e] = valid ? 0u : 0xffu;
            }
        }
        if (count_only) return;
        // range of every query (top bucket in LDS -> cell -> range) and its rank in the range, in
        // two phases of 8 (every LDS read of a phase issued before any is used)
#pragma unroll
        for (int h = 0; h < kSlPer; h += 8) {
            uint2 e[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) e[k] = l1[key[h + k] >> kCiLowBits];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const unsigned g = ci_cell(key[h + k], e[k]) >> kSlCellBits;
                // a query past the last cell (above every table key: it adds nothing) is dropped
                if (rk[h + k] == 0u) rk[h + k] = g < static_cast<unsigned>(G) ? g : 0xffu;
            }
        }
#pragma unroll
        for (int k = 0; k < kSlPer; ++k)
            if (rk[k] != 0xffu) rk[k] |= atomicAdd(&hist[rk[k]], 1u) << 8;
        lds_barrier();
        if (wid == 0) {
            // ranges 2 lane and 2 lane + 1: the runs' starts (an exclusive scan of the counts)
            const unsigned c0 = hist[2 * lane], c1 = hist[2 * lane + 1];
            unsigned incl = c0 + c1;
#pragma unroll
            for (int o = 1; o < kWave; o <<= 1) {
                const unsigned u = __shfl_up(incl, o, kWave);
                if (lane >= o) incl += u;
            }
            const unsigned base0 = incl - c0 - c1, base1 = base0 + c0;
            hist[2 * lane] = base0;
            hist[2 * lane + 1] = base1;
            if (2 * lane < G) off[t * kSlOffStride + 2 * lane] = base0;
            if (2 * lane + 1 < G) off[t * kSlOffStride + 2 * lane + 1] = base1;
            if (lane == kWave - 1) {
                tile_n = incl;
                off[t * kSlOffStride + G] = incl;
            }
        }
        lds_barrier();
#pragma unroll
        for (int k = 0; k < kSlPer; ++k)
            if (rk[k] != 0xffu) stage[hist[rk[k] & 0xffu] + (rk[k] >> 8)] = key[k];
        lds_barrier();
        // the stage out (16-byte stores; the tile's slice of `out` has room for a whole tile), and
        // the counters cleared for the next tile
        const unsigned q = tile_n;
        unsigned* o = out + t * kSlTile;
#pragma unroll
        for (int j = 0; j < kSlSlots; ++j) {
            const unsigned i = (j * kSlThreads + threadIdx.x) * 4;
            if (i < q) *reinterpret_cast<uint4*>(o + i) = *reinterpret_cast<const uint4*>(stage + i);
        }
        if (threadIdx.x < kSlMaxRanges) hist[threadIdx.x] = 0u;
        lds_barrier();
    };
    SlTile<LT> A, B;
    load(A, blockIdx.x);
    __syncthreads();
    for (int64_t t = blockIdx.x; t < ntiles; t += 2 * int64_t(gridDim.x)) {
        step(A, B, t);
        if (t + gridDim.x >= ntiles) break;
        step(B, A, t + gridDim.x);
    }
    const unsigned long long nfw = wave_sum(static_cast<unsigned long long>(nf));
    if (lane == 0 && nfw && nonfinite) atomicAdd(nonfinite, nfw);
}

// ---- prefix -----------------------------------------------------------------------------------

// Per range g (one workgroup each): the total of its runs, tot[g], and where each of its count
// chunks starts. Chunk c = the tiles whose run of range g starts at a query index (in the range's
// concatenation of runs over the tiles) in [c K, (c + 1) K), K = kSlChunk: its first tile is the t
// with prefix(t - 1) < c K <= prefix(t). A run is shorter than K, so each tile starts at most one
// chunk; a chunk no tile starts is empty (its queries, if any, are in the last tiles, which the
// chunk before it runs to the end) and keeps cstart = ntiles.
__global__ __launch_bounds__(kSlThreads) void sl_prefix_kernel(const unsigned* __restrict__ off, int64_t ntiles,
                                                               int64_t cstride, const unsigned* __restrict__ meta,
                                                               unsigned* __restrict__ tot,
                                                               unsigned* __restrict__ cstart) {
    static_assert(kSlTile < kSlChunk, "a run never spans a chunk");
    if (!sl_usable(meta) || blockIdx.x >= meta[kSmRanges]) return;
    __shared__ unsigned wtot[kSlThreads / kWave];
    const int64_t g = blockIdx.x;
    auto l = [&](int64_t t) { return off[t * kSlOffStride + g + 1] - off[t * kSlOffStride + g]; };
    unsigned* cs = cstart + int64_t(blockIdx.x) * cstride;
    for (int64_t c = threadIdx.x; c < cstride; c += kSlThreads) cs[c] = static_cast<unsigned>(ntiles);
    const int64_t per = (ntiles + kSlThreads - 1) / kSlThreads;
    const int64_t t0 = int64_t(threadIdx.x) * per;
    const int64_t t1 = t0 + per < ntiles ? t0 + per : ntiles;
    unsigned sum = 0u;
    for (int64_t t = t0; t < t1; ++t) sum += l(t);
    const unsigned incl = block_incl_scan1024<false>(sum, wtot);  // its barriers order the fill above
    unsigned run = incl - sum;                                     // prefix(t0)
    for (int64_t t = t0; t < t1; ++t) {
        const unsigned lt = l(t);
        // prefix(t) = run: chunk c = floor(run / K) starts here when prefix(t - 1) < c K
        const uint64_t c = uint64_t(run) / kSlChunk;
        if (t == 0)
            cs[0] = 0u;
        else if (c * kSlChunk > uint64_t(run) - l(t - 1) && c < uint64_t(cstride))
            cs[c] = static_cast<unsigned>(t);
        run += lt;
    }
    if (threadIdx.x == kSlThreads - 1) tot[blockIdx.x] = incl;
}

// ---- count ------------------------------------------------------------------------------------

constexpr int kSlU = 8;  // queries per lane per block (one block = 512 queries of one run)

// Persistent: one 1024-thread workgroup per CU takes a contiguous span of the chunks (chunk = the
// tiles whose run of one range starts in one ~kSlChunk-query stretch of the range's queries;
// chunks ordered by range), so it loads a range's slots into LDS once per range it meets, not once
// per chunk. Per chunk, wave w takes the chunk's tiles w, w + 16, ...; a run is read in blocks of
// 512 queries (8 per lane, all loads in flight together) and the NEXT block's loads -- the same
// run's or the wave's next run's -- are issued before this block is counted. Workgroup 0 writes
// the verdict (1 = counted, 2 = the caller takes the sorted path) and any workgroup that meets an
// inconsistency makes it 2.
__global__ __launch_bounds__(kSlThreads) void sl_query_kernel(
    const unsigned* __restrict__ out, const unsigned* __restrict__ off, const unsigned* __restrict__ tot,
    const unsigned* __restrict__ cstart, int64_t ntiles, int64_t cstride, const unsigned* __restrict__ meta,
    const uint2* __restrict__ l1g, const uint4* __restrict__ slotsg, const unsigned* __restrict__ rtot,
    const unsigned* __restrict__ table, const unsigned long long* __restrict__ Mp,
    unsigned long long* __restrict__ wt, unsigned* __restrict__ verdict) {
    // the verdict word starts at 0 (the caller zeroes it): max-combined, so a workgroup's 2 holds
    // whichever workgroup writes last
    const bool usable = sl_usable(meta);
    if (blockIdx.x == 0 && threadIdx.x == 0 && verdict) atomicMax(verdict, usable ? 1u : 2u);
    if (!usable) return;
    const int G = static_cast<int>(meta[kSmRanges]);
    __shared__ uint2 l1[kCiTop];
    __shared__ uint4 sl[kSlCells];
    __shared__ unsigned chfirst[kSlMaxRanges + 1];  // the first chunk of every range (+ the total)
    __shared__ unsigned kfirst[kSlMaxRanges];       // the first table key of every range
    __shared__ unsigned long long red[2][kSlWaves];
    __shared__ int bad_any;
    const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
    if (wid == 0) {
        // ranges 2 lane and 2 lane + 1: chunks of range g = ceil(tot_g / K); the prefixes of the
        // chunk counts and of the ranges' key counts
        unsigned ch[2], kt[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int g = 2 * lane + h;
            const unsigned tr = g < G ? tot[g] : 0u;
            ch[h] = static_cast<unsigned>((uint64_t(tr) + kSlChunk - 1) / kSlChunk);
            kt[h] = g < G ? rtot[g] : 0u;
        }
        unsigned incl = ch[0] + ch[1], kincl = kt[0] + kt[1];
#pragma unroll
        for (int o = 1; o < kWave; o <<= 1) {
            const unsigned u = __shfl_up(incl, o, kWave), ku = __shfl_up(kincl, o, kWave);
            if (lane >= o) {
                incl += u;
                kincl += ku;
            }
        }
        chfirst[2 * lane] = incl - ch[0] - ch[1];
        chfirst[2 * lane + 1] = incl - ch[1];
        kfirst[2 * lane] = kincl - kt[0] - kt[1];
        kfirst[2 * lane + 1] = kincl - kt[1];
        if (lane == kWave - 1) chfirst[kSlMaxRanges] = incl;
        if (lane == 0) bad_any = 0;
    }
    __syncthreads();
    const unsigned J = chfirst[kSlMaxRanges];
    const unsigned jlo = static_cast<unsigned>(uint64_t(blockIdx.x) * J / gridDim.x);
    const unsigned jhi = static_cast<unsigned>(uint64_t(blockIdx.x + 1) * J / gridDim.x);
    const unsigned M = static_cast<unsigned>(*Mp);
    unsigned long long W = 0, T = 0;
    bool bad = false;
    int loaded = -1;
    for (unsigned jc = jlo; jc < jhi; ++jc) {
        // the chunk's range: the last g with chfirst[g] <= jc (ranges without chunks share their
        // first chunk index with the next range: the last such g has the chunk)
        int g = 0;
        for (int step = kSlMaxRanges / 2; step > 0; step >>= 1)
            if (g + step < G && chfirst[g + step] <= jc) g += step;
        const unsigned c = jc - chfirst[g];
        const unsigned nch = chfirst[g + 1 < G ? g + 1 : kSlMaxRanges] - chfirst[g];
        const unsigned* cs = cstart + int64_t(g) * cstride;
        const int64_t t0 = cs[c];
        const int64_t t1 = c + 1 < nch ? int64_t(cs[c + 1]) : ntiles;
        if (g != loaded) {
            __syncthreads();  // every wave is done with the previous range's slots
            // the tables into LDS with every load of a thread in flight before its first LDS store
            constexpr int kSlotPer = kSlCells / kSlThreads;  // 8
            constexpr int kL1Per = kCiTop / kSlThreads;      // 2
            uint4 sv[kSlotPer];
            const uint4* src = slotsg + int64_t(g) * kSlCells;
#pragma unroll
            for (int j = 0; j < kSlotPer; ++j) sv[j] = src[j * kSlThreads + threadIdx.x];
            if (loaded < 0) {
                uint2 lv[kL1Per];
#pragma unroll
                for (int j = 0; j < kL1Per; ++j) lv[j] = l1g[j * kSlThreads + threadIdx.x];
#pragma unroll
                for (int j = 0; j < kL1Per; ++j) l1[j * kSlThreads + threadIdx.x] = lv[j];
            }
#pragma unroll
            for (int j = 0; j < kSlotPer; ++j) sl[j * kSlThreads + threadIdx.x] = sv[j];
            __syncthreads();
            loaded = g;
        }
        const unsigned cell0 = static_cast<unsigned>(g) << kSlCellBits;
        const unsigned rb = kfirst[g];
        // the wave's runs: tiles t0 + wid, + 16, ...; (o, L) of a run = its start in the tile, length
        struct Run {
            int64_t t;
            unsigned o, L;
        };
        auto run_of = [&](int64_t t) -> Run {
            if (t >= t1) return Run{t, 0u, 0u};
            const unsigned o0 = off[t * kSlOffStride + g], o1 = off[t * kSlOffStride + g + 1];
            return Run{t, o0, o1 - o0};
        };
        auto load_block = [&](unsigned (&x)[kSlU], const Run& r, unsigned j0) {
            const unsigned* q = out + (r.t < t1 ? r.t : 0) * kSlTile + r.o;
#pragma unroll
            for (int u = 0; u < kSlU; ++u) {
                const unsigned j = j0 + u * kWave + lane;
                x[u] = q[j < r.L ? j : 0u];  // lanes past the run re-read its first query (counted out below)
            }
        };
        // The block's queries per lane in phases (every LDS read of a phase issued before any is
        // used): top bucket, slot, counts. A cell of 4+ keys (~0.2 % of the queries at 2 cells per
        // key) reads the rest of its keys from the table after the block.
        auto count_block = [&](const unsigned (&x)[kSlU], const Run& r, unsigned j0) {
            uint2 e[kSlU];
#pragma unroll
            for (int u = 0; u < kSlU; ++u) e[u] = l1[x[u] >> kCiLowBits];
            unsigned cr[kSlU];
            bool in[kSlU];
#pragma unroll
            for (int u = 0; u < kSlU; ++u) {
                cr[u] = ci_cell(x[u], e[u]) - cell0;  // the cell, relative to the range
                in[u] = j0 + u * kWave + lane < r.L;
                bad |= in[u] && cr[u] >= static_cast<unsigned>(kSlCells);
                in[u] = in[u] && cr[u] < static_cast<unsigned>(kSlCells);
            }
            uint4 v[kSlU];
#pragma unroll
            for (int u = 0; u < kSlU; ++u) v[u] = sl[in[u] ? cr[u] : 0u];
            unsigned w32 = 0u, t32 = 0u;
            bool longer = false;
#pragma unroll
            for (int u = 0; u < kSlU; ++u) {
                const unsigned xv = x[u];
                // keys past the cell's count are +inf in the slot: above every query's key
                const unsigned lt = (v[u].y < xv) + (v[u].z < xv) + (v[u].w < xv);
                const unsigned le = (v[u].y <= xv) + (v[u].z <= xv) + (v[u].w <= xv);
                const unsigned rl = rb + (v[u].x & kSlRankMask);
                w32 += in[u] ? M - (rl + le) : 0u;
                t32 += in[u] ? le - lt : 0u;
                longer |= in[u] && (v[u].x >> 28) > 3u;
            }
            if (longer) {
                // the keys past the first 3 of a longer cell (<= 15: a table with a cell of 16+
                // keys is not usable), from the cell-ordered table, counted one by one
#pragma unroll
                for (int u = 0; u < kSlU; ++u) {
                    const unsigned cc = v[u].x >> 28;
                    if (!(in[u] && cc > 3u)) continue;
                    const unsigned rl = rb + (v[u].x & kSlRankMask);
                    unsigned lt = 0u, le = 0u;
                    for (unsigned q = 3; q < cc; ++q) {
                        const unsigned k = table[rl + q < M ? rl + q : 0u];
                        lt += k < x[u];
                        le += k <= x[u];
                    }
                    bad |= rl + cc > M;
                    w32 -= le;
                    t32 += le - lt;
                }
            }
            W += w32;
            T += t32;
        };
        Run cur = run_of(t0 + wid), nxt = run_of(t0 + wid + kSlWaves);
        unsigned jb0 = 0;
        unsigned xa[kSlU], xb[kSlU];
        load_block(xa, cur, 0);
        // next block: the same run's, or the next run's first; returns false past the wave's last run
        auto advance = [&](Run& r, unsigned& j0, Run& n) -> bool {
            if (j0 + kSlU * kWave < r.L) {
                j0 += kSlU * kWave;
                return true;
            }
            r = n;
            j0 = 0;
            n = run_of(r.t + kSlWaves);
            return r.t < t1;
        };
        while (cur.t < t1) {
            // A: count xa (block jb0 of cur) while the next block loads into xb
            Run rb2 = cur, nb = nxt;
            unsigned jb = jb0;
            const bool more = advance(rb2, jb, nb);
            load_block(xb, rb2, jb);  // unconditional (past the end: a valid address, counted out)
            count_block(xa, cur, jb0);
            if (!more) break;
            cur = rb2;
            nxt = nb;
            jb0 = jb;
            // B: the same with the register sets swapped
            Run ra = cur, na = nxt;
            unsigned ja = jb0;
            const bool more2 = advance(ra, ja, na);
            load_block(xa, ra, ja);
            count_block(xb, cur, jb0);
            if (!more2) break;
            cur = ra;
            nxt = na;
            jb0 = ja;
        }
    }
    W = wave_sum(W);
    T = wave_sum(T);
    if (__ballot(bad) != 0ull && lane == 0) bad_any = 1;
    if (lane == 0) {
        red[0][wid] = W;
        red[1][wid] = T;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long bw = 0, bt = 0;
        for (int i = 0; i < kSlWaves; ++i) {
            bw += red[0][i];
            bt += red[1][i];
        }
        if (bw) atomicAdd(wt + 0, bw);
        if (bt) atomicAdd(wt + 1, bt);
        if (bad_any && verdict) atomicMax(verdict, 2u);
    }
}

int sl_cu_count() {
    static int cus = 0;
    if (cus == 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) {
            (void)hipGetLastError();
            cus = 256;
        }
    }
    return cus;
}

constexpr size_t al256(size_t b) { return (b + 255) / 256 * 256; }

int64_t sl_tiles(int64_t q) { return (q + 3 + kSlTile - 1) / kSlTile; }  // + up to 3 scores before begin
int64_t sl_cstride(int64_t nt) { return nt * kSlTile / kSlChunk + 2; }  // chunks of one range, at most

struct SlWs {
    unsigned* meta;    // [16]
    unsigned* hist;    // [kCiTop]
    uint2* l1;         // [kCiTop]
    unsigned* rtot;    // [kSlMaxRanges]
    unsigned* tot;     // [kSlMaxRanges]
    unsigned* cnt;     // [kSlMaxCells]
    uint4* slots;      // [kSlMaxCells]
    unsigned* cell;    // [mcap]
    unsigned* table;   // [mcap + 64]
    unsigned* off;     // [ntiles][kSlOffStride]
    unsigned* cstart;  // [kSlMaxRanges][cstride]
    unsigned* out;     // [ntiles][kSlTile]
};

// the bytes zeroed before every build: meta + hist (the workspace's first two regions)
constexpr size_t kSlZeroed = 256 + al256(size_t(kCiTop) * 4);

size_t sl_ws_bytes(int64_t mcap, int64_t q, SlWs* w, void* base) {
    const int64_t nt = sl_tiles(q < 1 ? 1 : q);
    char* p = static_cast<char*>(base);
    size_t at = 0;
    auto take = [&](size_t bytes) {
        char* r = p + at;
        at += al256(bytes);
        return r;
    };
    char* meta = take(256);
    char* hist = take(size_t(kCiTop) * 4);
    char* l1 = take(size_t(kCiTop) * 8);
    char* rtot = take(size_t(kSlMaxRanges) * 4);
    char* tot = take(size_t(kSlMaxRanges) * 4);
    char* cnt = take(size_t(kSlMaxCells) * 4);
    char* slots = take(size_t(kSlMaxCells) * 16);
    char* cell = take(size_t(mcap) * 4);
    char* table = take(size_t(mcap + 64) * 4);
    char* off = take(size_t(nt) * kSlOffStride * 4);
    char* cst = take(size_t(sl_cstride(nt)) * kSlMaxRanges * 4);
    char* out = take(size_t(nt) * kSlTile * 4);
    if (w != nullptr) {
        w->meta = reinterpret_cast<unsigned*>(meta);
        w->hist = reinterpret_cast<unsigned*>(hist);
        w->l1 = reinterpret_cast<uint2*>(l1);
        w->rtot = reinterpret_cast<unsigned*>(rtot);
        w->tot = reinterpret_cast<unsigned*>(tot);
        w->cnt = reinterpret_cast<unsigned*>(cnt);
        w->slots = reinterpret_cast<uint4*>(slots);
        w->cell = reinterpret_cast<unsigned*>(cell);
        w->table = reinterpret_cast<unsigned*>(table);
        w->off = reinterpret_cast<unsigned*>(off);
        w->cstart = reinterpret_cast<unsigned*>(cst);
        w->out = reinterpret_cast<unsigned*>(out);
    }
    return at;
}

template <typename LT>
int launch_sl_split(const float* s, const LT* lab, int64_t begin, int64_t end, const SlWs& w,
                    const unsigned long long* Mp, int64_t ntiles, unsigned long long* nonfinite, hipStream_t st) {
    const int64_t a0 = begin & ~int64_t(3);
    // the last float4 slot wholly inside [a0, end) (the vector loads are clamped to it)
    const int64_t vmax = end - a0 >= 4 ? a0 + ((end - a0) / 4 - 1) * 4 : -1;
    const size_t lsz = sizeof(LT), lal = 4 * lsz < 16 ? 4 * lsz : 16;
    const bool vec = vmax >= 0 && (reinterpret_cast<uintptr_t>(s) & 15u) == 0 &&
                     (reinterpret_cast<uintptr_t>(lab) & (lal - 1)) == 0;
    int64_t grid = int64_t(sl_cu_count());  // persistent: one 1024-thread workgroup per CU (LDS + registers)
    if (grid > ntiles) grid = ntiles;
    if (vec)
        hipLaunchKernelGGL((sl_split_kernel<LT, true>), dim3(static_cast<unsigned>(grid)), dim3(kSlThreads), 0, st, s,
                           lab, a0, begin, end, vmax, ntiles, w.l1, w.meta, Mp, w.out, w.off, nonfinite);
    else
        hipLaunchKernelGGL((sl_split_kernel<LT, false>), dim3(static_cast<unsigned>(grid)), dim3(kSlThreads), 0, st, s,
                           lab, a0, begin, end, vmax, ntiles, w.l1, w.meta, Mp, w.out, w.off, nonfinite);
    return launch_status();
}

}  // namespace

int g_query_path = 1;
int eval_query_path() { return g_query_path; }

int64_t slot_index_capacity(int64_t n) {
    // 1.5 keys per cell at most, and the smaller class of n scores (a table of n / 2 + 1 keys)
    const int64_t cap = 3 * kSlMaxCells / 2, half = n / 2 + 1;
    return half < cap ? half : cap;
}

size_t slot_index_workspace_size(int64_t n) {
    return sl_ws_bytes(slot_index_capacity(n < 1 ? 1 : n), n < 1 ? 1 : n, nullptr, nullptr);
}

int counts_slotted(const float* pos, const unsigned long long* Mp, int64_t mcap, const float* scores,
                   const void* labels, int label_dtype, int64_t begin, int64_t end, unsigned long long* wins_ties,
                   unsigned long long* nonfinite, unsigned* verdict, void* workspace, size_t workspace_bytes,
                   hipStream_t st) {
    const int64_t q = end - begin;
    if (q <= 0) return DAUC_OK;
    if (pos == nullptr || Mp == nullptr || mcap < 1 || workspace == nullptr ||
        (reinterpret_cast<uintptr_t>(workspace) & 255u) != 0 ||
        workspace_bytes < sl_ws_bytes(mcap, q, nullptr, nullptr))
        return DAUC_EINVAL;
    SlWs w{};
    sl_ws_bytes(mcap, q, &w, workspace);
    const int64_t ntiles = sl_tiles(q);
    hipError_t e;
    if ((e = hipMemsetAsync(w.meta, 0, kSlZeroed, st)) != hipSuccess) return -static_cast<int>(e);
    const auto blocks = [](int64_t keys, int64_t per, int64_t cap) {
        const int64_t b = (keys + per - 1) / per;
        return dim3(static_cast<unsigned>(b < 1 ? 1 : b < cap ? b : cap));
    };
    hipLaunchKernelGGL(sl_hist_kernel, blocks(mcap, kSlBuildThreads * 8, 256), dim3(kSlBuildThreads), 0, st, pos, Mp,
                       w.hist, w.cnt);
    hipLaunchKernelGGL(sl_count_kernel, blocks(mcap, kSlBuildThreads, 1024), dim3(kSlBuildThreads), 0, st, pos, mcap,
                       w.hist, w.l1, w.meta, w.cnt, w.cell);
    hipLaunchKernelGGL(sl_scan_kernel, dim3(kSlMaxRanges), dim3(kSlThreads), 0, st, w.meta, w.cnt, w.rtot, w.slots);
    hipLaunchKernelGGL(sl_scatter_kernel, blocks(mcap, kSlBuildThreads, 1024), dim3(kSlBuildThreads), 0, st, pos, Mp,
                       w.meta, w.rtot, w.cnt, w.cell, w.slots, w.table);
    int rc = launch_status();
    if (rc) return rc;
    switch (label_dtype) {
        case DAUC_LABEL_I8:
            rc = launch_sl_split(scores, static_cast<const int8_t*>(labels), begin, end, w, Mp, ntiles, nonfinite, st);
            break;
        case DAUC_LABEL_I32:
            rc = launch_sl_split(scores, static_cast<const int32_t*>(labels), begin, end, w, Mp, ntiles, nonfinite, st);
            break;
        case DAUC_LABEL_I64:
            rc = launch_sl_split(scores, static_cast<const int64_t*>(labels), begin, end, w, Mp, ntiles, nonfinite, st);
            break;
        default:
            return DAUC_EINVAL;
    }
    if (rc) return rc;
    hipLaunchKernelGGL(sl_prefix_kernel, dim3(kSlMaxRanges), dim3(kSlThreads), 0, st, w.off, ntiles, sl_cstride(ntiles),
                       w.meta, w.tot, w.cstart);
    // persistent: one workgroup per CU, each a contiguous span of the chunks
    hipLaunchKernelGGL(sl_query_kernel, dim3(static_cast<unsigned>(sl_cu_count())), dim3(kSlThreads), 0, st, w.out, w.off,
                       w.tot, w.cstart, ntiles, sl_cstride(ntiles), w.meta, w.l1, w.slots, w.rtot, w.table, Mp,
                       wins_ties, verdict);
    return launch_status();
}

}  // namespace dauc

extern "C" int dauc_set_query_path(int path) {
    if (path < 1 || path > 2) return DAUC_EINVAL;
    dauc::g_query_path = path;
    return DAUC_OK;
}

#endif  // DAUC_TUNING
