// Exact AUC counts of the labeled queries through the count index, with no per-query gather.
//
// Reference: imagenet/main.py:79-81 -> sklearn roc_curve + auc (sklearn/metrics/_ranking.py:826-908):
// W = #{(positive, negative) : s_pos > s_neg}, T = #{s_pos == s_neg}. Every score whose label is
// not +1 is a query x against the positives' table: W += M - ub(x), T += ub(x) - lb(x), with
// lb / ub = #(table keys < x) / #(table keys <= x).
//
// Round 3's query pass located every query in the count index (LDS) and gathered its cell's keys
// from the L2-resident table: 81 M scattered 16-byte gathers per 134 M queries kept the CU's
// texture path 92 % busy. Here the queries are first SPLIT by key range, so that the
// count pass for one range holds that range's whole table -- its cells' block words AND its keys --
// in LDS, and no query touches global memory but its own key:
//
//   plan   (1 workgroup)  ranges = runs of 8-cell blocks holding at most ~12.4 k table keys and
//                         1024 blocks each (<= 64 ranges); a range id per block; the verdict.
//   split  (persistent)   scores + labels streamed once; every query's key -> top bucket (LDS) ->
//                         cell -> block -> range id (LDS); the tile's queries are ranked within
//                         their range by wave ballots and stored grouped by range in the tile's own
//                         slice of the output (no atomics, no cross-tile scan); per tile the runs'
//                         offsets, per range the runs' lengths; the non-finite queries are counted.
//   prefix (1 / range)    per range, the exclusive prefix of its run lengths over the tiles.
//   count  (1 / chunk)    a workgroup takes ~64 k queries of one range (whole tiles' runs), loads
//                         the range's block words and keys into LDS, and counts every query from
//                         LDS: cell -> block word -> rank_lo, cnt -> at most 8 keys compared.
// Traffic: 5 B per score read + 4 B per query written + 4 B per query read (the index and the
// plan's tables are ~1 % of that); every kernel checks every index it dereferences and turns an
// inconsistency into verdict 2 (the caller's sorted path), never an out-of-bounds access.

#include "count_index.h"

namespace dauc {
namespace {

constexpr int kBkMaxRanges = 64;                      // range ids fit 6 ballot bits
constexpr int kBkRangeBlocks = 1024;                  // blocks (8 cells each) per range: 8 KB of block words
constexpr int kBkKeyStep = 12288;                     // a new range every 12288 table keys (see plan)
constexpr int kBkMaxBlockKeys = kCiBlock * 14;        // a block holds at most 8 cells x 14 keys
constexpr int kBkRangeKeys = kBkKeyStep + kBkMaxBlockKeys;  // keys per range, at most
constexpr int kBkKeysLds = kBkRangeKeys + 16;         // + alignment (3) + the 8-key window past the end
constexpr int kPlanThreads = 1024;
constexpr int kSplitThreads = 1024;
constexpr int kSplitSlots = 2;                        // float4 slots per thread per tile
constexpr int kSplitTile = kSplitThreads * kSplitSlots * 4;  // 8192 scores per tile
constexpr int kCountThreads = 1024;
constexpr int kCountWaves = kCountThreads / kWave;
constexpr int64_t kChunkQueries = 65536;              // queries per count workgroup (whole tiles' runs)
constexpr int kOffStride = kBkMaxRanges + 1;          // per tile: the runs' starts and the tile's total
// bmeta words
constexpr int kBmRanges = 0, kBmOk = 1;

static_assert(kCiMaxBlocks / kBkRangeBlocks + (3 * kCiMaxCells / 2) / kBkKeyStep + 2 <= kBkMaxRanges,
              "ranges of the largest index fit the range ids");

// ---- plan -------------------------------------------------------------------------------------

// Range boundaries: block b starts a range when b = 0, b is a multiple of kBkRangeBlocks, or
// floor(rank(b) / kBkKeyStep) differs from block b-1's (rank(b) = table keys before block b). So a
// range's keys are < kBkKeyStep + one block's keys, and it spans <= kBkRangeBlocks blocks.
// rinfo[g] = {first block, end block, first key rank, end key rank}; rid[b] = the range of block b.
// Writes the verdict: 1 = the index holds the table and the ranges are built, 2 = the caller must
// take the sorted path.
__global__ __launch_bounds__(kPlanThreads) void bucket_plan_kernel(DirectIndex ix,
                                                                   const unsigned long long* __restrict__ Mp,
                                                                   uint4* __restrict__ rinfo,
                                                                   unsigned char* __restrict__ rid,
                                                                   unsigned* __restrict__ bmeta,
                                                                   unsigned* __restrict__ verdict) {
    __shared__ unsigned pre[kDirectMaxGroups];
    __shared__ unsigned wtot[kPlanThreads / kWave];
    __shared__ unsigned total;
    const bool usable = count_index_in_use(ix.meta);
    const int nb = usable ? static_cast<int>(ix.meta[kCiBlocks]) : 0;
    const unsigned M = static_cast<unsigned>(*Mp);
    if (!usable || nb < 1 || nb > kCiMaxBlocks) {
        if (threadIdx.x == 0) {
            bmeta[kBmOk] = 0u;
            bmeta[kBmRanges] = 0u;
            if (verdict) *verdict = 2u;
        }
        return;
    }
    group_prefix(ix.grp, (nb + kDirectGroup - 1) / kDirectGroup, pre);
    __syncthreads();
    constexpr int kPer = (kCiMaxBlocks + kPlanThreads - 1) / kPlanThreads;  // 18
    const int b0 = static_cast<int>(threadIdx.x) * kPer;
    auto rank = [&](int b) -> unsigned { return b >= nb ? M : pre[b / kDirectGroup] + ix.blk[b].x; };
    unsigned r[kPer];
    unsigned flags = 0u;
    int nflag = 0;
    unsigned prev = b0 > 0 && b0 - 1 < nb ? rank(b0 - 1) : 0u;
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
        const int b = b0 + j;
        r[j] = b < nb ? rank(b) : M;
        const bool start = b < nb && (b == 0 || b % kBkRangeBlocks == 0 || r[j] / kBkKeyStep != prev / kBkKeyStep);
        flags |= start ? (1u << j) : 0u;
        nflag += start;
        prev = r[j];
    }
    const unsigned incl = block_incl_scan1024<false>(static_cast<unsigned>(nflag), wtot);
    if (threadIdx.x == kPlanThreads - 1) total = incl;
    __syncthreads();
    const unsigned G = total;
    const bool ok = G >= 1 && G <= static_cast<unsigned>(kBkMaxRanges);
    if (threadIdx.x == 0) {
        bmeta[kBmOk] = ok ? 1u : 0u;
        bmeta[kBmRanges] = ok ? G : 0u;
        if (verdict) *verdict = ok ? 1u : 2u;
    }
    if (!ok) return;
    unsigned g = incl - static_cast<unsigned>(nflag);  // ranges started before this thread's blocks
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
        const int b = b0 + j;
        if (b >= nb) break;
        if (flags & (1u << j)) {
            // component stores: range g's end words are written by the thread starting range g+1
            rinfo[g].x = static_cast<unsigned>(b);
            rinfo[g].z = r[j];
            if (g > 0) {
                rinfo[g - 1].y = static_cast<unsigned>(b);
                rinfo[g - 1].w = r[j];
            }
            if (g == G - 1) {
                rinfo[g].y = static_cast<unsigned>(nb);
                rinfo[g].w = M;
            }
            ++g;
        }
        rid[b] = static_cast<unsigned char>(g - 1);
    }
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
struct SplitTile {
    f32x4 f[kSplitSlots];
    LabelWords<LT> l[kSplitSlots];
};

// The tile's queries grouped by range into out[t * kSplitTile, ...) by an LDS counting sort: a
// histogram of the tile's range ids (no-return LDS atomics), its exclusive scan (one wave), and a
// cursor per range that every query bumps for its slot (returning LDS atomics; the order inside a
// run is immaterial, the counts are sums). off[t][r] = the start of range r's run in the tile
// (r <= G: off[t][G] = the tile's query count); len[r][t] = range r's run length. Software-
// pipelined: the next tile's loads are issued before this tile is processed, the LDS state
// alternates between two buffers, and the tile's barriers order LDS only, so the stores of a tile
// are never waited for.
template <typename LT, bool VEC>
__global__ __launch_bounds__(kSplitThreads) void bucket_split_kernel(
    const float* __restrict__ s, const LT* __restrict__ lab, int64_t a0, int64_t begin, int64_t end, int64_t vmax,
    int64_t ntiles, const uint2* __restrict__ l1g, const unsigned char* __restrict__ ridg,
    const unsigned* __restrict__ bmeta, const unsigned long long* __restrict__ Mp, unsigned* __restrict__ out,
    unsigned* __restrict__ off, unsigned* __restrict__ len, unsigned long long* __restrict__ nonfinite) {
    // no index: nothing to split, except that with no positives at all (M = 0) the queries are
    // still checked for finiteness (sklearn raises on a non-finite score before its one-class
    // warning, _ranking.py:868-869 / 1191)
    const bool count_only = bmeta[kBmOk] == 0u;
    if (count_only && *Mp != 0ull) return;
    const unsigned G = bmeta[kBmRanges];
    constexpr int kRidWords = (kCiMaxBlocks + 3) / 4;
    __shared__ uint2 l1[kCiTop];
    __shared__ unsigned rid4[kRidWords];
    __shared__ unsigned hist[2][kBkMaxRanges];
    __shared__ unsigned cursor[2][kBkMaxRanges];
    {
        // every load of a thread in flight before its first LDS store
        constexpr int kL1Per = kCiTop / kSplitThreads, kRidPer = (kRidWords + kSplitThreads - 1) / kSplitThreads;
        uint2 a[kL1Per];
        unsigned r[kRidPer];
#pragma unroll
        for (int j = 0; j < kL1Per; ++j) a[j] = l1g[j * kSplitThreads + threadIdx.x];
#pragma unroll
        for (int j = 0; j < kRidPer; ++j) {
            const int i = j * kSplitThreads + threadIdx.x;
            r[j] = i < kRidWords ? reinterpret_cast<const unsigned*>(ridg)[i] : 0u;
        }
#pragma unroll
        for (int j = 0; j < kL1Per; ++j) l1[j * kSplitThreads + threadIdx.x] = a[j];
#pragma unroll
        for (int j = 0; j < kRidPer; ++j) {
            const int i = j * kSplitThreads + threadIdx.x;
            if (i < kRidWords) rid4[i] = r[j];
        }
        if (threadIdx.x < 2 * kBkMaxRanges) (&hist[0][0])[threadIdx.x] = 0u;
    }
    const unsigned char* rid = reinterpret_cast<const unsigned char*>(rid4);
    const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
    unsigned nf = 0;
    // loads of tile t: unconditional (a slot past the last full one re-reads it and is fixed up
    // from scalars; a tile past the end re-reads the last tile), so they are all in flight together
    auto load = [&](SplitTile<LT>& x, int64_t t) {
        if constexpr (VEC) {
            const int64_t tt = t < ntiles ? t : ntiles - 1;
#pragma unroll
            for (int j = 0; j < kSplitSlots; ++j) {
                const int64_t idx = a0 + tt * kSplitTile + (int64_t(j) * kSplitThreads + threadIdx.x) * 4;
                const int64_t ic = idx <= vmax ? idx : vmax;
                x.f[j] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(s + ic));
                x.l[j].load(lab + ic);
            }
        }
    };
    constexpr int K = kSplitSlots * 4;
    // one tile: sort `cur` (tile t) while `nxt`'s loads (tile t + grid) are in flight; called
    // alternately on two register sets, so no loaded register is copied at a back-edge
    auto step = [&](SplitTile<LT>& cur, SplitTile<LT>& nxt, int64_t t, int p) {
        load(nxt, t + gridDim.x);
        const int64_t i0 = a0 + t * kSplitTile;
        unsigned key[K], d[K];
        bool valid[K];
        float v[K];
#pragma unroll
        for (int j = 0; j < kSplitSlots; ++j) {
            v[4 * j] = cur.f[j].x;
            v[4 * j + 1] = cur.f[j].y;
            v[4 * j + 2] = cur.f[j].z;
            v[4 * j + 3] = cur.f[j].w;
#pragma unroll
            for (int e = 0; e < 4; ++e) valid[4 * j + e] = cur.l[j].not_positive(e);
        }
        // the first and the last tile hold scores outside [begin, end) (and the tail slot, or every
        // slot of unaligned arrays, takes scalar loads); every other tile is wholly inside
        const bool edge = !VEC || i0 < begin || i0 + kSplitTile > end;
        if (edge) {
#pragma unroll
            for (int j = 0; j < kSplitSlots; ++j) {
                const int64_t idx = i0 + (int64_t(j) * kSplitThreads + threadIdx.x) * 4;
                const bool scalar = !VEC || idx > vmax;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const bool in = idx + e >= begin && idx + e < end;
                    if (scalar) {
                        v[4 * j + e] = in ? s[idx + e] : 0.0f;
                        valid[4 * j + e] = in && lab[idx + e] != LT(1);
                    } else {
                        valid[4 * j + e] = valid[4 * j + e] && in;
                    }
                }
            }
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            nf += valid[k] && !isfinite(v[k]);
            key[k] = key_fast(v[k]);
        }
        if (count_only) return;
        // range id of every query: top bucket -> cell -> block -> range (LDS); the histogram
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const unsigned c = ci_cell(key[k], l1[key[k] >> kCiLowBits]);
            const unsigned b = c / kCiBlock;
            d[k] = rid[b < static_cast<unsigned>(kCiMaxBlocks) ? b : 0u];
        }
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (valid[k]) atomicAdd(&hist[p][d[k]], 1u);
        lds_barrier();
        if (wid == 0) {
            // range r = lane: its start in the tile (exclusive scan); the histogram is cleared for
            // the tile after next
            const unsigned c = hist[p][lane];
            unsigned incl = c;
#pragma unroll
            for (int o = 1; o < kWave; o <<= 1) {
                const unsigned u = __shfl_up(incl, o, kWave);
                if (lane >= o) incl += u;
            }
            const unsigned start = incl - c;
            cursor[p][lane] = start;
            hist[p][lane] = 0u;
            if (static_cast<unsigned>(lane) < G) {
                off[t * kOffStride + lane] = start;
                len[int64_t(lane) * ntiles + t] = c;
            }
            if (static_cast<unsigned>(lane) == G - 1u) off[t * kOffStride + G] = incl;
        }
        lds_barrier();
        unsigned* o = out + t * kSplitTile;
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (valid[k]) o[atomicAdd(&cursor[p][d[k]], 1u)] = key[k];
    };
    SplitTile<LT> A, B;
    load(A, blockIdx.x);
    __syncthreads();
    for (int64_t t = blockIdx.x; t < ntiles; t += 2 * int64_t(gridDim.x)) {
        step(A, B, t, 0);
        if (t + gridDim.x >= ntiles) break;
        step(B, A, t + gridDim.x, 1);
    }
    const unsigned long long nfw = wave_sum(static_cast<unsigned long long>(nf));
    if (lane == 0 && nfw && nonfinite) atomicAdd(nonfinite, nfw);
}

// ---- prefix -----------------------------------------------------------------------------------

// Per range r (one workgroup each): the total of its runs, tot[r], and where each of its count
// chunks starts. Chunk c = the tiles whose run of range r starts at a query index (in the range's
// concatenation of runs over the tiles) in [c K, (c + 1) K), K = kChunkQueries: its first tile is
// the t with prefix(t - 1) < c K <= prefix(t) (prefix = the exclusive prefix of the run lengths).
// A run is shorter than K, so each tile starts at most one chunk; a chunk no tile starts is empty
// (its queries, if any, are in the last tiles, which the chunk before it runs to the end) and
// keeps cstart = ntiles.
__global__ __launch_bounds__(kPlanThreads) void bucket_prefix_kernel(const unsigned* __restrict__ len,
                                                                     int64_t ntiles, int64_t cstride,
                                                                     const unsigned* __restrict__ bmeta,
                                                                     unsigned* __restrict__ tot,
                                                                     unsigned* __restrict__ cstart) {
    static_assert(kSplitTile < kChunkQueries, "a run never spans a chunk");
    if (bmeta[kBmOk] == 0u || blockIdx.x >= bmeta[kBmRanges]) return;
    __shared__ unsigned wtot[kPlanThreads / kWave];
    const unsigned* l = len + int64_t(blockIdx.x) * ntiles;
    unsigned* cs = cstart + int64_t(blockIdx.x) * cstride;
    for (int64_t c = threadIdx.x; c < cstride; c += kPlanThreads) cs[c] = static_cast<unsigned>(ntiles);
    const int64_t per = (ntiles + kPlanThreads - 1) / kPlanThreads;
    const int64_t t0 = int64_t(threadIdx.x) * per;
    const int64_t t1 = t0 + per < ntiles ? t0 + per : ntiles;
    unsigned sum = 0u;
    for (int64_t t = t0; t < t1; ++t) sum += l[t];
    const unsigned incl = block_incl_scan1024<false>(sum, wtot);  // its barriers order the fill above
    unsigned run = incl - sum;                                     // prefix(t0)
    for (int64_t t = t0; t < t1; ++t) {
        const unsigned lt = l[t];
        // prefix(t) = run: chunk c = floor(run / K) starts here when prefix(t - 1) < c K
        const uint64_t c = uint64_t(run) / kChunkQueries;
        if (t == 0)
            cs[0] = 0u;
        else if (c * kChunkQueries > uint64_t(run) - l[t - 1] && c < uint64_t(cstride))
            cs[c] = static_cast<unsigned>(t);
        run += lt;
    }
    if (threadIdx.x == kPlanThreads - 1) tot[blockIdx.x] = incl;
}

constexpr int kCountU = 4;  // queries per lane per block (one block = 256 queries of one run)

// One workgroup per chunk of ~kChunkQueries queries of one range (the tiles whose run of that
// range starts in the chunk). The range's block words (global ranks) and keys go to LDS; wave w
// takes the chunk's tiles w, w + 16, ...; a run is read in blocks of 512 queries (8 per lane, all
// loads in flight together) and the NEXT block's loads -- the same run's or the wave's next run's
// -- are issued before this block is counted.
__global__ __launch_bounds__(kCountThreads) void bucket_count_kernel(
    const unsigned* __restrict__ out, const unsigned* __restrict__ off, const unsigned* __restrict__ tot,
    const unsigned* __restrict__ cstart, int64_t ntiles, int64_t cstride, const uint4* __restrict__ rinfo,
    const unsigned* __restrict__ bmeta, DirectIndex ix,
    const unsigned long long* __restrict__ Mp, unsigned long long* __restrict__ wt, unsigned* __restrict__ verdict) {
    if (bmeta[kBmOk] == 0u) return;
    const unsigned G = bmeta[kBmRanges];
    __shared__ uint2 l1[kCiTop];
    __shared__ uint2 blk[kBkRangeBlocks];
    __shared__ __attribute__((aligned(16))) unsigned keys[kBkKeysLds];
    __shared__ unsigned pre[kDirectMaxGroups];
    __shared__ int64_t job[3];  // range, first tile, end tile (range < 0: no chunk)
    __shared__ unsigned long long red[2][kCountWaves];
    __shared__ int bad_any;
    const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
    if (wid == 0) {
        // which range and chunk: range r = lane; chunks of range r = ceil(total_r / kChunkQueries)
        const unsigned tr = static_cast<unsigned>(lane) < G ? tot[lane] : 0u;
        const unsigned ch = static_cast<unsigned>((uint64_t(tr) + kChunkQueries - 1) / kChunkQueries);
        unsigned incl = ch;
#pragma unroll
        for (int o = 1; o < kWave; o <<= 1) {
            const unsigned u = __shfl_up(incl, o, kWave);
            if (lane >= o) incl += u;
        }
        const unsigned b = blockIdx.x;
        const bool mine = b >= incl - ch && b < incl;
        if (lane == 0) {
            job[0] = -1;
            bad_any = 0;
        }
        if (mine) {
            const unsigned c = b - (incl - ch);
            const unsigned* cs = cstart + int64_t(lane) * cstride;
            job[0] = lane;
            job[1] = cs[c];
            job[2] = c + 1 < ch ? cs[c + 1] : ntiles;
        }
    }
    __syncthreads();
    const int64_t g = job[0];
    if (g < 0) return;
    const uint4 ri = rinfo[g];
    const unsigned nbr = ri.y - ri.x;  // blocks of the range (<= kBkRangeBlocks by the plan)
    const unsigned k4 = ri.z & ~3u, k0 = k4;  // LDS key 0 = table key k4
    const unsigned nkeys = ri.w + 8u - k4;     // the range's keys, aligned down, + 8 past them (+inf padded)
    const unsigned M = static_cast<unsigned>(*Mp);
    if (nbr > static_cast<unsigned>(kBkRangeBlocks) || nkeys > static_cast<unsigned>(kBkKeysLds) || ri.w > M) {
        if (threadIdx.x == 0 && verdict) *verdict = 2u;  // an inconsistent plan: the sorted path
        return;
    }
    group_prefix(ix.grp, (static_cast<int>(ix.meta[kCiBlocks]) + kDirectGroup - 1) / kDirectGroup, pre);
    {
        // the tables into LDS with every load of a thread in flight before its first LDS store
        constexpr int kKeysPer = (kBkKeysLds + kCountThreads - 1) / kCountThreads;  // 13
        constexpr int kL1Per = kCiTop / kCountThreads;                              // 2
        unsigned kv[kKeysPer];
        uint2 lv[kL1Per];
#pragma unroll
        for (int j = 0; j < kKeysPer; ++j) {
            const unsigned i = j * kCountThreads + threadIdx.x;
            kv[j] = i < nkeys ? ix.table[k4 + i] : kPadKey;  // the table has M + 16 words
        }
#pragma unroll
        for (int j = 0; j < kL1Per; ++j) lv[j] = ix.l1[j * kCountThreads + threadIdx.x];
        const uint2 bv = threadIdx.x < nbr ? ix.blk[ri.x + threadIdx.x] : uint2{0u, 0u};
#pragma unroll
        for (int j = 0; j < kKeysPer; ++j) {
            const unsigned i = j * kCountThreads + threadIdx.x;
            if (i < nkeys) keys[i] = kv[j];
        }
#pragma unroll
        for (int j = 0; j < kL1Per; ++j) l1[j * kCountThreads + threadIdx.x] = lv[j];
        __syncthreads();  // pre[]
        static_assert(kBkRangeBlocks <= kCountThreads, "one block word per thread");
        if (threadIdx.x < nbr) blk[threadIdx.x] = uint2{bv.x + pre[(ri.x + threadIdx.x) / kDirectGroup], bv.y};
    }
    __syncthreads();
    const int64_t t1 = job[2];
    const unsigned cell0 = ri.x * kCiBlock, ncell = nbr * kCiBlock;
    unsigned long long W = 0, T = 0;
    bool bad = false;
    // the wave's runs: tiles t0 + wid, + 16, ...; (o, L) of a run = its start in the tile, length
    struct Run {
        int64_t t;
        unsigned o, L;
    };
    auto run_of = [&](int64_t t) -> Run {
        if (t >= t1) return Run{t, 0u, 0u};
        const unsigned o0 = off[t * kOffStride + g], o1 = off[t * kOffStride + g + 1];
        return Run{t, o0, o1 - o0};
    };
    auto load_block = [&](unsigned (&x)[kCountU], const Run& r, unsigned j0) {
        const unsigned* q = out + (r.t < t1 ? r.t : 0) * kSplitTile + r.o;
#pragma unroll
        for (int u = 0; u < kCountU; ++u) {
            const unsigned j = j0 + u * kWave + lane;
            x[u] = q[j < r.L ? j : 0u];  // lanes past the run re-read its first query (counted out below)
        }
    };
    // The block's kCountU queries per lane, in phases (every LDS read of a phase issued before any
    // is used) and predicated instead of branched: top bucket, block word, the cell's first 4 keys
    // (read whatever the count: no branch), the counts. A cell of 5+ keys (~0.2 % of the queries
    // at 1.1 cells per key) is recounted key by key after the block.
    auto count_block = [&](const unsigned (&x)[kCountU], const Run& r, unsigned j0) {
#if defined(DAUC_BK_X) && DAUC_BK_X == 3
        for (int u = 0; u < kCountU; ++u) W += (j0 + u * kWave + lane < r.L) ? x[u] : 0u;
        return;
#endif
        uint2 e[kCountU], b[kCountU];
        unsigned cr[kCountU];
        bool in[kCountU];
#pragma unroll
        for (int u = 0; u < kCountU; ++u) e[u] = l1[x[u] >> kCiLowBits];
#pragma unroll
        for (int u = 0; u < kCountU; ++u) {
            cr[u] = ci_cell(x[u], e[u]) - cell0;  // the cell, relative to the range
            in[u] = j0 + u * kWave + lane < r.L;
            bad |= in[u] && cr[u] >= ncell;
            in[u] = in[u] && cr[u] < ncell;
            b[u] = blk[in[u] ? cr[u] / kCiBlock : 0u];
        }
        unsigned rl[kCountU], cnt[kCountU], li[kCountU];
#pragma unroll
        for (int u = 0; u < kCountU; ++u) {
            ci_decode(cr[u], b[u], rl[u], cnt[u]);  // cell0 is a multiple of 8: the same nibble
            li[u] = rl[u] - k0;                      // the cell's first key in LDS
            const bool fits = li[u] + cnt[u] <= nkeys;
            bad |= in[u] && !fits;
            in[u] = in[u] && fits;
            if (!in[u]) li[u] = 0u;
        }
        unsigned k[kCountU][4];
#pragma unroll
        for (int u = 0; u < kCountU; ++u) {
#pragma unroll
#if defined(DAUC_BK_X) && DAUC_BK_X == 2
            for (int q = 0; q < 4; ++q) k[u][q] = li[u] + q;
#else
            for (int q = 0; q < 4; ++q) k[u][q] = keys[li[u] + q];  // li + 3 < nkeys: 8 keys past the range
#endif
        }
        unsigned w32 = 0u, t32 = 0u;
        bool longer = false;
#pragma unroll
        for (int u = 0; u < kCountU; ++u) {
            const unsigned c = cnt[u], xv = x[u];
            const unsigned lt = (c > 0u && k[u][0] < xv) + (c > 1u && k[u][1] < xv) + (c > 2u && k[u][2] < xv) +
                                (c > 3u && k[u][3] < xv);
            const unsigned le = (c > 0u && k[u][0] <= xv) + (c > 1u && k[u][1] <= xv) + (c > 2u && k[u][2] <= xv) +
                                (c > 3u && k[u][3] <= xv);
            w32 += in[u] ? M - (rl[u] + le) : 0u;
            t32 += in[u] ? le - lt : 0u;
            longer |= in[u] && c > 4u;
        }
#if defined(DAUC_BK_X) && DAUC_BK_X == 1
        longer = false;
#endif
        if (longer) {
            // the keys past the first 4 of a longer cell (<= 14 keys: a nibble); the table is
            // ordered by cell only, so they are counted one by one
#pragma unroll
            for (int u = 0; u < kCountU; ++u) {
                if (!(in[u] && cnt[u] > 4u)) continue;
                unsigned lt = 0u, le = 0u;
                for (unsigned q = 4; q < cnt[u]; ++q) {
                    const unsigned v = keys[li[u] + q];
                    lt += v < x[u];
                    le += v <= x[u];
                }
                w32 -= le;
                t32 += le - lt;
            }
        }
        W += w32;
        T += t32;
    };
    Run cur = run_of(job[1] + wid), nxt = run_of(job[1] + wid + kCountWaves);
    unsigned jc = 0;
    unsigned xa[kCountU], xb[kCountU];
    load_block(xa, cur, 0);
    // next block: the same run's, or the next run's first; returns false past the wave's last run
    auto advance = [&](Run& r, unsigned& j0, Run& n) -> bool {
        if (j0 + kCountU * kWave < r.L) {
            j0 += kCountU * kWave;
            return true;
        }
        r = n;
        j0 = 0;
        n = run_of(r.t + kCountWaves);
        return r.t < t1;
    };
    while (cur.t < t1) {
        // A: count xa (block jc of cur) while the next block loads into xb
        Run rb = cur, nb = nxt;
        unsigned jb = jc;
        const bool more = advance(rb, jb, nb);
        load_block(xb, rb, jb);  // unconditional (past the end: a valid address, counted out)
        count_block(xa, cur, jc);
        if (!more) break;
        cur = rb;
        nxt = nb;
        jc = jb;
        // B: the same with the register sets swapped
        Run ra = cur, na = nxt;
        unsigned ja = jc;
        const bool more2 = advance(ra, ja, na);
        load_block(xa, ra, ja);
        count_block(xb, cur, jc);
        if (!more2) break;
        cur = ra;
        nxt = na;
        jc = ja;
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
        for (int i = 0; i < kCountWaves; ++i) {
            bw += red[0][i];
            bt += red[1][i];
        }
        if (bw) atomicAdd(wt + 0, bw);
        if (bt) atomicAdd(wt + 1, bt);
        if (bad_any && verdict) *verdict = 2u;
    }
}

int cu_count() {
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

inline size_t al256(size_t b) { return (b + 255) / 256 * 256; }

int64_t tiles_of(int64_t q) { return (q + 3 + kSplitTile - 1) / kSplitTile; }  // + up to 3 scores before begin
int64_t cstride_of(int64_t nt) { return nt * kSplitTile / kChunkQueries + 2; }  // chunks of one range, at most

struct BucketWs {
    unsigned* out;
    unsigned* off;
    unsigned* len;
    unsigned* tot;
    unsigned* cstart;
    uint4* rinfo;
    unsigned char* rid;
    unsigned* bmeta;
};

BucketWs bucket_ws(void* ws, int64_t q) {
    const int64_t nt = tiles_of(q);
    char* p = static_cast<char*>(ws);
    BucketWs w;
    w.bmeta = reinterpret_cast<unsigned*>(p);
    p += 256;
    w.rinfo = reinterpret_cast<uint4*>(p);
    p += al256(size_t(kBkMaxRanges) * 16);
    w.rid = reinterpret_cast<unsigned char*>(p);
    p += al256(size_t(kCiMaxBlocks) + 4);
    w.off = reinterpret_cast<unsigned*>(p);
    p += al256(size_t(nt) * kOffStride * 4);
    w.len = reinterpret_cast<unsigned*>(p);
    p += al256(size_t(nt) * kBkMaxRanges * 4);
    w.tot = reinterpret_cast<unsigned*>(p);
    p += al256(size_t(kBkMaxRanges) * 4);
    w.cstart = reinterpret_cast<unsigned*>(p);
    p += al256(size_t(cstride_of(nt)) * kBkMaxRanges * 4);
    w.out = reinterpret_cast<unsigned*>(p);
    return w;
}

template <typename LT>
int launch_split(const float* s, const LT* lab, int64_t begin, int64_t end, const DirectIndex& ix,
                 const unsigned long long* Mp, const BucketWs& w, int64_t ntiles, unsigned long long* nonfinite,
                 hipStream_t st) {
    const int64_t a0 = begin & ~int64_t(3);
    // the last float4 slot wholly inside [a0, end) (the vector loads are clamped to it)
    const int64_t vmax = end - a0 >= 4 ? a0 + ((end - a0) / 4 - 1) * 4 : -1;
    const size_t lsz = sizeof(LT), lal = 4 * lsz < 16 ? 4 * lsz : 16;
    const bool vec = vmax >= 0 && (reinterpret_cast<uintptr_t>(s) & 15u) == 0 &&
                     (reinterpret_cast<uintptr_t>(lab) & (lal - 1)) == 0;
    int64_t grid = int64_t(cu_count());  // persistent: one 1024-thread workgroup per CU (LDS + registers)
    if (grid > ntiles) grid = ntiles;
    if (vec)
        hipLaunchKernelGGL((bucket_split_kernel<LT, true>), dim3(static_cast<unsigned>(grid)), dim3(kSplitThreads), 0,
                           st, s, lab, a0, begin, end, vmax, ntiles, ix.l1, w.rid, w.bmeta, Mp, w.out, w.off, w.len,
                           nonfinite);
    else
        hipLaunchKernelGGL((bucket_split_kernel<LT, false>), dim3(static_cast<unsigned>(grid)), dim3(kSplitThreads), 0,
                           st, s, lab, a0, begin, end, vmax, ntiles, ix.l1, w.rid, w.bmeta, Mp, w.out, w.off, w.len,
                           nonfinite);
    return launch_status();
}

}  // namespace

size_t bucket_workspace_size(int64_t q) {
    const int64_t nt = tiles_of(q < 1 ? 1 : q);
    return 256 + al256(size_t(kBkMaxRanges) * 16) + al256(size_t(kCiMaxBlocks) + 4) + al256(size_t(nt) * kOffStride * 4) +
           al256(size_t(nt) * kBkMaxRanges * 4) + al256(size_t(kBkMaxRanges) * 4) +
           al256(size_t(cstride_of(nt)) * kBkMaxRanges * 4) +
           al256(size_t(nt) * kSplitTile * 4);
}

int counts_bucketed(const DirectIndex& ix, const unsigned long long* Mp, const float* scores, const void* labels,
                    int label_dtype, int64_t begin, int64_t end, unsigned long long* wins_ties,
                    unsigned long long* nonfinite, unsigned* verdict, void* workspace, size_t workspace_bytes,
                    hipStream_t st) {
    const int64_t q = end - begin;
    if (q <= 0) return DAUC_OK;
    if (workspace == nullptr || workspace_bytes < bucket_workspace_size(q) ||
        (reinterpret_cast<uintptr_t>(workspace) & 255u) != 0)
        return DAUC_EINVAL;
    const BucketWs w = bucket_ws(workspace, q);
    const int64_t ntiles = tiles_of(q);
    hipLaunchKernelGGL(bucket_plan_kernel, dim3(1), dim3(kPlanThreads), 0, st, ix, Mp, w.rinfo, w.rid, w.bmeta,
                       verdict);
    int rc = launch_status();
    if (rc) return rc;
    switch (label_dtype) {
        case DAUC_LABEL_I8:
            rc = launch_split(scores, static_cast<const int8_t*>(labels), begin, end, ix, Mp, w, ntiles, nonfinite, st);
            break;
        case DAUC_LABEL_I32:
            rc = launch_split(scores, static_cast<const int32_t*>(labels), begin, end, ix, Mp, w, ntiles, nonfinite, st);
            break;
        default:
            rc = launch_split(scores, static_cast<const int64_t*>(labels), begin, end, ix, Mp, w, ntiles, nonfinite, st);
            break;
    }
    if (rc) return rc;
    hipLaunchKernelGGL(bucket_prefix_kernel, dim3(kBkMaxRanges), dim3(kPlanThreads), 0, st, w.len, ntiles,
                       cstride_of(ntiles), w.bmeta, w.tot, w.cstart);
    // one workgroup per chunk of ~kChunkQueries queries of one range: at most q / kChunkQueries + one
    // partial chunk per range (the surplus workgroups find no chunk and return)
    const int64_t grid = (q + kChunkQueries - 1) / kChunkQueries + kBkMaxRanges;
    hipLaunchKernelGGL(bucket_count_kernel, dim3(static_cast<unsigned>(grid)), dim3(kCountThreads), 0, st, w.out,
                       w.off, w.tot, w.cstart, ntiles, cstride_of(ntiles), w.rinfo, w.bmeta, ix, Mp, wins_ties,
                       verdict);
    return launch_status();
}

}  // namespace dauc
