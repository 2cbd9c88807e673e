// Exact AUC by sorting: LSD radix sort of the SMALLER class's order-preserving keys,
// then every score of the larger class is located in it with an LDS-resident search
// tree. O(M log M + L log M) work (M = min(P, N), L = max(P, N)) instead of the pair
// count's O(P*N); the counts are the same integers (W, T).
//
// Reference: imagenet/main.py:79-81 -> sklearn roc_curve/auc, whose
// _binary_clf_curve (sklearn/metrics/_ranking.py:826-908) also sorts the scores
// (a stable mergesort on the CPU, :886). SURVEY §8f row 1.
//
// Keys: an fp32 score maps to a uint32 that orders like the float, with -0 and
// +0 on one key (fp32 equality semantics): k = bits ^ (sign ? 0xffffffff : 0x80000000).
//
// Sort (per 8-bit digit, 4 passes, keys only; 2048-key tiles, one 256-thread workgroup each):
//   hist    : LDS histogram of the tile's digit -> hist[digit][tile] (digit-major)
//   scan    : small sorts (<= 256 tiles) have none — every scatter workgroup derives its own
//             offsets from the raw histogram; larger sorts scan it in 1 or 3 launches
//   scatter : wave w owns the tile's keys [512w, 512w + 512); a key's stable rank among its
//             wave's keys with the same digit = the wave's running count of that digit (a
//             wave-private LDS row) + the same-digit lanes below it (8 ballots); one barrier turns
//             the per-wave counts into offsets; writes to out[offset[digit][tile] + rank].
// Search: every k-th sorted key (k a power of two, at most kMaxSplit splitters) is a key of a
//   5-ary search tree of 16-byte nodes (4 keys, one ds_read_b128 per level) that every query
//   workgroup copies into LDS; each level stores only its real prefix plus one all-padding
//   node. A query x, clamped below the largest splitter, walks <= 7 levels (p <- 5p + #(node
//   keys <= x)), then one 16-byte load of its k-key bucket from the (L2-resident) sorted table
//   finishes upper_bound and lower_bound. The queries are streamed once with float4 loads;
//   per-block integer sums, one 64-bit atomic each.
//   table = positives: W += M - ub(x), T += ub - lb;  table = negatives: W += lb(x), T += ub - lb.

#include <stdlib.h>
#include <type_traits>

#include "count_index.h"

namespace dauc {
namespace {

constexpr int kSortThreads = 256;
constexpr int kPerThread = 8;  // keys per thread per pass tile
constexpr int kTile = kSortThreads * kPerThread;  // 2048 keys (8 per thread: the hist pass 4.9 vs 6.1 us at 134k keys)
constexpr int kRadix = 256;
constexpr int kScanBlock = 1024;
constexpr int64_t kSingleScan = 32768;  // histogram entries one workgroup scans alone (<= 512K keys)

__device__ __forceinline__ unsigned key_of(float f) {
    if (f == 0.0f) f = 0.0f;  // -0 -> +0
    const unsigned u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

int64_t tiles_for(int64_t n) { return (n + kTile - 1) / kTile; }

// ---- pass kernels -------------------------------------------------------------------

// FROM_FLOAT: the first pass reads fp32 scores and converts them to keys on the fly.
template <bool FROM_FLOAT>
__global__ __launch_bounds__(kSortThreads) void radix_hist_kernel(const void* __restrict__ in, int64_t n,
                                                                  int shift, unsigned* __restrict__ hist,
                                                                  int64_t ntiles) {
    __shared__ unsigned h[kRadix];
    h[threadIdx.x] = 0;
    __syncthreads();
    const int64_t t0 = int64_t(blockIdx.x) * kTile;
    for (int k = 0; k < kPerThread; ++k) {
        const int64_t i = t0 + int64_t(k) * kSortThreads + threadIdx.x;
        if (i < n) {
            const unsigned key = FROM_FLOAT ? key_of(static_cast<const float*>(in)[i])
                                            : static_cast<const unsigned*>(in)[i];
            atomicAdd(&h[(key >> shift) & 0xffu], 1u);
        }
    }
    __syncthreads();
    hist[int64_t(threadIdx.x) * ntiles + blockIdx.x] = h[threadIdx.x];  // digit-major
}

// exclusive scan of m counts, in place: 3 steps (block sums, scan of block sums, add back)
__global__ __launch_bounds__(kScanBlock) void scan_blocks_kernel(unsigned* __restrict__ a, int64_t m,
                                                                 unsigned* __restrict__ block_sums) {
    __shared__ unsigned s[kScanBlock];
    const int64_t i = int64_t(blockIdx.x) * kScanBlock + threadIdx.x;
    const unsigned v = i < m ? a[i] : 0u;
    s[threadIdx.x] = v;
    __syncthreads();
    for (int d = 1; d < kScanBlock; d <<= 1) {
        const unsigned t = threadIdx.x >= d ? s[threadIdx.x - d] : 0u;
        __syncthreads();
        s[threadIdx.x] += t;
        __syncthreads();
    }
    if (i < m) a[i] = s[threadIdx.x] - v;  // exclusive within the block
    if (threadIdx.x == kScanBlock - 1) block_sums[blockIdx.x] = s[threadIdx.x];
}

__global__ __launch_bounds__(kScanBlock) void scan_sums_kernel(unsigned* __restrict__ sums, int64_t nb) {
    // one block: exclusive scan of nb block sums (nb <= kScanBlock * per-thread run)
    __shared__ unsigned s[kScanBlock];
    const int64_t per = (nb + kScanBlock - 1) / kScanBlock;
    const int64_t b0 = int64_t(threadIdx.x) * per;
    const int64_t b1 = (b0 + per < nb) ? b0 + per : nb;
    unsigned local = 0;
    for (int64_t b = b0; b < b1; ++b) local += sums[b];
    s[threadIdx.x] = local;
    __syncthreads();
    for (int d = 1; d < kScanBlock; d <<= 1) {
        const unsigned t = threadIdx.x >= d ? s[threadIdx.x - d] : 0u;
        __syncthreads();
        s[threadIdx.x] += t;
        __syncthreads();
    }
    unsigned run = s[threadIdx.x] - local;
    for (int64_t b = b0; b < b1; ++b) {
        const unsigned v = sums[b];
        sums[b] = run;
        run += v;
    }
}

__global__ __launch_bounds__(kScanBlock) void scan_add_kernel(unsigned* __restrict__ a, int64_t m,
                                                              const unsigned* __restrict__ sums) {
    const int64_t i = int64_t(blockIdx.x) * kScanBlock + threadIdx.x;
    if (i < m) a[i] += sums[blockIdx.x];
}

// FUSED_SCAN: offs is the raw digit-major histogram; every workgroup derives its own output
// offsets from it (its digit's count in the tiles before it + the exclusive scan of the digit
// totals): a small sort (<= kFusedScanTiles tiles) then needs no scan launches at all.
constexpr int64_t kFusedScanTiles = 256;

// exclusive scan of v over the block's 256 threads (thread t holds digit t): wave scans by
// shuffles, then the wave totals through LDS (one barrier); returns the exclusive prefix
__device__ __forceinline__ unsigned block_excl_scan256(unsigned v, unsigned* wtot) {
    static_assert(kSortThreads == 256, "4 waves");
    const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
    unsigned incl = v;
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
        const unsigned t = __shfl_up(incl, off, kWave);
        if (lane >= off) incl += t;
    }
    if (lane == kWave - 1) wtot[wid] = incl;
    __syncthreads();
    unsigned before = 0;
#pragma unroll
    for (int w = 0; w < kSortThreads / kWave; ++w) before += w < wid ? wtot[w] : 0u;
    return before + incl - v;
}

// Stable scatter of one tile. Wave w owns the tile's contiguous keys [w * 512, (w + 1) * 512),
// read as 8 chunks of 64 (one per lane). A key's rank among its wave's keys with the same digit
// = the wave's running count of that digit (wave-private LDS row: a wave's LDS reads and writes
// are ordered, so no barrier) + the same-digit lanes below it in its chunk (8 ballots: wave
// multisplit). One barrier, then per digit the waves' counts become offsets, and every key goes
// to base[digit] + offset[wave][digit] + rank: 2 barriers per pass instead of 4 per chunk.
template <bool FROM_FLOAT, bool FUSED_SCAN>
__global__ __launch_bounds__(kSortThreads) void radix_scatter_kernel(const void* __restrict__ in, int64_t n,
                                                                     int shift,
                                                                     const unsigned* __restrict__ offs,
                                                                     int64_t ntiles,
                                                                     unsigned* __restrict__ out) {
    constexpr int kWaves = kSortThreads / kWave;
    constexpr int kChunks = kTile / kSortThreads;  // chunks of 64 keys per wave
    __shared__ unsigned base[kRadix];             // output start of each digit for this tile
    __shared__ unsigned wcnt[kWaves][kRadix];     // per-wave running digit counts, then offsets
    __shared__ unsigned wtot[kWaves];
    const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
    const unsigned long long lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    const int64_t t0 = int64_t(blockIdx.x) * kTile + int64_t(wid) * (kChunks * kWave);
    unsigned key[kChunks];
#pragma unroll
    for (int c = 0; c < kChunks; ++c) {
        const int64_t i = t0 + c * kWave + lane;
        key[c] = 0u;
        if (i < n)
            key[c] = FROM_FLOAT ? key_of(static_cast<const float*>(in)[i]) : static_cast<const unsigned*>(in)[i];
    }
    // this tile's digit bases (thread t = digit t)
    if constexpr (FUSED_SCAN) {
        static_assert(kSortThreads == kRadix, "one thread per digit");
        const unsigned* h = offs + int64_t(threadIdx.x) * ntiles;
        unsigned before = 0, total = 0;
        int64_t b = 0;
        for (; b + 4 <= ntiles; b += 4) {
            const unsigned c0 = h[b], c1 = h[b + 1], c2 = h[b + 2], c3 = h[b + 3];
            before += (b < blockIdx.x ? c0 : 0u) + (b + 1 < blockIdx.x ? c1 : 0u) + (b + 2 < blockIdx.x ? c2 : 0u) +
                      (b + 3 < blockIdx.x ? c3 : 0u);
            total += c0 + c1 + c2 + c3;
        }
        for (; b < ntiles; ++b) {
            const unsigned c = h[b];
            before += b < blockIdx.x ? c : 0u;
            total += c;
        }
        base[threadIdx.x] = block_excl_scan256(total, wtot) + before;
    } else {
        base[threadIdx.x] = offs[int64_t(threadIdx.x) * ntiles + blockIdx.x];
    }
#pragma unroll
    for (int q = 0; q < kRadix / kWave; ++q) wcnt[wid][q * kWave + lane] = 0u;
    unsigned rank[kChunks];
#pragma unroll
    for (int c = 0; c < kChunks; ++c) {
        const bool valid = t0 + c * kWave + lane < n;
        const unsigned d = (key[c] >> shift) & 0xffu;
        unsigned long long same = __ballot(valid);
#pragma unroll
        for (int bit = 0; bit < 8; ++bit) {
            const unsigned long long m = __ballot((d >> bit) & 1u);
            same &= ((d >> bit) & 1u) ? m : ~m;
        }
        const unsigned below = __popcll(same & lt);
        const unsigned run = valid ? wcnt[wid][d] : 0u;  // every same-digit lane reads before the leader writes
        rank[c] = run + below;
        if (valid && below == 0) wcnt[wid][d] = run + __popcll(same);
    }
    __syncthreads();
    {
        // offsets of the waves within each digit (thread t = digit t)
        unsigned run = 0;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) {
            const unsigned c = wcnt[w][threadIdx.x];
            wcnt[w][threadIdx.x] = run;
            run += c;
        }
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < kChunks; ++c) {
        if (t0 + c * kWave + lane < n) {
            const unsigned d = (key[c] >> shift) & 0xffu;
            out[base[d] + wcnt[wid][d] + rank[c]] = key[c];
        }
    }
}

// the distinct-key index of tie-heavy tables (dk_*_kernel below)
constexpr int kDkMax = 14000;
// the plan's cells: 4 per distinct key (up to 3,500 of them), fewer but at least 1 past that, + 1 per used bucket
constexpr int kDkMaxCells = kDkMax + kCiTop;
constexpr int kDkTile = 1024;                     // table keys per tile of the mark / write passes (4 per thread)
constexpr int kDkUse = 0, kDkD = 1;              // meta words; kCiOk, kCiCells, kCiBlocks: the plan's
constexpr int kDkScanThreads = 1024;
static_assert(kDkMax < 16384, "the query's LDS holds a cell's first distinct key in 14 bits");

struct DkWs {
    unsigned* meta;    // [16]
    uint2* l1;         // [kCiTop]
    unsigned* cstart;  // [kDkMaxCells + 2] the first distinct key of every cell
    unsigned* kd;      // [kDkMax] the distinct keys, ascending
    unsigned* cd;      // [kDkMax] #(table keys <= kd[i])
    unsigned* tcnt;    // [tiles] distinct keys whose last copy is in the tile -> their exclusive prefix
};

__device__ __forceinline__ bool dk_ci_in_use(const unsigned* __restrict__ ci_meta) {
    return ci_meta != nullptr && count_index_in_use(ci_meta);
}

// ---- search ---------------------------------------------------------------------------

// Splitters (every k-th sorted key, k a power of two) kept in LDS: at most kMaxSplit of them
// (4 B each: 40000 -> 156 KB of the CU's 160 KB), so a bucket holds k <= 4 keys -- ONE 16-byte
// load -- up to M = 160,000 table keys (2^27 scores at 0.1 % positives: M = 134,447 -> k = 4).
constexpr int kMaxSplit = 40000;
constexpr size_t kTreeBytes = (size_t(kMaxSplit) + 64) * 4;  // nodes of 4 keys + per-level padding nodes
constexpr int kQueryThreads = 1024;

// The S splitters are the in-order keys of a perfect 5-ary search tree of height H (5^(H-1) <= S
// + 1 <= 5^H): a node is 4 keys (16 B, one ds_read_b128) and routes a query to child
// #(keys <= x), so a walk is H <= 7 dependent LDS reads (a binary tree needs ~16). Key i of node
// j on level d has in-order rank (5j + i + 1) * 5^(H-1-d) - 1; keys of rank >= S are padding
// (+inf). The nodes holding at least one real key form a prefix of every level (n_d nodes),
// stored level after level and followed by ONE all-padding node: a walk at position p of level
// d reads node off_d + min(p, n_d), and p <- 5p + #(node keys <= x); after H levels p =
// #splitters <= x. The sorted table is padded with kPadKey to a whole number of buckets.
constexpr int kTreeArity = 5;  // 4-key nodes, one ds_read_b128 (3-ary 8-byte nodes measured the same)
constexpr int kNodeKeys = kTreeArity - 1;
constexpr int kMaxTreeH = 7;  // 5^7 - 1 >= kMaxSplit
static_assert(kMaxSplit <= 78124, "tree height bound");
typedef uint4 TreeNode;

struct TreeGeom {
    int S, H;
    int nd[kMaxTreeH];   // stored real nodes of level d
    int off[kMaxTreeH];  // first node of level d
    int nodes;           // total stored nodes (incl. the per-level padding nodes)
};

// (round 2 measured the tree's top levels held in SGPRs instead of LDS: no faster)
struct TopKeys {
    unsigned last;  // the largest splitter (a finite score's key, so >= 0x007fffff > 0)
};

TreeGeom tree_geom(int S) {
    TreeGeom g{};
    g.S = S;
    int64_t pw = 1;
    g.H = 0;
    while (pw * kTreeArity - 1 < S) {
        pw *= kTreeArity;
        ++g.H;
    }
    ++g.H;  // A^(H-1) <= S + 1 <= A^H
    int off = 0;
    int64_t div = pw;  // A^(H-1-d)
    for (int d = 0; d < g.H; ++d) {
        const int64_t t = S / div;
        g.nd[d] = static_cast<int>((t + kTreeArity - 1) / kTreeArity);  // j with A j + 1 <= t
        g.off[d] = off;
        off += g.nd[d] + 1;
        div /= kTreeArity;
    }
    g.nodes = off;
    return g;
}

__device__ __forceinline__ void store_node(uint4* t, int64_t c, const unsigned (&k)[4]) { t[c] = uint4{k[0], k[1], k[2], k[3]}; }

__global__ __launch_bounds__(256) void build_tree_kernel(unsigned* __restrict__ sorted, int64_t M, int64_t pad, int k,
                                                         TreeGeom g, TreeNode* __restrict__ tree,
                                                         unsigned* __restrict__ ci_first, int n_first) {
    const int64_t c = int64_t(blockIdx.x) * 256 + threadIdx.x;
    if (c < g.nodes) {
        int d = 0;
        while (d + 1 < g.H && c >= g.off[d + 1]) ++d;
        const int j = static_cast<int>(c) - g.off[d];
        int64_t pw = 1;
        for (int e = d + 1; e < g.H; ++e) pw *= kTreeArity;
        unsigned key[4] = {kPadKey, kPadKey, kPadKey, kPadKey};
#pragma unroll
        for (int i = 0; i < kNodeKeys; ++i) {
            const int64_t r = (int64_t(kTreeArity) * j + i + 1) * pw - 1;  // in-order rank
            key[i] = (j < g.nd[d] && r < g.S) ? sorted[r * k] : kPadKey;
        }
        store_node(tree, c, key);
    }
    // keys M .. S*k of the last bucket (and at least 8 past M, for the count index's windows):
    // +inf, so bucket compares need no bounds
    if (c < pad || c < 8) sorted[M + c] = kPadKey;
    if (c < n_first) ci_first[c] = static_cast<unsigned>(M);  // count index: "no key in this bucket"
}

// p <- 5 p + #(node keys <= x): the compares' carries feed the adds (a carry-free form with
// saturating subtracts, 12 VALU instead of 8, measured 5 % slower in round 2)
__device__ __forceinline__ unsigned tree_step(unsigned p, uint4 n, unsigned x) {
    unsigned r = p * 5u;
    asm("v_cmp_le_u32_e32 vcc, %1, %5\n\t"
        "v_addc_co_u32_e32 %0, vcc, 0, %0, vcc\n\t"
        "v_cmp_le_u32_e32 vcc, %2, %5\n\t"
        "v_addc_co_u32_e32 %0, vcc, 0, %0, vcc\n\t"
        "v_cmp_le_u32_e32 vcc, %3, %5\n\t"
        "v_addc_co_u32_e32 %0, vcc, 0, %0, vcc\n\t"
        "v_cmp_le_u32_e32 vcc, %4, %5\n\t"
        "v_addc_co_u32_e32 %0, vcc, 0, %0, vcc"
        : "+v"(r)
        : "v"(n.x), "v"(n.y), "v"(n.z), "v"(n.w), "v"(x)
        : "vcc");
    return r;
}

// Q walks of the tree in lockstep: p[q] ends as #splitters <= x[q]. The level geometry is
// wave-uniform (kernel arguments, scalar registers).
template <int Q>
__device__ __forceinline__ void tree_walk(const unsigned (&x)[Q], unsigned (&p)[Q], const TreeNode* __restrict__ tree,
                                          const TreeGeom& g, const TopKeys& top) {
#pragma unroll
    for (int q = 0; q < Q; ++q) p[q] = 0;
    // A walk for x below the largest splitter only visits stored nodes: its node at level d is
    // floor(r / 5^(H-d)) for r = #splitters <= x <= S - 1, at most the level's one padding node
    // (n_d). So x is clamped below the largest splitter (no per-level index clamp) and the
    // queries at or above it get p = S.
    unsigned xc[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) xc[q] = x[q] < top.last ? x[q] : top.last - 1u;
#pragma unroll
    for (int d = 0; d < kMaxTreeH; ++d) {
        if (d < g.H) {
            const unsigned off = static_cast<unsigned>(g.off[d]);
            TreeNode v[Q];
#pragma unroll
            for (int q = 0; q < Q; ++q) v[q] = tree[off + p[q]];
#pragma unroll
            for (int q = 0; q < Q; ++q) p[q] = tree_step(p[q], v[q], xc[q]);
        }
    }
#pragma unroll
    for (int q = 0; q < Q; ++q) p[q] = x[q] < top.last ? p[q] : static_cast<unsigned>(g.S);
}

// #keys of bucket b (keys sorted[b*k .. min(b*k + k, M))) that are <= x, and that are < x;
// first = the bucket's smallest key (its splitter)
template <int K>
__device__ __forceinline__ void bucket_counts(const unsigned* __restrict__ sorted, int64_t M, int64_t b,
                                              unsigned x, int& le, int& lt, unsigned& first) {
    const int64_t base = b * K;
    unsigned v[K];
    if constexpr (K >= 4) {
#pragma unroll
        for (int q = 0; q < K / 4; ++q) {
            const uint4 u = reinterpret_cast<const uint4*>(sorted + base)[q];
            v[4 * q] = u.x;
            v[4 * q + 1] = u.y;
            v[4 * q + 2] = u.z;
            v[4 * q + 3] = u.w;
        }
    } else if constexpr (K == 2) {
        const uint2 u = *reinterpret_cast<const uint2*>(sorted + base);
        v[0] = u.x;
        v[1] = u.y;
    } else {
        v[0] = sorted[base];
    }
    first = v[0];
    le = 0;
    lt = 0;
#pragma unroll
    for (int j = 0; j < K; ++j) {  // the tail bucket is padded with kPadKey (> every finite key)
        le += v[j] <= x;
        lt += v[j] < x;
    }
}

// #keys in sorted[lo, hi) that are < x (LT) or <= x (!LT): binary search in global memory
template <bool LT>
__device__ __forceinline__ int64_t count_below(const unsigned* __restrict__ a, int64_t lo, int64_t hi, unsigned x) {
    int64_t len = hi - lo, base = lo;
    while (len > 0) {
        const int64_t half = len >> 1;
        const unsigned v = a[base + half];
        if (LT ? v < x : v <= x) {
            base += half + 1;
            len -= half + 1;
        } else {
            len = half;
        }
    }
    return base - lo;
}

// One query (K = 0: buckets of k > 32 keys, finished by binary searches in global memory).
template <int K, bool TABLE_POS>
__device__ __forceinline__ void count_query(unsigned x, const TreeNode* __restrict__ tree, const TreeGeom& g,
                                            const TopKeys& top, int k,
                                            const unsigned* __restrict__ sorted, int64_t M,
                                            unsigned long long& w, unsigned long long& t) {
    // splitters <= x (walk 0) and < x = <= x - 1 (walk 1; finite keys are >= 0x00800000, so
    // x - 1 never wraps)
    int64_t ub = 0, lb = 0;
    if constexpr (K <= 1) {
        const unsigned xs[2] = {x, x - 1u};
        unsigned i[2];
        tree_walk<2>(xs, i, tree, g, top);
        const int64_t su = i[0], sl = i[1];
        if constexpr (K == 1) {
            ub = su;
            lb = sl;
        } else {
            if (su > 0) {
                const int64_t b0 = (su - 1) * k, b1 = (b0 + k < M) ? b0 + k : M;
                ub = b0 + count_below<false>(sorted, b0, b1, x);
            }
            if (sl > 0) {
                const int64_t b0 = (sl - 1) * k, b1 = (b0 + k < M) ? b0 + k : M;
                lb = b0 + count_below<true>(sorted, b0, b1, x);
            }
        }
    } else {
        // one walk for x; the walk for x - 1 is needed only when the last splitter <= x
        // equals x (a run of x may then start in an earlier bucket)
        const unsigned xs[1] = {x};
        unsigned i[1];
        tree_walk<1>(xs, i, tree, g, top);
        const int64_t su = i[0];
        if (su > 0) {
            int le = 0, lt = 0;
            unsigned first = 0;
            bucket_counts<K>(sorted, M, su - 1, x, le, lt, first);
            ub = (su - 1) * K + le;
            if (first < x) {
                lb = (su - 1) * K + lt;
            } else {
                const unsigned xm[1] = {x - 1u};
                tree_walk<1>(xm, i, tree, g, top);
                const int64_t sl = i[0];
                if (sl > 0) {
                    bucket_counts<K>(sorted, M, sl - 1, x, le, lt, first);
                    lb = (sl - 1) * K + lt;
                }
            }
        }
    }
    w += TABLE_POS ? static_cast<unsigned long long>(M - ub) : static_cast<unsigned long long>(lb);
    t += static_cast<unsigned long long>(ub - lb);
}

// Q queries walked in lockstep (K = 1 .. 32): Q independent chains of LDS reads (and then Q
// bucket loads) in flight per lane. use[q] = false: the slot is walked but not counted.
template <int K>
constexpr int lockstep_queries() {
    return K <= 8 ? 4 : (K == 16 ? 2 : 1);
}

template <int K, int Q, bool TABLE_POS>
__device__ __forceinline__ void count_queries(const unsigned (&x)[Q], const bool (&use)[Q],
                                              const TreeNode* __restrict__ tree, const TreeGeom& g,
                                              const TopKeys& top,
                                              const unsigned* __restrict__ sorted, int64_t M,
                                              unsigned long long& w, unsigned long long& t) {
    static_assert(K >= 1 && K <= 32, "bucketed lockstep walk");
    if constexpr (K == 1) {
        // the tree holds every key: splitters <= x and <= x - 1 directly
        unsigned xs[2 * Q], i[2 * Q];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            xs[q] = x[q];
            xs[Q + q] = x[q] - 1u;
        }
        tree_walk<2 * Q>(xs, i, tree, g, top);
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            if (!use[q]) continue;
            const int64_t ub = i[q], lb = i[Q + q];
            w += TABLE_POS ? static_cast<unsigned long long>(M - ub) : static_cast<unsigned long long>(lb);
            t += static_cast<unsigned long long>(ub - lb);
        }
    } else {
        unsigned su[Q];
        tree_walk<Q>(x, su, tree, g, top);
        // every bucket load issued before any is examined (su = 0: bucket 0 is read, unused)
        int le[Q], lt[Q];
        unsigned first[Q];
#pragma unroll
        for (int q = 0; q < Q; ++q) bucket_counts<K>(sorted, M, su[q] ? su[q] - 1u : 0u, x[q], le[q], lt[q], first[q]);
        // 32-bit and branch-free: lb below is exact unless the bucket starts with x itself (then
        // a run of x may begin in an earlier bucket); those rare queries are fixed up after
        // the Q queries' counts summed in 32 bits (Q * M < 2^32), one 64-bit add each
        bool slow = false;
        unsigned wl = 0u, tl = 0u;
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const unsigned base = su[q] ? (su[q] - 1u) * static_cast<unsigned>(K) : 0u;
            const unsigned ub = su[q] ? base + static_cast<unsigned>(le[q]) : 0u;
            const unsigned lb = su[q] ? base + static_cast<unsigned>(lt[q]) : 0u;
            const unsigned wq = TABLE_POS ? static_cast<unsigned>(M) - ub : lb;
            wl += use[q] ? wq : 0u;
            tl += use[q] ? ub - lb : 0u;
            slow |= use[q] && su[q] != 0u && first[q] >= x[q];
        }
        w += wl;
        t += tl;
        if (slow) {
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                if (!(use[q] && su[q] != 0u && first[q] >= x[q])) continue;
                const unsigned xm[1] = {x[q] - 1u};
                unsigned j[1];
                tree_walk<1>(xm, j, tree, g, top);
                unsigned lb_true = 0u;
                if (j[0] != 0u) {
                    int le2 = 0, lt2 = 0;
                    unsigned f2 = 0;
                    bucket_counts<K>(sorted, M, j[0] - 1u, x[q], le2, lt2, f2);
                    lb_true = (j[0] - 1u) * static_cast<unsigned>(K) + static_cast<unsigned>(lt2);
                }
                const unsigned lb_fast = (su[q] - 1u) * static_cast<unsigned>(K);  // lt = 0: the bucket starts with x
                t += lb_fast - lb_true;                                             // ties: ub - lb_true
                if (!TABLE_POS) w -= lb_fast - lb_true;                             // wins: lb_true
            }
        }
    }
}

// Four keys (one float4 slot) with per-key use flags, through count_queries in groups of Q
// (K = 0, buckets > 32 keys finished in global memory: one key at a time).
template <int K, bool TABLE_POS>
__device__ __forceinline__ void count4(const unsigned (&x)[4], const bool (&use)[4], const TreeNode* __restrict__ tree,
                                       const TreeGeom& g, const TopKeys& top, int k, const unsigned* __restrict__ sorted, int64_t M,
                                       unsigned long long& w, unsigned long long& t) {
    if constexpr (K == 0) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (use[q]) count_query<0, TABLE_POS>(x[q], tree, g, top, k, sorted, M, w, t);
    } else {
        constexpr int Q = lockstep_queries<K>();
#pragma unroll
        for (int b = 0; b < 4; b += Q) {
            unsigned xs[Q];
            bool us[Q];
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                xs[q] = x[b + q];
                us[q] = use[b + q];
            }
            count_queries<K, Q, TABLE_POS>(xs, us, tree, g, top, sorted, M, w, t);
        }
    }
}

// the top levels' keys, read once per workgroup with uniform (scalar) loads
__device__ __forceinline__ TopKeys load_top(const TreeNode* __restrict__ gtree, const TreeGeom& g,
                                           const unsigned* __restrict__ sorted, int k) {
    (void)gtree;
    (void)g;
    TopKeys t{};
    t.last = sorted[int64_t(g.S - 1) * k];
    return t;
}

template <int K, bool TABLE_POS>
__global__ __launch_bounds__(kQueryThreads) void query_count_kernel(const float* __restrict__ q, int64_t L,
                                                                   const TreeNode* __restrict__ gtree, TreeGeom g,
                                                                   int k, const unsigned* __restrict__ sorted,
                                                                   int64_t M, unsigned long long* __restrict__ out,
                                                                   const unsigned* __restrict__ dk_meta) {
    if (dk_meta != nullptr && dk_meta[kDkUse] != 0u) return;  // the distinct-key index counts instead
    extern __shared__ TreeNode tree[];
    for (int i = threadIdx.x; i < g.nodes; i += kQueryThreads) tree[i] = gtree[i];
    const TopKeys top = load_top(gtree, g, sorted, k);
    __syncthreads();
    unsigned long long w = 0, t = 0;
    const bool vec = (reinterpret_cast<uintptr_t>(q) & 15u) == 0;
    const int64_t nvec = vec ? L / 4 : 0;
    const int64_t stride = int64_t(gridDim.x) * kQueryThreads;
    const bool all[4] = {true, true, true, true};
    for (int64_t v = int64_t(blockIdx.x) * kQueryThreads + threadIdx.x; v < nvec; v += stride) {
        const f32x4 f = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(q) + v);
        const unsigned x[4] = {key_of(f.x), key_of(f.y), key_of(f.z), key_of(f.w)};
        count4<K, TABLE_POS>(x, all, tree, g, top, k, sorted, M, w, t);
    }
    for (int64_t i = nvec * 4 + int64_t(blockIdx.x) * kQueryThreads + threadIdx.x; i < L; i += stride)
        count_query<K, TABLE_POS>(key_of(q[i]), tree, g, top, k, sorted, M, w, t);
    __shared__ unsigned long long red[2][kQueryThreads / kWave];
    w = wave_sum(w);
    t = wave_sum(t);
    const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
    if (lane == 0) {
        red[0][wid] = w;
        red[1][wid] = t;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long bw = 0, bt = 0;
        for (int i = 0; i < kQueryThreads / kWave; ++i) {
            bw += red[0][i];
            bt += red[1][i];
        }
        if (bw) atomicAdd(out + 0, bw);
        if (bt) atomicAdd(out + 1, bt);
    }
}


// Labeled queries: the negatives are not materialised. Elements [begin, end) of the full score
// and label arrays are streamed (float4 + 4 labels per slot); every element whose label is
// not +1 is a query against the sorted positives (table = positives).
template <typename LT>
__device__ __forceinline__ void label4(const LT* __restrict__ lab, int64_t i, bool full, int64_t end, bool (&neg)[4]) {
    if (full && sizeof(LT) == 1) {
        const char4 c = *reinterpret_cast<const char4*>(lab + i);
        neg[0] = c.x != 1;
        neg[1] = c.y != 1;
        neg[2] = c.z != 1;
        neg[3] = c.w != 1;
    } else if (full && sizeof(LT) == 4) {
        const int4 c = *reinterpret_cast<const int4*>(lab + i);
        neg[0] = c.x != 1;
        neg[1] = c.y != 1;
        neg[2] = c.z != 1;
        neg[3] = c.w != 1;
    } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) neg[q] = i + q < end && lab[i + q] != LT(1);
    }
}

// Region of the sort workspace that holds the direct build's 72 group totals (grp)
constexpr size_t kGrpBytes = 512;

// search structure: 0 automatic (the count index where it holds the table, else the distinct-key
// index where it holds it, else the tree); the tuning build can force the tree
// (dauc_set_search_mode(1)) or the distinct-key index (2) to test them on any table
#ifdef DAUC_TUNING
int g_search_mode = 0;
#else
constexpr int g_search_mode = 0;
#endif

// ---- count index (the default search where it fits: dauc_set_search_mode 0) -----------------
//
// The tree's cost per query is its one 16-byte bucket gather from L2 plus 7 dependent LDS reads
// and ~140 VALU. The count index answers ~40 % of the queries with no gather at all and the rest
// with one, from 2 LDS reads and ~60 VALU:
//   * the key's top 11 bits pick a top bucket t (sign, exponent, 2 mantissa bits); its n_t table
//     keys get C_t = ceil(n_t * R) cells that split its 2^21 low key values evenly
//     (cell = off_t + mulhi(low21 << 11, C_t)), R = cells per table key (~1.1 for the 2^27 @
//     0.1 % table, so ~40 % of the cells -- and of the queries -- are empty);
//   * LDS holds {off_t, C_t} (2048 x 8 B) and, per block of 8 cells, {the table keys before the
//     block, the 8 cells' key counts as nibbles} (8 B): 1 B per cell, 146,559 cells;
//   * rank_lo = block base + the nibbles below the cell = #(table keys < the cell) and cnt = the
//     cell's nibble: the aligned 16-byte window of the sorted table at rank_lo & ~3 (loaded only
//     by the lanes with cnt > 0; a second one when the cell runs past it, a binary search past 8
//     keys) gives lb and ub by counting its keys < x and <= x -- keys before the cell are < x,
//     keys after it > x or the +inf padding; cnt = 0 gives lb = ub = rank_lo.
// The builder keeps the tree (a device word both query kernels read) when the table needs more
// than 1.5 keys per cell or a cell holds 15 or more keys (a nibble): clustered or tie-heavy
// tables, for which the tree's cost does not depend on the key distribution.

constexpr int kCiPlanThreads = 1024;

struct CountWs {
    unsigned* meta;    // [16]
    unsigned* first;   // [kCiTop]      first table index of every top bucket (M = none)
    uint2* l1;         // [kCiTop]      {first cell, cells} of every top bucket
    unsigned* cstart;  // [kCiMaxCells + 2] first table index of every cell
    uint2* blk;        // [kCiMaxBlocks] {keys before the block, 8 nibble counts}
};

constexpr size_t kCountBytes = 256 + 3 * size_t(kCiTop) * 4 + ((size_t(kCiMaxCells) + 2) * 4 + 255) / 256 * 256 +
                               size_t(kCiMaxBlocks) * 8 + 256;





// first[t] = the first table index of top bucket t, for the buckets holding keys (first[] was set
// to M by build_tree_kernel)
__global__ __launch_bounds__(256) void ci_first_kernel(const unsigned* __restrict__ sorted, int64_t M,
                                                       unsigned* __restrict__ first) {
    const int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x;
    if (i >= M) return;
    const unsigned t = sorted[i] >> kCiLowBits;
    if (i == 0 || (sorted[i - 1] >> kCiLowBits) != t) first[t] = static_cast<unsigned>(i);
}

// One workgroup: n_t from the suffix minima of first[] (thread i owns the buckets 2047 - 2i and
// 2046 - 2i: descending, so the suffix minima are prefix minima over the threads), the cells per
// bucket C_t = ceil(n_t * num / M), num = min(cells left after one per used bucket, 2 M) (so
// sum C_t fits), and the first cell of every bucket (prefix sum).
// (the body is shared with the distinct-key index's plan: dk_index_kernel; `first` and `l1` may be
// LDS or global, `max_cells` the cells the consumer's LDS holds)
__device__ __forceinline__ void ci_plan_body(int64_t M, const unsigned* first, uint2* l1, unsigned* __restrict__ meta,
                                             int64_t max_cells, unsigned* wtot, unsigned* incl_min, unsigned* totals,
                                             int per_key = 2) {
    static_assert(kCiTop == 2 * kCiPlanThreads, "two top buckets per thread");
    const unsigned m32 = static_cast<unsigned>(M);
    int tj[2];
    unsigned st[2], run = ~0u;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        tj[j] = kCiTop - 1 - 2 * static_cast<int>(threadIdx.x) - j;
        const unsigned f = first[tj[j]];
        run = f < run ? f : run;
        st[j] = run;
    }
    const unsigned incl = block_incl_scan1024<true>(run, wtot);
    incl_min[threadIdx.x] = incl;
    __syncthreads();
    unsigned n[2];
    {
        const unsigned above = threadIdx.x == 0 ? m32 : incl_min[threadIdx.x - 1];
        unsigned hi = above < m32 ? above : m32;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const unsigned s0 = st[j] < hi ? st[j] : hi;
            n[j] = hi - s0;
            hi = s0;
        }
    }
    const unsigned used = block_incl_scan1024<false>((n[0] != 0u) + (n[1] != 0u), wtot);
    if (threadIdx.x == kCiPlanThreads - 1) totals[0] = used;
    __syncthreads();
    const int64_t avail = max_cells - int64_t(totals[0]);
    const int64_t num = avail < per_key * M ? avail : per_key * M;
    unsigned C[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) C[j] = n[j] ? static_cast<unsigned>((int64_t(n[j]) * num + M - 1) / M) : 0u;
    const unsigned csum = C[0] + C[1];
    const unsigned incl_c = block_incl_scan1024<false>(csum, wtot);
    if (threadIdx.x == kCiPlanThreads - 1) totals[1] = incl_c;
    __syncthreads();
    const unsigned total = totals[1];
    unsigned upto = incl_c - csum;  // cells of the buckets above this thread's
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        upto += C[j];
        l1[tj[j]] = uint2{total - upto, C[j]};
    }
    if (threadIdx.x == 0) {
        meta[kCiOk] = (3 * num >= 2 * M && total <= static_cast<unsigned>(max_cells)) ? 1u : 0u;  // <= 1.5 keys/cell
        meta[kCiCells] = total;
        meta[kCiBlocks] = (total + 1 + kCiBlock - 1) / kCiBlock;
        meta[kCiSkew] = 0u;
    }
}

__global__ __launch_bounds__(kCiPlanThreads) void ci_plan_kernel(int64_t M, const unsigned* __restrict__ first,
                                                                 uint2* __restrict__ l1,
                                                                 unsigned* __restrict__ meta) {
    __shared__ unsigned wtot[kCiPlanThreads / kWave];
    __shared__ unsigned incl_min[kCiPlanThreads];
    __shared__ unsigned totals[2];
    ci_plan_body(M, first, l1, meta, kCiMaxCells, wtot, incl_min, totals);
}

// One thread per table index i in [0, M] (i = M: past the last cell): cells (c(i-1), c(i)] start at i
__global__ __launch_bounds__(256) void ci_cells_kernel(const unsigned* __restrict__ sorted, int64_t M,
                                                       const uint2* __restrict__ l1, const unsigned* __restrict__ meta,
                                                       unsigned* __restrict__ cstart) {
    if (meta[kCiOk] == 0u) return;
    const int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x;
    if (i > M) return;
    auto cell = [&](int64_t j) -> int64_t {
        const unsigned key = sorted[j];
        return ci_cell(key, l1[key >> kCiLowBits]);
    };
    const int64_t ci = i < M ? cell(i) : int64_t(meta[kCiCells]) + 1;
    const int64_t cp = i > 0 ? cell(i - 1) : -1;
    for (int64_t c = cp + 1; c <= ci; ++c) cstart[c] = static_cast<unsigned>(i);
}

// One thread per block of 8 cells: the table keys before the block and the cells' counts as
// nibbles; a count of 15 or more marks the table skewed (the tree is used)
__global__ __launch_bounds__(256) void ci_blocks_kernel(const unsigned* __restrict__ cstart,
                                                        unsigned* __restrict__ meta, uint2* __restrict__ blk) {
    if (meta[kCiOk] == 0u) return;
    const int b = blockIdx.x * 256 + threadIdx.x;
    const int nb = static_cast<int>(meta[kCiBlocks]);
    const int last = static_cast<int>(meta[kCiCells]) + 1;  // cstart[0 .. last] are written
    bool skew = false;
    if (b < nb) {
        unsigned w = 0;
        const int c0 = b * kCiBlock;
        unsigned prev = cstart[c0 < last ? c0 : last];
        const unsigned base = prev;
#pragma unroll
        for (int j = 0; j < kCiBlock; ++j) {
            const int c = c0 + j + 1;
            const unsigned nxt = cstart[c < last ? c : last];
            const unsigned cnt = nxt - prev;
            skew |= cnt >= 15u;
            w |= (cnt < 15u ? cnt : 15u) << (4 * j);
            prev = nxt;
        }
        blk[b] = uint2{base, w};
    }
    if (__ballot(skew) != 0ull && (threadIdx.x & (kWave - 1)) == 0) atomicOr(meta + kCiSkew, 1u);
}

// a 16-byte window of the L2-resident table
__device__ __forceinline__ uint4 win_load(const unsigned* p) { return *reinterpret_cast<const uint4*>(p); }

// Counting in VGPRs only: gt01(a, b) = min(sat(a - b), 1) is 1 when a > b, else 0. A compare into
// an SGPR read back by a v_cndmask / v_addc costs the VALU-writes-SGPR hazard's wait states on
// every key (the round-3 loop issued 110 VALU per query, s_nop-padded, ~75 % of the SIMDs' issue
// cycles: DESIGN §3).
__device__ __forceinline__ unsigned gt01(unsigned a, unsigned b) {
    return min(__builtin_elementwise_sub_sat(a, b), 1u);
}
// the window's keys <= x and < x
__device__ __forceinline__ void win_le_lt(const uint4& k, unsigned x, unsigned& le, unsigned& lt) {
    le = 4u - (gt01(k.x, x) + gt01(k.y, x) + gt01(k.z, x) + gt01(k.w, x));
    lt = gt01(x, k.x) + gt01(x, k.y) + gt01(x, k.z) + gt01(x, k.w);
}

// Phase 1 of one query: cell, rank_lo, count and (lanes with cnt > 0) the window load
__device__ __forceinline__ void ci_locate(unsigned x, const uint2* __restrict__ l1, const uint2* __restrict__ blk,
                                          const unsigned* __restrict__ sorted, unsigned& rl, unsigned& cnt,
                                          uint4& k) {
    const unsigned c = ci_cell(x, l1[x >> kCiLowBits]);
    const uint2 b = blk[c / kCiBlock];
    const unsigned sh = 4u * (c % kCiBlock);
    const unsigned below = __builtin_amdgcn_ubfe(b.y, 0u, sh);           // nibbles of the cells before
    const unsigned bytes = (below & 0x0f0f0f0fu) + ((below >> 4) & 0x0f0f0f0fu);
    rl = b.x + __builtin_amdgcn_sad_u8(bytes, 0u, 0u);
    cnt = __builtin_amdgcn_ubfe(b.y, sh, 4u);
    k = uint4{kPadKey, kPadKey, kPadKey, kPadKey};
    if (cnt) k = *reinterpret_cast<const uint4*>(sorted + (rl & ~3u));
}

// Phase 2: lb, ub from the window (W += M - ub, T += ub - lb for use); returns whether the cell
// runs past the window (then ci_fix recounts it)
__device__ __forceinline__ bool ci_count(unsigned x, bool use, unsigned rl, unsigned cnt, const uint4& k, unsigned M,
                                         unsigned& wl, unsigned& tl) {
    const unsigned base = cnt ? (rl & ~3u) : rl;
    const unsigned lt = (k.x < x) + (k.y < x) + (k.z < x) + (k.w < x);
    const unsigned le = (k.x <= x) + (k.y <= x) + (k.z <= x) + (k.w <= x);
    wl += use ? M - (base + le) : 0u;
    tl += use ? le - lt : 0u;
    return use && (rl & 3u) + cnt > 4u;
}

// a cell past its window: the next 4 keys (or, past 8, every key of the cell); corrects W and T
__device__ __forceinline__ void ci_fix(unsigned x, unsigned rl, unsigned cnt, const uint4& k,
                                       const unsigned* __restrict__ sorted, unsigned long long& w,
                                       unsigned long long& t) {
    const unsigned a = rl & ~3u;
    const unsigned lt0 = (k.x < x) + (k.y < x) + (k.z < x) + (k.w < x);
    const unsigned le0 = (k.x <= x) + (k.y <= x) + (k.z <= x) + (k.w <= x);
    int64_t lb, ub;
    if ((rl & 3u) + cnt <= 8u) {
        const uint4 k2 = *reinterpret_cast<const uint4*>(sorted + a + 4);
        lb = int64_t(a) + lt0 + (k2.x < x) + (k2.y < x) + (k2.z < x) + (k2.w < x);
        ub = int64_t(a) + le0 + (k2.x <= x) + (k2.y <= x) + (k2.z <= x) + (k2.w <= x);
    } else {
        // <= 14 keys (a cell of 15+ keys marks the table skewed): counted one by one, so the order
        // of the keys inside the cell does not matter (the direct build orders the table by cell only)
        lb = rl;
        ub = rl;
        for (unsigned j = rl; j < rl + cnt; ++j) {
            const unsigned v = sorted[j];
            lb += v < x;
            ub += v <= x;
        }
    }
    const int64_t lbf = int64_t(a) + lt0, ubf = int64_t(a) + le0;
    w -= static_cast<unsigned long long>(ub - ubf);
    t += static_cast<unsigned long long>((ub - lb) - (ubf - lbf));
}

// SLOT: keys 8 .. cnt - 1 of cell c (its tertiary run), counted one by one after the two windows
// counted the first 8: W += M - ub loses the run's keys <= x, T gains its keys == x
__device__ __forceinline__ void slot_tertiary(unsigned x, unsigned c, unsigned cnt, const unsigned* __restrict__ tab,
                                              unsigned cells, unsigned long long& w, unsigned long long& t) {
    const unsigned* r = tab + slot_ter(cells, c);
    for (unsigned j = 0; j + 8u < cnt; ++j) {
        const unsigned v = r[j];
        w -= v <= x;
        t += (v <= x) - (v < x);
    }
}

// The labeled query pass over the count index (same stream and checks as query_labeled_kernel);
// returns at once when the builder kept the tree, so it is enqueued unconditionally. Per
// iteration every slot's window loads are issued BEFORE the next iteration's stream loads:
// vmcnt retires loads in issue order, so a wait for a window would otherwise also wait out a
// streaming load's HBM latency. CHECK (the two-step evaluation): *check += #queries over [begin,
// end) (mod 2^32) -- also when the index is not used (the pass then only reads the range for it) --
// so the caller can compare the range's positives with the ones another rank compacted from it.
// The loop runs at the 128-VGPR bound of 4 waves per SIMD, so the query count rides in the high
// half of the non-finite counter (per lane both stay far below 2^16): no extra register.
//
// SLOT (round 6): the cell-slotted table of direct_count_slots_kernel<true> (count_index.h). `blkg`
// is then the raw per-cell byte counts (8 per block: the block words' size), turned into block words
// in LDS by the workgroup itself (each thread sums its run of 18 blocks, one workgroup scan, written
// back in place); `sorted` is the slotted table of `slot_cells` cells. A cell's keys are its primary
// window (+inf past its count), its secondary window past 4 keys and, past 8 (rare), its tertiary
// run: W += M - (rank_lo + #keys <= x), T += #(== x); no straddling windows.
#ifdef DAUC_TUNING
// tuning builds: DAUC_QUERY_ABL (timing ablations of the SLOT query pass; WRONG counts): 1 = no
// query loop (the prologue and the reduction only), 2 = the block words zeroed instead of loaded
// and converted (every cell empty: the loop's windows all read the +inf pad window), 3 = no
// end-of-kernel atomics, 4 = 1 + 3 (the prologue only)
__device__ int g_query_abl = 0;
#endif
// SEC (SLOT only; round 6): ONE secondary window per lane per group of 4 queries instead of one per
// query: cells of 5+ keys are ~0.6 % of the queries, so a lane loads the secondary window of its
// group's first such query (the +inf pad when there is none) with the group's primaries, and counts
// it with them; a second such query in the same group (~2e-4 of lane-groups) is counted at once.
// 12 fewer live VGPRs per group and ~69 fewer VALU per group.
template <typename LT, bool CHECK = false, bool SLOT = false, bool SEC = true>
__global__ __launch_bounds__(kQueryThreads) void query_ci_kernel(const float* __restrict__ s,
                                                                const LT* __restrict__ lab, int64_t begin,
                                                                int64_t end, unsigned* __restrict__ meta,
                                                                const uint2* __restrict__ l1g,
                                                                const uint2* __restrict__ blkg,
                                                                const unsigned* __restrict__ sorted, int64_t M,
                                                                unsigned long long* __restrict__ out,
                                                                unsigned long long* __restrict__ nonfinite,
                                                                unsigned* __restrict__ verdict,
                                                                const unsigned* __restrict__ grp,
                                                                const unsigned long long* __restrict__ Mp,
                                                                unsigned* __restrict__ check, unsigned slot_cells = 0u,
                                                                unsigned long long* __restrict__ red8 = nullptr) {
    const unsigned pad_word = 4u * slot_cells;  // SLOT: the all-+inf primary slot past the last cell
    // SLOT: the index's loads (the l1 plan, the byte counts of every block the workspace holds) are
    // issued BEFORE the meta words are read, so the prologue waits one round trip, not two (meta ->
    // block count -> loads); blocks past the count are loaded and never stored
    constexpr int kL1Per = kCiTop / kQueryThreads;                                 // 2
    constexpr int kBlkPer = (kCiMaxBlocks + kQueryThreads - 1) / kQueryThreads;  // 18
    uint2 pre_a[SLOT ? kL1Per : 1], pre_v[SLOT ? kBlkPer : 1];
    if constexpr (SLOT) {
#pragma unroll
        for (int j = 0; j < kL1Per; ++j) pre_a[j] = l1g[j * kQueryThreads + threadIdx.x];
#pragma unroll
        for (int j = 0; j < kBlkPer; ++j) {
            const int i = j * kQueryThreads + threadIdx.x;
            pre_v[j] = i < kCiMaxBlocks ? blkg[i] : uint2{0u, 0u};
        }
    }
    const bool in_use = count_index_in_use(meta);
    if (Mp != nullptr) M = static_cast<int64_t>(*Mp);  // the direct build: the table size on the device
    if constexpr (SLOT) {
        // the slotted state is consumed (read after every count-pass workgroup finished: stream order)
        if (blockIdx.x == 0 && threadIdx.x == 0) meta[kCiConsumed] = 1u;
    }
    // the end-of-kernel reduction's rows (W, T, #non-finite, CHECK: #queries); static LDS on top of
    // the index's 163,232 dynamic bytes: the 160 KB limit leaves room for 4 rows, no more
    __shared__ unsigned long long red[CHECK ? 4 : 3][kQueryThreads / kWave];
    if (verdict != nullptr && blockIdx.x == 0 && threadIdx.x == 0) *verdict = in_use ? 1u : 2u;
    if (!in_use) {
        if constexpr (CHECK) {
            // the consistency word and the finiteness of every query, whatever the table
            unsigned nf = 0u, chk = 0u;
            for (int64_t i = begin + int64_t(blockIdx.x) * kQueryThreads + threadIdx.x; i < end;
                 i += int64_t(gridDim.x) * kQueryThreads) {
                if (lab[i] != LT(1)) {
                    nf += !isfinite(s[i]);
                    chk += 1u;
                }
            }
            // one atomic per workgroup and word (per-wave atomics on one address serialise)
            const unsigned long long nfw = wave_sum(static_cast<unsigned long long>(nf));
            const unsigned long long ckw = wave_sum(static_cast<unsigned long long>(chk));
            if ((threadIdx.x & (kWave - 1)) == 0) {
                red[0][threadIdx.x / kWave] = nfw;
                red[1][threadIdx.x / kWave] = ckw;
            }
            __syncthreads();
            if (threadIdx.x == 0) {
                unsigned long long bn = 0, bc = 0;
                for (int i = 0; i < kQueryThreads / kWave; ++i) {
                    bn += red[0][i];
                    bc += red[1][i];
                }
                if (bn && nonfinite != nullptr) atomicAdd(nonfinite, bn);
                if (bc) atomicAdd(check, static_cast<unsigned>(bc));
            }
            return;
        }
        // no positives at all: nothing to count, but the queries are still checked for finiteness
        // (sklearn raises on a non-finite score before its one-class warning, _ranking.py:868-869)
        if (M == 0 && nonfinite != nullptr) {
            unsigned nf = 0;
            for (int64_t i = begin + int64_t(blockIdx.x) * kQueryThreads + threadIdx.x; i < end;
                 i += int64_t(gridDim.x) * kQueryThreads)
                nf += lab[i] != LT(1) && !isfinite(s[i]);
            const unsigned long long nfw = wave_sum(static_cast<unsigned long long>(nf));
            if ((threadIdx.x & (kWave - 1)) == 0 && nfw) atomicAdd(nonfinite, nfw);
        }
        return;
    }
    extern __shared__ uint2 ci_lds[];
    const int nb = static_cast<int>(meta[kCiBlocks]);
    uint2* l1 = ci_lds;          // [2048]
    uint2* blk = ci_lds + kCiTop;  // [nb]
    {
        // the index into LDS with every load of a thread in flight before its first LDS store (a
        // load-store loop waits out one L2 round trip per iteration: 18 of them per thread)
        uint2 a[kL1Per], v[kBlkPer];
#ifdef DAUC_TUNING
        const bool abl2 = SLOT && g_query_abl == 2;
#else
        constexpr bool abl2 = false;
#endif
        if constexpr (SLOT) {  // (loaded above)
#pragma unroll
            for (int j = 0; j < kL1Per; ++j) a[j] = pre_a[j];
#pragma unroll
            for (int j = 0; j < kBlkPer; ++j) v[j] = abl2 ? uint2{0u, 0u} : pre_v[j];
        } else {
#pragma unroll
            for (int j = 0; j < kL1Per; ++j) a[j] = l1g[j * kQueryThreads + threadIdx.x];
#pragma unroll
            for (int j = 0; j < kBlkPer; ++j) {
                const int i = j * kQueryThreads + threadIdx.x;
                v[j] = i < nb && !abl2 ? blkg[i] : uint2{0u, 0u};
            }
        }
        if (grp != nullptr) {
            // the direct build's block words hold prefixes within groups of 256 blocks: add the groups'
            unsigned* pre = reinterpret_cast<unsigned*>(blk + kCiMaxBlocks);
            group_prefix(grp, (nb + kDirectGroup - 1) / kDirectGroup, pre);
            __syncthreads();
#pragma unroll
            for (int j = 0; j < kBlkPer; ++j) v[j].x += pre[(j * kQueryThreads + threadIdx.x) / kDirectGroup];
        }
#pragma unroll
        for (int j = 0; j < kL1Per; ++j) l1[j * kQueryThreads + threadIdx.x] = a[j];
#pragma unroll
        for (int j = 0; j < kBlkPer; ++j) {
            const int i = j * kQueryThreads + threadIdx.x;
            if (i < nb) blk[i] = v[j];
        }
    }
    if constexpr (SLOT) {
        // byte counts -> block words {keys before the block, the 8 counts as nibbles}, in place:
        // thread t owns blocks [18 t, 18 t + 18); its run total, one workgroup scan, then each
        // block rewritten with its exclusive prefix (counts <= 14: a skewed table never gets here)
        constexpr int kOwn = (kCiMaxBlocks + kQueryThreads - 1) / kQueryThreads;  // 18
        __syncthreads();
        const int b0 = threadIdx.x * kOwn;
        unsigned run = 0u;
#pragma unroll
        for (int j = 0; j < kOwn; ++j) {
            if (b0 + j < nb) {
                const uint2 r = blk[b0 + j];
                run += __builtin_amdgcn_sad_u8(r.x, 0u, 0u) + __builtin_amdgcn_sad_u8(r.y, 0u, 0u);
            }
        }
        unsigned before = block_incl_scan1024<false>(run, reinterpret_cast<unsigned*>(&red[0][0])) - run;
#pragma unroll
        for (int j = 0; j < kOwn; ++j) {
            if (b0 + j < nb) {
                const uint2 r = blk[b0 + j];
                // bytes b0..b3 (each <= 14) -> nibbles: 0x0b3b2b1b0 per half
                const unsigned tl = (r.x & 0x000f000fu) | ((r.x >> 4) & 0x00f000f0u);
                const unsigned th = (r.y & 0x000f000fu) | ((r.y >> 4) & 0x00f000f0u);
                const unsigned nib = (tl & 0xffu) | ((tl >> 8) & 0xff00u) | ((th & 0xffu) << 16) | ((th >> 8) & 0xff00u) << 16;
                blk[b0 + j] = uint2{before, nib};
                before += __builtin_amdgcn_sad_u8(r.x, 0u, 0u) + __builtin_amdgcn_sad_u8(r.y, 0u, 0u);
            }
        }
    }
    __syncthreads();
    const unsigned M32 = static_cast<unsigned>(M);
    unsigned long long w = 0, t = 0;
    unsigned nf = 0;  // CHECK: + #queries << 16
#ifdef DAUC_TUNING
    if (SLOT && (g_query_abl == 1 || g_query_abl == 4)) end = begin;  // no queries: the prologue (+ reduction)
#endif
    const int64_t a0 = (begin + 3) & ~int64_t(3);
    const int64_t head = a0 < end ? a0 : end;
    const int64_t stride = int64_t(gridDim.x) * kQueryThreads;
    const int64_t tid = int64_t(blockIdx.x) * kQueryThreads + threadIdx.x;
    auto one = [&](int64_t i) {
        if (lab[i] != LT(1)) {
            nf += !isfinite(s[i]) + (CHECK ? 0x10000u : 0u);
            const unsigned x = key_fast(s[i]);
            if constexpr (SLOT) {
                const unsigned c = ci_cell(x, l1[x >> kCiLowBits]);
                unsigned rl, cnt;
                ci_decode(c, blk[c / kCiBlock], rl, cnt);
                const uint4 k = win_load(sorted + (cnt ? 4u * c : pad_word));
                const uint4 k2 = win_load(sorted + (cnt > 4u ? slot_sec(slot_cells, c) : pad_word));
                unsigned le, lt, le2, lt2;
                win_le_lt(k, x, le, lt);
                win_le_lt(k2, x, le2, lt2);
                w += M32 - (rl + le + le2);
                t += (le - lt) + (le2 - lt2);
                if (cnt > 8u) slot_tertiary(x, c, cnt, sorted, slot_cells, w, t);
            } else {
                unsigned rl, cnt, wl = 0u, tl = 0u;
                uint4 k;
                ci_locate(x, l1, blk, sorted, rl, cnt, k);
                const bool more = ci_count(x, true, rl, cnt, k, M32, wl, tl);
                w += wl;
                t += tl;
                if (more) ci_fix(x, rl, cnt, k, sorted, w, t);
            }
        }
    };
    for (int64_t i = begin + tid; i < head; i += stride) one(i);
    const int64_t nvec = end > head ? (end - head) / 4 : 0;
    const bool aligned = (reinterpret_cast<uintptr_t>(s + head) & 15u) == 0 &&
                         (reinterpret_cast<uintptr_t>(lab + head) & (4 * sizeof(LT) - 1)) == 0;
    if (aligned) {
        // Software-pipelined over groups of NQ queries (U float4 slots per thread): the LDS lookups
        // of group g run while group g-1's window loads and group g+1's stream loads are in
        // flight, and group g-1 is counted after group g's windows are issued. Per group, in
        // issue order: keys(g) [waits for the stream loads issued one group earlier], stream
        // loads of g+1, LDS lookups of g, window loads of g, count of g-1 [waits for the windows
        // issued one group earlier; the younger loads stay in flight: vmcnt retires in order].
        constexpr int U = 1;  // one float4 slot per lane per group (more slots spill registers)
        constexpr int NQ = 4 * U;
        const int64_t step = int64_t(U) * stride;
        // two sets of every per-group register (A and B, used alternately by an unrolled pair of
        // iterations): a loop that rotated one set into the other would copy loaded registers at
        // its back-edge, i.e. wait there for the loads it had just issued
        struct Stream {
            f32x4 f[U];
            LabelWords<LT> l[U];
        };
        // Every load of the loop is issued unconditionally (out-of-range slots re-read slot 0 and are
        // masked; a lane without a window reads the table's first one): a load under a branch
        // leaves the number of younger loads in flight unknown, and the compiler then waits with
        // vmcnt(0) -- for every load in flight -- instead of a counted wait.
        auto load = [&](Stream& sg, int64_t v0) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t v = v0 + int64_t(u) * stride;
                const int64_t i = head + (v < nvec ? v : 0) * 4;
                sg.f[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(s + i));
                sg.l[u].load(lab + i);
                if (v >= nvec) sg.l[u].set_positive();
            }
        };
        // one group in flight: its keys, rank_lo | count << 28 (rank_lo < 2^28: M <= 2^27 here),
        // window and query mask
        constexpr bool ONE2 = SLOT && SEC;  // one secondary window per lane per group (see SEC)
        struct Group {
            unsigned x[NQ], rc[NQ];
            uint4 k[NQ];
            uint4 k2[ONE2 ? 1 : NQ];  // the next window, for cells that run past the first
            unsigned xs;              // ONE2: the key of the query k2[0] belongs to
            unsigned use;             // bit q: query q counts; ONE2: bit 8 + q: q's cell has 5+ keys
        };
        auto keys = [&](Group& g, const Stream& sg) {
            g.use = 0u;
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const float f[4] = {sg.f[u].x, sg.f[u].y, sg.f[u].z, sg.f[u].w};
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const bool use = sg.l[u].not_positive(q);
                    g.use |= unsigned(use) << (4 * u + q);
                    g.x[4 * u + q] = key_fast(f[q]);
                    nf += use && !isfinite(f[q]);
                }
            }
            // (a slot past the end loads as positive: no use bit, so it counts no query)
            if constexpr (CHECK) nf += static_cast<unsigned>(__builtin_popcount(g.use)) << 16;
        };
        // phase by phase over the group, so that every query's LDS read of a phase is issued before
        // the first wait (a per-query chain with its conditional window load in between keeps the
        // compiler from interleaving the queries: one LDS round trip per read per query)
        auto locate_lds = [&](Group& g, unsigned (&c)[NQ]) {
            uint2 e[NQ];
#pragma unroll
            for (int q = 0; q < NQ; ++q) e[q] = l1[g.x[q] >> kCiLowBits];
#pragma unroll
            for (int q = 0; q < NQ; ++q) c[q] = ci_cell(g.x[q], e[q]);
            uint2 b[NQ];
#pragma unroll
            for (int q = 0; q < NQ; ++q) b[q] = blk[c[q] / kCiBlock];
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const unsigned sh = 4u * (c[q] % kCiBlock);
                const unsigned below = __builtin_amdgcn_ubfe(b[q].y, 0u, sh);
                const unsigned bytes = (below & 0x0f0f0f0fu) + ((below >> 4) & 0x0f0f0f0fu);
                const unsigned rl = b[q].x + __builtin_amdgcn_sad_u8(bytes, 0u, 0u);
                const unsigned cnt = __builtin_amdgcn_ubfe(b[q].y, sh, 4u);
                g.rc[q] = rl | (cnt << 28);
            }
        };
        // an aligned window of +inf keys (the table is padded with at least 8 past M): the lanes with
        // no window to gather read it, so their counts need no mask
        const unsigned padoff = SLOT ? pad_word : (M32 + 3u) & ~3u;
        auto locate_win = [&](Group& g, const unsigned (&c)[NQ]) {
            if constexpr (SLOT) {
                // the cell's primary window (its first 4 keys), and its secondary one past 4 keys
#pragma unroll
                for (int q = 0; q < NQ; ++q) {
                    const unsigned cnt = g.rc[q] >> 28;
                    g.k[q] = win_load(sorted + (cnt && ((g.use >> q) & 1u) ? 4u * c[q] : padoff));
                }
                if constexpr (ONE2) {
                    unsigned pend = 0u;
#pragma unroll
                    for (int q = 0; q < NQ; ++q) pend |= unsigned(((g.use >> q) & 1u) && (g.rc[q] >> 28) > 4u) << q;
                    unsigned xs = 0u, cs = 0u;
#pragma unroll
                    for (int q = NQ - 1; q >= 0; --q) {  // the lowest such query
                        xs = (pend >> q) & 1u ? g.x[q] : xs;
                        cs = (pend >> q) & 1u ? c[q] : cs;
                    }
                    g.xs = xs;
                    g.use |= pend << 8;
                    g.k2[0] = win_load(sorted + (pend ? slot_sec(slot_cells, cs) : padoff));
                } else {
#pragma unroll
                    for (int q = 0; q < NQ; ++q) {
                        const unsigned cnt = g.rc[q] >> 28;
                        g.k2[q] = win_load(sorted + (((g.use >> q) & 1u) && cnt > 4u ? slot_sec(slot_cells, c[q]) : padoff));
                    }
                }
                return;
            }
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const unsigned rl = g.rc[q] & 0x0fffffffu, cnt = g.rc[q] >> 28;
                g.k[q] = win_load(sorted + (cnt && ((g.use >> q) & 1u) ? rl & ~3u : padoff));
            }
            // A cell that runs past its first window ((rank_lo & 3) + count > 4: ~7 % of the queries
            // at 1.1 cells per key) also loads the next one here, in the same straight-line issue: as
            // a branch after the count it was waited for with vmcnt(0) -- every load in flight,
            // the stream's included -- in nearly every iteration of every wave. Lanes that do not
            // need it read the +inf window (one shared line).
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const unsigned rl = g.rc[q] & 0x0fffffffu, cnt = g.rc[q] >> 28;
                g.k2[q] = win_load(sorted + (((g.use >> q) & 1u) && (rl & 3u) + cnt > 4u ? (rl & ~3u) + 4u : padoff));
            }
        };
        auto locate = [&](Group& g) {
            unsigned c[NQ];
            locate_lds(g, c);
            locate_win(g, c);
        };
        // ONE2: the group's secondary window, for its first query whose cell has 5+ keys (whose
        // primary window's count lacks the keys past the 4th); any further such query of the group
        // (rare) gets its secondary window now
        auto count_sec = [&](const Group& g) {
            const unsigned pend = (g.use >> 8) & 0xfu;
            unsigned les, lts;
            win_le_lt(g.k2[0], g.xs, les, lts);
            const unsigned hm = 0u - min(pend, 1u);
            w -= static_cast<unsigned long long>(les & hm);
            t += (les - lts) & hm;
            const unsigned rest = pend & (pend - 1u);
            if (__ballot(rest != 0u) != 0ull) {
#pragma unroll
                for (int q = 0; q < NQ; ++q) {
                    if ((rest >> q) & 1u) {
                        const unsigned x = g.x[q];
                        const uint4 k2 = win_load(sorted + slot_sec(slot_cells, ci_cell(x, l1[x >> kCiLowBits])));
                        unsigned le2, lt2;
                        win_le_lt(k2, x, le2, lt2);
                        w -= le2;
                        t += le2 - lt2;
                    }
                }
            }
        };
        auto count = [&](const Group& g) {
            unsigned wl = 0u, tl = 0u;
            bool more8 = false;
            if constexpr (ONE2) count_sec(g);
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                // lb = base + #(window keys < x), ub = base + #(<= x): the first window's keys before
                // the cell are < x, after it > x (or the +inf window of a lane without keys); the
                // second window (the cell's rest and later cells, or +inf) adds its own counts.
                // W += M - ub, T += ub - lb, for the queries only (um)
                const unsigned x = g.x[q], rl = g.rc[q] & 0x0fffffffu, cnt = g.rc[q] >> 28;
                const unsigned um = 0u - ((g.use >> q) & 1u);
                // rl & ~3 when the cell has keys (its window starts at the aligned rank); SLOT: the
                // window holds exactly the cell's keys, then +inf
                const unsigned base = SLOT ? rl : rl & ~(min(cnt, 1u) * 3u);
                unsigned le, lt, le2 = 0u, lt2 = 0u;
                win_le_lt(g.k[q], x, le, lt);
                if constexpr (!ONE2) win_le_lt(g.k2[q], x, le2, lt2);
                wl += (M32 - (base + le + le2)) & um;
                tl += ((le - lt) + (le2 - lt2)) & um;
                more8 |= um && (SLOT ? cnt : (rl & 3u) + cnt) > 8u;
            }
            w += wl;
            t += tl;
            if (more8) {  // a cell of 6+ keys across both windows: rare (the nibble caps it at 14)
                if constexpr (SLOT) {  // a cell of 9+ keys: its tertiary run, key by key
#pragma unroll
                    for (int q = 0; q < NQ; ++q) {
                        const unsigned cnt = g.rc[q] >> 28;
                        if (((g.use >> q) & 1u) && cnt > 8u) {
                            const unsigned x = g.x[q];
                            slot_tertiary(x, ci_cell(x, l1[x >> kCiLowBits]), cnt, sorted, slot_cells, w, t);
                        }
                    }
                    return;
                }
#pragma unroll
                for (int q = 0; q < NQ; ++q) {
                    const unsigned rl = g.rc[q] & 0x0fffffffu, cnt = g.rc[q] >> 28;
                    if (((g.use >> q) & 1u) && (rl & 3u) + cnt > 8u) {
                        // undo the two windows' counts, then count the cell key by key (ci_fix)
                        const unsigned x = g.x[q];
                        const uint4 k2 = g.k2[ONE2 ? 0 : q];
                        w += (k2.x <= x) + (k2.y <= x) + (k2.z <= x) + (k2.w <= x);
                        t -= ((k2.x <= x) + (k2.y <= x) + (k2.z <= x) + (k2.w <= x)) -
                             ((k2.x < x) + (k2.y < x) + (k2.z < x) + (k2.w < x));
                        ci_fix(x, rl, cnt, g.k[q], sorted, w, t);
                    }
                }
            }
        };
        // per group g: keys(g) [its stream loads were issued D groups earlier], stream loads of
        // g + D into the buffer just read, LDS lookups + window loads of g, count of g - 1 [its
        // windows were issued one group earlier; the younger loads stay in flight: vmcnt retires
        // in order]. D stream buffers keep D groups of score/label loads in flight per lane: with
        // one (D = 1) a wave holds 20 B per lane in flight, 5 MB over the chip, which at HBM's
        // loaded latency caps the stream far below the bandwidth.
        // (round 6: D = 2 for the slotted form with a secondary window per query needs 128 VGPRs +
        // 144-200 B of scratch per lane; with SEC's one secondary window per group it fits in 119-123
        // VGPRs for 1- and 4-byte labels, but ran 0.3-0.5 % slower at 2^27 and the same at 2^24)
        constexpr int D = 1;
        // groups in flight (windows issued GD - 1 groups before their count; round 6 measured 3 with
        // SEC: 127-128 VGPRs, the same time as 2 -- more loads in flight do not help)
        constexpr int GD = 2;
        static_assert(GD == 2 || (GD == 3 && D == 1), "the pipeline's unroll");
        constexpr int L = GD == 3 ? 3 : D % 2 == 0 ? D : 2 * D;  // unroll: every buffer index compile-time
        Stream sbuf[D];
        Group gbuf[GD];
#pragma unroll
        for (int j = 0; j < D; ++j) load(sbuf[j], tid + int64_t(j) * step);
#pragma unroll
        for (int p = 0; p < GD - 1; ++p) {  // groups 0 .. GD - 2 located (a group past the end counts nothing)
            keys(gbuf[p], sbuf[p % D]);
            load(sbuf[p % D], tid + int64_t(p + D) * step);
            locate(gbuf[p]);
        }
        int64_t v = tid + int64_t(GD - 1) * step;
        for (;;) {
#pragma unroll
            for (int j = 0; j < L; ++j) {
                // group v sits in stream buffer (j + GD - 1) % D and group slot (j + GD - 1) % GD
                Group& gc = gbuf[(j + GD - 1) % GD];
                Group& gp = gbuf[j % GD];
                if (v >= nvec) {
#pragma unroll
                    for (int p = 0; p < GD - 1; ++p) count(gbuf[(j + p) % GD]);
                    goto ci_stream_done;
                }
                keys(gc, sbuf[(j + GD - 1) % D]);
                load(sbuf[(j + GD - 1) % D], v + int64_t(D) * step);
                asm volatile("" ::: "memory");  // the stream loads stay older than this group's windows
                locate(gc);
                count(gp);
                v += step;
            }
        }
    ci_stream_done:;
    } else {
        for (int64_t v = tid; v < nvec; v += stride)
            for (int q = 0; q < 4; ++q) one(head + v * 4 + q);
    }
    for (int64_t i = head + nvec * 4 + tid; i < end; i += stride) one(i);
    // one atomic per workgroup and word: per-wave atomics on one address serialise across the
    // XCDs (~15 ns each: 4096 of them cost ~60 us)
    w = wave_sum(w);
    t = wave_sum(t);
    const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
    unsigned long long ckw = 0;
    if constexpr (CHECK) {
        ckw = wave_sum(static_cast<unsigned long long>(nf >> 16));
        nf &= 0xffffu;
    }
    const unsigned long long nfw = wave_sum(static_cast<unsigned long long>(nf));
    if (lane == 0) {
        red[0][wid] = w;
        red[1][wid] = t;
        red[2][wid] = nfw;
        if constexpr (CHECK) red[CHECK ? 3 : 0][wid] = ckw;
    }
    __syncthreads();
#ifdef DAUC_TUNING
    if (SLOT && g_query_abl >= 3) return;  // no end-of-kernel atomics
#endif
    if (threadIdx.x == 0) {
        unsigned long long bw = 0, bt = 0, bn = 0, bc = 0;
        for (int i = 0; i < kQueryThreads / kWave; ++i) {
            bw += red[0][i];
            bt += red[1][i];
            bn += red[2][i];
            if constexpr (CHECK) bc += red[CHECK ? 3 : 0][i];
        }
        if (red8 == nullptr) {
            if (bw) atomicAdd(out + 0, bw);
            if (bt) atomicAdd(out + 1, bt);
            if (bn && nonfinite) atomicAdd(nonfinite, bn);
            if (CHECK && bc) atomicAdd(check, static_cast<unsigned>(bc));
        } else {
            // round 6 (the two-step's query pass): its workgroups finish together, and 3-4 atomics
            // each on the record's one line serialise (~8 us at 256 workgroups and 2^21 queries,
            // DAUC_QUERY_ABL 3; the one-call pass, 8x the queries per workgroup, measured 1 us
            // slower with the groups and keeps the plain atomics). Group g = blockIdx % 8 adds into
            // its own line of red8 (256 B apart; zeroed by the count pass before this launch), takes
            // the group's ticket after its adds are acknowledged, and the group's last arriver adds
            // the group's sums to the record: <= 8 atomics per record word, 8 chains in parallel
            const unsigned g = blockIdx.x & 7u;
            unsigned long long* L = red8 + 32u * g;
            if (bw) atomicAdd(L + 0, bw);
            if (bt) atomicAdd(L + 1, bt);
            if (bn) atomicAdd(L + 2, bn);
            if (CHECK && bc) atomicAdd(L + 3, bc);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const unsigned members = (gridDim.x - g + 7u) / 8u;
            const unsigned tk = __hip_atomic_fetch_add(reinterpret_cast<unsigned*>(L + 4), 1u, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT);
            if (tk == members - 1u) {
                const unsigned long long gw = __hip_atomic_load(L + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const unsigned long long gt = __hip_atomic_load(L + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const unsigned long long gn = __hip_atomic_load(L + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const unsigned long long gc =
                    CHECK ? __hip_atomic_load(L + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
                if (gw) atomicAdd(out + 0, gw);
                if (gt) atomicAdd(out + 1, gt);
                if (gn && nonfinite) atomicAdd(nonfinite, gn);
                if (CHECK && gc) atomicAdd(check, static_cast<unsigned>(gc));
            }
        }
    }
}

// ---- the count index built straight from the unsorted table (the one-call evaluation) -------
//
// The count index needs the table ordered by CELL only: ci_count and ci_fix count a cell's keys
// whatever their order (keys of earlier cells are < x, of later cells > x). So the one-call
// evaluation skips the radix sort and the tree: a top-bucket histogram, the plan, per-cell counts,
// the block words and their prefix, and a scatter of every key into its cell's range -- 6 small
// launches over the table instead of 8 sort launches + the tree + the 4-launch build behind a
// sort. The table is not sorted inside a cell, so the tree cannot fall back on it: when the plan
// or the block pass finds the table unusable (more than 1.5 keys per cell, a cell of 15+ keys)
// the query kernel reports it (*verdict = 2) and the caller re-runs the sorted path.
constexpr int64_t kCiCntWords = ((int64_t(kCiMaxCells) + 2) * 4 + 255) / 256 * 64;  // the cstart region
constexpr int kDirectPerThread = 8;

// top-bucket histogram (LDS, then one global add per used bucket; `hist` zeroed by the caller);
// also zeroes the per-cell counters the count pass adds into
// The table size M is read from the device (the compaction's count), so the whole build and query
// are enqueued without the host knowing M: the grids are sized for the index's capacity and loop.
__global__ __launch_bounds__(256) void direct_hist_kernel(const float* __restrict__ pos,
                                                          const unsigned long long* __restrict__ Mp,
                                                          unsigned* __restrict__ hist, unsigned* __restrict__ cnt,
                                                          int64_t ncnt) {
    const int64_t M = static_cast<int64_t>(*Mp);
    __shared__ unsigned h[kCiTop];
    for (int i = threadIdx.x; i < kCiTop; i += 256) h[i] = 0u;
    __syncthreads();
    const int64_t gid = int64_t(blockIdx.x) * 256 + threadIdx.x, stride = int64_t(gridDim.x) * 256;
    for (int64_t i = gid; i < ncnt; i += stride) cnt[i] = 0u;
    for (int64_t i = gid; i < M; i += stride) atomicAdd(&h[key_fast(pos[i]) >> kCiLowBits], 1u);
    __syncthreads();
    for (int i = threadIdx.x; i < kCiTop; i += 256)
        if (h[i]) atomicAdd(hist + i, h[i]);
}

// The slotted build's insertion (count_index.h), one key per live lane; every lane of the wave
// calls it. The key's rank in its cell is the byte its returning add on the cell's packed counter
// found (a wave whose keys all fall in one cell -- tie-heavy tables -- adds once and ranks its lanes
// itself); ranks 0-3 go to the primary window, 4-7 to the secondary, 8-13 to the tertiary run.
// Returns true for a key past 14 in its cell (the caller marks the index skewed; a byte past 255
// also carries into the next cell's counter: skewed anyway).
__device__ __forceinline__ bool slot_insert(unsigned x, unsigned c, bool live, unsigned* __restrict__ cnt,
                                            unsigned* __restrict__ stab, unsigned cells, int lane) {
    const unsigned long long act = __ballot(live);
    if (act == 0ull) return false;
    const int first = __ffsll(static_cast<long long>(act)) - 1;
    const unsigned cf = __shfl(c, first, kWave);
    unsigned rank = 0u;
    if (__ballot(live && c == cf) == act) {
        unsigned old = 0u;
        if (lane == first) old = atomicAdd(cnt + (cf >> 2), static_cast<unsigned>(__popcll(act)) << (8u * (cf & 3u)));
        old = __shfl(old, first, kWave);
        const unsigned below = static_cast<unsigned>(__popcll(act & (lane == 0 ? 0ull : (~0ull >> (kWave - lane)))));
        rank = ((old >> (8u * (cf & 3u))) & 0xffu) + below;
    } else if (live) {
        const unsigned old = atomicAdd(cnt + (c >> 2), 1u << (8u * (c & 3u)));
        rank = (old >> (8u * (c & 3u))) & 0xffu;
    }
    if (!live) return false;
    if (rank < 4u) stab[4u * c + rank] = x;
    else if (rank < 8u) stab[slot_sec(cells, c) + rank - 4u] = x;
    else if (rank < kSlotMaxKeys) stab[slot_ter(cells, c) + rank - 8u] = x;
    else return true;
    return false;
}

// The plan of ci_plan_kernel from the bucket sizes themselves, computed by EVERY workgroup of the
// count pass in LDS (2048 buckets, 8 per thread: cheaper than a one-workgroup launch between the
// histogram and the counts): C_t = ceil(n_t * num / M) cells per used bucket, num = min(cells left
// after one per used bucket, 2 M), the first cell of every bucket (ascending). Workgroup 0 also
// writes the plan and the verdict words for the later passes. Then the per-cell key counts (a wave
// whose keys all fall in one cell adds once: tie-heavy tables) and every key's cell.

// SLOT (round 6, the one-call evaluation's default): every key inserted into the cell-slotted
// table instead (slot_insert; the compaction prepared the table, the packed counters and meta).
template <bool SLOT = false>
__global__ __launch_bounds__(kDirectThreads) void direct_count_kernel(const float* __restrict__ pos, int64_t mcap,
                                                                      const unsigned* __restrict__ hist,
                                                                      uint2* __restrict__ l1g,
                                                                      unsigned* __restrict__ meta,
                                                                      unsigned* __restrict__ cnt,
                                                                      unsigned* __restrict__ cell,
                                                                      unsigned* __restrict__ stab = nullptr,
                                                                      unsigned slot_cells = 0u,
                                                                      const unsigned long long* __restrict__ Mp =
                                                                          nullptr) {
    static_assert(kCiTop == 8 * kDirectThreads, "eight top buckets per thread");
    __shared__ uint2 l1[kCiTop];
    __shared__ unsigned wtot[kDirectThreads / kWave];
    __shared__ unsigned totals[3];
    // Mp (round 6, the slotted one-call form): the compaction's P, which is the histogram's total
    // (every positive is in it) -- loaded with the histogram, so only the used buckets are summed
    // (eight ballots per wave, one LDS sum) and the plan needs one workgroup scan instead of three
    const unsigned long long Mdev = Mp != nullptr ? *Mp : 0ull;
    const uint4 h0 = reinterpret_cast<const uint4*>(hist)[2 * threadIdx.x];
    const uint4 h1 = reinterpret_cast<const uint4*>(hist)[2 * threadIdx.x + 1];
    const unsigned n[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
    int64_t M, used_total;
    if (Mp != nullptr) {  // (uniform)
        const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
        unsigned wu = 0u;
#pragma unroll
        for (int j = 0; j < 8; ++j) wu += static_cast<unsigned>(__popcll(__ballot(n[j] != 0u)));
        if (lane == 0) wtot[wid] = wu;
        __syncthreads();
        unsigned u = 0u;
#pragma unroll
        for (int w = 0; w < kDirectThreads / kWave; ++w) u += wtot[w];
        __syncthreads();  // (wtot is the next scan's)
        M = static_cast<int64_t>(Mdev);
        used_total = u;
    } else {
        unsigned used = 0u, keys = 0u;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            used += n[j] != 0u;
            keys += n[j];
        }
        used = block_incl_scan1024<false>(used, wtot);
        if (threadIdx.x == kDirectThreads - 1) totals[0] = used;
        keys = block_incl_scan1024<false>(keys, wtot);  // M = the histogram's total (< 2^32: M <= n / 2)
        if (threadIdx.x == kDirectThreads - 1) totals[2] = keys;
        __syncthreads();
        M = totals[2];
        used_total = totals[0];
    }
    const int64_t avail = int64_t(kCiMaxCells) - used_total;
    const int64_t num = avail < 2 * M ? avail : 2 * M;
    unsigned C[8], csum = 0u;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        C[j] = n[j] ? static_cast<unsigned>((int64_t(n[j]) * num + M - 1) / M) : 0u;
        csum += C[j];
    }
    const unsigned incl = block_incl_scan1024<false>(csum, wtot);
    if (threadIdx.x == kDirectThreads - 1) totals[1] = incl;
    unsigned run = incl - csum;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        l1[8 * threadIdx.x + j] = uint2{run, C[j]};
        run += C[j];
    }
    __syncthreads();
    const unsigned total = totals[1];
    // usable: at most 1.5 keys per cell, and the table fits the workspace (M <= mcap)
    const bool ok = num > 0 && 3 * num >= 2 * M && total <= static_cast<unsigned>(kCiMaxCells) && M <= mcap;
    if (blockIdx.x == 0) {
        for (int t = threadIdx.x; t < kCiTop; t += kDirectThreads) l1g[t] = l1[t];
        // SLOT: `cell` is unused as such; it holds the query pass's 8 group lines (query_ci_kernel's
        // red8: 2 KB), zeroed here, before that launch
        if (SLOT && cell != nullptr && threadIdx.x < 256)
            reinterpret_cast<unsigned long long*>(cell)[threadIdx.x] = 0ull;
        if (threadIdx.x == 0) {
            meta[kCiOk] = ok ? 1u : 0u;
            meta[kCiCells] = total;
            meta[kCiBlocks] = (total + 1 + kCiBlock - 1) / kCiBlock;
            if constexpr (!SLOT) meta[kCiSkew] = 0u;  // SLOT: zeroed by the compaction (set by any workgroup)
        }
    }
    if (!ok) return;
    const int lane = threadIdx.x & (kWave - 1);
    if constexpr (SLOT) {
        bool skew = false;
        for (int64_t i0 = int64_t(blockIdx.x) * kDirectThreads; i0 < M; i0 += int64_t(gridDim.x) * kDirectThreads) {
            const int64_t i = i0 + threadIdx.x;
            const bool live = i < M;
            unsigned x = 0u, c = 0u;
            if (live) {
                x = key_fast(pos[i]);
                c = ci_cell(x, l1[x >> kCiLowBits]);
            }
            skew |= slot_insert(x, c, live, cnt, stab, slot_cells, lane);
        }
        if (__ballot(skew) != 0ull && lane == 0) atomicOr(meta + kCiSkew, 1u);
        return;
    }
    for (int64_t i0 = int64_t(blockIdx.x) * kDirectThreads; i0 < M; i0 += int64_t(gridDim.x) * kDirectThreads) {
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

// The two-step evaluation's count pass straight from the gathered slots (the gather copy folded
// in): every workgroup sums the slots' headers (wave 0: the stored scores' prefix per slot) and
// their histograms (two top buckets per thread), computes the plan as direct_count_kernel does,
// and counts its keys -- each key read from its slot, copied to the table position array `pos`
// (the scatter's input) with its cell. Workgroup 0 also writes the plan, the verdict words, the
// part's record (counts zeroed, P, the check word, the label counts) and m_eff (P, or past the
// index's capacity when a slot overflowed, so the plan refuses the table: verdict 2).
//
// SLOT (round 6, the two-step evaluation's default): the cell-slotted table instead (count_index.h:
// primary / secondary windows +inf filled by the compaction of step 1, a tertiary run), the per-cell
// counters bytes packed four to a word (zeroed by that compaction too), and each key inserted
// straight into its cell: its rank in the cell is the byte its returning atomic add found. No
// position array, no cell array, no block pass and no scatter: the query pass turns the byte counts
// into the block words itself (query_ci_kernel<.., SLOT>). A cell of 15+ keys marks the index skewed
// (verdict 2: the caller's sorted path), as in the direct build; meta[kCiSkew] was zeroed by the
// compaction, because this pass's workgroups set it while workgroup 0 writes the other meta words.
constexpr int kSlotCountThreads = 1024;
template <bool SLOT = false>
__global__ __launch_bounds__(kSlotCountThreads) void direct_count_slots_kernel(SlotSource src, int64_t mcap,
                                                                              uint2* __restrict__ l1g,
                                                                              unsigned* __restrict__ meta,
                                                                              unsigned* __restrict__ cnt,
                                                                              unsigned* __restrict__ cell,
                                                                              float* __restrict__ pos,
                                                                              unsigned* __restrict__ stab,
                                                                              unsigned slot_cells) {
    static_assert(kCiTop == 2 * kSlotCountThreads, "two top buckets per thread");
    __shared__ uint2 l1[kCiTop];
    __shared__ unsigned wtot[kSlotCountThreads / kWave];
    __shared__ unsigned totals[3];
    __shared__ unsigned long long off[kMaxSlotParts + 1];  // stored scores before slot r
    __shared__ unsigned long long hs[5];                   // P, #non-finite, #other, overflow, check
    const int parts = src.parts;
    const int lane = threadIdx.x & (kWave - 1);
    auto hdr = [&](int r) { return reinterpret_cast<const unsigned long long*>(src.slots + size_t(r) * src.sbytes); };
    const unsigned long long cap = static_cast<unsigned long long>(src.cap);
    // the summed histogram: buckets 2t, 2t + 1 -- every slot's load issued before the header work
    // (8 loads in flight per thread: one L2 round trip, not one per slot)
    unsigned n0 = 0u, n1 = 0u;
    {
        const uint2* hp = reinterpret_cast<const uint2*>(src.slots + src.hist_off) + threadIdx.x;
        const size_t sw = src.sbytes / sizeof(uint2);
        int r = 0;
        for (; r + 8 <= parts; r += 8) {
            uint2 v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = hp[size_t(r + j) * sw];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                n0 += v[j].x;
                n1 += v[j].y;
            }
        }
        for (; r < parts; ++r) {
            const uint2 v = hp[size_t(r) * sw];
            n0 += v.x;
            n1 += v.y;
        }
    }
    if (threadIdx.x < kWave) {
        unsigned long long run = 0, P = 0, nf = 0, other = 0, mism = 0;
        bool over = false;
        for (int r0 = 0; r0 < parts; r0 += kWave) {
            const int r = r0 + lane;
            unsigned long long stored = 0;
            if (r < parts) {
                const unsigned long long* h = hdr(r);
                const unsigned long long pr = h[0];
                P += pr;
                nf += h[2];
                other += h[3];
                mism += h[4] != static_cast<unsigned long long>(src.n);
                over |= pr > cap;
                stored = pr < cap ? pr : cap;
            }
            unsigned long long inc = stored;
#pragma unroll
            for (int d = 1; d < kWave; d <<= 1) {
                const unsigned long long t = __shfl_up(inc, d, kWave);
                if (lane >= d) inc += t;
            }
            if (r < parts) off[r] = run + inc - stored;
            run += __shfl(inc, kWave - 1, kWave);
        }
        P = wave_sum(P);
        nf = wave_sum(nf);
        other = wave_sum(other);
        mism = wave_sum(mism);
        over = __ballot(over) != 0ull;
        if (lane == 0) {
            off[parts] = run;
            hs[0] = P;
            hs[1] = nf;
            hs[2] = other;
            hs[3] = over ? 1ull : 0ull;
            // the check word: the queried slot's P - the range length (low half, mod 2^32; the
            // query pass adds its queries), the slots built for another n (high half)
            const unsigned long long* q = hdr((src.part + 1) % parts);
            const unsigned lo = static_cast<unsigned>(q[0]) - static_cast<unsigned>(src.qlen);
            hs[4] = (mism << 32) | lo;
        }
    }
    __syncthreads();  // (an overflow adds past-capacity keys to bucket 0)
    // SLOT: this thread's first key is loaded now, so its latency overlaps the plan's three scans
    // (one key per thread: the grid covers the index's capacity)
    const int64_t i_first = int64_t(blockIdx.x) * kSlotCountThreads + threadIdx.x;
    float v_first = 0.0f;
    if constexpr (SLOT) {
        if (hs[3] == 0ull && i_first < static_cast<int64_t>(hs[0])) {
            int lo = 0, hi = parts;
            while (hi - lo > 1) {
                const int mid = (lo + hi) >> 1;
                if (off[mid] <= static_cast<unsigned long long>(i_first)) lo = mid;
                else hi = mid;
            }
            v_first = reinterpret_cast<const float*>(src.slots + size_t(lo) * src.sbytes + src.data_off)
                [i_first - static_cast<int64_t>(off[lo])];
        }
    }
    const bool over = hs[3] != 0ull;
    if (threadIdx.x == 0 && over) n0 += static_cast<unsigned>(mcap) + 1u;
    // round 6: only the totals of the used buckets and of the keys are needed, not their scans: the
    // used buckets by two ballots per wave and one LDS sum, and the keys = the slots' P (every
    // positive is in its slot's histogram, stored or not; an overflow adds the past-capacity count,
    // as the overflow bucket did, so the plan refuses the table) -- two workgroup scans fewer
    {
        const int wid = threadIdx.x / kWave;
        const unsigned wu = static_cast<unsigned>(__popcll(__ballot(n0 != 0u)) + __popcll(__ballot(n1 != 0u)));
        if (lane == 0) wtot[wid] = wu;
    }
    __syncthreads();
    unsigned used_total = 0u;
#pragma unroll
    for (int w = 0; w < kSlotCountThreads / kWave; ++w) used_total += wtot[w];
    __syncthreads();  // (wtot is the next scan's)
    const int64_t M = static_cast<int64_t>(hs[0]) + (over ? mcap + 1 : 0);
    const int64_t avail = int64_t(kCiMaxCells) - int64_t(used_total);
    const int64_t num = avail < 2 * M ? avail : 2 * M;
    const unsigned C0 = n0 ? static_cast<unsigned>((int64_t(n0) * num + M - 1) / M) : 0u;
    const unsigned C1 = n1 ? static_cast<unsigned>((int64_t(n1) * num + M - 1) / M) : 0u;
    const unsigned incl = block_incl_scan1024<false>(C0 + C1, wtot);
    if (threadIdx.x == kSlotCountThreads - 1) totals[1] = incl;
    const unsigned run = incl - (C0 + C1);
    l1[2 * threadIdx.x] = uint2{run, C0};
    l1[2 * threadIdx.x + 1] = uint2{run + C0, C1};
    __syncthreads();
    const unsigned total = totals[1];
    const bool ok = num > 0 && 3 * num >= 2 * M && total <= static_cast<unsigned>(kCiMaxCells) && M <= mcap;
    const unsigned long long P = hs[0];
    if (blockIdx.x == 0) {
        l1g[2 * threadIdx.x] = l1[2 * threadIdx.x];
        l1g[2 * threadIdx.x + 1] = l1[2 * threadIdx.x + 1];
        // SLOT: `cell` holds the query pass's 8 group lines (query_ci_kernel's red8), zeroed here
        if (SLOT && cell != nullptr && threadIdx.x < 256)
            reinterpret_cast<unsigned long long*>(cell)[threadIdx.x] = 0ull;
        if (threadIdx.x == 0) {
            meta[kCiOk] = ok ? 1u : 0u;
            meta[kCiCells] = total;
            meta[kCiBlocks] = (total + 1 + kCiBlock - 1) / kCiBlock;
            if constexpr (!SLOT) meta[kCiSkew] = 0u;  // SLOT: zeroed by the compaction (see above)
            *src.m_eff = over ? static_cast<unsigned long long>(mcap) + 1ull : P;
        } else if (threadIdx.x < 4) {
            src.wt[threadIdx.x - 1] = 0ull;
        } else if (threadIdx.x == 4) {
            *src.verdict = 0ull;
        } else if (threadIdx.x < 9) {
            const int k = threadIdx.x - 5;  // stats: P, check, #non-finite, #other
            src.stats[k] = k == 0 ? P : k == 1 ? hs[4] : hs[k - 1];  // hs: P, #non-finite, #other, .., check
        }
    }
    if (!ok) return;
    const int64_t Mk = static_cast<int64_t>(P);  // no overflow here: every positive is stored
    if constexpr (SLOT) {
        // step 2 again on the same step-1 state: the counters and slots already hold the keys, so
        // inserting them twice would double every count -- refuse the index instead (verdict 2:
        // the caller's sorted path gives the exact integers)
        if (meta[kCiConsumed] != 0u) {
            if (threadIdx.x == 0) atomicOr(meta + kCiSkew, 1u);
            return;
        }
        bool skew = false;
        for (int64_t i0 = int64_t(blockIdx.x) * kSlotCountThreads; i0 < Mk;
             i0 += int64_t(gridDim.x) * kSlotCountThreads) {
            const int64_t i = i0 + threadIdx.x;
            const bool live = i < Mk;
            unsigned x = 0u, c = 0u;
            if (live) {
                float v = v_first;
                if (i != i_first) {  // past the first key (a grid smaller than the table)
                    int lo = 0, hi = parts;
                    while (hi - lo > 1) {
                        const int mid = (lo + hi) >> 1;
                        if (off[mid] <= static_cast<unsigned long long>(i)) lo = mid;
                        else hi = mid;
                    }
                    v = reinterpret_cast<const float*>(src.slots + size_t(lo) * src.sbytes + src.data_off)
                        [i - static_cast<int64_t>(off[lo])];
                }
                x = key_fast(v);
                c = ci_cell(x, l1[x >> kCiLowBits]);
            }
            skew |= slot_insert(x, c, live, cnt, stab, slot_cells, lane);
        }
        if (__ballot(skew) != 0ull && lane == 0) atomicOr(meta + kCiSkew, 1u);
        return;
    }
    for (int64_t i0 = int64_t(blockIdx.x) * kSlotCountThreads; i0 < Mk;
         i0 += int64_t(gridDim.x) * kSlotCountThreads) {
        const int64_t i = i0 + threadIdx.x;
        const bool live = i < Mk;
        unsigned c = 0u;
        if (live) {
            // the slot holding key i: the last r with off[r] <= i (binary search over the prefix)
            int lo = 0, hi = parts;  // off[lo] <= i < off[hi]
            while (hi - lo > 1) {
                const int mid = (lo + hi) >> 1;
                if (off[mid] <= static_cast<unsigned long long>(i)) lo = mid;
                else hi = mid;
            }
            const float v = reinterpret_cast<const float*>(src.slots + size_t(lo) * src.sbytes + src.data_off)
                [i - static_cast<int64_t>(off[lo])];
            pos[i] = v;
            const unsigned x = key_fast(v);
            c = ci_cell(x, l1[x >> kCiLowBits]);
            cell[i] = c;
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

// One thread per block of 8 cells, one workgroup per group of 256 blocks: blk[b] = {the table
// keys before block b within its group, the 8 cells' counts as nibbles}, grp[g] = the group's
// keys; a count of 15 or more marks the table skewed. The consumers add the groups' prefix
// (group_prefix), so no one-workgroup scan launch sits between this pass and the scatter.
__global__ __launch_bounds__(kDirectGroup) void direct_blocks_kernel(const unsigned* __restrict__ cnt,
                                                                     unsigned* __restrict__ meta,
                                                                     uint2* __restrict__ blk,
                                                                     unsigned* __restrict__ grp) {
    if (meta[kCiOk] == 0u) return;
    __shared__ unsigned wtot[kDirectGroup / kWave];
    const int b = blockIdx.x * kDirectGroup + threadIdx.x;
    const bool live = b < static_cast<int>(meta[kCiBlocks]);
    bool skew = false;
    unsigned w = 0u, sum = 0u;
    if (live) {
        const uint4 lo = reinterpret_cast<const uint4*>(cnt)[2 * b], hi = reinterpret_cast<const uint4*>(cnt)[2 * b + 1];
        const unsigned c[kCiBlock] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
#pragma unroll
        for (int j = 0; j < kCiBlock; ++j) {
            skew |= c[j] >= 15u;
            w |= (c[j] < 15u ? c[j] : 15u) << (4 * j);
            sum += c[j];
        }
    }
    const unsigned incl = block_incl_scan1024<false>(sum, wtot);
    if (live) blk[b] = uint2{incl - sum, w};
    if (threadIdx.x == kDirectGroup - 1) grp[blockIdx.x] = incl;
    if (__ballot(skew) != 0ull && (threadIdx.x & (kWave - 1)) == 0) atomicOr(meta + kCiSkew, 1u);
}

// every key into its cell's range of the table (the counters are counted back down to zero);
// the table's tail is padded with +inf keys for the 16-byte windows
__global__ __launch_bounds__(kDirectThreads) void direct_scatter_kernel(const float* __restrict__ pos,
                                                                        const unsigned long long* __restrict__ Mp,
                                                                        const uint2* __restrict__ blk,
                                                                        const unsigned* __restrict__ grp,
                                                                        unsigned* __restrict__ meta,
                                                                        unsigned* __restrict__ cnt,
                                                                        const unsigned* __restrict__ cell,
                                                                        unsigned* __restrict__ table,
                                                                        int64_t ncnt) {
    if (meta[kCiOk] == 0u) return;  // nothing was counted: the counters are still zero
    if (meta[kCiSkew] != 0u) {
        // a skewed table: no scatter, but the counters go back to zero for the next build (the
        // scatter of a good build counts them down to zero itself)
        for (int64_t i = int64_t(blockIdx.x) * kDirectThreads + threadIdx.x; i < ncnt;
             i += int64_t(gridDim.x) * kDirectThreads)
            cnt[i] = 0u;
        return;
    }
    const int64_t M = static_cast<int64_t>(*Mp);
    __shared__ unsigned pre[kDirectMaxGroups];
    group_prefix(grp, (static_cast<int>(meta[kCiBlocks]) + kDirectGroup - 1) / kDirectGroup, pre);
    __syncthreads();
    const int64_t gid = int64_t(blockIdx.x) * kDirectThreads + threadIdx.x;
    if (gid < 16) table[M + gid] = kPadKey;
    // Every index is checked before it is used (a producer bug must become a verdict-2 fallback,
    // never an out-of-bounds store): the cell must be one of the plan's, and its counter must still
    // hold a slot (the count pass counted exactly this many keys into it). A failed check marks the
    // index skewed, so the query passes return at once and the caller takes the sorted path.
    const unsigned ncells = meta[kCiCells];
    bool bad = false;
    for (int64_t i = gid; i < M; i += int64_t(gridDim.x) * kDirectThreads) {
        const unsigned x = key_fast(pos[i]);
        const unsigned c = cell[i];
        if (c >= ncells) {
            bad = true;
            continue;
        }
        const unsigned bi = c / kCiBlock;
        unsigned rl, ccount;
        ci_decode(c, blk[bi], rl, ccount);
        const unsigned left = atomicSub(cnt + c, 1u);  // slots of the cell not yet taken, before this one
        if (left == 0u || left > ccount) {
            bad = true;
            continue;
        }
        const unsigned pos_in_table = pre[bi / kDirectGroup] + rl + (left - 1u);
        if (pos_in_table >= static_cast<unsigned>(M)) {
            bad = true;
            continue;
        }
        table[pos_in_table] = x;
    }
    if (__ballot(bad) != 0ull && (threadIdx.x & (kWave - 1)) == 0) atomicOr(meta + kCiSkew, 1u);
}

// Every queried score is also checked to be finite (sklearn rejects NaN / inf scores,
// _ranking.py:868-869): nonfinite (nullable) += #queried non-finite scores. The negatives are
// never materialised, so this is the only pass that reads their scores. With a cell index
// built (meta != nullptr) the kernel returns at once unless the builder kept the tree.
template <int K, typename LT>
__global__ __launch_bounds__(kQueryThreads) void query_labeled_kernel(const float* __restrict__ s,
                                                                     const LT* __restrict__ lab, int64_t begin,
                                                                     int64_t end, const TreeNode* __restrict__ gtree,
                                                                     TreeGeom g, int k,
                                                                     const unsigned* __restrict__ sorted,
                                                                     int64_t M, unsigned long long* __restrict__ out,
                                                                     unsigned long long* __restrict__ nonfinite,
                                                                     const unsigned* __restrict__ meta,
                                                                     const unsigned* __restrict__ dk_meta) {
    // meta: the count index's builder verdict, dk_meta the distinct-key index's (the tree runs only
    // when neither is used)
    if (meta != nullptr && count_index_in_use(meta)) return;
    if (dk_meta != nullptr && dk_meta[kDkUse] != 0u) return;
    extern __shared__ TreeNode tree[];
    for (int i = threadIdx.x; i < g.nodes; i += kQueryThreads) tree[i] = gtree[i];
    const TopKeys top = load_top(gtree, g, sorted, k);
    __syncthreads();
    unsigned long long w = 0, t = 0;
    unsigned nf = 0;
    // scalar head up to a 4-element boundary, then float4 slots, then the scalar tail
    const int64_t a0 = (begin + 3) & ~int64_t(3);
    const int64_t head = a0 < end ? a0 : end;
    const int64_t stride = int64_t(gridDim.x) * kQueryThreads;
    const int64_t tid = int64_t(blockIdx.x) * kQueryThreads + threadIdx.x;
    for (int64_t i = begin + tid; i < head; i += stride) {
        if (lab[i] != LT(1)) {
            nf += !isfinite(s[i]);
            count_query<K, true>(key_of(s[i]), tree, g, top, k, sorted, M, w, t);
        }
    }
    const int64_t nvec = end > head ? (end - head) / 4 : 0;
    const bool aligned = (reinterpret_cast<uintptr_t>(s + head) & 15u) == 0 &&
                         (reinterpret_cast<uintptr_t>(lab + head) & (4 * sizeof(LT) - 1)) == 0;
    if (aligned) {
        // U float4 slots (4 queries each) per iteration, and the NEXT iteration's loads issued
        // before this one's walks: each walk is a chain of dependent LDS reads and a bucket load,
        // so without this the stream's HBM latency sits between every two iterations of a wave.
        // slots per iteration (prefetched one iteration ahead): register-bound
        constexpr int U = sizeof(LT) == 8 ? 2 : 4;
        f32x4 fc[U], fn[U];
        LabelWords<LT> lc[U], ln[U];
        auto load = [&](int64_t v0, f32x4 (&f)[U], LabelWords<LT> (&l)[U]) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t v = v0 + int64_t(u) * stride;
                if (v < nvec) {
                    const int64_t i = head + v * 4;
                    f[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(s + i));
                    l[u].load(lab + i);
                } else {
                    f[u] = f32x4{0.f, 0.f, 0.f, 0.f};
                    l[u].set_positive();  // past the end: no query
                }
            }
        };
        load(tid, fc, lc);
        for (int64_t v0 = tid; v0 < nvec; v0 += int64_t(U) * stride) {
            auto keys = [&](int u, unsigned (&x)[4], bool (&neg)[4]) {
                const float f[4] = {fc[u].x, fc[u].y, fc[u].z, fc[u].w};
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    neg[q] = lc[u].not_positive(q);
                    x[q] = key_of(f[q]);
                    nf += neg[q] && !isfinite(f[q]);
                }
            };
            load(v0 + int64_t(U) * stride, fn, ln);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                bool neg[4];
                unsigned x[4];
                keys(u, x, neg);
                count4<K, true>(x, neg, tree, g, top, k, sorted, M, w, t);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                fc[u] = fn[u];
                lc[u] = ln[u];
            }
        }
    } else {
        for (int64_t v = tid; v < nvec; v += stride) {
            const int64_t i = head + v * 4;
            float f[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) f[q] = s[i + q];
            bool neg[4];
            label4(lab, i, false, end, neg);
            unsigned x[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                x[q] = key_of(f[q]);
                nf += neg[q] && !isfinite(f[q]);
            }
            count4<K, true>(x, neg, tree, g, top, k, sorted, M, w, t);
        }
    }
    for (int64_t i = head + nvec * 4 + tid; i < end; i += stride) {
        if (lab[i] != LT(1)) {
            nf += !isfinite(s[i]);
            count_query<K, true>(key_of(s[i]), tree, g, top, k, sorted, M, w, t);
        }
    }
    __shared__ unsigned long long red[3][kQueryThreads / kWave];
    w = wave_sum(w);
    t = wave_sum(t);
    const unsigned long long nfw = wave_sum(static_cast<unsigned long long>(nf));
    const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
    if (lane == 0) {
        red[0][wid] = w;
        red[1][wid] = t;
        red[2][wid] = nfw;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long bw = 0, bt = 0, bn = 0;
        for (int i = 0; i < kQueryThreads / kWave; ++i) {
            bw += red[0][i];
            bt += red[1][i];
            bn += red[2][i];
        }
        if (bw) atomicAdd(out + 0, bw);
        if (bt) atomicAdd(out + 1, bt);
        if (bn && nonfinite) atomicAdd(nonfinite, bn);
    }
}

// ---- distinct-key index: tie-heavy tables (round 6) ---------------------------------------------
//
// The count index refuses a table whose cells hold 15+ keys. In practice that is a table of FEW
// DISTINCT values -- rounded scores, or the probabilities of a bf16 model (2^27 @ 0.1 % rounded to
// bf16: 134,447 positives on 1,329 values) -- whose equal keys no cell split can separate, and the
// tree it fell back to ran 1.05 ms at 2^27 (vs 0.47 ms for the index on spread scores). Its distinct
// keys, each with the number of table keys <= it (cum), answer a query exactly: #(table <= x) = the
// cum of the last distinct key <= x, #(== x) = that cum minus the previous one when the key IS x.
// Up to kDkMax distinct keys the whole structure fits the query's LDS: the count index's top-bucket
// plan over the distinct keys (l1, 16 KB), one word per cell {first distinct key, distinct keys in
// the cell} (2 cells per distinct key: <= 72 KB), and {key, cum} per distinct key (<= 64 KB). A
// query is then 3 dependent LDS reads -- l1, its cell word, the two entries at the cell's start --
// and no table gather at all; a cell of 2+ distinct keys (rare) adds a binary search over them.
// Built behind prepare_count from the sorted table in 4 small launches (mark, scan, write, index),
// every one deciding on the device (the count index in use: they return at once; more than kDkMax
// distinct keys: the tree runs), so the sorted path still needs no host readback. Round 6.
// the tile's 4 keys per thread and whether each is the LAST copy of its key (the table is +inf
// padded past M, and no finite key is +inf's)
__device__ __forceinline__ unsigned dk_flags(const unsigned* __restrict__ sorted, int64_t M, int64_t i0,
                                             unsigned (&k)[4]) {
    unsigned f = 0u;
#pragma unroll
    for (int j = 0; j < 4; ++j) k[j] = i0 + j < M ? sorted[i0 + j] : kPadKey;
    const unsigned nxt = i0 + 4 < M ? sorted[i0 + 4] : kPadKey;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const unsigned after = j < 3 ? k[j + 1] : nxt;
        f |= unsigned(i0 + j < M && k[j] != after) << j;
    }
    return f;
}

__global__ __launch_bounds__(kDkTile / 4) void dk_mark_kernel(const unsigned* __restrict__ sorted, int64_t M,
                                                              const unsigned* __restrict__ ci_meta,
                                                              unsigned* __restrict__ tcnt) {
    if (dk_ci_in_use(ci_meta)) return;
    __shared__ unsigned wsum[kDkTile / 4 / kWave];
    unsigned k[4];
    const unsigned f = dk_flags(sorted, M, int64_t(blockIdx.x) * kDkTile + 4 * int64_t(threadIdx.x), k);
    unsigned c = static_cast<unsigned>(__popc(f));
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, kWave);
    if ((threadIdx.x & (kWave - 1)) == 0) wsum[threadIdx.x / kWave] = c;
    __syncthreads();
    if (threadIdx.x == 0) tcnt[blockIdx.x] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
}

// one workgroup: the tiles' exclusive prefix in place, D, and whether the index is used
__global__ __launch_bounds__(kDkScanThreads) void dk_scan_kernel(const unsigned* __restrict__ ci_meta, DkWs dk,
                                                                 int64_t ntiles) {
    if (dk_ci_in_use(ci_meta)) return;
    __shared__ unsigned wtot[kDkScanThreads / kWave];
    const int64_t per = (ntiles + kDkScanThreads - 1) / kDkScanThreads;
    const int64_t t0 = int64_t(threadIdx.x) * per, t1 = t0 + per < ntiles ? t0 + per : ntiles;
    unsigned long long mine = 0;
    for (int64_t t = t0; t < t1; ++t) mine += dk.tcnt[t];
    // a thread's run past kDkMax: saturated (the total is then past it too, and nothing else is read)
    const unsigned m = mine > unsigned(kDkMax) ? unsigned(kDkMax) + 1u : static_cast<unsigned>(mine);
    const unsigned incl = block_incl_scan1024<false>(m, wtot);
    unsigned run = incl - m;
    for (int64_t t = t0; t < t1; ++t) {
        const unsigned c = dk.tcnt[t];
        dk.tcnt[t] = run;
        run += c;
    }
    if (threadIdx.x == kDkScanThreads - 1) {
        dk.meta[kDkD] = incl;
        dk.meta[kDkUse] = (incl >= 1u && incl <= static_cast<unsigned>(kDkMax)) ? 1u : 0u;
    }
}

// the distinct keys and their cums: the last copy of key kd[d] is table index cd[d] - 1
__global__ __launch_bounds__(kDkTile / 4) void dk_write_kernel(const unsigned* __restrict__ sorted, int64_t M,
                                                               const unsigned* __restrict__ ci_meta, DkWs dk) {
    if (dk_ci_in_use(ci_meta) || dk.meta[kDkUse] == 0u) return;
    __shared__ unsigned wsum[kDkTile / 4 / kWave];
    unsigned k[4];
    const int64_t i0 = int64_t(blockIdx.x) * kDkTile + 4 * int64_t(threadIdx.x);
    const unsigned f = dk_flags(sorted, M, i0, k);
    const unsigned c = static_cast<unsigned>(__popc(f));
    const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
    unsigned incl = c;
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
        const unsigned t = __shfl_up(incl, off, kWave);
        if (lane >= off) incl += t;
    }
    if (lane == kWave - 1) wsum[wid] = incl;
    __syncthreads();
    unsigned d = dk.tcnt[blockIdx.x] + incl - c;
    for (int w = 0; w < wid; ++w) d += wsum[w];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        if ((f >> j) & 1u) {
            dk.kd[d] = k[j];
            dk.cd[d] = static_cast<unsigned>(i0 + j + 1);
            ++d;
        }
    }
}

// one workgroup: the plan over the distinct keys (the count index's, ci_plan_body) and the first
// distinct key of every cell (cells (c(d-1), c(d)] start at d; d = D: up to the virtual last cell)
__global__ __launch_bounds__(kCiPlanThreads) void dk_index_kernel(const unsigned* __restrict__ ci_meta, DkWs dk) {
    if (dk_ci_in_use(ci_meta) || dk.meta[kDkUse] == 0u) return;
    __shared__ unsigned first[kCiTop];
    __shared__ uint2 l1[kCiTop];
    __shared__ unsigned wtot[kCiPlanThreads / kWave];
    __shared__ unsigned incl_min[kCiPlanThreads];
    __shared__ unsigned totals[2];
    const unsigned D = dk.meta[kDkD];
    for (int t = threadIdx.x; t < kCiTop; t += kCiPlanThreads) first[t] = D;
    __syncthreads();
    for (unsigned d = threadIdx.x; d < D; d += kCiPlanThreads) {
        const unsigned t = dk.kd[d] >> kCiLowBits;
        if (d == 0 || (dk.kd[d - 1] >> kCiLowBits) != t) first[t] = d;
    }
    __syncthreads();
    // up to 4 cells per distinct key while the LDS holds them (fewer cells of 2+ keys: less searching)
    ci_plan_body(D, first, l1, dk.meta, kDkMaxCells, wtot, incl_min, totals, 4);
    __syncthreads();
    for (int t = threadIdx.x; t < kCiTop; t += kCiPlanThreads) dk.l1[t] = l1[t];
    const unsigned cells = totals[1];
    auto cell = [&](unsigned d) -> int64_t {
        const unsigned key = dk.kd[d];
        return ci_cell(key, l1[key >> kCiLowBits]);
    };
    for (unsigned d = threadIdx.x; d <= D; d += kCiPlanThreads) {
        const int64_t cd = d < D ? cell(d) : int64_t(cells) + 1;
        const int64_t cp = d > 0 ? cell(d - 1) : -1;
        for (int64_t c = cp + 1; c <= cd; ++c) dk.cstart[c] = d;
    }
}

// Two LDS layouts of the index; the kernel built for the other one returns at once. Up to
// kDkSmall distinct keys (4 cells each) a cell word is 8 bytes {the cum before the cell, its first
// distinct key | its count << 16}: a query reads its cell word and, in a cell that holds keys, the
// cell's first {key, cum} -- 2 random LDS reads. Past it, to kDkMax, a cell word is 16 bits {first
// distinct key (14 bits), count saturated at 3} and a query reads the two entries at the cell's
// start -- 3 random reads. (The pass is bound by the LDS bank conflicts of those reads.)
constexpr int kDkSmall = 3200;
constexpr int kDkSmallCells = 4 * kDkSmall + kCiTop;

// the query kernels' LDS: l1, then {0, 0}, {key, cum} of every distinct key, {+inf, M} (read, never
// counted, past the last), then the cell words
template <bool SMALL>
struct DkLds {
    uint2* l1;
    uint2* kc;
    std::conditional_t<SMALL, uint2*, unsigned short*> cw;
};
template <bool SMALL>
__device__ __forceinline__ DkLds<SMALL> dk_load_lds(uint2* lds, const DkWs& dk, int64_t M) {
    constexpr int kMax = SMALL ? kDkSmall : kDkMax;
    using CW = std::conditional_t<SMALL, uint2*, unsigned short*>;
    DkLds<SMALL> r{lds, lds + kCiTop, reinterpret_cast<CW>(lds + kCiTop + kMax + 2)};
    const unsigned D = dk.meta[kDkD], cells = dk.meta[kCiCells];
    for (int i = threadIdx.x; i < kCiTop; i += blockDim.x) r.l1[i] = dk.l1[i];
    for (unsigned i = threadIdx.x; i < D + 2; i += blockDim.x)
        r.kc[i] = i == 0 ? uint2{0u, 0u}
                         : (i <= D ? uint2{dk.kd[i - 1], dk.cd[i - 1]} : uint2{kPadKey, static_cast<unsigned>(M)});
    for (unsigned c = threadIdx.x; c <= cells + (SMALL ? 0u : 1u); c += blockDim.x) {
        const unsigned a = dk.cstart[c], n = c <= cells ? dk.cstart[c + 1] - a : 0u;
        if constexpr (SMALL)
            r.cw[c] = uint2{a ? dk.cd[a - 1] : 0u, a | (n << 16)};
        else
            r.cw[c] = static_cast<unsigned short>(a | (min(n, 3u) << 14));
    }
    __syncthreads();
    return r;
}

// NQ queries of one lane: W += M - #(table <= x), T += #(table == x) for the queries in `use`
// (TABLE_POS false: the table is the negatives and the queries positives, W += #(table < x))
template <int NQ, bool TABLE_POS = true, bool SMALL = false>
__device__ __forceinline__ void dk_count(const unsigned (&x)[NQ], unsigned use, const DkLds<SMALL>& ld,
                                         unsigned long long M, unsigned long long& w, unsigned long long& t) {
    const uint2* kc = ld.kc;
    unsigned s0[NQ], n[NQ], cb[NQ], c[NQ];  // cb: the cum before s0 (SMALL)
    uint2 e[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) e[q] = ld.l1[x[q] >> kCiLowBits];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        c[q] = ci_cell(x[q], e[q]);
        if constexpr (SMALL) {
            const uint2 v = ld.cw[c[q]];
            cb[q] = v.x;
            s0[q] = v.y & 0xffffu;
            n[q] = v.y >> 16;
        } else {
            const unsigned v = ld.cw[c[q]];
            s0[q] = v & 0x3fffu;
            n[q] = v >> 14;
        }
    }
    bool many = false;
#pragma unroll
    for (int q = 0; q < NQ; ++q) many |= n[q] > 1u;
    if (many) {  // a cell of 2+ distinct keys: s0 <- the last one <= x (n = 1), or none (n = 0)
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            if (n[q] > 1u) {
                unsigned lo = s0[q], cnt = n[q];
                if constexpr (!SMALL) cnt = n[q] < 3u ? n[q] : (ld.cw[c[q] + 1] & 0x3fffu) - s0[q];
                while (cnt > 0u) {
                    const unsigned h = cnt >> 1;
                    if (kc[lo + h + 1].x <= x[q]) {
                        lo += h + 1;
                        cnt -= h + 1;
                    } else {
                        cnt = h;
                    }
                }
                if constexpr (SMALL) {  // the cum before the last key <= x, when that is not the cell's first
                    if (lo > s0[q] + 1) cb[q] = kc[lo - 1].y;
                }
                n[q] = lo > s0[q] ? 1u : 0u;
                s0[q] = lo > s0[q] ? lo - 1 : s0[q];
            }
        }
    }
    // kc[s0] = the distinct key before the cell's (or {0, 0}), kc[s0 + 1] = the cell's first one
    uint2 a[NQ], b[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        if constexpr (SMALL) {
            a[q] = uint2{0u, cb[q]};
            b[q] = uint2{kPadKey, 0u};
            if (n[q]) b[q] = kc[s0[q] + 1];  // only the lanes whose cell holds keys read it
        } else {
            a[q] = kc[s0[q]];
            b[q] = kc[s0[q] + 1];
        }
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const bool in = n[q] != 0u && b[q].x <= x[q];
        const bool eq = in && b[q].x == x[q];
        const unsigned le = in ? b[q].y : a[q].y;
        const unsigned lt = eq ? a[q].y : le;
        if ((use >> q) & 1u) {
            w += TABLE_POS ? M - le : lt;
            t += le - lt;
        }
    }
}

// the block's W, T (and non-finite count) into out[0..1] (and *nonfinite)
__device__ __forceinline__ void dk_reduce(unsigned long long w, unsigned long long t, unsigned nf,
                                          unsigned long long* __restrict__ out,
                                          unsigned long long* __restrict__ nonfinite) {
    __shared__ unsigned long long red[3][kQueryThreads / kWave];
    w = wave_sum(w);
    t = wave_sum(t);
    const unsigned long long nfw = wave_sum(static_cast<unsigned long long>(nf));
    const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
    if (lane == 0) {
        red[0][wid] = w;
        red[1][wid] = t;
        red[2][wid] = nfw;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long bw = 0, bt = 0, bn = 0;
        for (int i = 0; i < kQueryThreads / kWave; ++i) {
            bw += red[0][i];
            bt += red[1][i];
            bn += red[2][i];
        }
        if (bw) atomicAdd(out + 0, bw);
        if (bt) atomicAdd(out + 1, bt);
        if (bn && nonfinite) atomicAdd(nonfinite, bn);
    }
}

// dauc_auc_counts_sorted's form: every element of q[0, L) is a query (no labels); the table is the
// positives (TABLE_POS) or the negatives
template <bool TABLE_POS, bool SMALL>
__global__ __launch_bounds__(kQueryThreads) void dk_plain_kernel(const float* __restrict__ q, int64_t L, DkWs dk,
                                                                 int64_t M, unsigned long long* __restrict__ out) {
    if (dk.meta[kDkUse] == 0u || (dk.meta[kDkD] <= unsigned(kDkSmall)) != SMALL) return;
    extern __shared__ uint2 dk_lds[];
    const DkLds<SMALL> ld = dk_load_lds<SMALL>(dk_lds, dk, M);
    const unsigned long long MM = static_cast<unsigned long long>(M);
    unsigned long long w = 0, t = 0;
    const bool vec = (reinterpret_cast<uintptr_t>(q) & 15u) == 0;
    const int64_t nvec = vec ? L / 4 : 0;
    const int64_t stride = int64_t(gridDim.x) * kQueryThreads;
    const int64_t tid = int64_t(blockIdx.x) * kQueryThreads + threadIdx.x;
    if (nvec > 0) {
        constexpr int U = 2, NQ = 4 * U;
        f32x4 fc[U], fn[U];
        auto load = [&](int64_t v0, f32x4 (&f)[U]) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t v = v0 + int64_t(u) * stride;
                f[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(q) + (v < nvec ? v : 0));
            }
        };
        load(tid, fc);
        for (int64_t v0 = tid; v0 < nvec; v0 += int64_t(U) * stride) {
            load(v0 + int64_t(U) * stride, fn);
            unsigned x[NQ], use = 0u;
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const float f[4] = {fc[u].x, fc[u].y, fc[u].z, fc[u].w};
                const unsigned in = v0 + int64_t(u) * stride < nvec ? 0xfu : 0u;
                use |= in << (4 * u);
#pragma unroll
                for (int j = 0; j < 4; ++j) x[4 * u + j] = key_fast(f[j]);
            }
            dk_count<NQ, TABLE_POS, SMALL>(x, use, ld, MM, w, t);
#pragma unroll
            for (int u = 0; u < U; ++u) fc[u] = fn[u];
        }
    }
    for (int64_t i = nvec * 4 + tid; i < L; i += stride) {
        const unsigned x[1] = {key_fast(q[i])};
        dk_count<1, TABLE_POS, SMALL>(x, 1u, ld, MM, w, t);
    }
    dk_reduce(w, t, 0u, out, nullptr);
}

// The labeled query pass over the distinct-key index (the stream and checks of query_labeled_kernel);
// returns at once unless the count index is not in use and the distinct-key index is, in this layout
template <typename LT, bool SMALL, int U = 2>
__global__ __launch_bounds__(kQueryThreads) void dk_query_kernel(const float* __restrict__ s, const LT* __restrict__ lab,
                                                                 int64_t begin, int64_t end,
                                                                 const unsigned* __restrict__ ci_meta, DkWs dk,
                                                                 int64_t M, unsigned long long* __restrict__ out,
                                                                 unsigned long long* __restrict__ nonfinite) {
    if (dk_ci_in_use(ci_meta) || dk.meta[kDkUse] == 0u || (dk.meta[kDkD] <= unsigned(kDkSmall)) != SMALL) return;
    extern __shared__ uint2 dk_lds[];
    const DkLds<SMALL> ld = dk_load_lds<SMALL>(dk_lds, dk, M);
    const unsigned long long MM = static_cast<unsigned long long>(M);
    unsigned long long w = 0, t = 0;
    unsigned nf = 0;
    auto one = [&](int64_t i) {
        if (lab[i] != LT(1)) {
            const float f = s[i];
            nf += !isfinite(f);
            const unsigned x[1] = {key_fast(f)};
            dk_count<1, true, SMALL>(x, 1u, ld, MM, w, t);
        }
    };
    const int64_t a0 = (begin + 3) & ~int64_t(3);
    const int64_t head = a0 < end ? a0 : end;
    const int64_t stride = int64_t(gridDim.x) * kQueryThreads;
    const int64_t tid = int64_t(blockIdx.x) * kQueryThreads + threadIdx.x;
    for (int64_t i = begin + tid; i < head; i += stride) one(i);
    const int64_t nvec = end > head ? (end - head) / 4 : 0;
    const bool aligned = (reinterpret_cast<uintptr_t>(s + head) & 15u) == 0 &&
                         (reinterpret_cast<uintptr_t>(lab + head) & (4 * sizeof(LT) - 1)) == 0;
    if (aligned && nvec > 0) {
        // U float4 slots per iteration, the next iteration's loaded before this one's lookups
        constexpr int NQ = 4 * U;
        f32x4 fc[U], fn[U];
        LabelWords<LT> lc[U], ln[U];
        auto load = [&](int64_t v0, f32x4 (&f)[U], LabelWords<LT> (&l)[U]) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t v = v0 + int64_t(u) * stride;
                const int64_t i = head + (v < nvec ? v : 0) * 4;
                f[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(s + i));
                l[u].load(lab + i);
                if (v >= nvec) l[u].set_positive();  // past the end: no query
            }
        };
        load(tid, fc, lc);
        for (int64_t v0 = tid; v0 < nvec; v0 += int64_t(U) * stride) {
            load(v0 + int64_t(U) * stride, fn, ln);
            unsigned x[NQ], use = 0u;
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const float f[4] = {fc[u].x, fc[u].y, fc[u].z, fc[u].w};
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const bool neg = lc[u].not_positive(q);
                    use |= unsigned(neg) << (4 * u + q);
                    x[4 * u + q] = key_fast(f[q]);
                    nf += neg && !isfinite(f[q]);
                }
            }
            dk_count<NQ, true, SMALL>(x, use, ld, MM, w, t);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                fc[u] = fn[u];
                lc[u] = ln[u];
            }
        }
    } else if (!aligned) {
        for (int64_t i = head + tid; i < head + nvec * 4; i += stride) one(i);
    }
    for (int64_t i = head + nvec * 4 + tid; i < end; i += stride) one(i);
    dk_reduce(w, t, nf, out, nonfinite);
}
constexpr size_t kDkQueryLds = (size_t(kCiTop) + kDkMax + 2) * 8 + (size_t(kDkMaxCells) + 2) * 2;
constexpr size_t kDkQueryLdsSmall = (size_t(kCiTop) + kDkSmall + 2) * 8 + (size_t(kDkSmallCells) + 1) * 8;
static_assert(kDkQueryLds + 3 * (kQueryThreads / kWave) * 8 <= 160 * 1024, "the distinct-key query's LDS");
static_assert(kDkQueryLdsSmall + 3 * (kQueryThreads / kWave) * 8 <= 160 * 1024, "the distinct-key query's LDS");

int query_grid(int64_t L) {
    static int cus = 0;
    if (cus == 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) {
            (void)hipGetLastError();
            cus = 256;
        }
    }
#ifdef DAUC_TUNING
    // tuning builds: DAUC_QUERY_QPT = the queries per thread the grid aims at (default 4)
    static int qpt = 0;
    if (qpt == 0) {
        const char* e = getenv("DAUC_QUERY_QPT");
        qpt = e ? atoi(e) : 4;
        if (qpt < 1 || qpt > 1024) qpt = 4;
    }
#else
    constexpr int qpt = 4;
#endif
    int64_t g = (L + int64_t(qpt) * kQueryThreads - 1) / (int64_t(qpt) * kQueryThreads);
    if (g > 1 * cus) g = 1 * cus;  // 1024-thread workgroups
    if (g < 1) g = 1;
    return static_cast<int>(g);
}

template <bool TABLE_POS>
int launch_query(int k, const float* q, int64_t L, const TreeNode* tree, const TreeGeom& g, const unsigned* sorted,
                 int64_t M, unsigned long long* out, hipStream_t st, const unsigned* dk_meta = nullptr) {
    const dim3 grid(query_grid(L)), block(kQueryThreads);
    const size_t lds = size_t(g.nodes) * sizeof(TreeNode);
#define DAUC_QC(KV) \
    hipLaunchKernelGGL((query_count_kernel<KV, TABLE_POS>), grid, block, lds, st, q, L, tree, g, k, sorted, M, out, \
                       dk_meta)
    switch (k) {
        case 1: DAUC_QC(1); break;
        case 2: DAUC_QC(2); break;
        case 4: DAUC_QC(4); break;
        case 8: DAUC_QC(8); break;
        case 16: DAUC_QC(16); break;
        case 32: DAUC_QC(32); break;
        default: DAUC_QC(0); break;
    }
#undef DAUC_QC
    return launch_status();
}

struct SortWs {
    unsigned* keys_a;
    unsigned* keys_b;
    unsigned* hist;
    unsigned* sums;
    int64_t ntiles, m, nsum;
};

SortWs carve(void* ws, int64_t n) {
    SortWs w;
    w.ntiles = tiles_for(n);
    w.m = int64_t(kRadix) * w.ntiles;
    w.nsum = (w.m + kScanBlock - 1) / kScanBlock;
    auto* p = static_cast<unsigned char*>(ws);
    auto take = [&](int64_t count) {
        unsigned* r = reinterpret_cast<unsigned*>(p);
        p += ((count * 4 + 255) / 256) * 256;
        return r;
    };
    w.keys_a = take(n + 64);  // + room for the last bucket's kPadKey tail
    w.keys_b = take(n + 64);
    w.hist = take(w.m);
    w.sums = take(w.nsum);
    return w;
}

size_t sort_ws_bytes(int64_t n) {
    const int64_t nt = tiles_for(n), m = int64_t(kRadix) * nt, ns = (m + kScanBlock - 1) / kScanBlock;
    auto rnd = [](int64_t c) { return ((c * 4 + 255) / 256) * 256; };
    return static_cast<size_t>(rnd(n + 64) * 2 + rnd(m) + rnd(ns));
}

// Sorts the keys of neg[0..N) into the workspace; returns the sorted array.
int radix_sort_keys(const float* neg, int64_t N, const SortWs& w, hipStream_t st, const unsigned** sorted) {
    const unsigned* src = nullptr;
    unsigned* dst = w.keys_a;
    for (int pass = 0; pass < 4; ++pass) {
        const int shift = 8 * pass;
        if (pass == 0)
            hipLaunchKernelGGL(radix_hist_kernel<true>, dim3(w.ntiles), dim3(kSortThreads), 0, st,
                               static_cast<const void*>(neg), N, shift, w.hist, w.ntiles);
        else
            hipLaunchKernelGGL(radix_hist_kernel<false>, dim3(w.ntiles), dim3(kSortThreads), 0, st,
                               static_cast<const void*>(src), N, shift, w.hist, w.ntiles);
        const void* in = pass == 0 ? static_cast<const void*>(neg) : static_cast<const void*>(src);
        if (w.ntiles <= kFusedScanTiles) {
            // small sorts are launch-bound: the scatter workgroups scan the histogram themselves
            if (pass == 0)
                hipLaunchKernelGGL((radix_scatter_kernel<true, true>), dim3(w.ntiles), dim3(kSortThreads), 0, st,
                                   in, N, shift, w.hist, w.ntiles, dst);
            else
                hipLaunchKernelGGL((radix_scatter_kernel<false, true>), dim3(w.ntiles), dim3(kSortThreads), 0, st,
                                   in, N, shift, w.hist, w.ntiles, dst);
        } else {
            if (w.m <= kSingleScan) {
                hipLaunchKernelGGL(scan_sums_kernel, dim3(1), dim3(kScanBlock), 0, st, w.hist, w.m);
            } else {
                hipLaunchKernelGGL(scan_blocks_kernel, dim3(w.nsum), dim3(kScanBlock), 0, st, w.hist, w.m, w.sums);
                hipLaunchKernelGGL(scan_sums_kernel, dim3(1), dim3(kScanBlock), 0, st, w.sums, w.nsum);
                hipLaunchKernelGGL(scan_add_kernel, dim3(w.nsum), dim3(kScanBlock), 0, st, w.hist, w.m, w.sums);
            }
            if (pass == 0)
                hipLaunchKernelGGL((radix_scatter_kernel<true, false>), dim3(w.ntiles), dim3(kSortThreads), 0, st,
                                   in, N, shift, w.hist, w.ntiles, dst);
            else
                hipLaunchKernelGGL((radix_scatter_kernel<false, false>), dim3(w.ntiles), dim3(kSortThreads), 0, st,
                                   in, N, shift, w.hist, w.ntiles, dst);
        }
        const int rc = launch_status();
        if (rc) return rc;
        src = dst;
        dst = (dst == w.keys_a) ? w.keys_b : w.keys_a;
    }
    *sorted = src;
    return DAUC_OK;
}

CountWs carve_count(void* p) {
    char* c = static_cast<char*>(p);
    CountWs w;
    w.meta = reinterpret_cast<unsigned*>(c);
    c += 256;
    w.first = reinterpret_cast<unsigned*>(c);
    c += size_t(kCiTop) * 4;
    w.l1 = reinterpret_cast<uint2*>(c);
    c += size_t(kCiTop) * 8;
    w.cstart = reinterpret_cast<unsigned*>(c);
    c += ((size_t(kCiMaxCells) + 2) * 4 + 255) / 256 * 256;
    w.blk = reinterpret_cast<uint2*>(c);
    return w;
}

// the count index behind the sort and the tree (first[] was reset by build_tree_kernel): 4 small
// launches; the verdict (usable, skewed) stays on the device
int prepare_count(const unsigned* sorted, int64_t M, const CountWs& cw, hipStream_t st) {
    hipLaunchKernelGGL(ci_first_kernel, dim3(static_cast<unsigned>((M + 255) / 256)), dim3(256), 0, st, sorted, M,
                       cw.first);
    hipLaunchKernelGGL(ci_plan_kernel, dim3(1), dim3(kCiPlanThreads), 0, st, M, cw.first, cw.l1, cw.meta);
    hipLaunchKernelGGL(ci_cells_kernel, dim3(static_cast<unsigned>((M + 1 + 255) / 256)), dim3(256), 0, st, sorted, M,
                       cw.l1, cw.meta, cw.cstart);
    hipLaunchKernelGGL(ci_blocks_kernel, dim3((kCiMaxBlocks + 255) / 256), dim3(256), 0, st, cw.cstart, cw.meta,
                       cw.blk);
    return launch_status();
}

template <typename LT>
int launch_ci(const float* s, const LT* lab, int64_t begin, int64_t end, const CountWs& cw, const unsigned* sorted,
              int64_t M, unsigned long long* out, unsigned long long* nonfinite, hipStream_t st,
              unsigned* verdict = nullptr, const unsigned* grp = nullptr, const unsigned long long* Mp = nullptr,
              unsigned* check = nullptr, const uint2* slot_counts = nullptr, unsigned slot_cells = 0u,
              unsigned long long* red8 = nullptr) {
    const dim3 grid(query_grid(end - begin)), block(kQueryThreads);
    const size_t lds = (size_t(kCiTop) + kCiMaxBlocks) * 8 + (grp ? size_t(kDirectMaxGroups) * 4 : 0);
    bool sec = true;  // the carried secondary window (query_ci_kernel's SEC)
#ifdef DAUC_TUNING
    {
        static int abl = -1;
        if (abl < 0) {
            const char* e = getenv("DAUC_QUERY_ABL");
            abl = e ? atoi(e) : 0;
            if (hipMemcpyToSymbol(HIP_SYMBOL(g_query_abl), &abl, sizeof(int)) != hipSuccess) return DAUC_EINVAL;
        }
        const char* e = getenv("DAUC_QUERY_SEC");  // 0: a secondary window per query (the round-6 form)
        sec = !(e && atoi(e) == 0);
    }
#endif
    // dynamic + the kernel's static reduction rows must fit the CU's 160 KB of LDS (a launch past it
    // aborts the queue: HSA_STATUS_ERROR_INVALID_ALLOCATION)
    static_assert((size_t(kCiTop) + kCiMaxBlocks) * 8 + size_t(kDirectMaxGroups) * 4 +
                          4 * (kQueryThreads / kWave) * 8 <= 160 * 1024,
                  "the count-index query's LDS");
    if (slot_counts != nullptr && check != nullptr && sec)
        hipLaunchKernelGGL((query_ci_kernel<LT, true, true, true>), grid, block, lds, st, s, lab, begin, end, cw.meta,
                           cw.l1, slot_counts, sorted, M, out, nonfinite, verdict, nullptr, Mp, check, slot_cells, red8);
    else if (slot_counts != nullptr && sec)
        hipLaunchKernelGGL((query_ci_kernel<LT, false, true, true>), grid, block, lds, st, s, lab, begin, end, cw.meta,
                           cw.l1, slot_counts, sorted, M, out, nonfinite, verdict, nullptr, Mp, nullptr, slot_cells, red8);
#ifdef DAUC_TUNING
    else if (slot_counts != nullptr && check != nullptr)
        hipLaunchKernelGGL((query_ci_kernel<LT, true, true, false>), grid, block, lds, st, s, lab, begin, end, cw.meta,
                           cw.l1, slot_counts, sorted, M, out, nonfinite, verdict, nullptr, Mp, check, slot_cells, red8);
    else if (slot_counts != nullptr)
        hipLaunchKernelGGL((query_ci_kernel<LT, false, true, false>), grid, block, lds, st, s, lab, begin, end,
                           cw.meta, cw.l1, slot_counts, sorted, M, out, nonfinite, verdict, nullptr, Mp, nullptr,
                           slot_cells, red8);
#endif
    else if (check != nullptr)
        hipLaunchKernelGGL((query_ci_kernel<LT, true>), grid, block, lds, st, s, lab, begin, end, cw.meta, cw.l1,
                           cw.blk, sorted, M, out, nonfinite, verdict, grp, Mp, check, 0u);
    else
        hipLaunchKernelGGL((query_ci_kernel<LT>), grid, block, lds, st, s, lab, begin, end, cw.meta, cw.l1, cw.blk,
                           sorted, M, out, nonfinite, verdict, grp, Mp, check, 0u);
    return launch_status();
}

char* after_tree_of(void* workspace, int64_t P) {
    return static_cast<char*>(workspace) + ((sort_ws_bytes(P) + 255) / 256) * 256 + ((kTreeBytes + 255) / 256) * 256;
}

CountWs count_ws_of(void* workspace, int64_t P) {
    return carve_count(after_tree_of(workspace, P) + kGrpBytes);
}

int64_t dk_tiles(int64_t M) { return (M + kDkTile - 1) / kDkTile; }

size_t dk_ws_bytes(int64_t M) {  // (+ 256: the count region's end rounded up to 256 bytes)
    return 256 + 256 + size_t(kCiTop) * 8 + (size_t(kDkMaxCells) + 2 + 63) / 64 * 256 + 2 * size_t(kDkMax) * 4 +
           (size_t(dk_tiles(M < 1 ? 1 : M)) * 4 + 255) / 256 * 256;
}

// the distinct-key index's region: past the count index's
DkWs dk_ws_of(void* workspace, int64_t P) {
    char* c = after_tree_of(workspace, P) + kGrpBytes + (kCountBytes + 255) / 256 * 256;
    DkWs w;
    w.meta = reinterpret_cast<unsigned*>(c);
    c += 256;
    w.l1 = reinterpret_cast<uint2*>(c);
    c += size_t(kCiTop) * 8;
    w.cstart = reinterpret_cast<unsigned*>(c);
    c += (size_t(kDkMaxCells) + 2 + 63) / 64 * 256;
    w.kd = reinterpret_cast<unsigned*>(c);
    c += size_t(kDkMax) * 4;
    w.cd = reinterpret_cast<unsigned*>(c);
    c += size_t(kDkMax) * 4;
    w.tcnt = reinterpret_cast<unsigned*>(c);
    return w;
}

// the distinct-key index behind prepare_count (ci_meta: the count index's verdict, or nullptr when
// it was not built): 4 small launches, each returning at once when the index is not needed / not used
int prepare_dk(const unsigned* sorted, int64_t M, const unsigned* ci_meta, const DkWs& dk, hipStream_t st) {
    const int64_t nt = dk_tiles(M);
    hipLaunchKernelGGL(dk_mark_kernel, dim3(static_cast<unsigned>(nt)), dim3(kDkTile / 4), 0, st, sorted, M, ci_meta,
                       dk.tcnt);
    hipLaunchKernelGGL(dk_scan_kernel, dim3(1), dim3(kDkScanThreads), 0, st, ci_meta, dk, nt);
    hipLaunchKernelGGL(dk_write_kernel, dim3(static_cast<unsigned>(nt)), dim3(kDkTile / 4), 0, st, sorted, M, ci_meta,
                       dk);
    hipLaunchKernelGGL(dk_index_kernel, dim3(1), dim3(kCiPlanThreads), 0, st, ci_meta, dk);
    return launch_status();
}

template <bool TABLE_POS>
int launch_dk_plain(const float* q, int64_t L, const DkWs& dk, int64_t M, unsigned long long* out, hipStream_t st) {
    // both layouts enqueued: the one the device's distinct count does not select returns at once
    hipLaunchKernelGGL((dk_plain_kernel<TABLE_POS, true>), dim3(query_grid(L)), dim3(kQueryThreads), kDkQueryLdsSmall,
                       st, q, L, dk, M, out);
    hipLaunchKernelGGL((dk_plain_kernel<TABLE_POS, false>), dim3(query_grid(L)), dim3(kQueryThreads), kDkQueryLds, st,
                       q, L, dk, M, out);
    return launch_status();
}

template <typename LT>
int launch_dk(const float* s, const LT* lab, int64_t begin, int64_t end, const unsigned* ci_meta, const DkWs& dk,
              int64_t M, unsigned long long* out, unsigned long long* nonfinite, hipStream_t st) {
    // both layouts enqueued: the one the device's distinct count does not select returns at once
    const dim3 grid(query_grid(end - begin));
    hipLaunchKernelGGL((dk_query_kernel<LT, true>), grid, dim3(kQueryThreads), kDkQueryLdsSmall, st, s, lab, begin,
                       end, ci_meta, dk, M, out, nonfinite);
    hipLaunchKernelGGL((dk_query_kernel<LT, false>), grid, dim3(kQueryThreads), kDkQueryLds, st, s, lab, begin, end,
                       ci_meta, dk, M, out, nonfinite);
    return launch_status();
}

template <typename LT>
int launch_labeled(int k, const float* s, const LT* lab, int64_t begin, int64_t end, const TreeNode* tree,
                   const TreeGeom& g, const unsigned* sorted, int64_t M, unsigned long long* out, unsigned long long* nonfinite,
                   const unsigned* meta, hipStream_t st, const unsigned* dk_meta = nullptr) {
    const dim3 grid(query_grid(end - begin)), block(kQueryThreads);
    const size_t lds = size_t(g.nodes) * sizeof(TreeNode);
#define DAUC_QL(KV)                                                                                              \
    hipLaunchKernelGGL((query_labeled_kernel<KV, LT>), grid, block, lds, st, s, lab, begin, end, tree, g, k, \
                       sorted, M, out, nonfinite, meta, dk_meta)
    switch (k) {
        case 1: DAUC_QL(1); break;
        case 2: DAUC_QL(2); break;
        case 4: DAUC_QL(4); break;
        case 8: DAUC_QL(8); break;
        case 16: DAUC_QL(16); break;
        case 32: DAUC_QL(32); break;
        default: DAUC_QL(0); break;
    }
#undef DAUC_QL
    return launch_status();
}

// sort the table, build the tree; returns the tree pointer and geometry
int prepare_table(const float* table, int64_t M, void* workspace, hipStream_t st, const unsigned** sorted,
                  TreeNode** tree, int* k_out, TreeGeom* g_out, unsigned* ci_first = nullptr) {
    SortWs w = carve(workspace, M);
    int rc = radix_sort_keys(table, M, w, st, sorted);
    if (rc) return rc;
    int k = 1;
    while ((M + k - 1) / k > kMaxSplit) k *= 2;
    const int S = static_cast<int>((M + k - 1) / k);
    const TreeGeom g = tree_geom(S);
    *tree = reinterpret_cast<TreeNode*>(static_cast<char*>(workspace) + ((sort_ws_bytes(M) + 255) / 256) * 256);
    // buckets of <= 32 keys are read whole (one vector load), so their tail is padded; larger
    // ones are binary-searched with bounds (k - 1 < 64 keys of slack in the sort workspace)
    const int64_t pad = k <= 32 ? int64_t(S) * k - M : 0;
    const int n_first = ci_first ? kCiTop : 0;
    int64_t nthreads = (g.nodes > pad) ? g.nodes : pad;
    if (nthreads < 8) nthreads = 8;
    if (nthreads < n_first) nthreads = n_first;
    hipLaunchKernelGGL(build_tree_kernel, dim3(static_cast<unsigned>((nthreads + 255) / 256)), dim3(256), 0, st,
                       const_cast<unsigned*>(*sorted), M, pad, k, g, *tree, ci_first, n_first);
    *k_out = k;
    *g_out = g;
    return launch_status();
}

}  // namespace

bool direct_enabled() { return g_search_mode == 0; }

int64_t direct_capacity(int64_t n) {
    // the plan's bound (2 M <= 3 cells), and the smaller class of n scores (the evaluation's
    // workspace holds a table of n / 2 + 1 keys)
    const int64_t cap = 3 * int64_t(kCiMaxCells) / 2, half = n / 2 + 1;
    return half < cap ? half : cap;
}

unsigned* direct_cnt_ptr(void* workspace, int64_t Mcap) { return count_ws_of(workspace, Mcap).cstart; }

int64_t direct_cnt_words() { return kCiCntWords; }

int64_t direct_hist_offset(int64_t Mcap) {  // carve_count(...).first, relative to the workspace
    return int64_t(((sort_ws_bytes(Mcap) + 255) / 256) * 256 + ((kTreeBytes + 255) / 256) * 256 +
                   kGrpBytes + 256);
}

#ifdef DAUC_TUNING
// Tuning builds: dauc_set_direct_fault corrupts the direct build between its count and scatter
// passes, so a test can check that the scatter's index checks turn a producer bug into a verdict-2
// fallback (include/dauc_tuning.h): 1 = one key's cell past the plan's last cell, 2 = one key moved
// to the next cell (that cell's counter runs out), 3 = one cell's counter one above its count.
int g_direct_fault = 0;

__global__ void direct_fault_kernel(int mode, const unsigned long long* __restrict__ Mp,
                                    const unsigned* __restrict__ meta, unsigned* __restrict__ cnt,
                                    unsigned* __restrict__ cell) {
    const int64_t M = static_cast<int64_t>(*Mp);
    if (threadIdx.x != 0 || meta[kCiOk] == 0u || M == 0) return;
    const int64_t i = M / 2;
    const unsigned ncells = meta[kCiCells], c = cell[i];
    if (mode == 1) cell[i] = ncells + 7u;
    if (mode == 2) cell[i] = c + 1u < ncells ? c + 1u : 0u;
    if (mode == 3) cnt[c] += 1u;
}
#endif

// The count and scatter passes loop over the keys (up to 1024 workgroups; 256 measured the same:
// profiles/r04/query_ablations/r04q_*)
constexpr int64_t kDirectGrid = 1024;

int build_direct_index(const float* pos, const unsigned long long* Mp, int64_t Mcap, void* workspace,
                       size_t workspace_bytes, hipStream_t st, DirectIndex* ix, const unsigned* ready_hist) {
    if (pos == nullptr || Mp == nullptr || Mcap < 1 || workspace == nullptr || ix == nullptr ||
        workspace_bytes < dauc_sort_workspace_size(Mcap))
        return DAUC_EINVAL;
    const SortWs w = carve(workspace, Mcap);
    const CountWs nw = count_ws_of(workspace, Mcap);
    unsigned* table = w.keys_a;  // Mcap + 64 words: room for the +inf tail
    // the histogram aggregates 8 keys per thread in LDS; the count and scatter passes are chains of
    // dependent loads per key, so they take one key per thread per step (every chain in flight)
    unsigned* grp = reinterpret_cast<unsigned*>(after_tree_of(workspace, Mcap));  // [kDirectMaxGroups]
    const auto blocks = [](int64_t keys, int64_t per, int64_t cap) {
        const int64_t b = (keys + per - 1) / per;
        return dim3(static_cast<unsigned>(b < cap ? b : cap));
    };
    if (ready_hist == nullptr)
        hipLaunchKernelGGL(direct_hist_kernel, blocks(Mcap, 256 * kDirectPerThread, 256), dim3(256), 0, st, pos, Mp,
                           nw.first, nw.cstart, kCiCntWords);
    hipLaunchKernelGGL(direct_count_kernel<false>, blocks(Mcap, kDirectThreads, kDirectGrid), dim3(kDirectThreads), 0,
                       st, pos, Mcap, ready_hist ? ready_hist : nw.first, nw.l1, nw.meta, nw.cstart, w.keys_b,
                       nullptr, 0u);
    hipLaunchKernelGGL(direct_blocks_kernel, dim3(kDirectMaxGroups), dim3(kDirectGroup), 0, st, nw.cstart, nw.meta,
                       nw.blk, grp);
#ifdef DAUC_TUNING
    if (g_direct_fault != 0)
        hipLaunchKernelGGL(direct_fault_kernel, dim3(1), dim3(64), 0, st, g_direct_fault, Mp, nw.meta, nw.cstart,
                           w.keys_b);
#endif
    hipLaunchKernelGGL(direct_scatter_kernel, blocks(Mcap, kDirectThreads, kDirectGrid), dim3(kDirectThreads), 0, st, pos,
                       Mp, nw.blk, grp, nw.meta, nw.cstart, w.keys_b, table, kCiCntWords);
    *ix = DirectIndex{table, nw.l1, nw.blk, grp, nw.meta};
    return launch_status();
}

int counts_labeled_direct_slots(const SlotSource& src, float* pos, int64_t Mcap, const float* scores,
                                const void* labels, int label_dtype, int64_t begin, int64_t end,
                                unsigned long long* wins_ties, unsigned long long* nonfinite, unsigned* verdict,
                                void* workspace, size_t workspace_bytes, hipStream_t st, unsigned* check) {
    if (begin < 0 || end < begin || wins_ties == nullptr || pos == nullptr || src.slots == nullptr ||
        src.parts < 1 || src.parts > kMaxSlotParts || (end > begin && (scores == nullptr || labels == nullptr)) ||
        workspace == nullptr || Mcap < 1 || workspace_bytes < dauc_sort_workspace_size(Mcap))
        return DAUC_EINVAL;
    if (label_dtype != DAUC_LABEL_I8 && label_dtype != DAUC_LABEL_I32 && label_dtype != DAUC_LABEL_I64)
        return DAUC_EINVAL;
    const SortWs w = carve(workspace, Mcap);
    const CountWs nw = count_ws_of(workspace, Mcap);
    unsigned* table = w.keys_a;
    unsigned* grp = reinterpret_cast<unsigned*>(after_tree_of(workspace, Mcap));
    const int64_t gk = (Mcap + kSlotCountThreads - 1) / kSlotCountThreads;
    hipLaunchKernelGGL(direct_count_slots_kernel<false>, dim3(static_cast<unsigned>(gk)), dim3(kSlotCountThreads), 0,
                       st, src, Mcap, nw.l1, nw.meta, nw.cstart, w.keys_b, pos, nullptr, 0u);
    hipLaunchKernelGGL(direct_blocks_kernel, dim3(kDirectMaxGroups), dim3(kDirectGroup), 0, st, nw.cstart, nw.meta,
                       nw.blk, grp);
    const int64_t gs = (Mcap + kDirectThreads - 1) / kDirectThreads;
    hipLaunchKernelGGL(direct_scatter_kernel, dim3(static_cast<unsigned>(gs < kDirectGrid ? gs : kDirectGrid)),
                       dim3(kDirectThreads), 0, st, pos, src.m_eff, nw.blk, grp, nw.meta, nw.cstart, w.keys_b, table,
                       kCiCntWords);
    int rc = launch_status();
    if (rc || end == begin) return rc;
    const unsigned long long* Mp = src.m_eff;
    switch (label_dtype) {
        case DAUC_LABEL_I8:
            return launch_ci(scores, static_cast<const int8_t*>(labels), begin, end, nw, table, 0, wins_ties,
                             nonfinite, st, verdict, grp, Mp, check);
        case DAUC_LABEL_I32:
            return launch_ci(scores, static_cast<const int32_t*>(labels), begin, end, nw, table, 0, wins_ties,
                             nonfinite, st, verdict, grp, Mp, check);
        default:
            return launch_ci(scores, static_cast<const int64_t*>(labels), begin, end, nw, table, 0, wins_ties,
                             nonfinite, st, verdict, grp, Mp, check);
    }
}

int64_t slotted_cells(int64_t Mcap) {
    // the plan uses at most min(kCiMaxCells, 2 M + one per used bucket) cells
    const int64_t c = 2 * Mcap + kCiTop;
    return c < kCiMaxCells ? c : kCiMaxCells;
}

size_t slotted_table_bytes(int64_t Mcap) {  // primary + secondary + tertiary
    return size_t(slotted_cells(Mcap) + 1) * 8 * 4 + size_t(slotted_cells(Mcap)) * 8 * 4;
}

size_t slotted_fill_bytes(int64_t Mcap) { return size_t(slotted_cells(Mcap) + 1) * 8 * 4; }  // the +inf part

int64_t slotted_cnt_words() { return (int64_t(kCiMaxBlocks) * kCiBlock) / 4; }

unsigned* slotted_meta_ptr(void* workspace, int64_t Mcap) { return count_ws_of(workspace, Mcap).meta; }

int counts_labeled_slotted(const SlotSource& src, unsigned* stab, int64_t Mcap, const float* scores, const void* labels,
                           int label_dtype, int64_t begin, int64_t end, unsigned long long* wins_ties,
                           unsigned long long* nonfinite, unsigned* verdict, void* workspace, size_t workspace_bytes,
                           hipStream_t st, unsigned* check) {
    if (begin < 0 || end < begin || wins_ties == nullptr || stab == nullptr || src.slots == nullptr ||
        src.parts < 1 || src.parts > kMaxSlotParts || (end > begin && (scores == nullptr || labels == nullptr)) ||
        workspace == nullptr || Mcap < 1 || workspace_bytes < dauc_sort_workspace_size(Mcap) || check == nullptr)
        return DAUC_EINVAL;
    if (label_dtype != DAUC_LABEL_I8 && label_dtype != DAUC_LABEL_I32 && label_dtype != DAUC_LABEL_I64)
        return DAUC_EINVAL;
    const CountWs nw = count_ws_of(workspace, Mcap);
    const int64_t gk0 = (Mcap + kSlotCountThreads - 1) / kSlotCountThreads;
    const unsigned cells = static_cast<unsigned>(slotted_cells(Mcap));
#ifdef DAUC_TUNING
    // tuning builds: DAUC_SLOT_COUNT_WGS = this many count workgroups instead (each loops over keys)
    int64_t gk = gk0;
    if (const char* e = getenv("DAUC_SLOT_COUNT_WGS"); e && atoi(e) > 0 && atoi(e) <= 4096) gk = atoi(e);
#else
    const int64_t gk = gk0;
#endif
    hipLaunchKernelGGL(direct_count_slots_kernel<true>, dim3(static_cast<unsigned>(gk)), dim3(kSlotCountThreads), 0,
                       st, src, Mcap, nw.l1, nw.meta, nw.cstart, nw.first, nullptr, stab, cells);  // (SLOT: see above)
    int rc = launch_status();
    if (rc || end == begin) return rc;
    const unsigned long long* Mp = src.m_eff;
    const uint2* counts = reinterpret_cast<const uint2*>(nw.cstart);
    switch (label_dtype) {
        case DAUC_LABEL_I8:
            return launch_ci(scores, static_cast<const int8_t*>(labels), begin, end, nw, stab, 0, wins_ties, nonfinite,
                             st, verdict, nullptr, Mp, check, counts, cells,
                             reinterpret_cast<unsigned long long*>(nw.first));
        case DAUC_LABEL_I32:
            return launch_ci(scores, static_cast<const int32_t*>(labels), begin, end, nw, stab, 0, wins_ties, nonfinite,
                             st, verdict, nullptr, Mp, check, counts, cells,
                             reinterpret_cast<unsigned long long*>(nw.first));
        default:
            return launch_ci(scores, static_cast<const int64_t*>(labels), begin, end, nw, stab, 0, wins_ties, nonfinite,
                             st, verdict, nullptr, Mp, check, counts, cells,
                             reinterpret_cast<unsigned long long*>(nw.first));
    }
}

int counts_labeled_direct_slotted(const float* pos, const unsigned long long* Mp, int64_t Mcap, unsigned* stab,
                                  const float* scores, const void* labels, int label_dtype, int64_t begin,
                                  int64_t end, unsigned long long* wins_ties, unsigned long long* nonfinite,
                                  unsigned* verdict, void* workspace, size_t workspace_bytes, hipStream_t st,
                                  const unsigned* ready_hist) {
    if (begin < 0 || end < begin || wins_ties == nullptr || pos == nullptr || Mp == nullptr || stab == nullptr ||
        ready_hist == nullptr || Mcap < 1 || workspace == nullptr || workspace_bytes < dauc_sort_workspace_size(Mcap) ||
        (end > begin && (scores == nullptr || labels == nullptr)))
        return DAUC_EINVAL;
    if (label_dtype != DAUC_LABEL_I8 && label_dtype != DAUC_LABEL_I32 && label_dtype != DAUC_LABEL_I64)
        return DAUC_EINVAL;
    const CountWs nw = count_ws_of(workspace, Mcap);
    const unsigned cells = static_cast<unsigned>(slotted_cells(Mcap));
    const int64_t gb = (Mcap + kDirectThreads - 1) / kDirectThreads;
    hipLaunchKernelGGL(direct_count_kernel<true>, dim3(static_cast<unsigned>(gb < kDirectGrid ? gb : kDirectGrid)),
                       dim3(kDirectThreads), 0, st, pos, Mcap, ready_hist, nw.l1, nw.meta, nw.cstart, nullptr, stab,
                       cells, Mp);
    int rc = launch_status();
    if (rc || end == begin) return rc;
    const uint2* counts = reinterpret_cast<const uint2*>(nw.cstart);
    switch (label_dtype) {
        case DAUC_LABEL_I8:
            return launch_ci(scores, static_cast<const int8_t*>(labels), begin, end, nw, stab, 0, wins_ties, nonfinite,
                             st, verdict, nullptr, Mp, nullptr, counts, cells);
        case DAUC_LABEL_I32:
            return launch_ci(scores, static_cast<const int32_t*>(labels), begin, end, nw, stab, 0, wins_ties, nonfinite,
                             st, verdict, nullptr, Mp, nullptr, counts, cells);
        default:
            return launch_ci(scores, static_cast<const int64_t*>(labels), begin, end, nw, stab, 0, wins_ties, nonfinite,
                             st, verdict, nullptr, Mp, nullptr, counts, cells);
    }
}

int counts_labeled_direct(const float* pos, const unsigned long long* Mp, int64_t Mcap, const float* scores,
                          const void* labels, int label_dtype, int64_t begin, int64_t end,
                          unsigned long long* wins_ties, unsigned long long* nonfinite, unsigned* verdict,
                          void* workspace, size_t workspace_bytes, hipStream_t st, const unsigned* ready_hist,
                          unsigned* check) {
    if (begin < 0 || end < begin || wins_ties == nullptr || (end > begin && (scores == nullptr || labels == nullptr)))
        return DAUC_EINVAL;
    if (label_dtype != DAUC_LABEL_I8 && label_dtype != DAUC_LABEL_I32 && label_dtype != DAUC_LABEL_I64)
        return DAUC_EINVAL;
    DirectIndex ix{};
    int rc = build_direct_index(pos, Mp, Mcap, workspace, workspace_bytes, st, &ix, ready_hist);
    if (rc || end == begin) return rc;
    const CountWs nw = count_ws_of(workspace, Mcap);
    switch (label_dtype) {
        case DAUC_LABEL_I8:
            return launch_ci(scores, static_cast<const int8_t*>(labels), begin, end, nw, ix.table, 0, wins_ties,
                             nonfinite, st, verdict, ix.grp, Mp, check);
        case DAUC_LABEL_I32:
            return launch_ci(scores, static_cast<const int32_t*>(labels), begin, end, nw, ix.table, 0, wins_ties,
                             nonfinite, st, verdict, ix.grp, Mp, check);
        default:
            return launch_ci(scores, static_cast<const int64_t*>(labels), begin, end, nw, ix.table, 0, wins_ties,
                             nonfinite, st, verdict, ix.grp, Mp, check);
    }
}

int counts_sorted_labeled(const float* pos, int64_t P, const float* scores, const void* labels, int label_dtype,
                          int64_t begin, int64_t end, unsigned long long* wins_ties, unsigned long long* nonfinite,
                          void* workspace, size_t workspace_bytes, hipStream_t st, bool count_index) {
    if (P < 0 || begin < 0 || end < begin || wins_ties == nullptr || (P > 0 && pos == nullptr) ||
        (end > begin && (scores == nullptr || labels == nullptr)))
        return DAUC_EINVAL;
    if (label_dtype != DAUC_LABEL_I8 && label_dtype != DAUC_LABEL_I32 && label_dtype != DAUC_LABEL_I64)
        return DAUC_EINVAL;
    if (P == 0 || end == begin) return DAUC_OK;
    if (workspace == nullptr || workspace_bytes < dauc_sort_workspace_size(P) || P > 0xffffffffLL) return DAUC_EINVAL;
    const unsigned* sorted = nullptr;
    TreeNode* tree = nullptr;
    int k = 1;
    TreeGeom g{};
    // the search structure: mode 0 the count index where the table can use it, else the
    // distinct-key index where it holds the table, else the tree (every choice made on the device);
    // 1 the tree; 2 the distinct-key index, else the tree
    const int mode = g_search_mode;
    const bool count = count_index && mode == 0 && 2 * P <= 3 * int64_t(kCiMaxCells);
    const bool distinct = mode == 0 || mode == 2;  // the distinct-key index where the count index is not used
    const CountWs nw = count_ws_of(workspace, P);
    const DkWs dk = dk_ws_of(workspace, P);
    int rc = prepare_table(pos, P, workspace, st, &sorted, &tree, &k, &g, count ? nw.first : nullptr);
    if (rc) return rc;
    if (count && (rc = prepare_count(sorted, P, nw, st))) return rc;
    const unsigned* meta = count ? nw.meta : nullptr;
    if (distinct && (rc = prepare_dk(sorted, P, meta, dk, st))) return rc;
    auto run = [&](auto* lab) {
        int r = launch_labeled(k, scores, lab, begin, end, tree, g, sorted, P, wins_ties, nonfinite, meta, st,
                               distinct ? dk.meta : nullptr);
        if (r == DAUC_OK && count) r = launch_ci(scores, lab, begin, end, nw, sorted, P, wins_ties, nonfinite, st);
        if (r == DAUC_OK && distinct) r = launch_dk(scores, lab, begin, end, meta, dk, P, wins_ties, nonfinite, st);
        return r;
    };
    switch (label_dtype) {
        case DAUC_LABEL_I8: return run(static_cast<const int8_t*>(labels));
        case DAUC_LABEL_I32: return run(static_cast<const int32_t*>(labels));
        default: return run(static_cast<const int64_t*>(labels));
    }
}

}  // namespace dauc

using namespace dauc;

extern "C" {

size_t dauc_sort_workspace_size(int64_t n) {
    return sort_ws_bytes(n < 1 ? 1 : n) + kTreeBytes + 256 + kGrpBytes + kCountBytes + 256 + dk_ws_bytes(n);
}

#ifdef DAUC_TUNING
int dauc_set_search_mode(int mode) {
    if (mode < 0 || mode > 2) return DAUC_EINVAL;
    g_search_mode = mode;
    return DAUC_OK;
}

int dauc_set_direct_fault(int mode) {
    if (mode < 0 || mode > 3) return DAUC_EINVAL;
    g_direct_fault = mode;
    return DAUC_OK;
}
#endif

int dauc_sort_keys(const float* scores, int64_t n, unsigned* keys_out, void* workspace,
                   size_t workspace_bytes, dauc_stream_t stream) {
    if (n <= 0 || scores == nullptr || keys_out == nullptr || workspace == nullptr ||
        workspace_bytes < sort_ws_bytes(n) || n > 0xffffffffLL)
        return DAUC_EINVAL;
    SortWs w = carve(workspace, n);
    const unsigned* sorted = nullptr;
    hipStream_t st = as_hip(stream);
    int rc = radix_sort_keys(scores, n, w, st, &sorted);
    if (rc) return rc;
    return -static_cast<int>(hipMemcpyAsync(keys_out, sorted, size_t(n) * 4, hipMemcpyDeviceToDevice, st));
}

int dauc_auc_counts_sorted(const float* pos, int64_t P, const float* neg, int64_t N,
                           unsigned long long* wins_ties, void* workspace, size_t workspace_bytes,
                           dauc_stream_t stream) {
    if (P < 0 || N < 0 || wins_ties == nullptr || (P > 0 && pos == nullptr) ||
        (N > 0 && neg == nullptr))
        return DAUC_EINVAL;
    if (P == 0 || N == 0) return DAUC_OK;
    // the smaller class is sorted (the table); the larger one streams through the search
    const bool table_pos = P <= N;
    const int64_t M = table_pos ? P : N, L = table_pos ? N : P;
    if (workspace == nullptr || workspace_bytes < dauc_sort_workspace_size(M) || M > 0xffffffffLL) return DAUC_EINVAL;
    hipStream_t st = as_hip(stream);
    const unsigned* sorted = nullptr;
    TreeNode* tree = nullptr;
    int k = 1;
    TreeGeom g{};
    int rc = prepare_table(table_pos ? pos : neg, M, workspace, st, &sorted, &tree, &k, &g);
    if (rc) return rc;
    const float* q = table_pos ? neg : pos;
    // the distinct-key index where it holds the table (tie-heavy), else the tree: chosen on the device
    const bool distinct = g_search_mode != 1;
    const DkWs dk = dk_ws_of(workspace, M);
    if (distinct && (rc = prepare_dk(sorted, M, nullptr, dk, st))) return rc;
    const unsigned* dkm = distinct ? dk.meta : nullptr;
    rc = table_pos ? launch_query<true>(k, q, L, tree, g, sorted, M, wins_ties, st, dkm)
                   : launch_query<false>(k, q, L, tree, g, sorted, M, wins_ties, st, dkm);
    if (rc || !distinct) return rc;
    return table_pos ? launch_dk_plain<true>(q, L, dk, M, wins_ties, st)
                     : launch_dk_plain<false>(q, L, dk, M, wins_ties, st);
}

int dauc_auc_counts_sorted_labeled(const float* pos, int64_t P, const float* scores, const void* labels,
                                   int label_dtype, int64_t begin, int64_t end, unsigned long long* wins_ties,
                                   unsigned long long* nonfinite, void* workspace, size_t workspace_bytes,
                                   dauc_stream_t stream) {
    return counts_sorted_labeled(pos, P, scores, labels, label_dtype, begin, end, wins_ties, nonfinite, workspace,
                                 workspace_bytes, as_hip(stream), true);
}

}  // extern "C"
