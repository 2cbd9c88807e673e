// Exact AUC counts of one test set (the sort method), enqueued as one stream-ordered sequence.
//
// Reference: imagenet/main.py:79-81, AUC(label, scores) = sklearn roc_curve(pos_label=1) + auc,
// evaluated by rank 0 over the test set (main.py:237-250). The evaluation is:
//   1. memsets of the 64-byte record (the compaction's counters, the query counts, the verdict
//      word) and the top-bucket histogram: one when the record is the workspace header (the
//      blocking forms), two when it is the caller's part_out (the enqueued form);
//   2. the one-pass positive compaction: labels read once, the positives' scores gathered (in no
//      particular order), P counted on the device, their top-bucket histogram built;
//   3. the count index built straight from the unsorted positives, sized by the device's P
//      (auc_sort.hip, direct_*: the grids are sized for the index's capacity and loop), and the
//      labeled query pass over the scores [part * n / parts, (part + 1) * n / parts), which also
//      counts the non-finite queried scores (sklearn rejects them, _ranking.py:868-869) and writes
//      the verdict: 1 = counted, 2 = the index cannot hold this table (more than 219,838
//      positives, or clustered / tie-heavy ones);
//   4. the 64-byte record: W, T, #non-finite queried scores, P, #non-finite positives, #labels
//      outside {-1, 1}, the verdict -- counted straight into the caller's part_out by the enqueued
//      forms (no copy), into the workspace header by the blocking ones.
// Nothing in 1-4 waits for the host or allocates: dauc_auc_eval_enqueue is exactly that, and the
// sharded evaluation all-reduces its counts without a host synchronisation in between. The
// blocking forms add ONE readback into the caller's page-locked words and, only for verdict 2, the
// sorted path (radix sort of the positives, the LDS search tree or the count index behind it; or,
// when the negatives are the smaller class, both classes split and the negatives sorted). The
// calls keep no state between them: every input is an argument, every byte of state is in the
// caller's workspace and is re-initialised by the call.

#include <hip/hip_runtime.h>

#include "dauc.h"
#include "count_index.h"

namespace dauc {
namespace {

inline size_t align256(size_t b) { return (b + 255) / 256 * 256; }

// workspace header (bytes): [0, 24) W, T, #non-finite queried scores (u64, the query's atomics);
// [24, 56) the compaction's counters: P, tag (0), #non-finite positives, #labels outside {-1, 1};
// [56, 60) the verdict; [64, 96) a second counter slot the compaction's block 0 writes (unused);
// [256, 8448) the top-bucket histogram of the positives (the compaction's, handed to the direct
// build: no histogram pass). [0, 64) is the result record (the blocking forms'; the enqueued
// forms count into the caller's part_out instead); record and histogram are zeroed first.
constexpr size_t kHistOff = 256, kHdr = kHistOff + size_t(kCiTop) * 4, kRecord = 64;

struct EvalWs {
    unsigned long long* wt;       // [3]
    unsigned long long* slot;     // [4]
    unsigned* verdict;
    unsigned long long* spare;    // [4]
    unsigned* hist;               // [kCiTop]
    float* pos;                   // [n]   positive scores (P <= n)
    float* neg;                   // [n/2] negative scores (only when P > N, so N < n/2)
    int64_t* split_stats;         // [4]   the split's stats (sorted fallback)
    void* sws;                    // split workspace
    void* tws;                    // sort + tree + count-index workspace (a table of at most n/2 keys)
    size_t sws_bytes, tws_bytes;
    unsigned* stab;               // the two-step evaluation's cell-slotted table (+inf filled by step 1)
};

EvalWs eval_ws(void* ws, int64_t n) {
    char* p = static_cast<char*>(ws);
    EvalWs w;
    w.wt = reinterpret_cast<unsigned long long*>(p);
    w.slot = reinterpret_cast<unsigned long long*>(p + 24);
    w.verdict = reinterpret_cast<unsigned*>(p + 56);
    w.spare = reinterpret_cast<unsigned long long*>(p + 64);
    w.split_stats = reinterpret_cast<int64_t*>(p + 128);
    w.hist = reinterpret_cast<unsigned*>(p + kHistOff);
    p += kHdr;
    w.pos = reinterpret_cast<float*>(p);
    p += align256(size_t(n) * 4);
    w.neg = reinterpret_cast<float*>(p);
    p += align256(size_t(n / 2 + 1) * 4);
    w.sws_bytes = dauc_split_workspace_size(n);
    w.sws = p;
    p += align256(w.sws_bytes);
    w.tws_bytes = dauc_sort_workspace_size(n / 2 + 1);
    w.tws = p;
    p += align256(w.tws_bytes);
    w.stab = reinterpret_cast<unsigned*>(p);
    return w;
}

size_t eval_ws_bytes(int64_t n) {
    return kHdr + align256(size_t(n) * 4) + align256(size_t(n / 2 + 1) * 4) + align256(dauc_split_workspace_size(n)) +
           align256(dauc_sort_workspace_size(n / 2 + 1)) + align256(slotted_table_bytes(direct_capacity(n)));
}

bool valid_args(const float* scores, const void* labels, int label_dtype, int64_t n, int part, int parts,
                void* workspace, size_t workspace_bytes) {
    return n > 0 && scores != nullptr && labels != nullptr && workspace != nullptr &&
           workspace_bytes >= eval_ws_bytes(n) && (reinterpret_cast<uintptr_t>(workspace) & 255u) == 0 &&
           parts >= 1 && part >= 0 && part < parts &&
           (label_dtype == DAUC_LABEL_I8 || label_dtype == DAUC_LABEL_I32 || label_dtype == DAUC_LABEL_I64);
}

// [a, a + an) and [b, b + bn) overlap (byte ranges)
bool overlaps(const void* a, size_t an, const void* b, size_t bn) {
    const uintptr_t x = reinterpret_cast<uintptr_t>(a), y = reinterpret_cast<uintptr_t>(b);
    return x < y + bn && y < x + an;
}

// The record words of `w` moved to the caller's part_out (int64[8], 8-byte aligned): the
// kernels count straight into it, so the enqueued forms end without a record copy.
EvalWs with_record(EvalWs w, int64_t* rec) {
    w.wt = reinterpret_cast<unsigned long long*>(rec);
    w.slot = reinterpret_cast<unsigned long long*>(rec + 3);
    w.verdict = reinterpret_cast<unsigned*>(rec + 7);
    return w;
}

#ifdef DAUC_TUNING
// tuning builds: the count index's build (dauc_set_index_form), in the one-call and the two-step
// evaluation alike: 0 the slotted table (the product's), 1 round 5's direct build (count, blocks,
// scatter passes into the cell-ordered table)
int g_index_form = 0;
#else
constexpr int g_index_form = 0;
#endif

// Zeroes a[0, na) and b[0, nb) (8-byte words: part_out is only 8-byte aligned) in ONE launch of
// one workgroup: the evaluation's record and histogram before the compaction (round 6:
// hipMemsetAsync took a launch per region, 4-5 us each in the kernel trace, for 64 B + 8 KB)
__global__ __launch_bounds__(256) void zero2_kernel(unsigned long long* __restrict__ a, int na,
                                                    unsigned long long* __restrict__ b, int nb) {
    for (int i = threadIdx.x; i < na; i += 256) a[i] = 0ull;
    for (int i = threadIdx.x; i < nb; i += 256) b[i] = 0ull;
}

int zero2(void* a, size_t abytes, void* b, size_t bbytes, hipStream_t st) {
    hipLaunchKernelGGL(zero2_kernel, dim3(1), dim3(256), 0, st, static_cast<unsigned long long*>(a),
                       static_cast<int>(abytes / 8), static_cast<unsigned long long*>(b), static_cast<int>(bbytes / 8));
    return launch_status();
}

// Steps 1-3 (no host synchronisation, no allocation): the record at w.wt .. w.verdict (the
// workspace header, or the caller's part_out through with_record).
int enqueue(const float* scores, const void* labels, int label_dtype, int64_t n, int part, int parts,
            const EvalWs& w, hipStream_t st) {
    // the record and the histogram: one zeroing launch (one region when the record is the
    // workspace header's)
    const bool own = reinterpret_cast<char*>(w.hist) == reinterpret_cast<char*>(w.wt) + kHistOff;
    if (int z = own ? zero2(w.wt, kHdr, nullptr, 0, st) : zero2(w.wt, kRecord, w.hist, size_t(kCiTop) * 4, st))
        return z;
    const int64_t mcap = direct_capacity(n);
    // the compaction builds the index build's histogram and prepares its state (spread over its
    // grid): the per-cell counters zeroed, so the build skips its histogram pass; for the slotted
    // build (round 6) also the slotted table's +inf fill and meta words 8..13
    const bool slot = g_index_form == 0;
    unsigned* cnt = direct_cnt_ptr(w.tws, mcap);
    auto* meta8 = reinterpret_cast<unsigned long long*>(slotted_meta_ptr(w.tws, mcap) + 8);
    int rc = compact_unordered(scores, labels, label_dtype, n, w.pos, w.slot, 0ull, w.spare, 0ull,
                               slot ? meta8 : nullptr, cnt,
                               static_cast<int>(slot ? slotted_cnt_words() : direct_cnt_words()), st, INT64_MAX,
                               w.hist, nullptr, 0ull, slot ? w.stab : nullptr,
                               slot ? static_cast<int64_t>(slotted_fill_bytes(mcap) / 16) : 0);
    if (rc) return rc;
    const int64_t qlo = n * part / parts, qhi = n * (part + 1) / parts;
    if (qhi <= qlo) return DAUC_OK;  // an empty part: verdict 0, counts 0
    if (!direct_enabled()) {
        // a tuning build forcing another search structure: straight to the sorted path
        return -static_cast<int>(hipMemsetAsync(w.verdict, 2, 1, st));
    }
    if (slot)
        return counts_labeled_direct_slotted(w.pos, w.slot, mcap, w.stab, scores, labels, label_dtype, qlo, qhi, w.wt,
                                             w.wt + 2, w.verdict, w.tws, w.tws_bytes, st, w.hist);
    return counts_labeled_direct(w.pos, w.slot, mcap, scores, labels, label_dtype, qlo, qhi, w.wt, w.wt + 2,
                                 w.verdict, w.tws, w.tws_bytes, st, w.hist);
}

// The sorted path for a verdict-2 evaluation (P, N known): counts of part `part` into w.wt.
int sorted_path(const float* scores, const void* labels, int label_dtype, int64_t n, int part, int parts, int64_t P,
                int64_t N, const EvalWs& w, int64_t* pinned, hipStream_t st) {
    hipError_t e;
    if ((e = hipMemsetAsync(w.wt, 0, 24, st)) != hipSuccess) return -static_cast<int>(e);
    const dauc_stream_t ds = reinterpret_cast<dauc_stream_t>(st);
    if (P <= N) {
        // the positives are the table; every other score of the part is a query read in place
        const int64_t qlo = n * part / parts, qhi = n * (part + 1) / parts;
        if (qhi <= qlo) return DAUC_OK;
        // (the count index refused this table: its plan over the sorted copy would too)
        return counts_sorted_labeled(w.pos, P, scores, labels, label_dtype, qlo, qhi, w.wt, w.wt + 2, w.tws,
                                     w.tws_bytes, st, false);
    }
    // the negatives are the smaller class: materialise both (the split also checks every score)
    int rc = dauc_split_scores(scores, labels, label_dtype, n, w.pos, w.neg, w.split_stats, w.sws, w.sws_bytes, ds);
    if (rc) return rc;
    if ((e = hipMemcpyAsync(pinned, w.split_stats, 32, hipMemcpyDeviceToHost, st)) != hipSuccess ||
        (e = hipStreamSynchronize(st)) != hipSuccess)
        return -static_cast<int>(e);
    const int64_t Ps = pinned[0], Ns = pinned[1];
    if (pinned[2] != 0) {
        // non-finite negatives (the positives were checked by the compaction): counted once, by part
        // 0, as this evaluation's non-finite queried scores; the caller raises
        if (part == 0 && (e = hipMemcpyAsync(w.wt + 2, w.split_stats + 2, 8, hipMemcpyDeviceToDevice, st)) != hipSuccess)
            return -static_cast<int>(e);
        return DAUC_OK;
    }
    if (Ps == 0 || Ns == 0) return DAUC_OK;
    const int64_t plo = Ps * part / parts, phi = Ps * (part + 1) / parts;
    if (phi <= plo) return DAUC_OK;
    return dauc_auc_counts_sorted(w.pos + plo, phi - plo, w.neg, Ns, w.wt, w.tws, w.tws_bytes, ds);
}

// The blocking part: out[7] = { W_part, T_part, P, N, #non-finite positives + labels check below,
// #labels outside {-1, 1}, #non-finite queried scores of this part }.
int counts_part_blocking(const float* scores, const void* labels, int label_dtype, int64_t n, int part, int parts,
                         int64_t* out, int64_t* part_counts, int64_t* pinned, void* workspace, size_t workspace_bytes,
                         hipStream_t st) {
    if (out == nullptr || pinned == nullptr || !valid_args(scores, labels, label_dtype, n, part, parts, workspace,
                                                           workspace_bytes))
        return DAUC_EINVAL;
    const EvalWs w = eval_ws(workspace, n);
    int rc = enqueue(scores, labels, label_dtype, n, part, parts, w, st);
    if (rc) return rc;
    hipError_t e;
    auto readback = [&]() -> int {
        if ((e = hipMemcpyAsync(pinned, w.wt, kRecord, hipMemcpyDeviceToHost, st)) != hipSuccess ||
            (e = hipStreamSynchronize(st)) != hipSuccess)
            return -static_cast<int>(e);
        return DAUC_OK;
    };
    if ((rc = readback())) return rc;
    const int64_t P = pinned[3], N = n - P, nonfinite = pinned[5], other = pinned[6];
    const unsigned verdict = static_cast<unsigned>(pinned[7] & 0xffffffffLL);
    const bool need = P > 0 && N > 0 && nonfinite == 0;
    if (need && verdict == 2u) {
        if ((rc = sorted_path(scores, labels, label_dtype, n, part, parts, P, N, w, pinned, st)) || (rc = readback()))
            return rc;
    }
    // this part's counts stay on the device too, for the caller's all-reduce (same stream: no sync)
    if (part_counts != nullptr &&
        (e = hipMemcpyAsync(part_counts, w.wt, 3 * sizeof(int64_t), hipMemcpyDeviceToDevice, st)) != hipSuccess)
        return -static_cast<int>(e);
    out[0] = need ? pinned[0] : 0;
    out[1] = need ? pinned[1] : 0;
    out[2] = P;
    out[3] = N;
    out[4] = nonfinite;
    out[5] = other;
    out[6] = pinned[2];  // non-finite queried scores: counted whatever the verdict, one class included
    return DAUC_OK;
}

// ---- the sharded evaluation in two steps: each rank compacts only its slice -----------------
//
// Step 1 (dauc_auc_eval_compact_part): rank r compacts the positives of ITS slice of the labels
// (and zeroes the per-cell counters of step 2's build in its workspace) into a slot: a 256-byte
// header {P_r, 0, #non-finite positives, #labels outside {-1, 1}, n} (u64 words), the top-bucket
// histogram of its positives' keys (count_index.h, 2048 u32) and room for `cap` scores. The caller
// all-gathers the slots (one collective). Step 2 (dauc_auc_eval_query_part): the count index is
// built from the gathered slots read in place (the count pass sums their headers and histograms --
// no histogram pass -- and copies each key to the table's position array as it counts it: no
// gather launch), and the scores of the NEXT rank's slice are counted (rank r queries slice
// (r + 1) % parts): the record is dauc_auc_eval_enqueue's, with word 4 a consistency check -- this
// rank's labels over that slice against the slot the next rank compacted from it (low 32 bits: the
// P of that slot - the positives this rank's labels give over it, mod 2^32; high 32 bits: the
// number of slots built for another n). A slot
// holds an even share of the index's capacity plus 25 %, whatever n (so ranks called with different
// n still gather equal sizes and report the mismatch instead of hanging in the collective): a rank
// whose slice holds more positives (unshuffled test sets) overflows, and the evaluation reports
// verdict 2 (the caller's blocking sorted path), as it does for tables the index cannot hold.
constexpr size_t kSlotHist = 256, kSlotHdr = kSlotHist + size_t(kCiTop) * 4;
constexpr int kSlotN = 4;  // header word: the n the slot was built for


int64_t slot_cap(int parts) {
    const int64_t fair = (direct_capacity(INT64_MAX / 4) + parts - 1) / parts;
    return fair + fair / 4 + 64;
}

size_t slot_bytes(int parts) { return kSlotHdr + align256(size_t(slot_cap(parts)) * 4); }

// the slice of the labels rank `part` compacts: boundaries on 256-label multiples (int8 label
// loads stay 16-byte aligned for every slice of an aligned array)
int64_t slice_lo(int64_t n, int part, int parts) {
    return part == 0 ? 0 : part >= parts ? n : ((n * part / parts) & ~int64_t(255));
}

// the slice queried by part `part`: the next part's slice (the consistency check of the record)
int64_t query_lo(int64_t n, int part, int parts) { return slice_lo(n, (part + 1) % parts, parts); }
int64_t query_hi(int64_t n, int part, int parts) {
    const int q = (part + 1) % parts;
    return slice_lo(n, q + 1, parts);
}

// The two-step evaluation's sorted fallback (dauc_auc_eval_query_part_sorted): the gathered slots'
// positives copied into one contiguous table at their rank-order offsets; bad[0] = 1 when a slot
// overflowed (its positives are not all there) or the slots' total is not the caller's P.
__global__ __launch_bounds__(256) void slot_gather_kernel(const unsigned char* __restrict__ slots, size_t sbytes,
                                                          int parts, int64_t cap, int64_t P, float* __restrict__ pos,
                                                          unsigned* __restrict__ bad) {
    const int r = blockIdx.y;
    auto count = [&](int j) {
        return reinterpret_cast<const unsigned long long*>(slots + size_t(j) * sbytes)[0];
    };
    __shared__ unsigned long long off;
    if (threadIdx.x == 0) {
        unsigned long long before = 0, total = 0;
        bool over = false;
        for (int j = 0; j < parts; ++j) {
            const unsigned long long pj = count(j);
            before += j < r ? pj : 0ull;
            total += pj;
            over |= pj > static_cast<unsigned long long>(cap);
        }
        off = before;
        if (blockIdx.x == 0 && r == 0 && (over || total != static_cast<unsigned long long>(P))) bad[0] = 1u;
    }
    __syncthreads();
    const unsigned long long pr = count(r);
    if (pr > static_cast<unsigned long long>(cap)) return;  // overflowed: bad, nothing to copy
    const float* src = reinterpret_cast<const float*>(slots + size_t(r) * sbytes + kSlotHdr);
    for (unsigned long long i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < pr; i += uint64_t(gridDim.x) * 256) {
        const unsigned long long d = off + i;
        if (d < static_cast<unsigned long long>(P)) pos[d] = src[i];
    }
}

// record word 3 = P, word 7 = the verdict (1 counted, 2 the slots could not serve: the caller's
// whole-vector fallback)
__global__ void sorted_part_verdict_kernel(const unsigned* __restrict__ bad, int64_t P, int64_t* __restrict__ rec) {
    if (threadIdx.x == 0) {
        rec[3] = P;
        rec[7] = bad[0] ? 2 : 1;
    }
}

}  // namespace
}  // namespace dauc

using namespace dauc;

extern "C" {

size_t dauc_auc_eval_workspace_size(int64_t n) { return eval_ws_bytes(n < 1 ? 1 : n); }

int dauc_auc_eval_enqueue(const float* scores, const void* labels, int label_dtype, int64_t n, int part, int parts,
                          int64_t* part_out, void* workspace, size_t workspace_bytes, dauc_stream_t stream) {
    if (part_out == nullptr || !valid_args(scores, labels, label_dtype, n, part, parts, workspace, workspace_bytes))
        return DAUC_EINVAL;
    // the kernels count straight into part_out: it must not lie in the workspace they also write
    if ((reinterpret_cast<uintptr_t>(part_out) & 7u) != 0 || overlaps(part_out, kRecord, workspace, workspace_bytes))
        return DAUC_EINVAL;
    return enqueue(scores, labels, label_dtype, n, part, parts, with_record(eval_ws(workspace, n), part_out),
                   as_hip(stream));
}

size_t dauc_auc_slot_bytes(int64_t n, int parts) { return n < 1 || parts < 1 ? 0 : slot_bytes(parts); }

int dauc_auc_eval_compact_part(const float* scores, const void* labels, int label_dtype, int64_t n, int part,
                               int parts, void* slot, void* workspace, size_t workspace_bytes, dauc_stream_t stream) {
    if (slot == nullptr || (reinterpret_cast<uintptr_t>(slot) & 255u) != 0 ||
        !valid_args(scores, labels, label_dtype, n, part, parts, workspace, workspace_bytes) ||
        overlaps(slot, slot_bytes(parts), workspace, workspace_bytes))
        return DAUC_EINVAL;
    hipStream_t st = as_hip(stream);
    const EvalWs w = eval_ws(workspace, n);
    auto* hdr = static_cast<unsigned long long*>(slot);
    hipError_t e;
    if (int z = zero2(hdr, kSlotHdr, nullptr, 0, st)) return z;  // + histogram
    const int64_t lo = slice_lo(n, part, parts), hi = slice_lo(n, part + 1, parts);
    // step 2's slotted build state, reset here (the compaction's grid does it on the side): the
    // packed per-cell byte counters zeroed, the slotted table +inf, meta words 8..13 (the skew
    // word among them, which step 2's count pass sets from any workgroup) zeroed
    const int64_t mcap = direct_capacity(n);
    unsigned* cnt = direct_cnt_ptr(w.tws, mcap);
    auto* meta8 = reinterpret_cast<unsigned long long*>(slotted_meta_ptr(w.tws, mcap) + 8);
    // (form 1, tuning builds: round 5's direct build counts into one u32 per cell and fills nothing)
    const size_t tab = g_index_form == 0 ? slotted_fill_bytes(mcap) : 0;
    const int64_t ncnt = g_index_form == 0 ? slotted_cnt_words() : direct_cnt_words();
    if (hi <= lo) {
        // an empty slice: P_r = 0, the length word still set (its two halves), and step 2's state
        // reset by memsets (the compaction's job otherwise)
        auto* nw = reinterpret_cast<unsigned*>(hdr + kSlotN);
        const unsigned long long nv = static_cast<unsigned long long>(n);
        if ((e = hipMemsetD32Async(nw, static_cast<int>(nv & 0xffffffffull), 1, st)) != hipSuccess ||
            (e = hipMemsetD32Async(nw + 1, static_cast<int>(nv >> 32), 1, st)) != hipSuccess ||
            (e = hipMemsetAsync(cnt, 0, size_t(ncnt) * 4, st)) != hipSuccess ||
            (e = hipMemsetAsync(meta8, 0, 24, st)) != hipSuccess ||
            (tab && (e = hipMemsetD32Async(w.stab, -1, tab / 4, st)) != hipSuccess))
            return -static_cast<int>(e);
        return DAUC_OK;
    }
    const size_t lsz = label_dtype == DAUC_LABEL_I8 ? 1 : label_dtype == DAUC_LABEL_I32 ? 4 : 8;
    return compact_unordered(scores + lo, static_cast<const char*>(labels) + size_t(lo) * lsz, label_dtype, hi - lo,
                             reinterpret_cast<float*>(static_cast<char*>(slot) + kSlotHdr), hdr, 0ull, w.spare, 0ull,
                             meta8, cnt, static_cast<int>(ncnt), st, slot_cap(parts),
                             reinterpret_cast<unsigned*>(static_cast<char*>(slot) + kSlotHist), hdr + kSlotN,
                             static_cast<unsigned long long>(n), w.stab, static_cast<int64_t>(tab / 16));
}

int dauc_auc_eval_query_part(const float* scores, const void* labels, int label_dtype, int64_t n, int part, int parts,
                             const void* slots, int64_t* part_out, void* workspace, size_t workspace_bytes,
                             dauc_stream_t stream) {
    if (slots == nullptr || part_out == nullptr || (reinterpret_cast<uintptr_t>(slots) & 255u) != 0 ||
        (reinterpret_cast<uintptr_t>(part_out) & 7u) != 0 ||
        !valid_args(scores, labels, label_dtype, n, part, parts, workspace, workspace_bytes))
        return DAUC_EINVAL;
    // the record, the gathered slots and the workspace: written / read by the same launches
    const size_t sall = slot_bytes(parts) * size_t(parts);
    if (overlaps(part_out, kRecord, workspace, workspace_bytes) || overlaps(part_out, kRecord, slots, sall) ||
        overlaps(slots, sall, workspace, workspace_bytes))
        return DAUC_EINVAL;
    hipStream_t st = as_hip(stream);
    const EvalWs w = with_record(eval_ws(workspace, n), part_out);
    const int64_t mcap = direct_capacity(n);
    const int64_t qlo = query_lo(n, part, parts), qhi = query_hi(n, part, parts);
    // the build reads the gathered slots in place (no gather copy): its count pass sums their
    // headers and histograms, writes this part's record (counts zeroed, P, the check word, the
    // label counts) and m_eff (w.spare[0]: P, or past the index's capacity on an overflow); the
    // query pass brings the check word's low half back to zero
    SlotSource src{static_cast<const unsigned char*>(slots), slot_bytes(parts), kSlotHist, kSlotHdr, parts, part,
                   slot_cap(parts), n, qhi - qlo, w.wt, w.slot, reinterpret_cast<unsigned long long*>(w.verdict),
                   w.spare};
    if (g_index_form == 1)
        return counts_labeled_direct_slots(src, w.pos, mcap, scores, labels, label_dtype, qlo, qhi, w.wt, w.wt + 2,
                                           w.verdict, w.tws, w.tws_bytes, st, reinterpret_cast<unsigned*>(part_out + 4));
    return counts_labeled_slotted(src, w.stab, mcap, scores, labels, label_dtype, qlo, qhi, w.wt, w.wt + 2, w.verdict,
                                  w.tws, w.tws_bytes, st, reinterpret_cast<unsigned*>(part_out + 4));
}

int dauc_auc_eval_query_part_sorted(const float* scores, const void* labels, int label_dtype, int64_t n, int part,
                                    int parts, const void* slots, int64_t P, int64_t* part_out, void* workspace,
                                    size_t workspace_bytes, dauc_stream_t stream) {
    if (slots == nullptr || part_out == nullptr || (reinterpret_cast<uintptr_t>(slots) & 255u) != 0 ||
        (reinterpret_cast<uintptr_t>(part_out) & 7u) != 0 || P < 1 ||
        !valid_args(scores, labels, label_dtype, n, part, parts, workspace, workspace_bytes))
        return DAUC_EINVAL;
    const size_t sall = slot_bytes(parts) * size_t(parts);
    if (overlaps(part_out, kRecord, workspace, workspace_bytes) || overlaps(part_out, kRecord, slots, sall) ||
        overlaps(slots, sall, workspace, workspace_bytes))
        return DAUC_EINVAL;
    hipStream_t st = as_hip(stream);
    const EvalWs w = eval_ws(workspace, n);
    hipError_t e;
    auto* bad = reinterpret_cast<unsigned*>(w.spare);
    if ((e = hipMemsetAsync(part_out, 0, kRecord, st)) != hipSuccess ||
        (e = hipMemsetAsync(bad, 0, 4, st)) != hipSuccess)
        return -static_cast<int>(e);
    if (P > n - P) {
        // the negatives are the smaller class: the slots hold the wrong one (the caller's fallback)
        if ((e = hipMemsetAsync(bad, 1, 1, st)) != hipSuccess) return -static_cast<int>(e);
    } else {
        const int64_t cap = slot_cap(parts);
        const int64_t bx = (cap + 1023) / 1024 < 64 ? (cap + 1023) / 1024 : 64;
        hipLaunchKernelGGL(slot_gather_kernel, dim3(static_cast<unsigned>(bx), static_cast<unsigned>(parts)), dim3(256),
                           0, st, static_cast<const unsigned char*>(slots), slot_bytes(parts), parts, cap, P, w.pos, bad);
        int rc = launch_status();
        if (rc) return rc;
        // this rank's own slice of the scores against the sorted table (the count index would refuse
        // it again: the distinct-key index for tie-heavy tables, else the tree); on a bad gather the
        // counts are discarded with the verdict
        const int64_t qlo = slice_lo(n, part, parts), qhi = slice_lo(n, part + 1, parts);
        auto* rec = reinterpret_cast<unsigned long long*>(part_out);
        if (qhi > qlo &&
            (rc = counts_sorted_labeled(w.pos, P, scores, labels, label_dtype, qlo, qhi, rec, rec + 2, w.tws,
                                        w.tws_bytes, st, false)))
            return rc;
    }
    hipLaunchKernelGGL(sorted_part_verdict_kernel, dim3(1), dim3(64), 0, st, bad, P, part_out);
    return launch_status();
}

int dauc_auc_eval_counts(const float* scores, const void* labels, int label_dtype, int64_t n, int64_t* out,
                         int64_t* pinned, void* workspace, size_t workspace_bytes, dauc_stream_t stream) {
    int64_t o[7];
    const int rc = counts_part_blocking(scores, labels, label_dtype, n, 0, 1, o, nullptr, pinned, workspace,
                                        workspace_bytes, as_hip(stream));
    if (rc) return rc;
    for (int i = 0; i < 6; ++i) out[i] = o[i];
    out[4] += o[6];
    return DAUC_OK;
}

int dauc_auc_eval_counts_part(const float* scores, const void* labels, int label_dtype, int64_t n, int part,
                              int parts, int64_t* out, int64_t* part_counts, int64_t* pinned, void* workspace,
                              size_t workspace_bytes, dauc_stream_t stream) {
    return counts_part_blocking(scores, labels, label_dtype, n, part, parts, out, part_counts, pinned, workspace,
                                workspace_bytes, as_hip(stream));
}

#ifdef DAUC_TUNING
int dauc_set_index_form(int form) {
    if (form < 0 || form > 1) return DAUC_EINVAL;
    g_index_form = form;
    return DAUC_OK;
}
#endif

}  // extern "C"
