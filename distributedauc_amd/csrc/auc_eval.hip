// One-call exact AUC counts on one GPU (the sort method), host orchestration in C++.
//
// Reference: imagenet/main.py:79-81, AUC(label, scores) = sklearn roc_curve(pos_label=1) + auc,
// a blocking host call. This entry point is its blocking counterpart: it enqueues the
// compaction, reads the class sizes back (the sort needs the table size), enqueues the sort,
// the tree and the query pass, and reads the integer counts back. The stages are the ABI calls
// dauc_compact_positives and dauc_auc_counts_sorted_labeled (or, when the positives outnumber
// the negatives, dauc_split_scores and dauc_auc_counts_sorted), so it returns exactly their
// integers; what it removes is the host work between them: on the Python path each readback
// was followed by ~45 us of interpreter work and small torch launches before the sort began
// (profiles/r02/final/bench_kernel_trace gaps), here it is a few HIP calls.

#include <hip/hip_runtime.h>

#include "dauc.h"
#include "dauc_internal.h"

namespace dauc {
namespace {

inline size_t align256(size_t b) { return (b + 255) / 256 * 256; }

// pinned host words for the two readbacks (one set per host thread, allocated on first use)
int64_t* pinned_words() {
    static thread_local int64_t* p = nullptr;
    if (p == nullptr) {
        void* q = nullptr;
        if (hipHostMalloc(&q, 64 * sizeof(int64_t), hipHostMallocDefault) != hipSuccess) return nullptr;
        p = static_cast<int64_t*>(q);
    }
    return p;
}

struct EvalWs {
    float* pos;                   // [n]   positive scores (P <= n)
    float* neg;                   // [n/2] negative scores (only when P > N, so N < n/2)
    int64_t* stats;               // [4]   compaction / split stats
    unsigned long long* wt;       // [3]   wins, ties, non-finite queried scores
    void* cws;                    // compaction workspace
    void* sws;                    // split workspace
    void* tws;                    // sort + tree workspace (table of at most n/2 keys)
    size_t cws_bytes, sws_bytes, tws_bytes;
};

EvalWs eval_ws(void* ws, int64_t n) {
    char* p = static_cast<char*>(ws);
    EvalWs w;
    w.stats = reinterpret_cast<int64_t*>(p);
    w.wt = reinterpret_cast<unsigned long long*>(p + 64);
    p += 256;
    w.pos = reinterpret_cast<float*>(p);
    p += align256(size_t(n) * 4);
    w.neg = reinterpret_cast<float*>(p);
    p += align256(size_t(n / 2 + 1) * 4);
    w.cws_bytes = dauc_compact_workspace_size(n);
    w.cws = p;
    p += align256(w.cws_bytes);
    w.sws_bytes = dauc_split_workspace_size(n);
    w.sws = p;
    p += align256(w.sws_bytes);
    w.tws_bytes = dauc_sort_workspace_size(n / 2 + 1);
    w.tws = p;
    return w;
}

// the last evaluation's table size for its length and label type (one per host thread)
struct EvalMemo {
    int64_t n;
    int dtype;
    int64_t P;
    bool direct_ok;  // the count index built from the unsorted table was usable last time
};

EvalMemo& eval_memo() {
    static thread_local EvalMemo m{0, 0, 0, true};
    return m;
}

// The compaction's counters alternate between two 32-byte slots of the workspace header: a call
// uses slot epoch & 1 and its compaction zeroes the other one for the next call, so no memset
// launch precedes the compaction; a workspace seen for the first time is zeroed once.
struct EvalRing {
    const void* ws;
    unsigned epoch;
};

EvalRing& eval_ring() {
    static thread_local EvalRing r{nullptr, 0};
    return r;
}

constexpr size_t kRingOffset = 128;  // header bytes [128, 192): two slots of 4 counters

// slot word 1: the epoch that may use the slot (0 after the first-use memset). A workspace
// pointer this thread saw before but whose contents changed since (freed and reallocated at the
// same address) shows a different tag: the compaction then writes nothing and the call starts
// over with zeroed slots.
inline unsigned long long slot_tag(unsigned epoch) { return epoch ? (0xDA0C000000000000ull | epoch) : 0ull; }

size_t eval_ws_bytes(int64_t n) {
    return 256 + align256(size_t(n) * 4) + align256(size_t(n / 2 + 1) * 4) + align256(dauc_compact_workspace_size(n)) +
           align256(dauc_split_workspace_size(n)) + align256(dauc_sort_workspace_size(n / 2 + 1));
}

}  // namespace
}  // namespace dauc

using namespace dauc;

extern "C" {

size_t dauc_auc_eval_workspace_size(int64_t n) { return eval_ws_bytes(n < 1 ? 1 : n); }

}  // extern "C"

namespace dauc {
namespace {

// The evaluation of part `part` of `parts` (part 0 of 1 = the whole vector). Every part compacts
// ALL the positives (each rank holds the same scores: main.py:237-250 evaluates one test set), so
// the table is identical on every rank with no collective; only the queries are split -- the
// score-index range [part*n/parts, (part+1)*n/parts) when the positives are the table, the
// positive range [part*P/parts, (part+1)*P/parts) against the sorted negatives otherwise.
//   out[7] = { W_part, T_part, P, N, #non-finite (global checks), #labels not in {-1, 1},
//              #non-finite queried scores of this part }
int eval_counts_part(const float* scores, const void* labels, int label_dtype, int64_t n, int part, int parts,
                     int64_t* out, int64_t* part_counts, void* workspace, size_t workspace_bytes,
                     dauc_stream_t stream, bool retry = false) {
    if (n <= 0 || scores == nullptr || labels == nullptr || out == nullptr || workspace == nullptr ||
        workspace_bytes < eval_ws_bytes(n) || (reinterpret_cast<uintptr_t>(workspace) & 255u))
        return DAUC_EINVAL;
    if (parts < 1 || part < 0 || part >= parts) return DAUC_EINVAL;
    if (label_dtype != DAUC_LABEL_I8 && label_dtype != DAUC_LABEL_I32 && label_dtype != DAUC_LABEL_I64)
        return DAUC_EINVAL;
    int64_t* host = pinned_words();
    if (host == nullptr) return -static_cast<int>(hipErrorOutOfMemory);
    hipStream_t st = as_hip(stream);
    const EvalWs w = eval_ws(workspace, n);
    hipError_t e;
    // the direct build's verdict word (1 = the count index was usable, 2 = re-run sorted)
    unsigned* verdict = reinterpret_cast<unsigned*>(w.wt + 3);
    // the split's stats [0, 32), the counts [64, 88), the verdict [88, 92) and the compaction's
    // counter slots [128, 192) come back in one copy
    auto readback = [&]() -> int {
        if ((e = hipMemcpyAsync(host, w.stats, 192, hipMemcpyDeviceToHost, st)) != hipSuccess ||
            (e = hipStreamSynchronize(st)) != hipSuccess)
            return -static_cast<int>(e);
        return DAUC_OK;
    };
    const int64_t qlo = n * part / parts, qhi = n * (part + 1) / parts;
    // the sorted path: radix sort of the positives, the tree, the count index behind them
    auto query = [&](int64_t P) {
        if (qhi <= qlo) return static_cast<int>(DAUC_OK);
        return dauc_auc_counts_sorted_labeled(w.pos, P, scores, labels, label_dtype, qlo, qhi, w.wt, w.wt + 2, w.tws,
                                              w.tws_bytes, stream);
    };
    // the direct path: the count index straight from the unsorted positives (no sort, no tree);
    // its verdict says whether the table was usable (else the sorted path re-runs)
    auto direct = [&](int64_t P) {
        return counts_labeled_direct(w.pos, P, scores, labels, label_dtype, qlo, qhi, w.wt, w.wt + 2, verdict, w.tws,
                                     w.tws_bytes, st);
    };
    auto direct_verdict_ok = [&]() { return qhi <= qlo || static_cast<unsigned>(host[11] & 0xffffffffLL) == 1u; };
    // The table size P is known only after the compaction. An evaluation repeats on the same
    // test set (main.py evaluates it after every stage), so the last call's P for this n is
    // taken as the size and the build and query are enqueued behind the compaction WITHOUT a
    // readback in between; the one readback at the end returns the real P with the counts, and a
    // different P (other data of the same length) re-runs them at the real size.
    EvalMemo& memo = eval_memo();
    const bool same = memo.n == n && memo.dtype == label_dtype;
    bool direct_ok = same ? memo.direct_ok : true;
    const bool speculate = same && memo.P > 0 && memo.P <= n - memo.P;
    const bool spec_direct = speculate && direct_ok && direct_fits(memo.P);
    // the one-pass compaction (positives in no particular order: everything after it counts) also
    // zeroes the query's counters, the next call's counter slot and the direct build's histogram
    EvalRing& ring = eval_ring();
    auto* slots = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(w.stats) + kRingOffset);
    if (ring.ws != workspace) {
        if ((e = hipMemsetAsync(slots, 0, 64, st)) != hipSuccess) return -static_cast<int>(e);
        ring = EvalRing{workspace, 0u};
    }
    const unsigned slot = ring.epoch & 1u, epoch = ring.epoch;
    int rc = compact_unordered(
        scores, labels, label_dtype, n, w.pos, slots + 4 * slot, slot_tag(epoch), slots + 4 * (slot ^ 1u),
        slot_tag(epoch + 1), w.wt,
        spec_direct ? reinterpret_cast<unsigned*>(static_cast<char*>(w.tws) + direct_hist_offset(memo.P)) : nullptr,
        spec_direct ? direct_hist_words() : 0, st);
    if (rc) {
        ring.ws = nullptr;  // the slots' state is unknown: zero them again next time
        return rc;
    }
    ++ring.epoch;
    if (speculate && (rc = spec_direct ? direct(memo.P) : query(memo.P))) return rc;
    if ((rc = readback())) return rc;
    const int64_t* cst = host + (kRingOffset / 8) + 4 * slot;
    if (static_cast<unsigned long long>(cst[1]) != slot_tag(epoch)) {
        // stale slots (see slot_tag): nothing was compacted; zero them and start over, once
        ring.ws = nullptr;
        if (retry) return DAUC_EINVAL;
        return eval_counts_part(scores, labels, label_dtype, n, part, parts, out, part_counts, workspace,
                                workspace_bytes, stream, true);
    }
    int64_t P = cst[0], N = n - cst[0], nonfinite = cst[2];
    const int64_t other = cst[3];
    bool counted = false;
    if (speculate && P == memo.P) {
        if (!spec_direct || direct_verdict_ok()) counted = true;
        else direct_ok = false;  // a skewed table: the sorted path below
    }
    if (!counted && P > 0 && N > 0 && nonfinite == 0) {
        if ((e = hipMemsetAsync(w.wt, 0, 3 * sizeof(unsigned long long), st)) != hipSuccess)
            return -static_cast<int>(e);
        if (P <= N) {
            // the positives are the table; every other score is a query read in place
            if (direct_ok && direct_fits(P)) {
                unsigned* hist = reinterpret_cast<unsigned*>(static_cast<char*>(w.tws) + direct_hist_offset(P));
                if ((e = hipMemsetAsync(hist, 0, size_t(direct_hist_words()) * 4, st)) != hipSuccess)
                    return -static_cast<int>(e);
                if ((rc = direct(P)) || (rc = readback())) return rc;
                if (direct_verdict_ok()) {
                    counted = true;
                } else {
                    direct_ok = false;
                    if ((e = hipMemsetAsync(w.wt, 0, 3 * sizeof(unsigned long long), st)) != hipSuccess)
                        return -static_cast<int>(e);
                }
            }
            if (!counted) rc = query(P);
        } else {
            // the negatives are the smaller class: materialise both (the split checks every score)
            rc = dauc_split_scores(scores, labels, label_dtype, n, w.pos, w.neg, w.stats, w.sws, w.sws_bytes, stream);
            if (rc) return rc;
            if ((rc = readback())) return rc;
            P = host[0];
            N = host[1];
            nonfinite = host[2];
            const int64_t plo = P * part / parts, phi = P * (part + 1) / parts;
            if (nonfinite == 0 && phi > plo)
                rc = dauc_auc_counts_sorted(w.pos + plo, phi - plo, w.neg, N, w.wt, w.tws, w.tws_bytes, stream);
        }
        if (rc) return rc;
        if (!counted && (rc = readback())) return rc;
        counted = true;
    }
    memo = EvalMemo{n, label_dtype, P, direct_ok};
    const bool have = counted && P > 0 && N > 0 && nonfinite == 0;
    // this part's counts stay on the device too, for the caller's all-reduce (same stream: no sync)
    if (have && part_counts != nullptr &&
        (e = hipMemcpyAsync(part_counts, w.wt, 3 * sizeof(int64_t), hipMemcpyDeviceToDevice, st)) != hipSuccess)
        return -static_cast<int>(e);
    out[0] = have ? host[8] : 0;
    out[1] = have ? host[9] : 0;
    out[2] = P;
    out[3] = N;
    out[4] = nonfinite;
    out[5] = other;
    out[6] = have ? host[10] : 0;
    return DAUC_OK;
}

}  // namespace
}  // namespace dauc

extern "C" {

int dauc_auc_eval_counts(const float* scores, const void* labels, int label_dtype, int64_t n, int64_t* out,
                         void* workspace, size_t workspace_bytes, dauc_stream_t stream) {
    if (out == nullptr) return DAUC_EINVAL;
    int64_t o[7];
    const int rc = eval_counts_part(scores, labels, label_dtype, n, 0, 1, o, nullptr, workspace, workspace_bytes, stream);
    if (rc) return rc;
    for (int i = 0; i < 6; ++i) out[i] = o[i];
    out[4] += o[6];
    return DAUC_OK;
}

int dauc_auc_eval_counts_part(const float* scores, const void* labels, int label_dtype, int64_t n, int part,
                              int parts, int64_t* out, int64_t* part_counts, void* workspace, size_t workspace_bytes,
                              dauc_stream_t stream) {
    return eval_counts_part(scores, labels, label_dtype, n, part, parts, out, part_counts, workspace, workspace_bytes,
                            stream);
}

}  // extern "C"
