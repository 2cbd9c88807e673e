/*
 * Plain-C restatement of the reference's exact-AUC arithmetic and its fp32
 * primal-dual update. TEST INFRASTRUCTURE ONLY: linked by tests/ and
 * bench.py's cpu_baseline leg as the checker and the timed CPU path; the
 * product library (libdauc.so) never links or calls it.
 *
 * oracle_auc_counts
 *   restates sklearn/metrics/_ranking.py:826-908 (_binary_clf_curve), which the
 *   reference reaches through main.py:79-81 (roc_curve(pos_label=1) + auc):
 *   W = #{(pos, neg): s_pos > s_neg}, T = #{s_pos == s_neg} (fp32 equality, so
 *   -0 == +0). It sorts the negatives (LSD radix sort on order-preserving keys)
 *   and counts, for every positive, the negatives strictly below and equal to it
 *   with two binary searches: O(N log N + P log N), exact 64-bit integers.
 *
 * oracle_pd_update
 *   restates main.py:61 + 333-334 in fp32 with every operation separately
 *   rounded (this file must be compiled with -ffp-contract=off).
 *
 * Pinned against the reference's own outputs: tests/golden/auc_cases.npz and
 * tests/golden/dppd_sg.npz (see tests/test_oracle_golden.py).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* order-preserving uint32 key of a finite float; -0 and +0 share a key */
static inline uint32_t fkey(float f) {
    if (f == 0.0f) f = 0.0f; /* canonical +0 */
    uint32_t u;
    memcpy(&u, &f, 4);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

static void radix_sort_u32(uint32_t* a, uint32_t* tmp, int64_t n) {
    for (int shift = 0; shift < 32; shift += 8) {
        int64_t cnt[257] = {0};
        for (int64_t i = 0; i < n; ++i) cnt[((a[i] >> shift) & 255u) + 1]++;
        for (int b = 0; b < 256; ++b) cnt[b + 1] += cnt[b];
        for (int64_t i = 0; i < n; ++i) tmp[cnt[(a[i] >> shift) & 255u]++] = a[i];
        uint32_t* t = a;
        a = tmp;
        tmp = t;
    }
    /* 4 passes: the sorted data is back in the caller's `a` */
}

/* first index with key >= k */
static int64_t lower_bound(const uint32_t* a, int64_t n, uint32_t k) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        int64_t mid = lo + (hi - lo) / 2;
        if (a[mid] < k) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

static int64_t upper_bound(const uint32_t* a, int64_t n, uint32_t k) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        int64_t mid = lo + (hi - lo) / 2;
        if (a[mid] <= k) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

/*
 * labels: int64, positive iff == 1 (sklearn pos_label=1). Returns 0, or -1 if a
 * score is not finite (sklearn raises ValueError), -2 on allocation failure.
 * out[0..3] = W, T, P, N.
 */
int oracle_auc_counts(const float* scores, const int64_t* labels, int64_t n, uint64_t* out) {
    int64_t P = 0, N = 0;
    for (int64_t i = 0; i < n; ++i) {
        if (!isfinite(scores[i])) return -1;
        if (labels[i] == 1) ++P;
        else ++N;
    }
    uint32_t* neg = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(N > 0 ? N : 1));
    uint32_t* tmp = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(N > 0 ? N : 1));
    if (!neg || !tmp) {
        free(neg);
        free(tmp);
        return -2;
    }
    int64_t k = 0;
    for (int64_t i = 0; i < n; ++i)
        if (labels[i] != 1) neg[k++] = fkey(scores[i]);
    radix_sort_u32(neg, tmp, N);
    uint64_t W = 0, T = 0;
    for (int64_t i = 0; i < n; ++i) {
        if (labels[i] != 1) continue;
        const uint32_t key = fkey(scores[i]);
        const int64_t lo = lower_bound(neg, N, key);
        const int64_t hi = upper_bound(neg, N, key);
        W += (uint64_t)lo;
        T += (uint64_t)(hi - lo);
    }
    free(neg);
    free(tmp);
    out[0] = W;
    out[1] = T;
    out[2] = (uint64_t)P;
    out[3] = (uint64_t)N;
    return 0;
}

/* Brute-force O(P*N) count over explicit positive / negative lists (small n only). */
void oracle_pair_count_bruteforce(const float* pos, int64_t P, const float* neg, int64_t N,
                                  uint64_t* out) {
    uint64_t W = 0, T = 0;
    for (int64_t i = 0; i < P; ++i)
        for (int64_t j = 0; j < N; ++j) {
            W += pos[i] > neg[j];
            T += pos[i] == neg[j];
        }
    out[0] = W;
    out[1] = T;
}

/* main.py:61 + 333-334: w <- w - lr*(g + invg*(w - w0)); avg <- avg + w (avg nullable) */
void oracle_pd_update(float* w, const float* g, const float* w0, float* avg, int64_t n, float lr,
                      float invg) {
    for (int64_t i = 0; i < n; ++i) {
        const float d = w[i] - w0[i];
        const float t = invg * d;
        const float gp = g[i] + t;
        const float u = lr * gp;
        const float r = w[i] - u;
        w[i] = r;
        if (avg) avg[i] = avg[i] + r;
    }
}
