/*
 * dauc_tuning.h -- entry points of the TUNING build of the library (tuning/libdauc_tuning.so:
 * the product sources compiled with -DDAUC_TUNING by distributedauc_amd/build.py).
 *
 * These are measured alternatives of the product kernels, kept selectable by number so the
 * measurements behind the product's choices can be repeated (scripts/micro_kernels.py) and so the
 * tests can check that every alternative gives the product's integers. The product library
 * (libdauc.so, include/dauc.h) exports none of them and runs the default of each.
 */
#ifndef DAUC_TUNING_H
#define DAUC_TUNING_H

#include "dauc.h"

#ifdef __cplusplus
extern "C" {
#endif

/*
 * dauc_surrogate_fwdbwd with an explicit kernel: 0 the product's dispatch, 1 the persistent
 * grid-stride kernel (the small-batch path) at any B, 2 the two-launch form (the streaming kernel
 * writes one fp64 row per workgroup, a second launch reduces them), 3 the streaming kernel alone
 * (dh only: no reduce, no scalar outputs), 20 the product's one-launch kernel (128 extra reducer
 * workgroups, the final one taking the last 512 rows itself) at any unit-stride B, 22 = 20 with its
 * reducers returning at once (the stream and its tagged row stores alone, no scalar outputs: the
 * in-launch hand-off's cost by difference), 23 = 20 with streaming workgroup nblocks / 2 never
 * publishing its row (the reducers' bounded wait times out: NaN outputs and the workspace's status
 * bit, dauc_surrogate_status; seconds of polling -- a test of the timeout path only). The other numbers of rounds 2-3 (round 2's 64 streaming
 * reducers, the early-reducer form, other R / K, stamps; profiles/r03/a) were removed in round 4.
 * Variants 2..23 need unit strides, 16-byte aligned h/dh and int8 labels.
 * Every variant but 23 returns bitwise-identical dh and counts; the fp64 sums agree to rounding.
 */
int dauc_surrogate_fwdbwd_variant(const float* h, int64_t h_stride, const void* y, int y_dtype, int64_t B,
                                  const float* abalpha, const float* p_hat, float* dh, int64_t dh_stride,
                                  double* out64, float* grad3, float* loss, void* workspace,
                                  size_t workspace_bytes, int variant, dauc_stream_t stream);

/*
 * dauc_pd_update_dense with an explicit kernel geometry: variant = v + 4*t, v selects
 * 2 / 1 / 4 / 3 float4 per thread, t = 1 turns the non-temporal loads of g and w0 off, t = 2 makes
 * every load and store non-temporal. Variant 0 is the product's. Results are bit-identical.
 */
int dauc_pd_update_dense_variant(float* w, const float* g, const float* w0, float* w_avg, int64_t n,
                                 float lr, float inv_gamma, int variant, dauc_stream_t stream);

/*
 * dauc_pair_count with an explicit kernel variant: variant = mode + 4*r, mode 0 = packed fp32
 * difference + clamp (exact-compare fallback for tiles with infinities or |score| < 2^-103; the
 * product's), 1 = per-lane VGPR compare counters, 2 = wave ballot + scalar popcount, 3 = mixed;
 * r selects 8 / 4 / 16 positives held per lane. Every variant returns identical counts.
 */
int dauc_pair_count_variant(const float* pos, int64_t P, const float* neg, int64_t N,
                            unsigned long long* wins_ties, int variant, dauc_stream_t stream);

/*
 * Search structure of dauc_auc_counts_sorted_labeled in THIS library (process-wide, default 0).
 * Same integers in every mode.
 *   0: the product's choice -- the count index for tables of up to 219,838 keys, unless the
 *      device finds the table skewed (a cell of 15+ keys, or more than 1.5 keys per cell): then,
 *      and for larger tables, the distinct-key index when the table holds at most 14,000 distinct
 *      keys (tie-heavy tables, round 6), else the LDS search tree;
 *   1: the LDS search tree always (the fallback's structure, tested on every table);
 *   2: the distinct-key index whenever the table holds at most 14,000 distinct keys (the count
 *      index is not built), else the tree -- to test it on any table.
 * Modes 1 and 2 also send dauc_auc_eval_* straight to the sorted path (no count index first).
 */
int dauc_set_search_mode(int mode);

/*
 * Fault injection into the direct count-index build (process-wide, default 0 = none): between the
 * build's count and scatter passes, 1 = one key's cell index past the plan's last cell, 2 = one
 * key moved to the next cell (that cell's counter runs out), 3 = one cell's counter one above its
 * key count. The scatter's index checks must turn each into verdict 2 (the sorted path), never
 * into an out-of-bounds store or wrong counts. Tests only.
 */
int dauc_set_direct_fault(int mode);

/*
 * The count index's build in the exact-AUC evaluations (dauc_auc_eval_counts / _enqueue / _counts_part
 * and the two-step dauc_auc_eval_compact_part / _query_part; process-wide, default 0): 0 the
 * product's cell-slotted build (one count pass inserting every key into its cell's slots, then the
 * query pass, which turns the byte counts into block words itself), 1 round 5's direct build (count,
 * block and scatter passes into the cell-ordered table, then the query; dauc_set_direct_fault acts on
 * it). Same integers; set it before the compaction (which prepares the chosen form's state).
 */
int dauc_set_index_form(int form);

/* The transposing LDS read of the 3x3 weight gradient (csrc/conv_wgrad.hip), for its lane-map test:
 * out[64 lanes][8] <- the 16x16x32 operand fragment (k-step 0, channel block 16) of a [32][64]
 * tile whose element (row, col) holds row * 64 + col. */
int dauc_probe_tr16(short* out, dauc_stream_t stream);

/* The 3x3 weight gradient's form: 0 automatic (stride 1: the window layout of least estimated cost
 * wherever one fits; stride 2: gather), 1 the gather form everywhere, 2 / 3 the window form with
 * per-output-row windows and 64 / 128-pixel chunks, 4 / 5 with shared window rows (stride 1) and
 * 64 / 128-pixel chunks, where they fit (tests, A/B runs). Process-global; tuning builds only. */
int dauc_set_wgrad_form(int form);

#ifdef __cplusplus
}
#endif

#endif /* DAUC_TUNING_H */
