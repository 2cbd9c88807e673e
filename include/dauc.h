/*
 * dauc.h — C ABI of libdauc.so, the MI355X (gfx950) hot path of CoDA
 * (communication-efficient distributed AUC maximization).
 *
 * This is the drop-in boundary for the data-parallel hot path of the reference
 * (ZhishuaiGuo/DistributedAUC, imagenet/main.py). The reference has no FFI: its
 * path is a handful of in-process Python functions and one inline loss
 * expression. Each entry point below replaces one of them; the citation names
 * the reference interface it replaces.
 *
 * Conventions (all entry points):
 *   - Every pointer argument is a DEVICE pointer owned by the caller, unless the
 *     parameter is documented as a host pointer.
 *   - The library never allocates or synchronises on the hot path. Scratch
 *     space is sized with the matching *_workspace_size() query and provided by
 *     the caller, zero-filled before its first use (the library leaves it
 *     zeroed again after every call).
 *   - Every call takes a hipStream_t (pass the caller's current stream). Work
 *     is enqueued on that stream, asynchronously and in stream order.
 *   - Return value: 0 on success, DAUC_EINVAL on a bad argument (nothing was
 *     enqueued), or -(hipError_t) if a HIP launch failed. No C++ exception ever
 *     crosses this boundary. dauc_strerror() turns a status into text.
 *   - One rank per process, one stream per call site: calls are
 *     thread-compatible, not thread-safe on one workspace.
 */
#ifndef DAUC_H_
#define DAUC_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* dauc_stream_t; /* == hipStream_t */

#define DAUC_OK 0
#define DAUC_EINVAL (-100000)

/* label element types accepted by the surrogate / class-sum kernels */
#define DAUC_LABEL_I8 1
#define DAUC_LABEL_I32 2
#define DAUC_LABEL_I64 3

/* element types of the logits accepted by the fused-softmax surrogate */
#define DAUC_DTYPE_F32 1
#define DAUC_DTYPE_BF16 2

/* dauc_pd_update modes */
#define DAUC_MODE_REFERENCE 0 /* main.py:58-64 as written: b prox uses (a_new-a0), alpha unchanged */
#define DAUC_MODE_PAPER 1     /* b prox uses (b-b0), alpha <- alpha + lr*dF/dalpha              */

/* ---------------------------------------------------------------- misc */

/* Library version as 100*major + minor. */
int dauc_version(void);

/* Human-readable text for a status returned by any dauc_* call (static storage). */
const char* dauc_strerror(int status);

/* ------------------------------------------------- a1: label map + p_hat */

/*
 * Replaces main.py:303-310 (label map, class counts and p_hat, including the
 * per-step device->host sync the reference pays at 309-310).
 *   y_out[i]  = (labels[i] <= split_index) ? -1 : +1               (int8)
 *   lcounts[0] += #{y == +1};  lcounts[1] += #{y == -1}              (fp32 accumulators; exact below 2^24)
 *   p_hat[0]  = (float)( (double)fp32(gpos+lpos) /
 *                        (double)fp32(((gpos+lpos)+gneg)+lneg) )    (gcounts = {gpos, gneg}, fp32)
 * labels: int64 [B] class indices. lcounts is normally the two count slots at
 * the tail of the CoDA flat buffer (so they ride in the averaging all-reduce).
 */
int dauc_label_map_phat(const int64_t* labels, int64_t B, int64_t split_index, int8_t* y_out,
                        float* lcounts, const float* gcounts, float* p_hat, dauc_stream_t stream);

/* ---------------------------------------------- a2+a3: fused surrogate */

/* Bytes of zero-initialised scratch dauc_surrogate_fwdbwd / dauc_class_sums need for B elements. */
size_t dauc_surrogate_workspace_size(int64_t B);

/*
 * Replaces the inline loss of main.py:313-317 and its autograd backward
 * (main.py:326) in ONE pass over the batch:
 *   F = (1-p) mean((h-a)^2 [y=1]) + p mean((h-b)^2 [y=-1])
 *       + 2(1+alpha) mean(p h [y=-1] - (1-p) h [y=1]) - p(1-p) alpha^2      (means divide by B)
 * Inputs : h [B] fp32 with element stride h_stride (e.g. 2 for column 1 of a [B,2] softmax),
 *          y [B] of type y_dtype (+1 positive, -1 negative, anything else in neither class),
 *          abalpha = {a, b, alpha} fp32 [3], p_hat fp32 [1].
 * Outputs: dh [B] fp32 with element stride dh_stride = dF/dh (nullable: skip),
 *          out64 [6] fp64 = {F, dF/da, dF/db, dF/dalpha, n_pos, n_neg} (nullable),
 *          grad3 [3] fp32 = {dF/da, dF/db, dF/dalpha} (nullable; normally the tail of the flat grad),
 *          loss [1] fp32 = F (nullable).
 * Reductions accumulate in fp64 in a fixed order: results are bitwise reproducible.
 */
int dauc_surrogate_fwdbwd(const float* h, int64_t h_stride, const void* y, int y_dtype, int64_t B,
                          const float* abalpha, const float* p_hat, float* dh, int64_t dh_stride,
                          double* out64, float* grad3, float* loss, void* workspace,
                          size_t workspace_bytes, dauc_stream_t stream);

/*
 * The sticky status of a surrogate workspace (a BLOCKING call: it synchronises `stream` and reads
 * one word into the HOST *status_out): 0 = every dauc_surrogate_fwdbwd on this workspace since the
 * last clear completed its reduction; bit 0 set = a reducer of the one-launch loss (unit-stride
 * batches of 2^22 or more) gave up waiting for a row, and that call's F and gradients are NaN --
 * a failed reduction, not a diverged loss. clear != 0 resets the word (the library never does).
 */
int dauc_surrogate_status(void* workspace, size_t workspace_bytes, unsigned* status_out, int clear,
                          dauc_stream_t stream);

/*
 * Replaces the stage-start alpha estimate of main.py:166-188 (per batch):
 *   sums4 (+)= { sum h[y=-1], #{y=-1}, sum h[y=1], #{y=1} }       (fp64 [4])
 * accumulate != 0 adds into sums4, otherwise overwrites it.
 */
int dauc_class_sums(const float* h, int64_t h_stride, const void* y, int y_dtype, int64_t B,
                    double* sums4, int accumulate, void* workspace, size_t workspace_bytes,
                    dauc_stream_t stream);

/*
 * the same loss straight from the 2-way logits z [B,2] (row stride
 * ldz, fp32 or bf16), i.e. with the backbone's final softmax (resnet.py:159, 218)
 * folded into the kernel: h = 1/(1+exp(z0-z1)) in fp32, and the backward through
 * the softmax column fused: dz[i,1] = dF/dh_i * h_i*(1-h_i), dz[i,0] = -dz[i,1]
 * (dz same dtype as z, row stride lddz; nullable). h_out [B] fp32 (nullable)
 * receives the probabilities. Other outputs as dauc_surrogate_fwdbwd.
 */
int dauc_surrogate_logits_fwdbwd(const void* z, int z_dtype, int64_t ldz, const void* y, int y_dtype,
                                 int64_t B, const float* abalpha, const float* p_hat, void* dz, int64_t lddz,
                                 float* h_out, double* out64, float* grad3, float* loss, void* workspace,
                                 size_t workspace_bytes, dauc_stream_t stream);

/* dauc_class_sums from the logits (h = softmax(z)[:,1] computed in the kernel; h_out nullable). */
int dauc_class_sums_logits(const void* z, int z_dtype, int64_t ldz, const void* y, int y_dtype, int64_t B,
                           float* h_out, double* sums4, int accumulate, void* workspace, size_t workspace_bytes,
                           dauc_stream_t stream);

/*
 * main.py:197: alpha[0] = (float)(sums4[0]/sums4[1] - sums4[2]/sums4[3]).
 */
int dauc_alpha_from_sums(const double* sums4, float* alpha, dauc_stream_t stream);

/* ---------------------------------------- a4+a5: primal-dual update */

/* One parameter tensor's gradient, located at w + offset inside the flat buffer. */
typedef struct dauc_grad_seg {
    const float* grad; /* device pointer, dense, same physical element order as the parameter */
    int64_t offset;    /* element offset of the parameter inside w / w0 / w_avg (offset+numel < 2^31) */
    int64_t numel;
} dauc_grad_seg;

/*
 * Replaces dppd_sg (main.py:56-64) for every named parameter, fused with the
 * per-step running average (main.py:333-334), over the flat parameter buffer:
 *   w[i]     <- w[i] - lr*(g[i] + inv_gamma*(w[i] - w0[i]))      (fp32, op order of main.py:61, no FMA)
 *   w_avg[i] <- w_avg[i] + w[i]                                  (if w_avg != NULL)
 * The gradients stay where autograd left them: segs (HOST array, nseg entries)
 * gives each parameter's gradient pointer and its offset in the flat buffer.
 * If scalars != NULL, the same launch also applies the scalar part:
 *   scalars = {a, b, alpha} fp32 [3], grad3 = {dF/da, dF/db, dF/dalpha}, anchor3 = {a0, b0, alpha0}
 *   a <- a - lr*(da + inv_gamma*(a - a0))
 *   b <- b - lr*(db + inv_gamma*(a_new - a0))     [REFERENCE] / (b - b0) [PAPER]
 *   alpha unchanged                                [REFERENCE] / alpha + lr*dalpha [PAPER]
 */
int dauc_pd_update(float* w, const float* w0, float* w_avg, const dauc_grad_seg* segs, int nseg,
                   float* scalars, const float* grad3, const float* anchor3, float lr,
                   float inv_gamma, int mode, dauc_stream_t stream);

/*
 * Same update over one dense gradient (w, g, w0, w_avg all [n]): the
 * single-tensor form used by the micro-benchmarks and by callers whose
 * gradient already lives in one buffer.
 */
int dauc_pd_update_dense(float* w, const float* g, const float* w0, float* w_avg, int64_t n,
                         float lr, float inv_gamma, dauc_stream_t stream);

/* ----------------------------------------------- a6: CoDA averaging */

/*
 * Completes one CoDA averaging round (main.py:33-54 + 297-301) after the
 * caller's SUM all-reduce of the flat buffer:
 *   flat[i] <- flat[i] / world            for i < n_avg        (parameters, a, b, alpha)
 *   gcounts[k] <- gcounts[k] + lcounts[k]; lcounts[k] <- 0     (k = 0 pos, 1 neg; fp32)
 * With world == 1 the caller skips the all-reduce and this only folds the counts.
 */
int dauc_coda_finalize(float* flat, int64_t n_avg, int world, float* lcounts, float* gcounts,
                       dauc_stream_t stream);

/* x[i] <- x[i] / divisor (fp32 IEEE division): stage-end average, main.py:338-339. */
int dauc_scale_div(float* x, int64_t n, float divisor, dauc_stream_t stream);

/* ------------------------------------------------ a8: exact AUC count */

/* Bytes of zero-initialised scratch dauc_split_scores needs for n scores. */
size_t dauc_split_workspace_size(int64_t n);

/*
 * Stable split of (scores, labels) into positive (label == 1) and negative
 * (label != 1) score lists, the sklearn roc_curve(pos_label=1) convention used
 * by main.py:79-80, in original order:
 *   pos_out[0..P), neg_out[0..N), each sized n by the caller (neg_out may be NULL:
 *   only the positives are written).
 *   stats[4] (int64) = { P, N, #non-finite scores, #labels not in {-1, 1} }
 */
int dauc_split_scores(const float* scores, const void* labels, int label_dtype, int64_t n,
                      float* pos_out, float* neg_out, int64_t* stats, void* workspace,
                      size_t workspace_bytes, dauc_stream_t stream);

/*
 * Stable compaction of the positive scores (label == 1) for the sort method of main.py:79-81
 * (sklearn roc_curve(pos_label=1) -> _binary_clf_curve, _ranking.py:826-908): every label is
 * read once and only the positives' scores are read, so a vector with few positives costs
 * about one label pass (1 B per score at int8) instead of a full split. Two launches (per-tile
 * counts and 1-bit positive masks; a write pass in which every tile sums the counts before it
 * itself and reads its masks instead of the labels).
 *   pos_out[0..P) = the positive scores in original order (capacity n)
 *   stats[4] (int64) = { P, n - P, #non-finite POSITIVE scores, #labels not in {-1, 1} }
 * The negatives' scores are checked by dauc_auc_counts_sorted_labeled (its nonfinite count).
 * workspace >= dauc_compact_workspace_size(n) bytes, 16-byte aligned; no zeroing needed.
 */
size_t dauc_compact_workspace_size(int64_t n);
int dauc_compact_positives(const float* scores, const void* labels, int label_dtype, int64_t n,
                           float* pos_out, int64_t* stats, void* workspace, size_t workspace_bytes,
                           dauc_stream_t stream);

/*
 * Exact pairwise count replacing sklearn roc_curve + auc (main.py:79-81):
 *   wins_ties[0] += #{(i, j): pos[i] >  neg[j]}
 *   wins_ties[1] += #{(i, j): pos[i] == neg[j]}      (fp32 equality: -0 == +0)
 * AUC = (2*wins + ties) / (2*P*N). Integer-exact; scores must be finite.
 */
int dauc_pair_count(const float* pos, int64_t P, const float* neg, int64_t N,
                    unsigned long long* wins_ties, dauc_stream_t stream);

/*
 * Bytes of scratch dauc_sort_keys needs for n keys, and dauc_auc_counts_sorted needs for
 * n = min(P, N) (the smaller class is the one sorted). No zeroing needed.
 */
size_t dauc_sort_workspace_size(int64_t n);

/*
 * Same counts as dauc_pair_count by sorting instead of enumerating pairs
 * (SURVEY §8f row 1): LSD radix sort of the smaller class's order-preserving uint32
 * keys (-0 == +0), then every score of the larger class is located in it through an
 * LDS-resident search tree of every k-th key plus one bucket load (upper_bound and
 * lower_bound). O(M log M + L log M), M = min(P, N), L = max(P, N); wins_ties
 * accumulates like dauc_pair_count. Scores must be finite.
 */
int dauc_auc_counts_sorted(const float* pos, int64_t P, const float* neg, int64_t N,
                           unsigned long long* wins_ties, void* workspace, size_t workspace_bytes,
                           dauc_stream_t stream);

/*
 * dauc_auc_counts_sorted without materialised negatives: the sorted table is the
 * positives pos[0..P); the queries are the elements of scores/labels in [begin, end)
 * whose label is not 1 (the full arrays, as given to dauc_compact_positives). Same
 * accumulation into wins_ties; nonfinite (device uint64 [1], nullable) += the number of
 * queried scores that are NaN or +-inf (the only check the negatives get: sklearn's
 * _ranking.py:868-869 rejects them). workspace >= dauc_sort_workspace_size(P). The search
 * structure behind the sort is chosen on the device: the LDS count index (one 16-byte window
 * gather per query) where it holds the table; else, for a table of at most 14,000 DISTINCT keys
 * (tie-heavy: rounded scores, a bf16 model's probabilities), the LDS distinct-key index (no
 * gather); else the LDS search tree. Same integers whichever runs.
 */
int dauc_auc_counts_sorted_labeled(const float* pos, int64_t P, const float* scores, const void* labels,
                                   int label_dtype, int64_t begin, int64_t end, unsigned long long* wins_ties,
                                   unsigned long long* nonfinite, void* workspace, size_t workspace_bytes,
                                   dauc_stream_t stream);

/*
 * The exact-AUC evaluation of main.py:79-81 (sklearn roc_curve + auc over one test set), as ONE
 * stream-ordered sequence with no host synchronisation and no allocation: one zeroing launch (the
 * record and the workspace's top-bucket histogram), a one-pass positive compaction (labels read once, P counted on the device),
 * the count index built straight from the unsorted positives with the table size read on the
 * device, and the query pass over this part's scores [part*n/parts, (part+1)*n/parts), whose
 * labels are not 1 (every part builds the index over ALL the positives itself: ranks holding the
 * same test set need no collective to share the table). The kernels count straight into the
 * record (no copy), so part_out must not overlap the workspace (DAUC_EINVAL if it does):
 *   part_out (DEVICE int64[8], 8-byte aligned) = { W_part, T_part, #non-finite queried scores of this part,
 *                                  P, 0, #non-finite positives, #labels not in {-1, 1}, verdict }
 * The first three sum over the parts (the caller's all-reduce); the rest are the same on every
 * part. verdict (low 32 bits): 0 = nothing to query (empty part), 1 = counted, 2 = the count index
 * cannot hold this table (more than 219,838 positives or n/2 + 1, or clustered / tie-heavy
 * positives): take dauc_auc_eval_counts(_part), which then runs the sorted path. N = n - P.
 * workspace >= dauc_auc_eval_workspace_size(n) bytes, 256-byte aligned; its contents need no
 * initialisation and are not used after the call (one workspace per stream at a time).
 */
size_t dauc_auc_eval_workspace_size(int64_t n);
int dauc_auc_eval_enqueue(const float* scores, const void* labels, int label_dtype, int64_t n, int part, int parts,
                          int64_t* part_out, void* workspace, size_t workspace_bytes, dauc_stream_t stream);

/*
 * The whole single-GPU evaluation as ONE blocking call (sklearn's roc_curve + auc is a blocking
 * host call too): the sequence above, ONE readback of its record into `pinned` (caller-owned
 * page-locked host memory of >= 8 int64, e.g. hipHostMalloc; the call writes and reads it) and a
 * synchronisation of `stream`; for verdict 2 the sorted path (radix sort of the positives + the
 * LDS distinct-key index for tie-heavy tables, or the search tree; or, when the negatives are the
 * smaller class, both classes split and the negatives sorted) and one more readback. Stateless:
 * same inputs, same work.
 *   out[6] (HOST int64) = { W, T, P, N, #non-finite scores, #labels not in {-1, 1} }
 *   (W = T = 0 when a class is empty or a score is non-finite: the caller raises like sklearn)
 */
int dauc_auc_eval_counts(const float* scores, const void* labels, int label_dtype, int64_t n, int64_t* out,
                         int64_t* pinned, void* workspace, size_t workspace_bytes, dauc_stream_t stream);

/*
 * Part `part` of `parts` of the blocking evaluation (the sorted path of a verdict-2 test set,
 * sharded: scores [part*n/parts, (part+1)*n/parts) when P <= N, positives [part*P/parts,
 * (part+1)*P/parts) against the sorted negatives when P > N). The parts' counts sum to
 * dauc_auc_eval_counts's for every `parts`.
 *   out[7] (HOST int64) = { W_part, T_part, P, N, #non-finite positives, #labels not in {-1, 1},
 *                           #non-finite queried scores of this part }
 *   part_counts (DEVICE int64[3], may be NULL): receives { W_part, T_part, out[6] } on `stream`
 *   (enqueued, not synchronised) -- the buffer the caller all-reduces.
 */
int dauc_auc_eval_counts_part(const float* scores, const void* labels, int label_dtype, int64_t n, int part,
                              int parts, int64_t* out, int64_t* part_counts, int64_t* pinned, void* workspace,
                              size_t workspace_bytes, dauc_stream_t stream);

/*
 * The sharded evaluation without a whole-vector compaction on every rank, in two enqueued steps
 * around the caller's collective (no host synchronisation in either). Slice r of n labels is
 * [lo(r), lo(r+1)) with lo(0) = 0, lo(parts) = n and lo(r) = (r*n/parts) rounded down to a multiple
 * of 256.
 *   1. dauc_auc_eval_compact_part: the positives of THIS rank's slice compacted, unordered, into
 *      `slot` (device, dauc_auc_slot_bytes(n, parts) bytes -- the same for every n --, 256-byte
 *      aligned, outside the workspace; step 2's index-build state in `workspace` is prepared --
 *      per-cell counters zeroed, the cell-slotted table filled with +inf --, so step 2 must use the
 *      same workspace, and each step 2 needs its own step 1: a second step 2 on the same state
 *      reports verdict 2 instead of counting twice): a header of int64 words {P_r, 0, #non-finite
 *      positives, #labels not in {-1, 1}, n} at byte 0, the top-bucket histogram of the positives'
 *      order-preserving keys (2048 uint32: key >> 21) from byte 256 and the scores from byte 8448;
 *   -- the caller all-gathers the `parts` slots, rank order, contiguous --
 *   2. dauc_auc_eval_query_part: the count index is built from the gathered slots read in place
 *      (headers and histograms summed) and the scores of the NEXT rank's slice, (part + 1) %
 *      parts, are counted straight into part_out (device int64[8], 8-byte aligned, outside the
 *      workspace and the slots; DAUC_EINVAL otherwise) = dauc_auc_eval_enqueue's record, except
 *      word 4, a consistency check that is 0 when the ranks agree: low 32 bits = the P of the
 *      queried slice's slot - the positives this rank's labels give over that slice, mod 2^32;
 *      high 32 bits = the number of slots built for another n (parts <= 1024). A slot holds an
 *      even share of the count index's capacity + 25 %:
 *      a slice with more positives (an unshuffled test set), like a table the index cannot hold,
 *      gives verdict 2 -- the caller then runs dauc_auc_eval_query_part_sorted on every rank, and
 *      where that reports verdict 2 too, dauc_auc_eval_counts_part.
 *   dauc_auc_eval_query_part_sorted (verdict-2 path, after the caller has read the records): the
 *      gathered slots' positives (P of them, the records' word 3) are copied into one table, which
 *      is sorted and searched (the distinct-key index for tie-heavy tables, else the LDS tree), and
 *      THIS rank's own slice of the scores is counted into part_out (zeroed first): {W_part,
 *      T_part, #non-finite queried scores, P, 0, 0, 0, verdict}; verdict 2 when a slot overflowed,
 *      the slots do not hold P positives, or P > n - P -- then dauc_auc_eval_counts_part. No host
 *      synchronisation; the same workspace, slots and alignment rules as step 2.
 * Replaces the reference's rank-0 evaluation (main.py:232-250) with a sharded one.
 */
size_t dauc_auc_slot_bytes(int64_t n, int parts);
int dauc_auc_eval_compact_part(const float* scores, const void* labels, int label_dtype, int64_t n, int part,
                               int parts, void* slot, void* workspace, size_t workspace_bytes, dauc_stream_t stream);
int dauc_auc_eval_query_part(const float* scores, const void* labels, int label_dtype, int64_t n, int part, int parts,
                             const void* slots, int64_t* part_out, void* workspace, size_t workspace_bytes,
                             dauc_stream_t stream);
int dauc_auc_eval_query_part_sorted(const float* scores, const void* labels, int label_dtype, int64_t n, int part,
                                    int parts, const void* slots, int64_t P, int64_t* part_out, void* workspace,
                                    size_t workspace_bytes, dauc_stream_t stream);

/* The radix sort alone: keys_out[0..n) = ascending order-preserving keys of scores (testing). */
int dauc_sort_keys(const float* scores, int64_t n, unsigned* keys_out, void* workspace,
                   size_t workspace_bytes, dauc_stream_t stream);

/* ------------------------------------- backbone: fused BatchNorm + add + ReLU */

/*
 * Training-mode BatchNorm over channels-last activations x [M, C] (M = N*H*W rows,
 * C contiguous; dtype bf16 or fp32; C a power-of-two multiple of the 16-byte vector,
 * 16-byte aligned pointers), fused with the residual add and the ReLU that follow it
 * in the ResNet blocks (resnet.py:47-64, 87-108, 203-206):
 *   y = relu?( (x - mean) * invstd * gamma + beta  (+ residual) )
 * with batch mean / biased variance over M, invstd = 1/sqrt(var + eps), and the
 * running statistics updated as torch does (unbiased variance, momentum). gamma,
 * beta, running_* are fp32 [C] (nullable: affine off / no running stats);
 * save_mean, save_invstd fp32 [C] receive the batch statistics for the backward.
 * relu_mask (nullable; relu only): one byte per 16-byte vector of y ([M * C * elem / 16] bytes),
 * bit i = (stored element i of the vector > 0): the backward's ReLU mask in 1/16 (bf16) of y's bytes.
 * Workspace: dauc_bn_workspace_size(M, C) bytes, 16-byte aligned, no zeroing needed.
 */
size_t dauc_bn_workspace_size(int64_t M, int C);
int dauc_bn_act_forward(const void* x, int dtype, int64_t M, int C, const void* residual, int relu,
                        const float* gamma, const float* beta, float* running_mean, float* running_var,
                        float momentum, float eps, void* y, uint8_t* relu_mask, float* save_mean, float* save_invstd,
                        void* workspace, size_t workspace_bytes, dauc_stream_t stream);

/*
 * Backward of dauc_bn_act_forward. g = dy * [y > 0] (relu; y = the forward output, or relu_mask --
 * the forward's mask bytes, read instead of y when non-null) or dy.
 *   dres (nullable) <- g: the gradient of the residual input;
 *   dx <- gamma*invstd*(g - mean(g) - xhat*mean(g*xhat)); dgamma <- sum g*xhat; dbeta <- sum g
 * (dgamma / dbeta fp32 [C], nullable).
 */
int dauc_bn_act_backward(const void* dy, const void* y, const uint8_t* relu_mask, const void* x, int dtype, int64_t M,
                         int C, int relu, const float* gamma, const float* save_mean, const float* save_invstd,
                         void* dres, void* dx, float* dgamma, float* dbeta, void* workspace, size_t workspace_bytes,
                         dauc_stream_t stream);

/* ------------------------------------------------ backbone: stem max-pool */

/*
 * Max pooling over channels-last x [N, H, W, C] (bf16 or fp32; C a multiple of the
 * 16-byte vector; 16-byte aligned; N <= 65535), square kernel, stride, zero-free padding
 * (pad <= kernel / 2, kernel^2 <= 127), floor mode: Ho = (H + 2 pad - kernel) / stride + 1.
 * Replaces torch's max_pool2d_with_indices of resnet.py:205 (the stem). argmax int8
 * [N, Ho, Wo, C] (8-byte aligned) receives each maximum's position inside its window
 * (row * kernel + column; -1 = no element compared greater than -inf, torch's index 0).
 * Output, comparisons (NaN wins) and the backward's fp32 summation order are torch's:
 * bit-identical results.
 */
int dauc_maxpool2d_forward(const void* x, int dtype, int64_t N, int H, int W, int C, int kernel, int stride,
                           int pad, void* y, int8_t* argmax, int Ho, int Wo, dauc_stream_t stream);

/* dx [N, H, W, C] <- the gradient of dauc_maxpool2d_forward given dy [N, Ho, Wo, C]. */
int dauc_maxpool2d_backward(const void* dy, const int8_t* argmax, int dtype, int64_t N, int H, int W, int C,
                            int kernel, int stride, int pad, int Ho, int Wo, void* dx, dauc_stream_t stream);

/* ---------------------------------- backbone: split-K weight-gradient sum */

/*
 * out[i] = sum over s = 0 .. S-1 (ascending) of part[s * n + i], fp32; n % 4 == 0, 16-byte
 * aligned pointers. The last step of the 1x1 convolutions' split-K weight gradient
 * (conv1x1.py: S slab GEMMs over the N*H*W rows). Bitwise reproducible.
 */
int dauc_slab_sum(const float* part, int64_t S, int64_t n, float* out, dauc_stream_t stream);

/* ---------------------------------- backbone: 3x3 convolution weight gradient */

/*
 * dw[co][kh][kw][ci] (fp32, the channels-last [Co, Ci, 3, 3] weight's memory order) <-
 *   sum over output pixels (n, ho, wo) of dy[n][ho][wo][co] * x[n][ho*stride - 1 + kh][wo*stride - 1 + kw][ci]
 * for a 3x3 convolution with padding 1 and stride 1 or 2: x [N, H, W, Ci] and dy [N, Ho, Wo, Co]
 * channels-last bf16 (dtype DAUC_DTYPE_BF16 only), Ci and Co multiples of 64, 16-byte aligned
 * pointers, N*H*W and N*Ho*Wo < 2^31. A split-K MFMA implicit GEMM with fp32 accumulation; the
 * splits' fp32 partials go to `workspace` (dauc_conv3x3_wgrad_workspace_size bytes; 0 = none
 * needed) and are summed in split order (dauc_slab_sum): bitwise reproducible. Replaces MIOpen's
 * backward-weights call of the ResNet 3x3 convolutions under bf16 autocast (resnet.py:72-108,
 * main.py:326) and autograd's bf16 -> fp32 cast of its result.
 */
size_t dauc_conv3x3_wgrad_workspace_size(int64_t N, int Ho, int Wo, int Ci, int Co);
int dauc_conv3x3_wgrad(const void* x, const void* dy, int dtype, int64_t N, int H, int W, int Ci, int Ho, int Wo,
                       int Co, int stride, float* dw, void* workspace, size_t workspace_bytes, dauc_stream_t stream);

/* ---------------------------------- backbone: the 7x7 / stride-2 stem convolution */

/*
 * The stem convolution conv1 = Conv2d(3, 64, 7, stride 2, padding 3, no bias) (imagenet/resnet.py:145)
 * on channels-last bf16 (dtype DAUC_DTYPE_BF16 only): x [N, H, W, 3], weight [64][7][7][3] (the
 * channels-last memory order of [64, 3, 7, 7]), y / dy [N, Ho, Wo, 64] with Ho = (H - 1) / 2 + 1,
 * Wo = (W - 1) / 2 + 1; x, y and dy 16-byte aligned, N*H*W*3 and N*Ho*Wo*64 < 2^31. MFMA with fp32
 * accumulation: forward y = bf16(sum) rounded once; weight gradient dw (fp32, [64][7][7][3])
 * through per-workgroup slabs in `workspace` (dauc_conv7x7s2_stem_wgrad_workspace_size bytes)
 * summed in workgroup order (dauc_slab_sum): bitwise reproducible. Replaces MIOpen's forward and
 * backward-weights calls for the stem under bf16 autocast (main.py:311-326) and autograd's
 * bf16 -> fp32 cast of the gradient. The stem's input gradient is never needed (the image).
 */
int dauc_conv7x7s2_stem_forward(const void* x, const void* w, int dtype, int64_t N, int H, int W, int Ho, int Wo,
                                void* y, dauc_stream_t stream);
size_t dauc_conv7x7s2_stem_wgrad_workspace_size(int64_t N, int Ho, int Wo);
int dauc_conv7x7s2_stem_wgrad(const void* x, const void* dy, int dtype, int64_t N, int H, int W, int Ho, int Wo,
                              float* dw, void* workspace, size_t workspace_bytes, dauc_stream_t stream);

/* ---------------------------------- backbone: strided and broadcast copies (channels-last bf16) */

/*
 * The strided 1x1 downsample's backward (conv1x1.py; resnet.py:87-108) and the average pool's
 * gradient (resnet.py:214), bf16 (DAUC_DTYPE_BF16) channels-last, C a multiple of 8, 16-byte
 * aligned pointers. Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1.
 *   dauc_strided_pick:  out[n][i][j][:] = x[n][stride i][stride j][:]   (x [N, H, W, C], out [N, Ho, Wo, C])
 *   dauc_strided_add:   dx[n][stride i][stride j][:] += src[n][i][j][:] (fp32 sum rounded to bf16,
 *                       bit-identical to torch's add_ on the strided view)
 *   dauc_broadcast_hw:  out[n][p][:] = g[n][:] for p < HW           (g [N, C], out [N, HW, C])
 */
int dauc_strided_pick(const void* x, int dtype, int64_t N, int H, int W, int C, int stride, void* out,
                      dauc_stream_t stream);
int dauc_strided_add(void* dx, int dtype, int64_t N, int H, int W, int C, int stride, const void* src,
                     dauc_stream_t stream);
int dauc_broadcast_hw(const void* g, int dtype, int64_t N, int64_t HW, int C, void* out, dauc_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* DAUC_H_ */
