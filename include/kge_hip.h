/*
 * kge_hip.h — C-ABI of libkge_hip.so, the MI355X (gfx950) knowledge-graph-embedding scoring path.
 *
 * This is the drop-in boundary for the hot path of NguyenThaiHoc1/CustomKnowledgeGraphEmbedding:
 * the score-function plugins (`TFKGEModel.model_func`, tensorflow_codes/model.py:109-112), the
 * per-mode gather + score + reduce of `TFKGEModel.call` (model.py:114-205), and the embedding
 * lookup / score path of the upstream PyTorch `KGEModel.forward` (KnowledgeGraphEmbedding/codes/
 * model.py — absent from the snapshot, restated in oracle/kge_oracle.py).
 *
 * Contract (all entry points):
 *   - every pointer is caller-owned DEVICE memory (the library never allocates or frees);
 *   - every launch is asynchronous on the caller's hipStream_t (`stream`, may be NULL = default
 *     stream); no host synchronisation happens inside the library, so calls are graph-capturable;
 *   - return 0 on success or a negative errno-style code (KGE_EINVAL, KGE_ENOTSUP, KGE_EHIP);
 *     the message for the calling thread is in kge_last_error();
 *   - forward results are deterministic (fixed reduction order, no atomics);
 *   - an out-of-range entity/relation index reads a ZERO row, like TF's GPU `tf.gather`
 *     (model.py:130-136,152-158,178-185); it never faults.
 *
 * Layout: tables are row-major fp32, row i of the entity table at ent + i*ent_ld.
 *   Split models keep the two halves of a row back to back: [re | im] for ComplEx/RotatE,
 *   [a | b] for InterHT (model.py:208,210), so a row holds 2*D floats; D is the per-half width
 *   (= hidden_dim). TransE/DistMult rows hold D floats.
 *   The relation part a score function reads starts at rel + r*rel_ld + rel_off: InterHT reads
 *   only the middle third (re_mid, model.py:209 -> rel_off = D), everything else rel_off = 0.
 */
#ifndef KGE_HIP_H
#define KGE_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KGE_ABI_VERSION 1

/* score functions: model_func keys (model.py:109-112 + upstream codes/model.py model_func) */
enum kge_fn {
    KGE_TRANSE = 0,   /* upstream TransE:   gamma - ||h + r - t||_1                        */
    KGE_DISTMULT = 1, /* upstream DistMult: sum(h * r * t)                                  */
    KGE_COMPLEX = 2,  /* upstream ComplEx:  Re<h, r, conj(t)>                               */
    KGE_ROTATE = 3,   /* upstream RotatE:   gamma - sum |h o e^{i theta_r} - t|             */
    KGE_INTERHT = 4,  /* model.py:207-224                                                   */
    KGE_PROTATE = 5   /* upstream pRotatE:  gamma - modulus * sum |sin(ph_h + ph_r - ph_t)| */
};

/* mode codes of the TF reference (Q1: model.py:124,203; supervisor.py:18) */
enum kge_mode {
    KGE_HEAD_BATCH = 0, /* candidates replace the head  (model.py:148-172) */
    KGE_TAIL_BATCH = 1, /* candidates replace the tail  (model.py:174-199) */
    KGE_SINGLE = 3      /* the positive triple only     (model.py:127-146) */
};

#define KGE_EINVAL (-22)
#define KGE_ENOTSUP (-95)
#define KGE_EHIP (-1000)

/* Version of this ABI (KGE_ABI_VERSION). */
int kge_abi_version(void);

/* Last error message of the calling thread ("" if none). */
const char* kge_last_error(void);

/* Largest per-half width D the forward kernels accept for a score function (in floats). */
int64_t kge_max_dim(int fn);

/* Which form kge_step_forward (without cand_stats) uses for a table of nentity rows and N negatives
 * per batch row: 0 = one launch, batch-row-major; 1 = two launches, XCD-sliced (see kge_step_forward). */
int kge_step_forward_order(int64_t nentity, int64_t N);

/*
 * Fused gather + score (replaces model.py:127-137,148-159,174-185 gathers + model_func calls at
 * :139-144,161-166,187-192; upstream KGEModel.forward gathers + model_func).
 *   pos    [B,3] int64 (h, r, t) rows of the batch, row stride 3
 *   neg    [B,N] int64 candidate entity ids (row stride neg_ld); ignored for KGE_SINGLE
 *   scores [B,N] fp32 raw scores out (row stride scores_ld); N is forced to 1 for KGE_SINGLE
 *   gamma, emb_range: model.py:60-63 (emb_range = (gamma + 2) / hidden_dim);
 *   modulus: pRotatE only (upstream 0.5 * emb_range initial value; pass the current parameter).
 */
int kge_score_indexed(int fn, int mode,
                      const float* ent, int64_t nentity, int64_t ent_ld,
                      const float* rel, int64_t nrelation, int64_t rel_ld, int64_t rel_off,
                      const int64_t* pos, const int64_t* neg, int64_t neg_ld,
                      int64_t B, int64_t N, int64_t D,
                      float gamma, float emb_range, float modulus,
                      float* scores, int64_t scores_ld, void* stream);

/*
 * Fused forward of one TF train step (supervisor.py:17-18): the negative call
 * model(((pos, neg), mode)) and the positive call model(((pos, neg), 3)). Two forms, chosen per call by
 * kge_step_forward_order (results bitwise identical):
 *   0: ONE launch: a block per batch row scores its negatives, then finishes the row (positive, reduction);
 *   1: TWO launches: the negatives and positives in XCD-sliced order (each XCD gathers only the rows of
 *      one eighth of the table, every wave in ascending id order, so repeat gathers of a row hit the
 *      XCD's L2 / the Infinity Cache), then one wave per row reduces it. Used for N >= 128 unless
 *      KGE_STEP_ORDER=row|xcd overrides; without cand_stats only.
 *   mode       KGE_HEAD_BATCH or KGE_TAIL_BATCH (the batch's negative mode)
 *   neg_scores [B,N] raw negative scores (out, row stride ns_ld) — kept for the backward
 *   out_neg    [B]   reduced negative branch: adversarial != 0 -> sum softmax(T s) logsigmoid(-s)
 *                    (model.py:168-171,195-198), else mean logsigmoid(-s)
 *   pos_scores [B]   raw positive scores, single-mode formula (out, may be NULL)
 *   out_pos    [B]   logsigmoid(positive score) (model.py:145)
 *   cand_stats [B*N] float2 (may be NULL): InterHT keeps each candidate's inverse half-norms here for
 *                    kge_step_backward(_adam), whose phase 1 then streams the candidates column-group-wise
 */
int kge_step_forward(int fn, int mode,
                     const float* ent, int64_t nentity, int64_t ent_ld,
                     const float* rel, int64_t nrelation, int64_t rel_ld, int64_t rel_off,
                     const int64_t* pos, const int64_t* neg, int64_t neg_ld,
                     int64_t B, int64_t N, int64_t D,
                     float gamma, float emb_range, float modulus,
                     float temperature, int adversarial,
                     float* neg_scores, int64_t ns_ld, float* out_neg,
                     float* pos_scores, float* out_pos, float* cand_stats, void* stream);

/*
 * Second half of kge_step_forward, on scores kge_score_indexed already wrote: one wave per batch
 * row scores the positive triple (single mode) and reduces the row's N negative scores.
 */
int kge_step_finish(int fn,
                    const float* ent, int64_t nentity, int64_t ent_ld,
                    const float* rel, int64_t nrelation, int64_t rel_ld, int64_t rel_off,
                    const int64_t* pos, int64_t B, int64_t D,
                    float gamma, float emb_range, float modulus,
                    const float* neg_scores, int64_t N, int64_t ns_ld,
                    float temperature, int adversarial,
                    float* out_neg, float* pos_scores, float* out_pos, void* stream);

/*
 * Owner-computes scoring on a ROW-SHARDED entity table. This shard holds global rows
 * [shard_lo, shard_lo + shard_rows). Query-entity rows are pre-assembled by the caller (row b of
 * `qent`, e.g. kge_gather_rows + a SUM all-reduce over shards); the relation table is replicated.
 * Candidates this shard does not own score exactly 0 and cost no memory traffic, so a SUM
 * reduce over shards yields the unsharded scores bitwise. For KGE_SINGLE the candidate is pos[b,2].
 */
int kge_score_sharded(int fn, int mode,
                      const float* qent, int64_t q_ld,
                      const float* rel, int64_t nrelation, int64_t rel_ld, int64_t rel_off,
                      const float* shard, int64_t shard_rows, int64_t shard_ld, int64_t shard_lo,
                      const int64_t* pos, const int64_t* neg, int64_t neg_ld,
                      int64_t B, int64_t N, int64_t D,
                      float gamma, float emb_range, float modulus,
                      float* scores, int64_t scores_ld, void* stream);

/*
 * out[i, 0:width] = table[ids[i*id_stride] - lo, 0:width] if 0 <= ids[..] - lo < rows, else 0.
 * Row gather from a (sharded) table; the zero rows make a SUM all-reduce over shards exact.
 */
int kge_gather_rows(const float* table, int64_t rows, int64_t ld, int64_t lo,
                    const int64_t* ids, int64_t id_stride, int64_t n, int64_t width,
                    float* out, int64_t out_ld, void* stream);

/*
 * Link-prediction evaluation against all entities (upstream KGEModel.test_step; BASELINE config C5).
 *
 * kge_eval_query: the query operand of the all-entity contraction for DistMult / ComplEx:
 *   Q[b] = h*r (tail-batch) or r*t (head-batch); ComplEx: [re_q | im_q] (width 2D). Then
 *   score(b, e) = Q[b] . E[e] for every entity e.
 * kge_gemm_nt: C[M,N] = A[M,K] . B[N,K]^T in fp32 on the matrix cores (v_mfma_f32_32x32x2_f32);
 *   K, lda, ldb multiples of 4; A, B 16-byte aligned.
 * kge_rank_filtered: ranks[q] = 1 + #{e != truth[q] : S[q,e] > S[q,truth[q]]}
 *                               - #{f in filter[q], f != truth[q] : S[q,f] > S[q,truth[q]]}
 *   filter[q] = filter_ids[filter_ptr[q] .. filter_ptr[q+1]) (CSR, distinct ids; NULL = no filter):
 *   the entities upstream's filter_bias pushes below the positive. Integer result, exact.
 * Any score function can also score all entities through kge_score_indexed with neg = [0..E)
 * and neg_ld = 0.
 */
int kge_eval_query(int fn, int mode,
                   const float* ent, int64_t nentity, int64_t ent_ld,
                   const float* rel, int64_t nrelation, int64_t rel_ld,
                   const int64_t* pos, int64_t B, int64_t D,
                   float* Q, int64_t ldq, void* stream);
int kge_gemm_nt(const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc,
                int64_t M, int64_t N, int64_t K, void* stream);
/*
 * kge_gemm_nt_bf16x3: the same contraction (arguments as kge_gemm_nt) at fp32 accuracy on the bf16 matrix
 *   cores: each fp32 operand is split in registers into three bf16 terms x = x0 + x1 + x2 (RNE, 24
 *   significant bits) and C = sum of the six products A_i . B_j^T with i + j <= 2 (v_mfma_f32_32x32x16_bf16,
 *   fp32 accumulation). Error vs the fp64 product: the fp32 MFMA path's (tests/test_eval_gpu.py).
 *   Non-finite inputs give NaN.
 */
int kge_gemm_nt_bf16x3(const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc,
                       int64_t M, int64_t N, int64_t K, void* stream);
int kge_rank_filtered(const float* scores, int64_t M, int64_t N, int64_t ld, const int64_t* truth,
                      const int64_t* filter_ptr, const int64_t* filter_ids, int64_t* ranks,
                      void* stream);

/*
 * Score pre-gathered rows: the model_func plugin surface itself,
 * `model_func[name](head, relation, tail, mode) -> [B, 1|N]` (model.py:109-112,207).
 *   head [B, Nh, *] rows (row stride head_ld), Nh = N for KGE_HEAD_BATCH else 1
 *   rel  [B, *]     rows (row stride rel_ld), the used part starts at rel_off
 *   tail [B, Nt, *] rows (row stride tail_ld), Nt = N for KGE_TAIL_BATCH else 1
 */
int kge_score_dense(int fn, int mode,
                    const float* head, int64_t head_ld,
                    const float* rel, int64_t rel_ld, int64_t rel_off,
                    const float* tail, int64_t tail_ld,
                    int64_t B, int64_t N, int64_t D,
                    float gamma, float emb_range, float modulus,
                    float* scores, int64_t scores_ld, void* stream);

/*
 * Per-row negative reduction of TFKGEModel (model.py:168-171,195-198; Q3) and upstream train_step:
 *   adversarial != 0: out[b] = sum_n softmax(T * s[b,:])_n * logsigmoid(-s[b,n])
 *   adversarial == 0: out[b] = mean_n logsigmoid(-s[b,n])
 * scores [B,N] (row stride ld), out [B].
 */
int kge_neg_reduce(const float* scores, int64_t B, int64_t N, int64_t ld,
                   float temperature, int adversarial, float* out, void* stream);

/* out[i] = logsigmoid(x[i]) (model.py:145), n elements. */
int kge_log_sigmoid(const float* x, int64_t n, float* out, void* stream);

/*
 * Backward of kge_neg_reduce: d_scores[b,n] = d_out[b] * d(out[b])/d(s[b,n]).
 *   detach != 0 stops the gradient through the softmax weights (upstream `.detach()`);
 *   detach == 0 is the TF reference (Q3: model.py:168-171 does not stop it).
 */
int kge_neg_reduce_bwd(const float* scores, int64_t B, int64_t N, int64_t ld,
                       float temperature, int adversarial, int detach,
                       const float* d_out, float* d_scores, int64_t d_ld, void* stream);

/* d_x[i] = d_out[i] * sigmoid(-x[i])  (backward of kge_log_sigmoid). */
/*
 * The weighted loss of the train step (supervisor.py:19-23) over the two [B] outputs of
 * kge_step_forward, and its gradient: loss = (-sum(w*pos)/sum(w) - sum(w*neg)/sum(w)) / 2 (device
 * scalar, may be NULL), d_out[b] = dloss/dout_neg[b] = dloss/dout_pos[b] = (-0.5/sum(w)) * w[b]
 * (may be NULL). One block, fixed reduction order (deterministic).
 */
int kge_step_loss(const float* out_neg, const float* out_pos, const float* weight, int64_t B, float* loss,
                  float* d_out, void* stream);

int kge_log_sigmoid_bwd(const float* x, const float* d_out, int64_t n, float* d_x, void* stream);

/*
 * Deterministic backward of kge_step_forward (supervisor.py:25 tape.gradient through both calls),
 * given dL/d(out_neg) and dL/d(out_pos) [B]. OVERWRITES every row of d_ent [nentity, ent_ld] and
 * d_rel [nrelation, rel_ld] (no memset needed) and *d_modulus (pRotatE; may be NULL). No float
 * atomics: phase 1 reduces each batch row's query-side gradient inside one block; phase 2 walks,
 * for every entity row, the gradient events bucketed to it (counting sort) in a fixed order, so
 * the result is bitwise reproducible. detach != 0: upstream's detached self-adversarial weights.
 * cand_stats: the buffer kge_step_forward filled (or NULL; InterHT then uses the register-resident
 * phase 1). workspace: device scratch of kge_step_backward_workspace_size(fn, nentity, B, N, D) bytes.
 */
int64_t kge_step_backward_workspace_size(int fn, int64_t nentity, int64_t B, int64_t N, int64_t D);
int kge_step_backward(int fn, int mode,
                      const float* ent, int64_t nentity, int64_t ent_ld,
                      const float* rel, int64_t nrelation, int64_t rel_ld, int64_t rel_off,
                      const int64_t* pos, const int64_t* neg, int64_t neg_ld,
                      int64_t B, int64_t N, int64_t D,
                      float gamma, float emb_range, float modulus,
                      float temperature, int adversarial, int detach,
                      const float* neg_scores, int64_t ns_ld, const float* pos_scores,
                      const float* d_out_neg, const float* d_out_pos,
                      float* d_ent, float* d_rel, float* d_modulus, const float* cand_stats,
                      void* workspace, int64_t workspace_bytes, void* stream);

/*
 * The whole train step's update (supervisor.py:25-26) with the optimizer FUSED into the backward:
 * the deterministic backward of kge_step_backward, where the entity-major phase applies Adam
 * (keras != 0: Keras rule, else torch.optim.Adam) to each entity row as it finishes its
 * gradient, in place on `ent` / m_ent / v_ent; then Adam on the relation table (and on the
 * pRotatE modulus if modulus_param != NULL). Bitwise identical to kge_step_backward followed by
 * kge_adam_update on every table, without materialising the entity gradient.
 * workspace: kge_step_backward_adam_workspace_size(...) bytes.
 */
int64_t kge_step_backward_adam_workspace_size(int fn, int64_t nentity, int64_t nrelation, int64_t rel_ld,
                                              int64_t B, int64_t N, int64_t D);
int kge_step_backward_adam(int fn, int mode,
                           float* ent, int64_t nentity, int64_t ent_ld,
                           float* rel, int64_t nrelation, int64_t rel_ld, int64_t rel_off,
                           const int64_t* pos, const int64_t* neg, int64_t neg_ld,
                           int64_t B, int64_t N, int64_t D,
                           float gamma, float emb_range, float* modulus_param, float modulus,
                           float temperature, int adversarial, int detach,
                           const float* neg_scores, int64_t ns_ld, const float* pos_scores,
                           const float* d_out_neg, const float* d_out_pos,
                           float* m_ent, float* v_ent, float* m_rel, float* v_rel, float* m_mod, float* v_mod,
                           float lr, float beta1, float beta2, float eps, int64_t step, int keras,
                           const float* cand_stats, void* workspace, int64_t workspace_bytes, void* stream);

/*
 * One whole train step, supervisor.py:15-26 (`train_step_fn`): both model calls (:17-18, negative
 * `mode` + positive single call), the weighted loss (:19-23; weight = subsampling_weight [B]), the
 * gradient (:25) and Adam (:26; keras != 0: Keras rule, else torch.optim.Adam) on both tables, in place.
 * It replaces what the reference spreads over TFKGEModel.call (model.py:114-205), tf.GradientTape and
 * optimizer.apply_gradients. Four launches at D <= 1024:
 *   forward with phase 1 of the backward fused in (each candidate row gathered once per step; online-
 *   softmax running sums, valid for the TF and upstream reductions) and the gradient events counted
 *   per entity; the bucket scan; an epilogue (event scatter, score gradients, query chains, loss);
 *   phase 2 with Adam fused into the entity pass, then the relation gradient with Adam.
 *   D > 1024 (or 4-B-only alignment with D > 256) falls back to the separate phase 1.
 *   pRotatE -> KGE_ENOTSUP (use kge_step_backward_adam).
 *   Outputs: loss [1], out_neg [B] (reduced negative branch), out_pos [B] (logsigmoid of the
 *   positive score), all device memory; loss_sum [1] (or NULL): the running Sum metric
 *   (supervisor.py:28 metrics.update_state), incremented by the loss on the device.
 *   Results equal kge_step_backward_adam's to fp32 rounding (the query gradient is summed in a
 *   different order); deterministic run to run.
 *   workspace: kge_train_step_workspace_size(...) bytes of scratch with NO state between calls: the
 *   call zeroes the per-entity event counters it keeps there itself (an async memset on `stream`), so
 *   any contents (uninitialised, reused at another shape, left by an aborted call) give the same result.
 */
int64_t kge_train_step_workspace_size(int fn, int64_t nentity, int64_t nrelation, int64_t rel_ld,
                                      int64_t B, int64_t N, int64_t D);
int kge_train_step(int fn, int mode,
                   float* ent, int64_t nentity, int64_t ent_ld,
                   float* rel, int64_t nrelation, int64_t rel_ld, int64_t rel_off,
                   const int64_t* pos, const int64_t* neg, int64_t neg_ld,
                   int64_t B, int64_t N, int64_t D,
                   float gamma, float emb_range, float temperature, int adversarial, int detach,
                   const float* weight, float* loss, float* loss_sum, float* out_neg, float* out_pos,
                   float* m_ent, float* v_ent, float* m_rel, float* v_rel,
                   float lr, float beta1, float beta2, float eps, int64_t step, int keras,
                   void* workspace, int64_t workspace_bytes, void* stream);

/*
 * Row-sharded train step (owner-computes): supervisor.py:15-26 (`train_step_fn`) over the
 * batches of W replicas (tf.distribute: each replica's loss on its own batch, gradients SUM-aggregated
 * by `apply_gradients`, metric += loss * num_replicas_in_sync), with the ENTITY TABLE ROW-SHARDED over
 * the W ranks instead of replicated. Rank r holds rows [shard_lo, shard_lo + shard_rows) (ent_ld
 * stride; updated in place, with its Adam moments m_ent / v_ent), the replicated relation table (every
 * rank applies the identical relation update), and the GLOBAL batch of Bg = W * home_B rows (pos [Bg,3],
 * neg [Bg,N], weight [Bg]; home rank h's replica batch is rows [h home_B, (h+1) home_B)), identical on
 * every rank. Candidate rows never leave their owner. Three calls, with the caller's collectives between:
 *   kge_shard_train_forward   owned candidates: scores, per-row partial softmax state -> stats [Bg*4];
 *                             owned positives' query gradients -> dq rows [Bg, 2Bg)
 *   (caller) all-gather stats -> stats_all [W*Bg*4] (rank-major)
 *   kge_shard_train_combine   merged row state; this rank's share of each negative slot's query
 *                             gradient -> dq rows [0, Bg); out_neg [Bg] (reduced negative branch),
 *                             out_pos_raw / out_pos [Bg] (positive score, logsigmoid)
 *   (caller) SUM all-reduce of dq [2*Bg*nq*D floats], nq = kge_shard_nq(fn)
 *   kge_shard_train_backward  owned score gradients, every slot's query chain, deterministic phase 2
 *                             with Adam on the shard, relation gradient with Adam; loss [W] (each
 *                             replica's loss), *loss_sum += W * sum(loss) (may be NULL)
 * qent [Bg, q_ld]: row b = entity row pos[b, mode == head ? 2 : 0]; qent_pos [Bg, q_ld]: row b = entity
 * row pos[b, 0] (the same buffer in tail-batch mode) — e.g. kge_gather_rows on every shard + SUM all-reduce.
 * The same argument prefix goes to all three calls; workspace (kge_shard_train_workspace_size bytes)
 * carries the step from forward to backward (no state between steps). Deterministic for a fixed W.
 * Out-of-range ids have no owner: they are dropped (the unsharded path scores them on a zero row).
 * D <= 1024 (per half), no pRotatE (KGE_ENOTSUP).
 */
int kge_shard_nq(int fn);
int64_t kge_shard_train_workspace_size(int fn, int64_t shard_rows, int64_t nrelation, int64_t rel_ld, int64_t Bg,
                                       int64_t N, int64_t D);
int kge_shard_train_forward(int fn, int mode, const float* shard, int64_t shard_rows, int64_t ent_ld, int64_t shard_lo,
                            const float* qent, const float* qent_pos, int64_t q_ld, const float* rel, int64_t nrelation,
                            int64_t rel_ld, int64_t rel_off, const int64_t* pos, const int64_t* neg, int64_t neg_ld,
                            int64_t Bg, int64_t N, int64_t D, int64_t home_B, int world, int rank, float gamma,
                            float emb_range, float temperature, int adversarial, int detach, const float* weight,
                            float* stats, float* dq, void* workspace, int64_t workspace_bytes, void* stream);
int kge_shard_train_combine(int fn, int mode, const float* shard, int64_t shard_rows, int64_t ent_ld, int64_t shard_lo,
                            const float* qent, const float* qent_pos, int64_t q_ld, const float* rel, int64_t nrelation,
                            int64_t rel_ld, int64_t rel_off, const int64_t* pos, const int64_t* neg, int64_t neg_ld,
                            int64_t Bg, int64_t N, int64_t D, int64_t home_B, int world, int rank, float gamma,
                            float emb_range, float temperature, int adversarial, int detach, const float* weight,
                            const float* stats_all, float* dq, float* out_neg, float* out_pos_raw, float* out_pos,
                            void* workspace, int64_t workspace_bytes, void* stream);
int kge_shard_train_backward(int fn, int mode, float* shard, int64_t shard_rows, int64_t ent_ld, int64_t shard_lo,
                             const float* qent, const float* qent_pos, int64_t q_ld, float* rel, int64_t nrelation,
                             int64_t rel_ld, int64_t rel_off, const int64_t* pos, const int64_t* neg, int64_t neg_ld,
                             int64_t Bg, int64_t N, int64_t D, int64_t home_B, int world, int rank, float gamma,
                             float emb_range, float temperature, int adversarial, int detach, const float* weight,
                             const float* dq, float* loss, float* loss_sum, float* m_ent, float* v_ent, float* m_rel,
                             float* v_rel, float lr, float beta1, float beta2, float eps, int64_t step, int keras,
                             void* workspace, int64_t workspace_bytes, void* stream);

/*
 * TranSparse scores (tensorflow_codes/model.py:226-235, gathers at :139-142, :161-164, :187-190; tables
 * :96-106) on the fp32 matrix cores. W and mask are [nrel, d, d] row-major contiguous; the score reads the
 * whole relation row (d floats, rel_ld stride) and needs entity_dim == relation_dim == d.
 *   mode KGE_HEAD_BATCH: out[b*out_ld + n] for n < N, head = E[neg[b*neg_ld + n]], relation pos[b,1]
 *   mode KGE_SINGLE / KGE_TAIL_BATCH: out[b*out_ld] only (the reference's [B, 1]: Q9 makes the score
 *        depend on the head alone, so tail-batch ignores the negatives); neg may be NULL.
 * Out-of-range ids read zero rows (scores NaN from the zero-norm normalisation, as on TF-GPU).
 * stats (may be NULL): per row float2 (||p||^2, sum_j |p_j c_j|) for the backward.
 * mask may be NULL: W then already holds mask * W (kge_transparse_premul), which halves the matrix reads.
 * d <= 8192. Deterministic (no atomics).
 */
int kge_transparse_score(int mode, const float* ent, int64_t nent, int64_t ent_ld, const float* rel, int64_t nrel,
                         int64_t rel_ld, const float* W, const float* mask, const int64_t* pos, const int64_t* neg,
                         int64_t neg_ld, int64_t B, int64_t N, int64_t d, float gamma, float* out, int64_t out_ld,
                         float* stats, void* stream);
/*
 * Backward of kge_transparse_score's raw scores (autograd of model.py:226-235 through the gathers).
 *   stats     [B*N] (head-batch) or [B] (single/tail) float2 written by the forward (stats != NULL)
 *   d_scores  dL/dscore, row b at d_scores + b*d_ld (column 0 only for single/tail)
 *   M         mask * W from kge_transparse_premul, or NULL (the product is then formed on the fly)
 *   d_ent [nent, ent_ld], d_rel [nrel, rel_ld], d_W [nrel, d, d]: gradients are ADDED (+=)
 * Bitwise deterministic (no float atomics). Workspace: kge_transparse_bwd_workspace_size bytes.
 */
/* M[i] = mask[i] * W[i] for n floats (n % 4 == 0, 16-byte aligned): the premultiplied relation matrices. */
int kge_transparse_premul(const float* W, const float* mask, int64_t n, float* M, void* stream);
size_t kge_transparse_bwd_workspace_size(int mode, int64_t nent, int64_t nrel, int64_t B, int64_t N, int64_t d);
int kge_transparse_score_bwd(int mode, const float* ent, int64_t nent, int64_t ent_ld, const float* rel, int64_t nrel,
                             int64_t rel_ld, const float* W, const float* mask, const float* M, const int64_t* pos,
                             const int64_t* neg,
                             int64_t neg_ld, int64_t B, int64_t N, int64_t d, const float* stats, const float* d_scores,
                             int64_t d_ld, float* d_ent, float* d_rel, float* d_W, void* workspace,
                             size_t workspace_bytes, void* stream);

/*
 * Negative sampler of the training batches (host memory, no GPU): the upstream KnowledgeGraphEmbedding
 * TrainDataset (call sites compress_data/main.py:64-73), bit-exact with its numpy code for the same RNG
 * state: negatives from numpy's legacy MT19937 `randint` (seeded like np.random.seed(seed)), filtered by
 * `np.in1d(..., assume_unique=True, invert=True)` exactly as numpy 2.2.6 evaluates it, weights
 * sqrt(1 / (count(h,r) + count(t,-r-1))) with count start 4.
 *   triples [T,3] int64 (h, r, t) training triples; mode KGE_HEAD_BATCH or KGE_TAIL_BATCH
 *   kge_sampler_get: for each idx[b] in order: pos[b] = triples[idx[b]], neg[b] [N], weight[b]
 */
typedef struct kge_sampler kge_sampler;
kge_sampler* kge_sampler_create(const int64_t* triples, int64_t ntriples, int64_t nentity, int64_t nrelation,
                                int64_t negative_sample_size, int mode);
int kge_sampler_seed(kge_sampler* sampler, uint32_t seed);
int kge_sampler_get(kge_sampler* sampler, const int64_t* idx, int64_t B, int64_t* pos, int64_t* neg,
                    float* weight);
void kge_sampler_destroy(kge_sampler* sampler);

/*
 * TFRecord IO of the reference's on-disk training batches (host memory, no GPU). One
 * tf.train.Example per batch with Int64List "positive_sample" [B*3], "negative_sample" [B*N],
 * FloatList "subsampling_weight" [B], Int64List "mode" [B]:
 *   writer = compress_data/main.py:117-131 + compress_data/utils.py:35-42 (create_example);
 *   reader = tensorflow_codes/run.py:40-51 (parse_tfrecord_fn, VarLenFeature + to_dense) over
 *            tf.data.TFRecordDataset(paths) (run.py:87), files read in order.
 * Framing and CRC-32C (masked) as TFRecord; CRCs are verified when verify_crc != 0.
 * kge_tfrecord_next: 1 = a record was parsed and counts[4] = {npos, nneg, nw, nmode}; 0 = end of the
 * last file; < 0 = error (truncated, CRC mismatch, malformed proto, wrong list type).
 */
typedef struct kge_tfrecord_reader kge_tfrecord_reader;
typedef struct kge_tfrecord_writer kge_tfrecord_writer;
uint32_t kge_crc32c(const void* data, int64_t n);
kge_tfrecord_reader* kge_tfrecord_open(const char* const* paths, int64_t npaths, int verify_crc);
int kge_tfrecord_next(kge_tfrecord_reader* reader, int64_t* counts);
int kge_tfrecord_copy(kge_tfrecord_reader* reader, int64_t* positive_sample, int64_t* negative_sample,
                      float* subsampling_weight, int64_t* mode);
int kge_tfrecord_rewind(kge_tfrecord_reader* reader);
void kge_tfrecord_close(kge_tfrecord_reader* reader);
kge_tfrecord_writer* kge_tfrecord_writer_open(const char* path);
int kge_tfrecord_write_example(kge_tfrecord_writer* writer, const int64_t* positive_sample, int64_t npos,
                               const int64_t* negative_sample, int64_t nneg, const float* subsampling_weight,
                               int64_t nw, const int64_t* mode, int64_t nmode);
int kge_tfrecord_writer_close(kge_tfrecord_writer* writer);

/*
 * Dense Adam step over n floats (supervisor.py:26 `optimizer.apply_gradients`, run.py:111 Keras Adam).
 *   keras != 0: Keras Adam  (m += (g-m)(1-b1); v += (g^2-v)(1-b2);
 *                            p -= m*alpha/(sqrt(v)+eps), alpha = lr*sqrt(1-b2^t)/(1-b1^t))
 *   keras == 0: torch.optim.Adam (p -= lr/(1-b1^t) * m / (sqrt(v)/sqrt(1-b2^t) + eps))
 *   step is the 1-based step t; zero_grad != 0 also zeroes grad in the same pass.
 * n floats each, 4-byte aligned; 16-byte aligned buffers take the float4 nontemporal path, others a
 * dword path with bitwise the same per-element result.
 */
int kge_adam_update(float* param, float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                    float lr, float beta1, float beta2, float eps, int64_t step,
                    int keras, int zero_grad, void* stream);

/*
 * Backward of kge_score_indexed (GradientTape through the gathers, supervisor.py:25).
 * Accumulates (+=) into d_ent [nentity, ent_ld] and d_rel [nrelation, rel_ld] (same strides as
 * the tables). The query-side rows get one deterministic per-row sum over the N candidates; the
 * candidate rows are scattered with fp32 atomics (order of accumulation between candidates that hit
 * the same entity is not fixed: results are reproducible to fp32 rounding, not bitwise).
 * workspace: device scratch of kge_score_bwd_workspace_size(...) bytes (caller-owned).
 */
int64_t kge_score_bwd_workspace_size(int fn, int mode, int64_t B, int64_t N, int64_t D);
int kge_score_indexed_bwd(int fn, int mode,
                          const float* ent, int64_t nentity, int64_t ent_ld,
                          const float* rel, int64_t nrelation, int64_t rel_ld, int64_t rel_off,
                          const int64_t* pos, const int64_t* neg, int64_t neg_ld,
                          int64_t B, int64_t N, int64_t D,
                          float gamma, float emb_range, float modulus,
                          const float* d_scores, int64_t d_ld,
                          float* d_ent, float* d_rel, float* d_modulus,
                          void* workspace, void* stream);

/*
 * Backward of kge_score_dense (gradient of the model_func plugin w.r.t. its gathered inputs).
 * Accumulates (+=) into d_head / d_rel / d_tail, laid out like head / rel / tail.
 */
int kge_score_dense_bwd(int fn, int mode,
                        const float* head, int64_t head_ld,
                        const float* rel, int64_t rel_ld, int64_t rel_off,
                        const float* tail, int64_t tail_ld,
                        int64_t B, int64_t N, int64_t D,
                        float gamma, float emb_range, float modulus,
                        const float* d_scores, int64_t d_ld,
                        float* d_head, float* d_rel, float* d_tail, float* d_modulus, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* KGE_HIP_H */
