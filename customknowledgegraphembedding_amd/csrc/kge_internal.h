// kge_internal.h — host/device shared definitions of libkge_hip.so (not part of the C-ABI).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kge_hip.h"

namespace kge_impl {

constexpr int kWave = 64;
constexpr int kBlock = 256;
constexpr int kWavesPerBlock = kBlock / kWave;
constexpr int kMaxG = 8;  // float4 groups per lane per half-row kept in VGPRs (D <= 2048)
constexpr int kBwdMaxG = 16;  // dword groups per lane of the backward's atomic-friendly layout (D <= 1024)

enum Kind {
    KIND_FWD = 0,
    KIND_BWD = 1,
    KIND_FINISH = 2,
    KIND_BWD_ROWS = 3,
    KIND_BWD_ENT = 4,
    KIND_BWD_STREAM = 5,  // phase 1, column-group streaming (one wave per column group, dq -> dqbuf)
    KIND_BWD_CHAIN = 6,   // phase 1 epilogue of the streaming form (one wave per slot)
    KIND_FWD_STATS = 7,   // forward that also keeps InterHT's candidate norms (train step)
    KIND_STEP_FWD = 8,    // fused train-step forward: block per batch row, negatives + finish in one launch
    KIND_STEP_FWD_STATS = 9,
    KIND_BWD_ENT_STREAM = 10,  // phase 2, column-group streaming (one block per entity row)
    KIND_STEP_FWD_GRAD = 11,   // train-step forward with phase 1 fused (kge_train_step)
    KIND_STEP_EPILOGUE = 12,   // kge_train_step: loss weights, score gradients, chains, loss (one wave per slot)
    KIND_SHARD_FWD_GRAD = 13,  // row-sharded train step: owned candidates' scores + partial softmax state
    KIND_SHARD_POS = 14,       // row-sharded train step: owned positives (score, gradient, query gradient)
    KIND_SHARD_EPILOGUE = 15,  // row-sharded train step: owned score gradients, every slot's chain, loss
    KIND_STEP_FWD_XCD = 16,    // kge_step_forward's negatives, XCD-sliced entity table, ascending ids per wave
    KIND_SCORE_SHARD_XCD = 17, // kge_score_indexed / kge_score_sharded in the same order (no positives)
    KIND_SHARD_BUCKET = 18,    // row-sharded forward: this rank's bucket (kge_shard_plan) scored, compact out
    KIND_STEP_FWD_TILE = 19,   // kge_step_forward's negatives + positives: row-group x XCD-slice tiles, one
                               // entity-sorted sweep per block (queries in LDS)
    KIND_SCORE_TILE = 20,      // kge_score_indexed in the same order (no positives)
};
constexpr int kTileBuckets = 256;  // entity buckets of a slice (the block's counting sort)
constexpr int kTileMaxRows = 16;
constexpr int kTileLdsMax = 160 * 1024;
constexpr int kTileSortRel = 64;     // relation buckets of the tile kernel's row sort (ids >= 62 share one)
constexpr int kTileSortMaxB = 2048;  // batch rows the tile kernel sorts by relation in LDS
// LDS query operands per batch row of the tile kernel (InterHT's third, the relation, is read per candidate)
constexpr int tile_nq(int fn) { return (fn == KGE_COMPLEX || fn == KGE_ROTATE || fn == KGE_INTERHT) ? 2 : 1; }
// query operands a score function's gradient has (q0 always; q1 for the complex / split forms; q2 InterHT)
constexpr int shard_nq(int fn) {
    return fn == KGE_INTERHT ? 3 : ((fn == KGE_COMPLEX || fn == KGE_ROTATE) ? 2 : 1);
}
constexpr int kFwdGradMaxG = 4;  // the fused forward + query gradient keeps 6 accumulators per element

// ---------------------------------------------------------------------------------------------
// The tile scorer's step plan (kge_step_plan / kge_step_forward_planned): everything step_fwd_tile_kernel
// derives from a batch's ids alone, made ahead of the step. int32 words:
//   [0, kPlanHdr)                 header: magic, B, N, mode, rows per group R, nentity, the relation sort flag
//   meta  [groups][R][4]          per row of a group in the block's row order: batch row b (-1 past the batch),
//                                 then its positive (h, r, t) with out-of-range ids as -1
//   soff  [groups][9]             per group, the start of each entity slice's items in its list, then the total
//   list  [groups][R (N + 1)][2]  per group, its items sorted by (slice, entity bucket): (candidate entity id
//                                 or -1 when out of range, row << 16 | column) — column N: the row's positive
// The plan is a snapshot of the batch's ids: the planned step reads no id but the plan's.
// ---------------------------------------------------------------------------------------------
constexpr int kPlanMagic = 0x4B475031;  // "KGP1"
constexpr int kPlanHdr = 16;
__host__ __device__ inline int64_t plan_groups(int64_t B, int R) { return (B + R - 1) / R; }
__host__ __device__ inline int64_t plan_soff(int64_t B, int R) { return kPlanHdr + plan_groups(B, R) * R * 4; }
__host__ __device__ inline int64_t plan_list(int64_t B, int R) { return (plan_soff(B, R) + plan_groups(B, R) * 9 + 3) & ~(int64_t)3; }
__host__ __device__ inline int64_t plan_words(int64_t B, int64_t N, int R) {
    return plan_list(B, R) + plan_groups(B, R) * R * (N + 1) * 2;
}
// one plan to make: the next batch's ids (same B, N) and where its plan goes
struct PlanArgs {
    const int64_t* pos;
    const int64_t* neg;
    int64_t neg_ld;
    int64_t B, N, nent, nrel;
    int mode;  // KGE_HEAD_BATCH / KGE_TAIL_BATCH
    int R;     // batch rows per group
    int sort;  // rows ranked by relation (InterHT, B <= kTileSortMaxB)
    int* plan;
};
// LDS ints of one plan block of NT threads: row list, (slice, bucket) counts, the relation sort's wave counts
__host__ __device__ constexpr int plan_lds_ints(int NT) {
    return kTileMaxRows + 8 * kTileBuckets + (kTileSortMaxB + NT - 1) / NT * (NT / 64) * kTileSortRel;
}

// Parameters of one scoring launch. Rows are addressed as base + row * ld (floats).
//   query entity row of batch row b:  q_idx ? q_idx[b * q_stride] : b
//   relation row of batch row b:      r_idx ? r_idx[b * r_stride] : b      (+ r_off floats)
//   candidate n of batch row b:       c_idx ? c_idx[b * c_stride + n] : b * c_dense + n
struct ScoreParams {
    const float* qent;
    const int64_t* q_idx;
    int64_t q_ld, q_stride, q_rows;
    const float* rel;
    const int64_t* r_idx;
    int64_t r_ld, r_stride, r_rows, r_off;
    const float* cent;
    const int64_t* c_idx;
    int64_t c_ld, c_stride, c_rows, c_dense;
    int64_t c_base;    // candidate ids are global: row = id - c_base (row-sharded tables)
    int skip_foreign;  // sharded scoring: a candidate outside [c_base, c_base + c_rows) scores 0, no work
    // compact output of the row-sharded score exchange (kge_shard_score): only this rank's owned scores are
    // written, row b's at out[cmp_off(b) + k], k = the candidate's rank among the row's owned ones in column
    // order (the positive last). cmp_off(b) = cmp_pre[b] + the owned counts of the launch's earlier homes:
    // the send block of an all-to-all, home-major.
    const int* cmp_pre;   // [B] home-local exclusive prefix of this rank's owned counts
    const int* cmp_cnt;   // [B] this rank's owned candidates of each row (negatives + the positive)
    const int* cmp_tot;   // [W * W] tot[h * W + o]: candidates of home h's rows owned by rank o
    int64_t cmp_home0;    // home of the launch's row 0 (its rows are whole homes of home_B rows)
    const int2* bk_ent;   // [B, bk_ld] kge_shard_plan's bucket: (local row, rank k) per owned candidate
    const int* bk_start;  // [B, 9] the bucket's XCD-slice starts per row
    int64_t bk_ld;
    int xcd_phases;       // step_fwd_xcd_kernel: the table's 8 slices cut again into this many phases (1: none)
    int tile_rows;        // step_fwd_tile_kernel: batch rows per block (their queries staged in LDS)
    int tile_lds;         // step_fwd_tile_kernel: dynamic LDS bytes of one block
    int tile_pos;         // step_fwd_tile_kernel: also score the rows' positives (kge_step_forward)
    int tile_q2slots;     // step_fwd_tile_kernel (InterHT): LDS slots of relation thirds
    int tile_sort;        // step_fwd_tile_kernel: 0, or the power of two >= B of the (relation, row) sort
    int tile_waves;       // step_fwd_tile_kernel: waves per block (8 or 16)
    int tile_dry;         // step_fwd_tile_kernel: setup only, no scoring (A/B knob KGE_TILE_DRY)
    int tile_rev;         // step_fwd_tile_kernel: sweep each block's sorted list in descending entity order
    const int* tile_plan; // step_fwd_tile_kernel: this batch's plan (kge_step_forward_planned), or null
    int tile_blocks;      // step_fwd_tile_kernel: scoring blocks; blocks past them make the next batch's plan
    PlanArgs tile_next;   // ... that plan (tile_next.plan null: none)
    float* out;
    int64_t out_ld;
    int64_t B, N;
    int D;    // per-half width
    int cpw;  // candidates per wave
    int wpr;  // waves per batch row = ceil(N / cpw)
    float gamma;
    float phase_div;  // emb_range / pi (RotatE) or emb_range / pi' (pRotatE), fp32 as torch does
    float modulus;    // pRotatE
    // backward only
    const float* d_scores;
    int64_t d_ld;
    float* d_qent;  // gradient table for query entity rows (== d_cent for indexed scoring)
    float* d_rel;
    float* d_cent;
    float* d_modulus;
    // finish kernel only (one wave per batch row: positive score + negative-row reduction)
    const float* neg_scores;
    int64_t ns_ld, n_neg;
    float temperature;
    int adversarial;
    int detach;                // self-adversarial weights detached (upstream) or not (TF, Q3)
    const float* dq_scale;     // [B] chain kernel: scale of the fused forward's query gradient
    // kge_train_step epilogue
    const float* weight;       // [B] subsampling weights
    const float* pos_raw;      // [B] raw positive scores
    float* loss;               // [1]
    float* loss_sum;           // [1] running Sum metric (may be null)
    int* ev_count;             // fused forward: per-entity event counts (atomics)
    int* ev_cursor;            // epilogue: bucket cursors (scatter)
    int* ev_code_w;            // epilogue: event codes grouped by entity
    const int* ev_tile_sum;    // epilogue: per-4096-entity tile totals of the counts (tile-local cursors), or null
    int* ev_off_fix;           // epilogue: the tile-local offsets it rewrites to global ones (phase 2 reads them)
    int ev_ntiles;
    float* out_neg;      // [B] reduced negative branch
    float* out_pos_raw;  // [B] raw positive score (may be null)
    float* out_pos_ls;   // [B] logsigmoid(positive score)
    // deterministic two-phase backward (kge_step_backward). A "slot" is one query side: slots
    // [0, Bn) are the negative call's batch rows, [Bn, 2 Bn) the positive (single) call's.
    float* qbuf;          // [slots, 3 D] query operands q0 | q1 | q2 (phase 1 writes, phase 2 reads)
    float* qg_ent;        // [slots, ent_w] gradient of each slot's raw query-entity row
    float* qg_rel;        // [slots, rel_w] gradient of each slot's used relation part
    float* dmod_part;     // [slots] pRotatE modulus gradient partials
    int64_t slot0;        // first slot of a phase-1 launch
    float2* cand_stats;   // [B * N] per-candidate (1/||a||, 1/||b||) of InterHT, written by the forward
    const int64_t* pos_base;  // [B, 3] positive triples (fused step forward)
    float* dqbuf;         // [B, 3 * D] phase-1 query-part gradients (streaming form)
    int64_t ent_w, rel_w; // floats per entity row / per used relation part
    const int* ev_off;    // [E + 1] bucket offsets of the per-entity gradient events (phase 2)
    const int* ev_code;   // event codes, grouped by entity (order inside a bucket: arbitrary)
    const float* d_ns;    // [Bn, N] dL/d(negative score), contiguous
    const float* d_ps;    // [Bn] dL/d(positive score)
    int64_t Bn, Nn;       // negative batch rows and candidates per row
    float* d_out_ent;     // [E, c_ld] entity gradient table, fully overwritten by phase 2
    // row-sharded train step (kge_shard_train_*; kge_shard.h). Batch rows are GLOBAL: [0, B) over all
    // W home ranks, home h owning rows [h * home_B, (h + 1) * home_B).
    const float* qent_pos;      // [B, q_ld] the positive call's query rows (h), assembled by the caller
    float* sh_stats;            // [B, 4] this shard's partial (M, Z, Ln, positive score)
    const float* sh_stats_all;  // [world, B, 4] every shard's partial stats (all-gathered)
    float* sh_dq;               // [2 B, nq D] this shard's share of each slot's query gradient (SUM-reduced)
    float* sh_A;                // [B, nq D] online-softmax query-gradient sums of the owned candidates
    float* sh_B;                // [B, nq D] (TF semantics only: the softmax term)
    float* sh_merged;           // [B, 4] merged (M, Z, R, positive score): identical on every shard
    int64_t home_B;
    int world, rank, nq;
    // fused optimizer in phase 2 (kge_step_backward_adam): row e of the table is updated in place
    struct {
        float* m;   // [E, c_ld] first moment
        float* v;   // [E, c_ld] second moment
        float b1, b2, eps, alpha, step_size, bc2_sqrt;
        int keras, on;
    } adam;
};

// Adam coefficients of step t (1-based), computed on the host in double
struct AdamArgs {
    float b1, b2, eps, alpha, step_size, bc2_sqrt;
    int keras, zero_grad;
};

// per-score-function launchers (one translation unit each, see kge_fn_*.hip)
int launch_transe(const ScoreParams& p, int kind, hipStream_t st, int blocks, bool ch, int V, int G);
int launch_distmult(const ScoreParams& p, int kind, hipStream_t st, int blocks, bool ch, int V, int G);
int launch_complex(const ScoreParams& p, int kind, hipStream_t st, int blocks, bool ch, int V, int G);
int launch_rotate(const ScoreParams& p, int kind, hipStream_t st, int blocks, bool ch, int V, int G);
int launch_interht(const ScoreParams& p, int kind, hipStream_t st, int blocks, bool ch, int V, int G);
int launch_protate(const ScoreParams& p, int kind, hipStream_t st, int blocks, bool ch, int V, int G);

// link-prediction evaluation (kge_eval.hip)
int launch_eval_query_any(int fn, bool ch, const ScoreParams& p, hipStream_t st, int blocks, int V, int G, float* Q,
                          int64_t ldq, void* P = nullptr, int64_t prows = 0);
int launch_gemm_nt(const float* A, const float* B, float* C, int M, int N, int K, int64_t lda, int64_t ldb,
                   int64_t ldc, hipStream_t st);
int launch_gemm_nt_f32x3(const float* A, const float* B, float* C, int M, int N, int K, int64_t lda, int64_t ldb,
                         int64_t ldc, hipStream_t st, int form = 0);
int launch_split3_planes(const float* X, int64_t rows, int64_t cols, int64_t ld, void* planes, int64_t plane_rows,
                         hipStream_t st);
// form 1: both operands staged through LDS per 16-k chunk (gemm_nt_x3p_kernel, 256 x 256 tiles); 2: B straight into
// registers, A staged per 32 k (gemm_nt_x3d_kernel); 3: gemm_nt_x3p_kernel with 256 x 192 tiles; 4: LDS-DMA staging
// in three stages (gemm_nt_x3l_kernel). Bitwise the same C.
int launch_gemm_nt_x3p(const void* Ap, int64_t a_rows, const void* Bp, int64_t b_rows, int64_t K, float* C, int64_t ldc,
                       int M, int N, hipStream_t st, int form);
// kge_eval_rank_planes: workspace bytes (truth scores and counts [M], filter-entry scores [F]) and the launches of
// the phases in `phases` (1 pair scores + count reset, 2 counting GEMM, 4 finish), in that order
int64_t eval_rank_ws_bytes(int64_t M, int64_t F);
int launch_eval_rank_planes(const void* Ap, int64_t a_rows, const void* Bp, int64_t b_rows, int64_t K, int M, int N,
                            const int64_t* truth, const int64_t* fptr, const int64_t* fids, int64_t F, int64_t* ranks,
                            void* ws, hipStream_t st, int form, int phases);
int launch_rank(const float* S, int64_t M, int64_t N, int64_t ld, const int64_t* truth, const int64_t* fptr,
                const int64_t* fids, int64_t* ranks, hipStream_t st);

}  // namespace kge_impl
