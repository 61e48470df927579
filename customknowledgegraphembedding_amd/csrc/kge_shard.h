// kge_shard.h — device kernels of the ROW-SHARDED train step (owner-computes).
// Included by kge_device.h ahead of its dispatch section; builds on its templates (Query, Cand,
// cand_score, group_jac, cand_grad, rows_finalize, for_owned_runs).
//
// W ranks each hold the entity rows [c_base, c_base + c_rows) of one table, the replicated relation
// table, the same global batch (B = W * home_B rows; home rank h's replica batch is rows
// [h home_B, (h + 1) home_B)) and the query-entity rows of every batch row (assembled by the caller:
// owners gather, SUM all-reduce). One step is supervisor.py:15-26 over the W replicas' batches with
// tf.distribute's SUM gradient aggregation (`apply_gradients`), in three library calls with two
// collectives between them:
//   forward  (owned candidates only) per-row partial online-softmax state (M_r, Z_r, Ln_r) and the
//            query-gradient sums A_r = sum e_n (-sigmoid(s_n) + T f_n) J_n, B_r = sum e_n J_n
//            (step_fwd_grad_kernel's algebra); owned positives: score, its gradient, its query
//            gradient                                                   -> stats [B, 4], dq[B + b]
//   [all-gather of the [B, 4] stats]
//   combine  merged (M, Z, R = Ln / Z) per row, the same on every rank (fixed order over ranks);
//            this rank's share go f_r (A_r - T R B_r) / Z of each row's query gradient  -> dq[b]
//   [SUM all-reduce of dq [2 B, nq D]]
//   backward owned candidates' score gradients from the merged state, every slot's query chain
//            (identical on all ranks), owned-row events, then phase 2 with Adam on the shard and the
//            relation gradient with Adam (identical on all ranks: the replicas stay equal)
// Candidate rows are gathered once per step (as kge_train_step); nothing shard-sized crosses ranks.
#pragma once

namespace kge_impl {

// merged per-row state from every rank's partial (M_r, Z_r, Ln_r, pos_r), in rank order
struct RowMerge {
    float M, Z, Ln, pos, f_me;
};

__device__ __forceinline__ RowMerge merge_row(const ScoreParams& p, int64_t b) {
    RowMerge r;
    r.M = -INFINITY;
    for (int w = 0; w < p.world; ++w) r.M = fmaxf(r.M, p.sh_stats_all[((int64_t)w * p.B + b) * 4 + 0]);
    r.Z = 0.f;
    r.Ln = 0.f;
    r.pos = 0.f;
    r.f_me = 0.f;
    for (int w = 0; w < p.world; ++w) {
        const float* s = p.sh_stats_all + ((int64_t)w * p.B + b) * 4;
        const float f = (s[0] == -INFINITY) ? 0.f : expf(s[0] - r.M);  // a rank with no owned candidate: 0
        r.Z += s[1] * f;
        r.Ln += s[2] * f;
        r.pos += s[3];
        if (w == p.rank) r.f_me = f;
    }
    return r;
}

// dL/d(out_neg_b) = dL/d(out_pos_b) = -w_b / (2 sum_{home of b} w)   (supervisor.py:19-23, per replica)
__device__ __forceinline__ float home_loss_weight(const ScoreParams& p, int64_t b, int lane) {
    const int64_t h0 = (b / p.home_B) * p.home_B;
    float sw = 0.f;
    for (int64_t i = lane; i < p.home_B; i += kWave) sw += p.weight[h0 + i];
    sw = wave_sum(sw);
    return (-0.5f / sw) * p.weight[b];
}

// ---------------------------------------------------------------------------------------------
// Forward (KIND_SHARD_FWD_GRAD): one block per global batch row b; the four waves split the row's
// candidates and each compacts the ones this shard owns (for_owned_runs). Per owned candidate: the
// score (kept for the backward's score gradients), the gradient event (counted into the local
// row's bucket) and the online-softmax running sums. The waves' partial states are merged to the
// block's maximum and added in wave order through one LDS image (deterministic).
//   RED: 0 mean, 1 self-adversarial with the softmax detached, 2 self-adversarial (TF semantics).
// ---------------------------------------------------------------------------------------------
template <int FN, bool CH, int V, int G, int RED>
__global__ __launch_bounds__(kBlock) void shard_fwd_grad_kernel(ScoreParams p) {
    static_assert(FN != KGE_PROTATE, "pRotatE's modulus gradient is not part of the fused query pass");
    constexpr bool TWO = RED == 2;
    constexpr int W = G * kWave;  // vecf<V> per operand per wave image
    constexpr int NQ = shard_nq(FN);
    __shared__ vecf<V> qimg[3][W];                // the row's query operands, shared by the four waves
    __shared__ vecf<V> acc[(TWO ? 2 : 1) * NQ][W];  // the block's A (and B), added in wave order
    __shared__ float st[kWavesPerBlock][3];
    const int64_t b = blockIdx.x;
    if (b >= p.B) return;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int DV = p.D / V;
    const float T = p.temperature;
    if (w == 1 && lane < 3 && p.ev_count) {
        // the row's other events, owned ones only: positive tail, negative call's query entity, positive head
        const int64_t k = p.pos_base[b * 3 + (lane == 0 ? 2 : (lane == 1 ? (CH ? 2 : 0) : 0))] - p.c_base;
        if (k >= 0 && k < p.c_rows) atomicAdd(p.ev_count + k, 1);
    }
    if (w == 0) {
        Query<FN, CH, V, G> qr;
        int64_t qi, ri;
        bool qok, rok;
        build_query_for<FN, CH, V, G>(p, b, lane, qr, qi, ri, qok, rok);
#pragma unroll
        for (int k = 0; k < G; ++k) {
            qimg[0][lane + k * kWave] = qr.q0[k];
            qimg[1][lane + k * kWave] = qr.q1[k];
            qimg[2][lane + k * kWave] = qr.q2[k];
        }
    }
    __syncthreads();
    vecf<V> a0[G], a1[G], a2[G], b0[G], b1[G], b2[G];
#pragma unroll
    for (int k = 0; k < G; ++k) a0[k] = a1[k] = a2[k] = b0[k] = b1[k] = b2[k] = vzero<V>();
    float mrun = -INFINITY, Z = 0.f, Ln = 0.f;
    {
        auto accumulate = [&](const Cand<FN, V, G>& c, const LdsQuery<V>& q, float s, float2 nst) {
            // the hardware exp / log / rcp, as the single-GPU fused forward (per candidate these were most of
            // a DistMult wave's VALU work); the merged stats stay within fp32 rounding of the libm ones
            auto expf = [](float x) { return fexp(x); };
            auto sigmoidf = [](float x) { return fsigmoid(x); };
            auto log_sigmoid = [](float x) { return flog_sigmoid(x); };
            float wa, wb = 0.f;
            if constexpr (RED == 0) {
                wa = -sigmoidf(s);
                Z += 1.f;
                Ln += log_sigmoid(-s);
            } else {
                const float t = T * s;
                if (t > mrun) {  // online softmax: rescale the running sums to the new maximum
                    const float sc = expf(mrun - t);
                    Z *= sc;
                    Ln *= sc;
#pragma unroll
                    for (int k = 0; k < G; ++k)
#pragma unroll
                        for (int i = 0; i < V; ++i) {
                            a0[k].a[i] *= sc;
                            a1[k].a[i] *= sc;
                            a2[k].a[i] *= sc;
                            if constexpr (TWO) {
                                b0[k].a[i] *= sc;
                                b1[k].a[i] *= sc;
                                b2[k].a[i] *= sc;
                            }
                        }
                    mrun = t;
                }
                const float e = expf(t - mrun);
                const float f = log_sigmoid(-s);
                Z += e;
                Ln += e * f;
                wa = e * -sigmoidf(s);
                if constexpr (TWO) {
                    wa += e * (T * f);
                    wb = e;
                }
            }
#pragma unroll
            for (int k = 0; k < G; ++k)
                group_jac<FN, CH, V, TWO>(c.ca[k], c.cb[k], q.q0[k], q.q1[k], q.q2[k], (lane + k * kWave) < DV, nst.x,
                                          nst.y, p, wa, wb, a0[k], a1[k], a2[k], b0[k], b1[k], b2[k]);
        };
        const int64_t per = (p.N + kWavesPerBlock - 1) / kWavesPerBlock;
        const int64_t lo = w * per, hi = min(p.N, lo + per);
        for_owned_runs(p, b, lo, hi, lane, false, [&](int row, int n, int nc) {
            const int64_t my_id = (int64_t)row + p.c_base;
            // the candidate's gradient event, counted into its local row's bucket (phase 2)
            if (p.ev_count && lane < nc) atomicAdd(p.ev_count + row, 1);
            float my_score = 0.f;
            Cand<FN, V, G> x0, x1;
            bool ok0, ok1;
            auto one = [&](const Cand<FN, V, G>& c, int jj) {
                int li = lane;
                asm volatile("" : "+v"(li));  // keep the LDS query reads inside the loop (VGPRs)
                const LdsQuery<V> q{{qimg[0], li}, {qimg[1], li}, {qimg[2], li}};
                float2 nst = make_float2(0.f, 0.f);
                const float s = cand_score<FN, CH, V, G>(c, q, p, &nst);
                if (lane == jj) my_score = s;
                asm volatile("" : "+v"(nst.x), "+v"(nst.y));
                accumulate(c, q, s, nst);
            };
            x0.load(cand_row(p, readlane64(my_id, 0), ok0), ok0, p.D, lane);
            int j = 0;
            for (; j + 2 < nc; j += 2) {
                x1.load(cand_row(p, readlane64(my_id, j + 1), ok1), ok1, p.D, lane);
                one(x0, j);
                x0.load(cand_row(p, readlane64(my_id, j + 2), ok0), ok0, p.D, lane);
                one(x1, j + 1);
            }
            if (j + 1 < nc) {
                x1.load(cand_row(p, readlane64(my_id, j + 1), ok1), ok1, p.D, lane);
                one(x0, j);
                one(x1, j + 1);
            } else {
                one(x0, j);
            }
            if (lane < nc) p.out[b * p.out_ld + n] = my_score;
        });
    }
    if (lane == 0) {
        st[w][0] = mrun;
        st[w][1] = Z;
        st[w][2] = Ln;
    }
    __syncthreads();
    float M = 0.f, Zt = 0.f, Lt = 0.f, sc = 1.f;
    if constexpr (RED == 0) {
#pragma unroll
        for (int ww = 0; ww < kWavesPerBlock; ++ww) {
            Zt += st[ww][1];
            Lt += st[ww][2];
        }
    } else {
        M = st[0][0];
#pragma unroll
        for (int ww = 1; ww < kWavesPerBlock; ++ww) M = fmaxf(M, st[ww][0]);
#pragma unroll
        for (int ww = 0; ww < kWavesPerBlock; ++ww) {
            const float f = (st[ww][0] == -INFINITY) ? 0.f : expf(st[ww][0] - M);
            Zt += st[ww][1] * f;
            Lt += st[ww][2] * f;
        }
        sc = (mrun == -INFINITY) ? 0.f : expf(mrun - M);
    }
    // the waves' sums, rescaled to the block maximum, added in wave order
    for (int ww = 0; ww < kWavesPerBlock; ++ww) {
        if (w == ww) {
#pragma unroll
            for (int k = 0; k < G; ++k) {
                const int gi = lane + k * kWave;
#pragma unroll
                for (int o = 0; o < (TWO ? 2 : 1) * NQ; ++o) {
                    const int op = o % NQ;
                    const bool isb = o >= NQ;
                    vecf<V> v = isb ? (op == 0 ? b0[k] : (op == 1 ? b1[k] : b2[k]))
                                    : (op == 0 ? a0[k] : (op == 1 ? a1[k] : a2[k]));
                    if (ww > 0) {
                        const vecf<V> prev = acc[o][gi];
#pragma unroll
                        for (int i = 0; i < V; ++i) v.a[i] = prev.a[i] + sc * v.a[i];
                    } else {
#pragma unroll
                        for (int i = 0; i < V; ++i) v.a[i] = sc * v.a[i];
                    }
                    acc[o][gi] = v;
                }
            }
        }
        __syncthreads();
    }
    if (w == 0) {
        const int D = p.D;
        float* A = p.sh_A + b * NQ * D;
        float* Bv = p.sh_B + b * NQ * D;
#pragma unroll
        for (int k = 0; k < G; ++k) {
            const int gi = lane + k * kWave;
            const bool in = gi < DV;
#pragma unroll
            for (int o = 0; o < NQ; ++o) {
                vstore<V>(A + o * D + gi * V, acc[o][gi], in);
                if constexpr (TWO) vstore<V>(Bv + o * D + gi * V, acc[NQ + o][gi], in);
            }
        }
        if (lane == 0) {
            p.sh_stats[b * 4 + 0] = RED == 0 ? 0.f : M;
            p.sh_stats[b * 4 + 1] = Zt;
            p.sh_stats[b * 4 + 2] = Lt;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Owned positives (KIND_SHARD_POS): one wave per global batch row b. The shard that owns the
// positive tail scores the triple with the single-mode (tail) formula (model.py:127-146), takes its
// gradient dL/ds = go sigmoid(-s) (logsigmoid backward; go is the replica's loss weight) and the
// query-side gradient of the positive slot; every other shard contributes zeros to the SUM.
// ---------------------------------------------------------------------------------------------
template <int FN, int V, int G>
__global__ __launch_bounds__(kBlock) void shard_pos_kernel(ScoreParams p) {
    constexpr int NQ = shard_nq(FN);
    const int64_t b = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (b >= p.B) return;
    const int lane = threadIdx.x & 63;
    const int D = p.D, DV = D / V;
    float* dq = p.sh_dq + (p.B + b) * NQ * D;
    const int64_t row = p.pos_base[b * 3 + 2] - p.c_base;
    if (!(row >= 0 && row < p.c_rows)) {
        for (int64_t i = lane; i < (int64_t)NQ * D; i += kWave) dq[i] = 0.f;
        if (lane == 0) p.sh_stats[b * 4 + 3] = 0.f;
        return;
    }
    Cand<FN, V, G> c;
    c.load(p.cent + row * p.c_ld, true, D, lane);
    const int64_t ri = p.pos_base[b * 3 + 1];
    const bool rok = ri >= 0 && ri < p.r_rows;
    Query<FN, false, V, G> q;
    q.build(p.qent_pos + b * p.q_ld, true, p.rel + (rok ? ri : 0) * p.r_ld + p.r_off, rok, D, lane, p);
    const float s = cand_score<FN, false, V, G>(c, q, p);
    const float g = home_loss_weight(p, b, lane) * sigmoidf(-s);
    if (lane == 0) {
        p.sh_stats[b * 4 + 3] = s;
        const_cast<float*>(p.d_ps)[b] = g;
    }
    vecf<V> dq0[G], dq1[G], dq2[G], dca[G], dcb[G];
#pragma unroll
    for (int k = 0; k < G; ++k) dq0[k] = dq1[k] = dq2[k] = vzero<V>();
    float dmod = 0.f;
    cand_grad<FN, false, V, G, true, false>(c, q, g, lane, DV, p, dq0, dq1, dq2, dca, dcb, dmod);
#pragma unroll
    for (int k = 0; k < G; ++k) {
        const int gi = lane + k * kWave;
        const bool in = gi < DV;
        vstore<V>(dq + gi * V, dq0[k], in);
        if constexpr (NQ > 1) vstore<V>(dq + D + gi * V, dq1[k], in);
        if constexpr (NQ > 2) vstore<V>(dq + 2 * D + gi * V, dq2[k], in);
    }
}

// (The combine step between the two collectives, shard_combine_kernel, lives in kge_abi.hip.)

// ---------------------------------------------------------------------------------------------
// Backward epilogue (KIND_SHARD_EPILOGUE; after the SUM all-reduce of dq): one wave per slot.
//   negative slot b: score gradients of the OWNED candidates from the merged state (the reduction
//     backward of model.py:168-171, as neg_row_bwd), then the chain of the slot's summed query
//     gradient into its query-entity and relation gradients (identical on every rank)
//   positive slot B + b: the chain of the positive slot's query gradient ((h, r) query)
//   all threads: the counting sort's scatter of the owned rows' gradient events
//   an extra last block: every replica's loss, and the running Sum metric += W * sum of the
//     replicas' losses (supervisor.py:28: each replica adds loss * num_replicas_in_sync)
// ---------------------------------------------------------------------------------------------
template <int FN, bool CH, int V, int G>
__global__ __launch_bounds__(kBlock) void shard_epilogue_kernel(ScoreParams p) {
    constexpr int NQ = shard_nq(FN);
    __shared__ float red[3][kBlock];
    const int64_t slot = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int64_t B = p.B;
    const int D = p.D;
    {
        constexpr int U = 4;
        const int total = (int)(B * p.N + 3 * B), nl = (int)gridDim.x * kBlock;
        for (int c0 = (int)blockIdx.x * kBlock + (int)threadIdx.x; c0 < total; c0 += U * nl) {
            int64_t k[U];
#pragma unroll
            for (int u = 0; u < U; ++u) k[u] = c0 + u * nl < total ? step_ev_key<CH>(p, c0 + u * nl) - p.c_base : -1;
            int at[U];
#pragma unroll
            for (int u = 0; u < U; ++u) at[u] = (k[u] >= 0 && k[u] < p.c_rows) ? atomicAdd(p.ev_cursor + k[u], 1) : -1;
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (at[u] >= 0 && at[u] < total) p.ev_code_w[at[u]] = c0 + u * nl;
        }
    }
    if (blockIdx.x == gridDim.x - 1) {
        const int t = threadIdx.x;
        float total_loss = 0.f;
        for (int h = 0; h < p.world; ++h) {
            float sw = 0.f, sp = 0.f, sn = 0.f;
            for (int64_t i = t; i < p.home_B; i += kBlock) {
                const int64_t bb = h * p.home_B + i;
                const float wi = p.weight[bb];
                sw += wi;
                sp += wi * log_sigmoid(p.sh_merged[bb * 4 + 3]);
                sn += wi * p.sh_merged[bb * 4 + 2];
            }
            red[0][t] = sw;
            red[1][t] = sp;
            red[2][t] = sn;
            __syncthreads();
            for (int o = kBlock / 2; o > 0; o >>= 1) {
                if (t < o) {
                    red[0][t] += red[0][t + o];
                    red[1][t] += red[1][t + o];
                    red[2][t] += red[2][t + o];
                }
                __syncthreads();
            }
            const float tw = red[0][0];
            const float loss = (-red[1][0] / tw + -red[2][0] / tw) / 2.f;
            total_loss += loss;
            if (t == 0) p.loss[h] = loss;
            __syncthreads();
        }
        if (t == 0 && p.loss_sum) *p.loss_sum += (float)p.world * total_loss;
        return;
    }
    if (slot >= 2 * B) return;
    const bool negslot = slot < B;
    const int64_t b = negslot ? slot : slot - B;
    vecf<V> dq0[G], dq1[G], dq2[G];
    {
        const float* dq = p.sh_dq + slot * NQ * D;
        const uint32_t nb = (uint32_t)D * 4u;
        const rsrc_t s0 = make_rsrc(dq, nb), s1 = make_rsrc(dq + D, NQ > 1 ? nb : 0u),
                     s2 = make_rsrc(dq + 2 * D, NQ > 2 ? nb : 0u);
#pragma unroll
        for (int k = 0; k < G; ++k) {
            dq0[k] = bload<V>(s0, goff<V>(lane, k));
            dq1[k] = bload<V>(s1, goff<V>(lane, k));
            dq2[k] = bload<V>(s2, goff<V>(lane, k));
        }
    }
    if (negslot) {
        // score gradients of this shard's candidates of row b (neg_row_bwd's arithmetic on the merged state)
        const float* m = p.sh_merged + b * 4;
        const float M = m[0], Z = m[1], R = m[2];
        const float go = home_loss_weight(p, b, lane);
        const float T = p.temperature;
        for (int64_t n = lane; n < p.N; n += kWave) {
            const int64_t row = p.c_idx[b * p.c_stride + n] - p.c_base;
            if (row < 0 || row >= p.c_rows) continue;
            const float x = p.neg_scores[b * p.ns_ld + n];
            float gsn;
            if (p.adversarial) {
                const float pn = expf(T * x - M) / Z;
                gsn = pn * (-sigmoidf(x));
                if (!p.detach) gsn += T * pn * (log_sigmoid(-x) - R);
            } else {
                gsn = (-sigmoidf(x)) * (1.f / (float)p.N);
            }
            const_cast<float*>(p.d_ns)[b * p.N + n] = go * gsn;
        }
        Query<FN, CH, V, G> q;
        int64_t qi, ri;
        bool qok, rok;
        build_query_for<FN, CH, V, G>(p, b, lane, q, qi, ri, qok, rok);
        rows_finalize<FN, CH, V, G>(p, slot, q, dq0, dq1, dq2, qi, ri, qok, rok, lane);
    } else {
        ScoreParams pp = p;
        pp.qent = p.qent_pos;  // the positive call's query: (h, r)
        const int64_t ri = p.pos_base[b * 3 + 1];
        const bool rok = ri >= 0 && ri < p.r_rows;
        Query<FN, false, V, G> q;
        q.build(pp.qent + b * pp.q_ld, true, pp.rel + (rok ? ri : 0) * pp.r_ld + pp.r_off, rok, D, lane, pp);
        rows_finalize<FN, false, V, G>(pp, slot, q, dq0, dq1, dq2, b, ri, true, rok, lane);
    }
}

template <int FN, bool CH, int V, int G>
void launch_shard(const ScoreParams& p, int kind, hipStream_t st, int blocks) {
    if constexpr (FN != KGE_PROTATE && G <= kFwdGradMaxG) {
        if (kind == KIND_SHARD_FWD_GRAD) {
            if (!p.adversarial)
                hipLaunchKernelGGL((shard_fwd_grad_kernel<FN, CH, V, G, 0>), dim3(blocks), dim3(kBlock), 0, st, p);
            else if (p.detach)
                hipLaunchKernelGGL((shard_fwd_grad_kernel<FN, CH, V, G, 1>), dim3(blocks), dim3(kBlock), 0, st, p);
            else
                hipLaunchKernelGGL((shard_fwd_grad_kernel<FN, CH, V, G, 2>), dim3(blocks), dim3(kBlock), 0, st, p);
        } else if (kind == KIND_SHARD_POS) {
            if constexpr (!CH) hipLaunchKernelGGL((shard_pos_kernel<FN, V, G>), dim3(blocks), dim3(kBlock), 0, st, p);
        } else if (kind == KIND_SHARD_EPILOGUE) {
            hipLaunchKernelGGL((shard_epilogue_kernel<FN, CH, V, G>), dim3(blocks), dim3(kBlock), 0, st, p);
        }
    }
}

}  // namespace kge_impl
