// kge_exchange.hip — the row-sharded scoring step's exchange (SURVEY §8e owner-computes), sized to the
// information it carries.
//
// The global batch (Bg = W * home_B rows, home rank h owning rows [h home_B, (h+1) home_B)) is identical
// on every rank, so every rank can compute, from the ids alone, who owns which query row and which
// candidate, and in which order each owner will send them. Nothing but payload crosses xGMI:
//   * query rows: owner o gathers the chunk's query-entity rows it owns, compacted in row order
//     (kge_shard_gather_queries), and every rank receives every owner's rows (an all-to-all whose pieces
//     are the same block, sized exactly: no padding); a row's place in the received block is implicit
//     (owner, rank among that owner's rows of the chunk);
//   * scores: owner o writes only the scores of the candidates it owns, compacted per row in column
//     order with the row's positive last (kge_shard_score), and sends home h exactly the
//     scores of h's rows (all-to-all, no indices); home h scatters them back with the same ranks
//     (kge_shard_finish) and reduces its rows.
// kge_shard_plan computes the ownership counts and ranks once per global batch (two launches, O(Bg N)
// integer work on device) and this rank's bucket of owned candidates; its small summary (the all-to-all
// split sizes) is the only thing the host reads.
#include <string>

#include "kge_device.h"

namespace kge_impl {

int set_error(int code, const char* msg);  // kge_abi.hip

namespace {

constexpr int kMaxWorld = 64;  // one lane per rank in the plan's per-owner counts
constexpr int kSlices = 8;     // XCD slices of a shard (the bucket's groups; kge_device.h's sliced kernels)

// floor(a / b) for 0 <= a < 2^53, b >= 1, a / b < 2^31, with inv = 1 / b: the double quotient is within
// one of the exact one, so one correction step makes it exact (no 64-bit integer division on the SIMD)
__device__ __forceinline__ int div_floor(int64_t a, int64_t b, double inv) {
    int q = (int)((double)a * inv);
    const int64_t r = a - (int64_t)q * b;
    q += (r >= b) - (r < 0);
    return q;
}

// Block partition of entity rows over W ranks (distributed.shard_bounds): the first E % W ranks hold
// one extra row. Returns the owner of id, or -1 for an id outside [0, E) (no owner: scores 0).
struct Owners {
    int64_t E, split;
    int W, extra;
    int64_t base;
    double inv_b1, inv_b;  // 1 / (base + 1), 1 / base
    __device__ __forceinline__ int of(int64_t id) const {
        if (id < 0 || id >= E) return -1;
        if (id < split) return div_floor(id, base + 1, inv_b1);
        return extra + div_floor(id - split, base, inv_b);
    }
};

Owners make_owners(int64_t E, int W) {
    Owners o;
    o.E = E;
    o.W = W;
    o.base = E / W;
    o.extra = (int)(E % W);
    o.split = (int64_t)o.extra * (o.base + 1);
    o.inv_b1 = 1.0 / (double)(o.base + 1);
    o.inv_b = 1.0 / (double)o.base;
    return o;
}

// Rank r's bucket (kge_shard_plan's optional output, the input of kge_shard_score): row g's negatives
// owned by r (and, tail-batch, its positive) as (local shard row, rank among the row's owned candidates in
// column order), grouped by XCD slice (local row / S), in no particular order inside a slice:
//   ent [Bg, N + 1] int2: row g's entries at ent[g, 0 .. start[g, 8]);
//   start [Bg, 9]: slice x's entries are ent[g, start[g, x] .. start[g, x + 1]).
struct Bucket {
    int2* ent;
    int* start;
    int64_t lo, S;  // this rank's first row, slice height ceil(rows / 8)
    double inv_S;
    int rank, pos_in;  // pos_in: the positive (candidate N) belongs in the bucket (tail-batch)
};

// candidate n of global row g (n < N: negative, n == N: the positive, owned by the owner of pos[g, pcol]),
// -1 past the row
__device__ __forceinline__ int64_t cand_id(const int64_t* pos, const int64_t* neg, int64_t neg_ld, int64_t N,
                                           int64_t g, int64_t n, int pcol) {
    if (n < N) return neg[g * neg_ld + n];
    if (n == N) return pos[g * 3 + pcol];
    return -1;
}

// inclusive prefix sum over the wave
__device__ __forceinline__ int wave_incl_scan(int v, int lane) {
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        const int u = __shfl_up(v, o, kWave);
        if (lane >= o) v += u;
    }
    return v;
}

// Plan pass 1, one wave per global row g: cnt[o * Bg + g] = candidates of row g (N negatives + the
// positive) owned by rank o; qown[c * Bg + g] = owner of the row's query entity of column c; with bk.ent,
// the row's bucket of rank bk.rank. NR > 0: the row's N + 1 <= 64 NR ids are loaded at once (NR loads in
// flight) and the bucket's local rows stay in registers between its two passes (per-slice counts, then
// placement); NR = 0: one 64-id chunk at a time, the ids re-read for the placement.
//
// The counts go through LDS atomics (one ds_add per 64 candidates instead of a ballot per owner): the
// kernel is VALU-issue bound, ~4 waves per SIMD each running its row's whole walk. Entries inside a slice
// land in LDS-atomic order; kge_shard_score does not depend on it (each entry carries its rank).
template <int NR>
__global__ __launch_bounds__(kBlock) void plan_count_kernel(const int64_t* __restrict__ pos,
                                                            const int64_t* __restrict__ neg, int64_t neg_ld,
                                                            int64_t Bg, int64_t N, Owners own, int ncol, int qc0,
                                                            int qc1, int pcol, int* __restrict__ cnt,
                                                            int* __restrict__ qown, Bucket bk) {
    __shared__ int ocnt[kWavesPerBlock][kMaxWorld];
    __shared__ int scur[kWavesPerBlock][kSlices];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t g = (int64_t)blockIdx.x * kWavesPerBlock + w;
    if (g >= Bg) return;  // whole waves: no block barrier below
    const bool buck = bk.ent != nullptr;
    const int nch = (int)((N + kWave) / kWave);  // 64-candidate chunks of the N + 1 candidates
    ocnt[w][lane] = 0;
    if (lane < kSlices) scur[w][lane] = 0;
    __builtin_amdgcn_wave_barrier();
    // one chunk's ownership counts; returns (slice << 25 | local row) if this lane's candidate goes in the
    // bucket, else -1
    auto count = [&](int k, int64_t id) -> int {
        const int64_t n = (int64_t)k * kWave + lane;
        const int o = own.of(id);
        if (o >= 0) atomicAdd(&ocnt[w][o], 1);
        if (!buck || o != bk.rank || (n >= N && !bk.pos_in)) return -1;
        const int l = (int)(id - bk.lo);
        const int x = div_floor(l, bk.S, bk.inv_S);
        atomicAdd(&scur[w][x], 1);
        return (x << 25) | l;
    };
    constexpr int NC = NR > 0 ? NR : 1;
    int loc[NC];
    if constexpr (NR > 0) {
        int64_t ids[NR];
#pragma unroll
        for (int k = 0; k < NR; ++k) ids[k] = cand_id(pos, neg, neg_ld, N, g, (int64_t)k * kWave + lane, pcol);
#pragma unroll
        for (int k = 0; k < NR; ++k) loc[k] = k < nch ? count(k, ids[k]) : -1;
    } else {
        for (int k = 0; k < nch; ++k) count(k, cand_id(pos, neg, neg_ld, N, g, (int64_t)k * kWave + lane, pcol));
    }
    __builtin_amdgcn_wave_barrier();
    if (lane < own.W) cnt[(int64_t)lane * Bg + g] = ocnt[w][lane];
    if (lane < ncol) qown[(int64_t)lane * Bg + g] = own.of(pos[g * 3 + (lane == 0 ? qc0 : qc1)]);
    if (!buck) return;
    // slice starts (lane x: exclusive prefix of the slice counts; lane 8: the row's total); the LDS
    // counters become the slices' cursors
    const int sv = lane < kSlices ? scur[w][lane] : 0;
    const int sbase = wave_incl_scan(sv, lane) - sv;
    if (lane <= kSlices) bk.start[g * (kSlices + 1) + lane] = sbase;
    __builtin_amdgcn_wave_barrier();
    if (lane < kSlices) scur[w][lane] = sbase;
    __builtin_amdgcn_wave_barrier();
    int run = 0;  // bucket entries met so far in column order: the next one's rank in the row
    int2* ent = bk.ent + g * (N + 1);
    auto place = [&](int xl) {
        const uint64_t mb = __ballot(xl >= 0);
        const int r = run + lanes_below(mb);
        run += __popcll(mb);
        if (xl >= 0) {
            const int at = atomicAdd(&scur[w][xl >> 25], 1);
            ent[at] = make_int2(xl & ((1 << 25) - 1), r);
        }
    };
    if constexpr (NR > 0) {
#pragma unroll
        for (int k = 0; k < NR; ++k) place(loc[k]);
    } else {
        for (int k = 0; k < nch; ++k) {
            const int64_t n = (int64_t)k * kWave + lane;
            const int64_t id = cand_id(pos, neg, neg_ld, N, g, n, pcol);
            int xl = -1;
            if (own.of(id) == bk.rank && (n < N || bk.pos_in)) {
                const int l = (int)(id - bk.lo);
                xl = (div_floor(l, bk.S, bk.inv_S) << 25) | l;
            }
            place(xl);
        }
    }
}

// Plan pass 2, one wave per task:
//   home task (h, o), W^2 of them:   hpre[o * Bg + g] = sum of cnt[o, g'] over the rows g' < g of home h
//                                    (exclusive), tot[h * W + o] = the home's total for owner o;
//   query task (k, c, o), K ncol W:  qslot[c * Bg + g] = rank of row g among chunk k's rows whose column-c
//                                    query entity rank o owns (the o = 0 task writes -1 for rows without
//                                    an owner), qtot[(k * ncol + c) * W + o] = their count.
// Each wave reads its segment 8 x 64 values at a time (8 loads in flight) and carries a running total.
constexpr int kScanU = 8;
__global__ __launch_bounds__(kBlock) void plan_scan_kernel(const int* __restrict__ cnt, const int* __restrict__ qown,
                                                           int64_t Bg, int64_t home_B, int64_t chunk_rows, int W,
                                                           int ncol, int chunks, int* __restrict__ hpre,
                                                           int* __restrict__ qslot, int* __restrict__ tot,
                                                           int* __restrict__ qtot) {
    const int64_t t = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int64_t nh = (int64_t)W * W;
    if (t < nh) {
        const int h = (int)(t / W), o = (int)(t % W);
        const int* src = cnt + (int64_t)o * Bg + (int64_t)h * home_B;
        int* dst = hpre + (int64_t)o * Bg + (int64_t)h * home_B;
        int carry = 0;
        for (int64_t i0 = 0; i0 < home_B; i0 += kScanU * kWave) {
            int v[kScanU];
#pragma unroll
            for (int u = 0; u < kScanU; ++u) {
                const int64_t i = i0 + u * kWave + lane;
                v[u] = i < home_B ? src[i] : 0;
            }
#pragma unroll
            for (int u = 0; u < kScanU; ++u) {
                const int64_t i = i0 + u * kWave + lane;
                const int inc = wave_incl_scan(v[u], lane);
                if (i < home_B) dst[i] = carry + inc - v[u];
                carry += __builtin_amdgcn_readlane(inc, kWave - 1);
            }
        }
        if (lane == 0) tot[(int64_t)h * W + o] = carry;
        return;
    }
    const int64_t j = t - nh;
    if (j >= (int64_t)chunks * ncol * W) return;
    const int o = (int)(j % W), c = (int)((j / W) % ncol), k = (int)(j / ((int64_t)W * ncol));
    const int64_t r0 = (int64_t)k * chunk_rows;
    const int* src = qown + (int64_t)c * Bg + r0;
    int* dst = qslot + (int64_t)c * Bg + r0;
    int carry = 0;
    for (int64_t i0 = 0; i0 < chunk_rows; i0 += kScanU * kWave) {
        int v[kScanU];
#pragma unroll
        for (int u = 0; u < kScanU; ++u) {
            const int64_t i = i0 + u * kWave + lane;
            v[u] = i < chunk_rows ? src[i] : -2;
        }
#pragma unroll
        for (int u = 0; u < kScanU; ++u) {
            const int64_t i = i0 + u * kWave + lane;
            const uint64_t m = __ballot(v[u] == o);
            if (v[u] == o)
                dst[i] = carry + lanes_below(m);
            else if (o == 0 && v[u] == -1)
                dst[i] = -1;
            carry += __popcll(m);
        }
    }
    if (lane == 0) qtot[((int64_t)k * ncol + c) * W + o] = carry;
}

// Sender side of the query exchange, one wave per (column c, row i of rows [row0, row0 + rows)). Owner o's
// rows of chunk k go to every rank (an all-to-all whose W pieces are the same block: NCCL has no
// all-gather of unequal sizes): piece = [column 0 rows | column 1 rows] in slot order, per = sum_c qtot[k,
// c, me] rows, written W times into chunk k's send block [W, per, width]. The all-to-all output holds the
// owners' pieces in rank order, so the row holding (owner o, column c, slot) is roff[o] + (c ? qtot[k, 0, o]
// : 0) + slot, roff[o] = sum over o' < o of the pieces: qidx[c * rows + i] (-1 without an owner). One launch
// may cover every chunk (rows = Bg): chunk k's send block then starts after chunks 0..k-1's (W per_k' rows
// each).
__global__ __launch_bounds__(kBlock) void gather_queries_kernel(const float* __restrict__ shard, int64_t shard_rows,
                                                                int64_t ld, int64_t lo, const int64_t* __restrict__ pos,
                                                                int64_t Bg, int64_t row0, int64_t rows,
                                                                int64_t chunk_rows, int ncol, int qc0, int qc1,
                                                                const int* __restrict__ qown,
                                                                const int* __restrict__ qslot,
                                                                const int* __restrict__ qtot_all, int W, int rank,
                                                                int64_t width, float* __restrict__ send,
                                                                int64_t* __restrict__ qidx, int vec4) {
    const int64_t t = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (t >= (int64_t)ncol * rows) return;
    const int lane = threadIdx.x & 63;
    const int c = (int)(t / rows);
    const int64_t i = t - (int64_t)c * rows, g = row0 + i;
    const int k = (int)(g / chunk_rows);
    const int* qtot = qtot_all + (int64_t)k * ncol * W;
    const int o = qown[(int64_t)c * Bg + g];
    const int64_t s = qslot[(int64_t)c * Bg + g];
    // lane l < W: rank l's piece size; exclusive prefix = where its piece starts
    int piece = 0, col0 = 0;
    if (lane < W) {
        col0 = qtot[lane];
        piece = col0 + (ncol > 1 ? qtot[W + lane] : 0);
    }
    const int roff = wave_incl_scan(piece, lane) - piece;
    // rows of this rank's send blocks of the launch's chunks before k (lane k' < k: W per_k')
    int64_t before = 0;
    const int k0 = (int)(row0 / chunk_rows);
    if (k > k0) {
        int mine = 0;
        if (lane < k - k0) {
            const int* qk = qtot_all + (int64_t)(k0 + lane) * ncol * W;
            mine = qk[rank] + (ncol > 1 ? qk[W + rank] : 0);
        }
        for (int off = 32; off > 0; off >>= 1) mine += __shfl_xor(mine, off, kWave);
        before = (int64_t)W * mine;
    }
    if (o < 0) {
        if (lane == 0) qidx[t] = -1;
        return;
    }
    // every cross-lane read happens with the whole wave active (inside `if (lane == 0)` the compiler may
    // compute roff for lane 0 only and read garbage from lane o)
    const int64_t inner = (c ? __builtin_amdgcn_readlane(col0, o) : 0) + s;
    const int64_t at = __builtin_amdgcn_readlane(roff, o) + inner;
    const int64_t per = __builtin_amdgcn_readlane(piece, rank);
    if (lane == 0) qidx[t] = at;
    if (o != rank) return;
    send += before * width;
    const int64_t r = pos[g * 3 + (c == 0 ? qc0 : qc1)] - lo;
    const bool ok = r >= 0 && r < shard_rows;  // o == rank implies it
    const float* src = shard + (ok ? r : 0) * ld;
    if (vec4) {
        const rsrc_t rs = make_rsrc(src, ok ? (uint32_t)(width * 4) : 0u);
        for (int64_t e = (int64_t)lane * 4; e < width; e += 4 * kWave) {
            const vecf<4> v = bload<4>(rs, (uint32_t)(e * 4));
            for (int d = 0; d < W; ++d) *reinterpret_cast<vecf<4>*>(send + (d * per + inner) * width + e) = v;
        }
    } else {
        for (int64_t e = lane; e < width; e += kWave) {
            const float v = ok ? src[e] : 0.f;
            for (int d = 0; d < W; ++d) send[(d * per + inner) * width + e] = v;
        }
    }
}

// Home side, one wave per home row b (global row g = h home_B + b): every candidate's score comes from the
// block its owner o sent (recv holds the owners' blocks in rank order, roff[o] = sum of tot[h, o' < o]),
// at the row's run start hpre[o, g] plus the candidate's rank among the row's o-owned ones. Candidates
// without an owner score 0. Writes scores [B, N], the positive's raw score and logsigmoid; the row
// reductions follow in shard_rows_reduce_kernel (rows of more than 20 x 64 columns).
__global__ __launch_bounds__(kBlock) void shard_finish_kernel(const float* __restrict__ recv, const int* __restrict__ tot,
                                                              const int* __restrict__ hpre,
                                                              const int64_t* __restrict__ pos,
                                                              const int64_t* __restrict__ neg, int64_t neg_ld,
                                                              int64_t Bg, int64_t B, int64_t N, Owners own, int h,
                                                              int pcol, float* __restrict__ scores, int64_t ns_ld,
                                                              float* __restrict__ pos_raw, float* __restrict__ pos_ls) {
    const int64_t b = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (b >= B) return;
    const int lane = threadIdx.x & 63;
    const int64_t g = (int64_t)h * B + b;
    const int W = own.W;
    const int t = lane < W ? tot[(int64_t)h * W + lane] : 0;
    const int base = (wave_incl_scan(t, lane) - t) + (lane < W ? hpre[(int64_t)lane * Bg + g] : 0);
    int seen = 0;  // lane o: candidates of this row owned by rank o met so far
    for (int64_t c0 = 0; c0 <= N; c0 += kWave) {
        const int64_t n = c0 + lane;
        const int o = own.of(cand_id(pos, neg, neg_ld, N, g, n, pcol));
        int idx = -1;
        for (int q = 0; q < W; ++q) {
            const uint64_t m = __ballot(o == q);
            if (m == 0) continue;  // wave-uniform
            const int start = __builtin_amdgcn_readlane(base, q) + __builtin_amdgcn_readlane(seen, q);
            if (o == q) idx = start + lanes_below(m);
            if (lane == q) seen += __popcll(m);
        }
        const float s = idx >= 0 ? recv[idx] : 0.f;
        if (n < N) {
            scores[b * ns_ld + n] = s;
        } else if (n == N) {
            pos_raw[b] = s;
            pos_ls[b] = log_sigmoid(s);
        }
    }
}

// The same with the row reductions, a block of 4 waves per home row b: wave w takes the row's 64-column slots [w SPW, (w+1) SPW)
// (the one-wave form above runs ~10K dependent instructions per row at half a wave per SIMD). Ranks: per
// slot a ballot per owner within the wave, plus the earlier waves' per-owner counts through LDS. The
// reduction keeps row_reduce's order bitwise: the row max over the waves (exact), every slot's softmax
// weight and logsigmoid computed by its wave into LDS, then wave 0 sums them lane-sequentially over the
// slots as row_reduce_vals does.
template <int SPW>
__global__ __launch_bounds__(kBlock) void shard_finish_block_kernel(
    const float* __restrict__ recv, const int* __restrict__ tot, const int* __restrict__ hpre,
    const int64_t* __restrict__ pos, const int64_t* __restrict__ neg, int64_t neg_ld, int64_t Bg, int64_t B, int64_t N,
    Owners own, int h, int pcol, float T, int adversarial, float* __restrict__ scores, int64_t ns_ld,
    float* __restrict__ out_neg, float* __restrict__ pos_raw, float* __restrict__ pos_ls) {
    constexpr int NR = kWavesPerBlock * SPW;
    __shared__ int base[kMaxWorld];                   // roff[o] + hpre[o, g]
    __shared__ int wcnt[kWavesPerBlock][kMaxWorld];   // per wave: its candidates owned by o
    __shared__ float ev[NR][kWave], lv[NR][kWave];    // per slot: softmax weight, logsigmoid(-s)
    __shared__ float wmax[kWavesPerBlock];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t b = blockIdx.x, g = (int64_t)h * B + b;
    const int W = own.W;
    if (w == 0) {
        const int t = lane < W ? tot[(int64_t)h * W + lane] : 0;
        base[lane] = (wave_incl_scan(t, lane) - t) + (lane < W ? hpre[(int64_t)lane * Bg + g] : 0);
    }
    int64_t ids[SPW];
#pragma unroll
    for (int j = 0; j < SPW; ++j) ids[j] = cand_id(pos, neg, neg_ld, N, g, (int64_t)(w * SPW + j) * kWave + lane, pcol);
    int rel[SPW], ow[SPW];
    int seen = 0;  // lane q: this wave's candidates owned by rank q met so far
#pragma unroll
    for (int j = 0; j < SPW; ++j) {
        const int o = own.of(ids[j]);
        int idx = -1;
        for (int q = 0; q < W; ++q) {
            const uint64_t m = __ballot(o == q);
            if (m == 0) continue;  // wave-uniform
            const int s0 = __builtin_amdgcn_readlane(seen, q);
            if (o == q) idx = s0 + lanes_below(m);
            if (lane == q) seen += __popcll(m);
        }
        rel[j] = idx;
        ow[j] = o;
    }
    wcnt[w][lane] = seen;
    __syncthreads();
    float v[SPW];
#pragma unroll
    for (int j = 0; j < SPW; ++j) {
        const int o = ow[j];
        v[j] = 0.f;
        if (o >= 0) {
            int at = base[o] + rel[j];
            for (int u = 0; u < w; ++u) at += wcnt[u][o];
            v[j] = recv[at];
        }
    }
#pragma unroll
    for (int j = 0; j < SPW; ++j) {
        const int64_t n = (int64_t)(w * SPW + j) * kWave + lane;
        if (n < N) {
            scores[b * ns_ld + n] = v[j];
        } else if (n == N) {
            pos_raw[b] = v[j];
            pos_ls[b] = log_sigmoid(v[j]);
        }
    }
    float m = 0.f;
    if (adversarial) {
        m = -INFINITY;
#pragma unroll
        for (int j = 0; j < SPW; ++j)
            if (lane + (int64_t)(w * SPW + j) * kWave < N) m = fmaxf(m, T * v[j]);
        m = wave_max(m);
        if (lane == 0) wmax[w] = m;
        __syncthreads();
        m = fmaxf(fmaxf(wmax[0], wmax[1]), fmaxf(wmax[2], wmax[3]));
    }
#pragma unroll
    for (int j = 0; j < SPW; ++j) {
        const int k = w * SPW + j;
        if (lane + (int64_t)k * kWave < N) {
            if (adversarial) ev[k][lane] = rr_exp(T * v[j] - m);  // row_reduce's exp / log (kge_device.h)
            lv[k][lane] = rr_log_sigmoid(-v[j]);
        }
    }
    __syncthreads();
    if (w) return;
    float z = 0.f, wsum = 0.f;
    if (adversarial) {
#pragma unroll
        for (int k = 0; k < NR; ++k)
            if (lane + (int64_t)k * kWave < N) {
                const float e = ev[k][lane];
                z += e;
                wsum += e * lv[k][lane];
            }
        const float r = wave_sum(wsum) / wave_sum(z);
        if (lane == 0) out_neg[b] = r;
    } else {
#pragma unroll
        for (int k = 0; k < NR; ++k)
            if (lane + (int64_t)k * kWave < N) wsum += lv[k][lane];
        const float r = wave_sum(wsum) / (float)N;
        if (lane == 0) out_neg[b] = r;
    }
}

// N > 1024: the reduction re-reads the written row (a second launch)
__global__ __launch_bounds__(kBlock) void shard_rows_reduce_kernel(const float* __restrict__ scores, int64_t ns_ld,
                                                                   int64_t B, int64_t N, float T, int adversarial,
                                                                   float* __restrict__ out_neg) {
    const int64_t b = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (b >= B) return;
    const int lane = threadIdx.x & 63;
    const float r = row_reduce(scores + b * ns_ld, N, T, adversarial, lane);
    if (lane == 0) out_neg[b] = r;
}

int launched(const char* what) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_error(KGE_EHIP, (std::string(what) + ": " + hipGetErrorString(e)).c_str());
    return set_error(0, "");
}

int check_world(int64_t Bg, int world, int64_t nentity) {
    if (world < 1 || world > kMaxWorld) return set_error(KGE_ENOTSUP, "row-sharded exchange: world must be 1..64");
    if (Bg < 0 || Bg % world) return set_error(KGE_EINVAL, "row-sharded exchange: Bg must split evenly over ranks");
    if (nentity < world) return set_error(KGE_EINVAL, "row-sharded exchange: fewer entities than ranks");
    return 0;
}

// The exchanged query columns and the column whose owner scores the positive. The forward (flags 0)
// exchanges only the negative call's query entity (head-batch: the tail, else the head); its positive is
// scored by the owner of the head in head-batch mode (query (h, r) from its shard, the tail row from the
// exchanged block), by the owner of the tail otherwise. KGE_SHARD_TWO_COLUMNS (the sharded train step)
// also exchanges the positive's query entity (the head) and leaves the positive with the tail's owner.
int query_cols(int mode, int flags, int& qc0, int& qc1, int& pcol) {
    const bool head = mode == KGE_HEAD_BATCH;
    qc0 = head ? 2 : 0;
    qc1 = 0;
    pcol = (head && !(flags & KGE_SHARD_TWO_COLUMNS)) ? 0 : 2;
    return (head && (flags & KGE_SHARD_TWO_COLUMNS)) ? 2 : 1;
}

}  // namespace
}  // namespace kge_impl

using namespace kge_impl;

extern "C" {

int kge_shard_plan(const int64_t* pos, const int64_t* neg, int64_t neg_ld, int64_t Bg, int64_t N, int64_t nentity,
                   int world, int chunks, int mode, int flags, int rank, int* cnt, int* hpre, int* qown, int* qslot,
                   int* summary, int* bucket, int* bucket_start, void* stream) {
    int rc = check_world(Bg, world, nentity);
    if (rc) return rc;
    if (mode != KGE_HEAD_BATCH && mode != KGE_TAIL_BATCH)
        return set_error(KGE_EINVAL, "kge_shard_plan: mode must be 0 (head-batch) or 1 (tail-batch)");
    if (N < 0 || chunks < 1 || world % chunks) return set_error(KGE_EINVAL, "kge_shard_plan: chunks must divide world");
    if ((bucket != nullptr) != (bucket_start != nullptr))
        return set_error(KGE_EINVAL, "kge_shard_plan: bucket and bucket_start go together");
    if (bucket && (flags != 0 || rank < 0 || rank >= world))
        return set_error(KGE_EINVAL, "kge_shard_plan: a bucket needs flags 0 and a rank in [0, world)");
    if (Bg == 0) return set_error(0, "");
    if (!pos || (N > 0 && !neg) || !cnt || !hpre || !qown || !qslot || !summary)
        return set_error(KGE_EINVAL, "kge_shard_plan: null pointer");
    int qc0, qc1, pcol;
    const int ncol = query_cols(mode, flags, qc0, qc1, pcol);
    const Owners own = make_owners(nentity, world);
    Bucket bk{};
    if (bucket) {
        const int64_t rows = own.base + (rank < own.extra ? 1 : 0);
        bk.ent = reinterpret_cast<int2*>(bucket);
        bk.start = bucket_start;
        bk.lo = rank < own.extra ? (int64_t)rank * (own.base + 1) : own.split + (int64_t)(rank - own.extra) * own.base;
        bk.S = (rows + kSlices - 1) / kSlices;
        bk.inv_S = 1.0 / (double)bk.S;
        bk.rank = rank;
        bk.pos_in = mode == KGE_TAIL_BATCH;  // head-batch: the head's owner scores the positive (kge_shard_score)
        if (rows >= ((int64_t)1 << 25)) return set_error(KGE_ENOTSUP, "kge_shard_plan: a bucket needs < 2^25 shard rows");
    }
    const hipStream_t st = (hipStream_t)stream;
    const dim3 grid((unsigned)((Bg + kWavesPerBlock - 1) / kWavesPerBlock));
    if (N + 1 <= 4 * kWave)
        hipLaunchKernelGGL(plan_count_kernel<4>, grid, dim3(kBlock), 0, st, pos, neg, neg_ld, Bg, N, own, ncol, qc0, qc1,
                           pcol, cnt, qown, bk);
    else if (N + 1 <= 17 * kWave)
        hipLaunchKernelGGL(plan_count_kernel<17>, grid, dim3(kBlock), 0, st, pos, neg, neg_ld, Bg, N, own, ncol, qc0, qc1,
                           pcol, cnt, qown, bk);
    else
        hipLaunchKernelGGL(plan_count_kernel<0>, grid, dim3(kBlock), 0, st, pos, neg, neg_ld, Bg, N, own, ncol, qc0, qc1,
                           pcol, cnt, qown, bk);
    rc = launched("kge_shard_plan counts");
    if (rc) return rc;
    const int64_t home_B = Bg / world, chunk_rows = Bg / chunks;
    const int64_t tasks = (int64_t)world * world + (int64_t)chunks * ncol * world;
    hipLaunchKernelGGL(plan_scan_kernel, dim3((unsigned)((tasks + kWavesPerBlock - 1) / kWavesPerBlock)), dim3(kBlock), 0,
                       st, cnt, qown, Bg, home_B, chunk_rows, world, ncol, chunks, hpre, qslot, summary,
                       summary + (int64_t)world * world);
    return launched("kge_shard_plan scans");
}

int kge_shard_gather_queries(const float* shard, int64_t shard_rows, int64_t ld, int64_t shard_lo,
                             const int64_t* pos, int64_t Bg, int chunks, int chunk, int64_t width, int world,
                             int rank, int mode, int flags, const int* qown, const int* qslot, const int* summary,
                             float* send, int64_t* qidx, void* stream) {
    if (world < 1 || world > kMaxWorld || rank < 0 || rank >= world)
        return set_error(KGE_EINVAL, "kge_shard_gather_queries: bad world/rank");
    if (mode != KGE_HEAD_BATCH && mode != KGE_TAIL_BATCH)
        return set_error(KGE_EINVAL, "kge_shard_gather_queries: mode must be 0 or 1");
    if (Bg < 0 || chunks < 1 || chunks > kWave || Bg % chunks || chunk < -1 || chunk >= chunks || width <= 0 ||
        shard_rows < 0)
        return set_error(KGE_EINVAL, "kge_shard_gather_queries: bad shape");
    if (Bg == 0) return set_error(0, "");
    if (!shard || !pos || !qown || !qslot || !summary || !qidx)
        return set_error(KGE_EINVAL, "kge_shard_gather_queries: null pointer");
    int qc0, qc1, pcol;
    const int ncol = query_cols(mode, flags, qc0, qc1, pcol);
    const int64_t chunk_rows = Bg / chunks;
    const int64_t row0 = chunk < 0 ? 0 : chunk * chunk_rows, rows = chunk < 0 ? Bg : chunk_rows;
    const int* qtot_all = summary + (int64_t)world * world;
    const int vec4 = (width % 4 == 0 && ld % 4 == 0 && ((uintptr_t)shard % 16) == 0 && ((uintptr_t)send % 16) == 0);
    const int64_t waves = ncol * rows;
    hipLaunchKernelGGL(gather_queries_kernel, dim3((unsigned)((waves + kWavesPerBlock - 1) / kWavesPerBlock)),
                       dim3(kBlock), 0, (hipStream_t)stream, shard, shard_rows, ld, shard_lo, pos, Bg, row0, rows,
                       chunk_rows, ncol, qc0, qc1, qown, qslot, qtot_all, world, rank, width, send, qidx, vec4);
    return launched("kge_shard_gather_queries");
}

int kge_shard_finish(const float* recv, const int* tot, const int* hpre, const int64_t* pos, const int64_t* neg,
                     int64_t neg_ld, int64_t Bg, int64_t N, int64_t nentity, int world, int home, int mode,
                     float temperature, int adversarial, float* scores, int64_t ns_ld, float* out_neg,
                     float* pos_scores, float* out_pos, void* stream) {
    int rc = check_world(Bg, world, nentity);
    if (rc) return rc;
    if (home < 0 || home >= world || N < 0) return set_error(KGE_EINVAL, "kge_shard_finish: bad home or N");
    if (mode != KGE_HEAD_BATCH && mode != KGE_TAIL_BATCH)
        return set_error(KGE_EINVAL, "kge_shard_finish: mode must be 0 or 1");
    const int64_t B = Bg / world;
    if (B == 0) return set_error(0, "");
    if (!tot || !hpre || !pos || (N > 0 && (!neg || !scores)) || !out_neg || !pos_scores || !out_pos)
        return set_error(KGE_EINVAL, "kge_shard_finish: null pointer");
    // recv may be NULL only when nothing was received (no candidate of these rows has an owner)
    int qc0, qc1, pcol;
    query_cols(mode, 0, qc0, qc1, pcol);
    const Owners own = make_owners(nentity, world);
    const hipStream_t st = (hipStream_t)stream;
    const dim3 grid((unsigned)((B + kWavesPerBlock - 1) / kWavesPerBlock));
    // the row's positive is column N: N + 1 columns cover ceil((N + 1) / 64) slots, 4 waves per row
    const dim3 rows_grid((unsigned)B);
    if (N + 1 <= 4 * kWave)
        hipLaunchKernelGGL(shard_finish_block_kernel<1>, rows_grid, dim3(kBlock), 0, st, recv, tot, hpre, pos, neg,
                           neg_ld, Bg, B, N, own, home, pcol, temperature, adversarial, scores, ns_ld, out_neg,
                           pos_scores, out_pos);
    else if (N + 1 <= 8 * kWave)
        hipLaunchKernelGGL(shard_finish_block_kernel<2>, rows_grid, dim3(kBlock), 0, st, recv, tot, hpre, pos, neg,
                           neg_ld, Bg, B, N, own, home, pcol, temperature, adversarial, scores, ns_ld, out_neg,
                           pos_scores, out_pos);
    else if (N + 1 <= 20 * kWave)
        hipLaunchKernelGGL(shard_finish_block_kernel<5>, rows_grid, dim3(kBlock), 0, st, recv, tot, hpre, pos, neg,
                           neg_ld, Bg, B, N, own, home, pcol, temperature, adversarial, scores, ns_ld, out_neg,
                           pos_scores, out_pos);
    else {
        hipLaunchKernelGGL(shard_finish_kernel, grid, dim3(kBlock), 0, st, recv, tot, hpre, pos, neg, neg_ld, Bg, B, N,
                           own, home, pcol, scores, ns_ld, pos_scores, out_pos);
        rc = launched("kge_shard_finish scatter");
        if (rc) return rc;
        hipLaunchKernelGGL(shard_rows_reduce_kernel, grid, dim3(kBlock), 0, st, scores, ns_ld, B, N, temperature,
                           adversarial, out_neg);
    }
    return launched("kge_shard_finish");
}

}  // extern "C"
