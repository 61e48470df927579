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
//     order with the row's positive last (kge_score_sharded_compact), and sends home h exactly the
//     scores of h's rows (all-to-all, no indices); home h scatters them back with the same ranks
//     (kge_shard_finish) and reduces its rows.
// kge_shard_plan computes the ownership counts and ranks once per global batch (two launches, O(Bg N)
// integer work on device); its small summary (the all-to-all split sizes) is the only thing the host reads.
#include <string>

#include "kge_device.h"

namespace kge_impl {

int set_error(int code, const char* msg);  // kge_abi.hip

namespace {

constexpr int kMaxWorld = 64;  // one lane per rank in the plan's per-owner counts

// Block partition of entity rows over W ranks (distributed.shard_bounds): the first E % W ranks hold
// one extra row. Returns the owner of id, or -1 for an id outside [0, E) (no owner: scores 0).
struct Owners {
    int64_t E, split;
    int W, extra;
    int64_t base;
    __device__ __forceinline__ int of(int64_t id) const {
        if (id < 0 || id >= E) return -1;
        if (id < split) return (int)(id / (base + 1));
        return extra + (int)((id - split) / base);
    }
};

Owners make_owners(int64_t E, int W) {
    Owners o;
    o.E = E;
    o.W = W;
    o.base = E / W;
    o.extra = (int)(E % W);
    o.split = (int64_t)o.extra * (o.base + 1);
    return o;
}

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
// positive) owned by rank o; qown[c * Bg + g] = owner of the row's query entity of column c.
__global__ __launch_bounds__(kBlock) void plan_count_kernel(const int64_t* __restrict__ pos,
                                                            const int64_t* __restrict__ neg, int64_t neg_ld,
                                                            int64_t Bg, int64_t N, Owners own, int ncol, int qc0,
                                                            int qc1, int pcol, int* __restrict__ cnt,
                                                            int* __restrict__ qown) {
    const int64_t g = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (g >= Bg) return;
    const int lane = threadIdx.x & 63;
    int acc = 0;  // lane o: candidates owned by rank o
    for (int64_t c0 = 0; c0 <= N; c0 += kWave) {
        const int o = own.of(cand_id(pos, neg, neg_ld, N, g, c0 + lane, pcol));
        for (int k = 0; k < own.W; ++k) {
            const int c = __popcll(__ballot(o == k));
            if (lane == k) acc += c;
        }
    }
    if (lane < own.W) cnt[(int64_t)lane * Bg + g] = acc;
    if (lane < ncol) qown[(int64_t)lane * Bg + g] = own.of(pos[g * 3 + (lane == 0 ? qc0 : qc1)]);
}

// Plan pass 2, one block per home h (blocks [0, W)) and per (query column c, chunk k) (blocks after):
//   home block:  hpre[o * Bg + g] = sum of cnt[o, g'] over the rows g' < g of home h (exclusive), and
//                tot[h * W + o] = the home's total for owner o;
//   query block: qslot[c * Bg + g] = rank of row g among the chunk's rows whose column-c query entity
//                has the same owner; qtot[(k * ncol + c) * W + o] = that owner's count in the chunk.
// 256 rows per step, one per thread: a wave prefix per owner, then the waves' totals through LDS.
__global__ __launch_bounds__(kBlock) void plan_scan_kernel(const int* __restrict__ cnt, const int* __restrict__ qown,
                                                           int64_t Bg, int64_t home_B, int64_t chunk_rows, int W,
                                                           int ncol, int* __restrict__ hpre, int* __restrict__ qslot,
                                                           int* __restrict__ tot, int* __restrict__ qtot) {
    __shared__ int wsum[kWavesPerBlock][kMaxWorld];
    __shared__ int carry[kMaxWorld];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const bool home_blk = (int)blockIdx.x < W;
    int64_t r0, rows;
    int c = 0, k = 0;
    if (home_blk) {
        r0 = (int64_t)blockIdx.x * home_B;
        rows = home_B;
    } else {
        const int i = blockIdx.x - W;
        k = i / ncol;
        c = i % ncol;
        r0 = (int64_t)k * chunk_rows;
        rows = chunk_rows;
    }
    if (tid < W) carry[tid] = 0;
    __syncthreads();
    for (int64_t t0 = 0; t0 < rows; t0 += kBlock) {
        const int64_t g = r0 + t0 + tid;
        const bool in = t0 + tid < rows;
        if (home_blk) {
            // one exclusive scan per owner column
            for (int o = 0; o < W; ++o) {
                const int v = in ? cnt[(int64_t)o * Bg + g] : 0;
                const int inc = wave_incl_scan(v, lane);
                if (lane == kWave - 1) wsum[w][o] = inc;
                __syncthreads();
                int before = carry[o];
                for (int j = 0; j < w; ++j) before += wsum[j][o];
                if (in) hpre[(int64_t)o * Bg + g] = before + inc - v;
                __syncthreads();
                if (tid == 0) {
                    int s = carry[o];
                    for (int j = 0; j < kWavesPerBlock; ++j) s += wsum[j][o];
                    carry[o] = s;
                }
                __syncthreads();
            }
        } else {
            // rank of the row among the chunk's rows with the same query owner
            const int o = in ? qown[(int64_t)c * Bg + g] : -1;
            int rank_w = 0;
            for (int q = 0; q < W; ++q) {
                const uint64_t m = __ballot(o == q);
                if (o == q) rank_w = lanes_below(m);
                if (lane == 0) wsum[w][q] = __popcll(m);
            }
            __syncthreads();
            if (o >= 0) {
                int before = carry[o];
                for (int j = 0; j < w; ++j) before += wsum[j][o];
                qslot[(int64_t)c * Bg + g] = before + rank_w;
            } else if (in) {
                qslot[(int64_t)c * Bg + g] = -1;
            }
            __syncthreads();
            if (tid < W) {
                int s = carry[tid];
                for (int j = 0; j < kWavesPerBlock; ++j) s += wsum[j][tid];
                carry[tid] = s;
            }
            __syncthreads();
        }
    }
    if (tid < W) {
        if (home_blk)
            tot[(int64_t)blockIdx.x * W + tid] = carry[tid];
        else
            qtot[((int64_t)k * ncol + c) * W + tid] = carry[tid];
    }
}

// Sender side of the query exchange, one wave per (column c, chunk row i). Owner o's rows of chunk k go
// to every rank (an all-to-all whose W pieces are the same block: NCCL has no all-gather of unequal
// sizes): piece = [column 0 rows | column 1 rows] in slot order, per = sum_c qtot[k, c, me] rows, written W
// times into send [W, per, width]. The all-to-all output holds the owners' pieces in rank order, so the row
// holding (owner o, column c, slot) is roff[o] + (c ? qtot[k, 0, o] : 0) + slot, roff[o] = sum over o' < o
// of the pieces: qidx[c * rows + i] (-1 without an owner).
__global__ __launch_bounds__(kBlock) void gather_queries_kernel(const float* __restrict__ shard, int64_t shard_rows,
                                                                int64_t ld, int64_t lo, const int64_t* __restrict__ pos,
                                                                int64_t Bg, int64_t row0, int64_t rows, int ncol,
                                                                int qc0, int qc1, const int* __restrict__ qown,
                                                                const int* __restrict__ qslot,
                                                                const int* __restrict__ qtot, int W, int rank,
                                                                int64_t width, float* __restrict__ send,
                                                                int64_t* __restrict__ qidx, int vec4) {
    const int64_t t = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (t >= (int64_t)ncol * rows) return;
    const int lane = threadIdx.x & 63;
    const int c = (int)(t / rows);
    const int64_t i = t - (int64_t)c * rows, g = row0 + i;
    const int o = qown[(int64_t)c * Bg + g];
    const int64_t s = qslot[(int64_t)c * Bg + g];
    // lane l < W: rank l's piece size; exclusive prefix = where its piece starts
    int piece = 0, col0 = 0;
    if (lane < W) {
        col0 = qtot[lane];
        piece = col0 + (ncol > 1 ? qtot[W + lane] : 0);
    }
    const int roff = wave_incl_scan(piece, lane) - piece;
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
// without an owner score 0. Writes scores [B, N], the positive's raw score and logsigmoid, and (NR > 0)
// the row's self-adversarial reduction from the registers it filled, in row_reduce's order.
template <int NR>
__global__ __launch_bounds__(kBlock) void shard_finish_kernel(const float* __restrict__ recv, const int* __restrict__ tot,
                                                              const int* __restrict__ hpre,
                                                              const int64_t* __restrict__ pos,
                                                              const int64_t* __restrict__ neg, int64_t neg_ld,
                                                              int64_t Bg, int64_t B, int64_t N, Owners own, int h,
                                                              int pcol, float T, int adversarial,
                                                              float* __restrict__ scores,
                                                              int64_t ns_ld, float* __restrict__ out_neg,
                                                              float* __restrict__ pos_raw, float* __restrict__ pos_ls) {
    const int64_t b = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (b >= B) return;
    const int lane = threadIdx.x & 63;
    const int64_t g = (int64_t)h * B + b;
    const int W = own.W;
    const int t = lane < W ? tot[(int64_t)h * W + lane] : 0;
    const int base = (wave_incl_scan(t, lane) - t) + (lane < W ? hpre[(int64_t)lane * Bg + g] : 0);
    int seen = 0;  // lane o: candidates of this row owned by rank o met so far
    float v[NR > 0 ? NR : 1];
    int k = 0;
    for (int64_t c0 = 0; c0 <= N; c0 += kWave, ++k) {
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
        if constexpr (NR > 0) {
#pragma unroll
            for (int j = 0; j < NR; ++j)
                if (j == k) v[j] = n < N ? s : 0.f;
        }
    }
    if constexpr (NR > 0) {
        const float r = row_reduce_vals<NR>(v, N, T, adversarial, lane);
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
                   int world, int chunks, int mode, int flags, int* cnt, int* hpre, int* qown, int* qslot,
                   int* summary, void* stream) {
    int rc = check_world(Bg, world, nentity);
    if (rc) return rc;
    if (mode != KGE_HEAD_BATCH && mode != KGE_TAIL_BATCH)
        return set_error(KGE_EINVAL, "kge_shard_plan: mode must be 0 (head-batch) or 1 (tail-batch)");
    if (N < 0 || chunks < 1 || world % chunks) return set_error(KGE_EINVAL, "kge_shard_plan: chunks must divide world");
    if (Bg == 0) return set_error(0, "");
    if (!pos || (N > 0 && !neg) || !cnt || !hpre || !qown || !qslot || !summary)
        return set_error(KGE_EINVAL, "kge_shard_plan: null pointer");
    int qc0, qc1, pcol;
    const int ncol = query_cols(mode, flags, qc0, qc1, pcol);
    const Owners own = make_owners(nentity, world);
    const hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(plan_count_kernel, dim3((unsigned)((Bg + kWavesPerBlock - 1) / kWavesPerBlock)), dim3(kBlock), 0,
                       st, pos, neg, neg_ld, Bg, N, own, ncol, qc0, qc1, pcol, cnt, qown);
    rc = launched("kge_shard_plan counts");
    if (rc) return rc;
    const int64_t home_B = Bg / world, chunk_rows = Bg / chunks;
    hipLaunchKernelGGL(plan_scan_kernel, dim3((unsigned)(world + chunks * ncol)), dim3(kBlock), 0, st, cnt, qown, Bg,
                       home_B, chunk_rows, world, ncol, hpre, qslot, summary, summary + (int64_t)world * world);
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
    if (Bg < 0 || chunks < 1 || Bg % chunks || chunk < 0 || chunk >= chunks || width <= 0 || shard_rows < 0)
        return set_error(KGE_EINVAL, "kge_shard_gather_queries: bad shape");
    if (Bg == 0) return set_error(0, "");
    if (!shard || !pos || !qown || !qslot || !summary || !qidx)
        return set_error(KGE_EINVAL, "kge_shard_gather_queries: null pointer");
    int qc0, qc1, pcol;
    const int ncol = query_cols(mode, flags, qc0, qc1, pcol);
    const int64_t rows = Bg / chunks;
    const int* qtot = summary + (int64_t)world * world + (int64_t)chunk * ncol * world;
    const int vec4 = (width % 4 == 0 && ld % 4 == 0 && ((uintptr_t)shard % 16) == 0 && ((uintptr_t)send % 16) == 0);
    const int64_t waves = ncol * rows;
    hipLaunchKernelGGL(gather_queries_kernel, dim3((unsigned)((waves + kWavesPerBlock - 1) / kWavesPerBlock)),
                       dim3(kBlock), 0, (hipStream_t)stream, shard, shard_rows, ld, shard_lo, pos, Bg, chunk * rows,
                       rows, ncol, qc0, qc1, qown, qslot, qtot, world, rank, width, send, qidx, vec4);
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
    // the row's positive is column N: N + 1 columns cover ceil((N + 1) / 64) register slots
    if (N + 1 <= 4 * kWave)
        hipLaunchKernelGGL(shard_finish_kernel<4>, grid, dim3(kBlock), 0, st, recv, tot, hpre, pos, neg, neg_ld, Bg, B,
                           N, own, home, pcol, temperature, adversarial, scores, ns_ld, out_neg, pos_scores, out_pos);
    else if (N + 1 <= 17 * kWave && N <= 16 * kWave)
        hipLaunchKernelGGL(shard_finish_kernel<17>, grid, dim3(kBlock), 0, st, recv, tot, hpre, pos, neg, neg_ld, Bg,
                           B, N, own, home, pcol, temperature, adversarial, scores, ns_ld, out_neg, pos_scores, out_pos);
    else {
        hipLaunchKernelGGL(shard_finish_kernel<0>, grid, dim3(kBlock), 0, st, recv, tot, hpre, pos, neg, neg_ld, Bg, B,
                           N, own, home, pcol, temperature, adversarial, scores, ns_ld, out_neg, pos_scores, out_pos);
        rc = launched("kge_shard_finish scatter");
        if (rc) return rc;
        hipLaunchKernelGGL(shard_rows_reduce_kernel, grid, dim3(kBlock), 0, st, scores, ns_ld, B, N, temperature,
                           adversarial, out_neg);
    }
    return launched("kge_shard_finish");
}

}  // extern "C"
