// kge_transparse.hip — TranSparse score function on the fp32 matrix cores,
// forward and deterministic backward.
//
// Reference: tensorflow_codes/model.py:226-235 with its call sites :139-142 (single), :161-164
// (head-batch), :187-190 (tail-batch) and the tables of :96-106:
//   M_r     = mask[r] * W[r]                        ([d, d], mask is a fixed 0/1 pattern)
//   p_head  = normalize(head @ M_r)                 (no epsilon, Q7)
//   p_tail  = normalize(head @ M_r)                 (Q9: computed from the HEAD, tail unused)
//   rel     = normalize(relation)
//   score   = gamma - || p_head * rel - p_tail ||_1 = gamma - sum_j |p_j c_j| / P,
//             P = ||p||, u = r / ||r||, c = u - 1
// Shapes follow the reference: head-batch head = E[neg] -> [B, N]; single and tail-batch head = E[pos_h]
// -> [B, 1] (Q9 makes the tail-batch score independent of the negatives).
//
// A "row" is one head vector to project. Two row sources share every kernel:
//   * per batch row  (head-batch): block = (b, 128 negatives); all rows share relation pos[b,1];
//   * per relation   (single/tail): block = (r, 128-row chunk of the batch rows with pos[b,1] == r),
//     found by an ordered ballot scan of pos[:,1]; bucket r = nrel collects out-of-range relations
//     (zero rows -> NaN scores, like TF-GPU gather).
//
// Forward (ts_rows_kernel<TS_FWD>): P[128, d] = H . M_r on v_mfma_f32_32x32x2_f32, block tile 128 x 128
// over the column tiles (2 x 2 waves of 64 x 64, K chunks of 16 double-buffered through LDS, the mask
// product fused into the M_r tile load). P never leaves registers: each column tile folds into per-row
// sums of p^2 and |p c|; optional per-row stats (P^2, sum |p c|) are kept for the backward.
//
// Backward of the raw scores, with G = dL/ds of a row:
//   dL/dp_j = (G / P) (p_j * S / P^2 - sign(p_j c_j) c_j),   S = sum_j |p_j c_j|
//   dL/du_j = -sign(c_j) sum_rows (G / P) |p_j|   ->  dL/dr = (g_u - u (u . g_u)) / ||r||
//   dL/dh   = dL/dp . M_r^T,      dL/dW_r = mask_r * sum_rows h^T dL/dp
// Kernels: (1) ts_rows_kernel<TS_GP> recomputes P tiles and writes dL/dp rows plus per-block column
// partials of g_u; (2) ts_rows_kernel<TS_DH> = dL/dp . M_r^T -> dH rows; (3) ts_dw_kernel: per
// (relation, 128 x 128 tile of dW, K split) MFMA over the relation's rows (relation CSR built by
// ordered compaction), split partials reduced in order; (4) entity buckets (count, scan, scatter,
// rank-sort by row id) and a wave per entity adding its dH rows in row order; (5) ts_drel_kernel per
// relation adds the g_u partials in block order. Every output element is produced by one thread in a
// fixed order: the backward is bitwise deterministic. Gradients ACCUMULATE into d_ent, d_rel, d_W.
#include <math.h>

#include <string>

#include "kge_device.h"
#include "kge_scan.h"

namespace kge_impl {
int set_error(int code, const char* msg);  // kge_abi.hip

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int TBM = 128, TBN = 128, TBK = 32;
constexpr int NU = TBK / 8;  // float4 per thread per operand and K chunk
constexpr int TLD = TBN + 4;  // row pitch of images stored with 16-B (ds_write_b128) rows: 16-B aligned
// row pitch of images stored TRANSPOSED (lane l writes k-row 4 (l % 8) + c, column l / 8 with
// ds_write_b32): a pitch of 1 (mod 8) puts a half-wave's 32 dwords on 32 distinct banks (the old
// TBM + 4 gave 4-way conflicts on every transposed store)
constexpr int ALD = TBM + 1;
constexpr int kMaxTsDim = 8192;
enum TsOp { TS_FWD = 0, TS_GP = 1, TS_DH = 2 };

struct TsParams {
    const float* ent;
    int64_t nent, ent_ld;
    const float* rel;
    int64_t nrel, rel_ld;
    const float* W;     // [R, d, d]
    const float* mask;  // [R, d, d]
    const float* Mpre;  // [R, d, d] mask * W precomputed, or null (then the product is fused in the loads)
    const int64_t* pos;
    const int64_t* neg;
    int64_t neg_ld;
    int64_t B, N;  // N = rows per batch row (1 for the grouped source)
    int d;
    float gamma;
    float* out;
    int64_t out_ld;
    float2* stats;  // [B * N] (P^2, sum |p c|) per row, row id = b * N + n
    int nchunk;
    bool grouped;
    // backward
    const float* d_scores;
    int64_t d_ld;
    float* gp;    // [rows, d]  dL/dp
    float* dh;    // [rows, d]  dL/dh
    float* upart;  // [blocks, d] per-block column sums of (G / P) |p|
    const int* rcnt;   // [R + 1] rows (batch rows) per relation bucket
    const int* roff;   // [R + 2]
    const int* rlist;  // [B] batch rows grouped by relation, ascending within a relation
    float* d_ent;
    float* d_rel;
    float* d_W;
    float* pdw;  // [S, R, d, d] split partials (S > 1)
    int S, T;
    // ts_fwd_x3g_kernel's split form (kge_transparse_score_ex with a workspace): each block of a row chunk takes
    // one of `xsplit` column ranges and one of `ksplit` K ranges and writes its rows' raw projections there to
    // xk [ksplit][B][xk_ld]; ts_xk_finish_kernel adds the K ranges in order and reduces each row
    int xsplit, ksplit;
    float* xk;
    int64_t xk_ld;
    int form;  // kge_forms.transparse_form: 0 the library's, 1 the forward's operands split per fragment, 2 the
               // head-batch split-once kernel in the compiler's instruction order
    // kge_transparse_step_forward: the negative call's row reduction (model.py:168-171, row_reduce_fast) in the
    // head-batch kernels' epilogue when one block holds a whole row (out_neg), and the positive call's
    // logsigmoid (model.py:145) in the split form's finish (out_pos_ls)
    float* out_neg;
    float* out_pos_ls;
    float temperature;
    int adversarial;
    // head-batch with a workspace: M_r (= W_r * mask_r) split once per call into three bf16 planes per relation,
    // [r][plane][K / 16][mp_cols][16] (ts_mplanes_kernel), staged by ts_fwd_x3s_kernel<.., true> with no conversion
    __bf16* mplanes;
    int mp_cols, mp_nk;
};

__device__ __forceinline__ int64_t row_entity(const TsParams& p, int64_t b, int64_t n) {
    return p.grouped ? p.pos[b * 3] : p.neg[b * p.neg_ld + n];
}

template <int VEC>
__device__ __forceinline__ float4 ld4(const float* base, int64_t off, int lim) {
    // lim: number of valid elements starting at off (<= 0: none)
    if constexpr (VEC == 4) {
        return lim > 0 ? *reinterpret_cast<const float4*>(base + off) : make_float4(0.f, 0.f, 0.f, 0.f);
    } else {
        float4 v;
        v.x = lim > 0 ? base[off] : 0.f;
        v.y = lim > 1 ? base[off + 1] : 0.f;
        v.z = lim > 2 ? base[off + 2] : 0.f;
        v.w = lim > 3 ? base[off + 3] : 0.f;
        return v;
    }
}

__device__ __forceinline__ float4 mul4(float4 a, float4 b) {
    return make_float4(a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w);
}

// one K chunk of the 2 x 2-wave 128 x 128 MFMA tile from the LDS images (k-major)
__device__ __forceinline__ void mfma_chunk(const float (*As)[TLD], const float (*Bs)[TLD], int wm, int wn, int half,
                                           int col, f32x16 (&acc)[2][2]) {
#pragma unroll
    for (int s = 0; s < TBK / 2; ++s) {
        const int kk = 2 * s + half;
        float a[2], bv[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) a[i] = As[kk][wm * 64 + i * 32 + col];
#pragma unroll
        for (int j = 0; j < 2; ++j) bv[j] = Bs[kk][wn * 64 + j * 32 + col];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], bv[j], acc[i][j], 0, 0, 0);
    }
}

// C/D map of the 32 x 32 MFMA: row within the wave tile for (i, register r, half-wave)
__device__ __forceinline__ int acc_row(int wm, int i, int r, int half) {
    return wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
}

// The g-th batch row in (relation bucket, row) order (bucket nrel collects out-of-range relations), computed
// by the whole block: bucket counts in LDS, the bucket holding position g (one wave, running prefix), then an
// ordered ballot scan for the k-th row of that bucket. Every thread returns the same row.
constexpr int kTsSortMaxRel = 1023;
// Each block finds its batch row in (relation, row) order by scanning the whole batch: O(B) per block, O(B^2)
// per launch, so the sorted order is used up to this many batch rows (natural order beyond).
constexpr int64_t kTsSortMaxB = 8192;
__device__ int64_t ts_sorted_row(const TsParams& p, int64_t g, int* hist, int* wcnt, int* sel) {
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int nb = (int)p.nrel + 1;
    auto bucket = [&](int64_t bb) {
        const int64_t rr = p.pos[bb * 3 + 1];
        return (rr >= 0 && rr < p.nrel) ? (int)rr : (int)p.nrel;
    };
    for (int i = t; i < nb; i += kBlock) hist[i] = 0;
    __syncthreads();
    for (int64_t bb = t; bb < p.B; bb += kBlock) atomicAdd(&hist[bucket(bb)], 1);
    __syncthreads();
    if (wave == 0) {
        int run = 0;
        for (int base = 0; base < nb; base += kWave) {
            const int i = base + lane;
            const int c = i < nb ? hist[i] : 0;
            int incl = c;
#pragma unroll
            for (int o = 1; o < kWave; o <<= 1) {
                const int y = __shfl_up(incl, o, kWave);
                if (lane >= o) incl += y;
            }
            const int excl = run + incl - c;
            const uint64_t m = __ballot(i < nb && g >= excl && g < excl + c);
            if (m) {
                const int src = __builtin_ctzll(m);
                if (lane == src) {
                    sel[0] = i;
                    sel[1] = (int)(g - excl);
                }
                break;
            }
            run += __shfl(incl, kWave - 1, kWave);
        }
    }
    __syncthreads();
    const int want = sel[0], k = sel[1];
    int64_t seen = 0;
    for (int64_t s0 = 0; s0 < p.B; s0 += kBlock) {
        const int64_t bb = s0 + t;
        const bool m = bb < p.B && bucket(bb) == want;
        const uint64_t bal = __ballot(m);
        if (lane == 0) wcnt[wave] = __popcll(bal);
        __syncthreads();
        int before = 0, total = 0;
        for (int w = 0; w < kWavesPerBlock; ++w) {
            before += (w < wave) ? wcnt[w] : 0;
            total += wcnt[w];
        }
        if (m && seen + before + __popcll(bal & ((1ull << lane) - 1ull)) == k) sel[2] = (int)bb;
        seen += total;
        __syncthreads();
        if (seen > k) break;  // uniform
    }
    return sel[2];
}

// ---------------------------------------------------------------------------------------------
// Row-block kernel: forward scores (TS_FWD), dL/dp rows (TS_GP) or dL/dh rows (TS_DH).
// ---------------------------------------------------------------------------------------------
template <int OP, int VEC, bool X3 = false>
__global__ __attribute__((amdgpu_flat_work_group_size(1, kBlock), amdgpu_waves_per_eu(X3 ? 2 : 1))) void
ts_rows_kernel(TsParams p) {
    static_assert(!X3 || (OP == TS_FWD && VEC == 4), "the bf16x3 form is the forward with float4 rows");
    __shared__ const float* rowp[TBM];
    __shared__ int rb[TBM], rn[TBM];  // (b, n) of each row; rb = -1 for padding rows
    __shared__ float2 red[TBM];
    __shared__ float colred[kWavesPerBlock][TBN];
    __shared__ float sa[TBM], sbv[TBM];
    __shared__ float wsum[kWavesPerBlock];
    __shared__ int wcnt[kWavesPerBlock];
    __shared__ int s_rows;
    __shared__ int hist[OP == TS_FWD ? kTsSortMaxRel + 1 : 1];
    __shared__ int sel[3];
    extern __shared__ float cs[];  // u - 1, d floats

    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int half = lane >> 5, col = lane & 31;
    const int d = p.d;
    const int64_t blk = blockIdx.x;
    const int64_t grp = blk / p.nchunk;
    const int chunk = (int)(blk % p.nchunk);

    // ---- rows of this block + its relation -----------------------------------------------------
    int64_t r;
    if (!p.grouped) {
        int64_t b = grp;
        int ch = chunk;
        if constexpr (OP == TS_FWD) {
            if (p.nrel <= kTsSortMaxRel && p.B <= kTsSortMaxB) {
                // Relation-sorted order: blocks i and i + 8 share an XCD, each XCD takes a contiguous run of ranks,
                // and rank k is the k-th batch row in (relation, row) order, so an XCD works through one or two
                // relations at a time and their M_r tiles (1 MB at d = 500) stay in its L2 (scripts/ts_rel_probe.py:
                // rows sorted by relation run 0.88x the time of random relations). Outputs go to (b, n) as before.
                const int64_t nblk = p.B * p.nchunk, q8 = nblk / 8, r8 = nblk % 8, x = blk % 8;
                const int64_t rank = (x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8) + blk / 8;
                ch = (int)(rank % p.nchunk);
                b = ts_sorted_row(p, rank / p.nchunk, hist, wcnt, sel);
            }
        }
        r = p.pos[b * 3 + 1];
        const int64_t n0 = (int64_t)ch * TBM;
        const int nrows = (int)min<int64_t>(TBM, p.N - n0);
        if (t < TBM) {
            rb[t] = t < nrows ? (int)b : -1;
            rn[t] = (int)(n0 + t);
        }
        if (t == 0) s_rows = nrows;
    } else {
        r = grp;  // == nrel: the out-of-range bucket
        const int64_t skip = (int64_t)chunk * TBM;
        int64_t seen = 0;
        if (t < TBM) {
            rb[t] = -1;
            rn[t] = 0;
        }
        for (int64_t s = 0; s < p.B; s += kBlock) {
            const int64_t b = s + t;
            bool m = false;
            if (b < p.B) {
                const int64_t rr = p.pos[b * 3 + 1];
                m = (r < p.nrel) ? (rr == r) : !(rr >= 0 && rr < p.nrel);
            }
            const uint64_t bal = __ballot(m);
            if (lane == 0) wcnt[wave] = __popcll(bal);
            __syncthreads();
            int before = 0, total = 0;
            for (int w = 0; w < kWavesPerBlock; ++w) {
                before += (w < wave) ? wcnt[w] : 0;
                total += wcnt[w];
            }
            if (m) {
                const int64_t k = seen + before + __popcll(bal & ((1ull << lane) - 1ull)) - skip;
                if (k >= 0 && k < TBM) rb[k] = (int)b;
            }
            seen += total;
            __syncthreads();
            if (seen >= skip + TBM) break;
        }
        const int64_t nrows = min<int64_t>(TBM, seen - skip);
        if (nrows <= 0) return;  // uniform: every thread computed the same `seen`
        if (t == 0) s_rows = (int)nrows;
    }
    __syncthreads();
    const bool rok = r >= 0 && r < p.nrel;
    if (t < TBM) {
        const float* rp = nullptr;
        float a = 0.f, bsc = 0.f;
        if (rb[t] >= 0) {
            const int64_t b = rb[t], n = rn[t];
            const int64_t row = b * p.N + n;
            if constexpr (OP == TS_DH) {
                rp = p.gp + row * d;
            } else {
                const int64_t id = row_entity(p, b, n);
                if (id >= 0 && id < p.nent) rp = p.ent + id * p.ent_ld;
            }
            if constexpr (OP == TS_GP) {
                const float2 st = p.stats[row];
                const float P = sqrtf(st.x);
                a = p.d_scores[b * p.d_ld + (p.grouped ? 0 : n)] / P;
                bsc = st.y / (P * P);
            }
        }
        rowp[t] = rp;
        sa[t] = a;
        sbv[t] = bsc;
    }

    // ---- u - 1 for the relation row ------------------------------------------------------------
    if constexpr (OP != TS_DH) {
        float ss = 0.f;
        for (int j = t; j < d; j += kBlock) {
            const float v = rok ? p.rel[r * p.rel_ld + j] : 0.f;
            cs[j] = v;
            ss += v * v;
        }
        for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o, kWave);
        if (lane == 0) wsum[wave] = ss;
        __syncthreads();
        const float rnorm = sqrtf(wsum[0] + wsum[1] + wsum[2] + wsum[3]);
        for (int j = t; j < d; j += kBlock) cs[j] = cs[j] / rnorm - 1.f;
    }
    const float* Wr = rok ? (p.Mpre ? p.Mpre : p.W) + r * (int64_t)d * d : nullptr;
    const float* Mr = (rok && !p.Mpre) ? p.mask + r * (int64_t)d * d : nullptr;
    __syncthreads();

    // wave w: rows [32 w, 32 w + 32) x all 128 columns of the tile (four 32 x 32 MFMA accumulators);
    // C/D map: row = 32 w + (r & 3) + 8 (r >> 2) + 4 (lane >> 5), column = 32 j + (lane & 31)
    f32x16 acc[4];
    float sq[16], ab[16];
#pragma unroll
    for (int r2 = 0; r2 < 16; ++r2) {
        sq[r2] = 0.f;
        ab[r2] = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j][r2] = 0.f;
    }
    auto row_of = [&](int r2) { return wave * 32 + (r2 & 3) + 8 * (r2 >> 2) + 4 * half; };

    const int nrows = s_rows;
    const int nk = (d + TBK - 1) / TBK, nct = (d + TBN - 1) / TBN;
    const int iters = nk * nct;
    // folds a finished column tile into the per-row sums of p^2 and |p c| (forward)
    auto fold = [&](int ct) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int cg = ct * TBN + j * 32 + col;
            const float c = cg < d ? cs[cg] : 0.f;
#pragma unroll
            for (int r2 = 0; r2 < 16; ++r2) {
                const float v = acc[j][r2];
                sq[r2] = fmaf(v, v, sq[r2]);
                ab[r2] += fabsf(v * c);
                acc[j][r2] = 0.f;
            }
        }
    };
    if constexpr (X3) {
        // ---- bf16x3 forward: P = H . M_r at fp32 accuracy on v_mfma_f32_32x32x16_bf16 ------------------
        // Each fp32 fragment value is split in registers into three bf16 terms (split3_bf16) and the six
        // products with i + j <= 2 accumulate in fp32 (kge_gemm_nt_bf16x3's numerics). LDS images hold the
        // tiles with k contiguous per row / per column (rows of 34 dwords: a fragment read, ds_read_b64 x 4 of
        // 32 rows, hits 32 distinct bank pairs): A = the 128 gathered rows [row][k]; B = the M_r tile stored
        // transposed [col][k] (lane l stages k = l & 31, so the transposing ds_write_b32 are conflict-free).
        constexpr int XLD = 34;
        __shared__ __attribute__((aligned(16))) float Ax[2][TBM * XLD];
        __shared__ __attribute__((aligned(16))) float Bx[2][TBN * XLD];
        const float* arow[NU];
    #pragma unroll
        for (int u = 0; u < NU; ++u) arow[u] = rowp[(t + kBlock * u) >> 3];
        float4 ra[NU], rbv[NU];
        auto gload = [&](int ct, int k0) {
    #pragma unroll
            for (int u = 0; u < NU; ++u) {
                const int f = t + kBlock * u, ka = k0 + 4 * (f & 7);
                ra[u] = arow[u] ? ld4<4>(arow[u], ka, d - ka) : make_float4(0.f, 0.f, 0.f, 0.f);
                const int kb = k0 + (lane & 31), j = ct * TBN + 4 * ((lane >> 5) + 2 * (wave + 4 * u));
                if (Wr && kb < d) {
                    const int64_t off = (int64_t)kb * d + j;
                    rbv[u] = Mr ? mul4(ld4<4>(Wr, off, d - j), ld4<4>(Mr, off, d - j)) : ld4<4>(Wr, off, d - j);
                } else {
                    rbv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
                }
            }
        };
        auto sstore = [&](int buf) {
    #pragma unroll
            for (int u = 0; u < NU; ++u) {
                const int f = t + kBlock * u, o = (f >> 3) * XLD + 4 * (f & 7);
                *reinterpret_cast<float2*>(&Ax[buf][o]) = make_float2(ra[u].x, ra[u].y);
                *reinterpret_cast<float2*>(&Ax[buf][o + 2]) = make_float2(ra[u].z, ra[u].w);
                const int kb = lane & 31, cg = 4 * ((lane >> 5) + 2 * (wave + 4 * u));
                Bx[buf][(cg + 0) * XLD + kb] = rbv[u].x;
                Bx[buf][(cg + 1) * XLD + kb] = rbv[u].y;
                Bx[buf][(cg + 2) * XLD + kb] = rbv[u].z;
                Bx[buf][(cg + 3) * XLD + kb] = rbv[u].w;
            }
        };
        auto frag = [&](const float* base) {
            f32x8 v;
    #pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float2 x = *reinterpret_cast<const float2*>(base + 2 * q);
                v[2 * q] = x.x;
                v[2 * q + 1] = x.y;
            }
            return v;
        };
        gload(0, 0);
        sstore(0);
        __syncthreads();
        for (int it = 0; it < iters; ++it) {
            const int buf = it & 1;
            const int ct = it / nk, kc = it - ct * nk;
            if (it + 1 < iters) {
                const int ct1 = (it + 1) / nk;
                gload(ct1, ((it + 1) - ct1 * nk) * TBK);
            }
    #pragma unroll
            for (int s2 = 0; s2 < TBK / 16; ++s2) {
                const int ko = 16 * s2 + 8 * half;
                bf16x8 a[3], b[4][3];
                split3_bf16(frag(&Ax[buf][(wave * 32 + col) * XLD + ko]), a[0], a[1], a[2]);
    #pragma unroll
                for (int j = 0; j < 4; ++j) split3_bf16(frag(&Bx[buf][(j * 32 + col) * XLD + ko]), b[j][0], b[j][1], b[j][2]);
    #pragma unroll
                for (int q = 0; q < 6; ++q)
    #pragma unroll
                    for (int j = 0; j < 4; ++j)
                        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[kX3A[q]], b[j][kX3B[q]], acc[j], 0, 0, 0);
            }
            if (kc == nk - 1) fold(ct);
            if (it + 1 < iters) {
                sstore(buf ^ 1);
                __syncthreads();
            }
        }
    } else {
        // ---- staging --------------------------------------------------------------------------------
        constexpr int BLD = OP == TS_DH ? ALD : TLD;  // TS_DH stages M_r transposed like A
        __shared__ __attribute__((aligned(16))) float As[2][TBK][ALD];
        __shared__ __attribute__((aligned(16))) float Bs[2][TBK][BLD];
        // A (rows): 128 rows x TBK k, NU float4 per thread, transposed into As[k][row].
        // B: FWD/GP: M_r[k][col] row segments (natural k-major); DH: M_r[col][k] (transposed like A).
        // thread t, unit u: A row = (t >> 3) + 32 u, k offset (t & 7) * 4; B k row = (t >> 5) + 8 u, col (t & 31) * 4
        const int akq = (t & 7) * 4, bjq = (t & 31) * 4;
        const float* arow[NU];
    #pragma unroll
        for (int u = 0; u < NU; ++u) arow[u] = rowp[(t >> 3) + 32 * u];
        float4 ra[NU], rbv[NU];
        auto gload = [&](int ct, int k0) {
            const int ka = k0 + akq;
    #pragma unroll
            for (int u = 0; u < NU; ++u) {
                ra[u] = arow[u] ? ld4<VEC>(arow[u], ka, d - ka) : make_float4(0.f, 0.f, 0.f, 0.f);
                if constexpr (OP == TS_DH) {
                    const int c = ct * TBN + (t >> 3) + 32 * u;
                    if (Wr && c < d) {
                        const int64_t off = (int64_t)c * d + ka;
                        rbv[u] = Mr ? mul4(ld4<VEC>(Wr, off, d - ka), ld4<VEC>(Mr, off, d - ka)) : ld4<VEC>(Wr, off, d - ka);
                    } else {
                        rbv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
                    }
                } else {
                    const int kb = k0 + (t >> 5) + 8 * u, j = ct * TBN + bjq;
                    if (Wr && kb < d) {
                        const int64_t off = (int64_t)kb * d + j;
                        rbv[u] = Mr ? mul4(ld4<VEC>(Wr, off, d - j), ld4<VEC>(Mr, off, d - j)) : ld4<VEC>(Wr, off, d - j);
                    } else {
                        rbv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
                    }
                }
            }
        };
        auto sstore = [&](int buf) {
    #pragma unroll
            for (int u = 0; u < NU; ++u) {
                const int ar = (t >> 3) + 32 * u;
                As[buf][akq + 0][ar] = ra[u].x;
                As[buf][akq + 1][ar] = ra[u].y;
                As[buf][akq + 2][ar] = ra[u].z;
                As[buf][akq + 3][ar] = ra[u].w;
                if constexpr (OP == TS_DH) {
                    Bs[buf][akq + 0][ar] = rbv[u].x;
                    Bs[buf][akq + 1][ar] = rbv[u].y;
                    Bs[buf][akq + 2][ar] = rbv[u].z;
                    Bs[buf][akq + 3][ar] = rbv[u].w;
                } else {
                    *reinterpret_cast<float4*>(&Bs[buf][(t >> 5) + 8 * u][bjq]) = rbv[u];
                }
            }
        };

        gload(0, 0);
        sstore(0);
        __syncthreads();
        for (int it = 0; it < iters; ++it) {
            const int buf = it & 1;
            const int ct = it / nk, kc = it - ct * nk;
            if (it + 1 < iters) {
                const int ct1 = (it + 1) / nk;
                gload(ct1, ((it + 1) - ct1 * nk) * TBK);
            }
    #pragma unroll
            for (int s2 = 0; s2 < TBK / 2; ++s2) {
                const int kk = 2 * s2 + half;
                const float a = As[buf][kk][wave * 32 + col];
                float bv[4];
    #pragma unroll
                for (int j = 0; j < 4; ++j) bv[j] = Bs[buf][kk][j * 32 + col];
    #pragma unroll
                for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bv[j], acc[j], 0, 0, 0);
            }
            if (kc == nk - 1) {
                if constexpr (OP == TS_FWD) {
                    fold(ct);
                } else if constexpr (OP == TS_GP) {
    #pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int cg = ct * TBN + j * 32 + col;
                        const bool cin = cg < d;
                        const float c = cin ? cs[cg] : 0.f;
                        float up = 0.f;
    #pragma unroll
                        for (int r2 = 0; r2 < 16; ++r2) {
                            const int m = row_of(r2);
                            const float v = acc[j][r2];
                            const float a = sa[m];
                            if (cin && m < nrows)
                                p.gp[((int64_t)rb[m] * p.N + rn[m]) * d + cg] = a * (v * sbv[m] - sgnf(v * c) * c);
                            up += a * fabsf(v);
                            acc[j][r2] = 0.f;
                        }
                        up += __shfl_xor(up, 32, kWave);
                        if (half == 0) colred[wave][j * 32 + col] = up;
                    }
                    __syncthreads();
                    if (t < TBN && ct * TBN + t < d)
                        p.upart[blk * d + ct * TBN + t] = (colred[0][t] + colred[1][t]) + (colred[2][t] + colred[3][t]);
                } else {  // TS_DH
    #pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int cg = ct * TBN + j * 32 + col;
    #pragma unroll
                        for (int r2 = 0; r2 < 16; ++r2) {
                            const int m = row_of(r2);
                            if (cg < d && m < nrows) p.dh[((int64_t)rb[m] * p.N + rn[m]) * d + cg] = acc[j][r2];
                            acc[j][r2] = 0.f;
                        }
                    }
                }
            }
            if (it + 1 < iters) {
                sstore(buf ^ 1);
                __syncthreads();
            }
        }
    }

    if constexpr (OP == TS_FWD) {
        // row reductions: the 32 lanes of a half-wave hold the columns of the same rows
#pragma unroll
        for (int r2 = 0; r2 < 16; ++r2) {
            float a = sq[r2], b = ab[r2];
#pragma unroll
            for (int o = 16; o > 0; o >>= 1) {
                a += __shfl_xor(a, o, kWave);
                b += __shfl_xor(b, o, kWave);
            }
            if (col == 0) red[row_of(r2)] = make_float2(a, b);
        }
        __syncthreads();
        if (t < nrows) {
            const float2 x = red[t];
            const int64_t b = rb[t], n = rn[t];
            p.out[b * p.out_ld + n] = p.gamma - x.y / sqrtf(x.x);
            if (p.stats) p.stats[b * p.N + n] = x;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Head-batch forward, 256-row blocks (ts_fwd_x3_kernel; the bf16x3 numerics of ts_rows_kernel<TS_FWD, 4,
// true>). One block = one batch row's 256 negatives, which share M_r: each staged M_r chunk serves all 256
// rows (the 128-row kernel stages the 1 MB M_r twice per batch row and its rows once per 128-column tile).
//   * 8 waves, a 4 x 2 grid of 64-row x 128-column wave tiles (eight 32 x 32 accumulators, 128 AGPRs);
//     the block's 256 x 256 tile sweeps the columns in ceil(d / 256) super-tiles;
//   * K in chunks of 32, DOUBLE-buffered in LDS (2 x (256 + 256) x 34 dwords = 139 KB: one block per CU,
//     2 waves per SIMD): the next chunk is loaded into registers while this one's 96 MFMAs per wave run,
//     stored into the other buffer, and one barrier per chunk orders the two;
//   * each finished super-tile is folded into per-row sums of p^2 and |p c| right away (half-wave shuffles,
//     the two column waves added through LDS), so no per-row state lives in registers across super-tiles.
// ---------------------------------------------------------------------------------------------
constexpr int XBR = 256, XBC = 256, XLDB = 34, kXThreads = 512, kXWaves = kXThreads / kWave;
constexpr int kTsBigMaxDim = 3072;  // the dynamic u - 1 image (d floats) beside ~146 KB of static LDS

// ts_sorted_row for a block of NT threads: the g-th batch row in (relation bucket, row) order. O(B) per
// block (so O(B^2) per launch): used up to kTsSortMaxB batch rows.
template <int NT>
__device__ int64_t ts_sorted_row_nt(const TsParams& p, int64_t g, int* hist, int* wcnt, int* sel) {
    constexpr int NW = NT / kWave;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int nb = (int)p.nrel + 1;
    auto bucket = [&](int64_t bb) {
        const int64_t rr = p.pos[bb * 3 + 1];
        return (rr >= 0 && rr < p.nrel) ? (int)rr : (int)p.nrel;
    };
    for (int i = t; i < nb; i += NT) hist[i] = 0;
    __syncthreads();
    for (int64_t bb = t; bb < p.B; bb += NT) atomicAdd(&hist[bucket(bb)], 1);
    __syncthreads();
    if (wave == 0) {
        int run = 0;
        for (int base = 0; base < nb; base += kWave) {
            const int i = base + lane;
            const int c = i < nb ? hist[i] : 0;
            int incl = c;
#pragma unroll
            for (int o = 1; o < kWave; o <<= 1) {
                const int y = __shfl_up(incl, o, kWave);
                if (lane >= o) incl += y;
            }
            const int excl = run + incl - c;
            const uint64_t m = __ballot(i < nb && g >= excl && g < excl + c);
            if (m) {
                const int src = __builtin_ctzll(m);
                if (lane == src) {
                    sel[0] = i;
                    sel[1] = (int)(g - excl);
                }
                break;
            }
            run += __shfl(incl, kWave - 1, kWave);
        }
    }
    __syncthreads();
    const int want = sel[0], k = sel[1];
    int64_t seen = 0;
    for (int64_t s0 = 0; s0 < p.B; s0 += NT) {
        const int64_t bb = s0 + t;
        const bool m = bb < p.B && bucket(bb) == want;
        const uint64_t bal = __ballot(m);
        if (lane == 0) wcnt[wave] = __popcll(bal);
        __syncthreads();
        int before = 0, total = 0;
        for (int w = 0; w < NW; ++w) {
            before += (w < wave) ? wcnt[w] : 0;
            total += wcnt[w];
        }
        if (m && seen + before + __popcll(bal & ((1ull << lane) - 1ull)) == k) sel[2] = (int)bb;
        seen += total;
        __syncthreads();
        if (seen > k) break;  // uniform
    }
    return sel[2];
}

__global__ __attribute__((amdgpu_flat_work_group_size(1, kXThreads), amdgpu_waves_per_eu(2))) void
ts_fwd_x3_kernel(TsParams p) {
    __shared__ __attribute__((aligned(16))) float Ax[2][XBR * XLDB];
    __shared__ __attribute__((aligned(16))) float Bx[2][XBC * XLDB];
    __shared__ const float* rowp[XBR];
    __shared__ float2 red[2][XBR];
    __shared__ float wsum[kXWaves];
    __shared__ int wcnt[kXWaves];
    __shared__ int hist[kTsSortMaxRel + 1];
    __shared__ int sel[3];
    extern __shared__ float cs[];  // u - 1, d floats

    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int half = lane >> 5, col = lane & 31;
    const int wr = wave >> 1, wc = wave & 1;
    const int d = p.d;
    const int64_t blk = blockIdx.x;
    int64_t b = blk / p.nchunk;
    int ch = (int)(blk % p.nchunk);
    if (p.nrel <= kTsSortMaxRel && p.B <= kTsSortMaxB) {
        // relation-sorted order (ts_rows_kernel's): blocks i and i + 8 share an XCD, each XCD takes a contiguous
        // run of ranks, rank k = the k-th batch row in (relation, row) order: M_r stays in the XCD's L2
        const int64_t nblk = p.B * p.nchunk, q8 = nblk / 8, r8 = nblk % 8, x = blk % 8;
        const int64_t rank = (x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8) + blk / 8;
        ch = (int)(rank % p.nchunk);
        b = ts_sorted_row_nt<kXThreads>(p, rank / p.nchunk, hist, wcnt, sel);
    }
    const int64_t r = p.pos[b * 3 + 1];
    const bool rok = r >= 0 && r < p.nrel;
    const int64_t n0 = (int64_t)ch * XBR;
    const int nrows = (int)min<int64_t>(XBR, p.N - n0);
    if (t < XBR) {
        const float* rp = nullptr;
        if (t < nrows) {
            const int64_t id = p.neg[b * p.neg_ld + n0 + t];
            if (id >= 0 && id < p.nent) rp = p.ent + id * p.ent_ld;
        }
        rowp[t] = rp;
        red[0][t] = red[1][t] = make_float2(0.f, 0.f);
    }
    // u - 1 for the relation row
    {
        float ss = 0.f;
        for (int j = t; j < d; j += kXThreads) {
            const float v = rok ? p.rel[r * p.rel_ld + j] : 0.f;
            cs[j] = v;
            ss += v * v;
        }
        for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o, kWave);
        if (lane == 0) wsum[wave] = ss;
        __syncthreads();
        float tot = 0.f;
#pragma unroll
        for (int w = 0; w < kXWaves; ++w) tot += wsum[w];
        const float rnorm = sqrtf(tot);
        for (int j = t; j < d; j += kXThreads) cs[j] = cs[j] / rnorm - 1.f;
    }
    const float* Wr = rok ? (p.Mpre ? p.Mpre : p.W) + r * (int64_t)d * d : nullptr;
    const float* Mr = (rok && !p.Mpre) ? p.mask + r * (int64_t)d * d : nullptr;
    __syncthreads();

    // staging: thread t, unit u < 4: A row (f >> 3), k 4 (f & 7), f = t + 512 u; B k = lane & 31, columns
    // 4 ((lane >> 5) + 2 (wave + 8 u)) .. + 3 of the super-tile (transposed into Bx[col][k])
    const float* arow[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) arow[u] = rowp[(t + kXThreads * u) >> 3];
    float4 ra[4], rbv[4];
    const int nk = (d + TBK - 1) / TBK, nct = (d + XBC - 1) / XBC;
    auto gload = [&](int ct, int k0) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int f = t + kXThreads * u, ka = k0 + 4 * (f & 7);
            ra[u] = arow[u] ? ld4<4>(arow[u], ka, d - ka) : make_float4(0.f, 0.f, 0.f, 0.f);
            const int kb = k0 + (lane & 31), j = ct * XBC + 4 * ((lane >> 5) + 2 * (wave + kXWaves * u));
            if (Wr && kb < d) {
                const int64_t off = (int64_t)kb * d + j;
                rbv[u] = Mr ? mul4(ld4<4>(Wr, off, d - j), ld4<4>(Mr, off, d - j)) : ld4<4>(Wr, off, d - j);
            } else {
                rbv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
    };
    auto sstore = [&](int buf) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int f = t + kXThreads * u, o = (f >> 3) * XLDB + 4 * (f & 7);
            *reinterpret_cast<float2*>(&Ax[buf][o]) = make_float2(ra[u].x, ra[u].y);
            *reinterpret_cast<float2*>(&Ax[buf][o + 2]) = make_float2(ra[u].z, ra[u].w);
            const int kb = lane & 31, cg = 4 * ((lane >> 5) + 2 * (wave + kXWaves * u));
            Bx[buf][(cg + 0) * XLDB + kb] = rbv[u].x;
            Bx[buf][(cg + 1) * XLDB + kb] = rbv[u].y;
            Bx[buf][(cg + 2) * XLDB + kb] = rbv[u].z;
            Bx[buf][(cg + 3) * XLDB + kb] = rbv[u].w;
        }
    };
    auto frag = [&](const float* base) {
        f32x8 v;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float2 x = *reinterpret_cast<const float2*>(base + 2 * q);
            v[2 * q] = x.x;
            v[2 * q + 1] = x.y;
        }
        return v;
    };
    for (int ct = 0; ct < nct; ++ct) {
        f32x16 acc[2][4];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int r2 = 0; r2 < 16; ++r2) acc[i][j][r2] = 0.f;
        gload(ct, 0);
        sstore(0);
        __syncthreads();
        for (int kc = 0; kc < nk; ++kc) {
            const int buf = kc & 1;
            if (kc + 1 < nk) gload(ct, (kc + 1) * TBK);
#pragma unroll
            for (int s2 = 0; s2 < TBK / 16; ++s2) {
                const int ko = 16 * s2 + 8 * half;
                bf16x8 a[2][3];
#pragma unroll
                for (int i = 0; i < 2; ++i)
                    split3_bf16(frag(&Ax[buf][(wr * 64 + i * 32 + col) * XLDB + ko]), a[i][0], a[i][1], a[i][2]);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    bf16x8 bb[3];
                    split3_bf16(frag(&Bx[buf][(wc * 128 + j * 32 + col) * XLDB + ko]), bb[0], bb[1], bb[2]);
#pragma unroll
                    for (int q = 0; q < 6; ++q)
#pragma unroll
                        for (int i = 0; i < 2; ++i)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][kX3A[q]], bb[kX3B[q]], acc[i][j], 0,
                                                                               0, 0);
                }
            }
            if (kc + 1 < nk) sstore(buf ^ 1);
            __syncthreads();
        }
        // fold the super-tile: per row sum over this wave's 128 columns of p^2 and |p c|
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int r2 = 0; r2 < 16; ++r2) {
                float sq = 0.f, ab = 0.f;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int cg = ct * XBC + wc * 128 + j * 32 + col;
                    const float c = cg < d ? cs[cg] : 0.f;
                    const float v = acc[i][j][r2];
                    sq = fmaf(v, v, sq);
                    ab += fabsf(v * c);
                }
#pragma unroll
                for (int o = 16; o > 0; o >>= 1) {
                    sq += __shfl_xor(sq, o, kWave);
                    ab += __shfl_xor(ab, o, kWave);
                }
                if (col == 0) {
                    const int row = wr * 64 + i * 32 + (r2 & 3) + 8 * (r2 >> 2) + 4 * half;
                    float2& x = red[wc][row];
                    x = make_float2(x.x + sq, x.y + ab);
                }
            }
    }
    __syncthreads();
    if (t < nrows) {
        const float2 x0 = red[0][t], x1 = red[1][t];
        const float2 x = make_float2(x0.x + x1.x, x0.y + x1.y);
        const int64_t n = n0 + t;
        p.out[b * p.out_ld + n] = p.gamma - x.y / sqrtf(x.x);
        if (p.stats) p.stats[b * p.N + n] = x;
    }
    if (p.out_neg) {  // the block holds the whole row (the launcher sets out_neg only then): its reduction
        __syncthreads();
        if (wave == 0) {
            const float rr = row_reduce_fast(p.out + b * p.out_ld, p.N, p.temperature, p.adversarial, lane);
            if (lane == 0) p.out_neg[b] = rr;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Head-batch forward with the operands split ONCE (ts_fwd_x3s_kernel): ts_fwd_x3_kernel's block tile,
// products and accumulation order (so bitwise its scores), restaged so that the MFMA loop does no VALU work:
//   * K in chunks of 16 (one 32x32x16 k-step). The staging threads load a chunk of the rows (A: 256 x 16)
//     and of M_r (B: 16 x 256) with raw buffer loads whose hardware range check zero-fills everything past
//     d and every invalid row (no branches, no waits inside the loop), split each fp32 value ONCE into its
//     three bf16 terms (split3_bf16's arithmetic) and store three bf16 planes per operand; ts_fwd_x3_kernel
//     split every fragment in the MFMA loop, A twice and B four times over, and its branchy loads compiled
//     to a vmcnt(0) wait per chunk plus 32 spilled VGPRs;
//   * planes [row or column][16 k] bf16 (32-B rows) with the 16-B halves swapped on every other group of
//     8 rows: the MFMA operand reads (ds_read_b128, one per fragment and plane) and the staging stores are
//     bank-conflict-free (B's transposing 4-B stores 2-way, which costs a ds_write_b32 nothing);
//   * two LDS stages (96 KB) and two register sets: chunk g + 2 is loaded while chunk g is multiplied and
//     chunk g + 1 stored, one barrier per chunk.
// The 48 MFMAs of a chunk per wave read 18 ds_read_b128 (2 A fragments x 3 planes, 4 B fragments x 3).
// SCHED (the default, round 6): the staging of chunk g + 1 (~110 VALU of splitting, 14-18 LDS stores) and the
// loads of chunk g + 3 are placed among the chunk's last 36 MFMAs (the eval GEMM's sched-group recipe); the
// compiler's own order (form 2) issues all 48 MFMAs first and then the staging, with both waves of a SIMD in the
// same phase, so the matrix pipe idles through that tail every chunk. The same instructions either way: bitwise.
// ---------------------------------------------------------------------------------------------
constexpr int kXsPlane = XBR * 16 * 2;  // bytes of one bf16 plane chunk (256 rows x 16 k)
constexpr int kXsStage = 6 * kXsPlane;  // A planes then B planes
constexpr int kXsMaxDim = 1024;         // u - 1 image beside the two stages
constexpr uint32_t kXsOOB = 0xFFFFFFF0u;

__device__ __forceinline__ int xs_off(int row, int h) { return row * 32 + ((h ^ ((row >> 3) & 1)) << 4); }

typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

// split3_bf16's arithmetic on 4 and 2 values (elementwise the same operations: the same three terms)
__device__ __forceinline__ void split3_x4(f32x4_t v, bf16x4_t& a0, bf16x4_t& a1, bf16x4_t& a2) {
    a0 = __builtin_convertvector(v, bf16x4_t);
    const f32x4_t r1 = v - __builtin_convertvector(a0, f32x4_t);
    a1 = __builtin_convertvector(r1, bf16x4_t);
    a2 = __builtin_convertvector(r1 - __builtin_convertvector(a1, f32x4_t), bf16x4_t);
}

struct XsRegs {
    float4 a[2], b[2], m[2];
    int4 bp[3];  // B from the pre-split planes (BPL)
};

// Knock-out builds for the step-cost breakdown probe (scripts/x3p_knockout_probe.py; wrong results by design,
// never the library's build), applied to the compiler-order step (transparse_form 2): bit 0 drops the per-chunk
// barrier, bit 1 the LDS stores (and the splits), bit 2 the global loads.
#ifndef KGE_TS_KO
#define KGE_TS_KO 0
#endif

template <bool MASK, bool BPL, bool SCHED>
__global__ __attribute__((amdgpu_flat_work_group_size(1, kXThreads), amdgpu_waves_per_eu(2))) void
ts_fwd_x3s_kernel(TsParams p) {
    extern __shared__ __attribute__((aligned(16))) unsigned char xs_smem[];  // 2 stages, then u - 1 (d floats)
    __shared__ int rowid[XBR];
    __shared__ float2 red[2][XBR];
    __shared__ float wsum[kXWaves];
    __shared__ int wcnt[kXWaves];
    __shared__ int hist[kTsSortMaxRel + 1];
    __shared__ int sel[3];
    float* cs = reinterpret_cast<float*>(xs_smem + 2 * kXsStage);

    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int half = lane >> 5, col = lane & 31;
    const int wr = wave >> 1, wc = wave & 1;
    const int d = p.d;
    const int64_t blk = blockIdx.x;
    int64_t b = blk / p.nchunk;
    int ch = (int)(blk % p.nchunk);
    if (p.nrel <= kTsSortMaxRel && p.B <= kTsSortMaxB) {  // ts_fwd_x3_kernel's relation-sorted order
        const int64_t nblk = p.B * p.nchunk, q8 = nblk / 8, r8 = nblk % 8, x = blk % 8;
        const int64_t rank = (x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8) + blk / 8;
        ch = (int)(rank % p.nchunk);
        b = ts_sorted_row_nt<kXThreads>(p, rank / p.nchunk, hist, wcnt, sel);
    }
    const int64_t r = p.pos[b * 3 + 1];
    const bool rok = r >= 0 && r < p.nrel;
    const int64_t n0 = (int64_t)ch * XBR;
    const int nrows = (int)min<int64_t>(XBR, p.N - n0);
    if (t < XBR) {
        int id = -1;
        if (t < nrows) {
            const int64_t e = p.neg[b * p.neg_ld + n0 + t];
            if (e >= 0 && e < p.nent) id = (int)e;
        }
        rowid[t] = id;
        red[0][t] = red[1][t] = make_float2(0.f, 0.f);
    }
    {  // u - 1 for the relation row (ts_fwd_x3_kernel's arithmetic)
        float ss = 0.f;
        for (int j = t; j < d; j += kXThreads) {
            const float v = rok ? p.rel[r * p.rel_ld + j] : 0.f;
            cs[j] = v;
            ss += v * v;
        }
        for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o, kWave);
        if (lane == 0) wsum[wave] = ss;
        __syncthreads();
        float tot = 0.f;
#pragma unroll
        for (int w = 0; w < kXWaves; ++w) tot += wsum[w];
        const float rnorm = sqrtf(tot);
        for (int j = t; j < d; j += kXThreads) cs[j] = cs[j] / rnorm - 1.f;
    }
    __syncthreads();
    // buffer descriptors: the entity table (rows by per-lane offset) and the relation's d x d matrix
    const rsrc_t ra = make_rsrc(p.ent, (uint32_t)(p.nent * p.ent_ld * 4));
    const float* Wr = rok ? (MASK ? p.W : p.Mpre) + r * (int64_t)d * d : p.W;
    const uint32_t mbytes = rok ? (uint32_t)((int64_t)d * d * 4) : 0u;
    const rsrc_t rw = make_rsrc(Wr, mbytes);
    constexpr bool fuse_mask = MASK;  // M_r = W_r * mask_r formed at staging (else p.Mpre holds the products)
    const rsrc_t rm = make_rsrc(fuse_mask && rok ? p.mask + r * (int64_t)d * d : p.W, fuse_mask ? mbytes : 0u);
    // BPL: the relation's three planes; thread t stages column t >> 1, k half t & 1 of each (16 B, x3p's pattern)
    const int64_t mp_plane = (int64_t)p.mp_nk * p.mp_cols * 16;  // elements of one plane of one relation
    const rsrc_t rp = make_rsrc(BPL && rok ? p.mplanes + r * 3 * mp_plane : nullptr,
                                BPL && rok ? (uint32_t)(3 * mp_plane * 2) : 0u);
    const int spc = t >> 1, sph = t & 1;
    // this thread's staging slots: A rows (t >> 2) + 128 u, k quad t & 3; B k pair t & 7 (+u), columns 4 (t >> 3)
    int aid[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) aid[u] = rowid[(t >> 2) + 128 * u];
    const int aq = t & 3, bkp = t & 7, bjq = t >> 3;
    const int nk = (d + 15) / 16, nct = (d + XBC - 1) / XBC, T = nk * nct;

    // every load is issued unconditionally (a chunk past the end reads zeros through the out-of-range offset):
    // with no branch around a load the wait before a store to LDS counts exactly the younger set's loads
    auto gload = [&](XsRegs& R, int g) {
        const bool in = g < T;
        const int ct = g / nk, k0 = (g - ct * nk) * 16;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int ka = in ? k0 + 4 * aq : d;
            const uint32_t oa = (aid[u] >= 0 && ka < d) ? (uint32_t)(((int64_t)aid[u] * p.ent_ld + ka) * 4) : kXsOOB;
            const auto va = __builtin_amdgcn_raw_buffer_load_b128(ra, oa, 0, 0);
            R.a[u] = make_float4(__uint_as_float(va[0]), __uint_as_float(va[1]), __uint_as_float(va[2]),
                                 __uint_as_float(va[3]));
            if constexpr (BPL) continue;
            const int kb = in ? k0 + 2 * bkp + u : d, j = ct * XBC + 4 * bjq;
            const uint32_t ob = (kb < d && j < d) ? (uint32_t)(((int64_t)kb * d + j) * 4) : kXsOOB;
            const auto vb = __builtin_amdgcn_raw_buffer_load_b128(rw, ob, 0, 0);
            R.b[u] = make_float4(__uint_as_float(vb[0]), __uint_as_float(vb[1]), __uint_as_float(vb[2]),
                                 __uint_as_float(vb[3]));
            if (fuse_mask) {
                const auto vm = __builtin_amdgcn_raw_buffer_load_b128(rm, ob, 0, 0);
                R.m[u] = make_float4(__uint_as_float(vm[0]), __uint_as_float(vm[1]), __uint_as_float(vm[2]),
                                     __uint_as_float(vm[3]));
            }
        }
        if constexpr (BPL) {
            // a chunk past the end (g >= T) reloads chunk 0: never multiplied, and no branch around the loads
            const int kc = in ? (k0 >> 4) : 0, cc = in ? ct * XBC : 0;
            const uint32_t ob = (uint32_t)((((int64_t)kc * p.mp_cols + cc + spc) * 16 + 8 * sph) * 2);
#pragma unroll
            for (int pl = 0; pl < 3; ++pl) {
                const auto v = __builtin_amdgcn_raw_buffer_load_b128(rp, ob + (uint32_t)(pl * mp_plane * 2), 0, 0);
                R.bp[pl] = make_int4(v[0], v[1], v[2], v[3]);
            }
        }
    };
    auto sstore = [&](const XsRegs& R, int stage) {
        unsigned char* A = xs_smem + stage * kXsStage;
        unsigned char* Bp = A + 3 * kXsPlane;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int row = (t >> 2) + 128 * u;
            bf16x4_t s0, s1, s2;
            split3_x4(f32x4_t{R.a[u].x, R.a[u].y, R.a[u].z, R.a[u].w}, s0, s1, s2);
            const int o = xs_off(row, aq >> 1) + (aq & 1) * 8;
            *reinterpret_cast<bf16x4_t*>(A + o) = s0;
            *reinterpret_cast<bf16x4_t*>(A + kXsPlane + o) = s1;
            *reinterpret_cast<bf16x4_t*>(A + 2 * kXsPlane + o) = s2;
        }
        if constexpr (BPL) {  // B: the planes' [column][16 k] rows as they are
#pragma unroll
            for (int pl = 0; pl < 3; ++pl) *reinterpret_cast<int4*>(Bp + pl * kXsPlane + xs_off(spc, sph)) = R.bp[pl];
            return;
        }
        // B: the two k rows of this thread's 4 columns, transposed into [column][k]
        float4 b0 = R.b[0], b1 = R.b[1];
        if (fuse_mask) {
            b0 = mul4(b0, R.m[0]);
            b1 = mul4(b1, R.m[1]);
        }
        const float lo_k[4] = {b0.x, b0.y, b0.z, b0.w}, hi_k[4] = {b1.x, b1.y, b1.z, b1.w};
        bf16x4_t e0, e1, e2, o0, o1, o2;  // the three terms of the four columns at k = 2 kp and 2 kp + 1
        split3_x4(f32x4_t{lo_k[0], lo_k[1], lo_k[2], lo_k[3]}, e0, e1, e2);
        split3_x4(f32x4_t{hi_k[0], hi_k[1], hi_k[2], hi_k[3]}, o0, o1, o2);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int cl = 4 * bjq + c;
            const int o = xs_off(cl, bkp >> 2) + (bkp & 3) * 4;
            *reinterpret_cast<bf16x2_t*>(Bp + o) = bf16x2_t{e0[c], o0[c]};
            *reinterpret_cast<bf16x2_t*>(Bp + kXsPlane + o) = bf16x2_t{e1[c], o1[c]};
            *reinterpret_cast<bf16x2_t*>(Bp + 2 * kXsPlane + o) = bf16x2_t{e2[c], o2[c]};
        }
    };
    f32x16 acc[2][4];
    auto zero_acc = [&]() {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int r2 = 0; r2 < 16; ++r2) acc[i][j][r2] = 0.f;
    };
    auto compute = [&](int stage) {
        const unsigned char* A = xs_smem + stage * kXsStage;
        const unsigned char* Bp = A + 3 * kXsPlane;
        bf16x8 a[2][3];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int o = xs_off(wr * 64 + i * 32 + col, half);
#pragma unroll
            for (int pl = 0; pl < 3; ++pl) a[i][pl] = *reinterpret_cast<const bf16x8*>(A + pl * kXsPlane + o);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int o = xs_off(wc * 128 + j * 32 + col, half);
            bf16x8 bb[3];
#pragma unroll
            for (int pl = 0; pl < 3; ++pl) bb[pl] = *reinterpret_cast<const bf16x8*>(Bp + pl * kXsPlane + o);
#pragma unroll
            for (int q = 0; q < 6; ++q)
#pragma unroll
                for (int i = 0; i < 2; ++i)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][kX3A[q]], bb[kX3B[q]], acc[i][j], 0, 0, 0);
        }
    };
    auto fold = [&](int ct) {  // ts_fwd_x3_kernel's per-row sums over this wave's 128 columns
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int r2 = 0; r2 < 16; ++r2) {
                float sq = 0.f, ab = 0.f;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int cg = ct * XBC + wc * 128 + j * 32 + col;
                    const float c = cg < d ? cs[cg] : 0.f;
                    const float v = acc[i][j][r2];
                    sq = fmaf(v, v, sq);
                    ab += fabsf(v * c);
                }
#pragma unroll
                for (int o = 16; o > 0; o >>= 1) {
                    sq += __shfl_xor(sq, o, kWave);
                    ab += __shfl_xor(ab, o, kWave);
                }
                if (col == 0) {
                    const int row = wr * 64 + i * 32 + (r2 & 3) + 8 * (r2 >> 2) + 4 * half;
                    float2& x = red[wc][row];
                    x = make_float2(x.x + sq, x.y + ab);
                }
            }
    };
    // SCHED: compute, sstore and gload of one step in the order the matrix pipe wants, written out in source
    // order between scheduling fences (the scheduler's own interleave of this step is undone by its register-
    // pressure check at 2 waves per SIMD, 254 VGPRs): B fragment j + 1 is read before fragment j's 12 MFMAs, and
    // after MFMAs 2, 6 and 10 of fragments 1-3 one piece of the staging runs (a row of A split and stored, half of
    // B's split, one column of B's stores, the loads of chunk g + 3 into the registers just stored). The same
    // MFMAs in the same order per accumulator, the same splits: bitwise the other order's scores.
    auto compute_staged = [&](int g, XsRegs& nxt) {
        const unsigned char* A = xs_smem + (g & 1) * kXsStage;
        const unsigned char* Bs = A + 3 * kXsPlane;
        unsigned char* SA = xs_smem + ((g + 1) & 1) * kXsStage;
        unsigned char* SB = SA + 3 * kXsPlane;
        bf16x4_t e0, e1, e2, o0, o1, o2;  // B's three terms at k = 2 kp (e) and 2 kp + 1 (o) of 4 columns
        auto piece = [&](int pc) {
            if (pc < 2) {  // A row u: split and store (sstore's)
                const int u = pc, row = (t >> 2) + 128 * u;
                bf16x4_t s0, s1, s2;
                split3_x4(f32x4_t{nxt.a[u].x, nxt.a[u].y, nxt.a[u].z, nxt.a[u].w}, s0, s1, s2);
                const int o = xs_off(row, aq >> 1) + (aq & 1) * 8;
                *reinterpret_cast<bf16x4_t*>(SA + o) = s0;
                *reinterpret_cast<bf16x4_t*>(SA + kXsPlane + o) = s1;
                *reinterpret_cast<bf16x4_t*>(SA + 2 * kXsPlane + o) = s2;
            } else if (pc < 8) {
                if constexpr (BPL) {
                    if (pc < 5) *reinterpret_cast<int4*>(SB + (pc - 2) * kXsPlane + xs_off(spc, sph)) = nxt.bp[pc - 2];
                } else if (pc < 4) {
                    float4 b = nxt.b[pc - 2];
                    if (fuse_mask) b = mul4(b, nxt.m[pc - 2]);
                    if (pc == 2)
                        split3_x4(f32x4_t{b.x, b.y, b.z, b.w}, e0, e1, e2);
                    else
                        split3_x4(f32x4_t{b.x, b.y, b.z, b.w}, o0, o1, o2);
                } else {
                    const int c = pc - 4, cl = 4 * bjq + c;
                    const int o = xs_off(cl, bkp >> 2) + (bkp & 3) * 4;
                    *reinterpret_cast<bf16x2_t*>(SB + o) = bf16x2_t{e0[c], o0[c]};
                    *reinterpret_cast<bf16x2_t*>(SB + kXsPlane + o) = bf16x2_t{e1[c], o1[c]};
                    *reinterpret_cast<bf16x2_t*>(SB + 2 * kXsPlane + o) = bf16x2_t{e2[c], o2[c]};
                }
            } else {
                gload(nxt, g + 3);
            }
        };
        bf16x8 a[2][3], bb[3], bn[3];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int o = xs_off(wr * 64 + i * 32 + col, half);
#pragma unroll
            for (int pl = 0; pl < 3; ++pl) a[i][pl] = *reinterpret_cast<const bf16x8*>(A + pl * kXsPlane + o);
        }
        {
            const int o = xs_off(wc * 128 + col, half);
#pragma unroll
            for (int pl = 0; pl < 3; ++pl) bb[pl] = *reinterpret_cast<const bf16x8*>(Bs + pl * kXsPlane + o);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (j < 3) {
                const int o = xs_off(wc * 128 + (j + 1) * 32 + col, half);
#pragma unroll
                for (int pl = 0; pl < 3; ++pl) bn[pl] = *reinterpret_cast<const bf16x8*>(Bs + pl * kXsPlane + o);
            }
#pragma unroll
            for (int m = 0; m < 12; ++m) {
                const int q = m >> 1, i = m & 1;
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][kX3A[q]], bb[kX3B[q]], acc[i][j], 0, 0, 0);
                if (j >= 1 && m % 4 == 1) {
                    __builtin_amdgcn_sched_barrier(0);
                    piece((j - 1) * 3 + m / 4);
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
#pragma unroll
            for (int pl = 0; pl < 3; ++pl) bb[pl] = bn[pl];
        }
    };
    // one chunk step: multiply stage g % 2, store chunk g + 1 (held in `nxt`) into the other stage, load chunk
    // g + 3 into `nxt` (chunk g + 2 is in flight in the other set), fold at the end of a column super-tile. The
    // store is unconditional (one basic block for the schedule): the last step's lands in a stage nothing reads
    // again, after the barrier that ended that stage's last multiply.
    auto step = [&](int g, XsRegs& nxt) {
        if constexpr (SCHED) {
            compute_staged(g, nxt);
        } else {
            compute(g & 1);
            if constexpr (!(KGE_TS_KO & 2)) sstore(nxt, (g + 1) & 1);
            if constexpr (!(KGE_TS_KO & 4)) gload(nxt, g + 3);
        }
        if ((g + 1) % nk == 0) {
            fold(g / nk);
            zero_acc();
        }
        if constexpr (!(KGE_TS_KO & 1)) __syncthreads();
    };
    XsRegs R0, R1;
    zero_acc();
    gload(R0, 0);
    gload(R1, 1);
    sstore(R0, 0);
    gload(R0, 2);
    __syncthreads();
    int g = 0;
    for (; g + 1 < T; g += 2) {
        step(g, R1);      // stores chunk g + 1 (R1), loads g + 3 into R1
        step(g + 1, R0);  // stores chunk g + 2 (R0), loads g + 4 into R0
    }
    if (g < T) step(g, R1);
    if (t < nrows) {
        const float2 x0 = red[0][t], x1 = red[1][t];
        const float2 x = make_float2(x0.x + x1.x, x0.y + x1.y);
        const int64_t n = n0 + t;
        p.out[b * p.out_ld + n] = p.gamma - x.y / sqrtf(x.x);
        if (p.stats) p.stats[b * p.N + n] = x;
    }
    if (p.out_neg) {  // the block holds the whole row (the launcher sets out_neg only then): its reduction
        __syncthreads();
        if (wave == 0) {
            const float rr = row_reduce_fast(p.out + b * p.out_ld, p.N, p.temperature, p.adversarial, lane);
            if (lane == 0) p.out_neg[b] = rr;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Single / tail-batch forward (the grouped row source: each batch row's own head, relation pos[b,1]) with the
// operands split once: ts_fwd_x3g_kernel. The B batch rows are few (512 at C6) and share M_r only within a
// relation (~B / R rows each), so ts_rows_kernel's 128-row blocks gave 4 chunk blocks per relation, most of
// them empty, each sweeping the columns 128 at a time: 279 us at C6 for 0.26 GFLOP. Here a block takes 64 rows
// of one relation and ALL columns at once (8 waves x 64 columns, up to 512 per pass), so one block per relation
// covers it in one pass over K; staging, planes and the pipeline are ts_fwd_x3s_kernel's.
//   A: 64 rows x 16 k (threads 0..255, one float4 each); B: 16 k x 512 columns (two k pairs x column quads per
//   thread), both split once into three bf16 planes, two LDS stages (108 KB), two register sets.
//   Per wave and chunk: 2 A and 2 B fragments x 3 planes (12 ds_read_b128), 24 MFMAs.
// The per-row sums over the columns are taken per wave (half-wave shuffles), then over the 8 waves in wave
// order: the products are ts_rows_kernel's, the column sums in another order (scores within fp32 rounding).
// ---------------------------------------------------------------------------------------------
// Split form (round 5): with the whole column range per block only one block per relation works (~12 CUs at
// C6). With a workspace, ts_fwd_x3g_kernel<4, 1, 2, MASK> gives a block 4 waves x 32 columns = 128 columns of its
// rows and one K range of 8 chunks (xsplit x ksplit blocks per row chunk: 16 at d = 500) and writes the rows' raw
// partial projections to the workspace; ts_xk_finish_kernel adds each row's K ranges in order and reduces it:
// deterministic, scores within fp32 rounding of the one-block form. A step of the K loop costs ~1.25 us whatever
// the block's width (profiles/r05_ts_xg_ab.txt: 2-wave blocks and deeper prefetch measured no faster), so the
// K split is what shortens the block: 32 steps -> 8.
constexpr int XGR = 64, XGC = 512;
constexpr int kXgAPlane = XGR * 32, kXgBPlane = XGC * 32;
constexpr int kXgStage = 3 * (kXgAPlane + kXgBPlane);
// LDS of one pipeline stage for a block of NWV waves x JPW column tiles of 32
constexpr int xg_bplane(int NWV, int JPW) { return NWV * JPW * 32 * 32; }
constexpr int xg_stage(int NWV, int JPW) { return 3 * (kXgAPlane + xg_bplane(NWV, JPW)); }

// the column-split form's block: 4 waves x 32 columns, two register sets (chunks loaded two steps ahead). Deeper
// prefetch (4 / 6 sets) and 2-wave 64-column blocks measured no faster (profiles/r05_ts_xg_ab.txt): a step costs
// ~1.3 us whatever its width, with or without the loads' latency exposed.
constexpr int kXgSplitWaves = 4, kXgSplitCols = 32 * kXgSplitWaves, kXgSplitDepth = 2;
// the split form's K range per block: 8 chunks of 16 (a 500-wide K in 4 ranges)
constexpr int kXgKChunks = 8;
__host__ __device__ constexpr int64_t xg_ksplit(int64_t d) { return ((d + 15) / 16 + kXgKChunks - 1) / kXgKChunks; }
__host__ __device__ constexpr int64_t xg_xsplit(int64_t d) { return (d + kXgSplitCols - 1) / kXgSplitCols; }

template <int JPW, int AP>
struct XgRegs {
    float4 a[AP], b[JPW][2], m[JPW][2];
};

template <int NWV, int JPW, int DEP, bool MASK>
__global__ __attribute__((amdgpu_flat_work_group_size(1, NWV * kWave), amdgpu_waves_per_eu(2))) void
ts_fwd_x3g_kernel(TsParams p) {
    constexpr int NT = NWV * kWave, CW = NWV * JPW * 32;  // threads, columns per pass
    constexpr int BPL = xg_bplane(NWV, JPW), STG = xg_stage(NWV, JPW);
    constexpr int AP = NT >= 4 * XGR ? 1 : 4 * XGR / NT;  // A float4 per thread per step
    static_assert(AP * NT == 4 * XGR || NT >= 4 * XGR, "A tile staging");
    using Regs = XgRegs<JPW, AP>;
    extern __shared__ __attribute__((aligned(16))) unsigned char xg_smem[];  // 2 stages, then u - 1 (d floats)
    __shared__ int rb[XGR], rid[XGR];
    __shared__ float2 part[NWV][XGR];
    __shared__ float2 red[XGR];
    __shared__ int wcnt[NWV];
    float* cs = reinterpret_cast<float*>(xg_smem + 2 * STG);

    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int half = lane >> 5, col = lane & 31;
    const int d = p.d;
    const bool sf = p.xk != nullptr;  // the split form
    const int xs = sf ? p.xsplit : 1, ks = sf ? p.ksplit : 1;
    const int split = (int)(blockIdx.x % xs);  // this block's column range
    const int64_t q0 = blockIdx.x / xs;
    const int kidx = (int)(q0 % ks);           // its K range
    // its (relation, row chunk): one-block form relation-major; split form chunk-major, so that the blocks of
    // every relation's first chunk (the ones with rows, unless a relation has more than 64) are dispatched first
    const int64_t q1 = q0 / ks;
    const int64_t r = sf ? q1 % (p.nrel + 1) : q1 / p.nchunk;  // == nrel: the out-of-range bucket
    const int64_t skip = (sf ? q1 / (p.nrel + 1) : q1 % p.nchunk) * XGR;
    // this block's rows: the batch rows of relation bucket r, ranks [skip, skip + 64), by an ordered ballot scan
    if (t < XGR) {
        rb[t] = -1;
        red[t] = make_float2(0.f, 0.f);
    }
    int64_t seen = 0;
    for (int64_t s = 0; s < p.B; s += NT) {
        const int64_t b = s + t;
        bool m = false;
        if (b < p.B) {
            const int64_t rr = p.pos[b * 3 + 1];
            m = (r < p.nrel) ? (rr == r) : !(rr >= 0 && rr < p.nrel);
        }
        const uint64_t bal = __ballot(m);
        if (lane == 0) wcnt[wave] = __popcll(bal);
        __syncthreads();
        int before = 0, total = 0;
#pragma unroll
        for (int w = 0; w < NWV; ++w) {
            before += (w < wave) ? wcnt[w] : 0;
            total += wcnt[w];
        }
        if (m) {
            const int64_t k = seen + before + __popcll(bal & ((1ull << lane) - 1ull)) - skip;
            if (k >= 0 && k < XGR) rb[k] = (int)b;
        }
        seen += total;
        __syncthreads();
        if (seen >= skip + XGR) break;  // uniform
    }
    const int nrows = (int)min<int64_t>(XGR, seen - skip);
    if (nrows <= 0) return;  // uniform (the finish skips a chunk without rows too)
    if (t < XGR) {
        int id = -1;
        if (rb[t] >= 0) {
            const int64_t e = p.pos[(int64_t)rb[t] * 3];  // the head (Q9: the tail-batch score uses the head too)
            if (e >= 0 && e < p.nent) id = (int)e;
        }
        rid[t] = id;
    }
    const bool rok = r >= 0 && r < p.nrel;
    if (!sf) {  // u - 1 for the relation row (the norm summed over 512 threads' strides in the same order at any
                // NWV, as ts_xk_finish_kernel sums it for the split form)
        float ss[kXThreads / NT];
#pragma unroll
        for (int q = 0; q < kXThreads / NT; ++q) {
            ss[q] = 0.f;
            for (int j = t + q * NT; j < d; j += kXThreads) {
                const float v = rok ? p.rel[r * p.rel_ld + j] : 0.f;
                cs[j] = v;
                ss[q] += v * v;
            }
            for (int o = 32; o > 0; o >>= 1) ss[q] += __shfl_xor(ss[q], o, kWave);
        }
        __shared__ float wsum8[kXWaves];
#pragma unroll
        for (int q = 0; q < kXThreads / NT; ++q)
            if (lane == 0) wsum8[q * NWV + wave] = ss[q];
        __syncthreads();
        float tot = 0.f;
#pragma unroll
        for (int w = 0; w < kXWaves; ++w) tot += wsum8[w];
        const float rnorm = sqrtf(tot);
        for (int j = t; j < d; j += NT) cs[j] = cs[j] / rnorm - 1.f;
    }
    __syncthreads();
    const rsrc_t ra = make_rsrc(p.ent, (uint32_t)(p.nent * p.ent_ld * 4));
    const float* Wr = rok ? (MASK ? p.W : p.Mpre) + r * (int64_t)d * d : p.W;
    const uint32_t mbytes = rok ? (uint32_t)((int64_t)d * d * 4) : 0u;
    const rsrc_t rw = make_rsrc(Wr, mbytes);
    constexpr bool fuse_mask = MASK;  // M_r = W_r * mask_r formed at staging (else p.Mpre holds the products)
    const rsrc_t rm = make_rsrc(fuse_mask && rok ? p.mask + r * (int64_t)d * d : p.W, fuse_mask ? mbytes : 0u);
    int aid[AP];
#pragma unroll
    for (int u = 0; u < AP; ++u) aid[u] = t + u * NT < 4 * XGR ? rid[(t + u * NT) >> 2] : -1;
    const int aq = t & 3, bkp = t & 7, bjq = t >> 3;
    // one-block form: every pass of CW columns over all of K; split form: the one pass of columns
    // [split CW, split CW + CW) over K chunks [kidx kXgKChunks, + kXgKChunks)
    const int nk0 = (d + 15) / 16;
    const int kc0 = sf ? kidx * kXgKChunks : 0, nk = sf ? min(kXgKChunks, nk0 - kc0) : nk0;
    const int npass = sf ? 1 : (d + CW - 1) / CW, T = nk * npass;
    const int col0 = sf ? split * CW : 0;

    // every load is issued unconditionally (a chunk past the end reads zeros through the out-of-range offset):
    // with no branch around a load the wait before a store to LDS counts exactly the younger sets' loads
    auto gload = [&](Regs& R, int g) {
        const bool in = g < T;
        const int pc = g / nk, k0 = (kc0 + g - pc * nk) * 16;
        const int ka = in ? k0 + 4 * aq : d;
#pragma unroll
        for (int u = 0; u < AP; ++u) {
            const uint32_t oa =
                (aid[u] >= 0 && ka < d) ? (uint32_t)(((int64_t)aid[u] * p.ent_ld + ka) * 4) : kXsOOB;
            const auto va = __builtin_amdgcn_raw_buffer_load_b128(ra, oa, 0, 0);
            R.a[u] = make_float4(__uint_as_float(va[0]), __uint_as_float(va[1]), __uint_as_float(va[2]),
                                 __uint_as_float(va[3]));
        }
#pragma unroll
        for (int u = 0; u < JPW; ++u)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int kb = in ? k0 + 2 * bkp + h : d, j = col0 + pc * CW + 4 * (bjq + (NT / 8) * u);
                const uint32_t ob = (kb < d && j < d) ? (uint32_t)(((int64_t)kb * d + j) * 4) : kXsOOB;
                const auto vb = __builtin_amdgcn_raw_buffer_load_b128(rw, ob, 0, 0);
                R.b[u][h] = make_float4(__uint_as_float(vb[0]), __uint_as_float(vb[1]), __uint_as_float(vb[2]),
                                        __uint_as_float(vb[3]));
                if (fuse_mask) {
                    const auto vm = __builtin_amdgcn_raw_buffer_load_b128(rm, ob, 0, 0);
                    R.m[u][h] = make_float4(__uint_as_float(vm[0]), __uint_as_float(vm[1]), __uint_as_float(vm[2]),
                                            __uint_as_float(vm[3]));
                }
            }
    };
    auto sstore = [&](const Regs& R, int stage) {
        unsigned char* A = xg_smem + stage * STG;
        unsigned char* Bp = A + 3 * kXgAPlane;
#pragma unroll
        for (int u = 0; u < AP; ++u)
            if (t + u * NT < 4 * XGR) {
                const int row = (t + u * NT) >> 2;
                bf16x4_t s0, s1, s2;
                split3_x4(f32x4_t{R.a[u].x, R.a[u].y, R.a[u].z, R.a[u].w}, s0, s1, s2);
                const int o = xs_off(row, aq >> 1) + (aq & 1) * 8;
                *reinterpret_cast<bf16x4_t*>(A + o) = s0;
                *reinterpret_cast<bf16x4_t*>(A + kXgAPlane + o) = s1;
                *reinterpret_cast<bf16x4_t*>(A + 2 * kXgAPlane + o) = s2;
            }
#pragma unroll
        for (int u = 0; u < JPW; ++u) {
            float4 b0 = R.b[u][0], b1 = R.b[u][1];
            if (fuse_mask) {
                b0 = mul4(b0, R.m[u][0]);
                b1 = mul4(b1, R.m[u][1]);
            }
            bf16x4_t e0, e1, e2, o0, o1, o2;
            split3_x4(f32x4_t{b0.x, b0.y, b0.z, b0.w}, e0, e1, e2);
            split3_x4(f32x4_t{b1.x, b1.y, b1.z, b1.w}, o0, o1, o2);
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int cl = 4 * (bjq + (NT / 8) * u) + c;
                const int o = xs_off(cl, bkp >> 2) + (bkp & 3) * 4;
                *reinterpret_cast<bf16x2_t*>(Bp + o) = bf16x2_t{e0[c], o0[c]};
                *reinterpret_cast<bf16x2_t*>(Bp + BPL + o) = bf16x2_t{e1[c], o1[c]};
                *reinterpret_cast<bf16x2_t*>(Bp + 2 * BPL + o) = bf16x2_t{e2[c], o2[c]};
            }
        }
    };
    f32x16 acc[2][JPW];
    auto zero_acc = [&]() {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < JPW; ++j)
#pragma unroll
                for (int r2 = 0; r2 < 16; ++r2) acc[i][j][r2] = 0.f;
    };
    auto compute = [&](int stage) {
        const unsigned char* A = xg_smem + stage * STG;
        const unsigned char* Bp = A + 3 * kXgAPlane;
        bf16x8 a[2][3];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int o = xs_off(i * 32 + col, half);
#pragma unroll
            for (int pl = 0; pl < 3; ++pl) a[i][pl] = *reinterpret_cast<const bf16x8*>(A + pl * kXgAPlane + o);
        }
#pragma unroll
        for (int j = 0; j < JPW; ++j) {
            const int o = xs_off(wave * JPW * 32 + j * 32 + col, half);
            bf16x8 bb[3];
#pragma unroll
            for (int pl = 0; pl < 3; ++pl) bb[pl] = *reinterpret_cast<const bf16x8*>(Bp + pl * BPL + o);
#pragma unroll
            for (int q = 0; q < 6; ++q)
#pragma unroll
                for (int i = 0; i < 2; ++i)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][kX3A[q]], bb[kX3B[q]], acc[i][j], 0, 0, 0);
        }
    };
    auto fold = [&](int pc) {  // this pass's per-row sums: per wave over its 64 columns, then over the waves
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int r2 = 0; r2 < 16; ++r2) {
                float sq = 0.f, ab = 0.f;
#pragma unroll
                for (int j = 0; j < JPW; ++j) {
                    const int cg = col0 + pc * CW + wave * JPW * 32 + j * 32 + col;
                    const float c = cg < d ? cs[cg] : 0.f;
                    const float v = acc[i][j][r2];
                    sq = fmaf(v, v, sq);
                    ab += fabsf(v * c);
                }
#pragma unroll
                for (int o = 16; o > 0; o >>= 1) {
                    sq += __shfl_xor(sq, o, kWave);
                    ab += __shfl_xor(ab, o, kWave);
                }
                if (col == 0) part[wave][i * 32 + (r2 & 3) + 8 * (r2 >> 2) + 4 * half] = make_float2(sq, ab);
            }
        __syncthreads();
        if (t < XGR) {
            float2 x = red[t];
#pragma unroll
            for (int w = 0; w < NWV; ++w) x = make_float2(x.x + part[w][t].x, x.y + part[w][t].y);
            red[t] = x;
        }
    };
    // DEP register sets: chunk c is held in set c % DEP from its load until its store to LDS, so a chunk's
    // loads are issued DEP steps before the step that stores it
    auto step = [&](int g, Regs& nxt) {
        compute(g & 1);
        if (g + 1 < T) sstore(nxt, (g + 1) & 1);
        gload(nxt, g + 1 + DEP);
        if (!sf && (g + 1) % nk == 0) {
            fold(g / nk);
            zero_acc();
        }
        __syncthreads();
    };
    Regs R[DEP];
    zero_acc();
#pragma unroll
    for (int c = 0; c < DEP; ++c) gload(R[c], c);
    sstore(R[0], 0);
    gload(R[0], DEP);
    __syncthreads();
    int g = 0;
    for (; g + DEP <= T; g += DEP) {
#pragma unroll
        for (int c = 0; c < DEP; ++c) step(g + c, R[(c + 1) % DEP]);
    }
#pragma unroll
    for (int c = 0; c < DEP - 1; ++c)
        if (g + c < T) step(g + c, R[(c + 1) % DEP]);
    if (sf) {  // the rows' raw projections over this block's columns and K range; ts_xk_finish_kernel reduces them
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int r2 = 0; r2 < 16; ++r2) {
                const int row = i * 32 + (r2 & 3) + 8 * (r2 >> 2) + 4 * half;
                if (row >= nrows) continue;
                float* xr = p.xk + ((int64_t)kidx * p.B + rb[row]) * p.xk_ld;
#pragma unroll
                for (int j = 0; j < JPW; ++j) {
                    const int cg = col0 + wave * JPW * 32 + j * 32 + col;
                    if (cg < d) xr[cg] = acc[i][j][r2];
                }
            }
        return;
    }
    if (t < nrows) {
        const float2 x = red[t];
        const int64_t b = rb[t];
        p.out[b * p.out_ld] = p.gamma - x.y / sqrtf(x.x);
        if (p.stats) p.stats[b * p.N] = x;
    }
}

// M_r split once per call into the planes ts_fwd_x3s_kernel<.., true> stages (split3_x4's arithmetic on the same
// products W * mask or Mpre, so the bf16 terms and the scores are bitwise the in-kernel split's): one thread per
// (relation, 16-k chunk, column), 16 k values -> 32 B per plane; columns past d and k past d are zero.
__global__ __launch_bounds__(kBlock) void ts_mplanes_kernel(const float* __restrict__ src, const float* __restrict__ mask,
                                                            int64_t nrel, int d, int cols, int nk,
                                                            __bf16* __restrict__ P) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= nrel * nk * cols) return;
    const int j = (int)(i % cols);
    const int64_t q = i / cols;
    const int kc = (int)(q % nk);
    const int64_t r = q / nk;
    const int64_t plane = (int64_t)nk * cols * 16;
    __bf16* o = P + r * 3 * plane + ((int64_t)kc * cols + j) * 16;
    // clamped addresses and a select (no branch around a load): the 16 loads (32 with the mask) issue together
    const int jc = min(j, d - 1);
    float x[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        const int k = min(kc * 16 + e, d - 1);
        const int64_t at = (r * d + k) * (int64_t)d + jc;
        x[e] = mask ? src[at] * mask[at] : src[at];
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        f32x4_t v;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int k = kc * 16 + 4 * g + e;
            v[e] = (k < d && j < d) ? x[4 * g + e] : 0.f;
        }
        bf16x4_t s0, s1, s2;
        split3_x4(v, s0, s1, s2);
        *reinterpret_cast<bf16x4_t*>(o + 4 * g) = s0;
        *reinterpret_cast<bf16x4_t*>(o + plane + 4 * g) = s1;
        *reinterpret_cast<bf16x4_t*>(o + 2 * plane + 4 * g) = s2;
    }
}

int64_t mplanes_bytes(int64_t nrel, int64_t d) {
    const int64_t cols = (d + XBC - 1) / XBC * XBC, nk = (d + 15) / 16;
    return nrel * 3 * nk * cols * 16 * 2;
}

template <bool MASK, bool BPL, bool SCHED>
void launch_x3s_form(const TsParams& q, unsigned grid, size_t lds, hipStream_t st) {
    static const bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(ts_fwd_x3s_kernel<MASK, BPL, SCHED>),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize,
                                                 2 * kXsStage + kXsMaxDim * 4) == hipSuccess;
    (void)attr;
    hipLaunchKernelGGL((ts_fwd_x3s_kernel<MASK, BPL, SCHED>), dim3(grid), dim3(kXThreads), lds, st, q);
}

// form 2: the compiler's instruction order (the A/B against the scheduled step; bitwise the same scores). The
// mask-product variant keeps it always: its scheduled step spills 26 VGPRs into the loop (613 against 404 us at
// c6's shape on 237 relations, profiles/r06_ts_sched_ab.txt).
template <bool MASK, bool BPL>
void launch_x3s(const TsParams& q, unsigned grid, size_t lds, hipStream_t st) {
    if (q.form == 2 || MASK)
        launch_x3s_form<MASK, BPL, false>(q, grid, lds, st);
    else
        launch_x3s_form<MASK, BPL, true>(q, grid, lds, st);
}

template <int NWV, int JPW, int DEP, bool MASK>
void launch_x3g(const TsParams& q, unsigned grid, size_t lds, size_t lds_max, hipStream_t st) {
    static const bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(ts_fwd_x3g_kernel<NWV, JPW, DEP, MASK>),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_max) == hipSuccess;
    (void)attr;
    hipLaunchKernelGGL((ts_fwd_x3g_kernel<NWV, JPW, DEP, MASK>), dim3(grid), dim3(NWV * kWave), lds, st, q);
}

// The split form's finish: one block per batch row. The row's projection is the sum of its K ranges' partial
// projections in range order (deterministic), reduced over the columns as the one-block form reduces it (u - 1
// of the row's relation in the same 512-thread order; the column sums in another order: scores within fp32
// rounding of the one-block form).
__global__ __launch_bounds__(kBlock) void ts_xk_finish_kernel(TsParams p) {
    extern __shared__ float xf_cs[];  // u - 1 (d floats)
    __shared__ float wsum8[kXWaves];
    __shared__ float2 wred[kWavesPerBlock];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int64_t b = blockIdx.x;
    const int d = p.d;
    const int64_t r = p.pos[b * 3 + 1];
    const bool rok = r >= 0 && r < p.nrel;
    {
        float ss[kXThreads / kBlock];
#pragma unroll
        for (int q = 0; q < kXThreads / kBlock; ++q) {
            ss[q] = 0.f;
            for (int j = t + q * kBlock; j < d; j += kXThreads) {
                const float v = rok ? p.rel[r * p.rel_ld + j] : 0.f;
                xf_cs[j] = v;
                ss[q] += v * v;
            }
            for (int o = 32; o > 0; o >>= 1) ss[q] += __shfl_xor(ss[q], o, kWave);
        }
#pragma unroll
        for (int q = 0; q < kXThreads / kBlock; ++q)
            if (lane == 0) wsum8[q * kWavesPerBlock + wave] = ss[q];
        __syncthreads();
        float tot = 0.f;
#pragma unroll
        for (int w = 0; w < kXWaves; ++w) tot += wsum8[w];
        const float rnorm = sqrtf(tot);
        for (int j = t; j < d; j += kBlock) xf_cs[j] = xf_cs[j] / rnorm - 1.f;
    }
    __syncthreads();
    float sq = 0.f, ab = 0.f;
    for (int c = t; c < d; c += kBlock) {
        float v = 0.f;
        for (int k = 0; k < p.ksplit; ++k) v += p.xk[((int64_t)k * p.B + b) * p.xk_ld + c];
        sq = fmaf(v, v, sq);
        ab += fabsf(v * xf_cs[c]);
    }
    for (int o = 32; o > 0; o >>= 1) {
        sq += __shfl_xor(sq, o, kWave);
        ab += __shfl_xor(ab, o, kWave);
    }
    if (lane == 0) wred[wave] = make_float2(sq, ab);
    __syncthreads();
    if (t == 0) {
        float2 x = make_float2(0.f, 0.f);
#pragma unroll
        for (int w = 0; w < kWavesPerBlock; ++w) x = make_float2(x.x + wred[w].x, x.y + wred[w].y);
        const float sc = p.gamma - x.y / sqrtf(x.x);
        p.out[b * p.out_ld] = sc;
        if (p.stats) p.stats[b * p.N] = x;
        if (p.out_pos_ls) p.out_pos_ls[b] = log_sigmoid(sc);
    }
    if (p.out_neg) {  // the tail-batch negative call's [B, 1] row (Q9): its reduction over the one score
        __syncthreads();
        if (wave == 0) {
            const float rr = row_reduce_fast(p.out + b * p.out_ld, 1, p.temperature, p.adversarial, lane);
            if (lane == 0) p.out_neg[b] = rr;
        }
    }
}

__global__ __launch_bounds__(kBlock) void ts_premul_kernel(const float4* __restrict__ W, const float4* __restrict__ mask,
                                                          float4* __restrict__ M, int64_t n4) {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n4; i += (int64_t)gridDim.x * kBlock)
        M[i] = mul4(W[i], mask[i]);
}

// ---------------------------------------------------------------------------------------------
// Relation CSR of the batch rows: count (one block per bucket), scan (one block), ordered list.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ bool in_bucket(const TsParams& p, int64_t b, int64_t r) {
    const int64_t rr = p.pos[b * 3 + 1];
    return r < p.nrel ? rr == r : !(rr >= 0 && rr < p.nrel);
}

__global__ __launch_bounds__(kBlock) void ts_rel_count_kernel(TsParams p, int* __restrict__ cnt) {
    __shared__ int wc[kWavesPerBlock];
    const int64_t r = blockIdx.x;
    int c = 0;
    for (int64_t b = threadIdx.x; b < p.B; b += kBlock) c += in_bucket(p, b, r) ? 1 : 0;
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, kWave);
    if ((threadIdx.x & 63) == 0) wc[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) cnt[r] = wc[0] + wc[1] + wc[2] + wc[3];
}

__global__ __launch_bounds__(kBlock) void ts_rel_list_kernel(TsParams p, const int* __restrict__ off,
                                                             int* __restrict__ list) {
    __shared__ int wcnt[kWavesPerBlock];
    const int64_t r = blockIdx.x;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    int base = off[r];
    for (int64_t s = 0; s < p.B; s += kBlock) {
        const int64_t b = s + t;
        const bool m = b < p.B && in_bucket(p, b, r);
        const uint64_t bal = __ballot(m);
        if (lane == 0) wcnt[wave] = __popcll(bal);
        __syncthreads();
        int before = 0, total = 0;
        for (int w = 0; w < kWavesPerBlock; ++w) {
            before += (w < wave) ? wcnt[w] : 0;
            total += wcnt[w];
        }
        if (m) list[base + before + __popcll(bal & ((1ull << lane) - 1ull))] = (int)b;
        base += total;
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------------------------
// dW: block = (relation r, tile (ti, tj) of dM_r, split s); dM_r[i][j] = sum_rows h[i] gp[j] over the
// rows of the relation (its batch rows x N), the split's contiguous part of that row list.
// ---------------------------------------------------------------------------------------------
template <int VEC>
__global__ __launch_bounds__(kBlock) void ts_dw_kernel(TsParams p) {
    __shared__ __attribute__((aligned(16))) float As[2][TBK][TLD];
    __shared__ __attribute__((aligned(16))) float Bs[2][TBK][TLD];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int half = lane >> 5, col = lane & 31;
    const int d = p.d, T = p.T, S = p.S;
    int64_t blk = blockIdx.x;
    const int s = (int)(blk % S);
    blk /= S;
    const int tj = (int)(blk % T);
    blk /= T;
    const int ti = (int)(blk % T);
    const int64_t r = blk / T;
    const int cnt = p.rcnt[r];
    if (cnt == 0) return;
    const int* lst = p.rlist + p.roff[r];
    const int64_t K = (int64_t)cnt * p.N;
    const int64_t q0 = K * s / S, q1 = K * (s + 1) / S;

    // thread t, unit u: k row (t >> 5) + 8 u of the chunk, columns (t & 31) * 4 .. + 3
    const int cq = (t & 31) * 4;
    float4 ra[NU], rbv[NU];
    auto gload = [&](int64_t k0) {
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            const int64_t q = k0 + (t >> 5) + 8 * u;
            ra[u] = make_float4(0.f, 0.f, 0.f, 0.f);
            rbv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (q < q1) {
                const int64_t b = lst[q / p.N], n = q % p.N;
                const int64_t id = row_entity(p, b, n);
                const int i = ti * TBM + cq, j = tj * TBN + cq;
                if (id >= 0 && id < p.nent) ra[u] = ld4<VEC>(p.ent + id * p.ent_ld, i, d - i);
                rbv[u] = ld4<VEC>(p.gp + (b * p.N + n) * d, j, d - j);
            }
        }
    };
    auto sstore = [&](int buf) {
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            *reinterpret_cast<float4*>(&As[buf][(t >> 5) + 8 * u][cq]) = ra[u];
            *reinterpret_cast<float4*>(&Bs[buf][(t >> 5) + 8 * u][cq]) = rbv[u];
        }
    };

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r2 = 0; r2 < 16; ++r2) {
            acc[i][0][r2] = 0.f;
            acc[i][1][r2] = 0.f;
        }
    const int64_t nk = (q1 - q0 + TBK - 1) / TBK;
    if (nk > 0) {
        gload(q0);
        sstore(0);
        __syncthreads();
        for (int64_t kc = 0; kc < nk; ++kc) {
            const int buf = (int)(kc & 1);
            if (kc + 1 < nk) gload(q0 + (kc + 1) * TBK);
            mfma_chunk(As[buf], Bs[buf], wm, wn, half, col, acc);
            if (kc + 1 < nk) {
                sstore(buf ^ 1);
                __syncthreads();
            }
        }
    }
    const int64_t dd = (int64_t)d * d;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int gj = tj * TBN + wn * 64 + j * 32 + col;
#pragma unroll
            for (int r2 = 0; r2 < 16; ++r2) {
                const int gi = ti * TBM + acc_row(wm, i, r2, half);
                if (gi < d && gj < d) {
                    const int64_t e = (int64_t)gi * d + gj;
                    if (S == 1) {
                        if (r < p.nrel) p.d_W[r * dd + e] += p.mask[r * dd + e] * acc[i][j][r2];
                    } else {
                        p.pdw[((int64_t)s * (p.nrel + 1) + r) * dd + e] = acc[i][j][r2];
                    }
                }
            }
        }
}

__global__ __launch_bounds__(kBlock) void ts_dw_reduce_kernel(TsParams p) {
    const int64_t dd = (int64_t)p.d * p.d;
    const int64_t total = p.nrel * dd;
    for (int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x; e < total; e += (int64_t)gridDim.x * kBlock) {
        const int64_t r = e / dd;
        if (p.rcnt[r] == 0) continue;
        float v = 0.f;
        for (int s = 0; s < p.S; ++s) v += p.pdw[((int64_t)s * (p.nrel + 1)) * dd + e];
        p.d_W[e] += p.mask[e] * v;
    }
}

// ---------------------------------------------------------------------------------------------
// d_rel: one block per relation; g_u = sum of the block partials of the relation's row blocks in
// block order, then the normalisation backward (g_u - u (u . g_u)) / ||r||.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void ts_drel_kernel(TsParams p) {
    extern __shared__ float gu[];  // d floats
    __shared__ float wsum[2][kWavesPerBlock];
    const int64_t r = blockIdx.x;
    const int cnt = p.rcnt[r];
    if (cnt == 0) return;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int d = p.d;
    const float* rr = p.rel + r * p.rel_ld;
    float ss = 0.f, dot = 0.f;
    for (int j = t; j < d; j += kBlock) {
        float g = 0.f;
        if (p.grouped) {
            const int nb = (cnt + TBM - 1) / TBM;
            for (int c = 0; c < nb; ++c) g += p.upart[(r * p.nchunk + c) * d + j];
        } else {
            const int* lst = p.rlist + p.roff[r];
            for (int q = 0; q < cnt; ++q) {
                const int64_t b = lst[q];
                for (int c = 0; c < p.nchunk; ++c) g += p.upart[(b * p.nchunk + c) * d + j];
            }
        }
        const float v = rr[j];
        gu[j] = g;
        ss += v * v;
    }
    for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o, kWave);
    if (lane == 0) wsum[0][wave] = ss;
    __syncthreads();
    const float rn = sqrtf(wsum[0][0] + wsum[0][1] + wsum[0][2] + wsum[0][3]);
    for (int j = t; j < d; j += kBlock) {
        const float u = rr[j] / rn;
        const float g = -sgnf(u - 1.f) * gu[j];
        gu[j] = g;
        dot += u * g;
    }
    for (int o = 32; o > 0; o >>= 1) dot += __shfl_xor(dot, o, kWave);
    if (lane == 0) wsum[1][wave] = dot;
    __syncthreads();
    const float ug = wsum[1][0] + wsum[1][1] + wsum[1][2] + wsum[1][3];
    for (int j = t; j < d; j += kBlock) {
        const float u = rr[j] / rn;
        p.d_rel[r * p.rel_ld + j] += (gu[j] - u * ug) / rn;
    }
}

// ---------------------------------------------------------------------------------------------
// d_ent: rows bucketed by entity (count, scan, scatter), each bucket rank-sorted by row id, then one
// wave per (entity, 256 columns) adds the bucket's dH rows in row order.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void ts_ent_count_kernel(TsParams p, int* __restrict__ count) {
    const int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (q >= p.B * p.N) return;
    const int64_t id = row_entity(p, q / p.N, q % p.N);
    if (id >= 0 && id < p.nent) atomicAdd(&count[id], 1);
}

__global__ __launch_bounds__(kBlock) void ts_ent_scatter_kernel(TsParams p, int* __restrict__ cursor,
                                                                int* __restrict__ code) {
    const int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (q >= p.B * p.N) return;
    const int64_t id = row_entity(p, q / p.N, q % p.N);
    if (id >= 0 && id < p.nent) code[atomicAdd(&cursor[id], 1)] = (int)q;
}

__global__ __launch_bounds__(kBlock) void ts_ent_sort_kernel(int64_t E, const int* __restrict__ off,
                                                             const int* __restrict__ code, int* __restrict__ sorted) {
    const int64_t e = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (e >= E) return;
    const int lane = threadIdx.x & 63;
    const int lo = off[e], n = off[e + 1] - lo;
    for (int i = lane; i < n; i += kWave) {  // codes are distinct: rank = # smaller
        const int v = code[lo + i];
        int rank = 0;
        for (int j = 0; j < n; ++j) rank += code[lo + j] < v ? 1 : 0;
        sorted[lo + rank] = v;
    }
}

__global__ __launch_bounds__(kBlock) void ts_dent_kernel(TsParams p, const int* __restrict__ off,
                                                         const int* __restrict__ sorted) {
    const int d = p.d;
    const int64_t chunks = (d + 255) / 256;
    const int64_t w = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    const int64_t e = w / chunks;
    if (e >= p.nent) return;
    const int lane = threadIdx.x & 63;
    const int c0 = (int)(w % chunks) * 256 + lane;
    const int lo = off[e], hi = off[e + 1];
    if (lo == hi) return;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int k = lo; k < hi; ++k) {
        const float* row = p.dh + (int64_t)sorted[k] * d;
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (c0 + 64 * u < d) acc[u] += row[c0 + 64 * u];
    }
    float* out = p.d_ent + e * p.ent_ld;
#pragma unroll
    for (int u = 0; u < 4; ++u)
        if (c0 + 64 * u < d) out[c0 + 64 * u] += acc[u];
}

// ---------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------
int check(const char* what) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_error(KGE_EHIP, (std::string(what) + ": " + hipGetErrorString(e)).c_str());
    return 0;
}

bool use_v4(const TsParams& p) {
    return p.d % 4 == 0 && p.ent_ld % 4 == 0 && ((uintptr_t)p.ent & 15) == 0 && ((uintptr_t)p.W & 15) == 0 &&
           ((uintptr_t)p.mask & 15) == 0 && ((uintptr_t)p.Mpre & 15) == 0;
}

int fill(TsParams& p, int mode, const float* ent, int64_t nent, int64_t ent_ld, const float* rel, int64_t nrel,
         int64_t rel_ld, const float* W, const float* mask, const int64_t* pos, const int64_t* neg, int64_t neg_ld,
         int64_t B, int64_t N, int64_t d, float gamma) {
    if (mode != KGE_HEAD_BATCH && mode != KGE_TAIL_BATCH && mode != KGE_SINGLE)
        return set_error(KGE_EINVAL, "TranSparse: mode must be 0, 1 or 3");
    if (B < 0 || N < 0 || d <= 0 || nent < 0 || nrel < 0) return set_error(KGE_EINVAL, "TranSparse: bad shape");
    if (d > kMaxTsDim) return set_error(KGE_ENOTSUP, "TranSparse: d > 8192");
    if (B > INT32_MAX / 4 || B * (N > 0 ? N : 1) > INT32_MAX) return set_error(KGE_EINVAL, "TranSparse: batch too large");
    p = TsParams{};
    p.ent = ent;
    p.nent = nent;
    p.ent_ld = ent_ld;
    p.rel = rel;
    p.nrel = nrel;
    p.rel_ld = rel_ld;
    p.W = W;
    p.mask = mask;
    p.pos = pos;
    p.neg = neg;
    p.neg_ld = neg_ld;
    p.B = B;
    p.grouped = mode != KGE_HEAD_BATCH;
    p.N = p.grouped ? 1 : N;
    p.d = (int)d;
    p.gamma = gamma;
    p.nchunk = (int)((p.grouped ? B : N) + TBM - 1) / TBM;
    if (p.nchunk == 0) p.nchunk = 1;
    return 0;
}

int64_t row_blocks(const TsParams& p) { return p.grouped ? (p.nrel + 1) * p.nchunk : p.B * p.nchunk; }

// true: the launch also produced p.out_neg / p.out_pos_ls (the fused epilogues); false: it ignored them
template <int OP>
bool launch_rows(const TsParams& p, hipStream_t st) {
    const unsigned blocks = (unsigned)row_blocks(p);
    const size_t lds = OP == TS_DH ? 0 : (size_t)p.d * sizeof(float);
    if constexpr (OP == TS_FWD) {
        // the bf16x3 forms (fp32 accuracy, 2.67x the fp32 MFMA rate) when rows take float4s, operands split once at
        // staging where the 32-bit buffer offsets reach (form 1: the forms that split each fragment in registers,
        // for the bitwise / rounding cross-checks)
        if (use_v4(p)) {
            const bool xs_ok = (p.form == 0 || p.form == 2) && p.d <= kXsMaxDim && p.nent * p.ent_ld * 4 < (int64_t)kXsOOB &&
                               (int64_t)p.d * p.d * 4 < (int64_t)kXsOOB;
            if (p.grouped && xs_ok) {
                // single / tail-batch rows: 64 rows of one relation per block (ts_fwd_x3g_kernel), all columns, or
                // with a workspace (xk) one of xsplit 128-column ranges x one of ksplit K ranges, then the finish
                TsParams q = p;
                q.nchunk = (int)((p.B + XGR - 1) / XGR);
                const int64_t chunks = (p.nrel + 1) * q.nchunk;
                if (p.xk) {
                    constexpr int ST = xg_stage(kXgSplitWaves, 1);
                    const size_t lds = 2 * (size_t)ST + (size_t)p.d * 4;
                    const unsigned grid = (unsigned)(chunks * p.xsplit * p.ksplit);
                    const size_t lmax = 2 * (size_t)ST + kXsMaxDim * 4;
                    if (q.Mpre)
                        launch_x3g<kXgSplitWaves, 1, kXgSplitDepth, false>(q, grid, lds, lmax, st);
                    else
                        launch_x3g<kXgSplitWaves, 1, kXgSplitDepth, true>(q, grid, lds, lmax, st);
                    hipLaunchKernelGGL(ts_xk_finish_kernel, dim3((unsigned)p.B), dim3(kBlock), (size_t)p.d * 4, st, q);
                    return true;
                }
                q.xk = nullptr;
                const size_t lds = 2 * (size_t)kXgStage + (size_t)p.d * 4;
                const size_t lmax = 2 * (size_t)kXgStage + kXsMaxDim * 4;
                if (q.Mpre)
                    launch_x3g<8, 2, 2, false>(q, (unsigned)chunks, lds, lmax, st);
                else
                    launch_x3g<8, 2, 2, true>(q, (unsigned)chunks, lds, lmax, st);
                return false;
            }
            if (!p.grouped && p.N > TBM && p.d <= kTsBigMaxDim) {
                // head-batch rows beyond one 128-row block: 256-row blocks that stage each M_r chunk once for all
                // the batch row's negatives
                TsParams q = p;
                q.nchunk = (int)((p.N + XBR - 1) / XBR);
                if (q.nchunk != 1) q.out_neg = nullptr;  // the epilogue reduces a row only when one block holds it
                if (xs_ok) {  // operands split once at staging (ts_fwd_x3s_kernel, bitwise ts_fwd_x3_kernel's scores)
                    const size_t lds = 2 * (size_t)kXsStage + (size_t)p.d * 4;
                    if (q.mplanes) {  // M_r split once for every block of the relation (workspace)
                        const int64_t n = (p.nrel) * q.mp_nk * (int64_t)q.mp_cols;
                        hipLaunchKernelGGL(ts_mplanes_kernel, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock),
                                           0, st, q.Mpre ? q.Mpre : q.W, q.Mpre ? nullptr : q.mask, p.nrel, p.d,
                                           q.mp_cols, q.mp_nk, q.mplanes);
                        launch_x3s<false, true>(q, (unsigned)(p.B * q.nchunk), lds, st);
                    } else if (q.Mpre) {
                        launch_x3s<false, false>(q, (unsigned)(p.B * q.nchunk), lds, st);
                    } else {
                        launch_x3s<true, false>(q, (unsigned)(p.B * q.nchunk), lds, st);
                    }
                    return q.nchunk == 1;
                }
                hipLaunchKernelGGL(ts_fwd_x3_kernel, dim3((unsigned)(p.B * q.nchunk)), dim3(kXThreads), lds, st, q);
                return q.nchunk == 1;
            }
            hipLaunchKernelGGL((ts_rows_kernel<OP, 4, true>), dim3(blocks), dim3(kBlock), lds, st, p);
            return false;
        }
    }
    if (use_v4(p))
        hipLaunchKernelGGL((ts_rows_kernel<OP, 4>), dim3(blocks), dim3(kBlock), lds, st, p);
    else
        hipLaunchKernelGGL((ts_rows_kernel<OP, 1>), dim3(blocks), dim3(kBlock), lds, st, p);
    return false;
}

size_t al(size_t x) { return (x + 255) & ~(size_t)255; }

struct TsWs {
    float *gp, *dh, *upart, *pdw;
    int *rcnt, *roff, *rcur, *rtiles, *rlist, *ecount, *eoff, *ecursor, *etiles, *ecode, *esorted;
    int S;
};

int pick_splits(int64_t nrel, int T) {
    const int64_t base = (nrel + 1) * (int64_t)T * T;
    int S = (int)((1024 + base - 1) / base);
    return S < 1 ? 1 : (S > 16 ? 16 : S);
}

size_t ws_layout(const TsParams& p, TsWs* w, char* base) {
    const int64_t rows = p.B * p.N, d = p.d, E = p.nent, R = p.nrel;
    const int T = (p.d + TBM - 1) / TBM;
    const int S = pick_splits(R, T);
    size_t o = 0;
    auto take = [&](size_t bytes) {
        char* ptr = base ? base + o : nullptr;
        o += al(bytes);
        return ptr;
    };
    TsWs x;
    x.gp = (float*)take((size_t)rows * d * 4);
    x.dh = (float*)take((size_t)rows * d * 4);
    x.upart = (float*)take((size_t)row_blocks(p) * d * 4);
    x.pdw = S > 1 ? (float*)take((size_t)S * (R + 1) * d * d * 4) : nullptr;
    x.rcnt = (int*)take((size_t)(R + 1) * 4);
    x.roff = (int*)take((size_t)(R + 2) * 4);
    x.rcur = (int*)take((size_t)(R + 1) * 4);
    x.rtiles = (int*)take((size_t)((R + 1 + 1023) / 1024 + 1) * 4);
    x.rlist = (int*)take((size_t)(p.B > 0 ? p.B : 1) * 4);
    x.ecount = (int*)take((size_t)(E > 0 ? E : 1) * 4);
    x.eoff = (int*)take((size_t)(E + 1) * 4);
    x.ecursor = (int*)take((size_t)(E > 0 ? E : 1) * 4);
    x.etiles = (int*)take((size_t)((E + 1023) / 1024 + 1) * 4);
    x.ecode = (int*)take((size_t)(rows > 0 ? rows : 1) * 4);
    x.esorted = (int*)take((size_t)(rows > 0 ? rows : 1) * 4);
    x.S = S;
    if (w) *w = x;
    return o;
}

}  // namespace
}  // namespace kge_impl

using namespace kge_impl;

extern "C" {

int kge_transparse_score(int mode, const float* ent, int64_t nent, int64_t ent_ld, const float* rel, int64_t nrel,
                         int64_t rel_ld, const float* W, const float* mask, const int64_t* pos, const int64_t* neg,
                         int64_t neg_ld, int64_t B, int64_t N, int64_t d, float gamma, float* out, int64_t out_ld,
                         float* stats, void* stream) {
    return kge_transparse_score_ex(mode, ent, nent, ent_ld, rel, nrel, rel_ld, W, mask, pos, neg, neg_ld, B, N, d,
                                   gamma, out, out_ld, stats, nullptr, nullptr, 0, stream);
}

// The head-batch planes split every M_r of the table on every call (nrel d^2 reads and 6 B written per element),
// whichever relations the batch uses: they are asked for only where the batch has many rows per relation (WN18RR:
// 11 relations, 512 rows; 346-360 against 365-380 us per call) and the planes stay small; otherwise 0, the staging
// split (the same scores; FB15k-237's 237 relations: 515-604 us with planes against 395-438 without, FB15k's 1 345:
// 1 320 against 417). The grouped split form stays on for every relation count: its extra blocks are mostly empty
// and cheap (1 345 relations: 444 us against 1 768 us for the one-block form). scripts/ts_many_rel_probe.py,
// profiles/r06_ts_many_rel_ab.txt.
constexpr int64_t kTsPlanesMinRowsPerRel = 16;
constexpr int64_t kTsPlanesMaxBytes = (int64_t)256 << 20;

size_t kge_transparse_score_workspace_size(int mode, int64_t nrel, int64_t B, int64_t d) {
    if (B <= 0 || d <= 0 || d > kXsMaxDim || nrel < 0) return 0;
    // head-batch: M_r as bf16 planes for the 256-row kernel
    if (mode == KGE_HEAD_BATCH)
        return ((nrel + 1) * kTsPlanesMinRowsPerRel <= B && mplanes_bytes(nrel, d) <= kTsPlanesMaxBytes)
                   ? (size_t)mplanes_bytes(nrel, d) : 0;
    // the grouped rows (single / tail-batch): the partial projections [ksplit][B][xsplit 128] floats
    const int64_t xs = xg_xsplit(d), ks = xg_ksplit(d);
    return xs * ks > 1 ? (size_t)(ks * B * xs * kXgSplitCols) * sizeof(float) : 0;
}

static int ts_score_impl(int mode, const float* ent, int64_t nent, int64_t ent_ld, const float* rel, int64_t nrel,
                         int64_t rel_ld, const float* W, const float* mask, const int64_t* pos, const int64_t* neg,
                         int64_t neg_ld, int64_t B, int64_t N, int64_t d, float gamma, float* out, int64_t out_ld,
                         float* stats, const kge_forms* forms, void* workspace, size_t workspace_bytes,
                         float* out_neg, float* out_pos_ls, float temperature, int adversarial, bool* fused,
                         void* stream) {
    if (fused) *fused = false;
    TsParams p;
    int rc = fill(p, mode, ent, nent, ent_ld, rel, nrel, rel_ld, W, mask, pos, neg, neg_ld, B, N, d, gamma);
    if (rc) return rc;
    p.form = forms ? forms->transparse_form : 0;
    const size_t need = kge_transparse_score_workspace_size(mode, nrel, B, d);
    if (workspace && need) {
        if (workspace_bytes < need) return set_error(KGE_EINVAL, "kge_transparse_score_ex: workspace too small");
        if ((uintptr_t)workspace & 15) return set_error(KGE_EINVAL, "kge_transparse_score_ex: workspace not 16-B aligned");
        if (p.grouped) {
            p.xsplit = (int)xg_xsplit(d);
            p.ksplit = (int)xg_ksplit(d);
            p.xk = reinterpret_cast<float*>(workspace);
            p.xk_ld = (int64_t)p.xsplit * kXgSplitCols;
        } else {
            p.mplanes = reinterpret_cast<__bf16*>(workspace);
            p.mp_cols = (int)((d + XBC - 1) / XBC * XBC);
            p.mp_nk = (int)((d + 15) / 16);
        }
    }
    if (B == 0 || (!p.grouped && N == 0)) return 0;
    if (!ent || !rel || !W || !pos || !out || (!p.grouped && !neg))
        return set_error(KGE_EINVAL, "kge_transparse_score: null pointer");
    if (!mask) p.Mpre = W;  // W already holds mask * W
    if (row_blocks(p) > INT32_MAX) return set_error(KGE_EINVAL, "kge_transparse_score: grid too large");
    p.out = out;
    p.out_ld = out_ld;
    p.stats = reinterpret_cast<float2*>(stats);
    p.out_neg = out_neg;
    p.out_pos_ls = out_pos_ls;
    p.temperature = temperature;
    p.adversarial = adversarial;
    const bool f = launch_rows<TS_FWD>(p, (hipStream_t)stream);
    if (fused) *fused = f;
    return check("kge_transparse_score");
}

int kge_transparse_score_ex(int mode, const float* ent, int64_t nent, int64_t ent_ld, const float* rel, int64_t nrel,
                            int64_t rel_ld, const float* W, const float* mask, const int64_t* pos, const int64_t* neg,
                            int64_t neg_ld, int64_t B, int64_t N, int64_t d, float gamma, float* out, int64_t out_ld,
                            float* stats, const kge_forms* forms, void* workspace, size_t workspace_bytes,
                            void* stream) {
    return ts_score_impl(mode, ent, nent, ent_ld, rel, nrel, rel_ld, W, mask, pos, neg, neg_ld, B, N, d, gamma, out,
                         out_ld, stats, forms, workspace, workspace_bytes, nullptr, nullptr, 1.f, 1, nullptr, stream);
}

size_t kge_transparse_step_workspace_size(int64_t nrel, int64_t B, int64_t d) {
    // the calls run in order on one stream: the head-batch planes, then the grouped rows' partial projections
    return std::max(kge_transparse_score_workspace_size(KGE_HEAD_BATCH, nrel, B, d),
                    kge_transparse_score_workspace_size(KGE_SINGLE, nrel, B, d));
}

int kge_transparse_step_forward(int mode, const float* ent, int64_t nent, int64_t ent_ld, const float* rel,
                                int64_t nrel, int64_t rel_ld, const float* W, const float* mask, const int64_t* pos,
                                const int64_t* neg, int64_t neg_ld, int64_t B, int64_t N, int64_t d, float gamma,
                                float temperature, int adversarial, float* neg_scores, int64_t ns_ld, float* out_neg,
                                float* pos_scores, float* out_pos, void* workspace, size_t workspace_bytes,
                                void* stream) {
    if (mode != KGE_HEAD_BATCH && mode != KGE_TAIL_BATCH)
        return set_error(KGE_EINVAL, "kge_transparse_step_forward: mode must be 0 (head-batch) or 1 (tail-batch)");
    if (B > 0 && (!out_neg || !out_pos || !neg_scores || !pos_scores))
        return set_error(KGE_EINVAL, "kge_transparse_step_forward: null output");
    // the negative call (model.py:121-125): scores, then its row reduction (model.py:168-171)
    bool fused = false;
    int rc = ts_score_impl(mode, ent, nent, ent_ld, rel, nrel, rel_ld, W, mask, pos, neg, neg_ld, B, N, d, gamma,
                           neg_scores, ns_ld, nullptr, nullptr, workspace, workspace_bytes, out_neg, nullptr,
                           temperature, adversarial, &fused, stream);
    if (rc) return rc;
    if (!fused && B > 0) {
        rc = kge_neg_reduce(neg_scores, B, mode == KGE_HEAD_BATCH ? N : 1, ns_ld, temperature, adversarial, out_neg,
                            stream);
        if (rc) return rc;
    }
    // the positive call (model.py:117-146): the single-mode scores and their logsigmoid (model.py:145)
    rc = ts_score_impl(KGE_SINGLE, ent, nent, ent_ld, rel, nrel, rel_ld, W, mask, pos, nullptr, 0, B, 1, d, gamma,
                       pos_scores, 1, nullptr, nullptr, workspace, workspace_bytes, nullptr, out_pos, temperature,
                       adversarial, &fused, stream);
    if (rc) return rc;
    if (!fused && B > 0) return kge_log_sigmoid(pos_scores, B, out_pos, stream);
    return 0;
}

size_t kge_transparse_bwd_workspace_size(int mode, int64_t nent, int64_t nrel, int64_t B, int64_t N, int64_t d) {
    TsParams p;
    if (fill(p, mode, nullptr, nent, 0, nullptr, nrel, 0, nullptr, nullptr, nullptr, nullptr, 0, B, N, d, 0.f))
        return 0;
    return ws_layout(p, nullptr, nullptr);
}

int kge_transparse_premul(const float* W, const float* mask, int64_t n, float* M, void* stream) {
    if (n < 0) return set_error(KGE_EINVAL, "kge_transparse_premul: bad size");
    if (n == 0) return 0;
    if (!W || !mask || !M || n % 4 || ((uintptr_t)W & 15) || ((uintptr_t)mask & 15) || ((uintptr_t)M & 15))
        return set_error(KGE_EINVAL, "kge_transparse_premul: needs 16-byte aligned buffers and n % 4 == 0");
    const int64_t n4 = n / 4;
    const int64_t nb = (n4 + kBlock - 1) / kBlock;
    const unsigned blocks = (unsigned)(nb < 4096 ? nb : 4096);
    hipLaunchKernelGGL(ts_premul_kernel, dim3(blocks), dim3(kBlock), 0, (hipStream_t)stream,
                       reinterpret_cast<const float4*>(W), reinterpret_cast<const float4*>(mask),
                       reinterpret_cast<float4*>(M), n4);
    return check("kge_transparse_premul");
}

int kge_transparse_score_bwd(int mode, const float* ent, int64_t nent, int64_t ent_ld, const float* rel,
                             int64_t nrel, int64_t rel_ld, const float* W, const float* mask, const float* M,
                             const int64_t* pos,
                             const int64_t* neg, int64_t neg_ld, int64_t B, int64_t N, int64_t d, const float* stats,
                             const float* d_scores, int64_t d_ld, float* d_ent, float* d_rel, float* d_W,
                             void* workspace, size_t workspace_bytes, void* stream) {
    TsParams p;
    int rc = fill(p, mode, ent, nent, ent_ld, rel, nrel, rel_ld, W, mask, pos, neg, neg_ld, B, N, d, 0.f);
    if (rc) return rc;
    if (B == 0 || (!p.grouped && N == 0)) return 0;
    if (!ent || !rel || !W || !mask || !pos || (!p.grouped && !neg) || !stats || !d_scores || !d_ent || !d_rel ||
        !d_W || !workspace)
        return set_error(KGE_EINVAL, "kge_transparse_score_bwd: null pointer");
    TsWs w;
    const size_t need = ws_layout(p, &w, (char*)workspace);
    if (workspace_bytes < need) return set_error(KGE_EINVAL, "kge_transparse_score_bwd: workspace too small");
    if (row_blocks(p) > INT32_MAX) return set_error(KGE_EINVAL, "kge_transparse_score_bwd: grid too large");
    hipStream_t st = (hipStream_t)stream;
    p.Mpre = M;
    p.stats = reinterpret_cast<float2*>(const_cast<float*>(stats));
    p.d_scores = d_scores;
    p.d_ld = d_ld;
    p.gp = w.gp;
    p.dh = w.dh;
    p.upart = w.upart;
    p.pdw = w.pdw;
    p.rcnt = w.rcnt;
    p.roff = w.roff;
    p.rlist = w.rlist;
    p.d_ent = d_ent;
    p.d_rel = d_rel;
    p.d_W = d_W;
    p.S = w.S;
    p.T = (p.d + TBM - 1) / TBM;
    const int64_t rows = p.B * p.N;
    // relation CSR
    hipLaunchKernelGGL(ts_rel_count_kernel, dim3((unsigned)(nrel + 1)), dim3(kBlock), 0, st, p, w.rcnt);
    launch_exclusive_scan(w.rcnt, nrel + 1, w.roff, w.rcur, w.rtiles, st);
    hipLaunchKernelGGL(ts_rel_list_kernel, dim3((unsigned)(nrel + 1)), dim3(kBlock), 0, st, p, w.roff, w.rlist);
    // dL/dp rows + g_u partials, then dL/dh rows
    launch_rows<TS_GP>(p, st);
    launch_rows<TS_DH>(p, st);
    // dW
    const int64_t dwb = (nrel + 1) * (int64_t)p.T * p.T * p.S;
    if (dwb > INT32_MAX) return set_error(KGE_EINVAL, "kge_transparse_score_bwd: dW grid too large");
    if (use_v4(p))
        hipLaunchKernelGGL(ts_dw_kernel<4>, dim3((unsigned)dwb), dim3(kBlock), 0, st, p);
    else
        hipLaunchKernelGGL(ts_dw_kernel<1>, dim3((unsigned)dwb), dim3(kBlock), 0, st, p);
    if (p.S > 1) hipLaunchKernelGGL(ts_dw_reduce_kernel, dim3(2048), dim3(kBlock), 0, st, p);
    // d_rel
    hipLaunchKernelGGL(ts_drel_kernel, dim3((unsigned)nrel), dim3(kBlock), (size_t)p.d * 4, st, p);
    // d_ent
    if (nent > 0) {
        if (hipMemsetAsync(w.ecount, 0, (size_t)nent * 4, st) != hipSuccess) return check("memset");
        const unsigned rb = (unsigned)((rows + kBlock - 1) / kBlock);
        hipLaunchKernelGGL(ts_ent_count_kernel, dim3(rb), dim3(kBlock), 0, st, p, w.ecount);
        launch_exclusive_scan(w.ecount, nent, w.eoff, w.ecursor, w.etiles, st);
        hipLaunchKernelGGL(ts_ent_scatter_kernel, dim3(rb), dim3(kBlock), 0, st, p, w.ecursor, w.ecode);
        hipLaunchKernelGGL(ts_ent_sort_kernel, dim3((unsigned)((nent + kWavesPerBlock - 1) / kWavesPerBlock)),
                           dim3(kBlock), 0, st, nent, w.eoff, w.ecode, w.esorted);
        const int64_t waves = nent * ((p.d + 255) / 256);
        hipLaunchKernelGGL(ts_dent_kernel, dim3((unsigned)((waves + kWavesPerBlock - 1) / kWavesPerBlock)),
                           dim3(kBlock), 0, st, p, w.eoff, w.esorted);
    }
    return check("kge_transparse_score_bwd");
}

}  // extern "C"
