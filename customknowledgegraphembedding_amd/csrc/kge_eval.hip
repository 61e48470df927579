// kge_eval.hip — filtered link-prediction evaluation against ALL entities (SURVEY §8f rank 3,
// BASELINE config C5: FB15k, each test triple vs all 14 951 entities, filtered MRR).
//
// Reference: upstream KGEModel.test_step (KnowledgeGraphEmbedding/codes/model.py, absent; restated in
// oracle/kge_oracle.py:eval_ranks): for every test triple and mode, score every entity as the
// candidate, push filtered candidates (other true triples) below the positive, and rank the positive.
//
//   * DistMult / ComplEx: scoring against all entities is a true dense contraction
//     S[q, e] = Q[q, :] . E[e, :]  (Q = h*r or r*t; ComplEx: [re_q | im_q] against [re_e | im_e]),
//     run on the fp32 matrix cores (v_mfma_f32_32x32x2_f32: exact f32, k-ordered fma chain).
//   * Every score function: S via the VALU scorer with the candidate row stride 0 (kge_abi.hip).
//   * kge_rank_filtered: exact integer ranks from S, the true entity and a CSR filter list.
#include <stdlib.h>

#include <string>

#include "kge_device.h"

namespace kge_impl {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

// ---------------------------------------------------------------------------------------------
// Query operand rows for the MFMA contraction: Q[b] = q0 (DistMult) or [q0 | q1] (ComplEx), built by
// the same Query<> code the scoring kernels use (tail mode: (h, r); head mode: (r, t)).
// ---------------------------------------------------------------------------------------------
typedef float xs_f32x4_t __attribute__((ext_vector_type(4)));
typedef __bf16 xs_bf16x4_t __attribute__((ext_vector_type(4)));
// xs_split3's arithmetic (the planes' three bf16 terms)
__device__ __forceinline__ void xs_split3_t(xs_f32x4_t v, xs_bf16x4_t& a0, xs_bf16x4_t& a1, xs_bf16x4_t& a2) {
    a0 = __builtin_convertvector(v, xs_bf16x4_t);
    const xs_f32x4_t r1 = v - __builtin_convertvector(a0, xs_f32x4_t);
    a1 = __builtin_convertvector(r1, xs_bf16x4_t);
    a2 = __builtin_convertvector(r1 - __builtin_convertvector(a1, xs_f32x4_t), xs_bf16x4_t);
}

template <int FN, bool CH, int V, int G>
__global__ __launch_bounds__(kBlock) void eval_query_kernel(ScoreParams p, float* __restrict__ Q, int64_t ldq,
                                                            __bf16* __restrict__ P, int64_t prows) {
    const int64_t b = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (b >= p.B) return;
    const int lane = threadIdx.x & 63;
    Query<FN, CH, V, G> q;
    int64_t qi, ri;
    bool qok, rok;
    build_query_for<FN, CH, V, G>(p, b, lane, q, qi, ri, qok, rok);
    const int DV = p.D / V;
    if constexpr (V == 4) {
        if (P) {  // kge_eval_query_planes: the row straight into the GEMM's bf16 planes (split3_planes_kernel's
                  // arithmetic and layout, [kp / 16][prows][16] per plane, k past K zero)
            const int K = FN == KGE_COMPLEX ? 2 * p.D : p.D, kp = (K + 15) / 16 * 16;
            const int64_t plane = prows * kp;
            auto put = [&](int k, const vecf<4>& v) {
                xs_bf16x4_t s0, s1, s2;
                xs_split3_t(xs_f32x4_t{v.a[0], v.a[1], v.a[2], v.a[3]}, s0, s1, s2);
                __bf16* d = P + ((int64_t)(k >> 4) * prows + b) * 16 + (k & 15);
                *reinterpret_cast<xs_bf16x4_t*>(d) = s0;
                *reinterpret_cast<xs_bf16x4_t*>(d + plane) = s1;
                *reinterpret_cast<xs_bf16x4_t*>(d + 2 * plane) = s2;
            };
#pragma unroll
            for (int k = 0; k < G; ++k) {
                const int g = lane + k * kWave;
                if (g < DV) {
                    put(4 * g, q.q0[k]);
                    if constexpr (FN == KGE_COMPLEX) put(p.D + 4 * g, q.q1[k]);
                }
            }
            for (int k = K + 4 * lane; k < kp; k += 4 * kWave) put(k, vzero<4>());  // the zero pad of the last chunk
            return;
        }
    }
    float* row = Q + b * ldq;
#pragma unroll
    for (int k = 0; k < G; ++k) {
        const int g = lane + k * kWave;
        if (g < DV) {
            *reinterpret_cast<vecf<V>*>(row + g * V) = q.q0[k];
            if constexpr (FN == KGE_COMPLEX) *reinterpret_cast<vecf<V>*>(row + p.D + g * V) = q.q1[k];
        }
    }
}

// ---------------------------------------------------------------------------------------------
// S[M, N] = A[M, K] . B[N, K]^T, fp32 in / fp32 out, on v_mfma_f32_32x32x2_f32.
// Block 256 threads = 2 x 2 waves, block tile 128 x BN (BN = 128 or 64), wave tile 64 x BN/2 (2 x JN
// MFMA tiles, independent accumulators -> back-to-back issue), K staged through LDS in chunks of 16,
// double buffered (next chunk's global loads in registers while the current chunk is multiplied).
// LDS images are k-major ([k][m]) so a wave's fragment read (lanes 0-31 one k, 32-63 the next)
// is 32 consecutive dwords per half-wave: conflict-free ds_read_b32. The staging stores are the
// transpose: lane l writes k-row 4 (l % 4) + c, column l / 4, so a half-wave's 32 dwords land on
// banks 4 (l % 4) LD + l / 4 (mod 32); a row pitch LD = 2 (mod 8) spreads them over all 32 banks
// (a pitch of BM + 4 put k-rows 0 and 8 on the same banks: 2-way conflicts on every store, which
// was every SQ_LDS_BANK_CONFLICT cycle the kernel had).
// BN = 64 halves the tile for grids too small to give every one of the 256 CUs a 128 x 128 tile.
// ---------------------------------------------------------------------------------------------
constexpr int GBM = 128, GBK = 16;  // BK = 32 measured 92 vs 96 TFLOP/s at C5
constexpr int GTPR = GBK / 4;       // threads per staged row
constexpr int GRPP = kBlock / GTPR;  // rows staged per unit
constexpr int GLD = GBM + 2;         // padded LDS row (floats): 2 (mod 8), conflict-free stores

template <int BN>
__global__ __launch_bounds__(kBlock) void gemm_nt_f32_kernel(const float* __restrict__ A, const float* __restrict__ Bm,
                                                             float* __restrict__ C, int M, int N, int K, int64_t lda,
                                                             int64_t ldb, int64_t ldc) {
    constexpr int JN = BN / 64;               // 32-wide MFMA tiles per wave in N
    constexpr int AU = GBM * GBK / 4 / kBlock;  // float4 per thread for A
    constexpr int BU = BN * GBK / 4 / kBlock;   // float4 per thread for B
    constexpr int BLD = BN + 2;  // 2 (mod 8) as GLD
    __shared__ __attribute__((aligned(16))) float As[2][GBK][GLD];
    __shared__ __attribute__((aligned(16))) float Bs[2][GBK][BLD];
    const int t = threadIdx.x;
    const int lane = t & 63;
    const int wave = t >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    // XCD-aware: blocks b and b+8 share an XCD (round-robin placement); give each XCD a contiguous
    // run of N-tiles (entity rows) so its L2 keeps reusing the same B rows across query tiles.
    const int ntn = (N + BN - 1) / BN, ntm = (M + GBM - 1) / GBM;
    const int nblk = ntn * ntm;
    int bid = blockIdx.x;
    if (nblk % 8 == 0) bid = (bid % 8) * (nblk / 8) + bid / 8;
    const int tn = bid / ntm, tm = bid % ntm;
    const int m0 = tm * GBM, n0 = tn * BN;

    // global -> register staging (thread t, unit u: row t / GTPR + GRPP u, k offset (t % GTPR) * 4)
    float4 ra[AU], rb[BU];
    const int kq = (t % GTPR) * 4;
    auto gload = [&](int k0) {
        const int ka = k0 + kq;
#pragma unroll
        for (int u = 0; u < AU; ++u) {
            const int gm = m0 + t / GTPR + GRPP * u;
            ra[u] = (gm < M && ka < K) ? *reinterpret_cast<const float4*>(A + (int64_t)gm * lda + ka)
                                       : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < BU; ++u) {
            const int gn = n0 + t / GTPR + GRPP * u;
            rb[u] = (gn < N && ka < K) ? *reinterpret_cast<const float4*>(Bm + (int64_t)gn * ldb + ka)
                                       : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    auto sstore = [&](int buf) {
#pragma unroll
        for (int u = 0; u < AU; ++u) {
            const int r = t / GTPR + GRPP * u;
            As[buf][kq + 0][r] = ra[u].x;
            As[buf][kq + 1][r] = ra[u].y;
            As[buf][kq + 2][r] = ra[u].z;
            As[buf][kq + 3][r] = ra[u].w;
        }
#pragma unroll
        for (int u = 0; u < BU; ++u) {
            const int r = t / GTPR + GRPP * u;
            Bs[buf][kq + 0][r] = rb[u].x;
            Bs[buf][kq + 1][r] = rb[u].y;
            Bs[buf][kq + 2][r] = rb[u].z;
            Bs[buf][kq + 3][r] = rb[u].w;
        }
    };

    f32x16 acc[2][JN];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < JN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int nk = (K + GBK - 1) / GBK;
    gload(0);
    sstore(0);
    __syncthreads();
    const int half = lane >> 5, col = lane & 31;
    for (int kc = 0; kc < nk; ++kc) {
        const int buf = kc & 1;
        if (kc + 1 < nk) gload((kc + 1) * GBK);  // next chunk in flight during the MFMAs
#pragma unroll
        for (int s = 0; s < GBK / 2; ++s) {
            const int kk = 2 * s + half;
            float a[2], b[JN];
#pragma unroll
            for (int i = 0; i < 2; ++i) a[i] = As[buf][kk][wm * 64 + i * 32 + col];
#pragma unroll
            for (int j = 0; j < JN; ++j) b[j] = Bs[buf][kk][wn * (BN / 2) + j * 32 + col];
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < JN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
        }
        if (kc + 1 < nk) {
            sstore(buf ^ 1);
            __syncthreads();
        }
    }
    // epilogue: C/D map of 32x32 MFMAs: col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < JN; ++j) {
            const int gn = n0 + wn * (BN / 2) + j * 32 + col;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int gm = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
                if (gm < M && gn < N) C[(int64_t)gm * ldc + gn] = acc[i][j][r];
            }
        }
}

// ---------------------------------------------------------------------------------------------
// fp32-accurate GEMM on the bf16 matrix cores: bf16x3 split, six products.
// Each fp32 operand x is split into three bf16 terms x = x0 + x1 + x2 (x0 = bf16(x), x1 = bf16(x - x0),
// x2 = bf16(x - x0 - x1); round-to-nearest-even; 24 significant bits, |x - x0 - x1 - x2| <= 2^-27 |x|),
// and A.B^T = sum of the six products Ai.Bj^T with i + j <= 2 (the three dropped ones are each
// <= 2^-26 |a||b| per term). v_mfma_f32_32x32x16_bf16 forms the bf16 products exactly and accumulates
// in fp32: the result is as close to the fp64 product as the fp32 MFMA path's (tests/test_eval_gpu.py),
// at 6 x 32 = 192 MFMA cycles per 16 k against 8 x 64 = 512 for v_mfma_f32_32x32x2_f32.
// ---------------------------------------------------------------------------------------------
constexpr int XBM = 128;

// The split is done on the fly: A and B tiles are staged through LDS as fp32, and each lane converts its
// fragment values to the three bf16 terms in registers (v_cvt_pk_bf16_f32, RNE) right before the MFMAs
// (pre-split bf16 planes staged instead moved 6 B per element and measured 1190 us against 920 us at C5). Block 128 x 128, 4 waves
// of 64 x 64, K in chunks of 32 double-buffered (LDS rows of 34 dwords: the ds_read_b64 fragment reads of
// 32 rows hit 32 distinct bank pairs; 70 KB per block, 2 blocks per CU). Non-finite inputs give NaN.
constexpr int YBK = 32, YLD = 34;

__global__ __launch_bounds__(kBlock) void gemm_nt_f32x3_kernel(const float* __restrict__ A, const float* __restrict__ Bm,
                                                               float* __restrict__ C, int M, int N, int K, int64_t lda,
                                                               int64_t ldb, int64_t ldc) {
    __shared__ __attribute__((aligned(16))) float As[2][XBM * YLD];
    __shared__ __attribute__((aligned(16))) float Bs[2][XBM * YLD];
    const int t = threadIdx.x;
    const int lane = t & 63, wave = t >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int ntn = (N + XBM - 1) / XBM, ntm = (M + XBM - 1) / XBM;
    const int nblk = ntn * ntm;
    int bid = blockIdx.x;
    {  // XCD-aware bijective remap: each XCD walks a contiguous run of N tiles (entity rows)
        const int q = nblk / 8, r = nblk % 8, x = bid % 8;
        bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
    }
    const int tn = bid / ntm, tm = bid % ntm;
    const int m0 = tm * XBM, n0 = tn * XBM;
    // staging: float4 f = t + 256 u (u < 4) of each 128 x 32 tile: row f >> 3, k 4 (f & 7)
    float4 ra[4], rb[4];
    auto gload = [&](int k0) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int f = t + kBlock * u, row = f >> 3, k = k0 + 4 * (f & 7);
            const int gm = m0 + row, gn = n0 + row;
            ra[u] = (gm < M && k < K) ? *reinterpret_cast<const float4*>(A + (int64_t)gm * lda + k)
                                      : make_float4(0.f, 0.f, 0.f, 0.f);
            rb[u] = (gn < N && k < K) ? *reinterpret_cast<const float4*>(Bm + (int64_t)gn * ldb + k)
                                      : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    auto sstore = [&](int buf) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int f = t + kBlock * u, o = (f >> 3) * YLD + 4 * (f & 7);
            *reinterpret_cast<float2*>(&As[buf][o]) = make_float2(ra[u].x, ra[u].y);
            *reinterpret_cast<float2*>(&As[buf][o + 2]) = make_float2(ra[u].z, ra[u].w);
            *reinterpret_cast<float2*>(&Bs[buf][o]) = make_float2(rb[u].x, rb[u].y);
            *reinterpret_cast<float2*>(&Bs[buf][o + 2]) = make_float2(rb[u].z, rb[u].w);
        }
    };
    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    const int nk = (K + YBK - 1) / YBK;
    gload(0);
    sstore(0);
    __syncthreads();
    const int r32 = lane & 31, half = lane >> 5;
    for (int kc = 0; kc < nk; ++kc) {
        const int buf = kc & 1;
        if (kc + 1 < nk) gload((kc + 1) * YBK);  // next chunk in flight during the MFMAs
#pragma unroll
        for (int s = 0; s < YBK / 16; ++s) {
            bf16x8 a[2][3], b[2][3];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const float* pa = &As[buf][(wm * 64 + i * 32 + r32) * YLD + 16 * s + 8 * half];
                const float* pb = &Bs[buf][(wn * 64 + i * 32 + r32) * YLD + 16 * s + 8 * half];
                f32x8 va, vb;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float2 x = *reinterpret_cast<const float2*>(pa + 2 * q);
                    const float2 y = *reinterpret_cast<const float2*>(pb + 2 * q);
                    va[2 * q] = x.x;
                    va[2 * q + 1] = x.y;
                    vb[2 * q] = y.x;
                    vb[2 * q + 1] = y.y;
                }
                split3_bf16(va, a[i][0], a[i][1], a[i][2]);
                split3_bf16(vb, b[i][0], b[i][1], b[i][2]);
            }
#pragma unroll
            for (int q = 0; q < 6; ++q)
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j)
                        acc[i][j] =
                            __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][kX3A[q]], b[j][kX3B[q]], acc[i][j], 0, 0, 0);
        }
        if (kc + 1 < nk) {
            sstore(buf ^ 1);
            __syncthreads();
        }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int gn = n0 + wn * 64 + j * 32 + r32;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int gm = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
                if (gm < M && gn < N) C[(int64_t)gm * ldc + gn] = acc[i][j][r];
            }
        }
}

// ---------------------------------------------------------------------------------------------
// Filtered rank of the true entity in each score row (one block per query row):
//   rank = 1 + #{ e != true : S[e] > S[true] } - #{ f in filt[q], f != true : S[f] > S[true] }
// The filter list of a row must hold distinct ids (the host dedups). Integer counts: exact.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void rank_kernel(const float* __restrict__ S, int64_t M, int64_t N, int64_t ld,
                                                      const int64_t* __restrict__ truth,
                                                      const int64_t* __restrict__ fptr,
                                                      const int64_t* __restrict__ fids, int64_t* __restrict__ ranks) {
    const int64_t q = blockIdx.x;
    if (q >= M) return;
    const float* row = S + q * ld;
    const int64_t tr = truth[q];
    const bool tok = tr >= 0 && tr < N;
    const float st = tok ? row[tr] : -INFINITY;
    unsigned long long cnt = 0;
    // a scalar head up to the first 16-B boundary, 16-B loads for the body, a scalar tail (the true
    // entity's own score is never > st, so the body needs no e != tr test)
    const int64_t head = min<int64_t>(N, (int64_t)((16 - ((uintptr_t)row & 15)) & 15) / 4);
    const int64_t nv = (N - head) / 4;
    for (int64_t e = threadIdx.x; e < head; e += kBlock) cnt += (e != tr && row[e] > st) ? 1ull : 0ull;
    {
        const rsrc_t rs = make_rsrc(row + head, (uint32_t)(nv * 16));
        for (int64_t g = threadIdx.x; g < nv; g += kBlock) {
            const vecf<4> v = bload<4>(rs, (uint32_t)(g * 16));
#pragma unroll
            for (int i = 0; i < 4; ++i) cnt += v.a[i] > st ? 1ull : 0ull;
        }
    }
    for (int64_t e = head + nv * 4 + threadIdx.x; e < N; e += kBlock) cnt += (e != tr && row[e] > st) ? 1ull : 0ull;
    if (fptr) {
        for (int64_t i = fptr[q] + threadIdx.x; i < fptr[q + 1]; i += kBlock) {
            const int64_t f = fids[i];
            if (f >= 0 && f < N && f != tr && row[f] > st) cnt -= 1ull;
        }
    }
    // block reduction of the (exact, wrapping) counts
    __shared__ unsigned long long red[kBlock / kWave];
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, kWave);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long c = 0;
        for (int w = 0; w < kBlock / kWave; ++w) c += red[w];
        ranks[q] = 1 + (int64_t)c;
    }
}

template <int FN, bool CH>
int launch_eval_query(const ScoreParams& p, hipStream_t st, int blocks, int V, int G, float* Q, int64_t ldq,
                      __bf16* P, int64_t prows) {
#define KGE_EQ(VV, GG)                                                                                   \
    if (V == VV && G == GG) {                                                                            \
        hipLaunchKernelGGL((eval_query_kernel<FN, CH, VV, GG>), dim3(blocks), dim3(kBlock), 0, st, p, Q, ldq, P, \
                           prows);                                                                       \
        return 0;                                                                                        \
    }
    KGE_EQ(4, 1) KGE_EQ(4, 2) KGE_EQ(4, 4) KGE_EQ(4, 8)
    KGE_EQ(2, 1) KGE_EQ(2, 2) KGE_EQ(2, 4) KGE_EQ(2, 8)
    KGE_EQ(1, 1) KGE_EQ(1, 2) KGE_EQ(1, 4) KGE_EQ(1, 8)
#undef KGE_EQ
    return KGE_ENOTSUP;
}

}  // namespace

int launch_eval_query_any(int fn, bool ch, const ScoreParams& p, hipStream_t st, int blocks, int V, int G, float* Q,
                          int64_t ldq, void* P, int64_t prows) {
    __bf16* pp = static_cast<__bf16*>(P);
    if (fn == KGE_DISTMULT)
        return ch ? launch_eval_query<KGE_DISTMULT, true>(p, st, blocks, V, G, Q, ldq, pp, prows)
                  : launch_eval_query<KGE_DISTMULT, false>(p, st, blocks, V, G, Q, ldq, pp, prows);
    if (fn == KGE_COMPLEX)
        return ch ? launch_eval_query<KGE_COMPLEX, true>(p, st, blocks, V, G, Q, ldq, pp, prows)
                  : launch_eval_query<KGE_COMPLEX, false>(p, st, blocks, V, G, Q, ldq, pp, prows);
    return KGE_ENOTSUP;
}

int launch_gemm_nt(const float* A, const float* B, float* C, int M, int N, int K, int64_t lda, int64_t ldb,
                   int64_t ldc, hipStream_t st) {
    // tile width: 128 x 128 unless that grid leaves CUs idle (fewer tiles than the 256 CUs); at C5
    // (936 tiles) 128 wide measured 102 TFLOP/s against 92 for 64 wide
    const int64_t tm = (M + GBM - 1) / GBM;
    const int64_t t128 = tm * ((N + 127) / 128), t64 = tm * ((N + 63) / 64);
    int bn = t128 < 256 ? 64 : 128;
    const int64_t t256 = tm * ((N + 255) / 256);
    if (bn == 256)
        hipLaunchKernelGGL(gemm_nt_f32_kernel<256>, dim3((unsigned)t256), dim3(kBlock), 0, st, A, B, C, M, N, K, lda,
                           ldb, ldc);
    else if (bn == 64)
        hipLaunchKernelGGL(gemm_nt_f32_kernel<64>, dim3((unsigned)t64), dim3(kBlock), 0, st, A, B, C, M, N, K, lda,
                           ldb, ldc);
    else
        hipLaunchKernelGGL(gemm_nt_f32_kernel<128>, dim3((unsigned)t128), dim3(kBlock), 0, st, A, B, C, M, N, K, lda,
                           ldb, ldc);
    return 0;
}

// ---------------------------------------------------------------------------------------------
// The same products with the operands split ONCE at staging (gemm_nt_x3s_kernel; the TranSparse forward's
// staging, ts_fwd_x3s_kernel): gemm_nt_f32x3_kernel splits every fragment in its MFMA loop (each A and B
// fragment twice over) behind branchy staging loads. Here:
//   * block tile 256 x 256, 8 waves of 64 x 128 (eight 32 x 32 accumulators), one block per CU at 2 waves per SIMD;
//   * K in chunks of 16; each thread loads one k quad of two A rows and two B rows per chunk with raw buffer
//     loads (the range check zero-fills past M, N and K: no branches) and splits each value once into three bf16
//     planes [row][16 k] (32-B rows, 16-B halves swapped every other 8 rows: conflict-free fragment reads);
//   * two LDS stages (96 KB) and two register sets: chunk g + 2 loads while chunk g multiplies.
// Per wave and chunk: 18 ds_read_b128 for 48 MFMAs and no other VALU work. The per-element products and their
// order are gemm_nt_f32x3_kernel's: C is bitwise the same.
// ---------------------------------------------------------------------------------------------
namespace {
constexpr int XS_T = 256;                      // block tile (rows of A and of B)
constexpr int XS_PLANE = XS_T * 32;            // one bf16 plane of a 16-k chunk: 256 rows x 32 B
constexpr int XS_STAGE = 6 * XS_PLANE;         // A planes then B planes (48 KB)
constexpr uint32_t XS_OOB = 0xFFFFFFF0u;

__device__ __forceinline__ int xs_off(int row, int h) { return row * 32 + ((h ^ ((row >> 3) & 1)) << 4); }

typedef float xs_f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 xs_bf16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void xs_split3(xs_f32x4 v, xs_bf16x4& a0, xs_bf16x4& a1, xs_bf16x4& a2) {
    a0 = __builtin_convertvector(v, xs_bf16x4);
    const xs_f32x4 r1 = v - __builtin_convertvector(a0, xs_f32x4);
    a1 = __builtin_convertvector(r1, xs_bf16x4);
    a2 = __builtin_convertvector(r1 - __builtin_convertvector(a1, xs_f32x4), xs_bf16x4);
}

struct XsGemmRegs {
    float4 a[2], b[2];
};

__global__ __attribute__((amdgpu_flat_work_group_size(1, 512), amdgpu_waves_per_eu(2))) void gemm_nt_x3s_kernel(
    const float* __restrict__ A, const float* __restrict__ Bm, float* __restrict__ C, int M, int N, int K, int64_t lda,
    int64_t ldb, int64_t ldc) {
    extern __shared__ __attribute__((aligned(16))) unsigned char gx_smem[];  // 2 stages
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int half = lane >> 5, col = lane & 31;
    const int wr = wave >> 1, wc = wave & 1;
    const int ntn = (N + XS_T - 1) / XS_T, ntm = (M + XS_T - 1) / XS_T;
    const int nblk = ntn * ntm;
    int bid = blockIdx.x;
    {  // XCD-aware bijective remap (gemm_nt_f32x3_kernel's): each XCD walks a contiguous run of N tiles
        const int q = nblk / 8, r = nblk % 8, x = bid % 8;
        bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
    }
    const int tn = bid / ntm, tm = bid % ntm;
    const int m0 = tm * XS_T, n0 = tn * XS_T;
    const rsrc_t ra = make_rsrc(A, (uint32_t)((int64_t)M * lda * 4));
    const rsrc_t rb = make_rsrc(Bm, (uint32_t)((int64_t)N * ldb * 4));
    const int q4 = t & 3;
    int arow[2], brow[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        arow[u] = m0 + (t >> 2) + 128 * u;
        brow[u] = n0 + (t >> 2) + 128 * u;
    }
    const int T = (K + 15) / 16;
    auto gload = [&](XsGemmRegs& R, int g) {
        const int k = g * 16 + 4 * q4;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const uint32_t oa = (arow[u] < M && k < K) ? (uint32_t)(((int64_t)arow[u] * lda + k) * 4) : XS_OOB;
            const uint32_t ob = (brow[u] < N && k < K) ? (uint32_t)(((int64_t)brow[u] * ldb + k) * 4) : XS_OOB;
            const auto va = __builtin_amdgcn_raw_buffer_load_b128(ra, oa, 0, 0);
            const auto vb = __builtin_amdgcn_raw_buffer_load_b128(rb, ob, 0, 0);
            R.a[u] = make_float4(__uint_as_float(va[0]), __uint_as_float(va[1]), __uint_as_float(va[2]),
                                 __uint_as_float(va[3]));
            R.b[u] = make_float4(__uint_as_float(vb[0]), __uint_as_float(vb[1]), __uint_as_float(vb[2]),
                                 __uint_as_float(vb[3]));
        }
    };
    auto sstore = [&](const XsGemmRegs& R, int stage) {
        unsigned char* As = gx_smem + stage * XS_STAGE;
        unsigned char* Bs = As + 3 * XS_PLANE;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int row = (t >> 2) + 128 * u;
            const int o = xs_off(row, q4 >> 1) + (q4 & 1) * 8;
            xs_bf16x4 s0, s1, s2;
            xs_split3(xs_f32x4{R.a[u].x, R.a[u].y, R.a[u].z, R.a[u].w}, s0, s1, s2);
            *reinterpret_cast<xs_bf16x4*>(As + o) = s0;
            *reinterpret_cast<xs_bf16x4*>(As + XS_PLANE + o) = s1;
            *reinterpret_cast<xs_bf16x4*>(As + 2 * XS_PLANE + o) = s2;
            xs_split3(xs_f32x4{R.b[u].x, R.b[u].y, R.b[u].z, R.b[u].w}, s0, s1, s2);
            *reinterpret_cast<xs_bf16x4*>(Bs + o) = s0;
            *reinterpret_cast<xs_bf16x4*>(Bs + XS_PLANE + o) = s1;
            *reinterpret_cast<xs_bf16x4*>(Bs + 2 * XS_PLANE + o) = s2;
        }
    };
    f32x16 acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r2 = 0; r2 < 16; ++r2) acc[i][j][r2] = 0.f;
    auto compute = [&](int stage) {
        const unsigned char* As = gx_smem + stage * XS_STAGE;
        const unsigned char* Bs = As + 3 * XS_PLANE;
        bf16x8 a[2][3];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int o = xs_off(wr * 64 + i * 32 + col, half);
#pragma unroll
            for (int pl = 0; pl < 3; ++pl) a[i][pl] = *reinterpret_cast<const bf16x8*>(As + pl * XS_PLANE + o);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int o = xs_off(wc * 128 + j * 32 + col, half);
            bf16x8 bb[3];
#pragma unroll
            for (int pl = 0; pl < 3; ++pl) bb[pl] = *reinterpret_cast<const bf16x8*>(Bs + pl * XS_PLANE + o);
#pragma unroll
            for (int q = 0; q < 6; ++q)
#pragma unroll
                for (int i = 0; i < 2; ++i)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][kX3A[q]], bb[kX3B[q]], acc[i][j], 0, 0, 0);
        }
    };
    // the loads are issued unconditionally (a chunk past K reads zeros through the out-of-range offset): with no
    // branch around a load, the wait before a store to LDS leaves the younger set's loads in flight (a
    // conditional load made it wait for every load, the pipeline one chunk deep)
    auto step = [&](int g, XsGemmRegs& nxt) {
        compute(g & 1);
        if (g + 1 < T) sstore(nxt, (g + 1) & 1);
        gload(nxt, g + 3);
        __syncthreads();
    };
    XsGemmRegs R0, R1;
    gload(R0, 0);
    gload(R1, 1);
    sstore(R0, 0);
    gload(R0, 2);
    __syncthreads();
    int g = 0;
    for (; g + 1 < T; g += 2) {
        step(g, R1);
        step(g + 1, R0);
    }
    if (g < T) step(g, R1);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int gn = n0 + wc * 128 + j * 32 + col;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int gm = m0 + wr * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
                if (gm < M && gn < N) C[(int64_t)gm * ldc + gn] = acc[i][j][r];
            }
        }
}

// ---------------------------------------------------------------------------------------------
// The same GEMM on operands split BEFORE it (round 5): gemm_nt_x3s_kernel spends ~190 VALU instructions per wave
// and 16-k chunk splitting its fp32 loads into bf16 terms and computing their addresses, against 48 MFMAs
// (PMC, profiles/r05_pmc_c5.json: the matrix cores busy 0.60 of the kernel, co-issuing with that VALU work 20 %
// of the time). The operands of the all-entity scores are reused: the entity table across every query batch of
// an evaluation pass, the query block across the 59 entity tiles. split3_planes_kernel writes each fp32 matrix as
// three bf16 planes (xs_split3's arithmetic, K rounded up to 16 with zeros), each plane k-chunk-major
// [K / 16][rows][16]: a block's 16-k chunk of 256 rows is 8 KB contiguous per plane, loaded in whole lines (a
// row-major [rows][K] plane gave each row's 32 B of a chunk its own 128-B line: 4x the L2 traffic, slower than
// staging from fp32). gemm_nt_x3p_kernel stages the pieces into the same LDS images with no conversion: the
// products, their order and C are bitwise gemm_nt_x3s_kernel's.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ int64_t rows_pad(int64_t plane, int kp) { return plane / kp; }

__global__ __launch_bounds__(kBlock) void split3_planes_kernel(const float* __restrict__ X, int64_t rows, int cols,
                                                               int64_t ld, int kp, __bf16* __restrict__ P,
                                                               int64_t plane) {
    const int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x;  // one k quad of one row
    const int kq = kp / 4;
    if (q >= rows * kq) return;
    const int64_t r = q / kq;
    const int k = (int)(q - r * kq) * 4;
    xs_f32x4 v;
    if (k + 3 < cols && (ld & 3) == 0 && ((uintptr_t)X & 15) == 0) {
        const float4 x = *reinterpret_cast<const float4*>(X + r * ld + k);
        v = xs_f32x4{x.x, x.y, x.z, x.w};
    } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = k + i < cols ? X[r * ld + k + i] : 0.f;
    }
    xs_bf16x4 s0, s1, s2;
    xs_split3(v, s0, s1, s2);
    __bf16* d = P + ((int64_t)(k >> 4) * rows_pad(plane, kp) + r) * 16 + (k & 15);
    *reinterpret_cast<xs_bf16x4*>(d) = s0;
    *reinterpret_cast<xs_bf16x4*>(d + plane) = s1;
    *reinterpret_cast<xs_bf16x4*>(d + 2 * plane) = s2;
}

struct XpGemmRegs {
    int4 a[3], b[3];
};

// Knock-out builds for the step-cost breakdown probe (scripts/x3p_knockout_probe.py; wrong results by design,
// never the library's build): bit 0 drops the per-chunk barrier, bit 1 the LDS stores, bit 2 the global loads,
// bit 3 the fragment reads (the MFMAs take fragments read once before the loop).
#ifndef KGE_X3P_KO
#define KGE_X3P_KO 0
#endif

// CNT (kge_eval_rank_planes): no C; the epilogue counts, per query row, the scores above the row's truth score
// ts[row] (columns < N) and adds the block's counts to gcnt[row] (integer atomics). The accumulators are the
// CNT = false kernel's, bitwise.
// JN: 32-column B tiles per wave; the block tile is 256 x 64 JN (JN 4: 256 x 256; JN 3: 256 x 192, whose 78 tiles
// per 4 096-query M tile at C5 fill 4.9 rounds of the CUs where 256-wide tiles fill 3.7). Every accumulator element
// takes the same products in the same order for either JN: C is bitwise the same.
template <bool CNT, int JN>
__global__ __attribute__((amdgpu_flat_work_group_size(1, 512), amdgpu_waves_per_eu(2))) void gemm_nt_x3p_kernel(
    const __bf16* __restrict__ Ap, int64_t a_plane, const __bf16* __restrict__ Bp, int64_t b_plane, int kp,
    float* __restrict__ C, int M, int N, int64_t ldc, const float* __restrict__ ts, int* __restrict__ gcnt) {
    extern __shared__ __attribute__((aligned(16))) unsigned char gp_smem[];  // 2 stages
    __shared__ int rowcnt[CNT ? XS_T : 1];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    if constexpr (CNT) {
        if (t < XS_T) rowcnt[t] = 0;  // visible after the prologue's barrier
    }
    const int half = lane >> 5, col = lane & 31;
    const int wr = wave >> 1, wc = wave & 1;
    constexpr int TN = 64 * JN;  // block tile columns
    const int ntn = (N + TN - 1) / TN, ntm = (M + XS_T - 1) / XS_T;
    const int nblk = ntn * ntm;
    int bid = blockIdx.x;
    {  // XCD-aware bijective remap (gemm_nt_x3s_kernel's)
        const int q = nblk / 8, r = nblk % 8, x = bid % 8;
        bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
    }
    const int tn = bid / ntm, tm = bid % ntm;
    const int m0 = tm * XS_T, n0 = tn * TN;
    const rsrc_t ra = make_rsrc(Ap, (uint32_t)(3 * a_plane * 2));
    const rsrc_t rb = make_rsrc(Bp, (uint32_t)(3 * b_plane * 2));
    // thread t stages row t >> 1, k half t & 1 of every plane; a plane is [K / 16][plane rows][16], so chunk g of
    // the block's rows is contiguous and the offsets advance one chunk slab (plane rows x 32 B) per chunk (B rows
    // past the tile's TN read zeros into LDS rows nothing reads)
    const int srow = t >> 1, sh = t & 1;
    const uint32_t oa0 = m0 + srow < M ? (uint32_t)(((int64_t)(m0 + srow) * 16 + 8 * sh) * 2) : XS_OOB;
    const uint32_t ob0 =
        (srow < TN && n0 + srow < N) ? (uint32_t)(((int64_t)(n0 + srow) * 16 + 8 * sh) * 2) : XS_OOB;
    const uint32_t pa = (uint32_t)(a_plane * 2), pb = (uint32_t)(b_plane * 2);
    const uint32_t sa = (uint32_t)(a_plane / kp * 32), sb = (uint32_t)(b_plane / kp * 32);  // one chunk slab
    const int so = xs_off(srow, sh);
    const int T = kp / 16;
    auto gload = [&](XpGemmRegs& R, int g) {  // unconditional (gemm_nt_x3s_kernel's): a chunk past K reads zeros
        const bool ina = oa0 != XS_OOB && g < T, inb = ob0 != XS_OOB && g < T;
#pragma unroll
        for (int p = 0; p < 3; ++p) {
            const auto va = __builtin_amdgcn_raw_buffer_load_b128(ra, ina ? oa0 + p * pa + g * sa : XS_OOB, 0, 0);
            const auto vb = __builtin_amdgcn_raw_buffer_load_b128(rb, inb ? ob0 + p * pb + g * sb : XS_OOB, 0, 0);
            R.a[p] = make_int4(va[0], va[1], va[2], va[3]);
            R.b[p] = make_int4(vb[0], vb[1], vb[2], vb[3]);
        }
    };
    auto sstore = [&](const XpGemmRegs& R, int stage) {
        unsigned char* As = gp_smem + stage * XS_STAGE;
        unsigned char* Bs = As + 3 * XS_PLANE;
#pragma unroll
        for (int p = 0; p < 3; ++p) {
            *reinterpret_cast<int4*>(As + p * XS_PLANE + so) = R.a[p];
            *reinterpret_cast<int4*>(Bs + p * XS_PLANE + so) = R.b[p];
        }
    };
    f32x16 acc[2][JN];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < JN; ++j)
#pragma unroll
            for (int r2 = 0; r2 < 16; ++r2) acc[i][j][r2] = 0.f;
    auto compute = [&](int stage) {  // gemm_nt_x3s_kernel's
        const unsigned char* As = gp_smem + stage * XS_STAGE;
        const unsigned char* Bs = As + 3 * XS_PLANE;
        bf16x8 a[2][3];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int o = xs_off(wr * 64 + i * 32 + col, half);
#pragma unroll
            for (int pl = 0; pl < 3; ++pl) a[i][pl] = *reinterpret_cast<const bf16x8*>(As + pl * XS_PLANE + o);
        }
#pragma unroll
        for (int j = 0; j < JN; ++j) {
            const int o = xs_off(wc * 32 * JN + j * 32 + col, half);
            bf16x8 bb[3];
#pragma unroll
            for (int pl = 0; pl < 3; ++pl) bb[pl] = *reinterpret_cast<const bf16x8*>(Bs + pl * XS_PLANE + o);
#pragma unroll
            for (int q = 0; q < 6; ++q)
#pragma unroll
                for (int i = 0; i < 2; ++i)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][kX3A[q]], bb[kX3B[q]], acc[i][j], 0, 0, 0);
        }
    };
    // one step: multiply stage g % 2, store chunk g + 1 into the other stage, load chunk g + 3. The stores and
    // loads are placed among the MFMAs (one store + one load per 4 MFMAs after the first B fragment's 12): 596 ->
    // 568 us at C5 against the compiler's order (MFMAs first, then the stores and loads; profiles/r05_x3p_sched_ab.txt;
    // an s_setprio(1) around the step on top measured the same). The last step's store lands in a stage nothing
    // reads again.
    bf16x8 ko_a[2][3], ko_b[3];  // KGE_X3P_KO bit 3: loop-invariant fragments
    auto step = [&](int g, XpGemmRegs& nxt) {
        if constexpr (KGE_X3P_KO & 8) {
#pragma unroll
            for (int j = 0; j < JN; ++j)
#pragma unroll
                for (int q = 0; q < 6; ++q)
#pragma unroll
                    for (int i = 0; i < 2; ++i)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ko_a[i][kX3A[q]], ko_b[kX3B[q]], acc[i][j],
                                                                            0, 0, 0);
        } else {
            compute(g & 1);
        }
        if constexpr (!(KGE_X3P_KO & 2)) sstore(nxt, (g + 1) & 1);
        if constexpr (!(KGE_X3P_KO & 4)) gload(nxt, g + 3);
        __builtin_amdgcn_sched_group_barrier(0x100, 9, 0);  // DS reads: the A fragments and B fragment 0
        __builtin_amdgcn_sched_group_barrier(0x008, 12, 0); // MFMA
        constexpr int WPJ = 6 / (JN - 1);  // the 6 stores and 6 loads spread over the later B fragments
#pragma unroll
        for (int j = 1; j < JN; ++j) {
            __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);  // B fragment j
#pragma unroll
            for (int u = 0; u < WPJ; ++u) {
                __builtin_amdgcn_sched_group_barrier(0x008, 12 / (WPJ + 1), 0);
                __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);  // DS write
                __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM read
            }
            __builtin_amdgcn_sched_group_barrier(0x008, 12 - WPJ * (12 / (WPJ + 1)), 0);
        }
        if constexpr (!(KGE_X3P_KO & 1)) __syncthreads();
    };
    XpGemmRegs R0, R1;
    gload(R0, 0);
    gload(R1, 1);
    sstore(R0, 0);
    gload(R0, 2);
    __syncthreads();
    if constexpr (KGE_X3P_KO & 8) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int pl = 0; pl < 3; ++pl)
                ko_a[i][pl] = *reinterpret_cast<const bf16x8*>(gp_smem + pl * XS_PLANE + xs_off(wr * 64 + i * 32 + col, half));
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
            ko_b[pl] = *reinterpret_cast<const bf16x8*>(gp_smem + 3 * XS_PLANE + pl * XS_PLANE + xs_off(wc * 32 * JN + col, half));
    }
    int g = 0;
    for (; g + 1 < T; g += 2) {
        step(g, R1);
        step(g + 1, R0);
    }
    if (g < T) step(g, R1);
    if constexpr (CNT) {
        // per query row: how many of this block's columns score above the row's truth (ties and NaN never
        // count; the truth's own column scores exactly ts, so it does not count either)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int lr = wr * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
                const float tv = m0 + lr < M ? ts[m0 + lr] : INFINITY;
                int c = 0;
#pragma unroll
                for (int j = 0; j < JN; ++j) {
                    const int gn = n0 + wc * 32 * JN + j * 32 + col;
                    const uint64_t bal = __ballot(gn < N && acc[i][j][r] > tv);
                    c += __popcll(half ? (bal >> 32) : (bal & 0xFFFFFFFFull));
                }
                if (col == 0 && c) atomicAdd(&rowcnt[lr], c);
            }
        __syncthreads();
        if (t < XS_T && rowcnt[t] && m0 + t < M) atomicAdd(&gcnt[m0 + t], rowcnt[t]);
        return;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < JN; ++j) {
            const int gn = n0 + wc * 32 * JN + j * 32 + col;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int gm = m0 + wr * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
                if (gm < M && gn < N) C[(int64_t)gm * ldc + gn] = acc[i][j][r];
            }
        }
}

// ---------------------------------------------------------------------------------------------
// The plane GEMM with LDS-DMA staging (round 6, form 4): gemm_nt_x3p_kernel's tile, waves, fragments, products and
// epilogue, with each chunk's six planes (A and B, 3 x 8 KB each) copied global -> LDS by `buffer_load_dwordx4 ...
// lds` (one 1-KB wave-instruction per plane: the LDS image of a wave's 32 rows is lane-linear, so xs_off's swizzle
// is put on the SOURCE address: lane L of row r loads half (L & 1) ^ ((r >> 3) & 1)). No staging registers, no
// ds_write pass: a knock-out build of gemm_nt_x3p_kernel without its stores and loads ran 483 against 572 us at
// C5's shape (profiles/r06_x3p_knockout.txt).
//   * three LDS stages (144 KB, static objects so the compiler's LDS-DMA wait tracking tells them apart); step g
//     issues chunk g + 2's copies into the stage step g - 1 multiplied, multiplies stage g % 3, waits for chunk
//     g + 1's copies (counted vmcnt: chunk g + 2's six stay in flight) and meets the others at a raw s_barrier
//     (a __syncthreads() fence would drain every copy in flight);
//   * the loop is unrolled by 3 so that every stage access names its object.
// Per accumulator the same products in the same order: C (and the counts) bitwise gemm_nt_x3p_kernel<.., 4>'s.
// ---------------------------------------------------------------------------------------------
typedef __attribute__((address_space(3))) void* xl_lds_t;

template <bool CNT>
__global__ __attribute__((amdgpu_flat_work_group_size(1, 512), amdgpu_waves_per_eu(2))) void gemm_nt_x3l_kernel(
    const __bf16* __restrict__ Ap, int64_t a_plane, const __bf16* __restrict__ Bp, int64_t b_plane, int kp,
    float* __restrict__ C, int M, int N, int64_t ldc, const float* __restrict__ ts, int* __restrict__ gcnt) {
    __shared__ __attribute__((aligned(16))) unsigned char xl0[XS_STAGE];
    __shared__ __attribute__((aligned(16))) unsigned char xl1[XS_STAGE];
    __shared__ __attribute__((aligned(16))) unsigned char xl2[XS_STAGE];
    __shared__ int rowcnt[CNT ? XS_T : 1];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    if constexpr (CNT) {
        if (t < XS_T) rowcnt[t] = 0;  // visible after the prologue's barrier
    }
    const int half = lane >> 5, col = lane & 31;
    const int wr = wave >> 1, wc = wave & 1;
    const int ntn = (N + XS_T - 1) / XS_T, ntm = (M + XS_T - 1) / XS_T;
    const int nblk = ntn * ntm;
    int bid = blockIdx.x;
    {  // XCD-aware bijective remap (gemm_nt_x3s_kernel's)
        const int q = nblk / 8, r = nblk % 8, x = bid % 8;
        bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
    }
    const int tn = bid / ntm, tm = bid % ntm;
    const int m0 = tm * XS_T, n0 = tn * XS_T;
    const rsrc_t ra = make_rsrc(Ap, (uint32_t)(3 * a_plane * 2));
    const rsrc_t rb = make_rsrc(Bp, (uint32_t)(3 * b_plane * 2));
    // lane t writes LDS bytes [16 t, 16 t + 16) of each plane image: row t >> 1, slot t & 1, which holds the row's
    // k half (t & 1) ^ ((row >> 3) & 1) (xs_off's swizzle, applied at the source)
    const int srow = t >> 1, sh = (t & 1) ^ ((srow >> 3) & 1);
    const uint32_t oa0 = m0 + srow < M ? (uint32_t)(((int64_t)(m0 + srow) * 16 + 8 * sh) * 2) : XS_OOB;
    const uint32_t ob0 = n0 + srow < N ? (uint32_t)(((int64_t)(n0 + srow) * 16 + 8 * sh) * 2) : XS_OOB;
    const uint32_t pa = (uint32_t)(a_plane * 2), pb = (uint32_t)(b_plane * 2);
    const uint32_t sa = (uint32_t)(a_plane / kp * 32), sb = (uint32_t)(b_plane / kp * 32);  // one chunk slab
    const int T = kp / 16;
    const int wo = wave * 1024;  // this wave's 1-KB piece of every plane image
    auto dma = [&](unsigned char* S, int g) {  // chunk g's six planes into stage S (past K: out of range, unread)
        const bool ina = oa0 != XS_OOB && g < T, inb = ob0 != XS_OOB && g < T;
#pragma unroll
        for (int p = 0; p < 3; ++p) {
            __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (xl_lds_t)(S + p * XS_PLANE + wo), 16,
                                                     ina ? oa0 + p * pa + g * sa : XS_OOB, 0, 0, 0);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (xl_lds_t)(S + (3 + p) * XS_PLANE + wo), 16,
                                                     inb ? ob0 + p * pb + g * sb : XS_OOB, 0, 0, 0);
        }
    };
    f32x16 acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r2 = 0; r2 < 16; ++r2) acc[i][j][r2] = 0.f;
    auto compute = [&](const unsigned char* As) {  // gemm_nt_x3p_kernel's
        const unsigned char* Bs = As + 3 * XS_PLANE;
        bf16x8 a[2][3];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int o = xs_off(wr * 64 + i * 32 + col, half);
#pragma unroll
            for (int pl = 0; pl < 3; ++pl) a[i][pl] = *reinterpret_cast<const bf16x8*>(As + pl * XS_PLANE + o);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int o = xs_off(wc * 128 + j * 32 + col, half);
            bf16x8 bb[3];
#pragma unroll
            for (int pl = 0; pl < 3; ++pl) bb[pl] = *reinterpret_cast<const bf16x8*>(Bs + pl * XS_PLANE + o);
#pragma unroll
            for (int q = 0; q < 6; ++q)
#pragma unroll
                for (int i = 0; i < 2; ++i)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][kX3A[q]], bb[kX3B[q]], acc[i][j], 0, 0, 0);
        }
    };
    // step g: copies of chunk g + 2 into N2 (multiplied at step g - 1, released by that step's barrier), multiply
    // Cur, then wait until chunk g + 1's copies (issued at step g - 1) have landed: 6 copies stay in flight
    auto step = [&](int g, const unsigned char* Cur, unsigned char* N2) {
        dma(N2, g + 2);
        __builtin_amdgcn_sched_barrier(0);  // the copies first: a full step for them to land
        compute(Cur);
        asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
    };
    dma(xl0, 0);
    dma(xl1, 1);
    asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    int g = 0;
    for (; g + 2 < T; g += 3) {
        step(g, xl0, xl2);
        step(g + 1, xl1, xl0);
        step(g + 2, xl2, xl1);
    }
    if (g < T) step(g, xl0, xl2);
    if (g + 1 < T) step(g + 1, xl1, xl0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // nothing in flight past the loop (copies of chunks >= T)
    if constexpr (CNT) {
        // gemm_nt_x3p_kernel's count epilogue
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int lr = wr * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
                const float tv = m0 + lr < M ? ts[m0 + lr] : INFINITY;
                int c = 0;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int gn = n0 + wc * 128 + j * 32 + col;
                    const uint64_t bal = __ballot(gn < N && acc[i][j][r] > tv);
                    c += __popcll(half ? (bal >> 32) : (bal & 0xFFFFFFFFull));
                }
                if (col == 0 && c) atomicAdd(&rowcnt[lr], c);
            }
        __syncthreads();
        if (t < XS_T && rowcnt[t] && m0 + t < M) atomicAdd(&gcnt[m0 + t], rowcnt[t]);
        return;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int gn = n0 + wc * 128 + j * 32 + col;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int gm = m0 + wr * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
                if (gm < M && gn < N) C[(int64_t)gm * ldc + gn] = acc[i][j][r];
            }
        }
}

// ---------------------------------------------------------------------------------------------
// The plane GEMM with B's fragments loaded straight into registers (round 6). gemm_nt_x3p_kernel stages both
// operands through LDS in 16-k chunks with one barrier per chunk, and each B fragment is read from LDS by the four
// waves of its column half (MFMA busy 0.72). Here each of the 8 waves of a 256 x 256 tile owns 32
// columns and all 256 rows: its B fragments (one 32-column tile) are read by no other wave, so they are loaded
// once per block straight from the chunk-major planes (1 KB contiguous per wave-instruction, one stage ahead) and
// never touch LDS; A (8 row tiles, shared by every wave) is staged, 32 k per stage (48 KB, two stages), so there
// is one barrier per 32 k. Per accumulator the products, their order (chunk by chunk; kX3A / kX3B within a chunk)
// and C are bitwise gemm_nt_x3p_kernel's.
// ---------------------------------------------------------------------------------------------
constexpr int XD_CH = 2;                        // 16-k chunks per stage
constexpr int XD_STAGE = XD_CH * 3 * XS_PLANE;  // A only: 2 chunks x 3 planes x 256 rows x 32 B = 48 KB

struct XdARegs {
    int4 a[XD_CH * 3];
};
struct XdBRegs {
    bf16x8 b[XD_CH][3];
};

__global__ __attribute__((amdgpu_flat_work_group_size(1, 512), amdgpu_waves_per_eu(2))) void gemm_nt_x3d_kernel(
    const __bf16* __restrict__ Ap, int64_t a_plane, const __bf16* __restrict__ Bp, int64_t b_plane, int kp,
    float* __restrict__ C, int M, int N, int64_t ldc) {
    extern __shared__ __attribute__((aligned(16))) unsigned char gd_smem[];  // 2 stages of A
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int half = lane >> 5, col = lane & 31;
    const int ntn = (N + XS_T - 1) / XS_T, ntm = (M + XS_T - 1) / XS_T;
    const int nblk = ntn * ntm;
    int bid = blockIdx.x;
    {  // XCD-aware bijective remap (gemm_nt_x3s_kernel's): each XCD walks a contiguous run of B tiles
        const int q = nblk / 8, r = nblk % 8, x = bid % 8;
        bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
    }
    const int tn = bid / ntm, tm = bid % ntm;
    const int m0 = tm * XS_T, n0 = tn * XS_T;
    const rsrc_t ra = make_rsrc(Ap, (uint32_t)(3 * a_plane * 2));
    const rsrc_t rb = make_rsrc(Bp, (uint32_t)(3 * b_plane * 2));
    const int T = kp / 16;            // 16-k chunks
    const int S = (T + XD_CH - 1) / XD_CH;  // stages
    const uint32_t pa = (uint32_t)(a_plane * 2), pb = (uint32_t)(b_plane * 2);
    const uint32_t sa = (uint32_t)(a_plane / kp * 32), sb = (uint32_t)(b_plane / kp * 32);  // one chunk slab
    // A staging: thread t takes row t >> 1, k half t & 1 of every (chunk, plane) piece of the stage
    const int srow = t >> 1, sh = t & 1;
    const uint32_t oa0 = m0 + srow < M ? (uint32_t)(((int64_t)(m0 + srow) * 16 + 8 * sh) * 2) : XS_OOB;
    const int so = xs_off(srow, sh);
    // B fragment of this lane: column n0 + 32 wave + col, k half `half` of each chunk
    const int bn = n0 + wave * 32 + col;
    const uint32_t ob0 = bn < N ? (uint32_t)(((int64_t)bn * 16 + 8 * half) * 2) : XS_OOB;
    auto gload_a = [&](XdARegs& R, int s) {  // a chunk past K reads zeros (and is never multiplied)
#pragma unroll
        for (int c = 0; c < XD_CH; ++c) {
            const int g = s * XD_CH + c;
            const bool in = oa0 != XS_OOB && g < T;
#pragma unroll
            for (int p = 0; p < 3; ++p) {
                const auto v = __builtin_amdgcn_raw_buffer_load_b128(ra, in ? oa0 + p * pa + g * sa : XS_OOB, 0, 0);
                R.a[c * 3 + p] = make_int4(v[0], v[1], v[2], v[3]);
            }
        }
    };
    auto sstore_a = [&](const XdARegs& R, int stage) {
        unsigned char* As = gd_smem + stage * XD_STAGE;
#pragma unroll
        for (int i = 0; i < XD_CH * 3; ++i) *reinterpret_cast<int4*>(As + i * XS_PLANE + so) = R.a[i];
    };
    auto gload_b = [&](XdBRegs& R, int s) {
#pragma unroll
        for (int c = 0; c < XD_CH; ++c) {
            const int g = s * XD_CH + c;
            const bool in = ob0 != XS_OOB && g < T;
#pragma unroll
            for (int p = 0; p < 3; ++p) {
                const auto v = __builtin_amdgcn_raw_buffer_load_b128(rb, in ? ob0 + p * pb + g * sb : XS_OOB, 0, 0);
                R.b[c][p] = __builtin_bit_cast(bf16x8, v);
            }
        }
    };
    f32x16 acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int r2 = 0; r2 < 16; ++r2) acc[i][r2] = 0.f;
    auto compute = [&](int stage, const XdBRegs& Bf, int s) {
        const unsigned char* As = gd_smem + stage * XD_STAGE;
#pragma unroll
        for (int c = 0; c < XD_CH; ++c) {
            if (s * XD_CH + c >= T) break;  // block-uniform: the last stage of an odd chunk count
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int o = xs_off(i * 32 + col, half);
                bf16x8 a[3];
#pragma unroll
                for (int pl = 0; pl < 3; ++pl) a[pl] = *reinterpret_cast<const bf16x8*>(As + (c * 3 + pl) * XS_PLANE + o);
#pragma unroll
                for (int q = 0; q < 6; ++q)
                    acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[kX3A[q]], Bf.b[c][kX3B[q]], acc[i], 0, 0, 0);
            }
        }
    };
    // one stage: B of the next stage requested first (its latency under this stage's MFMAs), A of this stage
    // multiplied from LDS, A of the next stage (in registers since the stage before) stored into the other LDS
    // stage, A of the stage after it requested
    XdARegs RA;
    XdBRegs B0, B1;
    gload_a(RA, 0);
    gload_b(B0, 0);
    sstore_a(RA, 0);
    gload_a(RA, 1);
    __syncthreads();
    auto step = [&](int s, const XdBRegs& Bc, XdBRegs& Bn) {
        gload_b(Bn, s + 1);
        compute(s & 1, Bc, s);
        sstore_a(RA, (s + 1) & 1);
        gload_a(RA, s + 2);
        __syncthreads();
    };
    int s = 0;
    for (; s + 1 < S; s += 2) {
        step(s, B0, B1);
        step(s + 1, B1, B0);
    }
    if (s < S) step(s, B0, B1);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int gm = m0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
            if (gm < M && bn < N) C[(int64_t)gm * ldc + bn] = acc[i][r];
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Filtered ranks without the score matrix (kge_eval_rank_planes, round 6). rank_kernel reads back the whole
// [M, N] score matrix the GEMM wrote (4 096 x 14 951 floats = 245 MB written and read per C5 batch). Here:
//   1. pair_dot_x3_kernel: the scores of the pairs a rank compares against, (q, truth[q]) and every filter entry
//      (q, f), each as the diagonal of one 32 x 32 MFMA tile whose row p is pair p's query row and column p its
//      entity row: the same planes, chunks and six products in the same order as the GEMM's element (q, e), so
//      bitwise its value (tests/test_eval_gpu.py checks that against the materialised scores);
//   2. gemm_nt_x3p_kernel<true>: the GEMM, counting per row the scores above the truth's;
//   3. rank_finish_kernel: rank = 1 + count - #{filter entries f != truth scoring above the truth}: rank_kernel's
//      rank exactly.
// ---------------------------------------------------------------------------------------------
// One wave per block (a C5 batch has ~4 100 pairs: 130 waves, each on a CU of its own) and 14 of its 16-k chunks of
// loads in flight: a wave's 63 chunks x 6 MFMAs are one dependent chain, so the loads must run far ahead of it (6
// chunks in flight and 4-wave blocks: 42.5 us per C5 batch, latency-bound).
constexpr int kPairDepth = 14;

__global__ __launch_bounds__(kWave) void pair_dot_x3_kernel(const __bf16* __restrict__ Ap, int64_t a_rows,
                                                             const __bf16* __restrict__ Bp, int64_t b_rows, int kp,
                                                             int64_t M, int64_t N, const int64_t* __restrict__ truth,
                                                             const int64_t* __restrict__ fptr,
                                                             const int64_t* __restrict__ fids, int64_t F,
                                                             float* __restrict__ ts, float* __restrict__ fs,
                                                             int* __restrict__ gcnt) {
    const int lane = threadIdx.x & 63, half = lane >> 5, col = lane & 31;
    for (int64_t i = (int64_t)blockIdx.x * kWave + lane; i < M; i += (int64_t)gridDim.x * kWave) gcnt[i] = 0;
    const int64_t p0 = (int64_t)blockIdx.x * 32;
    if (p0 >= M + F) return;  // wave-uniform
    const int64_t p = p0 + col;
    int64_t q = 0, e = -1;
    if (p < M) {
        q = p;
        e = truth[p];
    } else if (p < M + F) {
        const int64_t j = p - M;
        e = fids[j];
        int64_t lo = 0, hi = M;  // the query whose filter range holds j: the last q with fptr[q] <= j
        while (hi - lo > 1) {
            const int64_t mid = (lo + hi) >> 1;
            if (fptr[mid] <= j) lo = mid; else hi = mid;
        }
        q = lo;
    }
    const bool ev = e >= 0 && e < N;
    const int64_t a_plane = a_rows * kp, b_plane = b_rows * kp;
    const rsrc_t ra = make_rsrc(Ap, (uint32_t)(3 * a_plane * 2)), rb = make_rsrc(Bp, (uint32_t)(3 * b_plane * 2));
    const uint32_t oa = (uint32_t)((q * 16 + 8 * half) * 2), ob = (uint32_t)(((ev ? e : 0) * 16 + 8 * half) * 2);
    const uint32_t sa = (uint32_t)(a_rows * 32), sb = (uint32_t)(b_rows * 32);  // one chunk slab
    const uint32_t pa = (uint32_t)(a_plane * 2), pb = (uint32_t)(b_plane * 2);
    const int T = kp / 16;
    bf16x8 av[kPairDepth][3], bv[kPairDepth][3];
    auto load = [&](int slot, int g) {  // a chunk past K reads zeros (never multiplied)
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) {
            av[slot][pl] = __builtin_bit_cast(
                bf16x8, __builtin_amdgcn_raw_buffer_load_b128(ra, g < T ? oa + pl * pa + g * sa : XS_OOB, 0, 0));
            bv[slot][pl] = __builtin_bit_cast(
                bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rb, g < T ? ob + pl * pb + g * sb : XS_OOB, 0, 0));
        }
    };
    f32x16 acc;
#pragma unroll
    for (int r2 = 0; r2 < 16; ++r2) acc[r2] = 0.f;
#pragma unroll
    for (int s = 0; s < kPairDepth; ++s) load(s, s);
    for (int g0 = 0; g0 < T; g0 += kPairDepth) {
#pragma unroll
        for (int s = 0; s < kPairDepth; ++s) {
            if (g0 + s < T) {  // wave-uniform
#pragma unroll
                for (int q6 = 0; q6 < 6; ++q6)
                    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[s][kX3A[q6]], bv[s][kX3B[q6]], acc, 0, 0, 0);
            }
            load(s, g0 + s + kPairDepth);
        }
    }
    // the diagonal: pair c's score is row c, column c of the tile, held by the lane of column c in the half whose
    // rows hold c (rows 8 (r >> 2) + 4 half + (r & 3))
    if (half == ((col >> 2) & 1)) {
        float v = 0.f;
        const int rr = 4 * (col >> 3) + (col & 3);
#pragma unroll
        for (int r2 = 0; r2 < 16; ++r2)
            if (r2 == rr) v = acc[r2];
        if (p < M)
            ts[p] = ev ? v : -INFINITY;  // rank_kernel's score of an out-of-range truth
        else if (p < M + F)
            fs[p - M] = v;
    }
}

__global__ __launch_bounds__(kBlock) void rank_finish_kernel(int64_t M, int64_t N, const int64_t* __restrict__ truth,
                                                             const int64_t* __restrict__ fptr,
                                                             const int64_t* __restrict__ fids,
                                                             const float* __restrict__ ts, const float* __restrict__ fs,
                                                             const int* __restrict__ gcnt, int64_t* __restrict__ ranks) {
    const int64_t q = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (q >= M) return;
    const int lane = threadIdx.x & 63;
    const int64_t tr = truth[q];
    const float st = ts[q];
    int sub = 0;
    if (fptr)
        for (int64_t i = fptr[q] + lane; i < fptr[q + 1]; i += kWave) {
            const int64_t f = fids[i];
            if (f >= 0 && f < N && f != tr && fs[i] > st) ++sub;
        }
    for (int o = 32; o > 0; o >>= 1) sub += __shfl_xor(sub, o, kWave);
    if (lane == 0) ranks[q] = 1 + (int64_t)gcnt[q] - sub;
}

}  // namespace

int launch_gemm_nt_f32x3(const float* A, const float* B, float* C, int M, int N, int K, int64_t lda, int64_t ldb,
                         int64_t ldc, hipStream_t st, int form) {
    // the split-once kernel when its 32-bit buffer offsets cover both operands and its rows take float4 loads;
    // form 1 (kge_forms.gemm_form) keeps gemm_nt_f32x3_kernel, which splits each fragment in registers (a
    // SIMD-partner stagger, waves 4-7 storing before multiplying, measured no faster: profiles/r05_stagger_ab.txt)
    if (form != 1 && (int64_t)M * lda * 4 < (int64_t)XS_OOB && (int64_t)N * ldb * 4 < (int64_t)XS_OOB &&
        K % 4 == 0 && lda % 4 == 0 && ldb % 4 == 0 && ((uintptr_t)A & 15) == 0 && ((uintptr_t)B & 15) == 0) {
        static const bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_nt_x3s_kernel),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, 2 * XS_STAGE) == hipSuccess;
        (void)attr;
        const int64_t tiles = (int64_t)((M + XS_T - 1) / XS_T) * ((N + XS_T - 1) / XS_T);
        hipLaunchKernelGGL(gemm_nt_x3s_kernel, dim3((unsigned)tiles), dim3(512), 2 * XS_STAGE, st, A, B, C, M, N, K, lda,
                           ldb, ldc);
        return 0;
    }
    const int64_t tiles = (int64_t)((M + XBM - 1) / XBM) * ((N + XBM - 1) / XBM);
    hipLaunchKernelGGL(gemm_nt_f32x3_kernel, dim3((unsigned)tiles), dim3(kBlock), 0, st, A, B, C, M, N, K, lda, ldb,
                       ldc);
    return 0;
}

int launch_split3_planes(const float* X, int64_t rows, int64_t cols, int64_t ld, void* planes, int64_t plane_rows,
                         hipStream_t st) {
    const int kp = (int)((cols + 15) / 16 * 16);
    const int64_t q = rows * (kp / 4);
    hipLaunchKernelGGL(split3_planes_kernel, dim3((unsigned)((q + kBlock - 1) / kBlock)), dim3(kBlock), 0, st, X, rows,
                       (int)cols, ld, kp, static_cast<__bf16*>(planes), plane_rows * kp);
    return 0;
}

template <bool CNT, int JN>
void launch_x3p(const void* Ap, int64_t a_rows, const void* Bp, int64_t b_rows, int kp, float* C, int64_t ldc, int M,
                int N, const float* ts, int* gcnt, hipStream_t st) {
    static const bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_nt_x3p_kernel<CNT, JN>),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, 2 * XS_STAGE) == hipSuccess;
    (void)attr;
    const int64_t tiles = (int64_t)((M + XS_T - 1) / XS_T) * ((N + 64 * JN - 1) / (64 * JN));
    hipLaunchKernelGGL((gemm_nt_x3p_kernel<CNT, JN>), dim3((unsigned)tiles), dim3(512), 2 * XS_STAGE, st,
                       static_cast<const __bf16*>(Ap), a_rows * kp, static_cast<const __bf16*>(Bp), b_rows * kp, kp, C, M,
                       N, ldc, ts, gcnt);
}

template <bool CNT>
void launch_x3l(const void* Ap, int64_t a_rows, const void* Bp, int64_t b_rows, int kp, float* C, int64_t ldc, int M,
                int N, const float* ts, int* gcnt, hipStream_t st) {
    const int64_t tiles = (int64_t)((M + XS_T - 1) / XS_T) * ((N + XS_T - 1) / XS_T);
    hipLaunchKernelGGL((gemm_nt_x3l_kernel<CNT>), dim3((unsigned)tiles), dim3(512), 0, st,
                       static_cast<const __bf16*>(Ap), a_rows * kp, static_cast<const __bf16*>(Bp), b_rows * kp, kp, C, M,
                       N, ldc, ts, gcnt);
}

int launch_gemm_nt_x3p(const void* Ap, int64_t a_rows, const void* Bp, int64_t b_rows, int64_t K, float* C, int64_t ldc,
                       int M, int N, hipStream_t st, int form) {
    const int kp = (int)((K + 15) / 16 * 16);
    const int64_t tiles = (int64_t)((M + XS_T - 1) / XS_T) * ((N + XS_T - 1) / XS_T);
    if (form == 4) {  // LDS-DMA staging, three stages
        launch_x3l<false>(Ap, a_rows, Bp, b_rows, kp, C, ldc, M, N, nullptr, nullptr, st);
        return 0;
    }
    if (form == 3) {  // 256 x 192 block tiles
        launch_x3p<false, 3>(Ap, a_rows, Bp, b_rows, kp, C, ldc, M, N, nullptr, nullptr, st);
        return 0;
    }
    if (form == 2) {  // B straight into registers, A staged 32 k per barrier (gemm_nt_x3d_kernel)
        static const bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_nt_x3d_kernel),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, 2 * XD_STAGE) == hipSuccess;
        (void)attr;
        hipLaunchKernelGGL(gemm_nt_x3d_kernel, dim3((unsigned)tiles), dim3(512), 2 * XD_STAGE, st,
                           static_cast<const __bf16*>(Ap), a_rows * kp, static_cast<const __bf16*>(Bp), b_rows * kp, kp,
                           C, M, N, ldc);
        return 0;
    }
    launch_x3p<false, 4>(Ap, a_rows, Bp, b_rows, kp, C, ldc, M, N, nullptr, nullptr, st);
    return 0;
}

int64_t eval_rank_ws_bytes(int64_t M, int64_t F) { return ((M * 8 + 15) / 16 * 16) + ((F * 4 + 15) / 16 * 16); }

int launch_eval_rank_planes(const void* Ap, int64_t a_rows, const void* Bp, int64_t b_rows, int64_t K, int M, int N,
                            const int64_t* truth, const int64_t* fptr, const int64_t* fids, int64_t F, int64_t* ranks,
                            void* ws, hipStream_t st, int form, int phases) {
    const int kp = (int)((K + 15) / 16 * 16);
    float* ts = static_cast<float*>(ws);
    int* gcnt = reinterpret_cast<int*>(ts + M);
    float* fs = reinterpret_cast<float*>(static_cast<unsigned char*>(ws) + (((int64_t)M * 8 + 15) / 16 * 16));
    const int64_t pairs = (int64_t)M + F, waves = (pairs + 31) / 32;
    if (phases & 1)
        hipLaunchKernelGGL(pair_dot_x3_kernel, dim3((unsigned)waves), dim3(kWave), 0, st, static_cast<const __bf16*>(Ap),
                           a_rows, static_cast<const __bf16*>(Bp), b_rows, kp, (int64_t)M, (int64_t)N, truth, fptr, fids,
                           F, ts, fs, gcnt);
    if (phases & 2) {
        if (form == 4)
            launch_x3l<true>(Ap, a_rows, Bp, b_rows, kp, nullptr, 0, M, N, ts, gcnt, st);
        else if (form == 3)
            launch_x3p<true, 3>(Ap, a_rows, Bp, b_rows, kp, nullptr, 0, M, N, ts, gcnt, st);
        else
            launch_x3p<true, 4>(Ap, a_rows, Bp, b_rows, kp, nullptr, 0, M, N, ts, gcnt, st);
    }
    if (phases & 4)
        hipLaunchKernelGGL(rank_finish_kernel, dim3((unsigned)((M + kWavesPerBlock - 1) / kWavesPerBlock)), dim3(kBlock),
                           0, st, (int64_t)M, (int64_t)N, truth, fptr, fids, ts, fs, gcnt, ranks);
    return 0;
}

int launch_rank(const float* S, int64_t M, int64_t N, int64_t ld, const int64_t* truth, const int64_t* fptr,
                const int64_t* fids, int64_t* ranks, hipStream_t st) {
    hipLaunchKernelGGL(rank_kernel, dim3((unsigned)M), dim3(kBlock), 0, st, S, M, N, ld, truth, fptr, fids, ranks);
    return 0;
}

}  // namespace kge_impl
