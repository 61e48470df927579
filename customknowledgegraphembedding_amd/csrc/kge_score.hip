// kge_score.hip — fused gather + score kernels for knowledge-graph-embedding negative sampling on
// MI355X (gfx950, CDNA4), behind the C-ABI in include/kge_hip.h.
//
// What it replaces (reference, /root/reference):
//   tensorflow_codes/model.py:127-199  single/head-batch/tail-batch gathers (tf.gather) + model_func
//   tensorflow_codes/model.py:207-224  InterHT score
//   tensorflow_codes/model.py:168-171,195-198  self-adversarial per-row reduction (Q3)
//   KnowledgeGraphEmbedding/codes/model.py (absent; restated in oracle/kge_oracle.py):
//     TransE / DistMult / ComplEx / RotatE / pRotatE score functions and KGEModel.forward gathers.
//
// Work decomposition (forward and backward alike): one wave64 owns one batch row b and a run of
// `cpw` consecutive candidates of that row. The "query" side shared by every candidate of row b —
// (h, r) in tail-batch / single mode, (r, t) in head-batch mode — is built ONCE per wave and kept
// in VGPRs; each candidate row is then gathered straight from HBM into VGPRs with 16-B loads
// (lane l owns float4 groups l, l+64, l+128, ... of each half-row), two candidates in flight per
// wave, and reduced along the hidden dim by wave-wide butterflies. Nothing [B,N,d]-shaped is ever
// materialised: the HBM traffic is one read of every gathered row, the indices and the scores.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <string>
#include <math.h>

#include "kge_hip.h"

namespace {

// upstream RotatE uses pi = 3.14159265358979323846; upstream pRotatE has the literal
// 3.14159262358979323846 (sic) — both are kept as the reference has them (host side computes the
// fp32 phase divisor from them, see kge_abi.cpp).

constexpr int kWave = 64;
constexpr int kBlock = 256;
constexpr int kWavesPerBlock = kBlock / kWave;

template <int V>
struct alignas(4 * V) vecf {
    float a[V];
};

template <int V>
__device__ __forceinline__ vecf<V> vzero() {
    vecf<V> r;
#pragma unroll
    for (int i = 0; i < V; ++i) r.a[i] = 0.f;
    return r;
}

template <int V>
__device__ __forceinline__ vecf<V> vload(const float* p, bool ok) {
    if (ok) return *reinterpret_cast<const vecf<V>*>(p);
    return vzero<V>();
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
    return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
    return v;
}

__device__ __forceinline__ int64_t readlane64(int64_t v, int j) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(uint64_t)v, j);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), j);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ float readlanef(float v, int j) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), j));
}

__device__ __forceinline__ float sgnf(float x) { return (x > 0.f) ? 1.f : ((x < 0.f) ? -1.f : 0.f); }

// logsigmoid(x) = min(x,0) - log1p(exp(-|x|))   (tf.math.log_sigmoid, model.py:145,169)
__device__ __forceinline__ float log_sigmoid(float x) { return fminf(x, 0.f) - log1pf(expf(-fabsf(x))); }
__device__ __forceinline__ float sigmoidf(float x) {
    // stable for both signs
    if (x >= 0.f) return 1.f / (1.f + expf(-x));
    const float e = expf(x);
    return e / (1.f + e);
}

// ---------------------------------------------------------------------------------------------
// Parameters of one scoring launch. Rows are addressed as base + row * ld (floats).
//   query entity row of batch row b:  q_idx ? q_idx[b * q_stride] : b
//   relation row of batch row b:      r_idx ? r_idx[b * r_stride] : b      (+ r_off floats)
//   candidate n of batch row b:       c_idx ? c_idx[b * c_stride + n] : b * c_dense + n
// ---------------------------------------------------------------------------------------------
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
};

constexpr bool is_split(int fn) { return fn == KGE_COMPLEX || fn == KGE_ROTATE || fn == KGE_INTERHT; }
constexpr bool rel_split(int fn) { return fn == KGE_COMPLEX; }

// ---------------------------------------------------------------------------------------------
// Query side. CH = candidate is the head (head-batch); otherwise the candidate is the tail
// (tail-batch and single, which upstream scores with the same "else" branch).
//   q0,q1,q2: per-element query operands kept in VGPRs; zero on groups past D.
//   qa,qb:    raw query entity halves (kept for the backward chain rule)
//   ra,rb:    raw relation (halves for ComplEx)
//   na,nb:    InterHT query norms
// ---------------------------------------------------------------------------------------------
template <int FN, bool CH, int V, int G>
struct Query {
    vecf<V> q0[G], q1[G], q2[G];
    float na, nb;

    __device__ __forceinline__ void build(const float* qrow, bool qok, const float* rrow, bool rok,
                                          int D, int lane, const ScoreParams& p) {
        const int DV = D / V;
        vecf<V> ea[G], eb[G], ra[G], rb[G];
#pragma unroll
        for (int k = 0; k < G; ++k) {
            const int g = lane + k * kWave;
            const bool in = g < DV;
            const int e = g * V;
            ea[k] = vload<V>(qrow + e, qok && in);
            if constexpr (is_split(FN)) eb[k] = vload<V>(qrow + D + e, qok && in);
            ra[k] = vload<V>(rrow + e, rok && in);
            if constexpr (rel_split(FN)) rb[k] = vload<V>(rrow + D + e, rok && in);
        }
        na = nb = 0.f;
        if constexpr (FN == KGE_INTERHT) {
            float sa = 0.f, sb = 0.f;
#pragma unroll
            for (int k = 0; k < G; ++k)
#pragma unroll
                for (int i = 0; i < V; ++i) {
                    sa += ea[k].a[i] * ea[k].a[i];
                    sb += eb[k].a[i] * eb[k].a[i];
                }
            sa = wave_sum(sa);
            sb = wave_sum(sb);
            na = sqrtf(sa);
            nb = sqrtf(sb);
        }
#pragma unroll
        for (int k = 0; k < G; ++k) {
            const bool in = (lane + k * kWave) < DV;
#pragma unroll
            for (int i = 0; i < V; ++i) {
                const float x = ea[k].a[i], y = is_split(FN) ? eb[k].a[i] : 0.f;
                const float r = ra[k].a[i], s = rel_split(FN) ? rb[k].a[i] : 0.f;
                float o0 = 0.f, o1 = 0.f, o2 = 0.f;
                if constexpr (FN == KGE_TRANSE) {
                    // tail: (h + r) - t ; head: h + (r - t)
                    o0 = CH ? (r - x) : (x + r);
                } else if constexpr (FN == KGE_DISTMULT) {
                    // tail: (h * r) * t ; head: h * (r * t)
                    o0 = CH ? (r * x) : (x * r);
                } else if constexpr (FN == KGE_COMPLEX) {
                    if (!CH) {  // re_h*re_r - im_h*im_r ; re_h*im_r + im_h*re_r
                        o0 = x * r - y * s;
                        o1 = x * s + y * r;
                    } else {  // re_r*re_t + im_r*im_t ; re_r*im_t - im_r*re_t
                        o0 = r * x + s * y;
                        o1 = r * y - s * x;
                    }
                } else if constexpr (FN == KGE_ROTATE) {
                    const float ph = r / p.phase_div;
                    const float c = cosf(ph), sn = sinf(ph);
                    if (!CH) {  // re_h*re_r - im_h*im_r ; re_h*im_r + im_h*re_r
                        o0 = x * c - y * sn;
                        o1 = x * sn + y * c;
                    } else {  // re_r*re_t + im_r*im_t ; re_r*im_t - im_r*re_t
                        o0 = c * x + sn * y;
                        o1 = c * y - sn * x;
                    }
                    if (!in) o0 = o1 = 0.f;
                } else if constexpr (FN == KGE_PROTATE) {
                    const float pe = x / p.phase_div, pr = r / p.phase_div;
                    o0 = CH ? (pr - pe) : (pe + pr);
                } else if constexpr (FN == KGE_INTERHT) {
                    // query entity halves normalised (no epsilon, Q7), b-half shifted by u = 1
                    o0 = in ? x / na : 0.f;
                    o1 = in ? (y / nb + 1.f) : 0.f;
                    o2 = r;
                }
                q0[k].a[i] = o0;
                q1[k].a[i] = o1;
                q2[k].a[i] = o2;
            }
        }
    }
};

// Candidate registers: first half (or whole row) in ca, second half in cb.
template <int FN, int V, int G>
struct Cand {
    vecf<V> ca[G], cb[G];
    __device__ __forceinline__ void load(const float* row, bool ok, int D, int lane) {
        const int DV = D / V;
#pragma unroll
        for (int k = 0; k < G; ++k) {
            const int g = lane + k * kWave;
            const bool in = ok && g < DV;
            ca[k] = vload<V>(row + g * V, in);
            if constexpr (is_split(FN)) cb[k] = vload<V>(row + D + g * V, in);
        }
    }
};

// Forward score of one candidate held in registers (all lanes return the full score).
template <int FN, bool CH, int V, int G>
__device__ __forceinline__ float cand_score(const Cand<FN, V, G>& c, const Query<FN, CH, V, G>& q,
                                            const ScoreParams& p) {
    float acc = 0.f;
    if constexpr (FN == KGE_INTERHT) {
        float sa = 0.f, sb = 0.f;
#pragma unroll
        for (int k = 0; k < G; ++k)
#pragma unroll
            for (int i = 0; i < V; ++i) {
                sa += c.ca[k].a[i] * c.ca[k].a[i];
                sb += c.cb[k].a[i] * c.cb[k].a[i];
            }
        sa = wave_sum(sa);
        sb = wave_sum(sb);
        const float na = sqrtf(sa), nb = sqrtf(sb);
#pragma unroll
        for (int k = 0; k < G; ++k)
#pragma unroll
            for (int i = 0; i < V; ++i) {
                const float ah = c.ca[k].a[i] / na;        // normalised candidate a-half
                const float bh = c.cb[k].a[i] / nb + 1.f;  // normalised candidate b-half + u
                float x;
                if (CH)  // a_head * b_tail - a_tail * b_head + re_mid   (model.py:222)
                    x = ah * q.q1[k].a[i] - q.q0[k].a[i] * bh + q.q2[k].a[i];
                else
                    x = q.q0[k].a[i] * bh - ah * q.q1[k].a[i] + q.q2[k].a[i];
                acc += fabsf(x);
            }
        // groups past D: candidate zero-loaded, query zero -> x = 0 (bh = 1 * 0 query)
    } else {
#pragma unroll
        for (int k = 0; k < G; ++k)
#pragma unroll
            for (int i = 0; i < V; ++i) {
                const float x = c.ca[k].a[i];
                if constexpr (FN == KGE_TRANSE) {
                    acc += fabsf(CH ? (x + q.q0[k].a[i]) : (q.q0[k].a[i] - x));
                } else if constexpr (FN == KGE_DISTMULT) {
                    acc += CH ? (x * q.q0[k].a[i]) : (q.q0[k].a[i] * x);
                } else if constexpr (FN == KGE_COMPLEX) {
                    const float y = c.cb[k].a[i];
                    acc += CH ? (x * q.q0[k].a[i] + y * q.q1[k].a[i]) : (q.q0[k].a[i] * x + q.q1[k].a[i] * y);
                } else if constexpr (FN == KGE_ROTATE) {
                    const float y = c.cb[k].a[i];
                    const float xr = q.q0[k].a[i] - x, xi = q.q1[k].a[i] - y;
                    acc += sqrtf(xr * xr + xi * xi);
                } else if constexpr (FN == KGE_PROTATE) {
                    const float pc = x / p.phase_div;
                    acc += fabsf(sinf(CH ? (pc + q.q0[k].a[i]) : (q.q0[k].a[i] - pc)));
                }
            }
    }
    acc = wave_sum(acc);
    if constexpr (FN == KGE_DISTMULT || FN == KGE_COMPLEX) return acc;
    else if constexpr (FN == KGE_PROTATE) return p.gamma - acc * p.modulus;
    else return p.gamma - acc;
}

struct WaveTask {
    int64_t b, n0;
    int nc;
};

__device__ __forceinline__ bool wave_task(const ScoreParams& p, WaveTask& t) {
    const int64_t wid = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    t.b = wid / p.wpr;
    if (t.b >= p.B) return false;
    t.n0 = (wid - t.b * p.wpr) * (int64_t)p.cpw;
    if (t.n0 >= p.N) return false;
    t.nc = (int)min((int64_t)p.cpw, p.N - t.n0);
    return true;
}

template <int FN, bool CH, int V, int G>
__global__ __launch_bounds__(kBlock) void score_fwd_kernel(ScoreParams p) {
    WaveTask t;
    if (!wave_task(p, t)) return;
    const int lane = threadIdx.x & 63;

    const int64_t qi = p.q_idx ? p.q_idx[t.b * p.q_stride] : t.b;
    const int64_t ri = p.r_idx ? p.r_idx[t.b * p.r_stride] : t.b;
    const bool qok = qi >= 0 && qi < p.q_rows;
    const bool rok = ri >= 0 && ri < p.r_rows;
    Query<FN, CH, V, G> q;
    q.build(p.qent + (qok ? qi : 0) * p.q_ld, qok, p.rel + (rok ? ri : 0) * p.r_ld + p.r_off, rok, p.D, lane, p);

    int64_t my_id = 0;
    if (lane < t.nc) my_id = p.c_idx ? p.c_idx[t.b * p.c_stride + t.n0 + lane] : t.b * p.c_dense + t.n0 + lane;

    float my_score = 0.f;
    int j = 0;
    for (; j + 1 < t.nc; j += 2) {
        const int64_t c0 = readlane64(my_id, j), c1 = readlane64(my_id, j + 1);
        const bool ok0 = c0 >= 0 && c0 < p.c_rows, ok1 = c1 >= 0 && c1 < p.c_rows;
        Cand<FN, V, G> x0, x1;
        x0.load(p.cent + (ok0 ? c0 : 0) * p.c_ld, ok0, p.D, lane);
        x1.load(p.cent + (ok1 ? c1 : 0) * p.c_ld, ok1, p.D, lane);
        const float s0 = cand_score<FN, CH, V, G>(x0, q, p);
        const float s1 = cand_score<FN, CH, V, G>(x1, q, p);
        if (lane == j) my_score = s0;
        if (lane == j + 1) my_score = s1;
    }
    if (j < t.nc) {
        const int64_t c0 = readlane64(my_id, j);
        const bool ok0 = c0 >= 0 && c0 < p.c_rows;
        Cand<FN, V, G> x0;
        x0.load(p.cent + (ok0 ? c0 : 0) * p.c_ld, ok0, p.D, lane);
        const float s0 = cand_score<FN, CH, V, G>(x0, q, p);
        if (lane == j) my_score = s0;
    }
    if (lane < t.nc) p.out[t.b * p.out_ld + t.n0 + lane] = my_score;
}

// ---------------------------------------------------------------------------------------------
// Backward: recompute each candidate's per-element terms, scatter the candidate-row gradient with
// fp32 atomics, accumulate the query-side gradient in VGPRs over the wave's candidates and add it
// once per wave (atomics: query rows are shared across waves and batch rows).
// ---------------------------------------------------------------------------------------------
template <int V>
__device__ __forceinline__ void vatomic_add(float* dst, const vecf<V>& v, bool ok) {
    if (!ok) return;
#pragma unroll
    for (int i = 0; i < V; ++i) unsafeAtomicAdd(dst + i, v.a[i]);
}

template <int FN, bool CH, int V, int G>
__global__ __launch_bounds__(kBlock) void score_bwd_kernel(ScoreParams p) {
    WaveTask t;
    if (!wave_task(p, t)) return;
    const int lane = threadIdx.x & 63;
    const int D = p.D, DV = D / V;

    const int64_t qi = p.q_idx ? p.q_idx[t.b * p.q_stride] : t.b;
    const int64_t ri = p.r_idx ? p.r_idx[t.b * p.r_stride] : t.b;
    const bool qok = qi >= 0 && qi < p.q_rows;
    const bool rok = ri >= 0 && ri < p.r_rows;
    const float* qrow = p.qent + (qok ? qi : 0) * p.q_ld;
    const float* rrow = p.rel + (rok ? ri : 0) * p.r_ld + p.r_off;
    Query<FN, CH, V, G> q;
    q.build(qrow, qok, rrow, rok, D, lane, p);

    int64_t my_id = 0;
    float my_g = 0.f;
    if (lane < t.nc) {
        my_id = p.c_idx ? p.c_idx[t.b * p.c_stride + t.n0 + lane] : t.b * p.c_dense + t.n0 + lane;
        my_g = p.d_scores[t.b * p.d_ld + t.n0 + lane];
    }

    vecf<V> dq0[G], dq1[G], dq2[G];
#pragma unroll
    for (int k = 0; k < G; ++k) dq0[k] = dq1[k] = dq2[k] = vzero<V>();
    float dmod = 0.f;

    for (int j = 0; j < t.nc; ++j) {
        const int64_t ci = readlane64(my_id, j);
        const float g = readlanef(my_g, j);
        const bool ok = ci >= 0 && ci < p.c_rows;
        Cand<FN, V, G> c;
        c.load(p.cent + (ok ? ci : 0) * p.c_ld, ok, D, lane);
        vecf<V> dca[G], dcb[G];
        if constexpr (FN == KGE_INTERHT) {
            float sa = 0.f, sb = 0.f;
#pragma unroll
            for (int k = 0; k < G; ++k)
#pragma unroll
                for (int i = 0; i < V; ++i) {
                    sa += c.ca[k].a[i] * c.ca[k].a[i];
                    sb += c.cb[k].a[i] * c.cb[k].a[i];
                }
            sa = wave_sum(sa);
            sb = wave_sum(sb);
            const float na = sqrtf(sa), nb = sqrtf(sb);
            float dota = 0.f, dotb = 0.f;
#pragma unroll
            for (int k = 0; k < G; ++k)
#pragma unroll
                for (int i = 0; i < V; ++i) {
                    const float ah = c.ca[k].a[i] / na;
                    const float bn = c.cb[k].a[i] / nb;
                    const float bh = bn + 1.f;
                    const float q0 = q.q0[k].a[i], q1 = q.q1[k].a[i], q2 = q.q2[k].a[i];
                    float x, dah, dbn;
                    const bool in = (lane + k * kWave) < DV;
                    if (CH) {
                        x = ah * q1 - q0 * bh + q2;
                        const float Gx = in ? -g * sgnf(x) : 0.f;
                        dah = Gx * q1;
                        dbn = -Gx * q0;
                        dq1[k].a[i] += Gx * ah;
                        dq0[k].a[i] += -Gx * bh;
                        dq2[k].a[i] += Gx;
                    } else {
                        x = q0 * bh - ah * q1 + q2;
                        const float Gx = in ? -g * sgnf(x) : 0.f;
                        dah = -Gx * q1;
                        dbn = Gx * q0;
                        dq0[k].a[i] += Gx * bh;
                        dq1[k].a[i] += -Gx * ah;
                        dq2[k].a[i] += Gx;
                    }
                    dca[k].a[i] = dah;
                    dcb[k].a[i] = dbn;
                    dota += ah * dah;
                    dotb += bn * dbn;
                }
            dota = wave_sum(dota);
            dotb = wave_sum(dotb);
#pragma unroll
            for (int k = 0; k < G; ++k)
#pragma unroll
                for (int i = 0; i < V; ++i) {
                    const float ah = c.ca[k].a[i] / na;
                    const float bn = c.cb[k].a[i] / nb;
                    dca[k].a[i] = (dca[k].a[i] - ah * dota) / na;
                    dcb[k].a[i] = (dcb[k].a[i] - bn * dotb) / nb;
                }
        } else {
            float ysum = 0.f;
#pragma unroll
            for (int k = 0; k < G; ++k)
#pragma unroll
                for (int i = 0; i < V; ++i) {
                    const float x = c.ca[k].a[i];
                    const bool in = (lane + k * kWave) < DV;
                    float da = 0.f, db = 0.f;
                    if constexpr (FN == KGE_TRANSE) {
                        const float r = CH ? (x + q.q0[k].a[i]) : (q.q0[k].a[i] - x);
                        const float Gx = -g * sgnf(r);  // d/d(residual)
                        da = CH ? Gx : -Gx;
                        dq0[k].a[i] += Gx;
                    } else if constexpr (FN == KGE_DISTMULT) {
                        da = g * q.q0[k].a[i];
                        dq0[k].a[i] += g * x;
                    } else if constexpr (FN == KGE_COMPLEX) {
                        const float y = c.cb[k].a[i];
                        da = g * q.q0[k].a[i];
                        db = g * q.q1[k].a[i];
                        dq0[k].a[i] += g * x;
                        dq1[k].a[i] += g * y;
                    } else if constexpr (FN == KGE_ROTATE) {
                        const float y = c.cb[k].a[i];
                        const float xr = q.q0[k].a[i] - x, xi = q.q1[k].a[i] - y;
                        const float m = sqrtf(xr * xr + xi * xi);
                        const float fr = (m > 0.f) ? xr / m : 0.f, fi = (m > 0.f) ? xi / m : 0.f;
                        da = g * fr;
                        db = g * fi;
                        dq0[k].a[i] += -g * fr;
                        dq1[k].a[i] += -g * fi;
                    } else if constexpr (FN == KGE_PROTATE) {
                        const float pc = x / p.phase_div;
                        const float z = CH ? (pc + q.q0[k].a[i]) : (q.q0[k].a[i] - pc);
                        const float sz = sinf(z);
                        const float Gx = in ? -g * p.modulus * sgnf(sz) * cosf(z) : 0.f;
                        da = (CH ? Gx : -Gx) / p.phase_div;
                        dq0[k].a[i] += Gx;
                        ysum += in ? fabsf(sz) : 0.f;
                    }
                    dca[k].a[i] = in ? da : 0.f;
                    dcb[k].a[i] = in ? db : 0.f;
                }
            if constexpr (FN == KGE_PROTATE) dmod += -g * wave_sum(ysum);
        }
        // scatter the candidate-row gradient
        float* drow = p.d_cent + (ok ? ci : 0) * p.c_ld;
#pragma unroll
        for (int k = 0; k < G; ++k) {
            const int gi = lane + k * kWave;
            const bool in = ok && gi < DV;
            vatomic_add<V>(drow + gi * V, dca[k], in);
            if constexpr (is_split(FN)) vatomic_add<V>(drow + D + gi * V, dcb[k], in);
        }
    }

    // query-side chain rule -> raw query entity row (ge*) and relation row (gr*)
    float dna = 0.f, dnb = 0.f;
    if constexpr (FN == KGE_INTERHT) {
        // d(x/n) = (dy - y <y,dy>) / n  for both query halves (b-half: y = q1 - u)
        float da = 0.f, db = 0.f;
#pragma unroll
        for (int k = 0; k < G; ++k)
#pragma unroll
            for (int i = 0; i < V; ++i) {
                const bool in = (lane + k * kWave) < DV;
                da += q.q0[k].a[i] * dq0[k].a[i];
                db += (in ? q.q1[k].a[i] - 1.f : 0.f) * dq1[k].a[i];
            }
        dna = wave_sum(da);
        dnb = wave_sum(db);
    }
    float* dq_row = p.d_qent + (qok ? qi : 0) * p.q_ld;
    float* dr_row = p.d_rel + (rok ? ri : 0) * p.r_ld + p.r_off;
#pragma unroll
    for (int k = 0; k < G; ++k) {
        const int gi = lane + k * kWave;
        const bool in = gi < DV;
        const int e = gi * V;
        vecf<V> ea = vload<V>(qrow + e, qok && in), eb = vzero<V>(), ra = vload<V>(rrow + e, rok && in),
                rb = vzero<V>();
        if constexpr (is_split(FN)) eb = vload<V>(qrow + D + e, qok && in);
        if constexpr (rel_split(FN)) rb = vload<V>(rrow + D + e, rok && in);
        vecf<V> gea = vzero<V>(), geb = vzero<V>(), gra = vzero<V>(), grb = vzero<V>();
#pragma unroll
        for (int i = 0; i < V; ++i) {
            const float x = ea.a[i], y = eb.a[i], r = ra.a[i], s = rb.a[i];
            const float d0 = dq0[k].a[i], d1 = dq1[k].a[i], d2 = dq2[k].a[i];
            if constexpr (FN == KGE_TRANSE) {
                gea.a[i] = CH ? -d0 : d0;
                gra.a[i] = d0;
            } else if constexpr (FN == KGE_DISTMULT) {
                gea.a[i] = d0 * r;
                gra.a[i] = d0 * x;
            } else if constexpr (FN == KGE_COMPLEX) {
                if (!CH) {
                    gea.a[i] = d0 * r + d1 * s;
                    geb.a[i] = -d0 * s + d1 * r;
                    gra.a[i] = d0 * x + d1 * y;
                    grb.a[i] = -d0 * y + d1 * x;
                } else {
                    gea.a[i] = d0 * r - d1 * s;
                    geb.a[i] = d0 * s + d1 * r;
                    gra.a[i] = d0 * x + d1 * y;
                    grb.a[i] = d0 * y - d1 * x;
                }
            } else if constexpr (FN == KGE_ROTATE) {
                const float ph = r / p.phase_div;
                const float c = cosf(ph), sn = sinf(ph);
                const float Q0 = q.q0[k].a[i], Q1 = q.q1[k].a[i];
                float dth;
                if (!CH) {
                    gea.a[i] = d0 * c + d1 * sn;
                    geb.a[i] = -d0 * sn + d1 * c;
                    dth = -d0 * Q1 + d1 * Q0;
                } else {
                    gea.a[i] = d0 * c - d1 * sn;
                    geb.a[i] = d0 * sn + d1 * c;
                    dth = d0 * Q1 - d1 * Q0;
                }
                gra.a[i] = dth / p.phase_div;
            } else if constexpr (FN == KGE_PROTATE) {
                gea.a[i] = (CH ? -d0 : d0) / p.phase_div;
                gra.a[i] = d0 / p.phase_div;
            } else if constexpr (FN == KGE_INTERHT) {
                const float Q0 = q.q0[k].a[i];
                const float bn = in ? q.q1[k].a[i] - 1.f : 0.f;
                gea.a[i] = (d0 - Q0 * dna) / q.na;
                geb.a[i] = (d1 - bn * dnb) / q.nb;
                gra.a[i] = d2;
            }
            if (!in) gea.a[i] = geb.a[i] = gra.a[i] = grb.a[i] = 0.f;
        }
        vatomic_add<V>(dq_row + e, gea, qok && in);
        if constexpr (is_split(FN)) vatomic_add<V>(dq_row + D + e, geb, qok && in);
        vatomic_add<V>(dr_row + e, gra, rok && in);
        if constexpr (rel_split(FN)) vatomic_add<V>(dr_row + D + e, grb, rok && in);
    }
    if constexpr (FN == KGE_PROTATE) {
        if (lane == 0 && p.d_modulus) unsafeAtomicAdd(p.d_modulus, dmod);
    }
}

// ---------------------------------------------------------------------------------------------
// Per-row reductions (model.py:145, 168-171, 195-198; upstream train_step). One wave per row.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void neg_reduce_kernel(const float* __restrict__ s, int64_t B, int64_t N,
                                                            int64_t ld, float T, int adversarial,
                                                            float* __restrict__ out) {
    const int64_t b = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (b >= B) return;
    const int lane = threadIdx.x & 63;
    const float* row = s + b * ld;
    float res;
    if (adversarial) {
        float m = -INFINITY;
        for (int64_t n = lane; n < N; n += kWave) m = fmaxf(m, T * row[n]);
        m = wave_max(m);
        float z = 0.f, w = 0.f;
        for (int64_t n = lane; n < N; n += kWave) {
            const float x = row[n];
            const float e = expf(T * x - m);
            z += e;
            w += e * log_sigmoid(-x);
        }
        z = wave_sum(z);
        w = wave_sum(w);
        res = w / z;
    } else {
        float w = 0.f;
        for (int64_t n = lane; n < N; n += kWave) w += log_sigmoid(-row[n]);
        res = wave_sum(w) / (float)N;
    }
    if (lane == 0) out[b] = res;
}

__global__ __launch_bounds__(kBlock) void neg_reduce_bwd_kernel(const float* __restrict__ s, int64_t B, int64_t N,
                                                                int64_t ld, float T, int adversarial, int detach,
                                                                const float* __restrict__ d_out,
                                                                float* __restrict__ d_s, int64_t d_ld) {
    const int64_t b = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (b >= B) return;
    const int lane = threadIdx.x & 63;
    const float* row = s + b * ld;
    float* drow = d_s + b * d_ld;
    const float go = d_out[b];
    if (adversarial) {
        float m = -INFINITY;
        for (int64_t n = lane; n < N; n += kWave) m = fmaxf(m, T * row[n]);
        m = wave_max(m);
        float z = 0.f, w = 0.f;
        for (int64_t n = lane; n < N; n += kWave) {
            const float x = row[n];
            const float e = expf(T * x - m);
            z += e;
            w += e * log_sigmoid(-x);
        }
        z = wave_sum(z);
        w = wave_sum(w);
        const float outv = w / z;
        for (int64_t n = lane; n < N; n += kWave) {
            const float x = row[n];
            const float pn = expf(T * x - m) / z;
            float gsn = pn * (-sigmoidf(x));
            if (!detach) gsn += T * pn * (log_sigmoid(-x) - outv);
            drow[n] = go * gsn;
        }
    } else {
        const float inv = 1.f / (float)N;
        for (int64_t n = lane; n < N; n += kWave) drow[n] = go * (-sigmoidf(row[n])) * inv;
    }
}

__global__ __launch_bounds__(kBlock) void log_sigmoid_kernel(const float* __restrict__ x, int64_t n,
                                                             float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) out[i] = log_sigmoid(x[i]);
}

__global__ __launch_bounds__(kBlock) void log_sigmoid_bwd_kernel(const float* __restrict__ x,
                                                                 const float* __restrict__ d_out, int64_t n,
                                                                 float* __restrict__ d_x) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) d_x[i] = d_out[i] * sigmoidf(-x[i]);
}

// ---------------------------------------------------------------------------------------------
// Host side: error state, dispatch over (fn, candidate side, vector width, groups per lane)
// ---------------------------------------------------------------------------------------------
thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

int check_launch(const char* what) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(KGE_EHIP, std::string(what) + ": " + hipGetErrorString(e));
    g_last_error.clear();
    return 0;
}

constexpr int kMaxG = 8;

template <int FN, bool CH, int V, int G>
void launch_one(const ScoreParams& p, bool bwd, hipStream_t st, int blocks) {
    if (bwd)
        hipLaunchKernelGGL((score_bwd_kernel<FN, CH, V, G>), dim3(blocks), dim3(kBlock), 0, st, p);
    else
        hipLaunchKernelGGL((score_fwd_kernel<FN, CH, V, G>), dim3(blocks), dim3(kBlock), 0, st, p);
}

template <int FN, bool CH, int V>
int launch_g(const ScoreParams& p, bool bwd, hipStream_t st, int blocks, int G) {
    switch (G) {
        case 1: launch_one<FN, CH, V, 1>(p, bwd, st, blocks); return 0;
        case 2: launch_one<FN, CH, V, 2>(p, bwd, st, blocks); return 0;
        case 4: launch_one<FN, CH, V, 4>(p, bwd, st, blocks); return 0;
        case 8: launch_one<FN, CH, V, 8>(p, bwd, st, blocks); return 0;
        default: return fail(KGE_ENOTSUP, "unsupported groups-per-lane");
    }
}

template <int FN, bool CH>
int launch_v(const ScoreParams& p, bool bwd, hipStream_t st, int blocks, int V, int G) {
    switch (V) {
        case 4: return launch_g<FN, CH, 4>(p, bwd, st, blocks, G);
        case 2: return launch_g<FN, CH, 2>(p, bwd, st, blocks, G);
        case 1: return launch_g<FN, CH, 1>(p, bwd, st, blocks, G);
        default: return fail(KGE_ENOTSUP, "unsupported vector width");
    }
}

template <int FN>
int launch_ch(const ScoreParams& p, bool bwd, hipStream_t st, int blocks, bool ch, int V, int G) {
    return ch ? launch_v<FN, true>(p, bwd, st, blocks, V, G) : launch_v<FN, false>(p, bwd, st, blocks, V, G);
}

int launch_fn(int fn, const ScoreParams& p, bool bwd, hipStream_t st, int blocks, bool ch, int V, int G) {
    switch (fn) {
        case KGE_TRANSE: return launch_ch<KGE_TRANSE>(p, bwd, st, blocks, ch, V, G);
        case KGE_DISTMULT: return launch_ch<KGE_DISTMULT>(p, bwd, st, blocks, ch, V, G);
        case KGE_COMPLEX: return launch_ch<KGE_COMPLEX>(p, bwd, st, blocks, ch, V, G);
        case KGE_ROTATE: return launch_ch<KGE_ROTATE>(p, bwd, st, blocks, ch, V, G);
        case KGE_INTERHT: return launch_ch<KGE_INTERHT>(p, bwd, st, blocks, ch, V, G);
        case KGE_PROTATE: return launch_ch<KGE_PROTATE>(p, bwd, st, blocks, ch, V, G);
        default: return fail(KGE_EINVAL, "unknown score function id " + std::to_string(fn));
    }
}

bool aligned(const void* ptr, int bytes) { return ptr == nullptr || ((uintptr_t)ptr % (uintptr_t)bytes) == 0; }

// pick the widest vector width every operand allows, then the groups-per-lane bucket
int pick_vg(const ScoreParams& p, int& V, int& G) {
    const int cand[3] = {4, 2, 1};
    V = 1;
    for (int v : cand) {
        if (p.D % v == 0 && p.q_ld % v == 0 && p.r_ld % v == 0 && p.r_off % v == 0 && p.c_ld % v == 0 &&
            aligned(p.qent, 4 * v) && aligned(p.rel, 4 * v) && aligned(p.cent, 4 * v)) {
            V = v;
            break;
        }
    }
    const int groups = (p.D / V + kWave - 1) / kWave;
    G = 1;
    while (G < groups) G <<= 1;
    if (G > kMaxG)
        return fail(KGE_ENOTSUP, "per-half dim " + std::to_string(p.D) + " exceeds the register-resident limit " +
                                     std::to_string(kMaxG * kWave * V) + " for vector width " + std::to_string(V));
    return 0;
}

int pick_cpw(int64_t B, int64_t N) {
    // enough waves to fill 256 CUs several times over; long runs amortise the query build
    if (N <= 1) return 1;
    int64_t cpw = 16;
    while (cpw > 4 && B * ((N + cpw - 1) / cpw) < 8192) cpw >>= 1;
    return (int)cpw;
}

int run_score(int fn, int mode, ScoreParams& p, bool bwd, void* stream) {
    if (mode != KGE_HEAD_BATCH && mode != KGE_TAIL_BATCH && mode != KGE_SINGLE)
        return fail(KGE_EINVAL, "mode must be 0 (head-batch), 1 (tail-batch) or 3 (single)");
    if (p.B < 0 || p.N < 0 || p.D <= 0) return fail(KGE_EINVAL, "bad shape (B, N, D)");
    if (fn < KGE_TRANSE || fn > KGE_PROTATE) return fail(KGE_EINVAL, "unknown score function id " + std::to_string(fn));
    if (p.B == 0 || p.N == 0) {
        g_last_error.clear();
        return 0;
    }
    if (!p.qent || !p.rel || !p.cent || !p.out) return fail(KGE_EINVAL, "null table/output pointer");
    int V = 1, G = 1;
    int rc = pick_vg(p, V, G);
    if (rc) return rc;
    p.cpw = pick_cpw(p.B, p.N);
    p.wpr = (int)((p.N + p.cpw - 1) / p.cpw);
    const int64_t waves = p.B * p.wpr;
    const int64_t blocks = (waves + kWavesPerBlock - 1) / kWavesPerBlock;
    if (blocks > INT32_MAX) return fail(KGE_EINVAL, "problem too large for one launch");
    rc = launch_fn(fn, p, bwd, (hipStream_t)stream, (int)blocks, mode == KGE_HEAD_BATCH, V, G);
    if (rc) return rc;
    return check_launch(bwd ? "kge score backward launch" : "kge score launch");
}

void fill_indexed(ScoreParams& p, int mode, const float* ent, int64_t nentity, int64_t ent_ld, const float* rel,
                  int64_t nrelation, int64_t rel_ld, int64_t rel_off, const int64_t* pos, const int64_t* neg,
                  int64_t neg_ld, int64_t B, int64_t N, int64_t D) {
    memset(&p, 0, sizeof(p));
    const bool ch = mode == KGE_HEAD_BATCH;
    p.qent = ent;
    p.q_idx = pos ? pos + (ch ? 2 : 0) : nullptr;
    p.q_ld = ent_ld;
    p.q_stride = 3;
    p.q_rows = nentity;
    p.rel = rel;
    p.r_idx = pos ? pos + 1 : nullptr;
    p.r_ld = rel_ld;
    p.r_stride = 3;
    p.r_rows = nrelation;
    p.r_off = rel_off;
    p.cent = ent;
    p.c_ld = ent_ld;
    p.c_rows = nentity;
    if (mode == KGE_SINGLE) {
        p.c_idx = pos ? pos + 2 : nullptr;
        p.c_stride = 3;
        N = 1;
    } else {
        p.c_idx = neg;
        p.c_stride = neg_ld;
    }
    p.B = B;
    p.N = N;
    p.D = (int)D;
}

float phase_div_for(int fn, float emb_range) {
    // torch: tensor / (python float: emb_range.item() / pi) -> the divisor is rounded to fp32
    const double pi = (fn == KGE_PROTATE) ? 3.14159262358979323846 : 3.14159265358979323846;
    return (float)((double)emb_range / pi);
}

}  // namespace

// =============================================================================================
// C-ABI
// =============================================================================================
extern "C" {

int kge_abi_version(void) { return KGE_ABI_VERSION; }

const char* kge_last_error(void) { return g_last_error.c_str(); }

int64_t kge_max_dim(int fn) {
    if (fn < KGE_TRANSE || fn > KGE_PROTATE) return 0;
    return (int64_t)kMaxG * kWave * 4;
}

int kge_score_indexed(int fn, int mode, const float* ent, int64_t nentity, int64_t ent_ld, const float* rel,
                      int64_t nrelation, int64_t rel_ld, int64_t rel_off, const int64_t* pos, const int64_t* neg,
                      int64_t neg_ld, int64_t B, int64_t N, int64_t D, float gamma, float emb_range, float modulus,
                      float* scores, int64_t scores_ld, void* stream) {
    if (!pos) return fail(KGE_EINVAL, "pos must not be NULL");
    if (mode != KGE_SINGLE && !neg) return fail(KGE_EINVAL, "neg must not be NULL in head/tail-batch mode");
    ScoreParams p;
    fill_indexed(p, mode, ent, nentity, ent_ld, rel, nrelation, rel_ld, rel_off, pos, neg, neg_ld, B, N, D);
    p.out = scores;
    p.out_ld = scores_ld;
    p.gamma = gamma;
    p.phase_div = phase_div_for(fn, emb_range);
    p.modulus = modulus;
    return run_score(fn, mode, p, false, stream);
}

static void fill_dense(ScoreParams& p, int fn, int mode, const float* head, int64_t head_ld, const float* rel,
                       int64_t rel_ld, int64_t rel_off, const float* tail, int64_t tail_ld, int64_t B, int64_t N,
                       int64_t D, float gamma, float emb_range, float modulus) {
    memset(&p, 0, sizeof(p));
    const bool ch = mode == KGE_HEAD_BATCH;
    if (mode == KGE_SINGLE) N = 1;
    p.qent = ch ? tail : head;
    p.q_ld = ch ? tail_ld : head_ld;
    p.q_rows = B;
    p.rel = rel;
    p.r_ld = rel_ld;
    p.r_off = rel_off;
    p.r_rows = B;
    p.cent = ch ? head : tail;
    p.c_ld = ch ? head_ld : tail_ld;
    p.c_dense = N;
    p.c_rows = B * N;
    p.B = B;
    p.N = N;
    p.D = (int)D;
    p.gamma = gamma;
    p.phase_div = phase_div_for(fn, emb_range);
    p.modulus = modulus;
}

int kge_score_dense(int fn, int mode, const float* head, int64_t head_ld, const float* rel, int64_t rel_ld,
                    int64_t rel_off, const float* tail, int64_t tail_ld, int64_t B, int64_t N, int64_t D, float gamma,
                    float emb_range, float modulus, float* scores, int64_t scores_ld, void* stream) {
    ScoreParams p;
    fill_dense(p, fn, mode, head, head_ld, rel, rel_ld, rel_off, tail, tail_ld, B, N, D, gamma, emb_range, modulus);
    p.out = scores;
    p.out_ld = scores_ld;
    return run_score(fn, mode, p, false, stream);
}

int kge_score_dense_bwd(int fn, int mode, const float* head, int64_t head_ld, const float* rel, int64_t rel_ld,
                        int64_t rel_off, const float* tail, int64_t tail_ld, int64_t B, int64_t N, int64_t D,
                        float gamma, float emb_range, float modulus, const float* d_scores, int64_t d_ld,
                        float* d_head, float* d_rel, float* d_tail, float* d_modulus, void* stream) {
    if (!d_scores || !d_head || !d_rel || !d_tail) return fail(KGE_EINVAL, "null gradient pointer");
    ScoreParams p;
    fill_dense(p, fn, mode, head, head_ld, rel, rel_ld, rel_off, tail, tail_ld, B, N, D, gamma, emb_range, modulus);
    const bool ch = mode == KGE_HEAD_BATCH;
    p.out = d_head;  // unused by the backward kernel; non-null for the argument check
    p.d_scores = d_scores;
    p.d_ld = d_ld;
    p.d_qent = ch ? d_tail : d_head;
    p.d_cent = ch ? d_head : d_tail;
    p.d_rel = d_rel;
    p.d_modulus = d_modulus;
    return run_score(fn, mode, p, true, stream);
}

int kge_neg_reduce(const float* scores, int64_t B, int64_t N, int64_t ld, float temperature, int adversarial,
                   float* out, void* stream) {
    if (B < 0 || N <= 0) return fail(KGE_EINVAL, "bad shape (B, N)");
    if (B == 0) return 0;
    if (!scores || !out) return fail(KGE_EINVAL, "null pointer");
    const int64_t blocks = (B + kWavesPerBlock - 1) / kWavesPerBlock;
    hipLaunchKernelGGL(neg_reduce_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, (hipStream_t)stream, scores, B, N,
                       ld, temperature, adversarial, out);
    return check_launch("kge_neg_reduce");
}

int kge_neg_reduce_bwd(const float* scores, int64_t B, int64_t N, int64_t ld, float temperature, int adversarial,
                       int detach, const float* d_out, float* d_scores, int64_t d_ld, void* stream) {
    if (B < 0 || N <= 0) return fail(KGE_EINVAL, "bad shape (B, N)");
    if (B == 0) return 0;
    if (!scores || !d_out || !d_scores) return fail(KGE_EINVAL, "null pointer");
    const int64_t blocks = (B + kWavesPerBlock - 1) / kWavesPerBlock;
    hipLaunchKernelGGL(neg_reduce_bwd_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, (hipStream_t)stream, scores,
                       B, N, ld, temperature, adversarial, detach, d_out, d_scores, d_ld);
    return check_launch("kge_neg_reduce_bwd");
}

int kge_log_sigmoid(const float* x, int64_t n, float* out, void* stream) {
    if (n < 0) return fail(KGE_EINVAL, "bad size");
    if (n == 0) return 0;
    if (!x || !out) return fail(KGE_EINVAL, "null pointer");
    hipLaunchKernelGGL(log_sigmoid_kernel, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       (hipStream_t)stream, x, n, out);
    return check_launch("kge_log_sigmoid");
}

int kge_log_sigmoid_bwd(const float* x, const float* d_out, int64_t n, float* d_x, void* stream) {
    if (n < 0) return fail(KGE_EINVAL, "bad size");
    if (n == 0) return 0;
    if (!x || !d_out || !d_x) return fail(KGE_EINVAL, "null pointer");
    hipLaunchKernelGGL(log_sigmoid_bwd_kernel, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       (hipStream_t)stream, x, d_out, n, d_x);
    return check_launch("kge_log_sigmoid_bwd");
}

int64_t kge_score_bwd_workspace_size(int fn, int mode, int64_t B, int64_t N, int64_t D) {
    (void)fn;
    (void)mode;
    (void)B;
    (void)N;
    (void)D;
    return 0;  // the atomic-scatter backward needs no scratch
}

int kge_score_indexed_bwd(int fn, int mode, const float* ent, int64_t nentity, int64_t ent_ld, const float* rel,
                          int64_t nrelation, int64_t rel_ld, int64_t rel_off, const int64_t* pos, const int64_t* neg,
                          int64_t neg_ld, int64_t B, int64_t N, int64_t D, float gamma, float emb_range, float modulus,
                          const float* d_scores, int64_t d_ld, float* d_ent, float* d_rel, float* d_modulus,
                          void* workspace, void* stream) {
    (void)workspace;
    if (!pos) return fail(KGE_EINVAL, "pos must not be NULL");
    if (mode != KGE_SINGLE && !neg) return fail(KGE_EINVAL, "neg must not be NULL in head/tail-batch mode");
    if (!d_scores || !d_ent || !d_rel) return fail(KGE_EINVAL, "null gradient pointer");
    ScoreParams p;
    fill_indexed(p, mode, ent, nentity, ent_ld, rel, nrelation, rel_ld, rel_off, pos, neg, neg_ld, B, N, D);
    p.out = d_ent;  // unused by the backward kernel; non-null for the argument check
    p.gamma = gamma;
    p.phase_div = phase_div_for(fn, emb_range);
    p.modulus = modulus;
    p.d_scores = d_scores;
    p.d_ld = d_ld;
    p.d_qent = d_ent;
    p.d_cent = d_ent;
    p.d_rel = d_rel;
    p.d_modulus = d_modulus;
    return run_score(fn, mode, p, true, stream);
}

}  // extern "C"
