// kge_device.h — device templates of the fused gather + score kernels (gfx950 / CDNA4).
//
// What they replace (reference, /root/reference):
//   tensorflow_codes/model.py:127-199  single/head-batch/tail-batch gathers (tf.gather) + model_func
//   tensorflow_codes/model.py:207-224  InterHT score
//   tensorflow_codes/model.py:145,168-171,195-198  logsigmoid / self-adversarial reduction (Q3, Q4)
//   KnowledgeGraphEmbedding/codes/model.py (absent; restated in oracle/kge_oracle.py):
//     TransE / DistMult / ComplEx / RotatE / pRotatE score functions and KGEModel.forward gathers.
//
// Work decomposition: one wave64 owns one batch row b and a run of `cpw` consecutive candidates of
// that row. The query side shared by every candidate of row b — (h, r) in tail-batch / single
// mode, (r, t) in head-batch mode — is built ONCE per wave and kept in VGPRs. Candidate rows are
// gathered from HBM straight into VGPRs with 16-B loads (lane l owns float4 groups l, l+64, ...
// of each half-row) and software-pipelined: the next row is in flight while the current one is
// reduced. Reductions along the hidden dim are DPP row butterflies + 4 readlanes (fixed order:
// deterministic). Nothing [B, N, d]-shaped is materialised.
#pragma once

#include <math.h>

#include <type_traits>

#include "kge_internal.h"

namespace kge_impl {

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

template <int V>
__device__ __forceinline__ void vstore(float* dst, const vecf<V>& v, bool ok) {
    if (ok) *reinterpret_cast<vecf<V>*>(dst) = v;
}

// Raw buffer descriptor over `bytes` bytes at `base`, built from wave-uniform values only (the
// readfirstlanes make that provable to the compiler, so no waterfall loop is emitted). Loads at or
// past `bytes` return 0 (hardware range check): rows past D, or a whole invalid row (bytes = 0),
// need no masks or branches.
using rsrc_t = __amdgpu_buffer_rsrc_t;
__device__ __forceinline__ rsrc_t make_rsrc(const void* base, uint32_t bytes) {
    const uint64_t a = (uint64_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    const uint32_t n = __builtin_amdgcn_readfirstlane(bytes);
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0, (int)n, 0x00020000);
}

// AUX: cache policy bits of the buffer instruction (gfx950: 2 = nt, 16 = sc1)
constexpr int kAuxNT = 2, kAuxSC1 = 16;
// cache policy of bwd_ent_stream_kernel's streamed table row and Adam moments: nt loads AND nt
// stores (either alone measured no faster; together the C2 train step drops 0.636 -> 0.606 ms,
// scripts/ab_cache_policy.sh)
constexpr int kEntLdAux = kAuxNT, kEntStAux = kAuxNT;

template <int V, int AUX = 0>
__device__ __forceinline__ vecf<V> bload(rsrc_t r, uint32_t off) {
    vecf<V> o;
    if constexpr (V == 4) {
        const auto u = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, AUX);
        o.a[0] = __uint_as_float(u[0]);
        o.a[1] = __uint_as_float(u[1]);
        o.a[2] = __uint_as_float(u[2]);
        o.a[3] = __uint_as_float(u[3]);
    } else if constexpr (V == 2) {
        const auto u = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, AUX);
        o.a[0] = __uint_as_float(u[0]);
        o.a[1] = __uint_as_float(u[1]);
    } else {
        o.a[0] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, off, 0, AUX));
    }
    return o;
}

// buffer store (range-checked: bytes at or past the descriptor's size are dropped)
template <int V, int AUX = 0>
__device__ __forceinline__ void bstore(rsrc_t r, uint32_t off, const vecf<V>& v) {
    if constexpr (V == 4) {
        __attribute__((ext_vector_type(4))) unsigned u;
        u[0] = __float_as_uint(v.a[0]);
        u[1] = __float_as_uint(v.a[1]);
        u[2] = __float_as_uint(v.a[2]);
        u[3] = __float_as_uint(v.a[3]);
        __builtin_amdgcn_raw_buffer_store_b128(u, r, off, 0, AUX);
    } else if constexpr (V == 2) {
        __attribute__((ext_vector_type(2))) unsigned u;
        u[0] = __float_as_uint(v.a[0]);
        u[1] = __float_as_uint(v.a[1]);
        __builtin_amdgcn_raw_buffer_store_b64(u, r, off, 0, AUX);
    } else {
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v.a[0]), r, off, 0, AUX);
    }
}

// byte offset of lane `lane`'s group k in a half-row
template <int V>
__device__ __forceinline__ uint32_t goff(int lane, int k) {
    return (uint32_t)((lane + k * kWave) * V * 4);
}

__device__ __forceinline__ float rsqrt_f(float x) { return __builtin_amdgcn_rsqf(x); }

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}

// Sum over the 64 lanes, result in every lane: quad_perm xor1, xor2, row_half_mirror, row_mirror
// (each 16-lane row then holds its sum in all lanes), then the 4 row sums via readlane.
__device__ __forceinline__ float wave_sum(float v) {
    v += dpp<0xB1>(v);   // quad_perm [1,0,3,2]
    v += dpp<0x4E>(v);   // quad_perm [2,3,0,1]
    v += dpp<0x141>(v);  // row_half_mirror
    v += dpp<0x140>(v);  // row_mirror
    const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
    const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
    const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
    const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
    return (r0 + r1) + (r2 + r3);
}

__device__ __forceinline__ float wave_max(float v) {
    v = fmaxf(v, dpp<0xB1>(v));
    v = fmaxf(v, dpp<0x4E>(v));
    v = fmaxf(v, dpp<0x141>(v));
    v = fmaxf(v, dpp<0x140>(v));
    const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
    const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
    const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
    const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
    return fmaxf(fmaxf(r0, r1), fmaxf(r2, r3));
}

__device__ __forceinline__ int64_t readlane64(int64_t v, int j) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(uint64_t)v, j);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), j);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ float readlanef(float v, int j) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), j));
}

// ascending bitonic sort of one int per lane across the wave
__device__ __forceinline__ int wave_sort_asc(int v, int lane) {
#pragma unroll
    for (int k = 2; k <= kWave; k <<= 1)
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            const int o = __shfl_xor(v, j, kWave);
            const bool keep_min = ((lane & k) == 0) == ((lane & j) == 0);
            v = keep_min ? min(v, o) : max(v, o);
        }
    return v;
}

__device__ __forceinline__ int wave_min_i(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, kWave));
    return v;
}

__device__ __forceinline__ float sgnf(float x) { return (x > 0.f) ? 1.f : ((x < 0.f) ? -1.f : 0.f); }

// logsigmoid(x) = min(x,0) - log1p(exp(-|x|))   (tf.math.log_sigmoid, model.py:145,169)
__device__ __forceinline__ float log_sigmoid(float x) { return fminf(x, 0.f) - log1pf(expf(-fabsf(x))); }
__device__ __forceinline__ float sigmoidf(float x) {
    if (x >= 0.f) return 1.f / (1.f + expf(-x));
    const float e = expf(x);
    return e / (1.f + e);
}

// fp32 -> three bf16 terms, x = x0 + x1 + x2 to 24 significant bits (RNE v_cvt_pk_bf16_f32 each): the
// operand form of the fp32-accurate products on the bf16 matrix cores (kge_eval.hip, kge_transparse.hip).
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ void split3_bf16(const f32x8& v, bf16x8& a0, bf16x8& a1, bf16x8& a2) {
    a0 = __builtin_convertvector(v, bf16x8);
    const f32x8 r1 = v - __builtin_convertvector(a0, f32x8);
    a1 = __builtin_convertvector(r1, bf16x8);
    a2 = __builtin_convertvector(r1 - __builtin_convertvector(a1, f32x8), bf16x8);
}
// the six products A_i . B_j (i + j <= 2), smallest first
constexpr int kX3A[6] = {2, 1, 0, 1, 0, 0}, kX3B[6] = {0, 1, 2, 0, 1, 0};

// One Adam update (supervisor.py:26; run.py:111 Keras Adam, or torch.optim.Adam), shared by the
// dense optimizer kernel and the fused backward so both give bitwise-identical results.
//   keras: m += (g - m)(1 - b1); v += (g^2 - v)(1 - b2); p -= m * alpha / (sqrt(v) + eps)
//   torch: m = lerp(m, g, 1 - b1); v = v b2 + (1 - b2) g^2; p -= step_size m / (sqrt(v) / bc2_sqrt + eps)
__device__ __forceinline__ void adam_update(float& p, float g, float& m, float& v, float b1, float b2, float eps,
                                            float alpha, float step_size, float bc2_sqrt, int keras) {
    if (keras) {
        m += (g - m) * (1.f - b1);
        v += (g * g - v) * (1.f - b2);
        p -= (m * alpha) / (sqrtf(v) + eps);
    } else {
        m = m + (1.f - b1) * (g - m);
        v = v * b2 + (1.f - b2) * g * g;
        p -= step_size * m / (sqrtf(v) / bc2_sqrt + eps);
    }
}

constexpr bool is_split(int fn) { return fn == KGE_COMPLEX || fn == KGE_ROTATE || fn == KGE_INTERHT; }
constexpr bool rel_split(int fn) { return fn == KGE_COMPLEX; }

// ---------------------------------------------------------------------------------------------
// Query side. CH = candidate is the head (head-batch); otherwise the candidate is the tail
// (tail-batch and single, which upstream scores with the same "else" branch).
//   q0,q1,q2: per-element query operands kept in VGPRs; zero on groups past D.
//   na_inv,nb_inv: InterHT query reciprocal norms (1/||a||, 1/||b||; no epsilon, Q7)
// ---------------------------------------------------------------------------------------------
// The hardware v_sin_f32 / v_cos_f32 take their argument in revolutions and are defined for |x| <= 256 of
// them. hw_sin / hw_cos scale a phase in radians to revolutions and keep only its fraction (v_fract_f32) before
// the instruction: one more VALU op, and a phase of any size (trained embeddings are unconstrained) stays in the
// instruction's range. The scaled phase carries the fp32 rounding of x / 2 pi: at |x| = 500 rad (80 revolutions)
// that is <= 2.4e-5 rad, against the scores' 1e-4 relative bar (tests/test_parity_gpu.py::test_trained_range_*).
constexpr float kInv2Pi = 0.15915494309189535f;
__device__ __forceinline__ float hw_sin(float x) { return __builtin_amdgcn_sinf(__builtin_amdgcn_fractf(x * kInv2Pi)); }
__device__ __forceinline__ float hw_cos(float x) { return __builtin_amdgcn_cosf(__builtin_amdgcn_fractf(x * kInv2Pi)); }

template <int FN, bool CH, int V, int G>
struct Query {
    vecf<V> q0[G], q1[G], q2[G];
    float na_inv, nb_inv;

    __device__ __forceinline__ void build(const float* qrow, bool qok, const float* rrow, bool rok,
                                          int D, int lane, const ScoreParams& p) {
        const int DV = D / V;
        const uint32_t qb = qok ? (uint32_t)D * 4u : 0u, rbytes = rok ? (uint32_t)D * 4u : 0u;
        const rsrc_t sqa = make_rsrc(qrow, qb), sra = make_rsrc(rrow, rbytes);
        vecf<V> ea[G], eb[G], ra[G], rb[G];
#pragma unroll
        for (int k = 0; k < G; ++k) {
            ea[k] = bload<V>(sqa, goff<V>(lane, k));
            ra[k] = bload<V>(sra, goff<V>(lane, k));
        }
        if constexpr (is_split(FN)) {
            const rsrc_t sqb = make_rsrc(qrow + D, qb);
#pragma unroll
            for (int k = 0; k < G; ++k) eb[k] = bload<V>(sqb, goff<V>(lane, k));
        } else {
#pragma unroll
            for (int k = 0; k < G; ++k) eb[k] = vzero<V>();
        }
        if constexpr (rel_split(FN)) {
            const rsrc_t srb = make_rsrc(rrow + D, rbytes);
#pragma unroll
            for (int k = 0; k < G; ++k) rb[k] = bload<V>(srb, goff<V>(lane, k));
        } else {
#pragma unroll
            for (int k = 0; k < G; ++k) rb[k] = vzero<V>();
        }
        na_inv = nb_inv = 0.f;
        if constexpr (FN == KGE_INTERHT) {
            float sa = 0.f, sb = 0.f;
#pragma unroll
            for (int k = 0; k < G; ++k)
#pragma unroll
                for (int i = 0; i < V; ++i) {
                    sa += ea[k].a[i] * ea[k].a[i];
                    sb += eb[k].a[i] * eb[k].a[i];
                }
            na_inv = rsqrt_f(wave_sum(sa));
            nb_inv = rsqrt_f(wave_sum(sb));
        }
        // RotatE: the relation phases' cos / sin on the hardware units (hw_cos / hw_sin: two instructions and a
        // fract per element; libm's argument reduction put the query build of the tile kernel's setup and of the
        // head-batch positives on a long VALU chain, and G V of them interleaved spilled the tile kernel)
        float rc[G][V], rs[G][V];
        if constexpr (FN == KGE_ROTATE) {
#pragma unroll
            for (int k = 0; k < G; ++k)
#pragma unroll
                for (int i = 0; i < V; ++i) {
                    const float ph = ra[k].a[i] / p.phase_div;
                    rc[k][i] = hw_cos(ph);
                    rs[k][i] = hw_sin(ph);
                }
        }
#pragma unroll
        for (int k = 0; k < G; ++k) {
            const bool in = (lane + k * kWave) < DV;
#pragma unroll
            for (int i = 0; i < V; ++i) {
                const float x = ea[k].a[i], y = eb[k].a[i];
                const float r = ra[k].a[i], s = rb[k].a[i];
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
                    const float c = rc[k][i], sn = rs[k][i];
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
                    // query entity halves normalised (Q7), b-half shifted by u = 1 (model.py:215-220)
                    o0 = in ? x * na_inv : 0.f;
                    o1 = in ? (y * nb_inv + 1.f) : 0.f;
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
        const uint32_t nb = ok ? (uint32_t)D * 4u : 0u;
        const rsrc_t sa = make_rsrc(row, nb);
#pragma unroll
        for (int k = 0; k < G; ++k) ca[k] = bload<V>(sa, goff<V>(lane, k));
        if constexpr (is_split(FN)) {
            const rsrc_t sb = make_rsrc(row + D, nb);
#pragma unroll
            for (int k = 0; k < G; ++k) cb[k] = bload<V>(sb, goff<V>(lane, k));
        }
    }
};

// Forward score of one candidate held in registers (every lane returns the full score).
// Query operands held in LDS (one copy per block, shared by its waves): q.q0[k] reads lane's group k.
template <int V>
struct LdsOperand {
    const vecf<V>* base;  // the operand image
    int idx;              // lane
    __device__ __forceinline__ vecf<V> operator[](int k) const { return base[idx + k * kWave]; }
};
template <int V>
struct LdsQuery {
    LdsOperand<V> q0, q1, q2;
};

template <int FN, bool CH, int V, int G, class Q>
__device__ __forceinline__ float cand_score(const Cand<FN, V, G>& c, const Q& q, const ScoreParams& p,
                                            float2* stats = nullptr, vecf<V>* nsg = nullptr) {
    float acc = 0.f;
    if constexpr (FN == KGE_INTERHT && V % 2 == 0) {
        // on packed fp32 pairs (v_pk_fma_f32 / v_pk_mul_f32: two elements per instruction): the fused
        // train forward is VALU-bound and this is most of its per-candidate work
        typedef float f2 __attribute__((ext_vector_type(2)));
        f2 sa2 = {0.f, 0.f}, sb2 = {0.f, 0.f};
#pragma unroll
        for (int k = 0; k < G; ++k)
#pragma unroll
            for (int i = 0; i < V; i += 2) {
                const f2 a{c.ca[k].a[i], c.ca[k].a[i + 1]}, bb{c.cb[k].a[i], c.cb[k].a[i + 1]};
                sa2 = a * a + sa2;
                sb2 = bb * bb + sb2;
            }
        const float ia = rsqrt_f(wave_sum(sa2.x + sa2.y)), ib = rsqrt_f(wave_sum(sb2.x + sb2.y));
        if (stats) *stats = make_float2(ia, ib);  // kept for the streaming phase-1 backward
#pragma unroll
        for (int k = 0; k < G; ++k) {
            const vecf<V> q0 = q.q0[k], q1 = q.q1[k], q2 = q.q2[k];
#pragma unroll
            for (int i = 0; i < V; i += 2) {
                const f2 ah = f2{c.ca[k].a[i], c.ca[k].a[i + 1]} * ia;        // normalised candidate a-half
                const f2 bh = f2{c.cb[k].a[i], c.cb[k].a[i + 1]} * ib + 1.f;  // normalised b-half + u
                const f2 Q0{q0.a[i], q0.a[i + 1]}, Q1{q1.a[i], q1.a[i + 1]}, Q2{q2.a[i], q2.a[i + 1]};
                // head: a_head * b_tail - a_tail * b_head + re_mid; tail: the other way round (model.py:222)
                const f2 x = CH ? (ah * Q1 - Q0 * bh + Q2) : (Q0 * bh - ah * Q1 + Q2);
                acc += fabsf(x.x);
                acc += fabsf(x.y);
                if (nsg) {  // the Jacobian's sign (0 past D: x = 0 there)
                    nsg[k].a[i] = -sgnf(x.x);
                    nsg[k].a[i + 1] = -sgnf(x.y);
                }
            }
        }
    } else if constexpr (FN == KGE_INTERHT) {
        float sa = 0.f, sb = 0.f;
#pragma unroll
        for (int k = 0; k < G; ++k)
#pragma unroll
            for (int i = 0; i < V; ++i) {
                sa += c.ca[k].a[i] * c.ca[k].a[i];
                sb += c.cb[k].a[i] * c.cb[k].a[i];
            }
        const float ia = rsqrt_f(wave_sum(sa)), ib = rsqrt_f(wave_sum(sb));
        if (stats) *stats = make_float2(ia, ib);  // kept for the streaming phase-1 backward
#pragma unroll
        for (int k = 0; k < G; ++k)
#pragma unroll
            for (int i = 0; i < V; ++i) {
                const float ah = c.ca[k].a[i] * ia;        // normalised candidate a-half
                const float bh = c.cb[k].a[i] * ib + 1.f;  // normalised candidate b-half + u
                float x;
                if (CH)  // a_head * b_tail - a_tail * b_head + re_mid   (model.py:222)
                    x = ah * q.q1[k].a[i] - q.q0[k].a[i] * bh + q.q2[k].a[i];
                else
                    x = q.q0[k].a[i] * bh - ah * q.q1[k].a[i] + q.q2[k].a[i];
                acc += fabsf(x);
                if (nsg) nsg[k].a[i] = -sgnf(x);  // the Jacobian's sign (0 past D: x = 0 there)
            }
        // groups past D: candidate zero-loaded and query zero -> x = 0
    } else if constexpr (FN == KGE_ROTATE && V % 2 == 0) {
        // per-element modulus |q - c| on packed fp32 pairs and the hardware v_sqrt_f32 (1 ulp): the IEEE
        // sqrtf expansion (denormal scaling + two Newton corrections, ~15 instructions per element) made the
        // C3 tile kernel issue-bound (SQ_WAIT_ANY 30 % of the wave cycles, slower than C2 on the same bytes)
        typedef float f2 __attribute__((ext_vector_type(2)));
#pragma unroll
        for (int k = 0; k < G; ++k) {
            const vecf<V> q0 = q.q0[k], q1 = q.q1[k];
#pragma unroll
            for (int i = 0; i < V; i += 2) {
                const f2 xr = f2{q0.a[i], q0.a[i + 1]} - f2{c.ca[k].a[i], c.ca[k].a[i + 1]};
                const f2 xi = f2{q1.a[i], q1.a[i + 1]} - f2{c.cb[k].a[i], c.cb[k].a[i + 1]};
                const f2 s2 = xr * xr + xi * xi;
                acc += __builtin_amdgcn_sqrtf(s2.x);
                acc += __builtin_amdgcn_sqrtf(s2.y);
            }
        }
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
                    acc += __builtin_amdgcn_sqrtf(xr * xr + xi * xi);  // hardware sqrt, as the packed form
                } else if constexpr (FN == KGE_PROTATE) {
                    const float pc = x / p.phase_div;
                    const float z = CH ? (pc + q.q0[k].a[i]) : (q.q0[k].a[i] - pc);
                    acc += fabsf(hw_sin(z));  // the hardware v_sin_f32 on the fraction of z's revolutions
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
__device__ __forceinline__ void build_query_for(const ScoreParams& p, int64_t b, int lane, Query<FN, CH, V, G>& q,
                                                int64_t& qi, int64_t& ri, bool& qok, bool& rok) {
    qi = p.q_idx ? p.q_idx[b * p.q_stride] : b;
    ri = p.r_idx ? p.r_idx[b * p.r_stride] : b;
    qok = qi >= 0 && qi < p.q_rows;
    rok = ri >= 0 && ri < p.r_rows;
    q.build(p.qent + (qok ? qi : 0) * p.q_ld, qok, p.rel + (rok ? ri : 0) * p.r_ld + p.r_off, rok, p.D, lane, p);
}

__device__ __forceinline__ const float* cand_row(const ScoreParams& p, int64_t id, bool& ok) {
    id -= p.c_base;
    ok = id >= 0 && id < p.c_rows;
    return p.cent + (ok ? id : 0) * p.c_ld;
}

// Scores up to 64 candidates held one per lane (lane j: global id my_id, j < nc) against the wave's
// query; returns candidate j's score in lane j (and, with ST, InterHT's candidate inverse half-norms
// in my_st). Software pipeline: row j+1 is in flight while row j is reduced.
// Query with InterHT's third operand (the relation's middle third, shared by every candidate) read
// from a wave-private LDS image: 4 x G fewer VGPRs per lane (the XCD-sliced kernel then holds 4 waves
// per SIMD at D = 1000). fresh() launders the LDS index before each candidate so the reads are not
// hoisted back into loop-invariant registers.
template <int FN, bool CH, int V, int G>
struct QueryL2 {
    vecf<V> q0[G], q1[G];
    LdsOperand<V> q2;
};
template <class Q>
__device__ __forceinline__ const Q& fresh(const Q& q) {
    return q;
}
template <int FN, bool CH, int V, int G>
__device__ __forceinline__ QueryL2<FN, CH, V, G> fresh(const QueryL2<FN, CH, V, G>& q) {
    QueryL2<FN, CH, V, G> r = q;
    int li = q.q2.idx;
    asm volatile("" : "+v"(li));
    r.q2.idx = li;
    return r;
}

template <int FN, bool CH, int V, int G, bool ST, class Q, int DEPTH = 2>
__device__ __forceinline__ float score_lanes(const ScoreParams& p, const Q& q, int64_t my_id, int nc, int lane,
                                             float2& my_st) {
    float my_score = 0.f;
    float2 st;
    float2* stp = ST ? &st : nullptr;
    if constexpr (DEPTH == 1) {
        // one row in registers at a time: fewer VGPRs, more waves per SIMD hide the gather latency
        for (int j = 0; j < nc; ++j) {
            Cand<FN, V, G> x;
            bool ok;
            x.load(cand_row(p, readlane64(my_id, j), ok), ok, p.D, lane);
            const float sc = cand_score<FN, CH, V, G>(x, fresh(q), p, stp);
            if (lane == j) {
                my_score = sc;
                if constexpr (ST) my_st = st;
            }
        }
        return my_score;
    }
    Cand<FN, V, G> x0, x1;
    bool ok0, ok1;
    const float* row = cand_row(p, readlane64(my_id, 0), ok0);
    x0.load(row, ok0, p.D, lane);
    int j = 0;
    auto keep = [&](int jj, float sc) {
        if (lane == jj) {
            my_score = sc;
            if constexpr (ST) my_st = st;
        }
    };
    for (; j + 2 < nc; j += 2) {
        row = cand_row(p, readlane64(my_id, j + 1), ok1);
        x1.load(row, ok1, p.D, lane);
        keep(j, cand_score<FN, CH, V, G>(x0, fresh(q), p, stp));
        row = cand_row(p, readlane64(my_id, j + 2), ok0);
        x0.load(row, ok0, p.D, lane);
        keep(j + 1, cand_score<FN, CH, V, G>(x1, fresh(q), p, stp));
    }
    if (j + 1 < nc) {
        row = cand_row(p, readlane64(my_id, j + 1), ok1);
        x1.load(row, ok1, p.D, lane);
        keep(j, cand_score<FN, CH, V, G>(x0, fresh(q), p, stp));
        keep(j + 1, cand_score<FN, CH, V, G>(x1, fresh(q), p, stp));
    } else {
        keep(j, cand_score<FN, CH, V, G>(x0, fresh(q), p, stp));
    }
    return my_score;
}

// Scores candidates [n0, n0 + nc) (nc <= 64) of batch row b against the wave's query; score n0 + j
// is produced in lane j and stored coalesced (and, with ST, InterHT's candidate inverse half-norms).
template <int FN, bool CH, int V, int G, bool ST>
__device__ __forceinline__ void score_run(const ScoreParams& p, const Query<FN, CH, V, G>& q, int64_t b, int64_t n0,
                                          int nc, int lane) {
    int64_t my_id = 0;
    if (lane < nc) my_id = p.c_idx ? p.c_idx[b * p.c_stride + n0 + lane] : b * p.c_dense + n0 + lane;
    float2 my_st = make_float2(0.f, 0.f);
    const float my_score = score_lanes<FN, CH, V, G, ST>(p, q, my_id, nc, lane, my_st);
    if (lane < nc) p.out[b * p.out_ld + n0 + lane] = my_score;
    if constexpr (ST) {
        if (lane < nc) p.cand_stats[b * p.N + n0 + lane] = my_st;
    }
}

// ---------------------------------------------------------------------------------------------
// Row-sharded tables (SURVEY §8e owner-computes): this shard holds global entity rows
// [c_base, c_base + c_rows). A batch row's candidates are spread over every shard, so each shard
// COMPACTS the candidates it owns before scoring: per 64 ids one coalesced load, a ballot and a few
// lane permutes; only owned candidates take a slot of the gather pipeline. Per-shard work is then
// O(owned candidates) + O(ids), not O(all candidates).
// ---------------------------------------------------------------------------------------------
// position of the k-th (0-based) set bit of m (k < popcount(m))
__device__ __forceinline__ int kth_set_bit(uint64_t m, int k) {
    int pos = 0;
#pragma unroll
    for (int s = 32; s > 0; s >>= 1) {
        const uint64_t low = m & ((1ull << s) - 1ull);
        const int c = __popcll(low);
        if (k >= c) {
            k -= c;
            m >>= s;
            pos += s;
        } else {
            m = low;
        }
    }
    return pos;
}

// value of `v` in lane `src` (every lane must execute this)
__device__ __forceinline__ int lane_pull(int v, int src) { return __builtin_amdgcn_ds_bpermute(src << 2, v); }

// number of set bits of m in the lanes below this one
__device__ __forceinline__ int lanes_below(uint64_t m) {
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Start of batch row b's run in the compact send block (ScoreParams::cmp_pre, kge_shard_score): the row's
// home-local prefix plus this rank's owned counts of the launch's earlier homes.
__device__ __forceinline__ int64_t cmp_row_off(const ScoreParams& p, int64_t b) {
    const int64_t h = b / p.home_B;
    int64_t off = p.cmp_pre[b];
    for (int64_t k = 0; k < h; ++k) off += p.cmp_tot[(p.cmp_home0 + k) * p.world + p.rank];
    return off;
}

// Walks candidates [lo, hi) of batch row b and calls body(row, n, cnt) with the owned ones compacted
// into lanes 0..cnt-1 (row: local shard row, n: candidate column), in candidate order; every call but
// the last has cnt = 64. With zero_out, a foreign candidate's score slot p.out[b, n] is written 0 (the
// partial score block a SUM over shards assembles).
template <class Body>
__device__ __forceinline__ void for_owned_runs(const ScoreParams& p, int64_t b, int64_t lo, int64_t hi, int lane,
                                               bool zero_out, Body&& body) {
    int buf_row = 0, buf_n = 0, fill = 0;
    // the ids of 4 chunks are requested at once (one latency per 256 candidates instead of per 64)
    constexpr int PF = 4;
    int64_t ids[PF];
    for (int64_t c0 = lo; c0 < hi; c0 += kWave) {
        const int u = (int)(((c0 - lo) / kWave) % PF);
        if (u == 0) {
#pragma unroll
            for (int v = 0; v < PF; ++v) {
                const int64_t nv = c0 + v * kWave + lane;
                ids[v] = nv < hi ? (p.c_idx ? p.c_idx[b * p.c_stride + nv] : b * p.c_dense + nv) : 0;
            }
        }
        int64_t picked = ids[0];
#pragma unroll
        for (int v = 1; v < PF; ++v)
            if (u == v) picked = ids[v];
        const int64_t n = c0 + lane;
        int64_t row = -1;
        if (n < hi) row = picked - p.c_base;
        const bool own = n < hi && row >= 0 && row < p.c_rows;
        if (zero_out && n < hi && !own) p.out[b * p.out_ld + n] = 0.f;
        const uint64_t m = __ballot(own);
        const int cnt = __popcll(m);
        const int n32 = (int)n;
        if (cnt == 0) continue;  // wave-uniform
        const int row32 = (int)row;
        // lanes [fill, min(fill + cnt, 64)) take the first owned candidates of this chunk
        const int d = lane - fill;
        const bool take = d >= 0 && d < cnt;
        const int src = kth_set_bit(m, take ? d : 0);
        const int r1 = lane_pull(row32, src), n1 = lane_pull(n32, src);
        if (take) {
            buf_row = r1;
            buf_n = n1;
        }
        if (fill + cnt >= kWave) {
            body(buf_row, buf_n, kWave);
            // the chunk's remaining owned candidates [64 - fill, cnt) move to lanes [0, fill + cnt - 64)
            const int rest = fill + cnt - kWave;
            const int src2 = kth_set_bit(m, lane < rest ? (kWave - fill) + lane : 0);
            buf_row = lane_pull(row32, src2);
            buf_n = lane_pull(n32, src2);
            fill = rest;
        } else {
            fill += cnt;
        }
    }
    if (fill > 0) body(buf_row, buf_n, fill);
}

// Scores the owned candidates of [lo, hi) of row b (foreign ones score 0 in p.out): kge_score_sharded.
template <int FN, bool CH, int V, int G>
__device__ __forceinline__ void score_owned(const ScoreParams& p, const Query<FN, CH, V, G>& q, int64_t b, int64_t lo,
                                            int64_t hi, int lane) {
    for_owned_runs(p, b, lo, hi, lane, true, [&](int row, int n, int cnt) {
        const int64_t my_id = (int64_t)row + p.c_base;
        float2 st;
        const float s = score_lanes<FN, CH, V, G, false>(p, q, my_id, cnt, lane, st);
        if (lane < cnt) p.out[b * p.out_ld + n] = s;
    });
}

// ---------------------------------------------------------------------------------------------
// XCD-sliced scoring (kge_step_forward's negatives, KIND_STEP_FWD_XCD). The entity table is cut into 8
// slices of S = ceil(E / 8) rows; block i scores, for the 4 batch rows b = 4 (i / 8) + w, only the
// candidates whose id falls in slice x = i % 8. Blocks i and i + 8 share an XCD (round-robin dispatch),
// so every gather of an entity row is issued by one XCD, and each wave walks its candidates in
// ascending id order: the XCD's waves sweep their slice together and the repeat gathers of a row (row
// reuse ~3.4x at C2) hit that XCD's L2 or the Infinity Cache instead of HBM (tools/locality_probe.hip:
// the same gathers run 0.84-0.86x the time of the batch-row-major order). The scores are those of
// step_fwd_kernel bitwise (same query build, same per-candidate code).
// ---------------------------------------------------------------------------------------------
// Walks the ids of batch row b, compacting the candidates of slice [e_lo, e_hi) (and, with
// take_invalid, every id outside [0, c_rows), which scores against a zero row) into lanes; calls
// body(id32, n, cnt) with up to 64 of them, sorted by id (id32 = id, or -1 for an invalid one; n its
// candidate column).
// Ids are global: the table holds rows [c_base, c_base + c_rows) (a shard, or the whole table with c_base
// = 0); e_lo, e_hi are global too. With zero_foreign, the score of every id outside the table is written 0
// (the sharded scorer's partial block, which a SUM over the shards assembles).
template <class Body>
__device__ __forceinline__ void for_slice_runs_sorted(const ScoreParams& p, int64_t b, int64_t e_lo, int64_t e_hi,
                                                      bool take_invalid, bool zero_foreign, int lane, Body&& body) {
    int buf_key = INT32_MAX, buf_id = -1, buf_n = 0, fill = 0;
    auto flush = [&](int cnt) {
        // sort key: (id - e_lo) << 6 | source lane (invalid ids first, as id - e_lo = 0)
        const int key = wave_sort_asc(lane < cnt ? buf_key : INT32_MAX, lane);
        const int src = key & (kWave - 1);
        const int id = lane_pull(buf_id, src), n = lane_pull(buf_n, src);
        body(id, n, cnt);
    };
    for (int64_t c0 = 0; c0 < p.N; c0 += kWave) {
        const int64_t n = c0 + lane;
        int64_t id = -1;
        if (n < p.N) id = p.c_idx[b * p.c_stride + n];
        const bool valid = id >= p.c_base && id < p.c_base + p.c_rows;
        const bool own = n < p.N && (valid ? (id >= e_lo && id < e_hi) : take_invalid);
        if (zero_foreign && n < p.N && !valid) p.out[b * p.out_ld + n] = 0.f;
        const int n32 = (int)n;
        const uint64_t m = __ballot(own);
        const int cnt = __popcll(m);
        if (cnt == 0) continue;  // wave-uniform
        const int id32 = valid ? (int)id : -1, rl = valid ? (int)(id - e_lo) : 0;
        const int d = lane - fill;
        const bool take = d >= 0 && d < cnt;
        const int src = kth_set_bit(m, take ? d : 0);
        const int i1 = lane_pull(id32, src), n1 = lane_pull(n32, src), r1 = lane_pull(rl, src);
        if (take) {
            buf_id = i1;
            buf_n = n1;
            buf_key = (r1 << 6) | lane;
        }
        if (fill + cnt >= kWave) {
            flush(kWave);
            const int rest = fill + cnt - kWave;
            const int src2 = kth_set_bit(m, lane < rest ? (kWave - fill) + lane : 0);
            buf_id = lane_pull(id32, src2);
            buf_n = lane_pull(n32, src2);
            buf_key = (lane_pull(rl, src2) << 6) | lane;
            fill = rest;
        } else {
            fill += cnt;
        }
    }
    if (fill > 0) flush(fill);
}

// The XCD-sliced kernel also scores the row's positive triple (single mode, tail formula, model.py:127-146):
// the wave whose slice holds the positive's tail does it (slice 0 for an out-of-range tail). The row's
// self-adversarial reduction needs every slice's scores and runs in neg_rows_kernel after it.
// One candidate row in registers at a time (score_lanes<DEPTH = 1>) and 4 waves per SIMD up to D = 1024:
// every wave of a C2-sized launch (8 x 512) is resident at once, so the XCDs' sweeps stay together
// (2-deep pipelining at 3 waves per SIMD measured 140 us against 133 us for this form at C2).
// Phases (p.xcd_phases = P > 1): the table is cut into 8 P slices and the grid into P consecutive runs of
// blocks, run f taking slices 8 f .. 8 f + 7: blocks are dispatched in order, so the chip sweeps 1/P of
// the table at a time and the repeat gathers of a phase hit a working set P times smaller (the Infinity
// Cache's 256 MB against a C2 table of 327.5 MB). Every candidate is still scored by the same code.
template <int FN, bool CH, int V, int G>
__global__ __attribute__((amdgpu_flat_work_group_size(1, kBlock), amdgpu_waves_per_eu(G <= 4 ? 4 : 1))) void
step_fwd_xcd_kernel(ScoreParams p) {
    __shared__ vecf<V> q2img[kWavesPerBlock][FN == KGE_INTERHT ? G * kWave : 1];
    const int P = p.xcd_phases > 1 ? p.xcd_phases : 1;
    const int64_t per_phase = (p.B + kWavesPerBlock - 1) / kWavesPerBlock * 8;  // blocks of one phase
    const int phase = (int)(blockIdx.x / per_phase);
    const int64_t bi = blockIdx.x - phase * per_phase;
    const int x = (int)(bi & 7) + 8 * phase;  // slice
    const int w = threadIdx.x >> 6;
    const int64_t b = (bi >> 3) * kWavesPerBlock + w;
    if (b >= p.B) return;
    const int lane = threadIdx.x & 63;
    const int64_t S = (p.c_rows + 8 * P - 1) / (8 * P);
    const int64_t e_lo = min((int64_t)x * S, p.c_rows), e_hi = min(p.c_rows, e_lo + S);
    const int64_t t = p.pos_base[b * 3 + 2];
    const bool t_here = (t >= 0 && t < p.c_rows) ? (t >= e_lo && t < e_hi) : x == 0;
    Query<FN, CH, V, G> q;
    int64_t qi, ri;
    bool qok, rok;
    build_query_for<FN, CH, V, G>(p, b, lane, q, qi, ri, qok, rok);
    auto run = [&](const auto& qq) {
        for_slice_runs_sorted(p, b, e_lo, e_hi, x == 0, false, lane, [&](int id, int n, int cnt) {
            float2 st;
            // one row in flight: two (C4, DistMult d = 500, 59 VGPRs) measured 128.5-129 us against 124-126 us
            const float s = score_lanes<FN, CH, V, G, false, std::decay_t<decltype(qq)>, 1>(p, qq, (int64_t)id, cnt, lane, st);
            if (lane < cnt) p.out[b * p.out_ld + n] = s;
        });
        if (!t_here) return;  // wave-uniform
        bool ok;
        Cand<FN, V, G> c;
        c.load(cand_row(p, t, ok), ok, p.D, lane);
        float s;
        if constexpr (!CH) {  // tail-batch: the positive's query (h, r) is the negatives' query
            s = cand_score<FN, false, V, G>(c, fresh(qq), p);
        } else {
            Query<FN, false, V, G> qp;
            const int64_t hi = p.pos_base[b * 3], rj = p.pos_base[b * 3 + 1];
            const bool hok = hi >= 0 && hi < p.q_rows, rjok = rj >= 0 && rj < p.r_rows;
            qp.build(p.qent + (hok ? hi : 0) * p.q_ld, hok, p.rel + (rjok ? rj : 0) * p.r_ld + p.r_off, rjok, p.D,
                     lane, p);
            s = cand_score<FN, false, V, G>(c, qp, p);
        }
        if (lane == 0) {
            if (p.out_pos_raw) p.out_pos_raw[b] = s;
            p.out_pos_ls[b] = log_sigmoid(s);
        }
    };
    if constexpr (FN == KGE_INTERHT) {
        QueryL2<FN, CH, V, G> ql;
#pragma unroll
        for (int k = 0; k < G; ++k) {
            q2img[w][lane + k * kWave] = q.q2[k];
            ql.q0[k] = q.q0[k];
            ql.q1[k] = q.q1[k];
        }
        ql.q2 = LdsOperand<V>{q2img[w], lane};
        run(ql);
    } else {
        run(q);
    }
}


// ---------------------------------------------------------------------------------------------
// Row-group tiles (kge_step_forward KIND_STEP_FWD_TILE, kge_score_indexed KIND_SCORE_TILE). Block i takes
// entity slice x = i % 8 of the table (S = ceil(c_rows / 8) rows; blocks i and i + 8 share an XCD) and the
// R = p.tile_rows batch rows [g R, g R + R), g = i / 8:
//   1. the R rows' query operands are built once into LDS (InterHT's third operand, the relation's middle
//      third, stays in the relation table: it is re-read per candidate from L2);
//   2. the rows' candidates that fall in slice x (slice 0 also takes the out-of-range ids, which score
//      against a zero row), plus, with tile_pos, each row's positive whose tail falls there, are counting-
//      sorted into kTileBuckets entity buckets in LDS (order inside a bucket: arbitrary);
//   3. the block's NWV waves (12 for candidate rows of 4 KB or more, else 16) take the sorted list round-robin,
//      two candidate rows in flight per wave; head-batch positives (their own (h, r) query) after the sweep.
// The block sweeps its slice in ONE ascending front, and the ~32 blocks of an XCD sweep the same slice
// together, so the ~3.4 gathers of an entity row (C2) are issued by one XCD close in time and the repeats
// hit its L2. Against step_fwd_xcd_kernel (one wave per (row, slice, phase), which rebuilds its row's query
// and walks its row's ids once per phase) a row's query is built 8 times per launch, not 8 P times.
// Every candidate is scored by cand_score with the same operand values as every other form: the scores
// are bitwise those of step_fwd_kernel / step_fwd_xcd_kernel.
// LDS (dynamic, p.tile_lds bytes): query images [R][tile_nq][G * 64] vecf<V>, relation rows, batch rows and
// query entity ids [R] (int64 each),
// bucket counts / cursors [kTileBuckets], the item count, the sorted list [R (N + 1)] of (row << 16 | column)
// (column N: the row's positive).
// ---------------------------------------------------------------------------------------------
template <int V, int G>
struct TileQueryIH {  // InterHT: q0, q1 from LDS, the relation third in registers
    LdsOperand<V> q0, q1;
    vecf<V> q2[G];
};

// One group of a step plan (kge_internal.h: the plan layout), made by one block of NWV waves: the group's batch
// rows (InterHT: ranks [g R, g R + R) of the batch in (relation, row) order, the same stable counting sort as
// step_fwd_tile_kernel's step 0; else rows g R + r), their positives, and the group's items — every candidate
// of its rows, and in tail-batch mode each row's positive as column N — counting-sorted by (entity slice,
// entity bucket) into the group's list. The tile kernel's block (g, x) then sweeps list[soff[x], soff[x + 1]).
// Order inside a bucket: arbitrary (LDS atomics); every item is scored on its own, so the scores do not depend
// on it. sm: plan_lds_ints(NWV * 64) ints of LDS.
template <int NWV>
__device__ void tile_plan_group(const PlanArgs& a, int g, int* sm) {
    constexpr int NT = NWV * kWave, NB = kTileSortRel, MU = (kTileSortMaxB + NT - 1) / NT;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int R = a.R;
    const int64_t g0 = (int64_t)g * R;
    const int nr = (int)min<int64_t>(R, a.B - g0);
    int* brow = sm;                        // [kTileMaxRows]
    int* hist = brow + kTileMaxRows;       // [8][kTileBuckets]
    int* wc = hist + 8 * kTileBuckets;     // [MU NWV][NB] the sort's per-wave bucket counts
    if (a.sort) {  // step_fwd_tile_kernel's step 0 on the relation ids pos[i][1]
        int bk[MU], wr[MU];
        int64_t rv[MU];
#pragma unroll
        for (int u = 0; u < MU; ++u) rv[u] = a.pos[min<int64_t>(u * NT + t, a.B - 1) * 3 + 1];  // all in flight
#pragma unroll
        for (int u = 0; u < MU; ++u) {
            const int64_t rr = rv[u];
            bk[u] = u * NT + t >= a.B ? NB : ((rr >= 0 && rr < a.nrel) ? (int)min<int64_t>(rr, NB - 2) : NB - 1);
        }
        for (int i = t; i < MU * NWV * NB; i += NT) wc[i] = 0;
        __syncthreads();
#pragma unroll
        for (int u = 0; u < MU; ++u) {
            wr[u] = 0;
            if (u * NT >= a.B) continue;  // block-uniform
            uint64_t todo = __ballot(bk[u] < NB);
            while (todo) {
                const int v = __builtin_amdgcn_readlane(bk[u], __builtin_ctzll(todo));
                const uint64_t m = __ballot(bk[u] == v);
                if (bk[u] == v) wr[u] = lanes_below(m);
                if (lane == 0) wc[(u * NWV + w) * NB + v] = __popcll(m);
                todo &= ~m;
            }
        }
        __syncthreads();
        if (w == 0) {
            int y[MU * NWV];
#pragma unroll
            for (int c = 0; c < MU * NWV; ++c) y[c] = wc[c * NB + lane];
            int run = 0;
#pragma unroll
            for (int c = 0; c < MU * NWV; ++c) {
                const int v = y[c];
                y[c] = run;
                run += v;
            }
            int incl = run;
#pragma unroll
            for (int o = 1; o < kWave; o <<= 1) {
                const int v = __shfl_up(incl, o, kWave);
                if (lane >= o) incl += v;
            }
            const int base = incl - run;
#pragma unroll
            for (int c = 0; c < MU * NWV; ++c) wc[c * NB + lane] = y[c] + base;
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < MU; ++u) {
            if (bk[u] >= NB) continue;
            const int64_t rank = wc[(u * NWV + w) * NB + bk[u]] + wr[u];
            if (rank >= g0 && rank < g0 + nr) brow[rank - g0] = u * NT + t;
        }
    } else if (t < nr) {
        brow[t] = (int)(g0 + t);
    }
    for (int i = t; i < 8 * kTileBuckets; i += NT) hist[i] = 0;
    __syncthreads();
    // the items: (slice, bucket) key, checked id, code
    const int Np = a.mode == KGE_HEAD_BATCH ? (int)a.N : (int)a.N + 1;
    const int nf = nr * Np;
    const int64_t S = (a.nent + 7) / 8;
    const int S32 = (int)S;  // nent < 2^31 (kge_step_plan_size): slice math in 32 bits
    const float invS = 1.f / (float)S, bscale = (float)kTileBuckets / (float)S, inv_np = 1.f / (float)Np;
    // an item's id, by address select and one load (no branch: a walk's loads all go out together)
    auto item_row = [&](int f, int& r) {
        r = (int)((float)f * inv_np);  // f < 2^21: the float quotient corrected to the exact one
        if (r * Np > f) --r;
        if ((r + 1) * Np <= f) ++r;
        const int n = f - r * Np;
        const int64_t b = brow[r];
        const int64_t* src = n < a.N ? a.neg + b * a.neg_ld + n : a.pos + b * 3 + 2;
        return src;
    };
    auto classify = [&](int f, int r, int64_t id, int& key, int& idc, int& code) {
        const int n = f - r * Np;
        const bool valid = id >= 0 && id < a.nent;
        const int i32 = valid ? (int)id : 0;
        int x = min(7, (int)((float)i32 * invS));  // the products below stay <= 7 S < 2^31
        if (x * S32 > i32) --x;
        if (x < 7 && (x + 1) * S32 <= i32) ++x;
        const int bk = valid ? min(kTileBuckets - 1, (int)((float)(i32 - x * S32) * bscale)) : 0;
        if (!valid) x = 0;
        key = x * kTileBuckets + bk;
        idc = valid ? (int)id : -1;
        code = (r << 16) | n;
    };
    auto item = [&](int f, int& key, int& idc, int& code) {
        int r;
        const int64_t id = *item_row(f, r);
        classify(f, r, id, key, idc, code);
    };
    constexpr int TPI = 17;  // C2's 16 x 257 items over 768 threads walked once; larger groups twice
    const bool in_regs = nf <= TPI * NT;
    int ky[TPI], ic[TPI], cd[TPI], rk[TPI];
    // the rows' positives (b, h, r, t), loaded with the walk's ids (one round trip), stored at the end
    int64_t ph = -1, pr = -1, pt = -1;
    if (t < nr) {
        const int64_t b = brow[t];
        ph = a.pos[b * 3];
        pr = a.pos[b * 3 + 1];
        pt = a.pos[b * 3 + 2];
    }
    if (in_regs) {
        int64_t idv[TPI];
        int rr[TPI];
#pragma unroll
        for (int u = 0; u < TPI; ++u) idv[u] = *item_row(min(u * NT + t, nf - 1), rr[u]);
#pragma unroll
        for (int u = 0; u < TPI; ++u) {
            const int f = u * NT + t;
            ky[u] = -1;
            if (f < nf) classify(f, rr[u], idv[u], ky[u], ic[u], cd[u]);
        }
        // the counting atomic's old value is the item's rank in its bin: the scatter then needs no second atomic
#pragma unroll
        for (int u = 0; u < TPI; ++u)
            if (ky[u] >= 0) rk[u] = atomicAdd(&hist[ky[u]], 1);
    } else {
        for (int f = t; f < nf; f += NT) {
            int k, i, c;
            item(f, k, i, c);
            atomicAdd(&hist[k], 1);
        }
    }
    __syncthreads();
    if (w == 0) {  // exclusive scan of the 8 x 256 counts, 32 per lane; the slice starts
        constexpr int PL = 8 * kTileBuckets / kWave;
        int v[PL], sum = 0;
#pragma unroll
        for (int i = 0; i < PL; ++i) {
            v[i] = hist[lane * PL + i];
            sum += v[i];
        }
        int incl = sum;
#pragma unroll
        for (int o = 1; o < kWave; o <<= 1) {
            const int y = __shfl_up(incl, o, kWave);
            if (lane >= o) incl += y;
        }
        int run = incl - sum;
        int* soff = a.plan + plan_soff(a.B, R) + (int64_t)g * 9;
        if ((lane * PL) % kTileBuckets == 0) soff[lane * PL / kTileBuckets] = run;  // slice x starts at lane 8 x
        if (lane == kWave - 1) soff[8] = incl;
#pragma unroll
        for (int i = 0; i < PL; ++i) {
            hist[lane * PL + i] = run;
            run += v[i];
        }
    }
    __syncthreads();
    int2* list = reinterpret_cast<int2*>(a.plan + plan_list(a.B, R)) + (int64_t)g * R * (a.N + 1);
    if (in_regs) {
#pragma unroll
        for (int u = 0; u < TPI; ++u)
            if (ky[u] >= 0) list[hist[ky[u]] + rk[u]] = make_int2(ic[u], cd[u]);
    } else {
        for (int f = t; f < nf; f += NT) {
            int k, i, c;
            item(f, k, i, c);
            list[atomicAdd(&hist[k], 1)] = make_int2(i, c);
        }
    }
    // the rows' (b, h, r, t), ids checked (-1: out of range); the header
    auto chk = [](int64_t id, int64_t n) { return (id >= 0 && id < n) ? (int)id : -1; };
    if (t < R)
        reinterpret_cast<int4*>(a.plan + kPlanHdr)[(int64_t)g * R + t] =
            t < nr ? make_int4(brow[t], chk(ph, a.nent), chk(pr, a.nrel), chk(pt, a.nent)) : make_int4(-1, -1, -1, -1);
    if (g == 0 && t == 0) {
        int* h = a.plan;
        h[0] = kPlanMagic;
        h[1] = (int)a.B;
        h[2] = (int)a.N;
        h[3] = a.mode;
        h[4] = R;
        h[5] = (int)a.nent;
        h[6] = a.sort;
    }
}

// kge_step_plan: a batch's plan on its own (the first batch of a planned run; later plans come from the tail
// blocks of the step before)
template <int NWV>
__global__ __launch_bounds__(NWV * kWave) void tile_plan_kernel(PlanArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char plan_smem[];
    tile_plan_group<NWV>(a, (int)blockIdx.x, reinterpret_cast<int*>(plan_smem));
}

template <int FN, bool CH, int V, int G, int NWV>
__global__ __launch_bounds__(NWV * kWave) void step_fwd_tile_kernel(ScoreParams p) {
    extern __shared__ __attribute__((aligned(16))) unsigned char tile_smem[];
    constexpr int NQ = tile_nq(FN);
    constexpr int W = G * kWave;
    constexpr int NT = NWV * kWave;
    const int R = p.tile_rows, QS = p.tile_q2slots;
    vecf<V>* qimg = reinterpret_cast<vecf<V>*>(tile_smem);  // [R][NQ][W]
    vecf<V>* q2img = qimg + (size_t)R * NQ * W;               // [QS][W] InterHT relation thirds
    int64_t* rrow = reinterpret_cast<int64_t*>(q2img + (size_t)QS * W);
    int64_t* brow = rrow + R;
    int64_t* qid = brow + R;  // the rows' query entity ids, read with the relation ids in step 0
    int* q2slot = reinterpret_cast<int*>(qid + R);
    int* hist = q2slot + R;
    int* cntp = hist + kTileBuckets;
    int* list = cntp + 4;  // also the relation sort's keys before the list is built
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    if (p.tile_next.plan && (int)blockIdx.x >= p.tile_blocks) {
        // a tail block: the NEXT batch's plan, on the CUs the scoring blocks free up at the end of the launch
        tile_plan_group<NWV>(p.tile_next, (int)blockIdx.x - p.tile_blocks, reinterpret_cast<int*>(tile_smem));
        return;
    }
    const int x = (int)(blockIdx.x & 7);
    const int gi = (int)(blockIdx.x >> 3);
    const int64_t g0 = (int64_t)gi * R;
    const int nr = (int)min<int64_t>(R, p.B - g0);
    if (nr <= 0) return;  // block-uniform
    // a planned step (kge_step_forward_planned): rows, ids and this block's sorted items come from the plan
    const int* pl = p.tile_plan;
    const int4* pmeta = pl ? reinterpret_cast<const int4*>(pl + kPlanHdr) + (int64_t)gi * R : nullptr;
    const int2* plist = pl ? reinterpret_cast<const int2*>(pl + plan_list(p.B, R)) + (int64_t)gi * R * (p.N + 1) : nullptr;
    int plo = 0, pcnt = 0;
    if (pl) {
        const int mode = CH ? KGE_HEAD_BATCH : KGE_TAIL_BATCH;
        if (pl[0] != kPlanMagic || pl[1] != (int)p.B || pl[2] != (int)p.N || pl[3] != mode || pl[4] != R ||
            pl[5] != (int)p.c_rows || (pl[6] != 0) != (p.tile_sort != 0)) {
            // not this batch shape's plan (or a plan made for a score function with the other row order): every
            // output of the block's rows (by index) becomes NaN, loudly. A plan of the same shape made from other
            // ids is not detectable here: kge_step_planner_* (ops.StepPlanner) pairs plans with batches
            if (x == 0)
                for (int r = w; r < nr; r += NWV) {
                    for (int64_t n = lane; n < p.N; n += kWave) p.out[(g0 + r) * p.out_ld + n] = __builtin_nanf("");
                    if (lane == 0) {
                        if (p.out_pos_raw) p.out_pos_raw[g0 + r] = __builtin_nanf("");
                        p.out_pos_ls[g0 + r] = __builtin_nanf("");
                    }
                }
            return;
        }
        const int* so = pl + plan_soff(p.B, R) + (int64_t)gi * 9;
        plo = so[x];
        pcnt = so[x + 1] - plo;
    }
    const int64_t S = (p.c_rows + 7) / 8;
    const int64_t e_lo = min((int64_t)x * S, p.c_rows), e_hi = min(p.c_rows, e_lo + S);
    // column N: the row's positive (its tail) in tail-batch mode, where it shares the negatives' query; head-batch
    // positives need their own (h, r) query and are scored after the sweep
    const int64_t Np = (p.tile_pos && !CH) ? p.N + 1 : p.N;

    // 0. the block's batch rows: ranks [g0, g0 + nr) of the batch in (relation, row) order (p.tile_sort: InterHT,
    //    so that a block's rows share few relations and their relation thirds fit QS LDS slots), else rows g0 + r.
    //    A stable counting sort over kTileSortRel relation buckets: row i = (u NWV + w) 64 + lane is ranked inside
    //    its wave by ballots (one per distinct bucket of the wave), then by the bucket counts of the earlier waves.
    if (pl) {
        if (t < nr) {
            const int4 m = pmeta[t];
            brow[t] = m.x;
            qid[t] = CH ? m.w : m.y;
            rrow[t] = m.z;
        }
    } else if (p.tile_sort) {
        constexpr int MU = (kTileSortMaxB + NT - 1) / NT, NB = kTileSortRel;
        int* wc = list;  // [MU NWV][NB] per-wave bucket counts, then their exclusive prefixes
        int bk[MU], wr[MU];
        int64_t rv[MU], qv[MU];
#pragma unroll
        for (int u = 0; u < MU; ++u) {
            const int i = u * NT + t;
            bk[u] = NB;
            rv[u] = qv[u] = 0;
            if (i < p.B) {
                const int64_t rr = p.r_idx ? p.r_idx[i * p.r_stride] : i;
                rv[u] = rr;
                qv[u] = p.q_idx ? p.q_idx[i * p.q_stride] : i;
                bk[u] = (rr >= 0 && rr < p.r_rows) ? (int)min<int64_t>(rr, NB - 2) : NB - 1;
            }
        }
        for (int i = t; i < MU * NWV * NB; i += NT) wc[i] = 0;
        __syncthreads();
#pragma unroll
        for (int u = 0; u < MU; ++u) {
            wr[u] = 0;
            if (u * NT >= p.B) continue;  // block-uniform
            uint64_t todo = __ballot(bk[u] < NB);
            while (todo) {  // wave-uniform: one round per distinct bucket of the wave
                const int v = __builtin_amdgcn_readlane(bk[u], __builtin_ctzll(todo));
                const uint64_t m = __ballot(bk[u] == v);
                if (bk[u] == v) wr[u] = lanes_below(m);
                if (lane == 0) wc[(u * NWV + w) * NB + v] = __popcll(m);
                todo &= ~m;
            }
        }
        __syncthreads();
        if (w == 0) {  // bucket v = lane: prefix over the waves in row order, then over the buckets
            // (the counts are loaded all together and summed in registers: a dependent LDS round trip per wave
            // slot cost ~1.5 us of the block's setup)
            int y[MU * NWV];
#pragma unroll
            for (int c = 0; c < MU * NWV; ++c) y[c] = wc[c * NB + lane];
            int run = 0;
#pragma unroll
            for (int c = 0; c < MU * NWV; ++c) {
                const int v = y[c];
                y[c] = run;
                run += v;
            }
            int incl = run;
#pragma unroll
            for (int o = 1; o < kWave; o <<= 1) {
                const int v = __shfl_up(incl, o, kWave);
                if (lane >= o) incl += v;
            }
            const int base = incl - run;
#pragma unroll
            for (int c = 0; c < MU * NWV; ++c) wc[c * NB + lane] = y[c] + base;
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < MU; ++u) {
            if (bk[u] >= NB) continue;
            const int64_t rank = wc[(u * NWV + w) * NB + bk[u]] + wr[u];
            if (rank >= g0 && rank < g0 + nr) {
                brow[rank - g0] = u * NT + t;
                qid[rank - g0] = qv[u];
                rrow[rank - g0] = rv[u];
            }
        }
    } else if (t < nr) {
        const int64_t b = g0 + t;
        brow[t] = b;
        qid[t] = p.q_idx ? p.q_idx[b * p.q_stride] : b;
        rrow[t] = p.r_idx ? p.r_idx[b * p.r_stride] : b;
    }
    __syncthreads();
    if (p.tile_dry == 1) return;  // A/B knob KGE_TILE_DRY=<level>: the setup up to this point alone

    // 2. counting sort of the block's items of slice x by entity bucket
    const int64_t nf = (int64_t)nr * Np;
    // no 64-bit divisions in the walk (an emulated int64 divide is ~100 instructions): the item's row by a
    // float reciprocal corrected to the exact quotient (f < R (N + 1) < 2^21), the entity bucket by a float
    // scale (any monotone map of the slice onto the buckets orders the sweep)
    const int Np32 = (int)Np;
    const float inv_np = 1.f / (float)Np32, bscale = (float)kTileBuckets / (float)S;
    auto item = [&](int64_t f64, int& bucket, int& code) -> bool {
        const int f = (int)f64;
        int r = (int)((float)f * inv_np);
        if (r * Np32 > f) --r;
        if ((r + 1) * Np32 <= f) ++r;
        const int n = f - r * Np32;
        const int64_t b = brow[r];
        const int64_t id = n < p.N ? p.c_idx[b * p.c_stride + n] : p.pos_base[b * 3 + 2];
        const int64_t row = id - p.c_base;
        const bool valid = row >= 0 && row < p.c_rows;
        if (valid ? (row < e_lo || row >= e_hi) : x != 0) return false;
        bucket = valid ? min(kTileBuckets - 1, (int)((float)(int)(row - e_lo) * bscale)) : 0;
        code = (r << 16) | n;
        return true;
    };
    // the ids are loaded once, all in flight together, when the block's walk fits TPI per thread (C2: 4 112
    // items over 768 threads); otherwise the walk is made twice (count, then scatter)
    // 17 at 16 waves: a 16-row block's 16 x 1 025 tail-batch items at N = 1 024 (C4) over 1 024 threads, walked
    // once (C4 tail-batch 94.5 -> 88 us); 16 at fewer waves, where the 17th slot measured ~1 us slower at C3
    constexpr int TPI = NWV >= 16 ? 17 : 16;
    int wbk[TPI], wcd[TPI];
    const bool in_regs = !pl && nf <= (int64_t)TPI * NT;  // block-uniform
    // (their loads are issued here, before the query build, so both latencies overlap)
    if (in_regs) {
#pragma unroll
        for (int u = 0; u < TPI; ++u) {
            const int64_t f = (int64_t)u * NT + t;
            wbk[u] = -1;
            if (f < nf && !item(f, wbk[u], wcd[u])) wbk[u] = -1;
        }
    }

    // 1. the rows' query operands; with fewer waves than rows, two rows per wave built side by side (branch-free:
    //    both rows' loads in flight together). The ids come from LDS (step 0 read them with the relation ids), so
    //    the rows' loads are not behind a dependent id load
    auto build_row = [&](int r, Query<FN, CH, V, G>& q, int64_t& ri, bool& rok) {
        const int64_t qi = qid[r];
        ri = rrow[r];  // the raw relation id until put() replaces it with the checked one
        bool qok = qi >= 0 && qi < p.q_rows;
        rok = ri >= 0 && ri < p.r_rows;
        q.build(p.qent + (qok ? qi : 0) * p.q_ld, qok, p.rel + (rok ? ri : 0) * p.r_ld + p.r_off, rok, p.D, lane, p);
    };
    auto put = [&](int r, const Query<FN, CH, V, G>& q, int64_t ri, bool rok) {
        vecf<V>* qr = qimg + (size_t)r * NQ * W;
#pragma unroll
        for (int k = 0; k < G; ++k) {
            qr[lane + k * kWave] = q.q0[k];
            if constexpr (NQ > 1) qr[W + lane + k * kWave] = q.q1[k];
        }
        if (lane == 0) rrow[r] = rok ? ri : -1;
    };
    if constexpr (2 * NWV <= kTileMaxRows) {
        for (int r = w; r < nr; r += 2 * NWV) {
            const int r2 = r + NWV < nr ? r + NWV : r;
            Query<FN, CH, V, G> qa, qb;
            int64_t ri, ri2;
            bool rok, rok2;
            build_row(r, qa, ri, rok);
            build_row(r2, qb, ri2, rok2);
            put(r, qa, ri, rok);
            if (r2 != r) put(r2, qb, ri2, rok2);
        }
    } else {
        for (int r = w; r < nr; r += NWV) {
            Query<FN, CH, V, G> q;
            int64_t ri;
            bool rok;
            build_row(r, q, ri, rok);
            put(r, q, ri, rok);
        }
    }
    for (int i = t; i < kTileBuckets; i += NT) hist[i] = 0;
    __syncthreads();
    if (p.tile_dry == 2) return;
    if constexpr (FN == KGE_INTERHT) {
        // relation slots: one per run of equal relations among the block's rows (first QS runs; the rows of
        // later runs read their relation third from the table per candidate)
        static_assert(kTileMaxRows <= kWave, "one lane per row");
        if (w == 0) {  // lane r: row r opens a run when its relation differs from row r - 1's
            const bool in = lane < nr;
            const int64_t cur = in ? rrow[lane] : 0;
            const bool open = in && (lane == 0 || cur != rrow[lane - 1]);
            const uint64_t m = __ballot(open);
            if (in) {
                const int sl = __popcll(m & (lane == 63 ? ~0ull : (2ull << lane) - 1)) - 1;
                q2slot[lane] = sl < QS ? sl : -1;
            }
        }
    }
    int wrk[TPI];  // the item's rank in its bucket, from the counting atomic (no second atomic in the scatter)
    if (pl) {
    } else if (in_regs) {
#pragma unroll
        for (int u = 0; u < TPI; ++u)
            if (wbk[u] >= 0) wrk[u] = atomicAdd(&hist[wbk[u]], 1);
    } else {
        for (int64_t f = t; f < nf; f += NT) {
            int bk, code;
            if (item(f, bk, code)) atomicAdd(&hist[bk], 1);
        }
    }
    __syncthreads();
    if (p.tile_dry == 3) return;
    if constexpr (FN == KGE_INTERHT) {
        for (int r = w; r < nr; r += NWV) {
            const int sl = q2slot[r];
            if (sl < 0 || (r > 0 && q2slot[r - 1] == sl)) continue;  // wave-uniform: the run's first row fills
            const int64_t ri = rrow[r];
            const rsrc_t sr = make_rsrc(p.rel + (ri >= 0 ? ri : 0) * p.r_ld + p.r_off, ri >= 0 ? (uint32_t)p.D * 4u : 0u);
#pragma unroll
            for (int k = 0; k < G; ++k) q2img[(size_t)sl * W + lane + k * kWave] = bload<V>(sr, goff<V>(lane, k));
        }
    }
    if (!pl && w == 0) {  // exclusive scan of the bucket counts (4 per lane)
        constexpr int PL = kTileBuckets / kWave;
        int v[PL], s = 0;
#pragma unroll
        for (int i = 0; i < PL; ++i) {
            v[i] = hist[lane * PL + i];
            s += v[i];
        }
        int incl = s;
#pragma unroll
        for (int o = 1; o < kWave; o <<= 1) {
            const int y = __shfl_up(incl, o, kWave);
            if (lane >= o) incl += y;
        }
        int run = incl - s;
#pragma unroll
        for (int i = 0; i < PL; ++i) {
            hist[lane * PL + i] = run;
            run += v[i];
        }
        if (lane == kWave - 1) cntp[0] = incl;
    }
    __syncthreads();
    if (pl) {
    } else if (in_regs) {
#pragma unroll
        for (int u = 0; u < TPI; ++u)
            if (wbk[u] >= 0) list[hist[wbk[u]] + wrk[u]] = wcd[u];
    } else {
        for (int64_t f = t; f < nf; f += NT) {
            int bk, code;
            if (item(f, bk, code)) list[atomicAdd(&hist[bk], 1)] = code;
        }
    }
    __syncthreads();
    const int cnt = pl ? pcnt : cntp[0];

    if (p.tile_dry) return;
    // 3. the sweep: wave w takes items w, w + NWV, w + 2 NWV, ...; the next item's
    // candidate row (and InterHT's relation third) is in flight while this one is scored
    struct Item {
        Cand<FN, V, G> c;
        vecf<V> q2[FN == KGE_INTERHT ? G : 1];
    };
    for (int c0 = w; c0 < cnt; c0 += NT) {
        const int nc = min(kWave, (cnt - c0 + NWV - 1) / NWV);
        int code = 0;
        int64_t my_id = 0;
        if (lane < nc) {
            // p.tile_rev: the list walked from its end (descending entity order), the same items
            const int ci = p.tile_rev ? cnt - 1 - (c0 + NWV * lane) : c0 + NWV * lane;
            if (pl) {  // (checked entity id, code): no dependent id load
                const int2 e = plist[plo + ci];
                code = e.y;
                my_id = e.x;
            } else {
                code = list[ci];
                const int r = code >> 16, n = code & 0xFFFF;
                const int64_t b = brow[r];
                my_id = n < p.N ? p.c_idx[b * p.c_stride + n] : p.pos_base[b * 3 + 2];
            }
        }
        auto load = [&](Item& it, int j) {
            bool ok;
            it.c.load(cand_row(p, readlane64(my_id, j), ok), ok, p.D, lane);
            if constexpr (FN == KGE_INTERHT) {
                const int r = __builtin_amdgcn_readlane(code, j) >> 16;
                const int sl = q2slot[r];
                if (sl >= 0) {  // wave-uniform
#pragma unroll
                    for (int k = 0; k < G; ++k) it.q2[k] = q2img[(size_t)sl * W + lane + k * kWave];
                } else {
                    const int64_t ri = rrow[r];
                    const rsrc_t sr = make_rsrc(p.rel + (ri >= 0 ? ri : 0) * p.r_ld + p.r_off,
                                                ri >= 0 ? (uint32_t)p.D * 4u : 0u);
#pragma unroll
                    for (int k = 0; k < G; ++k) it.q2[k] = bload<V>(sr, goff<V>(lane, k));
                }
            }
        };
        auto score = [&](const Item& it, int j) -> float {
            const int cj = __builtin_amdgcn_readlane(code, j);
            const int r = cj >> 16, n = cj & 0xFFFF;
            const vecf<V>* qr = qimg + (size_t)r * NQ * W;
            (void)n;
            if constexpr (FN == KGE_INTERHT) {
                TileQueryIH<V, G> q{{qr, lane}, {qr + W, lane}, {}};
#pragma unroll
                for (int k = 0; k < G; ++k) q.q2[k] = it.q2[k];
                return cand_score<FN, CH, V, G>(it.c, q, p);
            } else {
                const LdsQuery<V> q{{qr, lane}, {qr + (NQ > 1 ? W : 0), lane}, {qr, lane}};
                return cand_score<FN, CH, V, G>(it.c, q, p);
            }
        };
        float my_score = 0.f;
        {
            Item x0, x1;
            load(x0, 0);
            for (int j = 0; j < nc; j += 2) {
                if (j + 1 < nc) load(x1, j + 1);
                float s = score(x0, j);
                if (lane == j) my_score = s;
                if (j + 1 < nc) {
                    if (j + 2 < nc) load(x0, j + 2);
                    s = score(x1, j + 1);
                    if (lane == j + 1) my_score = s;
                }
            }
        }
        if (lane < nc) {
            const int r = code >> 16, n = code & 0xFFFF;
            const int64_t b = brow[r];
            if (n < p.N) {
                p.out[b * p.out_ld + n] = my_score;
            } else {
                if (p.out_pos_raw) p.out_pos_raw[b] = my_score;
                p.out_pos_ls[b] = log_sigmoid(my_score);
            }
        }
    }
    if constexpr (CH) {
        if (!p.tile_pos) return;
        // head-batch positives whose tail falls in this slice: the single-mode (h, r) query, tail formula
        // (model.py:127-146), one wave per row
        for (int r = w; r < nr; r += NWV) {
            const int64_t b = brow[r];
            const int4 pm = pl ? pmeta[r] : make_int4(0, 0, 0, 0);
            const int64_t tt = pl ? pm.w : p.pos_base[b * 3 + 2], row = tt - p.c_base;
            const bool valid = row >= 0 && row < p.c_rows;
            if (valid ? (row < e_lo || row >= e_hi) : x != 0) continue;  // wave-uniform
            Query<FN, false, V, G> qp;
            const int64_t hi = pl ? pm.y : p.pos_base[b * 3], rj = pl ? pm.z : p.pos_base[b * 3 + 1];
            const bool hok = hi >= 0 && hi < p.q_rows, rjok = rj >= 0 && rj < p.r_rows;
            qp.build(p.qent + (hok ? hi : 0) * p.q_ld, hok, p.rel + (rjok ? rj : 0) * p.r_ld + p.r_off, rjok, p.D,
                     lane, p);
            bool ok;
            Cand<FN, V, G> c;
            c.load(cand_row(p, tt, ok), ok, p.D, lane);
            const float s = cand_score<FN, false, V, G>(c, qp, p);
            if (lane == 0) {
                if (p.out_pos_raw) p.out_pos_raw[b] = s;
                p.out_pos_ls[b] = log_sigmoid(s);
            }
        }
    }
}

// Scoring in the XCD-sliced order (kge_score_indexed / kge_score_sharded, N >= 128): the table's rows
// [c_base, c_base + c_rows) are cut into 8 slices and scored as step_fwd_xcd_kernel scores them, without the
// positives. Sharded (skip_foreign): a candidate outside the shard scores 0 (written by the slice-0 wave);
// at the north star's 8-way split of YAGO3-10 a slice is 3.9 MB, so each XCD's L2 holds its whole slice
// while its waves sweep it. Unsharded: out-of-range ids go to slice 0 and score against a zero row.
template <int FN, bool CH, int V, int G>
__global__ __attribute__((amdgpu_flat_work_group_size(1, kBlock), amdgpu_waves_per_eu(G <= 4 ? 4 : 1))) void
score_sharded_xcd_kernel(ScoreParams p) {
    __shared__ vecf<V> q2img[kWavesPerBlock][FN == KGE_INTERHT ? G * kWave : 1];
    const int x = blockIdx.x & 7;
    const int w = threadIdx.x >> 6;
    const int64_t b = (int64_t)(blockIdx.x >> 3) * kWavesPerBlock + w;
    if (b >= p.B) return;
    const int lane = threadIdx.x & 63;
    const int64_t S = (p.c_rows + 7) / 8;
    const int64_t e_lo = p.c_base + min((int64_t)x * S, p.c_rows), e_hi = p.c_base + min(p.c_rows, (int64_t)(x + 1) * S);
    Query<FN, CH, V, G> q;
    int64_t qi, ri;
    bool qok, rok;
    build_query_for<FN, CH, V, G>(p, b, lane, q, qi, ri, qok, rok);
    auto run = [&](const auto& qq) {
        const bool sh = p.skip_foreign != 0;
        for_slice_runs_sorted(p, b, e_lo, e_hi, !sh && x == 0, sh && x == 0, lane, [&](int id, int n, int cnt) {
            float2 st;
            const float s = score_lanes<FN, CH, V, G, false, std::decay_t<decltype(qq)>, 1>(p, qq, (int64_t)id, cnt, lane, st);
            if (lane < cnt) p.out[b * p.out_ld + n] = s;
        });
    };
    if constexpr (FN == KGE_INTERHT) {
        QueryL2<FN, CH, V, G> ql;
#pragma unroll
        for (int k = 0; k < G; ++k) {
            q2img[w][lane + k * kWave] = q.q2[k];
            ql.q0[k] = q.q0[k];
            ql.q1[k] = q.q1[k];
        }
        ql.q2 = LdsOperand<V>{q2img[w], lane};
        run(ql);
    } else {
        run(q);
    }
}

// ---------------------------------------------------------------------------------------------
// The row-sharded forward's owner-computes scoring (kge_shard_score, KIND_SHARD_BUCKET). Block i scores,
// for the 4 batch rows b = 4 (i / 8) + w, slice x = i % 8 of each row's bucket (kge_shard_plan: this
// rank's owned candidates grouped by XCD slice of S = ceil(rows / 8) shard rows), so, as in
// step_fwd_xcd_kernel, every gather of a shard row is issued by one XCD and each XCD's waves sweep their
// slice together (3.9 MB at the north star's 8-way YAGO3-10 split: the XCD's L2 holds it). A wave reads its
// ~N / 64 entries with one load per 64 (no walk over the row's ids), sorts them by row, gathers and scores
// them two rows deep and writes each score at the row's compact run start + its rank: the send
// block of the score all-to-all. Head-batch positives: the exchanged block holds the TAIL (the negatives'
// query entity), so the wave of the head's slice on the head's owner scores query (h, r), built from its
// shard row, against the tail row (the single-mode formula, bitwise every other positive's).
// ---------------------------------------------------------------------------------------------
template <int FN, bool CH, int V, int G>
__global__ __attribute__((amdgpu_flat_work_group_size(1, kBlock), amdgpu_waves_per_eu(G <= 4 ? 4 : 1))) void
shard_bucket_kernel(ScoreParams p) {
    __shared__ vecf<V> q2img[kWavesPerBlock][FN == KGE_INTERHT ? G * kWave : 1];
    const int x = blockIdx.x & 7;
    const int w = threadIdx.x >> 6;
    const int64_t b = (int64_t)(blockIdx.x >> 3) * kWavesPerBlock + w;
    if (b >= p.B) return;
    const int lane = threadIdx.x & 63;
    const int e0 = p.bk_start[b * 9 + x], e1 = p.bk_start[b * 9 + x + 1];
    const int64_t S = (p.c_rows + 7) / 8;
    int64_t hloc = -1;
    bool pos_here = false;
    if constexpr (CH) {
        hloc = p.pos_base[b * 3] - p.c_base;
        pos_here = hloc >= 0 && hloc < p.c_rows && hloc / S == x;
    }
    if (e0 >= e1 && !pos_here) return;  // wave-uniform
    const int64_t off = cmp_row_off(p, b);
    if (e0 < e1) {
        Query<FN, CH, V, G> q;
        int64_t qi, ri;
        bool qok, rok;
        build_query_for<FN, CH, V, G>(p, b, lane, q, qi, ri, qok, rok);
        const int2* ent = p.bk_ent + b * p.bk_ld;
        const int sl0 = (int)(x * S);
        auto run = [&](const auto& qq) {
            for (int s0 = e0; s0 < e1; s0 += kWave) {
                const int cnt = min(kWave, e1 - s0);
                const int2 e = lane < cnt ? ent[s0 + lane] : make_int2(0, 0);
                // ascending rows: key = (row - slice start) << 6 | lane
                const int key = wave_sort_asc(lane < cnt ? ((e.x - sl0) << 6) | lane : INT32_MAX, lane);
                const int src = key & (kWave - 1);
                const int row = lane_pull(e.x, src), k = lane_pull(e.y, src);
                float2 st;
                const float sc = score_lanes<FN, CH, V, G, false, std::decay_t<decltype(qq)>, (FN == KGE_INTERHT ? 1 : 2)>(
                    p, qq, (int64_t)row + p.c_base, cnt, lane, st);
                if (lane < cnt) p.out[off + k] = sc;
            }
        };
        if constexpr (FN == KGE_INTERHT) {
            QueryL2<FN, CH, V, G> ql;
#pragma unroll
            for (int k = 0; k < G; ++k) {
                q2img[w][lane + k * kWave] = q.q2[k];
                ql.q0[k] = q.q0[k];
                ql.q1[k] = q.q1[k];
            }
            ql.q2 = LdsOperand<V>{q2img[w], lane};
            run(ql);
        } else {
            run(q);
        }
    }
    if constexpr (CH) {
        if (!pos_here) return;  // wave-uniform
        const int64_t rj = p.pos_base[b * 3 + 1];
        const bool rok = rj >= 0 && rj < p.r_rows;
        Query<FN, false, V, G> qp;
        qp.build(p.cent + hloc * p.c_ld, true, p.rel + (rok ? rj : 0) * p.r_ld + p.r_off, rok, p.D, lane, p);
        const int64_t ti = p.q_idx[b * p.q_stride];
        const bool tok = ti >= 0 && ti < p.q_rows;
        Cand<FN, V, G> c;
        c.load(p.qent + (tok ? ti : 0) * p.q_ld, tok, p.D, lane);
        const float sc = cand_score<FN, false, V, G>(c, qp, p);
        if (lane == 0) p.out[off + p.cmp_cnt[b] - 1] = sc;
    }
}

template <int FN, bool CH, int V, int G, bool ST = false>
__global__ __launch_bounds__(kBlock) void score_fwd_kernel(ScoreParams p) {
    WaveTask t;
    if (!wave_task(p, t)) return;
    const int lane = threadIdx.x & 63;
    Query<FN, CH, V, G> q;
    int64_t qi, ri;
    bool qok, rok;
    build_query_for<FN, CH, V, G>(p, t.b, lane, q, qi, ri, qok, rok);
    if (!ST && p.skip_foreign)
        score_owned<FN, CH, V, G>(p, q, t.b, t.n0, t.n0 + t.nc, lane);  // runs of up to cpw (> 64) candidates
    else
        score_run<FN, CH, V, G, ST>(p, q, t.b, t.n0, t.nc, lane);
}

// ---------------------------------------------------------------------------------------------
// Finish kernel of the fused train-step forward (supervisor.py:17-18): one wave per batch row b
//   * positive triple: single-mode score (tail formula) -> raw + logsigmoid   (model.py:127-146)
//   * negative row b: sum softmax(T s) logsigmoid(-s) or mean logsigmoid(-s)  (model.py:168-171)
// ---------------------------------------------------------------------------------------------
// The forward row reductions' exp / log on the hardware v_exp_f32 / v_log_f32 (~1 ulp, well inside the 1e-4
// parity bar): with libm's expf / log1pf the C4 reduction (1 024 scores per row, 16 per lane, three
// transcendentals each) was compute-bound at 8.1 us per launch, 4.8 us on the hardware units
// (profiles/r04_tile_setup_ab.txt). Every form's reduction (fused, neg_rows, neg_reduce, the row-sharded finish)
// uses these two, so the forms stay bitwise equal to one another.
// log1p(e) for e = exp(-|x|) in [0, 1]: below 1/128 the series e (1 - e (1/2 - e / 3)) (relative error < e^3 / 4,
// under 2^-22), above it the hardware log of 1 + e. log(1 + e) alone returns 0 for e < 2^-24 and loses the
// relative accuracy of a small row loss (a well-separated row's logsigmoid(-s) ~ -e^s).
__device__ __forceinline__ float rr_log1p(float e) {
    const float series = e * (1.f - e * (0.5f - e * (1.f / 3.f)));
    return e < (1.f / 128.f) ? series : __logf(1.f + e);
}
__device__ __forceinline__ float rr_exp(float x) { return __expf(x); }
__device__ __forceinline__ float rr_log_sigmoid(float x) { return fminf(x, 0.f) - rr_log1p(__expf(-fabsf(x))); }

__device__ __forceinline__ float row_reduce(const float* row, int64_t N, float T, int adversarial, int lane) {
    if (adversarial) {
        float m = -INFINITY;
        for (int64_t n = lane; n < N; n += kWave) m = fmaxf(m, T * row[n]);
        m = wave_max(m);
        float z = 0.f, w = 0.f;
        for (int64_t n = lane; n < N; n += kWave) {
            const float x = row[n];
            const float e = rr_exp(T * x - m);
            z += e;
            w += e * rr_log_sigmoid(-x);
        }
        return wave_sum(w) / wave_sum(z);
    }
    float w = 0.f;
    for (int64_t n = lane; n < N; n += kWave) w += rr_log_sigmoid(-row[n]);
    return wave_sum(w) / (float)N;
}

// The row reduction of kge_step_forward's XCD-sliced form: out_neg[b] = sum softmax(T s) logsigmoid(-s)
// or mean logsigmoid(-s) over row b's scores (model.py:168-171), one wave per row. The row is loaded
// into registers in one round (N <= 64 NR) and reduced in row_reduce's exact order (bitwise its result).
// row_reduce_vals: the same reduction on values already in registers (v[k] = row[lane + 64 k]).
template <int NR>
__device__ __forceinline__ float row_reduce_vals(const float (&v)[NR], int64_t N, float T, int adversarial, int lane) {
    if (adversarial) {
        float m = -INFINITY;
#pragma unroll
        for (int k = 0; k < NR; ++k)
            if (lane + (int64_t)k * kWave < N) m = fmaxf(m, T * v[k]);
        m = wave_max(m);
        float z = 0.f, wsum = 0.f;
#pragma unroll
        for (int k = 0; k < NR; ++k)
            if (lane + (int64_t)k * kWave < N) {
                const float e = rr_exp(T * v[k] - m);
                z += e;
                wsum += e * rr_log_sigmoid(-v[k]);
            }
        return wave_sum(wsum) / wave_sum(z);
    }
    float wsum = 0.f;
#pragma unroll
    for (int k = 0; k < NR; ++k)
        if (lane + (int64_t)k * kWave < N) wsum += rr_log_sigmoid(-v[k]);
    return wave_sum(wsum) / (float)N;
}

template <int NR>
__device__ __forceinline__ float row_reduce_regs(const float* row, int64_t N, float T, int adversarial, int lane) {
    float v[NR];
#pragma unroll
    for (int k = 0; k < NR; ++k) {
        const int64_t n = lane + (int64_t)k * kWave;
        v[k] = n < N ? row[n] : 0.f;
    }
    return row_reduce_vals<NR>(v, N, T, adversarial, lane);
}

// row_reduce with the row loaded in one round for N <= 1024 (bitwise row_reduce's result)
__device__ __forceinline__ float row_reduce_fast(const float* row, int64_t N, float T, int adversarial, int lane) {
    if (N <= 4 * kWave) return row_reduce_regs<4>(row, N, T, adversarial, lane);
    if (N <= 16 * kWave) return row_reduce_regs<16>(row, N, T, adversarial, lane);
    return row_reduce(row, N, T, adversarial, lane);
}

// Backward of one row's reduction (model.py:168-171): drow[n] = go * d(row_reduce)/d s_n.
//   d/ds_n [sum_m p_m L_m] = p_n * dL_n/ds_n + T p_n (L_n - out)   (second term: softmax not detached)
__device__ __forceinline__ void neg_row_bwd(const float* row, int64_t N, float T, int adversarial, int detach,
                                            float go, float* drow, int lane) {
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

// One batch row's finish: the positive (h, r, t) scored with the single-mode (tail) formula, and the
// reduction of the row's N negative scores. `pos` is the [B, 3] positive batch.
template <int FN, int V, int G>
__device__ __forceinline__ void finish_row(const ScoreParams& p, const int64_t* pos, int64_t b, int lane,
                                           const float* scores, int64_t n_neg) {
    // issue every independent load before the first reduction: the positive tail row, then the
    // query rows (h, r), then the negative row's scores (latency-bound: one wave per batch row)
    bool ok;
    const float* row = cand_row(p, pos[b * 3 + 2], ok);
    Cand<FN, V, G> c;
    c.load(row, ok, p.D, lane);
    Query<FN, false, V, G> q;
    const int64_t qi = pos[b * 3], ri = pos[b * 3 + 1];
    const bool qok = qi >= 0 && qi < p.q_rows, rok = ri >= 0 && ri < p.r_rows;
    q.build(p.qent + (qok ? qi : 0) * p.q_ld, qok, p.rel + (rok ? ri : 0) * p.r_ld + p.r_off, rok, p.D, lane, p);
    const float red = row_reduce_fast(scores, n_neg, p.temperature, p.adversarial, lane);
    const float s = cand_score<FN, false, V, G>(c, q, p);
    if (lane == 0) {
        if (p.out_pos_raw) p.out_pos_raw[b] = s;
        p.out_pos_ls[b] = log_sigmoid(s);
        p.out_neg[b] = red;
    }
}

template <int FN, int V, int G>
__global__ __launch_bounds__(kBlock) void finish_kernel(ScoreParams p) {
    const int64_t b = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (b >= p.B) return;
    // single-mode parameters: q_idx = pos (h column), stride 3
    finish_row<FN, V, G>(p, p.q_idx, b, threadIdx.x & 63, p.neg_scores + b * p.ns_ld, p.n_neg);
}

// Fused train-step forward (kge_step_forward): one block per batch row. The four waves score a
// quarter of the row's negatives each (the scoring code above), then wave 0 runs the row's finish
// (positive + reduction) once the block's scores are written: one launch instead of two, and the
// finish's latency overlaps the other rows' gathers instead of following the whole negative pass.
template <int FN, bool CH, int V, int G, bool ST>
__global__ __launch_bounds__(kBlock) void step_fwd_kernel(ScoreParams p) {
    const int64_t b = blockIdx.x;
    if (b >= p.B) return;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    {
        Query<FN, CH, V, G> q;
        int64_t qi, ri;
        bool qok, rok;
        build_query_for<FN, CH, V, G>(p, b, lane, q, qi, ri, qok, rok);
        const int64_t per = (p.N + kWavesPerBlock - 1) / kWavesPerBlock;
        const int64_t lo = w * per, hi = min(p.N, lo + per);
        for (int64_t c0 = lo; c0 < hi; c0 += kWave)
            score_run<FN, CH, V, G, ST>(p, q, b, c0, (int)min((int64_t)kWave, hi - c0), lane);
    }
    __syncthreads();  // the row's scores are in memory, visible to the block
    if (w == 0) finish_row<FN, V, G>(p, p.pos_base, b, lane, p.out + b * p.out_ld, p.N);
}

// ---------------------------------------------------------------------------------------------
// Train-step forward with the query side of the backward fused in (kge_train_step; KIND_STEP_FWD_GRAD).
//
// The negative branch's loss term of row b is R_b = sum_n p_n f_n (p = softmax(T s), f = logsigmoid(-s),
// model.py:168-171) or mean_n f_n, so dR_b/ds_n = p_n (-sigmoid(s_n) + T (f_n - R_b)) (TF: softmax not
// detached, Q3), p_n (-sigmoid(s_n)) (detached) or -sigmoid(s_n)/N (mean). The query-side gradient
// sum_n dR_b/ds_n J_n (J_n = ds_n/dq, elementwise in the candidate row) therefore needs only two running
// sums while the row is still in registers: A = sum e_n (-sigmoid(s_n) + T f_n) J_n and B = sum e_n J_n
// with e_n = exp(T s_n - m) under a running max m (rescaled when m grows, as an online softmax does),
// and the row's gradient is (A - T R_b B) / Z. This removes phase 1's second gather of every candidate
// row (1.05 GB at C2). The result is written unscaled: the loss weight dL/dR_b = -w_b / (2 sum w) is a
// whole-batch quantity, applied by the chain kernel (dq_scale).
//   RED: 0 mean, 1 self-adversarial with the softmax detached, 2 self-adversarial (TF semantics).
// Scores, the row finish and the per-candidate code are the step forward's (bitwise the same scores).
// ---------------------------------------------------------------------------------------------
// InterHT's Jacobian sums on packed fp32 pairs (v_pk_mul / v_pk_fma_f32: two elements per instruction):
//   x = q0 bh - ah q1 + q2 (tail) or ah q1 - q0 bh + q2 (head), J = -sgn(x) (bh, -ah, 1) resp. (-bh, ah, 1)
// sgn(x) exactly (0 at x = 0, as tf.abs' gradient) as med3(x 2^127 2^127, -1, 1); the sums take nwa = -wa
// and nwb = -wb so that nwa sgn(x) = wa Gx. No range mask: past D the candidate, q0, q1 and q2 are 0, so
// x = 0 and the element adds nothing.
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 sgn2(f32x2 x) {
    x = x * 0x1p127f;
    x = x * 0x1p127f;
    return f32x2{__builtin_amdgcn_fmed3f(x.x, -1.f, 1.f), __builtin_amdgcn_fmed3f(x.y, -1.f, 1.f)};
}
template <bool CH, int V, bool TWO>
__device__ __forceinline__ void group_jac_ih(const vecf<V>& ca, const vecf<V>& cb, const vecf<V>& q0,
                                             const vecf<V>& q1, const vecf<V>& q2, float ia, float ib, float nwa,
                                             float nwb, vecf<V>& a0, vecf<V>& a1, vecf<V>& a2, vecf<V>& b0,
                                             vecf<V>& b1, vecf<V>& b2) {
    static_assert(V % 2 == 0, "pairs");
#pragma unroll
    for (int i = 0; i < V; i += 2) {
        const f32x2 ah = f32x2{ca.a[i], ca.a[i + 1]} * ia;
        const f32x2 bh = f32x2{cb.a[i], cb.a[i + 1]} * ib + 1.f;
        const f32x2 Q0{q0.a[i], q0.a[i + 1]}, Q1{q1.a[i], q1.a[i + 1]}, Q2{q2.a[i], q2.a[i + 1]};
        const f32x2 x = CH ? (ah * Q1 - Q0 * bh + Q2) : (Q0 * bh - ah * Q1 + Q2);
        const f32x2 sg = sgn2(x);
        auto acc = [&](float nw, vecf<V>& s0, vecf<V>& s1, vecf<V>& s2) {
            const f32x2 g = sg * nw;  // w Gx
            f32x2 u0{s0.a[i], s0.a[i + 1]}, u1{s1.a[i], s1.a[i + 1]}, u2{s2.a[i], s2.a[i + 1]};
            if (CH) {
                u0 = u0 - g * bh;
                u1 = u1 + g * ah;
            } else {
                u0 = u0 + g * bh;
                u1 = u1 - g * ah;
            }
            u2 = u2 + g;
            s0.a[i] = u0.x;
            s0.a[i + 1] = u0.y;
            s1.a[i] = u1.x;
            s1.a[i + 1] = u1.y;
            s2.a[i] = u2.x;
            s2.a[i + 1] = u2.y;
        };
        acc(nwa, a0, a1, a2);
        if constexpr (TWO) acc(nwb, b0, b1, b2);
    }
}

// Softmax / sigmoid weights of the fused query pass on the hardware exp / log / rcp (v_exp_f32, v_log_f32,
// v_rcp_f32). They weight gradient terms only (the forward's outputs are row_reduce's, in full precision). The
// log-sigmoid is the row reductions' (rr_log1p's series below 1/128): with log(1 + e) a well-separated row's
// f = logsigmoid(-s) ~ -e^s flushed to 0 under e^s < 2^-24, dropping the T f half of its weight wa.
__device__ __forceinline__ float fexp(float x) { return __expf(x); }
__device__ __forceinline__ float fsigmoid(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
__device__ __forceinline__ float flog_sigmoid(float x) { return rr_log_sigmoid(x); }

// (xr, xi) / |(xr, xi)| and 0 at (and, fast form, within FLT_MIN of) the origin: the derivative of RotatE's
// modulus, in every gradient path. One hardware reciprocal square root for both components
// instead of a square root and two IEEE divisions (the RotatE fused forward 340 -> 193 us at C3).
__device__ __forceinline__ void rot_unit(float xr, float xi, float& fr, float& fi) {
    const float s2 = xr * xr + xi * xi;
    const float im = s2 >= 1.17549435e-38f ? __builtin_amdgcn_rsqf(s2) : 0.f;
    fr = xr * im;
    fi = xi * im;
}

template <int FN, bool CH, int V, bool TWO>
__device__ __forceinline__ void group_jac(const vecf<V>& ca, const vecf<V>& cb, const vecf<V>& q0, const vecf<V>& q1,
                                          const vecf<V>& q2, bool in, float ia, float ib, const ScoreParams& p,
                                          float wa, float wb, vecf<V>& a0, vecf<V>& a1, vecf<V>& a2, vecf<V>& b0,
                                          vecf<V>& b1, vecf<V>& b2, const vecf<V>* nsg = nullptr) {
#pragma unroll
    for (int i = 0; i < V; ++i) {
        const float x = ca.a[i];
        float j0 = 0.f, j1 = 0.f, j2 = 0.f;  // d score / d (q0, q1, q2) of this element
        if constexpr (FN == KGE_INTERHT) {
            const float ah = x * ia;
            const float bh = cb.a[i] * ib + 1.f;
            if (CH) {
                const float xx = nsg ? 0.f : ah * q1.a[i] - q0.a[i] * bh + q2.a[i];
                const float Gx = nsg ? nsg->a[i] : (in ? -sgnf(xx) : 0.f);
                j1 = Gx * ah;
                j0 = -Gx * bh;
                j2 = Gx;
            } else {
                const float xx = nsg ? 0.f : q0.a[i] * bh - ah * q1.a[i] + q2.a[i];
                const float Gx = nsg ? nsg->a[i] : (in ? -sgnf(xx) : 0.f);
                j0 = Gx * bh;
                j1 = -Gx * ah;
                j2 = Gx;
            }
        } else if constexpr (FN == KGE_TRANSE) {
            const float r = CH ? (x + q0.a[i]) : (q0.a[i] - x);
            j0 = -sgnf(r);
        } else if constexpr (FN == KGE_DISTMULT) {
            j0 = x;
        } else if constexpr (FN == KGE_COMPLEX) {
            j0 = x;
            j1 = cb.a[i];
        } else if constexpr (FN == KGE_ROTATE) {
            const float xr = q0.a[i] - x, xi = q1.a[i] - cb.a[i];
            float fr, fi;
            rot_unit(xr, xi, fr, fi);
            j0 = -fr;
            j1 = -fi;
        }
        a0.a[i] += wa * j0;
        a1.a[i] += wa * j1;
        a2.a[i] += wa * j2;
        if constexpr (TWO) {
            b0.a[i] += wb * j0;
            b1.a[i] += wb * j1;
            b2.a[i] += wb * j2;
        }
    }
}

template <int FN, bool CH, int V, int G, int RED>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(2))) void step_fwd_grad_kernel(ScoreParams p) {
    static_assert(FN != KGE_PROTATE, "pRotatE's modulus gradient is not part of the fused query pass");
    constexpr bool TWO = RED == 2;
    constexpr int W = G * kWave;  // vecf<V> per operand per wave image
    __shared__ vecf<V> part[kWavesPerBlock - 1][3][W];
    __shared__ vecf<V> qimg[3][W];  // the row's query operands, shared by the four waves
    __shared__ float st[kWavesPerBlock][3];
    const int64_t b = blockIdx.x;
    if (b >= p.B) return;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int DV = p.D / V;
    const float T = p.temperature;
    if (w == 1 && lane < 3 && p.ev_count) {
        // the row's other events: positive candidate (tail), the negative call's query entity, the
        // positive call's head (step_ev_key order)
        const int64_t k = p.pos_base[b * 3 + (lane == 0 ? 2 : (lane == 1 ? (CH ? 2 : 0) : 0))];
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

        // one candidate's contribution (s is wave-uniform)
        auto accumulate = [&](const Cand<FN, V, G>& c, const LdsQuery<V>& q, float s, float2 nst,
                              const vecf<V>* nsg) {
            auto xexp = [](float x) { return fexp(x); };
            auto xsig = [](float x) { return fsigmoid(x); };
            auto xlogsig = [](float x) { return flog_sigmoid(x); };
            float wa, wb = 0.f;
            if constexpr (RED == 0) {
                wa = -xsig(s);
            } else {
                const float t = T * s;
                if (t > mrun) {  // online softmax: rescale the running sums to the new maximum
                    const float sc = xexp(mrun - t);
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
                const float e = xexp(t - mrun);
                const float f = xlogsig(-s);
                Z += e;
                Ln += e * f;
                wa = e * -xsig(s);
                if constexpr (TWO) {
                    wa += e * (T * f);
                    wb = e;
                }
            }
            if constexpr (FN == KGE_INTERHT && V % 2 == 0) {
#pragma unroll
                for (int k = 0; k < G; ++k)
                    group_jac_ih<CH, V, TWO>(c.ca[k], c.cb[k], q.q0[k], q.q1[k], q.q2[k], nst.x, nst.y, -wa, -wb, a0[k],
                                             a1[k], a2[k], b0[k], b1[k], b2[k]);
                return;
            }
#pragma unroll
            for (int k = 0; k < G; ++k)
                group_jac<FN, CH, V, TWO>(c.ca[k], c.cb[k], q.q0[k], q.q1[k], q.q2[k], (lane + k * kWave) < DV, nst.x,
                                          nst.y, p, wa, wb, a0[k], a1[k], a2[k], b0[k], b1[k], b2[k], nsg ? nsg + k : nullptr);
        };
        const int64_t per = (p.N + kWavesPerBlock - 1) / kWavesPerBlock;
        const int64_t lo = w * per, hi = min(p.N, lo + per);
        for (int64_t c0 = lo; c0 < hi; c0 += kWave) {
            const int nc = (int)min((int64_t)kWave, hi - c0);
            int64_t my_id = 0;
            if (lane < nc) {
                my_id = p.c_idx[b * p.c_stride + c0 + lane];
                // the candidate's gradient event, counted into its entity's bucket (phase 2's counting sort)
                if (p.ev_count && my_id >= 0 && my_id < p.c_rows) atomicAdd(p.ev_count + my_id, 1);
            }
            // gather the chunk's rows in ascending id order (lane j then holds the j-th smallest id): the
            // block's waves sweep the table together and repeat gathers of a row land close in time
            // (tools/locality_probe.hip: 0.95x the time of candidate order); sort key (id << 6) | lane
            int key = INT32_MAX;
            if (lane < nc)
                key = (my_id >= 0 && my_id < p.c_rows && p.c_rows < (1 << 25)) ? (int)((my_id << 6) | lane) : lane;
            key = wave_sort_asc(key, lane);
            const int src = key & (kWave - 1);
            {
                const int lo32 = lane_pull((int)(uint32_t)(uint64_t)my_id, src);
                const int hi32 = lane_pull((int)((uint64_t)my_id >> 32), src);
                my_id = (int64_t)(((uint64_t)(uint32_t)hi32 << 32) | (uint32_t)lo32);
            }
            float my_score = 0.f;
            Cand<FN, V, G> x0, x1;
            bool ok0, ok1;
            auto one = [&](const Cand<FN, V, G>& c, int jj) {
                // the query is re-read from LDS for every candidate: an opaque lane index keeps the
                // compiler from hoisting the reads into 48 loop-invariant VGPRs
                int li = lane;
                asm volatile("" : "+v"(li));
                const LdsQuery<V> q{{qimg[0], li}, {qimg[1], li}, {qimg[2], li}};
                float2 nst = make_float2(0.f, 0.f);
                const float s = cand_score<FN, CH, V, G>(c, q, p, &nst);
                if (lane == jj) my_score = s;
                // opaque copies of the half-norms: the gradient recomputes the candidate's terms
                // instead of keeping the score's per-element values alive across the reductions
                asm volatile("" : "+v"(nst.x), "+v"(nst.y));
                accumulate(c, q, s, nst, nullptr);
            };
            // software pipeline (as score_run): row j + 1 is in flight while row j is reduced
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
            if (lane < nc) p.out[b * p.out_ld + c0 + src] = my_score;
        }
    }
    // combine the four waves' partial sums in wave order
    if (lane == 0) {
        st[w][0] = mrun;
        st[w][1] = Z;
        st[w][2] = Ln;
    }
    __syncthreads();  // also: the row's scores are in memory, visible to the block
    float scale, TR = 0.f;
    if constexpr (RED == 0) {
        scale = 1.f / (float)p.N;
    } else {
        float M = st[0][0];
#pragma unroll
        for (int ww = 1; ww < kWavesPerBlock; ++ww) M = fmaxf(M, st[ww][0]);
        float Zt = 0.f, Lt = 0.f;
#pragma unroll
        for (int ww = 0; ww < kWavesPerBlock; ++ww) {
            const float f = expf(st[ww][0] - M);  // 0 for a wave without candidates (m = -inf)
            Zt += st[ww][1] * f;
            Lt += st[ww][2] * f;
        }
        scale = expf(mrun - M) / Zt;
        if constexpr (TWO) TR = T * (Lt / Zt);
    }
#pragma unroll
    for (int k = 0; k < G; ++k)
#pragma unroll
        for (int i = 0; i < V; ++i) {
            if constexpr (TWO) {
                a0[k].a[i] = scale * (a0[k].a[i] - TR * b0[k].a[i]);
                a1[k].a[i] = scale * (a1[k].a[i] - TR * b1[k].a[i]);
                a2[k].a[i] = scale * (a2[k].a[i] - TR * b2[k].a[i]);
            } else {
                a0[k].a[i] *= scale;
                a1[k].a[i] *= scale;
                a2[k].a[i] *= scale;
            }
        }
    if (w > 0) {
#pragma unroll
        for (int k = 0; k < G; ++k) {
            part[w - 1][0][lane + k * kWave] = a0[k];
            part[w - 1][1][lane + k * kWave] = a1[k];
            part[w - 1][2][lane + k * kWave] = a2[k];
        }
    }
    __syncthreads();
    if (w == 0) {
        float* dq = p.dqbuf + b * 3 * p.D;
#pragma unroll
        for (int k = 0; k < G; ++k) {
#pragma unroll
            for (int ww = 0; ww < kWavesPerBlock - 1; ++ww) {
                const vecf<V> u0 = part[ww][0][lane + k * kWave], u1 = part[ww][1][lane + k * kWave],
                              u2 = part[ww][2][lane + k * kWave];
#pragma unroll
                for (int i = 0; i < V; ++i) {
                    a0[k].a[i] += u0.a[i];
                    a1[k].a[i] += u1.a[i];
                    a2[k].a[i] += u2.a[i];
                }
            }
            const int gi = lane + k * kWave;
            const bool in = gi < DV;
            vstore<V>(dq + gi * V, a0[k], in);
            vstore<V>(dq + p.D + gi * V, a1[k], in);
            vstore<V>(dq + 2 * p.D + gi * V, a2[k], in);
        }
    } else if (w == 1) {
        finish_row<FN, V, G>(p, p.pos_base, b, lane, p.out + b * p.out_ld, p.N);
    }
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

// Gradient of one candidate's score w.r.t. the candidate row (dca, dcb; WANT_C) and the query
// operands (dq0..dq2 accumulated; ACC_Q), given dL/dscore = g. Also accumulates the pRotatE
// modulus gradient. Every lane must call it (it reduces across the wave).
template <int FN, bool CH, int V, int G, bool ACC_Q, bool WANT_C>
__device__ __forceinline__ void cand_grad(const Cand<FN, V, G>& c, const Query<FN, CH, V, G>& q, float g, int lane,
                                          int DV, const ScoreParams& p, vecf<V> (&dq0)[G], vecf<V> (&dq1)[G],
                                          vecf<V> (&dq2)[G], vecf<V> (&dca)[G], vecf<V> (&dcb)[G], float& dmod) {
    if constexpr (FN == KGE_INTERHT) {
        float sa = 0.f, sb = 0.f;
#pragma unroll
        for (int k = 0; k < G; ++k)
#pragma unroll
            for (int i = 0; i < V; ++i) {
                sa += c.ca[k].a[i] * c.ca[k].a[i];
                sb += c.cb[k].a[i] * c.cb[k].a[i];
            }
        const float ia = rsqrt_f(wave_sum(sa)), ib = rsqrt_f(wave_sum(sb));
        float dota = 0.f, dotb = 0.f;
#pragma unroll
        for (int k = 0; k < G; ++k)
#pragma unroll
            for (int i = 0; i < V; ++i) {
                const float ah = c.ca[k].a[i] * ia;
                const float bn = c.cb[k].a[i] * ib;
                const float bh = bn + 1.f;
                const float q0 = q.q0[k].a[i], q1 = q.q1[k].a[i], q2 = q.q2[k].a[i];
                const bool in = (lane + k * kWave) < DV;
                float dah, dbn;
                if (CH) {  // x = a_head * b_tail - a_tail * b_head + re_mid, candidate = head
                    const float x = ah * q1 - q0 * bh + q2;
                    const float Gx = in ? -g * sgnf(x) : 0.f;
                    dah = Gx * q1;
                    dbn = -Gx * q0;
                    if (ACC_Q) {
                        dq1[k].a[i] += Gx * ah;
                        dq0[k].a[i] += -Gx * bh;
                        dq2[k].a[i] += Gx;
                    }
                } else {
                    const float x = q0 * bh - ah * q1 + q2;
                    const float Gx = in ? -g * sgnf(x) : 0.f;
                    dah = -Gx * q1;
                    dbn = Gx * q0;
                    if (ACC_Q) {
                        dq0[k].a[i] += Gx * bh;
                        dq1[k].a[i] += -Gx * ah;
                        dq2[k].a[i] += Gx;
                    }
                }
                if (WANT_C) {
                    dca[k].a[i] = dah;
                    dcb[k].a[i] = dbn;
                    dota += ah * dah;
                    dotb += bn * dbn;
                }
            }
        if constexpr (WANT_C) {
            dota = wave_sum(dota);
            dotb = wave_sum(dotb);
            // d(x/n) = (dy - y <y, dy>) / n
#pragma unroll
            for (int k = 0; k < G; ++k)
#pragma unroll
                for (int i = 0; i < V; ++i) {
                    const float ah = c.ca[k].a[i] * ia;
                    const float bn = c.cb[k].a[i] * ib;
                    dca[k].a[i] = (dca[k].a[i] - ah * dota) * ia;
                    dcb[k].a[i] = (dcb[k].a[i] - bn * dotb) * ib;
                }
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
                    const float Gx = -g * sgnf(r);  // dL/d(residual)
                    da = CH ? Gx : -Gx;
                    if (ACC_Q) dq0[k].a[i] += Gx;
                } else if constexpr (FN == KGE_DISTMULT) {
                    da = g * q.q0[k].a[i];
                    if (ACC_Q) dq0[k].a[i] += g * x;
                } else if constexpr (FN == KGE_COMPLEX) {
                    const float y = c.cb[k].a[i];
                    da = g * q.q0[k].a[i];
                    db = g * q.q1[k].a[i];
                    if (ACC_Q) {
                        dq0[k].a[i] += g * x;
                        dq1[k].a[i] += g * y;
                    }
                } else if constexpr (FN == KGE_ROTATE) {
                    const float y = c.cb[k].a[i];
                    const float xr = q.q0[k].a[i] - x, xi = q.q1[k].a[i] - y;
                    float fr, fi;
                    rot_unit(xr, xi, fr, fi);
                    da = g * fr;
                    db = g * fi;
                    if (ACC_Q) {
                        dq0[k].a[i] += -g * fr;
                        dq1[k].a[i] += -g * fi;
                    }
                } else if constexpr (FN == KGE_PROTATE) {
                    const float pc = x / p.phase_div;
                    const float z = CH ? (pc + q.q0[k].a[i]) : (q.q0[k].a[i] - pc);
                    const float sz = sinf(z);
                    const float Gx = in ? -g * p.modulus * sgnf(sz) * cosf(z) : 0.f;
                    da = (CH ? Gx : -Gx) / p.phase_div;
                    if (ACC_Q) dq0[k].a[i] += Gx;
                    ysum += in ? fabsf(sz) : 0.f;
                }
                if (WANT_C) {
                    dca[k].a[i] = in ? da : 0.f;
                    dcb[k].a[i] = in ? db : 0.f;
                }
            }
        if constexpr (FN == KGE_PROTATE) {
            if (ACC_Q) dmod += -g * wave_sum(ysum);
        }
    }
}

// Query-side chain rule: accumulated query-operand grads (dq0..dq2) -> gradient of the raw query
// entity row (gea: first half / whole row, geb: second half) and of the used relation part (gra,
// grb). qrow / rrow are the raw rows (relation row already offset by r_off).
template <int FN, bool CH, int V, int G>
__device__ __forceinline__ void query_chain(const Query<FN, CH, V, G>& q, const vecf<V> (&dq0)[G],
                                            const vecf<V> (&dq1)[G], const vecf<V> (&dq2)[G], const float* qrow,
                                            bool qok, const float* rrow, bool rok, int lane, int D,
                                            const ScoreParams& p, vecf<V> (&gea)[G], vecf<V> (&geb)[G],
                                            vecf<V> (&gra)[G], vecf<V> (&grb)[G]) {
    const int DV = D / V;
    float dna = 0.f, dnb = 0.f;
    if constexpr (FN == KGE_INTERHT) {
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
    const uint32_t qb = qok ? (uint32_t)D * 4u : 0u, rbytes = rok ? (uint32_t)D * 4u : 0u;
    const rsrc_t sqa = make_rsrc(qrow, qb), sqb = make_rsrc(qrow + D, is_split(FN) ? qb : 0u);
    const rsrc_t sra = make_rsrc(rrow, rbytes), srb = make_rsrc(rrow + D, rel_split(FN) ? rbytes : 0u);
#pragma unroll
    for (int k = 0; k < G; ++k) {
        const bool in = (lane + k * kWave) < DV;
        const vecf<V> ea = bload<V>(sqa, goff<V>(lane, k)), eb = bload<V>(sqb, goff<V>(lane, k));
        const vecf<V> ra = bload<V>(sra, goff<V>(lane, k)), rb = bload<V>(srb, goff<V>(lane, k));
#pragma unroll
        for (int i = 0; i < V; ++i) {
            const float x = ea.a[i], y = eb.a[i], r = ra.a[i], s = rb.a[i];
            const float d0 = dq0[k].a[i], d1 = dq1[k].a[i], d2 = dq2[k].a[i];
            float o_ea = 0.f, o_eb = 0.f, o_ra = 0.f, o_rb = 0.f;
            if constexpr (FN == KGE_TRANSE) {
                o_ea = CH ? -d0 : d0;
                o_ra = d0;
            } else if constexpr (FN == KGE_DISTMULT) {
                o_ea = d0 * r;
                o_ra = d0 * x;
            } else if constexpr (FN == KGE_COMPLEX) {
                if (!CH) {
                    o_ea = d0 * r + d1 * s;
                    o_eb = -d0 * s + d1 * r;
                    o_ra = d0 * x + d1 * y;
                    o_rb = -d0 * y + d1 * x;
                } else {
                    o_ea = d0 * r - d1 * s;
                    o_eb = d0 * s + d1 * r;
                    o_ra = d0 * x + d1 * y;
                    o_rb = d0 * y - d1 * x;
                }
            } else if constexpr (FN == KGE_ROTATE) {
                const float ph = r / p.phase_div;
                const float c = cosf(ph), sn = sinf(ph);
                const float Q0 = q.q0[k].a[i], Q1 = q.q1[k].a[i];
                float dth;
                if (!CH) {
                    o_ea = d0 * c + d1 * sn;
                    o_eb = -d0 * sn + d1 * c;
                    dth = -d0 * Q1 + d1 * Q0;
                } else {
                    o_ea = d0 * c - d1 * sn;
                    o_eb = d0 * sn + d1 * c;
                    dth = d0 * Q1 - d1 * Q0;
                }
                o_ra = dth / p.phase_div;
            } else if constexpr (FN == KGE_PROTATE) {
                o_ea = (CH ? -d0 : d0) / p.phase_div;
                o_ra = d0 / p.phase_div;
            } else if constexpr (FN == KGE_INTERHT) {
                const float Q0 = q.q0[k].a[i];
                const float bn = in ? q.q1[k].a[i] - 1.f : 0.f;
                o_ea = (d0 - Q0 * dna) * q.na_inv;
                o_eb = (d1 - bn * dnb) * q.nb_inv;
                o_ra = d2;
            }
            gea[k].a[i] = in ? o_ea : 0.f;
            geb[k].a[i] = in ? o_eb : 0.f;
            gra[k].a[i] = in ? o_ra : 0.f;
            grb[k].a[i] = in ? o_rb : 0.f;
        }
    }
}

// Atomic-scatter backward (used by kge_score_indexed_bwd / kge_score_dense_bwd): recompute each
// candidate's terms, scatter its row gradient with fp32 atomics, accumulate the query-side
// gradient over the wave's run and add it once per wave.
template <int FN, bool CH, int V, int G>
__global__ __launch_bounds__(kBlock) void score_bwd_kernel(ScoreParams p) {
    WaveTask t;
    if (!wave_task(p, t)) return;
    const int lane = threadIdx.x & 63;
    const int D = p.D, DV = D / V;

    Query<FN, CH, V, G> q;
    int64_t qi, ri;
    bool qok, rok;
    build_query_for<FN, CH, V, G>(p, t.b, lane, q, qi, ri, qok, rok);
    const float* qrow = p.qent + (qok ? qi : 0) * p.q_ld;
    const float* rrow = p.rel + (rok ? ri : 0) * p.r_ld + p.r_off;

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
        bool ok;
        const float* crow = cand_row(p, ci, ok);
        Cand<FN, V, G> c;
        c.load(crow, ok, D, lane);
        vecf<V> dca[G], dcb[G];
        cand_grad<FN, CH, V, G, true, true>(c, q, g, lane, DV, p, dq0, dq1, dq2, dca, dcb, dmod);
        float* drow = p.d_cent + (ok ? ci - p.c_base : 0) * p.c_ld;
#pragma unroll
        for (int k = 0; k < G; ++k) {
            const int gi = lane + k * kWave;
            const bool in = ok && gi < DV;
            vatomic_add<V>(drow + gi * V, dca[k], in);
            if constexpr (is_split(FN)) vatomic_add<V>(drow + D + gi * V, dcb[k], in);
        }
    }

    vecf<V> gea[G], geb[G], gra[G], grb[G];
    query_chain<FN, CH, V, G>(q, dq0, dq1, dq2, qrow, qok, rrow, rok, lane, D, p, gea, geb, gra, grb);
    float* dq_row = p.d_qent + (qok ? qi : 0) * p.q_ld;
    float* dr_row = p.d_rel + (rok ? ri : 0) * p.r_ld + p.r_off;
#pragma unroll
    for (int k = 0; k < G; ++k) {
        const int gi = lane + k * kWave;
        const bool in = gi < DV;
        const int e = gi * V;
        vatomic_add<V>(dq_row + e, gea[k], qok && in);
        if constexpr (is_split(FN)) vatomic_add<V>(dq_row + D + e, geb[k], qok && in);
        vatomic_add<V>(dr_row + e, gra[k], rok && in);
        if constexpr (rel_split(FN)) vatomic_add<V>(dr_row + D + e, grb[k], rok && in);
    }
    if constexpr (FN == KGE_PROTATE) {
        if (lane == 0 && p.d_modulus) unsafeAtomicAdd(p.d_modulus, dmod);
    }
}

// ---------------------------------------------------------------------------------------------
// Deterministic two-phase backward of the fused train step (kge_step_backward). No atomics on
// floats anywhere: every sum has a fixed order, so gradients are bitwise reproducible.
//
// Phase 1 (bwd_rows_kernel): one block of 4 waves per batch row (a "slot"); the waves split the
//   row's candidates, accumulate the query-side gradient in VGPRs (cand_grad, ACC_Q), combine the
//   four partials through LDS in wave order, and wave 0 applies the query chain rule. Writes the
//   slot's query operands (for phase 2), its query-entity row gradient and relation gradient.
// Phase 2 (bwd_ent_kernel): one wave per entity row e. It loads row e once and walks the gradient
//   events bucketed to e (counting sort by entity) in ascending event-code order: a candidate event
//   (slot, dL/dscore) recomputes the candidate-row gradient against the slot's stored query; a row
//   event adds a slot's query-entity gradient. Every row of the gradient table is written once
//   (no memset; rows without events are written as zeros).
// ---------------------------------------------------------------------------------------------
template <int FN, bool CH, int V, int G>
__device__ __forceinline__ void load_prebuilt_query(Query<FN, CH, V, G>& q, const float* row, int D, int lane) {
    const uint32_t nb = (uint32_t)D * 4u;
    const rsrc_t s0 = make_rsrc(row, nb), s1 = make_rsrc(row + D, nb), s2 = make_rsrc(row + 2 * D, nb);
#pragma unroll
    for (int k = 0; k < G; ++k) {
        q.q0[k] = bload<V>(s0, goff<V>(lane, k));
        q.q1[k] = bload<V>(s1, goff<V>(lane, k));
        q.q2[k] = bload<V>(s2, goff<V>(lane, k));
    }
    q.na_inv = q.nb_inv = 0.f;
}

// Phase-1 epilogue of one slot: the query chain (gradients of the raw query-entity and relation rows)
// and the rows phase 2 reads (prebuilt query, query-entity gradient), relation gradient rows.
template <int FN, bool CH, int V, int G>
__device__ __forceinline__ void rows_finalize(const ScoreParams& p, int64_t slot, const Query<FN, CH, V, G>& q,
                                              vecf<V> (&dq0)[G], vecf<V> (&dq1)[G], vecf<V> (&dq2)[G], int64_t qi,
                                              int64_t ri, bool qok, bool rok, int lane) {
    const int D = p.D, DV = D / V;
    const float* qrow = p.qent + (qok ? qi : 0) * p.q_ld;
    const float* rrow = p.rel + (rok ? ri : 0) * p.r_ld + p.r_off;
    vecf<V> gea[G], geb[G], gra[G], grb[G];
    query_chain<FN, CH, V, G>(q, dq0, dq1, dq2, qrow, qok, rrow, rok, lane, D, p, gea, geb, gra, grb);
    float* qb = p.qbuf + slot * 3 * D;
    float* ge = p.qg_ent + slot * p.ent_w;
    float* gr = p.qg_rel + slot * p.rel_w;
#pragma unroll
    for (int k = 0; k < G; ++k) {
        const int gi = lane + k * kWave;
        const bool in = gi < DV;
        const int e = gi * V;
        vstore<V>(qb + e, q.q0[k], in);
        vstore<V>(qb + D + e, q.q1[k], in);
        vstore<V>(qb + 2 * D + e, q.q2[k], in);
        // a query row that is out of range (TF zero-fill) receives no gradient
        vstore<V>(ge + e, qok ? gea[k] : vzero<V>(), in);
        if constexpr (is_split(FN)) vstore<V>(ge + D + e, qok ? geb[k] : vzero<V>(), in);
        vstore<V>(gr + e, rok ? gra[k] : vzero<V>(), in);
        if constexpr (rel_split(FN)) vstore<V>(gr + D + e, rok ? grb[k] : vzero<V>(), in);
    }
}

template <int FN, bool CH, int V, int G>
__global__ __launch_bounds__(kBlock) void bwd_rows_kernel(ScoreParams p) {
    constexpr int W = G * V * kWave;  // floats per operand per wave image
    __shared__ float red[kWavesPerBlock][3][W];
    __shared__ float red_mod[kWavesPerBlock];
    const int64_t b = blockIdx.x;
    if (b >= p.B) return;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int D = p.D, DV = D / V;
    Query<FN, CH, V, G> q;
    int64_t qi, ri;
    bool qok, rok;
    build_query_for<FN, CH, V, G>(p, b, lane, q, qi, ri, qok, rok);

    vecf<V> dq0[G], dq1[G], dq2[G], dca[G], dcb[G];
#pragma unroll
    for (int k = 0; k < G; ++k) dq0[k] = dq1[k] = dq2[k] = vzero<V>();
    float dmod = 0.f;
    const int64_t per = (p.N + kWavesPerBlock - 1) / kWavesPerBlock;
    const int64_t n_lo = w * per, n_hi = min(p.N, n_lo + per);
    for (int64_t c0 = n_lo; c0 < n_hi; c0 += kWave) {
        const int nc = (int)min((int64_t)kWave, n_hi - c0);
        int64_t my_id = 0;
        float my_g = 0.f;
        if (lane < nc) {
            my_id = p.c_idx ? p.c_idx[b * p.c_stride + c0 + lane] : b * p.c_dense + c0 + lane;
            my_g = p.d_scores[b * p.d_ld + c0 + lane];
        }
        Cand<FN, V, G> x0, x1;
        bool ok0, ok1;
        x0.load(cand_row(p, readlane64(my_id, 0), ok0), ok0, D, lane);
        for (int j = 0; j < nc; ++j) {
            if (j + 1 < nc) {  // next row in flight while this one is reduced
                if (j & 1)
                    x0.load(cand_row(p, readlane64(my_id, j + 1), ok0), ok0, D, lane);
                else
                    x1.load(cand_row(p, readlane64(my_id, j + 1), ok1), ok1, D, lane);
            }
            const float g = readlanef(my_g, j);
            if (j & 1)
                cand_grad<FN, CH, V, G, true, false>(x1, q, g, lane, DV, p, dq0, dq1, dq2, dca, dcb, dmod);
            else
                cand_grad<FN, CH, V, G, true, false>(x0, q, g, lane, DV, p, dq0, dq1, dq2, dca, dcb, dmod);
        }
    }
    // combine the four waves' partials in wave order through LDS
#pragma unroll
    for (int k = 0; k < G; ++k)
#pragma unroll
        for (int i = 0; i < V; ++i) {
            const int e = (lane + k * kWave) * V + i;
            red[w][0][e] = dq0[k].a[i];
            red[w][1][e] = dq1[k].a[i];
            red[w][2][e] = dq2[k].a[i];
        }
    if (lane == 0) red_mod[w] = dmod;
    __syncthreads();
    if (w != 0) return;
#pragma unroll
    for (int k = 0; k < G; ++k)
#pragma unroll
        for (int i = 0; i < V; ++i) {
            const int e = (lane + k * kWave) * V + i;
            float s0 = red[0][0][e], s1 = red[0][1][e], s2 = red[0][2][e];
#pragma unroll
            for (int ww = 1; ww < kWavesPerBlock; ++ww) {
                s0 += red[ww][0][e];
                s1 += red[ww][1][e];
                s2 += red[ww][2][e];
            }
            dq0[k].a[i] = s0;
            dq1[k].a[i] = s1;
            dq2[k].a[i] = s2;
        }
    rows_finalize<FN, CH, V, G>(p, p.slot0 + b, q, dq0, dq1, dq2, qi, ri, qok, rok, lane);
    if (lane == 0 && p.dmod_part) {
        float m = red_mod[0];
        for (int ww = 1; ww < kWavesPerBlock; ++ww) m += red_mod[ww];
        p.dmod_part[p.slot0 + b] = m;
    }
}

template <int FN, bool CH, int V, int G>
__device__ __forceinline__ void ent_event(const ScoreParams& p, const Cand<FN, V, G>& c, int code, int lane,
                                          vecf<V> (&acc_a)[G], vecf<V> (&acc_b)[G]) {
    const int D = p.D, DV = D / V;
    const int64_t BN = p.Bn * p.Nn;
    vecf<V> dq0[G], dq1[G], dq2[G], dca[G], dcb[G];
    float dmod = 0.f;
    if (code < BN + p.Bn) {
        // candidate event: negative (slot = row b) or positive (slot = Bn + b, tail formula)
        const bool neg = code < BN;
        const int64_t slot = neg ? code / p.Nn : p.Bn + (code - BN);
        const float g = neg ? p.d_ns[code] : p.d_ps[code - BN];
        if (neg) {
            Query<FN, CH, V, G> q;
            load_prebuilt_query<FN, CH, V, G>(q, p.qbuf + slot * 3 * D, D, lane);
            cand_grad<FN, CH, V, G, false, true>(c, q, g, lane, DV, p, dq0, dq1, dq2, dca, dcb, dmod);
        } else {
            Query<FN, false, V, G> q;
            load_prebuilt_query<FN, false, V, G>(q, p.qbuf + slot * 3 * D, D, lane);
            cand_grad<FN, false, V, G, false, true>(c, q, g, lane, DV, p, dq0, dq1, dq2, dca, dcb, dmod);
        }
#pragma unroll
        for (int k = 0; k < G; ++k)
#pragma unroll
            for (int i = 0; i < V; ++i) {
                acc_a[k].a[i] += dca[k].a[i];
                if constexpr (is_split(FN)) acc_b[k].a[i] += dcb[k].a[i];
            }
    } else {
        // row event: a slot's query-entity gradient (negative call's query, then positive's h)
        const int64_t slot = code - BN - p.Bn;
        const float* row = p.qg_ent + slot * p.ent_w;
        const rsrc_t sa = make_rsrc(row, (uint32_t)D * 4u);
        const rsrc_t sb = make_rsrc(row + D, is_split(FN) ? (uint32_t)D * 4u : 0u);
#pragma unroll
        for (int k = 0; k < G; ++k) {
            const vecf<V> a = bload<V>(sa, goff<V>(lane, k)), bb = bload<V>(sb, goff<V>(lane, k));
#pragma unroll
            for (int i = 0; i < V; ++i) {
                acc_a[k].a[i] += a.a[i];
                if constexpr (is_split(FN)) acc_b[k].a[i] += bb.a[i];
            }
        }
    }
}

template <int FN, bool CH, int V, int G>
__global__ __launch_bounds__(kBlock) void bwd_ent_kernel(ScoreParams p) {
    const int64_t e = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (e >= p.c_rows) return;
    const int lane = threadIdx.x & 63;
    const int D = p.D, DV = D / V;
    vecf<V> acc_a[G], acc_b[G];
#pragma unroll
    for (int k = 0; k < G; ++k) acc_a[k] = acc_b[k] = vzero<V>();
    // bucket bounds and codes are validated against the event count: a corrupted bucket table (a
    // workspace that was not zero-filled) gives wrong gradients, never an out-of-range access
    const int ntot = (int)(p.Bn * p.Nn + 3 * p.Bn);
    const int lo = min(max(p.ev_off[e], 0), ntot), hi = min(max(p.ev_off[e + 1], lo), ntot);
    const int n = hi - lo;
    Cand<FN, V, G> c;
    if (n > 0 || p.adam.on) c.load(p.cent + e * p.c_ld, true, D, lane);
    // fused optimizer: the row's Adam moments are requested now, so their latency overlaps the
    // event walk instead of following it
    constexpr int NH = is_split(FN) ? 2 : 1;
    vecf<V> mm[NH][G], vv[NH][G];
    if (p.adam.on) {
        const rsrc_t sm = make_rsrc(p.adam.m + e * p.c_ld, (uint32_t)p.ent_w * 4u);
        const rsrc_t sv = make_rsrc(p.adam.v + e * p.c_ld, (uint32_t)p.ent_w * 4u);
#pragma unroll
        for (int h = 0; h < NH; ++h)
#pragma unroll
            for (int k = 0; k < G; ++k) {
                const uint32_t off = (uint32_t)(h * D * 4) + goff<V>(lane, k);
                mm[h][k] = bload<V>(sm, off);
                vv[h][k] = bload<V>(sv, off);
            }
    }
    if (n > 0) {
        if (n <= kWave) {
            int code = lane < n ? p.ev_code[lo + lane] : INT32_MAX;
            if ((unsigned)code >= (unsigned)ntot) code = INT32_MAX;  // never index with a stray code
            const int nv = __popcll(__ballot(code != INT32_MAX));
            code = wave_sort_asc(code, lane);
            for (int j = 0; j < nv; ++j)
                ent_event<FN, CH, V, G>(p, c, __builtin_amdgcn_readlane(code, j), lane, acc_a, acc_b);
        } else {
            // large bucket: extract codes in ascending order (O(n^2 / 64), rare for random ids)
            int last = -1;
            for (int it = 0; it < n; ++it) {
                int m = INT32_MAX;
                for (int i = lo + lane; i < hi; i += kWave) {
                    const int v = p.ev_code[i];
                    if (v > last && v < m && v < ntot) m = v;
                }
                m = wave_min_i(m);
                if (m == INT32_MAX) break;
                ent_event<FN, CH, V, G>(p, c, m, lane, acc_a, acc_b);
                last = m;
            }
        }
    }
    if (p.adam.on) {
        // fused optimizer: row e of the table (already in registers) and its Adam moments
        float* prow = const_cast<float*>(p.cent) + e * p.c_ld;
        float* mrow = p.adam.m + e * p.c_ld;
        float* vrow = p.adam.v + e * p.c_ld;
#pragma unroll
        for (int k = 0; k < G; ++k) {
            const int gi = lane + k * kWave;
            const bool in = gi < DV;
#pragma unroll
            for (int h = 0; h < NH; ++h) {
                vecf<V> pp = h ? c.cb[k] : c.ca[k];
                const vecf<V>& gg = h ? acc_b[k] : acc_a[k];
#pragma unroll
                for (int i = 0; i < V; ++i)
                    adam_update(pp.a[i], gg.a[i], mm[h][k].a[i], vv[h][k].a[i], p.adam.b1, p.adam.b2, p.adam.eps,
                                p.adam.alpha, p.adam.step_size, p.adam.bc2_sqrt, p.adam.keras);
                const int64_t col = (int64_t)h * D + gi * V;
                vstore<V>(prow + col, pp, in);
                vstore<V>(mrow + col, mm[h][k], in);
                vstore<V>(vrow + col, vv[h][k], in);
            }
        }
        return;
    }
    float* out = p.d_out_ent + e * p.c_ld;
#pragma unroll
    for (int k = 0; k < G; ++k) {
        const int gi = lane + k * kWave;
        const bool in = gi < DV;
        vstore<V>(out + gi * V, acc_a[k], in);
        if constexpr (is_split(FN)) vstore<V>(out + D + gi * V, acc_b[k], in);
    }
}

// ---------------------------------------------------------------------------------------------
// Phase 1, streaming form (KIND_BWD_STREAM + KIND_BWD_CHAIN; used when each lane holds >= 4 column
// groups). The query-side gradient of a slot is a sum over its N candidates of elementwise terms; the
// only full-row quantities, InterHT's candidate half-norms, come from the forward (cand_stats). So the
// block's four waves split the COLUMNS (wave w owns groups k = w, w + 4, ...) and each streams all N
// candidates through its own columns: a wave holds only its query and accumulator groups (no full
// candidate row), which keeps the kernel at high occupancy with 8 candidates' loads in flight.
// The chain (normalisation backward of the query, full-row dots) runs afterwards, one wave per slot.
// ---------------------------------------------------------------------------------------------
template <int FN, bool CH, int V>
__device__ __forceinline__ void group_grad(const vecf<V>& ca, const vecf<V>& cb, const vecf<V>& q0, const vecf<V>& q1,
                                           const vecf<V>& q2, bool in, float g, float ia, float ib,
                                           const ScoreParams& p, vecf<V>& dq0, vecf<V>& dq1, vecf<V>& dq2,
                                           float& dmod) {
#pragma unroll
    for (int i = 0; i < V; ++i) {
        const float x = ca.a[i];
        if constexpr (FN == KGE_INTERHT) {
            const float ah = x * ia;
            const float bh = cb.a[i] * ib + 1.f;
            if (CH) {
                const float xx = ah * q1.a[i] - q0.a[i] * bh + q2.a[i];
                const float Gx = in ? -g * sgnf(xx) : 0.f;
                dq1.a[i] += Gx * ah;
                dq0.a[i] += -Gx * bh;
                dq2.a[i] += Gx;
            } else {
                const float xx = q0.a[i] * bh - ah * q1.a[i] + q2.a[i];
                const float Gx = in ? -g * sgnf(xx) : 0.f;
                dq0.a[i] += Gx * bh;
                dq1.a[i] += -Gx * ah;
                dq2.a[i] += Gx;
            }
        } else if constexpr (FN == KGE_TRANSE) {
            const float r = CH ? (x + q0.a[i]) : (q0.a[i] - x);
            dq0.a[i] += -g * sgnf(r);
        } else if constexpr (FN == KGE_DISTMULT) {
            dq0.a[i] += g * x;
        } else if constexpr (FN == KGE_COMPLEX) {
            dq0.a[i] += g * x;
            dq1.a[i] += g * cb.a[i];
        } else if constexpr (FN == KGE_ROTATE) {
            const float xr = q0.a[i] - x, xi = q1.a[i] - cb.a[i];
            float fr, fi;
            rot_unit(xr, xi, fr, fi);
            dq0.a[i] += -g * fr;
            dq1.a[i] += -g * fi;
        } else if constexpr (FN == KGE_PROTATE) {
            const float pc = x / p.phase_div;
            const float z = CH ? (pc + q0.a[i]) : (q0.a[i] - pc);
            const float sz = sinf(z);
            dq0.a[i] += in ? -g * p.modulus * sgnf(sz) * cosf(z) : 0.f;
            dmod += in ? -g * fabsf(sz) : 0.f;
        }
    }
}

template <int FN, bool CH, int V, int G>
__global__ __launch_bounds__(kBlock) void bwd_stream_kernel(ScoreParams p) {
    static_assert(G % kWavesPerBlock == 0, "the streaming phase 1 needs a multiple of 4 groups per lane");
    constexpr int GW = G / kWavesPerBlock;  // column groups per wave
    constexpr int U = 8;                     // candidates in flight per wave
    constexpr bool SPLIT = is_split(FN);
    __shared__ float red_mod[kWavesPerBlock];
    const int64_t b = blockIdx.x;
    if (b >= p.B) return;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int D = p.D, DV = D / V;
    vecf<V> q0w[GW], q1w[GW], q2w[GW], d0[GW], d1[GW], d2[GW];
    {
        Query<FN, CH, V, G> q;
        int64_t qi, ri;
        bool qok, rok;
        build_query_for<FN, CH, V, G>(p, b, lane, q, qi, ri, qok, rok);
#pragma unroll
        for (int gg = 0; gg < GW; ++gg) {
#pragma unroll
            for (int kk = 0; kk < G; ++kk)
                if (kk == w + kWavesPerBlock * gg) {
                    q0w[gg] = q.q0[kk];
                    q1w[gg] = q.q1[kk];
                    q2w[gg] = q.q2[kk];
                }
            d0[gg] = d1[gg] = d2[gg] = vzero<V>();
        }
    }
    uint32_t goffs[GW];
    bool gin[GW];
#pragma unroll
    for (int gg = 0; gg < GW; ++gg) {
        const int k = w + kWavesPerBlock * gg;
        goffs[gg] = goff<V>(lane, k);
        gin[gg] = (lane + k * kWave) < DV;
    }
    float dmod = 0.f;
    for (int64_t c0 = 0; c0 < p.N; c0 += kWave) {
        const int nc = (int)min((int64_t)kWave, p.N - c0);
        int64_t my_id = 0;
        float my_g = 0.f;
        float2 my_st = make_float2(0.f, 0.f);
        if (lane < nc) {
            my_id = p.c_idx ? p.c_idx[b * p.c_stride + c0 + lane] : b * p.c_dense + c0 + lane;
            my_g = p.d_scores[b * p.d_ld + c0 + lane];
            if constexpr (FN == KGE_INTERHT) my_st = p.cand_stats[b * p.N + c0 + lane];
        }
        for (int j = 0; j < nc; j += U) {
            vecf<V> xa[U][GW], xb[U][GW];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                bool ok = false;
                const float* row = cand_row(p, readlane64(my_id, min(j + u, nc - 1)), ok);
                ok = ok && (j + u < nc);
                const uint32_t nb = ok ? (uint32_t)D * 4u : 0u;
                const rsrc_t sa = make_rsrc(row, nb);
#pragma unroll
                for (int gg = 0; gg < GW; ++gg) xa[u][gg] = bload<V>(sa, goffs[gg]);
                if constexpr (SPLIT) {
                    const rsrc_t sb = make_rsrc(row + D, nb);
#pragma unroll
                    for (int gg = 0; gg < GW; ++gg) xb[u][gg] = bload<V>(sb, goffs[gg]);
                } else {
#pragma unroll
                    for (int gg = 0; gg < GW; ++gg) xb[u][gg] = vzero<V>();
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (j + u < nc) {  // wave-uniform
                    const float g = readlanef(my_g, j + u);
                    float ia = 0.f, ib = 0.f;
                    if constexpr (FN == KGE_INTERHT) {
                        ia = readlanef(my_st.x, j + u);
                        ib = readlanef(my_st.y, j + u);
                    }
#pragma unroll
                    for (int gg = 0; gg < GW; ++gg)
                        group_grad<FN, CH, V>(xa[u][gg], xb[u][gg], q0w[gg], q1w[gg], q2w[gg], gin[gg], g, ia, ib, p,
                                              d0[gg], d1[gg], d2[gg], dmod);
                }
            }
        }
    }
    // the slot's query-part gradients, in the row layout the chain kernel reads
    float* dq = p.dqbuf + b * 3 * D;
#pragma unroll
    for (int gg = 0; gg < GW; ++gg) {
        const int e = (lane + (w + kWavesPerBlock * gg) * kWave) * V;
        vstore<V>(dq + e, d0[gg], gin[gg]);
        vstore<V>(dq + D + e, d1[gg], gin[gg]);
        vstore<V>(dq + 2 * D + e, d2[gg], gin[gg]);
    }
    if constexpr (FN == KGE_PROTATE) {
        dmod = wave_sum(dmod);
        if (lane == 0) red_mod[w] = dmod;
        __syncthreads();
        if (threadIdx.x == 0 && p.dmod_part) {
            float m = red_mod[0];
            for (int ww = 1; ww < kWavesPerBlock; ++ww) m += red_mod[ww];
            p.dmod_part[p.slot0 + b] = m;
        }
    } else if (threadIdx.x == 0 && p.dmod_part) {
        p.dmod_part[p.slot0 + b] = 0.f;
    }
}

template <int FN, bool CH, int V, int G>
__global__ __launch_bounds__(kBlock) void bwd_chain_kernel(ScoreParams p) {
    const int64_t b = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (b >= p.B) return;
    const int lane = threadIdx.x & 63;
    const int D = p.D;
    Query<FN, CH, V, G> q;
    int64_t qi, ri;
    bool qok, rok;
    build_query_for<FN, CH, V, G>(p, b, lane, q, qi, ri, qok, rok);
    const float* dq = p.dqbuf + b * 3 * D;
    const uint32_t nb = (uint32_t)D * 4u;
    const rsrc_t s0 = make_rsrc(dq, nb), s1 = make_rsrc(dq + D, nb), s2 = make_rsrc(dq + 2 * D, nb);
    vecf<V> dq0[G], dq1[G], dq2[G];
#pragma unroll
    for (int k = 0; k < G; ++k) {
        dq0[k] = bload<V>(s0, goff<V>(lane, k));
        dq1[k] = bload<V>(s1, goff<V>(lane, k));
        dq2[k] = bload<V>(s2, goff<V>(lane, k));
    }
    if (p.dq_scale) {  // the fused forward's unscaled query gradient: times dL/d(reduced row b)
        const float sc = p.dq_scale[b];
#pragma unroll
        for (int k = 0; k < G; ++k)
#pragma unroll
            for (int i = 0; i < V; ++i) {
                dq0[k].a[i] *= sc;
                dq1[k].a[i] *= sc;
                dq2[k].a[i] *= sc;
            }
    }
    rows_finalize<FN, CH, V, G>(p, p.slot0 + b, q, dq0, dq1, dq2, qi, ri, qok, rok, lane);
}

// ---------------------------------------------------------------------------------------------
// Train-step epilogue (kge_train_step; KIND_STEP_EPILOGUE): everything between the fused forward and
// phase 2 in one launch, one wave per slot.
//   loss weights: dL/d(out_neg_b) = dL/d(out_pos_b) = -w_b / (2 sum w)         (supervisor.py:19-23)
//   negative slot b: the row's score gradients d_ns[b, :] (reduction backward), then the chain of the
//     fused forward's query gradient (dqbuf, scaled by the loss weight)
//   positive slot B + b: d_ps[b] (logsigmoid backward), the single candidate's query gradient and its
//     chain (the positive call scores the tail, model.py:127-146)
//   all threads: the counting sort's scatter of the gradient events (the forward counted them)
//   an extra last block: the loss value and the running Sum metric (supervisor.py:19-23, :28)
// ---------------------------------------------------------------------------------------------
// Entity key of gradient event `code` of the train step (the order of kge_abi.hip's ev_key):
//   [0, BN) candidate n of row b; then per row: positive tail, negative call's query, positive head.
template <bool CH>
__device__ __forceinline__ int64_t step_ev_key(const ScoreParams& p, int code) {
    const int BN = (int)(p.B * p.N);
    if (code < BN) {
        const int b = code / (int)p.N;
        return p.c_idx[(int64_t)b * p.c_stride + (code - b * (int)p.N)];
    }
    int b = code - BN;
    if (b < p.B) return p.pos_base[(int64_t)b * 3 + 2];
    b -= (int)p.B;
    if (b < p.B) return p.pos_base[(int64_t)b * 3 + (CH ? 2 : 0)];
    b -= (int)p.B;
    return p.pos_base[(int64_t)b * 3];
}

// the tile-local bucket scan (scan_tiles4k_kernel): entities per tile, and the most tiles the epilogue takes
constexpr int kEvTile = 4096, kEvMaxTiles = 1024;

template <int FN, bool CH, int V, int G>
__global__ __launch_bounds__(kBlock) void step_epilogue_kernel(ScoreParams p) {
    __shared__ float red[3][kBlock];
    __shared__ int tpre[kEvMaxTiles + 1];  // exclusive prefix of the tile totals (tile-local scan), and the total
    const int64_t slot = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int64_t B = p.B;
    const int D = p.D, DV = D / V;
    const int total = (int)(B * p.N + 3 * B);
    const bool tiled = p.ev_tile_sum != nullptr;
    // blocks [0, nsb): slots; [nsb, last): the event scatter; last: the loss. The scatter's chain (key
    // load -> cursor atomic -> code store) runs beside the slots' chains instead of ahead of them.
    const int nsb = (int)((3 * B + kWavesPerBlock - 1) / kWavesPerBlock), last = (int)gridDim.x - 1;
    const int sblk = (int)blockIdx.x - nsb, nscat = last - nsb;
    if (sblk >= 0 && sblk < nscat) {
        if (tiled) {
            if (threadIdx.x < kWave) {
                int carry = 0;
                for (int base = 0; base < p.ev_ntiles; base += kWave) {
                    const int i = base + lane;
                    const int v = i < p.ev_ntiles ? p.ev_tile_sum[i] : 0;
                    int incl = v;
#pragma unroll
                    for (int o = 1; o < kWave; o <<= 1) {
                        const int y = __shfl_up(incl, o, kWave);
                        if (lane >= o) incl += y;
                    }
                    if (i < p.ev_ntiles) tpre[i] = carry + incl - v;
                    carry += __shfl(incl, kWave - 1, kWave);
                }
                if (lane == 0) tpre[p.ev_ntiles] = carry;
            }
            __syncthreads();
        }
        {
            // scatter the gradient events into their entity buckets (offsets from the scan kernel)
            // four codes per thread per round, their key loads and cursor atomics all in flight together
            constexpr int U = 4;
            const int nl = nscat * kBlock;
            for (int c0 = sblk * kBlock + (int)threadIdx.x; c0 < total; c0 += U * nl) {
                int64_t k[U];
#pragma unroll
                for (int u = 0; u < U; ++u) k[u] = c0 + u * nl < total ? step_ev_key<CH>(p, c0 + u * nl) : -1;
                int at[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    at[u] = (k[u] >= 0 && k[u] < p.c_rows) ? atomicAdd(p.ev_cursor + k[u], 1) : -1;
                    if (tiled && at[u] >= 0) at[u] += tpre[k[u] / kEvTile];
                }
#pragma unroll
                for (int u = 0; u < U; ++u)
                    if (at[u] >= 0 && at[u] < total) p.ev_code_w[at[u]] = c0 + u * nl;
            }
            if (tiled) {
                // phase 2's bucket offsets: tile-local -> global (clamped to the event count)
                for (int64_t e = (int64_t)sblk * kBlock + threadIdx.x; e <= p.c_rows; e += nl)
                    p.ev_off_fix[e] = e < p.c_rows ? min(p.ev_off_fix[e] + tpre[e / kEvTile], total)
                                                   : min(tpre[p.ev_ntiles], total);
            }
        }
        return;
    }
    if ((int)blockIdx.x == last) {
        // the last block: the loss of supervisor.py:19-23 (fixed reduction order) and the Sum metric
        const int t = threadIdx.x;
        float sw = 0.f, sp = 0.f, sn = 0.f;
        for (int64_t i = t; i < B; i += kBlock) {
            const float wi = p.weight[i];
            sw += wi;
            sp += wi * p.out_pos_ls[i];
            sn += wi * p.out_neg[i];
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
        if (t == 0) {
            const float tw = red[0][0];
            const float loss = (-red[1][0] / tw + -red[2][0] / tw) / 2.f;
            *p.loss = loss;
            if (p.loss_sum) *p.loss_sum += loss;
        }
        return;
    }
    // waves [0, B): the negative slots' query chains; [B, 2B): the positive slots; [2B, 3B): the negative rows'
    // score gradients (split from the chains: neither waits for the other's loads and stores)
    if (slot >= 3 * B) return;
    {
        const bool negslot = slot < B, rowgrad = slot >= 2 * B;
        const int64_t b = negslot ? slot : (rowgrad ? slot - 2 * B : slot - B);
        // sum w in a fixed order: every wave gets the same value
        float sw = 0.f;
        for (int64_t i = lane; i < B; i += kWave) sw += p.weight[i];
        sw = wave_sum(sw);
        const float wb = p.weight[b];
        const float go = (-0.5f / sw) * wb;
        if (rowgrad) {
            neg_row_bwd(p.neg_scores + b * p.ns_ld, p.N, p.temperature, p.adversarial, p.detach, go,
                        const_cast<float*>(p.d_ns) + b * p.N, lane);
        } else if (negslot) {
            Query<FN, CH, V, G> q;
            int64_t qi, ri;
            bool qok, rok;
            build_query_for<FN, CH, V, G>(p, b, lane, q, qi, ri, qok, rok);
            const float* dq = p.dqbuf + b * 3 * D;
            const uint32_t nb = (uint32_t)D * 4u;
            const rsrc_t s0 = make_rsrc(dq, nb), s1 = make_rsrc(dq + D, nb), s2 = make_rsrc(dq + 2 * D, nb);
            vecf<V> dq0[G], dq1[G], dq2[G];
#pragma unroll
            for (int k = 0; k < G; ++k) {
                dq0[k] = bload<V>(s0, goff<V>(lane, k));
                dq1[k] = bload<V>(s1, goff<V>(lane, k));
                dq2[k] = bload<V>(s2, goff<V>(lane, k));
#pragma unroll
                for (int i = 0; i < V; ++i) {
                    dq0[k].a[i] *= go;
                    dq1[k].a[i] *= go;
                    dq2[k].a[i] *= go;
                }
            }
            rows_finalize<FN, CH, V, G>(p, slot, q, dq0, dq1, dq2, qi, ri, qok, rok, lane);
        } else {
            const float g = go * sigmoidf(-p.pos_raw[b]);
            if (lane == 0) const_cast<float*>(p.d_ps)[b] = g;
            const int64_t* pr = p.pos_base + b * 3;
            const int64_t qi = pr[0], ri = pr[1];
            const bool qok = qi >= 0 && qi < p.q_rows, rok = ri >= 0 && ri < p.r_rows;
            bool cok;
            Cand<FN, V, G> c;
            c.load(cand_row(p, pr[2], cok), cok, D, lane);
            Query<FN, false, V, G> q;
            q.build(p.qent + (qok ? qi : 0) * p.q_ld, qok, p.rel + (rok ? ri : 0) * p.r_ld + p.r_off, rok, D, lane, p);
            vecf<V> dq0[G], dq1[G], dq2[G], dca[G], dcb[G];
#pragma unroll
            for (int k = 0; k < G; ++k) dq0[k] = dq1[k] = dq2[k] = vzero<V>();
            float dmod = 0.f;
            cand_grad<FN, false, V, G, true, false>(c, q, g, lane, DV, p, dq0, dq1, dq2, dca, dcb, dmod);
            rows_finalize<FN, false, V, G>(p, slot, q, dq0, dq1, dq2, qi, ri, qok, rok, lane);
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Phase 2, streaming form (KIND_BWD_ENT_STREAM; same condition as the streaming phase 1). One block
// per entity row; wave w owns column groups w, w + 4, ... A candidate event's contribution is
// elementwise against the slot's stored query once the row's InterHT half-norms are known, and the
// normalisation backward d(x/n) = (dy - y<y,dy>)/n is linear in dy: so the block sums the
// normalised-space terms of all candidate events (code order, per column), applies the chain once
// with two block-wide dots, and adds the row events (query-entity gradients, code order). A wave
// holds one row slice, its Adam moments and U events' query slices in flight (~100 VGPRs instead of
// the register-resident form's 250), so the Adam stream over the table runs at high occupancy.
// ---------------------------------------------------------------------------------------------
template <int FN, bool CH, int V>
__device__ __forceinline__ void ent_group_term(const vecf<V>& ca, const vecf<V>& cb, const vecf<V>& q0,
                                               const vecf<V>& q1, const vecf<V>& q2, bool in, float g, float ia,
                                               float ib, const ScoreParams& p, vecf<V>& sa, vecf<V>& sb) {
#pragma unroll
    for (int i = 0; i < V; ++i) {
        const float x = ca.a[i];
        float da = 0.f, db = 0.f;
        if constexpr (FN == KGE_INTERHT) {  // normalised-space terms (dy of d(x/n))
            const float ah = x * ia;
            const float bh = cb.a[i] * ib + 1.f;
            if (CH) {
                const float xx = ah * q1.a[i] - q0.a[i] * bh + q2.a[i];
                const float Gx = in ? -g * sgnf(xx) : 0.f;
                da = Gx * q1.a[i];
                db = -Gx * q0.a[i];
            } else {
                const float xx = q0.a[i] * bh - ah * q1.a[i] + q2.a[i];
                const float Gx = in ? -g * sgnf(xx) : 0.f;
                da = -Gx * q1.a[i];
                db = Gx * q0.a[i];
            }
        } else if constexpr (FN == KGE_TRANSE) {
            const float r = CH ? (x + q0.a[i]) : (q0.a[i] - x);
            const float Gx = -g * sgnf(r);
            da = CH ? Gx : -Gx;
        } else if constexpr (FN == KGE_DISTMULT) {
            da = g * q0.a[i];
        } else if constexpr (FN == KGE_COMPLEX) {
            da = g * q0.a[i];
            db = g * q1.a[i];
        } else if constexpr (FN == KGE_ROTATE) {
            const float xr = q0.a[i] - x, xi = q1.a[i] - cb.a[i];
            float fr, fi;
            rot_unit(xr, xi, fr, fi);
            da = g * fr;
            db = g * fi;
        } else if constexpr (FN == KGE_PROTATE) {
            const float pc = x / p.phase_div;
            const float z = CH ? (pc + q0.a[i]) : (q0.a[i] - pc);
            const float Gx = in ? -g * p.modulus * sgnf(sinf(z)) * cosf(z) : 0.f;
            da = (CH ? Gx : -Gx) / p.phase_div;
        }
        sa.a[i] += in ? da : 0.f;
        sb.a[i] += in ? db : 0.f;
    }
}

// block-wide sum of two per-lane partials, waves combined in wave order (deterministic)
__device__ __forceinline__ float2 block_sum2(float a, float b, float (*red)[kWavesPerBlock], int lane, int w) {
    a = wave_sum(a);
    b = wave_sum(b);
    __syncthreads();  // red may still be read from a previous call
    if (lane == 0) {
        red[0][w] = a;
        red[1][w] = b;
    }
    __syncthreads();
    float sa = red[0][0], sb = red[1][0];
#pragma unroll
    for (int ww = 1; ww < kWavesPerBlock; ++ww) {
        sa += red[0][ww];
        sb += red[1][ww];
    }
    return make_float2(sa, sb);
}

// largest entity bucket phase 2 sorts block-wide in LDS (larger ones fall back to ordered extraction)
constexpr int kEntSortMax = 2048;

// query operands a candidate event of function FN reads from the slot's stored query (InterHT's third,
// the relation row, is read from the relation table instead: it stays in L2)
constexpr int ent_nq(int fn) { return (fn == KGE_COMPLEX || fn == KGE_ROTATE || fn == KGE_INTERHT) ? 2 : 1; }

template <int FN, bool CH, int V, int G>
__global__ __launch_bounds__(kBlock) void bwd_ent_stream_kernel(ScoreParams p) {
    static_assert(G % kWavesPerBlock == 0, "the streaming phase 2 needs a multiple of 4 groups per lane");
    constexpr int GW = G / kWavesPerBlock;
    constexpr int U0 = GW == 1 ? 4 : (GW == 2 ? 2 : 1);  // events whose query slices are in flight
    constexpr int U = U0 < 2 ? U0 : 2;  // 2 events in flight (4: 398-400 us against 369-374 at C2, 93 VGPRs)
    constexpr bool SPLIT = is_split(FN);
    constexpr int NH = SPLIT ? 2 : 1;
    constexpr int NQ = ent_nq(FN);
    __shared__ float red[2][kWavesPerBlock];
    __shared__ int srt[kEntSortMax];  // a large bucket's codes, sorted block-wide
    const int64_t e = blockIdx.x;
    if (e >= p.c_rows) return;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int D = p.D, DV = D / V;
    const int64_t BN = p.Bn * p.Nn;
    const uint32_t nb = (uint32_t)D * 4u;
    uint32_t goffs[GW];
    bool gin[GW];
#pragma unroll
    for (int gg = 0; gg < GW; ++gg) {
        const int k = w + kWavesPerBlock * gg;
        goffs[gg] = goff<V>(lane, k);
        gin[gg] = (lane + k * kWave) < DV;
    }
    // streamed (read-once) operands: the table row and its Adam moments, nontemporal (kEntLdAux)
    auto sload = [&](rsrc_t r, uint32_t off) { return bload<V, kEntLdAux>(r, off); };
    // bucket bounds and codes are validated against the event count: a corrupted bucket table (a
    // workspace that was not zero-filled) gives wrong gradients, never an out-of-range access
    const int ntot = (int)(p.Bn * p.Nn + 3 * p.Bn);
    const int lo = min(max(p.ev_off[e], 0), ntot), hi = min(max(p.ev_off[e + 1], lo), ntot);
    const int n = hi - lo;
    // a small bucket's codes are requested before the row and its moments: the vector-memory counter
    // retires in order, so the code -> relation index -> event-slice chain then runs under the row's
    // HBM latency instead of after it
    int code0 = (n <= kWave && lane < n) ? p.ev_code[lo + lane] : INT32_MAX;
    // the row slice, and the Adam moments requested up front so their latency overlaps the walk
    vecf<V> ca[GW], cb[GW], mm[NH][GW], vv[NH][GW];
    {
        const float* row = p.cent + e * p.c_ld;
        const uint32_t rb = (n > 0 || p.adam.on) ? nb : 0u;
        const rsrc_t sa = make_rsrc(row, rb), sb = make_rsrc(row + D, SPLIT ? rb : 0u);
#pragma unroll
        for (int gg = 0; gg < GW; ++gg) {
            ca[gg] = sload(sa, goffs[gg]);
            cb[gg] = SPLIT ? sload(sb, goffs[gg]) : vzero<V>();
        }
    }
    auto load_mv = [&]() {
        if (p.adam.on) {
#pragma unroll
            for (int h = 0; h < NH; ++h) {
                const rsrc_t sm = make_rsrc(p.adam.m + e * p.c_ld + h * D, nb);
                const rsrc_t sv = make_rsrc(p.adam.v + e * p.c_ld + h * D, nb);
#pragma unroll
                for (int gg = 0; gg < GW; ++gg) {
                    mm[h][gg] = sload(sm, goffs[gg]);
                    vv[h][gg] = sload(sv, goffs[gg]);
                }
            }
        }
    };
    vecf<V> sa[GW], sb[GW], ra[GW], rb[GW];  // candidate terms (normalised space), row events
#pragma unroll
    for (int gg = 0; gg < GW; ++gg) sa[gg] = sb[gg] = ra[gg] = rb[gg] = vzero<V>();
    float ia = 0.f, ib = 0.f;
    bool any_cand = false;
    if (n > 0) {
        // InterHT's half-norms of the row (block-wide; every wave calls this at the same point)
        auto norms = [&]() {
            if constexpr (FN == KGE_INTERHT) {
                float s2a = 0.f, s2b = 0.f;
#pragma unroll
                for (int gg = 0; gg < GW; ++gg)
#pragma unroll
                    for (int i = 0; i < V; ++i) {
                        s2a += ca[gg].a[i] * ca[gg].a[i];
                        s2b += cb[gg].a[i] * cb[gg].a[i];
                    }
                const float2 s = block_sum2(s2a, s2b, red, lane, w);
                ia = rsqrt_f(s.x);
                ib = rsqrt_f(s.y);
            }
        };
        // one event: its slice of the slot's stored query (candidate event) or of the slot's
        // query-entity gradient (row event)
        auto load_ev = [&](int code, vecf<V>(&x0)[GW], vecf<V>(&x1)[GW], vecf<V>(&x2)[GW]) {
            const float *b0, *b1, *b2 = p.rel;
            uint32_t n1, n2 = 0u;
            if (code < BN + p.Bn) {
                const int64_t slot = code < BN ? code / p.Nn : p.Bn + (code - BN);
                b0 = p.qbuf + slot * 3 * D;
                b1 = b0 + D;
                n1 = NQ > 1 ? nb : 0u;
                if constexpr (FN == KGE_INTERHT) {  // q2 = the slot's relation row (zero when out of range)
                    const int64_t bb = slot < p.Bn ? slot : slot - p.Bn;
                    const int64_t ri = p.r_idx ? p.r_idx[bb * p.r_stride] : bb;
                    const bool rok = ri >= 0 && ri < p.r_rows;
                    b2 = p.rel + (rok ? ri : 0) * p.r_ld + p.r_off;
                    n2 = rok ? nb : 0u;
                }
            } else {
                b0 = p.qg_ent + (code - BN - p.Bn) * p.ent_w;
                b1 = b0 + D;
                n1 = SPLIT ? nb : 0u;
            }
            const rsrc_t s0 = make_rsrc(b0, nb), s1 = make_rsrc(b1, n1), s2 = make_rsrc(b2, n2);
#pragma unroll
            for (int gg = 0; gg < GW; ++gg) {
                x0[gg] = bload<V>(s0, goffs[gg]);
                x1[gg] = (NQ > 1 || SPLIT) ? bload<V>(s1, goffs[gg]) : vzero<V>();
                x2[gg] = FN == KGE_INTERHT ? bload<V>(s2, goffs[gg]) : vzero<V>();
            }
        };
        auto apply_ev = [&](int code, const vecf<V>(&x0)[GW], const vecf<V>(&x1)[GW], const vecf<V>(&x2)[GW]) {
            if (code < BN + p.Bn) {
                const bool neg = code < BN;
                const float g = neg ? p.d_ns[code] : p.d_ps[code - BN];
                any_cand = true;
#pragma unroll
                for (int gg = 0; gg < GW; ++gg) {
                    if (neg)
                        ent_group_term<FN, CH, V>(ca[gg], cb[gg], x0[gg], x1[gg], x2[gg], gin[gg], g, ia, ib, p,
                                                  sa[gg], sb[gg]);
                    else  // the positive call scores the tail
                        ent_group_term<FN, false, V>(ca[gg], cb[gg], x0[gg], x1[gg], x2[gg], gin[gg], g, ia, ib, p,
                                                     sa[gg], sb[gg]);
                }
            } else {
#pragma unroll
                for (int gg = 0; gg < GW; ++gg)
#pragma unroll
                    for (int i = 0; i < V; ++i) {
                        ra[gg].a[i] += x0[gg].a[i];
                        if constexpr (SPLIT) rb[gg].a[i] += x1[gg].a[i];
                    }
            }
        };
        if (n <= kWave) {
            int code = code0;
            if ((unsigned)code >= (unsigned)ntot) code = INT32_MAX;  // never index with a stray code
            const int nv = __popcll(__ballot(code != INT32_MAX));
            code = wave_sort_asc(code, lane);
            for (int j = 0; j < nv; j += U) {
                vecf<V> x0[U][GW], x1[U][GW], x2[U][GW];
#pragma unroll
                for (int u = 0; u < U; ++u)
                    if (j + u < nv) load_ev(__builtin_amdgcn_readlane(code, j + u), x0[u], x1[u], x2[u]);
                // the norms after the first events' loads are issued (nv is block-uniform)
                if (j == 0) norms();
#pragma unroll
                for (int u = 0; u < U; ++u)
                    if (j + u < nv) apply_ev(__builtin_amdgcn_readlane(code, j + u), x0[u], x1[u], x2[u]);
            }
        } else if (n <= kEntSortMax) {
            norms();
            // large bucket (a hub entity, or a small table): one block-wide bitonic sort of its codes in LDS,
            // then the same ordered walk, U events in flight (n is block-uniform: every barrier is reached)
            int np2 = 2 * kWave;
            while (np2 < n) np2 <<= 1;
            for (int i = threadIdx.x; i < np2; i += kBlock) {
                int v = i < n ? p.ev_code[lo + i] : INT32_MAX;
                if ((unsigned)v >= (unsigned)ntot) v = INT32_MAX;  // never index with a stray code
                srt[i] = v;
            }
            __syncthreads();
            for (int k = 2; k <= np2; k <<= 1)
                for (int j = k >> 1; j > 0; j >>= 1) {
                    for (int i = threadIdx.x; i < np2; i += kBlock) {
                        const int ij = i ^ j;
                        if (ij > i) {
                            const int a = srt[i], c = srt[ij];
                            if ((a > c) == ((i & k) == 0)) {
                                srt[i] = c;
                                srt[ij] = a;
                            }
                        }
                    }
                    __syncthreads();
                }
            int nv = 0;  // valid codes (stray ones sorted to the end)
            for (int i = lane; i < n; i += kWave) nv += srt[i] != INT32_MAX ? 1 : 0;
            nv = (int)wave_sum((float)nv);
            for (int j = 0; j < nv; j += U) {
                vecf<V> x0[U][GW], x1[U][GW], x2[U][GW];
#pragma unroll
                for (int u = 0; u < U; ++u)
                    if (j + u < nv) load_ev(srt[j + u], x0[u], x1[u], x2[u]);
#pragma unroll
                for (int u = 0; u < U; ++u)
                    if (j + u < nv) apply_ev(srt[j + u], x0[u], x1[u], x2[u]);
            }
        } else {
            norms();
            // larger still: extract codes in ascending order (O(n^2 / 64))
            int last = -1;
            for (int it = 0; it < n; ++it) {
                int m = INT32_MAX;
                for (int i = lo + lane; i < hi; i += kWave) {
                    const int v = p.ev_code[i];
                    if (v > last && v < m && v < ntot) m = v;
                }
                m = wave_min_i(m);
                if (m == INT32_MAX) break;
                vecf<V> x0[GW], x1[GW], x2[GW];
                load_ev(m, x0, x1, x2);
                apply_ev(m, x0, x1, x2);
                last = m;
            }
        }
        load_mv();  // the moments' latency overlaps the row's closing dot
        if constexpr (FN == KGE_INTERHT) {
            // any_cand is block-uniform (every wave walks the same events)
            if (any_cand) {
                float da = 0.f, db = 0.f;
#pragma unroll
                for (int gg = 0; gg < GW; ++gg)
#pragma unroll
                    for (int i = 0; i < V; ++i) {
                        da += (ca[gg].a[i] * ia) * sa[gg].a[i];
                        db += (cb[gg].a[i] * ib) * sb[gg].a[i];
                    }
                const float2 dot = block_sum2(da, db, red, lane, w);
#pragma unroll
                for (int gg = 0; gg < GW; ++gg)
#pragma unroll
                    for (int i = 0; i < V; ++i) {
                        sa[gg].a[i] = (sa[gg].a[i] - (ca[gg].a[i] * ia) * dot.x) * ia;
                        sb[gg].a[i] = (sb[gg].a[i] - (cb[gg].a[i] * ib) * dot.y) * ib;
                    }
            }
        }
#pragma unroll
        for (int gg = 0; gg < GW; ++gg)
#pragma unroll
            for (int i = 0; i < V; ++i) {
                sa[gg].a[i] += ra[gg].a[i];
                sb[gg].a[i] += rb[gg].a[i];
            }
    }
    if (n <= 0) load_mv();
    auto sstore = [&](rsrc_t r, uint32_t off, const vecf<V>& v) { bstore<V, kEntStAux>(r, off, v); };
    if (p.adam.on) {
#pragma unroll
        for (int h = 0; h < NH; ++h) {
            const rsrc_t sp = make_rsrc(p.cent + e * p.c_ld + h * D, nb);
            const rsrc_t sm = make_rsrc(p.adam.m + e * p.c_ld + h * D, nb);
            const rsrc_t sv = make_rsrc(p.adam.v + e * p.c_ld + h * D, nb);
#pragma unroll
            for (int gg = 0; gg < GW; ++gg) {
                vecf<V> pp = h ? cb[gg] : ca[gg];
                const vecf<V>& gr = h ? sb[gg] : sa[gg];
#pragma unroll
                for (int i = 0; i < V; ++i)
                    adam_update(pp.a[i], gr.a[i], mm[h][gg].a[i], vv[h][gg].a[i], p.adam.b1, p.adam.b2, p.adam.eps,
                                p.adam.alpha, p.adam.step_size, p.adam.bc2_sqrt, p.adam.keras);
                sstore(sp, goffs[gg], pp);
                sstore(sm, goffs[gg], mm[h][gg]);
                sstore(sv, goffs[gg], vv[h][gg]);
            }
        }
        return;
    }
#pragma unroll
    for (int h = 0; h < NH; ++h) {
        const rsrc_t so = make_rsrc(p.d_out_ent + e * p.c_ld + h * D, nb);
#pragma unroll
        for (int gg = 0; gg < GW; ++gg) sstore(so, goffs[gg], h ? sb[gg] : sa[gg]);
    }
}

}  // namespace kge_impl

#include "kge_shard.h"

namespace kge_impl {

// ---------------------------------------------------------------------------------------------
// dispatch over (kind, candidate side, vector width, groups per lane) for one score function
// ---------------------------------------------------------------------------------------------
template <int FN, bool CH, int V, int G, int NWV>
void launch_tile(const ScoreParams& p, hipStream_t st, int blocks) {
    // up to the whole 160 KB of a CU's LDS per block (set once per instantiation)
    static const bool lds_ok = hipFuncSetAttribute(reinterpret_cast<const void*>(step_fwd_tile_kernel<FN, CH, V, G, NWV>),
                                                   hipFuncAttributeMaxDynamicSharedMemorySize, kTileLdsMax) == hipSuccess;
    (void)lds_ok;
    hipLaunchKernelGGL((step_fwd_tile_kernel<FN, CH, V, G, NWV>), dim3(blocks), dim3(NWV * kWave), p.tile_lds, st, p);
}

template <int FN, bool CH, int V, int G>
void launch_one(const ScoreParams& p, int kind, hipStream_t st, int blocks) {
    if (kind == KIND_SHARD_FWD_GRAD || kind == KIND_SHARD_POS || kind == KIND_SHARD_EPILOGUE)
        launch_shard<FN, CH, V, G>(p, kind, st, blocks);
    else if (kind == KIND_BWD)
        hipLaunchKernelGGL((score_bwd_kernel<FN, CH, V, G>), dim3(blocks), dim3(kBlock), 0, st, p);
    else if (kind == KIND_BWD_ROWS)
        hipLaunchKernelGGL((bwd_rows_kernel<FN, CH, V, G>), dim3(blocks), dim3(kBlock), 0, st, p);
    else if (kind == KIND_BWD_ENT)
        hipLaunchKernelGGL((bwd_ent_kernel<FN, CH, V, G>), dim3(blocks), dim3(kBlock), 0, st, p);
    else if (kind == KIND_BWD_STREAM) {
        if constexpr (G % kWavesPerBlock == 0)
            hipLaunchKernelGGL((bwd_stream_kernel<FN, CH, V, G>), dim3(blocks), dim3(kBlock), 0, st, p);
    } else if (kind == KIND_BWD_ENT_STREAM) {
        if constexpr (G % kWavesPerBlock == 0)
            hipLaunchKernelGGL((bwd_ent_stream_kernel<FN, CH, V, G>), dim3(blocks), dim3(kBlock), 0, st, p);
    } else if (kind == KIND_BWD_CHAIN)
        hipLaunchKernelGGL((bwd_chain_kernel<FN, CH, V, G>), dim3(blocks), dim3(kBlock), 0, st, p);
    else if (kind == KIND_FWD_STATS) {
        if constexpr (FN == KGE_INTERHT)
            hipLaunchKernelGGL((score_fwd_kernel<FN, CH, V, G, true>), dim3(blocks), dim3(kBlock), 0, st, p);
    }
    else if (kind == KIND_STEP_FWD)
        hipLaunchKernelGGL((step_fwd_kernel<FN, CH, V, G, false>), dim3(blocks), dim3(kBlock), 0, st, p);
    else if (kind == KIND_STEP_FWD_XCD)
        hipLaunchKernelGGL((step_fwd_xcd_kernel<FN, CH, V, G>), dim3(blocks), dim3(kBlock), 0, st, p);
    else if (kind == KIND_STEP_FWD_TILE || kind == KIND_SCORE_TILE) {
        if constexpr (G <= kFwdGradMaxG) {
            if (p.tile_waves == 16)
                launch_tile<FN, CH, V, G, 16>(p, st, blocks);
            else if (p.tile_waves == 12)
                launch_tile<FN, CH, V, G, 12>(p, st, blocks);
            else
                launch_tile<FN, CH, V, G, 8>(p, st, blocks);
        }
    }
    else if (kind == KIND_SCORE_SHARD_XCD)
        hipLaunchKernelGGL((score_sharded_xcd_kernel<FN, CH, V, G>), dim3(blocks), dim3(kBlock), 0, st, p);
    else if (kind == KIND_SHARD_BUCKET)
        hipLaunchKernelGGL((shard_bucket_kernel<FN, CH, V, G>), dim3(blocks), dim3(kBlock), 0, st, p);
    else if (kind == KIND_STEP_FWD_GRAD) {
        if constexpr (FN != KGE_PROTATE && G <= kFwdGradMaxG) {
            if (!p.adversarial)
                hipLaunchKernelGGL((step_fwd_grad_kernel<FN, CH, V, G, 0>), dim3(blocks), dim3(kBlock), 0, st, p);
            else if (p.detach)
                hipLaunchKernelGGL((step_fwd_grad_kernel<FN, CH, V, G, 1>), dim3(blocks), dim3(kBlock), 0, st, p);
            else
                hipLaunchKernelGGL((step_fwd_grad_kernel<FN, CH, V, G, 2>), dim3(blocks), dim3(kBlock), 0, st, p);
        }
    }
    else if (kind == KIND_STEP_EPILOGUE) {
        if constexpr (FN != KGE_PROTATE && G <= kFwdGradMaxG)
            hipLaunchKernelGGL((step_epilogue_kernel<FN, CH, V, G>), dim3(blocks), dim3(kBlock), 0, st, p);
    }
    else if (kind == KIND_STEP_FWD_STATS) {
        if constexpr (FN == KGE_INTERHT)
            hipLaunchKernelGGL((step_fwd_kernel<FN, CH, V, G, true>), dim3(blocks), dim3(kBlock), 0, st, p);
    }
    else if (kind == KIND_FINISH) {
        if constexpr (!CH) hipLaunchKernelGGL((finish_kernel<FN, V, G>), dim3(blocks), dim3(kBlock), 0, st, p);
    } else
        hipLaunchKernelGGL((score_fwd_kernel<FN, CH, V, G>), dim3(blocks), dim3(kBlock), 0, st, p);
}

template <int FN, bool CH, int V>
int launch_g(const ScoreParams& p, int kind, hipStream_t st, int blocks, int G) {
    switch (G) {
        case 1: launch_one<FN, CH, V, 1>(p, kind, st, blocks); return 0;
        case 2: launch_one<FN, CH, V, 2>(p, kind, st, blocks); return 0;
        case 4: launch_one<FN, CH, V, 4>(p, kind, st, blocks); return 0;
        case 8: launch_one<FN, CH, V, 8>(p, kind, st, blocks); return 0;
        case 16:
            // dword-per-lane backward for D <= 1024 (kBwdMaxG): every atomic wave-instruction then
            // covers 256 contiguous bytes, the full-rate shape for global float atomics
            if constexpr (V == 1) {
                if (kind == KIND_BWD) {
                    hipLaunchKernelGGL((score_bwd_kernel<FN, CH, 1, 16>), dim3(blocks), dim3(kBlock), 0, st, p);
                    return 0;
                }
            }
            return KGE_ENOTSUP;
        default: return KGE_ENOTSUP;
    }
}

template <int FN, bool CH>
int launch_v(const ScoreParams& p, int kind, hipStream_t st, int blocks, int V, int G) {
    switch (V) {
        case 4: return launch_g<FN, CH, 4>(p, kind, st, blocks, G);
        case 2: return launch_g<FN, CH, 2>(p, kind, st, blocks, G);
        case 1: return launch_g<FN, CH, 1>(p, kind, st, blocks, G);
        default: return KGE_ENOTSUP;
    }
}

template <int FN>
int launch_fn_tmpl(const ScoreParams& p, int kind, hipStream_t st, int blocks, bool ch, int V, int G) {
    return ch ? launch_v<FN, true>(p, kind, st, blocks, V, G) : launch_v<FN, false>(p, kind, st, blocks, V, G);
}

}  // namespace kge_impl
