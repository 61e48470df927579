// kge_abi.hip — the C-ABI of libkge_hip.so (include/kge_hip.h): argument checking, kernel
// selection, the per-row reduction kernels and the extern "C" entry points.
#include <string.h>

#include <algorithm>
#include <cmath>

#include <string>

#include "kge_device.h"
#include "kge_scan.h"

namespace kge_impl {
namespace {

// ---------------------------------------------------------------------------------------------
// Per-row reductions (model.py:145, 168-171, 195-198; upstream train_step). One wave per row.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void neg_reduce_kernel(const float* __restrict__ s, int64_t B, int64_t N,
                                                            int64_t ld, float T, int adversarial,
                                                            float* __restrict__ out) {
    const int64_t b = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (b >= B) return;
    const int lane = threadIdx.x & 63;
    const float res = row_reduce_fast(s + b * ld, N, T, adversarial, lane);
    if (lane == 0) out[b] = res;
}

// kge_step_forward's XCD-sliced form: the row reductions after step_fwd_xcd_kernel (one wave per row)
__global__ __launch_bounds__(kBlock) void neg_rows_kernel(ScoreParams p) {
    const int64_t b = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (b >= p.B) return;
    const int lane = threadIdx.x & 63;
    const float* row = p.out + b * p.out_ld;
    const float r = row_reduce_fast(row, p.N, p.temperature, p.adversarial, lane);
    if (lane == 0) p.out_neg[b] = r;
}

// With `ps` set it also writes the positive branch's d_ps[b] = d_out_pos[b] * sigmoid(-ps[b])
// (logsigmoid backward, model.py:145), saving the separate launch in the train step.
__global__ __launch_bounds__(kBlock) void neg_reduce_bwd_kernel(const float* __restrict__ s, int64_t B, int64_t N,
                                                                int64_t ld, float T, int adversarial, int detach,
                                                                const float* __restrict__ d_out,
                                                                float* __restrict__ d_s, int64_t d_ld,
                                                                const float* __restrict__ ps,
                                                                const float* __restrict__ d_out_pos,
                                                                float* __restrict__ d_ps) {
    const int64_t b = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (b >= B) return;
    const int lane = threadIdx.x & 63;
    if (ps && lane == 0) d_ps[b] = d_out_pos[b] * sigmoidf(-ps[b]);
    neg_row_bwd(s + b * ld, N, T, adversarial, detach, d_out[b], d_s + b * d_ld, lane);
}

__global__ __launch_bounds__(kBlock) void log_sigmoid_kernel(const float* __restrict__ x, int64_t n,
                                                             float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) out[i] = log_sigmoid(x[i]);
}

// Weighted train-step loss of supervisor.py:19-23 and its gradient, one block, fixed reduction order:
//   loss = (-sum(w * pos) / sum(w) - sum(w * neg) / sum(w)) / 2,   d_out[b] = (-0.5 / sum(w)) * w[b]
constexpr int kLossBlock = 1024;
__global__ __launch_bounds__(kLossBlock) void step_loss_kernel(const float* __restrict__ out_neg,
                                                               const float* __restrict__ out_pos,
                                                               const float* __restrict__ w, int64_t B,
                                                               float* __restrict__ loss, float* __restrict__ d_out) {
    __shared__ float red[3][kLossBlock];
    const int t = threadIdx.x;
    float sw = 0.f, sp = 0.f, sn = 0.f;
    for (int64_t b = t; b < B; b += kLossBlock) {
        const float wb = w[b];
        sw += wb;
        sp += wb * out_pos[b];
        sn += wb * out_neg[b];
    }
    red[0][t] = sw;
    red[1][t] = sp;
    red[2][t] = sn;
    __syncthreads();
    for (int o = kLossBlock / 2; o > 0; o >>= 1) {
        if (t < o) {
            red[0][t] += red[0][t + o];
            red[1][t] += red[1][t + o];
            red[2][t] += red[2][t + o];
        }
        __syncthreads();
    }
    const float tw = red[0][0];
    if (t == 0 && loss) *loss = (-red[1][0] / tw + -red[2][0] / tw) / 2.f;
    if (d_out) {
        const float c = -0.5f / tw;
        for (int64_t b = t; b < B; b += kLossBlock) d_out[b] = c * w[b];
    }
}

__global__ void add_scalar_kernel(const float* __restrict__ x, float* __restrict__ acc) { *acc += *x; }

__global__ __launch_bounds__(kBlock) void log_sigmoid_bwd_kernel(const float* __restrict__ x,
                                                                 const float* __restrict__ d_out, int64_t n,
                                                                 float* __restrict__ d_x) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) d_x[i] = d_out[i] * sigmoidf(-x[i]);
}

// ---------------------------------------------------------------------------------------------
// Dense Adam over a whole table (supervisor.py:26 optimizer.apply_gradients; run.py:111 Keras Adam).
//   keras: m += (g - m)(1 - b1); v += (g^2 - v)(1 - b2); p -= m * alpha / (sqrt(v) + eps),
//          alpha = lr * sqrt(1 - b2^t) / (1 - b1^t)
//   torch: m = lerp(m, g, 1 - b1); v = v * b2 + (1 - b2) g^2;
//          p -= (lr / (1 - b1^t)) * m / (sqrt(v) / sqrt(1 - b2^t) + eps)
// HBM-bound elementwise pass: 16-B loads/stores, grid-stride; optionally zeroes the gradient.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void adam_one(float& p, float& g, float& m, float& v, const AdamArgs& a) {
    adam_update(p, g, m, v, a.b1, a.b2, a.eps, a.alpha, a.step_size, a.bc2_sqrt, a.keras);
    if (a.zero_grad) g = 0.f;
}

// one thread per 2 float4 (8 floats): all eight 16-B loads issued before any math
constexpr int kAdamVec = 2;

// Streamed (touch-once) float4 i of a table: nontemporal loads and stores. On gfx950 nt on both
// sides lifts a 3-read/3-write stream from ~4.9 to ~5.4 TB/s (profiles/r01_stream_probe_nt.txt).
typedef float f4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 nt_ld4(const float* base, int64_t i) {
    const f4v x = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(base) + i);
    return make_float4(x[0], x[1], x[2], x[3]);
}
__device__ __forceinline__ void nt_st4(float* base, int64_t i, const float4& v) {
    const f4v x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<f4v*>(base) + i);
}

__global__ __launch_bounds__(kBlock) void adam_kernel(float* __restrict__ p, float* __restrict__ g,
                                                      float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                      AdamArgs a) {
    const int64_t n4 = n / 4;
    const int64_t i0 = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * kAdamVec;
    float4 P[kAdamVec], G[kAdamVec], M[kAdamVec], Vv[kAdamVec];
#pragma unroll
    for (int u = 0; u < kAdamVec; ++u) {
        const int64_t i = i0 + u;
        if (i < n4) {
            P[u] = nt_ld4(p, i);
            G[u] = nt_ld4(g, i);
            M[u] = nt_ld4(m, i);
            Vv[u] = nt_ld4(v, i);
        }
    }
#pragma unroll
    for (int u = 0; u < kAdamVec; ++u) {
        const int64_t i = i0 + u;
        if (i < n4) {
            adam_one(P[u].x, G[u].x, M[u].x, Vv[u].x, a);
            adam_one(P[u].y, G[u].y, M[u].y, Vv[u].y, a);
            adam_one(P[u].z, G[u].z, M[u].z, Vv[u].z, a);
            adam_one(P[u].w, G[u].w, M[u].w, Vv[u].w, a);
            nt_st4(p, i, P[u]);
            nt_st4(m, i, M[u]);
            nt_st4(v, i, Vv[u]);
            if (a.zero_grad) nt_st4(g, i, G[u]);
        }
    }
    if (blockIdx.x == 0)  // scalar tail (n % 4)
        for (int64_t i = n4 * 4 + threadIdx.x; i < n; i += kBlock) adam_one(p[i], g[i], m[i], v[i], a);
}

// The same update for buffers that are not all 16-byte aligned (e.g. a parameter that is an offset
// view of a larger allocation): dword accesses, grid-stride. Bitwise the same per element.
__global__ __launch_bounds__(kBlock) void adam_scalar_kernel(float* __restrict__ p, float* __restrict__ g,
                                                             float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                             AdamArgs a) {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock)
        adam_one(p[i], g[i], m[i], v[i], a);
}

// ---------------------------------------------------------------------------------------------
// Owned-row gather of a row-sharded table: out[i] = table[ids[i*stride] - lo] if this shard owns
// the id, else zeros (so a SUM all-reduce over shards assembles the rows exactly). One wave per row.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void gather_owned_kernel(const float* __restrict__ tab, int64_t rows, int64_t ld,
                                                              int64_t lo, const int64_t* __restrict__ ids,
                                                              int64_t stride, int64_t n, int64_t width,
                                                              float* __restrict__ out, int64_t out_ld, int vec4) {
    const int64_t i = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (i >= n) return;
    const int lane = threadIdx.x & 63;
    const int64_t id = ids[i * stride] - lo;
    const bool ok = id >= 0 && id < rows;
    const float* src = tab + (ok ? id : 0) * ld;
    float* dst = out + i * out_ld;
    if (vec4) {
        const rsrc_t r = make_rsrc(src, ok ? (uint32_t)(width * 4) : 0u);
        for (int64_t e = (int64_t)lane * 4; e < width; e += 4 * kWave) {
            const vecf<4> v = bload<4>(r, (uint32_t)(e * 4));
            *reinterpret_cast<vecf<4>*>(dst + e) = v;
        }
    } else {
        for (int64_t e = lane; e < width; e += kWave) dst[e] = ok ? src[e] : 0.f;
    }
}

// ---------------------------------------------------------------------------------------------
// Gradient events of the deterministic backward, bucketed by entity (counting sort).
//   code in [0, BN)            negative candidate (b = code / N, n = code % N)  key neg[b, n]
//   code in [BN, BN+B)         positive candidate of row b (single mode)        key pos[b, 2]
//   code in [BN+B, BN+2B)      query-entity gradient of the negative call's b   key pos[b, 2|0]
//   code in [BN+2B, BN+3B)     query-entity (h) gradient of the positive call   key pos[b, 0]
// ---------------------------------------------------------------------------------------------
struct EvArgs {
    const int64_t* pos;
    const int64_t* neg;
    int64_t neg_ld, B, N, E;
    int qcol;  // query-entity column of the negative call: 2 (head-batch) or 0
    int total;
};

__device__ __forceinline__ int64_t ev_key(const EvArgs& a, int code) {
    const int64_t BN = a.B * a.N;
    if (code < BN) return a.neg[(code / a.N) * a.neg_ld + code % a.N];
    int64_t b = code - BN;
    if (b < a.B) return a.pos[b * 3 + 2];
    b -= a.B;
    if (b < a.B) return a.pos[b * 3 + a.qcol];
    b -= a.B;
    return a.pos[b * 3 + 0];
}

__global__ __launch_bounds__(kBlock) void ev_count_kernel(EvArgs a, int* __restrict__ count) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= a.total) return;
    const int64_t k = ev_key(a, i);
    if (k >= 0 && k < a.E) atomicAdd(&count[k], 1);
}

__global__ __launch_bounds__(kBlock) void ev_scatter_kernel(EvArgs a, int* __restrict__ cursor, int* __restrict__ code) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= a.total) return;
    const int64_t k = ev_key(a, i);
    if (k >= 0 && k < a.E) {
        const int at = atomicAdd(&cursor[k], 1);
        if (at >= 0 && at < a.total) code[at] = i;
    }
}

// Relation gradient: one block per (relation, 64-column chunk). Its four waves split the slots (a
// quarter each), find the slots that use the relation 64 at a time (ballot) and add their rows in
// slot order with 8 rows' loads in flight; the partials are combined in wave order (deterministic).
// With `ra.on` the block then applies Adam to its 64 columns of the relation table in place (the
// dense optimizer of supervisor.py:26: columns no score function reads get a zero gradient).
struct RelAdam {
    float *p, *m, *v;
    AdamArgs a;
    int on;
};

constexpr int kRelWaves = 16;  // waves per relation chunk: each scans 1/16 of the slots (fewer dependent rounds)
__global__ __launch_bounds__(kRelWaves * kWave) void bwd_rel_kernel(const int64_t* __restrict__ pos, int64_t B, int64_t R,
                                                         const float* __restrict__ qg_rel, int64_t rel_w,
                                                         int64_t rel_off, float* __restrict__ d_rel, int64_t rel_ld,
                                                         int64_t rel_dim, const float* __restrict__ dmod_part,
                                                         float* __restrict__ d_mod, RelAdam ra) {
    __shared__ float red[kRelWaves][kWave];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (blockIdx.x == 0 && threadIdx.x == 0 && d_mod && dmod_part) {
        float m = 0.f;
        for (int64_t s = 0; s < 2 * B; ++s) m += dmod_part[s];
        *d_mod = m;
    }
    const int64_t chunks = (rel_dim + kWave - 1) / kWave;
    const int64_t rho = blockIdx.x / chunks;
    if (rho >= R) return;
    const int64_t c = (blockIdx.x - rho * chunks) * kWave + lane;  // column of the full relation row
    const bool used = c >= rel_off && c < rel_off + rel_w;
    const int64_t cu = c - rel_off;
    const int64_t S = 2 * B, per = (S + kRelWaves - 1) / kRelWaves;
    const int64_t s_lo = w * per, s_hi = min(S, s_lo + per);
    float acc = 0.f;
    if (__ballot(used)) {
        for (int64_t s0 = s_lo; s0 < s_hi; s0 += kWave) {
            const int64_t s = s0 + lane;
            unsigned long long m = __ballot(s < s_hi && pos[(s % B) * 3 + 1] == rho);  // slot s: row s % B
            while (m) {
                float v[8];
                int nv = 0;
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    v[u] = 0.f;
                    if (m) {
                        const int bit = __builtin_ctzll(m);
                        m &= m - 1;
                        v[u] = used ? qg_rel[(s0 + bit) * rel_w + cu] : 0.f;
                        ++nv;
                    }
                }
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    if (u < nv) acc += v[u];
            }
        }
    }
    red[w][lane] = acc;
    __syncthreads();
    if (w != 0 || c >= rel_dim) return;
    float g = 0.f;
#pragma unroll
    for (int ww = 0; ww < kRelWaves; ++ww) g += red[ww][lane];
    g = used ? g : 0.f;  // parts no score function reads get 0
    if (ra.on) {
        const int64_t e = rho * rel_ld + c;
        float p = ra.p[e], m = ra.m[e], v = ra.v[e];
        adam_update(p, g, m, v, ra.a.b1, ra.a.b2, ra.a.eps, ra.a.alpha, ra.a.step_size, ra.a.bc2_sqrt, ra.a.keras);
        ra.p[e] = p;
        ra.m[e] = m;
        ra.v[e] = v;
    } else {
        d_rel[rho * rel_ld + c] = g;
    }
}

// ---------------------------------------------------------------------------------------------
// Combine (between the two collectives; one wave per global batch row b): the merged row state and
// this shard's share of the negative slot's query gradient, scaled by the loss weight:
//   TF (RED 2):     go f_r (A_r - T R B_r) / Z      detached (1): go f_r A_r / Z      mean (0): go A_r / N
// Also the forward's outputs for every row: out_neg = R (the reduced negative branch), the positive's
// raw score and logsigmoid. Every rank computes identical merged values (same inputs, same order).
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void shard_combine_kernel(ScoreParams p) {
    const int64_t b = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (b >= p.B) return;
    const int lane = threadIdx.x & 63;
    const RowMerge r = merge_row(p, b);
    const float go = home_loss_weight(p, b, lane);
    const bool mean = !p.adversarial;
    const float R = mean ? r.Ln / (float)p.N : (r.Z > 0.f ? r.Ln / r.Z : 0.f);
    float ca = 0.f, cb = 0.f;
    if (mean) {
        ca = go / (float)p.N;
    } else if (r.Z > 0.f) {
        ca = go * r.f_me / r.Z;
        if (!p.detach) cb = -ca * (p.temperature * R);
    }
    const int64_t w = (int64_t)p.nq * p.D;
    const float* A = p.sh_A + b * w;
    const float* Bv = p.sh_B + b * w;
    float* dq = p.sh_dq + b * w;
    for (int64_t i = lane; i < w; i += kWave) {
        float v = ca * A[i];
        if (cb != 0.f) v += cb * Bv[i];
        dq[i] = v;
    }
    if (lane == 0) {
        float* m = p.sh_merged + b * 4;
        m[0] = r.M;
        m[1] = r.Z;
        m[2] = R;
        m[3] = r.pos;
        p.out_neg[b] = R;
        if (p.out_pos_raw) p.out_pos_raw[b] = r.pos;
        p.out_pos_ls[b] = log_sigmoid(r.pos);
    }
}

// ---------------------------------------------------------------------------------------------
// host helpers
// ---------------------------------------------------------------------------------------------
thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

int ok() {
    g_last_error.clear();
    return 0;
}

int check_launch(const char* what) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(KGE_EHIP, std::string(what) + ": " + hipGetErrorString(e));
    return ok();
}

bool aligned(const void* ptr, int bytes) { return ptr == nullptr || ((uintptr_t)ptr % (uintptr_t)bytes) == 0; }

// widest vector width every operand allows, then the groups-per-lane bucket
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

// candidates per wave: long runs amortise the per-wave query build; keep >= 8192 waves in flight
int pick_cpw(int64_t B, int64_t N) {
    if (N <= 1) return 1;
    int64_t cpw = 16;
    while (cpw > 4 && B * ((N + cpw - 1) / cpw) < 8192) cpw >>= 1;
    return (int)cpw;
}

int pick_cpw_sharded(int64_t B, int64_t N) {
    if (N <= 1) return 1;
    int64_t cpw = 512;
    while (cpw > 16 && B * ((N + cpw - 1) / cpw) < 8192) cpw >>= 1;
    return (int)cpw;
}

int dispatch(int fn, const ScoreParams& p, int kind, hipStream_t st, int blocks, bool ch, int V, int G) {
    switch (fn) {
        case KGE_TRANSE: return launch_transe(p, kind, st, blocks, ch, V, G);
        case KGE_DISTMULT: return launch_distmult(p, kind, st, blocks, ch, V, G);
        case KGE_COMPLEX: return launch_complex(p, kind, st, blocks, ch, V, G);
        case KGE_ROTATE: return launch_rotate(p, kind, st, blocks, ch, V, G);
        case KGE_INTERHT: return launch_interht(p, kind, st, blocks, ch, V, G);
        case KGE_PROTATE: return launch_protate(p, kind, st, blocks, ch, V, G);
        default: return KGE_EINVAL;
    }
}

int check_fn_mode(int fn, int mode) {
    if (mode != KGE_HEAD_BATCH && mode != KGE_TAIL_BATCH && mode != KGE_SINGLE)
        return fail(KGE_EINVAL, "mode must be 0 (head-batch), 1 (tail-batch) or 3 (single)");
    if (fn < KGE_TRANSE || fn > KGE_PROTATE) return fail(KGE_EINVAL, "unknown score function id " + std::to_string(fn));
    return 0;
}

int run_score(int fn, int mode, ScoreParams& p, int kind, void* stream) {
    int rc = check_fn_mode(fn, mode);
    if (rc) return rc;
    if (p.B < 0 || p.N < 0 || p.D <= 0) return fail(KGE_EINVAL, "bad shape (B, N, D)");
    if (p.B == 0 || p.N == 0) return ok();
    if (!p.qent || !p.rel || !p.cent) return fail(KGE_EINVAL, "null table pointer");
    int V = 1, G = 1;
    rc = pick_vg(p, V, G);
    if (rc) return rc;
    if (kind == KIND_BWD) {
        // backward: dword-per-lane layout (lane l owns elements l + 64k) so the gradient atomics are
        // 256-B contiguous per wave-instruction; falls back to the forward layout past D = 1024
        int g1 = 1;
        while (g1 * kWave < p.D) g1 <<= 1;
        if (g1 <= kBwdMaxG) {
            V = 1;
            G = g1;
        }
    }
    int64_t waves;
    if (kind == KIND_FINISH) {
        p.cpw = 1;
        p.wpr = 1;
        waves = p.B;
    } else if (kind == KIND_BWD_ROWS || kind == KIND_BWD_STREAM || kind == KIND_STEP_FWD ||
               kind == KIND_STEP_FWD_STATS || kind == KIND_STEP_FWD_GRAD || kind == KIND_SHARD_FWD_GRAD) {
        waves = p.B * kWavesPerBlock;  // one block per slot / batch row
    } else if (kind == KIND_STEP_FWD_TILE || kind == KIND_SCORE_TILE) {
        if (p.tile_rows < 1 || p.tile_lds > kTileLdsMax) return fail(KGE_EINVAL, "tile plan missing");
        // one block of tile_waves waves per (group of tile_rows batch rows, entity slice): run_score's
        // block count is waves / kWavesPerBlock; then, for a planned step, one tail block per group of the
        // next batch's plan
        const int64_t groups = (p.B + p.tile_rows - 1) / p.tile_rows;
        p.tile_blocks = (int)(groups * 8);
        waves = (groups * 8 + (p.tile_next.plan ? plan_groups(p.tile_next.B, p.tile_next.R) : 0)) * kWavesPerBlock;
    } else if (kind == KIND_STEP_FWD_XCD || kind == KIND_SCORE_SHARD_XCD || kind == KIND_SHARD_BUCKET) {
        waves = (p.B + kWavesPerBlock - 1) / kWavesPerBlock * kWavesPerBlock * 8;  // 8 slice blocks per 4 rows
        if (kind == KIND_STEP_FWD_XCD && p.xcd_phases > 1) waves *= p.xcd_phases;
    } else if (kind == KIND_BWD_CHAIN || kind == KIND_SHARD_POS) {
        waves = p.B;  // one wave per slot
    } else if (kind == KIND_STEP_EPILOGUE) {
        // one wave per slot (negative rows' chains, positives, negative rows' score gradients), then the
        // event-scatter blocks (about four codes per thread, at most 256 blocks), then one block for the loss
        const int64_t ev = p.B * p.N + 3 * p.B;
        const int64_t sb = std::min<int64_t>(std::max<int64_t>((ev + 4 * kBlock - 1) / (4 * kBlock), 1), 256);
        waves = (3 * p.B + kWavesPerBlock - 1) / kWavesPerBlock * kWavesPerBlock + (sb + 1) * kWavesPerBlock;
    } else if (kind == KIND_SHARD_EPILOGUE) {
        // one wave per slot (negative rows, then positives), then one block for the loss
        waves = (2 * p.B + kWavesPerBlock - 1) / kWavesPerBlock * kWavesPerBlock + kWavesPerBlock;
    } else if (kind == KIND_BWD_ENT) {
        waves = p.c_rows;  // one wave per entity row
    } else if (kind == KIND_BWD_ENT_STREAM) {
        waves = p.c_rows * kWavesPerBlock;  // one block per entity row
    } else {
        // sharded scoring compacts each wave's owned candidates: long runs (up to 512 ids, ~64 owned
        // at 8 shards) keep the per-wave query build amortised; >= 8192 waves still fill the chip
        p.cpw = p.skip_foreign ? pick_cpw_sharded(p.B, p.N) : pick_cpw(p.B, p.N);
        p.wpr = (int)((p.N + p.cpw - 1) / p.cpw);
        waves = p.B * p.wpr;
    }
    const int64_t blocks = (waves + kWavesPerBlock - 1) / kWavesPerBlock;
    if (blocks > INT32_MAX) return fail(KGE_EINVAL, "problem too large for one launch");
    const bool ch = (kind != KIND_FINISH && kind != KIND_SHARD_POS) && mode == KGE_HEAD_BATCH;
    if ((kind == KIND_BWD_ROWS || kind == KIND_BWD_ENT || kind == KIND_BWD_STREAM || kind == KIND_BWD_CHAIN ||
         kind == KIND_BWD_ENT_STREAM) &&
        G > kMaxG)
        return fail(KGE_ENOTSUP, "dimension too large");
    if ((kind == KIND_STEP_FWD_GRAD || kind == KIND_STEP_EPILOGUE || kind == KIND_SHARD_FWD_GRAD ||
         kind == KIND_SHARD_POS || kind == KIND_SHARD_EPILOGUE) &&
        (G > kFwdGradMaxG || fn == KGE_PROTATE))
        return fail(KGE_ENOTSUP, "the fused forward + query gradient needs D <= 1024 and no pRotatE");
    if ((kind == KIND_BWD_STREAM || kind == KIND_BWD_ENT_STREAM) && G % kWavesPerBlock)
        return fail(KGE_ENOTSUP, "the streaming backward needs G % 4 == 0");
    rc = dispatch(fn, p, kind, (hipStream_t)stream, (int)blocks, ch, V, G);
    if (rc) return fail(rc, "no kernel for this (function, width) combination");
    return check_launch(kind == KIND_BWD ? "kge score backward launch"
                                         : (kind == KIND_FINISH ? "kge finish launch" : "kge score launch"));
}

float phase_div_for(int fn, float emb_range) {
    // torch: tensor / (python float: emb_range.item() / pi) -> the divisor is rounded to fp32
    const double pi = (fn == KGE_PROTATE) ? 3.14159262358979323846 : 3.14159265358979323846;
    return (float)((double)emb_range / pi);
}

void fill_indexed(ScoreParams& p, int fn, int mode, const float* ent, int64_t nentity, int64_t ent_ld,
                  const float* rel, int64_t nrelation, int64_t rel_ld, int64_t rel_off, const int64_t* pos,
                  const int64_t* neg, int64_t neg_ld, int64_t B, int64_t N, int64_t D, float gamma, float emb_range,
                  float modulus) {
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
    p.gamma = gamma;
    p.phase_div = phase_div_for(fn, emb_range);
    p.modulus = modulus;
}

void fill_dense(ScoreParams& p, int fn, int mode, const float* head, int64_t head_ld, const float* rel,
                int64_t rel_ld, int64_t rel_off, const float* tail, int64_t tail_ld, int64_t B, int64_t N, int64_t D,
                float gamma, float emb_range, float modulus) {
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

bool empty(int64_t B, int64_t N) { return B == 0 || N == 0; }

// phases of kge_step_forward's XCD-sliced order (step_fwd_xcd_kernel): forms->xcd_phases chooses (A/B runs)
int xcd_phases(int64_t nentity, int64_t ent_ld, const kge_forms* forms) {
    const int forced = forms ? forms->xcd_phases : 0;
    if (forced > 0) return std::min(forced, 16);
    // a table larger than the 256 MB Infinity Cache is swept in phases of ~96 MB (C2's 327.5 MB: 4 phases,
    // 139 -> 128.5 us); a table that fits gains nothing and pays the extra id walks (C3's 116 MB at 4
    // phases: 144 -> 162 us)
    const int64_t bytes = nentity * ent_ld * 4, mall = (int64_t)256 << 20, phase = (int64_t)96 << 20;
    if (bytes <= mall) return 1;
    return (int)std::min<int64_t>((bytes + phase - 1) / phase, 8);
}

// kge_step_forward's candidate order: 0 batch-row-major (KIND_STEP_FWD), 1 XCD-sliced ascending ids per wave
// (KIND_STEP_FWD_XCD), 2 row-group x XCD-slice tiles (KIND_STEP_FWD_TILE, when its LDS plan fits).
// forms->step_order chooses (A/B runs and the cross-form tests).
int step_order(int64_t nentity, int64_t N, const kge_forms* forms = nullptr) {
    const int forced = forms ? forms->step_order : -1;
    if (nentity >= (int64_t)8 << 25) return 0;  // sort keys hold (id - slice start) << 6
    if (forced >= 0 && forced <= 2) return forced;
    return N >= 128 ? 2 : 0;
}
bool use_xcd_order(int64_t nentity, int64_t N, const kge_forms* forms = nullptr) {
    return step_order(nentity, N, forms) != 0;
}

// Rows per block of the tile kernel (step_fwd_tile_kernel) and its dynamic LDS: 0 when the plan does not fit
// (then the XCD-sliced form runs). forms->tile_rows caps the row count, tile_waves / tile_q2slots choose.
int tile_plan(int fn, ScoreParams& p, const kge_forms* forms = nullptr) {
    int V = 1, G = 1;
    if (pick_vg(p, V, G)) return 0;
    if (G > kFwdGradMaxG || p.N + 1 > 65536 || p.c_rows <= 0) return 0;
    const int64_t opb = (int64_t)G * kWave * V * 4;  // bytes of one query operand image
    // InterHT: batch rows sorted by relation (B <= kTileSortMaxB), relation thirds in LDS slots
    int64_t P2 = 0;
    if (fn == KGE_INTERHT && p.B <= kTileSortMaxB) {
        P2 = kWave;
        while (P2 < p.B) P2 <<= 1;
    }
    // waves per block (each two candidate rows deep): 12 for candidate rows of 4 KB or more (3 waves per SIMD
    // at <= 168 VGPRs; C2 InterHT 105 -> 95 us and C3 RotatE 124-131 -> 115-120 us against 8 waves, whose
    // 2 waves per SIMD leave the score's VALU exposed; 16 spills), 16 for smaller rows (C4 DistMult: 2 KB rows
    // need the waves for bytes in flight). forms->tile_waves chooses (8, 12, 16).
    const int64_t row_bytes = (int64_t)p.D * 4 * (is_split(fn) ? 2 : 1);
    p.tile_waves = row_bytes >= 4096 ? 12 : 16;
    const int fw = forms ? forms->tile_waves : 0;
    if (fw == 8 || fw == 12 || fw == 16) p.tile_waves = fw;
    const int64_t NT = (int64_t)p.tile_waves * kWave;
    const int64_t qrow = tile_nq(fn) * opb + 8 + 8 + 8 + 4, lrow = (p.N + 1) * 4;  // + rrow, brow, qid, q2slot
    const int64_t fixed = kTileBuckets * 4 + 16;
    // the list region also holds the relation sort's per-wave bucket counts ([ceil(kTileSortMaxB / NT) NWV][64],
    // step_fwd_tile_kernel step 0), sized for the block's actual wave count
    const int64_t sort_ints = P2 ? (kTileSortMaxB + NT - 1) / NT * p.tile_waves * kTileSortRel : 0;
    auto lds = [&](int64_t R, int64_t QS) { return R * qrow + QS * opb + fixed + std::max(R * lrow, sort_ints * 4); };
    int64_t R = kTileMaxRows;
    if (forms && forms->tile_rows > 0) R = std::min<int64_t>(R, forms->tile_rows);
    while (R >= 1 && lds(R, 0) > kTileLdsMax) --R;
    if (R < 1) return 0;
    int64_t QS = 0;
    if (fn == KGE_INTERHT)
        while (QS < R && lds(R, QS + 1) <= kTileLdsMax) ++QS;
    if (forms && forms->tile_q2slots >= 0) QS = std::min<int64_t>(QS, forms->tile_q2slots);
#ifdef KGE_PROFILING_KNOBS
    // profiling-only A/B knobs (a build with -DKGE_PROFILING_KNOBS): KGE_TILE_DRY=<level> runs the setup alone and
    // writes no scores; KGE_TILE_NOSORT keeps the batch-row order
    p.tile_dry = getenv("KGE_TILE_DRY") ? std::max(1, atoi(getenv("KGE_TILE_DRY"))) : 0;
    if (getenv("KGE_TILE_NOSORT")) P2 = 0;
#endif
    p.tile_rows = (int)R;
    p.tile_q2slots = (int)QS;
    p.tile_sort = (int)P2;
    p.tile_lds = (int)lds(R, QS);
    return 1;
}

// The tile parameters of a planned step (kge_step_plan / kge_step_forward_planned): tile_plan's choice for
// 16-B aligned tables of these shapes, so that a plan is made without the tables. Returns the rows per group
// (0: the tile form does not apply).
int planned_tile_params(int fn, int64_t nentity, int64_t ent_ld, int64_t nrelation, int64_t rel_ld, int64_t rel_off,
                        int64_t B, int64_t N, int64_t D, ScoreParams& p) {
    if (B <= 0 || N <= 0 || D <= 0 || nentity <= 0 || nentity >= ((int64_t)1 << 31) || B >= ((int64_t)1 << 31))
        return 0;
    const float* tab = reinterpret_cast<const float*>((uintptr_t)4096);
    fill_indexed(p, fn, KGE_TAIL_BATCH, tab, nentity, ent_ld, tab, nrelation, rel_ld, rel_off, nullptr, nullptr, 0, B,
                 N, D, 0.f, 1.f, 0.f);
    return tile_plan(fn, p) ? p.tile_rows : 0;
}

PlanArgs plan_args(const ScoreParams& tp, int mode, int64_t nentity, int64_t nrelation, const int64_t* pos,
                   const int64_t* neg, int64_t neg_ld, int64_t B, int64_t N, void* plan) {
    PlanArgs a;
    a.pos = pos;
    a.neg = neg;
    a.neg_ld = neg_ld;
    a.B = B;
    a.N = N;
    a.nent = nentity;
    a.nrel = nrelation;
    a.mode = mode;
    a.R = tp.tile_rows;
    a.sort = tp.tile_sort != 0;
    a.plan = reinterpret_cast<int*>(plan);
    return a;
}

}  // namespace

int set_error(int code, const char* msg) { return fail(code, msg); }
}  // namespace kge_impl

using namespace kge_impl;

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

int kge_step_forward_order(int64_t nentity, int64_t N) { return step_order(nentity, N); }

int kge_score_indexed(int fn, int mode, const float* ent, int64_t nentity, int64_t ent_ld, const float* rel,
                      int64_t nrelation, int64_t rel_ld, int64_t rel_off, const int64_t* pos, const int64_t* neg,
                      int64_t neg_ld, int64_t B, int64_t N, int64_t D, float gamma, float emb_range, float modulus,
                      float* scores, int64_t scores_ld, void* stream) {
    return kge_score_indexed_ex(fn, mode, ent, nentity, ent_ld, rel, nrelation, rel_ld, rel_off, pos, neg, neg_ld, B,
                                N, D, gamma, emb_range, modulus, scores, scores_ld, nullptr, stream);
}

int kge_score_indexed_ex(int fn, int mode, const float* ent, int64_t nentity, int64_t ent_ld, const float* rel,
                         int64_t nrelation, int64_t rel_ld, int64_t rel_off, const int64_t* pos, const int64_t* neg,
                         int64_t neg_ld, int64_t B, int64_t N, int64_t D, float gamma, float emb_range, float modulus,
                         float* scores, int64_t scores_ld, const kge_forms* forms, void* stream) {
    int rc = check_fn_mode(fn, mode);
    if (rc) return rc;
    if (B < 0 || N < 0 || D <= 0) return fail(KGE_EINVAL, "bad shape (B, N, D)");
    if (empty(B, mode == KGE_SINGLE ? 1 : N)) return ok();
    if (!pos) return fail(KGE_EINVAL, "pos must not be NULL");
    if (mode != KGE_SINGLE && !neg) return fail(KGE_EINVAL, "neg must not be NULL in head/tail-batch mode");
    if (!scores) return fail(KGE_EINVAL, "scores must not be NULL");
    ScoreParams p;
    fill_indexed(p, fn, mode, ent, nentity, ent_ld, rel, nrelation, rel_ld, rel_off, pos, neg, neg_ld, B, N, D, gamma,
                 emb_range, modulus);
    p.out = scores;
    p.out_ld = scores_ld;
    if (mode != KGE_SINGLE && nentity < ((int64_t)1 << 31) && use_xcd_order(nentity, N, forms)) {
        if (step_order(nentity, N, forms) == 2 && tile_plan(fn, p, forms))
            return run_score(fn, mode, p, KIND_SCORE_TILE, stream);  // row-group x XCD-slice tiles (§3.0)
        return run_score(fn, mode, p, KIND_SCORE_SHARD_XCD, stream);  // XCD-sliced gather order (§3.0)
    }
    return run_score(fn, mode, p, KIND_FWD, stream);
}

int kge_step_finish(int fn, const float* ent, int64_t nentity, int64_t ent_ld, const float* rel, int64_t nrelation,
                    int64_t rel_ld, int64_t rel_off, const int64_t* pos, int64_t B, int64_t D, float gamma,
                    float emb_range, float modulus, const float* neg_scores, int64_t N, int64_t ns_ld,
                    float temperature, int adversarial, float* out_neg, float* pos_scores, float* out_pos,
                    void* stream) {
    int rc = check_fn_mode(fn, KGE_SINGLE);
    if (rc) return rc;
    if (B < 0 || N <= 0 || D <= 0) return fail(KGE_EINVAL, "bad shape (B, N, D)");
    if (B == 0) return ok();
    if (!pos || !neg_scores || !out_neg || !out_pos) return fail(KGE_EINVAL, "null pointer");
    ScoreParams f;
    fill_indexed(f, fn, KGE_SINGLE, ent, nentity, ent_ld, rel, nrelation, rel_ld, rel_off, pos, nullptr, 0, B, 1, D,
                 gamma, emb_range, modulus);
    f.neg_scores = neg_scores;
    f.ns_ld = ns_ld;
    f.n_neg = N;
    f.temperature = temperature;
    f.adversarial = adversarial;
    f.out_neg = out_neg;
    f.out_pos_raw = pos_scores;
    f.out_pos_ls = out_pos;
    return run_score(fn, KGE_SINGLE, f, KIND_FINISH, stream);
}

int kge_step_forward(int fn, int mode, const float* ent, int64_t nentity, int64_t ent_ld, const float* rel,
                     int64_t nrelation, int64_t rel_ld, int64_t rel_off, const int64_t* pos, const int64_t* neg,
                     int64_t neg_ld, int64_t B, int64_t N, int64_t D, float gamma, float emb_range, float modulus,
                     float temperature, int adversarial, float* neg_scores, int64_t ns_ld, float* out_neg,
                     float* pos_scores, float* out_pos, float* cand_stats, void* stream) {
    return kge_step_forward_ex(fn, mode, ent, nentity, ent_ld, rel, nrelation, rel_ld, rel_off, pos, neg, neg_ld, B, N,
                               D, gamma, emb_range, modulus, temperature, adversarial, neg_scores, ns_ld, out_neg,
                               pos_scores, out_pos, cand_stats, nullptr, stream);
}

int kge_step_forward_ex(int fn, int mode, const float* ent, int64_t nentity, int64_t ent_ld, const float* rel,
                        int64_t nrelation, int64_t rel_ld, int64_t rel_off, const int64_t* pos, const int64_t* neg,
                        int64_t neg_ld, int64_t B, int64_t N, int64_t D, float gamma, float emb_range, float modulus,
                        float temperature, int adversarial, float* neg_scores, int64_t ns_ld, float* out_neg,
                        float* pos_scores, float* out_pos, float* cand_stats, const kge_forms* forms, void* stream) {
    int rc = check_fn_mode(fn, mode);
    if (rc) return rc;
    if (mode == KGE_SINGLE) return fail(KGE_EINVAL, "kge_step_forward needs a negative mode (0 or 1)");
    if (B < 0 || N <= 0 || D <= 0) return fail(KGE_EINVAL, "bad shape (B, N, D)");
    if (B == 0) return ok();
    if (!pos || !neg || !neg_scores || !out_neg || !out_pos) return fail(KGE_EINVAL, "null pointer");
    ScoreParams p;
    fill_indexed(p, fn, mode, ent, nentity, ent_ld, rel, nrelation, rel_ld, rel_off, pos, neg, neg_ld, B, N, D, gamma,
                 emb_range, modulus);
    p.out = neg_scores;
    p.out_ld = ns_ld;
    p.cand_stats = reinterpret_cast<float2*>(cand_stats);
    p.pos_base = pos;
    p.temperature = temperature;
    p.adversarial = adversarial;
    p.out_neg = out_neg;
    p.out_pos_raw = pos_scores;
    p.out_pos_ls = out_pos;
    const int order = step_order(nentity, N, forms);
    if (!(cand_stats && fn == KGE_INTERHT) && order != 0) {
        // two launches: the negatives (and the positives) in row-group x XCD-slice tiles or in XCD-sliced
        // ascending-id order, then the rows' self-adversarial reductions
        if (order == 2 && tile_plan(fn, p, forms)) {
            p.tile_pos = 1;
            rc = run_score(fn, mode, p, KIND_STEP_FWD_TILE, stream);
        } else {
            p.xcd_phases = xcd_phases(nentity, ent_ld, forms);
            rc = run_score(fn, mode, p, KIND_STEP_FWD_XCD, stream);
        }
        if (rc) return rc;
        const int64_t blocks = (B + kWavesPerBlock - 1) / kWavesPerBlock;
        hipLaunchKernelGGL(neg_rows_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, (hipStream_t)stream, p);
        return check_launch("kge_step_forward row reductions");
    }
    // one launch: negatives + the per-row finish (positive, reduction)
    return run_score(fn, mode, p, (cand_stats && fn == KGE_INTERHT) ? KIND_STEP_FWD_STATS : KIND_STEP_FWD, stream);
}

int64_t kge_step_plan_size(int fn, int64_t nentity, int64_t ent_ld, int64_t nrelation, int64_t rel_ld,
                           int64_t rel_off, int64_t B, int64_t N, int64_t D) {
    if (fn < KGE_TRANSE || fn > KGE_PROTATE) return 0;
    ScoreParams tp;
    const int R = planned_tile_params(fn, nentity, ent_ld, nrelation, rel_ld, rel_off, B, N, D, tp);
    return R ? plan_words(B, N, R) * 4 : 0;
}

int kge_step_plan(int fn, int mode, int64_t nentity, int64_t ent_ld, int64_t nrelation, int64_t rel_ld,
                  int64_t rel_off, const int64_t* pos, const int64_t* neg, int64_t neg_ld, int64_t B, int64_t N,
                  int64_t D, void* plan, void* stream) {
    if (fn < KGE_TRANSE || fn > KGE_PROTATE) return fail(KGE_EINVAL, "unknown score function id " + std::to_string(fn));
    if (mode != KGE_HEAD_BATCH && mode != KGE_TAIL_BATCH)
        return fail(KGE_EINVAL, "kge_step_plan needs a negative mode (0 or 1)");
    if (B <= 0 || N <= 0 || D <= 0) return fail(KGE_EINVAL, "bad shape (B, N, D)");
    if (!pos || !neg || !plan) return fail(KGE_EINVAL, "null pointer");
    if (!aligned(plan, 16)) return fail(KGE_EINVAL, "the plan must be 16-B aligned");
    ScoreParams tp;
    if (!planned_tile_params(fn, nentity, ent_ld, nrelation, rel_ld, rel_off, B, N, D, tp))
        return fail(KGE_ENOTSUP, "the tile form does not apply to this shape (kge_step_plan_size is 0)");
    const PlanArgs a = plan_args(tp, mode, nentity, nrelation, pos, neg, neg_ld, B, N, plan);
    const unsigned groups = (unsigned)plan_groups(B, tp.tile_rows);
    if (tp.tile_waves == 16)
        hipLaunchKernelGGL(tile_plan_kernel<16>, dim3(groups), dim3(16 * kWave), plan_lds_ints(16 * kWave) * 4,
                           (hipStream_t)stream, a);
    else
        hipLaunchKernelGGL(tile_plan_kernel<12>, dim3(groups), dim3(12 * kWave), plan_lds_ints(12 * kWave) * 4,
                           (hipStream_t)stream, a);
    return check_launch("kge_step_plan");
}

static int step_forward_planned(int fn, int mode, const float* ent, int64_t nentity, int64_t ent_ld, const float* rel,
                                int64_t nrelation, int64_t rel_ld, int64_t rel_off, int64_t B, int64_t N, int64_t D,
                                float gamma, float emb_range, float modulus, float temperature, int adversarial,
                                const void* plan, const int64_t* next_pos, const int64_t* next_neg,
                                int64_t next_neg_ld, int next_mode, void* next_plan, float* neg_scores, int64_t ns_ld,
                                float* out_neg, float* pos_scores, float* out_pos, int reverse, void* stream);

int kge_step_forward_planned(int fn, int mode, const float* ent, int64_t nentity, int64_t ent_ld, const float* rel,
                             int64_t nrelation, int64_t rel_ld, int64_t rel_off, int64_t B, int64_t N, int64_t D,
                             float gamma, float emb_range, float modulus, float temperature, int adversarial,
                             const void* plan, const int64_t* next_pos, const int64_t* next_neg, int64_t next_neg_ld,
                             int next_mode, void* next_plan, float* neg_scores, int64_t ns_ld, float* out_neg,
                             float* pos_scores, float* out_pos, void* stream) {
    return step_forward_planned(fn, mode, ent, nentity, ent_ld, rel, nrelation, rel_ld, rel_off, B, N, D, gamma,
                                emb_range, modulus, temperature, adversarial, plan, next_pos, next_neg, next_neg_ld,
                                next_mode, next_plan, neg_scores, ns_ld, out_neg, pos_scores, out_pos, 0, stream);
}

static int step_forward_planned(int fn, int mode, const float* ent, int64_t nentity, int64_t ent_ld, const float* rel,
                                int64_t nrelation, int64_t rel_ld, int64_t rel_off, int64_t B, int64_t N, int64_t D,
                                float gamma, float emb_range, float modulus, float temperature, int adversarial,
                                const void* plan, const int64_t* next_pos, const int64_t* next_neg,
                                int64_t next_neg_ld, int next_mode, void* next_plan, float* neg_scores, int64_t ns_ld,
                                float* out_neg, float* pos_scores, float* out_pos, int reverse, void* stream) {
    int rc = check_fn_mode(fn, mode);
    if (rc) return rc;
    if (mode == KGE_SINGLE) return fail(KGE_EINVAL, "kge_step_forward_planned needs a negative mode (0 or 1)");
    if (B <= 0 || N <= 0 || D <= 0) return fail(KGE_EINVAL, "bad shape (B, N, D)");
    if (!ent || !rel || !plan || !neg_scores || !out_neg || !out_pos) return fail(KGE_EINVAL, "null pointer");
    if (next_plan) {
        if (next_mode != KGE_HEAD_BATCH && next_mode != KGE_TAIL_BATCH)
            return fail(KGE_EINVAL, "the next batch needs a negative mode (0 or 1)");
        if (!next_pos || !next_neg) return fail(KGE_EINVAL, "next_plan needs next_pos and next_neg");
        if (next_plan == plan) return fail(KGE_EINVAL, "next_plan must not be the plan this step reads");
        if (!aligned(next_plan, 16)) return fail(KGE_EINVAL, "the plan must be 16-B aligned");
    }
    if (!aligned(plan, 16)) return fail(KGE_EINVAL, "the plan must be 16-B aligned");
    ScoreParams tp;
    const int R = planned_tile_params(fn, nentity, ent_ld, nrelation, rel_ld, rel_off, B, N, D, tp);
    ScoreParams p;
    fill_indexed(p, fn, mode, ent, nentity, ent_ld, rel, nrelation, rel_ld, rel_off, nullptr, nullptr, 0, B, N, D,
                 gamma, emb_range, modulus);
    if (!R || !tile_plan(fn, p) || p.tile_rows != R)
        return fail(KGE_ENOTSUP, "the tile form does not apply to these tables (unaligned rows, or "
                                 "kge_step_plan_size is 0): use kge_step_forward");
    p.out = neg_scores;
    p.out_ld = ns_ld;
    p.pos_base = nullptr;
    p.temperature = temperature;
    p.adversarial = adversarial;
    p.out_neg = out_neg;
    p.out_pos_raw = pos_scores;
    p.out_pos_ls = out_pos;
    p.tile_pos = 1;
    p.tile_rev = reverse;
    p.tile_plan = reinterpret_cast<const int*>(plan);
    // the next batch's plan: the scoring launch's tail blocks, on the CUs its scoring blocks free up at its end
    // (C2 device time per step, alternating modes: 93.6 us; made beside the row reductions 99.5 us, as a launch
    // of its own 101.6 us, not planned 101.9 us; scripts/plan_probe.py, profiles/r05_plan_ab.txt)
    if (next_plan) {
        p.tile_next = plan_args(tp, next_mode, nentity, nrelation, next_pos, next_neg, next_neg_ld, B, N, next_plan);
        p.tile_lds = std::max(p.tile_lds, plan_lds_ints(p.tile_waves * kWave) * 4);
    }
    rc = run_score(fn, mode, p, KIND_STEP_FWD_TILE, stream);
    if (rc) return rc;
    const int64_t blocks = (B + kWavesPerBlock - 1) / kWavesPerBlock;
    hipLaunchKernelGGL(neg_rows_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, (hipStream_t)stream, p);
    return check_launch("kge_step_forward_planned row reductions");
}

// The planned step loop as a handle (kge_step_planner_*): the tables, shapes and the two plan buffers are given
// once; a step then passes only the next batch and the outputs (9 arguments instead of 29: at C2 the device
// step is ~93 us and the host issues one step per step, so its per-call cost is part of the loop's rate).
struct kge_step_planner {
    int fn = 0, adversarial = 1;
    const float* ent = nullptr;
    const float* rel = nullptr;
    int64_t nentity = 0, ent_ld = 0, nrelation = 0, rel_ld = 0, rel_off = 0, B = 0, N = 0, D = 0;
    float gamma = 0.f, emb_range = 0.f, modulus = 0.f, temperature = 1.f;
    void* plans[2] = {nullptr, nullptr};
    int cur = -1;  // the buffer holding the next step's plan (-1: none)
    int mode = 0;  // that plan's batch mode
    // kge_step_planner_set_sweep: 1 (default) = the tile sweep's direction alternates step by step, so a step starts
    // on the entity rows the step before touched last, which the Infinity Cache still holds when the table is larger
    // than it (C2's 327.5 MB: 92.8 -> 86.3 us per step, scripts/sweep_probe.py, profiles/r06_sweep_ab.txt)
    int sweep = 1;
    int64_t steps = 0;  // steps issued
    void* stream = nullptr;
};

int kge_step_planner_create(kge_step_planner** out, int fn, const float* ent, int64_t nentity, int64_t ent_ld,
                            const float* rel, int64_t nrelation, int64_t rel_ld, int64_t rel_off, int64_t B, int64_t N,
                            int64_t D, float gamma, float emb_range, float modulus, float temperature, int adversarial,
                            void* plan0, void* plan1, int64_t plan_bytes, void* stream) {
    if (!out) return fail(KGE_EINVAL, "kge_step_planner_create: null pointer");
    *out = nullptr;
    const int64_t need = kge_step_plan_size(fn, nentity, ent_ld, nrelation, rel_ld, rel_off, B, N, D);
    if (need <= 0) return fail(KGE_ENOTSUP, "kge_step_planner_create: the tile form does not apply to this shape");
    if (!ent || !rel || !plan0 || !plan1 || plan0 == plan1) return fail(KGE_EINVAL, "kge_step_planner_create: bad pointers");
    if (plan_bytes < need || !aligned(plan0, 16) || !aligned(plan1, 16))
        return fail(KGE_EINVAL, "kge_step_planner_create: plan buffers too small or not 16-B aligned");
    kge_step_planner* sp = new kge_step_planner;
    sp->fn = fn;
    sp->ent = ent;
    sp->nentity = nentity;
    sp->ent_ld = ent_ld;
    sp->rel = rel;
    sp->nrelation = nrelation;
    sp->rel_ld = rel_ld;
    sp->rel_off = rel_off;
    sp->B = B;
    sp->N = N;
    sp->D = D;
    sp->gamma = gamma;
    sp->emb_range = emb_range;
    sp->modulus = modulus;
    sp->temperature = temperature;
    sp->adversarial = adversarial;
    sp->plans[0] = plan0;
    sp->plans[1] = plan1;
    sp->stream = stream;
    *out = sp;
    return ok();
}

int kge_step_planner_set_modulus(kge_step_planner* sp, float modulus) {
    if (!sp) return fail(KGE_EINVAL, "kge_step_planner_set_modulus: null pointer");
    sp->modulus = modulus;
    return ok();
}

int kge_step_planner_set_sweep(kge_step_planner* sp, int alternate) {
    if (!sp) return fail(KGE_EINVAL, "kge_step_planner_set_sweep: null pointer");
    if (alternate != 0 && alternate != 1) return fail(KGE_EINVAL, "kge_step_planner_set_sweep: 0 or 1");
    sp->sweep = alternate;
    return ok();
}

int kge_step_planner_plan(kge_step_planner* sp, const int64_t* pos, const int64_t* neg, int64_t neg_ld, int mode) {
    if (!sp) return fail(KGE_EINVAL, "kge_step_planner_plan: null pointer");
    const int buf = sp->cur < 0 ? 0 : sp->cur;
    const int rc = kge_step_plan(sp->fn, mode, sp->nentity, sp->ent_ld, sp->nrelation, sp->rel_ld, sp->rel_off, pos, neg,
                                 neg_ld, sp->B, sp->N, sp->D, sp->plans[buf], sp->stream);
    if (rc) return rc;
    sp->cur = buf;
    sp->mode = mode;
    return ok();
}

int kge_step_planner_step(kge_step_planner* sp, const int64_t* next_pos, const int64_t* next_neg, int64_t next_neg_ld,
                          int next_mode, float* neg_scores, float* out_neg, float* pos_scores, float* out_pos) {
    if (!sp) return fail(KGE_EINVAL, "kge_step_planner_step: null pointer");
    if (sp->cur < 0) return fail(KGE_EINVAL, "kge_step_planner_step: no batch planned (kge_step_planner_plan first)");
    const bool nxt = next_pos && next_neg;
    const int rc = step_forward_planned(
        sp->fn, sp->mode, sp->ent, sp->nentity, sp->ent_ld, sp->rel, sp->nrelation, sp->rel_ld, sp->rel_off, sp->B,
        sp->N, sp->D, sp->gamma, sp->emb_range, sp->modulus, sp->temperature, sp->adversarial, sp->plans[sp->cur],
        next_pos, next_neg, next_neg_ld, next_mode, nxt ? sp->plans[1 - sp->cur] : nullptr, neg_scores, sp->N, out_neg,
        pos_scores, out_pos, sp->sweep ? (int)(sp->steps & 1) : 0, sp->stream);
    if (rc) return rc;
    ++sp->steps;
    if (nxt) {
        sp->cur = 1 - sp->cur;
        sp->mode = next_mode;
    } else {
        sp->cur = -1;
    }
    return ok();
}

int kge_step_planner_destroy(kge_step_planner* sp) {
    delete sp;
    return ok();
}

int kge_score_sharded(int fn, int mode, const float* qent, int64_t q_ld, const float* rel, int64_t nrelation,
                      int64_t rel_ld, int64_t rel_off, const float* shard, int64_t shard_rows, int64_t shard_ld,
                      int64_t shard_lo, const int64_t* pos, const int64_t* neg, int64_t neg_ld, int64_t B, int64_t N,
                      int64_t D, float gamma, float emb_range, float modulus, float* scores, int64_t scores_ld,
                      void* stream) {
    int rc = check_fn_mode(fn, mode);
    if (rc) return rc;
    if (B < 0 || N < 0 || D <= 0 || shard_rows < 0) return fail(KGE_EINVAL, "bad shape");
    if (empty(B, mode == KGE_SINGLE ? 1 : N)) return ok();
    if (!pos || (mode != KGE_SINGLE && !neg) || !scores || !qent || !shard)
        return fail(KGE_EINVAL, "null pointer");
    ScoreParams p;
    fill_indexed(p, fn, mode, shard, shard_rows, shard_ld, rel, nrelation, rel_ld, rel_off, pos, neg, neg_ld, B, N,
                 D, gamma, emb_range, modulus);
    // query entity rows come pre-assembled (row b of qent); candidates from the local shard
    p.qent = qent;
    p.q_idx = nullptr;
    p.q_ld = q_ld;
    p.q_rows = B;
    p.c_base = shard_lo;
    p.skip_foreign = 1;
    p.out = scores;
    p.out_ld = scores_ld;
    if (mode != KGE_SINGLE && shard_lo >= 0 && shard_lo + shard_rows < ((int64_t)1 << 31) &&
        use_xcd_order(shard_rows, N))
        return run_score(fn, mode, p, KIND_SCORE_SHARD_XCD, stream);  // XCD-sliced order over the shard
    return run_score(fn, mode, p, KIND_FWD, stream);
}

int kge_shard_score(int fn, int mode, const float* qent, int64_t q_rows, int64_t q_ld, const int64_t* q_idx,
                    const float* rel, int64_t nrelation, int64_t rel_ld, int64_t rel_off, const float* shard,
                    int64_t shard_rows, int64_t shard_ld, int64_t shard_lo, const int64_t* pos, int64_t B, int64_t N,
                    int64_t D, float gamma, float emb_range, float modulus, const int* bucket,
                    const int* bucket_start, const int* pre, const int* cnt, const int* tot, int world, int rank,
                    int64_t home_B, int64_t home0, float* send, void* stream) {
    if (mode != KGE_HEAD_BATCH && mode != KGE_TAIL_BATCH)
        return fail(KGE_EINVAL, "kge_shard_score: mode must be 0 (head-batch) or 1 (tail-batch)");
    int rc = check_fn_mode(fn, mode);
    if (rc) return rc;
    if (B < 0 || N < 0 || D <= 0 || shard_rows <= 0 || q_rows < 0) return fail(KGE_EINVAL, "bad shape");
    if (world < 1 || rank < 0 || rank >= world || home_B <= 0 || B % home_B || home0 < 0 ||
        home0 + B / home_B > world)
        return fail(KGE_EINVAL, "kge_shard_score: rows must be whole homes of home_B rows");
    if (shard_lo < 0 || shard_rows >= ((int64_t)1 << 25))
        return fail(KGE_ENOTSUP, "kge_shard_score: the shard must hold < 2^25 rows");
    if (B == 0) return ok();
    if (!pos || !send || !qent || !q_idx || !shard || !bucket || !bucket_start || !pre || !cnt || !tot)
        return fail(KGE_EINVAL, "null pointer");
    ScoreParams p;
    fill_indexed(p, fn, mode, shard, shard_rows, shard_ld, rel, nrelation, rel_ld, rel_off, pos, nullptr, 0, B, N + 1,
                 D, gamma, emb_range, modulus);
    // query entity rows: row q_idx[b] of the exchanged query block; candidates: the bucket's shard rows
    p.qent = qent;
    p.q_idx = q_idx;
    p.q_stride = 1;
    p.q_ld = q_ld;
    p.q_rows = q_rows;
    p.c_idx = nullptr;
    p.c_base = shard_lo;
    p.skip_foreign = 1;
    p.pos_base = pos;
    p.bk_ent = reinterpret_cast<const int2*>(bucket);
    p.bk_start = bucket_start;
    p.bk_ld = N + 1;
    p.cmp_pre = pre;
    p.cmp_cnt = cnt;
    p.cmp_tot = tot;
    p.cmp_home0 = home0;
    p.home_B = home_B;
    p.world = world;
    p.rank = rank;
    p.out = send;
    p.out_ld = 0;
    return run_score(fn, mode, p, KIND_SHARD_BUCKET, stream);
}

int kge_gather_rows(const float* table, int64_t rows, int64_t ld, int64_t lo, const int64_t* ids, int64_t id_stride,
                    int64_t n, int64_t width, float* out, int64_t out_ld, void* stream) {
    if (n < 0 || width < 0 || rows < 0) return fail(KGE_EINVAL, "bad shape");
    if (n == 0 || width == 0) return ok();
    if (!table || !ids || !out) return fail(KGE_EINVAL, "null pointer");
    const int vec4 = (width % 4 == 0 && ld % 4 == 0 && out_ld % 4 == 0 && aligned(table, 16) && aligned(out, 16));
    const int64_t blocks = (n + kWavesPerBlock - 1) / kWavesPerBlock;
    hipLaunchKernelGGL(gather_owned_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, (hipStream_t)stream, table, rows,
                       ld, lo, ids, id_stride, n, width, out, out_ld, vec4);
    return check_launch("kge_gather_rows");
}

int kge_eval_query(int fn, int mode, const float* ent, int64_t nentity, int64_t ent_ld, const float* rel,
                   int64_t nrelation, int64_t rel_ld, const int64_t* pos, int64_t B, int64_t D, float* Q, int64_t ldq,
                   void* stream) {
    int rc = check_fn_mode(fn, mode);
    if (rc) return rc;
    if (fn != KGE_DISTMULT && fn != KGE_COMPLEX)
        return fail(KGE_ENOTSUP, "kge_eval_query: only DistMult and ComplEx score as a dense contraction");
    if (mode == KGE_SINGLE) return fail(KGE_EINVAL, "kge_eval_query needs mode 0 or 1");
    if (B < 0 || D <= 0) return fail(KGE_EINVAL, "bad shape");
    if (B == 0) return ok();
    if (!ent || !rel || !pos || !Q) return fail(KGE_EINVAL, "null pointer");
    ScoreParams p;
    fill_indexed(p, fn, mode, ent, nentity, ent_ld, rel, nrelation, rel_ld, 0, pos, nullptr, 0, B, 1, D, 0.f, 1.f,
                 0.f);
    int V = 1, G = 1;
    rc = pick_vg(p, V, G);
    if (rc) return rc;
    if (ldq % V) V = 1;
    while (V > 1 && !aligned(Q, 4 * V)) V >>= 1;
    G = 1;
    while (G * kWave * V < D) G <<= 1;
    if (G > kMaxG) return fail(KGE_ENOTSUP, "dimension too large");
    const int64_t blocks = (B + kWavesPerBlock - 1) / kWavesPerBlock;
    rc = launch_eval_query_any(fn, mode == KGE_HEAD_BATCH, p, (hipStream_t)stream, (int)blocks, V, G, Q, ldq);
    if (rc) return fail(rc, "no eval-query kernel for this width");
    return check_launch("kge_eval_query");
}

int kge_eval_query_planes(int fn, int mode, const float* ent, int64_t nentity, int64_t ent_ld, const float* rel,
                          int64_t nrelation, int64_t rel_ld, const int64_t* pos, int64_t B, int64_t D, void* planes,
                          int64_t plane_rows, void* stream) {
    int rc = check_fn_mode(fn, mode);
    if (rc) return rc;
    if (fn != KGE_DISTMULT && fn != KGE_COMPLEX)
        return fail(KGE_ENOTSUP, "kge_eval_query_planes: only DistMult and ComplEx score as a dense contraction");
    if (mode == KGE_SINGLE) return fail(KGE_EINVAL, "kge_eval_query_planes needs mode 0 or 1");
    if (B < 0 || D <= 0 || plane_rows < B) return fail(KGE_EINVAL, "bad shape");
    if (B == 0) return ok();
    if (!ent || !rel || !pos || !planes) return fail(KGE_EINVAL, "null pointer");
    if (!aligned(planes, 16)) return fail(KGE_EINVAL, "kge_eval_query_planes: planes not 16-B aligned");
    ScoreParams p;
    fill_indexed(p, fn, mode, ent, nentity, ent_ld, rel, nrelation, rel_ld, 0, pos, nullptr, 0, B, 1, D, 0.f, 1.f,
                 0.f);
    int V = 1, G = 1;
    rc = pick_vg(p, V, G);
    if (rc) return rc;
    if (V != 4) return fail(KGE_ENOTSUP, "kge_eval_query_planes needs D % 4 == 0 and 16-B aligned tables");
    G = 1;
    while (G * kWave * V < D) G <<= 1;
    if (G > kMaxG) return fail(KGE_ENOTSUP, "dimension too large");
    const int64_t blocks = (B + kWavesPerBlock - 1) / kWavesPerBlock;
    rc = launch_eval_query_any(fn, mode == KGE_HEAD_BATCH, p, (hipStream_t)stream, (int)blocks, V, G, nullptr, 0,
                               planes, plane_rows);
    if (rc) return fail(rc, "no eval-query kernel for this width");
    return check_launch("kge_eval_query_planes");
}

int kge_gemm_nt(const float* A, int64_t lda, const float* Bm, int64_t ldb, float* C, int64_t ldc, int64_t M,
                int64_t N, int64_t K, void* stream) {
    if (M < 0 || N < 0 || K < 0) return fail(KGE_EINVAL, "bad shape");
    if (M == 0 || N == 0) return ok();
    if (!A || !Bm || !C) return fail(KGE_EINVAL, "null pointer");
    if (M > INT32_MAX || N > INT32_MAX || K > INT32_MAX) return fail(KGE_EINVAL, "shape exceeds int32");
    if (K % 4 || lda % 4 || ldb % 4 || !aligned(A, 16) || !aligned(Bm, 16))
        return fail(KGE_ENOTSUP, "kge_gemm_nt needs K, lda, ldb multiples of 4 and 16-byte aligned A, B");
    launch_gemm_nt(A, Bm, C, (int)M, (int)N, (int)K, lda, ldb, ldc, (hipStream_t)stream);
    return check_launch("kge_gemm_nt");
}

int64_t kge_split_bf16x3_bytes(int64_t rows, int64_t cols) {
    if (rows < 0 || cols <= 0) return 0;
    return 3 * rows * ((cols + 15) / 16 * 16) * 2;
}

int kge_split_bf16x3(const float* X, int64_t rows, int64_t cols, int64_t ld, void* planes, int64_t plane_rows,
                     void* stream) {
    if (rows < 0 || cols <= 0 || ld < cols || plane_rows < rows) return fail(KGE_EINVAL, "kge_split_bf16x3: bad shape");
    if (rows == 0) return ok();
    if (!X || !planes) return fail(KGE_EINVAL, "kge_split_bf16x3: null pointer");
    if (!aligned(planes, 16)) return fail(KGE_EINVAL, "kge_split_bf16x3: planes must be 16-B aligned");
    if (kge_split_bf16x3_bytes(plane_rows, cols) >= ((int64_t)1 << 32) - 16)
        return fail(KGE_ENOTSUP, "kge_split_bf16x3: planes past 4 GB (the GEMM's 32-bit buffer offsets)");
    launch_split3_planes(X, rows, cols, ld, planes, plane_rows, (hipStream_t)stream);
    return check_launch("kge_split_bf16x3");
}

int kge_gemm_nt_bf16x3_planes(const void* A_planes, int64_t a_rows, const void* B_planes, int64_t b_rows, int64_t K,
                              float* C, int64_t ldc, int64_t M, int64_t N, void* stream) {
    return kge_gemm_nt_bf16x3_planes_ex(A_planes, a_rows, B_planes, b_rows, K, C, ldc, M, N, nullptr, stream);
}

// the plane GEMM the library runs (forms->gemm_form 0): 1 = gemm_nt_x3p_kernel 256 x 256, 2 = gemm_nt_x3d_kernel,
// 3 = gemm_nt_x3p_kernel 256 x 192, 4 = gemm_nt_x3l_kernel (LDS-DMA staging, three stages; 546 against 551 us at
// C5's shape, 568 against 572 us for the rank call: profiles/r06_gemm_dma_ab.txt)
constexpr int kPlanesGemmForm = 4;

int kge_gemm_nt_bf16x3_planes_ex(const void* A_planes, int64_t a_rows, const void* B_planes, int64_t b_rows, int64_t K,
                                 float* C, int64_t ldc, int64_t M, int64_t N, const kge_forms* forms, void* stream) {
    const int form = forms && forms->gemm_form >= 1 && forms->gemm_form <= 4 ? forms->gemm_form : kPlanesGemmForm;
    if (M < 0 || N < 0 || K <= 0 || M > a_rows || N > b_rows) return fail(KGE_EINVAL, "bad shape");
    if (M == 0 || N == 0) return ok();
    if (!A_planes || !B_planes || !C) return fail(KGE_EINVAL, "null pointer");
    if (M > INT32_MAX || N > INT32_MAX || !aligned(A_planes, 16) || !aligned(B_planes, 16))
        return fail(KGE_EINVAL, "kge_gemm_nt_bf16x3_planes: int32 shapes and 16-B aligned planes");
    if (kge_split_bf16x3_bytes(a_rows, K) >= ((int64_t)1 << 32) - 16 ||
        kge_split_bf16x3_bytes(b_rows, K) >= ((int64_t)1 << 32) - 16)
        return fail(KGE_ENOTSUP, "kge_gemm_nt_bf16x3_planes: planes past 4 GB");
    launch_gemm_nt_x3p(A_planes, a_rows, B_planes, b_rows, K, C, ldc, (int)M, (int)N, (hipStream_t)stream, form);
    return check_launch("kge_gemm_nt_bf16x3_planes");
}

int kge_gemm_nt_bf16x3(const float* A, int64_t lda, const float* Bm, int64_t ldb, float* C, int64_t ldc, int64_t M,
                      int64_t N, int64_t K, void* stream) {
    return kge_gemm_nt_bf16x3_ex(A, lda, Bm, ldb, C, ldc, M, N, K, nullptr, stream);
}

int kge_gemm_nt_bf16x3_ex(const float* A, int64_t lda, const float* Bm, int64_t ldb, float* C, int64_t ldc, int64_t M,
                          int64_t N, int64_t K, const kge_forms* forms, void* stream) {
    if (M < 0 || N < 0 || K < 0) return fail(KGE_EINVAL, "bad shape");
    if (M == 0 || N == 0) return ok();
    if (!A || !Bm || !C) return fail(KGE_EINVAL, "null pointer");
    if (M > INT32_MAX || N > INT32_MAX || K > INT32_MAX) return fail(KGE_EINVAL, "shape exceeds int32");
    if (K % 4 || lda % 4 || ldb % 4 || !aligned(A, 16) || !aligned(Bm, 16))
        return fail(KGE_ENOTSUP, "kge_gemm_nt_bf16x3 needs K, lda, ldb multiples of 4 and 16-byte aligned A, B");
    launch_gemm_nt_f32x3(A, Bm, C, (int)M, (int)N, (int)K, lda, ldb, ldc, (hipStream_t)stream, forms ? forms->gemm_form : 0);
    return check_launch("kge_gemm_nt_bf16x3");
}

int kge_rank_filtered(const float* scores, int64_t M, int64_t N, int64_t ld, const int64_t* truth,
                      const int64_t* filter_ptr, const int64_t* filter_ids, int64_t* ranks, void* stream) {
    if (M < 0 || N < 0) return fail(KGE_EINVAL, "bad shape");
    if (M == 0) return ok();
    if (!scores || !truth || !ranks || (filter_ptr && !filter_ids)) return fail(KGE_EINVAL, "null pointer");
    if (M > INT32_MAX) return fail(KGE_EINVAL, "too many rows");
    launch_rank(scores, M, N, ld, truth, filter_ptr, filter_ids, ranks, (hipStream_t)stream);
    return check_launch("kge_rank_filtered");
}

int64_t kge_eval_rank_planes_workspace_size(int64_t M, int64_t nfilter) {
    if (M < 0 || nfilter < 0) return 0;
    return eval_rank_ws_bytes(M, nfilter);
}

int kge_eval_rank_planes(const void* A_planes, int64_t a_rows, const void* B_planes, int64_t b_rows, int64_t K,
                         int64_t M, int64_t N, const int64_t* truth, const int64_t* filter_ptr,
                         const int64_t* filter_ids, int64_t nfilter, int64_t* ranks, void* workspace,
                         size_t workspace_bytes, void* stream) {
    return kge_eval_rank_planes_ex(A_planes, a_rows, B_planes, b_rows, K, M, N, truth, filter_ptr, filter_ids, nfilter,
                                   ranks, workspace, workspace_bytes, nullptr, stream);
}

int kge_eval_rank_planes_ex(const void* A_planes, int64_t a_rows, const void* B_planes, int64_t b_rows, int64_t K,
                            int64_t M, int64_t N, const int64_t* truth, const int64_t* filter_ptr,
                            const int64_t* filter_ids, int64_t nfilter, int64_t* ranks, void* workspace,
                            size_t workspace_bytes, const kge_forms* forms, void* stream) {
    return kge_eval_rank_planes_phases(A_planes, a_rows, B_planes, b_rows, K, M, N, truth, filter_ptr, filter_ids,
                                       nfilter, ranks, workspace, workspace_bytes, KGE_RANK_ALL, forms, stream);
}

int kge_eval_rank_planes_phases(const void* A_planes, int64_t a_rows, const void* B_planes, int64_t b_rows, int64_t K,
                                int64_t M, int64_t N, const int64_t* truth, const int64_t* filter_ptr,
                                const int64_t* filter_ids, int64_t nfilter, int64_t* ranks, void* workspace,
                                size_t workspace_bytes, int phases, const kge_forms* forms, void* stream) {
    if (phases <= 0 || phases > KGE_RANK_ALL) return fail(KGE_EINVAL, "kge_eval_rank_planes: phases must be 1..7");
    const int form = forms && (forms->gemm_form == 1 || forms->gemm_form >= 3) && forms->gemm_form <= 4
                         ? forms->gemm_form
                         : (kPlanesGemmForm == 2 ? 1 : kPlanesGemmForm);
    if (M < 0 || N <= 0 || K <= 0 || M > a_rows || N > b_rows || nfilter < 0) return fail(KGE_EINVAL, "bad shape");
    if (M == 0) return ok();
    if (!A_planes || !B_planes || !truth || !ranks || !workspace || (filter_ptr && !filter_ids && nfilter > 0) ||
        (nfilter > 0 && !filter_ptr))
        return fail(KGE_EINVAL, "null pointer");
    if (M > INT32_MAX || N > INT32_MAX || !aligned(A_planes, 16) || !aligned(B_planes, 16) || !aligned(workspace, 16))
        return fail(KGE_EINVAL, "kge_eval_rank_planes: int32 shapes and 16-B aligned planes / workspace");
    if (kge_split_bf16x3_bytes(a_rows, K) >= ((int64_t)1 << 32) - 16 ||
        kge_split_bf16x3_bytes(b_rows, K) >= ((int64_t)1 << 32) - 16)
        return fail(KGE_ENOTSUP, "kge_eval_rank_planes: planes past 4 GB");
    if ((int64_t)workspace_bytes < eval_rank_ws_bytes(M, nfilter))
        return fail(KGE_EINVAL, "kge_eval_rank_planes: workspace too small");
    launch_eval_rank_planes(A_planes, a_rows, B_planes, b_rows, K, (int)M, (int)N, truth, filter_ptr, filter_ids,
                            nfilter, ranks, workspace, (hipStream_t)stream, form, phases);
    return check_launch("kge_eval_rank_planes");
}

int kge_score_dense(int fn, int mode, const float* head, int64_t head_ld, const float* rel, int64_t rel_ld,
                    int64_t rel_off, const float* tail, int64_t tail_ld, int64_t B, int64_t N, int64_t D, float gamma,
                    float emb_range, float modulus, float* scores, int64_t scores_ld, void* stream) {
    int rc = check_fn_mode(fn, mode);
    if (rc) return rc;
    if (B < 0 || N < 0 || D <= 0) return fail(KGE_EINVAL, "bad shape (B, N, D)");
    if (empty(B, mode == KGE_SINGLE ? 1 : N)) return ok();
    if (!scores) return fail(KGE_EINVAL, "scores must not be NULL");
    ScoreParams p;
    fill_dense(p, fn, mode, head, head_ld, rel, rel_ld, rel_off, tail, tail_ld, B, N, D, gamma, emb_range, modulus);
    p.out = scores;
    p.out_ld = scores_ld;
    return run_score(fn, mode, p, KIND_FWD, stream);
}

int kge_score_dense_bwd(int fn, int mode, const float* head, int64_t head_ld, const float* rel, int64_t rel_ld,
                        int64_t rel_off, const float* tail, int64_t tail_ld, int64_t B, int64_t N, int64_t D,
                        float gamma, float emb_range, float modulus, const float* d_scores, int64_t d_ld,
                        float* d_head, float* d_rel, float* d_tail, float* d_modulus, void* stream) {
    int rc = check_fn_mode(fn, mode);
    if (rc) return rc;
    if (B < 0 || N < 0 || D <= 0) return fail(KGE_EINVAL, "bad shape (B, N, D)");
    if (empty(B, mode == KGE_SINGLE ? 1 : N)) return ok();
    if (!d_scores || !d_head || !d_rel || !d_tail) return fail(KGE_EINVAL, "null gradient pointer");
    ScoreParams p;
    fill_dense(p, fn, mode, head, head_ld, rel, rel_ld, rel_off, tail, tail_ld, B, N, D, gamma, emb_range, modulus);
    const bool ch = mode == KGE_HEAD_BATCH;
    p.d_scores = d_scores;
    p.d_ld = d_ld;
    p.d_qent = ch ? d_tail : d_head;
    p.d_cent = ch ? d_head : d_tail;
    p.d_rel = d_rel;
    p.d_modulus = d_modulus;
    return run_score(fn, mode, p, KIND_BWD, stream);
}

int kge_neg_reduce(const float* scores, int64_t B, int64_t N, int64_t ld, float temperature, int adversarial,
                   float* out, void* stream) {
    if (B < 0 || N <= 0) return fail(KGE_EINVAL, "bad shape (B, N)");
    if (B == 0) return ok();
    if (!scores || !out) return fail(KGE_EINVAL, "null pointer");
    const int64_t blocks = (B + kWavesPerBlock - 1) / kWavesPerBlock;
    hipLaunchKernelGGL(neg_reduce_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, (hipStream_t)stream, scores, B, N,
                       ld, temperature, adversarial, out);
    return check_launch("kge_neg_reduce");
}

int kge_neg_reduce_bwd(const float* scores, int64_t B, int64_t N, int64_t ld, float temperature, int adversarial,
                       int detach, const float* d_out, float* d_scores, int64_t d_ld, void* stream) {
    if (B < 0 || N <= 0) return fail(KGE_EINVAL, "bad shape (B, N)");
    if (B == 0) return ok();
    if (!scores || !d_out || !d_scores) return fail(KGE_EINVAL, "null pointer");
    const int64_t blocks = (B + kWavesPerBlock - 1) / kWavesPerBlock;
    hipLaunchKernelGGL(neg_reduce_bwd_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, (hipStream_t)stream, scores,
                       B, N, ld, temperature, adversarial, detach, d_out, d_scores, d_ld, nullptr, nullptr, nullptr);
    return check_launch("kge_neg_reduce_bwd");
}

int kge_log_sigmoid(const float* x, int64_t n, float* out, void* stream) {
    if (n < 0) return fail(KGE_EINVAL, "bad size");
    if (n == 0) return ok();
    if (!x || !out) return fail(KGE_EINVAL, "null pointer");
    hipLaunchKernelGGL(log_sigmoid_kernel, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       (hipStream_t)stream, x, n, out);
    return check_launch("kge_log_sigmoid");
}

int kge_step_loss(const float* out_neg, const float* out_pos, const float* weight, int64_t B, float* loss,
                  float* d_out, void* stream) {
    if (B <= 0) return fail(KGE_EINVAL, "kge_step_loss needs B > 0");
    if (!out_neg || !out_pos || !weight || (!loss && !d_out)) return fail(KGE_EINVAL, "null pointer");
    hipLaunchKernelGGL(step_loss_kernel, dim3(1), dim3(kLossBlock), 0, (hipStream_t)stream, out_neg, out_pos, weight, B,
                       loss, d_out);
    return check_launch("kge_step_loss");
}

int kge_log_sigmoid_bwd(const float* x, const float* d_out, int64_t n, float* d_x, void* stream) {
    if (n < 0) return fail(KGE_EINVAL, "bad size");
    if (n == 0) return ok();
    if (!x || !d_out || !d_x) return fail(KGE_EINVAL, "null pointer");
    hipLaunchKernelGGL(log_sigmoid_bwd_kernel, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       (hipStream_t)stream, x, d_out, n, d_x);
    return check_launch("kge_log_sigmoid_bwd");
}

int kge_adam_update(float* param, float* grad, float* exp_avg, float* exp_avg_sq, int64_t n, float lr, float beta1,
                    float beta2, float eps, int64_t step, int keras, int zero_grad, void* stream) {
    if (n < 0 || step < 1) return fail(KGE_EINVAL, "bad size or step (step is 1-based)");
    if (n == 0) return ok();
    if (!param || !grad || !exp_avg || !exp_avg_sq) return fail(KGE_EINVAL, "null pointer");
    if (!aligned(param, 4) || !aligned(grad, 4) || !aligned(exp_avg, 4) || !aligned(exp_avg_sq, 4))
        return fail(KGE_EINVAL, "adam buffers must be 4-byte aligned fp32");
    const bool vec = aligned(param, 16) && aligned(grad, 16) && aligned(exp_avg, 16) && aligned(exp_avg_sq, 16);
    const double bc1 = 1.0 - std::pow((double)beta1, (double)step);
    const double bc2 = 1.0 - std::pow((double)beta2, (double)step);
    AdamArgs a;
    a.b1 = beta1;
    a.b2 = beta2;
    a.eps = eps;
    a.alpha = (float)((double)lr * std::sqrt(bc2) / bc1);
    a.step_size = (float)((double)lr / bc1);
    a.bc2_sqrt = (float)std::sqrt(bc2);
    a.keras = keras;
    a.zero_grad = zero_grad;
    const int64_t per_block = (int64_t)kBlock * kAdamVec;
    const int64_t want = (n / 4 + per_block - 1) / per_block;
    if (want > INT32_MAX) return fail(KGE_EINVAL, "tensor too large for one launch");
    const int blocks = (int)std::max<int64_t>(1, want);
    if (vec)
        hipLaunchKernelGGL(adam_kernel, dim3(blocks), dim3(kBlock), 0, (hipStream_t)stream, param, grad, exp_avg,
                           exp_avg_sq, n, a);
    else
        hipLaunchKernelGGL(adam_scalar_kernel, dim3((unsigned)std::min<int64_t>(4096, (n + kBlock - 1) / kBlock)),
                           dim3(kBlock), 0, (hipStream_t)stream, param, grad, exp_avg, exp_avg_sq, n, a);
    return check_launch("kge_adam_update");
}

// ---------------------------------------------------------------------------------------------
// Deterministic backward of the fused train step
// ---------------------------------------------------------------------------------------------
struct StepWs {
    float *d_ns, *d_ps, *qbuf, *qg_ent, *qg_rel, *dmod, *dqbuf;
    int *count, *off, *cursor, *code, *tiles;
    int64_t bytes;
};

static int64_t align256(int64_t x) { return (x + 255) & ~(int64_t)255; }

static StepWs step_ws_layout(char* base, int64_t E, int64_t B, int64_t N, int64_t D, int64_t ent_w, int64_t rel_w) {
    StepWs w;
    int64_t o = 0;
    auto take = [&](int64_t bytes) {
        char* p = base ? base + o : nullptr;
        o += align256(bytes);
        return p;
    };
    w.d_ns = (float*)take(B * N * 4);
    w.d_ps = (float*)take(B * 4);
    w.qbuf = (float*)take(2 * B * 3 * D * 4);
    w.qg_ent = (float*)take(2 * B * ent_w * 4);
    w.qg_rel = (float*)take(2 * B * rel_w * 4);
    w.dmod = (float*)take(2 * B * 4);
    w.dqbuf = (float*)take(B * 3 * D * 4);
    w.count = (int*)take(E * 4);
    w.off = (int*)take((E + 1) * 4);
    w.cursor = (int*)take(E * 4);
    w.code = (int*)take((B * N + 3 * B) * 4);
    w.tiles = (int*)take(((E + 1023) / 1024 + 1) * 4);
    w.bytes = o;
    return w;
}

static int64_t ent_width(int fn, int64_t D) { return is_split(fn) ? 2 * D : D; }
static int64_t rel_width(int fn, int64_t D) { return fn == KGE_COMPLEX ? 2 * D : D; }

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
    int rc = check_fn_mode(fn, mode);
    if (rc) return rc;
    if (B < 0 || N < 0 || D <= 0) return fail(KGE_EINVAL, "bad shape (B, N, D)");
    if (empty(B, mode == KGE_SINGLE ? 1 : N)) return ok();
    if (!pos) return fail(KGE_EINVAL, "pos must not be NULL");
    if (mode != KGE_SINGLE && !neg) return fail(KGE_EINVAL, "neg must not be NULL in head/tail-batch mode");
    if (!d_scores || !d_ent || !d_rel) return fail(KGE_EINVAL, "null gradient pointer");
    ScoreParams p;
    fill_indexed(p, fn, mode, ent, nentity, ent_ld, rel, nrelation, rel_ld, rel_off, pos, neg, neg_ld, B, N, D, gamma,
                 emb_range, modulus);
    p.d_scores = d_scores;
    p.d_ld = d_ld;
    p.d_qent = d_ent;
    p.d_cent = d_ent;
    p.d_rel = d_rel;
    p.d_modulus = d_modulus;
    return run_score(fn, mode, p, KIND_BWD, stream);
}

int64_t kge_step_backward_workspace_size(int fn, int64_t nentity, int64_t B, int64_t N, int64_t D) {
    if (fn < KGE_TRANSE || fn > KGE_PROTATE || nentity < 0 || B < 0 || N < 0 || D <= 0) return -1;
    return step_ws_layout(nullptr, nentity, B, N, D, ent_width(fn, D), rel_width(fn, D)).bytes;
}

// Options of the shared backward body. The defaults are kge_step_backward's behaviour.
struct StepOpts {
    bool dq_ready = false;      // phase 1 done by the fused forward: dqbuf holds unscaled query gradients
    bool events_ready = false;  // the entity buckets were built by the caller (e.g. on a side stream)
    bool fused_dscores = false; // the positive score gradient comes out of the neg_reduce_bwd launch
    bool epilogue_done = false; // score gradients and both slots' chains done (KIND_STEP_EPILOGUE)
    float *rel_p = nullptr, *rel_m = nullptr, *rel_v = nullptr;  // Adam on the relation table, fused
};

static EvArgs ev_args(const int64_t* pos, const int64_t* neg, int64_t neg_ld, int64_t B, int64_t N, int64_t E,
                      int mode) {
    EvArgs a;
    a.pos = pos;
    a.neg = neg;
    a.neg_ld = neg_ld;
    a.B = B;
    a.N = N;
    a.E = E;
    a.qcol = mode == KGE_HEAD_BATCH ? 2 : 0;
    a.total = (int)(B * N + 3 * B);
    return a;
}

// bucket the gradient events by entity: count, exclusive scan, scatter (counting sort)
static int launch_events(const EvArgs& a, const StepWs& w, hipStream_t st) {
    if (hipMemsetAsync(w.count, 0, (size_t)(a.E * 4), st) != hipSuccess) return check_launch("memset");
    const unsigned eb = (unsigned)((a.total + kBlock - 1) / kBlock);
    if (a.total > 0) hipLaunchKernelGGL(ev_count_kernel, dim3(eb), dim3(kBlock), 0, st, a, w.count);
    if (a.E > 0)
        hipLaunchKernelGGL(scan_block_kernel, dim3(1), dim3(kScanTile), 0, st, w.count, a.E, w.off, w.cursor, 1,
                           a.total);
    if (a.total > 0) hipLaunchKernelGGL(ev_scatter_kernel, dim3(eb), dim3(kBlock), 0, st, a, w.cursor, w.code);
    return check_launch("kge_step_backward events");
}

static int step_backward_impl(int fn, int mode, const float* ent, int64_t nentity, int64_t ent_ld, const float* rel,
                              int64_t nrelation, int64_t rel_ld, int64_t rel_off, const int64_t* pos,
                              const int64_t* neg, int64_t neg_ld, int64_t B, int64_t N, int64_t D, float gamma,
                              float emb_range, float modulus, float temperature, int adversarial, int detach,
                              const float* neg_scores, int64_t ns_ld, const float* pos_scores, const float* d_out_neg,
                              const float* d_out_pos, float* d_ent, float* d_rel, float* d_modulus,
                              const float* cand_stats, void* workspace, int64_t workspace_bytes, void* stream,
                              const AdamArgs* adam, float* m_ent, float* v_ent, const StepOpts& o = StepOpts()) {
    int rc = check_fn_mode(fn, mode);
    if (rc) return rc;
    if (mode == KGE_SINGLE) return fail(KGE_EINVAL, "kge_step_backward needs a negative mode (0 or 1)");
    if (B < 0 || N <= 0 || D <= 0 || nentity < 0 || nrelation < 0) return fail(KGE_EINVAL, "bad shape");
    if (!ent || !rel || !pos || !neg || !neg_scores || !pos_scores || !d_out_neg || !d_out_pos || !d_rel ||
        (!adam && !d_ent) || (adam && (!m_ent || !v_ent)))
        return fail(KGE_EINVAL, "null pointer");
    if (B * N + 3 * B >= (int64_t)INT32_MAX || nentity >= (int64_t)INT32_MAX)
        return fail(KGE_EINVAL, "too many gradient events for 32-bit codes");
    const int64_t ent_w = ent_width(fn, D), rel_w = rel_width(fn, D);
    const int64_t rel_dim = rel_ld;  // rows are written over their full stride (padding included)
    StepWs w = step_ws_layout((char*)workspace, nentity, B, N, D, ent_w, rel_w);
    if (!workspace || workspace_bytes < w.bytes) return fail(KGE_EINVAL, "workspace too small");
    hipStream_t st = (hipStream_t)stream;
    if (B == 0 && !adam) {
        if (hipMemsetAsync(d_ent, 0, (size_t)(nentity * ent_ld * 4), st) != hipSuccess ||
            hipMemsetAsync(d_rel, 0, (size_t)(nrelation * rel_ld * 4), st) != hipSuccess)
            return check_launch("kge_step_backward memset");
        if (d_modulus && hipMemsetAsync(d_modulus, 0, 4, st) != hipSuccess) return check_launch("memset");
        return ok();
    }
    // 1. loss -> score gradients
    if (o.epilogue_done) {
        rc = 0;
    } else if (o.fused_dscores) {
        const unsigned nb = (unsigned)((B + kWavesPerBlock - 1) / kWavesPerBlock);
        hipLaunchKernelGGL(neg_reduce_bwd_kernel, dim3(nb), dim3(kBlock), 0, st, neg_scores, B, N, ns_ld,
                           temperature, adversarial, detach, d_out_neg, w.d_ns, N, pos_scores, d_out_pos, w.d_ps);
        rc = check_launch("kge_step_backward score gradients");
    } else {
        rc = kge_neg_reduce_bwd(neg_scores, B, N, ns_ld, temperature, adversarial, detach, d_out_neg, w.d_ns, N,
                                stream);
        if (rc) return rc;
        rc = kge_log_sigmoid_bwd(pos_scores, d_out_pos, B, w.d_ps, stream);
    }
    if (rc) return rc;
    // 2. phase 1: per-slot query gradients (negative call, then positive call)
    ScoreParams p;
    fill_indexed(p, fn, mode, ent, nentity, ent_ld, rel, nrelation, rel_ld, rel_off, pos, neg, neg_ld, B, N, D, gamma,
                 emb_range, modulus);
    p.d_scores = w.d_ns;
    p.d_ld = N;
    p.qbuf = w.qbuf;
    p.qg_ent = w.qg_ent;
    p.qg_rel = w.qg_rel;
    p.dmod_part = w.dmod;
    p.ent_w = ent_w;
    p.rel_w = rel_w;
    p.slot0 = 0;
    // streaming form when every wave of the block owns whole column groups (G a multiple of 4) and
    // InterHT's candidate norms are available from the forward; the register-resident form otherwise
    int V1 = 1, G1 = 1;
    rc = pick_vg(p, V1, G1);
    if (rc) return rc;
    if (o.epilogue_done) {
        rc = 0;
    } else if (o.dq_ready) {
        // the fused forward (KIND_STEP_FWD_GRAD) left each row's query gradient, unscaled, in dqbuf
        p.dqbuf = w.dqbuf;
        p.dq_scale = d_out_neg;
        rc = run_score(fn, mode, p, KIND_BWD_CHAIN, stream);
    } else if (G1 >= kWavesPerBlock && G1 % kWavesPerBlock == 0 && G1 <= kMaxG && (fn != KGE_INTERHT || cand_stats)) {
        p.cand_stats = reinterpret_cast<float2*>(const_cast<float*>(cand_stats));
        p.dqbuf = w.dqbuf;
        rc = run_score(fn, mode, p, KIND_BWD_STREAM, stream);
        if (rc) return rc;
        rc = run_score(fn, mode, p, KIND_BWD_CHAIN, stream);
    } else {
        rc = run_score(fn, mode, p, KIND_BWD_ROWS, stream);
    }
    if (rc) return rc;
    ScoreParams pp;
    fill_indexed(pp, fn, KGE_SINGLE, ent, nentity, ent_ld, rel, nrelation, rel_ld, rel_off, pos, nullptr, 0, B, 1, D,
                 gamma, emb_range, modulus);
    pp.d_scores = w.d_ps;
    pp.d_ld = 1;
    pp.qbuf = w.qbuf;
    pp.qg_ent = w.qg_ent;
    pp.qg_rel = w.qg_rel;
    pp.dmod_part = w.dmod;
    pp.ent_w = ent_w;
    pp.rel_w = rel_w;
    pp.slot0 = B;
    if (!o.epilogue_done) {
        rc = run_score(fn, KGE_SINGLE, pp, KIND_BWD_ROWS, stream);
        if (rc) return rc;
    }
    // 3. bucket the gradient events by entity
    if (!o.events_ready) {
        rc = launch_events(ev_args(pos, neg, neg_ld, B, N, nentity, mode), w, st);
        if (rc) return rc;
    }
    // 4. phase 2: one wave per entity row, events in code order -> every row of d_ent written
    ScoreParams q;
    fill_indexed(q, fn, mode, ent, nentity, ent_ld, rel, nrelation, rel_ld, rel_off, pos, neg, neg_ld, B, N, D, gamma,
                 emb_range, modulus);
    q.qbuf = w.qbuf;
    q.qg_ent = w.qg_ent;
    q.ev_off = w.off;
    q.ev_code = w.code;
    q.d_ns = w.d_ns;
    q.d_ps = w.d_ps;
    q.Bn = B;
    q.Nn = N;
    q.ent_w = ent_w;
    q.d_out_ent = d_ent;
    if (adam) {
        q.adam.on = 1;
        q.adam.m = m_ent;
        q.adam.v = v_ent;
        q.adam.b1 = adam->b1;
        q.adam.b2 = adam->b2;
        q.adam.eps = adam->eps;
        q.adam.alpha = adam->alpha;
        q.adam.step_size = adam->step_size;
        q.adam.bc2_sqrt = adam->bc2_sqrt;
        q.adam.keras = adam->keras;
    }
    if (nentity > 0) {
        // streaming form (block per row, waves split the columns) under the same condition as phase 1
        const bool ent_stream = G1 >= kWavesPerBlock && G1 % kWavesPerBlock == 0 && G1 <= kMaxG;
        rc = run_score(fn, mode, q, ent_stream ? KIND_BWD_ENT_STREAM : KIND_BWD_ENT, stream);
        if (rc) return rc;
    }
    // 5. relation rows (slot order) and the pRotatE modulus
    if (nrelation > 0 || d_modulus) {
        const int64_t rb = std::max<int64_t>(1, nrelation * ((rel_dim + kWave - 1) / kWave));
        RelAdam ra;
        memset(&ra, 0, sizeof(ra));
        if (adam && o.rel_p) {
            ra.p = o.rel_p;
            ra.m = o.rel_m;
            ra.v = o.rel_v;
            ra.a = *adam;
            ra.on = 1;
        }
        hipLaunchKernelGGL(bwd_rel_kernel, dim3((unsigned)rb), dim3(kRelWaves * kWave), 0, st, pos, B, nrelation, w.qg_rel, rel_w,
                           rel_off, d_rel, rel_ld, rel_dim, w.dmod, d_modulus, ra);
    }
    return check_launch("kge_step_backward");
}

int kge_step_backward(int fn, int mode, const float* ent, int64_t nentity, int64_t ent_ld, const float* rel,
                      int64_t nrelation, int64_t rel_ld, int64_t rel_off, const int64_t* pos, const int64_t* neg,
                      int64_t neg_ld, int64_t B, int64_t N, int64_t D, float gamma, float emb_range, float modulus,
                      float temperature, int adversarial, int detach, const float* neg_scores, int64_t ns_ld,
                      const float* pos_scores, const float* d_out_neg, const float* d_out_pos, float* d_ent,
                      float* d_rel, float* d_modulus, const float* cand_stats, void* workspace,
                      int64_t workspace_bytes, void* stream) {
    return step_backward_impl(fn, mode, ent, nentity, ent_ld, rel, nrelation, rel_ld, rel_off, pos, neg, neg_ld, B, N,
                              D, gamma, emb_range, modulus, temperature, adversarial, detach, neg_scores, ns_ld,
                              pos_scores, d_out_neg, d_out_pos, d_ent, d_rel, d_modulus, cand_stats, workspace,
                              workspace_bytes, stream, nullptr, nullptr, nullptr);
}

// Adam coefficients of step t (1-based), in double on the host
static AdamArgs adam_args(float lr, float beta1, float beta2, float eps, int64_t step, int keras) {
    const double bc1 = 1.0 - std::pow((double)beta1, (double)step);
    const double bc2 = 1.0 - std::pow((double)beta2, (double)step);
    AdamArgs a;
    a.b1 = beta1;
    a.b2 = beta2;
    a.eps = eps;
    a.alpha = (float)((double)lr * std::sqrt(bc2) / bc1);
    a.step_size = (float)((double)lr / bc1);
    a.bc2_sqrt = (float)std::sqrt(bc2);
    a.keras = keras;
    a.zero_grad = 0;
    return a;
}

int64_t kge_step_backward_adam_workspace_size(int fn, int64_t nentity, int64_t nrelation, int64_t rel_ld, int64_t B,
                                              int64_t N, int64_t D) {
    const int64_t base = kge_step_backward_workspace_size(fn, nentity, B, N, D);
    if (base < 0 || nrelation < 0 || rel_ld < 0) return -1;
    return base + align256(nrelation * rel_ld * 4) + 256;
}

int kge_step_backward_adam(int fn, int mode, float* ent, int64_t nentity, int64_t ent_ld, float* rel,
                           int64_t nrelation, int64_t rel_ld, int64_t rel_off, const int64_t* pos, const int64_t* neg,
                           int64_t neg_ld, int64_t B, int64_t N, int64_t D, float gamma, float emb_range,
                           float* modulus_param, float modulus, float temperature, int adversarial, int detach,
                           const float* neg_scores, int64_t ns_ld, const float* pos_scores, const float* d_out_neg,
                           const float* d_out_pos, float* m_ent, float* v_ent, float* m_rel, float* v_rel,
                           float* m_mod, float* v_mod, float lr, float beta1, float beta2, float eps, int64_t step,
                           int keras, const float* cand_stats, void* workspace, int64_t workspace_bytes,
                           void* stream) {
    if (step < 1) return fail(KGE_EINVAL, "step is 1-based");
    if (!m_rel || !v_rel || (modulus_param && (!m_mod || !v_mod))) return fail(KGE_EINVAL, "null optimizer state");
    const int64_t base = kge_step_backward_workspace_size(fn, nentity, B, N, D);
    if (base < 0) return fail(KGE_EINVAL, "bad shape");
    if (!workspace || workspace_bytes < kge_step_backward_adam_workspace_size(fn, nentity, nrelation, rel_ld, B, N, D))
        return fail(KGE_EINVAL, "workspace too small");
    float* d_rel = (float*)((char*)workspace + base);
    float* d_mod = (float*)((char*)workspace + base + align256(nrelation * rel_ld * 4));
    const AdamArgs a = adam_args(lr, beta1, beta2, eps, step, keras);
    StepOpts o;
    o.rel_p = rel;  // Adam on the relation table inside the relation-gradient kernel
    o.rel_m = m_rel;
    o.rel_v = v_rel;
    int rc = step_backward_impl(fn, mode, ent, nentity, ent_ld, rel, nrelation, rel_ld, rel_off, pos, neg, neg_ld, B,
                                N, D, gamma, emb_range, modulus, temperature, adversarial, detach, neg_scores, ns_ld,
                                pos_scores, d_out_neg, d_out_pos, nullptr, d_rel, modulus_param ? d_mod : nullptr,
                                cand_stats, workspace, base, stream, &a, m_ent, v_ent, o);
    if (rc) return rc;
    // the pRotatE modulus (one element) goes through the dense optimizer kernel, with the same
    // adam_update as the fused rows
    if (modulus_param) {
        rc = kge_adam_update(modulus_param, d_mod, m_mod, v_mod, 1, lr, beta1, beta2, eps, step, keras, 0, stream);
        if (rc) return rc;
    }
    return ok();
}

// ---------------------------------------------------------------------------------------------
// One whole train step (supervisor.py:15-26 train_step_fn): both model calls with phase 1 of the
// backward fused into the forward, the weighted loss and its gradient, the deterministic backward
// with Adam fused into the entity pass, and Adam on the relation table.
// ---------------------------------------------------------------------------------------------
struct TrainWs {
    float *ns, *ps, *d_out, *stats;
    int64_t bwd_bytes, bytes;
};

static TrainWs train_ws_layout(char* base, int fn, int64_t E, int64_t R, int64_t rel_ld, int64_t B, int64_t N,
                               int64_t D) {
    TrainWs t;
    t.bwd_bytes = kge_step_backward_adam_workspace_size(fn, E, R, rel_ld, B, N, D);
    int64_t o = t.bwd_bytes;
    auto take = [&](int64_t bytes) {
        char* p = base ? base + o : nullptr;
        o += align256(bytes);
        return (float*)p;
    };
    t.ns = take(B * N * 4);
    t.ps = take(B * 4);
    t.d_out = take(B * 4);
    t.stats = take(B * N * 8);
    t.bytes = o;
    return t;
}

int64_t kge_train_step_workspace_size(int fn, int64_t nentity, int64_t nrelation, int64_t rel_ld, int64_t B, int64_t N,
                                      int64_t D) {
    if (kge_step_backward_adam_workspace_size(fn, nentity, nrelation, rel_ld, B, N, D) < 0) return -1;
    return train_ws_layout(nullptr, fn, nentity, nrelation, rel_ld, B, N, D).bytes;
}

int kge_train_step(int fn, int mode, float* ent, int64_t nentity, int64_t ent_ld, float* rel, int64_t nrelation,
                   int64_t rel_ld, int64_t rel_off, const int64_t* pos, const int64_t* neg, int64_t neg_ld, int64_t B,
                   int64_t N, int64_t D, float gamma, float emb_range, float temperature, int adversarial, int detach,
                   const float* weight, float* loss, float* loss_sum, float* out_neg, float* out_pos,
                   float* m_ent, float* v_ent, float* m_rel, float* v_rel, float lr, float beta1, float beta2,
                   float eps, int64_t step, int keras, void* workspace, int64_t workspace_bytes, void* stream) {
    int rc = check_fn_mode(fn, mode);
    if (rc) return rc;
    if (fn == KGE_PROTATE) return fail(KGE_ENOTSUP, "kge_train_step: pRotatE uses kge_step_backward_adam");
    if (mode == KGE_SINGLE) return fail(KGE_EINVAL, "kge_train_step needs a negative mode (0 or 1)");
    if (B <= 0 || N <= 0 || D <= 0 || nentity < 0 || nrelation < 0) return fail(KGE_EINVAL, "bad shape");
    if (step < 1) return fail(KGE_EINVAL, "step is 1-based");
    if (!ent || !rel || !pos || !neg || !weight || !loss || !out_neg || !out_pos || !m_ent || !v_ent || !m_rel ||
        !v_rel)
        return fail(KGE_EINVAL, "null pointer");
    if (B * N + 3 * B >= (int64_t)INT32_MAX || nentity >= (int64_t)INT32_MAX)
        return fail(KGE_EINVAL, "too many gradient events for 32-bit codes");
    const TrainWs t = train_ws_layout((char*)workspace, fn, nentity, nrelation, rel_ld, B, N, D);
    if (!workspace || workspace_bytes < t.bytes) return fail(KGE_EINVAL, "workspace too small");
    const int64_t base = kge_step_backward_workspace_size(fn, nentity, B, N, D);
    const StepWs w = step_ws_layout((char*)workspace, nentity, B, N, D, ent_width(fn, D), rel_width(fn, D));
    float* d_rel = (float*)((char*)workspace + base);
    hipStream_t st = (hipStream_t)stream;
    StepOpts o;
    o.fused_dscores = true;
    o.events_ready = true;
    o.rel_p = rel;
    o.rel_m = m_rel;
    o.rel_v = v_rel;

    // 1. forward of both model calls (supervisor.py:17-18); phase 1 of the backward fused in where its
    //    accumulators fit, and the gradient events counted into their entity buckets
    ScoreParams p;
    fill_indexed(p, fn, mode, ent, nentity, ent_ld, rel, nrelation, rel_ld, rel_off, pos, neg, neg_ld, B, N, D, gamma,
                 emb_range, 0.f);
    p.out = t.ns;
    p.out_ld = N;
    p.pos_base = pos;
    p.temperature = temperature;
    p.adversarial = adversarial;
    p.detach = detach;
    p.out_neg = out_neg;
    p.out_pos_raw = t.ps;
    p.out_pos_ls = out_pos;
    p.dqbuf = w.dqbuf;
    int V = 1, G = 1;
    rc = pick_vg(p, V, G);
    if (rc) return rc;
    const AdamArgs a = adam_args(lr, beta1, beta2, eps, step, keras);
    if (G > kFwdGradMaxG) {
        // fallback (D > 1024): the step forward, the loss kernel, then the backward with its own phase 1
        o.events_ready = false;
        p.cand_stats = reinterpret_cast<float2*>(t.stats);
        rc = run_score(fn, mode, p, fn == KGE_INTERHT ? KIND_STEP_FWD_STATS : KIND_STEP_FWD, stream);
        if (rc) return rc;
        hipLaunchKernelGGL(step_loss_kernel, dim3(1), dim3(kLossBlock), 0, st, out_neg, out_pos, weight, B, loss,
                           t.d_out);
        if (loss_sum) hipLaunchKernelGGL(add_scalar_kernel, dim3(1), dim3(1), 0, st, loss, loss_sum);
        rc = check_launch("kge_train_step loss");
        if (rc) return rc;
        return step_backward_impl(fn, mode, ent, nentity, ent_ld, rel, nrelation, rel_ld, rel_off, pos, neg, neg_ld, B,
                                  N, D, gamma, emb_range, 0.f, temperature, adversarial, detach, t.ns, N, t.ps,
                                  t.d_out, t.d_out, nullptr, d_rel, nullptr, t.stats, workspace, base, stream, &a,
                                  m_ent, v_ent, o);
    }
    // the per-entity event counters are zeroed here, on every call: the workspace carries no state
    // between calls, so any workspace contents (fresh, shared, or left by an aborted call) are valid. The
    // size is rounded up inside the 256-B aligned region: an unaligned tail costs the runtime a second
    // fill kernel (~3-5 us on the step's critical path)
    if (nentity > 0 && hipMemsetAsync(w.count, 0, (size_t)align256(nentity * 4), st) != hipSuccess)
        return check_launch("kge_train_step memset");
    p.ev_count = w.count;
    rc = run_score(fn, mode, p, KIND_STEP_FWD_GRAD, stream);
    if (rc) return rc;
    // 2. bucket offsets (one launch): every 4096-entity tile scanned at once, the tiles' prefix added by the
    //    epilogue; one block walking all tiles for tables of more than 4M entities
    const int64_t ntiles = (nentity + kTile4k - 1) / kTile4k;
    const bool tiled = nentity > 0 && ntiles <= kEvMaxTiles;
    if (tiled)
        hipLaunchKernelGGL(scan_tiles4k_kernel, dim3((unsigned)ntiles), dim3(kScanTile), 0, st, w.count, nentity, w.off,
                           w.cursor, w.tiles);
    else
        hipLaunchKernelGGL(scan_block_kernel, dim3(1), dim3(kScanTile), 0, st, w.count, nentity, w.off, w.cursor, 0,
                           (int)(B * N + 3 * B));
    rc = check_launch("kge_train_step scan");
    if (rc) return rc;
    // 3. one launch: event scatter, loss weights, score gradients, both slots' query chains, the loss
    ScoreParams e = p;
    e.ev_count = nullptr;
    e.neg_scores = t.ns;
    e.ns_ld = N;
    e.d_ns = w.d_ns;
    e.d_ps = w.d_ps;
    e.qbuf = w.qbuf;
    e.qg_ent = w.qg_ent;
    e.qg_rel = w.qg_rel;
    e.ent_w = ent_width(fn, D);
    e.rel_w = rel_width(fn, D);
    e.weight = weight;
    e.pos_raw = t.ps;
    e.loss = loss;
    e.loss_sum = loss_sum;
    e.ev_cursor = w.cursor;
    e.ev_code_w = w.code;
    if (tiled) {
        e.ev_tile_sum = w.tiles;
        e.ev_off_fix = w.off;
        e.ev_ntiles = (int)ntiles;
    }
    rc = run_score(fn, mode, e, KIND_STEP_EPILOGUE, stream);
    if (rc) return rc;
    // 4. phase 2 with Adam fused into the entity pass, relation gradient with Adam (supervisor.py:25-26)
    o.dq_ready = o.epilogue_done = true;
    return step_backward_impl(fn, mode, ent, nentity, ent_ld, rel, nrelation, rel_ld, rel_off, pos, neg, neg_ld, B, N,
                              D, gamma, emb_range, 0.f, temperature, adversarial, detach, t.ns, N, t.ps, t.d_out,
                              t.d_out, nullptr, d_rel, nullptr, nullptr, workspace, base, stream, &a, m_ent, v_ent, o);
}

}  // extern "C"

// ---------------------------------------------------------------------------------------------
// Row-sharded train step (owner-computes; kge_shard.h): supervisor.py:15-26 over the
// W replicas' batches, the entity table row-sharded over the W ranks, in three calls with the
// caller's two collectives between them.
// ---------------------------------------------------------------------------------------------
struct ShardWs {
    StepWs step;
    float *d_rel, *ns, *A, *Bv, *merged;
    int64_t base, bytes;
};

static ShardWs shard_ws_layout(char* ws, int fn, int64_t rows, int64_t R, int64_t rel_ld, int64_t Bg, int64_t N,
                               int64_t D) {
    ShardWs s;
    s.step = step_ws_layout(ws, rows, Bg, N, D, ent_width(fn, D), rel_width(fn, D));
    s.base = s.step.bytes;
    int64_t o = kge_step_backward_adam_workspace_size(fn, rows, R, rel_ld, Bg, N, D);
    s.d_rel = ws ? (float*)(ws + s.base) : nullptr;
    auto take = [&](int64_t bytes) {
        char* q = ws ? ws + o : nullptr;
        o += align256(bytes);
        return (float*)q;
    };
    const int64_t nqd = (int64_t)shard_nq(fn) * D;
    s.ns = take(Bg * N * 4);
    s.A = take(Bg * nqd * 4);
    s.Bv = take(Bg * nqd * 4);
    s.merged = take(Bg * 4 * 4);
    s.bytes = o;
    return s;
}

static int shard_check(int fn, int mode, const float* shard, int64_t rows, const float* qent, const float* qent_pos,
                       const float* rel, const int64_t* pos, const int64_t* neg, int64_t Bg, int64_t N, int64_t D,
                       int64_t home_B, int world, int rank, const float* weight, void* ws, int64_t ws_bytes) {
    int rc = check_fn_mode(fn, mode);
    if (rc) return rc;
    if (fn == KGE_PROTATE) return fail(KGE_ENOTSUP, "the sharded train step has no pRotatE modulus gradient");
    if (mode == KGE_SINGLE) return fail(KGE_EINVAL, "the sharded train step needs a negative mode (0 or 1)");
    if (Bg <= 0 || N <= 0 || D <= 0 || rows < 0 || world < 1 || rank < 0 || rank >= world || home_B <= 0 ||
        home_B * world != Bg)
        return fail(KGE_EINVAL, "bad shape: need Bg = world * home_B > 0, N, D > 0, 0 <= rank < world");
    if (!shard || !qent || !qent_pos || !rel || !pos || !neg || !weight) return fail(KGE_EINVAL, "null pointer");
    if (Bg * N + 3 * Bg >= (int64_t)INT32_MAX || rows >= (int64_t)INT32_MAX)
        return fail(KGE_EINVAL, "too many gradient events for 32-bit codes");
    if (!ws || ws_bytes < shard_ws_layout(nullptr, fn, rows, 0, 0, Bg, N, D).bytes) return fail(KGE_EINVAL, "workspace too small");
    return 0;
}

static void shard_params(ScoreParams& p, int fn, int mode, const float* shard, int64_t rows, int64_t ent_ld,
                         int64_t shard_lo, const float* qent, const float* qent_pos, int64_t q_ld, const float* rel,
                         int64_t nrelation, int64_t rel_ld, int64_t rel_off, const int64_t* pos, const int64_t* neg,
                         int64_t neg_ld, int64_t Bg, int64_t N, int64_t D, int64_t home_B, int world, int rank,
                         float gamma, float emb_range, float temperature, int adversarial, int detach,
                         const float* weight, const ShardWs& w) {
    fill_indexed(p, fn, mode, shard, rows, ent_ld, rel, nrelation, rel_ld, rel_off, pos, neg, neg_ld, Bg, N, D, gamma,
                 emb_range, 0.f);
    p.qent = qent;  // row b: the negative call's query entity (assembled by the caller)
    p.q_idx = nullptr;
    p.q_ld = q_ld;
    p.q_rows = Bg;
    p.qent_pos = qent_pos;
    p.c_base = shard_lo;
    p.pos_base = pos;
    p.temperature = temperature;
    p.adversarial = adversarial;
    p.detach = detach;
    p.weight = weight;
    p.home_B = home_B;
    p.world = world;
    p.rank = rank;
    p.nq = shard_nq(fn);
    p.out = w.ns;
    p.out_ld = N;
    p.neg_scores = w.ns;
    p.ns_ld = N;
    p.d_ns = w.step.d_ns;
    p.d_ps = w.step.d_ps;
    p.sh_A = w.A;
    p.sh_B = w.Bv;
    p.sh_merged = w.merged;
}

extern "C" {

int kge_shard_nq(int fn) { return (fn < KGE_TRANSE || fn > KGE_PROTATE) ? 0 : shard_nq(fn); }

int64_t kge_shard_train_workspace_size(int fn, int64_t shard_rows, int64_t nrelation, int64_t rel_ld, int64_t Bg,
                                       int64_t N, int64_t D) {
    if (fn < KGE_TRANSE || fn > KGE_PROTATE || shard_rows < 0 || nrelation < 0 || rel_ld < 0 || Bg < 0 || N < 0 ||
        D <= 0)
        return -1;
    return shard_ws_layout(nullptr, fn, shard_rows, nrelation, rel_ld, Bg, N, D).bytes;
}

int kge_shard_train_forward(int fn, int mode, const float* shard, int64_t shard_rows, int64_t ent_ld, int64_t shard_lo,
                            const float* qent, const float* qent_pos, int64_t q_ld, const float* rel, int64_t nrelation,
                            int64_t rel_ld, int64_t rel_off, const int64_t* pos, const int64_t* neg, int64_t neg_ld,
                            int64_t Bg, int64_t N, int64_t D, int64_t home_B, int world, int rank, float gamma,
                            float emb_range, float temperature, int adversarial, int detach, const float* weight,
                            float* stats, float* dq, void* workspace, int64_t workspace_bytes, void* stream) {
    int rc = shard_check(fn, mode, shard, shard_rows, qent, qent_pos, rel, pos, neg, Bg, N, D, home_B, world, rank,
                         weight, workspace, workspace_bytes);
    if (rc) return rc;
    if (!stats || !dq) return fail(KGE_EINVAL, "null pointer");
    const ShardWs w = shard_ws_layout((char*)workspace, fn, shard_rows, nrelation, rel_ld, Bg, N, D);
    if (workspace_bytes < w.bytes) return fail(KGE_EINVAL, "workspace too small");
    hipStream_t st = (hipStream_t)stream;
    // per-call state only: the local rows' event counters are zeroed here
    if (shard_rows > 0 && hipMemsetAsync(w.step.count, 0, (size_t)align256(shard_rows * 4), st) != hipSuccess)
        return check_launch("kge_shard_train_forward memset");
    ScoreParams p;
    shard_params(p, fn, mode, shard, shard_rows, ent_ld, shard_lo, qent, qent_pos, q_ld, rel, nrelation, rel_ld,
                 rel_off, pos, neg, neg_ld, Bg, N, D, home_B, world, rank, gamma, emb_range, temperature, adversarial,
                 detach, weight, w);
    p.ev_count = w.step.count;
    p.sh_stats = stats;
    p.sh_dq = dq;
    rc = run_score(fn, mode, p, KIND_SHARD_FWD_GRAD, stream);
    if (rc) return rc;
    p.ev_count = nullptr;
    return run_score(fn, KGE_TAIL_BATCH, p, KIND_SHARD_POS, stream);  // owned positives (tail formula)
}

int kge_shard_train_combine(int fn, int mode, const float* shard, int64_t shard_rows, int64_t ent_ld, int64_t shard_lo,
                            const float* qent, const float* qent_pos, int64_t q_ld, const float* rel, int64_t nrelation,
                            int64_t rel_ld, int64_t rel_off, const int64_t* pos, const int64_t* neg, int64_t neg_ld,
                            int64_t Bg, int64_t N, int64_t D, int64_t home_B, int world, int rank, float gamma,
                            float emb_range, float temperature, int adversarial, int detach, const float* weight,
                            const float* stats_all, float* dq, float* out_neg, float* out_pos_raw, float* out_pos,
                            void* workspace, int64_t workspace_bytes, void* stream) {
    int rc = shard_check(fn, mode, shard, shard_rows, qent, qent_pos, rel, pos, neg, Bg, N, D, home_B, world, rank,
                         weight, workspace, workspace_bytes);
    if (rc) return rc;
    if (!stats_all || !dq || !out_neg || !out_pos) return fail(KGE_EINVAL, "null pointer");
    const ShardWs w = shard_ws_layout((char*)workspace, fn, shard_rows, nrelation, rel_ld, Bg, N, D);
    if (workspace_bytes < w.bytes) return fail(KGE_EINVAL, "workspace too small");
    ScoreParams p;
    shard_params(p, fn, mode, shard, shard_rows, ent_ld, shard_lo, qent, qent_pos, q_ld, rel, nrelation, rel_ld,
                 rel_off, pos, neg, neg_ld, Bg, N, D, home_B, world, rank, gamma, emb_range, temperature, adversarial,
                 detach, weight, w);
    p.sh_stats_all = stats_all;
    p.sh_dq = dq;
    p.out_neg = out_neg;
    p.out_pos_raw = out_pos_raw;
    p.out_pos_ls = out_pos;
    const int64_t blocks = (Bg + kWavesPerBlock - 1) / kWavesPerBlock;
    hipLaunchKernelGGL(shard_combine_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, (hipStream_t)stream, p);
    return check_launch("kge_shard_train_combine");
}

int kge_shard_train_backward(int fn, int mode, float* shard, int64_t shard_rows, int64_t ent_ld, int64_t shard_lo,
                             const float* qent, const float* qent_pos, int64_t q_ld, float* rel, int64_t nrelation,
                             int64_t rel_ld, int64_t rel_off, const int64_t* pos, const int64_t* neg, int64_t neg_ld,
                             int64_t Bg, int64_t N, int64_t D, int64_t home_B, int world, int rank, float gamma,
                             float emb_range, float temperature, int adversarial, int detach, const float* weight,
                             const float* dq, float* loss, float* loss_sum, float* m_ent, float* v_ent, float* m_rel,
                             float* v_rel, float lr, float beta1, float beta2, float eps, int64_t step, int keras,
                             void* workspace, int64_t workspace_bytes, void* stream) {
    int rc = shard_check(fn, mode, shard, shard_rows, qent, qent_pos, rel, pos, neg, Bg, N, D, home_B, world, rank,
                         weight, workspace, workspace_bytes);
    if (rc) return rc;
    if (step < 1) return fail(KGE_EINVAL, "step is 1-based");
    if (!dq || !loss || !m_ent || !v_ent || !m_rel || !v_rel) return fail(KGE_EINVAL, "null pointer");
    const ShardWs w = shard_ws_layout((char*)workspace, fn, shard_rows, nrelation, rel_ld, Bg, N, D);
    if (workspace_bytes < w.bytes) return fail(KGE_EINVAL, "workspace too small");
    hipStream_t st = (hipStream_t)stream;
    // bucket offsets of the owned rows' events (counted by the forward)
    if (shard_rows > 0)
        hipLaunchKernelGGL(scan_block_kernel, dim3(1), dim3(kScanTile), 0, st, w.step.count, shard_rows, w.step.off,
                           w.step.cursor, 0, (int)(Bg * N + 3 * Bg));
    rc = check_launch("kge_shard_train_backward scan");
    if (rc) return rc;
    ScoreParams e;
    shard_params(e, fn, mode, shard, shard_rows, ent_ld, shard_lo, qent, qent_pos, q_ld, rel, nrelation, rel_ld,
                 rel_off, pos, neg, neg_ld, Bg, N, D, home_B, world, rank, gamma, emb_range, temperature, adversarial,
                 detach, weight, w);
    e.sh_dq = const_cast<float*>(dq);
    e.qbuf = w.step.qbuf;
    e.qg_ent = w.step.qg_ent;
    e.qg_rel = w.step.qg_rel;
    e.ent_w = ent_width(fn, D);
    e.rel_w = rel_width(fn, D);
    e.loss = loss;
    e.loss_sum = loss_sum;
    e.ev_cursor = w.step.cursor;
    e.ev_code_w = w.step.code;
    rc = run_score(fn, mode, e, KIND_SHARD_EPILOGUE, stream);
    if (rc) return rc;
    // phase 2 with Adam fused into the shard's rows, relation gradient with Adam (supervisor.py:25-26)
    const AdamArgs a = adam_args(lr, beta1, beta2, eps, step, keras);
    StepOpts o;
    o.dq_ready = o.epilogue_done = o.events_ready = true;
    o.rel_p = rel;
    o.rel_m = m_rel;
    o.rel_v = v_rel;
    return step_backward_impl(fn, mode, shard, shard_rows, ent_ld, rel, nrelation, rel_ld, rel_off, pos, neg, neg_ld,
                              Bg, N, D, gamma, emb_range, 0.f, temperature, adversarial, detach, w.ns, N, w.ns,
                              w.step.d_ps, w.step.d_ps, nullptr, w.d_rel, nullptr, nullptr, workspace, w.base, stream,
                              &a, m_ent, v_ent, o);
}

}  // extern "C"
