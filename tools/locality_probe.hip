// locality_probe.hip — does the order of the candidate gathers change the memory-system ceiling of the
// scoring kernel (C2: 131 072 random 8 000-B rows of a 327 MB table per launch, row reuse ~3.2x)?
//
// Every variant gathers exactly the same (batch row, candidate) pairs with trivial compute; only the
// assignment of candidates to waves and their order inside a wave change:
//   rowmajor        wave = (batch row, quarter of its candidates), candidate order   (= step_fwd_kernel)
//   rowmajor-sorted same waves, each wave's 64 ids ascending
//   xcd             wave = (batch row, entity slice x of E/8 ids); block i holds 4 batch rows of slice
//                   x = i % 8, so every gather of an entity row is issued by the same XCD (blocks b and
//                   b + 8 share an XCD), ids in candidate order
//   xcd-sorted      the same, ids ascending: the XCD's waves sweep their slice together, so the repeat
//                   gathers of a row land close in time (L2 / Infinity Cache hits)
// Build: hipcc --offload-arch=gfx950 -O3 -o locality_probe locality_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

using rsrc_t = __amdgpu_buffer_rsrc_t;
__device__ __forceinline__ rsrc_t make_rsrc(const void* base, uint32_t bytes) {
    const uint64_t a = (uint64_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0,
                                             (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

constexpr int G = 8;  // float4 groups per lane: 2000 floats = 500 float4 (last group partial, range-checked)
struct Row {
    float a[G][4];
};

__device__ __forceinline__ void load_row(Row& r, const float* base, int lane, uint32_t bytes) {
    const rsrc_t s = make_rsrc(base, bytes);
#pragma unroll
    for (int k = 0; k < G; ++k) {
        const auto u = __builtin_amdgcn_raw_buffer_load_b128(s, (uint32_t)((lane + 64 * k) * 16), 0, 0);
        r.a[k][0] = __uint_as_float(u[0]);
        r.a[k][1] = __uint_as_float(u[1]);
        r.a[k][2] = __uint_as_float(u[2]);
        r.a[k][3] = __uint_as_float(u[3]);
    }
}

__device__ __forceinline__ float row_sum(const Row& r) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < G; ++k) s += (r.a[k][0] + r.a[k][1]) + (r.a[k][2] + r.a[k][3]);
    return s;
}

// wave gw gathers list wl[gw] = ids[off[l], off[l+1]) in runs of 64, two rows in flight
__global__ __launch_bounds__(256) void gather_lists(const float* __restrict__ tab, int64_t rowf, uint32_t row_bytes,
                                                    const int* __restrict__ off, const int* __restrict__ ids,
                                                    const int* __restrict__ wl, int nw, float* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (gw >= nw) return;
    const int l = wl[gw];
    if (l < 0) return;
    const int lo = off[l], hi = off[l + 1];
    for (int c0 = lo; c0 < hi; c0 += 64) {
        const int nc = min(64, hi - c0);
        const int my = lane < nc ? ids[c0 + lane] : 0;
        Row r0, r1;
        float mine = 0.f;
        load_row(r0, tab + (int64_t)__builtin_amdgcn_readlane(my, 0) * rowf, lane, row_bytes);
        int j = 0;
        for (; j + 2 < nc; j += 2) {
            load_row(r1, tab + (int64_t)__builtin_amdgcn_readlane(my, j + 1) * rowf, lane, row_bytes);
            float s = row_sum(r0);
            if (lane == j) mine = s;
            load_row(r0, tab + (int64_t)__builtin_amdgcn_readlane(my, j + 2) * rowf, lane, row_bytes);
            s = row_sum(r1);
            if (lane == j + 1) mine = s;
        }
        if (j + 1 < nc) {
            load_row(r1, tab + (int64_t)__builtin_amdgcn_readlane(my, j + 1) * rowf, lane, row_bytes);
            float s = row_sum(r0);
            if (lane == j) mine = s;
            s = row_sum(r1);
            if (lane == j + 1) mine = s;
        } else {
            const float s = row_sum(r0);
            if (lane == j) mine = s;
        }
        if (lane < nc) out[c0 + lane] = mine;
    }
}


// entity-major: wave gw walks the (entity, batch row) pairs of list wl[gw] (sorted by entity): an entity
// row is loaded once per run of equal entities and kept in registers; every pair also loads its batch
// row's query (q0, q1: 2 x HALF floats of qbuf [B, 2 HALF]) and relation row (rel [11, HALF]) — the
// operands an entity-major InterHT score reads. Two pairs in flight.
constexpr int GH = 4;  // float4 groups per lane per half row (HALF = 1000 floats = 250 float4)
struct Half {
    float a[GH][4];
};
__device__ __forceinline__ void load_half(Half& r, const float* base, int lane, uint32_t bytes) {
    const rsrc_t s = make_rsrc(base, bytes);
#pragma unroll
    for (int k = 0; k < GH; ++k) {
        const auto u = __builtin_amdgcn_raw_buffer_load_b128(s, (uint32_t)((lane + 64 * k) * 16), 0, 0);
        r.a[k][0] = __uint_as_float(u[0]);
        r.a[k][1] = __uint_as_float(u[1]);
        r.a[k][2] = __uint_as_float(u[2]);
        r.a[k][3] = __uint_as_float(u[3]);
    }
}
struct Pair {
    Half ea, eb, q0, q1, q2;
};
__device__ __forceinline__ float pair_score(const Pair& p) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < GH; ++k)
#pragma unroll
        for (int i = 0; i < 4; ++i) s += fabsf(p.q0.a[k][i] * p.eb.a[k][i] - p.ea.a[k][i] * p.q1.a[k][i] + p.q2.a[k][i]);
    return s;
}
__global__ __launch_bounds__(256) void gather_pairs(const float* __restrict__ tab, const float* __restrict__ qbuf,
                                                    const float* __restrict__ rel, const int* __restrict__ off,
                                                    const int* __restrict__ pe, const int* __restrict__ pb,
                                                    const int* __restrict__ wl, int nw, float* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (gw >= nw) return;
    const int l = wl[gw];
    if (l < 0) return;
    const int lo = off[l], hi = off[l + 1];
    const uint32_t hb = 1000 * 4;
    for (int c0 = lo; c0 < hi; c0 += 64) {
        const int nc = min(64, hi - c0);
        const int my_e = lane < nc ? pe[c0 + lane] : 0, my_b = lane < nc ? pb[c0 + lane] : 0;
        float mine = 0.f;
        Pair cur, nxt;
        int e = __builtin_amdgcn_readlane(my_e, 0), b = __builtin_amdgcn_readlane(my_b, 0);
        load_half(cur.ea, tab + (int64_t)e * 2000, lane, hb);
        load_half(cur.eb, tab + (int64_t)e * 2000 + 1000, lane, hb);
        load_half(cur.q0, qbuf + (int64_t)b * 2000, lane, hb);
        load_half(cur.q1, qbuf + (int64_t)b * 2000 + 1000, lane, hb);
        load_half(cur.q2, rel + (int64_t)(b % 11) * 1000, lane, hb);
        for (int j = 0; j < nc; ++j) {
            if (j + 1 < nc) {
                const int e1 = __builtin_amdgcn_readlane(my_e, j + 1), b1 = __builtin_amdgcn_readlane(my_b, j + 1);
                if (e1 != e) {
                    load_half(nxt.ea, tab + (int64_t)e1 * 2000, lane, hb);
                    load_half(nxt.eb, tab + (int64_t)e1 * 2000 + 1000, lane, hb);
                } else {
                    nxt.ea = cur.ea;
                    nxt.eb = cur.eb;
                }
                load_half(nxt.q0, qbuf + (int64_t)b1 * 2000, lane, hb);
                load_half(nxt.q1, qbuf + (int64_t)b1 * 2000 + 1000, lane, hb);
                load_half(nxt.q2, rel + (int64_t)(b1 % 11) * 1000, lane, hb);
                e = e1;
            }
            float s = pair_score(cur);
            s += __shfl_xor(s, 1);
            if (lane == j) mine = s;
            cur = nxt;
        }
        if (lane < nc) out[c0 + lane] = mine;
    }
}

// row-group tiles: block = (group of R batch rows, entity slice x = blockIdx % 8). The R rows' queries (q0, q1:
// 2 x 1000 floats each) are staged once into LDS; the block's (entity, row) pairs, sorted by entity, are dealt
// round-robin to its NWV waves, so the block sweeps its slice in one ascending front and the slice's 32 blocks
// on one XCD sweep it together. Per pair: the candidate row from global (8 KB), the query from LDS (8 KB), the
// relation third from a small global table (L2-resident).
template <int R, int NWV, int DEPTH, bool Q2LDS = false>
__global__ __launch_bounds__(NWV * 64) void tile_pairs(const float* __restrict__ tab, const float* __restrict__ qbuf,
                                                       const float* __restrict__ rel, const int* __restrict__ off,
                                                       const int* __restrict__ pe, const int* __restrict__ pb,
                                                       float* __restrict__ out) {
    __shared__ float4 q[R][2][64 * GH];
    __shared__ float4 q2s[Q2LDS ? 3 : 1][64 * GH];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int blk = blockIdx.x, grp = blk / 8;
    for (int i = t; i < R * 2 * 64 * GH; i += NWV * 64) {
        const int r = i / (2 * 64 * GH), j = i % (2 * 64 * GH), hf = j / (64 * GH), k = j % (64 * GH);
        q[r][hf][k] = k < 250 ? reinterpret_cast<const float4*>(qbuf)[(int64_t)(grp * R + r) * 500 + hf * 250 + k]
                              : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if constexpr (Q2LDS)
        for (int i = t; i < 3 * 64 * GH; i += NWV * 64) {
            const int sl = i / (64 * GH), k = i % (64 * GH);
            q2s[sl][k] = k < 250 ? reinterpret_cast<const float4*>(rel)[sl * 250 + k] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    __syncthreads();
    const int lo = off[blk], hi = off[blk + 1];
    const uint32_t hb = 1000 * 4;
    auto score = [&](const Half& ea, const Half& eb, int b) {
        Half q2;
        if constexpr (Q2LDS) {
#pragma unroll
            for (int k = 0; k < GH; ++k) {
                const float4 v = q2s[b % 3][lane + 64 * k];
                q2.a[k][0] = v.x;
                q2.a[k][1] = v.y;
                q2.a[k][2] = v.z;
                q2.a[k][3] = v.w;
            }
        } else {
            load_half(q2, rel + (int64_t)((grp * R + b) % 11) * 1000, lane, hb);
        }
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < GH; ++k) {
            const float4 a = q[b][0][lane + 64 * k], c = q[b][1][lane + 64 * k];
            s += fabsf(a.x * eb.a[k][0] - ea.a[k][0] * c.x + q2.a[k][0]);
            s += fabsf(a.y * eb.a[k][1] - ea.a[k][1] * c.y + q2.a[k][1]);
            s += fabsf(a.z * eb.a[k][2] - ea.a[k][2] * c.z + q2.a[k][2]);
            s += fabsf(a.w * eb.a[k][3] - ea.a[k][3] * c.w + q2.a[k][3]);
        }
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
        return s;
    };
    for (int c0 = lo + wave; c0 < hi; c0 += NWV * 64) {
        const int nc = min(64, (hi - c0 + NWV - 1) / NWV);
        const int my = c0 + NWV * lane;
        const int my_e = lane < nc ? pe[my] : 0, my_b = lane < nc ? pb[my] : 0;
        float mine = 0.f;
        if constexpr (DEPTH == 1) {
            for (int j = 0; j < nc; ++j) {
                Half ea, eb;
                const int e = __builtin_amdgcn_readlane(my_e, j), b = __builtin_amdgcn_readlane(my_b, j);
                load_half(ea, tab + (int64_t)e * 2000, lane, hb);
                load_half(eb, tab + (int64_t)e * 2000 + 1000, lane, hb);
                const float s = score(ea, eb, b);
                if (lane == j) mine = s;
            }
        } else {
            Half a0, b0, a1, b1;
            int e = __builtin_amdgcn_readlane(my_e, 0);
            load_half(a0, tab + (int64_t)e * 2000, lane, hb);
            load_half(b0, tab + (int64_t)e * 2000 + 1000, lane, hb);
            for (int j = 0; j < nc; j += 2) {
                if (j + 1 < nc) {
                    e = __builtin_amdgcn_readlane(my_e, j + 1);
                    load_half(a1, tab + (int64_t)e * 2000, lane, hb);
                    load_half(b1, tab + (int64_t)e * 2000 + 1000, lane, hb);
                }
                float s = score(a0, b0, __builtin_amdgcn_readlane(my_b, j));
                if (lane == j) mine = s;
                if (j + 1 < nc) {
                    if (j + 2 < nc) {
                        e = __builtin_amdgcn_readlane(my_e, j + 2);
                        load_half(a0, tab + (int64_t)e * 2000, lane, hb);
                        load_half(b0, tab + (int64_t)e * 2000 + 1000, lane, hb);
                    }
                    s = score(a1, b1, __builtin_amdgcn_readlane(my_b, j + 1));
                    if (lane == j + 1) mine = s;
                }
            }
        }
        if (lane < nc) out[my] = mine;
    }
}

// tile_pairs with the XCD's waves paced together: the block's sorted pairs are cut into NG entity groups
// (group g: entities [g S / NG, (g + 1) S / NG) of the slice); a wave starts group g only when every wave of
// its XCD has finished group g - L - 1 (per-(XCD, group) counters, agent-scope atomics; the wait is bounded,
// so pacing never deadlocks, it only bounds the spread of the fronts to L + 1 groups). Counters accumulate
// over launches: launch `epoch` (0-based) waits for nwx * (epoch + 1).
template <int R, int NWV, int NG, int L>
__global__ __launch_bounds__(NWV * 64) void tile_pairs_sync(const float* __restrict__ tab,
                                                            const float* __restrict__ qbuf,
                                                            const float* __restrict__ rel, const int* __restrict__ goff,
                                                            const int* __restrict__ pe, const int* __restrict__ pb,
                                                            float* __restrict__ out, int* sync, int nwx, int epoch) {
    __shared__ float4 q[R][2][64 * GH];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int blk = blockIdx.x, grp = blk / 8, x = blk % 8;
    for (int i = t; i < R * 2 * 64 * GH; i += NWV * 64) {
        const int r = i / (2 * 64 * GH), j = i % (2 * 64 * GH), hf = j / (64 * GH), k = j % (64 * GH);
        q[r][hf][k] = k < 250 ? reinterpret_cast<const float4*>(qbuf)[(int64_t)(grp * R + r) * 500 + hf * 250 + k]
                              : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    __syncthreads();
    const uint32_t hb = 1000 * 4;
    auto score = [&](const Half& ea, const Half& eb, int b) {
        Half q2;
        load_half(q2, rel + (int64_t)((grp * R + b) % 11) * 1000, lane, hb);
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < GH; ++k) {
            const float4 a = q[b][0][lane + 64 * k], c = q[b][1][lane + 64 * k];
            s += fabsf(a.x * eb.a[k][0] - ea.a[k][0] * c.x + q2.a[k][0]);
            s += fabsf(a.y * eb.a[k][1] - ea.a[k][1] * c.y + q2.a[k][1]);
            s += fabsf(a.z * eb.a[k][2] - ea.a[k][2] * c.z + q2.a[k][2]);
            s += fabsf(a.w * eb.a[k][3] - ea.a[k][3] * c.w + q2.a[k][3]);
        }
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
        return s;
    };
    for (int g = 0; g < NG; ++g) {
        if (g > L) {
            int* c = sync + x * NG + (g - L - 1);
            const int want = nwx * (epoch + 1);
            int polls = 0;
            int v = 0;
            if (lane == 0) v = __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            v = __shfl(v, 0);
            while (v < want && polls < 4000) {
                __builtin_amdgcn_s_sleep(4);
                ++polls;
                if (lane == 0) v = __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                v = __shfl(v, 0);
            }
        }
        const int lo = goff[blk * (NG + 1) + g], hi = goff[blk * (NG + 1) + g + 1];
        for (int c0 = lo + wave; c0 < hi; c0 += NWV * 64) {
            const int nc = min(64, (hi - c0 + NWV - 1) / NWV);
            const int my = c0 + NWV * lane;
            const int my_e = lane < nc ? pe[my] : 0, my_b = lane < nc ? pb[my] : 0;
            float mine = 0.f;
            Half a0, b0, a1, b1;
            int e = __builtin_amdgcn_readlane(my_e, 0);
            load_half(a0, tab + (int64_t)e * 2000, lane, hb);
            load_half(b0, tab + (int64_t)e * 2000 + 1000, lane, hb);
            for (int j = 0; j < nc; j += 2) {
                if (j + 1 < nc) {
                    e = __builtin_amdgcn_readlane(my_e, j + 1);
                    load_half(a1, tab + (int64_t)e * 2000, lane, hb);
                    load_half(b1, tab + (int64_t)e * 2000 + 1000, lane, hb);
                }
                float s = score(a0, b0, __builtin_amdgcn_readlane(my_b, j));
                if (lane == j) mine = s;
                if (j + 1 < nc) {
                    if (j + 2 < nc) {
                        e = __builtin_amdgcn_readlane(my_e, j + 2);
                        load_half(a0, tab + (int64_t)e * 2000, lane, hb);
                        load_half(b0, tab + (int64_t)e * 2000 + 1000, lane, hb);
                    }
                    s = score(a1, b1, __builtin_amdgcn_readlane(my_b, j + 1));
                    if (lane == j + 1) mine = s;
                }
            }
            if (lane < nc) out[my] = mine;
        }
        if (lane == 0) __hip_atomic_fetch_add(sync + x * NG + g, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

struct Lists {
    std::vector<int> off, ids, wl;
};

static double run(const char* name, const Lists& L, const float* tab, int64_t rowf, float* out, double bytes) {
    int *off, *ids, *wl;
    CHECK(hipMalloc(&off, L.off.size() * 4));
    CHECK(hipMalloc(&ids, L.ids.size() * 4));
    CHECK(hipMalloc(&wl, L.wl.size() * 4));
    CHECK(hipMemcpy(off, L.off.data(), L.off.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(ids, L.ids.data(), L.ids.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(wl, L.wl.data(), L.wl.size() * 4, hipMemcpyHostToDevice));
    const int nw = (int)L.wl.size(), blocks = (nw + 3) / 4;
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    const int reps = 20;
    for (int i = 0; i < 3; ++i)
        hipLaunchKernelGGL(gather_lists, dim3(blocks), dim3(256), 0, 0, tab, rowf, (uint32_t)(rowf * 4), off, ids, wl, nw, out);
    CHECK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL(gather_lists, dim3(blocks), dim3(256), 0, 0, tab, rowf, (uint32_t)(rowf * 4), off, ids, wl, nw, out);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    ms /= reps;
    printf("%-44s %8.1f us  %7.0f GB/s (gathered bytes)\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e9);
    CHECK(hipFree(off));
    CHECK(hipFree(ids));
    CHECK(hipFree(wl));
    return ms;
}

int main() {
    const int64_t E = 40943, ROWF = 2000, B = 512, N = 256;
    std::vector<float> h((size_t)(E * ROWF));
    std::mt19937 g(0);
    std::uniform_real_distribution<float> U(-1.f, 1.f);
    for (auto& x : h) x = U(g);
    std::vector<int> neg((size_t)(B * N));
    std::uniform_int_distribution<int> I(0, (int)E - 1);
    for (auto& x : neg) x = I(g);
    float *tab, *out;
    CHECK(hipMalloc(&tab, h.size() * 4));
    CHECK(hipMalloc(&out, B * N * 4));
    CHECK(hipMemcpy(tab, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    const double bytes = (double)B * N * ROWF * 4;

    for (int sorted = 0; sorted < 2; ++sorted) {  // row-major: wave = (b, quarter)
        Lists L;
        L.off.push_back(0);
        for (int64_t b = 0; b < B; ++b)
            for (int q = 0; q < 4; ++q) {
                std::vector<int> v(neg.begin() + b * N + q * 64, neg.begin() + b * N + q * 64 + 64);
                if (sorted) std::sort(v.begin(), v.end());
                L.ids.insert(L.ids.end(), v.begin(), v.end());
                L.off.push_back((int)L.ids.size());
                L.wl.push_back((int)L.wl.size());
            }
        run(sorted ? "rowmajor-sorted (4 waves per batch row)" : "rowmajor (4 waves per batch row)", L, tab, ROWF,
            out, bytes);
    }
    const int64_t slice = (E + 7) / 8;
    for (int sorted = 0; sorted < 2; ++sorted) {
        for (int spread = 0; spread < 2; ++spread) {
            // list (b, x) = row b's candidates in entity slice x
            Lists L;
            L.off.push_back(0);
            for (int64_t b = 0; b < B; ++b)
                for (int x = 0; x < 8; ++x) {
                    std::vector<int> v;
                    for (int64_t n = 0; n < N; ++n)
                        if (neg[b * N + n] / slice == x) v.push_back(neg[b * N + n]);
                    if (sorted) std::sort(v.begin(), v.end());
                    L.ids.insert(L.ids.end(), v.begin(), v.end());
                    L.off.push_back((int)L.ids.size());
                }
            // block i: slice x = i % 8, batch rows 4 (i / 8) .. + 3 (spread: slice x = (i / 64) % 8, no XCD affinity)
            const int nblk = (int)(B / 4 * 8);
            for (int i = 0; i < nblk; ++i)
                for (int w = 0; w < 4; ++w) {
                    const int x = spread ? (i / 64) % 8 : i % 8;
                    const int grp = spread ? (i % 64) + 64 * (i / 512) : i / 8;
                    const int b = 4 * grp + w;
                    L.wl.push_back(b < B ? (int)(b * 8 + x) : -1);
                }
            char nm[96];
            snprintf(nm, sizeof nm, "%s%s", spread ? "slices, no XCD affinity" : "xcd slices",
                     sorted ? " sorted" : "");
            run(nm, L, tab, ROWF, out, bytes);
        }
    }
    {
        // slice x's (b, e) pairs sorted by e, cut into lists of 32 consecutive pairs, dealt to slice x's
        // XCD: repeat gathers of a row fall in one wave's list (the gather side of an entity-major walk)
        Lists L;
        L.off.push_back(0);
        std::vector<std::vector<int>> per(8);
        for (int64_t i = 0; i < B * N; ++i) per[neg[i] / slice].push_back(neg[i]);
        std::vector<std::vector<int>> lists_of(8);
        for (int x = 0; x < 8; ++x) {
            std::sort(per[x].begin(), per[x].end());
            for (size_t c = 0; c < per[x].size(); c += 32) {
                lists_of[x].push_back((int)L.off.size() - 1);
                const size_t e = std::min(per[x].size(), c + 32);
                L.ids.insert(L.ids.end(), per[x].begin() + c, per[x].begin() + e);
                L.off.push_back((int)L.ids.size());
            }
        }
        size_t mx = 0;
        for (int x = 0; x < 8; ++x) mx = std::max(mx, lists_of[x].size());
        const int nblk = (int)(8 * ((mx + 3) / 4));
        for (int i = 0; i < nblk; ++i)
            for (int w = 0; w < 4; ++w) {
                const size_t k = 4 * (size_t)(i / 8) + w;
                const int x = i % 8;
                L.wl.push_back(k < lists_of[x].size() ? lists_of[x][k] : -1);
            }
        run("xcd slices, entity-sorted chunks of 32", L, tab, ROWF, out, bytes);
    }
    {
        // entity-major with queries: (e, b) pairs of entity slice x (x = XCD group, or spread), sorted by
        // e, in lists of 32 pairs that never split an entity's run unless it is longer than 32
        float *qbuf, *rel;
        CHECK(hipMalloc(&qbuf, (size_t)B * 2000 * 4));
        CHECK(hipMalloc(&rel, (size_t)11 * 1000 * 4));
        CHECK(hipMemcpy(qbuf, h.data(), (size_t)B * 2000 * 4, hipMemcpyHostToDevice));
        CHECK(hipMemcpy(rel, h.data(), (size_t)11 * 1000 * 4, hipMemcpyHostToDevice));
        for (int halves : {1, 2}) {
            // halves = 2: slice group = (batch half, entity quarter): each XCD sees 256 batch rows' queries
            const int nsl = 8 / halves;
            const int64_t sl = (E + nsl - 1) / nsl;
            std::vector<std::vector<std::pair<int, int>>> per(8);
            for (int64_t i = 0; i < B * N; ++i) {
                const int e = neg[i], b = (int)(i / N);
                const int x = (int)(e / sl) + nsl * (halves == 2 ? (b >= B / 2) : 0);
                per[x].push_back({e, b});
            }
            std::vector<int> off{0}, pe, pb;
            std::vector<std::vector<int>> lists_of(8);
            for (int x = 0; x < 8; ++x) {
                std::sort(per[x].begin(), per[x].end());
                size_t c = 0;
                while (c < per[x].size()) {
                    size_t e = std::min(per[x].size(), c + 32);
                    while (e < per[x].size() && e > c + 1 && per[x][e].first == per[x][e - 1].first && e - c > 24) --e;
                    lists_of[x].push_back((int)off.size() - 1);
                    for (size_t k = c; k < e; ++k) {
                        pe.push_back(per[x][k].first);
                        pb.push_back(per[x][k].second);
                    }
                    off.push_back((int)pe.size());
                    c = e;
                }
            }
            size_t mx = 0;
            for (int x = 0; x < 8; ++x) mx = std::max(mx, lists_of[x].size());
            std::vector<int> wl;
            const int nblk = (int)(8 * ((mx + 3) / 4));
            for (int i = 0; i < nblk; ++i)
                for (int w = 0; w < 4; ++w) {
                    const size_t k = 4 * (size_t)(i / 8) + w;
                    wl.push_back(k < lists_of[i % 8].size() ? lists_of[i % 8][k] : -1);
                }
            int *doff, *dpe, *dpb, *dwl;
            CHECK(hipMalloc(&doff, off.size() * 4));
            CHECK(hipMalloc(&dpe, pe.size() * 4));
            CHECK(hipMalloc(&dpb, pb.size() * 4));
            CHECK(hipMalloc(&dwl, wl.size() * 4));
            CHECK(hipMemcpy(doff, off.data(), off.size() * 4, hipMemcpyHostToDevice));
            CHECK(hipMemcpy(dpe, pe.data(), pe.size() * 4, hipMemcpyHostToDevice));
            CHECK(hipMemcpy(dpb, pb.data(), pb.size() * 4, hipMemcpyHostToDevice));
            CHECK(hipMemcpy(dwl, wl.data(), wl.size() * 4, hipMemcpyHostToDevice));
            const int nw = (int)wl.size(), blocks = (nw + 3) / 4;
            hipEvent_t a, bb;
            CHECK(hipEventCreate(&a));
            CHECK(hipEventCreate(&bb));
            for (int i = 0; i < 3; ++i)
                hipLaunchKernelGGL(gather_pairs, dim3(blocks), dim3(256), 0, 0, tab, qbuf, rel, doff, dpe, dpb, dwl, nw, out);
            CHECK(hipEventRecord(a));
            for (int i = 0; i < 20; ++i)
                hipLaunchKernelGGL(gather_pairs, dim3(blocks), dim3(256), 0, 0, tab, qbuf, rel, doff, dpe, dpb, dwl, nw, out);
            CHECK(hipEventRecord(bb));
            CHECK(hipEventSynchronize(bb));
            float ms;
            CHECK(hipEventElapsedTime(&ms, a, bb));
            ms /= 20;
            printf("%-44s %8.1f us  %7.0f GB/s (gathered bytes)\n",
                   halves == 1 ? "entity-major + 12 KB query/pair, 8 slices" : "entity-major + query, 2 halves x 4 slices",
                   ms * 1e3, bytes / (ms * 1e-3) / 1e9);
        }
        // row-group tiles (tile_pairs): R rows per block, pairs of slice x sorted by entity
        auto tiles = [&](auto kern, int R, int nwv, const char* nm) {
            const int ngrp = (int)(B / R), nblk = ngrp * 8;
            std::vector<std::vector<std::pair<int, int>>> per(nblk);
            for (int64_t i = 0; i < B * N; ++i) {
                const int e = neg[i], b = (int)(i / N);
                per[(b / R) * 8 + (int)(e / slice)].push_back({e, b % R});
            }
            std::vector<int> off{0}, pe, pb;
            for (auto& v : per) {
                std::sort(v.begin(), v.end());
                for (auto& pr : v) {
                    pe.push_back(pr.first);
                    pb.push_back(pr.second);
                }
                off.push_back((int)pe.size());
            }
            int *doff, *dpe, *dpb;
            CHECK(hipMalloc(&doff, off.size() * 4));
            CHECK(hipMalloc(&dpe, pe.size() * 4));
            CHECK(hipMalloc(&dpb, pb.size() * 4));
            CHECK(hipMemcpy(doff, off.data(), off.size() * 4, hipMemcpyHostToDevice));
            CHECK(hipMemcpy(dpe, pe.data(), pe.size() * 4, hipMemcpyHostToDevice));
            CHECK(hipMemcpy(dpb, pb.data(), pb.size() * 4, hipMemcpyHostToDevice));
            hipEvent_t a, bb;
            CHECK(hipEventCreate(&a));
            CHECK(hipEventCreate(&bb));
            for (int i = 0; i < 3; ++i)
                hipLaunchKernelGGL(kern, dim3(nblk), dim3(nwv * 64), 0, 0, tab, qbuf, rel, doff, dpe, dpb, out);
            CHECK(hipGetLastError());
            CHECK(hipEventRecord(a));
            for (int i = 0; i < 20; ++i)
                hipLaunchKernelGGL(kern, dim3(nblk), dim3(nwv * 64), 0, 0, tab, qbuf, rel, doff, dpe, dpb, out);
            CHECK(hipEventRecord(bb));
            CHECK(hipEventSynchronize(bb));
            float ms;
            CHECK(hipEventElapsedTime(&ms, a, bb));
            ms /= 20;
            printf("%-44s %8.1f us  %7.0f GB/s (gathered bytes)\n", nm, ms * 1e3, bytes / (ms * 1e-3) / 1e9);
            CHECK(hipFree(doff));
            CHECK(hipFree(dpe));
            CHECK(hipFree(dpb));
        };
        tiles(tile_pairs<16, 16, 1>, 16, 16, "tiles R=16, 16 waves, depth 1");
        tiles(tile_pairs<16, 16, 2>, 16, 16, "tiles R=16, 16 waves, depth 2");
        tiles(tile_pairs<16, 8, 2>, 16, 8, "tiles R=16, 8 waves, depth 2");
        tiles(tile_pairs<8, 8, 1>, 8, 8, "tiles R=8, 8 waves, depth 1");
        tiles(tile_pairs<8, 8, 2>, 8, 8, "tiles R=8, 8 waves, depth 2");
        tiles(tile_pairs<8, 16, 1>, 8, 16, "tiles R=8, 16 waves, depth 1");
        tiles(tile_pairs<4, 8, 2>, 4, 8, "tiles R=4, 8 waves, depth 2");
        tiles(tile_pairs<16, 8, 2, true>, 16, 8, "tiles R=16, 8 waves, depth 2, q2 in LDS");
        tiles(tile_pairs<16, 16, 1, true>, 16, 16, "tiles R=16, 16 waves, depth 1, q2 in LDS");
        tiles(tile_pairs<16, 16, 2, true>, 16, 16, "tiles R=16, 16 waves, depth 2, q2 in LDS");
        // paced tiles (tile_pairs_sync): R = 16 rows, 8 waves, NG entity groups, lookahead L
        int* sync;
        CHECK(hipMalloc(&sync, 8 * 64 * 4));
        auto paced = [&](auto kern, int NG, const char* nm) {
            const int R = 16, nwv = 8, ngrp = (int)(B / R), nblk = ngrp * 8;
            std::vector<std::vector<std::pair<int, int>>> per(nblk);
            for (int64_t i = 0; i < B * N; ++i) {
                const int e = neg[i], b = (int)(i / N);
                per[(b / R) * 8 + (int)(e / slice)].push_back({e, b % R});
            }
            std::vector<int> goff, pe, pb;
            for (int blk = 0; blk < nblk; ++blk) {
                auto& v = per[blk];
                std::sort(v.begin(), v.end());
                const int x = blk % 8;
                size_t k = 0;
                for (int g = 0; g < NG; ++g) {
                    goff.push_back((int)pe.size());
                    const int64_t ehi = x * slice + (slice * (g + 1)) / NG;
                    while (k < v.size() && v[k].first < ehi) {
                        pe.push_back(v[k].first);
                        pb.push_back(v[k].second);
                        ++k;
                    }
                }
                goff.push_back((int)pe.size());
            }
            int *dgo, *dpe, *dpb;
            CHECK(hipMalloc(&dgo, goff.size() * 4));
            CHECK(hipMalloc(&dpe, pe.size() * 4));
            CHECK(hipMalloc(&dpb, pb.size() * 4));
            CHECK(hipMemcpy(dgo, goff.data(), goff.size() * 4, hipMemcpyHostToDevice));
            CHECK(hipMemcpy(dpe, pe.data(), pe.size() * 4, hipMemcpyHostToDevice));
            CHECK(hipMemcpy(dpb, pb.data(), pb.size() * 4, hipMemcpyHostToDevice));
            CHECK(hipMemset(sync, 0, 8 * 64 * 4));
            const int nwx = ngrp * nwv;  // waves per XCD
            hipEvent_t a, bb;
            CHECK(hipEventCreate(&a));
            CHECK(hipEventCreate(&bb));
            int ep = 0;
            for (int i = 0; i < 3; ++i, ++ep)
                hipLaunchKernelGGL(kern, dim3(nblk), dim3(nwv * 64), 0, 0, tab, qbuf, rel, dgo, dpe, dpb, out, sync, nwx, ep);
            CHECK(hipGetLastError());
            CHECK(hipEventRecord(a));
            for (int i = 0; i < 20; ++i, ++ep)
                hipLaunchKernelGGL(kern, dim3(nblk), dim3(nwv * 64), 0, 0, tab, qbuf, rel, dgo, dpe, dpb, out, sync, nwx, ep);
            CHECK(hipEventRecord(bb));
            CHECK(hipEventSynchronize(bb));
            float ms;
            CHECK(hipEventElapsedTime(&ms, a, bb));
            ms /= 20;
            printf("%-44s %8.1f us  %7.0f GB/s (gathered bytes)\n", nm, ms * 1e3, bytes / (ms * 1e-3) / 1e9);
            CHECK(hipFree(dgo));
            CHECK(hipFree(dpe));
            CHECK(hipFree(dpb));
        };
        (void)paced;  // paced tiles (every XCD-group barrier a bounded spin): 6-17x slower, same fetched bytes

    }
    return 0;
}
