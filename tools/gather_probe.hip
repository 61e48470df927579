// gather_probe.hip — memory-system ceiling for the scoring kernel's access pattern on MI355X.
//
// Measures, with hipEvents, how fast a wave64 can gather random fp32 rows of ROW floats from a
// table of E rows when the per-row compute is trivial (sum of the row): the same decomposition
// as score_fwd_kernel (one wave per (b, run of CPW candidates), 16-B buffer loads, DEPTH rows in
// flight per wave). Also a contiguous stream of the same byte count (HBM streaming ceiling) and a
// small, Infinity-Cache-resident table. Build: hipcc --offload-arch=gfx950 -O3 -o gather_probe gather_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#define CHECK(x)                                                                          \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
            exit(1);                                                                      \
        }                                                                                 \
    } while (0)

using rsrc_t = __amdgpu_buffer_rsrc_t;
__device__ __forceinline__ rsrc_t make_rsrc(const void* base, uint32_t bytes) {
    const uint64_t a = (uint64_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0,
                                             (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

__device__ __forceinline__ int64_t readlane64(int64_t v, int j) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(uint64_t)v, j);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), j);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

template <int G>  // float4 groups per lane per row: ROW = 256 * G floats
struct Row {
    float a[G][4];
};

template <int G>
__device__ __forceinline__ void load_row(Row<G>& r, const float* base, int lane, uint32_t bytes) {
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

template <int G>
__device__ __forceinline__ float row_sum(const Row<G>& r) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < G; ++k) s += (r.a[k][0] + r.a[k][1]) + (r.a[k][2] + r.a[k][3]);
    return s;
}

// DEPTH rows in flight per wave (ring of DEPTH row buffers)
template <int G, int DEPTH>
__global__ __launch_bounds__(256) void gather_kernel(const float* __restrict__ tab, int64_t row_floats,
                                                     const int64_t* __restrict__ idx, int64_t total, int cpw,
                                                     uint32_t row_bytes, float* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t n0 = w * cpw;
    if (n0 >= total) return;
    const int nc = (int)min((int64_t)cpw, total - n0);
    int64_t my = lane < nc ? idx[n0 + lane] : 0;
    Row<G> r[DEPTH];
    float acc = 0.f, mine = 0.f;
#pragma unroll
    for (int d = 0; d < DEPTH; ++d)
        if (d < nc) load_row<G>(r[d], tab + readlane64(my, d) * row_floats, lane, row_bytes);
    for (int j = 0; j < nc; j += DEPTH) {
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
            if (j + d < nc) {
                const float s = row_sum<G>(r[d]);
                acc += s;
                if (lane == j + d) mine = s;
                if (j + d + DEPTH < nc) load_row<G>(r[d], tab + readlane64(my, j + d + DEPTH) * row_floats, lane, row_bytes);
            }
        }
    }
    if (lane < nc) out[n0 + lane] = mine + acc * 1e-30f;
}

__global__ __launch_bounds__(256) void stream_kernel(const float4* __restrict__ src, int64_t n4, float* __restrict__ out) {
    float s = 0.f;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
        const float4 v = src[i];
        s += (v.x + v.y) + (v.z + v.w);
    }
    if (s == 12345.678f) out[0] = s;
}

template <int G, int DEPTH>
double time_gather(const float* tab, int64_t rowf, const int64_t* idx, int64_t total, int cpw, float* out, int reps) {
    const int64_t waves = (total + cpw - 1) / cpw;
    const int blocks = (int)((waves + 3) / 4);
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i)
        hipLaunchKernelGGL((gather_kernel<G, DEPTH>), dim3(blocks), dim3(256), 0, 0, tab, rowf, idx, total, cpw,
                           (uint32_t)(rowf * 4), out);
    CHECK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL((gather_kernel<G, DEPTH>), dim3(blocks), dim3(256), 0, 0, tab, rowf, idx, total, cpw,
                           (uint32_t)(rowf * 4), out);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main(int argc, char** argv) {
    const int64_t E = 40943, ROWF = 2000, B = 512, N = 256;
    const int64_t total = B * N;
    const int reps = 20;
    std::vector<float> h((size_t)(E * ROWF));
    std::mt19937 g(0);
    std::uniform_real_distribution<float> U(-1.f, 1.f);
    for (auto& x : h) x = U(g);
    std::vector<int64_t> hidx((size_t)total);
    std::uniform_int_distribution<int64_t> I(0, E - 1);
    for (auto& x : hidx) x = I(g);
    // small table: 5000 rows (40 MB) -> Infinity-Cache resident
    std::vector<int64_t> hsmall((size_t)total);
    std::uniform_int_distribution<int64_t> Is(0, 4999);
    for (auto& x : hsmall) x = Is(g);

    float *tab, *out, *big;
    int64_t *idx, *sidx;
    CHECK(hipMalloc(&tab, h.size() * 4));
    CHECK(hipMalloc(&out, total * 4));
    CHECK(hipMalloc(&idx, total * 8));
    CHECK(hipMalloc(&sidx, total * 8));
    CHECK(hipMemcpy(tab, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(idx, hidx.data(), total * 8, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(sidx, hsmall.data(), total * 8, hipMemcpyHostToDevice));
    const double bytes = (double)total * ROWF * 4;
    // ROW = 2000 floats = 500 float4 -> 8 groups of 64 lanes (last partial, range-checked)
    struct V {
        const char* name;
        double ms;
    };
    std::vector<V> res;
    for (int cpw : {8, 16, 32}) {
        char nm[128];
        snprintf(nm, sizeof nm, "gather 327MB table depth1 cpw%d", cpw);
        res.push_back({strdup(nm), time_gather<8, 1>(tab, ROWF, idx, total, cpw, out, reps)});
        snprintf(nm, sizeof nm, "gather 327MB table depth2 cpw%d", cpw);
        res.push_back({strdup(nm), time_gather<8, 2>(tab, ROWF, idx, total, cpw, out, reps)});
        snprintf(nm, sizeof nm, "gather 327MB table depth3 cpw%d", cpw);
        res.push_back({strdup(nm), time_gather<8, 3>(tab, ROWF, idx, total, cpw, out, reps)});
    }
    res.push_back({"gather 40MB table depth2 cpw16", time_gather<8, 2>(tab, ROWF, sidx, total, 16, out, reps)});
    // contiguous stream of the same bytes (first 1.05 GB of a fresh buffer)
    CHECK(hipMalloc(&big, (size_t)bytes));
    CHECK(hipMemset(big, 0, (size_t)bytes));
    {
        hipEvent_t a, b;
        CHECK(hipEventCreate(&a));
        CHECK(hipEventCreate(&b));
        const int64_t n4 = (int64_t)(bytes / 16);
        for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(stream_kernel, dim3(4096), dim3(256), 0, 0, (const float4*)big, n4, out);
        CHECK(hipEventRecord(a));
        for (int i = 0; i < reps; ++i)
            hipLaunchKernelGGL(stream_kernel, dim3(4096), dim3(256), 0, 0, (const float4*)big, n4, out);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        res.push_back({"stream 1.05GB contiguous", ms / reps});
    }
    for (auto& v : res) printf("%-40s %8.1f us  %7.0f GB/s\n", v.name, v.ms * 1e3, bytes / (v.ms * 1e-3) / 1e9);
    return 0;
}
