// stream_probe.hip — mixed read/write streaming ceilings on MI355X for the optimizer pass.
//
// The train step's dense Adam touches every row of the entity table: parameters, m and v are read and
// written (fused into the entity pass: 3 reads + 3 writes), or additionally the gradient is read (the
// standalone kernel: 4 + 3). This probe times those patterns, plus a plain copy and a read-only sum,
// (and with nontemporal stores / loads, the `NT` variants)
// over 327.5 MB arrays (the C2 table), each with float4 per thread and U float4 per thread per
// iteration, grid-stride, 256 threads, `blocks` CUs x waves. Reports total bytes moved / time.
// Build: hipcc --offload-arch=gfx950 -O3 -o stream_probe stream_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

template <int U>
__global__ __launch_bounds__(256) void read_k(const float4* __restrict__ a, int64_t n4, float* out) {
    float s = 0.f;
    for (int64_t i = (int64_t)blockIdx.x * 256 * U + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256 * U) {
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = (i + u * 256 < n4) ? a[i + u * 256] : make_float4(0, 0, 0, 0);
#pragma unroll
        for (int u = 0; u < U; ++u) s += v[u].x + v[u].y + v[u].z + v[u].w;
    }
    if (s == 12345.f) out[0] = s;
}

// NT: 0 plain, 1 nontemporal stores, 2 nontemporal loads and stores
template <int NT>
__device__ __forceinline__ void st4(float4* dst, const float4& x) {
    if constexpr (NT >= 1) {
        float* d = reinterpret_cast<float*>(dst);
        __builtin_nontemporal_store(x.x, d + 0);
        __builtin_nontemporal_store(x.y, d + 1);
        __builtin_nontemporal_store(x.z, d + 2);
        __builtin_nontemporal_store(x.w, d + 3);
    } else {
        *dst = x;
    }
}
template <int NT>
__device__ __forceinline__ float4 ld4(const float4* src) {
    if constexpr (NT >= 2) {
        const float* s = reinterpret_cast<const float*>(src);
        return make_float4(__builtin_nontemporal_load(s + 0), __builtin_nontemporal_load(s + 1),
                           __builtin_nontemporal_load(s + 2), __builtin_nontemporal_load(s + 3));
    } else {
        return *src;
    }
}

template <int U, int NT = 0>
__global__ __launch_bounds__(256) void copy_k(const float4* __restrict__ a, float4* __restrict__ b, int64_t n4) {
    for (int64_t i = (int64_t)blockIdx.x * 256 * U + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256 * U) {
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i + u * 256 < n4) v[u] = ld4<NT>(a + i + u * 256);
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i + u * 256 < n4) st4<NT>(b + i + u * 256, v[u]);
    }
}

// Adam-shaped: NR reads (p, m, v [, g]) and 3 writes (p, m, v)
template <int U, bool G, int NT = 0>
__global__ __launch_bounds__(256) void adam_k(float4* __restrict__ p, float4* __restrict__ m, float4* __restrict__ v,
                                              const float4* __restrict__ g, int64_t n4) {
    for (int64_t i = (int64_t)blockIdx.x * 256 * U + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256 * U) {
        float4 pp[U], mm[U], vv[U], gg[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j = i + u * 256;
            if (j < n4) {
                pp[u] = ld4<NT>(p + j);
                mm[u] = ld4<NT>(m + j);
                vv[u] = ld4<NT>(v + j);
                gg[u] = G ? ld4<NT>(g + j) : make_float4(1e-3f, 1e-3f, 1e-3f, 1e-3f);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j = i + u * 256;
            if (j < n4) {
                float4 a = pp[u], b = mm[u], c = vv[u], d = gg[u];
#define UPD(X)                                 \
    b.X = b.X + (d.X - b.X) * 0.1f;            \
    c.X = c.X + (d.X * d.X - c.X) * 0.001f;    \
    a.X = a.X - b.X * 1e-3f / (sqrtf(c.X) + 1e-7f);
                UPD(x) UPD(y) UPD(z) UPD(w)
#undef UPD
                st4<NT>(p + j, a);
                st4<NT>(m + j, b);
                st4<NT>(v + j, c);
            }
        }
    }
}

int main() {
    const int64_t bytes = 40943LL * 2000 * 4;  // C2 entity table
    const int64_t n4 = bytes / 16;
    float4 *a, *b, *c, *d;
    float* o;
    CHECK(hipMalloc(&a, bytes));
    CHECK(hipMalloc(&b, bytes));
    CHECK(hipMalloc(&c, bytes));
    CHECK(hipMalloc(&d, bytes));
    CHECK(hipMalloc(&o, 4));
    CHECK(hipMemset(a, 0, bytes));
    CHECK(hipMemset(b, 0, bytes));
    CHECK(hipMemset(c, 0, bytes));
    CHECK(hipMemset(d, 0, bytes));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    auto timeit = [&](const char* name, double moved, auto launch) {
        for (int i = 0; i < 3; ++i) launch();
        CHECK(hipEventRecord(e0));
        const int reps = 20;
        for (int i = 0; i < reps; ++i) launch();
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / reps;
        printf("%-40s %9.1f us  %7.3f TB/s\n", name, us, moved / (us * 1e-6) / 1e12);
    };
    for (int blocks : {1024, 2048, 4096, 8192}) {
        printf("-- grid %d blocks\n", blocks);
        timeit("read 1x", bytes, [&] { hipLaunchKernelGGL(read_k<2>, dim3(blocks), dim3(256), 0, 0, a, n4, o); });
        timeit("copy 1r+1w", 2.0 * bytes, [&] { hipLaunchKernelGGL(copy_k<2>, dim3(blocks), dim3(256), 0, 0, a, b, n4); });
        timeit("adam fused 3r+3w U1", 6.0 * bytes,
               [&] { hipLaunchKernelGGL((adam_k<1, false>), dim3(blocks), dim3(256), 0, 0, a, b, c, d, n4); });
        timeit("adam fused 3r+3w U2", 6.0 * bytes,
               [&] { hipLaunchKernelGGL((adam_k<2, false>), dim3(blocks), dim3(256), 0, 0, a, b, c, d, n4); });
        timeit("adam dense 4r+3w U1", 7.0 * bytes,
               [&] { hipLaunchKernelGGL((adam_k<1, true>), dim3(blocks), dim3(256), 0, 0, a, b, c, d, n4); });
        timeit("adam dense 4r+3w U2", 7.0 * bytes,
               [&] { hipLaunchKernelGGL((adam_k<2, true>), dim3(blocks), dim3(256), 0, 0, a, b, c, d, n4); });
        timeit("copy 1r+1w nt-store", 2.0 * bytes,
               [&] { hipLaunchKernelGGL((copy_k<2, 1>), dim3(blocks), dim3(256), 0, 0, a, b, n4); });
        timeit("copy 1r+1w nt-load+store", 2.0 * bytes,
               [&] { hipLaunchKernelGGL((copy_k<2, 2>), dim3(blocks), dim3(256), 0, 0, a, b, n4); });
        timeit("adam fused 3r+3w U2 nt-store", 6.0 * bytes,
               [&] { hipLaunchKernelGGL((adam_k<2, false, 1>), dim3(blocks), dim3(256), 0, 0, a, b, c, d, n4); });
        timeit("adam fused 3r+3w U2 nt-load+store", 6.0 * bytes,
               [&] { hipLaunchKernelGGL((adam_k<2, false, 2>), dim3(blocks), dim3(256), 0, 0, a, b, c, d, n4); });
    }
    return 0;
}
