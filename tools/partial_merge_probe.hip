// partial_merge_probe.hip — what the fused train forward would pay for per-slice partial states.
//
// In the XCD-sliced (or tile) order a batch row's candidates are split over 8 slices, so the fused train forward's
// online-softmax gradient sums (A and B: 2 x 3 x D floats per row, plus the running max / normaliser) would be
// written once per (row, slice) and merged in fixed slice order before the row's closing (A - T R B) / Z
// (DESIGN §3.3). This probe times exactly that extra traffic at C2's shape (B = 512 rows, 8 slices, D = 1000):
//   write  — one wave per (row, slice) stores its 6 D partial floats + 4 scalars (98.3 MB per step), blocks mapped
//            slice = blockIdx & 7 as the sliced kernels are;
//   merge  — one (or 4) block(s) per row read its 8 slices' scalars, rescales by exp(m_s - M) and sums the 8 partial vectors
//            in slice order, writing the merged 6 D floats (reads 98.3 MB, writes 12.3 MB); plain and
//            nontemporal partial stores, 1 and 4 merge blocks per row: the cheapest pair is reported;
//   base   — what the epilogue reads today instead: one 6 D vector per row, copied (12.3 MB read, 12.3 MB written).
// Extra cost of the sliced form = write + merge - base, to be added to the sliced order's gather time.
// Build: hipcc --offload-arch=gfx950 -O3 -o partial_merge_probe partial_merge_probe.hip
#include <hip/hip_runtime.h>

#include <cmath>
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

constexpr int kSlices = 8, kVec = 6;

// one wave per (row, slice); 4 waves per block; the block's slice is blockIdx & 7 (the sliced kernels' mapping)
template <bool NT>
__global__ __launch_bounds__(256) void write_partials(float4* __restrict__ part, float4* __restrict__ stats, int B,
                                                      int d4, float seed) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int s = blockIdx.x & 7;
    const int b = (blockIdx.x >> 3) * 4 + w;
    if (b >= B) return;
    const int64_t ps = (int64_t)b * kSlices + s;
    float4* dst = part + ps * kVec * d4;
    const float base = seed + (float)ps;
    for (int i = lane; i < kVec * d4; i += 64) {
        const float v = base + (float)i;
        const float4 x = make_float4(v, v + 1.f, v + 2.f, v + 3.f);
        if constexpr (NT) {
            __builtin_nontemporal_store(x.x, &dst[i].x);
            __builtin_nontemporal_store(x.y, &dst[i].y);
            __builtin_nontemporal_store(x.z, &dst[i].z);
            __builtin_nontemporal_store(x.w, &dst[i].w);
        } else {
            dst[i] = x;
        }
    }
    if (lane == 0) stats[ps] = make_float4(0.01f * (float)s, 1.f + (float)s, 0.5f, 0.f);
}

// gridDim.y blocks per row: scale factors from the slices' maxima, then the 8 partial vectors summed in slice order
__global__ __launch_bounds__(256) void merge_partials(const float4* __restrict__ part, const float4* __restrict__ stats,
                                                      float4* __restrict__ out, int d4) {
    const int b = blockIdx.x;
    __shared__ float f[kSlices];
    if (threadIdx.x < kSlices) {
        float m = -INFINITY;
        for (int s = 0; s < kSlices; ++s) m = fmaxf(m, stats[(int64_t)b * kSlices + s].x);
        f[threadIdx.x] = __expf(stats[(int64_t)b * kSlices + threadIdx.x].x - m);
    }
    __syncthreads();
    const float4* src = part + (int64_t)b * kSlices * kVec * d4;
    float4* dst = out + (int64_t)b * kVec * d4;
    for (int i = blockIdx.y * 256 + threadIdx.x; i < kVec * d4; i += 256 * gridDim.y) {
        float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int s = 0; s < kSlices; ++s) {
            const float4 v = src[(int64_t)s * kVec * d4 + i];
            a.x += f[s] * v.x;
            a.y += f[s] * v.y;
            a.z += f[s] * v.z;
            a.w += f[s] * v.w;
        }
        dst[i] = a;
    }
}

__global__ __launch_bounds__(256) void base_copy(const float4* __restrict__ src, float4* __restrict__ dst, int d4) {
    const int64_t o = (int64_t)blockIdx.x * kVec * d4;
    for (int i = threadIdx.x; i < kVec * d4; i += 256) dst[o + i] = src[o + i];
}

int main(int argc, char** argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 512;
    const int D = argc > 2 ? atoi(argv[2]) : 1000;
    const int reps = argc > 3 ? atoi(argv[3]) : 50;
    if (D % 4 != 0 || B <= 0 || reps <= 0) {
        fprintf(stderr, "usage: partial_merge_probe [B] [D, multiple of 4] [reps]\n");
        return 1;
    }
    const int d4 = D / 4;
    const size_t part_n = (size_t)B * kSlices * kVec * d4, row_n = (size_t)B * kVec * d4;
    float4 *part, *stats, *merged, *rowv, *rowo;
    CHECK(hipMalloc(&part, part_n * sizeof(float4)));
    CHECK(hipMalloc(&stats, (size_t)B * kSlices * sizeof(float4)));
    CHECK(hipMalloc(&merged, row_n * sizeof(float4)));
    CHECK(hipMalloc(&rowv, row_n * sizeof(float4)));
    CHECK(hipMalloc(&rowo, row_n * sizeof(float4)));
    CHECK(hipMemset(rowv, 0, row_n * sizeof(float4)));
    hipEvent_t e[4];
    for (auto& x : e) CHECK(hipEventCreate(&x));
    const int wblocks = ((B + 3) / 4) * kSlices;
    // variants: (write plain | nontemporal) x (merge 1 | 4 blocks per row); the best pair is the lower bound
    double best = 1e30, bw = 0, bm = 0, bb = 0;
    for (int var = 0; var < 4; ++var) {
        const bool nt = var & 1;
        const dim3 mgrid(B, (var & 2) ? 4 : 1);
        double tw = 0, tm = 0, tb = 0;
        for (int it = -5; it < reps; ++it) {
            CHECK(hipEventRecord(e[0]));
            if (nt)
                write_partials<true><<<wblocks, 256>>>(part, stats, B, d4, (float)it);
            else
                write_partials<false><<<wblocks, 256>>>(part, stats, B, d4, (float)it);
            CHECK(hipEventRecord(e[1]));
            merge_partials<<<mgrid, 256>>>(part, stats, merged, d4);
            CHECK(hipEventRecord(e[2]));
            base_copy<<<B, 256>>>(rowv, rowo, d4);
            CHECK(hipEventRecord(e[3]));
            CHECK(hipEventSynchronize(e[3]));
            float a, b, c;
            CHECK(hipEventElapsedTime(&a, e[0], e[1]));
            CHECK(hipEventElapsedTime(&b, e[1], e[2]));
            CHECK(hipEventElapsedTime(&c, e[2], e[3]));
            if (it >= 0) tw += a, tm += b, tb += c;
        }
        tw *= 1e3 / reps, tm *= 1e3 / reps, tb *= 1e3 / reps;
        printf("{\"variant\": \"write_%s merge_x%d\", \"write_us\": %.2f, \"merge_us\": %.2f, \"base_us\": %.2f, "
               "\"extra_us\": %.2f}\n", nt ? "nt" : "plain", mgrid.y, tw, tm, tb, tw + tm - tb);
        if (tw + tm - tb < best) best = tw + tm - tb, bw = tw, bm = tm, bb = tb;
    }
    CHECK(hipGetLastError());
    const double mb_part = part_n * 16.0 / 1e6, mb_row = row_n * 16.0 / 1e6;
    printf("{\"B\": %d, \"D\": %d, \"reps\": %d, \"partial_MB\": %.1f, \"row_MB\": %.1f, \"write_us\": %.2f, "
           "\"merge_us\": %.2f, \"base_us\": %.2f, \"extra_us\": %.2f, \"best_of\": 4}\n",
           B, D, reps, mb_part, mb_row, bw, bm, bb, best);
    CHECK(hipFree(part));
    CHECK(hipFree(stats));
    CHECK(hipFree(merged));
    CHECK(hipFree(rowv));
    CHECK(hipFree(rowo));
    return 0;
}
