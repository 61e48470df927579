// kge_scan.h — exclusive scan of int counts (entity buckets of the deterministic backward passes).
// Included by several translation units; every kernel has internal linkage.
#pragma once

#include "kge_internal.h"

namespace kge_impl {
namespace {

// exclusive scan of count[0..E) -> off[0..E] (and cursor = off), three launches:
//   tiles of 1024 (block scan, tile totals) -> scan of the tile totals (one block) -> add prefix
constexpr int kScanTile = 1024;

__device__ __forceinline__ int block_exclusive_scan_1024(int v, int* part, int& total) {
    const int t = threadIdx.x;
    part[t] = v;
    __syncthreads();
    for (int o = 1; o < kScanTile; o <<= 1) {  // Hillis-Steele inclusive scan in LDS
        const int u = t >= o ? part[t - o] : 0;
        __syncthreads();
        part[t] += u;
        __syncthreads();
    }
    total = part[kScanTile - 1];
    return part[t] - v;
}

__global__ __launch_bounds__(kScanTile) void scan_tiles_kernel(const int* __restrict__ count, int64_t E,
                                                               int* __restrict__ off, int* __restrict__ tile_sum) {
    __shared__ int part[kScanTile];
    const int64_t i = (int64_t)blockIdx.x * kScanTile + threadIdx.x;
    const int v = i < E ? count[i] : 0;
    int total;
    const int ex = block_exclusive_scan_1024(v, part, total);
    if (i < E) off[i] = ex;
    if (threadIdx.x == 0) tile_sum[blockIdx.x] = total;
}

__global__ __launch_bounds__(kScanTile) void scan_sums_kernel(int* __restrict__ tile_sum, int ntiles,
                                                              int* __restrict__ off_end) {
    __shared__ int part[kScanTile];
    int carry = 0;
    for (int base = 0; base < ntiles; base += kScanTile) {  // ntiles > 1024 loops (E > 1M rows)
        const int i = base + threadIdx.x;
        const int v = i < ntiles ? tile_sum[i] : 0;
        int total;
        const int ex = block_exclusive_scan_1024(v, part, total);
        __syncthreads();
        if (i < ntiles) tile_sum[i] = carry + ex;
        carry += total;
        __syncthreads();
    }
    if (threadIdx.x == 0) *off_end = carry;
}

__global__ __launch_bounds__(kBlock) void scan_add_kernel(int* __restrict__ off, int* __restrict__ cursor, int64_t E,
                                                          const int* __restrict__ tile_sum) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= E) return;
    const int v = off[i] + tile_sum[i / kScanTile];
    off[i] = v;
    cursor[i] = v;
}

// count[0..E) -> off[0..E] (exclusive, off[E] = total) and cursor[0..E) = off; `tiles` holds
// ceil(E / 1024) ints of scratch.
inline void launch_exclusive_scan(const int* count, int64_t E, int* off, int* cursor, int* tiles, hipStream_t st) {
    if (E <= 0) return;
    const int ntiles = (int)((E + kScanTile - 1) / kScanTile);
    hipLaunchKernelGGL(scan_tiles_kernel, dim3(ntiles), dim3(kScanTile), 0, st, count, E, off, tiles);
    hipLaunchKernelGGL(scan_sums_kernel, dim3(1), dim3(kScanTile), 0, st, tiles, ntiles, off + E);
    hipLaunchKernelGGL(scan_add_kernel, dim3((unsigned)((E + kBlock - 1) / kBlock)), dim3(kBlock), 0, st, off,
                       cursor, E, tiles);
}

}  // namespace
}  // namespace kge_impl
