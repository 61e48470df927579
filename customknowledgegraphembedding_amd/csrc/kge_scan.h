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

// One-launch exclusive scan for the train step's entity buckets: a single block of 1024 threads.
// The counts are read as int4 through a range-checked buffer descriptor (zero past E), 8 tiles of
// 4096 ints at a time, every load in flight at once; each tile is scanned across the block (wave
// shuffles, 16 wave totals in LDS) and the tiles are chained in order. With `zero` the counts are
// reset to 0 on the way (the train step keeps its count array zero between calls, so no memset is
// needed). off[E] = total; cursor = off. Needs 16-B aligned count/off/cursor.
constexpr int kScanK = 8;  // tiles in flight per super-tile
typedef int scan_i4 __attribute__((ext_vector_type(4)));
typedef unsigned scan_u4 __attribute__((ext_vector_type(4)));

// (unused attribute: kge_transparse.hip includes this header for launch_exclusive_scan only)
__global__ __launch_bounds__(kScanTile) __attribute__((unused)) void scan_block_kernel(int* __restrict__ count, int64_t E, int* __restrict__ off,
                                                               int* __restrict__ cursor, int zero, int cap) {
    constexpr int NW = kScanTile / kWave;  // 16 waves
    __shared__ int wtot[kScanK][NW];
    __shared__ int carry_s;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const uint32_t bytes = (uint32_t)(E * 4);
    const auto rc = __builtin_amdgcn_make_buffer_rsrc(count, (short)0, (int)bytes, 0x00020000);
    const auto ro = __builtin_amdgcn_make_buffer_rsrc(off, (short)0, (int)bytes, 0x00020000);
    const auto ru = __builtin_amdgcn_make_buffer_rsrc(cursor, (short)0, (int)bytes, 0x00020000);
    int carry = 0;
    for (int64_t base = 0; base < E; base += (int64_t)kScanK * kScanTile * 4) {
        scan_i4 x[kScanK];
#pragma unroll
        for (int r = 0; r < kScanK; ++r) {
            const int64_t e0 = base + ((int64_t)r * kScanTile + t) * 4;
            x[r] = e0 < E ? __builtin_bit_cast(scan_i4, __builtin_amdgcn_raw_buffer_load_b128(rc, (uint32_t)(e0 * 4), 0, 0))
                          : scan_i4{0, 0, 0, 0};
        }
        int incl[kScanK];
#pragma unroll
        for (int r = 0; r < kScanK; ++r) {
            int v = x[r][0] + x[r][1] + x[r][2] + x[r][3];
#pragma unroll
            for (int o = 1; o < kWave; o <<= 1) {
                const int y = __shfl_up(v, o, kWave);
                if (lane >= o) v += y;
            }
            incl[r] = v;
            if (lane == kWave - 1) wtot[r][w] = v;
        }
        __syncthreads();
        // exclusive prefix of this thread's int4 in each tile, tiles chained in order
        int tile_base = carry;
#pragma unroll
        for (int r = 0; r < kScanK; ++r) {
            int before = 0, all = 0;
#pragma unroll
            for (int ww = 0; ww < NW; ++ww) {
                const int v = wtot[r][ww];
                before += ww < w ? v : 0;
                all += v;
            }
            int run = tile_base + before + incl[r] - (x[r][0] + x[r][1] + x[r][2] + x[r][3]);
            scan_i4 o4;  // offsets clamped to `cap` (the number of events): corrupt counts stay in bounds
            o4[0] = min(run, cap);
            run += x[r][0];
            o4[1] = min(run, cap);
            run += x[r][1];
            o4[2] = min(run, cap);
            run += x[r][2];
            o4[3] = min(run, cap);
            const int64_t e0 = base + ((int64_t)r * kScanTile + t) * 4;
            if (e0 < E) {
                const scan_u4 u = __builtin_bit_cast(scan_u4, o4);
                __builtin_amdgcn_raw_buffer_store_b128(u, ro, (uint32_t)(e0 * 4), 0, 0);
                __builtin_amdgcn_raw_buffer_store_b128(u, ru, (uint32_t)(e0 * 4), 0, 0);
                if (zero) __builtin_amdgcn_raw_buffer_store_b128(scan_u4{0u, 0u, 0u, 0u}, rc, (uint32_t)(e0 * 4), 0, 0);
            }
            tile_base += all;
        }
        carry = tile_base;
        __syncthreads();  // wtot is rewritten by the next super-tile
    }
    if (t == 0) carry_s = carry;
    __syncthreads();
    if (t == 0) off[E] = min(carry_s, cap);
}

// Tile-local exclusive scan for the train step's entity buckets: block i (1024 threads, one int4 each)
// scans the 4096 counts of tile i, writes the tile-LOCAL exclusive offsets to off and cursor and the tile's
// total to tile_sum[i]. The consumer (step_epilogue_kernel) adds the tiles' prefix itself: the scatter adds
// it to each cursor it draws, and it rewrites off to the global offsets for phase 2. All tiles run at once
// (one launch, no cross-block wait), instead of one block walking every tile.
constexpr int kTile4k = 4 * kScanTile;
__global__ __launch_bounds__(kScanTile) __attribute__((unused)) void scan_tiles4k_kernel(const int* __restrict__ count, int64_t E,
                                                                 int* __restrict__ off, int* __restrict__ cursor,
                                                                 int* __restrict__ tile_sum) {
    constexpr int NW = kScanTile / kWave;
    __shared__ int wtot[NW];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int64_t e0 = (int64_t)blockIdx.x * kTile4k + (int64_t)t * 4;
    const uint32_t bytes = (uint32_t)(E * 4);
    const auto rc = __builtin_amdgcn_make_buffer_rsrc(const_cast<int*>(count), (short)0, (int)bytes, 0x00020000);
    const scan_i4 x = e0 < E ? __builtin_bit_cast(scan_i4, __builtin_amdgcn_raw_buffer_load_b128(rc, (uint32_t)(e0 * 4), 0, 0))
                             : scan_i4{0, 0, 0, 0};
    const int v = x[0] + x[1] + x[2] + x[3];
    int incl = v;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        const int y = __shfl_up(incl, o, kWave);
        if (lane >= o) incl += y;
    }
    if (lane == kWave - 1) wtot[w] = incl;
    __syncthreads();
    int before = 0, all = 0;
#pragma unroll
    for (int ww = 0; ww < NW; ++ww) {
        const int s = wtot[ww];
        before += ww < w ? s : 0;
        all += s;
    }
    int run = before + incl - v;
    scan_i4 o4;
    o4[0] = run;
    run += x[0];
    o4[1] = run;
    run += x[1];
    o4[2] = run;
    run += x[2];
    o4[3] = run;
    if (e0 < E) {
        const auto ro = __builtin_amdgcn_make_buffer_rsrc(off, (short)0, (int)bytes, 0x00020000);
        const auto ru = __builtin_amdgcn_make_buffer_rsrc(cursor, (short)0, (int)bytes, 0x00020000);
        const scan_u4 u = __builtin_bit_cast(scan_u4, o4);
        __builtin_amdgcn_raw_buffer_store_b128(u, ro, (uint32_t)(e0 * 4), 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(u, ru, (uint32_t)(e0 * 4), 0, 0);
    }
    if (t == 0) tile_sum[blockIdx.x] = all;
}

}  // namespace
}  // namespace kge_impl
