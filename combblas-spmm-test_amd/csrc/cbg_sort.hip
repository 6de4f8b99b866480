// cbg_sort.hip -- device radix sort of (key, value) pairs and reduce-by-key,
// hand-written for gfx950 (no hipCUB): the global expand-sort-compress of the
// thin big columns (cbg_thin.hip), SpDCCols::Transpose (SpDCCols.cpp:853-873,
// whose SpTuples::SortRowBased is a sort of (row, col) keys) and the
// restriction operator's construction (cbg_ops.hip).  Counts are 64-bit.
//
// LSD radix sort, 8-bit digits, only over the digits of `varying` (a mask of
// the key bits that can differ; a digit that is constant over every key is a
// stable no-op and is skipped).  Per pass, over tiles of 4096 items (256
// threads x 16):
//   k_rs_hist     per-tile digit counts (LDS atomics), digit-major
//   scan          exclusive scan of the 256 x tiles counts (int64 offsets)
//   k_rs_scatter  the tile's items in registers; stable ranks inside the tile
//                 from wave-level digit matching (8 ballots) and per-wave digit
//                 counts; the tile is reordered by digit in LDS and written out
//                 in digit runs (coalesced stores), each run at its global offset.
// Stability makes reduce-by-key sums deterministic: equal keys keep their
// expansion order (as hipCUB's onesweep sort did).
#include <algorithm>

#include "cbg_device.h"
#include "cbg_internal.h"

namespace cbg {

namespace {

constexpr int RS_BS = 256;
constexpr int RS_ITEMS = 16;
constexpr int RS_TILE = RS_BS * RS_ITEMS;  // 4096
constexpr int RS_RADIX = 256;
constexpr int RS_NW = RS_BS / WAVE;

template <typename K>
__global__ __launch_bounds__(RS_BS) void k_rs_hist(const K* __restrict__ keys, int64_t n, int shift, int64_t ntiles,
                                                   int32_t* __restrict__ counts) {
  __shared__ int c[RS_RADIX];
  const int tid = threadIdx.x;
  c[tid] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * RS_TILE;
#pragma unroll
  for (int j = 0; j < RS_ITEMS; ++j) {
    const int64_t i = base + j * RS_BS + tid;
    if (i < n) atomicAdd(&c[(int)((keys[i] >> shift) & 0xFF)], 1);
  }
  __syncthreads();
  counts[(int64_t)tid * ntiles + blockIdx.x] = c[tid];  // digit-major: one scan gives every (digit, tile) offset
}

// lanes of this wave holding the same 8-bit digit (match by 8 ballots)
__device__ __forceinline__ unsigned long long digit_peers(int d) {
  unsigned long long m = __ballot(1);
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    const unsigned long long x = __ballot((d >> b) & 1);
    m &= ((d >> b) & 1) ? x : ~x;
  }
  return m;
}

template <typename K>
__global__ __launch_bounds__(RS_BS) void k_rs_scatter(const K* __restrict__ kin, const double* __restrict__ vin,
                                                      int64_t n, int shift, int64_t ntiles,
                                                      const int64_t* __restrict__ offs, K* __restrict__ kout,
                                                      double* __restrict__ vout) {
  __shared__ int wcnt[2][RS_NW][RS_RADIX];  // digit counts per wave, double-buffered over the rounds
  __shared__ int run[RS_RADIX];             // items of each digit in the earlier rounds (then the tile's offsets)
  __shared__ K sk[RS_TILE];
  __shared__ double sv[RS_TILE];
  const int tid = threadIdx.x, lane = lane_id(), w = tid / WAVE;
  const int64_t base = (int64_t)blockIdx.x * RS_TILE;
  const int nt = (int)std::min<int64_t>(RS_TILE, n - base);
  run[tid] = 0;
#pragma unroll
  for (int q = 0; q < RS_NW; ++q) wcnt[0][q][tid] = 0;
  K k[RS_ITEMS];
  double v[RS_ITEMS];
  int rk[RS_ITEMS];  // rank among the tile's items of the same digit
#pragma unroll
  for (int j = 0; j < RS_ITEMS; ++j) {
    const int64_t i = base + j * RS_BS + tid;
    if (i < n) {
      k[j] = kin[i];
      v[j] = vin[i];
    }
  }
  __syncthreads();
  const unsigned long long lt = (1ull << lane) - 1;
#pragma unroll
  for (int j = 0; j < RS_ITEMS; ++j) {
    // items j * 256 + tid of the tile: index order = (round, wave, lane) order
    int(*wc)[RS_RADIX] = wcnt[j & 1];
    int(*wn)[RS_RADIX] = wcnt[(j + 1) & 1];
    const bool ok = j * RS_BS + tid < nt;
    const int d = ok ? (int)((k[j] >> shift) & 0xFF) : 0;
    const unsigned long long peers = digit_peers(d) & __ballot(ok);
    const int r = __popcll(peers & lt);
    if (ok && r == 0) wc[w][d] = __popcll(peers);  // the digit's lowest lane reports the wave's count
    __syncthreads();
    {
      // digit tid: offsets of the waves inside this round, after the earlier
      // rounds; the other buffer is cleared for the next round (whose counts
      // are written after the barrier below, and whose offsets are taken after
      // every thread has read this round's)
      int acc = run[tid];
#pragma unroll
      for (int q = 0; q < RS_NW; ++q) {
        const int c = wc[q][tid];
        wc[q][tid] = acc;
        acc += c;
        wn[q][tid] = 0;
      }
      run[tid] = acc;
    }
    __syncthreads();
    if (ok) rk[j] = wc[w][d] + r;
  }
  __syncthreads();
  // the tile's digit offsets: exclusive scan of run[] (the tile's digit counts)
  int tot;
  const int cnt_d = run[tid];
  __syncthreads();
  const int ex = block_excl_scan<RS_BS>(cnt_d, &wcnt[0][0][0], &tot);
  run[tid] = ex;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < RS_ITEMS; ++j)
    if (j * RS_BS + tid < nt) {
      const int d = (int)((k[j] >> shift) & 0xFF);
      const int p = run[d] + rk[j];
      sk[p] = k[j];
      sv[p] = v[j];
    }
  __syncthreads();
  // digit runs of the reordered tile, each to its global offset (consecutive
  // positions of one digit are consecutive addresses)
  for (int p = tid; p < nt; p += RS_BS) {
    const K key = sk[p];
    const int d = (int)((key >> shift) & 0xFF);
    const int64_t o = offs[(int64_t)d * ntiles + blockIdx.x] + (p - run[d]);
    kout[o] = key;
    vout[o] = sv[p];
  }
}

// reduce-by-key over sorted keys: run heads, their scan, one thread per run
template <typename K>
__global__ void k_rbk_flags(const K* __restrict__ k, int64_t n, int32_t* __restrict__ flag) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < n) flag[i] = (i == 0 || k[i] != k[i - 1]) ? 1 : 0;
}
template <typename K, int SR>
__global__ void k_rbk_runs(const K* __restrict__ k, const double* __restrict__ v, int64_t n,
                           const int64_t* __restrict__ pos, K* __restrict__ uk, double* __restrict__ uv) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n || (i > 0 && k[i] == k[i - 1])) return;
  const K key = k[i];
  double acc = v[i];
  for (int64_t q = i + 1; q < n && k[q] == key; ++q) acc = Sem<SR>::add(acc, v[q]);  // in sorted (= expansion) order
  uk[pos[i]] = key;
  uv[pos[i]] = acc;
}

}  // namespace

template <typename K>
void radix_sort_pairs(DBuf<K>& keys, DBuf<double>& vals, int64_t n, unsigned long long varying, hipStream_t s,
                      DeferredFree* df) {
  if (n <= 1) return;
  const int64_t ntiles = (n + RS_TILE - 1) / RS_TILE;
  DBuf<K> k2(n);
  DBuf<double> v2(n);
  DBuf<int32_t> counts(ntiles * RS_RADIX + 1);
  DBuf<int64_t> offs(ntiles * RS_RADIX + 1);
  for (int shift = 0; shift < (int)(8 * sizeof(K)); shift += 8) {
    if (!((varying >> shift) & 0xFFull)) continue;
    hipLaunchKernelGGL(k_rs_hist<K>, dim3((unsigned)ntiles), dim3(RS_BS), 0, s, keys.p, n, shift, ntiles, counts.p);
    exclusive_scan_i32_to_i64(counts.p, offs.p, ntiles * RS_RADIX, s, df);
    hipLaunchKernelGGL(k_rs_scatter<K>, dim3((unsigned)ntiles), dim3(RS_BS), 0, s, keys.p, vals.p, n, shift, ntiles,
                       offs.p, k2.p, v2.p);
    std::swap(keys.p, k2.p);
    std::swap(vals.p, v2.p);
  }
  if (df) {  // the temporaries go back to the pool after the caller's synchronization
    df->take(k2);
    df->take(v2);
    df->take(counts);
    df->take(offs);
    return;
  }
  CBG_HIP(hipStreamSynchronize(s));  // k2 / v2 / counts go back to the pool
}

template <typename K>
int64_t reduce_by_key(const K* keys, const double* vals, int64_t n, int semiring, K* ukeys, double* uvals,
                      hipStream_t s, DeferredFree* df) {
  if (n <= 0) return 0;
  DBuf<int32_t> flag(n + 1);
  DBuf<int64_t> pos(n + 1);
  const unsigned g = (unsigned)((n + 255) / 256);
  hipLaunchKernelGGL(k_rbk_flags<K>, dim3(g), dim3(256), 0, s, keys, n, flag.p);
  exclusive_scan_i32_to_i64(flag.p, pos.p, n, s, df);
  if (semiring == CBG_MIN_PLUS)
    hipLaunchKernelGGL((k_rbk_runs<K, 1>), dim3(g), dim3(256), 0, s, keys, vals, n, pos.p, ukeys, uvals);
  else
    hipLaunchKernelGGL((k_rbk_runs<K, 0>), dim3(g), dim3(256), 0, s, keys, vals, n, pos.p, ukeys, uvals);
  int64_t runs = 0;
  CBG_HIP(hipMemcpyAsync(&runs, pos.p + n, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  CBG_HIP(hipStreamSynchronize(s));  // the one readback: the run count
  if (df) {
    df->take(flag);
    df->take(pos);
  }
  return runs;
}

template void radix_sort_pairs<uint32_t>(DBuf<uint32_t>&, DBuf<double>&, int64_t, unsigned long long, hipStream_t,
                                         DeferredFree*);
template void radix_sort_pairs<unsigned long long>(DBuf<unsigned long long>&, DBuf<double>&, int64_t,
                                                   unsigned long long, hipStream_t, DeferredFree*);
template int64_t reduce_by_key<uint32_t>(const uint32_t*, const double*, int64_t, int, uint32_t*, double*,
                                         hipStream_t, DeferredFree*);
template int64_t reduce_by_key<unsigned long long>(const unsigned long long*, const double*, int64_t, int,
                                                   unsigned long long*, double*, hipStream_t, DeferredFree*);

}  // namespace cbg
