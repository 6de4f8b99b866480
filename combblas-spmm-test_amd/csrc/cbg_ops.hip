// cbg_ops.hip -- tile operations of the Galerkin triple-product path
// (reference ReleaseTests/GalerkinNew.cpp:96-153):
//   tile_transpose     SpDCCols::Transpose (SpDCCols.cpp:853-873): DCSC of T^T
//   tile_dim_apply     SpParMat::DimApply (SpParMat.cpp:801): x(i,j) = op(x(i,j), v[j] or v[i])
//   restriction_tile   the restriction operator T of the multigrid driver
//                      (mfiles/genrestrict.m:11 sprand(n, n/order, order/n): Poisson(1)
//                      nonzeros per fine row in uniform coarse columns, values in (0,1])
// Sorts: cbg_sort.hip (radix sort over the key bits that vary, 64-bit counts).
#include <algorithm>
#include <type_traits>

#include "cbg_device.h"
#include "cbg_internal.h"

namespace cbg {

namespace {
__device__ __forceinline__ unsigned long long mix(unsigned long long z) {
  z += 0x9e3779b97f4a7c15ULL;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
}  // namespace

// (row << 32 | col) keys of every nonzero, wave per column
__global__ void k_transpose_keys(int64_t nzc, const int64_t* __restrict__ cp, const int32_t* __restrict__ jc,
                                 const int32_t* __restrict__ ir, unsigned long long* __restrict__ key) {
  const int64_t i = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / WAVE;
  if (i >= nzc) return;
  const unsigned long long c = (unsigned)jc[i];
  for (int64_t q = cp[i] + lane_id(); q < cp[i + 1]; q += WAVE) key[q] = ((unsigned long long)(unsigned)ir[q] << 32) | c;
}

// sorted (major << 32 | minor) keys -> DCSC with major as the column: flags of
// column starts, then ir/val/jc/cp from their scan
__global__ void k_key_flags(int64_t n, const unsigned long long* __restrict__ k, int64_t* __restrict__ flag) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < n) flag[i] = (i == 0 || (k[i] >> 32) != (k[i - 1] >> 32)) ? 1 : 0;
}
__global__ void k_key_fill(int64_t n, const unsigned long long* __restrict__ k, const double* __restrict__ v,
                           const int64_t* __restrict__ pos, int32_t* __restrict__ ir, double* __restrict__ val,
                           int32_t* __restrict__ jc, int64_t* __restrict__ cp) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  ir[i] = (int32_t)(k[i] & 0xFFFFFFFFULL);
  val[i] = v[i];
  if (i == 0 || (k[i] >> 32) != (k[i - 1] >> 32)) {
    jc[pos[i]] = (int32_t)(k[i] >> 32);
    cp[pos[i]] = i;
  }
}

// n sorted keys (+ values) -> DCSC tile m x nn
static void keys_to_tile(unsigned long long* keys, double* vals, int64_t n, int64_t m, int64_t nn, cbg_tile& out,
                         hipStream_t s) {
  if (n == 0) {
    tile_alloc_device(out, m, nn, 0, 0);
    return;
  }
  DBuf<int64_t> flag(n + 1), pos(n + 1);
  hipLaunchKernelGGL(k_key_flags, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, keys, flag.p);
  exclusive_scan_i64(flag.p, pos.p, n, s);
  int64_t nzc = 0;
  CBG_HIP(hipMemcpyAsync(&nzc, pos.p + n, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  CBG_HIP(hipStreamSynchronize(s));
  tile_alloc_device(out, m, nn, n, nzc);
  hipLaunchKernelGGL(k_key_fill, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, keys, vals, pos.p, out.ir,
                     out.val, out.jc, out.cp);
  CBG_HIP(hipMemcpyAsync(out.cp + nzc, &n, sizeof(int64_t), hipMemcpyHostToDevice, s));
  CBG_HIP(hipStreamSynchronize(s));
}

static unsigned long long low_bits(int64_t maxval) {  // mask of the bits of values in [0, maxval]
  unsigned long long m = 0;
  while ((unsigned long long)maxval > m) m = (m << 1) | 1ull;
  return m;
}

void tile_transpose(const cbg_tile& T, cbg_tile& out, hipStream_t s) {
  out = cbg_tile{};
  out.on_device = 1;
  const int64_t n = T.nnz;
  if (n == 0) {
    tile_alloc_device(out, T.n, T.m, 0, 0);
    return;
  }
  DBuf<unsigned long long> k0(n);
  DBuf<double> v0(n);
  hipLaunchKernelGGL(k_transpose_keys, dim3((unsigned)((T.nzc * WAVE + 255) / 256)), dim3(256), 0, s, T.nzc, T.cp,
                     T.jc, T.ir, k0.p);
  CBG_HIP(hipMemcpyAsync(v0.p, T.val, sizeof(double) * n, hipMemcpyDeviceToDevice, s));
  // (row << 32 | col): SpTuples::SortRowBased (SpTuples.h:86-91) as a radix sort over the bits rows and columns use
  radix_sort_pairs(k0, v0, n, (low_bits(T.m - 1) << 32) | low_bits(T.n - 1), s);
  keys_to_tile(k0.p, v0.p, n, T.n, T.m, out, s);
}

// dim 0 (Column): x(i,j) op= v[j];  dim 1 (Row): x(i,j) op= v[i]
__global__ void k_dim_apply(int64_t nzc, const int64_t* __restrict__ cp, const int32_t* __restrict__ jc,
                            const int32_t* __restrict__ ir, double* __restrict__ val, const double* __restrict__ v,
                            int dim, int op) {
  const int64_t i = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / WAVE;
  if (i >= nzc) return;
  const double vc = dim == 0 ? v[jc[i]] : 0.0;
  for (int64_t q = cp[i] + lane_id(); q < cp[i + 1]; q += WAVE) {
    const double b = dim == 0 ? vc : v[ir[q]];
    const double a = val[q];
    val[q] = op == 0 ? a * b : op == 1 ? a + b : op == 2 ? fmin(a, b) : fmax(a, b);
  }
}

void tile_dim_apply(cbg_tile& t, int dim, const double* vec_host, int op, hipStream_t s) {
  const int64_t len = dim == 0 ? t.n : t.m;
  DBuf<double> v(std::max<int64_t>(len, 1));
  if (len) CBG_HIP(hipMemcpyAsync(v.p, vec_host, sizeof(double) * len, hipMemcpyHostToDevice, s));
  if (t.nzc > 0)
    hipLaunchKernelGGL(k_dim_apply, dim3((unsigned)((t.nzc * WAVE + 255) / 256)), dim3(256), 0, s, t.nzc, t.cp, t.jc,
                       t.ir, t.val, v.p, dim, op);
  CBG_HIP(hipStreamSynchronize(s));
}

// The restriction operator of genrestrict.m:11, sprand(n, n/order, order/n):
// every one of the n * n/order positions is a nonzero with probability
// order/n, so a fine row holds Poisson(1) nonzeros (about 37 % of the rows
// none) and a coarse column Poisson(order), at uniformly random columns, with
// values uniform in (0, 1].  MATLAB's generator cannot be reproduced; this one
// draws, from a counter-based hash of (seed, fine row i): the row's count k_i
// by inversion of the Poisson(1) CDF (a table of doubles, identical in the
// host restatement tests/helpers.py restriction_host), then for j < k_i the
// column c_ij = mix(h_i + (j+1) golden) mod nc and the value.  A column drawn
// twice in one row is one nonzero holding the sum (sparse() sums duplicates).
// Every grid cell generates its own tile (rows of its row block whose columns
// fall in its column block) without communication: the global T does not
// depend on the grid.
__constant__ double c_poisson1_cdf[12] = {
    0.36787944117144233, 0.7357588823428847, 0.9196986029286058, 0.9810118431238463,
    0.9963401531726563,  0.9994058151824183, 0.999916758850712,  0.9999897508033253,
    0.999998874797402,   0.9999998885745216, 0.9999999899522336, 0.9999999991683892};
__device__ __forceinline__ unsigned long long restrict_row_hash(unsigned long long seed, unsigned long long i) {
  return mix(seed ^ (i * 0xd1b54a32d192ed03ULL));
}
__device__ __forceinline__ int restrict_row_count(unsigned long long h) {
  const double u = (double)(mix(h ^ 0x5851f42d4c957f2dULL) >> 11) * (1.0 / 9007199254740992.0);  // [0, 1)
  int k = 0;
  while (k < 12 && u >= c_poisson1_cdf[k]) ++k;
  return k;
}
// entry j of fine row i: column and value
__device__ __forceinline__ unsigned long long restrict_entry_hash(unsigned long long h, int j) {
  return mix(h + (unsigned long long)(j + 1) * 0x9e3779b97f4a7c15ULL);
}
__global__ void k_restrict_count(int64_t r0, int64_t rows, int64_t c0, int64_t c1, int64_t nc,
                                 unsigned long long seed, int32_t* __restrict__ cnt) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t >= rows) return;
  const unsigned long long h = restrict_row_hash(seed, (unsigned long long)(r0 + t));
  const int k = restrict_row_count(h);
  int mine = 0;
  for (int j = 0; j < k; ++j) {
    const int64_t c = (int64_t)(restrict_entry_hash(h, j) % (unsigned long long)nc);
    mine += c >= c0 && c < c1;
  }
  cnt[t] = mine;
}
__global__ void k_restrict_fill(int64_t r0, int64_t rows, int64_t c0, int64_t c1, int64_t nc, unsigned long long seed,
                                const int64_t* __restrict__ pos, unsigned long long* __restrict__ key,
                                double* __restrict__ val) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t >= rows) return;
  const unsigned long long h = restrict_row_hash(seed, (unsigned long long)(r0 + t));
  const int k = restrict_row_count(h);
  int64_t o = pos[t];
  for (int j = 0; j < k; ++j) {
    const unsigned long long hj = restrict_entry_hash(h, j);
    const int64_t c = (int64_t)(hj % (unsigned long long)nc);
    if (c < c0 || c >= c1) continue;
    key[o] = ((unsigned long long)(c - c0) << 32) | (unsigned long long)t;
    val[o] = (double)((mix(hj) >> 11) + 1) * (1.0 / 9007199254740992.0);  // (0, 1]
    ++o;
  }
}

void restriction_tile(int scale, int order, uint64_t seed, int pr, int pc, int prow, int pcol, cbg_tile& out,
                      hipStream_t s) {
  const int64_t n = (int64_t)1 << scale, nc = n / order;
  // block distribution of SpParMat::Owner (SpParMat.cpp:5068-5097)
  const int64_t mper = n / pr, nper = nc / pc;
  const int64_t r0 = prow * mper, r1 = prow == pr - 1 ? n : r0 + mper;
  const int64_t c0 = pcol * nper, c1 = pcol == pc - 1 ? nc : c0 + nper;
  const int64_t rows = r1 - r0;
  out = cbg_tile{};
  out.on_device = 1;
  DBuf<int32_t> cnt(rows + 1);
  DBuf<int64_t> pos(rows + 1);
  const unsigned g = (unsigned)((rows + 255) / 256);
  hipLaunchKernelGGL(k_restrict_count, dim3(g), dim3(256), 0, s, r0, rows, c0, c1, nc, (unsigned long long)seed,
                     cnt.p);
  exclusive_scan_i32_to_i64(cnt.p, pos.p, rows, s);
  int64_t e = 0;
  CBG_HIP(hipMemcpyAsync(&e, pos.p + rows, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  CBG_HIP(hipStreamSynchronize(s));
  DBuf<unsigned long long> k0(std::max<int64_t>(e, 1)), uk(std::max<int64_t>(e, 1));
  DBuf<double> v0(std::max<int64_t>(e, 1)), uv(std::max<int64_t>(e, 1));
  if (e > 0)
    hipLaunchKernelGGL(k_restrict_fill, dim3(g), dim3(256), 0, s, r0, rows, c0, c1, nc, (unsigned long long)seed,
                       pos.p, k0.p, v0.p);
  // (column, row) order, then duplicates summed (sparse() of the drawn triples)
  radix_sort_pairs(k0, v0, e, (low_bits(c1 - c0 - 1) << 32) | low_bits(rows - 1), s);
  const int64_t u = reduce_by_key(k0.p, v0.p, e, CBG_PLUS_TIMES, uk.p, uv.p, s);
  keys_to_tile(uk.p, uv.p, u, rows, c1 - c0, out, s);
}

// SURVEY 8(d)'s random-valued inputs: every nonzero (i, j) of the global
// matrix gets U[-1, 1) from a counter hash of (seed, j, i) -- the R-MAT
// structure with values whose sums are not exact in any order (and not f32,
// so the slab kernels read A's f64 values).  (k >> 11) * 2^-52 - 1 is exact
// in double: tests/helpers.py random_values_host gives the same bits.
__device__ __forceinline__ double random_value(unsigned long long seed, unsigned long long row, unsigned long long col) {
  const unsigned long long z = mix(((col << 32) | row) ^ (seed * 0xd1b54a32d192ed03ULL));
  return (double)(z >> 11) * (1.0 / 4503599627370496.0) - 1.0;
}
__global__ void k_random_values(int64_t nzc, const int64_t* __restrict__ cp, const int32_t* __restrict__ jc,
                                const int32_t* __restrict__ ir, double* __restrict__ val, unsigned long long seed,
                                int64_t roff, int64_t coff) {
  const int64_t i = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / WAVE;
  if (i >= nzc) return;
  const unsigned long long c = (unsigned long long)(jc[i] + coff);
  for (int64_t q = cp[i] + lane_id(); q < cp[i + 1]; q += WAVE)
    val[q] = random_value(seed, (unsigned long long)(ir[q] + roff), c);
}
void tile_random_values(cbg_tile& t, uint64_t seed, int64_t roff, int64_t coff, hipStream_t s) {
  if (t.nzc > 0)
    hipLaunchKernelGGL(k_random_values, dim3((unsigned)((t.nzc * WAVE + 255) / 256)), dim3(256), 0, s, t.nzc, t.cp,
                       t.jc, t.ir, t.val, (unsigned long long)seed, roff, coff);
  CBG_HIP(hipStreamSynchronize(s));
}

// ---------------------------------------------------------------- HBM copy roofline
// The measured side of the roofline: a streaming copy, 16 B per lane, each
// lane keeping 4 loads in flight before its stores (MI355X_MICROARCH.md:
// 6.29 TB/s for a float4 copy).  Bytes moved = 2 x the buffer (read + write).
__global__ __launch_bounds__(256) void k_copy16(const uint4* __restrict__ src, uint4* __restrict__ dst, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n; i += 4 * stride) {
    const uint4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
    dst[i] = a;
    dst[i + stride] = b;
    dst[i + 2 * stride] = c;
    dst[i + 3 * stride] = d;
  }
  for (; i < n; i += stride) dst[i] = src[i];
}

// the same with nontemporal loads and stores (streamed once: keep them out of L2/MALL)
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_copy16_nt(const uint4* __restrict__ src_, uint4* __restrict__ dst_,
                                                   int64_t n) {
  const v4u* __restrict__ src = reinterpret_cast<const v4u*>(src_);
  v4u* __restrict__ dst = reinterpret_cast<v4u*>(dst_);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n; i += 4 * stride) {
    const v4u a = __builtin_nontemporal_load(src + i), b = __builtin_nontemporal_load(src + i + stride),
              c = __builtin_nontemporal_load(src + i + 2 * stride),
              d = __builtin_nontemporal_load(src + i + 3 * stride);
    __builtin_nontemporal_store(a, dst + i);
    __builtin_nontemporal_store(b, dst + i + stride);
    __builtin_nontemporal_store(c, dst + i + 2 * stride);
    __builtin_nontemporal_store(d, dst + i + 3 * stride);
  }
  for (; i < n; i += stride) __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

// one block per 256 x U consecutive 16-B elements, U loads in flight per lane
// (no grid-stride loop: the launch itself streams over the buffer)
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_copy16_flat(const uint4* __restrict__ src_, uint4* __restrict__ dst_,
                                                     int64_t n) {
  const v4u* __restrict__ src = reinterpret_cast<const v4u*>(src_);
  v4u* __restrict__ dst = reinterpret_cast<v4u*>(dst_);
  const int64_t i0 = (int64_t)blockIdx.x * (256 * U) + threadIdx.x;
  v4u x[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = i0 + u * 256;
    if (i < n) x[u] = NT ? __builtin_nontemporal_load(src + i) : src[i];
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = i0 + u * 256;
    if (i < n) {
      if (NT) __builtin_nontemporal_store(x[u], dst + i);
      else dst[i] = x[u];
    }
  }
}

// The measured side of the roofline: the best of several 16-B-per-lane copy
// shapes (grid-stride with 4 loads in flight, nontemporal or not; one launch
// streaming the buffer with 1 / 4 / 8 loads per lane), swept on the first call
// and the winner reused (MI355X_MICROARCH.md: 6.29 TB/s for a float4 copy).
// Bytes moved = 2 x the buffer.
// WRITE_SIZE calibration: n stores of W bytes, lane-consecutive, grid-stride
template <int W>
__global__ __launch_bounds__(256) void k_store_probe(char* __restrict__ dst, int64_t n) {
  using T = typename std::conditional<W == 4, int, long long>::type;
  T* d = reinterpret_cast<T*>(dst);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    d[i] = (T)i;
}
void store_probe(int64_t bytes, int width) {
  DBuf<char> buf(bytes);
  const int64_t n = bytes / width;
  const unsigned g = (unsigned)std::min<int64_t>((n + 255) / 256, 256 * 64);
  if (width == 4) hipLaunchKernelGGL(k_store_probe<4>, dim3(g), dim3(256), 0, nullptr, buf.p, n);
  else hipLaunchKernelGGL(k_store_probe<8>, dim3(g), dim3(256), 0, nullptr, buf.p, n);
  CBG_HIP(hipDeviceSynchronize());
}

double hbm_copy_gbps(int64_t bytes, int reps) {
  const int64_t n = std::max<int64_t>(bytes / 16, 1);
  DBuf<uint4> ba(n), bb(n);  // from the pool (it drops its cache and retries when the device is full)
  uint4 *a = ba.p, *b = bb.p;
  CBG_HIP(hipMemset(a, 1, n * 16));
  CBG_HIP(hipMemset(b, 0, n * 16));
  CBG_HIP(hipDeviceSynchronize());
  int dev = 0, cus = 256;
  CBG_HIP(hipGetDevice(&dev));
  CBG_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  hipStream_t st = nullptr;
  CBG_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  constexpr int NV = 8;
  auto launch = [&](int v, const uint4* src, uint4* dst) {
    auto flat = [&](int u) { return dim3((unsigned)((n + 256 * u - 1) / (256 * u))); };
    switch (v) {
      case 0: hipLaunchKernelGGL(k_copy16_nt, dim3(cus * 128), dim3(256), 0, st, src, dst, n); break;
      case 1: hipLaunchKernelGGL(k_copy16, dim3(cus * 128), dim3(256), 0, st, src, dst, n); break;
      case 2: hipLaunchKernelGGL((k_copy16_flat<1, false>), flat(1), dim3(256), 0, st, src, dst, n); break;
      case 3: hipLaunchKernelGGL((k_copy16_flat<1, true>), flat(1), dim3(256), 0, st, src, dst, n); break;
      case 4: hipLaunchKernelGGL((k_copy16_flat<4, false>), flat(4), dim3(256), 0, st, src, dst, n); break;
      case 5: hipLaunchKernelGGL((k_copy16_flat<4, true>), flat(4), dim3(256), 0, st, src, dst, n); break;
      case 6: hipLaunchKernelGGL((k_copy16_flat<8, false>), flat(8), dim3(256), 0, st, src, dst, n); break;
      default: hipLaunchKernelGGL((k_copy16_flat<8, true>), flat(8), dim3(256), 0, st, src, dst, n); break;
    }
  };
  hipEvent_t e0, e1;
  CBG_HIP(hipEventCreate(&e0));
  CBG_HIP(hipEventCreate(&e1));
  auto measure = [&](int v, int r_) {
    launch(v, a, b);  // warm-up
    CBG_HIP(hipEventRecord(e0, st));
    for (int r = 0; r < r_; ++r) launch(v, (r & 1) ? b : a, (r & 1) ? a : b);
    CBG_HIP(hipEventRecord(e1, st));
    CBG_HIP(hipEventSynchronize(e1));
    float ms = 0.f;
    CBG_HIP(hipEventElapsedTime(&ms, e0, e1));
    return 2.0 * 16.0 * (double)n * r_ / (ms * 1e-3) / 1e9;
  };
  static int best = -1;
  double gbps = 0.0;
  if (best < 0) {
    for (int v = 0; v < NV; ++v) {
      const double g = measure(v, std::max(2, reps / 2));
      if (g > gbps) {
        gbps = g;
        best = v;
      }
    }
  }
  gbps = std::max(gbps, measure(best, reps));
  CBG_HIP(hipEventDestroy(e0));
  CBG_HIP(hipEventDestroy(e1));
  CBG_HIP(hipStreamDestroy(st));  // (synchronized above: the pool may reuse a and b)
  return gbps;
}

}  // namespace cbg
