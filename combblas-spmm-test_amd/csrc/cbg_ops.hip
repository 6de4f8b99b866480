// cbg_ops.hip -- tile operations of the Galerkin triple-product path
// (reference ReleaseTests/GalerkinNew.cpp:96-153):
//   tile_transpose     SpDCCols::Transpose (SpDCCols.cpp:853-873): DCSC of T^T
//   tile_dim_apply     SpParMat::DimApply (SpParMat.cpp:801): x(i,j) = op(x(i,j), v[j] or v[i])
//   restriction_tile   the restriction operator T of the multigrid driver
//                      (mfiles/genrestrict.m: n x n/order, ~n nonzeros, values in (0,1])
#include <algorithm>

#include <hipcub/hipcub.hpp>

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

static void sort_pairs(DBuf<unsigned long long>& k0, DBuf<double>& v0, DBuf<unsigned long long>& k1,
                       DBuf<double>& v1, int64_t n, hipStream_t s) {
  if (n >= (int64_t)INT32_MAX) throw HipError("transpose: nnz must stay below 2^31", CBG_ERR_NOTSUPPORTED);
  size_t bytes = 0;
  CBG_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, k0.p, k1.p, v0.p, v1.p, (int)n, 0, 64, s));
  DBuf<char> tmp(bytes);
  CBG_HIP(hipcub::DeviceRadixSort::SortPairs(tmp.p, bytes, k0.p, k1.p, v0.p, v1.p, (int)n, 0, 64, s));
}

void tile_transpose(const cbg_tile& T, cbg_tile& out, hipStream_t s) {
  out = cbg_tile{};
  out.on_device = 1;
  const int64_t n = T.nnz;
  if (n == 0) {
    tile_alloc_device(out, T.n, T.m, 0, 0);
    return;
  }
  DBuf<unsigned long long> k0(n), k1(n);
  DBuf<double> v0(n), v1(n);
  hipLaunchKernelGGL(k_transpose_keys, dim3((unsigned)((T.nzc * WAVE + 255) / 256)), dim3(256), 0, s, T.nzc, T.cp,
                     T.jc, T.ir, k0.p);
  CBG_HIP(hipMemcpyAsync(v0.p, T.val, sizeof(double) * n, hipMemcpyDeviceToDevice, s));
  sort_pairs(k0, v0, k1, v1, n, s);
  keys_to_tile(k1.p, v1.p, n, T.n, T.m, out, s);
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

// T(i, c(i)) = v(i) for the fine rows i of this tile's row block whose
// aggregate c(i) = mix(seed, i) mod nc falls in its column block; keys
// (col << 32 | row) of the others are all-ones and sort to the end
__global__ void k_restrict_keys(int64_t r0, int64_t rows, int64_t c0, int64_t c1, int64_t nc, unsigned long long seed,
                                unsigned long long* __restrict__ key, double* __restrict__ val) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t >= rows) return;
  const unsigned long long i = (unsigned long long)(r0 + t);
  const unsigned long long h = mix(seed ^ (i * 0xd1b54a32d192ed03ULL));
  const int64_t c = (int64_t)(h % (unsigned long long)nc);
  const bool mine = c >= c0 && c < c1;
  key[t] = mine ? ((unsigned long long)(c - c0) << 32) | (unsigned long long)t : ~0ULL;
  val[t] = (double)((mix(h) >> 11) + 1) * (1.0 / 9007199254740992.0);  // (0, 1]
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
  DBuf<unsigned long long> k0(rows), k1(rows);
  DBuf<double> v0(rows), v1(rows);
  hipLaunchKernelGGL(k_restrict_keys, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, s, r0, rows, c0, c1, nc,
                     (unsigned long long)seed, k0.p, v0.p);
  sort_pairs(k0, v0, k1, v1, rows, s);
  // kept entries are the prefix of keys != ~0
  int64_t lo = 0, hi = rows;
  while (lo < hi) {  // first all-ones key (binary search on the host over device reads)
    const int64_t mid = (lo + hi) / 2;
    unsigned long long k = 0;
    CBG_HIP(hipMemcpyAsync(&k, k1.p + mid, sizeof(k), hipMemcpyDeviceToHost, s));
    CBG_HIP(hipStreamSynchronize(s));
    if (k == ~0ULL) hi = mid; else lo = mid + 1;
  }
  keys_to_tile(k1.p, v1.p, lo, rows, c1 - c0, out, s);
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

double hbm_copy_gbps(int64_t bytes, int reps) {
  const int64_t n = std::max<int64_t>(bytes / 16, 1);
  uint4 *a = nullptr, *b = nullptr;
  // from the pool (no hipMalloc: after a large multiply the pool's cache may
  // hold most of the device; pool().alloc drops the cache and retries)
  DBuf<uint4> ba(n), bb(n);
  a = ba.p;
  b = bb.p;
  CBG_HIP(hipMemset(a, 1, n * 16));
  CBG_HIP(hipMemset(b, 0, n * 16));
  CBG_HIP(hipDeviceSynchronize());
  int dev = 0, cus = 256;
  CBG_HIP(hipGetDevice(&dev));
  CBG_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  static const char* eg = getenv("CBG_COPY_BLOCKS_PER_CU");  // tuning knob
  const int grid = cus * (eg ? atoi(eg) : 128);  // 8: 4.7, 32: 5.0, 128: 5.3-5.5 TB/s (nt)
  static const char* em = getenv("CBG_COPY_NT");
  const bool nt = !em || atoi(em) != 0;
  hipStream_t st = nullptr;
  CBG_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  auto launch = [&](const uint4* src, uint4* dst) {
    if (nt)
      hipLaunchKernelGGL(k_copy16_nt, dim3(grid), dim3(256), 0, st, src, dst, n);
    else
      hipLaunchKernelGGL(k_copy16, dim3(grid), dim3(256), 0, st, src, dst, n);
  };
  hipEvent_t e0, e1;
  CBG_HIP(hipEventCreate(&e0));
  CBG_HIP(hipEventCreate(&e1));
  launch(a, b);  // warm-up
  CBG_HIP(hipEventRecord(e0, st));
  for (int r = 0; r < reps; ++r) launch((r & 1) ? b : a, (r & 1) ? a : b);
  CBG_HIP(hipEventRecord(e1, st));
  CBG_HIP(hipEventSynchronize(e1));
  float ms = 0.f;
  CBG_HIP(hipEventElapsedTime(&ms, e0, e1));
  CBG_HIP(hipEventDestroy(e0));
  CBG_HIP(hipEventDestroy(e1));
  CBG_HIP(hipStreamDestroy(st));  // (synchronized above: the pool may reuse a and b)
  return 2.0 * 16.0 * (double)n * reps / (ms * 1e-3) / 1e9;
}

}  // namespace cbg
