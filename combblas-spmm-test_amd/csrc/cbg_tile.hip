// cbg_tile.hip -- device DCSC tiles: pool allocator, scans, split/concat, digest.
//
// Split/concat replace the reference's tile surgery on the DoubleBuff path:
//   SpDCCols::Split / Dcsc::Split      SpDCCols.cpp:905-930, dcsc.cpp:1100-1138
//   B row split by Transpose/Split/Transpose (ParFriends.h:824-829) -> tile_split_rows
//   SpDCCols::Merge / Dcsc::Merge      SpDCCols.cpp:1194-1223, dcsc.cpp:1204-1230
#include "cbg_device.h"
#include "cbg_internal.h"

namespace cbg {

// ----------------------------------------------------------------------------
// caching device allocator
// ----------------------------------------------------------------------------
static size_t round_bytes(size_t b) {
  if (b < 4096) return 4096;
  if (b < (2u << 20)) {
    size_t r = 4096;
    while (r < b) r <<= 1;
    return r;
  }
  const size_t g = 2u << 20;
  return (b + g - 1) / g * g;
}

void* DevicePool::alloc(size_t bytes) {
  const size_t rb = round_bytes(bytes);
  {
    std::lock_guard<std::mutex> lk(mu_);
    // best fit among cached blocks no larger than 2x the request
    auto it = free_.lower_bound(rb);
    if (it != free_.end() && it->first <= 2 * rb + (2u << 20)) {
      void* p = it->second;
      size_t sz = it->first;
      free_.erase(it);
      cached_ -= sz;
      live_[p] = sz;
      in_use_ += sz;
      return p;
    }
  }
  void* p = nullptr;
  hipError_t e = hipMalloc(&p, rb);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    trim();  // drop the cache and retry once
    e = hipMalloc(&p, rb);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      throw HipError("device allocation of " + std::to_string(rb) + " bytes failed (" + hipGetErrorString(e) + ")",
                     CBG_ERR_OOM);
    }
  }
  std::lock_guard<std::mutex> lk(mu_);
  live_[p] = rb;
  in_use_ += rb;
  return p;
}

void DevicePool::free(void* p) {
  if (!p) return;
  std::lock_guard<std::mutex> lk(mu_);
  auto it = live_.find(p);
  if (it == live_.end()) return;
  free_.emplace(it->second, p);
  cached_ += it->second;
  in_use_ -= it->second;
  live_.erase(it);
}

void DevicePool::trim() {
  std::lock_guard<std::mutex> lk(mu_);
  for (auto& kv : free_) (void)hipFree(kv.second);
  free_.clear();
  cached_ = 0;
}

DevicePool& pool() {
  static DevicePool* p = new DevicePool();  // leaked on purpose: outlives static destructors
  return *p;
}

// ----------------------------------------------------------------------------
// scans (prefixsum, mtSpGEMM.h:23-70)
// ----------------------------------------------------------------------------
constexpr int SCAN_BS = 256, SCAN_IPT = 8, SCAN_TILE = SCAN_BS * SCAN_IPT;

template <class TI>
__global__ __launch_bounds__(SCAN_BS) void k_scan_tile(const TI* __restrict__ in, int64_t n, int64_t* __restrict__ out,
                                                       int64_t* __restrict__ tile_sum) {
  __shared__ long long wsum[SCAN_BS / WAVE + 1];
  const int tid = threadIdx.x;
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)tid * SCAN_IPT;
  long long v[SCAN_IPT];
  long long s = 0;
#pragma unroll
  for (int k = 0; k < SCAN_IPT; ++k) {
    v[k] = (base + k < n) ? (long long)in[base + k] : 0;
    s += v[k];
  }
  long long incl = wave_incl_scan64(s);
  const int w = tid / WAVE;
  if (lane_id() == WAVE - 1) wsum[w] = incl;
  __syncthreads();
  if (tid == 0) {
    long long a = 0;
    for (int i = 0; i < SCAN_BS / WAVE; ++i) {
      long long t = wsum[i];
      wsum[i] = a;
      a += t;
    }
    wsum[SCAN_BS / WAVE] = a;
  }
  __syncthreads();
  long long run = wsum[w] + incl - s;
#pragma unroll
  for (int k = 0; k < SCAN_IPT; ++k) {
    if (base + k < n) out[base + k] = run;
    run += v[k];
  }
  if (tid == 0) tile_sum[blockIdx.x] = wsum[SCAN_BS / WAVE];
}

__global__ void k_scan_add(int64_t* __restrict__ out, int64_t n, const int64_t* __restrict__ toff) {
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < n) out[i] += toff[i / SCAN_TILE];
}

template <class TI>
static void scan_impl(const TI* in, int64_t* out, int64_t n, hipStream_t s) {
  const int64_t nt = (n + SCAN_TILE - 1) / SCAN_TILE;
  if (nt <= 1) {
    if (n == 0) {
      CBG_HIP(hipMemsetAsync(out, 0, sizeof(int64_t), s));
      return;
    }
    hipLaunchKernelGGL(k_scan_tile<TI>, dim3(1), dim3(SCAN_BS), 0, s, in, n, out, out + n);
    return;
  }
  DBuf<int64_t> sums(nt), offs(nt + 1);
  hipLaunchKernelGGL(k_scan_tile<TI>, dim3((unsigned)nt), dim3(SCAN_BS), 0, s, in, n, out, sums.p);
  scan_impl<int64_t>(sums.p, offs.p, nt, s);
  hipLaunchKernelGGL(k_scan_add, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, out, n, offs.p);
  CBG_HIP(hipMemcpyAsync(out + n, offs.p + nt, sizeof(int64_t), hipMemcpyDeviceToDevice, s));
  CBG_HIP(hipStreamSynchronize(s));  // sums/offs go back to the pool
}

void exclusive_scan_i64(const int64_t* in, int64_t* out, int64_t n, hipStream_t s) { scan_impl<int64_t>(in, out, n, s); }
void exclusive_scan_i32_to_i64(const int32_t* in, int64_t* out, int64_t n, hipStream_t s) {
  scan_impl<int32_t>(in, out, n, s);
}

// ----------------------------------------------------------------------------
// tile allocation
// ----------------------------------------------------------------------------
void tile_alloc_device(cbg_tile& t, int64_t m, int64_t n, int64_t nnz, int64_t nzc) {
  t.m = m;
  t.n = n;
  t.nnz = nnz;
  t.nzc = nzc;
  t.on_device = 1;
  t.cp = static_cast<int64_t*>(pool().alloc(sizeof(int64_t) * (nzc + 1)));
  t.jc = static_cast<int32_t*>(pool().alloc(sizeof(int32_t) * std::max<int64_t>(nzc, 1)));
  t.ir = static_cast<int32_t*>(pool().alloc(sizeof(int32_t) * std::max<int64_t>(nnz, 1)));
  t.val = static_cast<double*>(pool().alloc(sizeof(double) * std::max<int64_t>(nnz, 1)));
  if (nzc == 0) CBG_HIP(hipMemset(t.cp, 0, sizeof(int64_t)));
}

void tile_free_device(cbg_tile& t) {
  if (t.on_device) {
    pool().free(t.cp);
    pool().free(t.jc);
    pool().free(t.ir);
    pool().free(t.val);
  }
  t.cp = nullptr;
  t.jc = nullptr;
  t.ir = nullptr;
  t.val = nullptr;
  t.nnz = t.nzc = 0;
}

// ----------------------------------------------------------------------------
// column split (Dcsc::Split: lower_bound on jc, re-base the right part)
// ----------------------------------------------------------------------------
__global__ void k_lower_bound_jc(const int32_t* __restrict__ jc, int64_t nzc, int64_t key, int64_t* __restrict__ out) {
  int64_t lo = 0, hi = nzc;
  while (lo < hi) {
    int64_t mid = (lo + hi) / 2;
    if (jc[mid] < key) lo = mid + 1; else hi = mid;
  }
  *out = lo;
}
__global__ void k_copy_cols(int64_t cnt, const int32_t* __restrict__ jc, const int64_t* __restrict__ cp,
                            int64_t jc_sub, int64_t cp_sub, int32_t* __restrict__ ojc, int64_t* __restrict__ ocp) {
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < cnt) ojc[i] = (int32_t)(jc[i] - jc_sub);
  if (i <= cnt) ocp[i] = cp[i] - cp_sub;
}

void tile_split_cols(const cbg_tile& T, int64_t cut, cbg_tile& L, cbg_tile& R, hipStream_t s) {
  int64_t pos = 0, cpos[2] = {0, 0};
  if (T.nzc > 0) {
    DBuf<int64_t> d(1);
    hipLaunchKernelGGL(k_lower_bound_jc, dim3(1), dim3(1), 0, s, T.jc, T.nzc, cut, d.p);
    CBG_HIP(hipMemcpyAsync(&pos, d.p, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    CBG_HIP(hipStreamSynchronize(s));
    CBG_HIP(hipMemcpyAsync(&cpos[0], T.cp + pos, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    CBG_HIP(hipStreamSynchronize(s));
  }
  const int64_t lnnz = cpos[0], rnnz = T.nnz - cpos[0];
  tile_alloc_device(L, T.m, cut, lnnz, pos);
  tile_alloc_device(R, T.m, T.n - cut, rnnz, T.nzc - pos);
  if (T.nzc > 0) {
    hipLaunchKernelGGL(k_copy_cols, dim3((unsigned)((pos + 256) / 256)), dim3(256), 0, s, pos, T.jc, T.cp, (int64_t)0,
                       (int64_t)0, L.jc, L.cp);
    hipLaunchKernelGGL(k_copy_cols, dim3((unsigned)((T.nzc - pos + 256) / 256)), dim3(256), 0, s, T.nzc - pos,
                       T.jc + pos, T.cp + pos, cut, cpos[0], R.jc, R.cp);
    if (lnnz) {
      CBG_HIP(hipMemcpyAsync(L.ir, T.ir, sizeof(int32_t) * lnnz, hipMemcpyDeviceToDevice, s));
      CBG_HIP(hipMemcpyAsync(L.val, T.val, sizeof(double) * lnnz, hipMemcpyDeviceToDevice, s));
    }
    if (rnnz) {
      CBG_HIP(hipMemcpyAsync(R.ir, T.ir + lnnz, sizeof(int32_t) * rnnz, hipMemcpyDeviceToDevice, s));
      CBG_HIP(hipMemcpyAsync(R.val, T.val + lnnz, sizeof(double) * rnnz, hipMemcpyDeviceToDevice, s));
    }
  }
  CBG_HIP(hipStreamSynchronize(s));
}

// ----------------------------------------------------------------------------
// row split: per column, rows < cut go to Top, rows >= cut (re-based) to Bot
// ----------------------------------------------------------------------------
__global__ void k_rowsplit_count(int64_t nzc, const int64_t* __restrict__ cp, const int32_t* __restrict__ ir, int cut,
                                 int64_t* __restrict__ ntop, int64_t* __restrict__ nbot, int64_t* __restrict__ ftop,
                                 int64_t* __restrict__ fbot) {
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= nzc) return;
  const int a = (int)cp[i], b = (int)cp[i + 1];
  const int k = lower_bound_g(ir, a, b, cut) - a;
  ntop[i] = k;
  nbot[i] = (b - a) - k;
  ftop[i] = k > 0;
  fbot[i] = (b - a - k) > 0;
}
__global__ void k_rowsplit_copy(int64_t nzc, const int64_t* __restrict__ cp, const int32_t* __restrict__ jc,
                                const int32_t* __restrict__ ir, const double* __restrict__ val, int cut,
                                const int64_t* __restrict__ otop, const int64_t* __restrict__ obot,
                                const int64_t* __restrict__ ctop, const int64_t* __restrict__ cbot,
                                int32_t* __restrict__ tjc, int64_t* __restrict__ tcp, int32_t* __restrict__ tir,
                                double* __restrict__ tval, int32_t* __restrict__ bjc, int64_t* __restrict__ bcp,
                                int32_t* __restrict__ bir, double* __restrict__ bval) {
  const int64_t i = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / WAVE;
  if (i >= nzc) return;
  const int lane = lane_id();
  const int64_t a = cp[i], b = cp[i + 1];
  const int64_t k = otop[i + 1] - otop[i];
  if (k > 0) {
    if (lane == 0) {
      tjc[ctop[i]] = jc[i];
      tcp[ctop[i]] = otop[i];
    }
    for (int64_t q = lane; q < k; q += WAVE) {
      tir[otop[i] + q] = ir[a + q];
      tval[otop[i] + q] = val[a + q];
    }
  }
  const int64_t r = (b - a) - k;
  if (r > 0) {
    if (lane == 0) {
      bjc[cbot[i]] = jc[i];
      bcp[cbot[i]] = obot[i];
    }
    for (int64_t q = lane; q < r; q += WAVE) {
      bir[obot[i] + q] = ir[a + k + q] - cut;
      bval[obot[i] + q] = val[a + k + q];
    }
  }
}

void tile_split_rows(const cbg_tile& T, int64_t cut, cbg_tile& Top, cbg_tile& Bot, hipStream_t s) {
  const int64_t nz = T.nzc;
  if (nz == 0) {
    tile_alloc_device(Top, cut, T.n, 0, 0);
    tile_alloc_device(Bot, T.m - cut, T.n, 0, 0);
    return;
  }
  DBuf<int64_t> ntop(nz + 1), nbot(nz + 1), ftop(nz + 1), fbot(nz + 1);
  DBuf<int64_t> otop(nz + 1), obot(nz + 1), ctop(nz + 1), cbot(nz + 1);
  hipLaunchKernelGGL(k_rowsplit_count, dim3((unsigned)((nz + 255) / 256)), dim3(256), 0, s, nz, T.cp, T.ir, (int)cut,
                     ntop.p, nbot.p, ftop.p, fbot.p);
  exclusive_scan_i64(ntop.p, otop.p, nz, s);
  exclusive_scan_i64(nbot.p, obot.p, nz, s);
  exclusive_scan_i64(ftop.p, ctop.p, nz, s);
  exclusive_scan_i64(fbot.p, cbot.p, nz, s);
  int64_t h[4];
  CBG_HIP(hipMemcpyAsync(&h[0], otop.p + nz, 8, hipMemcpyDeviceToHost, s));
  CBG_HIP(hipMemcpyAsync(&h[1], obot.p + nz, 8, hipMemcpyDeviceToHost, s));
  CBG_HIP(hipMemcpyAsync(&h[2], ctop.p + nz, 8, hipMemcpyDeviceToHost, s));
  CBG_HIP(hipMemcpyAsync(&h[3], cbot.p + nz, 8, hipMemcpyDeviceToHost, s));
  CBG_HIP(hipStreamSynchronize(s));
  tile_alloc_device(Top, cut, T.n, h[0], h[2]);
  tile_alloc_device(Bot, T.m - cut, T.n, h[1], h[3]);
  hipLaunchKernelGGL(k_rowsplit_copy, dim3((unsigned)((nz * WAVE + 255) / 256)), dim3(256), 0, s, nz, T.cp, T.jc, T.ir,
                     T.val, (int)cut, otop.p, obot.p, ctop.p, cbot.p, Top.jc, Top.cp, Top.ir, Top.val, Bot.jc, Bot.cp,
                     Bot.ir, Bot.val);
  CBG_HIP(hipMemcpyAsync(Top.cp + h[2], &h[0], 8, hipMemcpyHostToDevice, s));
  CBG_HIP(hipMemcpyAsync(Bot.cp + h[3], &h[1], 8, hipMemcpyHostToDevice, s));
  CBG_HIP(hipStreamSynchronize(s));
}

// ----------------------------------------------------------------------------
// concatenation along columns (disjoint, ascending column blocks)
// ----------------------------------------------------------------------------
__global__ void k_cat_cols(int64_t cnt, const int32_t* __restrict__ jc, const int64_t* __restrict__ cp, int64_t jadd,
                           int64_t cadd, int32_t* __restrict__ ojc, int64_t* __restrict__ ocp) {
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < cnt) {
    ojc[i] = (int32_t)(jc[i] + jadd);
    ocp[i] = cp[i] + cadd;
  }
}

void tile_concat_cols(const std::vector<cbg_tile>& parts, const std::vector<int64_t>& col_off, int64_t m, int64_t n,
                      cbg_tile& out, hipStream_t s) {
  int64_t nnz = 0, nzc = 0;
  for (auto& p : parts) {
    nnz += p.nnz;
    nzc += p.nzc;
  }
  tile_alloc_device(out, m, n, nnz, nzc);
  int64_t e = 0, c = 0;
  for (size_t k = 0; k < parts.size(); ++k) {
    const cbg_tile& p = parts[k];
    if (p.nzc > 0)
      hipLaunchKernelGGL(k_cat_cols, dim3((unsigned)((p.nzc + 255) / 256)), dim3(256), 0, s, p.nzc, p.jc, p.cp,
                         col_off[k], e, out.jc + c, out.cp + c);
    if (p.nnz > 0) {
      CBG_HIP(hipMemcpyAsync(out.ir + e, p.ir, sizeof(int32_t) * p.nnz, hipMemcpyDeviceToDevice, s));
      CBG_HIP(hipMemcpyAsync(out.val + e, p.val, sizeof(double) * p.nnz, hipMemcpyDeviceToDevice, s));
    }
    e += p.nnz;
    c += p.nzc;
  }
  CBG_HIP(hipMemcpyAsync(out.cp + nzc, &nnz, sizeof(int64_t), hipMemcpyHostToDevice, s));
  CBG_HIP(hipStreamSynchronize(s));
}

// ----------------------------------------------------------------------------
// concatenation along rows (parts share the column space; row blocks ascending)
// ----------------------------------------------------------------------------
__global__ void k_rowcat_count(int64_t nzc, const int32_t* __restrict__ jc, const int64_t* __restrict__ cp,
                               int64_t* __restrict__ len) {
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < nzc) len[jc[i]] += cp[i + 1] - cp[i];  // one part per launch: no two threads share jc[i]
}
__global__ void k_flag_nonzero(int64_t n, const int64_t* __restrict__ len, int64_t* __restrict__ flag) {
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < n) flag[i] = len[i] > 0;
}
__global__ void k_rowcat_cols(int64_t n, const int64_t* __restrict__ len, const int64_t* __restrict__ pos,
                              const int64_t* __restrict__ off, int32_t* __restrict__ jc, int64_t* __restrict__ cp) {
  int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (j < n && len[j] > 0) {
    jc[pos[j]] = (int32_t)j;
    cp[pos[j]] = off[j];
  }
}
__global__ void k_rowcat_copy(int64_t nzc, const int32_t* __restrict__ jc, const int64_t* __restrict__ cp,
                              const int32_t* __restrict__ ir, const double* __restrict__ val, int64_t roff,
                              int64_t* __restrict__ fill, int32_t* __restrict__ oir, double* __restrict__ oval) {
  const int64_t i = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / WAVE;
  if (i >= nzc) return;
  const int64_t a = cp[i], b = cp[i + 1], j = jc[i];
  const int64_t dst = fill[j];
  for (int64_t q = a + lane_id(); q < b; q += WAVE) {
    oir[dst + (q - a)] = (int32_t)(ir[q] + roff);
    oval[dst + (q - a)] = val[q];
  }
  __builtin_amdgcn_wave_barrier();
  if (lane_id() == 0) fill[j] = dst + (b - a);
}

void tile_concat_rows(const std::vector<cbg_tile>& parts, const std::vector<int64_t>& row_off, int64_t m, int64_t n,
                      cbg_tile& out, hipStream_t s) {
  DBuf<int64_t> len(n + 1), flag(n + 1), pos(n + 1), off(n + 1);
  CBG_HIP(hipMemsetAsync(len.p, 0, sizeof(int64_t) * (n + 1), s));
  int64_t nnz = 0;
  for (auto& p : parts) {
    nnz += p.nnz;
    if (p.nzc > 0)
      hipLaunchKernelGGL(k_rowcat_count, dim3((unsigned)((p.nzc + 255) / 256)), dim3(256), 0, s, p.nzc, p.jc, p.cp,
                         len.p);
  }
  hipLaunchKernelGGL(k_flag_nonzero, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, len.p, flag.p);
  exclusive_scan_i64(flag.p, pos.p, n, s);
  exclusive_scan_i64(len.p, off.p, n, s);
  int64_t nzc = 0;
  CBG_HIP(hipMemcpyAsync(&nzc, pos.p + n, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  CBG_HIP(hipStreamSynchronize(s));
  tile_alloc_device(out, m, n, nnz, nzc);
  hipLaunchKernelGGL(k_rowcat_cols, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, len.p, pos.p, off.p, out.jc,
                     out.cp);
  CBG_HIP(hipMemcpyAsync(out.cp + nzc, &nnz, sizeof(int64_t), hipMemcpyHostToDevice, s));
  // `off` doubles as the running fill pointer per column
  for (size_t k = 0; k < parts.size(); ++k) {
    const cbg_tile& p = parts[k];
    if (p.nzc > 0)
      hipLaunchKernelGGL(k_rowcat_copy, dim3((unsigned)((p.nzc * WAVE + 255) / 256)), dim3(256), 0, s, p.nzc, p.jc,
                         p.cp, p.ir, p.val, row_off[k], off.p, out.ir, out.val);
  }
  CBG_HIP(hipStreamSynchronize(s));
}

// ----------------------------------------------------------------------------
// digest (tests/golden/make_golden.py definition)
// ----------------------------------------------------------------------------
__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
__global__ void k_digest(int64_t nzc, const int64_t* __restrict__ cp, const int32_t* __restrict__ jc,
                         const int32_t* __restrict__ ir, const double* __restrict__ val, int64_t roff, int64_t coff,
                         unsigned long long* __restrict__ acc, double* __restrict__ vsum) {
  const int64_t i = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / WAVE;
  if (i >= nzc) return;
  const unsigned long long col = (unsigned long long)(jc[i] + coff);
  unsigned long long hs = 0, hv = 0;
  double vs = 0.0;
  for (int64_t q = cp[i] + lane_id(); q < cp[i + 1]; q += WAVE) {
    const unsigned long long h = mix64((col << 32) | (unsigned long long)(ir[q] + roff));
    const double v = val[q];
    hs += h;
    hv += h * mix64(__double_as_longlong(v));
    vs += v;
  }
#pragma unroll
  for (int d = WAVE / 2; d > 0; d >>= 1) {
    hs += __shfl_xor(hs, d, WAVE);
    hv += __shfl_xor(hv, d, WAVE);
    vs += __shfl_xor(vs, d, WAVE);
  }
  if (lane_id() == 0) {
    atomicAdd(&acc[0], hs);
    atomicAdd(&acc[1], hv);
    atomicAdd(vsum, vs);
  }
}

void tile_digest(const cbg_tile& t, int64_t roff, int64_t coff, uint64_t* hs, uint64_t* hv, double* vsum,
                 hipStream_t s) {
  DBuf<unsigned long long> acc(2);
  DBuf<double> vs(1);
  CBG_HIP(hipMemsetAsync(acc.p, 0, 16, s));
  CBG_HIP(hipMemsetAsync(vs.p, 0, 8, s));
  if (t.nzc > 0)
    hipLaunchKernelGGL(k_digest, dim3((unsigned)((t.nzc * WAVE + 255) / 256)), dim3(256), 0, s, t.nzc, t.cp, t.jc, t.ir,
                       t.val, roff, coff, acc.p, vs.p);
  unsigned long long h[2];
  CBG_HIP(hipMemcpyAsync(h, acc.p, 16, hipMemcpyDeviceToHost, s));
  CBG_HIP(hipMemcpyAsync(vsum, vs.p, 8, hipMemcpyDeviceToHost, s));
  CBG_HIP(hipStreamSynchronize(s));
  *hs = h[0];
  *hv = h[1];
}

// ---------------------------------------------------------------------------
// SpDCCols::operator== (SpDCCols.h:74-81) + Dcsc::operator== (dcsc.cpp:472-510):
// structure exact (cp, jc, ir), values ErrorTolerantEqual (Compare.h:47-65):
// a == b, or |a-b| < eps, or |a-b| / max(|a|,|b|) < eps (eps = SpDefs.h:64 EPSILON)
// ---------------------------------------------------------------------------
__global__ void k_tile_diff(int64_t nzc, int64_t nnz, const int64_t* __restrict__ cpa,
                            const int64_t* __restrict__ cpb, const int32_t* __restrict__ jca,
                            const int32_t* __restrict__ jcb, const int32_t* __restrict__ ira,
                            const int32_t* __restrict__ irb, const double* __restrict__ va,
                            const double* __restrict__ vb, double eps, unsigned long long* __restrict__ bad) {
  unsigned long long mine = 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nnz || i <= nzc; i += stride) {
    if (i <= nzc && cpa[i] != cpb[i]) ++mine;
    if (i < nzc && jca[i] != jcb[i]) ++mine;
    if (i < nnz) {
      if (ira[i] != irb[i]) ++mine;
      const double a = va[i], b = vb[i];
      if (!(a == b)) {
        const double d = fabs(a - b);
        if (!(d < eps || d / fmax(fabs(a), fabs(b)) < eps)) ++mine;
      }
    }
  }
  mine = wave_sum64((long long)mine);
  if (lane_id() == 0 && mine) atomicAdd(bad, mine);
}

bool tile_equal(const cbg_tile& a, const cbg_tile& b, double eps, hipStream_t s) {
  if (a.nnz == 0 && b.nnz == 0) return true;
  if (a.nnz != b.nnz || a.m != b.m || a.n != b.n || a.nzc != b.nzc) return false;
  DBuf<unsigned long long> bad(1);
  CBG_HIP(hipMemsetAsync(bad.p, 0, sizeof(unsigned long long), s));
  const int64_t work = std::max(a.nnz, a.nzc + 1);
  const unsigned blocks = (unsigned)std::min<int64_t>((work + 255) / 256, 65536);
  hipLaunchKernelGGL(k_tile_diff, dim3(blocks), dim3(256), 0, s, a.nzc, a.nnz, a.cp, b.cp, a.jc, b.jc, a.ir, b.ir,
                     a.val, b.val, eps, bad.p);
  unsigned long long h = 0;
  CBG_HIP(hipMemcpyAsync(&h, bad.p, sizeof(h), hipMemcpyDeviceToHost, s));
  CBG_HIP(hipStreamSynchronize(s));
  return h == 0;
}

}  // namespace cbg
