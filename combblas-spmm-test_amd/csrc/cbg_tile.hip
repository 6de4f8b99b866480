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
  // 2 MiB granules up to 1 GiB; above, 1/16 of the size's power of two (<= 6.25 %
  // rounding), so that the C arrays of consecutive MemEfficientSpGEMM phases --
  // tens of GB whose sizes differ by a few percent -- reuse one cached block
  // instead of each allocating another next to the cached one
  size_t g = 2u << 20;
  if (b >= ((size_t)1 << 30)) {
    int l = 63 - __builtin_clzll(b);
    g = (size_t)1 << (l - 4);
  }
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
      serial_[p] = ++next_serial_;
      in_use_ += sz;
      return p;
    }
  }
  void* p = nullptr;
  hipError_t e = hipMalloc(&p, rb);
  // out of memory: release cached blocks largest first until the request fits
  // (dropping the whole cache would make every later request allocate again)
  while (e != hipSuccess && release_largest_cached()) {
    (void)hipGetLastError();
    e = hipMalloc(&p, rb);
  }
  if (e != hipSuccess) {
    (void)hipGetLastError();
    trim();  // drop the cache (growable blocks included) and retry once
    e = hipMalloc(&p, rb);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      throw HipError("device allocation of " + std::to_string(rb) + " bytes failed (" + hipGetErrorString(e) + ")",
                     CBG_ERR_OOM);
    }
  }
  std::lock_guard<std::mutex> lk(mu_);
  live_[p] = rb;
  serial_[p] = ++next_serial_;
  in_use_ += rb;
  return p;
}

uint64_t DevicePool::serial_of(const void* p) {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = serial_.upper_bound(const_cast<void*>(p));
  if (it == serial_.begin()) return 0;
  --it;
  size_t size = 0;
  auto l = live_.find(it->first);
  if (l != live_.end()) {
    size = l->second;
  } else {
    auto g = grow_.find(it->first);
    if (g != grow_.end()) size = g->second.reserved;
  }
  return static_cast<const char*>(p) < static_cast<const char*>(it->first) + size ? it->second : 0;
}

bool DevicePool::release_largest_cached() {
  std::lock_guard<std::mutex> lk(mu_);
  if (free_.empty()) return false;
  auto it = std::prev(free_.end());
  (void)hipFree(it->second);
  cached_ -= it->first;
  free_.erase(it);
  return true;
}

DevicePool::DevicePool() {
  const char* e = getenv("CBG_POOL_QUARANTINE");
  quarantine_ = e && atoi(e) > 0;
}

void DevicePool::quarantine_release() {
  if (!quarantine_) return;
  (void)hipDeviceSynchronize();  // no kernel uses a quarantined block any more, the poison has landed
  std::lock_guard<std::mutex> lk(mu_);
  for (auto& q : quar_) {
    free_.emplace(q.second, q.first);
    cached_ += q.second;
  }
  quar_.clear();
}

void DevicePool::free(void* p) {
  if (!p) return;
  std::lock_guard<std::mutex> lk(mu_);
  serial_.erase(p);
  auto it = live_.find(p);
  if (it != live_.end() && quarantine_) {
    if (!poison_) (void)hipStreamCreateWithFlags(&poison_, hipStreamNonBlocking);
    (void)hipMemsetAsync(p, 0xff, it->second, poison_);
    quar_.emplace_back(p, it->second);
    in_use_ -= it->second;
    live_.erase(it);
    return;
  }
  if (it == live_.end()) {
    auto g = grow_.find(p);
    if (g != grow_.end()) {  // keep it mapped for the next growable request
      in_use_ -= g->second.mapped;
      cached_ += g->second.mapped;
      grow_cache_.emplace(p, std::move(g->second));
      grow_.erase(g);
    }
    return;
  }
  free_.emplace(it->second, p);
  cached_ += it->second;
  in_use_ -= it->second;
  live_.erase(it);
}

// physical granule of the growable arrays (hipMemGetAllocationGranularity)
static hipMemAllocationProp device_prop() {
  int dev = 0;
  (void)hipGetDevice(&dev);
  hipMemAllocationProp prop{};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = dev;
  return prop;
}
// Mapping sizes and offsets are multiples of 64 MiB: a multiple of the
// recommended granularity and of the 2 MiB GPU page (a 545 MiB mapping after a
// 256 MiB one made hipMemSetAccess fail with "invalid argument" on the box).
static size_t granule() {
  static thread_local size_t g = 0;
  if (!g) {
    hipMemAllocationProp prop = device_prop();
    size_t rec = 0;
    CBG_HIP(hipMemGetAllocationGranularity(&rec, &prop, hipMemAllocationGranularityRecommended));
    g = (size_t)64 << 20;
    while (rec > g) g <<= 1;
  }
  return g;
}

void* DevicePool::reserve_growable(size_t max_bytes) {
  const size_t g = granule();
  const size_t r = (std::max<size_t>(max_bytes, 1) + g - 1) / g * g;
  {
    // a cached block large enough, the most mapped first
    std::lock_guard<std::mutex> lk(mu_);
    auto best = grow_cache_.end();
    for (auto it = grow_cache_.begin(); it != grow_cache_.end(); ++it)
      if (it->second.reserved >= r && (best == grow_cache_.end() || it->second.mapped > best->second.mapped))
        best = it;
    if (best != grow_cache_.end()) {
      void* p = best->first;
      cached_ -= best->second.mapped;
      in_use_ += best->second.mapped;
      grow_.emplace(p, std::move(best->second));
      grow_cache_.erase(best);
      serial_[p] = ++next_serial_;
      return p;
    }
  }
  void* p = nullptr;
  CBG_HIP(hipMemAddressReserve(&p, r, g, nullptr, 0));
  std::lock_guard<std::mutex> lk(mu_);
  grow_[p].reserved = r;
  serial_[p] = ++next_serial_;
  return p;
}

void DevicePool::grow(void* base, size_t bytes) {
  std::unique_lock<std::mutex> lk(mu_);
  auto it = grow_.find(base);
  if (it == grow_.end()) throw HipError("grow: not a growable block", CBG_ERR_HIP);
  Growable& gr = it->second;
  if (bytes <= gr.mapped) return;
  if (bytes > gr.reserved) throw HipError("growable block exhausted its reservation", CBG_ERR_OOM);
  // map at least 256 MiB at a time (few mappings for tiles of 10^10 entries)
  const size_t g = granule();
  size_t step = std::max<size_t>(bytes - gr.mapped, (size_t)256 << 20);
  step = std::min((step + g - 1) / g * g, gr.reserved - gr.mapped);
  if (gr.mapped + step < bytes) step = (bytes - gr.mapped + g - 1) / g * g;
  hipMemAllocationProp prop = device_prop();
  hipMemGenericAllocationHandle_t h{};
  hipError_t e = hipMemCreate(&h, step, &prop, 0);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    lk.unlock();
    trim();  // drop the pool cache and retry once
    lk.lock();
    e = hipMemCreate(&h, step, &prop, 0);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      throw HipError("device allocation of " + std::to_string(step) + " bytes (growable) failed", CBG_ERR_OOM);
    }
  }
  char* at = static_cast<char*>(base) + gr.mapped;
  const char* what = "hipMemMap";
  e = hipMemMap(at, step, 0, h, 0);
  if (e == hipSuccess) {
    hipMemAccessDesc d{};
    d.location = prop.location;
    d.flags = hipMemAccessFlagsProtReadWrite;
    what = "hipMemSetAccess";
    // access is set over the whole mapped range from the reservation's base
    // (setting it on the new chunk alone failed with "invalid argument" on the box
    // once other processes had used the device)
    e = hipMemSetAccess(base, gr.mapped + step, &d, 1);
    if (e != hipSuccess) (void)hipMemUnmap(at, step);
  }
  if (e != hipSuccess) {
    (void)hipGetLastError();
    (void)hipMemRelease(h);
    size_t fr = 0, tot = 0;
    (void)hipMemGetInfo(&fr, &tot);
    throw HipError(std::string(what) + ": " + hipGetErrorString(e) + " (mapping " + std::to_string(step >> 20) +
                       " MiB at offset " + std::to_string(gr.mapped >> 20) + " MiB of a " +
                       std::to_string(gr.reserved >> 30) + " GiB range; device free " + std::to_string(fr >> 30) +
                       " of " + std::to_string(tot >> 30) + " GiB)",
                   CBG_ERR_OOM);
  }
  gr.chunks.emplace_back(h, step);
  gr.mapped += step;
  in_use_ += step;
}

void DevicePool::release_growable(void* base, Growable& gr) {
  // callers free a tile only after the kernels that use it have completed.
  // The physical pages go back to the driver, but the virtual range stays
  // reserved for the life of the process: measured on the MI355X box, a range
  // freed with hipMemAddressFree and handed out again (to a new growable block
  // or to hipMalloc) read back stale or zero data in the next kernels
  // (tests/test_multiprocess.py::test_fault_injection_gpu caught it); never
  // reusing a virtual address avoids it, at no cost beyond address space.
  (void)hipDeviceSynchronize();
  size_t off = 0;
  for (auto& c : gr.chunks) {
    (void)hipMemUnmap(static_cast<char*>(base) + off, c.second);
    (void)hipMemRelease(c.first);
    off += c.second;
  }
  in_use_ -= gr.mapped;
  gr.chunks.clear();
  gr.mapped = 0;
}

// ----------------------------------------------------------------------------
// EntryArena: C entries of consecutive multiplies, end to end
// ----------------------------------------------------------------------------
EntryArena::EntryArena() {
  size_t fr = 0, tot = 0;
  CBG_HIP(hipMemGetInfo(&fr, &tot));
  // virtual reservations only: room for a tile filling the whole device
  // (12 bytes per entry: a third of the bytes for the row ids)
  ir = static_cast<int32_t*>(pool().reserve_growable(tot / 3 + ((size_t)256 << 20)));
  val = static_cast<double*>(pool().reserve_growable(2 * (tot / 3) + ((size_t)512 << 20)));
}
EntryArena::~EntryArena() {
  pool().free(ir);
  pool().free(val);
}
void EntryArena::place(int64_t nnz, int32_t** pir, double** pval) {
  pool().grow(ir, sizeof(int32_t) * (size_t)std::max<int64_t>(used + nnz, 1));
  pool().grow(val, sizeof(double) * (size_t)std::max<int64_t>(used + nnz, 1));
  *pir = ir + used;
  *pval = val + used;
  used += nnz;
}

void DevicePool::trim() {
  std::lock_guard<std::mutex> lk(mu_);
  for (auto& kv : free_) (void)hipFree(kv.second);
  free_.clear();
  for (auto& kv : grow_cache_) {
    in_use_ += kv.second.mapped;  // release_growable accounts it as in use
    release_growable(kv.first, kv.second);
  }
  grow_cache_.clear();
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

// also out[n] = the total (toff[nt]): a separate 8-byte device copy is a blit
// kernel that waits for a free CU slot behind a concurrent stream's kernels
// (up to 150 us seen in GalerkinNew's thin-column sort)
__global__ void k_scan_add(int64_t* __restrict__ out, int64_t n, const int64_t* __restrict__ toff, int64_t nt) {
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < n) out[i] += toff[i / SCAN_TILE];
  if (i == 0) out[n] = toff[nt];
}

template <class TI>
static void scan_impl(const TI* in, int64_t* out, int64_t n, hipStream_t s, DeferredFree* df) {
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
  scan_impl<int64_t>(sums.p, offs.p, nt, s, df);
  hipLaunchKernelGGL(k_scan_add, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, out, n, offs.p, nt);
  if (df) {  // released when the caller's work on `s` has been synchronized
    df->take(sums);
    df->take(offs);
  } else {
    CBG_HIP(hipStreamSynchronize(s));  // sums/offs go back to the pool
  }
}

void exclusive_scan_i64(const int64_t* in, int64_t* out, int64_t n, hipStream_t s, DeferredFree* df) {
  scan_impl<int64_t>(in, out, n, s, df);
}
void exclusive_scan_i32_to_i64(const int32_t* in, int64_t* out, int64_t n, hipStream_t s, DeferredFree* df) {
  scan_impl<int32_t>(in, out, n, s, df);
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
    if (!(t.reserved & TILE_BORROWED_ENTRIES)) {
      pool().free(t.ir);
      pool().free(t.val);
    }
  }
  t.cp = nullptr;
  t.jc = nullptr;
  t.ir = nullptr;
  t.val = nullptr;
  t.nnz = t.nzc = 0;
  t.reserved = 0;
}

TileGuard::~TileGuard() { tile_free_device(t); }
TileGuard& TileGuard::operator=(TileGuard&& o) noexcept {
  if (this != &o) {
    tile_free_device(t);
    t = o.release();
  }
  return *this;
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
  const int64_t a = cp[i], b = cp[i + 1];  // 64-bit: tiles may hold 2^31 or more entries
  const int64_t k = lower_bound_g64(ir, a, b, cut) - a;
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
// slices: columns [a, b) or rows [a, b) of a tile, re-based, one copy
// (the stage pieces of the generalized SUMMA and the pipeline's B pieces)
// ----------------------------------------------------------------------------
void tile_slice_cols(const cbg_tile& T, int64_t a, int64_t b, cbg_tile& out, hipStream_t s) {
  int64_t pos[2] = {0, 0}, cpos[2] = {0, 0};
  if (T.nzc > 0) {
    DBuf<int64_t> d(2);
    hipLaunchKernelGGL(k_lower_bound_jc, dim3(1), dim3(1), 0, s, T.jc, T.nzc, a, d.p);
    hipLaunchKernelGGL(k_lower_bound_jc, dim3(1), dim3(1), 0, s, T.jc, T.nzc, b, d.p + 1);
    CBG_HIP(hipMemcpyAsync(pos, d.p, 2 * sizeof(int64_t), hipMemcpyDeviceToHost, s));
    CBG_HIP(hipStreamSynchronize(s));
    CBG_HIP(hipMemcpyAsync(&cpos[0], T.cp + pos[0], sizeof(int64_t), hipMemcpyDeviceToHost, s));
    CBG_HIP(hipMemcpyAsync(&cpos[1], T.cp + pos[1], sizeof(int64_t), hipMemcpyDeviceToHost, s));
    CBG_HIP(hipStreamSynchronize(s));
  }
  const int64_t nzc = pos[1] - pos[0], nnz = cpos[1] - cpos[0];
  tile_alloc_device(out, T.m, b - a, nnz, nzc);
  if (nzc > 0) {
    hipLaunchKernelGGL(k_copy_cols, dim3((unsigned)((nzc + 256) / 256)), dim3(256), 0, s, nzc, T.jc + pos[0],
                       T.cp + pos[0], a, cpos[0], out.jc, out.cp);
    if (nnz) {
      CBG_HIP(hipMemcpyAsync(out.ir, T.ir + cpos[0], sizeof(int32_t) * nnz, hipMemcpyDeviceToDevice, s));
      CBG_HIP(hipMemcpyAsync(out.val, T.val + cpos[0], sizeof(double) * nnz, hipMemcpyDeviceToDevice, s));
    }
  }
  CBG_HIP(hipStreamSynchronize(s));
}

__global__ void k_rowslice_count(int64_t nzc, const int64_t* __restrict__ cp, const int32_t* __restrict__ ir, int lo,
                                 int hi, int64_t* __restrict__ first, int64_t* __restrict__ cnt,
                                 int64_t* __restrict__ flag) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= nzc) return;
  const int64_t a = lower_bound_g64(ir, cp[i], cp[i + 1], lo);
  const int64_t b = lower_bound_g64(ir, a, cp[i + 1], hi);
  first[i] = a;
  cnt[i] = b - a;
  flag[i] = b > a;
}
__global__ void k_rowslice_copy(int64_t nzc, const int32_t* __restrict__ jc, const int32_t* __restrict__ ir,
                                const double* __restrict__ val, int lo, const int64_t* __restrict__ first,
                                const int64_t* __restrict__ off, const int64_t* __restrict__ col,
                                int32_t* __restrict__ ojc, int64_t* __restrict__ ocp, int32_t* __restrict__ oir,
                                double* __restrict__ oval) {
  const int64_t i = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / WAVE;
  if (i >= nzc) return;
  const int64_t k = off[i + 1] - off[i];
  if (k == 0) return;
  if (lane_id() == 0) {
    ojc[col[i]] = jc[i];
    ocp[col[i]] = off[i];
  }
  const int64_t a = first[i];
  for (int64_t q = lane_id(); q < k; q += WAVE) {
    oir[off[i] + q] = ir[a + q] - lo;
    oval[off[i] + q] = val[a + q];
  }
}

void tile_slice_rows(const cbg_tile& T, int64_t a, int64_t b, cbg_tile& out, hipStream_t s) {
  const int64_t nz = T.nzc;
  if (nz == 0) {
    tile_alloc_device(out, b - a, T.n, 0, 0);
    return;
  }
  DBuf<int64_t> first(nz + 1), cnt(nz + 1), flag(nz + 1), off(nz + 1), col(nz + 1);
  hipLaunchKernelGGL(k_rowslice_count, dim3((unsigned)((nz + 255) / 256)), dim3(256), 0, s, nz, T.cp, T.ir, (int)a,
                     (int)b, first.p, cnt.p, flag.p);
  exclusive_scan_i64(cnt.p, off.p, nz, s);
  exclusive_scan_i64(flag.p, col.p, nz, s);
  int64_t h[2];
  CBG_HIP(hipMemcpyAsync(&h[0], off.p + nz, 8, hipMemcpyDeviceToHost, s));
  CBG_HIP(hipMemcpyAsync(&h[1], col.p + nz, 8, hipMemcpyDeviceToHost, s));
  CBG_HIP(hipStreamSynchronize(s));
  tile_alloc_device(out, b - a, T.n, h[0], h[1]);
  hipLaunchKernelGGL(k_rowslice_copy, dim3((unsigned)((nz * WAVE + 255) / 256)), dim3(256), 0, s, nz, T.jc, T.ir,
                     T.val, (int)a, first.p, off.p, col.p, out.jc, out.cp, out.ir, out.val);
  CBG_HIP(hipMemcpyAsync(out.cp + h[1], &h[0], 8, hipMemcpyHostToDevice, s));
  CBG_HIP(hipStreamSynchronize(s));
}

// ----------------------------------------------------------------------------
// column assembly of arena-backed parts (no entry copies)
// ----------------------------------------------------------------------------
void tile_assemble_cols(const std::vector<cbg_tile>& parts, const std::vector<int64_t>& col_off, int64_t m, int64_t n,
                        EntryArena& arena, cbg_tile& out, hipStream_t s) {
  int64_t nnz = 0, nzc = 0;
  for (size_t k = 0; k < parts.size(); ++k) {
    if (parts[k].nnz > 0 && parts[k].ir != arena.ir + nnz)
      throw HipError("tile_assemble_cols: parts are not laid out end to end in the arena", CBG_ERR_HIP);
    nnz += parts[k].nnz;
    nzc += parts[k].nzc;
  }
  if (nnz != arena.used) throw HipError("tile_assemble_cols: arena holds other entries", CBG_ERR_HIP);
  out = cbg_tile{};
  out.m = m;
  out.n = n;
  out.nnz = nnz;
  out.nzc = nzc;
  out.on_device = 1;
  out.cp = static_cast<int64_t*>(pool().alloc(sizeof(int64_t) * (nzc + 1)));
  out.jc = static_cast<int32_t*>(pool().alloc(sizeof(int32_t) * std::max<int64_t>(nzc, 1)));
  int64_t e = 0, c = 0;
  for (size_t k = 0; k < parts.size(); ++k) {
    const cbg_tile& p = parts[k];
    if (p.nzc > 0)
      hipLaunchKernelGGL(k_cat_cols, dim3((unsigned)((p.nzc + 255) / 256)), dim3(256), 0, s, p.nzc, p.jc, p.cp,
                         col_off[k], e, out.jc + c, out.cp + c);
    e += p.nnz;
    c += p.nzc;
  }
  CBG_HIP(hipMemcpyAsync(out.cp + nzc, &nnz, sizeof(int64_t), hipMemcpyHostToDevice, s));
  CBG_HIP(hipStreamSynchronize(s));
  if (nnz > 0) {
    out.ir = arena.ir;
    out.val = arena.val;
    arena.detach();
  } else {
    out.ir = static_cast<int32_t*>(pool().alloc(sizeof(int32_t)));
    out.val = static_cast<double*>(pool().alloc(sizeof(double)));
  }
}

// ----------------------------------------------------------------------------
// digest (tests/golden/make_golden.py definition)
// ----------------------------------------------------------------------------
__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
// acc[2] counts order violations, as the reference driver's digest does: a
// row id not strictly above its predecessor in the column, a column id not
// strictly above the previous nonempty column, a decreasing or empty cp step
__global__ void k_digest(int64_t nzc, const int64_t* __restrict__ cp, const int32_t* __restrict__ jc,
                         const int32_t* __restrict__ ir, const double* __restrict__ val, int64_t roff, int64_t coff,
                         unsigned long long* __restrict__ acc, double* __restrict__ vsum) {
  const int64_t i = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / WAVE;
  if (i >= nzc) return;
  const unsigned long long col = (unsigned long long)(jc[i] + coff);
  const int64_t a = cp[i], b = cp[i + 1];
  unsigned long long hs = 0, hv = 0, bad = 0;
  double vs = 0.0;
  for (int64_t q = a + lane_id(); q < b; q += WAVE) {
    const int r = ir[q];
    const unsigned long long h = mix64((col << 32) | (unsigned long long)(r + roff));
    const double v = val[q];
    hs += h;
    hv += h * mix64(__double_as_longlong(v));
    vs += v;
    if (q > a && ir[q - 1] >= r) ++bad;
  }
  if (lane_id() == 0) {
    if (b <= a) ++bad;                     // DCSC columns are nonempty
    if (i > 0 && jc[i - 1] >= jc[i]) ++bad;
  }
#pragma unroll
  for (int d = WAVE / 2; d > 0; d >>= 1) {
    hs += __shfl_xor(hs, d, WAVE);
    hv += __shfl_xor(hv, d, WAVE);
    vs += __shfl_xor(vs, d, WAVE);
    bad += __shfl_xor(bad, d, WAVE);
  }
  if (lane_id() == 0) {
    atomicAdd(&acc[0], hs);
    atomicAdd(&acc[1], hv);
    if (bad) atomicAdd(&acc[2], bad);
    atomicAdd(vsum, vs);
  }
}

void tile_digest(const cbg_tile& t, int64_t roff, int64_t coff, uint64_t* hs, uint64_t* hv, double* vsum,
                 uint64_t* unsorted, hipStream_t s) {
  DBuf<unsigned long long> acc(3);
  DBuf<double> vs(1);
  CBG_HIP(hipMemsetAsync(acc.p, 0, 24, s));
  CBG_HIP(hipMemsetAsync(vs.p, 0, 8, s));
  if (t.nzc > 0)
    hipLaunchKernelGGL(k_digest, dim3((unsigned)((t.nzc * WAVE + 255) / 256)), dim3(256), 0, s, t.nzc, t.cp, t.jc, t.ir,
                       t.val, roff, coff, acc.p, vs.p);
  unsigned long long h[3];
  int64_t ends[2] = {0, 0};
  CBG_HIP(hipMemcpyAsync(h, acc.p, 24, hipMemcpyDeviceToHost, s));
  CBG_HIP(hipMemcpyAsync(vsum, vs.p, 8, hipMemcpyDeviceToHost, s));
  CBG_HIP(hipMemcpyAsync(&ends[0], t.cp, 8, hipMemcpyDeviceToHost, s));
  CBG_HIP(hipMemcpyAsync(&ends[1], t.cp + t.nzc, 8, hipMemcpyDeviceToHost, s));
  CBG_HIP(hipStreamSynchronize(s));
  *hs = h[0];
  *hv = h[1];
  // cp[0] == 0 and cp[nzc] == nnz close the chain of per-column checks
  if (unsorted) *unsorted = h[2] + (ends[0] != 0) + (ends[1] != t.nnz);
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

// ---------------------------------------------------------------------------
// phase planning (MemEfficientSpGEMM's memory-driven phase count,
// ParFriends.h:482-535): the flops of a SUMMA product from the column counts
// of A's tiles and the row counts of B's tiles, and a column sample of B for
// the compression ratio
// ---------------------------------------------------------------------------
__global__ void k_col_counts(int64_t nzc, const int64_t* __restrict__ cp, const int32_t* __restrict__ jc,
                             int32_t* __restrict__ cnt) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < nzc) cnt[jc[i]] = (int32_t)(cp[i + 1] - cp[i]);
}
__global__ void k_row_counts(int64_t nnz, const int32_t* __restrict__ ir, int32_t* __restrict__ cnt) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nnz; i += (int64_t)gridDim.x * blockDim.x)
    atomicAdd(&cnt[ir[i]], 1);
}
void tile_counts_device(const cbg_tile& t, int dim, int32_t* d, int64_t padded, hipStream_t s) {
  if (padded > 0) CBG_HIP(hipMemsetAsync(d, 0, sizeof(int32_t) * padded, s));
  if (dim == 0 && t.nzc > 0)
    hipLaunchKernelGGL(k_col_counts, dim3((unsigned)((t.nzc + 255) / 256)), dim3(256), 0, s, t.nzc, t.cp, t.jc, d);
  if (dim == 1 && t.nnz > 0)
    hipLaunchKernelGGL(k_row_counts, dim3((unsigned)std::min<int64_t>((t.nnz + 255) / 256, 8192)), dim3(256), 0, s,
                       t.nnz, t.ir, d);
  CBG_HIP(hipStreamSynchronize(s));  // the comm stream reads the counts next
}

// sum over k < K of a[k] * b[k], where a is split into segments aoff[s]..aoff[s+1]
// stored at a + s * astride (b likewise): the inner index walks A's column
// blocks and B's row blocks at once
struct DotSegs {
  int na, nb;
  int64_t aoff[65], boff[65];
};
__device__ __forceinline__ int seg_of_k(const int64_t* off, int n, int64_t k) {
  int s = 0;
  while (s + 1 < n && off[s + 1] <= k) ++s;
  return s;
}
__global__ void k_blocked_dot(const int32_t* __restrict__ a, int64_t astride, const int32_t* __restrict__ b,
                              int64_t bstride, DotSegs sg, int64_t K, unsigned long long* __restrict__ out) {
  unsigned long long acc = 0;
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < K; k += (int64_t)gridDim.x * blockDim.x) {
    const int sa = seg_of_k(sg.aoff, sg.na, k), sb = seg_of_k(sg.boff, sg.nb, k);
    acc += (unsigned long long)a[sa * astride + (k - sg.aoff[sa])] * (unsigned long long)b[sb * bstride + (k - sg.boff[sb])];
  }
  acc = (unsigned long long)wave_sum64((long long)acc);
  if (lane_id() == 0 && acc) atomicAdd(out, acc);
}
// sum over the entries (k, j) of B of a[k]: the flops of A*B when a holds A's
// column counts (estimateFLOP's total without row counts of B)
__global__ void k_entry_sum(int64_t nnz, const int32_t* __restrict__ ir, const int32_t* __restrict__ a,
                            unsigned long long* __restrict__ out) {
  unsigned long long acc = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nnz; i += (int64_t)gridDim.x * blockDim.x)
    acc += (unsigned)a[ir[i]];
  acc = (unsigned long long)wave_sum64((long long)acc);
  if (lane_id() == 0 && acc) atomicAdd(out, acc);
}
int64_t entry_sum_device(const cbg_tile& B, const int32_t* a, hipStream_t s) {
  DBuf<unsigned long long> d(1);
  CBG_HIP(hipMemsetAsync(d.p, 0, sizeof(unsigned long long), s));
  if (B.nnz > 0)
    hipLaunchKernelGGL(k_entry_sum, dim3((unsigned)std::min<int64_t>((B.nnz + 255) / 256, 4096)), dim3(256), 0, s,
                       B.nnz, B.ir, a, d.p);
  unsigned long long h = 0;
  CBG_HIP(hipMemcpyAsync(&h, d.p, sizeof(h), hipMemcpyDeviceToHost, s));
  CBG_HIP(hipStreamSynchronize(s));
  return (int64_t)h;
}

int64_t blocked_dot_device(const int32_t* a, int64_t astride, const std::vector<int64_t>& aoff, const int32_t* b,
                           int64_t bstride, const std::vector<int64_t>& boff, int64_t K, hipStream_t s) {
  DotSegs sg{};
  if (aoff.size() > 65 || boff.size() > 65) throw HipError("phase plan: grid dimension above 64", CBG_ERR_NOTSUPPORTED);
  sg.na = (int)aoff.size() - 1;
  sg.nb = (int)boff.size() - 1;
  for (size_t i = 0; i < aoff.size(); ++i) sg.aoff[i] = aoff[i];
  for (size_t i = 0; i < boff.size(); ++i) sg.boff[i] = boff[i];
  DBuf<unsigned long long> d(1);
  CBG_HIP(hipMemsetAsync(d.p, 0, sizeof(unsigned long long), s));
  if (K > 0)
    hipLaunchKernelGGL(k_blocked_dot, dim3((unsigned)std::min<int64_t>((K + 255) / 256, 4096)), dim3(256), 0, s, a,
                       astride, b, bstride, sg, K, d.p);
  unsigned long long h = 0;
  CBG_HIP(hipMemcpyAsync(&h, d.p, sizeof(h), hipMemcpyDeviceToHost, s));
  CBG_HIP(hipStreamSynchronize(s));
  return (int64_t)h;
}

// Samples of a tile for the compression estimate: the columns whose id is a
// multiple of `stride` (every tile of a grid column keeps the same columns), or
// the rows whose id is a multiple of `stride`, renumbered row / stride (every
// tile of a grid row keeps the same rows).  Ids, not positions: R-MAT's ids are
// scrambled, so either is a uniform sample.
__global__ void k_sample_col_len(int64_t nzc, int stride, const int64_t* __restrict__ cp, const int32_t* __restrict__ jc,
                                 int64_t* __restrict__ len, int64_t* __restrict__ flag) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= nzc) return;
  const bool keep = jc[i] % stride == 0;
  len[i] = keep ? cp[i + 1] - cp[i] : 0;
  flag[i] = keep;
}
__global__ void k_sample_row_len(int64_t nzc, int stride, const int64_t* __restrict__ cp,
                                 const int32_t* __restrict__ ir, int64_t* __restrict__ len, int64_t* __restrict__ flag) {
  const int64_t i = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / WAVE;
  if (i >= nzc) return;
  int c = 0;
  for (int64_t q = cp[i] + lane_id(); q < cp[i + 1]; q += WAVE) c += ir[q] % stride == 0;
  c = wave_sum(c);
  if (lane_id() == 0) {
    len[i] = c;
    flag[i] = c > 0;
  }
}
// a wave per kept column; rows == true: keep only rows % stride == 0, renumbered
__global__ void k_sample_copy(int64_t nzc, int stride, bool rows, const int64_t* __restrict__ cp,
                              const int32_t* __restrict__ jc, const int32_t* __restrict__ ir,
                              const double* __restrict__ val, const int64_t* __restrict__ len,
                              const int64_t* __restrict__ off, const int64_t* __restrict__ col,
                              int64_t* __restrict__ ocp, int32_t* __restrict__ ojc, int32_t* __restrict__ oir,
                              double* __restrict__ oval) {
  const int64_t i = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / WAVE;
  if (i >= nzc || len[i] == 0) return;
  const int lane = lane_id();
  if (lane == 0) {
    ojc[col[i]] = jc[i];
    ocp[col[i]] = off[i];
  }
  int64_t dst = off[i];
  for (int64_t q0 = cp[i]; q0 < cp[i + 1]; q0 += WAVE) {
    const int64_t q = q0 + lane;
    const bool in = q < cp[i + 1];
    const int r = in ? ir[q] : 0;
    const bool keep = in && (!rows || r % stride == 0);
    const unsigned long long m = __ballot(keep);
    if (keep) {
      const int64_t at = dst + __popcll(m & ((1ull << lane) - 1ull));
      oir[at] = rows ? r / stride : r;
      oval[at] = val[q];
    }
    dst += __popcll(m);
  }
}
static void tile_sample(const cbg_tile& T, int stride, bool rows, cbg_tile& out, hipStream_t s) {
  const int64_t m = rows ? (T.m + stride - 1) / stride : T.m;
  const int64_t nz = T.nzc;
  if (nz == 0) {
    tile_alloc_device(out, m, T.n, 0, 0);
    return;
  }
  DBuf<int64_t> len(nz + 1), flag(nz + 1), off(nz + 1), col(nz + 1);
  if (rows)
    hipLaunchKernelGGL(k_sample_row_len, dim3((unsigned)((nz * WAVE + 255) / 256)), dim3(256), 0, s, nz, stride, T.cp,
                       T.ir, len.p, flag.p);
  else
    hipLaunchKernelGGL(k_sample_col_len, dim3((unsigned)((nz + 255) / 256)), dim3(256), 0, s, nz, stride, T.cp, T.jc,
                       len.p, flag.p);
  exclusive_scan_i64(len.p, off.p, nz, s);
  exclusive_scan_i64(flag.p, col.p, nz, s);
  int64_t h[2];
  CBG_HIP(hipMemcpyAsync(&h[0], off.p + nz, 8, hipMemcpyDeviceToHost, s));
  CBG_HIP(hipMemcpyAsync(&h[1], col.p + nz, 8, hipMemcpyDeviceToHost, s));
  CBG_HIP(hipStreamSynchronize(s));
  tile_alloc_device(out, m, T.n, h[0], h[1]);
  hipLaunchKernelGGL(k_sample_copy, dim3((unsigned)((nz * WAVE + 255) / 256)), dim3(256), 0, s, nz, stride, rows, T.cp,
                     T.jc, T.ir, T.val, len.p, off.p, col.p, out.cp, out.jc, out.ir, out.val);
  CBG_HIP(hipMemcpyAsync(out.cp + h[1], &h[0], 8, hipMemcpyHostToDevice, s));
  CBG_HIP(hipStreamSynchronize(s));
}
void tile_sample_cols(const cbg_tile& T, int stride, cbg_tile& out, hipStream_t s) { tile_sample(T, stride, false, out, s); }
void tile_sample_rows(const cbg_tile& T, int stride, cbg_tile& out, hipStream_t s) { tile_sample(T, stride, true, out, s); }

}  // namespace cbg
