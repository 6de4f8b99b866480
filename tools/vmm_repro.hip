// vmm_repro.hip -- minimal single-process reproducer for the virtual-memory
// event recorded in cbg_tile.hip (DevicePool::release_growable): a virtual range
// unmapped, freed and handed out again "read back stale or zero data".
//
//   hipcc --offload-arch=gfx950 -O2 tools/vmm_repro.hip -o tools/vmm_repro && tools/vmm_repro
//
// Every variant maps physical memory into a virtual range, fills it with a
// pattern from a kernel on all CUs, verifies it from another kernel, then
// releases the mapping and maps NEW physical memory at the same (or a re-reserved)
// address, fills a second pattern and verifies again.  A stale translation would
// show as words of the first pattern (or zeros) in the second verification.
//   A: unmap + release, map a new handle at the SAME reservation
//   B: unmap + release + hipMemAddressFree, re-reserve (same VA if the driver
//      returns it), map a new handle
//   C: as B, then hipMalloc of the same size (may land on the freed VA)
//   D: as A, with hipMemSetAccess on the new chunk only (cbg_tile.hip saw
//      "invalid argument" for this on a shared box)
// Prints one line per trial; exits 0 whatever it finds (it is a measurement).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

#define CHK(x)                                                                  \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::printf("  %s -> %s\n", #x, hipGetErrorString(e_));                   \
      ok = false;                                                               \
    }                                                                           \
  } while (0)

__global__ void k_fill(unsigned* p, size_t n, unsigned pat) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = pat ^ (unsigned)i;
}
__global__ void k_check(const unsigned* p, size_t n, unsigned pat, unsigned old, unsigned long long* bad) {
  unsigned long long b[3] = {0, 0, 0};  // wrong, equal to the old pattern, zero
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const unsigned v = p[i];
    if (v != (pat ^ (unsigned)i)) {
      ++b[0];
      if (v == (old ^ (unsigned)i)) ++b[1];
      if (v == 0) ++b[2];
    }
  }
  for (int k = 0; k < 3; ++k)
    if (b[k]) atomicAdd(&bad[k], b[k]);
}

static const size_t kBytes = (size_t)256 << 20, kWords = kBytes / 4;

static bool fill_check(unsigned* p, unsigned pat, unsigned old, unsigned long long* dbad, unsigned long long hb[3]) {
  bool ok = true;
  CHK(hipMemset(dbad, 0, 24));
  hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, 0, p, kWords, pat);
  CHK(hipDeviceSynchronize());
  hipLaunchKernelGGL(k_check, dim3(2048), dim3(256), 0, 0, p, kWords, pat, old, dbad);
  CHK(hipDeviceSynchronize());
  CHK(hipMemcpy(hb, dbad, 24, hipMemcpyDeviceToHost));
  // and one host read-back of a sample
  unsigned s[4] = {0, 0, 0, 0};
  CHK(hipMemcpy(s, p + kWords / 2, sizeof(s), hipMemcpyDeviceToHost));
  for (int k = 0; k < 4; ++k)
    if (s[k] != (pat ^ (unsigned)(kWords / 2 + k))) ++hb[0];
  return ok;
}

int main() {
  bool ok = true;
  int dev = 0;
  CHK(hipSetDevice(dev));
  hipMemAllocationProp prop{};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = dev;
  size_t gran = 0;
  CHK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended));
  const size_t align = (size_t)64 << 20;
  hipMemAccessDesc acc{};
  acc.location = prop.location;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  unsigned long long* dbad = nullptr;
  CHK(hipMalloc(&dbad, 24));
  std::printf("granularity %zu bytes; %zu MiB per mapping\n", gran, kBytes >> 20);
  const char* names[4] = {"A same-reservation remap", "B free + re-reserve", "C free + hipMalloc",
                          "D remap, access on chunk only"};
  int problems = 0;
  for (int v = 0; v < 4; ++v) {
    for (int trial = 0; trial < 4; ++trial) {
      ok = true;
      void* R = nullptr;
      CHK(hipMemAddressReserve(&R, 2 * kBytes, align, nullptr, 0));
      hipMemGenericAllocationHandle_t h1{}, h2{};
      CHK(hipMemCreate(&h1, kBytes, &prop, 0));
      CHK(hipMemMap(R, kBytes, 0, h1, 0));
      CHK(hipMemSetAccess(R, kBytes, &acc, 1));
      if (!ok) {
        std::printf("%s trial %d: setup failed\n", names[v], trial);
        return 0;
      }
      const unsigned p1 = 0x11110000u + trial, p2 = 0x22220000u + trial;
      unsigned long long b1[3] = {0, 0, 0}, b2[3] = {0, 0, 0};
      fill_check((unsigned*)R, p1, 0, dbad, b1);
      CHK(hipMemUnmap(R, kBytes));
      CHK(hipMemRelease(h1));
      void* R2 = R;
      void* M = nullptr;
      if (v == 1 || v == 2) {
        CHK(hipMemAddressFree(R, 2 * kBytes));
        R2 = nullptr;
        if (v == 1) {
          CHK(hipMemAddressReserve(&R2, 2 * kBytes, align, nullptr, 0));
        } else {
          CHK(hipMalloc(&M, kBytes));
        }
      }
      bool mapped = false;
      if (v != 2) {
        CHK(hipMemCreate(&h2, kBytes, &prop, 0));
        CHK(hipMemMap(R2, kBytes, 0, h2, 0));
        if (v == 3) {
          CHK(hipMemSetAccess(R2, kBytes, &acc, 1));  // the whole (only) chunk
        } else {
          CHK(hipMemSetAccess(R2, kBytes, &acc, 1));
        }
        mapped = ok;
      }
      unsigned* target = v == 2 ? (unsigned*)M : (unsigned*)R2;
      const bool run = v == 2 ? (M != nullptr) : mapped;
      if (run) fill_check(target, p2, p1, dbad, b2);
      std::printf("%s trial %d: VA %p -> %p (same %d); first %llu wrong; second %llu wrong (%llu old pattern, %llu zero)%s\n",
                  names[v], trial, R, (void*)target, (void*)target == R, b1[0], b2[0], b2[1], b2[2],
                  run ? "" : " [not run: mapping failed]");
      if (b1[0] || b2[0]) ++problems;
      if (v != 2) {
        if (mapped) CHK(hipMemUnmap(R2, kBytes));
        if (h2) CHK(hipMemRelease(h2));
        CHK(hipMemAddressFree(R2, 2 * kBytes));
      } else {
        if (M) CHK(hipFree(M));
      }
    }
  }
  // D': a second chunk mapped after the first, access set on the new chunk alone
  {
    ok = true;
    void* R = nullptr;
    hipMemGenericAllocationHandle_t h1{}, h2{};
    CHK(hipMemAddressReserve(&R, 2 * kBytes, align, nullptr, 0));
    CHK(hipMemCreate(&h1, kBytes, &prop, 0));
    CHK(hipMemMap(R, kBytes, 0, h1, 0));
    CHK(hipMemSetAccess(R, kBytes, &acc, 1));
    CHK(hipMemCreate(&h2, kBytes, &prop, 0));
    CHK(hipMemMap((char*)R + kBytes, kBytes, 0, h2, 0));
    hipError_t e = hipMemSetAccess((char*)R + kBytes, kBytes, &acc, 1);
    std::printf("second chunk, access on it alone: %s\n", hipGetErrorString(e));
    unsigned long long b[3] = {0, 0, 0};
    if (e == hipSuccess) {
      fill_check((unsigned*)((char*)R + kBytes), 0x33330000u, 0, dbad, b);
      std::printf("  second chunk fill/check: %llu wrong\n", b[0]);
    } else {
      (void)hipGetLastError();
    }
    (void)hipMemUnmap((char*)R + kBytes, kBytes);
    (void)hipMemUnmap(R, kBytes);
    (void)hipMemRelease(h1);
    (void)hipMemRelease(h2);
    (void)hipMemAddressFree(R, 2 * kBytes);
  }
  std::printf("VMM REPRO DONE: %d trial(s) with wrong data\n", problems);
  return 0;
}
