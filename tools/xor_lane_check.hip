// Checks the VALU cross-lane helpers of csrc/cbg_device.h (xor_lane<D>: DPP and
// gfx950 permlane swaps) against ds_bpermute (__shfl_xor) on the device.
// Build: hipcc --offload-arch=gfx950 -O3 -I include -I combblas-spmm-test_amd/csrc tools/xor_lane_check.hip -o build/xor_check
#include <hip/hip_runtime.h>
#include <cstdio>
#include "cbg_device.h"
using namespace cbg;

__global__ void k_check(int* bad) {
  const int lane = threadIdx.x & 63;
  const int v = lane * 7 + 3 + (threadIdx.x >> 6) * 1000;
  const double dv = v * 0.5 + 1e-3;
  int e = 0;
  e |= (xor_lane<1>(v) != __shfl_xor(v, 1)) << 0;
  e |= (xor_lane<2>(v) != __shfl_xor(v, 2)) << 1;
  e |= (xor_lane<4>(v) != __shfl_xor(v, 4)) << 2;
  e |= (xor_lane<8>(v) != __shfl_xor(v, 8)) << 3;
  e |= (xor_lane<16>(v) != __shfl_xor(v, 16)) << 4;
  e |= (xor_lane<32>(v) != __shfl_xor(v, 32)) << 5;
  e |= (xor_lane<1>(dv) != __shfl_xor(dv, 1)) << 6;
  e |= (xor_lane<16>(dv) != __shfl_xor(dv, 16)) << 7;
  e |= (xor_lane<32>(dv) != __shfl_xor(dv, 32)) << 8;
  if (e) atomicOr(bad, e);
}

int main() {
  int* d;
  hipMalloc(&d, 4);
  hipMemset(d, 0, 4);
  hipLaunchKernelGGL(k_check, dim3(4), dim3(256), 0, 0, d);
  int h = -1;
  hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
  printf("xor_lane check: %s (mask 0x%x)\n", h == 0 ? "OK" : "BAD", h);
  return h == 0 ? 0 : 1;
}
