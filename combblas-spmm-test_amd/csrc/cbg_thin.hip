// cbg_thin.hip -- "thin" big columns of the local multiply by a global
// expand-sort-compress.
//
// A big column of B (flops > the big threshold) normally runs as R (column,
// row panel) pairs, each of which stages ALL of the column's B entries to find
// the ones whose A run reaches its panel.  That pays when every B entry brings
// many products (R-MAT A*A: ~50 per entry).  It does not for a long B column
// whose A columns are short -- GalerkinNew's S*(A*T): S = T^T has ONE nonzero
// per column, so a 50 K-entry column of A*T brings 50 K products spread over
// R panels, and the R pairs staged 8 x 50 K entries for them (the pair kernels
// took 1.5 ms of the 7 ms product for 6 % of its flops).  Such columns (flops
// x 4 < B entries x R) are expanded here instead: every product becomes a
// (column << rowbits | row, value) pair (32-bit keys when they fit), one radix sort orders them
// (cbg_sort.hip, 64-bit counts), one reduce-by-key combines equal (column, row) keys with the
// semiring's add in expansion order, and
// the unique entries land in the fused columns' temporary, from which the
// column-order copy (k_copy_fused) moves them to C after the column scan --
// estimateNNZ_Hash and the hash accumulation of mtSpGEMM.h:362-440, 805-933
// for these columns, as one sort.
#include "cbg_device.h"
#include "cbg_internal.h"

namespace cbg {

namespace {

// thin column i: its B entry count and products; eoff / poff are their scans
__global__ void k_thin_sizes(const int32_t* __restrict__ perm, int n, const int64_t* __restrict__ cpB,
                             int64_t* __restrict__ nbe) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) nbe[i] = cpB[perm[i] + 1] - cpB[perm[i]];
}

// flattened thin entry e (of E): its column index, B position and product count
__global__ void k_thin_entries(const int32_t* __restrict__ perm, int n, const int64_t* __restrict__ eoff,
                               int64_t E, const int64_t* __restrict__ cpB, const int32_t* __restrict__ irB,
                               const int2* __restrict__ cmap, const int4* __restrict__ ainl,
                               int32_t* __restrict__ ecol, int64_t* __restrict__ epos, int64_t* __restrict__ elen) {
  const int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (e >= E) return;
  int lo = 0, hi = n - 1;  // the last i with eoff[i] <= e
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (eoff[mid] <= e) lo = mid; else hi = mid - 1;
  }
  const int64_t p = cpB[perm[lo]] + (e - eoff[lo]);
  ecol[e] = lo;
  epos[e] = p;
  elen[e] = ainl ? ainl[2 * (int64_t)irB[p]].x : cmap[irB[p]].y;
}

// a wave per 64 flattened entries: their products, one per lane per round,
// from the wave's first output position poff[e0]
// INL: the rows and values of an A column of one or two entries come from the entry's lane (k_inline_cols)
template <typename K, int SR, bool INL>
__global__ __launch_bounds__(256) void k_thin_expand(int64_t E, const int32_t* __restrict__ ecol,
                                                     const int64_t* __restrict__ epos,
                                                     const int64_t* __restrict__ poff, const int32_t* __restrict__ irB,
                                                     const double* __restrict__ valB, const int2* __restrict__ cmap,
                                                     const int4* __restrict__ ainl,
                                                     const int32_t* __restrict__ irA, const double* __restrict__ valA,
                                                     int rowbits, K* __restrict__ keys, double* __restrict__ vals) {
  const int64_t e0 = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / WAVE * WAVE;
  if (e0 >= E) return;
  const int lane = lane_id();
  const int64_t e = e0 + lane;
  int s = 0, len = 0, c = 0, r1 = 0;
  double bv = 0.0, v0 = 0.0, v1 = 0.0;
  if (e < E) {
    const int64_t p = epos[e];
    if constexpr (INL) {
      const int k = irB[p];
      const int4 r = ainl[2 * (int64_t)k], v = ainl[2 * (int64_t)k + 1];
      len = r.x;
      s = r.y;
      r1 = r.z;
      v0 = __hiloint2double(v.y, v.x);
      v1 = __hiloint2double(v.w, v.z);
    } else {
      const int2 m = cmap[irB[p]];
      s = m.x;
      len = m.y;
    }
    bv = valB[p];
    c = ecol[e];
  }
  const int incl = wave_incl_scan(len);
  const int total = wave_last(incl);
  const int64_t o = poff[e0];
  for (int q0 = 0; q0 < total; q0 += WAVE) {
    const int q = q0 + lane;
    // product q's entry: the first lane whose inclusive count exceeds q
    int lo = 0, hi = WAVE - 1;
#pragma unroll
    for (int it = 0; it < 6; ++it) {
      const int mid = (lo + hi) >> 1;
      if (__shfl(incl, mid) > q) hi = mid; else lo = mid + 1;
    }
    const int e_s = __shfl(s, lo), e_ex = __shfl(incl - len, lo), e_c = __shfl(c, lo);
    const double e_bv = __shfl(bv, lo);
    bool inl = false, second = false;
    int e_r1 = 0;
    double e_v0 = 0.0, e_v1 = 0.0;
    if constexpr (INL) {
      inl = __shfl(len, lo) <= 2;
      second = q - e_ex == 1;
      e_r1 = __shfl(r1, lo);
      e_v0 = __shfl(v0, lo);
      e_v1 = __shfl(v1, lo);
    }
    if (q < total) {
      if (INL && inl) {
        keys[o + q] = ((K)e_c << rowbits) | (K)(unsigned)(second ? e_r1 : e_s);
        vals[o + q] = Sem<SR>::mul(second ? e_v1 : e_v0, e_bv);
      } else {
        const int a = e_s + (q - e_ex);
        keys[o + q] = ((K)e_c << rowbits) | (K)(unsigned)irA[a];
        vals[o + q] = Sem<SR>::mul(valA[a], e_bv);
      }
    }
  }
}

// unique keys -> rows in the temporary, and the first unique of every column
template <typename K>
__global__ void k_thin_rows(const K* __restrict__ uk, int64_t nruns, int rowbits, int32_t* __restrict__ tir,
                            int64_t* __restrict__ first) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= nruns) return;
  const K k = uk[i];
  tir[i] = (int32_t)(k & (((K)1 << rowbits) - 1));
  if (i == 0 || (uk[i - 1] >> rowbits) != (k >> rowbits)) first[k >> rowbits] = i;
}

__global__ void k_thin_slots(const int32_t* __restrict__ perm, int n, const int64_t* __restrict__ first,
                             int64_t nruns, int64_t base, int32_t* __restrict__ cnt, int64_t* __restrict__ tslot) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int col = perm[i];
  const int64_t f0 = first[i], f1 = i + 1 < n ? first[i + 1] : nruns;
  cnt[col] = (int32_t)(f1 - f0);
  tslot[col] = base + f0;
}

template <typename K>
void thin_impl(const int32_t* perm, int n, int64_t E, int64_t fthin, const cbg_tile& A, const cbg_tile& B,
               const int2* cmap, const int4* ainl, int semiring, int32_t* cnt, int64_t* tslot, int32_t* tir,
               double* tval, int64_t base, int rowbits, int colbits, hipStream_t s, DeferredFree& df) {
  DBuf<int64_t> nbe(n + 1), eoff(n + 1), first(n);
  hipLaunchKernelGGL(k_thin_sizes, dim3((n + 255) / 256), dim3(256), 0, s, perm, n, B.cp, nbe.p);
  exclusive_scan_i64(nbe.p, eoff.p, n, s, &df);
  DBuf<int32_t> ecol(E);
  DBuf<int64_t> epos(E), elen(E + 1), poff(E + 1);
  hipLaunchKernelGGL(k_thin_entries, dim3((unsigned)((E + 255) / 256)), dim3(256), 0, s, perm, n, eoff.p, E, B.cp,
                     B.ir, cmap, ainl, ecol.p, epos.p, elen.p);
  exclusive_scan_i64(elen.p, poff.p, E, s, &df);
  DBuf<K> k0(fthin), uk(fthin);
  DBuf<double> v0(fthin);
  const dim3 g((unsigned)((E + 255) / 256));
#define CBG_THIN_EXPAND(SR, INL)                                                                                  \
  hipLaunchKernelGGL((k_thin_expand<K, SR, INL>), g, dim3(256), 0, s, E, ecol.p, epos.p, poff.p, B.ir, B.val, cmap, \
                     ainl, A.ir, A.val, rowbits, k0.p, v0.p)
  if (semiring == CBG_MIN_PLUS) {
    if (ainl) CBG_THIN_EXPAND(1, true);
    else CBG_THIN_EXPAND(1, false);
  } else {
    if (ainl) CBG_THIN_EXPAND(0, true);
    else CBG_THIN_EXPAND(0, false);
  }
#undef CBG_THIN_EXPAND
  const int end_bit = rowbits + colbits;
  radix_sort_pairs<K>(k0, v0, fthin, end_bit >= 64 ? ~0ull : (1ull << end_bit) - 1, s, &df);
  const int64_t nruns = reduce_by_key<K>(k0.p, v0.p, fthin, semiring, uk.p, tval + base, s, &df);
  hipLaunchKernelGGL(k_thin_rows<K>, dim3((unsigned)((nruns + 255) / 256)), dim3(256), 0, s, uk.p, nruns, rowbits,
                     tir + base, first.p);
  hipLaunchKernelGGL(k_thin_slots, dim3((n + 255) / 256), dim3(256), 0, s, perm, n, first.p, nruns, base, cnt,
                     tslot);
  df.take(nbe);
  df.take(eoff);
  df.take(first);
  df.take(ecol);
  df.take(epos);
  df.take(elen);
  df.take(poff);
  df.take(k0);
  df.take(uk);
  df.take(v0);
}

void thin_any(const int32_t* perm, int n, int64_t E, int64_t fthin, const cbg_tile& A, const cbg_tile& B,
              const int2* cmap, const int4* ainl, int semiring, int32_t* cnt, int64_t* tslot, int32_t* tir,
              double* tval, int64_t base, hipStream_t s, DeferredFree& df) {
  int rowbits = 1, colbits = 1;
  while ((1LL << rowbits) < A.m) ++rowbits;
  while ((1LL << colbits) < (int64_t)n) ++colbits;
  // (column, row) keys in 32 bits when they fit: fewer radix passes, half the key traffic
  if (rowbits + colbits <= 32)
    thin_impl<uint32_t>(perm, n, E, fthin, A, B, cmap, ainl, semiring, cnt, tslot, tir, tval, base, rowbits, colbits, s,
                        df);
  else
    thin_impl<unsigned long long>(perm, n, E, fthin, A, B, cmap, ainl, semiring, cnt, tslot, tir, tval, base, rowbits,
                                  colbits, s, df);
}

}  // namespace

void thin_columns(const int32_t* perm, int n, int64_t E, int64_t fthin, const cbg_tile& A, const cbg_tile& B,
                  const int2* cmap, const int4* ainl, int semiring, int32_t* cnt, int64_t* tslot, int32_t* tir,
                  double* tval, int64_t base, hipStream_t s, DeferredFree& df) {
  if (n <= 0 || fthin <= 0 || E <= 0) return;
  thin_any(perm, n, E, fthin, A, B, cmap, ainl, semiring, cnt, tslot, tir, tval, base, s, df);
}

// the thin columns' entries -> C: a block per column (k_copy_fused's few
// threads per column would walk a 25 K-entry column serially)
__global__ __launch_bounds__(256) void k_copy_thin(const int32_t* __restrict__ perm, const int64_t* __restrict__ tslot,
                                                   const int32_t* __restrict__ cnt, const int64_t* __restrict__ colptr,
                                                   const int32_t* __restrict__ tir, const double* __restrict__ tval,
                                                   int32_t* __restrict__ out_ir, double* __restrict__ out_val) {
  const int col = perm[blockIdx.x];
  const int64_t src = tslot[col], o = colptr[col];
  const int c = cnt[col];
  for (int e = threadIdx.x; e < c; e += blockDim.x) {
    out_ir[o + e] = tir[src + e];
    out_val[o + e] = tval[src + e];
  }
}
void thin_copy(const int32_t* perm, int n, const int64_t* tslot, const int32_t* cnt, const int64_t* colptr,
               const int32_t* tir, const double* tval, int32_t* out_ir, double* out_val, hipStream_t s) {
  if (n > 0)
    hipLaunchKernelGGL(k_copy_thin, dim3(n), dim3(256), 0, s, perm, tslot, cnt, colptr, tir, tval, out_ir, out_val);
}

}  // namespace cbg
