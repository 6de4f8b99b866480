// cbg_local.hip -- per-tile SpGEMM C = A*B on MI355X (gfx950).
//
// Replaces LocalHybridSpGEMM (reference include/CombBLAS/mtSpGEMM.h:212-460)
// with the same contract: for every nonempty column j of B (DCSC order),
// C(:,j) = sum_k A(:,k) * B(k,j) on the semiring, rows ascending, explicit
// zeros kept, empty output columns dropped (SpDCCols(SpTuples) SpDCCols.cpp:108-190).
//
// Pipeline (all on one HIP stream):
//   k_colmap      dense column map of A            (Dcsc::ConstructAux/FillColInds, dcsc.cpp:982-1343)
//   k_flops_seg   flops per B column               (estimateFLOP, mtSpGEMM.h:1056-1134)
//   classify/bin  columns binned by flops
//   k_sym_*       exact nnz per C column            (estimateNNZ_Hash, mtSpGEMM.h:805-933)
//                 wave-level LDS hash (F<=512), block LDS hash (F<=4096),
//                 LDS bitmap over row passes for big columns (+ slab plan)
//   scan          column pointers of C              (prefixsum, mtSpGEMM.h:23-70)
//   k_num_*       numeric: LDS hash accumulate + in-LDS bitonic sort (small/medium),
//                 row slabs with dense LDS accumulators or LDS hash (big columns)
//                 (hash path mtSpGEMM.h:362-440; the heap path :311-360 gives the
//                 same result and is not replicated)
//   compaction    DCSC cp/jc of C
// Products of one B column are expanded "flattened": a chunk of B entries is
// staged in LDS with a prefix sum of A-column lengths, and consecutive lanes
// take consecutive products, so reads of A's columns are coalesced whatever
// their length (R-MAT hub columns included).
#include <atomic>
#include <map>
#include <mutex>
#include <tuple>
#include <cstring>
#include <type_traits>

#include "cbg_device.h"
#include "cbg_internal.h"

namespace cbg {

// Diagnostic ablation mask (CBG_DBG env, default 0; results are WRONG when set):
//   1: k_sym_panel skips its product loop     2: k_num_slab skips pass 0 products
//   4: k_num_slab skips pass 1 products       8: k_num_slab skips the output writes
__constant__ int c_dbg;
//   16: k_num_slab accumulates per-phase wall time (thread 0 of every block) into g_phase
__device__ unsigned long long g_phase[24];
//   32: k_num_slab counts into g_stat: slabs, non-full slabs, B entries, B entries of non-full slabs, products, nout
//   64: k_sym_panel skips the hash-count products of sparse pairs and panel groups
//  128: k_sym_panel does not store the kept bitmaps (their slots are still handed out)
//  256: k_sym_panel leaves a panel group right after its staging
//  512: k_num_slab_hash skips its products       1024: k_num_slab_hash skips its emit
__device__ unsigned long long g_stat[16];  // [4] bitmap slab products, [7] panel hash, [8] column hash products, [9] hash nnz,
                                          // [12..15] symbolic groups: counted, their products, run by panels, their products
__device__ __forceinline__ void phase_mark(unsigned long long& t, int k) {
  if ((c_dbg & 16) && threadIdx.x == 0) {
    const unsigned long long n = wall_clock64();
    atomicAdd(&g_phase[k], n - t);
    t = n;
  }
}

// ----------------------------------------------------------------------------
// small kernels
// ----------------------------------------------------------------------------
// cmap and clen8 (the column lengths clamped at 255, for k_flops_seg: an
// A-sized byte array stays in each XCD's L2, where the 8-byte cmap entries of
// a random gather went to the Infinity Cache -- GalerkinNew's S*(AT) gathers
// 68 M of them)
__global__ void k_colmap(int64_t nzc, const int64_t* __restrict__ cp, const int32_t* __restrict__ jc,
                         int2* __restrict__ cmap, unsigned char* __restrict__ clen8) {
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < nzc) {
    const int len = (int)(cp[i + 1] - cp[i]);
    cmap[jc[i]] = make_int2((int)cp[i], len);
    clen8[jc[i]] = (unsigned char)min(len, 255);
  }
}

// A's columns as inline records for the small-column passes (INL), two int4 per
// column: [2k] = {length, the first row (<= 2 entries) or the start, the second
// row, 0}, [2k+1] = the one or two values (a 32-byte record: one line)
__global__ void k_inline_cols(int64_t n1, const int2* __restrict__ cmap, const int32_t* __restrict__ irA,
                              const double* __restrict__ valA, int4* __restrict__ ainl) {
  const int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (k >= n1) return;
  const int2 m = cmap[k];
  int4 r = make_int4(m.y, m.x, 0, 0), v = make_int4(0, 0, 0, 0);
  if (m.y >= 1 && m.y <= 2) {
    const long long b0 = __double_as_longlong(valA[m.x]);
    r.y = irA[m.x];
    v.x = (int)b0;
    v.y = (int)(b0 >> 32);
    if (m.y == 2) {
      const long long b1 = __double_as_longlong(valA[m.x + 1]);
      r.z = irA[m.x + 1];
      v.z = (int)b1;
      v.w = (int)(b1 >> 32);
    }
  }
  ainl[2 * k] = r;
  ainl[2 * k + 1] = v;
}


// flops of every B column, load-balanced over B's ENTRIES (merge-path style):
// block b takes entries [b*E, (b+1)*E), finds the column holding its first
// entry with a wave-cooperative 64-ary search of cpB, marks where its other
// columns start, and reduces each column's A lengths in LDS; a column cut by a
// block boundary gets one global atomic per block.  Replaces a group of lanes
// per column, whose serial walk over a column's entries (up to FLOP_HEAD, the
// rest on a tail kernel) set the kernel's time on skewed B (GalerkinNew's A*T
// columns: 0.69 ms; the hub tail of S*(AT): 0.39 ms).  Block sums go to
// part[] and one block adds them up (a single-address atomic per block
// serialized 60 K blocks).
constexpr int FSEG_T = 256, FSEG_PER = 8, FSEG_E = FSEG_T * FSEG_PER;
// k[j] = ir[e + j] (j < 8; -1 at or past end); two 16-byte loads when aligned:
// a lane's 8 consecutive entries as 8 scalar loads touch 16 lines per wave
// instruction, eight times over
__device__ __forceinline__ void load8_rows(const int32_t* __restrict__ ir, int64_t e, int64_t end, int (&k)[8]) {
  if (e + 8 <= end && ((reinterpret_cast<uintptr_t>(ir + e) & 15) == 0)) {
    const int4 a = reinterpret_cast<const int4*>(ir + e)[0];
    const int4 b = reinterpret_cast<const int4*>(ir + e)[1];
    k[0] = a.x, k[1] = a.y, k[2] = a.z, k[3] = a.w, k[4] = b.x, k[5] = b.y, k[6] = b.z, k[7] = b.w;
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) k[j] = e + j < end ? ir[e + j] : -1;
  }
}
// the column holding each k_flops_seg block's first entry, from the column
// side: a thread per B column writes its index for the blocks whose first
// entry it holds (one coalesced pass over cpB instead of a 4-round dependent
// 64-ary search at the start of every block: GalerkinNew's S*(AT), 33 K
// blocks, 0.66 ms)
__global__ void k_flops_starts(int64_t nzcB, const int64_t* __restrict__ cpB, int64_t* __restrict__ c_lo) {
  const int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (c >= nzcB) return;
  const int64_t b0 = (cpB[c] + FSEG_E - 1) / FSEG_E, b1 = (cpB[c + 1] + FSEG_E - 1) / FSEG_E;
  for (int64_t b = b0; b < b1; ++b) c_lo[b] = c;
}
__global__ __launch_bounds__(FSEG_T) void k_flops_seg(int64_t nzcB, int64_t nnzB, const int64_t* __restrict__ cpB,
                                                    const int32_t* __restrict__ irB, const int2* __restrict__ cmap,
                                                    const unsigned char* __restrict__ clen8,
                                                    const int64_t* __restrict__ c_lo_blk,
                                                    unsigned long long* __restrict__ flops,
                                                    unsigned long long* __restrict__ part) {
  __shared__ unsigned long long lsum[FSEG_E];
  __shared__ __attribute__((aligned(16))) int head[FSEG_E];  // columns starting at each entry (empty ones too)
  __shared__ int tmp[FSEG_T / WAVE + 4];
  __shared__ unsigned long long wsum[FSEG_T / WAVE];
  const int tid = threadIdx.x;
  const int64_t e0 = blockIdx.x * (int64_t)FSEG_E;
  const int64_t e1 = min(e0 + (int64_t)FSEG_E, nnzB);
  // the largest c with cpB[c] <= e0 (cpB[0] = 0 <= e0 < cpB[nzcB] = nnzB)
  const int64_t c_lo = c_lo_blk[blockIdx.x];
  // the entries' A lengths first: their two dependent loads overlap the
  // column-start marking below instead of following it
  const int i0 = tid * FSEG_PER;
  int k[FSEG_PER];
  load8_rows(irB, e0 + i0, e1, k);
  int len[FSEG_PER];
#pragma unroll
  for (int j = 0; j < FSEG_PER; ++j) len[j] = k[j] >= 0 ? clen8[k[j]] : 0;
  for (int i = tid; i < FSEG_E; i += FSEG_T) lsum[i] = 0ull;
  for (int i = tid; i < FSEG_E / 4; i += FSEG_T) reinterpret_cast<int4*>(head)[i] = make_int4(0, 0, 0, 0);
  __syncthreads();
  // starts of the block's other columns (DCSC columns are nonempty: at most E
  // of them; an empty column would count at its position like any other)
  for (int64_t c = c_lo + 1 + tid; c < nzcB; c += FSEG_T) {
    const int64_t p = cpB[c];
    if (p >= e1) break;
    atomicAdd(&head[p - e0], 1);
  }
  __syncthreads();
  int hd[FSEG_PER];
  {
    const int4 a = *reinterpret_cast<const int4*>(head + i0), b = *reinterpret_cast<const int4*>(head + i0 + 4);
    hd[0] = a.x, hd[1] = a.y, hd[2] = a.z, hd[3] = a.w, hd[4] = b.x, hd[5] = b.y, hd[6] = b.z, hd[7] = b.w;
  }
  static_assert(FSEG_PER == 8, "two int4 head reads per thread");
  int hc = 0;
#pragma unroll
  for (int j = 0; j < FSEG_PER; ++j) hc += hd[j];
  int ncol;
  int col = block_excl_scan<FSEG_T>(hc, tmp, &ncol);  // local column of entry i0, before its own head
#pragma unroll
  for (int j = 0; j < FSEG_PER; ++j)
    if (len[j] == 255) len[j] = cmap[k[j]].y;  // 255 or longer
  unsigned long long acc = 0, bsum = 0;
#pragma unroll
  for (int j = 0; j < FSEG_PER; ++j) {
    if (hd[j]) {
      if (acc) atomicAdd(&lsum[col], acc);
      acc = 0;
      col += hd[j];
    }
    acc += (unsigned long long)len[j];
    bsum += (unsigned long long)len[j];
  }
  if (acc) atomicAdd(&lsum[col], acc);
  __syncthreads();
  for (int t = tid; t <= ncol; t += FSEG_T) {
    const unsigned long long v = lsum[t];
    if (v) atomicAdd(&flops[c_lo + t], v);
  }
  bsum = (unsigned long long)wave_sum64((long long)bsum);
  if (lane_id() == 0) wsum[tid / WAVE] = bsum;
  __syncthreads();
  if (tid == 0) {
    unsigned long long t = 0;
    for (int w = 0; w < FSEG_T / WAVE; ++w) t += wsum[w];
    part[blockIdx.x] = t;
  }
}
// (An LDS-free variant -- a wave per 512 entries, column starts from a global
// bitmap, a DPP segmented scan of the lanes' last-column sums and one global
// atomic per column piece -- measured slower than k_flops_seg: GalerkinNew at
// scale 22 6.76-6.96 vs 6.62-6.80 ms, removed.)

// flops when every A column has exactly one entry: the B column lengths, and
// their total (nnz(B)) in flops[nz]
__global__ void k_flops_unit(int64_t nz, const int64_t* __restrict__ cpB, int64_t* __restrict__ flops) {
  const int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (j < nz) flops[j] = cpB[j + 1] - cpB[j];
  if (j == 0) flops[nz] = cpB[nz];
}
// total of part[0, n) into *out (one block)
__global__ __launch_bounds__(1024) void k_sum_parts(const unsigned long long* __restrict__ part, int64_t n,
                                                    unsigned long long* __restrict__ out) {
  __shared__ unsigned long long ws[1024 / WAVE];
  unsigned long long s = 0;
  for (int64_t i = threadIdx.x; i < n; i += 1024) s += part[i];
  s = (unsigned long long)wave_sum64((long long)s);
  if (lane_id() == 0) ws[threadIdx.x / WAVE] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
    for (int w = 0; w < 1024 / WAVE; ++w) t += ws[w];
    *out = t;
  }
}

// panel column map when A has a single row panel: {start, end} from cmap
__global__ void k_colmap_panel1(int64_t nA1, const int2* __restrict__ cmap, int2* __restrict__ cmapP) {
  const int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (k < nA1) {
    const int2 e = cmap[k];
    cmapP[k] = make_int2(e.x, e.x + e.y);
  }
}

constexpr int MAXBINS = 24;
struct BinThr {
  int64_t t[MAXBINS];  // bin b <=> key <= t[b] (first match); last bin catches the rest
  int nb;
};

// mode 0: key = flops; mode 1: key = (flops > big) ? +inf : cnt.
// A block takes BIN_ITEMS x 256 columns (strided, coalesced), so that the
// per-block histogram atomics -- a few hundred blocks on 16 addresses -- do
// not serialize (one block per 256 columns: 80 us for 2 M columns).
constexpr int BIN_ITEMS = 16;
// big_entries (mode 0, optional): B entries of the columns in bins >= big_bin,
// [0] the big ones, [1] the thin ones
// thin_R > 0: big columns with flops * THIN_RATIO < B entries * thin_R go to
// thin_bin (mode 0) / are skipped like the fused ones (mode 1)
constexpr int64_t THIN_RATIO = 4;
// copy1: a column with one B entry and 0 < flops <= big is C(:,j) = A(:,k) * b,
// nnz = flops: mode 0 writes cnt and bins it with the empty columns, mode 1
// skips it (k_copy_single writes it)
__global__ __launch_bounds__(256) void k_classify(int64_t n, const int64_t* __restrict__ flops,
                                                  int32_t* __restrict__ cnt, int mode, int copy1, int64_t big, BinThr thr,
                                                  uint8_t* __restrict__ bin, int* __restrict__ hist,
                                                  int64_t fused_max, const int64_t* __restrict__ cpB, int big_bin,
                                                  unsigned long long* __restrict__ big_entries,
                                                  unsigned long long* __restrict__ bin_flops, int thin_R,
                                                  int thin_bin) {
  __shared__ int lh[MAXBINS];
  __shared__ unsigned long long lf[MAXBINS];
  __shared__ unsigned long long lbe, lbt;
  if (threadIdx.x < MAXBINS) {
    lh[threadIdx.x] = 0;
    lf[threadIdx.x] = 0;
  }
  if (threadIdx.x == 0) lbe = lbt = 0;
  __syncthreads();
  unsigned long long be = 0, bt = 0;
  const int64_t i0 = blockIdx.x * (int64_t)(256 * BIN_ITEMS) + threadIdx.x;
#pragma unroll 4
  for (int j = 0; j < BIN_ITEMS; ++j) {
    const int64_t i = i0 + j * 256;
    if (i < n) {
      const int64_t f = flops[i];
      int64_t key = f;
      // thin big columns (cbg_thin.hip): few products per B entry, so the R
      // (column, panel) pairs would each stage the whole column for little
      const bool thin = thin_R > 0 && f > big && f * THIN_RATIO < (cpB[i + 1] - cpB[i]) * (int64_t)thin_R;
      const bool single = copy1 && f > 0 && (f <= big || copy1 > 1) && cpB[i + 1] - cpB[i] == 1;
      // numeric bins: big columns last; columns computed by the fused small-column
      // pass (0 < flops <= fused_max), the thin pass or the single-entry copy in
      // bin 0, which the numeric skips
      if (mode == 1) key = (thin || single) ? 0 : (key > big) ? INT64_MAX : (key <= fused_max) ? 0 : (int64_t)cnt[i];
      int b = thr.nb - 1;
      for (int q = 0; q < thr.nb - 1; ++q)
        if (key <= thr.t[q]) { b = q; break; }
      if (mode == 0 && thin) b = thin_bin;
      if (single) {
        b = 0;
        if (mode == 0) cnt[i] = (int32_t)f;
      }
      bin[i] = (uint8_t)b;
      atomicAdd(&lh[b], 1);
      if (f > 0) atomicAdd(&lf[b], (unsigned long long)f);
      if (big_entries && b >= big_bin) (thin ? bt : be) += (unsigned long long)(cpB[i + 1] - cpB[i]);
    }
  }
  if (big_entries && be) atomicAdd(&lbe, be);
  if (big_entries && bt) atomicAdd(&lbt, bt);
  __syncthreads();
  if (threadIdx.x < thr.nb && lh[threadIdx.x]) atomicAdd(&hist[threadIdx.x], lh[threadIdx.x]);
  if (threadIdx.x < thr.nb && lf[threadIdx.x]) atomicAdd(&bin_flops[threadIdx.x], lf[threadIdx.x]);
  if (big_entries && threadIdx.x == 0 && lbe) atomicAdd(big_entries, lbe);
  if (big_entries && threadIdx.x == 0 && lbt) atomicAdd(big_entries + 1, lbt);
}

// hist: the bins' counts (their exclusive prefix is each bin's offset in perm);
// cursor: per-bin fill counters, zero on entry
__global__ __launch_bounds__(256) void k_bin_scatter(int64_t n, const uint8_t* __restrict__ bin, int nb,
                                                     const int* __restrict__ hist, int* __restrict__ cursor,
                                                     int32_t* __restrict__ perm) {
  __shared__ int lc[MAXBINS], lb[MAXBINS], loff[MAXBINS];
  if (threadIdx.x < MAXBINS) lc[threadIdx.x] = 0;
  if (threadIdx.x == 0) {
    int a = 0;
    for (int q = 0; q < nb; ++q) {
      loff[q] = a;
      a += hist[q];
    }
  }
  __syncthreads();
  const int64_t i0 = blockIdx.x * (int64_t)(256 * BIN_ITEMS) + threadIdx.x;
  int b[BIN_ITEMS], slot[BIN_ITEMS];
#pragma unroll
  for (int j = 0; j < BIN_ITEMS; ++j) {
    const int64_t i = i0 + j * 256;
    b[j] = i < n ? bin[i] : -1;
  }
#pragma unroll
  for (int j = 0; j < BIN_ITEMS; ++j) slot[j] = b[j] >= 0 ? atomicAdd(&lc[b[j]], 1) : 0;
  __syncthreads();
  if (threadIdx.x < nb)
    lb[threadIdx.x] = loff[threadIdx.x] + (lc[threadIdx.x] ? atomicAdd(&cursor[threadIdx.x], lc[threadIdx.x]) : 0);
  __syncthreads();
#pragma unroll
  for (int j = 0; j < BIN_ITEMS; ++j)
    if (b[j] >= 0) perm[lb[b[j]] + slot[j]] = (int32_t)(i0 + j * 256);
}

struct RowVal {
  int row;
  double v;
};
struct alignas(8) PackedRV {
  int row;
  float v;
};
// (row, f64 value) records of A's entries for the f64-valued path: 12 bytes,
// one dwordx3 gather per product instead of a row load and a value load
struct alignas(4) PackedRVD {
  int row, vlo, vhi;
};

// claim `row` in an LDS hash of mask + 1 slots (linear probing from h):
// 1 if this call inserted it, 0 if it was there
__device__ __forceinline__ int hash_claim(int* keys, unsigned h, unsigned mask, int row) {
  while (true) {
    const int old = atomicCAS(&keys[h], EMPTY_KEY, row);
    if (old == EMPTY_KEY) return 1;
    if (old == row) return 0;
    h = (h + 1) & mask;
  }
}

// insert-or-accumulate into an LDS hash table (linear probing)
template <int SR, int LOGT>
__device__ __forceinline__ void hash_acc(int* keys, double* vals, int row, double v) {
  constexpr int T = 1 << LOGT;
  unsigned h = hash_slot<LOGT>(row);
  while (true) {
    const int old = atomicCAS(&keys[h], EMPTY_KEY, row);
    if (old == EMPTY_KEY || old == row) {
      Sem<SR>::lds_acc(&vals[h], v);
      return;
    }
    h = (h + 1) & (T - 1);
  }
}

// the same for a table of any size T (multiplicative hash scaled to [0, T))
template <int T>
__device__ __forceinline__ unsigned hash_slot_t(int key) {
  return (unsigned)(((unsigned long long)((unsigned)key * 0x9E3779B1u) * T) >> 32);
}
template <int SR, int T>
__device__ __forceinline__ void hash_acc_t(int* keys, double* vals, int row, double v) {
  unsigned h = hash_slot_t<T>(row);
  while (true) {
    const int old = atomicCAS(&keys[h], EMPTY_KEY, row);
    if (old == EMPTY_KEY || old == row) {
      Sem<SR>::lds_acc(&vals[h], v);
      return;
    }
    h = h + 1 == T ? 0u : h + 1;
  }
}
// rank of this lane among the active lanes of mask m below it
__device__ __forceinline__ int lane_rank(unsigned long long m) {
  return __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}

// ----------------------------------------------------------------------------
// symbolic: wave per column, LDS hash of row ids
// ----------------------------------------------------------------------------
template <int LOGT>
struct SymWaveLds {
  static constexpr int T = 1 << LOGT;
  static constexpr int INTS = T + (WAVE + 4) + WAVE;  // keys, pref[65]+pad, st[64]
};

template <int LOGT>
__global__ __launch_bounds__(256) void k_sym_wave(const int32_t* __restrict__ perm, int n,
                                                  const int64_t* __restrict__ cpB, const int32_t* __restrict__ irB,
                                                  const int2* __restrict__ cmap, const int32_t* __restrict__ irA,
                                                  int32_t* __restrict__ cnt) {
  constexpr int T = 1 << LOGT;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int w = threadIdx.x / WAVE, lane = lane_id();
  int* keys = reinterpret_cast<int*>(smem) + w * SymWaveLds<LOGT>::INTS;
  int* pref = keys + T;
  int* st = pref + WAVE + 4;
  const int idx = blockIdx.x * (blockDim.x / WAVE) + w;
  if (idx >= n) return;
  const int col = perm[idx];
  for (int j = lane; j < T; j += WAVE) keys[j] = EMPTY_KEY;
  const int64_t p1 = cpB[col + 1];
  int count = 0;
  for (int64_t c0 = cpB[col]; c0 < p1; c0 += WAVE) {
    const int64_t p = c0 + lane;
    int s = 0, len = 0;
    if (p < p1) {
      int2 e = cmap[irB[p]];
      s = e.x;
      len = e.y;
    }
    const int incl = wave_incl_scan(len);
    const int total = wave_last(incl);
    pref[lane + 1] = incl;
    if (lane == 0) pref[0] = 0;
    st[lane] = seg_stage(s, incl - len);
    wave_sync();
    wave_products(
        pref, WAVE, 0, total, [&](int sg) { return SegI{seg_off(st, pref, sg)}; },
        [&](const SegI& g, int u) { return irA[g.off + u]; },
        [&](int row) {
          count += hash_claim(keys, hash_slot<LOGT>(row), T - 1, row);
        });
    wave_sync();
  }
  count = wave_sum(count);
  if (lane == 0) cnt[col] = count;
}

// symbolic: block per column
template <int LOGT, int BS>
struct SymBlockLds {
  static constexpr int T = 1 << LOGT;
  static constexpr int INTS = T + (BS + 4) + BS + (BS / WAVE + 8) + 2 * BS;  // + inline first-product index, 2nd row
};
// a staged segment of an inline-record A column (INL): rows of the one or two
// entries (ex = the segment's first product, -1: rows in irA)
struct SegIL {
  int off, ex, r1;
};

template <int LOGT, int BS, bool INL>
__global__ __launch_bounds__(BS) void k_sym_block(const int32_t* __restrict__ perm, const int64_t* __restrict__ cpB,
                                                  const int32_t* __restrict__ irB, const int2* __restrict__ cmap,
                                                  const int4* __restrict__ ainl, const int32_t* __restrict__ irA,
                                                  int32_t* __restrict__ cnt) {
  constexpr int T = 1 << LOGT;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int* keys = reinterpret_cast<int*>(smem);
  int* pref = keys + T;
  int* st = pref + BS + 4;
  int* tmp = st + BS;
  int& s_count = tmp[BS / WAVE + 4];  // outside block_excl_scan's scratch
  int* sx = tmp + BS / WAVE + 8;  // INL: inline segment's first product (-1: none)
  int* sr1 = sx + BS;             // INL: its second row
  const int tid = threadIdx.x;
  const int col = perm[blockIdx.x];
  for (int j = tid; j < T; j += BS) keys[j] = EMPTY_KEY;
  if (tid == 0) s_count = 0;
  __syncthreads();
  const int64_t p1 = cpB[col + 1];
  int count = 0;
  for (int64_t c0 = cpB[col]; c0 < p1; c0 += BS) {
    const int64_t p = c0 + tid;
    int s = 0, len = 0, r1 = 0;
    if (p < p1) {
      if constexpr (INL) {
        const int4 r = ainl[2 * (int64_t)irB[p]];
        len = r.x;
        s = r.y;
        r1 = r.z;
      } else {
        int2 e = cmap[irB[p]];
        s = e.x;
        len = e.y;
      }
    }
    int total;
    const int ex = block_excl_scan<BS>(len, tmp, &total);
    pref[tid] = ex;
    if (tid == BS - 1) pref[BS] = total;
    st[tid] = seg_stage(s, ex);
    if constexpr (INL) {
      sx[tid] = len <= 2 ? ex : -1;
      sr1[tid] = r1;
    }
    __syncthreads();
    if constexpr (INL) {
      block_products<BS>(
          pref, total, [&](int sg) { return SegIL{seg_off(st, pref, sg), sx[sg], sr1[sg]}; },
          [&](const SegIL& g, int u) { return g.ex < 0 ? irA[g.off + u] : u == g.ex ? g.off + u : g.r1; },
          [&](int row) { count += hash_claim(keys, hash_slot<LOGT>(row), T - 1, row); });
    } else {
      block_products<BS>(
          pref, total, [&](int sg) { return SegI{seg_off(st, pref, sg)}; },
          [&](const SegI& g, int u) { return irA[g.off + u]; },
          [&](int row) { count += hash_claim(keys, hash_slot<LOGT>(row), T - 1, row); });
    }
    __syncthreads();
  }
  count = wave_sum(count);
  if (lane_id() == 0 && count) atomicAdd(&s_count, count);
  __syncthreads();
  if (tid == 0) cnt[col] = s_count;
}

// ----------------------------------------------------------------------------
// big columns: row panels x bitmap + rank
//
// The rows of A are cut into panels of P = 2^plog rows (P <= 2^18, so a
// panel's bitmap is <= 32 KiB of LDS); A(:,k) restricted to panel r is a
// contiguous run of A's column (rows are sorted), located once by
// k_colmap_panels_col.  A big column j of B is then processed as R independent
// (j, r) sub-problems: C(panel r, j) = A(panel r, :) * B(:, j), whose sorted
// outputs concatenate in panel order.  Each (j, r) is one workgroup in the
// symbolic (bitmap -> counts, slab plan) and numeric (bitmap -> ranks ->
// accumulate at rank) kernels; a (j, r) holding more than SLAB_CAP nonzeros is
// cut into row slabs of whole fine ranges.
// ----------------------------------------------------------------------------
#ifndef CBG_FINE_LOG
#define CBG_FINE_LOG 13
#endif
#ifndef CBG_SLAB_CAP
#define CBG_SLAB_CAP 12032
#endif
#ifndef CBG_PANEL_LOG_MAX
#define CBG_PANEL_LOG_MAX 18
#endif
#ifndef CBG_SLAB_LARGE_BS
#define CBG_SLAB_LARGE_BS 1024
#endif
constexpr int FINE_LOG = CBG_FINE_LOG;            // fine row range (default 8192 rows = 256 bitmap words)
constexpr int SLAB_CAP = CBG_SLAB_CAP;            // max nnz of a slab (LDS value array, default 94 KiB)
constexpr int PANEL_LOG_MAX = CBG_PANEL_LOG_MAX;  // max rows of a panel (LDS bitmap, default 32 KiB)
static_assert(SLAB_CAP >= (1 << FINE_LOG), "a fine range must fit one slab");
constexpr int SLAB_WORDS = 1 << (PANEL_LOG_MAX - 5);
constexpr int NFINE_MAX = 1 << (PANEL_LOG_MAX - FINE_LOG);  // fine ranges (= max slabs) per panel
#ifndef CBG_BIG_BS
#define CBG_BIG_BS 512
#endif
constexpr int BIG_BS = CBG_BIG_BS;
#ifndef CBG_PAIR_LOAD_NUM  // symbolic hash of a (column, panel) pair: T >= (NUM/DEN) * products
#define CBG_PAIR_LOAD_NUM 2
#define CBG_PAIR_LOAD_DEN 1
#endif
#ifndef CBG_SPARSE_SLAB_MAX
#define CBG_SPARSE_SLAB_MAX 4096
#endif
constexpr int SPARSE_SLAB_MAX = CBG_SPARSE_SLAB_MAX;  // products of a (column, panel) pair counted by hash -> hash slab
// group rank slabs (k_num_slab_grank): spans <= 2^22 rows (level 1: a bit per
// 32 rows, <= 4096 words), <= GRANK_PMAX products (8 per thread: 80 VGPRs, 3
// blocks per CU; sym_group flags the groups with more, which stay hash slabs)
constexpr int GRANK_SPAN_LOG = 22;
constexpr int GRANK_PMAX = 4096;
constexpr int SLAB_SPARSE = 1 << 30;    // desc.w flag: hash-mode slab (count in the low bits)
constexpr int SLAB_MANYP = 1 << 29;     // desc.w flag: a panel group's slab of > GRANK_PMAX products
constexpr int SLAB_CNT_MASK = SLAB_MANYP - 1;

// Panel column maps of A: entry (r, k) = (first, end) of column k's entries
// in row panel r (layout: PMap below).  A panel without rows of A(:,k) gets (q, q) with q
// the lower bound of the panel's first row, so that (cmapP[r0].x,
// cmapP[r1].y) is A(:,k)'s run over panels r0..r1 (panel groups); columns
// absent from A stay (0, 0) (the caller's memset).  One
// thread per nonempty A column walks its rows once (short columns) or
// binary-searches each panel boundary (long ones) and writes its R entries,
// so every store of a wave is one row of the map at consecutive columns
// (coalesced; one thread per entry scattering over R rows was 3x slower).
//
// Layout: entry (r, k) at r * sr + k * sk.  Panel-major (sr = n + 1, sk = 1)
// or column-major (sr = 1, sk = R: a column's R entries share one or two
// lines, read once by the column's R units when they run together on one
// XCD); the whole-column map of the column bins as a map of one panel (sr = 0,
// sk = 1).
struct PMap {
  const int2* p;
  int64_t sr;
  int sk;
  __device__ __forceinline__ int2 at(int r, int k) const { return p[(int64_t)r * sr + (int64_t)k * sk]; }
};
// A(:,k) = rows irA[a, e): its run inside every row panel, one thread
__device__ __forceinline__ void panel_runs(const int32_t* __restrict__ irA, int a, int e, int plog, int R,
                                           int64_t sr, int sk, int64_t k, int2* __restrict__ cmapP) {
  int pos = a;
  for (int r = 0; r < R; ++r) {
    const int lo = pos;
    if (r == R - 1) {
      pos = e;
    } else {
      const int bound = (r + 1) << plog;
      if (e - pos <= 32) {
        while (pos < e && irA[pos] < bound) ++pos;
      } else {
        pos = lower_bound_g(irA, pos, e, bound);
      }
    }
    cmapP[r * sr + k * sk] = make_int2(lo, pos);
  }
}
__global__ void k_colmap_panels_col(int64_t nzcA, const int64_t* __restrict__ cpA, const int32_t* __restrict__ jcA,
                                    const int32_t* __restrict__ irA, int plog, int R, int64_t sr, int sk,
                                    int2* __restrict__ cmapP) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= nzcA) return;
  panel_runs(irA, (int)cpA[i], (int)cpA[i + 1], plog, R, sr, sk, jcA[i], cmapP);
}
// the same for the A columns the big B columns reference only (a wave per big
// column, a lane per entry; a column referenced twice is written twice alike)
__global__ void k_colmap_panels_entries(const int32_t* __restrict__ perm_big, int nbig,
                                        const int64_t* __restrict__ cpB, const int32_t* __restrict__ irB,
                                        const int2* __restrict__ cmap, const int32_t* __restrict__ irA, int plog,
                                        int R, int64_t sr, int sk, int2* __restrict__ cmapP) {
  const int64_t w = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / WAVE;
  if (w >= nbig) return;
  const int col = perm_big[w];
  for (int64_t p = cpB[col] + lane_id(); p < cpB[col + 1]; p += WAVE) {
    const int k = irB[p];
    const int2 e = cmap[k];
    panel_runs(irA, e.x, e.x + e.y, plog, R, sr, sk, k, cmapP);
  }
}

// symbolic of the big columns, one block per (column, panel group).
//
// A pair (column, panel) is counted into a bitmap of the panel's rows with
// per fine range counts and a slab plan (the bitmap optionally kept for the
// numeric phase); a pair with few products is counted with an LDS hash sized
// to it and becomes ONE sparse (hash) slab, so that its cost scales with its
// products, not with the panel's 2^plog rows.
//
// Panel groups: a column with few products per panel (R-MAT rows are
// scrambled, so a column's products spread evenly over the panels) is taken
// 2^glog panels at a time -- the launch class fixes glog from the column's
// flops -- and a group whose nonzeros fit one hash slab becomes ONE sparse
// slab over the group's rows.  That shares the B column staging and column
// map hops of up to 16 panels and reads A's runs over the group contiguously.
constexpr int GROUP_LOG_MAX = 6;      // groups of up to 64 panels (scale 24: R = 64 panels per column)
#ifndef CBG_GROUP_PRODUCTS
#define CBG_GROUP_PRODUCTS 4096
#endif
// expected products of a group (launch class thresholds).  With hash-slab
// numerics 3072 was best (1536/2048/4096 slower); with the group rank slabs
// 4096 is: scale 22 317-321 ms vs 332 (3072), 323 (3584), 333 (4608), 357
// (2048), 357 (5120), 393 (6144) -- past ~4096 expected products the groups
// overflow the symbolic's table and the group rank slab's products
constexpr int GROUP_PRODUCTS = CBG_GROUP_PRODUCTS;
#ifndef CBG_SYM_WAVES_OF_UNITS  // persistent symbolic grid: resident blocks x this
#define CBG_SYM_WAVES_OF_UNITS 32  // 1: -2 % (static stride meets hub-column imbalance); 16-32: +1 % at scale 22
#endif
#ifndef CBG_GROUP_T
#define CBG_GROUP_T 8192  // = the panel bitmap words: group launches keep 4 blocks/CU (+1 % at scale 22 over 16384 at load 1/2)
#endif
#ifndef CBG_SYM_LOAD_NUM  // symbolic group hash: T >= (NUM/DEN) * products
#define CBG_SYM_LOAD_NUM 3
#define CBG_SYM_LOAD_DEN 2
#endif
constexpr int GROUP_T = CBG_GROUP_T;  // LDS hash of a group's symbolic (ints)
constexpr int SPARSE_NNZ_MAX = 4096;  // nonzeros of a hash slab (largest numeric table: 8192)

struct SymPanelArgs {
  const int32_t* perm_big;
  int R, plog, glog, boff, hwords;
  int ncls;  // columns of this launch class (units = ncls x panel groups)
  const int64_t* cpB;
  const int32_t* irB;
  PMap pm;
  const int32_t* irA;
  int64_t m;
  int32_t* cnt;
  int32_t* cnt_br;
  int4* desc;
  int32_t* nslab;
  unsigned* gbm;
  int gbm_slots;
  int* gbm_next;
  int* gbm_slot;
  // a multi-slab pair's cut positions (offsets into each B entry's run at every
  // inner slab boundary) for the numeric: cuts[pcoff[br] + (s - 1) * nb + j]
  int* cuts;
  unsigned long long* cuts_next;
  long long cuts_cap;
  int* pcoff;  // per (column, panel) pair, -1: none (pre-set)
  // group units whose products or nonzeros overflow one hash slab (rare: a few
  // per phase at scale 22 / 24), run by panels in k_sym_deferred: (b, col, r0, r1)
  int4* defer;
  int* defer_n;
};

// staging of a unit fetched ahead: ok = 1: p0/p1 of the column; ok = 2: also
// this thread's first-chunk A run (s, len) over the unit's rows
struct SymPre {
  int64_t p0 = 0, p1 = 0;
  int s = 0, len = 0;
  int ok = 0;
};

struct SymPanelLds {
  unsigned* bm;  // [hwords]: panel bitmap or hash keys
  int* fine;     // [NFINE_MAX]
  int* pref;     // [BIG_BS + 4]
  int* st;       // [BIG_BS]
  int* tmp;      // scan scratch [BIG_BS / WAVE + 4]; tmp[NW + 3]: overflow count
  int* ovf;      // [SYM_OVF_CAP] rows deferred by hash_claim_bounded
};
#ifndef CBG_SYM_OVF  // probes of a symbolic hash insert before it is deferred (0: unbounded)
#define CBG_SYM_OVF 2
#endif
// rows of the symbolic overflow list: what is left of 160 KiB / 4 blocks per
// CU after the 8192-word bitmap and the staging arrays (the launch keeps 4 blocks)
constexpr int SYM_OVF_CAP = CBG_SYM_OVF > 0 ? 896 : 0;
static_assert(SYM_OVF_CAP >= NFINE_MAX + 2, "the cut pass keeps a pair's slab rows in the overflow list");

// hash_claim with at most NPROBE probes; a row without a slot by then goes to
// an LDS overflow list (one atomic per wave) that dense waves insert after the
// product loop, resuming at probe NPROBE.  A wave's linear-probe loop runs
// until its slowest lane has found a slot; bounding it and finishing the few
// long probes with full waves was +1.2 % at scale 22 in the symbolic (s8 vs
// s8n, profiles/r04_ab_hash_sym.json).  The same in the numeric hash slabs was
// -1 % (their LDS time is not in the probes: the atomics counted by rocprofv3
// dropped 8 %) and an expand-sort-compress numeric without a hash table
// (products into LDS at their index, counting sort by row bucket, heads
// compressed per bucket) -12 %: its products ran 20 % faster, the sort and
// compression twice as long as the hash emit (profiles/r04_hash_pmc.txt).
// Returns 1 if this call inserted the row.  A full list falls back to inline probing.
template <int NPROBE>
__device__ __forceinline__ int hash_claim_bounded(int* keys, unsigned h, unsigned mask, int row, int* ocount,
                                                  int* orow, int cap) {
  int got = 0;
  bool done = false;
#pragma unroll
  for (int k = 0; k < NPROBE; ++k) {
    if (!done) {
      const int old = atomicCAS(&keys[h], EMPTY_KEY, row);
      if (old == EMPTY_KEY || old == row) {
        got = old == EMPTY_KEY;
        done = true;
      } else {
        h = (h + 1) & mask;
      }
    }
  }
  const unsigned long long m = __ballot(!done);
  if (m) {
    const int leader = __ffsll((long long)m) - 1;
    int base = 0;
    if (lane_id() == leader) base = atomicAdd(ocount, __popcll(m));
    base = __builtin_amdgcn_readlane(base, leader);
    if (!done) {
      const int idx = base + lane_rank(m);
      if (idx < cap) orow[idx] = row;
      else got = hash_claim(keys, h, mask, row);
    }
  }
  return got;
}
// the deferred rows (after a barrier): this thread's insertions
template <int NPROBE>
__device__ __forceinline__ int hash_claim_drain(int* keys, unsigned mask, const int* orow, int n) {
  int got = 0;
  for (int i = threadIdx.x; i < n; i += BIG_BS) {
    const int row = orow[i];
    got += hash_claim(keys, (((unsigned)row * 0x9E3779B1u) + NPROBE) & mask, mask, row);
  }
  return got;
}

// one (column, panel) pair
template <class H>
__device__ __forceinline__ void sym_pair(const SymPanelArgs& a, const SymPanelLds& L, int b, int col, int r,
                                         const SymPre& pre, H& hook) {
  constexpr int BS = BIG_BS;
  const int R = a.R, plog = a.plog;
  const int64_t* __restrict__ cpB = a.cpB;
  const int32_t* __restrict__ irB = a.irB;
  const int32_t* __restrict__ irA = a.irA;
  int32_t* __restrict__ cnt = a.cnt;
  int32_t* __restrict__ cnt_br = a.cnt_br;
  int4* __restrict__ desc = a.desc;
  int32_t* __restrict__ nslab = a.nslab;
  unsigned* __restrict__ gbm = a.gbm;
  const int gbm_slots = a.gbm_slots;
  int* __restrict__ gbm_next = a.gbm_next;
  int* __restrict__ gbm_slot = a.gbm_slot;
  const int pwords = 1 << (plog - 5);
  const int nfine = 1 << (plog - FINE_LOG);
  unsigned* bm = L.bm;
  int* fine = L.fine;
  int* pref = L.pref;
  int* st = L.st;
  int* tmp = L.tmp;
  const int tid = threadIdx.x;
  const int64_t br = (int64_t)b * R + r;
  const int R0 = r << plog;
  const int R1 = (int)min((int64_t)R0 + (1LL << plog), a.m);
  const int words = (R1 - R0 + 31) >> 5;
  auto cm = [&](int k) { return a.pm.at(r, k); };
  unsigned long long tmark = wall_clock64();
  const int64_t p0 = pre.ok ? pre.p0 : cpB[col], p1 = pre.ok ? pre.p1 : cpB[col + 1];
  if (p1 - p0 <= BS) {
    // single chunk: stage once; a pair with few products is counted with an
    // LDS hash sized to it and becomes ONE sparse (hash) slab -- its cost then
    // scales with its products, not with the panel's 2^plog rows
    const int64_t p = p0 + tid;
    int s = 0, len = 0;
    if (pre.ok == 2) {
      s = pre.s;
      len = pre.len;
    } else if (p < p1) {
      const int2 e = cm(irB[p]);
      s = e.x;
      len = e.y - e.x;
    }
    int total;
    const int ex = block_excl_scan<BS>(len, tmp, &total);
    pref[tid] = ex;
    if (tid == BS - 1) pref[BS] = total;
    st[tid] = seg_stage(s, ex);
    hook(1);
    phase_mark(tmark, 8);
    int T = 512;
    while (T * CBG_PAIR_LOAD_DEN < CBG_PAIR_LOAD_NUM * total) T <<= 1;
    if (total <= SPARSE_SLAB_MAX && T <= pwords) {
      // the count of a sparse pair from the panel bitmap: one ds_or per product
      // (no returning CAS, no probes), a popcount of the panel's words; the
      // zeroing is the hash table's for pairs of 2048-4096 products (32 KiB).
      // (An LDS hash with bounded probes, before round 5: 0.8 % slower at 22.)
      for (int j = tid; j < pwords / 4; j += BS) reinterpret_cast<uint4*>(bm)[j] = make_uint4(0u, 0u, 0u, 0u);
      if (tid == 0) fine[0] = 0;
      __syncthreads();
      if (!(c_dbg & 64))
        block_products<BS>(
            pref, total, [&](int sg) { return SegI{seg_off(st, pref, sg)}; },
            [&](const SegI& g, int u) { return irA[g.off + u] - R0; },
            [&](int row) { atomicOr(&bm[row >> 5], 1u << (row & 31)); });
      hook(2);
      __syncthreads();
      int count = 0;
      for (int j = tid; j < words / 4 + 1; j += BS)
        if (4 * j < words) {
          const uint4 x = reinterpret_cast<const uint4*>(bm)[j];
          count += __popc(x.x) + __popc(x.y) + __popc(x.z) + __popc(x.w);  // (words past the panel's end are zero)
        }
      count = wave_sum(count);
      if (lane_id() == 0 && count) atomicAdd(&fine[0], count);
      __syncthreads();
      if (tid == 0) {
        const int cnt_pair = fine[0];
        nslab[br] = cnt_pair ? 1 : 0;
        if (cnt_pair) desc[(int64_t)br * NFINE_MAX] = make_int4(R0, R1, 0, cnt_pair | SLAB_SPARSE);
        cnt_br[br] = cnt_pair;
        if (gbm_slot) gbm_slot[br] = -1;
        if (cnt_pair) atomicAdd(&cnt[col], cnt_pair);
      }
      phase_mark(tmark, 9);
      return;
    }
    for (int j = tid; j < pwords / 4; j += BS) reinterpret_cast<uint4*>(bm)[j] = make_uint4(0u, 0u, 0u, 0u);
    if (tid < NFINE_MAX) fine[tid] = 0;
    __syncthreads();
    if (!(c_dbg & 1))
      block_products<BS>(
          pref, total, [&](int sg) { return SegI{seg_off(st, pref, sg)}; },
          [&](const SegI& g, int u) { return irA[g.off + u] - R0; },
          [&](int row) { atomicOr(&bm[row >> 5], 1u << (row & 31)); });
    __syncthreads();
  } else {
  for (int j = tid; j < pwords / 4; j += BS) reinterpret_cast<uint4*>(bm)[j] = make_uint4(0u, 0u, 0u, 0u);
  if (tid < NFINE_MAX) fine[tid] = 0;
  __syncthreads();
  for (int64_t c0 = p0; c0 < p1; c0 += BS) {    const int64_t p = c0 + tid;
    int s = 0, len = 0;
    if (p < p1) {
      const int2 e = cm(irB[p]);
      s = e.x;
      len = e.y - e.x;
    }
    int total;
    const int ex = block_excl_scan<BS>(len, tmp, &total);
    pref[tid] = ex;
    if (tid == BS - 1) pref[BS] = total;
    st[tid] = seg_stage(s, ex);
    hook(1);
    __syncthreads();
    if (!(c_dbg & 1))
      block_products<BS>(
          pref, total, [&](int sg) { return SegI{seg_off(st, pref, sg)}; },
          [&](const SegI& g, int u) { return irA[g.off + u] - R0; },
          [&](int row) { atomicOr(&bm[row >> 5], 1u << (row & 31)); });
    __syncthreads();
  }
  }
  hook(2);
  phase_mark(tmark, 10);
  // per fine range popcounts: coalesced words; a wave's 64 words lie in one
  // fine range (2^(FINE_LOG-5) >= 64 words)
  static_assert(FINE_LOG - 5 >= 6, "fine range must hold a wave's words");
  // keep this pair's bitmap for the numeric phase while bitmap slots last
  // (every bitmap-mode pair: re-marking the ones of 8 K-32 K products in the
  // numeric instead measured 3-5 % slower, rounds 2 and 5)
  unsigned* gdst = nullptr;
  if (gbm) {
    if (tid == 0) {
      int slot = atomicAdd(gbm_next, 1);
      if (slot >= gbm_slots) slot = -1;
      gbm_slot[br] = slot;
      tmp[0] = slot;
    }
    __syncthreads();
    if (tmp[0] >= 0) gdst = gbm + (int64_t)tmp[0] * pwords;
  }
  {
    // wave w owns the fine ranges w, w + 8, ...: its lanes read (and store)
    // 64 consecutive words per step, and one wave reduction per fine range
    // (16-byte vectors: a lane takes 4 consecutive words; words past the
    // panel's end are the zeroed tail of the bitmap)
    constexpr int FW = 1 << (FINE_LOG - 5);  // words per fine range
    static_assert(FW % (4 * WAVE) == 0, "fine range of whole 16-byte lane vectors");
    const int w = tid / WAVE, lane = lane_id();
    for (int f = w; f * FW < words; f += BS / WAVE) {
      int c = 0;
#pragma unroll
      for (int q = 0; q < FW; q += 4 * WAVE) {
        const int j = f * FW + q + 4 * lane;
        if (j < words) {
          const uint4 x = *reinterpret_cast<const uint4*>(bm + j);
          if (gdst && !(c_dbg & 128)) st_stream4(&gdst[j], x);
          c += __popc(x.x) + __popc(x.y) + __popc(x.z) + __popc(x.w);
        }
      }
      c = wave_sum(c);
      if (lane == 0) fine[f] = c;
    }
  }
  __syncthreads();
  phase_mark(tmark, 11);
  if (tid < WAVE) {
    // slab plan by wave 0 (nfine <= 64): one slab from the first to the last
    // non-empty fine range when the pair fits SLAB_CAP, else lane 0 groups
    // consecutive fine ranges greedily while a slab holds <= SLAB_CAP
    static_assert(NFINE_MAX <= WAVE, "fine ranges per panel");
    const int cf = tid < nfine ? fine[tid] : 0;
    const int total = wave_sum(cf);
    const unsigned long long nzmask = __ballot(cf != 0);
    int4* d = desc + (int64_t)br * NFINE_MAX;
    if (tid == 0) {
      int ns = 0;
      if (total > 0 && total <= SLAB_CAP) {
        const int f0 = __ffsll((long long)nzmask) - 1;
        const int f1 = 63 - __clzll((long long)nzmask);
        d[0] = make_int4(R0 + (f0 << FINE_LOG), min(R0 + ((f1 + 1) << FINE_LOG), R1), 0, total);
        ns = 1;
      } else if (total > 0) {
        int run = 0, g_lo = -1, g_hi = 0, g_cnt = 0;
        for (int f = 0; f < nfine; ++f) {
          const int c = fine[f];
          if (c == 0) continue;
          const int lo = R0 + (f << FINE_LOG);
          const int hi = min(lo + (1 << FINE_LOG), R1);
          if (g_cnt && g_cnt + c > SLAB_CAP) {
            d[ns++] = make_int4(g_lo, g_hi, run - g_cnt, g_cnt);
            g_cnt = 0;
          }
          if (g_cnt == 0) g_lo = lo;
          g_hi = hi;
          g_cnt += c;
          run += c;
        }
        if (g_cnt) d[ns++] = make_int4(g_lo, g_hi, run - g_cnt, g_cnt);
      }
      cnt_br[br] = total;
      nslab[br] = ns;
      if (total) atomicAdd(&cnt[col], total);
      // for the cut pass: the slab count and the slabs' first rows (in the
      // overflow list, idle on the bitmap path)
      for (int q = 1; q < ns; ++q) L.ovf[1 + q] = d[q].x;
      L.ovf[0] = ns;
    }
  }
  if (a.cuts) {
    // Cut positions of a multi-slab pair, once: for every B entry the start of
    // its A run's part in each slab after the first (a lower bound per slab
    // boundary, the run's rows ascending), as offsets from the run's start.
    // The numeric staged two binary searches per entry per slab instead.
    __syncthreads();
    const int ns = L.ovf[0];
    if (ns > 1) {
      const int64_t nb = p1 - p0;
      if (tid == 0) {
        const long long need = (long long)(ns - 1) * nb;
        long long off = (long long)atomicAdd(a.cuts_next, (unsigned long long)need);
        if (off + need > a.cuts_cap) off = -1;
        a.pcoff[br] = (int)off;
        L.ovf[1] = (int)off;
      }
      __syncthreads();
      const int off = L.ovf[1];
      if (off >= 0)
        for (int64_t j = tid; j < nb; j += BS) {
          const int2 ce = cm(irB[p0 + j]);
          int pos = ce.x;
          for (int q = 1; q < ns; ++q) {
            pos = lower_bound_g(irA, pos, ce.y, L.ovf[1 + q]);
            a.cuts[(int64_t)off + (int64_t)(q - 1) * nb + j] = pos - ce.x;
          }
        }
    }
  }
  if (c_dbg & 16) {
    __syncthreads();
    phase_mark(tmark, 12);
  }
}

// a panel group (column, panels r0..r1) counted as ONE hash slab over its
// rows when its products fit the LDS hash and its nonzeros one hash slab;
// false: nothing was written and the caller runs the panels one by one
template <class H>
__device__ __forceinline__ bool sym_group(const SymPanelArgs& a, const SymPanelLds& L, int b, int col, int r0,
                                          int r1, const SymPre& pre, H& hook) {
  constexpr int BS = BIG_BS;
  const int tid = threadIdx.x;
  const int64_t p0 = pre.ok ? pre.p0 : a.cpB[col], p1 = pre.ok ? pre.p1 : a.cpB[col + 1];
  if (p1 - p0 > BS) return false;
  const int64_t p = p0 + tid;
  int s = 0, len = 0;
  if (pre.ok == 2) {
    s = pre.s;
    len = pre.len;
  } else if (p < p1) {
    const int k = a.irB[p];
    s = a.pm.at(r0, k).x;
    len = a.pm.at(r1, k).y - s;
  }
  int total;
  const int ex = block_excl_scan<BS>(len, L.tmp, &total);
  L.pref[tid] = ex;
  if (tid == BS - 1) L.pref[BS] = total;
  L.st[tid] = seg_stage(s, ex);
  hook(1);
  int T = 512;
  while (T * CBG_SYM_LOAD_DEN < CBG_SYM_LOAD_NUM * total) T <<= 1;
  if (T > a.hwords) {
    if ((c_dbg & 32) && tid == 0) {
      atomicAdd(&g_stat[14], 1ull);
      atomicAdd(&g_stat[15], (unsigned long long)total);
    }
    __syncthreads();
    return false;
  }
  if ((c_dbg & 256) && total <= SPARSE_NNZ_MAX) {
    __syncthreads();
    if (tid <= r1 - r0) {
      const int64_t br = (int64_t)b * a.R + r0 + tid;
      a.nslab[br] = 0;
      a.cnt_br[br] = 0;
      if (a.gbm_slot) a.gbm_slot[br] = -1;
    }
    return true;
  }
  int* keys = reinterpret_cast<int*>(L.bm);
  int* ocount = L.tmp + BS / WAVE + 3;
  for (int j = tid; j < T / 4; j += BS)
    reinterpret_cast<int4*>(keys)[j] = make_int4(EMPTY_KEY, EMPTY_KEY, EMPTY_KEY, EMPTY_KEY);
  if (tid == 0) {
    L.fine[0] = 0;
    *ocount = 0;
  }
  __syncthreads();
  int count = 0;
  const int32_t* __restrict__ irA = a.irA;
  const int* pref = L.pref;
  const int* st = L.st;
  const unsigned mask = (unsigned)(T - 1);
  if (!(c_dbg & 64))
  block_products<BS>(
      pref, total, [&](int sg) { return SegI{seg_off(st, pref, sg)}; },
      [&](const SegI& g, int u) { return irA[g.off + u]; },
      [&](int row) {
        const unsigned h = ((unsigned)row * 0x9E3779B1u) & mask;
        if (CBG_SYM_OVF > 0)
          count += hash_claim_bounded<CBG_SYM_OVF>(keys, h, mask, row, ocount, L.ovf, SYM_OVF_CAP);
        else
          count += hash_claim(keys, h, mask, row);
      });
  hook(2);
  if (CBG_SYM_OVF > 0) {
    __syncthreads();
    const int no = *ocount;
    if (no > 0) count += hash_claim_drain<CBG_SYM_OVF>(keys, mask, L.ovf, min(no, SYM_OVF_CAP));
  }
  count = wave_sum(count);
  if (lane_id() == 0 && count) atomicAdd(&L.fine[0], count);
  __syncthreads();
  const int cg = L.fine[0];
  __syncthreads();
  if ((c_dbg & 32) && tid == 0) {
    const bool ok = cg <= SPARSE_NNZ_MAX;
    atomicAdd(&g_stat[ok ? 12 : 14], 1ull);
    atomicAdd(&g_stat[ok ? 13 : 15], (unsigned long long)total);
  }
  if (cg > SPARSE_NNZ_MAX) return false;
  if (tid <= r1 - r0) {
    const int64_t br = (int64_t)b * a.R + r0 + tid;
    const bool first = tid == 0;
    a.nslab[br] = (first && cg) ? 1 : 0;
    a.cnt_br[br] = first ? cg : 0;
    if (a.gbm_slot) a.gbm_slot[br] = -1;
    if (first && cg)
      a.desc[br * NFINE_MAX] =
          make_int4(r0 << a.plog, (int)min((int64_t)(r1 + 1) << a.plog, a.m), 0,
                    cg | SLAB_SPARSE | (total > GRANK_PMAX ? SLAB_MANYP : 0));
  }
  if (tid == 0 && cg) atomicAdd(&a.cnt[col], cg);
  return true;
}

// grid: RG groups x (columns of the class) in XCD column order (k_sym_panel)
#ifndef CBG_SYM_WPE  // waves per SIMD k_sym_panel is compiled for (0: the compiler's choice)
// 8: at most 64 VGPRs, so 4 blocks of 512 threads per CU (the LDS allows 4; at
// 65 VGPRs only 3 fit): +4.2 % at scale 22 (profiles/r04_ab_hash_sym.json)
#define CBG_SYM_WPE 8
#endif
#if CBG_SYM_WPE > 0
#define CBG_SYM_WPE_ATTR __attribute__((amdgpu_waves_per_eu(CBG_SYM_WPE)))
#else
#define CBG_SYM_WPE_ATTR
#endif
__device__ __forceinline__ SymPanelLds sym_lds(char* smem, int hwords) {
  SymPanelLds L;
  L.bm = reinterpret_cast<unsigned*>(smem);
  L.fine = reinterpret_cast<int*>(L.bm + hwords);
  L.pref = L.fine + NFINE_MAX;
  L.st = L.pref + BIG_BS + 4;
  L.tmp = L.st + BIG_BS;
  L.ovf = L.tmp + BIG_BS / WAVE + 4;
  return L;
}
// GROUPS: the launch's units span several panels (sym_group); false for the
// single-panel class, whose kernel then carries no group code (fewer spills)
template <bool GROUPS>
__global__ __launch_bounds__(BIG_BS) CBG_SYM_WPE_ATTR void k_sym_panel(SymPanelArgs a) {
  // Persistent blocks stride over the units (group-major order kept); the
  // next unit's dependent loads -- column id, B column range, B rows, A run
  // bounds -- are issued one per stage of the current unit (hook 1 after its
  // staging, 2 after its products, 3 at its end) instead of back to back at
  // the start of every block.
  constexpr int BS = BIG_BS;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const SymPanelLds L = sym_lds(smem, a.hwords);
  const int tid = threadIdx.x;
  const int g = 1 << a.glog;
  const int RG = (a.R + g - 1) >> a.glog;
  const int ncls = a.ncls;
  // next unit's fetch state
  int n_b = 0, n_r0 = 0, n_r1 = 0, n_col = 0, n_k = -1, stage = -1;
  int64_t n_p0 = 0, n_p1 = 0;
  // XCD column order: unit u goes to the blocks b = u (mod 8), which MI355X
  // places on one XCD (blocks are dealt round-robin over the 8 XCDs, and the
  // grid is a multiple of 8); they take the columns x, x + 8, ... of the class,
  // each column's RG units one after the other, so the blocks in flight on an
  // XCD are a few columns' panels, which read the same B entries, the same
  // column-major map lines and -- A's short columns -- the same lines of A:
  // L2 hits 27.6 -> 44.5 % (single panels) and 13.9 -> 40.1 % (groups), the
  // kernel 87 -> 72.7 ms per scale-22 step (profiles/r06_l2_s22_*.txt).  The
  // panel-major order before kept every block on one panel, reusing the hub
  // columns' runs in the Infinity Cache instead; bands of 8 / 4 / 2 panels
  // (column order inside a band) were 0.3 / 0.6 / 1.7 % slower than the whole
  // column (profiles/r06_ab_sym_bands.json).
  // false: no unit left for this block
  auto start = [&](int unit) {
    stage = -1;
    const int x = unit & 7, s = unit >> 3, cq = s / RG;
    const int ci = x + 8 * cq, rg = s - cq * RG;
    if (ci >= ncls) return false;
    n_b = a.boff + ci;
    n_r0 = rg << a.glog;
    n_r1 = min(n_r0 + g, a.R) - 1;
    n_col = a.perm_big[n_b];
    stage = 0;
    return true;
  };
  SymPre nxt;
  auto hook = [&](int k) {
    if (stage < 0) return;
    if (k >= 1 && stage < 1) {
      n_p0 = a.cpB[n_col];
      n_p1 = a.cpB[n_col + 1];
      stage = 1;
    }
    if (k >= 2 && stage < 2) {
      n_k = (n_p1 - n_p0 <= BS && tid < n_p1 - n_p0) ? a.irB[n_p0 + tid] : -1;
      stage = 2;
    }
    if (k >= 3 && stage < 3) {
      nxt.p0 = n_p0;
      nxt.p1 = n_p1;
      nxt.s = nxt.len = 0;
      nxt.ok = n_p1 - n_p0 <= BS ? 2 : 1;
      if (n_k >= 0) {
        const int2 e0 = a.pm.at(n_r0, n_k);
        const int e1y = n_r1 > n_r0 ? a.pm.at(n_r1, n_k).y : e0.y;
        nxt.s = e0.x;
        nxt.len = e1y - e0.x;
      }
      stage = 3;
    }
  };
  int unit = blockIdx.x;
  bool valid = start(unit);
  hook(3);
  while (valid) {
    const SymPre cur = nxt;
    const int b = n_b, col = n_col, r0 = n_r0, r1 = n_r1;
    const int next = unit + (int)gridDim.x;
    const bool nvalid = start(next);
    if constexpr (GROUPS) {
      // (the panel-by-panel fallback lives in k_sym_deferred, so this kernel
      // carries only the group hash: no VGPR spills at its 64-VGPR cap)
      const bool done = r1 > r0 && sym_group(a, L, b, col, r0, r1, cur, hook);
      if (!done && tid == 0) a.defer[atomicAdd(a.defer_n, 1)] = make_int4(b, col, r0, r1);
    } else {
      sym_pair(a, L, b, col, r0, cur, hook);  // (single-panel units: r1 == r0)
    }
    hook(3);
    __syncthreads();  // LDS is reused by the next unit
    unit = next;
    valid = nvalid;
  }
}

// the deferred group units, panel by panel (their pairs as in k_sym_panel<false>)
__global__ __launch_bounds__(BIG_BS) CBG_SYM_WPE_ATTR void k_sym_deferred(SymPanelArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const SymPanelLds L = sym_lds(smem, a.hwords);
  const int n = *a.defer_n;
  auto hook = [](int) {};
  for (int e = blockIdx.x; e < n; e += gridDim.x) {
    const int4 d = a.defer[e];
    const SymPre pp;  // (ok = 0: the pair loads its column range itself)
    for (int r = d.z; r <= d.w; ++r) {
      sym_pair(a, L, d.x, d.y, r, pp, hook);
      __syncthreads();  // LDS is reused by the next panel
    }
  }
}

// one numeric work item: everything a slab block needs in one 48-byte load
struct __attribute__((aligned(16))) SlabRec {
  int64_t obase;  // first output position in C
  int64_t p0;     // B column range [p0, p0 + nb)
  int nb;
  int r;          // panel
  int lo, hi;     // row range
  int nout;       // nnz of the slab
  int slot;       // kept symbolic bitmap (-1: none)
  // bit 0: first slab of its (column, panel) pair, bit 1: last, bit 2 (SLAB_FULL):
  // A's whole panel runs are the slab's products (the slab is its panel, or its
  // pair's only slab); bits 3+: the slab's index in its pair
  int flags;
  int coff;       // the pair's precomputed cut offsets in `cuts` (-1: search them)
};
constexpr int SLAB_FULL = 4;

#ifndef CBG_HASH_LOAD_NUM  // numeric hash slab tables: T >= (NUM/DEN) * nnz
#define CBG_HASH_LOAD_NUM 3  // 3/2: +4.6 % at scale 22 over 2/1 (more hash slabs in the smaller, higher-occupancy classes)
#define CBG_HASH_LOAD_DEN 2
#endif
// slab work lists per launch class.  Classes: 0 bitmap small (nnz <=
// small_cap), 1 bitmap large, 2+k hash slab with table HASH_T[k] slots: powers
// of two and 1.5x powers of two, so that the LDS a slab reserves (12 B per
// slot) tracks its nnz and more slabs fit a CU
constexpr int SLAB_HASH_NCLS = 9;
#define CBG_HASH_TABLES 512, 768, 1024, 1536, 2048, 3072, 4096, 6144, 8192
__constant__ int c_hash_t[SLAB_HASH_NCLS] = {CBG_HASH_TABLES};
// + rank slabs (k_num_slab_rank) of <= 1024 / 2048 / 4096 nonzeros: the
// hash-mode slabs of more than rank_min nonzeros spanning <= rank_span rows
// (one panel; rank_span 0: none)
constexpr int SLAB_RANK_NCLS = 3;
static_assert(CBG_WORK_RANK0 - CBG_WORK_HASH0 == SLAB_HASH_NCLS && CBG_WORK_SYM_PANEL_UNITS - CBG_WORK_RANK0 == SLAB_RANK_NCLS,
              "cbg_last_work_stats classes");
constexpr int SLAB_RANK0 = 2 + SLAB_HASH_NCLS;
// + group rank slabs (k_num_slab_grank) of <= 2048 / 4096 nonzeros: the
// panel-group slabs of more than grank_min nonzeros spanning <= 2^22 rows
constexpr int SLAB_GRANK_NCLS = 2;
constexpr int SLAB_GRANK0 = SLAB_RANK0 + SLAB_RANK_NCLS;
static_assert(CBG_WORK_GRANK0 == CBG_WORK_IACC + 1 && CBG_WORK_N == CBG_WORK_GRANK0 + SLAB_GRANK_NCLS,
              "cbg_last_work_stats group rank classes");
constexpr int SLAB_NCLS = 2 + SLAB_HASH_NCLS + SLAB_RANK_NCLS + SLAB_GRANK_NCLS;
__device__ __forceinline__ int slab_class(const int4& d, int small_cap, int rank_span, int rank_min, int grank_min) {
  const int w = d.w;
  if (w & SLAB_SPARSE) {
    const int c = w & SLAB_CNT_MASK;
    if (c > rank_min && rank_span > 0 && d.y - d.x <= rank_span)
      return SLAB_RANK0 + (c <= 1024 ? 0 : c <= 2048 ? 1 : 2);
    if (c > grank_min && !(w & SLAB_MANYP) && d.y - d.x > rank_span && d.y - d.x <= (1 << GRANK_SPAN_LOG))
      return SLAB_GRANK0 + (c <= 2048 ? 0 : 1);
    int k = 0;
    while (k + 1 < SLAB_HASH_NCLS && c_hash_t[k] * CBG_HASH_LOAD_DEN < CBG_HASH_LOAD_NUM * c) ++k;  // load <= NUM/DEN
    return 2 + k;
  }
  return w <= small_cap ? 0 : 1;
}
// The slab list is ordered by (class, panel): a class is one launch, and
// inside it the slabs of panel r run together, so the A rows they gather
// (A's panel-r segments, ~1/R of A) stay in L2 / Infinity Cache.  key = c *
// KR + r with KR = R (KR = 1, class order only, if the keys overflow LDS).
constexpr int SLAB_KEYS_MAX = 8192;
__host__ __device__ inline int slab_kr(int R) { return SLAB_NCLS * R <= SLAB_KEYS_MAX ? R : 1; }

// pass 1: within-panel -> within-column offsets, (class, panel) counts
__global__ void k_slab_count(int nbig, int R, const int32_t* __restrict__ nslab, const int32_t* __restrict__ cnt_br,
                             int4* __restrict__ desc, int small_cap, int rank_span, int rank_min,
                             int grank_min, int* __restrict__ counts) {
  extern __shared__ int lc[];  // [SLAB_NCLS * KR]
  const int KR = slab_kr(R), NK = SLAB_NCLS * KR;
  for (int k = threadIdx.x; k < NK; k += blockDim.x) lc[k] = 0;
  __syncthreads();
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < nbig) {
    int off = 0;
    for (int r = 0; r < R; ++r) {
      const int br = b * R + r;
      for (int s = 0; s < nslab[br]; ++s) {
        int4& d = desc[(int64_t)br * NFINE_MAX + s];
        d.z += off;
        atomicAdd(&lc[slab_class(d, small_cap, rank_span, rank_min, grank_min) * KR + (KR > 1 ? r : 0)], 1);
      }
      off += cnt_br[br];
    }
  }
  __syncthreads();
  for (int k = threadIdx.x; k < NK; k += blockDim.x)
    if (lc[k]) atomicAdd(&counts[k], lc[k]);
}
// key bases (exclusive prefix of the counts) into cursor[], class totals into cls[]
__global__ void k_slab_bases(int R, const int* __restrict__ counts, int* __restrict__ cursor, int* __restrict__ cls) {
  if (threadIdx.x == 0) {
    const int KR = slab_kr(R);
    int s = 0;
    for (int c = 0; c < SLAB_NCLS; ++c) {
      int t = 0;
      for (int r = 0; r < KR; ++r) {
        cursor[c * KR + r] = s;
        s += counts[c * KR + r];
        t += counts[c * KR + r];
      }
      cls[c] = t;
    }
  }
}
// pass 2: slab records into their (class, panel) segment of one list
__global__ void k_slab_fill(int nbig, int R, const int32_t* __restrict__ nslab, const int4* __restrict__ desc,
                            int small_cap, int rank_span, int rank_min, int grank_min, int* __restrict__ cursor,
                            SlabRec* __restrict__ list,
                            const int32_t* __restrict__ perm_big, const int64_t* __restrict__ cpB,
                            const int64_t* __restrict__ colptr, const int* __restrict__ gbm_slot, int plog,
                            int64_t m_rows, const int* __restrict__ pcoff) {
  extern __shared__ int lsh[];  // lc[NK] | lb[NK]
  const int KR = slab_kr(R), NK = SLAB_NCLS * KR;
  int* lc = lsh;
  int* lb = lsh + NK;
  for (int k = threadIdx.x; k < NK; k += blockDim.x) lc[k] = 0;
  __syncthreads();
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < nbig)
    for (int r = 0; r < R; ++r) {
      const int br = b * R + r;
      for (int s = 0; s < nslab[br]; ++s)
        atomicAdd(&lc[slab_class(desc[(int64_t)br * NFINE_MAX + s], small_cap, rank_span, rank_min, grank_min) * KR +
                      (KR > 1 ? r : 0)],
                  1);
    }
  __syncthreads();
  for (int k = threadIdx.x; k < NK; k += blockDim.x) {
    lb[k] = lc[k] ? atomicAdd(&cursor[k], lc[k]) : 0;
    lc[k] = 0;
  }
  __syncthreads();
  if (b >= nbig) return;
  const int col = perm_big[b];
  const int64_t p0 = cpB[col], nb = cpB[col + 1] - p0, cbase = colptr[col];
  for (int r = 0; r < R; ++r) {
    const int br = b * R + r;
    const int R0 = r << plog;
    const int R1 = (int)min((int64_t)R0 + (1LL << plog), m_rows);
    for (int s = 0; s < nslab[br]; ++s) {
      const int4 d = desc[(int64_t)br * NFINE_MAX + s];
      const int key = slab_class(d, small_cap, rank_span, rank_min, grank_min) * KR + (KR > 1 ? r : 0);
      SlabRec rec;
      rec.obase = cbase + d.z;
      rec.p0 = p0;
      rec.nb = (int)nb;
      rec.r = r;
      rec.lo = d.x;
      rec.hi = d.y;
      rec.nout = (d.w & SLAB_SPARSE) ? (d.w & SLAB_CNT_MASK) : d.w;
      rec.slot = gbm_slot ? gbm_slot[br] : -1;
      // a pair's only slab holds every row its products reach (the plan trims
      // empty fine ranges only), so A's whole panel runs are its products
      const bool full = (d.x == R0 && d.y == R1) || nslab[br] == 1;
      rec.flags = (s == 0 ? 1 : 0) | (s == nslab[br] - 1 ? 2 : 0) | (full ? SLAB_FULL : 0) | (s << 3);
      rec.coff = pcoff ? pcoff[br] : -1;
      list[lb[key] + atomicAdd(&lc[key], 1)] = rec;
    }
  }
}

// ----------------------------------------------------------------------------
// numeric: wave per column (n <= 256), LDS hash + wave bitonic sort
// ----------------------------------------------------------------------------
template <int LOGT>
struct NumWaveLds {
  static constexpr int T = 1 << LOGT;
  // vals[T] f64 | bv[64] f64 | keys[T] | pref[68] | st[64]
  static constexpr int BYTES = T * 8 + WAVE * 8 + T * 4 + (WAVE + 4) * 4 + WAVE * 4;
};

template <int LOGT, int SR>
__global__ __launch_bounds__(256) void k_num_wave(const int32_t* __restrict__ perm, int n,
                                                  const int64_t* __restrict__ cpB, const int32_t* __restrict__ irB,
                                                  const double* __restrict__ valB, const int2* __restrict__ cmap,
                                                  const int32_t* __restrict__ irA, const double* __restrict__ valA,
                                                  const int64_t* __restrict__ colptr, int32_t* __restrict__ out_ir,
                                                  double* __restrict__ out_val) {
  constexpr int T = 1 << LOGT;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int w = threadIdx.x / WAVE, lane = lane_id();
  char* base = smem + w * NumWaveLds<LOGT>::BYTES;
  double* vals = reinterpret_cast<double*>(base);
  double* bv = vals + T;
  int* keys = reinterpret_cast<int*>(bv + WAVE);
  int* pref = keys + T;
  int* st = pref + WAVE + 4;
  const int idx = blockIdx.x * (blockDim.x / WAVE) + w;
  if (idx >= n) return;
  const int col = perm[idx];
  for (int j = lane; j < T; j += WAVE) {
    keys[j] = EMPTY_KEY;
    vals[j] = Sem<SR>::identity();
  }
  const int64_t p1 = cpB[col + 1];
  for (int64_t c0 = cpB[col]; c0 < p1; c0 += WAVE) {
    const int64_t p = c0 + lane;
    int s = 0, len = 0;
    double bval = 0.0;
    if (p < p1) {
      int2 e = cmap[irB[p]];
      s = e.x;
      len = e.y;
      bval = valB[p];
    }
    const int incl = wave_incl_scan(len);
    const int total = wave_last(incl);
    pref[lane + 1] = incl;
    if (lane == 0) pref[0] = 0;
    st[lane] = seg_stage(s, incl - len);
    bv[lane] = bval;
    wave_sync();
    wave_products(
        pref, WAVE, 0, total, [&](int sg) { return SegV{seg_off(st, pref, sg), bv[sg]}; },
        [&](const SegV& g, int u) { return RowVal{irA[g.off + u], Sem<SR>::mul(valA[g.off + u], g.b)}; },
        [&](const RowVal& x) { hash_acc<SR, LOGT>(keys, vals, x.row, x.v); });
    wave_sync();
  }
  const int64_t o = colptr[col];
  const int nout = (int)(colptr[col + 1] - o);
  if constexpr (T == WAVE) {  // one slot per lane: sort in registers (-28 % kernel time)
    int key = keys[lane];
    double val = vals[lane];
    wave_bitonic_sort_kv(key, val, lane);
    if (lane < nout) {
      st_stream(&out_ir[o + lane], key);
      st_stream(&out_val[o + lane], val);
    }
    return;
  }
  bitonic_sort_kv<T, WAVE>(keys, vals, lane, WaveSync());
  for (int e = lane; e < nout; e += WAVE) {
    st_stream(&out_ir[o + e], keys[e]);
    st_stream(&out_val[o + e], vals[e]);
  }
}

// Small columns by expand-sort-compress in registers (flops <= fmax = 64 *
// NPL / CPW per column): a wave takes CPW consecutive columns of its bin,
// expands their <= 64 * NPL products (NPL per lane, product q in register q /
// 64 of lane q % 64), sorts the (column, row) keys with their values across
// the wave (bitonic), combines equal keys (segmented scan) and writes each
// column's sorted entries to its temporary slot idx * fmax, and cnt[col] =
// its nnz.  No LDS hash and no wave per column: GalerkinNew's columns carry 7
// products on average, so a wave per column left 7/8 of its lanes idle through
// every load of the column's chain.  key = c << SH | row needs A.m < 2^SH (the
// host launches CPW = 1 when it is not).
template <int NPL>
__device__ __forceinline__ void wave_bitonic_sort_kvn(int (&key)[NPL], double (&val)[NPL], int lane) {
  // element i = j * 64 + lane
#pragma unroll
  for (int k = 2; k <= WAVE * NPL; k <<= 1) {
#pragma unroll
    for (int d = k >> 1; d > 0; d >>= 1) {
      if (d >= WAVE) {
        const int dj = d / WAVE;
#pragma unroll
        for (int j = 0; j < NPL; ++j) {
          if (j & dj) continue;
          const int i = j * WAVE + lane;
          const bool up = (i & k) == 0;
          const int j2 = j | dj;
          if (up ? key[j2] < key[j] : key[j2] > key[j]) {
            const int tk = key[j];
            key[j] = key[j2];
            key[j2] = tk;
            const double tv = val[j];
            val[j] = val[j2];
            val[j2] = tv;
          }
        }
      } else {
#pragma unroll
        for (int j = 0; j < NPL; ++j) {
          const int i = j * WAVE + lane;
          const int ok = xor_lane_d(key[j], d);
          const double ov = xor_lane_d(val[j], d);
          const bool up = (i & k) == 0;
          const bool lower = (lane & d) == 0;
          if (lower == up ? ok < key[j] : ok > key[j]) {
            key[j] = ok;
            val[j] = ov;
          }
        }
      }
    }
  }
}

// One step of a DPP segmented scan: lanes whose source lane (CTRL, rows ROWM)
// holds the same key add its partial; invalid sources read EMPTY_KEY.
template <int SR, int CTRL, int ROWM>
__device__ __forceinline__ void seg_scan_step(int key, double& val) {
  const int ok = __builtin_amdgcn_update_dpp(EMPTY_KEY, key, CTRL, ROWM, 0xf, false);
  const long long b = __double_as_longlong(val);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, ROWM, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, ROWM, 0xf, false);
  if (ok == key) val = Sem<SR>::add(__longlong_as_double(((long long)hi << 32) | (unsigned)lo), val);
}
// Inclusive segmented scan (the semiring's add) over runs of equal keys of a
// wave whose keys are sorted ascending: Hillis-Steele with row_shr 1/2/4/8
// inside rows of 16, then row_bcast 15/31 carry runs across rows (sorted keys:
// equal keys at a distance are equal in between, so the carried partial
// covers exactly the run's lanes below).  Six VALU steps instead of six
// __shfl_up pairs (ds_bpermute).
template <int SR>
__device__ __forceinline__ double wave_seg_scan_sorted(int key, double val) {
#if CBG_XOR_DPP
  seg_scan_step<SR, 0x111, 0xf>(key, val);
  seg_scan_step<SR, 0x112, 0xf>(key, val);
  seg_scan_step<SR, 0x114, 0xf>(key, val);
  seg_scan_step<SR, 0x118, 0xf>(key, val);
  seg_scan_step<SR, 0x142, 0xa>(key, val);  // row_bcast:15 -> rows 1, 3
  seg_scan_step<SR, 0x143, 0xc>(key, val);  // row_bcast:31 -> rows 2, 3
#else
  const int lane = lane_id();
#pragma unroll
  for (int d = 1; d < WAVE; d <<= 1) {
    const int ok = __shfl_up(key, d);
    const double ov = __shfl_up(val, d);
    if (lane >= d && ok == key) val = Sem<SR>::add(ov, val);
  }
#endif
  return val;
}
__device__ __forceinline__ double readlane_f64(double v, int l) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// INL: A's columns as inline records (k_inline_cols); a product of an A column
// of one or two entries takes its row and value from the B entry's lane
// (shuffles) instead of two random gathers -- GalerkinNew's S = T^T, Poisson(1)
// entries per column
template <int CPW, int NPL, int SR, bool INL>
__global__ __launch_bounds__(256) void k_esc_wave(const int32_t* __restrict__ perm, int n, int fmax,
                                                  const int64_t* __restrict__ cpB, const int32_t* __restrict__ irB,
                                                  const double* __restrict__ valB, const int2* __restrict__ cmap,
                                                  const int4* __restrict__ ainl,
                                                  const int32_t* __restrict__ irA, const double* __restrict__ valA,
                                                  int32_t* __restrict__ cnt, int32_t* __restrict__ tir,
                                                  double* __restrict__ tval, int64_t slot_base,
                                                  int64_t* __restrict__ tslot) {
  constexpr int LOGC = CPW <= 1 ? 0 : CPW <= 2 ? 1 : CPW <= 4 ? 2 : CPW <= 8 ? 3 : CPW <= 16 ? 4 : 5;
  static_assert((1 << LOGC) == CPW && CPW <= 32, "columns per wave");
  static_assert(NPL == 1 || NPL == 2 || NPL == 4 || NPL == 8, "products per lane");
  constexpr int SH = 31 - LOGC;
  const int lane = lane_id();
  const int64_t idx0 = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / WAVE * CPW;
  if (idx0 >= n) return;
  int col = -1;
  int64_t p0 = 0, p1 = 0;
  if (lane < CPW && idx0 + lane < n) {
    col = perm[idx0 + lane];
    p0 = cpB[col];
    p1 = cpB[col + 1];
  }
  const int nb = (int)(p1 - p0);
  const int binc = wave_incl_scan(nb);  // B entries of columns 0..lane
  const int bexc = binc - nb;
  const int totalB = wave_last(binc);
  int key[NPL];
  double val[NPL];
#pragma unroll
  for (int j = 0; j < NPL; ++j) {
    key[j] = EMPTY_KEY;
    val[j] = 0.0;
  }
  int pbase = 0;  // products placed so far (element index)
  for (int e0 = 0; e0 < totalB; e0 += WAVE) {
    const int e = e0 + lane;
    int c = 0;  // column of B entry e
#pragma unroll
    for (int cc = 1; cc < CPW; ++cc) c += __builtin_amdgcn_readlane(bexc, cc) <= e ? 1 : 0;
    const int ex_c = __shfl(bexc, c);
    const int64_t p0_c = __shfl(p0, c);
    int s = 0, len = 0, r1 = 0;
    double bv = 0.0, v0 = 0.0, v1 = 0.0;
    if (e < totalB) {
      const int64_t p = p0_c + (e - ex_c);
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
    }
    const int pincl = wave_incl_scan(len);
    const int ptot = wave_last(pincl);
    if (ptot == 0) continue;
#pragma unroll
    for (int j = 0; j < NPL; ++j) {
      if (pbase + ptot <= j * WAVE || pbase >= (j + 1) * WAVE) continue;  // uniform
      // element j * 64 + lane takes product q of this round: its entry is the
      // first lane whose inclusive product count exceeds q
      const int q = j * WAVE + lane - pbase;
      int lo = 0, hi = WAVE - 1;
#pragma unroll
      for (int it = 0; it < 6; ++it) {
        const int mid = (lo + hi) >> 1;
        const int v = __shfl(pincl, mid);
        if (v > q) hi = mid; else lo = mid + 1;
      }
      const int o = lo;
      const int o_s = __shfl(s, o), o_ex = __shfl(pincl - len, o), o_c = __shfl(c, o);
      const double o_bv = __shfl(bv, o);
      bool inl = false, second = false;
      int o_r1 = 0;
      double o_v0 = 0.0, o_v1 = 0.0;
      if constexpr (INL) {
        inl = __shfl(len, o) <= 2;
        second = q - o_ex == 1;
        o_r1 = __shfl(r1, o);
        o_v0 = __shfl(v0, o);
        o_v1 = __shfl(v1, o);
      }
      if (q >= 0 && q < ptot) {
        if (INL && inl) {
          key[j] = (o_c << SH) | (second ? o_r1 : o_s);
          val[j] = Sem<SR>::mul(second ? o_v1 : o_v0, o_bv);
        } else {
          const int a = o_s + (q - o_ex);
          key[j] = (o_c << SH) | irA[a];
          val[j] = Sem<SR>::mul(valA[a], o_bv);
        }
      }
    }
    pbase += ptot;
  }
  if constexpr (NPL == 1) {
    wave_bitonic_sort_kv(key[0], val[0], lane);
  } else {
    wave_bitonic_sort_kvn<NPL>(key, val, lane);
  }
  // combine equal keys: segmented inclusive scan per register (keys are sorted,
  // so a lane d below with the same key means every lane in between has it
  // too), then the run that continues from the previous register's top lane
#pragma unroll
  for (int j = 0; j < NPL; ++j) {
    val[j] = wave_seg_scan_sorted<SR>(key[j], val[j]);
    if (j > 0) {
      const int pk = __builtin_amdgcn_readlane(key[j - 1], WAVE - 1);
      const double pv = readlane_f64(val[j - 1], WAVE - 1);
      if (key[j] == pk) val[j] = Sem<SR>::add(pv, val[j]);
    }
  }
  const unsigned long long lt = (1ull << lane) - 1ull;
  int pos[NPL], mycount = 0;
  bool tail[NPL];
  int cj[NPL];
#pragma unroll
  for (int j = 0; j < NPL; ++j) {
#if CBG_XOR_DPP
    int nk = __builtin_amdgcn_update_dpp(EMPTY_KEY, key[j], 0x130, 0xf, 0xf, false);  // wave_shl:1
#else
    int nk = __shfl_down(key[j], 1);
#endif
    if (j + 1 < NPL) {
      const int f = __builtin_amdgcn_readlane(key[j + 1 < NPL ? j + 1 : j], 0);
      if (lane == WAVE - 1) nk = f;
    }
    tail[j] = key[j] != EMPTY_KEY && ((lane == WAVE - 1 && j == NPL - 1) || nk != key[j]);
    cj[j] = key[j] != EMPTY_KEY ? key[j] >> SH : 0;
    pos[j] = 0;
  }
#pragma unroll
  for (int cc = 0; cc < CPW; ++cc) {
    int before = 0;  // tails of column cc in the registers below
#pragma unroll
    for (int j = 0; j < NPL; ++j) {
      const unsigned long long m = __ballot(tail[j] && cj[j] == cc);
      if (cj[j] == cc) pos[j] = before + __popcll(m & lt);
      before += __popcll(m);
    }
    if (lane == cc) mycount = before;
  }
#pragma unroll
  for (int j = 0; j < NPL; ++j) {
    if (tail[j]) {
      const int64_t o = (idx0 + cj[j]) * (int64_t)fmax + pos[j];
      tir[o] = key[j] & (int)((1u << SH) - 1u);
      tval[o] = val[j];
    }
  }
  if (col >= 0) {
    cnt[col] = mycount;
    tslot[col] = slot_base + (idx0 + lane) * (int64_t)fmax;
  }
}

// the fused columns' temporary slots -> C, in COLUMN order: a wave takes 64
// consecutive columns, flattens the entries of its fused ones (tslot[col] in
// [0, thin_base); -1: not fused, >= thin_base: a thin column, thin_copy) and
// copies them one per lane, so the stores run along C (a few threads per
// column, in bin order or column order, left C's lines written in pieces and
// walked each column serially: 0.4 ms per GalerkinNew product)
__global__ __launch_bounds__(256) void k_copy_fused(int64_t nz, const int64_t* __restrict__ tslot,
                                                    const int32_t* __restrict__ cnt,
                                                    const int64_t* __restrict__ colptr,
                                                    const int32_t* __restrict__ tir, const double* __restrict__ tval,
                                                    int32_t* __restrict__ out_ir, double* __restrict__ out_val,
                                                    int64_t thin_base) {
  const int64_t c0 = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / WAVE * WAVE;
  if (c0 >= nz) return;
  const int lane = lane_id();
  const int64_t col = c0 + lane;
  int64_t src = -1, dst = 0;
  int c = 0;
  if (col < nz) {
    src = tslot[col];
    if (src >= 0 && src < thin_base) {
      c = cnt[col];
      dst = colptr[col];
    }
  }
  const int incl = wave_incl_scan(c);
  const int total = wave_last(incl);
  for (int q0 = 0; q0 < total; q0 += WAVE) {
    const int q = q0 + lane;
    int lo = 0, hi = WAVE - 1;  // the column of flattened entry q
#pragma unroll
    for (int it = 0; it < 6; ++it) {
      const int mid = (lo + hi) >> 1;
      if (__shfl(incl, mid) > q) hi = mid; else lo = mid + 1;
    }
    const int64_t o_src = __shfl(src, lo), o_dst = __shfl(dst, lo);
    const int o_ex = __shfl(incl - c, lo);
    if (q < total) {
      const int e = q - o_ex;
      out_ir[o_dst + e] = tir[o_src + e];
      out_val[o_dst + e] = tval[o_src + e];
    }
  }
}

// single-entry columns of <= big flops (k_classify copy1): C(:,j) = A(:,k) * b, flattened per
// wave along C like k_copy_fused (rows are A's, already ascending)
template <int SR>
__global__ __launch_bounds__(256) void k_copy_single(int64_t nz, const int64_t* __restrict__ cpB,
                                                     const int32_t* __restrict__ irB, const double* __restrict__ valB,
                                                     const int2* __restrict__ cmap, const int64_t* __restrict__ flops,
                                                     int64_t big, const int32_t* __restrict__ irA,
                                                     const double* __restrict__ valA, const int64_t* __restrict__ colptr,
                                                     int32_t* __restrict__ out_ir, double* __restrict__ out_val) {
  const int64_t c0 = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / WAVE * WAVE;
  if (c0 >= nz) return;
  const int lane = lane_id();
  const int64_t col = c0 + lane;
  int64_t dst = 0;
  int src = 0, c = 0;
  double b = 0.0;
  if (col < nz) {
    const int64_t p = cpB[col], f = flops[col];
    if (cpB[col + 1] - p == 1 && f > 0 && f <= big) {
      const int2 m = cmap[irB[p]];
      src = m.x;
      c = m.y;
      b = valB[p];
      dst = colptr[col];
    }
  }
  const int incl = wave_incl_scan(c);
  const int total = wave_last(incl);
  for (int q0 = 0; q0 < total; q0 += WAVE) {
    const int q = q0 + lane;
    int lo = 0, hi = WAVE - 1;  // the column of flattened entry q
#pragma unroll
    for (int it = 0; it < 6; ++it) {
      const int mid = (lo + hi) >> 1;
      if (__shfl(incl, mid) > q) hi = mid; else lo = mid + 1;
    }
    const int o_src = __shfl(src, lo), o_ex = __shfl(incl - c, lo);
    const int64_t o_dst = __shfl(dst, lo);
    const double o_b = __shfl(b, lo);
    if (q < total) {
      const int e = q - o_ex;
      out_ir[o_dst + e] = irA[o_src + e];
      out_val[o_dst + e] = Sem<SR>::mul(valA[o_src + e], o_b);
    }
  }
}

// the single-entry columns of more than `big` flops (copy1 = 2): their sizes
// (flops = the A column's length) for an exclusive scan, so that the copy can be
// split into equal chunks.  A block per column (round 4) left a hub column of
// ~10^5 entries to 256 threads: at scale 24 that kernel ran 80 ms per phase
// for a few blocks (the side stream), beside k_num_slab.
__global__ void k_single_big_sizes(int64_t nz, const int64_t* __restrict__ cpB, const int64_t* __restrict__ flops,
                                   int64_t big, int64_t* __restrict__ sz) {
  const int64_t col = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (col < nz) sz[col] = (flops[col] > big && cpB[col + 1] - cpB[col] == 1) ? flops[col] : 0;
}
// chunk of ch = min(SB_CHUNK, big + 1) entries of the flattened copies (off:
// the scan of the sizes, off[nz] = total); a chunk spans at most two columns
// (each holds > big >= ch - 1 entries)
constexpr int SB_CHUNK = 4096;
__device__ __forceinline__ int64_t upper_bound_i64(const int64_t* __restrict__ a, int64_t n, int64_t key) {
  int64_t lo = 0, hi = n;  // first i in [0, n) with a[i] > key
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (a[mid] <= key) lo = mid + 1; else hi = mid;
  }
  return lo;
}
template <int SR>
__global__ __launch_bounds__(256) void k_copy_single_big(int64_t nz, const int64_t* __restrict__ off, int ch,
                                                         const int64_t* __restrict__ cpB,
                                                         const int32_t* __restrict__ irB,
                                                         const double* __restrict__ valB,
                                                         const int2* __restrict__ cmap,
                                                         const int32_t* __restrict__ irA,
                                                         const double* __restrict__ valA,
                                                         const int64_t* __restrict__ colptr,
                                                         int32_t* __restrict__ out_ir, double* __restrict__ out_val) {
  __shared__ int64_t col[2], base[2], dst[2];
  __shared__ int src[2];
  __shared__ double bv[2];
  const int64_t total = off[nz];
  const int64_t q0 = (int64_t)blockIdx.x * ch;
  if (q0 >= total) return;
  const int64_t q1 = min(q0 + ch, total);
  if (threadIdx.x < 2) {
    // the columns holding entries q0 and q1 - 1 (the last column whose offset is <= q)
    const int64_t c = upper_bound_i64(off, nz + 1, threadIdx.x ? q1 - 1 : q0) - 1;
    const int64_t p = cpB[c];
    col[threadIdx.x] = c;
    base[threadIdx.x] = off[c];
    dst[threadIdx.x] = colptr[c];
    src[threadIdx.x] = cmap[irB[p]].x;
    bv[threadIdx.x] = valB[p];
  }
  __syncthreads();
  for (int64_t q = q0 + threadIdx.x; q < q1; q += blockDim.x) {
    const int w = q >= base[1] ? 1 : 0;
    const int64_t e = q - base[w];
    out_ir[dst[w] + e] = irA[src[w] + e];
    out_val[dst[w] + e] = Sem<SR>::mul(valA[src[w] + e], bv[w]);
  }
}

// numeric: block per column

// numeric: one row slab of a big column by bitmap + rank.
// Pass 1 marks the slab's rows in an LDS bitmap, a scan turns the bitmap into
// ranks (= output positions, rows ascending), pass 2 accumulates each product
// into the LDS value slot of its rank.  No hashing, no sort, coalesced output.
// Two launch classes by slab size so that small slabs run 2 workgroups per CU
// (their phases overlap) while large ones get the full LDS for values.
#ifndef CBG_VEC_INIT  // slab LDS initialisation with 16-byte stores
#define CBG_VEC_INIT 1
#endif
#ifndef CBG_ROWS_DIRECT  // bitmap slabs store C's rows from the bitmap words directly
#define CBG_ROWS_DIRECT 1
#endif
#ifndef CBG_ROWS_DIRECT_NT  // ... as nontemporal stores: +66 GB of partial-line writes per scale-22 step
#define CBG_ROWS_DIRECT_NT 0
#endif
template <int CAP, int BS>
struct SlabLds {
  // vals[CAP] f64 | bv[BS] f64 | bm[SLAB_WORDS] | pref[BS+4] | st[BS] | tmp[BS/64+4] | (pad 16) wpre[SLAB_WORDS] u16
  static constexpr int WPRE_OFF =
      ((CAP * 8 + BS * 8 + SLAB_WORDS * 4 + (BS + 4) * 4 + BS * 4 + (BS / WAVE + 4) * 4) + 15) & ~15;
  static constexpr int BYTES = WPRE_OFF + SLAB_WORDS * 2;
  static_assert(BYTES <= 160 * 1024, "slab LDS");
};
#ifndef CBG_SLAB_SMALL_CAP  // the largest value array that keeps 2 blocks of 512 per CU (81856 B of LDS):
#define CBG_SLAB_SMALL_CAP 3056  // 412.6-414.4 vs 418.2-419.4 ms at 2048 (scale 22, same box)
#endif
constexpr int SLAB_SMALL_CAP = CBG_SLAB_SMALL_CAP, SLAB_SMALL_BS = 512;
constexpr int SLAB_LARGE_CAP = SLAB_CAP, SLAB_LARGE_BS = CBG_SLAB_LARGE_BS;

// A's (row, value) of product position q
// (VA = float: A's values narrowed losslessly, see k_vals_f32; the widening is
// exact; VA = PackedRV: the same as (row, f32) records, one gather per product)
template <int SR, typename VA>
__device__ __forceinline__ RowVal a_rowval(const int32_t* __restrict__ irA, const VA* __restrict__ valA, int q,
                                           double b, int lo) {
  if constexpr (std::is_same<VA, PackedRV>::value) {
    const PackedRV e = valA[q];
    return RowVal{e.row - lo, Sem<SR>::mul((double)e.v, b)};
  } else if constexpr (std::is_same<VA, PackedRVD>::value) {
    const PackedRVD e = valA[q];
    return RowVal{e.row - lo, Sem<SR>::mul(__hiloint2double(e.vhi, e.vlo), b)};
  } else {
    return RowVal{irA[q] - lo, Sem<SR>::mul((double)valA[q], b)};
  }
}

struct RankVal {
  int rank, row;
  double v;
};
// IA: int32 sums in vals' first CAP ints, and each product's row written at its
// rank into rows[] (the value region's second half; duplicates write the same
// row), so the output copies the rows instead of walking the bitmap
template <int SR, int BS, typename VA, bool IA>
__device__ __forceinline__ void slab_products(int pass, int total, const int* pref, const int* st, const double* bv,
                                              const int32_t* __restrict__ irA, const VA* __restrict__ valA,
                                              int lo, unsigned* bm, const unsigned short* wpre, double* vals,
                                              int* rows) {
  if (pass == 0) {
    block_products<BS>(
        pref, total, [&](int sg) { return SegI{seg_off(st, pref, sg)}; },
        [&](const SegI& g, int u) { return irA[g.off + u] - lo; },
        [&](int r) { atomicOr(&bm[r >> 5], 1u << (r & 31)); });
  } else {
    // ranks of a group of products are looked up before any accumulates
    block_products3<BS>(
        pref, total, [&](int sg) { return SegV{seg_off(st, pref, sg), bv[sg]}; },
        [&](const SegV& g, int u) { return a_rowval<SR>(irA, valA, g.off + u, g.b, lo); },
        [&](const RowVal& x) {
          const int w = x.row >> 5;
          return RankVal{(int)(wpre[w] + __popc(bm[w] & ((1u << (x.row & 31)) - 1u))), x.row, x.v};
        },
        [&](const RankVal& x) {
          if constexpr (IA) {
            SemI<SR>::lds_acc(reinterpret_cast<int*>(vals) + x.rank, x.v);
            rows[x.rank] = lo + x.row;
          } else {
            Sem<SR>::lds_acc(&vals[x.rank], x.v);
          }
        });
  }
}

// KEPT: every slab of the launch has its kept symbolic bitmap (the host saw
// that no bitmap-mode pair went without a slot), so the kernel carries no
// marking pass: 397.5-397.9 vs 403.0-404.4 ms at scale 22 (same box)
// IA: exact int32 accumulation (IACC, see k_int_bound): the value slots hold
// int32 sums, stored to C as f64
template <int SR, int CAP, int BS, typename VA, bool KEPT, bool IA>
__global__ __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(4))) void k_num_slab(const SlabRec* __restrict__ list, int n, int* __restrict__ queue,
                                                 int plog, const int32_t* __restrict__ irB,
                                                 const double* __restrict__ valB, PMap pm,
                                                 const int32_t* __restrict__ irA,
                                                 const VA* __restrict__ valA,
                                                 int32_t* __restrict__ out_ir,
                                                 double* __restrict__ out_val, const unsigned* __restrict__ gbm,
                                                 const int* __restrict__ cuts) {
  // Persistent blocks (one per CU at this LDS size) pull slabs from a queue.
  // With one block per CU nothing else hides a slab's dependent global reads,
  // so the next slab's record, kept bitmap words and B staging (irB/valB,
  // then the A column map hop) are loaded into registers while the current
  // slab runs its rank scan, products and output.
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* vals = reinterpret_cast<double*>(smem);                          // [CAP]
  double* bv = vals + CAP;                                                 // [BS]
  unsigned* bm = reinterpret_cast<unsigned*>(bv + BS);                     // [SLAB_WORDS]
  int* pref = reinterpret_cast<int*>(bm + SLAB_WORDS);                     // [BS+1]
  int* st = pref + BS + 4;                                                 // [BS]
  int* tmp = st + BS;                                                      // scan scratch + queue slot
  // [SLAB_WORDS], 16-B aligned; a constant offset from smem keeps the LDS
  // address space (a uintptr_t round-up would turn its reads into flat loads)
  unsigned short* wpre = reinterpret_cast<unsigned short*>(smem + SlabLds<CAP, BS>::WPRE_OFF);
  constexpr int WPT = SLAB_WORDS / BS;
  static_assert(WPT % 8 == 0 && (CAP * 8 + BS * 8) % 16 == 0, "rank scan vectors");
  const int tid = threadIdx.x;
  const int wslot = 1 << (plog - 5);
  constexpr int NW = BS / WAVE;
  int i = blockIdx.x;
  if (i >= n) return;
  // prefetch registers (bitmap words in 16-byte lane vectors: words 4 (k*BS + tid) .. +3)
  constexpr int WV = WPT / 4;
  uint4 pw[WV];
  int p_ir = 0;
  double p_bv = 0.0;
  int2 p_ce = make_int2(0, 0);
  auto rec_words = [&](const SlabRec& r) { return (r.hi - r.lo + 31) >> 5; };
  auto staged = [&](const SlabRec& r) { return (r.flags & SLAB_FULL) && r.nb <= BS; };
  auto fetch_words = [&](const SlabRec& r) {
    if (r.slot < 0) return;
    const unsigned* src = gbm + (int64_t)r.slot * wslot + ((r.lo - (r.r << plog)) >> 5);
    const int words = rec_words(r);
#pragma unroll
    for (int k = 0; k < WV; ++k) {
      const int j = 4 * (k * BS + tid);
      if (j + 3 < words) {
        pw[k] = ld_stream4(src + j);
      } else {  // the slab's last partial vector (never past the slab's words)
        pw[k] = make_uint4(j < words ? ld_stream(&src[j]) : 0u, j + 1 < words ? ld_stream(&src[j + 1]) : 0u,
                           j + 2 < words ? ld_stream(&src[j + 2]) : 0u, 0u);
      }
    }
  };
  auto fetch_stage1 = [&](const SlabRec& r) {
    if (staged(r) && tid < r.nb) {
      p_ir = irB[r.p0 + tid];
      p_bv = valB[r.p0 + tid];
    }
  };
  auto fetch_stage2 = [&](const SlabRec& r) {
    if (staged(r) && tid < r.nb) p_ce = pm.at(r.r, p_ir);
  };
  SlabRec rec = list[i];
  // (thread 0) the dequeue in flight: the slab after the next one -- issued a
  // slab ahead, so its returning atomic is not waited for at a slab's start
  int qnext = 0;
  if (tid == 0) qnext = (int)gridDim.x + atomicAdd(queue, 1);
  fetch_words(rec);
  fetch_stage1(rec);
  fetch_stage2(rec);
  while (true) {
    // ---- next work item (its record arrives while this slab fills LDS)
    if (tid == 0) {
      tmp[NW + 2] = qnext;  // the next slab (dequeued during this block's previous slab)
      qnext = (int)gridDim.x + atomicAdd(queue, 1);
    }
    const int nout = rec.nout;
    const int lo = rec.lo, hi = rec.hi;
    const int words = rec_words(rec);
    const int64_t obase = rec.obase;
    const bool have_bm = KEPT || rec.slot >= 0;  // bitmap kept by the symbolic phase: no marking pass
    const bool pre = staged(rec);        // chunk 0 staging came in registers
    if ((c_dbg & 32) && tid == 0) {
      atomicAdd(&g_stat[0], 1ull);
      atomicAdd(&g_stat[1], (rec.flags & SLAB_FULL) ? 0ull : 1ull);
      atomicAdd(&g_stat[2], (unsigned long long)rec.nb);
      atomicAdd(&g_stat[3], (rec.flags & SLAB_FULL) ? 0ull : (unsigned long long)rec.nb);
      atomicAdd(&g_stat[5], (unsigned long long)rec.nout);
      atomicAdd(&g_stat[6], rec.nb > BS ? 1ull : 0ull);
    }
    unsigned long long tmark = wall_clock64();
#pragma unroll
    for (int k = 0; k < WV; ++k) {
      const int j = 4 * (k * BS + tid);
      if (j < words) *reinterpret_cast<uint4*>(bm + j) = have_bm ? pw[k] : make_uint4(0u, 0u, 0u, 0u);
    }
    if (IA) {
      const int id = SemI<SR>::identity();
      int4* v4 = reinterpret_cast<int4*>(vals);
      for (int j = tid; j < (nout + 3) >> 2; j += BS) v4[j] = make_int4(id, id, id, id);
    } else if (CBG_VEC_INIT) {  // 16-byte LDS stores (CAP is even, vals is 16-byte aligned)
      const double id = Sem<SR>::identity();
      double2* v2 = reinterpret_cast<double2*>(vals);
      for (int j = tid; j < (nout + 1) >> 1; j += BS) v2[j] = make_double2(id, id);
    } else {
      for (int j = tid; j < nout; j += BS) vals[j] = Sem<SR>::identity();
    }
    int total = 0;
    if (pre) {
      const int len = tid < rec.nb ? p_ce.y - p_ce.x : 0;
      const int ex = block_excl_scan<BS>(len, tmp, &total);
      pref[tid] = ex;
      if (tid == BS - 1) pref[BS] = total;
      st[tid] = seg_stage(tid < rec.nb ? p_ce.x : 0, ex);
      bv[tid] = tid < rec.nb ? p_bv : 0.0;
    }
    __syncthreads();
    const int inext = tmp[NW + 2];
    const bool has_next = inext < n;
    SlabRec nrec;
    if (has_next) nrec = list[inext];
    phase_mark(tmark, 0);
    const int64_t p0 = rec.p0, p1 = rec.p0 + rec.nb;
    const int first_pass = KEPT ? 1 : have_bm ? 1 : 0;
    for (int pass = first_pass; pass < 2; ++pass) {
      if (pass == 1) {
        // ranks: exclusive prefix of popcounts over the slab's words; thread t
        // owns WPT consecutive words, read and written as 16-byte LDS vectors
        const int w0 = tid * WPT;
        auto word4 = [&](int k) {  // words w0+k .. w0+k+3, zero past the slab
          uint4 v = *reinterpret_cast<const uint4*>(bm + w0 + k);
          if (w0 + k >= words) v.x = 0u;
          if (w0 + k + 1 >= words) v.y = 0u;
          if (w0 + k + 2 >= words) v.z = 0u;
          if (w0 + k + 3 >= words) v.w = 0u;
          return v;
        };
        int sum = 0;
#pragma unroll
        for (int k = 0; k < WPT; k += 4) {
          const uint4 v = word4(k);
          sum += __popc(v.x) + __popc(v.y) + __popc(v.z) + __popc(v.w);
        }
        int tot;
        int run = block_excl_scan<BS>(sum, tmp, &tot);
#pragma unroll
        for (int k = 0; k < WPT; k += 8) {
          const uint4 a = word4(k), b = word4(k + 4);
          const unsigned q[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
          unsigned pk[4];
#pragma unroll
          for (int h = 0; h < 4; ++h) {
            const unsigned x = (unsigned)run;
            run += __popc(q[2 * h]);
            pk[h] = x | ((unsigned)run << 16);
            run += __popc(q[2 * h + 1]);
          }
          *reinterpret_cast<uint4*>(wpre + w0 + k) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
        }
        __syncthreads();
        phase_mark(tmark, 3);
        // next slab: bitmap words and B entries fly while this one multiplies
        if (has_next) {
          fetch_words(nrec);
          fetch_stage1(nrec);
        }
      }
      for (int64_t c0 = p0; c0 < p1; c0 += BS) {
        if (!(pre && c0 == p0)) {
          const int64_t p = c0 + tid;
          int s = 0, len = 0;
          double bval = 0.0;
          if (p < p1) {
            const int2 ce = pm.at(rec.r, irB[p]);
            if (rec.flags & SLAB_FULL) {
              s = ce.x;
              len = ce.y - ce.x;
            } else if (ce.y > ce.x) {
              // the pair's first slab starts at its run's start, the last ends at
              // its end; the cuts between are the symbolic's (offsets into the
              // run, cuts[coff + (slab - 1) * nb + entry]) or searched here
              int a, z;
              if (rec.coff >= 0) {
                const int si = rec.flags >> 3;
                const int64_t j = p - p0;
                a = (rec.flags & 1) ? ce.x : ce.x + cuts[(int64_t)rec.coff + (int64_t)(si - 1) * rec.nb + j];
                z = (rec.flags & 2) ? ce.y : ce.x + cuts[(int64_t)rec.coff + (int64_t)si * rec.nb + j];
              } else {
                a = (rec.flags & 1) ? ce.x : lower_bound_g(irA, ce.x, ce.y, lo);
                z = (rec.flags & 2) ? ce.y : lower_bound_g(irA, a, ce.y, hi);
              }
              s = a;
              len = z - a;
            }
            bval = valB[p];
          }
          const int ex = block_excl_scan<BS>(len, tmp, &total);
          pref[tid] = ex;
          if (tid == BS - 1) pref[BS] = total;
          st[tid] = seg_stage(s, ex);
          bv[tid] = bval;
          __syncthreads();
          phase_mark(tmark, 1);
        } else {
          total = pref[BS];
        }
        if ((c_dbg & 32) && pass == 1 && tid == 0) atomicAdd(&g_stat[4], (unsigned long long)total);
        if (!(c_dbg & (2 << pass)))
          slab_products<SR, BS, VA, IA>(pass, total, pref, st, bv, irA, valA, lo, bm, wpre, vals,
                                        reinterpret_cast<int*>(vals) + CAP);
        __syncthreads();
        phase_mark(tmark, 4 + pass);
      }
    }
    if (has_next) fetch_stage2(nrec);
    // values: coalesced copy; rows: each word scatters its set bits to their
    // ranks in LDS (reusing the value array), then a coalesced copy
    if (IA && !(c_dbg & 8)) {
      // rows and values in rank order (C's order): coalesced copies
      const int* ivals = reinterpret_cast<const int*>(vals);
      for (int j = tid; j < nout; j += BS) {
        out_ir[obase + j] = ivals[CAP + j];
        st_stream(&out_val[obase + j], (double)ivals[j]);
      }
    } else if (!(c_dbg & 8) && CBG_ROWS_DIRECT) {
      // rows straight from the bitmap words to C (a wave's lanes hold
      // consecutive words, so their ranks -- the store addresses -- are
      // consecutive too): no LDS staging of the rows, no barriers
      for (int w = tid; w < words; w += BS) {
        unsigned x = bm[w];
        int pos = wpre[w];
        while (x) {
#if CBG_ROWS_DIRECT_NT
          st_stream(&out_ir[obase + pos++], lo + w * 32 + __ffs(x) - 1);
#else
          out_ir[obase + pos++] = lo + w * 32 + __ffs(x) - 1;  // L2 merges the partial lines
#endif
          x &= x - 1;
        }
      }
      for (int j = tid; j < nout; j += BS)
        st_stream(&out_val[obase + j], IA ? (double)reinterpret_cast<const int*>(vals)[j] : vals[j]);
    } else if (!(c_dbg & 8)) {
      for (int j = tid; j < nout; j += BS)
        st_stream(&out_val[obase + j], IA ? (double)reinterpret_cast<const int*>(vals)[j] : vals[j]);
      __syncthreads();
      int* rows = reinterpret_cast<int*>(vals);
      for (int w = tid; w < words; w += BS) {
        unsigned x = bm[w];
        int pos = wpre[w];
        while (x) {
          rows[pos++] = lo + w * 32 + __ffs(x) - 1;
          x &= x - 1;
        }
      }
      __syncthreads();
      for (int j = tid; j < nout; j += BS) st_stream(&out_ir[obase + j], rows[j]);
    }
    __syncthreads();  // LDS is refilled by the next slab
    phase_mark(tmark, 6);
    if (!has_next) break;
    i = inext;
    rec = nrec;
  }
}

// ----------------------------------------------------------------------------
// per-product segment ids (hash and rank slabs)
// ----------------------------------------------------------------------------
// The flattened product loop (wave_products3) finds a product's segment (its
// B entry) with a per-lane cursor that walks forward one segment per LDS read.
// Where segments are short -- a (column, panel) pair reads A's columns inside
// one row panel: 1-3 rows each at scale 22 -- a lane whose products lie 64
// apart walks ~10 segments per product, a chain of dependent LDS reads before
// each gather.  Instead the staging marks every nonempty segment's first
// product (seg16[ex] = t) and a block max-scan spreads the marks, so each
// product finds its segment with one LDS read and its (A offset, B value) with
// a second: all of a thread's products issue their gathers back to back.
struct __attribute__((aligned(16))) SegRec {
  int off;  // A index of the segment's products minus the segment's first product index
  int pad;
  double b;  // the B entry's value
};
// inclusive max-scan over a wave of non-negative values (DPP, as wave_incl_scan)
__device__ __forceinline__ int wave_incl_max(int v) {
  v = max(v, dpp0<0x111>(v));
  v = max(v, dpp0<0x112>(v));
  v = max(v, dpp0<0x114>(v));
  v = max(v, dpp0<0x118>(v));
  v = max(v, dpp0<0x142, 0xa>(v));
  v = max(v, dpp0<0x143, 0xc>(v));
  return v;
}
// seg16[0, E*BS) zeroed, the heads written (seg16[ex] = t for every nonempty
// segment t) and a barrier passed: spreads every head over its products (block
// max-scan, thread t owns products E t .. E t + E - 1).  Ends with a barrier.
template <int BS, int E>
__device__ __forceinline__ void build_segids(unsigned short* seg16, int* tmp) {
  constexpr int NW = BS / WAVE;
  const int tid = threadIdx.x, lane = lane_id(), w = tid / WAVE;
  int h[E];
  if constexpr (E % 8 == 0) {
#pragma unroll
    for (int j = 0; j < E; j += 8) {
      const uint4 q = reinterpret_cast<const uint4*>(seg16 + tid * E + j)[0];
      const unsigned v[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        h[j + 2 * k] = (int)(v[k] & 0xffffu);
        h[j + 2 * k + 1] = (int)(v[k] >> 16);
      }
    }
  } else if constexpr (E % 4 == 0) {
#pragma unroll
    for (int j = 0; j < E; j += 4) {
      const uint2 q = reinterpret_cast<const uint2*>(seg16 + tid * E + j)[0];
      h[j] = (int)(q.x & 0xffffu);
      h[j + 1] = (int)(q.x >> 16);
      h[j + 2] = (int)(q.y & 0xffffu);
      h[j + 3] = (int)(q.y >> 16);
    }
  } else {
#pragma unroll
    for (int j = 0; j < E; ++j) h[j] = seg16[tid * E + j];
  }
  int m = 0;
#pragma unroll
  for (int j = 0; j < E; ++j) m = max(m, h[j]);
  const int incl = wave_incl_max(m);
  if (lane == WAVE - 1) tmp[w] = incl;
  __syncthreads();
  int before = 0;
#pragma unroll
  for (int v = 0; v < NW; ++v)
    if (v < w) before = max(before, tmp[v]);
  const int lprev = __shfl_up(incl, 1, WAVE);
  int run = max(before, lane > 0 ? lprev : 0);
#pragma unroll
  for (int j = 0; j < E; ++j) {
    run = max(run, h[j]);
    h[j] = run;
  }
  if constexpr (E % 8 == 0) {
#pragma unroll
    for (int j = 0; j < E; j += 8) {
      unsigned v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = (unsigned)h[j + 2 * k] | ((unsigned)h[j + 2 * k + 1] << 16);
      reinterpret_cast<uint4*>(seg16 + tid * E + j)[0] = make_uint4(v[0], v[1], v[2], v[3]);
    }
  } else if constexpr (E % 4 == 0) {
#pragma unroll
    for (int j = 0; j < E; j += 4)
      reinterpret_cast<uint2*>(seg16 + tid * E + j)[0] =
          make_uint2((unsigned)h[j] | ((unsigned)h[j + 1] << 16), (unsigned)h[j + 2] | ((unsigned)h[j + 3] << 16));
  } else {
#pragma unroll
    for (int j = 0; j < E; ++j) seg16[tid * E + j] = (unsigned short)h[j];
  }
  __syncthreads();
}
// products [0, total) by segment ids: thread t takes t + BS k (consecutive
// threads, consecutive products: coalesced inside a segment), U in flight
template <int BS, int U, class L, class A>
__device__ __forceinline__ void block_products_sid(int total, const unsigned short* seg16, const SegRec* srec,
                                                   L&& load, A&& apply) {
  for (int u0 = threadIdx.x; u0 < total; u0 += U * BS) {
    int sg[U];
#pragma unroll
    for (int j = 0; j < U; ++j) sg[j] = u0 + j * BS < total ? seg16[u0 + j * BS] : -1;
    decltype(load(SegRec{}, 0)) x[U];
#pragma unroll
    for (int j = 0; j < U; ++j)
      if (sg[j] >= 0) x[j] = load(srec[sg[j]], u0 + j * BS);
#pragma unroll
    for (int j = 0; j < U; ++j)
      if (sg[j] >= 0) apply(x[j]);
  }
}

// numeric of a sparse (column, panel) pair (hash-mode slab, <= SPARSE_SLAB_MAX
// products): LDS hash sized to the pair's nnz, sorted emit by row buckets
#ifndef CBG_EMIT_MOFF  // emit ranks from cached in-bucket row offsets (1 LDS read per bucket member)
#define CBG_EMIT_MOFF 1
#endif
#ifndef CBG_EMIT_REG  // hash_emit_reg: slots held in registers across the emit's passes
#define CBG_EMIT_REG 1
#endif
#ifndef CBG_EMIT_NB_DIV  // emit buckets of a hash slab: power of two <= T / DIV
#define CBG_EMIT_NB_DIV 4
#endif
#ifndef CBG_HASH_MEMB_ALIAS  // emit member list in the idle staging arrays (3072-slot slabs: 3 blocks per CU, not 2)
#define CBG_HASH_MEMB_ALIAS 0  // 1: +0.4 % at 22, -0.7 % at 18 (same box, 2 runs): within noise, off
#endif
template <int T_, int BS>
struct SlabHashLds {
  static constexpr int T = T_;
  static constexpr int LOGNB = 31 - __builtin_clz(T / CBG_EMIT_NB_DIV);
  static constexpr int NB = 1 << LOGNB;  // row buckets of the sorted emit (power of two <= T/4)
  static constexpr int MEMB = (T * CBG_HASH_LOAD_DEN + CBG_HASH_LOAD_NUM - 1) / CBG_HASH_LOAD_NUM;  // max nnz
  // vals[T] f64 | keys[T] | bv[BS] f64 | pref[BS+4] | st[BS] | tmp | boff[NB+4] | cur[NB] | members[MEMB] u16
  // bv|pref|st: idle during the emit, which reuses them for its in-bucket row
  // offsets (u16, MOFF) and, where both fit, its member list
  static constexpr int PBYTES = BS * 8 + (BS + 4) * 4 + BS * 4;  // staging region bv | pref | st
  static constexpr int IDLE = PBYTES;
  static constexpr bool MOFF_FITS = MEMB * 2 <= IDLE;
  static constexpr bool MEMB_ALIAS = CBG_HASH_MEMB_ALIAS && 2 * MEMB * 2 <= IDLE;
  static constexpr int TMP_OFF = T * 12 + PBYTES;
  static constexpr int BYTES = TMP_OFF + (BS / WAVE + 4) * 4 + (2 * NB + 4) * 4 + (MEMB_ALIAS ? 0 : MEMB * 2);
};

#ifndef CBG_HASH_WPE  // waves per SIMD the hash-slab kernels are compiled for (0: the compiler's choice)
#define CBG_HASH_WPE 0
#endif
#if CBG_HASH_WPE > 0
#define CBG_HASH_WPE_ATTR __attribute__((amdgpu_waves_per_eu(CBG_HASH_WPE)))
#else
#define CBG_HASH_WPE_ATTR
#endif
// CMLEN: cmapP entries are (start, len) -- the whole-column map of the
// column bins -- instead of the panel maps' (first, end)
// INL (with CMLEN): A's columns as inline records (k_inline_cols): an entry of
// B whose A column holds <= 2 entries adds its products at once from the
// record (no map hop, no gathers of A, no staging); the longer ones are staged
// as usual, and a chunk without any skips the scan
template <int SR, int TT, int BS, bool CMLEN, typename VA = double, bool INL = false>
__global__ __launch_bounds__(BS) CBG_HASH_WPE_ATTR void k_num_slab_hash(const SlabRec* __restrict__ list, int n, int* __restrict__ queue,
                                                      int plog, const int32_t* __restrict__ irB,
                                                      const double* __restrict__ valB, PMap pm,
                                                      const int32_t* __restrict__ irA,
                                                      const VA* __restrict__ valA,
                                                      int32_t* __restrict__ out_ir,
                                                      double* __restrict__ out_val,
                                                      const int4* __restrict__ ainl = nullptr) {
  static_assert(!INL || CMLEN, "inline A records: whole-column slabs only");
  // persistent blocks over a queue of hash slabs; the next slab's record and
  // B staging (irB/valB, then the A column map hop) are prefetched into
  // registers while the current slab multiplies and emits (see k_num_slab)
  using L = SlabHashLds<TT, BS>;
  constexpr int T = L::T, NB = L::NB;
  constexpr int LOGNB = L::LOGNB;
  constexpr int NW = BS / WAVE;
  constexpr int PF = (BIG_BS + BS - 1) / BS;  // prefetched chunks (hash slabs have <= BIG_BS B entries)
  static_assert(PF <= 2, "prefetch chunks");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* vals = reinterpret_cast<double*>(smem);
  int* keys = reinterpret_cast<int*>(vals + T);
  double* bv = reinterpret_cast<double*>(keys + T);  // T even: 8-B aligned
  int* pref = reinterpret_cast<int*>(bv + BS);
  int* st = pref + BS + 4;
  int* tmp = reinterpret_cast<int*>(smem + L::TMP_OFF);
  int* boff = tmp + BS / WAVE + 4;
  int* cur = boff + NB + 4;
  unsigned short* members = L::MEMB_ALIAS ? reinterpret_cast<unsigned short*>(bv) + L::MEMB
                                          : reinterpret_cast<unsigned short*>(cur + NB);
  const int tid = threadIdx.x;
  int i = blockIdx.x;
  if (i >= n) return;
  int p_ir0 = 0, p_ir1 = 0;
  double p_bv0 = 0.0, p_bv1 = 0.0;
  int2 p_ce0 = make_int2(0, 0), p_ce1 = make_int2(0, 0);
  auto staged = [&](const SlabRec& r) { return !INL && r.nb <= PF * BS; };
  auto fetch1 = [&](const SlabRec& r) {
    if (!staged(r)) return;
    if (tid < r.nb) {
      p_ir0 = irB[r.p0 + tid];
      p_bv0 = valB[r.p0 + tid];
    }
    if (PF > 1 && BS + tid < r.nb) {
      p_ir1 = irB[r.p0 + BS + tid];
      p_bv1 = valB[r.p0 + BS + tid];
    }
  };
  // A(:,k)'s run over the slab's rows: one map entry, or the first and last
  // panels' entries of a panel group (rows [lo, hi) span panels r .. r1)
  auto seg_of = [&](const SlabRec& r, int k) -> int2 {
    const int2 e = pm.at(r.r, k);
    if (CMLEN) return make_int2(e.x, e.x + e.y);
    const int r1 = (r.hi - 1) >> plog;
    if (r1 == r.r) return e;
    return make_int2(e.x, pm.at(r1, k).y);
  };
  auto fetch2 = [&](const SlabRec& r) {
    if (!staged(r)) return;
    if (tid < r.nb) p_ce0 = seg_of(r, p_ir0);
    if (PF > 1 && BS + tid < r.nb) p_ce1 = seg_of(r, p_ir1);
  };
  SlabRec rec = list[i];
  // (thread 0) the dequeue in flight: the slab after the next one -- issued a
  // slab ahead, so its returning atomic is not waited for at a slab's start
  int qnext = 0;
  if (tid == 0) qnext = (int)gridDim.x + atomicAdd(queue, 1);
  fetch1(rec);
  fetch2(rec);
  while (true) {
    if (tid == 0) {
      tmp[NW + 2] = qnext;  // the next slab (dequeued during this block's previous slab)
      qnext = (int)gridDim.x + atomicAdd(queue, 1);
    }
    const bool pre = staged(rec);
    unsigned long long tmark = wall_clock64();
    if (CBG_VEC_INIT) {  // 16-byte LDS stores (T is a multiple of 256; vals and keys are 16-byte aligned)
      const double id = Sem<SR>::identity();
      double2* v2 = reinterpret_cast<double2*>(vals);
      int4* k4 = reinterpret_cast<int4*>(keys);
      for (int j = tid; j < T / 2; j += BS) v2[j] = make_double2(id, id);
      for (int j = tid; j < T / 4; j += BS) k4[j] = make_int4(EMPTY_KEY, EMPTY_KEY, EMPTY_KEY, EMPTY_KEY);
    } else {
      for (int j = tid; j < T; j += BS) {
        keys[j] = EMPTY_KEY;
        vals[j] = Sem<SR>::identity();
      }
    }
    __syncthreads();
    phase_mark(tmark, 7);
    const int inext = tmp[NW + 2];
    const bool has_next = inext < n;
    SlabRec nrec;
    if (has_next) nrec = list[inext];
    const int64_t p1 = rec.p0 + rec.nb;
    const int nch = (int)((rec.nb + BS - 1) / BS);
    for (int c = 0; c < nch; ++c) {
      const int64_t p = rec.p0 + (int64_t)c * BS + tid;
      int s = 0, len = 0;
      double bval = 0.0;
      if (INL) {
        if (p < p1) {
          const int k = irB[p];
          bval = valB[p];
          const int4 r = ainl[2 * (int64_t)k];
          if (r.x <= 2) {
            if (r.x >= 1) {
              const int4 v = ainl[2 * (int64_t)k + 1];
              hash_acc_t<SR, T>(keys, vals, r.y, Sem<SR>::mul(__hiloint2double(v.y, v.x), bval));
              if (r.x == 2) hash_acc_t<SR, T>(keys, vals, r.z, Sem<SR>::mul(__hiloint2double(v.w, v.z), bval));
            }
          } else {
            s = r.y;
            len = r.x;
          }
        }
        if (!__syncthreads_or(len > 0)) {
          if (c == nch - 1 && has_next) fetch1(nrec);
          continue;
        }
      } else if (p < p1) {
        int2 ce;
        if (pre) {
          ce = c == 0 ? p_ce0 : p_ce1;
          bval = c == 0 ? p_bv0 : p_bv1;
        } else {
          ce = seg_of(rec, irB[p]);
          bval = valB[p];
        }
        s = ce.x;
        len = ce.y - ce.x;
      }
      int total;
      const int ex = block_excl_scan<BS>(len, tmp, &total);
      pref[tid] = ex;
      if (tid == BS - 1) pref[BS] = total;
      st[tid] = seg_stage(s, ex);
      bv[tid] = bval;
      __syncthreads();
      phase_mark(tmark, 13);
      if (c == nch - 1 && has_next) fetch1(nrec);
      if ((c_dbg & 32) && tid == 0) atomicAdd(&g_stat[CMLEN ? 8 : 7], (unsigned long long)total);
      if (!(c_dbg & 512))
        block_products<BS>(
            pref, total, [&](int sg) { return SegV{seg_off(st, pref, sg), bv[sg]}; },
            [&](const SegV& g, int u) { return a_rowval<SR, VA>(irA, valA, g.off + u, g.b, 0); },
            [&](const RowVal& x) { hash_acc_t<SR, T>(keys, vals, x.row, x.v); });
      __syncthreads();
      phase_mark(tmark, 14);
    }
    if (has_next) fetch2(nrec);
    if ((c_dbg & 32) && tid == 0) atomicAdd(&g_stat[9], (unsigned long long)rec.nout);
    int sl = plog;  // emit buckets span 2^sl rows from lo (a panel group spans several panels)
    if (!CMLEN)
      while ((1LL << sl) < (int64_t)(rec.hi - rec.lo)) ++sl;
    const int bshift = sl > LOGNB ? sl - LOGNB : 0;
    // in-bucket offsets fit u16 for panel-group slabs (span <= 2^(plog+4) rows,
    // bshift <= 15, 17 for groups of 64 panels); every slab uses them while bshift <= 16
    constexpr bool MOFF = L::MOFF_FITS && CBG_EMIT_MOFF;
    if (c_dbg & 1024)
      ;
    else if (MOFF && CBG_EMIT_REG && bshift <= 16)
      hash_emit_reg<T, BS, NB>(keys, vals, rec.lo, bshift, boff, cur, members, tmp,
                               reinterpret_cast<unsigned short*>(bv), out_ir, out_val, rec.obase);
    else if (MOFF && bshift <= 16)
      hash_emit_sorted<T, BS, NB, MOFF>(keys, vals, rec.lo, bshift, boff, cur, members, tmp, out_ir, out_val,
                                        rec.obase, reinterpret_cast<unsigned short*>(bv));
    else
      hash_emit_sorted<T, BS, NB, false>(keys, vals, rec.lo, bshift, boff, cur, members, tmp, out_ir, out_val,
                                         rec.obase);
    __syncthreads();  // LDS is reset for the next slab
    phase_mark(tmark, 15);
    if (!has_next) break;
    i = inext;
    rec = nrec;
  }
}

// ----------------------------------------------------------------------------
// numeric of a hash-mode (column, panel) pair by bitmap rank: no hash, no sort
// ----------------------------------------------------------------------------
// A single-panel hash pair (<= SPARSE_SLAB_MAX products, one chunk of <=
// BIG_BS B entries, rows inside one 2^plog panel).  The hash slab pays a
// returning CAS chain per product and a bucket counting sort per entry; here:
//   1. every lane gathers its <= RK products at once (all loads in flight) and
//      keeps (row, value) in registers; it marks the rows in an LDS bitmap of
//      the panel (ds_or, no return);
//   2. a block scan of the popcounts of 4-word groups gives every group its
//      first output rank (u16);
//   3. each product's rank = group rank + popcount of the bits below it in its
//      group; products accumulate at their ranks (vals[nout]);
//   4. C's rows come straight out of the bitmap words, already in order
//      (consecutive lanes own consecutive groups: the stores are consecutive
//      positions), values copied from vals with coalesced stores.
// The bitmap (32 KiB) is zeroed per slab and read twice in 16-byte vectors; every
// random LDS access is one ds_or, two reads (group, its rank) and the semiring's
// atomic per product.
template <int NCAP, int BS, int VB = 8>
struct SlabRankLds {
  // ust: during the products seg16[SPARSE_SLAB_MAX] u16 (each product's segment) |
  //      srec[BS] (segment: A offset minus its first product index, B value);
  //      from the rank scan on vals[NCAP] (f64, or int32 under IACC: VB = 4)
  // bm[SLAB_WORDS] | gpre[SLAB_WORDS / 4] u16 | tmp[BS/64+4]
  static constexpr int SEG_BYTES = SPARSE_SLAB_MAX * 2;
  static constexpr int UST = NCAP * VB > SEG_BYTES + BS * 16 ? NCAP * VB : SEG_BYTES + BS * 16;
  static constexpr int BM_OFF = UST;
  static constexpr int GPRE_OFF = BM_OFF + SLAB_WORDS * 4;
  static constexpr int TMP_OFF = GPRE_OFF + (SLAB_WORDS / 4) * 2;
  static constexpr int BYTES = TMP_OFF + (BS / WAVE + 4) * 4;
  static_assert(SEG_BYTES % 16 == 0 && BM_OFF % 16 == 0 && GPRE_OFF % 16 == 0, "rank slab LDS alignment");
};
constexpr int RANK_BS = 512;
static_assert(SPARSE_NNZ_MAX <= 4096 && BIG_BS <= RANK_BS && GRANK_PMAX % RANK_BS == 0,
              "group rank slab: nonzeros, B entries, products per thread");
static_assert(4096 <= SLAB_WORDS, "a rank slab's rows (<= 4096) are written into its bitmap's words");
// a rank slab stages one B entry per thread: the symbolic's sparse pairs (the
// rank slabs' source, sym_pair) have <= BIG_BS B entries
static_assert(BIG_BS <= RANK_BS, "rank slabs stage <= RANK_BS B entries");
static_assert(SPARSE_SLAB_MAX % RANK_BS == 0 && SPARSE_SLAB_MAX / RANK_BS <= 16, "rank slab products per lane");
static_assert(SPARSE_SLAB_MAX == 8 * RANK_BS, "segment scan: 8 products per thread");

__device__ __forceinline__ int popc4(const uint4& q) {
  return __popc(q.x) + __popc(q.y) + __popc(q.z) + __popc(q.w);
}
template <int SR, int NCAP, int BS, typename VA, bool IA>
__global__ __launch_bounds__(BS) void k_num_slab_rank(const SlabRec* __restrict__ list, int n,
                                                      int* __restrict__ queue, const int32_t* __restrict__ irB,
                                                      const double* __restrict__ valB,
                                                      PMap pm,
                                                      const int32_t* __restrict__ irA, const VA* __restrict__ valA,
                                                      int32_t* __restrict__ out_ir, double* __restrict__ out_val) {
  using L = SlabRankLds<NCAP, BS, IA ? 4 : 8>;
  constexpr int NW = BS / WAVE;
  constexpr int RK = SPARSE_SLAB_MAX / BS;  // products per thread
  constexpr int NG = SLAB_WORDS / 4;        // 4-word groups of a panel
  constexpr int GPT = NG / BS;              // groups per thread in the rank scan
  static_assert(GPT == 4, "rank scan packs 4 u16 group ranks per thread");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* vals = reinterpret_cast<double*>(smem);
  unsigned short* seg16 = reinterpret_cast<unsigned short*>(smem);
  SegRec* srec = reinterpret_cast<SegRec*>(smem + L::SEG_BYTES);
  unsigned* bm = reinterpret_cast<unsigned*>(smem + L::BM_OFF);
  uint4* bm4 = reinterpret_cast<uint4*>(smem + L::BM_OFF);
  unsigned short* gpre = reinterpret_cast<unsigned short*>(smem + L::GPRE_OFF);
  int* tmp = reinterpret_cast<int*>(smem + L::TMP_OFF);
  const int tid = threadIdx.x, lane = lane_id(), w = tid / WAVE;
  int i = blockIdx.x;
  if (i >= n) return;
  // next slab's staging (one B entry per thread), fetched while this one runs
  int p_ir = 0;
  double p_bv = 0.0;
  int2 p_ce = make_int2(0, 0);
  auto fetch1 = [&](const SlabRec& r) {
    if (tid < r.nb) {
      p_ir = irB[r.p0 + tid];
      p_bv = valB[r.p0 + tid];
    }
  };
  auto fetch2 = [&](const SlabRec& r) {
    if (tid < r.nb) p_ce = pm.at(r.r, p_ir);
  };
  SlabRec rec = list[i];
  // (thread 0) the dequeue in flight: the slab after the next one -- issued a
  // slab ahead, so its returning atomic is not waited for at a slab's start
  int qnext = 0;
  if (tid == 0) qnext = (int)gridDim.x + atomicAdd(queue, 1);
  fetch1(rec);
  fetch2(rec);
  while (true) {
    if (tid == 0) {
      tmp[NW + 2] = qnext;  // the next slab (dequeued during this block's previous slab)
      qnext = (int)gridDim.x + atomicAdd(queue, 1);
    }
    unsigned long long tmark = wall_clock64();
    const int lo = rec.lo, nout = rec.nout;
    const int ng = (((rec.hi - lo + 31) >> 5) + 3) >> 2;
    const int64_t obase = rec.obase;
    for (int g = tid; g < ng; g += BS) bm4[g] = make_uint4(0u, 0u, 0u, 0u);
    reinterpret_cast<uint4*>(seg16)[tid] = make_uint4(0u, 0u, 0u, 0u);  // 8 products per thread
    // staging: segment t = B entry t; its first product at ex; heads of the
    // nonempty segments marked at their first product
    const int len = tid < rec.nb ? p_ce.y - p_ce.x : 0;
    int total;
    const int ex = block_excl_scan<BS>(len, tmp, &total);  // (its barriers order the zeroing above)
    srec[tid] = SegRec{(tid < rec.nb ? p_ce.x : 0) - ex, 0, tid < rec.nb ? p_bv : 0.0};
    if (len > 0) seg16[ex] = (unsigned short)tid;
    const int inext = tmp[NW + 2];
    const bool has_next = inext < n;
    SlabRec nrec;
    if (has_next) nrec = list[inext];
    __syncthreads();
    build_segids<BS, RK>(seg16, tmp);  // every product's segment
    phase_mark(tmark, 16);
    // 1. products into registers (thread t: t + BS k), rows marked in the bitmap
    int xr[RK];
    typename std::conditional<IA, int, double>::type xv[RK];  // (exact integers as int: fewer VGPRs)
    {
      int sg[RK];
#pragma unroll
      for (int k = 0; k < RK; ++k) {
        const int u = tid + k * BS;
        sg[k] = u < total ? seg16[u] : -1;
      }
#pragma unroll
      for (int k = 0; k < RK; ++k) {
        xr[k] = -1;
        if (sg[k] >= 0 && !(c_dbg & 512)) {
          const SegRec r = srec[sg[k]];
          const RowVal x = a_rowval<SR, VA>(irA, valA, r.off + tid + k * BS, r.b, lo);
          xr[k] = x.row;
          if constexpr (IA) xv[k] = (int)x.v;
          else xv[k] = x.v;
        }
      }
#pragma unroll
      for (int k = 0; k < RK; ++k)
        if (xr[k] >= 0) atomicOr(&bm[xr[k] >> 5], 1u << (xr[k] & 31));
    }
    if (has_next) fetch1(nrec);
    __syncthreads();
    phase_mark(tmark, 17);
    // 2. group ranks: thread t owns groups 4t .. 4t+3 (one 8-byte store of 4
    // u16); vals (aliasing the staging, now idle) set to the semiring's identity
    {
      if (IA) {
        const int id = SemI<SR>::identity();
        int4* v4 = reinterpret_cast<int4*>(vals);
        for (int j = tid; j < (nout + 3) >> 2; j += BS) v4[j] = make_int4(id, id, id, id);
      } else {
        const double id = Sem<SR>::identity();
        double2* v2 = reinterpret_cast<double2*>(vals);
        for (int j = tid; j < (nout + 1) >> 1; j += BS) v2[j] = make_double2(id, id);
      }
      uint4 q[GPT];
      int sum = 0;
#pragma unroll
      for (int j = 0; j < GPT; ++j) {
        const int g = tid * GPT + j;
        q[j] = g < ng ? bm4[g] : make_uint4(0u, 0u, 0u, 0u);
        sum += popc4(q[j]);
      }
      int tot;
      int run = block_excl_scan<BS>(sum, tmp, &tot);
      unsigned pk[GPT / 2];
#pragma unroll
      for (int j = 0; j < GPT; j += 2) {
        const unsigned a = (unsigned)run;
        run += popc4(q[j]);
        pk[j / 2] = a | ((unsigned)run << 16);
        run += popc4(q[j + 1]);
      }
      *reinterpret_cast<uint2*>(gpre + tid * GPT) = make_uint2(pk[0], pk[1]);
    }
    __syncthreads();
    phase_mark(tmark, 18);
    // 3. accumulate at the ranks (all lookups first, then the atomics); each
    // product also writes its row at its rank into the bitmap's words, which
    // no lookup reads any more after the barrier (duplicates write the same
    // row), so C's rows come out in order with a coalesced copy
    {
      int rk[RK];
#pragma unroll
      for (int k = 0; k < RK; ++k) {
        rk[k] = -1;
        if (xr[k] >= 0) {
          const int r = xr[k], wd = r >> 5, g = wd >> 2, j = wd & 3;
          const uint4 q = bm4[g];
          const unsigned below = (1u << (r & 31)) - 1u;
          int x = gpre[g];
          x += j > 0 ? __popc(q.x) : __popc(q.x & below);
          if (j >= 1) x += j > 1 ? __popc(q.y) : __popc(q.y & below);
          if (j >= 2) x += j > 2 ? __popc(q.z) : __popc(q.z & below);
          if (j >= 3) x += __popc(q.w & below);
          rk[k] = x;
        }
      }
      __syncthreads();
      int* rows = reinterpret_cast<int*>(bm);  // [nout] (nout <= NCAP <= SLAB_WORDS)
#pragma unroll
      for (int k = 0; k < RK; ++k)
        if (rk[k] >= 0) {
          if constexpr (IA) SemI<SR>::lds_acc(reinterpret_cast<int*>(vals) + rk[k], (double)xv[k]);
          else Sem<SR>::lds_acc(&vals[rk[k]], xv[k]);
          rows[rk[k]] = lo + xr[k];
        }
    }
    if (has_next) fetch2(nrec);
    __syncthreads();
    phase_mark(tmark, 19);
    // 4. rows and values in rank order (C's order): coalesced copies
    if (!(c_dbg & 1024)) {
      const int* rows = reinterpret_cast<const int*>(bm);
      for (int j = tid; j < nout; j += BS) {
        out_ir[obase + j] = rows[j];
        st_emit(&out_val[obase + j], IA ? (double)reinterpret_cast<const int*>(vals)[j] : vals[j]);
      }
    }
    if ((c_dbg & 32) && tid == 0) {
      atomicAdd(&g_stat[10], (unsigned long long)total);
      atomicAdd(&g_stat[11], (unsigned long long)nout);
    }
    __syncthreads();  // LDS is reset for the next slab
    phase_mark(tmark, 20);
    if (!has_next) break;
    i = inext;
    rec = nrec;
  }
}

// ----------------------------------------------------------------------------
// numeric of a panel-group hash slab by two-level rank: no hash, no sort
// ----------------------------------------------------------------------------
// A panel group's slab (sym_group: <= BIG_BS B entries, <= GROUP_T * 2/3
// products, <= SPARSE_NNZ_MAX nonzeros) spans up to 2^22 rows, too many for the
// rank slab's one-bit-per-row bitmap (32 KiB per 2^18 rows).  Its rows are
// sparse, so the bitmap is split in two levels:
//   1. level 1, a bit per 32-row block of the span (<= 2^17 bits, 16 KiB):
//      every product marks its block (ds_or); a scan of the popcounts gives
//      every touched block its slot, in row order (slots <= nonzeros);
//   2. level 2, a word per slot: every product marks its row's bit in its
//      block's word (ds_or); a scan of those popcounts gives every slot its
//      first rank;
//   3. a product's rank = its slot's rank + the bits below it in the word;
//      the products accumulate at their ranks and write their rows at them
//      (into level 1's words, idle by then, when they fit): C's rows and
//      values come out in order with coalesced copies.
// Against the hash slab (a returning CAS chain per product, then a bucket
// counting sort of the table) this is two ds_or, two lookups and the
// semiring's atomic per product.
template <int NCAP, int BS, int SPANLOG, int PMAX, int VB = 8>
struct SlabGRankLds {
  // ust: seg16[PMAX] u16 | srec[BS]; from step 2 on vals[NCAP] (f64, or int32
  // under IACC: VB = 4)
  // l1[L1W] (level 1; then C's rows when NCAP <= L1W) | g1pre[L1W/4] u16 |
  // l2[NCAP] | g2pre[NCAP/4] u16 | rows[NCAP] (when NCAP > L1W) | tmp[BS/64+4]
  static constexpr int L1W = 1 << (SPANLOG - 10);
  static constexpr bool ROWS_IN_L1 = NCAP <= L1W;
  static constexpr int SEG_BYTES = PMAX * 2;
  static constexpr int UST = NCAP * VB > SEG_BYTES + BS * 16 ? NCAP * VB : SEG_BYTES + BS * 16;
  static constexpr int L1_OFF = UST;
  static constexpr int G1_OFF = L1_OFF + L1W * 4;
  static constexpr int L2_OFF = G1_OFF + (L1W / 4 * 2 + 15) / 16 * 16;
  static constexpr int G2_OFF = L2_OFF + NCAP * 4;
  static constexpr int ROWS_OFF = G2_OFF + (NCAP / 4) * 2;
  static constexpr int TMP_OFF = ROWS_OFF + (ROWS_IN_L1 ? 0 : NCAP * 4);
  static constexpr int BYTES = TMP_OFF + (BS / WAVE + 4) * 4;
  static_assert(SEG_BYTES % 16 == 0 && L1_OFF % 16 == 0 && G1_OFF % 16 == 0 && L2_OFF % 16 == 0 &&
                    G2_OFF % 16 == 0 && ROWS_OFF % 16 == 0 && TMP_OFF % 16 == 0,
                "group rank slab LDS alignment");
};
// the rank of bit b of a bitmap: its 4-word group's rank + the bits below it
__device__ __forceinline__ int bitmap_rank(const uint4* bm4, const unsigned short* gpre, int b) {
  const int wd = b >> 5, g = wd >> 2, j = wd & 3;
  const uint4 q = bm4[g];
  const unsigned below = (1u << (b & 31)) - 1u;
  int x = gpre[g];
  x += j > 0 ? __popc(q.x) : __popc(q.x & below);
  if (j >= 1) x += j > 1 ? __popc(q.y) : __popc(q.y & below);
  if (j >= 2) x += j > 2 ? __popc(q.z) : __popc(q.z & below);
  if (j >= 3) x += __popc(q.w & below);
  return x;
}
// the first rank of every 4-word group of bm4[0, ng) into gpre (u16, GPT groups
// per thread, GPT even); returns the total (block-uniform)
template <int BS, int GPT>
__device__ __forceinline__ int bitmap_group_ranks(const uint4* bm4, int ng, unsigned short* gpre, int* tmp) {
  const int tid = threadIdx.x;
  uint4 q[GPT];
  int sum = 0;
#pragma unroll
  for (int j = 0; j < GPT; ++j) {
    const int g = tid * GPT + j;
    q[j] = g < ng ? bm4[g] : make_uint4(0u, 0u, 0u, 0u);
    sum += popc4(q[j]);
  }
  int tot;
  int run = block_excl_scan<BS>(sum, tmp, &tot);
  unsigned pk[GPT / 2];
#pragma unroll
  for (int j = 0; j < GPT; j += 2) {
    const unsigned a = (unsigned)run;
    run += popc4(q[j]);
    pk[j / 2] = a | ((unsigned)run << 16);
    run += popc4(q[j + 1]);
  }
  if (tid * GPT < ng) {
    if constexpr (GPT == 2) *reinterpret_cast<unsigned*>(gpre + tid * GPT) = pk[0];
    else if constexpr (GPT == 4) *reinterpret_cast<uint2*>(gpre + tid * GPT) = make_uint2(pk[0], pk[1]);
    else {
#pragma unroll
      for (int j = 0; j < GPT / 2; ++j) reinterpret_cast<unsigned*>(gpre + tid * GPT)[j] = pk[j];
    }
  }
  return tot;
}
template <int SR, int NCAP, int BS, int SPANLOG, int PMAX, typename VA, bool IA>
__global__ __launch_bounds__(BS) void k_num_slab_grank(const SlabRec* __restrict__ list, int n,
                                                       int* __restrict__ queue, int plog,
                                                       const int32_t* __restrict__ irB,
                                                       const double* __restrict__ valB, PMap pm,
                                                       const int32_t* __restrict__ irA, const VA* __restrict__ valA,
                                                       int32_t* __restrict__ out_ir, double* __restrict__ out_val) {
  using L = SlabGRankLds<NCAP, BS, SPANLOG, PMAX, IA ? 4 : 8>;
  constexpr int NW = BS / WAVE;
  constexpr int RK = PMAX / BS;  // products per thread
  static_assert(PMAX % BS == 0, "products per thread");
  constexpr int G1PT = (L::L1W / 4 + BS - 1) / BS < 2 ? 2 : (L::L1W / 4 + BS - 1) / BS;  // level-1 groups per thread
  constexpr int G2PT = (NCAP / 4 + BS - 1) / BS < 2 ? 2 : (NCAP / 4 + BS - 1) / BS;
  static_assert(G1PT >= 2 && G1PT % 2 == 0 && G2PT % 2 == 0, "group rank scans: pairs of u16 ranks");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* vals = reinterpret_cast<double*>(smem);
  unsigned short* seg16 = reinterpret_cast<unsigned short*>(smem);
  SegRec* srec = reinterpret_cast<SegRec*>(smem + L::SEG_BYTES);
  unsigned* l1 = reinterpret_cast<unsigned*>(smem + L::L1_OFF);
  uint4* l1q = reinterpret_cast<uint4*>(smem + L::L1_OFF);
  unsigned short* g1pre = reinterpret_cast<unsigned short*>(smem + L::G1_OFF);
  unsigned* l2 = reinterpret_cast<unsigned*>(smem + L::L2_OFF);
  uint4* l2q = reinterpret_cast<uint4*>(smem + L::L2_OFF);
  unsigned short* g2pre = reinterpret_cast<unsigned short*>(smem + L::G2_OFF);
  int* tmp = reinterpret_cast<int*>(smem + L::TMP_OFF);
  const int tid = threadIdx.x;
  int i = blockIdx.x;
  if (i >= n) return;
  int p_ir = 0;
  double p_bv = 0.0;
  int2 p_ce = make_int2(0, 0);
  auto fetch1 = [&](const SlabRec& r) {
    if (tid < r.nb) {
      p_ir = irB[r.p0 + tid];
      p_bv = valB[r.p0 + tid];
    }
  };
  // A(:,k)'s run over the group's panels r .. r1: the first panel's start to
  // the last one's end
  auto fetch2 = [&](const SlabRec& r) {
    if (tid < r.nb) {
      const int r1 = (r.hi - 1) >> plog;
      p_ce = pm.at(r.r, p_ir);
      if (r1 != r.r) p_ce.y = pm.at(r1, p_ir).y;
    }
  };
  SlabRec rec = list[i];
  int qnext = 0;
  if (tid == 0) qnext = (int)gridDim.x + atomicAdd(queue, 1);
  fetch1(rec);
  fetch2(rec);
  while (true) {
    if (tid == 0) {
      tmp[NW + 2] = qnext;
      qnext = (int)gridDim.x + atomicAdd(queue, 1);
    }
    unsigned long long tmark = wall_clock64();
    const int lo = rec.lo, nout = rec.nout;
    const int ng1 = (((rec.hi - lo + 1023) >> 10) + 3) >> 2;  // level-1 groups (32 rows a bit, 32 bits a word)
    const int64_t obase = rec.obase;
    for (int g = tid; g < ng1; g += BS) l1q[g] = make_uint4(0u, 0u, 0u, 0u);
    for (int g = tid; g < (nout + 3) >> 2; g += BS) l2q[g] = make_uint4(0u, 0u, 0u, 0u);
    for (int g = tid; g < PMAX / 8; g += BS) reinterpret_cast<uint4*>(seg16)[g] = make_uint4(0u, 0u, 0u, 0u);
    const int len = tid < rec.nb ? p_ce.y - p_ce.x : 0;
    int total;
    const int ex = block_excl_scan<BS>(len, tmp, &total);  // (its barriers order the zeroing above)
    srec[tid] = SegRec{(tid < rec.nb ? p_ce.x : 0) - ex, 0, tid < rec.nb ? p_bv : 0.0};
    if (len > 0) seg16[ex] = (unsigned short)tid;
    const int inext = tmp[NW + 2];
    const bool has_next = inext < n;
    SlabRec nrec;
    if (has_next) nrec = list[inext];
    __syncthreads();
    build_segids<BS, RK>(seg16, tmp);
    phase_mark(tmark, 16);
    // 1. products into registers, their 32-row blocks marked in level 1
    // (exact integers as int: fewer VGPRs, more blocks per CU)
    int xr[RK];
    typename std::conditional<IA, int, double>::type xv[RK];
    {
      int sg[RK];
#pragma unroll
      for (int k = 0; k < RK; ++k) {
        const int u = tid + k * BS;
        sg[k] = u < total ? seg16[u] : -1;
      }
#pragma unroll
      for (int k = 0; k < RK; ++k) {
        xr[k] = -1;
        if (sg[k] >= 0) {
          const SegRec r = srec[sg[k]];
          const RowVal x = a_rowval<SR, VA>(irA, valA, r.off + tid + k * BS, r.b, lo);
          xr[k] = x.row;
          if constexpr (IA) xv[k] = (int)x.v;
          else xv[k] = x.v;
        }
      }
#pragma unroll
      for (int k = 0; k < RK; ++k)
        if (xr[k] >= 0) atomicOr(&l1[xr[k] >> 10], 1u << ((xr[k] >> 5) & 31));
    }
    if (has_next) fetch1(nrec);
    __syncthreads();
    phase_mark(tmark, 17);
    // 2. level-1 slots; vals (aliasing the staging, idle now) set to the identity
    if (IA) {
      const int id = SemI<SR>::identity();
      int4* v4 = reinterpret_cast<int4*>(vals);
      for (int j = tid; j < (nout + 3) >> 2; j += BS) v4[j] = make_int4(id, id, id, id);
    } else {
      const double id = Sem<SR>::identity();
      double2* v2 = reinterpret_cast<double2*>(vals);
      for (int j = tid; j < (nout + 1) >> 1; j += BS) v2[j] = make_double2(id, id);
    }
    const int nslot = bitmap_group_ranks<BS, G1PT>(l1q, ng1, g1pre, tmp);
    __syncthreads();
    int sl[RK];
#pragma unroll
    for (int k = 0; k < RK; ++k) {
      sl[k] = -1;
      if (xr[k] >= 0) {
        sl[k] = bitmap_rank(l1q, g1pre, xr[k] >> 5);
        atomicOr(&l2[sl[k]], 1u << (xr[k] & 31));
      }
    }
    __syncthreads();
    phase_mark(tmark, 18);
    // 3. ranks: level-2 group ranks, then every product's rank; accumulate and
    // write the rows at their ranks (into level 1, which nothing reads now)
    bitmap_group_ranks<BS, G2PT>(l2q, (nslot + 3) >> 2, g2pre, tmp);
    __syncthreads();
    {
      int* rows = reinterpret_cast<int*>(smem + (L::ROWS_IN_L1 ? L::L1_OFF : L::ROWS_OFF));
#pragma unroll
      for (int k = 0; k < RK; ++k)
        if (sl[k] >= 0) {
          const int rk = bitmap_rank(l2q, g2pre, (sl[k] << 5) | (xr[k] & 31));
          if constexpr (IA) SemI<SR>::lds_acc(reinterpret_cast<int*>(vals) + rk, (double)xv[k]);
          else Sem<SR>::lds_acc(&vals[rk], xv[k]);
          rows[rk] = lo + xr[k];
        }
    }
    if (has_next) fetch2(nrec);
    __syncthreads();
    phase_mark(tmark, 19);
    // 4. rows and values in rank order: coalesced copies
    {
      const int* rows = reinterpret_cast<const int*>(smem + (L::ROWS_IN_L1 ? L::L1_OFF : L::ROWS_OFF));
      for (int j = tid; j < nout; j += BS) {
        out_ir[obase + j] = rows[j];
        st_emit(&out_val[obase + j], IA ? (double)reinterpret_cast<const int*>(vals)[j] : vals[j]);
      }
    }
    if ((c_dbg & 32) && tid == 0) {
      atomicAdd(&g_stat[10], (unsigned long long)total);
      atomicAdd(&g_stat[11], (unsigned long long)nout);
    }
    __syncthreads();
    phase_mark(tmark, 20);
    if (!has_next) break;
    i = inext;
    rec = nrec;
  }
}

// ----------------------------------------------------------------------------
// column compaction of C
// ----------------------------------------------------------------------------
__global__ void k_col_flags(int64_t n, const int32_t* __restrict__ cnt, int64_t* __restrict__ flag) {
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < n) flag[i] = cnt[i] > 0 ? 1 : 0;
}
__global__ void k_col_scatter(int64_t n, const int32_t* __restrict__ cnt, const int64_t* __restrict__ pos,
                              const int32_t* __restrict__ jcB, const int64_t* __restrict__ colptr,
                              int32_t* __restrict__ jcC, int64_t* __restrict__ cpC) {
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < n && cnt[i] > 0) {
    jcC[pos[i]] = jcB[i];
    cpC[pos[i]] = colptr[i];
  }
  if (i == n) cpC[pos[n]] = colptr[n];
}

// ----------------------------------------------------------------------------
// host orchestration
// ----------------------------------------------------------------------------
void local_spgemm_impl(const cbg_tile& A, const cbg_tile& B, int semiring, cbg_tile& C, hipStream_t s, LocalStats* st,
                       OutSink* sink, bool sym_only = false);
static inline unsigned nblk(int64_t n, int bs) { return (unsigned)((n + bs - 1) / bs); }

// Device properties and occupancy are cached per (device, kernel, block size,
// LDS bytes): a process may drive several GPUs from several threads (one
// thread per GPU), and one kernel is launched at several LDS sizes.
static std::mutex& occ_mutex() {
  static std::mutex m;
  return m;
}
static int device_cus() {
  static std::map<int, int> cache;
  int dev = 0;
  CBG_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(occ_mutex());
  auto it = cache.find(dev);
  if (it != cache.end()) return it->second;
  int cus = 0;
  CBG_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  cache[dev] = cus;
  return cus;
}
// resident blocks per CU of `kernel` at BS threads and `lds` bytes of LDS (>= 1)
template <class K>
static int blocks_per_cu(K kernel, int bs, size_t lds) {
  static std::map<std::tuple<int, const void*, int, size_t>, int> cache;
  int dev = 0;
  CBG_HIP(hipGetDevice(&dev));
  const auto key = std::make_tuple(dev, (const void*)kernel, bs, lds);
  std::lock_guard<std::mutex> lk(occ_mutex());
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  int n = 0;
  CBG_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, (const void*)kernel, bs, lds));
  n = std::max(n, 1);
  cache[key] = n;
  return n;
}

// CUs the persistent kernels (slab queues) may fill: all of them, less
// comm_reserve_cus() while a broadcast of the SUMMA is in flight on the comm
// stream.  A persistent block never retires before its queue drains, so a grid
// of one block per CU would keep RCCL's broadcast kernels off the GPU until the
// kernel ends; the reserved CUs let them run beside it.
int& comm_reserve_cus() {
  static thread_local int r = 0;
  return r;
}
static int active_cus() { return std::max(1, device_cus() - comm_reserve_cus()); }

template <class K>
static void set_lds(K kernel, size_t bytes) {
  if (bytes > 65536) CBG_HIP(hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
}

// bins of the symbolic phase (key = flops)
//  0: F == 0 | 1: <=32 wave T64 | 2: <=128 wave T256 | 3: <=512 wave T1024 |
//  4: <=1024 block T2048 | 5: <=2048 block T4096 | 6: <=4096 block T8192 | 7: big
// symbolic bins: 1-9 (flops <= 2 ... 512) expand-sort-compress waves of 32 ... 1
// columns (symbolic and numeric in one pass; CBG_SYM_FUSED_LAST = 8 leaves bin 9
// to the wave hash), 10-12 block hash
#ifndef CBG_SYM_FUSED_LAST
#define CBG_SYM_FUSED_LAST 9
#endif
static const int64_t kSymThr[] = {0, 2, 4, 8, 16, 32, 64, 128, 256, 512, 1024, 2048, 4096};
constexpr int SYM_FUSED_LAST = CBG_SYM_FUSED_LAST;
// columns with more flops than this take the bitmap+rank slab path (runtime
// override: CBG_BIG_FLOPS); it must stay <= 4096 so that every other column's
// nnz fits the largest numeric hash bin
static int64_t big_flops(int64_t m) {
  static const char* e = getenv("CBG_BIG_FLOPS");
  // measured on R-MAT (scale 18/20): 4096 once hash slabs take the sparse
  // (column, panel) pairs and the block hash bins emit by bucket sort
  int64_t b = e ? atoll(e) : 4096;
  if (b < 64) b = 64;
  if (b > 4096) b = 4096;
  return b;
}
// bins of the numeric phase (key = exact nnz, big columns forced to the last bin)
//  0: 0 | 1: <=32 wave T64 | 2: <=64 wave T128 | 3: <=128 wave T256 | 4: <=256 wave T512 |
//  5: <=512 block T1024 | 6: <=1024 block T2048 | 7: <=2048 block T4096 | 8: <=4096 block T8192 | 9: big
static const int64_t kNumThr[] = {0, 32, 64, 128, 256, 512, 1024, 2048, 4096};

template <int LOGT>
static void launch_sym_wave(const int32_t* perm, int n, const cbg_tile& B, const int2* cmap, const cbg_tile& A,
                            int32_t* cnt, hipStream_t s) {
  if (n <= 0) return;
  const size_t lds = 4 * SymWaveLds<LOGT>::INTS * sizeof(int);
  set_lds(k_sym_wave<LOGT>, lds);
  hipLaunchKernelGGL(k_sym_wave<LOGT>, dim3(nblk(n, 4)), dim3(256), lds, s, perm, n, B.cp, B.ir, cmap, A.ir, cnt);
}
// expand-sort-compress bin b (flops <= fmax = 64 >> (b - 1)... as CPW = 64 / fmax
// columns per wave; one column per wave when A's rows leave no room for the
// column bits of the sort key)
// (2 products per lane for the bins of <= 64 flops, twice the columns per
// wave: GalerkinNew 7.33 vs 7.26 ms; 16 per lane for the 513-1024-flop bin
// instead of its block hash passes: 148 VGPRs, 3 waves per SIMD, 8.47 vs
// 6.28 ms and 463 vs 447 ms at scale 22 -- neither kept)
template <int CPW, int NPL, int SR>
static void launch_esc1(const int32_t* perm, int n, int fmax, const cbg_tile& B, const int2* cmap,
                        const int4* ainl, const cbg_tile& A, int32_t* cnt, int32_t* tir, double* tval, int64_t base,
                        int64_t* tslot, hipStream_t s) {
  const dim3 g(nblk((n + CPW - 1) / CPW, 4));
  if (ainl)
    hipLaunchKernelGGL((k_esc_wave<CPW, NPL, SR, true>), g, dim3(256), 0, s, perm, n, fmax, B.cp, B.ir, B.val, cmap,
                       ainl, A.ir, A.val, cnt, tir + base, tval + base, base, tslot);
  else
    hipLaunchKernelGGL((k_esc_wave<CPW, NPL, SR, false>), g, dim3(256), 0, s, perm, n, fmax, B.cp, B.ir, B.val, cmap,
                       ainl, A.ir, A.val, cnt, tir + base, tval + base, base, tslot);
}
// expand-sort-compress bin of flops <= fmax: CPW = 64 * NPL / fmax columns per
// wave (one column per wave when A's rows leave no room for the column bits of
// the sort key); fmax 128 / 256 / 512 sort 2 / 4 / 8 products per lane
template <int SR>
static void launch_esc(const int32_t* perm, int n, int fmax, const cbg_tile& B, const int2* cmap, const int4* ainl,
                       const cbg_tile& A, int32_t* cnt, int32_t* tir, double* tval, int64_t base, int64_t* tslot,
                       hipStream_t s) {
  if (n <= 0) return;
#define CBG_ESC_ARGS perm, n, fmax, B, cmap, ainl, A, cnt, tir, tval, base, tslot, s
  if (fmax > 4 * WAVE) return launch_esc1<1, 8, SR>(CBG_ESC_ARGS);
  if (fmax > 2 * WAVE) return launch_esc1<1, 4, SR>(CBG_ESC_ARGS);
  if (fmax > WAVE) return launch_esc1<1, 2, SR>(CBG_ESC_ARGS);
  int cpw = 1;
  while (cpw * fmax * 2 <= WAVE && cpw < 32) cpw <<= 1;  // CPW * fmax <= 64
  int logc = 0;
  while ((1 << logc) < cpw) ++logc;
  if (A.m >= (1LL << (31 - logc))) cpw = 1;  // key = c << (31 - logc) | row must stay below EMPTY_KEY
  switch (cpw) {
    case 32: launch_esc1<32, 1, SR>(CBG_ESC_ARGS); break;
    case 16: launch_esc1<16, 1, SR>(CBG_ESC_ARGS); break;
    case 8: launch_esc1<8, 1, SR>(CBG_ESC_ARGS); break;
    case 4: launch_esc1<4, 1, SR>(CBG_ESC_ARGS); break;
    case 2: launch_esc1<2, 1, SR>(CBG_ESC_ARGS); break;
    default: launch_esc1<1, 1, SR>(CBG_ESC_ARGS); break;
  }
#undef CBG_ESC_ARGS
}
template <int LOGT, int BS>
static void launch_sym_block(const int32_t* perm, int n, const cbg_tile& B, const int2* cmap, const int4* ainl,
                             const cbg_tile& A, int32_t* cnt, hipStream_t s) {
  if (n <= 0) return;
  const size_t lds = SymBlockLds<LOGT, BS>::INTS * sizeof(int);
  if (ainl) {
    set_lds(k_sym_block<LOGT, BS, true>, lds);
    hipLaunchKernelGGL((k_sym_block<LOGT, BS, true>), dim3(n), dim3(BS), lds, s, perm, B.cp, B.ir, cmap, ainl, A.ir,
                       cnt);
  } else {
    set_lds(k_sym_block<LOGT, BS, false>, lds);
    hipLaunchKernelGGL((k_sym_block<LOGT, BS, false>), dim3(n), dim3(BS), lds, s, perm, B.cp, B.ir, cmap, ainl, A.ir,
                       cnt);
  }
}
template <int LOGT, int SR>
static void launch_num_wave(const int32_t* perm, int n, const cbg_tile& B, const int2* cmap, const cbg_tile& A,
                            const int64_t* colptr, cbg_tile& C, hipStream_t s) {
  if (n <= 0) return;
  const size_t lds = 4 * NumWaveLds<LOGT>::BYTES;
  set_lds(k_num_wave<LOGT, SR>, lds);
  hipLaunchKernelGGL((k_num_wave<LOGT, SR>), dim3(nblk(n, 4)), dim3(256), lds, s, perm, n, B.cp, B.ir, B.val, cmap,
                     A.ir, A.val, colptr, C.ir, C.val);
}

// records of the block hash bins: a column is a hash slab over all rows
__global__ void k_col_records(const int32_t* __restrict__ perm, int n, const int64_t* __restrict__ cpB,
                              const int64_t* __restrict__ colptr, int m, SlabRec* __restrict__ rec) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int col = perm[i];
  SlabRec r;
  r.obase = colptr[col];
  r.p0 = cpB[col];
  r.nb = (int)(cpB[col + 1] - r.p0);
  r.r = 0;
  r.lo = 0;
  r.hi = m;  // the rows the slab spans
  r.nout = (int)(colptr[col + 1] - r.obase);
  r.slot = -1;
  r.flags = 3 | SLAB_FULL;
  r.coff = -1;
  rec[i] = r;
}

template <int LOGT, int BS, int SR>
static void launch_num_block_hash(const int32_t* perm, int n, const cbg_tile& B, const int2* cmap,
                                  const int4* ainl, const cbg_tile& A, const float* valAf, const int64_t* colptr,
                                  cbg_tile& C, hipStream_t s, DeferredFree& df) {
  if (n <= 0) return;
  DBuf<SlabRec> rec(n);
  hipLaunchKernelGGL(k_col_records, dim3(nblk(n, 256)), dim3(256), 0, s, perm, n, B.cp, colptr, (int)A.m, rec.p);
  constexpr int L = SlabHashLds<1 << LOGT, BS>::BYTES;
  int lm = 0;
  while ((1LL << lm) < A.m) ++lm;  // emit buckets span [0, 2^lm)
  DBuf<int> queue(1);
  CBG_HIP(hipMemsetAsync(queue.p, 0, sizeof(int), s));
  auto go = [&](auto k, const auto* valA) {
    set_lds(k, L);
    const int per_cu = blocks_per_cu(k, BS, L);
    // (a quarter / a 16th of the resident blocks, leaving the big-column slabs on
    // the main stream more CUs: 424 / 537 vs 418.5 ms at scale 22)
    const int grid = (int)std::min<int64_t>(n, (int64_t)per_cu * active_cus());
    hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(BS), L, s, rec.p, n, queue.p, lm, B.ir, B.val, PMap{cmap, 0, 1},
                       A.ir, valA, C.ir, C.val, ainl);
  };
  // A's f32 values (exact, see k_vals_f32) when the big-column path made them;
  // A's columns as inline records when the small-column passes have them
  if (ainl) go(k_num_slab_hash<SR, 1 << LOGT, BS, true, double, true>, A.val);
  else if (valAf) go(k_num_slab_hash<SR, 1 << LOGT, BS, true, float>, valAf);
  else go(k_num_slab_hash<SR, 1 << LOGT, BS, true, double>, A.val);
  df.take(rec);
  df.take(queue);
}

struct BigPlan {
  int nbig = 0, R = 1, plog = 0;
  const int32_t* perm_big = nullptr;
  const int2* cmapP = nullptr;  // panel column maps (cached across phases, or cmapP_own)
  DBuf<int2> cmapP_own;
  bool kmajor = false;  // cmapP column-major (PMap)
  int64_t n1 = 0;       // A's columns + 1
  PMap pm() const { return kmajor ? PMap{cmapP, 1, R} : PMap{cmapP, n1, 1}; }
  DBuf<int4> desc;
  DBuf<int32_t> nslab, cnt_br;
  DBuf<unsigned> gbm;       // kept symbolic bitmaps, slots of 2^(plog-5) words
  DBuf<int> gbm_slot;        // slot of a (column, panel) pair, -1 = none
  const float* valAf = nullptr;  // A's values as f32 when that is exact (slab kernels read 4 B, not 8)
  const PackedRV* valAp = nullptr;  // ... and as (row, f32) records
  const PackedRVD* valAd = nullptr;  // A's (row, f64) records when its values are not f32-exact
  DBuf<int> cuts, pcoff;  // multi-slab pairs' cut positions (sym_pair), per-pair offsets
  const int* gbm_next = nullptr;  // kept-bitmap slots handed out (device), of gbm_slots
  int64_t gbm_slots = 0;
  bool all_kept = false;  // no bitmap-mode pair went without a slot (read with sync 3)
  bool iacc = false;      // exact int32 accumulation (k_int_bound; read with sync 2)
};


template <int SR, int T, int BS>
static void launch_slab_hash(const SlabRec* list, int n, const BigPlan& bp, const cbg_tile& A,
                             const cbg_tile& B, cbg_tile& C, hipStream_t s, DeferredFree& df) {
  if (n <= 0) return;
  constexpr int L = SlabHashLds<T, BS>::BYTES;
  DBuf<int> queue(1);
  CBG_HIP(hipMemsetAsync(queue.p, 0, sizeof(int), s));
  auto go = [&](auto k, const auto* valA) {
    set_lds(k, L);
    const int per_cu = blocks_per_cu(k, BS, L);
    const int grid = (int)std::min<int64_t>(n, (int64_t)per_cu * active_cus());
    hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(BS), L, s, list, n, queue.p, bp.plog, B.ir, B.val, bp.pm(),
                       A.ir, valA, C.ir, C.val, (const int4*)nullptr);
  };
  // (A's exact f32 values come as (row, f32) records whenever they exist; f64
  // values as (row, f64) records when they were worth packing, see k_pack_rvd)
  if (bp.valAp) go(k_num_slab_hash<SR, T, BS, false, PackedRV>, bp.valAp);
  else if (bp.valAd) go(k_num_slab_hash<SR, T, BS, false, PackedRVD>, bp.valAd);
  else go(k_num_slab_hash<SR, T, BS, false, double>, A.val);
  df.take(queue);
}

template <int SR, int CAP, int BS>
static void launch_slab_bitmap(const SlabRec* list, int n, const BigPlan& bp, const cbg_tile& A,
                               const cbg_tile& B, cbg_tile& C, hipStream_t s, DeferredFree& df) {
  if (n <= 0) return;
  constexpr int L = SlabLds<CAP, BS>::BYTES;
  DBuf<int> queue(1);
  CBG_HIP(hipMemsetAsync(queue.p, 0, sizeof(int), s));
  auto go = [&](auto k, const auto* valA) {
    set_lds(k, L);
    const int per_cu = blocks_per_cu(k, BS, L);
    const int grid = (int)std::min<int64_t>(n, (int64_t)per_cu * active_cus());
    hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(BS), L, s, list, n, queue.p, bp.plog, B.ir, B.val, bp.pm(),
                       A.ir, valA, C.ir, C.val, bp.gbm.p, bp.cuts.p);
  };
  // (IACC only with the packed records: integers of magnitude <= 2^24 are f32-exact)
  if (bp.all_kept) {
    if (bp.iacc) go(k_num_slab<SR, CAP, BS, PackedRV, true, true>, bp.valAp);
    else if (bp.valAp) go(k_num_slab<SR, CAP, BS, PackedRV, true, false>, bp.valAp);
    else if (bp.valAd) go(k_num_slab<SR, CAP, BS, PackedRVD, true, false>, bp.valAd);
    else go(k_num_slab<SR, CAP, BS, double, true, false>, A.val);
  } else {
    if (bp.iacc) go(k_num_slab<SR, CAP, BS, PackedRV, false, true>, bp.valAp);
    else if (bp.valAp) go(k_num_slab<SR, CAP, BS, PackedRV, false, false>, bp.valAp);
    else if (bp.valAd) go(k_num_slab<SR, CAP, BS, PackedRVD, false, false>, bp.valAd);
    else go(k_num_slab<SR, CAP, BS, double, false, false>, A.val);
  }
  df.take(queue);
}

template <int SR, int NCAP>
static void launch_slab_rank(const SlabRec* list, int n, const BigPlan& bp, const cbg_tile& A,
                             const cbg_tile& B, cbg_tile& C, hipStream_t s, DeferredFree& df) {
  if (n <= 0) return;
  DBuf<int> queue(1);
  CBG_HIP(hipMemsetAsync(queue.p, 0, sizeof(int), s));
  auto go = [&](auto k, const auto* valA) {
    const int L = bp.iacc ? SlabRankLds<NCAP, RANK_BS, 4>::BYTES : SlabRankLds<NCAP, RANK_BS, 8>::BYTES;
    set_lds(k, L);
    const int per_cu = blocks_per_cu(k, RANK_BS, L);
    const int grid = (int)std::min<int64_t>(n, (int64_t)per_cu * active_cus());
    hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(RANK_BS), L, s, list, n, queue.p, B.ir, B.val, bp.pm(),
                       A.ir, valA, C.ir, C.val);
  };
  if (bp.iacc) go(k_num_slab_rank<SR, NCAP, RANK_BS, PackedRV, true>, bp.valAp);
  else if (bp.valAp) go(k_num_slab_rank<SR, NCAP, RANK_BS, PackedRV, false>, bp.valAp);
  else if (bp.valAd) go(k_num_slab_rank<SR, NCAP, RANK_BS, PackedRVD, false>, bp.valAd);
  else go(k_num_slab_rank<SR, NCAP, RANK_BS, double, false>, A.val);
  df.take(queue);
}

// hash-mode single-panel slabs of more than this many nonzeros run as rank
// slabs (scale 24: 400 / 1000 measured 3789 / 3825 vs 3795 ms; scale 22 flat)
constexpr int RANK_SLABS_MIN = 683;
// panel-group slabs of more than this many nonzeros run as group rank slabs
constexpr int GRANK_SLABS_MIN = 683;

template <int SR, int NCAP, int SPANLOG = GRANK_SPAN_LOG, int PMAX = GRANK_PMAX>
static void launch_slab_grank(const SlabRec* list, int n, const BigPlan& bp, const cbg_tile& A,
                              const cbg_tile& B, cbg_tile& C, hipStream_t s, DeferredFree& df) {
  if (n <= 0) return;
  DBuf<int> queue(1);
  CBG_HIP(hipMemsetAsync(queue.p, 0, sizeof(int), s));
  auto go = [&](auto k, const auto* valA) {
    const int L = bp.iacc ? SlabGRankLds<NCAP, RANK_BS, SPANLOG, PMAX, 4>::BYTES
                          : SlabGRankLds<NCAP, RANK_BS, SPANLOG, PMAX, 8>::BYTES;
    set_lds(k, L);
    const int per_cu = blocks_per_cu(k, RANK_BS, L);
    const int grid = (int)std::min<int64_t>(n, (int64_t)per_cu * active_cus());
    hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(RANK_BS), L, s, list, n, queue.p, bp.plog, B.ir, B.val, bp.pm(),
                       A.ir, valA, C.ir, C.val);
  };
  if (bp.iacc) go(k_num_slab_grank<SR, NCAP, RANK_BS, SPANLOG, PMAX, PackedRV, true>, bp.valAp);
  else if (bp.valAp) go(k_num_slab_grank<SR, NCAP, RANK_BS, SPANLOG, PMAX, PackedRV, false>, bp.valAp);
  else if (bp.valAd) go(k_num_slab_grank<SR, NCAP, RANK_BS, SPANLOG, PMAX, PackedRVD, false>, bp.valAd);
  else go(k_num_slab_grank<SR, NCAP, RANK_BS, SPANLOG, PMAX, double, false>, A.val);
  df.take(queue);
}

// ncls[c] slabs of class c, stored consecutively in `list` (k_slab_fill)

template <int SR>
static void launch_slabs(const SlabRec* list, const int* ncls, const BigPlan& bp, const cbg_tile& A,
                         const cbg_tile& B, cbg_tile& C, hipStream_t s, hipStream_t side, DeferredFree& df) {
  const SlabRec* at[SLAB_NCLS];
  int64_t o = 0;
  for (int c = 0; c < SLAB_NCLS; ++c) {
    at[c] = list + o;
    o += ncls[c];
  }
  // (hash classes queued behind the small-column bins on the side stream were
  // 3-4 % slower at scale 22: every slab class runs on the main stream)
  auto hs = [&](int) { return s; };
  launch_slab_bitmap<SR, SLAB_SMALL_CAP, SLAB_SMALL_BS>(at[0], ncls[0], bp, A, B, C, s, df);
  launch_slab_bitmap<SR, SLAB_LARGE_CAP, SLAB_LARGE_BS>(at[1], ncls[1], bp, A, B, C, s, df);
  static_assert(SLAB_HASH_NCLS == 9, "hash slab classes (CBG_HASH_TABLES)");
  launch_slab_hash<SR, 512, 256>(at[2], ncls[2], bp, A, B, C, hs(0), df);
  launch_slab_hash<SR, 768, 256>(at[3], ncls[3], bp, A, B, C, hs(1), df);
  launch_slab_hash<SR, 1024, 256>(at[4], ncls[4], bp, A, B, C, hs(2), df);
  launch_slab_hash<SR, 1536, 256>(at[5], ncls[5], bp, A, B, C, hs(3), df);
  launch_slab_hash<SR, 2048, 256>(at[6], ncls[6], bp, A, B, C, hs(4), df);
  launch_slab_hash<SR, 3072, 512>(at[7], ncls[7], bp, A, B, C, hs(5), df);
  launch_slab_hash<SR, 4096, 512>(at[8], ncls[8], bp, A, B, C, hs(6), df);
  launch_slab_hash<SR, 6144, 512>(at[9], ncls[9], bp, A, B, C, hs(7), df);
  launch_slab_hash<SR, 8192, 512>(at[10], ncls[10], bp, A, B, C, hs(8), df);
  // (class order: rank and group rank slabs first, or between the two bitmap
  // classes: 347.5 / 346.2 vs 343.5 ms at scale 22)
  // (the single-panel rank slabs by the two-level rank of the group slabs, 1
  // KiB of level 1 for 2^18 rows and 2-3x the blocks per CU: 352.1 vs 344.0 ms
  // at scale 22 -- the second lookup costs more than the occupancy buys)
  launch_slab_rank<SR, 4096>(at[SLAB_RANK0 + 2], ncls[SLAB_RANK0 + 2], bp, A, B, C, s, df);
  launch_slab_rank<SR, 2048>(at[SLAB_RANK0 + 1], ncls[SLAB_RANK0 + 1], bp, A, B, C, s, df);
  launch_slab_rank<SR, 1024>(at[SLAB_RANK0], ncls[SLAB_RANK0], bp, A, B, C, s, df);
  launch_slab_grank<SR, 4096>(at[SLAB_GRANK0 + 1], ncls[SLAB_GRANK0 + 1], bp, A, B, C, s, df);
  launch_slab_grank<SR, 2048>(at[SLAB_GRANK0], ncls[SLAB_GRANK0], bp, A, B, C, s, df);

}


// kept symbolic bitmaps (32 KiB per (column, panel) pair): CBG_BITMAP_BUDGET_GB,
// default 48 GB (scale 22 on one GPU: 16 GB -> 32 GB was +3.7 %), never more
// than a quarter of the device memory still available (free + pool cache), so
// that C, allocated after the symbolic phase, keeps room
static double bitmap_budget_bytes() {
  static const char* e = getenv("CBG_BITMAP_BUDGET_GB");
  const double want = (e ? atof(e) : 48.0) * 1e9;
  size_t fr = 0, tot = 0;
  if (hipMemGetInfo(&fr, &tot) != hipSuccess) {
    (void)hipGetLastError();
    return std::min(want, 16e9);
  }
  return std::min(want, 0.25 * (double)(fr + pool().bytes_cached()));
}

struct Binned {
  std::vector<int> count, offset;
  std::vector<unsigned long long> flops;  // per bin
  DBuf<int32_t> perm;
};

// Binning in two halves so that the histogram's trip to the host rides on a
// synchronization the caller makes anyway: bin_classify launches k_classify
// and an async copy of the histogram; after the caller's next stream sync,
// bin_scatter turns it into offsets and launches the scatter.
// Small device -> host readbacks go through pinned staging (a copy into
// pageable memory is staged by the runtime and holds the host thread once per
// copy: ~20 us each, several per multiply): slot k of the calling thread's
// page, read after the caller's next synchronization.
// Rule: at most ONE local multiply per host thread has readbacks in flight at a
// time -- the slots are fixed per thread and each is read right after the
// synchronization that follows its copy (every caller runs its multiply to
// completion on the thread, through its 4 host syncs, before the next one
// starts).  An asynchronous or nested multiply on one thread would need a page
// of its own.  The page lives for the thread (8 x 4 KiB pinned).
static char* host_stage(int slot) {
  static thread_local char* p = nullptr;
  if (!p) CBG_HIP(hipHostMalloc((void**)&p, 8 * 4096, hipHostMallocDefault));
  return p + (size_t)slot * 4096;
}
enum { STAGE_BINS_SYM = 0, STAGE_BINS_NUM = 1, STAGE_SCALARS = 2, STAGE_SLABS = 3, STAGE_AF = 4 };
struct BinPending {
  BinThr bt;
  DBuf<uint8_t> bin;
  DBuf<int> hist;
  char* host = nullptr;  // pinned copy of hist (after the caller's sync: read())
  std::vector<int> h;
  std::vector<unsigned long long> hf;  // flops per bin
  unsigned long long big_entries[2] = {0, 0};  // B entries of the big / thin columns
  void read() {
    const int* hi = reinterpret_cast<const int*>(host);
    h.assign(hi, hi + MAXBINS);
    const unsigned long long* be = reinterpret_cast<const unsigned long long*>(hi + 2 * MAXBINS);
    big_entries[0] = be[0];
    big_entries[1] = be[1];
    const unsigned long long* bf = reinterpret_cast<const unsigned long long*>(hi + 2 * MAXBINS + 4);
    hf.assign(bf, bf + MAXBINS);
  }
};
// cpB/big_bin (mode 0): also count the B entries of the bins >= big_bin into bp.big_entries
static void bin_classify(int64_t n, const int64_t* flops, int32_t* cnt, int mode, const int64_t* thr,
                         int nthr, int64_t big, BinPending& bp, hipStream_t s, int64_t fused_max = 0,
                         const int64_t* cpB = nullptr, int big_bin = MAXBINS, int thin_R = 0, int thin_bin = 0,
                         int copy1 = 0) {
  bp.bt.nb = nthr + 1;
  for (int i = 0; i < nthr; ++i) bp.bt.t[i] = thr[i];
  bp.bin.reset(n);
  // counts | offsets | big, thin entries (u64) | flops per bin (u64)
  bp.hist.reset(2 * MAXBINS + 4 + 2 * MAXBINS);
  CBG_HIP(hipMemsetAsync(bp.hist.p, 0, sizeof(int) * (4 * MAXBINS + 4), s));
  unsigned long long* be = (cpB && mode == 0) ? reinterpret_cast<unsigned long long*>(bp.hist.p + 2 * MAXBINS) : nullptr;
  unsigned long long* bf = reinterpret_cast<unsigned long long*>(bp.hist.p + 2 * MAXBINS + 4);
  hipLaunchKernelGGL(k_classify, dim3(nblk(n, 256 * BIN_ITEMS)), dim3(256), 0, s, n, flops, cnt, mode, copy1, big, bp.bt,
                     bp.bin.p, bp.hist.p, fused_max, cpB, big_bin, be, bf, thin_R, thin_bin);
  // one copy of counts | offsets | big entries | flops per bin
  bp.host = host_stage(mode == 0 ? STAGE_BINS_SYM : STAGE_BINS_NUM);
  CBG_HIP(hipMemcpyAsync(bp.host, bp.hist.p, sizeof(int) * (4 * MAXBINS + 4), hipMemcpyDeviceToHost, s));
}
static void bin_scatter(int64_t n, BinPending& bp, Binned& out, hipStream_t s, DeferredFree& df) {
  const int nb = bp.bt.nb;
  if (bp.h.empty()) bp.read();
  out.count.assign(nb, 0);
  out.offset.assign(nb + 1, 0);
  for (int b = 0; b < nb; ++b) {
    out.count[b] = bp.h[b];
    out.offset[b + 1] = out.offset[b] + bp.h[b];
  }
  out.flops = bp.hf;
  out.perm.reset(n);
  hipLaunchKernelGGL(k_bin_scatter, dim3(nblk(n, 256 * BIN_ITEMS)), dim3(256), 0, s, n, bp.bin.p, nb, bp.hist.p,
                     bp.hist.p + MAXBINS, out.perm.p);
  df.take(bp.bin);  // released after the multiply's final synchronization
  df.take(bp.hist);
}

// bytes the thin columns' expand-sort-reduce holds per product at most: two
// (key, value) buffers of the radix sort, the unique keys and values, the run
// flags and positions (64-bit keys)
constexpr double THIN_BYTES_PER_PRODUCT = 2 * 16 + 16 + 4 + 8;
static double device_bytes_available() {
  size_t fr = 0, tot = 0;
  if (hipMemGetInfo(&fr, &tot) != hipSuccess) {
    (void)hipGetLastError();
    return 0.0;
  }
  return (double)fr + (double)pool().bytes_cached();
}

static int pick_panel_log(int64_t m) {
  int l = FINE_LOG;
  while ((1LL << l) < m && l < PANEL_LOG_MAX) ++l;
  return l;
}


template <int SR>
static void numeric_dispatch(const Binned& nb, const cbg_tile& A, const float* valAf, const cbg_tile& B,
                             const int2* cmap, const int4* ainl, const int64_t* colptr, cbg_tile& C, const hipStream_t* sb,
                             DeferredFree& df) {
  const int32_t* P = nb.perm.p;
  auto at = [&](int b) { return P + nb.offset[b]; };
  launch_num_wave<6, SR>(at(1), nb.count[1], B, cmap, A, colptr, C, sb[1]);
  launch_num_wave<7, SR>(at(2), nb.count[2], B, cmap, A, colptr, C, sb[2]);
  launch_num_wave<8, SR>(at(3), nb.count[3], B, cmap, A, colptr, C, sb[3]);
  launch_num_wave<9, SR>(at(4), nb.count[4], B, cmap, A, colptr, C, sb[4]);
  launch_num_block_hash<10, 256, SR>(at(5), nb.count[5], B, cmap, ainl, A, valAf, colptr, C, sb[5], df);
  launch_num_block_hash<11, 256, SR>(at(6), nb.count[6], B, cmap, ainl, A, valAf, colptr, C, sb[6], df);
  launch_num_block_hash<12, 512, SR>(at(7), nb.count[7], B, cmap, ainl, A, valAf, colptr, C, sb[7], df);
  launch_num_block_hash<13, 1024, SR>(at(8), nb.count[8], B, cmap, ainl, A, valAf, colptr, C, sb[8], df);
}

// Stream of each small-column bin: the big columns run on the main stream,
// the small bins on the side stream concurrently -- unless the big columns
// carry less work than the small ones (GalerkinNew: 6 % of the flops), when
// bins from the largest down go to whichever stream has less work so far, so
// that both finish together.  Work = flops x the bin's relative cost.
// (bal = false: every bin to the side stream)
static void balance_bins(const std::vector<unsigned long long>& fl, int first, int last, double main_work,
                         double side_work, const double* cost, hipStream_t main, hipStream_t side,
                         hipStream_t* out, bool bal = false) {
  for (int b = last; b >= first; --b) {
    const double w = (double)fl[b] * (cost ? cost[b] : 1.0);
    if (!bal || side == main || side_work <= main_work) {
      out[b] = side;
      side_work += w;
    } else {
      out[b] = main;
      main_work += w;
    }
  }
}

struct APrep {
  bool active = false;
  const void* ir = nullptr;
  const void* cp = nullptr;
  uint64_t ser_ir = 0, ser_cp = 0;  // pool allocation serials of ir / cp (0: not pool memory)
  int64_t nnz = -1, nzc = -1, m = -1, n = -1;
  DBuf<int2> cmap, cmapP;  // cmapP: built by the first call that had big columns
  DBuf<unsigned char> clen8;  // A's column lengths clamped at 255
  int plog = -1;
  bool kmajor = false;  // cmapP's layout
  DBuf<float> valf;  // A's values as f32 (af == 1)
  int ai = -1, amax = 0;  // A's values all integers of magnitude <= 2^24 (k_int_bound; -1: not checked), max |a|
  DBuf<PackedRV> valp;  // (row, f32) records (af == 1)
  DBuf<PackedRVD> valpd;  // (row, f64) records (af == 0)
  int af = -1;       // -1 not checked yet, 0 some value is not an exact f32, 1 valf holds A's values
};

// A's values narrowed to f32, and whether every one survives the round trip
// exactly (NaN and values outside f32's range or precision do not).  When they
// all do, the slab kernels read 4 B per product instead of 8 and widen them:
// the products and sums are the f64 ones, bit for bit.
// (stops early once some value is inexact: the copy is then not used --
// GalerkinNew's A = L + D carries random diagonal values, and each of its
// products checked all 68 M values for nothing: 0.21 ms)
// pk (optional): A's (row, f32 value) records, one 8-byte gather per numeric product
__global__ void k_vals_f32(int64_t n, const double* __restrict__ v, float* __restrict__ f, int* __restrict__ inexact,
                           const int32_t* __restrict__ ir, PackedRV* __restrict__ pk) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  while (i < n) {
    if (*reinterpret_cast<volatile int*>(inexact)) return;
    bool bad = false;
#pragma unroll
    for (int u = 0; u < 8; ++u, i += stride) {
      if (i < n) {
        const double x = v[i];
        const float y = (float)x;
        f[i] = y;
        if (pk) pk[i] = PackedRV{ir[i], y};
        bad |= !((double)y == x);
      }
    }
    // one store per wave, and none once the flag is up: a million threads
    // storing to one address serialized at L2 (0.3 ms)
    const unsigned long long any = __ballot(bad);
    if (any) {
      if (lane_id() == __ffsll((long long)any) - 1 && !*reinterpret_cast<volatile int*>(inexact))
        *reinterpret_cast<volatile int*>(inexact) = 1;
      return;
    }
  }
}
// Exact integer accumulation (IACC): when every value of A and B is an integer
// of magnitude <= 2^24 (not -0.0) and every sum the slabs form is bounded below
// 2^31 -- plus-times: max|A| max_j sum_k |B(k,j)| bounds |sum_k a_ik b_kj|;
// min-plus: max|A| + max|B| -- the slab kernels accumulate in int32 LDS
// atomics and store the sums as f64: every partial sum is an integer the f64
// path also holds exactly, so C is the same, bit for bit, in any order.
// k_int_bound: out[0] |= 1 if some value is not such an integer, out[1] =
// max |value|; k_col_int_bound (a wave per column): the same and out[2] = the
// largest column sum of |values| (capped at INT32_MAX).  (R-MAT scale 22: max
// value 225, max column length 50,401, max column |sum| 79,824: the column-sum
// bound is 1.8e7, the length bound 2.6e9 would fail.)
__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
  for (int d = WAVE / 2; d > 0; d >>= 1) v = max(v, __shfl_xor(v, d, WAVE));
  return v;
}
// the block's (flag, max, max) to out[0..2]: one set of atomics per block
// (a wave each on three words serialized 2 M waves: 25 ms per scale-22 phase)
__device__ __forceinline__ void block_int_bound_out(int bad, int mx, int cs, int* __restrict__ out) {
  __shared__ int r[3];
  if (threadIdx.x == 0) r[0] = r[1] = r[2] = 0;
  __syncthreads();
  const unsigned long long any = __ballot(bad);
  mx = wave_max_i(mx);
  cs = wave_max_i(cs);
  if (lane_id() == 0) {
    if (any) atomicOr(&r[0], 1);
    atomicMax(&r[1], mx);
    atomicMax(&r[2], cs);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (r[0]) atomicOr(&out[0], 1);
    if (r[1]) atomicMax(&out[1], r[1]);
    if (r[2]) atomicMax(&out[2], r[2]);
  }
}
__device__ __forceinline__ bool int_value_bad(double x) {
  const double ax = fabs(x);
  return !(ax <= 16777216.0) || x != trunc(x) || (x == 0.0 && signbit(x));
}
// fail fast: a wave that sees a bad value raises out[0] at once (one store per
// wave), and every wave stops at its next check once it is up; k_int_bound
// does nothing when k_vals_f32 (before it on the stream) found A not
// f32-exact (skip[0]), k_col_int_bound nothing when A is not integral (skip:
// A's flags, in this call; the host skips the launch for a cached verdict)
// (GalerkinNew scale 22, f64 values: the two checks read 0.47 ms for nothing)
__device__ __forceinline__ bool int_bound_raise(int bad, int* __restrict__ out) {
  const unsigned long long any = __ballot(bad);
  if (any && lane_id() == __ffsll((long long)any) - 1 && !*reinterpret_cast<volatile int*>(out))
    *reinterpret_cast<volatile int*>(out) = 1;
  return any || *reinterpret_cast<volatile int*>(out);
}
__global__ __launch_bounds__(256) void k_int_bound(int64_t n, const double* __restrict__ v, int* __restrict__ out,
                                                   const int* __restrict__ skip) {
  if (*skip) return;  // (uniform: written by an earlier kernel)
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int bad = 0, mx = 0;
  for (int64_t i0 = blockIdx.x * (int64_t)blockDim.x; i0 < n; i0 += stride) {
    const int64_t i = i0 + threadIdx.x;
    if (i < n) {
      const double x = v[i];
      if (int_value_bad(x)) bad = 1;
      else mx = max(mx, (int)fabs(x));
    }
    if (int_bound_raise(bad, out)) break;
  }
  block_int_bound_out(bad, mx, 0, out);
}
// a wave per column, grid-stride over the columns
__global__ __launch_bounds__(256) void k_col_int_bound(int64_t nzc, const int64_t* __restrict__ cp,
                                                       const double* __restrict__ v, int* __restrict__ out,
                                                       const int* __restrict__ skip) {
  if (skip && (skip[0] | skip[1])) return;
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x / WAVE);
  int bad = 0, mx = 0, cs = 0;
  for (int64_t c = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / WAVE; c < nzc; c += nw) {
    double sum = 0.0;  // integers: exact below 2^53
    for (int64_t q = cp[c] + lane_id(); q < cp[c + 1]; q += WAVE) {
      const double x = v[q];
      if (int_value_bad(x)) bad = 1;
      else mx = max(mx, (int)fabs(x));
      sum += fabs(x);
    }
#pragma unroll
    for (int d = WAVE / 2; d > 0; d >>= 1) sum += __shfl_xor(sum, d, WAVE);
    cs = max(cs, sum < 2147483647.0 ? (int)sum : INT32_MAX);
    if (int_bound_raise(bad, out)) break;
  }
  block_int_bound_out(bad, mx, cs, out);
}
static bool iacc_bound_ok(int semiring, int amax, int bmax, int bcolsum) {
  if (semiring == CBG_MIN_PLUS) return (int64_t)amax + bmax < (1LL << 30);
  return (double)amax * (double)bcolsum < 2147483648.0;
}

// A's (row, f64) records for the f64-valued slab path
__global__ void k_pack_rvd(int64_t n, const int32_t* __restrict__ ir, const double* __restrict__ v,
                           PackedRVD* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const long long b = __double_as_longlong(v[i]);
    out[i] = PackedRVD{ir[i], (int)b, (int)(b >> 32)};
  }
}

// flops[0, nz) per B column and their total in flops[nz] (B.nnz > 0)
static void launch_flops(const cbg_tile& B, const int2* cmap, const unsigned char* clen8, bool A_one_per_col,
                         int64_t* flops, hipStream_t s, DeferredFree& df) {
  const int64_t nz = B.nzc;
  if (A_one_per_col) {
    // every A column holds exactly one entry (a restriction operator's
    // transpose, GalerkinNew's S): flops(j) = nnz(B(:, j)), no gathers
    hipLaunchKernelGGL(k_flops_unit, dim3(nblk(nz, 256)), dim3(256), 0, s, nz, B.cp, flops);
    return;
  }
  const int64_t nb = (B.nnz + FSEG_E - 1) / FSEG_E;
  DBuf<unsigned long long> part(nb);
  DBuf<int64_t> c_lo(nb);
  CBG_HIP(hipMemsetAsync(flops, 0, sizeof(int64_t) * nz, s));
  hipLaunchKernelGGL(k_flops_starts, dim3(nblk(nz, 256)), dim3(256), 0, s, nz, B.cp, c_lo.p);
  hipLaunchKernelGGL(k_flops_seg, dim3((unsigned)nb), dim3(FSEG_T), 0, s, nz, B.nnz, B.cp, B.ir, cmap, clen8, c_lo.p,
                     reinterpret_cast<unsigned long long*>(flops), part.p);
  hipLaunchKernelGGL(k_sum_parts, dim3(1), dim3(1024), 0, s, part.p, nb,
                     reinterpret_cast<unsigned long long*>(flops + nz));
  df.take(part);
  df.take(c_lo);
}

static APrep& aprep() {
  static thread_local APrep a;
  return a;
}
void aprep_begin() { aprep().active = true; }
void aprep_end() {
  APrep& a = aprep();
  a.cmap.release();
  a.clen8.release();
  a.cmapP.release();
  a.valf.release();
  a.valp.release();
  a.valpd.release();
  a.af = -1;
  a.ai = -1;
  a.active = false;
  a.ir = a.cp = nullptr;
  a.ser_ir = a.ser_cp = 0;
  a.nnz = a.nzc = a.m = a.n = -1;
  a.plog = -1;
}

LocalStats& thread_stats() {
  static thread_local LocalStats t;
  return t;
}

void local_spgemm(const cbg_tile& A, const cbg_tile& B, int semiring, cbg_tile& C, hipStream_t s, LocalStats* st,
                  OutSink* sink) {
  LocalStats mine;
  local_spgemm_impl(A, B, semiring, C, s, &mine, sink);
  LocalStats& t = thread_stats();
  t.flops += mine.flops;
  t.nnz += mine.nnz;
  t.n_big += mine.n_big;
  t.n_slabs += mine.n_slabs;
  t.ms_symbolic += mine.ms_symbolic;
  t.ms_numeric += mine.ms_numeric;
  for (int i = 0; i < CBG_WORK_N; ++i) t.work[i] += mine.work[i];
  if (st) *st = mine;
}

// estimateFLOP + estimateNNZ_Hash (mtSpGEMM.h:1056-1134, 805-933) alone: the
// multiply's flops, binning and symbolic kernels (no bitmaps kept), totals read
// back, no C
void local_symbolic(const cbg_tile& A, const cbg_tile& B, hipStream_t s, int64_t* flops, int64_t* nnz) {
  cbg_tile C{};
  LocalStats st;
  local_spgemm_impl(A, B, CBG_PLUS_TIMES, C, s, &st, nullptr, true);
  tile_free_device(C);
  if (flops) *flops = st.flops;
  if (nnz) *nnz = st.nnz;
}

void local_spgemm_impl(const cbg_tile& A, const cbg_tile& B, int semiring, cbg_tile& C, hipStream_t s, LocalStats* st,
                       OutSink* sink, bool sym_only) {
  C = cbg_tile{};
  C.m = A.m;
  C.n = B.n;
  C.on_device = 1;
  if (A.nnz == 0 || B.nnz == 0 || B.nzc == 0 || A.nzc == 0) {  // mtSpGEMM.h:224-227
    tile_alloc_device(C, A.m, B.n, 0, 0);
    if (st) *st = LocalStats{};
    return;
  }
  TileGuard Cg;  // C's arrays until the multiply has completed (exceptions included)
  DeferredFree df;
  // side stream for the small-column bins (independent of the big columns)
  // (and a copy stream for the numeric's direct copies into C)
  static thread_local hipStream_t side = nullptr, scopy = nullptr;
  static thread_local hipEvent_t ev_fork = nullptr, ev_join = nullptr, ev_cjoin = nullptr;
  if (!side) {
    CBG_HIP(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));
    CBG_HIP(hipStreamCreateWithFlags(&scopy, hipStreamNonBlocking));
    CBG_HIP(hipEventCreateWithFlags(&ev_fork, hipEventDisableTiming));
    CBG_HIP(hipEventCreateWithFlags(&ev_join, hipEventDisableTiming));
    CBG_HIP(hipEventCreateWithFlags(&ev_cjoin, hipEventDisableTiming));
  }
  // the small-column bins of the symbolic and the numeric run on the side stream
  // (serialized on the main one: -0.5 % at scale 22, -5 % at 18), the symbolic's
  // on the main one where the big columns dominate (below)
  const hipStream_t ssym = side, snum = side;
  auto fork = [&](hipStream_t main) {
    CBG_HIP(hipEventRecord(ev_fork, main));
    CBG_HIP(hipStreamWaitEvent(side, ev_fork, 0));
  };
  auto join = [&](hipStream_t main) {
    CBG_HIP(hipEventRecord(ev_join, side));
    CBG_HIP(hipStreamWaitEvent(main, ev_join, 0));
  };
  // timing events, created once per thread and reused by every multiply
  static thread_local hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr;
  if (!ev0) {
    CBG_HIP(hipEventCreate(&ev0));
    CBG_HIP(hipEventCreate(&ev1));
    CBG_HIP(hipEventCreate(&ev2));
  }
  CBG_HIP(hipEventRecord(ev0, s));
  const int64_t nz = B.nzc;
  int64_t work[CBG_WORK_N] = {};  // cbg_last_work_stats
  reinterpret_cast<int64_t*>(host_stage(STAGE_SCALARS))[5] = 0;  // deferred group units (sync 2)
  // A column map (reused across the phases of one MemEfficientSpGEMM)
  APrep& ap = aprep();
  const uint64_t ser_ir = ap.active ? pool().serial_of(A.ir) : 0, ser_cp = ap.active ? pool().serial_of(A.cp) : 0;
  const bool a_hit = ap.active && ap.ir == A.ir && ap.cp == A.cp && ap.ser_ir == ser_ir && ap.ser_cp == ser_cp &&
                     ap.nnz == A.nnz && ap.nzc == A.nzc && ap.m == A.m && ap.n == A.n;
  if (ap.active && !a_hit) {
    ap.cmap.release();
    ap.clen8.release();
    ap.cmapP.release();
    ap.valf.release();
    ap.valp.release();
    ap.valpd.release();
    ap.af = -1;
    ap.ai = -1;
    ap.ir = A.ir;
    ap.cp = A.cp;
    ap.ser_ir = ser_ir;
    ap.ser_cp = ser_cp;
    ap.nnz = A.nnz;
    ap.nzc = A.nzc;
    ap.m = A.m;
    ap.n = A.n;
    ap.plog = -1;
  }
  DBuf<int2> cmap_own;
  DBuf<unsigned char> clen8_own;
  DBuf<int2>& cmap = ap.active ? ap.cmap : cmap_own;
  DBuf<unsigned char>& clen8 = ap.active ? ap.clen8 : clen8_own;
  if (!a_hit) {
    cmap.reset(A.n + 1);
    clen8.reset(A.n + 1);
    CBG_HIP(hipMemsetAsync(cmap.p, 0, sizeof(int2) * (A.n + 1), s));
    CBG_HIP(hipMemsetAsync(clen8.p, 0, A.n + 1, s));
    hipLaunchKernelGGL(k_colmap, dim3(nblk(A.nzc, 256)), dim3(256), 0, s, A.nzc, A.cp, A.jc, cmap.p, clen8.p);
  }

  // flops per B column
  DBuf<int64_t> flops(nz + 1);
  launch_flops(B, cmap.p, clen8.p, A.nnz == A.n && A.nzc == A.n, flops.p, s, df);
  DBuf<int32_t> cnt(nz + 1);
  CBG_HIP(hipMemsetAsync(cnt.p, 0, sizeof(int32_t) * (nz + 1), s));
  // symbolic
  Binned sb;
  const int64_t big = big_flops(A.m);
  {
    // once per device (c_dbg exists once per device; a pageable copy holds the host ~20 us)
    static const int dbg = getenv("CBG_DBG") ? atoi(getenv("CBG_DBG")) : 0;
    static std::atomic<unsigned long long> dbg_set{0};
    if (dbg) {
      int dev = 0;
      CBG_HIP(hipGetDevice(&dev));
      const unsigned long long bit = 1ull << (dev & 63);
      if (!(dbg_set.fetch_or(bit) & bit))
        CBG_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(c_dbg), &dbg, sizeof(int), 0, hipMemcpyHostToDevice, s));
    }
  }
  // symbolic bins: kSymThr (clipped at `big`), then the big columns by panel
  // group size 2^GROUP_LOG_MAX .. 1 (columns with F * g / R <= GROUP_PRODUCTS
  // expected products per group; CBG_GROUPS=0 keeps every pair on its own)
  BigPlan bp;
  int64_t big_entries = 0, thin_entries = 0;  // B entries of the big / thin columns (read back with sync 1)
  // small columns' symbolic and numeric in one pass (bins 1..SYM_FUSED_LAST)
  constexpr bool fused = true;
  // single-entry columns as scaled copies of A's columns (CBG_COPY1=0: off)
  // (default 2: also those of more than `big` flops -- R-MAT columns whose one
  // entry hits a hub -- instead of (column, panel) pairs: s22 446.4 -> 440.9 ms;
  // 1: only the small ones)
  constexpr int copy1 = 2;
  bp.plog = pick_panel_log(A.m);
  bp.R = (int)((A.m + (1LL << bp.plog) - 1) >> bp.plog);
  constexpr int NSMALL = 13, NGCLS = GROUP_LOG_MAX + 1, THIN_BIN = NSMALL + NGCLS;
  static_assert(THIN_BIN < MAXBINS, "bins");
  int thin_R = 0;
  {
    static const char* eg = getenv("CBG_GROUPS");
    const bool groups = !(eg && !strcmp(eg, "0"));
    const int64_t gp = GROUP_PRODUCTS;
    int64_t thr[NSMALL + NGCLS];
    for (int i = 0; i < NSMALL; ++i) thr[i] = std::min(kSymThr[i], big);
    thr[NSMALL + NGCLS - 1] = INT64_MAX;  // the single-panel big columns; bin NSMALL + NGCLS: thin ones
    const int glmax = GROUP_LOG_MAX;
    for (int c = 0; c + 1 < NGCLS; ++c) {
      const int64_t g = 1LL << (GROUP_LOG_MAX - c);
      thr[NSMALL + c] = (groups && g <= bp.R && g <= (1LL << glmax)) ? gp * bp.R / g : -1;
    }
    BinPending sp;
    const bool thin_on = !(getenv("CBG_THIN") && !strcmp(getenv("CBG_THIN"), "0"));  // read per call (tests)
    // thin when flops * THIN_RATIO < B entries * R (1 and 2 measured equal at scales 22/24)
    const int ratio = (int)THIN_RATIO;
    thin_R = (fused && thin_on && bp.R >= 4) ? (int)(bp.R * THIN_RATIO / ratio) : 0;
    bin_classify(nz, flops.p, cnt.p, 0, thr, NSMALL + NGCLS, big, sp, s, 0, B.cp, NSMALL, thin_R, THIN_BIN, copy1);
    CBG_HIP(hipStreamSynchronize(s));  // host sync 1 of 4: the symbolic bins' sizes
    sp.read();
    if (thin_R && (double)sp.hf[THIN_BIN] * THIN_BYTES_PER_PRODUCT > 0.25 * device_bytes_available()) {
      // the sort's temporaries (64-bit counts, cbg_sort.hip) would take more than a
      // quarter of the device memory left: classify again without thin columns
      thin_R = 0;
      bin_classify(nz, flops.p, cnt.p, 0, thr, NSMALL + NGCLS, big, sp, s, 0, B.cp, NSMALL, 0, THIN_BIN, copy1);
      CBG_HIP(hipStreamSynchronize(s));
      sp.read();
    }
    bin_scatter(nz, sp, sb, s, df);
    big_entries = (int64_t)sp.big_entries[0];
    thin_entries = (int64_t)sp.big_entries[1];
  }
  // small-column symbolic bins on the side stream, big columns on the main one
  // (bins 1..SYM_FUSED_LAST fused with their numeric)
  DBuf<int32_t> fused_ir;
  DBuf<double> fused_val;
  DBuf<int64_t> fused_slot;  // temporary slot of each fused column (-1: none)
  size_t fused_off[SYM_FUSED_LAST + 2] = {};  // temporary slots of the fused bins 1..SYM_FUSED_LAST
  // slot width of fused bin b: its flops bound (big >= 64 never clips bins 1..6,
  // and a clipped bin 7 .. 9 holds columns of <= big flops)
  auto fmax_of = [&](int b) { return (int)kSymThr[b]; };
  if (fused) {
    fused_slot.reset(nz);
    CBG_HIP(hipMemsetAsync(fused_slot.p, 0xff, sizeof(int64_t) * nz, s));  // -1: not fused (before the fork)
  }
  // inline records of A's columns for the small-column and thin passes when A's
  // columns are short (<= 2 entries on average) and each entry is gathered many
  // times (flops >= 4 nnz(A)): GalerkinNew's S*(AT), S = T^T
  DBuf<int4> ainl;
  {
    unsigned long long fsmall = 0;
    for (int b = 1; b < NSMALL; ++b) fsmall += sb.flops[b];
    fsmall += thin_R ? sb.flops[THIN_BIN] : 0;
    if (fused && A.nnz <= 2 * A.nzc && (double)fsmall >= 4.0 * (double)A.nnz) {
      ainl.reset(2 * (A.n + 1));
      hipLaunchKernelGGL(k_inline_cols, dim3(nblk(A.n + 1, 256)), dim3(256), 0, s, A.n + 1, cmap.p, A.ir, A.val,
                         ainl.p);
    }
  }
  fork(s);
  // streams of the small symbolic bins (balance_bins; the fused bins also do
  // their numeric work: cost 2 per flop)
  hipStream_t symst[NSMALL];
  bool big_dominant = false;  // the (column, panel) units carry most of the flops over >= 8 row panels
  {
    double main_w = 0.0;
    for (int b = NSMALL; b < NSMALL + NGCLS; ++b) main_w += (double)sb.flops[b];
    double cost[NSMALL];
    for (int b = 0; b < NSMALL; ++b) cost[b] = (fused && b >= 1 && b <= SYM_FUSED_LAST) ? 2.0 : 1.0;
    // The small symbolic bins join the main stream, ahead of
    // the (column, panel) units, when those carry most of the flops over >= 8
    // row panels -- on the side stream they co-ran with k_sym_panel for its
    // whole length and slowed it (scale 22: 436.3 vs 443.1 ms, scale 24:
    // 3948 vs 3965 ms); small products (scale 18: R = 1) and small-column
    // products (GalerkinNew) keep the concurrency (side: 6.67 vs 6.79 ms and
    // 6.37 vs 6.85 ms)
    hipStream_t sy = ssym;
    if (bp.R >= 8) {
      double small_w = 0.0;
      for (int b = 1; b < NSMALL; ++b) small_w += (double)sb.flops[b];
      big_dominant = main_w >= small_w;
    }
    if (big_dominant) sy = s;
    symst[0] = sy;
    balance_bins(sb.flops, 1, NSMALL - 1, main_w, 0.0, cost, s, sy, symst, !big_dominant);
  }
  {
    const int32_t* P = sb.perm.p;
    auto at = [&](int b) { return P + sb.offset[b]; };
    if (fused) {
      // bins 1..SYM_FUSED_LAST (flops <= 512): symbolic and numeric in one pass into fused_ir/val
      for (int b = 1; b <= SYM_FUSED_LAST; ++b)
        fused_off[b + 1] = fused_off[b] + (size_t)sb.count[b] * (size_t)fmax_of(b);
      // the thin columns' unique entries follow the fused bins' slots
      const size_t ftot = fused_off[SYM_FUSED_LAST + 1] + (thin_R ? (size_t)sb.flops[THIN_BIN] : 0);
      fused_ir.reset(ftot + 1);
      fused_val.reset(ftot + 1);
      for (int b = 1; b <= SYM_FUSED_LAST; ++b) {
        if (semiring == CBG_MIN_PLUS)
          launch_esc<1>(at(b), sb.count[b], fmax_of(b), B, cmap.p, ainl.p, A, cnt.p, fused_ir.p, fused_val.p,
                        (int64_t)fused_off[b], fused_slot.p, symst[b]);
        else
          launch_esc<0>(at(b), sb.count[b], fmax_of(b), B, cmap.p, ainl.p, A, cnt.p, fused_ir.p, fused_val.p,
                        (int64_t)fused_off[b], fused_slot.p, symst[b]);
      }
    }
    static_assert(SYM_FUSED_LAST == 8 || SYM_FUSED_LAST == 9, "fused bins");
    if (SYM_FUSED_LAST < 9) launch_sym_wave<10>(at(9), sb.count[9], B, cmap.p, A, cnt.p, symst[9]);
    launch_sym_block<11, 256>(at(10), sb.count[10], B, cmap.p, ainl.p, A, cnt.p, symst[10]);
    launch_sym_block<12, 256>(at(11), sb.count[11], B, cmap.p, ainl.p, A, cnt.p, symst[11]);
    launch_sym_block<13, 512>(at(12), sb.count[12], B, cmap.p, ainl.p, A, cnt.p, symst[12]);
  }
  bp.nbig = sb.offset[NSMALL + NGCLS] - sb.offset[NSMALL];
  bp.perm_big = sb.perm.p + sb.offset[NSMALL];
  const int nbig = bp.nbig;
  const int64_t nbr = (int64_t)nbig * bp.R;
  // f32 copy of A's values for the slab kernels (checked once per A; the
  // verdict is read back with host sync 2)
  DBuf<float> valf_own;
  DBuf<float>& valf = ap.active ? ap.valf : valf_own;
  DBuf<PackedRV> valp_own;
  DBuf<PackedRV>& valp = ap.active ? ap.valp : valp_own;
  DBuf<PackedRVD> valpd_own;
  int af = ap.active ? ap.af : -1, af_inexact = 0;
  int ai = ap.active ? ap.ai : -1, amax = ap.active ? ap.amax : 0;
  DBuf<int> af_flag;
  // [0] A not f32-exact | [1] A not integral, [2] max |a| | [4] B not integral,
  // [5] max |b|, [6] B's largest column |sum| (IACC; read with sync 2)
  int* afh = reinterpret_cast<int*>(host_stage(STAGE_AF));
  if (nbig > 0 && af < 0 && !sym_only) {
    valf.reset(A.nnz);
    valp.reset(A.nnz);
    af_flag.reset(4);  // ([3]: k_int_bound's unused column-sum slot)
    CBG_HIP(hipMemsetAsync(af_flag.p, 0, 4 * sizeof(int), s));
    const int64_t nb = std::min<int64_t>(nblk(A.nnz, 256), (int64_t)device_cus() * 16);
    hipLaunchKernelGGL(k_vals_f32, dim3((unsigned)nb), dim3(256), 0, s, A.nnz, A.val, valf.p, af_flag.p, A.ir,
                       valp.p);
    hipLaunchKernelGGL(k_int_bound, dim3((unsigned)nb), dim3(256), 0, s, A.nnz, A.val, af_flag.p + 1, af_flag.p);
    CBG_HIP(hipMemcpyAsync(afh, af_flag.p, 3 * sizeof(int), hipMemcpyDeviceToHost, s));
  }
  DBuf<int> bint;
  afh[4] = 1;  // (no check: not integral)
  if (nbig > 0 && !sym_only && af != 0 && ai != 0) {
    bint.reset(3);
    CBG_HIP(hipMemsetAsync(bint.p, 0, 3 * sizeof(int), s));
    hipLaunchKernelGGL(k_col_int_bound, dim3((unsigned)std::min<int64_t>(nblk(B.nzc * WAVE, 256), (int64_t)device_cus() * 8)),
                       dim3(256), 0, s, B.nzc, B.cp, B.val, bint.p, af_flag.p);
    CBG_HIP(hipMemcpyAsync(afh + 4, bint.p, 3 * sizeof(int), hipMemcpyDeviceToHost, s));
  }
  if (nbig > 0) {
    // panel column maps of A (reused across phases like cmap)
    constexpr int pm_entries = 64;  // map only the referenced A columns when big-column entries * 64 < A's columns
    bp.n1 = A.n + 1;
    // column-major panel maps for the symbolic's XCD column order: a column's R
    // entries in one or two lines (scale 22: 399.6 -> 395.5 ms alone, with the
    // order 384 ms; the numeric slabs, panel-major, read them at the same speed)
    bp.kmajor = bp.R > 1;
    if (ap.active && ap.cmapP.p && ap.plog == bp.plog && ap.kmajor == bp.kmajor) {
      bp.cmapP = ap.cmapP.p;
    } else if (bp.R > 1 && pm_entries > 0 && big_entries * pm_entries < A.nzc) {
      // few big-column entries (GalerkinNew's A*T: ~10^3 of A's 4 M columns;
      // not the phase plan's sample of scale 22, 1/10 of them, whose hub
      // references would each search their long A column again):
      // map only the A columns they reference, without the memset of the
      // R x n map; this B's own map, never cached for other pieces / phases
      bp.cmapP_own.reset((size_t)bp.R * (A.n + 1));
      hipLaunchKernelGGL(k_colmap_panels_entries, dim3(nblk((int64_t)nbig * WAVE, 256)), dim3(256), 0, s,
                         bp.perm_big, nbig, B.cp, B.ir, cmap.p, A.ir, bp.plog, bp.R, bp.pm().sr, bp.pm().sk,
                         bp.cmapP_own.p);
      bp.cmapP = bp.cmapP_own.p;
    } else {
      DBuf<int2>& cp = ap.active ? ap.cmapP : bp.cmapP_own;
      cp.reset((size_t)bp.R * (A.n + 1));
      if (bp.R == 1) {
        hipLaunchKernelGGL(k_colmap_panel1, dim3(nblk(A.n + 1, 256)), dim3(256), 0, s, A.n + 1, cmap.p, cp.p);
      } else {
        CBG_HIP(hipMemsetAsync(cp.p, 0, sizeof(int2) * bp.R * (A.n + 1), s));
        hipLaunchKernelGGL(k_colmap_panels_col, dim3(nblk(A.nzc, 256)), dim3(256), 0, s, A.nzc, A.cp, A.jc, A.ir,
                           bp.plog, bp.R, bp.pm().sr, bp.pm().sk, cp.p);
      }
      if (ap.active) {
        ap.plog = bp.plog;
        ap.kmajor = bp.kmajor;
      }
      bp.cmapP = cp.p;
    }
    bp.desc.reset((size_t)nbr * NFINE_MAX);
    bp.nslab.reset(nbr);
    bp.cnt_br.reset(nbr);
    // keep the symbolic bitmaps for the numeric phase when they fit a budget
    // (saves the numeric marking pass); otherwise numeric rebuilds them
    // slots are handed out in launch order by the bitmap-mode pairs
    const int64_t slot_bytes = (int64_t)4 << (bp.plog - 5);
    const int64_t nslots = sym_only ? 0 : std::min<int64_t>(nbr, (int64_t)(bitmap_budget_bytes() / slot_bytes));
    DBuf<int> gbm_next;
    if (nslots > 0) {
      bp.gbm.reset((size_t)nslots << (bp.plog - 5));
      bp.gbm_slot.reset(nbr);
      gbm_next.reset(1);
      CBG_HIP(hipMemsetAsync(gbm_next.p, 0, sizeof(int), s));
    }
    if (nbr >= (int64_t)INT32_MAX) throw HipError("too many (column, panel) pairs", CBG_ERR_NOTSUPPORTED);
    // the multi-slab pairs' cut positions, handed out by an atomic counter up to
    // a budget (pairs past it leave their cuts to the numeric's searches)
    DBuf<unsigned long long> cuts_next;
    long long cuts_cap = 0;
    if (!sym_only) {
      // at most min(1.5 GB, 2 % of the free HBM), and never more than the cuts of
      // every pair cut into NFINE_MAX slabs (GalerkinNew's few big columns need
      // little); CBG_CUTS_CAP (entries, read per call) is a test hook that leaves
      // pairs past it to the numeric's searches
      cuts_cap = std::min<long long>(INT32_MAX, (long long)(std::min(1.5e9, 0.02 * device_bytes_available()) / 4));
      cuts_cap = std::min<long long>(cuts_cap, (long long)big_entries * bp.R * (NFINE_MAX - 1));
      if (const char* e = getenv("CBG_CUTS_CAP")) cuts_cap = std::min<long long>(cuts_cap, atoll(e));
      bp.cuts.reset(std::max<long long>(cuts_cap, 1));
      bp.pcoff.reset(nbr);
      cuts_next.reset(1);
      CBG_HIP(hipMemsetAsync(bp.pcoff.p, 0xff, sizeof(int) * nbr, s));
      CBG_HIP(hipMemsetAsync(cuts_next.p, 0, sizeof(unsigned long long), s));
    }
    const int pwords = 1 << (bp.plog - 5);
    auto lds_of = [&](int hw) {
      return (size_t)hw * 4 + NFINE_MAX * 4 + (BIG_BS + 4) * 4 + BIG_BS * 4 + (BIG_BS / WAVE + 4) * 4 +
             (size_t)SYM_OVF_CAP * 4;
    };
    set_lds(k_sym_panel<true>, lds_of(std::max(pwords, GROUP_T)));
    set_lds(k_sym_panel<false>, lds_of(std::max(pwords, GROUP_T)));
    SymPanelArgs sa{bp.perm_big, bp.R, bp.plog, 0, 0, pwords, 0, B.cp, B.ir, bp.pm(), A.ir, A.m,
                    cnt.p, bp.cnt_br.p, bp.desc.p, bp.nslab.p, bp.gbm.p, (int)nslots, gbm_next.p,
                    bp.gbm_slot.p,
                    bp.cuts.p, cuts_next.p, cuts_cap,
                    bp.pcoff.p, nullptr, nullptr};
    // group units that overflow one hash slab, collected for k_sym_deferred
    int64_t group_units = 0;
    for (int c = 0; c < NGCLS; ++c)
      if (GROUP_LOG_MAX - c > 0)
        group_units += (int64_t)sb.count[NSMALL + c] * ((bp.R + (1 << (GROUP_LOG_MAX - c)) - 1) >> (GROUP_LOG_MAX - c));
    DBuf<int4> defer;
    DBuf<int> defer_n;
    if (group_units > 0) {
      defer.reset(group_units);
      defer_n.reset(1);
      CBG_HIP(hipMemsetAsync(defer_n.p, 0, sizeof(int), s));
      sa.defer = defer.p;
      sa.defer_n = defer_n.p;
    }
    // one launch per group class (largest groups first)
    for (int c = 0; c < NGCLS; ++c) {
      const int nc = sb.count[NSMALL + c];
      if (nc == 0) continue;
      sa.glog = GROUP_LOG_MAX - c;
      sa.boff = sb.offset[NSMALL + c] - sb.offset[NSMALL];
      sa.hwords = sa.glog > 0 ? std::max(pwords, GROUP_T) : pwords;
      const int64_t RG = (bp.R + (1 << sa.glog) - 1) >> sa.glog;
      sa.ncls = nc;
      work[sa.glog > 0 ? CBG_WORK_SYM_GROUP_UNITS : CBG_WORK_SYM_PANEL_UNITS] += RG * nc;
      // resident blocks per CU at this launch's LDS size
      const int per_cu = sa.glog > 0 ? blocks_per_cu(k_sym_panel<true>, BIG_BS, lds_of(sa.hwords))
                                     : blocks_per_cu(k_sym_panel<false>, BIG_BS, lds_of(sa.hwords));
      // (a multiple of 8: the XCD column order; 8 x ceil(nc / 8) x RG units)
      const int64_t grid = std::min<int64_t>(RG * ((nc + 7) / 8) * 8,
                                             ((int64_t)per_cu * device_cus() * CBG_SYM_WAVES_OF_UNITS) & ~7LL);
      if (sa.glog > 0)
        hipLaunchKernelGGL(k_sym_panel<true>, dim3((unsigned)grid), dim3(BIG_BS), lds_of(sa.hwords), s, sa);
      else
        hipLaunchKernelGGL(k_sym_panel<false>, dim3((unsigned)grid), dim3(BIG_BS), lds_of(sa.hwords), s, sa);
    }
    if (group_units > 0) {
      sa.hwords = std::max(pwords, GROUP_T);
      set_lds(k_sym_deferred, lds_of(sa.hwords));
      hipLaunchKernelGGL(k_sym_deferred, dim3((unsigned)std::min<int64_t>(group_units, device_cus() * 4)),
                         dim3(BIG_BS), lds_of(sa.hwords), s, sa);
      CBG_HIP(hipMemcpyAsync(reinterpret_cast<int64_t*>(host_stage(STAGE_SCALARS)) + 5, defer_n.p, sizeof(int),
                             hipMemcpyDeviceToHost, s));
      df.take(defer);
      df.take(defer_n);
    }
    // the symbolic kernels may still run: the counters stay allocated until the
    // multiply's last synchronization
    bp.gbm_next = gbm_next.p;
    bp.gbm_slots = nslots;
    df.take(gbm_next);
    df.take(cuts_next);
  }
  // the thin columns' sort after the big columns' launches (its host
  // synchronizations would otherwise hold them back)
  {
    // CBG_DBG bit 16: the symbolic bins' sizes
    static const int dbg = getenv("CBG_DBG") ? atoi(getenv("CBG_DBG")) : 0;
    if (dbg & 16) {
      unsigned long long fs = 0, fh = 0, fb = 0;
      for (int b = 1; b <= SYM_FUSED_LAST; ++b) fs += sb.flops[b];
      for (int b = SYM_FUSED_LAST + 1; b < NSMALL; ++b) fh += sb.flops[b];
      for (int b = NSMALL; b < NSMALL + NGCLS; ++b) fb += sb.flops[b];
      std::fprintf(stderr,
                   "[cbg bins] fused cols %d flops %llu | hash cols %d flops %llu | big cols %d flops %llu | "
                   "thin cols %d entries %lld flops %llu | inline A %d\n",
                   sb.offset[SYM_FUSED_LAST + 1] - sb.offset[1], fs, sb.offset[NSMALL] - sb.offset[SYM_FUSED_LAST + 1],
                   fh, nbig, fb, thin_R ? sb.count[THIN_BIN] : 0, (long long)thin_entries,
                   thin_R ? (unsigned long long)sb.flops[THIN_BIN] : 0ull, ainl.p != nullptr);
    }
  }
  if (thin_R && sb.count[THIN_BIN] > 0) {
    // on the copy stream (idle until the numeric), from the fork point, so the
    // sort runs beside the small-column bins of both streams instead of behind
    // the main stream's (its readback then waits for the sort alone)
    CBG_HIP(hipStreamWaitEvent(scopy, ev_fork, 0));
    thin_columns(sb.perm.p + sb.offset[THIN_BIN], sb.count[THIN_BIN], thin_entries, (int64_t)sb.flops[THIN_BIN], A,
                 B, cmap.p, ainl.p, semiring, cnt.p, fused_slot.p, fused_ir.p, fused_val.p,
                 (int64_t)fused_off[SYM_FUSED_LAST + 1], scopy, df);
    CBG_HIP(hipEventRecord(ev_cjoin, scopy));
    CBG_HIP(hipStreamWaitEvent(s, ev_cjoin, 0));
  }
  join(s);
  // Everything that depends only on the per-column counts is launched now and
  // read back in ONE synchronization: nnz(C) (column pointers), the number of
  // slabs, the numeric bins' histogram and the number of nonempty C columns.
  DBuf<int64_t> colptr(nz + 1);
  exclusive_scan_i32_to_i64(cnt.p, colptr.p, nz, s, &df);
  // nnz(C), slabs, nonempty C columns, flops: one pinned slot, read after sync 2
  int64_t* scal = reinterpret_cast<int64_t*>(host_stage(STAGE_SCALARS));
  scal[1] = 0;
  CBG_HIP(hipMemcpyAsync(&scal[0], colptr.p + nz, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  // slab lists of big columns
  DBuf<int64_t> sbase;
  DBuf<SlabRec> slist;
  int64_t nslabs = 0;
  if (nbig > 0) {
    sbase.reset(nbr + 1);
    exclusive_scan_i32_to_i64(bp.nslab.p, sbase.p, nbr, s, &df);
    CBG_HIP(hipMemcpyAsync(&scal[1], sbase.p + nbr, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  }
  BinPending npend;
  bin_classify(nz, flops.p, cnt.p, 1, kNumThr, 9, big, npend, s, fused ? kSymThr[SYM_FUSED_LAST] : 0, B.cp,
               MAXBINS, thin_R, 0, copy1);
  // compaction of C's columns (SpDCCols(SpTuples): nonempty columns only)
  DBuf<int64_t> flag(nz + 1), pos(nz + 1);
  hipLaunchKernelGGL(k_col_flags, dim3(nblk(nz, 256)), dim3(256), 0, s, nz, cnt.p, flag.p);
  exclusive_scan_i64(flag.p, pos.p, nz, s, &df);
  CBG_HIP(hipMemcpyAsync(&scal[2], pos.p + nz, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  CBG_HIP(hipMemcpyAsync(&scal[3], flops.p + nz, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  // single-entry big columns: their sizes' scan (the chunked copy), total read back with sync 2
  DBuf<int64_t> sb_sz, sb_off;
  scal[4] = 0;
  if (copy1 > 1 && !sym_only) {
    sb_sz.reset(nz);
    sb_off.reset(nz + 1);
    hipLaunchKernelGGL(k_single_big_sizes, dim3(nblk(nz, 256)), dim3(256), 0, s, nz, B.cp, flops.p, big, sb_sz.p);
    exclusive_scan_i64(sb_sz.p, sb_off.p, nz, s, &df);
    CBG_HIP(hipMemcpyAsync(&scal[4], sb_off.p + nz, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  }
  CBG_HIP(hipEventRecord(ev1, s));
  CBG_HIP(hipStreamSynchronize(s));  // host sync 2 of 4
  const int64_t nnzc = scal[0], nzcC = scal[2], flops_total = scal[3];
  nslabs = scal[1];
  const int64_t single_big_entries = scal[4];
  work[CBG_WORK_SYM_DEFERRED_UNITS] = scal[5];
  for (int b = 1; fused && b <= SYM_FUSED_LAST; ++b) work[CBG_WORK_ESC_COLUMNS] += sb.count[b];
  work[CBG_WORK_THIN_COLUMNS] = thin_R ? sb.count[THIN_BIN] : 0;
  work[CBG_WORK_SINGLE_BIG_ENTRIES] = copy1 > 1 ? single_big_entries : 0;
  if (sym_only) {
    df.synced = true;
    if (st) {
      float a = 0;
      CBG_HIP(hipEventElapsedTime(&a, ev0, ev1));
      *st = LocalStats{};
      st->ms_symbolic = a;
      st->nnz = nnzc;
      st->n_big = nbig;
      st->flops = flops_total;
      std::memcpy(st->work, work, sizeof(work));
    }
    return;
  }
  if (af_flag.p) {
    af_inexact = afh[0];
    af = af_inexact ? 0 : 1;
    ai = afh[1] ? 0 : 1;
    amax = afh[2];
    if (ap.active) {
      ap.af = af;
      ap.ai = ai;
      ap.amax = amax;
    }
    if (!af) {
      valf.release();
      valp.release();
    }
  }
  if (af == 1) bp.valAf = valf.p;
  if (af == 1 && valp.p) bp.valAp = valp.p;
  uint64_t big_fl = 0;
  for (int b = NSMALL; b < NSMALL + NGCLS; ++b) big_fl += sb.flops[b];
  DBuf<PackedRVD>& vd = ap.active ? ap.valpd : valpd_own;
  if (af == 0 && nbig > 0 && (vd.p || big_fl >= 4 * (uint64_t)A.nnz)) {
    // the f64-valued slab path reads A as (row, f64) records (built once per A,
    // when the big columns' products are enough to pay for its 24 B per entry:
    // GalerkinNew scale 22 packed 68 M entries, 0.34 ms, for 3.7 M products)
    if (!vd.p) {
      vd.reset(A.nnz);
      hipLaunchKernelGGL(k_pack_rvd, dim3((unsigned)std::min<int64_t>(nblk(A.nnz, 256), (int64_t)device_cus() * 16)),
                         dim3(256), 0, s, A.nnz, A.ir, A.val, vd.p);
    }
    bp.valAd = vd.p;
  }
  bp.iacc = bp.valAp && ai == 1 && !afh[4] && iacc_bound_ok(semiring, amax, afh[5], afh[6]);
  work[CBG_WORK_IACC] = bp.iacc ? 1 : 0;
  {
    // test hook (CBG_FAULT_C_BYTES, read per call): C larger than this fails as
    // an out-of-memory would, after the symbolic pass -- the phase splitting of
    // MemEfficientSpGEMM (cbg_summa.cpp multiply_to_fn) is tested with it
    const char* e = getenv("CBG_FAULT_C_BYTES");
    if (e && 12.0 * (double)nnzc > atof(e)) {
      df.synced = true;
      throw HipError("C of " + std::to_string(nnzc) + " entries exceeds CBG_FAULT_C_BYTES", CBG_ERR_OOM);
    }
  }
  C.nzc = nzcC;
  C.cp = static_cast<int64_t*>(pool().alloc(sizeof(int64_t) * (nzcC + 1)));
  C.jc = static_cast<int32_t*>(pool().alloc(sizeof(int32_t) * std::max<int64_t>(nzcC, 1)));
  Cg.t = C;
  hipLaunchKernelGGL(k_col_scatter, dim3(nblk(nz + 1, 256)), dim3(256), 0, s, nz, cnt.p, pos.p, B.jc, colptr.p, C.jc,
                     C.cp);
  int ncls[SLAB_NCLS] = {};
  if (nbig > 0 && nslabs > 0) {
    slist.reset(nslabs);
    const int NK = SLAB_NCLS * slab_kr(bp.R);
    DBuf<int> counters(2 * NK + SLAB_NCLS);  // counts[NK] | cursor[NK] | class totals
    CBG_HIP(hipMemsetAsync(counters.p, 0, (2 * NK + SLAB_NCLS) * sizeof(int), s));
    const int rank_span = 1 << bp.plog, rank_min = RANK_SLABS_MIN;
    // (CBG_GRANK_MIN, read per call: group slabs of more nonzeros than this run
    // as group rank slabs; -1 none)
    const char* egm = getenv("CBG_GRANK_MIN");
    const int grank_min = egm ? (atoi(egm) < 0 ? INT32_MAX : atoi(egm)) : GRANK_SLABS_MIN;
    hipLaunchKernelGGL(k_slab_count, dim3(nblk(nbig, 256)), dim3(256), NK * sizeof(int), s, nbig, bp.R, bp.nslab.p,
                       bp.cnt_br.p, bp.desc.p, SLAB_SMALL_CAP, rank_span, rank_min, grank_min, counters.p);
    hipLaunchKernelGGL(k_slab_bases, dim3(1), dim3(64), 0, s, bp.R, counters.p, counters.p + NK,
                       counters.p + 2 * NK);
    hipLaunchKernelGGL(k_slab_fill, dim3(nblk(nbig, 256)), dim3(256), 2 * NK * sizeof(int), s, nbig, bp.R,
                       bp.nslab.p, bp.desc.p, SLAB_SMALL_CAP, rank_span, rank_min, grank_min, counters.p + NK, slist.p,
                       bp.perm_big, B.cp, colptr.p,
                       bp.gbm_slot.p, bp.plog, A.m, bp.pcoff.p);
    int* ncls_h = reinterpret_cast<int*>(host_stage(STAGE_SLABS));
    CBG_HIP(hipMemcpyAsync(ncls_h, counters.p + 2 * NK, SLAB_NCLS * sizeof(int), hipMemcpyDeviceToHost, s));
    if (bp.gbm_next)
      CBG_HIP(hipMemcpyAsync(ncls_h + SLAB_NCLS, bp.gbm_next, sizeof(int), hipMemcpyDeviceToHost, s));
    CBG_HIP(hipStreamSynchronize(s));  // host sync 3 of 4: the slab classes' sizes
    std::memcpy(ncls, ncls_h, sizeof(int) * SLAB_NCLS);
    // (CBG_DBG bit 128 hands out slots without storing the bitmaps: the
    // marking pass must run)
    static const int dbg_kept = getenv("CBG_DBG") ? atoi(getenv("CBG_DBG")) : 0;
    bp.all_kept = bp.gbm_next && (int64_t)ncls_h[SLAB_NCLS] <= bp.gbm_slots && !(dbg_kept & 128);
    df.take(counters);
    work[bp.all_kept ? CBG_WORK_BITMAP_SMALL_KEPT : CBG_WORK_BITMAP_SMALL_MARK] = ncls[0];
    work[bp.all_kept ? CBG_WORK_BITMAP_LARGE_KEPT : CBG_WORK_BITMAP_LARGE_MARK] = ncls[1];
    for (int k = 0; k < SLAB_HASH_NCLS; ++k) work[CBG_WORK_HASH0 + k] = ncls[2 + k];
    for (int k = 0; k < SLAB_RANK_NCLS; ++k) work[CBG_WORK_RANK0 + k] = ncls[SLAB_RANK0 + k];
    for (int k = 0; k < SLAB_GRANK_NCLS; ++k) work[CBG_WORK_GRANK0 + k] = ncls[SLAB_GRANK0 + k];
    static const int dbg = getenv("CBG_DBG") ? atoi(getenv("CBG_DBG")) : 0;
    if (dbg & 16)
    {
      static const int ht[SLAB_HASH_NCLS] = {CBG_HASH_TABLES};
      std::fprintf(stderr, "[cbg slabs] bitmap small %d large %d | hash", ncls[0], ncls[1]);
      for (int k = 0; k < SLAB_HASH_NCLS; ++k) std::fprintf(stderr, " T%d %d", ht[k], ncls[2 + k]);
      std::fprintf(stderr, " | rank N1024 %d N2048 %d N4096 %d | group rank N2048 %d N4096 %d", ncls[SLAB_RANK0],
                   ncls[SLAB_RANK0 + 1], ncls[SLAB_RANK0 + 2], ncls[SLAB_GRANK0], ncls[SLAB_GRANK0 + 1]);
      std::fprintf(stderr, "\n");
    }
  }
  // output arrays
  C.nnz = nnzc;
  if (sink) {
    sink->place(nnzc, &C.ir, &C.val);
    C.reserved |= TILE_BORROWED_ENTRIES;
  } else {
    C.ir = static_cast<int32_t*>(pool().alloc(sizeof(int32_t) * std::max<int64_t>(nnzc, 1)));
    C.val = static_cast<double*>(pool().alloc(sizeof(double) * std::max<int64_t>(nnzc, 1)));
  }
  Cg.t = C;
  // numeric
  Binned nbn;
  bin_scatter(nz, npend, nbn, s, df);
  for (int b = 1; b <= 4; ++b) work[CBG_WORK_WAVE_BIN_COLUMNS] += nbn.count[b];
  for (int b = 5; b <= 8; ++b) work[CBG_WORK_HASH_BIN_COLUMNS] += nbn.count[b];
  // small-column bins on the side stream, big-column slabs on the main one,
  // the copies (fused bins, single-entry columns) on the copy stream: they only
  // need colptr and stream at HBM rate beside the latency-bound kernels
  // (GalerkinNew at 22: 5.92 / 5.98 vs 6.45 / 6.38 ms); not where the big
  // columns' slabs dominate, which they slow (scale 22: 418.4 vs 413.0 ms)
  const bool copy_stream = !big_dominant;
  fork(s);
  const hipStream_t sc = copy_stream ? scopy : snum;
  if (copy_stream) CBG_HIP(hipStreamWaitEvent(scopy, ev_fork, 0));
  hipStream_t numst[10];
  {
    // the slabs of the big columns on the main stream; the fused bins' copies on
    // the side one (about a quarter of a product's cost per entry)
    double fused_w = 0.0;
    if (fused && !copy_stream)
      for (int b = 1; b <= SYM_FUSED_LAST; ++b) fused_w += 0.25 * (double)sb.flops[b];
    numst[0] = numst[9] = snum;
    // balanced when the copies have their own stream (GalerkinNew 6.01 vs 6.07 ms,
    // 3 rounds; round 3, before the copy stream: 9.9-10.2 vs 10.0 ms, off)
    balance_bins(nbn.flops, 1, 8, (double)nbn.flops[9], fused_w, nullptr, s, snum, numst, copy_stream);
  }
  // (the whole-column bins on the side stream overlap the slabs: serialized after
  // them on the main stream they take ~13 ms per scale-22 step and the step is
  // 1 ms longer, before them 0.6 ms longer -- profiles/r06_ab_numbins.json)
  if (semiring == CBG_MIN_PLUS) numeric_dispatch<1>(nbn, A, bp.valAf, B, cmap.p, ainl.p, colptr.p, C, numst, df);
  else numeric_dispatch<0>(nbn, A, bp.valAf, B, cmap.p, ainl.p, colptr.p, C, numst, df);
  if (fused && (fused_off[SYM_FUSED_LAST + 1] > 0 || (thin_R && sb.count[THIN_BIN] > 0)))
  {
    hipLaunchKernelGGL(k_copy_fused, dim3(nblk(nz, 256)), dim3(256), 0, sc, nz, fused_slot.p, cnt.p,
                       colptr.p, fused_ir.p, fused_val.p, C.ir, C.val, (int64_t)fused_off[SYM_FUSED_LAST + 1]);
    if (thin_R)
      thin_copy(sb.perm.p + sb.offset[THIN_BIN], sb.count[THIN_BIN], fused_slot.p, cnt.p, colptr.p, fused_ir.p,
                fused_val.p, C.ir, C.val, s);
  }
  if (copy1) {
    if (semiring == CBG_MIN_PLUS)
      hipLaunchKernelGGL(k_copy_single<1>, dim3(nblk(nz, 256)), dim3(256), 0, sc, nz, B.cp, B.ir, B.val, cmap.p,
                         flops.p, big, A.ir, A.val, colptr.p, C.ir, C.val);
    else
      hipLaunchKernelGGL(k_copy_single<0>, dim3(nblk(nz, 256)), dim3(256), 0, sc, nz, B.cp, B.ir, B.val, cmap.p,
                         flops.p, big, A.ir, A.val, colptr.p, C.ir, C.val);
  }
  if (copy1 > 1 && single_big_entries > 0) {
    const int ch = (int)std::min<int64_t>(SB_CHUNK, big + 1);
    const unsigned g = (unsigned)((single_big_entries + ch - 1) / ch);
    if (semiring == CBG_MIN_PLUS)
      hipLaunchKernelGGL(k_copy_single_big<1>, dim3(g), dim3(256), 0, sc, nz, sb_off.p, ch, B.cp, B.ir, B.val,
                         cmap.p, A.ir, A.val, colptr.p, C.ir, C.val);
    else
      hipLaunchKernelGGL(k_copy_single_big<0>, dim3(g), dim3(256), 0, sc, nz, sb_off.p, ch, B.cp, B.ir, B.val,
                         cmap.p, A.ir, A.val, colptr.p, C.ir, C.val);
  }
  if (nslabs > 0) {
    if (semiring == CBG_MIN_PLUS) launch_slabs<1>(slist.p, ncls, bp, A, B, C, s, side, df);
    else launch_slabs<0>(slist.p, ncls, bp, A, B, C, s, side, df);
  }
  join(s);
  if (copy_stream) {
    CBG_HIP(hipEventRecord(ev_cjoin, scopy));
    CBG_HIP(hipStreamWaitEvent(s, ev_cjoin, 0));
  }
  CBG_HIP(hipEventRecord(ev2, s));
  CBG_HIP(hipStreamSynchronize(s));  // host sync 4 of 4: C complete
  df.synced = true;
  CBG_HIP(hipGetLastError());
  {
    static const int dbg = getenv("CBG_DBG") ? atoi(getenv("CBG_DBG")) : 0;
    if (dbg & 16) {
      if (dbg & 32) {
        unsigned long long gs[16];
        CBG_HIP(hipMemcpyFromSymbol(gs, HIP_SYMBOL(g_stat), sizeof(gs)));
        std::fprintf(stderr, "[cbg k_num_slab] slabs %llu nonfull %llu nb %llu nb_nonfull %llu nout %llu multichunk %llu "
                     "products %llu | hash products panel %llu column %llu nout %llu | rank products %llu nout %llu"
                     " | symbolic groups %llu products %llu, by panels %llu products %llu\n",
                     gs[0], gs[1], gs[2], gs[3], gs[5], gs[6], gs[4], gs[7], gs[8], gs[9], gs[10], gs[11], gs[12], gs[13],
                     gs[14], gs[15]);
        std::memset(gs, 0, sizeof(gs));
        CBG_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_stat), gs, sizeof(gs)));
      }
      unsigned long long ph[24];
      CBG_HIP(hipMemcpyFromSymbol(ph, HIP_SYMBOL(g_phase), sizeof(ph)));
      const char* names[7] = {"init", "staging", "-", "rankscan", "pass0", "pass1", "output"};
      std::fprintf(stderr, "[cbg phases, block-us summed / 256 CUs]");
      for (int k = 0; k < 7; ++k)
        if (k != 2) std::fprintf(stderr, " %s=%.3fms", names[k], ph[k] / 100.0 / 256.0 / 1000.0);
      const char* snames[5] = {"sym_staging", "sym_hash", "sym_bitmap_products", "sym_counts_store", "sym_plan"};
      for (int k = 8; k < 13; ++k) std::fprintf(stderr, " %s=%.3fms", snames[k - 8], ph[k] / 100.0 / 256.0 / 1000.0);
      const char* hnames[4] = {"hash_clear", "hash_staging", "hash_products", "hash_emit"};
      const int hk[4] = {7, 13, 14, 15};
      for (int k = 0; k < 4; ++k) std::fprintf(stderr, " %s=%.3fms", hnames[k], ph[hk[k]] / 100.0 / 256.0 / 1000.0);
      const char* rnames[5] = {"rank_stage", "rank_products", "rank_scan", "rank_acc", "rank_emit"};
      for (int k = 0; k < 5; ++k) std::fprintf(stderr, " %s=%.3fms", rnames[k], ph[16 + k] / 100.0 / 256.0 / 1000.0);
      std::fprintf(stderr, "\n");
      std::memset(ph, 0, sizeof(ph));
      CBG_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_phase), ph, sizeof(ph)));
    }
  }
  if (st) {
    float a = 0, b = 0;
    CBG_HIP(hipEventElapsedTime(&a, ev0, ev1));
    CBG_HIP(hipEventElapsedTime(&b, ev1, ev2));
    st->ms_symbolic = a;
    st->ms_numeric = b;
    st->nnz = nnzc;
    st->n_big = nbig;
    st->n_slabs = nslabs;
    st->flops = flops_total;  // total flops (k_flops), read back with sync 2
    std::memcpy(st->work, work, sizeof(work));
  }
  Cg.release();  // completed: the caller owns C
}

}  // namespace cbg
