// cbg_device.h -- device-side building blocks for gfx950 (wave64) kernels.
#pragma once
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cstdint>

namespace cbg {

constexpr int WAVE = 64;
#ifndef CBG_PRODUCTS_U
#define CBG_PRODUCTS_U 4  // products in flight per lane in wave_products (2 or 4; 8 measured equal to 4)
#endif
constexpr int EMPTY_KEY = 0x7FFFFFFF;  // empty hash slot; sorts after every row id

// streaming stores/loads for data written or read once (C's entries, the kept
// symbolic bitmaps): nontemporal, so they do not evict A's rows from L2
#ifndef CBG_NT_OUT
#define CBG_NT_OUT 1  // +2.8 % at scale 22, +6 % at 18 (same-box A/B)
#endif
#ifndef CBG_NT_EMIT
#define CBG_NT_EMIT 1  // hash-slab emit stores too: +0.3 % at 22
#endif
template <class T>
__device__ __forceinline__ void st_stream(T* p, T v) {
#if CBG_NT_OUT
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}
template <class T>
__device__ __forceinline__ T ld_stream(const T* p) {
#if CBG_NT_OUT
  return __builtin_nontemporal_load(p);
#else
  return *p;
#endif
}
// 16-byte nontemporal store / load of 4 words (p 16-byte aligned)
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st_stream4(unsigned* p, uint4 v) {
  u32x4 x = {v.x, v.y, v.z, v.w};
#if CBG_NT_OUT
  __builtin_nontemporal_store(x, reinterpret_cast<u32x4*>(p));
#else
  *reinterpret_cast<u32x4*>(p) = x;
#endif
}
__device__ __forceinline__ uint4 ld_stream4(const unsigned* p) {
#if CBG_NT_OUT
  const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
#else
  const u32x4 x = *reinterpret_cast<const u32x4*>(p);
#endif
  return make_uint4(x.x, x.y, x.z, x.w);
}
template <class T>
__device__ __forceinline__ void st_emit(T* p, T v) {
#if CBG_NT_EMIT
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}

// Order LDS traffic between the lanes of ONE wave (LDS executes a wave's
// instructions in issue order; this stops the compiler from reordering).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & (WAVE - 1); }

// DPP lane move with zero fill: lanes whose source is outside the row (or in
// a row masked off by ROWM) read 0
template <int CTRL, int ROWM = 0xf>
__device__ __forceinline__ int dpp0(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, ROWM, 0xf, false);
}

// inclusive scan over the 64 lanes of a wave, on the VALU: row_shr 1/2/4/8
// inside rows of 16 lanes, then row_bcast 15/31 across rows (no LDS
// permutes, whose latency a __shfl_up ladder would pay six times)
__device__ __forceinline__ int wave_incl_scan(int v) {
  v += dpp0<0x111>(v);       // row_shr:1
  v += dpp0<0x112>(v);       // row_shr:2
  v += dpp0<0x114>(v);       // row_shr:4
  v += dpp0<0x118>(v);       // row_shr:8
  v += dpp0<0x142, 0xa>(v);  // row_bcast:15 -> rows 1, 3
  v += dpp0<0x143, 0xc>(v);  // row_bcast:31 -> rows 2, 3
  return v;
}
// value of lane 63 in every lane
__device__ __forceinline__ int wave_last(int v) { return __builtin_amdgcn_readlane(v, WAVE - 1); }
__device__ __forceinline__ long long wave_incl_scan64(long long v) {
  const int lane = lane_id();
#pragma unroll
  for (int d = 1; d < WAVE; d <<= 1) {
    long long t = __shfl_up(v, d, WAVE);
    if (lane >= d) v += t;
  }
  return v;
}
__device__ __forceinline__ long long wave_sum64(long long v) {
#pragma unroll
  for (int d = WAVE / 2; d > 0; d >>= 1) v += __shfl_xor(v, d, WAVE);
  return v;
}
__device__ __forceinline__ int wave_sum(int v) { return wave_last(wave_incl_scan(v)); }

// Block-wide exclusive scan of one int per thread.  `tmp` holds >= BS/64+1 ints.
// Returns the exclusive prefix; *total receives the block sum.  Contains barriers.
// The wave totals are combined by every wave on its own (one LDS read per
// lane and a DPP scan), not by a serial loop of thread 0 behind a second barrier.
template <int BS>
__device__ __forceinline__ int block_excl_scan(int v, int* tmp, int* total) {
  constexpr int NW = BS / WAVE;
  static_assert(NW <= WAVE, "block size");
  const int lane = lane_id(), w = threadIdx.x / WAVE;
  const int incl = wave_incl_scan(v);
  if (lane == WAVE - 1) tmp[w] = incl;
  __syncthreads();
  const int ws = wave_incl_scan(lane < NW ? tmp[lane] : 0);
  const int before = w > 0 ? __builtin_amdgcn_readlane(ws, w > 0 ? w - 1 : 0) : 0;
  *total = __builtin_amdgcn_readlane(ws, NW - 1);
  __syncthreads();  // tmp is reused by the caller
  return before + incl - v;
}

// Block-wide exclusive scan of get(i), i in [0, n), in index order: put(i, prefix)
// for every i; returns the total.  Wave w owns a contiguous span of indices and
// its lanes take consecutive ones (conflict-free LDS access for array-backed
// get/put, unlike a per-thread contiguous chunk).  get() is called twice per
// index.  tmp holds >= BS/64+1 ints.  Contains barriers.
template <int BS, class G, class P>
__device__ __forceinline__ int block_ordered_scan(int n, G&& get, P&& put, int* tmp) {
  constexpr int NW = BS / WAVE;
  const int lane = lane_id(), w = threadIdx.x / WAVE;
  const int span = ((n + BS - 1) / BS) * WAVE;
  const int b0 = min(w * span, n), b1 = min(b0 + span, n);
  int tot = 0;
  for (int i = b0 + lane; i - lane < b1; i += WAVE) tot += (i < b1) ? get(i) : 0;
  tot = wave_sum(tot);
  if (lane == 0) tmp[w] = tot;
  __syncthreads();
  const int ws = wave_incl_scan(lane < NW ? tmp[lane] : 0);  // every wave combines the wave totals itself
  int run = w > 0 ? __builtin_amdgcn_readlane(ws, w > 0 ? w - 1 : 0) : 0;
  const int total = __builtin_amdgcn_readlane(ws, NW - 1);
  for (int i = b0 + lane; i - lane < b1; i += WAVE) {
    const int c = (i < b1) ? get(i) : 0;
    const int incl = wave_incl_scan(c);
    if (i < b1) put(i, run + incl - c);
    run += wave_last(incl);
  }
  __syncthreads();
  return total;
}

// largest i in [0, n) with pref[i] <= u, for a non-decreasing pref[0..n] with pref[0] = 0 <= u
__device__ __forceinline__ int seg_search(const int* pref, int n, int u) {
  int lo = 0, hi = n;  // invariant: pref[lo] <= u < pref[hi]
  while (hi - lo > 1) {
    int mid = (lo + hi) >> 1;
    if (pref[mid] <= u) lo = mid; else hi = mid;
  }
  return lo;
}

// seg_search for the 64 consecutive products [u0, umax] of a wave (all lanes
// active, nseg a multiple of 64): one sampled read per lane and two ballots
// narrow every lane's search to the samples spanning [u0, umax], so a lane
// pays ~log2(nseg/64) + 2 dependent LDS reads instead of log2(nseg)
__device__ __forceinline__ int seg_search_wave(const int* pref, int nseg, int u, int u0, int umax) {
  const int S = nseg / WAVE;
  const int smp = pref[lane_id() * S];
  const int c0 = __popcll(__ballot(smp <= u0)), c1 = __popcll(__ballot(smp <= umax));
  int lo = (c0 - 1) * S, hi = c1 * S;  // pref[lo] <= u0 <= u <= umax < pref[hi]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (pref[mid] <= u) lo = mid; else hi = mid;
  }
  return lo;
}

// Flattened product loop over a staged chunk of B entries.  pref[0..nseg] is
// the prefix sum of the segment lengths (A sub-columns); product u belongs to
// segment sg with pref[sg] <= u < pref[sg+1].  Lanes of a wave take
// consecutive products (coalesced reads of A's columns) and keep a per-lane
// segment cursor that only moves forward; the segment's data (SEG, from
// seg(sg)) is cached in registers while the cursor stays, so a product costs
// its global loads and its apply() only.  Two products per lane are in flight
// per iteration (load() both, then apply() both) for memory-level parallelism.
//   seg(sg)        -> SEG           (per segment, e.g. {A offset, B value})
//   load(SEG, u)   -> X             (global loads of product u)
//   apply(X)                        (LDS update)
// pre(X) -> Y runs the apply's reads (e.g. LDS lookups) for all products of
// an unrolled group before any apply(Y) writes, so their latencies overlap.
template <class S, class L, class P, class A>
__device__ __forceinline__ void wave_products3(const int* pref, int nseg, int u0, int u1, S&& seg, L&& load, P&& pre,
                                               A&& apply) {
  if (u0 >= u1) return;  // (uniform: the whole wave)
  const int umax = min(u0 + WAVE - 1, u1 - 1);
  int u = u0 + lane_id();
  int sg = seg_search_wave(pref, nseg, min(u, umax), u0, umax);
  if (u >= u1) return;
  int nxt = pref[sg + 1];
  auto cur = seg(sg);
  // (reading a segment's data together with its bound, or prefetching the next
  // segment's on entering one, measured flat / -2.5 % at scale 22:
  // profiles/r04_ab_cursor.json -- the loop is bound by A's gathers, not by this chain)
  auto advance = [&](int v) {
    if (v >= nxt) {
      do nxt = pref[++sg + 1]; while (v >= nxt);
      cur = seg(sg);
    }
  };
#if CBG_PRODUCTS_U >= 4
  for (; u + 3 * WAVE < u1; u += 4 * WAVE) {
    advance(u);
    auto x0 = load(cur, u);
    advance(u + WAVE);
    auto x1 = load(cur, u + WAVE);
    advance(u + 2 * WAVE);
    auto x2 = load(cur, u + 2 * WAVE);
    advance(u + 3 * WAVE);
    auto x3 = load(cur, u + 3 * WAVE);
    auto y0 = pre(x0);
    auto y1 = pre(x1);
    auto y2 = pre(x2);
    auto y3 = pre(x3);
    apply(y0);
    apply(y1);
    apply(y2);
    apply(y3);
  }
#endif
  for (; u + WAVE < u1; u += 2 * WAVE) {
    advance(u);
    auto x0 = load(cur, u);
    advance(u + WAVE);
    auto x1 = load(cur, u + WAVE);
    auto y0 = pre(x0);
    auto y1 = pre(x1);
    apply(y0);
    apply(y1);
  }
  if (u < u1) {
    advance(u);
    apply(pre(load(cur, u)));
  }
}

struct PreIdentity {
  template <class X>
  __device__ __forceinline__ X operator()(const X& x) const {
    return x;
  }
};

template <class S, class L, class A>
__device__ __forceinline__ void wave_products(const int* pref, int nseg, int u0, int u1, S&& seg, L&& load, A&& apply) {
  wave_products3(pref, nseg, u0, u1, seg, load, PreIdentity(), apply);
}

// block-wide versions: wave w takes the contiguous range [w*per, (w+1)*per)
template <int BS, class S, class L, class P, class A>
__device__ __forceinline__ void block_products3(const int* pref, int total, S&& seg, L&& load, P&& pre, A&& apply) {
  constexpr int NW = BS / WAVE;
  const int w = threadIdx.x / WAVE;
  const int per = (total + NW - 1) / NW;
  const int u0 = min(w * per, total), u1 = min(u0 + per, total);
  wave_products3(pref, BS, u0, u1, seg, load, pre, apply);
}
template <int BS, class S, class L, class A>
__device__ __forceinline__ void block_products(const int* pref, int total, S&& seg, L&& load, A&& apply) {
  block_products3<BS>(pref, total, seg, load, PreIdentity(), apply);
}

// Staged segments: st[sg] holds A's start minus the segment's first product
// index (CBG_SEG_OFF=1), so a segment switch reads one LDS word less
#ifndef CBG_SEG_OFF
#define CBG_SEG_OFF 1
#endif
__device__ __forceinline__ int seg_stage(int s, int ex) { return CBG_SEG_OFF ? s - ex : s; }
__device__ __forceinline__ int seg_off(const int* st, const int* pref, int sg) {
  return CBG_SEG_OFF ? st[sg] : st[sg] - pref[sg];
}
// per-segment register cache: A offset (st[sg] - pref[sg]) and B value
struct SegI {
  int off;
};
struct SegV {
  int off;
  double b;
};

// first position in sorted a[lo,hi) with a[pos] >= key
__device__ __forceinline__ int lower_bound_g(const int32_t* __restrict__ a, int lo, int hi, int key) {
  while (lo < hi) {
    int mid = (lo + hi) >> 1;
    if (a[mid] < key) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// the same over 64-bit positions (tiles with 2^31 or more entries)
__device__ __forceinline__ int64_t lower_bound_g64(const int32_t* __restrict__ a, int64_t lo, int64_t hi, int key) {
  while (lo < hi) {
    const int64_t mid = lo + ((hi - lo) >> 1);
    if (a[mid] < key) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// multiplicative hash into a power-of-two table
template <int LOGT>
__device__ __forceinline__ unsigned hash_slot(int key) {
  return ((unsigned)key * 0x9E3779B1u) >> (32 - LOGT);
}

// ---- semirings (Semirings.h:212-255) ----
template <int SR>
struct Sem;
template <>
struct Sem<0> {  // PlusTimesSRing<double,double>
  static __device__ __forceinline__ double mul(double a, double b) { return a * b; }
  static __device__ __forceinline__ double identity() { return 0.0; }
  static __device__ __forceinline__ void lds_acc(double* p, double v) { atomicAdd(p, v); }
  static __device__ __forceinline__ double add(double a, double b) { return a + b; }
};
template <>
struct Sem<1> {  // MinPlusSRing<double,double>: multiply = inf_plus (Semirings.h:40-47), add = min
  static __device__ __forceinline__ double mul(double a, double b) {
    return (a == DBL_MAX || b == DBL_MAX) ? DBL_MAX : a + b;
  }
  // +inf as "empty" makes the first min() store the product exactly, like the
  // reference's first-insert (mtSpGEMM.h:410-414), also for an overflowing a+b.
  static __device__ __forceinline__ double identity() { return __builtin_inf(); }
  static __device__ __forceinline__ void lds_acc(double* p, double v) {
    __hip_atomic_fetch_min(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  static __device__ __forceinline__ double add(double a, double b) { return b < a ? b : a; }
};

// The same semirings accumulating exact integers in int32 LDS slots (IACC in
// cbg_local.hip: every product an integer of magnitude < 2^31, which the f64
// product v holds exactly)
template <int SR>
struct SemI;
template <>
struct SemI<0> {
  static __device__ __forceinline__ int identity() { return 0; }
  static __device__ __forceinline__ void lds_acc(int* p, double v) { atomicAdd(p, (int)v); }
};
template <>
struct SemI<1> {
  static __device__ __forceinline__ int identity() { return INT32_MAX; }
  static __device__ __forceinline__ void lds_acc(int* p, double v) { atomicMin(p, (int)v); }
};

// In-LDS bitonic sort of N (power of two) (key,val) pairs by key, ascending,
// by NT cooperating threads (tid in [0,NT)).  SYNC is a barrier functor.
template <int N, int NT, class SYNC>
__device__ __forceinline__ void bitonic_sort_kv(int* keys, double* vals, int tid, SYNC sync) {
#pragma unroll 1
  for (int k = 2; k <= N; k <<= 1) {
#pragma unroll 1
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int idx = tid; idx < N / 2; idx += NT) {
        int i = 2 * idx - (idx & (j - 1));
        int l = i + j;
        int ki = keys[i], kl = keys[l];
        bool up = (i & k) == 0;
        if ((ki > kl) == up) {
          keys[i] = kl;
          keys[l] = ki;
          double t = vals[i];
          vals[i] = vals[l];
          vals[l] = t;
        }
      }
      sync();
    }
  }
}

// Value of lane ^ D (D a power of two below 64) on the VALU: DPP inside rows
// (quad_perm for 1 and 2, row_half_mirror + quad reversal for 4, row_ror:8
// for 8) and gfx950's permlane swaps across rows (16, 32).  A __shfl_xor is a
// ds_bpermute: an LDS instruction shared by the CU's four SIMDs, which the
// wave sorts issued ~1200 of per wave (CBG_XOR_DPP=0 restores them).
#ifndef CBG_XOR_DPP
#define CBG_XOR_DPP 1
#endif
template <int D>
__device__ __forceinline__ int xor_lane(int v) {
#if CBG_XOR_DPP
  if constexpr (D == 1) {
    return __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xf, 0xf, false);  // quad_perm [1,0,3,2]
  } else if constexpr (D == 2) {
    return __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xf, 0xf, false);  // quad_perm [2,3,0,1]
  } else if constexpr (D == 4) {
    const int m = __builtin_amdgcn_update_dpp(0, v, 0x141, 0xf, 0xf, false);  // row_half_mirror: 7 - i
    return __builtin_amdgcn_update_dpp(0, m, 0x1B, 0xf, 0xf, false);         // quad_perm [3,2,1,0]
  } else if constexpr (D == 8) {
    return __builtin_amdgcn_update_dpp(0, v, 0x128, 0xf, 0xf, false);  // row_ror:8
  } else if constexpr (D == 16) {
    // odd rows of the first operand <-> even rows of the second: {r0 r0 r2 r2}, {r1 r1 r3 r3}
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return (threadIdx.x & 16) ? (int)r[0] : (int)r[1];
  } else {
    static_assert(D == 32, "xor distance");
    // upper half of the first operand <-> lower half of the second: {lo lo}, {hi hi}
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return (threadIdx.x & 32) ? (int)r[0] : (int)r[1];
  }
#else
  return __shfl_xor(v, D);
#endif
}
template <int D>
__device__ __forceinline__ double xor_lane(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = xor_lane<D>((int)b), hi = xor_lane<D>((int)(b >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
// runtime distance (unrolled loops make d a constant after inlining)
template <typename V>
__device__ __forceinline__ V xor_lane_d(V v, int d) {
  switch (d) {
    case 1: return xor_lane<1>(v);
    case 2: return xor_lane<2>(v);
    case 4: return xor_lane<4>(v);
    case 8: return xor_lane<8>(v);
    case 16: return xor_lane<16>(v);
    default: return xor_lane<32>(v);
  }
}

// Ascending bitonic sort of one (key, val) per lane across the 64 lanes of a
// wave, in registers (cross-lane swaps; no LDS, no barriers).  Used for the
// 64-slot wave tables; for 2-8 slots per lane the LDS sort was as fast.
__device__ __forceinline__ void wave_bitonic_sort_kv(int& key, double& val, int lane) {
#pragma unroll
  for (int k = 2; k <= WAVE; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      const int ok = xor_lane_d(key, j);
      const double ov = xor_lane_d(val, j);
      const bool up = (lane & k) == 0;     // this block of k lanes sorts ascending
      const bool lower = (lane & j) == 0;  // lower lane of the pair keeps the min when ascending
      if (lower == up ? ok < key : ok > key) {
        key = ok;
        val = ov;
      }
    }
  }
}

// Emit the n occupied slots of an LDS hash table (keys[T], vals[T]; empty =
// EMPTY_KEY) in ascending key order to out[obase ...] without a full sort:
// keys are bucketed by (key - lo) >> bshift into NB buckets (counting sort),
// and each entry's position inside its bucket is its rank among the few
// entries of that bucket.  O(T + n * bucket size) work, 3 barriers.
// Scratch: boff[NB+1], cur[NB] ints, members[n] (slot ids).
#ifndef CBG_EMIT_STAGE
#define CBG_EMIT_STAGE 0  // staged coalesced emit: -1.7 % at 22, -0.8 % at 18 (same box, 2 runs): scattered stores kept
#endif
template <int T, int BS, int NB, bool MOFF = false, bool STAGE = (CBG_EMIT_STAGE != 0)>
__device__ __forceinline__ void hash_emit_sorted(int* keys, double* vals, int lo, int bshift, int* boff,
                                                 int* cur, unsigned short* members, int* tmp,
                                                 int32_t* __restrict__ out_ir, double* __restrict__ out_val,
                                                 int64_t obase, unsigned short* moff = nullptr) {
  // MOFF: pass 2 also stores each entry's row offset inside its bucket
  // ((key - lo) mod 2^bshift, < 2^16), so the rank loop reads one u16 per
  // bucket member instead of a slot id and then that slot's key
  const int tid = threadIdx.x;
  const int omask = (1 << bshift) - 1;
  for (int b = tid; b < NB; b += BS) cur[b] = 0;
  __syncthreads();
  for (int j = tid; j < T; j += BS) {
    const int k = keys[j];
    if (k != EMPTY_KEY) atomicAdd(&cur[(k - lo) >> bshift], 1);
  }
  __syncthreads();
  // exclusive scan of the bucket counts
  const int total = block_ordered_scan<BS>(
      NB, [&](int b) { return cur[b]; },
      [&](int b, int x) {
        boff[b] = x;
        cur[b] = x;
      },
      tmp);
  if (tid == 0) boff[NB] = total;
  __syncthreads();
  for (int j = tid; j < T; j += BS) {
    const int k = keys[j];
    if (k != EMPTY_KEY) {
      const int pos = atomicAdd(&cur[(k - lo) >> bshift], 1);
      members[pos] = (unsigned short)j;
      if (MOFF) moff[pos] = (unsigned short)((k - lo) & omask);
    }
  }
  __syncthreads();
  auto rank_of = [&](int k) {
    const int b = (k - lo) >> bshift;
    int r = boff[b];
    const int e = boff[b + 1];
    if (MOFF) {
      const int mo = (k - lo) & omask;
      for (int q = boff[b]; q < e; ++q) r += (int)moff[q] < mo;
    } else {
      for (int q = boff[b]; q < e; ++q) r += keys[members[q]] < k;
    }
    return r;
  };
  // STAGE: every thread holds its entries' (rank, row, value) in registers,
  // then the table itself is overwritten in rank order and copied out with
  // coalesced stores (instead of one scattered store per entry); tables up
  // to load 2/3 (more entries: the scattered stores)
  constexpr int E = (2 * T / 3 + BS - 1) / BS;
  if (STAGE && total <= E * BS) {
    int rr[E], kk[E];
    double vv[E];
#pragma unroll
    for (int q = 0; q < E; ++q) {
      const int p = tid + q * BS;
      rr[q] = -1;
      if (p < total) {
        const int j = members[p];
        kk[q] = keys[j];
        vv[q] = vals[j];
        rr[q] = rank_of(kk[q]);
      }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < E; ++q)
      if (rr[q] >= 0) {
        keys[rr[q]] = kk[q];
        vals[rr[q]] = vv[q];
      }
    __syncthreads();
    for (int p = tid; p < total; p += BS) {
      st_emit(&out_ir[obase + p], keys[p]);
      st_emit(&out_val[obase + p], vals[p]);
    }
    return;
  }
  for (int p = tid; p < total; p += BS) {
    const int j = members[p];
    const int k = keys[j];
    const int r = rank_of(k);
    st_emit(&out_ir[obase + r], k);
    st_emit(&out_val[obase + r], vals[j]);
  }
}

// The same emit (MOFF) with each thread's slots kept in registers between the
// counting and the scatter pass: the counting pass's returning atomic gives
// every entry its index inside its bucket, so the scatter pass re-reads no key
// and needs no second atomic.  The rank pass still walks the bucket-ordered
// list (its output stores then land nearly in order: ranking each thread's
// own slots instead scatters the stores over the slab, 2.3x slower).
template <int T, int BS, int NB>
__device__ __forceinline__ void hash_emit_reg(const int* keys, const double* vals, int lo, int bshift, int* boff,
                                              int* cur, unsigned short* members, int* tmp, unsigned short* moff,
                                              int32_t* __restrict__ out_ir, double* __restrict__ out_val,
                                              int64_t obase) {
  constexpr int E = (T + BS - 1) / BS;
  const int tid = threadIdx.x;
  const int omask = (1 << bshift) - 1;
  for (int b = tid; b < NB; b += BS) cur[b] = 0;
  __syncthreads();
  int kk[E], ix[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int j = tid + e * BS;
    kk[e] = (T % BS == 0 || j < T) ? keys[j] : EMPTY_KEY;
    ix[e] = kk[e] != EMPTY_KEY ? atomicAdd(&cur[(kk[e] - lo) >> bshift], 1) : 0;
  }
  __syncthreads();
  const int total = block_ordered_scan<BS>(
      NB, [&](int b) { return cur[b]; }, [&](int b, int x) { boff[b] = x; }, tmp);
  if (tid == 0) boff[NB] = total;
  __syncthreads();
#pragma unroll
  for (int e = 0; e < E; ++e)
    if (kk[e] != EMPTY_KEY) {
      const int pos = boff[(kk[e] - lo) >> bshift] + ix[e];
      members[pos] = (unsigned short)(tid + e * BS);
      moff[pos] = (unsigned short)((kk[e] - lo) & omask);
    }
  __syncthreads();
  for (int p = tid; p < total; p += BS) {
    const int j = members[p];
    const int k = keys[j];
    const int b = (k - lo) >> bshift;
    const int mo = (k - lo) & omask;
    const int q0 = boff[b], q1 = boff[b + 1];
    int r = q0;
    for (int q = q0; q < q1; ++q) r += (int)moff[q] < mo;
    st_emit(&out_ir[obase + r], k);
    st_emit(&out_val[obase + r], vals[j]);
  }
}

struct WaveSync {
  __device__ __forceinline__ void operator()() const { wave_sync(); }
};
struct BlockSync {
  __device__ __forceinline__ void operator()() const { __syncthreads(); }
};

}  // namespace cbg
