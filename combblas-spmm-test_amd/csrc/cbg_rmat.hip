// cbg_rmat.hip -- Graph500 Kronecker R-MAT tiles generated on device.
//
// Reproduces, edge for edge, DistEdgeList::GenGraph500Data(packed=true,
// scramble=true) (reference DistEdgeList.cpp:223-280) -> RefGen21::make_graph /
// generate_kronecker_range / make_one_edge / scramble (RefGen21.h:185-304) on
// the graph500 MRG5 generator (graph500-1.2/generator/splittable_mrg.c), then
// SpParMat(DistEdgeList, false) (SpParMat.cpp:3140-3254: row = v0, col = v1,
// block distribution SpParMat::Owner :5068-5097), SpTuples(edges)
// (SpTuples.cpp:70-123: column-major sort, duplicates summed into the value)
// and RemoveLoops (SpParMat.cpp:3257-3272).
//
// Every edge is independent (the MRG state of edge e is A^(e*2^64) * seed), so
// one thread generates one edge; skip-ahead uses per-byte tables of powers of
// the 5x5 MRG transition matrix, built on the host by square-and-multiply
// (the role of the generated mrg_transitions.c table).

#include "cbg_device.h"
#include "cbg_internal.h"

namespace cbg {

static constexpr uint64_t MRG_P = 0x7FFFFFFFULL, MRG_X = 107374182ULL, MRG_Y = 104480ULL;
static constexpr int SKIP_BYTES = 5;  // edge index < 2^40

struct Mat5 {
  uint64_t a[5][5];
};
static Mat5 m5_mul(const Mat5& x, const Mat5& y) {
  Mat5 r;
  for (int i = 0; i < 5; ++i)
    for (int j = 0; j < 5; ++j) {
      uint64_t s = 0;
      for (int k = 0; k < 5; ++k) s = (s + x.a[i][k] * y.a[k][j]) % MRG_P;
      r.a[i][j] = s;
    }
  return r;
}
static Mat5 m5_id() {
  Mat5 r{};
  for (int i = 0; i < 5; ++i) r.a[i][i] = 1;
  return r;
}
static Mat5 m5_A() {  // mrg_orig_step: z1' = x z1 + y z5, shift down
  Mat5 r{};
  r.a[0][0] = MRG_X;
  r.a[0][4] = MRG_Y;
  for (int i = 1; i < 5; ++i) r.a[i][i - 1] = 1;
  return r;
}
static Mat5 m5_pow(Mat5 m, uint64_t e) {
  Mat5 r = m5_id();
  while (e) {
    if (e & 1) r = m5_mul(r, m);
    m = m5_mul(m, m);
    e >>= 1;
  }
  return r;
}
static void m5_apply(const Mat5& m, uint64_t z[5]) {
  uint64_t o[5];
  for (int i = 0; i < 5; ++i) {
    uint64_t s = 0;
    for (int k = 0; k < 5; ++k) s = (s + m.a[i][k] * z[k]) % MRG_P;
    o[i] = s;
  }
  for (int i = 0; i < 5; ++i) z[i] = o[i];
}
static uint32_t mrg_next(uint64_t z[5]) {
  uint64_t n = (MRG_X * z[0] + MRG_Y * z[4]) % MRG_P;
  z[4] = z[3];
  z[3] = z[2];
  z[2] = z[1];
  z[1] = z[0];
  z[0] = n;
  return (uint32_t)n;
}

struct SkipTables {
  uint32_t* dev = nullptr;  // [SKIP_BYTES][256][25]
  Mat5 skip50_7;
};
static SkipTables& skip_tables() {
  static SkipTables t;
  static std::once_flag once;
  std::call_once(once, [] {
    std::vector<uint32_t> h((size_t)SKIP_BYTES * 256 * 25);
    Mat5 base = m5_pow(m5_pow(m5_A(), 1ULL << 32), 1ULL << 32);  // A^(2^64)
    Mat5 p64 = base;
    for (int b = 0; b < SKIP_BYTES; ++b) {
      Mat5 cur = m5_id();
      for (int v = 0; v < 256; ++v) {
        for (int i = 0; i < 25; ++i) h[((size_t)b * 256 + v) * 25 + i] = (uint32_t)cur.a[i / 5][i % 5];
        cur = m5_mul(cur, base);
      }
      base = m5_pow(base, 256);
    }
    Mat5 p128 = m5_pow(m5_pow(p64, 1ULL << 32), 1ULL << 32);
    t.skip50_7 = m5_mul(m5_pow(p128, 50), m5_pow(p64, 7));  // mrg_skip(50, 7, 0), RefGen21.h:230
    CBG_HIP(hipMalloc(&t.dev, h.size() * sizeof(uint32_t)));
    CBG_HIP(hipMemcpy(t.dev, h.data(), h.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
  });
  return t;
}

__device__ __forceinline__ uint32_t mod_p(uint64_t x) {  // x < 2^63
  x = (x & 0x7FFFFFFFULL) + (x >> 31);
  x = (x & 0x7FFFFFFFULL) + (x >> 31);
  return (uint32_t)(x >= 0x7FFFFFFFULL ? x - 0x7FFFFFFFULL : x);
}
__device__ __forceinline__ uint64_t bitrev64_d(uint64_t x) { return __builtin_bitreverse64(x); }
__device__ __forceinline__ int64_t scramble_d(int64_t v0, int lgN, uint64_t val0, uint64_t val1) {
  uint64_t v = (uint64_t)v0;
  v += val0 + val1;
  v *= (val0 | 0x4519840211493211ULL);
  v = bitrev64_d(v) >> (64 - lgN);
  v *= (val1 | 0x3050852102C843A5ULL);
  v = bitrev64_d(v) >> (64 - lgN);
  return (int64_t)v;
}

struct RmatParams {
  uint32_t seed[5];
  uint64_t val0, val1;
  int scale;
  int pr, pc, prow, pcol;
  int64_t mper, nper;
  unsigned long long drop_key;  // key of a dropped edge (loop / other tile): sorts last
};
// mask of the bits of values in [0, maxval]
static unsigned long long rmat_bits(unsigned long long maxval) {
  unsigned long long m = 0;
  while (m < maxval) m = (m << 1) | 1ull;
  return m;
}

// keys of this tile's edges, appended in any order (the sort follows); dropped
// edges (loops, other tiles) are not written -- 7/8 of a 2x4 grid's edges,
// whose one long run of equal keys would serialize a reduce-by-key thread
__global__ __launch_bounds__(256) void k_rmat_edges(int64_t e0, int64_t ne, const uint32_t* __restrict__ tab,
                                                    RmatParams P, unsigned long long* __restrict__ keys,
                                                    unsigned long long* __restrict__ nkept) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t >= ne) return;
  const uint64_t ei = (uint64_t)(e0 + t);
  uint32_t z[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) z[i] = P.seed[i];
  // mrg_skip(state, 0, ei, 0): state <- A^(ei * 2^64) state (splittable_mrg.c:202-216)
  for (int b = 0; b < SKIP_BYTES; ++b) {
    const unsigned v = (unsigned)((ei >> (8 * b)) & 0xFF);
    if (!v) continue;
    const uint32_t* M = tab + ((size_t)b * 256 + v) * 25;
    uint32_t o[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      uint64_t s = 0;  // reduce per term: s < 2^31, M*z < 2^62
#pragma unroll
      for (int k = 0; k < 5; ++k) s = mod_p(s + (uint64_t)M[i * 5 + k] * z[k]);
      o[i] = (uint32_t)s;
    }
#pragma unroll
    for (int i = 0; i < 5; ++i) z[i] = o[i];
  }
  // make_one_edge (RefGen21.h:199-225) with generate_4way_bernoulli (:102-125)
  int64_t nverts = (int64_t)1 << P.scale, bs = 0, bt = 0;
  const uint32_t limit = 0xFFFFFFFFu % 10000u;
  while (nverts > 1) {
    uint32_t val;
    do {
      const uint32_t nz = mod_p((uint64_t)MRG_X * z[0] + (uint64_t)MRG_Y * z[4]);
      z[4] = z[3];
      z[3] = z[2];
      z[2] = z[1];
      z[1] = z[0];
      z[0] = nz;
      val = nz;
    } while (val < limit);
    val %= 10000u;
    int sq;
    if (val < 1900u) sq = 1;
    else if (val < 3800u) sq = 2;
    else if (val < 9500u) sq = 0;
    else sq = 3;
    int so = sq / 2, to = sq % 2;
    if (bs == bt && so > to) {
      const int x = so;
      so = to;
      to = x;
    }
    nverts /= 2;
    bs += nverts * so;
    bt += nverts * to;
  }
  const int64_t src = scramble_d(bs, P.scale, P.val0, P.val1);
  const int64_t dst = scramble_d(bt, P.scale, P.val0, P.val1);
  unsigned long long key = P.drop_key;  // sorts after every kept edge
  if (src != dst) {  // RemoveLoops
    const int orow = P.mper ? (int)min(src / P.mper, (int64_t)P.pr - 1) : P.pr - 1;
    const int ocol = P.nper ? (int)min(dst / P.nper, (int64_t)P.pc - 1) : P.pc - 1;
    if (orow == P.prow && ocol == P.pcol) {
      const uint64_t lr = (uint64_t)(src - (int64_t)orow * P.mper), lc = (uint64_t)(dst - (int64_t)ocol * P.nper);
      key = (lc << 32) | lr;
    }
  }
  const bool kept = key != P.drop_key;
  const unsigned long long m = __ballot(kept);  // one atomic per wave
  if (m) {
    const int lane = lane_id(), leader = __ffsll((long long)m) - 1;
    unsigned long long base = 0;
    if (lane == leader) base = atomicAdd(nkept, (unsigned long long)__popcll(m));
    base = __shfl(base, leader);
    if (kept) keys[base + __popcll(m & ((1ull << lane) - 1ull))] = key;
  }
}

__global__ void k_rmat_flags(int64_t n, const unsigned long long* __restrict__ uk, int64_t* __restrict__ flag) {
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < n) flag[i] = (i == 0 || (uk[i] >> 32) != (uk[i - 1] >> 32)) ? 1 : 0;
}
__global__ void k_ones(int64_t n, double* __restrict__ v) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < n) v[i] = 1.0;
}
__global__ void k_rmat_fill(int64_t n, const unsigned long long* __restrict__ uk, const double* __restrict__ cnt,
                            const int64_t* __restrict__ pos, int32_t* __restrict__ ir, double* __restrict__ val,
                            int32_t* __restrict__ jc, int64_t* __restrict__ cp) {
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  ir[i] = (int32_t)(uk[i] & 0xFFFFFFFFULL);
  val[i] = cnt[i];  // multiplicity of the edge (SpTuples.cpp:95-101)
  if (i == 0 || (uk[i] >> 32) != (uk[i - 1] >> 32)) {
    jc[pos[i]] = (int32_t)(uk[i] >> 32);
    cp[pos[i]] = i;
  }
}

void rmat_tile(int scale, int ef, uint64_t userseed, int pr, int pc, int prow, int pcol, cbg_tile& out, hipStream_t s) {
  SkipTables& tb = skip_tables();
  RmatParams P;
  // make_mrg_seed(userseed, userseed) (graph500 utils.c:83-89, RefGen21.h:279-282)
  uint64_t z[5] = {(userseed & 0x3FFFFFFF) + 1, ((userseed >> 30) & 0x3FFFFFFF) + 1, (userseed & 0x3FFFFFFF) + 1,
                   ((userseed >> 30) & 0x3FFFFFFF) + 1, ((userseed >> 60) << 4) + (userseed >> 60) + 1};
  for (int i = 0; i < 5; ++i) P.seed[i] = (uint32_t)z[i];
  uint64_t ns[5] = {z[0], z[1], z[2], z[3], z[4]};
  m5_apply(tb.skip50_7, ns);  // MakeScrambleValues (RefGen21.h:227-240)
  uint64_t v0 = mrg_next(ns);
  v0 *= 0xFFFFFFFFULL;
  v0 += mrg_next(ns);
  uint64_t v1 = mrg_next(ns);
  v1 *= 0xFFFFFFFFULL;
  v1 += mrg_next(ns);
  P.val0 = v0;
  P.val1 = v1;
  P.scale = scale;
  P.pr = pr;
  P.pc = pc;
  P.prow = prow;
  P.pcol = pcol;
  const int64_t nv = (int64_t)1 << scale;
  P.mper = nv / pr;
  P.nper = nv / pc;
  const int64_t M = nv * ef;
  const int64_t lm = (prow == pr - 1) ? nv - prow * P.mper : P.mper;
  const int64_t ln = (pcol == pc - 1) ? nv - pcol * P.nper : P.nper;
  // keys (local col << 32 | local row); dropped edges (loops, other tiles) get
  // column ln, one past the tile, so they sort last; the radix sort only runs
  // over the bits these keys can use
  P.drop_key = (unsigned long long)ln << 32;
  const unsigned long long varying = (rmat_bits((unsigned long long)ln) << 32) | rmat_bits((unsigned long long)(lm - 1));

  // edges -> (key, 1.0); sort; duplicates summed = the multiplicities
  // (cbg_sort.hip: the repo's radix sort and reduce-by-key, 64-bit counts)
  DBuf<unsigned long long> k0(M), nk(1);
  CBG_HIP(hipMemsetAsync(nk.p, 0, sizeof(unsigned long long), s));
  hipLaunchKernelGGL(k_rmat_edges, dim3((unsigned)((M + 255) / 256)), dim3(256), 0, s, (int64_t)0, M, tb.dev, P, k0.p,
                     nk.p);
  unsigned long long kept = 0;
  CBG_HIP(hipMemcpyAsync(&kept, nk.p, sizeof(kept), hipMemcpyDeviceToHost, s));
  CBG_HIP(hipStreamSynchronize(s));
  const int64_t E = (int64_t)kept;
  DBuf<unsigned long long> uk(std::max<int64_t>(E, 1));
  DBuf<double> w0(std::max<int64_t>(E, 1)), uv(std::max<int64_t>(E, 1));
  if (E > 0) hipLaunchKernelGGL(k_ones, dim3((unsigned)((E + 255) / 256)), dim3(256), 0, s, E, w0.p);
  radix_sort_pairs<unsigned long long>(k0, w0, E, varying, s);
  const int64_t runs = reduce_by_key<unsigned long long>(k0.p, w0.p, E, CBG_PLUS_TIMES, uk.p, uv.p, s);
  k0.release();
  w0.release();
  const int64_t nnz = runs;
  DBuf<int64_t> flag(nnz + 1), pos(nnz + 1);
  hipLaunchKernelGGL(k_rmat_flags, dim3((unsigned)((nnz + 255) / 256 + 1)), dim3(256), 0, s, nnz, uk.p, flag.p);
  exclusive_scan_i64(flag.p, pos.p, nnz, s);
  int64_t nzc = 0;
  CBG_HIP(hipMemcpyAsync(&nzc, pos.p + nnz, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  CBG_HIP(hipStreamSynchronize(s));
  tile_alloc_device(out, lm, ln, nnz, nzc);
  if (nnz > 0)
    hipLaunchKernelGGL(k_rmat_fill, dim3((unsigned)((nnz + 255) / 256)), dim3(256), 0, s, nnz, uk.p, uv.p, pos.p,
                       out.ir, out.val, out.jc, out.cp);
  CBG_HIP(hipMemcpyAsync(out.cp + nzc, &nnz, sizeof(int64_t), hipMemcpyHostToDevice, s));
  CBG_HIP(hipStreamSynchronize(s));
}

}  // namespace cbg
