/* cbg_oracle.c -- TEST INFRASTRUCTURE ONLY (see cbg_oracle.h).
 *
 * Plain-C restatement of the reference CombBLAS 2D-SUMMA SpGEMM hot path.
 * Every function cites the reference file:line it follows.  Parity of this
 * restatement is pinned by tests/test_oracle.py against tests/golden/, which
 * the reference itself produced (oracle/_ref).  Only tests/, smoke() and
 * bench.py's cpu_baseline use it; the product path never does.
 */
#define _GNU_SOURCE
#include "cbg_oracle.h"

#include <float.h>
#include <math.h>
#include <omp.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* Graph500 MRG5 generator (graph500-1.2/generator/splittable_mrg.c:19-60,   */
/* mod_arith_64bit.h) restated with full 5x5 transition matrices mod 2^31-1. */
/* ------------------------------------------------------------------------ */
#define MRG_P 0x7FFFFFFFULL
#define MRG_X 107374182ULL
#define MRG_Y 104480ULL

typedef struct { uint64_t a[5][5]; } mat5;
typedef struct { uint64_t z[5]; } mrg5;

static mat5 mat5_mul(const mat5* x, const mat5* y) {
  mat5 r;
  for (int i = 0; i < 5; ++i)
    for (int j = 0; j < 5; ++j) {
      uint64_t s = 0;
      for (int k = 0; k < 5; ++k) s = (s + x->a[i][k] * y->a[k][j]) % MRG_P;
      r.a[i][j] = s;
    }
  return r;
}
static mat5 mat5_identity(void) {
  mat5 r;
  memset(&r, 0, sizeof r);
  for (int i = 0; i < 5; ++i) r.a[i][i] = 1;
  return r;
}
/* one step of mrg_orig_step (splittable_mrg.c:190-198): z1' = x z1 + y z5, shift */
static mat5 mat5_A(void) {
  mat5 r;
  memset(&r, 0, sizeof r);
  r.a[0][0] = MRG_X;
  r.a[0][4] = MRG_Y;
  for (int i = 1; i < 5; ++i) r.a[i][i - 1] = 1;
  return r;
}
static mat5 mat5_pow(mat5 m, uint64_t e) {
  mat5 r = mat5_identity();
  while (e) {
    if (e & 1) r = mat5_mul(&r, &m);
    m = mat5_mul(&m, &m);
    e >>= 1;
  }
  return r;
}
static void mat5_apply(const mat5* m, mrg5* s) {
  uint64_t o[5];
  for (int i = 0; i < 5; ++i) {
    uint64_t acc = 0;
    for (int k = 0; k < 5; ++k) acc = (acc + m->a[i][k] * s->z[k]) % MRG_P;
    o[i] = acc;
  }
  memcpy(s->z, o, sizeof o);
}
static inline uint32_t mrg_get_uint_orig(mrg5* s) { /* splittable_mrg.c:280-283 */
  uint64_t n = (MRG_X * s->z[0] + MRG_Y * s->z[4]) % MRG_P;
  s->z[4] = s->z[3];
  s->z[3] = s->z[2];
  s->z[2] = s->z[1];
  s->z[1] = s->z[0];
  s->z[0] = n;
  return (uint32_t)n;
}

/* skip tables: A^(v * 256^b * 2^64) for b = 0..7, v = 0..255 (the role of
 * mrg_skip_matrices[8+b][v] in mrg_skip, splittable_mrg.c:202-216) */
static mat5 g_skip_50_7;
static mat5* skip_tables(void) {
  static mat5* tab = NULL;
  if (tab) return tab;
#pragma omp critical(ocbg_skip)
  {
    if (!tab) {
      mat5* t = (mat5*)malloc(sizeof(mat5) * 8 * 256);
      mat5 base = mat5_pow(mat5_A(), 1ULL << 32);
      base = mat5_pow(base, 1ULL << 32); /* A^(2^64) */
      for (int b = 0; b < 8; ++b) {
        t[b * 256] = mat5_identity();
        for (int v = 1; v < 256; ++v) t[b * 256 + v] = mat5_mul(&t[b * 256 + v - 1], &base);
        base = mat5_pow(base, 256);
      }
      /* skip(50, 7, 0) = 50 * 2^128 + 7 * 2^64 (RefGen21.h:230) */
      mat5 p64 = mat5_pow(mat5_pow(mat5_A(), 1ULL << 32), 1ULL << 32);
      mat5 p128 = mat5_pow(mat5_pow(p64, 1ULL << 32), 1ULL << 32);
      mat5 a = mat5_pow(p128, 50), b = mat5_pow(p64, 7);
      g_skip_50_7 = mat5_mul(&a, &b);
      tab = t;
    }
  }
  return tab;
}
static void mrg_skip_mid(mrg5* s, uint64_t e) { /* mrg_skip(state, 0, e, 0) */
  mat5* t = skip_tables();
  for (int b = 0; e; ++b, e >>= 8) {
    unsigned v = (unsigned)(e & 0xFF);
    if (v) mat5_apply(&t[b * 256 + v], s);
  }
}

/* make_mrg_seed (graph500 utils.c:83-89) with userseed1 == userseed2, as in
 * RefGen21::make_graph (RefGen21.h:279-282) */
static void make_seed(uint64_t u, mrg5* s) {
  s->z[0] = (u & 0x3FFFFFFF) + 1;
  s->z[1] = ((u >> 30) & 0x3FFFFFFF) + 1;
  s->z[2] = (u & 0x3FFFFFFF) + 1;
  s->z[3] = ((u >> 30) & 0x3FFFFFFF) + 1;
  s->z[4] = ((u >> 60) << 4) + (u >> 60) + 1;
}

static inline uint64_t bitrev64(uint64_t x) { /* RefGen21::bitreverse, RefGen21.h:127-178 */
  x = __builtin_bswap64(x);
  x = ((x >> 4) & 0x0F0F0F0F0F0F0F0FULL) | ((x & 0x0F0F0F0F0F0F0F0FULL) << 4);
  x = ((x >> 2) & 0x3333333333333333ULL) | ((x & 0x3333333333333333ULL) << 2);
  x = ((x >> 1) & 0x5555555555555555ULL) | ((x & 0x5555555555555555ULL) << 1);
  return x;
}
static inline int64_t scramble(int64_t v0, int lgN, uint64_t val0, uint64_t val1) { /* RefGen21.h:185-196 */
  uint64_t v = (uint64_t)v0;
  v += val0 + val1;
  v *= (val0 | 0x4519840211493211ULL);
  v = bitrev64(v) >> (64 - lgN);
  v *= (val1 | 0x3050852102C843A5ULL);
  v = bitrev64(v) >> (64 - lgN);
  return (int64_t)v;
}
static inline int bernoulli4(mrg5* st) { /* RefGen21.h:102-125, SPK_NOISE_LEVEL 0 */
  const uint32_t limit = 0xFFFFFFFFu % 10000u;
  uint32_t val = mrg_get_uint_orig(st);
  while (val < limit) val = mrg_get_uint_orig(st);
  val %= 10000u;
  if (val < 1900u) return 1;
  val -= 1900u;
  if (val < 1900u) return 2;
  val -= 1900u;
  if (val < 5700u) return 0;
  return 3;
}

void ocbg_rmat_edges(int scale, int64_t e0, int64_t e1, uint64_t userseed, int64_t* src, int64_t* dst) {
  /* RefGen21::generate_kronecker_range (RefGen21.h:246-262) + make_one_edge (:199-225) */
  mrg5 state;
  make_seed(userseed, &state);
  skip_tables();
  mrg5 ns = state;
  mat5_apply(&g_skip_50_7, &ns); /* MakeScrambleValues, RefGen21.h:227-240 */
  uint64_t val0 = mrg_get_uint_orig(&ns);
  val0 *= 0xFFFFFFFFULL;
  val0 += mrg_get_uint_orig(&ns);
  uint64_t val1 = mrg_get_uint_orig(&ns);
  val1 *= 0xFFFFFFFFULL;
  val1 += mrg_get_uint_orig(&ns);
#pragma omp parallel for schedule(static)
  for (int64_t ei = e0; ei < e1; ++ei) {
    mrg5 st = state;
    mrg_skip_mid(&st, (uint64_t)ei);
    int64_t nverts = (int64_t)1 << scale, bs = 0, bt = 0;
    while (nverts > 1) {
      int sq = bernoulli4(&st);
      int so = sq / 2, to = sq % 2;
      if (bs == bt && so > to) { int t = so; so = to; to = t; }
      nverts /= 2;
      bs += nverts * so;
      bt += nverts * to;
    }
    src[ei - e0] = scramble(bs, scale, val0, val1);
    dst[ei - e0] = scramble(bt, scale, val0, val1);
  }
}

/* LSD radix sort of 64-bit keys, 16-bit digits */
static void radix_sort_u64(uint64_t* a, int64_t n, int bits) {
  uint64_t* buf = (uint64_t*)malloc(sizeof(uint64_t) * (n > 0 ? n : 1));
  int64_t* cnt = (int64_t*)malloc(sizeof(int64_t) * 65536);
  uint64_t *src = a, *dst = buf;
  for (int sh = 0; sh < bits; sh += 16) {
    memset(cnt, 0, sizeof(int64_t) * 65536);
    for (int64_t i = 0; i < n; ++i) cnt[(src[i] >> sh) & 0xFFFF]++;
    int64_t s = 0;
    for (int d = 0; d < 65536; ++d) { int64_t c = cnt[d]; cnt[d] = s; s += c; }
    for (int64_t i = 0; i < n; ++i) dst[cnt[(src[i] >> sh) & 0xFFFF]++] = src[i];
    uint64_t* t = src; src = dst; dst = t;
  }
  if (src != a) memcpy(a, src, sizeof(uint64_t) * n);
  free(buf);
  free(cnt);
}

void ocbg_free(ocbg_tile* t) {
  free(t->cp); free(t->jc); free(t->ir); free(t->val);
  memset(t, 0, sizeof *t);
}

static void tile_alloc(ocbg_tile* t, int64_t m, int64_t n, int64_t nnz, int64_t nzc) {
  t->m = m; t->n = n; t->nnz = nnz; t->nzc = nzc;
  t->cp = (int64_t*)calloc((size_t)nzc + 1, sizeof(int64_t));
  t->jc = (int32_t*)malloc(sizeof(int32_t) * (size_t)(nzc > 0 ? nzc : 1));
  t->ir = (int32_t*)malloc(sizeof(int32_t) * (size_t)(nnz > 0 ? nnz : 1));
  t->val = (double*)malloc(sizeof(double) * (size_t)(nnz > 0 ? nnz : 1));
}

int ocbg_rmat_tile(int scale, int ef, uint64_t userseed, int nthreads, ocbg_tile* out) {
  if (nthreads > 0) omp_set_num_threads(nthreads);
  int64_t nv = (int64_t)1 << scale, M = nv * ef;
  int64_t* s = (int64_t*)malloc(sizeof(int64_t) * M);
  int64_t* d = (int64_t*)malloc(sizeof(int64_t) * M);
  ocbg_rmat_edges(scale, 0, M, userseed, s, d);
  /* SpParMat(DistEdgeList) -> SpTuples(edges): row = v0, col = v1 (SpParMat.cpp:3176-3184),
   * sort column-major, sum duplicates (SpTuples.cpp:70-123); RemoveLoops (SpParMat.cpp:3257) */
  uint64_t* key = (uint64_t*)malloc(sizeof(uint64_t) * M);
  for (int64_t i = 0; i < M; ++i) key[i] = ((uint64_t)d[i] << 32) | (uint64_t)s[i];
  free(s); free(d);
  radix_sort_u64(key, M, 64);
  int64_t nnz = 0, nzc = 0;
  for (int64_t i = 0; i < M;) {
    int64_t j = i + 1;
    while (j < M && key[j] == key[i]) ++j;
    uint32_t r = (uint32_t)key[i], c = (uint32_t)(key[i] >> 32);
    if (r != c) nnz++;
    i = j;
  }
  tile_alloc(out, nv, nv, nnz, 0);
  int64_t p = 0;
  int64_t lastc = -1;
  int64_t* cpt = (int64_t*)malloc(sizeof(int64_t) * (nnz + 1));
  int32_t* jct = (int32_t*)malloc(sizeof(int32_t) * (nnz > 0 ? nnz : 1));
  for (int64_t i = 0; i < M;) {
    int64_t j = i + 1;
    while (j < M && key[j] == key[i]) ++j;
    uint32_t r = (uint32_t)key[i], c = (uint32_t)(key[i] >> 32);
    if (r != c) {
      if ((int64_t)c != lastc) { jct[nzc] = (int32_t)c; cpt[nzc] = p; nzc++; lastc = c; }
      out->ir[p] = (int32_t)r;
      out->val[p] = (double)(j - i);
      p++;
    }
    i = j;
  }
  cpt[nzc] = p;
  free(key);
  free(out->cp); free(out->jc);
  out->cp = (int64_t*)realloc(cpt, sizeof(int64_t) * (nzc + 1));
  out->jc = jct;
  out->nzc = nzc;
  return 0;
}

/* ------------------------------------------------------------------------ */
/* Semirings (Semirings.h:212-255)                                           */
/* ------------------------------------------------------------------------ */
static inline double sr_mul(int sr, double a, double b) {
  if (sr == OCBG_MIN_PLUS) return (a == DBL_MAX || b == DBL_MAX) ? DBL_MAX : a + b; /* inf_plus :40-47 */
  return a * b;
}
static inline double sr_add(int sr, double a, double b) {
  if (sr == OCBG_MIN_PLUS) return a < b ? a : b; /* std::min(arg1,arg2) */
  return a + b;
}

/* ------------------------------------------------------------------------ */
/* Local SpGEMM                                                              */
/* ------------------------------------------------------------------------ */
/* Dense column lookup for A: the role of Dcsc::ConstructAux / FillColInds
 * (dcsc.cpp:982-1013, 1280-1343): B's row index k -> [start,end) of A(:,k). */
typedef struct { int64_t* start; int32_t* len; } colmap;
static colmap build_colmap(const ocbg_tile* A) {
  colmap c;
  c.start = (int64_t*)calloc((size_t)A->n + 1, sizeof(int64_t));
  c.len = (int32_t*)calloc((size_t)A->n + 1, sizeof(int32_t));
  for (int64_t i = 0; i < A->nzc; ++i) {
    c.start[A->jc[i]] = A->cp[i];
    c.len[A->jc[i]] = (int32_t)(A->cp[i + 1] - A->cp[i]);
  }
  return c;
}
static void free_colmap(colmap* c) { free(c->start); free(c->len); }

int ocbg_symbolic(const ocbg_tile* A, const ocbg_tile* B, int64_t* flops, int64_t* nnzc, int nthreads) {
  if (nthreads > 0) omp_set_num_threads(nthreads);
  if (A->nnz == 0 || B->nnz == 0) {
    for (int64_t i = 0; i < B->nzc; ++i) flops[i] = nnzc[i] = 0;
    return 0;
  }
  colmap cm = build_colmap(A);
#pragma omp parallel
  {
    int64_t cap = 0;
    int64_t* ht = NULL;
#pragma omp for schedule(dynamic, 64)
    for (int64_t i = 0; i < B->nzc; ++i) {
      int64_t f = 0; /* estimateFLOP, mtSpGEMM.h:1120-1124 */
      for (int64_t p = B->cp[i]; p < B->cp[i + 1]; ++p) f += cm.len[B->ir[p]];
      flops[i] = f;
      int64_t hs = 16; /* estimateNNZ_Hash, mtSpGEMM.h:880-925 */
      while (hs < f) hs <<= 1;
      if (hs > cap) { free(ht); cap = hs; ht = (int64_t*)malloc(sizeof(int64_t) * cap); }
      for (int64_t j = 0; j < hs; ++j) ht[j] = -1;
      int64_t cnt = 0;
      for (int64_t p = B->cp[i]; p < B->cp[i + 1]; ++p) {
        int64_t k = B->ir[p];
        for (int64_t q = cm.start[k]; q < cm.start[k] + cm.len[k]; ++q) {
          int64_t key = A->ir[q];
          int64_t h = (key * 107) & (hs - 1);
          while (1) {
            if (ht[h] == key) break;
            if (ht[h] == -1) { ht[h] = key; cnt++; break; }
            h = (h + 1) & (hs - 1);
          }
        }
      }
      nnzc[i] = cnt;
    }
    free(ht);
  }
  free_colmap(&cm);
  return 0;
}

typedef struct { int32_t key; int32_t runr; double num; } heapent; /* HeapEntry.h:36-56 */
static inline void heap_sift_down(heapent* h, int64_t n, int64_t i) {
  for (;;) {
    int64_t l = 2 * i + 1, r = l + 1, s = i;
    if (l < n && h[l].key < h[s].key) s = l;
    if (r < n && h[r].key < h[s].key) s = r;
    if (s == i) return;
    heapent t = h[i]; h[i] = h[s]; h[s] = t;
    i = s;
  }
}
static inline void heap_sift_up(heapent* h, int64_t i) {
  while (i > 0) {
    int64_t p = (i - 1) / 2;
    if (h[p].key <= h[i].key) return;
    heapent t = h[i]; h[i] = h[p]; h[p] = t;
    i = p;
  }
}
typedef struct { int32_t key; double val; } hashent;
static int cmp_hashent(const void* a, const void* b) {
  int32_t x = ((const hashent*)a)->key, y = ((const hashent*)b)->key;
  return (x > y) - (x < y);
}

/* heap k-way merge of one column (mtSpGEMM.h:311-360); returns entries written */
static int64_t col_heap(const ocbg_tile* A, const ocbg_tile* B, const colmap* cm, int64_t i, int sr,
                        heapent* wset, int64_t* cur, int64_t* end, int32_t* oir, double* oval) {
  int64_t nb = B->cp[i + 1] - B->cp[i], hsize = 0;
  for (int64_t j = 0; j < nb; ++j) {
    int64_t k = B->ir[B->cp[i] + j];
    cur[j] = cm->start[k];
    end[j] = cm->start[k] + cm->len[k];
    if (cur[j] != end[j]) {
      wset[hsize].key = A->ir[cur[j]];
      wset[hsize].runr = (int32_t)j;
      wset[hsize].num = A->val[cur[j]];
      hsize++;
    }
  }
  for (int64_t j = hsize / 2 - 1; j >= 0; --j) heap_sift_down(wset, hsize, j);
  int64_t out = 0;
  while (hsize > 0) {
    heapent top = wset[0];
    int32_t locb = top.runr;
    double mrhs = sr_mul(sr, top.num, B->val[B->cp[i] + locb]);
    if (out > 0 && oir[out - 1] == top.key)
      oval[out - 1] = sr_add(sr, oval[out - 1], mrhs);
    else {
      oir[out] = top.key;
      oval[out] = mrhs;
      out++;
    }
    if (++cur[locb] != end[locb]) {
      wset[0].key = A->ir[cur[locb]];
      wset[0].num = A->val[cur[locb]];
      heap_sift_down(wset, hsize, 0);
    } else {
      wset[0] = wset[hsize - 1];
      hsize--;
      heap_sift_down(wset, hsize, 0);
    }
  }
  return out;
}

/* hash accumulate of one column (mtSpGEMM.h:362-440) */
static int64_t col_hash(const ocbg_tile* A, const ocbg_tile* B, const colmap* cm, int64_t i, int sr,
                        int64_t nnzcol, hashent* ht, int32_t* oir, double* oval) {
  int64_t hs = 16;
  while (hs < nnzcol) hs <<= 1;
  for (int64_t j = 0; j < hs; ++j) ht[j].key = -1;
  for (int64_t p = B->cp[i]; p < B->cp[i + 1]; ++p) {
    int64_t k = B->ir[p];
    double bv = B->val[p];
    for (int64_t q = cm->start[k]; q < cm->start[k] + cm->len[k]; ++q) {
      double mrhs = sr_mul(sr, A->val[q], bv);
      int64_t key = A->ir[q];
      int64_t h = (key * 107) & (hs - 1);
      while (1) {
        if (ht[h].key == key) { ht[h].val = sr_add(sr, mrhs, ht[h].val); break; }
        if (ht[h].key == -1) { ht[h].key = (int32_t)key; ht[h].val = mrhs; break; }
        h = (h + 1) & (hs - 1);
      }
    }
  }
  int64_t idx = 0;
  for (int64_t j = 0; j < hs; ++j)
    if (ht[j].key != -1) ht[idx++] = ht[j];
  qsort(ht, (size_t)idx, sizeof(hashent), cmp_hashent);
  for (int64_t j = 0; j < idx; ++j) { oir[j] = ht[j].key; oval[j] = ht[j].val; }
  return idx;
}

/* builds DCSC C from per-B-column counts + filled ir/val (compacts empty columns) */
static void finish_tile(const ocbg_tile* A, const ocbg_tile* B, const int64_t* colptr, int32_t* ir, double* val,
                        ocbg_tile* C) {
  int64_t nzc = 0;
  for (int64_t i = 0; i < B->nzc; ++i) nzc += (colptr[i + 1] > colptr[i]);
  C->m = A->m; C->n = B->n; C->nnz = colptr[B->nzc]; C->nzc = nzc;
  C->cp = (int64_t*)malloc(sizeof(int64_t) * (nzc + 1));
  C->jc = (int32_t*)malloc(sizeof(int32_t) * (nzc > 0 ? nzc : 1));
  C->ir = ir;
  C->val = val;
  int64_t c = 0;
  for (int64_t i = 0; i < B->nzc; ++i)
    if (colptr[i + 1] > colptr[i]) { C->jc[c] = B->jc[i]; C->cp[c] = colptr[i]; c++; }
  C->cp[nzc] = colptr[B->nzc];
}

static int local_mult(const ocbg_tile* A, const ocbg_tile* B, int sr, int nthreads, int hybrid, ocbg_tile* C) {
  if (nthreads > 0) omp_set_num_threads(nthreads);
  if (A->nnz == 0 || B->nnz == 0) { /* mtSpGEMM.h:224-227 */
    tile_alloc(C, A->m, B->n, 0, 0);
    return 0;
  }
  int64_t nz = B->nzc;
  int64_t* flops = (int64_t*)malloc(sizeof(int64_t) * (nz + 1));
  int64_t* cnt = (int64_t*)malloc(sizeof(int64_t) * (nz + 1));
  ocbg_symbolic(A, B, flops, cnt, nthreads); /* estimateFLOP + estimateNNZ_Hash (:253-259) */
  int64_t* colptr = (int64_t*)malloc(sizeof(int64_t) * (nz + 1));
  colptr[0] = 0; /* prefixsum (:23-70) */
  for (int64_t i = 0; i < nz; ++i) colptr[i + 1] = colptr[i] + cnt[i];
  int64_t nnzc = colptr[nz];
  int32_t* ir = (int32_t*)malloc(sizeof(int32_t) * (nnzc > 0 ? nnzc : 1));
  double* val = (double*)malloc(sizeof(double) * (nnzc > 0 ? nnzc : 1));
  colmap cm = build_colmap(A);
  int64_t maxnb = 0;
  for (int64_t i = 0; i < nz; ++i) if (B->cp[i + 1] - B->cp[i] > maxnb) maxnb = B->cp[i + 1] - B->cp[i];
#pragma omp parallel
  {
    heapent* wset = (heapent*)malloc(sizeof(heapent) * (maxnb + 1));
    int64_t* cur = (int64_t*)malloc(sizeof(int64_t) * (maxnb + 1));
    int64_t* end = (int64_t*)malloc(sizeof(int64_t) * (maxnb + 1));
    int64_t hcap = 0;
    hashent* ht = NULL;
#pragma omp for schedule(dynamic, 64)
    for (int64_t i = 0; i < nz; ++i) {
      int64_t nc = colptr[i + 1] - colptr[i];
      double cr = (double)flops[i] / (double)nc; /* :309 (0/0 = NaN -> hash) */
      if (!hybrid || cr < 2.0) {
        col_heap(A, B, &cm, i, sr, wset, cur, end, ir + colptr[i], val + colptr[i]);
      } else {
        int64_t hs = 16;
        while (hs < nc) hs <<= 1;
        if (hs > hcap) { free(ht); hcap = hs; ht = (hashent*)malloc(sizeof(hashent) * hcap); }
        col_hash(A, B, &cm, i, sr, nc, ht, ir + colptr[i], val + colptr[i]);
      }
    }
    free(wset); free(cur); free(end); free(ht);
  }
  free_colmap(&cm);
  finish_tile(A, B, colptr, ir, val, C);
  free(flops); free(cnt); free(colptr);
  return 0;
}

int ocbg_local_hybrid(const ocbg_tile* A, const ocbg_tile* B, int sr, int nthreads, ocbg_tile* C) {
  return local_mult(A, B, sr, nthreads, 1, C);
}
int ocbg_local_heap(const ocbg_tile* A, const ocbg_tile* B, int sr, int nthreads, ocbg_tile* C) {
  return local_mult(A, B, sr, nthreads, 0, C);
}

/* ------------------------------------------------------------------------ */
/* Merging partial products                                                  */
/* ------------------------------------------------------------------------ */
/* k-way heap merge of column-sorted lists over column range [c0,c1),
 * summing equal (row,col) with SR::add (MergeAll Friends.h:657-741,
 * SerialMerge MultiwayMerge.h:184-233).  count_only -> SerialMergeNNZ (:129-180). */
typedef struct { int64_t col; int32_t row; int32_t src; } mkey;
static inline int mkey_less(const mkey* a, const mkey* b) { /* ColLexiCompare, Compare.h:95-109 */
  return a->col != b->col ? a->col < b->col : a->row < b->row;
}
typedef struct { const ocbg_tile* t; int64_t ci, p; } mcur; /* column index, position */

static int mcur_next(mcur* c, int64_t c1, mkey* k, int src) {
  while (c->ci < c->t->nzc && c->p >= c->t->cp[c->ci + 1]) c->ci++;
  if (c->ci >= c->t->nzc || c->t->jc[c->ci] >= c1) return 0;
  k->col = c->t->jc[c->ci];
  k->row = c->t->ir[c->p];
  k->src = src;
  return 1;
}
static void mheap_down(mkey* h, int n, int i) {
  for (;;) {
    int l = 2 * i + 1, r = l + 1, s = i;
    if (l < n && mkey_less(&h[l], &h[s])) s = l;
    if (r < n && mkey_less(&h[r], &h[s])) s = r;
    if (s == i) return;
    mkey t = h[i]; h[i] = h[s]; h[s] = t;
    i = s;
  }
}
static int64_t lower_col(const ocbg_tile* t, int64_t c) {
  int64_t lo = 0, hi = t->nzc;
  while (lo < hi) { int64_t mid = (lo + hi) / 2; if (t->jc[mid] < c) lo = mid + 1; else hi = mid; }
  return lo;
}
/* merges column range [c0,c1); writes to (ocol, oir, oval) if non-NULL; returns count */
static int64_t merge_range(ocbg_tile** L, int nl, int64_t c0, int64_t c1, int sr, int32_t* ocol, int32_t* oir,
                           double* oval) {
  mcur* cur = (mcur*)malloc(sizeof(mcur) * (nl > 0 ? nl : 1));
  mkey* h = (mkey*)malloc(sizeof(mkey) * (nl > 0 ? nl : 1));
  int hs = 0;
  for (int s = 0; s < nl; ++s) {
    cur[s].t = L[s];
    cur[s].ci = lower_col(L[s], c0);
    cur[s].p = cur[s].ci < L[s]->nzc ? L[s]->cp[cur[s].ci] : L[s]->nnz;
    if (mcur_next(&cur[s], c1, &h[hs], s)) hs++;
  }
  for (int j = hs / 2 - 1; j >= 0; --j) mheap_down(h, hs, j);
  int64_t cnz = 0, lastc = -1;
  int32_t lastr = -1;
  while (hs > 0) {
    mkey top = h[0];
    int s = top.src;
    double v = L[s]->val[cur[s].p];
    if (cnz > 0 && lastc == top.col && lastr == top.row) {
      if (oval) oval[cnz - 1] = sr_add(sr, oval[cnz - 1], v);
    } else {
      if (oir) { ocol[cnz] = (int32_t)top.col; oir[cnz] = top.row; oval[cnz] = v; }
      cnz++;
      lastc = top.col;
      lastr = top.row;
    }
    cur[s].p++;
    if (mcur_next(&cur[s], c1, &h[0], s)) {
      mheap_down(h, hs, 0);
    } else {
      h[0] = h[hs - 1];
      hs--;
      mheap_down(h, hs, 0);
    }
  }
  free(cur); free(h);
  return cnz;
}

static void tuples_to_tile(int64_t m, int64_t n, int64_t nnz, int32_t* col, int32_t* ir, double* val, ocbg_tile* C) {
  /* SpDCCols(SpTuples, false), SpDCCols.cpp:108-190 (column run-lengths) */
  int64_t nzc = 0;
  for (int64_t i = 0; i < nnz; ++i) nzc += (i == 0 || col[i] != col[i - 1]);
  C->m = m; C->n = n; C->nnz = nnz; C->nzc = nzc;
  C->cp = (int64_t*)malloc(sizeof(int64_t) * (nzc + 1));
  C->jc = (int32_t*)malloc(sizeof(int32_t) * (nzc > 0 ? nzc : 1));
  int64_t c = 0;
  for (int64_t i = 0; i < nnz; ++i)
    if (i == 0 || col[i] != col[i - 1]) { C->jc[c] = col[i]; C->cp[c] = i; c++; }
  C->cp[nzc] = nnz;
  C->ir = ir;
  C->val = val;
}

/* MergeAll (serial) when nsplits == 1, MultiwayMerge (threaded, column splits
 * findColSplitters MultiwayMerge.h:84-103) otherwise */
static void merge_lists(ocbg_tile** L, int nl, int64_t m, int64_t n, int sr, int nsplits, ocbg_tile* C) {
  if (nsplits < 1) nsplits = 1;
  if (nsplits > n) nsplits = (int)(n > 0 ? n : 1);
  int64_t* cnt = (int64_t*)calloc((size_t)nsplits + 1, sizeof(int64_t));
#pragma omp parallel for schedule(dynamic) if (nsplits > 1)
  for (int s = 0; s < nsplits; ++s) {
    int64_t c0 = (s == 0) ? 0 : s * (n / nsplits), c1 = (s == nsplits - 1) ? n : (s + 1) * (n / nsplits);
    cnt[s + 1] = merge_range(L, nl, c0, c1, sr, NULL, NULL, NULL);
  }
  for (int s = 0; s < nsplits; ++s) cnt[s + 1] += cnt[s];
  int64_t tot = cnt[nsplits];
  int32_t* col = (int32_t*)malloc(sizeof(int32_t) * (tot > 0 ? tot : 1));
  int32_t* ir = (int32_t*)malloc(sizeof(int32_t) * (tot > 0 ? tot : 1));
  double* val = (double*)malloc(sizeof(double) * (tot > 0 ? tot : 1));
#pragma omp parallel for schedule(dynamic) if (nsplits > 1)
  for (int s = 0; s < nsplits; ++s) {
    int64_t c0 = (s == 0) ? 0 : s * (n / nsplits), c1 = (s == nsplits - 1) ? n : (s + 1) * (n / nsplits);
    merge_range(L, nl, c0, c1, sr, col + cnt[s], ir + cnt[s], val + cnt[s]);
  }
  tuples_to_tile(m, n, tot, col, ir, val, C);
  free(col);
  free(cnt);
}

/* ------------------------------------------------------------------------ */
/* 2D SUMMA emulation                                                        */
/* ------------------------------------------------------------------------ */
/* extract rows [r0,r1) x cols [c0,c1) of a global tile, re-based */
static void sub_tile(const ocbg_tile* G, int64_t r0, int64_t r1, int64_t c0, int64_t c1, ocbg_tile* T) {
  int64_t a = lower_col(G, c0), b = lower_col(G, c1);
  int64_t nnz = 0, nzc = 0;
  for (int64_t i = a; i < b; ++i) {
    int64_t k = 0;
    for (int64_t p = G->cp[i]; p < G->cp[i + 1]; ++p) k += (G->ir[p] >= r0 && G->ir[p] < r1);
    nnz += k;
    nzc += (k > 0);
  }
  tile_alloc(T, r1 - r0, c1 - c0, nnz, nzc);
  int64_t q = 0, c = 0;
  for (int64_t i = a; i < b; ++i) {
    int64_t q0 = q;
    for (int64_t p = G->cp[i]; p < G->cp[i + 1]; ++p)
      if (G->ir[p] >= r0 && G->ir[p] < r1) { T->ir[q] = (int32_t)(G->ir[p] - r0); T->val[q] = G->val[p]; q++; }
    if (q > q0) { T->jc[c] = (int32_t)(G->jc[i] - c0); T->cp[c] = q0; c++; }
  }
  T->cp[nzc] = q;
}

int ocbg_summa(const ocbg_tile* A, const ocbg_tile* B, int pr, int algo, int sr, int nthreads, ocbg_tile* C) {
  if (A->n != B->m) return 3002; /* CheckSpGEMMCompliance DIMMISMATCH, ParFriends.h:162-170 */
  if (A == B) return 3005;       /* MATRIXALIAS, :171-178 */
  if (nthreads > 0) omp_set_num_threads(nthreads);
  int nt = omp_get_max_threads();
  int64_t m = A->m, n = B->n, kk = A->n;
  int64_t mper = m / pr, nper = n / pr, kper = kk / pr;
  ocbg_tile* Ct = (ocbg_tile*)calloc((size_t)pr * pr, sizeof(ocbg_tile));
  for (int r = 0; r < pr; ++r)
    for (int c = 0; c < pr; ++c) {
      int64_t rr0 = r * mper, rr1 = (r == pr - 1) ? m : rr0 + mper;
      int64_t cc0 = c * nper, cc1 = (c == pr - 1) ? n : cc0 + nper;
      ocbg_tile* parts = (ocbg_tile*)calloc((size_t)2 * pr, sizeof(ocbg_tile));
      ocbg_tile** L = (ocbg_tile**)malloc(sizeof(ocbg_tile*) * 2 * pr);
      int nl = 0;
      int halves = (algo == 0) ? 2 : 1;
      for (int h = 0; h < halves; ++h)
        for (int s = 0; s < pr; ++s) { /* stage s: A(r,s) x B(s,c) */
          int64_t k0 = s * kper, k1 = (s == pr - 1) ? kk : k0 + kper;
          if (halves == 2) { /* Split at local ncol/2 (SpDCCols.cpp:905-930); B row split via transposes (ParFriends.h:823-829) */
            int64_t cut = (k1 - k0) / 2;
            if (h == 0) k1 = k0 + cut; else k0 = k0 + cut;
          }
          ocbg_tile At, Bt;
          sub_tile(A, rr0, rr1, k0, k1, &At);
          sub_tile(B, k0, k1, cc0, cc1, &Bt);
          ocbg_tile* P = &parts[nl];
          local_mult(&At, &Bt, sr, nthreads, 1, P);
          ocbg_free(&At);
          ocbg_free(&Bt);
          if (P->nnz > 0) L[nl++] = P; else ocbg_free(P);
        }
      if (algo == 0) merge_lists(L, nl, rr1 - rr0, cc1 - cc0, sr, 1, &Ct[r * pr + c]);      /* MergeAll */
      else merge_lists(L, nl, rr1 - rr0, cc1 - cc0, sr, 4 * nt, &Ct[r * pr + c]);           /* MultiwayMerge */
      for (int i = 0; i < nl; ++i) ocbg_free(L[i]);
      free(parts);
      free(L);
    }
  /* gather tiles into a global DCSC (block offsets of SpParMat::Owner) */
  int64_t nnz = 0;
  for (int t = 0; t < pr * pr; ++t) nnz += Ct[t].nnz;
  int32_t* col = (int32_t*)malloc(sizeof(int32_t) * (nnz > 0 ? nnz : 1));
  int32_t* ir = (int32_t*)malloc(sizeof(int32_t) * (nnz > 0 ? nnz : 1));
  double* val = (double*)malloc(sizeof(double) * (nnz > 0 ? nnz : 1));
  int64_t q = 0;
  for (int c = 0; c < pr; ++c) {
    int64_t* ci = (int64_t*)calloc((size_t)pr, sizeof(int64_t));
    int64_t cc0 = c * nper, cc1 = (c == pr - 1) ? n : cc0 + nper;
    for (int64_t gc = cc0; gc < cc1; ++gc)
      for (int r = 0; r < pr; ++r) {
        ocbg_tile* T = &Ct[r * pr + c];
        if (ci[r] < T->nzc && T->jc[ci[r]] + cc0 == gc) {
          for (int64_t p = T->cp[ci[r]]; p < T->cp[ci[r] + 1]; ++p) {
            col[q] = (int32_t)gc;
            ir[q] = (int32_t)(T->ir[p] + r * mper);
            val[q] = T->val[p];
            q++;
          }
          ci[r]++;
        }
      }
    free(ci);
  }
  for (int t = 0; t < pr * pr; ++t) ocbg_free(&Ct[t]);
  free(Ct);
  tuples_to_tile(m, n, nnz, col, ir, val, C);
  free(col);
  return 0;
}
