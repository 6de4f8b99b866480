/* cbg_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement ("oracle") of the reference CombBLAS SpGEMM hot path, used
 * by tests/ (as the checker), by __graft_entry__.smoke() (as the checker) and
 * by bench.py's cpu_baseline leg (as the timed host baseline).  It is never
 * linked into, loaded by, or called from the product library.
 *
 * Parity is pinned against tests/golden/golden.json, produced by the reference
 * itself (oracle/_ref/ref_driver, see tests/golden/make_golden.py).
 *
 * Tiles are DCSC (reference Dcsc, dcsc.h:85-91): cp[nzc+1] (int64 here),
 * jc[nzc], ir[nnz] (int32 local indices), val[nnz] (fp64).
 */
#ifndef CBG_ORACLE_H
#define CBG_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct ocbg_tile {
  int64_t m, n, nnz, nzc;
  int64_t* cp;
  int32_t* jc;
  int32_t* ir;
  double* val;
} ocbg_tile;

enum { OCBG_PLUS_TIMES = 0, OCBG_MIN_PLUS = 1 };

/* frees arrays allocated by the oracle */
void ocbg_free(ocbg_tile* t);

/* Graph500 Kronecker R-MAT (RefGen21.h:73-318 + graph500 splittable_mrg.c):
 * global edges [e0,e1) of the (scale, ef) graph for userseed. */
void ocbg_rmat_edges(int scale, int64_t e0, int64_t e1, uint64_t userseed, int64_t* src, int64_t* dst);
/* Whole matrix as one 1x1 tile: duplicates summed (value = multiplicity),
 * self loops removed (SpTuples.cpp:70-123, SpParMat.cpp:3257-3272). */
int ocbg_rmat_tile(int scale, int ef, uint64_t userseed, int nthreads, ocbg_tile* out);

/* estimateFLOP (mtSpGEMM.h:1056-1134) and estimateNNZ_Hash (:805-933) */
int ocbg_symbolic(const ocbg_tile* A, const ocbg_tile* B, int64_t* flops, int64_t* nnzc, int nthreads);

/* LocalHybridSpGEMM (mtSpGEMM.h:212-460) -> C as DCSC (tuples are already
 * column-major/row-sorted, so the SpDCCols(SpTuples) conversion,
 * SpDCCols.cpp:108-190, is a run-length pass). */
int ocbg_local_hybrid(const ocbg_tile* A, const ocbg_tile* B, int semiring, int nthreads, ocbg_tile* C);
/* LocalSpGEMM (heap only, mtSpGEMM.h:73-202) */
int ocbg_local_heap(const ocbg_tile* A, const ocbg_tile* B, int semiring, int nthreads, ocbg_tile* C);

/* 2D SUMMA emulated on one host over a pr x pr grid (block distribution of
 * SpParMat::Owner, SpParMat.cpp:5068-5097):
 *   algo 0 = Mult_AnXBn_DoubleBuff (ParFriends.h:798-997, serial MergeAll Friends.h:657-741)
 *   algo 1 = Mult_AnXBn_Synch      (ParFriends.h:1004-1108, MultiwayMerge.h:409-526)
 * A and B are global 1x1 tiles; the result is returned as a global tile. */
int ocbg_summa(const ocbg_tile* A, const ocbg_tile* B, int pr, int algo, int semiring, int nthreads, ocbg_tile* C);

#ifdef __cplusplus
}
#endif
#endif
