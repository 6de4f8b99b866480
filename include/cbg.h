/* cbg.h -- C ABI of libcbg, the MI355X-native CombBLAS 2D-SUMMA SpGEMM hot path.
 *
 * Plain C types only (pointers + sizes): this is the drop-in boundary that a
 * CombBLAS build (C++ shim: combblas-spmm-test_amd/include/combblas_amd/) or
 * any FFI (ctypes stub in INTEGRATION.md) binds.  Each entry point names the
 * reference interface it replaces (paths relative to the reference root).
 *
 * Tiles are DCSC, the reference's Dcsc<IT,NT> (include/CombBLAS/dcsc.h:85-91):
 *   cp[nzc+1] column pointers (int64 here: C tiles exceed 2^31 nnz at scale>=20),
 *   jc[nzc]   ids of the nonempty columns (ascending),
 *   ir[nnz]   row ids, ascending inside each column,
 *   val[nnz]  fp64 values.
 * Local indices are int32 (SpDCCols<int32_t,double>, MultTiming.cpp:18-23);
 * A and B tiles need nnz < 2^31.
 *
 * Error model: the reference MPI_Aborts with SpDefs.h:69-76 codes; libcbg
 * returns the same code instead (3001 GRIDMISMATCH, 3002 DIMMISMATCH,
 * 3003 NOTSQUARE, 3005 MATRIXALIAS, 3007 INVALIDPARAMS) and >= 3100 for
 * device/runtime failures.  cbg_last_error() gives the message.
 */
#ifndef CBG_H
#define CBG_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct cbg_tile {
  int64_t m, n, nnz, nzc;
  int64_t* cp;
  int32_t* jc;
  int32_t* ir;
  double* val;
  int32_t on_device; /* 1: arrays are device memory (owned by libcbg when produced by it) */
  int32_t reserved;
} cbg_tile;

/* semirings: PlusTimesSRing<double,double> Semirings.h:212-233,
 *            MinPlusSRing<double,double>   Semirings.h:235-255 */
enum { CBG_PLUS_TIMES = 0, CBG_MIN_PLUS = 1 };

/* SUMMA variants */
enum {
  CBG_DOUBLEBUFF = 0, /* Mult_AnXBn_DoubleBuff ParFriends.h:798-997 */
  CBG_SYNCH = 1       /* Mult_AnXBn_Synch      ParFriends.h:1004-1108 (PSpGEMM SpParMat.h:454-467) */
};
/* how the stages are executed on device (identical results up to fp order) */
enum {
  CBG_EXEC_PANEL = 0, /* gather the A block-row, receive the B block-column in column pieces
                         (piece p+1 broadcast while piece p multiplies), one local multiply per
                         piece, C entries written end to end: no partial products, no merge */
  CBG_EXEC_STAGED = 1 /* the reference's stages (any pr x pc grid: inner dimension cut at the union
                         of A's column-block and B's row-block boundaries), stage s+1 broadcast while
                         stage s multiplies, then an on-device multiway merge of the partials */
};

enum {
  CBG_OK = 0,
  CBG_ERR_GRIDMISMATCH = 3001,
  CBG_ERR_DIMMISMATCH = 3002,
  CBG_ERR_NOTSQUARE = 3003,
  CBG_ERR_MATRIXALIAS = 3005,
  CBG_ERR_INVALIDPARAMS = 3007,
  CBG_ERR_HIP = 3100,
  CBG_ERR_RCCL = 3101,
  CBG_ERR_OOM = 3102,
  CBG_ERR_NOTSUPPORTED = 3103
};

/* ---------------- library ---------------- */
const char* cbg_version(void);
const char* cbg_last_error(void);
/* select the HIP device for the calling thread (default: current device) */
int cbg_set_device(int device);
int cbg_device_count(int* count);
/* device memory of libcbg's caching pool (bytes) */
int cbg_pool_stats(size_t* in_use, size_t* cached);
int cbg_pool_trim(void);
int cbg_synchronize(void);
/* measured side of the HBM roofline (no reference counterpart): a 16-byte-per-lane
 * device copy of `bytes` run `reps` times; *gbps = 2 * bytes * reps / time (GB/s) */
int cbg_hbm_copy_bandwidth(int64_t bytes, int reps, double* gbps);
/* known-bytes store probe for the PMC traffic calibration (tools/traffic.py, no
 * reference counterpart): writes exactly `bytes` (a multiple of 256) of a scratch
 * buffer with `width`-byte stores (4 or 8) per lane -- the SpGEMM kernels' C row
 * ids and values -- consecutive lanes at consecutive addresses (k_store_probe<W>) */
int cbg_store_probe(int64_t bytes, int width);

/* ---------------- tiles ---------------- */
/* host -> device copy (arrays of *dst are allocated by libcbg) */
int cbg_tile_upload(const cbg_tile* host, cbg_tile* dst);
/* device -> host into caller-provided arrays sized from dev->nnz/nzc */
int cbg_tile_download(const cbg_tile* dev, cbg_tile* host);
/* frees a device tile produced by libcbg (no-op for host tiles) */
int cbg_tile_free(cbg_tile* t);
/* SpDCCols::CreateImpl(essentials) (SpDCCols.cpp:733-745): an uninitialised device
 * tile of the given sizes (cp[0] = 0), e.g. the receive buffers of BCastMatrix */
int cbg_tile_alloc(int64_t m, int64_t n, int64_t nnz, int64_t nzc, cbg_tile* out);
/* SpDCCols::ColConcatenate / Merge (SpDCCols.cpp:1194-1223, ParFriends.h:724-725):
 * parts side by side (part k's columns shifted by the widths of parts 0..k-1),
 * all with the same row count; device tiles */
int cbg_tile_concat_cols(const cbg_tile* parts, int nparts, cbg_tile* out);
/* device memory: free and total bytes (hipMemGetInfo) */
int cbg_device_memory(size_t* free_bytes, size_t* total_bytes);
/* SpDCCols::Split (SpDCCols.cpp:905-930): columns [0,cut) and [cut,n) (device) */
int cbg_tile_split_cols(const cbg_tile* t, int64_t cut, cbg_tile* left, cbg_tile* right);
/* row split of B as DoubleBuff does with Transpose/Split/Transpose (ParFriends.h:824-829), no transposes */
int cbg_tile_split_rows(const cbg_tile* t, int64_t cut, cbg_tile* top, cbg_tile* bottom);
/* structural + value digest (same definition as tests/golden/make_golden.py), device tile.
 * unsorted (may be NULL) receives the number of DCSC order violations: a row id not
 * strictly above its predecessor in its column, a column id not strictly above the
 * previous one, an empty column, cp[0] != 0 or cp[nzc] != nnz (0 for a valid tile). */
int cbg_tile_digest(const cbg_tile* t, int64_t row_off, int64_t col_off, uint64_t* hs, uint64_t* hv, double* vsum,
                    uint64_t* unsorted);
/* SpDCCols::operator== (SpDCCols.h:74-81, Dcsc::operator== dcsc.cpp:472-510):
 * two empty tiles are equal; else m, n, nnz, nzc, cp, jc, ir must match and
 * values be ErrorTolerantEqual (Compare.h:47-65: equal, or absolute or
 * relative difference < epsilon; the reference's EPSILON is 0.01, SpDefs.h:64).
 * Device tiles; *equal receives 1 or 0. */
int cbg_tile_equal(const cbg_tile* a, const cbg_tile* b, double epsilon, int* equal);

/* ---------------- Galerkin triple-product path (GalerkinNew.cpp:96-153) ---------------- */
/* SpDCCols::Transpose (SpDCCols.cpp:853-873): out = t^T as a device DCSC tile */
int cbg_tile_transpose(const cbg_tile* t, cbg_tile* out);
/* SpParMat::DimApply (SpParMat.cpp:801): dim CBG_DIM_COLUMN: x(i,j) = op(x(i,j), vec[j]);
 * CBG_DIM_ROW: x(i,j) = op(x(i,j), vec[i]); vec is HOST memory of t->n (t->m) values,
 * the tile's slice of the distributed dense vector.  In place. */
enum { CBG_DIM_COLUMN = 0, CBG_DIM_ROW = 1 };
enum { CBG_OP_MULTIPLIES = 0, CBG_OP_PLUS = 1, CBG_OP_MIN = 2, CBG_OP_MAX = 3 };
int cbg_tile_dim_apply(cbg_tile* t, int dim, const double* vec, int op);
/* Restriction operator of the Galerkin driver (mfiles/genrestrict.m:11,
 * sprand(n, n/order, order/n)): n x n/order, Poisson(1) nonzeros per fine row
 * (~37 % of the rows empty) in uniform coarse columns (Poisson(order) per
 * column), values in (0,1]; counts, columns and values from a counter-based
 * hash of (seed, row), a column drawn twice in a row summed, so every grid
 * shape sees the same global T.  Tile (prow,pcol) of the pr x pc block
 * distribution. */
int cbg_restriction_tile(int scale, int order, uint64_t seed, int pr, int pc, int prow, int pcol, cbg_tile* out);
/* Test inputs with random values: every nonzero (i, j) of the
 * tile, at global row i + row_off and column j + col_off, gets a value
 * U[-1, 1) from a counter hash of (seed, column, row) (exact in double; the
 * structure is kept).  In place. */
int cbg_tile_random_values(cbg_tile* t, uint64_t seed, int64_t row_off, int64_t col_off);

/* ---------------- generator ---------------- */
/* Graph500 Kronecker R-MAT as DistEdgeList::GenGraph500Data(packed, scrambled)
 * (DistEdgeList.cpp:223-280, RefGen21.h:73-318) -> SpParMat(DEL,false)
 * (SpParMat.cpp:3140-3254) -> RemoveLoops (SpParMat.cpp:3257-3272), on device.
 * Produces the tile of grid cell (prow,pcol) of a pr x pc grid (1x1: whole matrix). */
int cbg_rmat_tile(int scale, int edgefactor, uint64_t userseed, int pr, int pc, int prow, int pcol,
                  cbg_tile* out);

/* ---------------- local multiply ---------------- */
/* LocalHybridSpGEMM (mtSpGEMM.h:212-460) + SpDCCols(SpTuples) (SpDCCols.cpp:108-190):
 * C = A*B on the semiring, C as a device DCSC tile (columns where C has nonzeros,
 * rows ascending, explicit zeros kept).  A, B device tiles.  stream may be NULL. */
int cbg_local_spgemm(const cbg_tile* A, const cbg_tile* B, int semiring, cbg_tile* C, void* hip_stream);
/* estimateFLOP + estimateNNZ_Hash (mtSpGEMM.h:1056-1134, 805-933): totals only */
int cbg_local_symbolic(const cbg_tile* A, const cbg_tile* B, int64_t* flops, int64_t* nnz, void* hip_stream);
/* MergeAll / MultiwayMerge (Friends.h:657-741, MultiwayMerge.h:409-526) of
 * column-sorted device tiles of equal shape, summing duplicates with SR::add. */
int cbg_merge(const cbg_tile* parts, int nparts, int semiring, cbg_tile* C, void* hip_stream);
/* last call's local-multiply statistics (summed over its multiplies): flops, nnz,
 * per-phase device ms, big columns, slabs.  Merges are not counted here. */
int cbg_last_stats(int64_t* flops, int64_t* nnz, double* ms_symbolic, double* ms_numeric, int64_t* n_big,
                   int64_t* n_slabs);
/* ... and the work of each kernel family (summed over the call's multiplies), so a
 * test can prove which code paths ran: numeric slabs per launch class (bitmap
 * slabs with kept symbolic bitmaps / with the marking pass, hash slabs by table
 * size 512 ... 8192, rank slabs of <= 1024 / 2048 / 4096 nonzeros), symbolic
 * (column, panel) units and panel-group units, group units run panel by panel,
 * columns of the one-pass small-column kernels, thin columns, entries of the
 * single-entry big columns, columns of the numeric hash / wave bins, and the
 * multiplies whose slab kernels accumulated exact integers in int32 (A's and B's
 * values integers of magnitude <= 2^24 whose sums stay below 2^31).
 * counts[i] for i < min(n, CBG_WORK_N); returns CBG_WORK_N. */
enum {
  CBG_WORK_BITMAP_SMALL_KEPT = 0,
  CBG_WORK_BITMAP_SMALL_MARK = 1,
  CBG_WORK_BITMAP_LARGE_KEPT = 2,
  CBG_WORK_BITMAP_LARGE_MARK = 3,
  CBG_WORK_HASH0 = 4, /* + k: tables of 512, 768, 1024, 1536, 2048, 3072, 4096, 6144, 8192 slots */
  CBG_WORK_RANK0 = 13, /* + k: rank slabs of <= 1024, 2048, 4096 nonzeros */
  CBG_WORK_SYM_PANEL_UNITS = 16,
  CBG_WORK_SYM_GROUP_UNITS = 17,
  CBG_WORK_SYM_DEFERRED_UNITS = 18,
  CBG_WORK_ESC_COLUMNS = 19,
  CBG_WORK_THIN_COLUMNS = 20,
  CBG_WORK_SINGLE_BIG_ENTRIES = 21,
  CBG_WORK_HASH_BIN_COLUMNS = 22,
  CBG_WORK_WAVE_BIN_COLUMNS = 23,
  CBG_WORK_IACC = 24, /* multiplies whose slabs accumulated exact integers in int32 */
  CBG_WORK_GRANK0 = 25, /* + k: panel-group rank slabs of <= 2048, 4096 nonzeros */
  CBG_WORK_N = 27
};
int cbg_last_work_stats(int64_t* counts, int n);
/* last call's multiway merges (MergeAll / MultiwayMerge): partial entries in,
 * merged entries out, device ms */
int cbg_merge_stats(int64_t* entries_in, int64_t* entries_out, double* ms);
/* last PANEL SUMMA call's double buffering: B-column pieces multiplied (1 = the
 * broadcast was not pipelined), measured broadcast ms of the first piece, the
 * estimated broadcast ms of the rest that pipelining would hide, and the ms an
 * extra piece is taken to cost: max(CBG_PIPELINE_MIN_MS (3), CBG_PIPELINE_COST_FRAC
 * (0.04) x the previous such call's local multiply ms); pipelined when the
 * hidden ms exceed the cost on some rank */
int cbg_last_summa_info(int* pieces, double* bcast_ms_piece0, double* est_hidden_ms, double* piece_cost_ms);
/* ... and its communication: the double-buffering rule applied (0 one piece,
 * 1 pipelined because the B block column has > 1 remote tile on an RCCL grid,
 * 2 adaptive and pipelined, 3 adaptive and rejoined, 4 a fixed pipeline of
 * several pieces: CBG_PIPELINE or phases given as pieces), the bytes of the remote
 * A and B tiles this rank received, and the exposed communication: the summed
 * ms the compute stream waited for broadcasts (HIP events around each wait) */
int cbg_last_summa_comm(int* rule, int64_t* bytes_recv, double* exposed_comm_ms);

/* ---------------- 2D SUMMA over RCCL ---------------- */
typedef struct cbg_grid cbg_grid;
#define CBG_UNIQUE_ID_BYTES 128
/* ncclGetUniqueId: called by rank 0, bytes shipped to the others by the host */
int cbg_get_unique_id(void* id);
/* CommGrid(MPI_COMM_WORLD, rows, cols) (CommGrid.cpp:37-75): rows=cols=0 => square
 * grid or CBG_ERR_NOTSQUARE; rank r -> (r / cols, r % cols); row/col
 * communicators via ncclCommSplit.  One process (rank) per GPU. */
int cbg_grid_create(int rank, int nranks, int grid_rows, int grid_cols, const void* unique_id, cbg_grid** out);
/* host-transport grid for testing the SUMMA logic with several processes on
 * one GPU: collectives are delegated to host callbacks (e.g. gloo). */
typedef struct cbg_host_comm {
  /* comm: 0 = world, 1 = row communicator, 2 = column communicator; root is the
   * rank inside that communicator; buf is HOST memory */
  int (*bcast)(void* user, int comm, void* buf, size_t bytes, int root);
  int (*allgather)(void* user, int comm, const void* in, void* out, size_t bytes_each);
  void* user;
} cbg_host_comm;
int cbg_grid_create_host(int rank, int nranks, int grid_rows, int grid_cols, const cbg_host_comm* comm,
                         cbg_grid** out);
int cbg_grid_destroy(cbg_grid* g);
int cbg_grid_info(const cbg_grid* g, int* rank, int* nranks, int* grid_rows, int* grid_cols, int* prow, int* pcol);
/* world-communicator helpers used by drivers for barrier + max-over-ranks timing */
int cbg_grid_barrier(cbg_grid* g);
/* collective error agreement (no reference counterpart: the reference MPI_Aborts,
 * SpDefs.h:69-76): *agreed = max over the grid's ranks of local_rc.  Every
 * collective entry point below runs it after each of its steps, so a failure on
 * one rank (CBG_ERR_OOM in its local multiply, a bad argument) is returned by
 * every rank instead of leaving the others blocked in a broadcast.  An RCCL
 * async error, or no progress for CBG_COMM_TIMEOUT_S seconds (default 600),
 * aborts the grid's communicators (ncclCommAbort): later calls on that grid
 * return CBG_ERR_RCCL. */
int cbg_grid_agree(cbg_grid* g, int local_rc, int* agreed);
int cbg_grid_allreduce_max(cbg_grid* g, double* value);
int cbg_grid_allreduce_sum_i64(cbg_grid* g, int64_t* value);

/* Mult_AnXBn_DoubleBuff / Mult_AnXBn_Synch (ParFriends.h:798-1108):
 * collective over the grid; A_local/B_local are this rank's device tiles of
 * the block distribution (SpParMat::Owner, SpParMat.cpp:5068-5097).
 * A_gncol/B_gnrow are the global inner dimensions (CheckSpGEMMCompliance).
 * A and B are left unchanged (the reference mutates and restores them).
 * C_local receives this rank's tile C(prow,pcol). */
int cbg_summa_spgemm(cbg_grid* g, const cbg_tile* A_local, const cbg_tile* B_local, int64_t A_gncol,
                     int64_t B_gnrow, int semiring, int algo, int exec, cbg_tile* C_local);

/* MemEfficientSpGEMM (ParFriends.h:449-730) without its Markov-clustering
 * pruning: this rank's B tile is cut into `phases` column pieces
 * (SpDCCols::ColSplit, SpDCCols.cpp:936-970: cuts at (i+1)*(n/phases)), each
 * piece goes through the SUMMA above, and the phase results are
 *   fn == NULL: column-concatenated on device into C_local
 *               (SpDCCols::ColConcatenate, ParFriends.h:724-725);
 *   fn != NULL: handed to fn(user, phase, col_offset, C_phase) one at a time
 *               and freed after the call (C streamed when it does not fit HBM;
 *               C_local may be NULL).  fn runs on every rank between the
 *               collectives; a nonzero return is reported after all phases.
 *               fn may be called SEVERAL times per phase, each time with a
 *               column piece of that phase's C at its own col_offset: with
 *               phases == 1 and EXEC_PANEL the SUMMA's pipeline pieces are
 *               handed over one by one (phase 0 each), and with EXEC_PANEL a
 *               phase whose C does not fit the device after all is computed as
 *               column halves of its B piece (same phase index).  With
 *               EXEC_STAGED such a phase fails with CBG_ERR_OOM.
 * phases < 1 or >= A_gncol is reset to 1 (ParFriends.h:468-473).  Every rank needs
 * B_local->n >= phases (CBG_ERR_INVALIDPARAMS otherwise, collectively). */
typedef int (*cbg_phase_fn)(void* user, int phase, int64_t col_offset, const cbg_tile* C_phase);
int cbg_summa_spgemm_phased(cbg_grid* g, const cbg_tile* A_local, const cbg_tile* B_local, int64_t A_gncol,
                            int64_t B_gnrow, int semiring, int algo, int exec, int phases, cbg_phase_fn fn,
                            void* user, cbg_tile* C_local);
/* The same with MemEfficientSpGEMM's perProcessMemory (GB, ParFriends.h:482-535):
 * when per_process_memory_gb > 0, or phases == CBG_PHASES_AUTO (this library's
 * extension: the device's free memory), the phase count comes from memory: the flops of this rank's product (from the column counts of A's tiles
 * and the row counts of B's tiles, allgathered along the grid row / column), an
 * nnz(C) estimate (flops, times the compression of an exact symbolic of a sample
 * of the product when the flops bound asks for more than one phase), and 60 % of
 * the memory left after the tiles the SUMMA gathers -- perProcessMemory, or the device's free memory when it is 0;
 * the maximum over the grid.  If that memory is already taken by the inputs the
 * given phases are kept, like the reference. */
#define CBG_PHASES_AUTO (-1)
int cbg_summa_spgemm_memeff(cbg_grid* g, const cbg_tile* A_local, const cbg_tile* B_local, int64_t A_gncol,
                            int64_t B_gnrow, int semiring, int algo, int exec, int phases,
                            int64_t per_process_memory_gb, cbg_phase_fn fn, void* user, cbg_tile* C_local);
/* the last (memeff / phased) call's phase plan: phases run, whether they were
 * chosen from memory, this rank's product flops and estimated nnz(C), the C bytes
 * a phase was allowed, phases split in halves after an out-of-memory, and the
 * host ms the planning took */
int cbg_last_phase_plan(int* phases, int* automatic, int64_t* flops, int64_t* nnz_est, double* c_budget_bytes,
                        int* oom_splits, double* plan_ms);

/* SpParMat::Transpose (SpParMat.cpp:3528-3590), collective over a square grid:
 * out = this rank's tile of the transposed matrix (the transpose of the
 * complement rank's tile, exchanged with RCCL send/recv).  CBG_ERR_NOTSQUARE
 * on non-square grids, like the reference. */
int cbg_grid_transpose(cbg_grid* g, const cbg_tile* local, cbg_tile* out);

/* SpParMat::BlockSplit (SpParMat.cpp:2974-3058) as BlockSpGEMM uses it
 * (BlockSpGEMM.h:39-45, bi = 1), collective over the grid: the global rows
 * [lo, hi) (dim 0) or columns [lo, hi) (dim 1) of the gm x gn distributed
 * matrix whose local tile is `local`, as a distributed matrix of their own on
 * the same grid (standard block layout, SpParMat::Owner SpParMat.cpp:5068);
 * out = this rank's tile of it. */
int cbg_grid_block_extract(cbg_grid* g, const cbg_tile* local, int64_t gm, int64_t gn, int dim, int64_t lo,
                           int64_t hi, cbg_tile* out);

#ifdef __cplusplus
}
#endif
#endif /* CBG_H */
