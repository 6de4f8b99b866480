// cbg_summa.cpp -- 2D Sparse SUMMA over RCCL (xGMI), one process per GPU.
//
// Replaces, for the SpGEMM path:
//   CommGrid (reference src/CommGrid.cpp:37-75; rank -> (rank / cols, rank % cols),
//             row/col communicators by MPI_Comm_split)       -> ncclCommInitRank + ncclCommSplit
//   ProductGrid (CommGrid.cpp:164-180)                        -> grid reuse (no per-call dup)
//   SpParHelper::GetSetSizes (SpParHelper.cpp:797-809)        -> one allgather of {m,n,nnz,nzc}
//   SpParHelper::BCastMatrix (SpParHelper.cpp:582-600)        -> 4 x ncclBroadcast in a group
//   Mult_AnXBn_DoubleBuff / Mult_AnXBn_Synch (ParFriends.h:798-1108)
//
// Two execution modes with identical results (up to fp summation order):
//   PANEL  : every rank gathers its A block row and B block column (the same
//            broadcasts as the SUMMA stages, issued back to back on the comm
//            stream), concatenates them in HBM and runs ONE local multiply.
//            No partial products, no merge (the reference's dominant cost,
//            69 % of DoubleBuff at 1x1).  Works on any pr x pc grid because
//            the inner coordinates are global.
//   STAGED : the reference's stage structure on square grids (sqrt(P) stages
//            for Synch, 2 sqrt(P) half-tile stages for DoubleBuff); the
//            broadcast of stage s+1 runs on the comm stream while stage s
//            multiplies on the compute stream; partial products are merged
//            on device (cbg_merge.hip).
#include <rccl/rccl.h>

#include <cstring>
#include <memory>

#include "cbg_internal.h"

namespace cbg {

struct RcclError : std::runtime_error {
  explicit RcclError(const std::string& s) : std::runtime_error(s) {}
};
#define CBG_NCCL(x)                                                                                   \
  do {                                                                                                \
    ncclResult_t r_ = (x);                                                                            \
    if (r_ != ncclSuccess)                                                                            \
      throw ::cbg::HipError(std::string(#x) + ": " + ncclGetErrorString(r_), CBG_ERR_RCCL);           \
  } while (0)

}  // namespace cbg

struct cbg_grid {
  int rank = 0, nranks = 1, pr = 1, pc = 1, prow = 0, pcol = 0;
  bool host_mode = false;
  cbg_host_comm hc{};
  ncclComm_t world = nullptr, row = nullptr, col = nullptr;
  hipStream_t compute = nullptr, comm = nullptr;
  hipEvent_t ev_comm = nullptr;
};

namespace cbg {

enum { COMM_WORLD = 0, COMM_ROW = 1, COMM_COL = 2 };

static ncclComm_t pick(cbg_grid* g, int which) {
  return which == COMM_ROW ? g->row : which == COMM_COL ? g->col : g->world;
}
static int comm_size(cbg_grid* g, int which) { return which == COMM_ROW ? g->pc : which == COMM_COL ? g->pr : g->nranks; }
static int comm_rank(cbg_grid* g, int which) { return which == COMM_ROW ? g->pcol : which == COMM_COL ? g->prow : g->rank; }

void grid_setup_streams(cbg_grid* g) {
  CBG_HIP(hipStreamCreateWithFlags(&g->compute, hipStreamNonBlocking));
  CBG_HIP(hipStreamCreateWithFlags(&g->comm, hipStreamNonBlocking));
  CBG_HIP(hipEventCreateWithFlags(&g->ev_comm, hipEventDisableTiming));
}

int grid_shape(int nranks, int& rows, int& cols) {
  if (rows == 0 && cols == 0) {  // CommGrid.cpp:44-53: square or NOTSQUARE
    int r = 1;
    while ((r + 1) * (r + 1) <= nranks) ++r;
    if (r * r != nranks) return CBG_ERR_NOTSQUARE;
    rows = cols = r;
  }
  if (rows <= 0 || cols <= 0 || rows * cols != nranks) return CBG_ERR_INVALIDPARAMS;
  return CBG_OK;
}

cbg_grid* grid_create_rccl(int rank, int nranks, int rows, int cols, const void* uid) {
  std::unique_ptr<cbg_grid> g(new cbg_grid());
  g->rank = rank;
  g->nranks = nranks;
  g->pr = rows;
  g->pc = cols;
  g->prow = rank / cols;
  g->pcol = rank % cols;
  grid_setup_streams(g.get());
  ncclUniqueId id;
  std::memcpy(&id, uid, sizeof(id));
  CBG_NCCL(ncclCommInitRank(&g->world, nranks, id, rank));
  CBG_NCCL(ncclCommSplit(g->world, g->prow, g->pcol, &g->row, nullptr));  // row comm: rank = pcol
  CBG_NCCL(ncclCommSplit(g->world, g->pcol, g->prow, &g->col, nullptr));  // col comm: rank = prow
  return g.release();
}

cbg_grid* grid_create_host(int rank, int nranks, int rows, int cols, const cbg_host_comm* hc) {
  std::unique_ptr<cbg_grid> g(new cbg_grid());
  g->rank = rank;
  g->nranks = nranks;
  g->pr = rows;
  g->pc = cols;
  g->prow = rank / cols;
  g->pcol = rank % cols;
  g->host_mode = true;
  g->hc = *hc;
  grid_setup_streams(g.get());
  return g.release();
}

void grid_destroy(cbg_grid* g) {
  if (!g) return;
  if (g->row) ncclCommDestroy(g->row);
  if (g->col) ncclCommDestroy(g->col);
  if (g->world) ncclCommDestroy(g->world);
  if (g->compute) (void)hipStreamDestroy(g->compute);
  if (g->comm) (void)hipStreamDestroy(g->comm);
  if (g->ev_comm) (void)hipEventDestroy(g->ev_comm);
  delete g;
}

// ---------------------------------------------------------------------------
// collectives
// ---------------------------------------------------------------------------
static void host_check(int rc, const char* what) {
  if (rc != 0) throw HipError(std::string("host transport ") + what + " failed", CBG_ERR_RCCL);
}

// allgather of n int64 per rank (host buffers)
void allgather_i64(cbg_grid* g, int which, const int64_t* in, int64_t* out, int n) {
  const int P = comm_size(g, which);
  if (P == 1) {
    std::memcpy(out, in, sizeof(int64_t) * n);
    return;
  }
  if (g->host_mode) {
    host_check(g->hc.allgather(g->hc.user, which, in, out, sizeof(int64_t) * n), "allgather");
    return;
  }
  DBuf<int64_t> d(P * n + n);
  CBG_HIP(hipMemcpyAsync(d.p + P * n, in, sizeof(int64_t) * n, hipMemcpyHostToDevice, g->comm));
  CBG_NCCL(ncclAllGather(d.p + P * n, d.p, n, ncclInt64, pick(g, which), g->comm));
  CBG_HIP(hipMemcpyAsync(out, d.p, sizeof(int64_t) * P * n, hipMemcpyDeviceToHost, g->comm));
  CBG_HIP(hipStreamSynchronize(g->comm));
}

void allreduce_f64(cbg_grid* g, double* v, bool max) {
  if (g->nranks == 1) return;
  if (g->host_mode) {
    std::vector<double> all(g->nranks);
    host_check(g->hc.allgather(g->hc.user, COMM_WORLD, v, all.data(), sizeof(double)), "allgather");
    double r = all[0];
    for (double x : all) r = max ? std::max(r, x) : r + x;
    *v = r;
    return;
  }
  DBuf<double> d(1);
  CBG_HIP(hipMemcpyAsync(d.p, v, sizeof(double), hipMemcpyHostToDevice, g->comm));
  CBG_NCCL(ncclAllReduce(d.p, d.p, 1, ncclFloat64, max ? ncclMax : ncclSum, g->world, g->comm));
  CBG_HIP(hipMemcpyAsync(v, d.p, sizeof(double), hipMemcpyDeviceToHost, g->comm));
  CBG_HIP(hipStreamSynchronize(g->comm));
}

void allreduce_sum_i64(cbg_grid* g, int64_t* v) {
  if (g->nranks == 1) return;
  std::vector<int64_t> all(g->nranks);
  allgather_i64(g, COMM_WORLD, v, all.data(), 1);
  int64_t s = 0;
  for (auto x : all) s += x;
  *v = s;
}

void barrier(cbg_grid* g) {
  double z = 0;
  allreduce_f64(g, &z, true);
}

// Broadcast a tile within a row/col communicator (BCastMatrix: the essentials
// {m,n,nnz,nzc} are known from the allgather; Create(ess) then 4 broadcasts).
// `t` holds the root's tile on the root; on the others it is allocated here.
// Enqueued on g->comm; the caller orders the consumer with g->ev_comm.
static void bcast_tile(cbg_grid* g, int which, int root, const int64_t ess[4], cbg_tile& t, bool mine) {
  if (!mine) tile_alloc_device(t, ess[0], ess[1], ess[2], ess[3]);
  const int64_t nnz = ess[2], nzc = ess[3];
  if (comm_size(g, which) == 1) return;
  if (g->host_mode) {
    CBG_HIP(hipStreamSynchronize(g->comm));
    auto hb = [&](void* dptr, size_t bytes) {
      if (bytes == 0) return;
      std::vector<char> h(bytes);
      if (mine) CBG_HIP(hipMemcpy(h.data(), dptr, bytes, hipMemcpyDeviceToHost));
      host_check(g->hc.bcast(g->hc.user, which, h.data(), bytes, root), "bcast");
      if (!mine) CBG_HIP(hipMemcpy(dptr, h.data(), bytes, hipMemcpyHostToDevice));
    };
    hb(t.cp, sizeof(int64_t) * (nzc + 1));
    hb(t.jc, sizeof(int32_t) * nzc);
    hb(t.ir, sizeof(int32_t) * nnz);
    hb(t.val, sizeof(double) * nnz);
    return;
  }
  ncclComm_t c = pick(g, which);
  CBG_NCCL(ncclGroupStart());
  CBG_NCCL(ncclBroadcast(t.cp, t.cp, nzc + 1, ncclInt64, root, c, g->comm));
  if (nzc) CBG_NCCL(ncclBroadcast(t.jc, t.jc, nzc, ncclInt32, root, c, g->comm));
  if (nnz) {
    CBG_NCCL(ncclBroadcast(t.ir, t.ir, nnz, ncclInt32, root, c, g->comm));
    CBG_NCCL(ncclBroadcast(t.val, t.val, nnz, ncclFloat64, root, c, g->comm));
  }
  CBG_NCCL(ncclGroupEnd());
}

static void tile_ess(const cbg_tile& t, int64_t e[4]) {
  e[0] = t.m;
  e[1] = t.n;
  e[2] = t.nnz;
  e[3] = t.nzc;
}

// ---------------------------------------------------------------------------
// Mult_AnXBn_{DoubleBuff,Synch}
// ---------------------------------------------------------------------------
int summa_spgemm(cbg_grid* g, const cbg_tile& A, const cbg_tile& B, int64_t A_gncol, int64_t B_gnrow, int sr, int algo,
                 int exec, cbg_tile& C) {
  // CheckSpGEMMCompliance (ParFriends.h:160-183)
  if (A_gncol != B_gnrow) return CBG_ERR_DIMMISMATCH;
  if (&A == &B || (A.ir == B.ir && A.nnz > 0)) return CBG_ERR_MATRIXALIAS;
  // GetSetSizes: essentials of every A tile in my grid row, every B tile in my grid column
  int64_t ea[4], eb[4];
  tile_ess(A, ea);
  tile_ess(B, eb);
  std::vector<int64_t> EA((size_t)4 * g->pc), EB((size_t)4 * g->pr);
  allgather_i64(g, COMM_ROW, ea, EA.data(), 4);
  allgather_i64(g, COMM_COL, eb, EB.data(), 4);
  int64_t kA = 0, kB = 0;
  for (int s = 0; s < g->pc; ++s) kA += EA[4 * s + 1];
  for (int s = 0; s < g->pr; ++s) kB += EB[4 * s + 0];
  if (kA != A_gncol || kB != B_gnrow) return CBG_ERR_DIMMISMATCH;
  const int64_t Cm = A.m, Cn = B.n;
  hipStream_t cs = g->compute;

  if (exec == CBG_EXEC_PANEL) {
    // gather the A block row and the B block column
    std::vector<cbg_tile> Ar(g->pc), Bc(g->pr);
    std::vector<int64_t> aoff(g->pc), boff(g->pr);
    int64_t o = 0;
    for (int s = 0; s < g->pc; ++s) {
      aoff[s] = o;
      o += EA[4 * s + 1];
      if (s == g->pcol) Ar[s] = A; else Ar[s] = cbg_tile{};
      bcast_tile(g, COMM_ROW, s, &EA[4 * s], Ar[s], s == g->pcol);
    }
    o = 0;
    for (int s = 0; s < g->pr; ++s) {
      boff[s] = o;
      o += EB[4 * s + 0];
      if (s == g->prow) Bc[s] = B; else Bc[s] = cbg_tile{};
      bcast_tile(g, COMM_COL, s, &EB[4 * s], Bc[s], s == g->prow);
    }
    CBG_HIP(hipStreamSynchronize(g->comm));
    cbg_tile Ap{}, Bp{};
    const cbg_tile* Ause = &A;
    const cbg_tile* Buse = &B;
    if (g->pc > 1) {
      tile_concat_cols(Ar, aoff, Cm, A_gncol, Ap, cs);
      Ause = &Ap;
    }
    if (g->pr > 1) {
      tile_concat_rows(Bc, boff, B_gnrow, Cn, Bp, cs);
      Buse = &Bp;
    }
    for (int s = 0; s < g->pc; ++s)
      if (s != g->pcol) tile_free_device(Ar[s]);
    for (int s = 0; s < g->pr; ++s)
      if (s != g->prow) tile_free_device(Bc[s]);
    local_spgemm(*Ause, *Buse, sr, C, cs, nullptr);
    if (g->pc > 1) tile_free_device(Ap);
    if (g->pr > 1) tile_free_device(Bp);
    return CBG_OK;
  }

  // ---------------- STAGED (reference stage structure, square grids) ----------------
  if (g->pr != g->pc) return CBG_ERR_NOTSQUARE;
  const int stages = g->pc;  // ProductGrid: innerdim = grcols
  std::vector<cbg_tile> partials;
  auto run_half = [&](const cbg_tile& Aseq, const cbg_tile& Bseq) {
    int64_t a4[4], b4[4];
    tile_ess(Aseq, a4);
    tile_ess(Bseq, b4);
    std::vector<int64_t> SA((size_t)4 * stages), SB((size_t)4 * stages);
    allgather_i64(g, COMM_ROW, a4, SA.data(), 4);  // GetSetSizes (ParFriends.h:834-835 / :1025-1026)
    allgather_i64(g, COMM_COL, b4, SB.data(), 4);
    // double buffer: stage s+1's broadcast is enqueued on the comm stream
    // before stage s's multiply runs on the compute stream
    std::vector<cbg_tile> Ar(stages), Bc(stages);
    auto post = [&](int s) {
      Ar[s] = (s == g->pcol) ? Aseq : cbg_tile{};
      Bc[s] = (s == g->prow) ? Bseq : cbg_tile{};
      bcast_tile(g, COMM_ROW, s, &SA[4 * s], Ar[s], s == g->pcol);
      bcast_tile(g, COMM_COL, s, &SB[4 * s], Bc[s], s == g->prow);
    };
    post(0);
    for (int s = 0; s < stages; ++s) {
      CBG_HIP(hipEventRecord(g->ev_comm, g->comm));
      CBG_HIP(hipStreamWaitEvent(cs, g->ev_comm, 0));
      if (s + 1 < stages) post(s + 1);
      cbg_tile P{};
      local_spgemm(Ar[s], Bc[s], sr, P, cs, nullptr);  // LocalHybridSpGEMM (ParFriends.h:888-891)
      if (s != g->pcol) tile_free_device(Ar[s]);
      if (s != g->prow) tile_free_device(Bc[s]);
      if (P.nnz > 0) partials.push_back(P); else tile_free_device(P);
    }
  };
  cbg_tile A1{}, A2{}, B1{}, B2{};
  if (algo == CBG_DOUBLEBUFF) {
    // A split by columns at n/2, B by rows at m/2 (ParFriends.h:823-829)
    tile_split_cols(A, A.n / 2, A1, A2, cs);
    tile_split_rows(B, B.m / 2, B1, B2, cs);
    run_half(A1, B1);
    run_half(A2, B2);
    tile_free_device(A1);
    tile_free_device(A2);
    tile_free_device(B1);
    tile_free_device(B2);
  } else {
    run_half(A, B);
  }
  // MergeAll (DoubleBuff, Friends.h:657-741) / MultiwayMerge (Synch, MultiwayMerge.h:409-526)
  if (partials.size() == 1) {
    C = partials[0];
  } else {
    merge_tiles(partials, Cm, Cn, sr, C, cs);
    for (auto& p : partials) tile_free_device(p);
  }
  return CBG_OK;
}


// ---------------------------------------------------------------------------
// MemEfficientSpGEMM (ParFriends.h:449-730) minus its Markov-clustering pruning:
// B's local tile is cut into `phases` column pieces like SpDCCols::ColSplit
// (SpDCCols.cpp:936-970), each piece goes through summa_spgemm, and the phase
// results are streamed to `fn` or column-concatenated (ColConcatenate,
// ParFriends.h:724-725).  Column pieces keep every C column's products inside
// one phase, so the result is identical to the unphased product.
// ---------------------------------------------------------------------------
int summa_spgemm_phased(cbg_grid* g, const cbg_tile& A, const cbg_tile& B, int64_t A_gncol, int64_t B_gnrow, int sr,
                        int algo, int exec, int phases, cbg_phase_fn fn, void* user, cbg_tile* C) {
  if (phases < 1 || phases >= A_gncol) phases = 1;  // "Resetting to 1" (ParFriends.h:469-473)
  int64_t small = B.n < phases ? 1 : 0;              // ColSplit: "Matrix is too small to be splitted"
  allreduce_sum_i64(g, &small);
  if (small) return CBG_ERR_INVALIDPARAMS;
  hipStream_t cs = g->compute;
  // column pieces of B: [p * (n / phases), (p + 1) * (n / phases)), the last takes the rest
  std::vector<cbg_tile> pieces(phases);
  std::vector<int64_t> off(phases);
  const int64_t w = B.n / phases;
  // the reference copies B first, so A and B may alias here (ParFriends.h:547-549)
  const bool alias = (&A == &B) || (A.ir == B.ir && A.nnz > 0);
  const bool copied = phases > 1 || alias;
  if (!copied) {
    pieces[0] = B;
  } else if (phases == 1) {
    cbg_tile right{};
    tile_split_cols(B, B.n, pieces[0], right, cs);
    tile_free_device(right);
  } else {
    cbg_tile rest = B;
    for (int p = 0; p < phases - 1; ++p) {
      cbg_tile left{}, right{};
      tile_split_cols(rest, w, left, right, cs);
      if (p > 0) tile_free_device(rest);
      pieces[p] = left;
      rest = right;
    }
    pieces[phases - 1] = rest;
  }
  for (int p = 0; p < phases; ++p) off[p] = (int64_t)p * w;
  std::vector<cbg_tile> parts;
  int cb_rc = 0;
  // every phase multiplies the caller's A itself when the PANEL execution needs
  // no A row concatenation (one grid column): keep its column maps across the
  // phases (other executions multiply per-stage / per-phase copies of A)
  std::unique_ptr<APrepScope> aprep_scope;
  if (exec == CBG_EXEC_PANEL && g->pc == 1) aprep_scope.reset(new APrepScope());
  for (int p = 0; p < phases; ++p) {
    cbg_tile Cp{};
    const int rc = summa_spgemm(g, A, pieces[p], A_gncol, B_gnrow, sr, algo, exec, Cp);
    if (copied) tile_free_device(pieces[p]);
    if (rc) {
      for (int q = p + 1; q < phases; ++q)
        if (copied) tile_free_device(pieces[q]);
      for (auto& t : parts) tile_free_device(t);
      return rc;
    }
    if (fn) {
      CBG_HIP(hipStreamSynchronize(cs));
      const int r = fn(user, p, off[p], &Cp);
      if (r && !cb_rc) cb_rc = r;
      tile_free_device(Cp);
    } else {
      parts.push_back(Cp);
    }
  }
  if (fn) return cb_rc ? CBG_ERR_INVALIDPARAMS : CBG_OK;
  if (parts.size() == 1) {
    *C = parts[0];
  } else {
    tile_concat_cols(parts, off, A.m, B.n, *C, cs);
    for (auto& t : parts) tile_free_device(t);
  }
  return CBG_OK;
}


// ---------------------------------------------------------------------------
// SpParMat::Transpose (SpParMat.cpp:3528-3590) on a square grid: a diagonal
// rank transposes its tile; rank (r,c) transposes the tile of its complement
// (c,r) (GetComplementRank), received over RCCL send/recv (host transport:
// world broadcasts, test only).  `out` is this rank's tile of the transpose.
// ---------------------------------------------------------------------------
int grid_transpose(cbg_grid* g, const cbg_tile& T, cbg_tile& out) {
  if (g->pr != g->pc) return CBG_ERR_NOTSQUARE;
  hipStream_t cs = g->compute;
  // essentials of every rank's tile (world allgather: collective, diagonal ranks too)
  int64_t e[4] = {T.m, T.n, T.nnz, T.nzc};
  std::vector<int64_t> E((size_t)4 * g->nranks);
  allgather_i64(g, COMM_WORLD, e, E.data(), 4);
  const bool diag = g->prow == g->pcol;
  const int peer = g->pcol * g->pc + g->prow;
  const int64_t* pe = &E[4 * (size_t)peer];
  cbg_tile R{};
  if (!diag) tile_alloc_device(R, pe[0], pe[1], pe[2], pe[3]);
  if (g->host_mode && g->nranks > 1) {
    // every off-diagonal rank broadcasts its tile over the world communicator
    for (int q = 0; q < g->nranks; ++q) {
      const int qr = q / g->pc, qc = q % g->pc;
      if (qr == qc) continue;
      const int64_t* qe = &E[4 * (size_t)q];
      const bool mine = q == g->rank, keep = !diag && q == peer;
      auto hb = [&](void* dst, const void* src, size_t bytes) {
        if (bytes == 0) return;
        std::vector<char> h(bytes);
        if (mine) CBG_HIP(hipMemcpy(h.data(), src, bytes, hipMemcpyDeviceToHost));
        host_check(g->hc.bcast(g->hc.user, COMM_WORLD, h.data(), bytes, q), "transpose bcast");
        if (keep) CBG_HIP(hipMemcpy(dst, h.data(), bytes, hipMemcpyHostToDevice));
      };
      hb(R.cp, T.cp, sizeof(int64_t) * (qe[3] + 1));
      hb(R.jc, T.jc, sizeof(int32_t) * qe[3]);
      hb(R.ir, T.ir, sizeof(int32_t) * qe[2]);
      hb(R.val, T.val, sizeof(double) * qe[2]);
    }
  } else if (!diag) {
    ncclComm_t c = g->world;
    CBG_NCCL(ncclGroupStart());
    CBG_NCCL(ncclSend(T.cp, T.nzc + 1, ncclInt64, peer, c, g->comm));
    CBG_NCCL(ncclRecv(R.cp, pe[3] + 1, ncclInt64, peer, c, g->comm));
    if (T.nzc) CBG_NCCL(ncclSend(T.jc, T.nzc, ncclInt32, peer, c, g->comm));
    if (pe[3]) CBG_NCCL(ncclRecv(R.jc, pe[3], ncclInt32, peer, c, g->comm));
    if (T.nnz) {
      CBG_NCCL(ncclSend(T.ir, T.nnz, ncclInt32, peer, c, g->comm));
      CBG_NCCL(ncclSend(T.val, T.nnz, ncclFloat64, peer, c, g->comm));
    }
    if (pe[2]) {
      CBG_NCCL(ncclRecv(R.ir, pe[2], ncclInt32, peer, c, g->comm));
      CBG_NCCL(ncclRecv(R.val, pe[2], ncclFloat64, peer, c, g->comm));
    }
    CBG_NCCL(ncclGroupEnd());
    CBG_HIP(hipStreamSynchronize(g->comm));
  }
  if (diag) {
    tile_transpose(T, out, cs);
  } else {
    tile_transpose(R, out, cs);
    tile_free_device(R);
  }
  return CBG_OK;
}

// ---------------------------------------------------------------------------
// SpParMat::BlockSplit (SpParMat.cpp:2974-3058) for the splits BlockSpGEMM
// uses (bi = 1, BlockSpGEMM.h:39-45): global rows [lo, hi) of a distributed
// matrix (dim 0) or columns [lo, hi) (dim 1) as a distributed matrix of its
// own on the same grid, in the standard block layout (Owner,
// SpParMat.cpp:5068-5097).  Rows only move inside a grid column (columns
// inside a grid row): every rank broadcasts its slice of the range to its
// column (row) communicator and keeps the part of each slice that falls in
// its new block.
// ---------------------------------------------------------------------------
int grid_block_extract(cbg_grid* g, const cbg_tile& T, int64_t gm, int64_t gn, int dim, int64_t lo, int64_t hi,
                       cbg_tile& out) {
  if (dim != 0 && dim != 1) return CBG_ERR_INVALIDPARAMS;
  const int64_t gext = dim == 0 ? gm : gn;
  if (lo < 0 || hi < lo || hi > gext) return CBG_ERR_INVALIDPARAMS;
  hipStream_t cs = g->compute;
  const int which = dim == 0 ? COMM_COL : COMM_ROW;
  const int np = comm_size(g, which), me = comm_rank(g, which);
  // my old range [S0, S1) along dim and my new range [lo + T0, lo + T1)
  auto span = [](int64_t ext, int np_, int i, int64_t& a, int64_t& b) {
    const int64_t per = ext / np_;
    a = (int64_t)i * per;
    b = i == np_ - 1 ? ext : a + per;
  };
  int64_t S0, S1, T0, T1;
  span(gext, np, me, S0, S1);
  span(hi - lo, np, me, T0, T1);
  T0 += lo;
  T1 += lo;
  auto cut = [&](const cbg_tile& X, int64_t a, int64_t b, cbg_tile& piece) {  // local range [a, b) of X
    cbg_tile head{}, rest{}, tail{};
    if (dim == 0) {
      tile_split_rows(X, b, head, tail, cs);
      tile_free_device(tail);
      tile_split_rows(head, a, rest, piece, cs);
    } else {
      tile_split_cols(X, b, head, tail, cs);
      tile_free_device(tail);
      tile_split_cols(head, a, rest, piece, cs);
    }
    tile_free_device(rest);
    tile_free_device(head);
  };
  // my slice of [lo, hi)
  const int64_t x0 = std::max(S0, lo), x1 = std::max(x0, std::min(S1, hi));
  cbg_tile mine{};
  cut(T, x0 - S0, x1 - S0, mine);
  int64_t e[4] = {mine.m, mine.n, mine.nnz, mine.nzc};
  std::vector<int64_t> E((size_t)4 * np);
  allgather_i64(g, which, e, E.data(), 4);
  std::vector<cbg_tile> parts;
  std::vector<int64_t> offs;
  for (int q = 0; q < np; ++q) {
    int64_t Q0, Q1;
    span(gext, np, q, Q0, Q1);
    const int64_t y0 = std::max(Q0, lo), y1 = std::max(y0, std::min(Q1, hi));  // slice of rank q
    cbg_tile sl = q == me ? mine : cbg_tile{};
    bcast_tile(g, which, q, &E[4 * (size_t)q], sl, q == me);
    CBG_HIP(hipStreamSynchronize(g->comm));
    const int64_t z0 = std::max(y0, T0), z1 = std::min(y1, T1);  // the part of it in my new range
    if (z1 > z0) {
      cbg_tile piece{};
      cut(sl, z0 - y0, z1 - y0, piece);
      parts.push_back(piece);
      offs.push_back(z0 - T0);
    }
    if (q != me) tile_free_device(sl);
  }
  tile_free_device(mine);
  const int64_t om = dim == 0 ? T1 - T0 : T.m, on = dim == 0 ? T.n : T1 - T0;
  if (parts.empty()) {
    tile_alloc_device(out, om, on, 0, 0);
  } else if (dim == 0) {
    tile_concat_rows(parts, offs, om, on, out, cs);
  } else {
    tile_concat_cols(parts, offs, om, on, out, cs);
  }
  for (auto& t : parts) tile_free_device(t);
  CBG_HIP(hipStreamSynchronize(cs));
  return CBG_OK;
}

}  // namespace cbg

extern "C" int cbg_get_unique_id(void* id) {
  if (!id) return CBG_ERR_INVALIDPARAMS;
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return CBG_ERR_RCCL;
  std::memcpy(id, &u, sizeof(u));
  return CBG_OK;
}

extern "C" int cbg_grid_info(const cbg_grid* g, int* rank, int* nranks, int* rows, int* cols, int* prow, int* pcol) {
  if (!g) return CBG_ERR_INVALIDPARAMS;
  if (rank) *rank = g->rank;
  if (nranks) *nranks = g->nranks;
  if (rows) *rows = g->pr;
  if (cols) *cols = g->pc;
  if (prow) *prow = g->prow;
  if (pcol) *pcol = g->pcol;
  return CBG_OK;
}
