/*
 * spmv_ref.c — TEST INFRASTRUCTURE (oracle).  Plain-C restatement of the
 * reference's CPU hot path, used as bench.py's CPU baseline
 * (cpu_baseline.kind = "port") and as the checker at BASELINE sizes, where
 * the Python oracle is too slow.  Never linked into the product.
 *
 * Restated (reference paths relative to /root/reference):
 *  - the local kernel mul!(C, A::SubSparseMatrix{SparseMatrixCSC}, B, α, β)
 *    SparseUtils.jl:157-187: column loop, Int64 colptr/rowval,
 *    `i = invrows[I]*rflag; if i>0: C[i] += nzv[p]*αxj`, after
 *    `fill!(C, 0)` for β = 0 (SparseUtils.jl:167-168, Interfaces.jl:2261-2266);
 *  - mul!(c::PVector, a::PSparseMatrix, b::PVector) (Interfaces.jl:2246-2275)
 *    on Cartesian parts: the owned_owned block (columns by oid), then the
 *    owned_ghost block (columns by hid) after the exchange;
 *  - the partition of the benchmark driver (partitionedarrays.jl_amd/
 *    drivers.py stencil_partition): rows = PRange(parts, (N,N,N)) (Cartesian,
 *    Interfaces.jl:1114-1137, _oid_to_gid 1307-1319), cols = rows + the ghosts
 *    that add_gids!(rows, J) (Interfaces.jl:579-603, 1515-1533) appends in
 *    first-touch order of the row-wise COO (owned rows by oid, neighbours in
 *    (dz,dy,dx) lexicographic order);
 *  - the operators: the 27-point Q1-hex FE operator of test_fem_sa.jl's
 *    pattern in 3D (Dirichlet rows keep their diagonal, one 1.0 per touching
 *    cell; entries summed over the cells holding both nodes in ascending cell
 *    order), or test_fdm.jl's 7-point operator (Dirichlet rows: identity),
 *    assembled as `sparse` does (CSC, rows ascending in each column);
 *  - IterativeSolvers.cg! v0.9 (not vendored; SURVEY.md §3.5, called at
 *    test_fdm.jl:115): u = 0; r = b; c = A*x; r .-= c; residual = norm(r);
 *    tol = max(reltol*norm(b), abstol); prev = 1; per iteration
 *    β = res²/prev²; u .= r .+ β.*u; mul!(c,A,u); α = res²/dot(u,c);
 *    x .+= α.*u; r .-= α.*c; prev = res; res = norm(r).  dot and norm fold
 *    the parts' owned partials in part order (reduce(+; init=0),
 *    Interfaces.jl:221-238, 1767-1772, 1985-1992); the local sums run over
 *    the owned values in oid order (the reference's BLAS internals are
 *    unpinned).
 *
 * Modes (F64; x fastest; gids 0-based in the files):
 *  spmv_ref --kind 27|7 --n N [--reps R] [--xin f --yout f]
 *      one part, literal CSC column loop over the whole operator
 *  spmv_ref ... --parts PX PY PZ [--threads T] [--literal] --xin f --yout f
 *      partitioned mul!: each owned row summed in the reference's order
 *      (owned columns by oid, then ghost columns by hid).  Row-wise by
 *      default (the per-row sequence of the column loop); --literal builds
 *      each part's local CSC and runs the column loop itself over the
 *      owned_owned then owned_ghost views (small sizes: the cross-check).
 *  spmv_ref ... [--parts ...] --cg K --bin f [--xin f] [--hist f] [--xout f]
 *      [--reltol r] [--abstol a] [--dot seq|pairwise]
 *      cg! with maxiter = K (x0 = 0 without --xin); --dot: the local
 *      summation order of dot/norm (below)
 *  spmv_ref --kind 27|7 --n N --seconds S --ranks P
 *      CPU baseline: MPIBackend with P ranks on P host threads; the rows
 *      split into P contiguous blocks (PRange(parts, n), Interfaces.jl:
 *      1014-1030), each rank holding the CSC of its owned rows over its local
 *      columns and running the column loop on its own copy of x, then a
 *      barrier (the halo exchange and PTimer's max-over-ranks).
 *  spmv_ref --kind 27|7 (--n N | --dims X Y Z) --parts PX PY PZ --mpi
 *      (--seconds S | --reps R) [--xin f --yout f]
 *      CPU baseline beside the multi-GPU lines: MPIBackend over the Cartesian
 *      parts, one rank (thread, core) per part, each with its local CSC, its
 *      Exchanger and a halo exchange of x in every mul! (run_mpi below)
 *  spmv_ref --kind 27|7 --n N --dtype f32|c128 --xin f --yout f
 *      one part, the literal column loop in Float32 / ComplexF64
 *      (Float32.(A) / A .* (1+0.5im))
 * --dims gives the global nodes per dimension (default N N N; the operator's
 * h follows N[0], as drivers.py stencil_coeffs).
 * Every mode prints one JSON line.
 */
#define _POSIX_C_SOURCE 200809L
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static double now(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

static void* xmalloc(size_t n) {
  void* p = malloc(n ? n : 1);
  if (!p) { fprintf(stderr, "out of memory (%zu bytes)\n", n); exit(1); }
  return p;
}

/* ---- the operators ------------------------------------------------------ */
static double Ke[64];
static int64_t N3[3];          /* global nodes per dim (x, y, z) */
static int kind;
static double fd_diag, fd_off;
static int K;                 /* stencil points */
static int off_d[27][3];      /* (dx,dy,dz) in (dz,dy,dx) lexicographic order */
static double interior_val[27];

static void q1_hex_ke(double h) {
  const double K1[2][2] = {{1.0, -1.0}, {-1.0, 1.0}};
  const double M1[2][2] = {{1.0 / 3.0, 1.0 / 6.0}, {1.0 / 6.0, 1.0 / 3.0}};
  for (int a = 0; a < 8; ++a)
    for (int b = 0; b < 8; ++b) {
      int ax = a & 1, ay = (a >> 1) & 1, az = a >> 2;
      int bx = b & 1, by = (b >> 1) & 1, bz = b >> 2;
      double t1 = (K1[az][bz] * M1[ay][by]) * M1[ax][bx];
      double t2 = (M1[az][bz] * K1[ay][by]) * M1[ax][bx];
      double t3 = (M1[az][bz] * M1[ay][by]) * K1[ax][bx];
      Ke[a * 8 + b] = h * ((t1 + t2) + t3);
    }
}

static int dirichlet(int64_t x, int64_t y, int64_t z) {
  return x == 0 || y == 0 || z == 0 || x == N3[0] - 1 || y == N3[1] - 1 || z == N3[2] - 1;
}

/* entry (row node g, column node g+d): Ke summed over the cells holding both,
 * in ascending cell order (the cell loop's COO order, combined by sparse) */
static double fe_value(int64_t gx, int64_t gy, int64_t gz, int dx, int dy, int dz) {
  double acc = 0.0;
  int first = 1;
  for (int cz = -1; cz <= 0; ++cz) {
    int64_t c2 = gz + cz;
    int bz = (int)(gz + dz - c2);
    if (c2 < 0 || c2 > N3[2] - 2 || bz < 0 || bz > 1) continue;
    for (int cy = -1; cy <= 0; ++cy) {
      int64_t c1 = gy + cy;
      int by = (int)(gy + dy - c1);
      if (c1 < 0 || c1 > N3[1] - 2 || by < 0 || by > 1) continue;
      for (int cx = -1; cx <= 0; ++cx) {
        int64_t c0 = gx + cx;
        int bx = (int)(gx + dx - c0);
        if (c0 < 0 || c0 > N3[0] - 2 || bx < 0 || bx > 1) continue;
        int a = (int)(gx - c0) + 2 * (int)(gy - c1) + 4 * (int)(gz - c2);
        double v = Ke[a * 8 + bx + 2 * by + 4 * bz];
        acc = first ? v : acc + v;
        first = 0;
      }
    }
  }
  return acc;
}

static double ncells(int64_t gx, int64_t gy, int64_t gz) {
  double acc = 0.0;
  int first = 1;
  for (int cz = -1; cz <= 0; ++cz) {
    if (gz + cz < 0 || gz + cz > N3[2] - 2) continue;
    for (int cy = -1; cy <= 0; ++cy) {
      if (gy + cy < 0 || gy + cy > N3[1] - 2) continue;
      for (int cx = -1; cx <= 0; ++cx) {
        if (gx + cx < 0 || gx + cx > N3[0] - 2) continue;
        acc = first ? 1.0 : acc + 1.0;
        first = 0;
      }
    }
  }
  return acc;
}

static double dirichlet_val(int64_t x, int64_t y, int64_t z) { return kind == 7 ? 1.0 : ncells(x, y, z); }

static void setup_operator(void) {
  const double h = 2.0 / (double)(N3[0] - 1);  /* drivers.py stencil_coeffs: h from N[0] */
  q1_hex_ke(h);
  fd_diag = -((-6.0) / (h * h));
  fd_off = -(1.0 / (h * h));
  K = 0;
  for (int dz = -1; dz <= 1; ++dz)
    for (int dy = -1; dy <= 1; ++dy)
      for (int dx = -1; dx <= 1; ++dx) {
        int nz = (dx != 0) + (dy != 0) + (dz != 0);
        if (kind == 7 && nz > 1) continue;
        off_d[K][0] = dx; off_d[K][1] = dy; off_d[K][2] = dz;
        /* every non-Dirichlet node has all 8 cells: the same values as node (1,1,1) */
        interior_val[K] = kind == 7 ? (nz == 0 ? fd_diag : fd_off) : (N3[0] >= 3 && N3[1] >= 3 && N3[2] >= 3 ? fe_value(1, 1, 1, dx, dy, dz) : 0.0);
        ++K;
      }
}

/* row r's entries (ascending column = lexicographic neighbour order) */
static int row_entries(int64_t r, int64_t* cols, double* vals) {
  int64_t x = r % N3[0], y = (r / N3[0]) % N3[1], z = r / (N3[0] * N3[1]);
  if (dirichlet(x, y, z)) {
    cols[0] = r;
    vals[0] = dirichlet_val(x, y, z);
    return 1;
  }
  for (int k = 0; k < K; ++k) {
    cols[k] = (x + off_d[k][0]) + N3[0] * ((y + off_d[k][1]) + N3[1] * (z + off_d[k][2]));
    vals[k] = interior_val[k]; /* == fe_value at every non-Dirichlet node (checked by --literal) */
  }
  return K;
}

/* ---- a tiny thread pool: parallel_for over [0, n) in chunks ------------- */
typedef void (*range_fn)(void* ctx, int64_t lo, int64_t hi);
typedef struct { range_fn fn; void* ctx; int64_t n; int t, T; } PFArg;
static int g_threads = 1;

static void* pf_run(void* a) {
  PFArg* p = (PFArg*)a;
  const int64_t lo = p->n * p->t / p->T, hi = p->n * (p->t + 1) / p->T;
  if (lo < hi) p->fn(p->ctx, lo, hi);
  return NULL;
}

static void parallel_for(int64_t n, range_fn fn, void* ctx) {
  int T = g_threads;
  if (T > n) T = (int)(n > 0 ? n : 1);
  if (T <= 1) { if (n > 0) fn(ctx, 0, n); return; }
  pthread_t th[256];
  PFArg args[256];
  if (T > 256) T = 256;
  for (int t = 0; t < T; ++t) {
    args[t] = (PFArg){fn, ctx, n, t, T};
    pthread_create(&th[t], NULL, pf_run, &args[t]);
  }
  for (int t = 0; t < T; ++t) pthread_join(th[t], NULL);
}

/* ---- Cartesian parts ---------------------------------------------------- */
/* _oid_to_gid (Interfaces.jl:1307-1319), 0-based first and length */
static void oid_range(int64_t ng, int np, int p, int64_t* first, int64_t* len) {
  const int64_t ol = ng / np, off = ol * (p - 1), rem = ng % np;
  if (rem < (np - p + 1)) { *first = off; *len = ol; }
  else { *first = off + p - (np - rem) - 1; *len = ol + 1; }
}

typedef struct {
  int64_t lo[3], n[3];      /* owned box, 0-based global origin */
  int64_t nown, nghost;
  int32_t* shell;           /* (n+2)^3 extended box → hid (0-based) or -1 */
} Part;

static int P3[3] = {1, 1, 1};
static int nparts = 1;
static Part* parts;

static inline int64_t shell_idx(const Part* q, int64_t ex, int64_t ey, int64_t ez) {
  return ex + (q->n[0] + 2) * (ey + (q->n[1] + 2) * ez);
}

/* add_gids!(rows, J) over the row-wise COO: ghosts in first-touch order */
static void build_part(Part* q, int part) {
  int c[3] = {(part - 1) % P3[0], ((part - 1) / P3[0]) % P3[1], (part - 1) / (P3[0] * P3[1])};
  for (int d = 0; d < 3; ++d) oid_range(N3[d], P3[d], c[d] + 1, &q->lo[d], &q->n[d]);
  q->nown = q->n[0] * q->n[1] * q->n[2];
  const int64_t ext = (q->n[0] + 2) * (q->n[1] + 2) * (q->n[2] + 2);
  q->shell = xmalloc((size_t)ext * sizeof(int32_t));
  for (int64_t i = 0; i < ext; ++i) q->shell[i] = -1;
  int64_t nh = 0;
  for (int64_t lz = 0; lz < q->n[2]; ++lz)
    for (int64_t ly = 0; ly < q->n[1]; ++ly)
      for (int64_t lx = 0; lx < q->n[0]; ++lx) {
        const int face = lx == 0 || ly == 0 || lz == 0 || lx == q->n[0] - 1 || ly == q->n[1] - 1 || lz == q->n[2] - 1;
        if (!face) continue;  /* no neighbour outside the box */
        const int64_t gx = q->lo[0] + lx, gy = q->lo[1] + ly, gz = q->lo[2] + lz;
        if (dirichlet(gx, gy, gz)) continue;  /* its only column is itself */
        for (int k = 0; k < K; ++k) {
          const int64_t ex = lx + off_d[k][0], ey = ly + off_d[k][1], ez = lz + off_d[k][2];
          if (ex >= 0 && ey >= 0 && ez >= 0 && ex < q->n[0] && ey < q->n[1] && ez < q->n[2]) continue;
          const int64_t s = shell_idx(q, ex + 1, ey + 1, ez + 1);
          if (q->shell[s] < 0) q->shell[s] = (int32_t)nh++;
        }
      }
  q->nghost = nh;
}

static inline int64_t gid3(int64_t x, int64_t y, int64_t z) { return x + N3[0] * (y + N3[1] * z); }

/* y[owned row] of one part, in the reference's order: the owned_owned
 * block's columns by oid, then the owned_ghost block's by hid */
static inline double row_apply(const Part* q, int64_t lx, int64_t ly, int64_t lz, const double* x) {
  const int64_t gx = q->lo[0] + lx, gy = q->lo[1] + ly, gz = q->lo[2] + lz;
  double acc = 0.0; /* fill!(co, 0) */
  if (dirichlet(gx, gy, gz)) return acc + dirichlet_val(gx, gy, gz) * x[gid3(gx, gy, gz)];
  int64_t key[27];
  double v[27], xv[27];
  int m = 0;
  for (int k = 0; k < K; ++k) {
    const int64_t ex = lx + off_d[k][0], ey = ly + off_d[k][1], ez = lz + off_d[k][2];
    int64_t kk;
    if (ex >= 0 && ey >= 0 && ez >= 0 && ex < q->n[0] && ey < q->n[1] && ez < q->n[2])
      kk = ex + q->n[0] * (ey + q->n[1] * ez);                        /* oid - 1 */
    else
      kk = q->nown + q->shell[shell_idx(q, ex + 1, ey + 1, ez + 1)];  /* nown + hid - 1 */
    /* insertion by key: owned (ascending oid) before ghosts (ascending hid) */
    int t = m++;
    while (t > 0 && key[t - 1] > kk) { key[t] = key[t - 1]; v[t] = v[t - 1]; xv[t] = xv[t - 1]; --t; }
    key[t] = kk;
    v[t] = interior_val[k];
    xv[t] = x[gid3(gx + off_d[k][0], gy + off_d[k][1], gz + off_d[k][2])];
  }
  for (int t = 0; t < m; ++t) acc += v[t] * xv[t]; /* C[i] += nzv[p]*αxj, α = 1 */
  return acc;
}

typedef struct { const double* x; double* y; } SpmvCtx;

/* work item = (part, z-plane) */
static void spmv_range(void* vctx, int64_t lo, int64_t hi) {
  SpmvCtx* c = (SpmvCtx*)vctx;
  for (int64_t w = lo; w < hi; ++w) {
    int64_t acc = 0;
    int p = 0;
    while (w >= acc + parts[p].n[2]) { acc += parts[p].n[2]; ++p; }
    const Part* q = &parts[p];
    const int64_t lz = w - acc;
    for (int64_t ly = 0; ly < q->n[1]; ++ly)
      for (int64_t lx = 0; lx < q->n[0]; ++lx)
        c->y[gid3(q->lo[0] + lx, q->lo[1] + ly, q->lo[2] + lz)] = row_apply(q, lx, ly, lz, c->x);
  }
}

static int64_t total_planes(void) {
  int64_t s = 0;
  for (int p = 0; p < nparts; ++p) s += parts[p].n[2];
  return s;
}

static void spmv_parts(const double* x, double* y) {
  SpmvCtx c = {x, y};
  parallel_for(total_planes(), spmv_range, &c);
}

/* --literal: each part's local CSC (rows: owned lids; columns: owned oids,
 * then ghosts by hid) and the column loop of SparseUtils.jl:176-185 over the
 * owned_owned view (flag (1,1)), then the owned_ghost view (flag (1,-1)) */
static void spmv_parts_literal(const double* x, double* y) {
  for (int p = 0; p < nparts; ++p) {
    const Part* q = &parts[p];
    const int64_t nl = q->nown + q->nghost;
    int64_t* colptr = calloc((size_t)nl + 1, sizeof(int64_t));
    int64_t* lid_gid = xmalloc((size_t)nl * sizeof(int64_t));
    for (int64_t lz = 0; lz < q->n[2]; ++lz)
      for (int64_t ly = 0; ly < q->n[1]; ++ly)
        for (int64_t lx = 0; lx < q->n[0]; ++lx)
          lid_gid[lx + q->n[0] * (ly + q->n[1] * lz)] = gid3(q->lo[0] + lx, q->lo[1] + ly, q->lo[2] + lz);
    for (int64_t ez = 0; ez < q->n[2] + 2; ++ez)
      for (int64_t ey = 0; ey < q->n[1] + 2; ++ey)
        for (int64_t ex = 0; ex < q->n[0] + 2; ++ex) {
          const int32_t h = q->shell[shell_idx(q, ex, ey, ez)];
          if (h >= 0) lid_gid[q->nown + h] = gid3(q->lo[0] + ex - 1, q->lo[1] + ey - 1, q->lo[2] + ez - 1);
        }
    /* entries (row lid, col lid, value) of the owned rows */
    int64_t cap = q->nown * K, ne = 0;
    int64_t* er = xmalloc((size_t)cap * sizeof(int64_t));
    int64_t* ec = xmalloc((size_t)cap * sizeof(int64_t));
    double* ev = xmalloc((size_t)cap * sizeof(double));
    for (int64_t lz = 0; lz < q->n[2]; ++lz)
      for (int64_t ly = 0; ly < q->n[1]; ++ly)
        for (int64_t lx = 0; lx < q->n[0]; ++lx) {
          const int64_t gx = q->lo[0] + lx, gy = q->lo[1] + ly, gz = q->lo[2] + lz;
          const int64_t row = lx + q->n[0] * (ly + q->n[1] * lz);
          if (dirichlet(gx, gy, gz)) {
            er[ne] = row; ec[ne] = row; ev[ne] = dirichlet_val(gx, gy, gz); ++ne;
            continue;
          }
          for (int k = 0; k < K; ++k) {
            const int64_t ex = lx + off_d[k][0], ey = ly + off_d[k][1], ez = lz + off_d[k][2];
            int64_t cl;
            if (ex >= 0 && ey >= 0 && ez >= 0 && ex < q->n[0] && ey < q->n[1] && ez < q->n[2])
              cl = ex + q->n[0] * (ey + q->n[1] * ez);
            else
              cl = q->nown + q->shell[shell_idx(q, ex + 1, ey + 1, ez + 1)];
            er[ne] = row; ec[ne] = cl;
            ev[ne] = kind == 7 ? interior_val[k] : fe_value(gx, gy, gz, off_d[k][0], off_d[k][1], off_d[k][2]);
            ++ne;
          }
        }
    for (int64_t e = 0; e < ne; ++e) colptr[ec[e] + 1]++;
    for (int64_t j = 0; j < nl; ++j) colptr[j + 1] += colptr[j];
    int64_t* rowval = xmalloc((size_t)ne * sizeof(int64_t));
    double* nzval = xmalloc((size_t)ne * sizeof(double));
    int64_t* cur = xmalloc((size_t)nl * sizeof(int64_t));
    memcpy(cur, colptr, (size_t)nl * sizeof(int64_t));
    for (int64_t e = 0; e < ne; ++e) { /* entries by ascending row → rows ascending per column */
      const int64_t pp = cur[ec[e]]++;
      rowval[pp] = er[e] + 1;
      nzval[pp] = ev[e];
    }
    for (int64_t j = 0; j <= nl; ++j) colptr[j] += 1;
    double* C = xmalloc((size_t)q->nown * sizeof(double));
    for (int64_t i = 0; i < q->nown; ++i) C[i] = 0.0; /* fill!(co, 0) */
    for (int blk = 0; blk < 2; ++blk) {  /* owned_owned, then owned_ghost */
      const int64_t j0 = blk == 0 ? 0 : q->nown, j1 = blk == 0 ? q->nown : nl;
      for (int64_t J = j0; J < j1; ++J) {
        const double axj = x[lid_gid[J]] * 1.0;
        for (int64_t pp = colptr[J] - 1; pp < colptr[J + 1] - 1; ++pp) {
          const int64_t i = rowval[pp]; /* invrows: owned row lids are their oids */
          if (i > 0) C[i - 1] += nzval[pp] * axj;
        }
      }
    }
    for (int64_t i = 0; i < q->nown; ++i) y[lid_gid[i]] = C[i];
    free(C); free(cur); free(rowval); free(nzval); free(er); free(ec); free(ev); free(colptr); free(lid_gid);
  }
}

/* ---- reductions over parts (owned values, oid order, folded in part order)
 * The local sum of a part runs over its owned values in oid order:
 * sequentially (default), or pairwise (--dot pairwise: halves down to 128
 * values, as blocked BLAS kernels do).  The reference's local dot/nrm2 is
 * BLAS, whose order is unpinned; the two orders bound the
 * rounding spread a CG trajectory inherits from that choice.              */
static int g_pairwise = 0;

static double pair_sum(const double* a, const double* b, const int64_t* idx, int64_t n) {
  if (n <= 128) {
    double s = 0.0;
    for (int64_t i = 0; i < n; ++i) s += a[idx[i]] * b[idx[i]];
    return s;
  }
  const int64_t h = n / 2;
  return pair_sum(a, b, idx, h) + pair_sum(a, b, idx + h, n - h);
}

typedef struct { const double* a; const double* b; double* part_sum; } DotCtx;
static void dot_range(void* vctx, int64_t lo, int64_t hi) {
  DotCtx* c = (DotCtx*)vctx;
  for (int64_t p = lo; p < hi; ++p) {
    const Part* q = &parts[p];
    double s = 0.0;
    if (g_pairwise) {
      int64_t* idx = xmalloc((size_t)q->nown * sizeof(int64_t));
      int64_t k = 0;
      for (int64_t lz = 0; lz < q->n[2]; ++lz)
        for (int64_t ly = 0; ly < q->n[1]; ++ly)
          for (int64_t lx = 0; lx < q->n[0]; ++lx) idx[k++] = gid3(q->lo[0] + lx, q->lo[1] + ly, q->lo[2] + lz);
      s = pair_sum(c->a, c->b, idx, q->nown);
      free(idx);
    } else {
      for (int64_t lz = 0; lz < q->n[2]; ++lz)
        for (int64_t ly = 0; ly < q->n[1]; ++ly) {
          const int64_t g = gid3(q->lo[0], q->lo[1] + ly, q->lo[2] + lz);
          for (int64_t lx = 0; lx < q->n[0]; ++lx) s += c->a[g + lx] * c->b[g + lx];
        }
    }
    c->part_sum[p] = s;
  }
}
static double pdot(const double* a, const double* b) {
  double* ps = xmalloc((size_t)nparts * sizeof(double));
  DotCtx c = {a, b, ps};
  parallel_for(nparts, dot_range, &c);
  double s = 0.0; /* reduce(+, …; init=0) in part order */
  for (int p = 0; p < nparts; ++p) s = s + ps[p];
  free(ps);
  return s;
}
static double pnorm(const double* a) { return sqrt(pdot(a, a)); }

typedef struct { double* y; const double* x; double a; int mode; int64_t n; } AxCtx;
static void ax_range(void* vctx, int64_t lo, int64_t hi) {
  AxCtx* c = (AxCtx*)vctx;
  for (int64_t i = lo; i < hi; ++i) {
    switch (c->mode) {
      case 0: c->y[i] = c->x[i] + c->a * c->y[i]; break; /* u .= r .+ β.*u */
      case 1: c->y[i] = c->y[i] + c->a * c->x[i]; break; /* x .+= α.*u */
      case 2: c->y[i] = c->y[i] - c->a * c->x[i]; break; /* r .-= α.*c */
      case 3: c->y[i] = c->y[i] - c->x[i]; break;        /* r .-= c */
    }
  }
}
static void axpby(double* y, const double* x, double a, int mode, int64_t n) {
  AxCtx c = {y, x, a, mode, n};
  parallel_for(n, ax_range, &c);
}

/* ---- the MPIBackend-like CPU baseline (ranks on threads) ---------------- */
typedef struct {
  int64_t r0, r1;          /* owned global rows [r0, r1) */
  int64_t c0, nc;          /* local columns: global c0 .. c0+nc-1 (owned + ghosts) */
  int64_t *colptr, *rowval;
  double *nzval, *x, *y;
  int32_t* invrows;        /* local row lid → ohid (all owned here) */
  int64_t nnz;
  const double* B;
} Rank;

static pthread_barrier_t g_bar;
static volatile int g_stop;
static int g_reps_target;
static double g_seconds;
static int g_done;

static void* rank_build(void* arg) {
  Rank* R = (Rank*)arg;
  const int64_t nrow = R->r1 - R->r0;
  int64_t cols[27];
  double vals[27];
  int64_t lo = R->r0, hi = R->r1 - 1;
  for (int64_t r = R->r0; r < R->r1; ++r) {
    int k = row_entries(r, cols, vals);
    for (int t = 0; t < k; ++t) {
      if (cols[t] < lo) lo = cols[t];
      if (cols[t] > hi) hi = cols[t];
    }
  }
  R->c0 = lo;
  R->nc = hi - lo + 1;
  R->colptr = calloc((size_t)R->nc + 1, sizeof(int64_t));
  int64_t nnz = 0;
  for (int64_t r = R->r0; r < R->r1; ++r) {
    int k = row_entries(r, cols, vals);
    for (int t = 0; t < k; ++t) R->colptr[cols[t] - lo + 1]++;
    nnz += k;
  }
  R->nnz = nnz;
  for (int64_t j = 0; j < R->nc; ++j) R->colptr[j + 1] += R->colptr[j];
  R->rowval = xmalloc((size_t)nnz * sizeof(int64_t));
  R->nzval = xmalloc((size_t)nnz * sizeof(double));
  int64_t* cur = xmalloc((size_t)R->nc * sizeof(int64_t));
  memcpy(cur, R->colptr, (size_t)R->nc * sizeof(int64_t));
  for (int64_t r = R->r0; r < R->r1; ++r) {
    int k = row_entries(r, cols, vals);
    for (int t = 0; t < k; ++t) {
      int64_t p = cur[cols[t] - lo]++;
      R->rowval[p] = r - R->r0 + 1;
      R->nzval[p] = vals[t];
    }
  }
  free(cur);
  for (int64_t j = 0; j <= R->nc; ++j) R->colptr[j] += 1;
  R->invrows = xmalloc((size_t)nrow * sizeof(int32_t));
  for (int64_t i = 0; i < nrow; ++i) R->invrows[i] = (int32_t)(i + 1);
  R->x = xmalloc((size_t)R->nc * sizeof(double));
  memcpy(R->x, R->B + lo, (size_t)R->nc * sizeof(double));
  R->y = xmalloc((size_t)nrow * sizeof(double));
  return NULL;
}

static void* rank_run(void* arg) {
  Rank* R = (Rank*)arg;
  const int64_t nrow = R->r1 - R->r0;
  const double alpha = 1.0;
  double t0 = 0.0;
  for (int it = 0;; ++it) {
    pthread_barrier_wait(&g_bar);
    if (it == 0) t0 = now();
    if (g_stop) break;
    memset(R->y, 0, (size_t)(nrow > 0 ? nrow : 1) * sizeof(double));
    for (int64_t j = 0; j < R->nc; ++j) {
      const double axj = R->x[j] * alpha;
      for (int64_t p = R->colptr[j] - 1; p < R->colptr[j + 1] - 1; ++p) {
        const int32_t i = R->invrows[R->rowval[p] - 1];
        if (i > 0) R->y[i - 1] += R->nzval[p] * axj;
      }
    }
    if (pthread_barrier_wait(&g_bar) == PTHREAD_BARRIER_SERIAL_THREAD) {
      ++g_done;
      if (g_reps_target > 0 ? g_done >= g_reps_target : (now() - t0) >= g_seconds) g_stop = 1;
    }
  }
  return NULL;
}

static void* read_bytes(const char* path, size_t nbytes) {
  void* v = xmalloc(nbytes);
  FILE* f = fopen(path, "rb");
  if (!f || fread(v, 1, nbytes, f) != nbytes) { fprintf(stderr, "bad input file %s\n", path); exit(1); }
  fclose(f);
  return v;
}

static void write_bytes(const char* path, const void* v, size_t nbytes) {
  FILE* f = fopen(path, "wb");
  if (!f || fwrite(v, 1, nbytes, f) != nbytes) { fprintf(stderr, "cannot write %s\n", path); exit(1); }
  fclose(f);
}

static double* read_vec(const char* path, int64_t n) { return read_bytes(path, (size_t)n * sizeof(double)); }
static void write_vec(const char* path, const double* v, int64_t n) { write_bytes(path, v, (size_t)n * sizeof(double)); }

static void seeded_vec(double* B, int64_t n) {
  uint64_t s = 20250114u;
  for (int64_t i = 0; i < n; ++i) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    B[i] = ((double)(s >> 11) / 9007199254740992.0) * 2.0 - 1.0;
  }
}

static int run_ranks(int ranks, int reps, double seconds, const double* B, int64_t n) {
  Rank* Rk = calloc((size_t)ranks, sizeof(Rank));
  pthread_t* th = xmalloc((size_t)ranks * sizeof(pthread_t));
  for (int q = 0; q < ranks; ++q) { /* _oid_to_gid (Interfaces.jl:1307-1319), 0-based */
    int64_t off, len;
    oid_range(n, ranks, q + 1, &off, &len);
    Rk[q].r0 = off;
    Rk[q].r1 = off + len;
    Rk[q].B = B;
    pthread_create(&th[q], NULL, rank_build, &Rk[q]); /* each rank assembles its own CSC */
  }
  int64_t nnz = 0;
  for (int q = 0; q < ranks; ++q) { pthread_join(th[q], NULL); nnz += Rk[q].nnz; }
  pthread_barrier_init(&g_bar, NULL, (unsigned)ranks);
  g_reps_target = reps;
  g_seconds = seconds;
  double t0 = now();
  for (int q = 0; q < ranks; ++q) pthread_create(&th[q], NULL, rank_run, &Rk[q]);
  for (int q = 0; q < ranks; ++q) pthread_join(th[q], NULL);
  double t1 = now();
  const double per = (t1 - t0) / g_done;
  const double bytes = (double)nnz * 12.0 + (double)(n + 1) * 4.0 + (double)n * 16.0;
  double cs = 0.0;
  for (int q = 0; q < ranks; ++q)
    for (int64_t i = 0; i < Rk[q].r1 - Rk[q].r0; ++i) cs += Rk[q].y[i];
  printf("{\"kind\": %d, \"n_per_dim\": %lld, \"rows\": %lld, \"nnz\": %lld, \"ranks\": %d, \"reps\": %d, "
         "\"sec_per_spmv\": %.9g, \"gbps\": %.6g, \"bytes_per_spmv\": %.0f, \"checksum\": %.17g}\n",
         kind, (long long)N3[0], (long long)n, (long long)nnz, ranks, g_done, per, bytes / per / 1e9, bytes, cs);
  return 0;
}

/* ---- MPIBackend over Cartesian parts (--mpi): the CPU baseline beside the
 * multi-GPU lines.  One rank per part (one thread each, one core each, as
 * `mpiexec -n P` with one core per rank), each holding what MPIBackend's
 * part holds: the local CSC of its owned rows over its local columns (owned
 * oids, then ghosts by hid; Int64 colptr/rowval, 1-based), its x with the
 * ghost layer, and the Exchanger of x (Interfaces.jl:723-786: parts_rcv the
 * sorted owners of its ghosts, lids_rcv its ghost lids grouped by owner in
 * ascending lid, lids_snd the owner's lids in the receiver's order).  One
 * mul! (Interfaces.jl:2246-2275) per step:
 *   async_exchange!(b): pack lids_snd into the send buffers, post (barrier:
 *   every message delivered once every rank has packed, MPIBackend.jl:
 *   261-309's Isend/Irecv + Waitall);
 *   the owned_owned block: fill!(c, 0), column loop over the owned columns
 *   (SparseUtils.jl:157-187, `i>0` filter);
 *   wait: copy each received segment from the sender's buffer and unpack it
 *   into the ghost lids;
 *   the owned_ghost block: column loop over the ghost columns;
 *   then PTimer's barrier (max over ranks).                               */
typedef struct {
  int p;                       /* 0-based part */
  const Part* q;
  int64_t nl, nnz;
  int64_t *colptr, *rowval;    /* 1-based, Julia's CSC */
  double* nzval;
  int32_t* invrows;            /* lid_to_ohid of the rows (all owned) */
  double *x, *y;
  int nin, nout;               /* neighbours: receive from / send to */
  int *in_part, *out_part;     /* sorted */
  int64_t *in_ptr, *out_ptr;
  int32_t *in_lids, *in_oid;   /* my ghost lids by owner; the owner's oid of each */
  int32_t* out_lids;           /* my owned lids, in each receiver's order */
  double *snd, *rcv;
  const double** in_src;       /* per incoming segment: the sender's send segment */
} MRank;

static MRank* g_mr;
static const double* g_mpi_x;   /* --xin: the global x (else sin(0.001*gid)) */

static int owner_coord(int64_t ng, int np, int64_t g) {
  for (int c = 0; c < np; ++c) {
    int64_t f, l;
    oid_range(ng, np, c + 1, &f, &l);
    if (g >= f && g < f + l) return c;
  }
  return -1;
}

static int64_t col_lid(const Part* q, int64_t lx, int64_t ly, int64_t lz, int k) {
  const int64_t ex = lx + off_d[k][0], ey = ly + off_d[k][1], ez = lz + off_d[k][2];
  if (ex >= 0 && ey >= 0 && ez >= 0 && ex < q->n[0] && ey < q->n[1] && ez < q->n[2])
    return ex + q->n[0] * (ey + q->n[1] * ez);
  return q->nown + q->shell[shell_idx(q, ex + 1, ey + 1, ez + 1)];
}

static void* mrank_build(void* arg) {
  MRank* R = (MRank*)arg;
  const Part* q = R->q;
  R->nl = q->nown + q->nghost;
  /* ghosts: global coords → owner part and its oid, hid order */
  int32_t* own_part = xmalloc((size_t)(q->nghost + 1) * sizeof(int32_t));
  int32_t* own_oid = xmalloc((size_t)(q->nghost + 1) * sizeof(int32_t));
  int64_t* ghost_gid = xmalloc((size_t)(q->nghost + 1) * sizeof(int64_t));
  for (int64_t ez = 0; ez < q->n[2] + 2; ++ez)
    for (int64_t ey = 0; ey < q->n[1] + 2; ++ey)
      for (int64_t ex = 0; ex < q->n[0] + 2; ++ex) {
        const int32_t h = q->shell[shell_idx(q, ex, ey, ez)];
        if (h < 0) continue;
        const int64_t g[3] = {q->lo[0] + ex - 1, q->lo[1] + ey - 1, q->lo[2] + ez - 1};
        int c[3];
        int64_t f[3], l[3];
        for (int d = 0; d < 3; ++d) {
          c[d] = owner_coord(N3[d], P3[d], g[d]);
          oid_range(N3[d], P3[d], c[d] + 1, &f[d], &l[d]);
        }
        own_part[h] = c[0] + P3[0] * (c[1] + P3[1] * c[2]);
        own_oid[h] = (int32_t)((g[0] - f[0]) + l[0] * ((g[1] - f[1]) + l[1] * (g[2] - f[2])));
        ghost_gid[h] = gid3(g[0], g[1], g[2]);
      }
  /* parts_rcv / lids_rcv: ghosts grouped by owner (sorted), ascending lid */
  int* cnt = calloc((size_t)nparts, sizeof(int));
  for (int64_t h = 0; h < q->nghost; ++h) cnt[own_part[h]]++;
  R->nin = 0;
  for (int t = 0; t < nparts; ++t) R->nin += cnt[t] > 0;
  R->in_part = xmalloc((size_t)(R->nin + 1) * sizeof(int));
  R->in_ptr = xmalloc((size_t)(R->nin + 1) * sizeof(int64_t));
  int64_t* start = xmalloc((size_t)nparts * sizeof(int64_t));
  R->in_ptr[0] = 0;
  for (int t = 0, k = 0; t < nparts; ++t) {
    start[t] = R->in_ptr[k];
    if (!cnt[t]) continue;
    R->in_part[k] = t;
    R->in_ptr[k + 1] = R->in_ptr[k] + cnt[t];
    ++k;
  }
  R->in_lids = xmalloc((size_t)(q->nghost + 1) * sizeof(int32_t));
  R->in_oid = xmalloc((size_t)(q->nghost + 1) * sizeof(int32_t));
  for (int64_t h = 0; h < q->nghost; ++h) {
    const int64_t t = start[own_part[h]]++;
    R->in_lids[t] = (int32_t)(q->nown + h);
    R->in_oid[t] = own_oid[h];
  }
  free(cnt); free(start); free(own_part); free(own_oid);
  R->rcv = xmalloc((size_t)(q->nghost + 1) * sizeof(double));
  R->in_src = xmalloc((size_t)(R->nin + 1) * sizeof(double*));
  /* the local CSC: count per column, then fill in row (= oid) order, so the
   * rows of each column ascend (sparse's CSC) */
  R->colptr = calloc((size_t)R->nl + 1, sizeof(int64_t));
  int64_t nnz = 0;
  for (int64_t lz = 0; lz < q->n[2]; ++lz)
    for (int64_t ly = 0; ly < q->n[1]; ++ly)
      for (int64_t lx = 0; lx < q->n[0]; ++lx) {
        const int64_t row = lx + q->n[0] * (ly + q->n[1] * lz);
        if (dirichlet(q->lo[0] + lx, q->lo[1] + ly, q->lo[2] + lz)) { R->colptr[row + 1]++; ++nnz; continue; }
        for (int k = 0; k < K; ++k) R->colptr[col_lid(q, lx, ly, lz, k) + 1]++;
        nnz += K;
      }
  for (int64_t j = 0; j < R->nl; ++j) R->colptr[j + 1] += R->colptr[j];
  R->nnz = nnz;
  R->rowval = xmalloc((size_t)nnz * sizeof(int64_t));
  R->nzval = xmalloc((size_t)nnz * sizeof(double));
  int64_t* cur = xmalloc((size_t)R->nl * sizeof(int64_t));
  memcpy(cur, R->colptr, (size_t)R->nl * sizeof(int64_t));
  for (int64_t lz = 0; lz < q->n[2]; ++lz)
    for (int64_t ly = 0; ly < q->n[1]; ++ly)
      for (int64_t lx = 0; lx < q->n[0]; ++lx) {
        const int64_t gx = q->lo[0] + lx, gy = q->lo[1] + ly, gz = q->lo[2] + lz;
        const int64_t row = lx + q->n[0] * (ly + q->n[1] * lz);
        if (dirichlet(gx, gy, gz)) {
          const int64_t pp = cur[row]++;
          R->rowval[pp] = row + 1;
          R->nzval[pp] = dirichlet_val(gx, gy, gz);
          continue;
        }
        for (int k = 0; k < K; ++k) {
          const int64_t pp = cur[col_lid(q, lx, ly, lz, k)]++;
          R->rowval[pp] = row + 1;
          R->nzval[pp] = interior_val[k];
        }
      }
  free(cur);
  for (int64_t j = 0; j <= R->nl; ++j) R->colptr[j] += 1;
  R->invrows = xmalloc((size_t)(q->nown + 1) * sizeof(int32_t));
  for (int64_t i = 0; i < q->nown; ++i) R->invrows[i] = (int32_t)(i + 1);
  /* x: the seeded global vector's owned and ghost values */
  R->x = xmalloc((size_t)(R->nl + 1) * sizeof(double));
  R->y = xmalloc((size_t)(q->nown + 1) * sizeof(double));
  for (int64_t lz = 0; lz < q->n[2]; ++lz)
    for (int64_t ly = 0; ly < q->n[1]; ++ly)
      for (int64_t lx = 0; lx < q->n[0]; ++lx) {
        const int64_t g = gid3(q->lo[0] + lx, q->lo[1] + ly, q->lo[2] + lz);
        R->x[lx + q->n[0] * (ly + q->n[1] * lz)] = g_mpi_x ? g_mpi_x[g] : sin(0.001 * (double)g);
      }
  for (int64_t h = 0; h < q->nghost; ++h) R->x[q->nown + h] = 0.0;  /* filled by the exchange */
  free(ghost_gid);
  return NULL;
}

/* lids_snd of every part: for each receiver (sorted), the oids it listed */
static void mrank_link(void) {
  for (int s = 0; s < nparts; ++s) {
    MRank* S = &g_mr[s];
    S->nout = 0;
    int64_t tot = 0;
    for (int r = 0; r < nparts; ++r)
      for (int k = 0; k < g_mr[r].nin; ++k)
        if (g_mr[r].in_part[k] == s) { S->nout++; tot += g_mr[r].in_ptr[k + 1] - g_mr[r].in_ptr[k]; }
    S->out_part = xmalloc((size_t)(S->nout + 1) * sizeof(int));
    S->out_ptr = xmalloc((size_t)(S->nout + 1) * sizeof(int64_t));
    S->out_lids = xmalloc((size_t)(tot + 1) * sizeof(int32_t));
    S->snd = xmalloc((size_t)(tot + 1) * sizeof(double));
    S->out_ptr[0] = 0;
    int m = 0;
    for (int r = 0; r < nparts; ++r)
      for (int k = 0; k < g_mr[r].nin; ++k) {
        if (g_mr[r].in_part[k] != s) continue;
        const int64_t a = g_mr[r].in_ptr[k], b = g_mr[r].in_ptr[k + 1];
        S->out_part[m] = r;
        for (int64_t t = a; t < b; ++t) S->out_lids[S->out_ptr[m] + t - a] = g_mr[r].in_oid[t];
        S->out_ptr[m + 1] = S->out_ptr[m] + (b - a);
        g_mr[r].in_src[k] = S->snd + S->out_ptr[m];
        ++m;
      }
  }
}

static void mrank_cols(MRank* R, int64_t j0, int64_t j1) {
  const double alpha = 1.0;
  for (int64_t j = j0; j < j1; ++j) {
    const double axj = R->x[j] * alpha;
    for (int64_t p = R->colptr[j] - 1; p < R->colptr[j + 1] - 1; ++p) {
      const int32_t i = R->invrows[R->rowval[p] - 1];
      if (i > 0) R->y[i - 1] += R->nzval[p] * axj;
    }
  }
}

static void* mrank_run(void* arg) {
  MRank* R = (MRank*)arg;
  const Part* q = R->q;
  double t0 = 0.0;
  for (int it = 0;; ++it) {
    pthread_barrier_wait(&g_bar);
    if (it == 0) t0 = now();
    if (g_stop) break;
    for (int k = 0; k < R->nout; ++k)  /* pack + post */
      for (int64_t t = R->out_ptr[k]; t < R->out_ptr[k + 1]; ++t) R->snd[t] = R->x[R->out_lids[t]];
    pthread_barrier_wait(&g_bar);      /* delivered */
    memset(R->y, 0, (size_t)(q->nown > 0 ? q->nown : 1) * sizeof(double));
    mrank_cols(R, 0, q->nown);         /* owned_owned */
    for (int k = 0; k < R->nin; ++k) { /* wait: receive + unpack */
      const int64_t a = R->in_ptr[k], b = R->in_ptr[k + 1];
      memcpy(R->rcv + a, R->in_src[k], (size_t)(b - a) * sizeof(double));
      for (int64_t t = a; t < b; ++t) R->x[R->in_lids[t]] = R->rcv[t];
    }
    mrank_cols(R, q->nown, R->nl);     /* owned_ghost */
    if (pthread_barrier_wait(&g_bar) == PTHREAD_BARRIER_SERIAL_THREAD) {
      ++g_done;
      if (g_reps_target > 0 ? g_done >= g_reps_target : (now() - t0) >= g_seconds) g_stop = 1;
    }
  }
  return NULL;
}

static int run_mpi(int reps, double seconds, const char* yout) {
  g_mr = calloc((size_t)nparts, sizeof(MRank));
  pthread_t* th = xmalloc((size_t)nparts * sizeof(pthread_t));
  double tb = now();
  for (int p = 0; p < nparts; ++p) {
    g_mr[p].p = p;
    g_mr[p].q = &parts[p];
    pthread_create(&th[p], NULL, mrank_build, &g_mr[p]); /* each rank assembles its own CSC */
  }
  for (int p = 0; p < nparts; ++p) pthread_join(th[p], NULL);
  mrank_link();
  tb = now() - tb;
  pthread_barrier_init(&g_bar, NULL, (unsigned)nparts);
  g_reps_target = reps;
  g_seconds = seconds;
  double t0 = now();
  for (int p = 0; p < nparts; ++p) pthread_create(&th[p], NULL, mrank_run, &g_mr[p]);
  for (int p = 0; p < nparts; ++p) pthread_join(th[p], NULL);
  const double per = (now() - t0) / g_done;
  double bytes = 0.0, cs = 0.0;
  int64_t nnz = 0, ghosts = 0, halo = 0;
  for (int p = 0; p < nparts; ++p) {
    const MRank* R = &g_mr[p];
    const int64_t no = R->q->nown, ng = R->q->nghost, ns = R->out_ptr[R->nout], nr = R->in_ptr[R->nin];
    /* nnz(S+I) + (n_own+1)I + (n_own+n_ghost)S + n_own S + (n_snd+n_rcv)(I+2S) */
    bytes += (double)R->nnz * 12.0 + (double)(no + 1) * 4.0 + (double)(no + ng) * 8.0 + (double)no * 8.0 +
             (double)(ns + nr) * 20.0;
    nnz += R->nnz;
    ghosts += ng;
    halo += nr;
    for (int64_t i = 0; i < no; ++i) cs += R->y[i];
  }
  if (yout) {  /* y by gid (the owned values of every part) */
    double* Y = xmalloc((size_t)N3[0] * N3[1] * N3[2] * sizeof(double));
    for (int p = 0; p < nparts; ++p) {
      const Part* q = g_mr[p].q;
      for (int64_t lz = 0; lz < q->n[2]; ++lz)
        for (int64_t ly = 0; ly < q->n[1]; ++ly)
          for (int64_t lx = 0; lx < q->n[0]; ++lx)
            Y[gid3(q->lo[0] + lx, q->lo[1] + ly, q->lo[2] + lz)] = g_mr[p].y[lx + q->n[0] * (ly + q->n[1] * lz)];
    }
    write_vec(yout, Y, N3[0] * N3[1] * N3[2]);
    free(Y);
  }
  printf("{\"mode\": \"mpi\", \"kind\": %d, \"dims\": [%lld, %lld, %lld], \"parts\": [%d, %d, %d], \"ranks\": %d, "
         "\"nnz\": %lld, \"ghosts\": %lld, \"halo_values\": %lld, \"reps\": %d, \"build_s\": %.3f, "
         "\"sec_per_spmv\": %.9g, \"gbps\": %.6g, \"bytes_per_spmv\": %.0f, \"checksum\": %.17g}\n",
         kind, (long long)N3[0], (long long)N3[1], (long long)N3[2], P3[0], P3[1], P3[2], nparts, (long long)nnz,
         (long long)ghosts, (long long)halo, g_done, tb, per, bytes / per / 1e9, bytes, cs);
  return 0;
}

/* ---- one part, the literal CSC column loop, in Float32 / ComplexF64 -------
 * A in T (Float32: Float32.(A), each Float64 value rounded once; ComplexF64:
 * A .* (1+0.5im) entrywise, Complex(v*1, v*0.5), as BASELINE config 5 and
 * the device stencil build it), x and y in T; C[i] += nzv[p]*(B[j]*α) with α = 1,
 * Julia's complex product (re = a.re*b.re - a.im*b.im, im = a.re*b.im +
 * a.im*b.re), no FMA (-ffp-contract=off).                                   */
typedef struct { double re, im; } cplx;

static void onepart_f32(int64_t n, const int64_t* colptr, const int64_t* rowval, const double* nz64,
                        const int32_t* invrows, const float* B, float* Cv) {
  for (int64_t i = 0; i < n; ++i) Cv[i] = 0.0f;
  for (int64_t j = 0; j < n; ++j) {
    const float axj = B[j];
    for (int64_t p = colptr[j] - 1; p < colptr[j + 1] - 1; ++p) {
      const int32_t i = invrows[rowval[p] - 1];
      if (i > 0) Cv[i - 1] += (float)nz64[p] * axj;
    }
  }
}

static void onepart_c128(int64_t n, const int64_t* colptr, const int64_t* rowval, const double* nz64,
                         const int32_t* invrows, const cplx* B, cplx* Cv) {
  for (int64_t i = 0; i < n; ++i) Cv[i].re = Cv[i].im = 0.0;
  for (int64_t j = 0; j < n; ++j) {
    const cplx axj = B[j];
    for (int64_t p = colptr[j] - 1; p < colptr[j + 1] - 1; ++p) {
      const int32_t i = invrows[rowval[p] - 1];
      if (i > 0) {
        const cplx a = {nz64[p] * 1.0, nz64[p] * 0.5};  /* A .* (1+0.5im), BASELINE config 5 */
        const double pr = a.re * axj.re - a.im * axj.im, pi = a.re * axj.im + a.im * axj.re;
        Cv[i - 1].re = Cv[i - 1].re + pr;
        Cv[i - 1].im = Cv[i - 1].im + pi;
      }
    }
  }
}

int main(int argc, char** argv) {
  N3[0] = N3[1] = N3[2] = 64;
  int mpi = 0;
  const char* dtype = "f64";
  kind = 27;
  double seconds = 10.0, reltol = 0.0, abstol = 0.0;
  int reps = 0, ranks = 1, literal = 0, have_parts = 0, cg = 0;
  const char *xin = NULL, *yout = NULL, *bin = NULL, *hist = NULL, *xout = NULL;
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "--n") && i + 1 < argc) N3[0] = N3[1] = N3[2] = atoll(argv[++i]);
    else if (!strcmp(argv[i], "--dims") && i + 3 < argc) { for (int d = 0; d < 3; ++d) N3[d] = atoll(argv[++i]); }
    else if (!strcmp(argv[i], "--mpi")) mpi = 1;
    else if (!strcmp(argv[i], "--dtype") && i + 1 < argc) dtype = argv[++i];
    else if (!strcmp(argv[i], "--kind") && i + 1 < argc) kind = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--seconds") && i + 1 < argc) seconds = atof(argv[++i]);
    else if (!strcmp(argv[i], "--reps") && i + 1 < argc) reps = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--ranks") && i + 1 < argc) ranks = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--threads") && i + 1 < argc) g_threads = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--parts") && i + 3 < argc) {
      for (int d = 0; d < 3; ++d) P3[d] = atoi(argv[++i]);
      have_parts = 1;
    }
    else if (!strcmp(argv[i], "--literal")) literal = 1;
    else if (!strcmp(argv[i], "--dot") && i + 1 < argc) g_pairwise = !strcmp(argv[++i], "pairwise");
    else if (!strcmp(argv[i], "--cg") && i + 1 < argc) cg = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--reltol") && i + 1 < argc) reltol = atof(argv[++i]);
    else if (!strcmp(argv[i], "--abstol") && i + 1 < argc) abstol = atof(argv[++i]);
    else if (!strcmp(argv[i], "--xin") && i + 1 < argc) xin = argv[++i];
    else if (!strcmp(argv[i], "--yout") && i + 1 < argc) yout = argv[++i];
    else if (!strcmp(argv[i], "--bin") && i + 1 < argc) bin = argv[++i];
    else if (!strcmp(argv[i], "--hist") && i + 1 < argc) hist = argv[++i];
    else if (!strcmp(argv[i], "--xout") && i + 1 < argc) xout = argv[++i];
    else { fprintf(stderr, "unknown argument %s\n", argv[i]); return 2; }
  }
  if (kind != 7 && kind != 27) { fprintf(stderr, "kind must be 7 or 27\n"); return 2; }
  if (N3[0] < 3 || N3[1] < 3 || N3[2] < 3) { fprintf(stderr, "n must be >= 3\n"); return 2; }
  const int dt = !strcmp(dtype, "f32") ? 1 : !strcmp(dtype, "c128") ? 2 : !strcmp(dtype, "f64") ? 0 : -1;
  if (dt < 0) { fprintf(stderr, "dtype must be f64, f32 or c128\n"); return 2; }
  if (dt != 0 && (have_parts || cg || ranks > 1 || mpi)) { fprintf(stderr, "--dtype f32|c128: one-part mode only\n"); return 2; }
  if (g_threads < 1) g_threads = 1;
  setup_operator();
  const int64_t n = N3[0] * N3[1] * N3[2];

  if (ranks > 1) {
    double* B = xmalloc((size_t)n * sizeof(double));
    if (xin) { free(B); B = read_vec(xin, n); } else seeded_vec(B, n);
    return run_ranks(ranks, reps, seconds, B, n);
  }

  if (have_parts || cg) {
    nparts = P3[0] * P3[1] * P3[2];
    if (nparts < 1) { fprintf(stderr, "bad --parts\n"); return 2; }
    for (int d = 0; d < 3; ++d)
      if (P3[d] > N3[d]) { fprintf(stderr, "more parts than nodes\n"); return 2; }
    parts = calloc((size_t)nparts, sizeof(Part));
    int64_t nghost = 0;
    for (int p = 0; p < nparts; ++p) { build_part(&parts[p], p + 1); nghost += parts[p].nghost; }
    if (mpi) {
      if (xin) g_mpi_x = read_vec(xin, n);
      return run_mpi(reps, seconds, yout);
    }
    void (*spmv)(const double*, double*) = literal ? spmv_parts_literal : spmv_parts;
    double t0 = now();
    if (!cg) {
      if (!xin || !yout) { fprintf(stderr, "--parts needs --xin and --yout\n"); return 2; }
      double* x = read_vec(xin, n);
      double* y = xmalloc((size_t)n * sizeof(double));
      spmv(x, y);
      write_vec(yout, y, n);
      double cs = 0.0;
      for (int64_t i = 0; i < n; ++i) cs += y[i];
      printf("{\"mode\": \"spmv\", \"kind\": %d, \"n_per_dim\": %lld, \"parts\": [%d, %d, %d], \"ghosts\": %lld, "
             "\"literal\": %d, \"seconds\": %.3f, \"checksum\": %.17g}\n",
             kind, (long long)N3[0], P3[0], P3[1], P3[2], (long long)nghost, literal, now() - t0, cs);
      return 0;
    }
    if (!bin) { fprintf(stderr, "--cg needs --bin\n"); return 2; }
    double* b = read_vec(bin, n);
    double* x = xin ? read_vec(xin, n) : calloc((size_t)n, sizeof(double));
    double* u = calloc((size_t)n, sizeof(double));
    double* r = xmalloc((size_t)n * sizeof(double));
    double* c = xmalloc((size_t)n * sizeof(double));
    double* h = xmalloc((size_t)(cg > 0 ? cg : 1) * sizeof(double));
    memcpy(r, b, (size_t)n * sizeof(double));      /* copyto!(r, b) */
    spmv(x, c);                                   /* mul!(c, A, x) */
    axpby(r, c, 0.0, 3, n);                       /* r .-= c */
    double residual = pnorm(r);
    const double nb = pnorm(b);
    const double tol = fmax(reltol * nb, abstol);
    double prev = 1.0;
    int it = 0;
    while (!(it >= cg || residual <= tol)) {
      const double beta = (residual * residual) / (prev * prev);
      axpby(u, r, beta, 0, n);                    /* u .= r .+ β.*u */
      spmv(u, c);                                 /* mul!(c, A, u) */
      const double alpha = (residual * residual) / pdot(u, c);
      axpby(x, u, alpha, 1, n);                   /* x .+= α.*u */
      axpby(r, c, alpha, 2, n);                   /* r .-= α.*c */
      prev = residual;
      residual = pnorm(r);
      h[it++] = residual;
    }
    if (hist) write_vec(hist, h, it);
    if (xout) write_vec(xout, x, n);
    printf("{\"mode\": \"cg\", \"kind\": %d, \"n_per_dim\": %lld, \"parts\": [%d, %d, %d], \"iterations\": %d, "
           "\"residual0_norm_b\": %.17g, \"residual\": %.17g, \"seconds\": %.3f}\n",
           kind, (long long)N3[0], P3[0], P3[1], P3[2], it, nb, residual, now() - t0);
    return 0;
  }

  /* one part, the literal CSC column loop over the whole operator */
  int64_t* colptr = calloc((size_t)n + 1, sizeof(int64_t));
  int64_t cols[27];
  double vals[27];
  int64_t nnz = 0;
  for (int64_t r = 0; r < n; ++r) {
    int k = row_entries(r, cols, vals);
    for (int t = 0; t < k; ++t) colptr[cols[t] + 1]++;
    nnz += k;
  }
  for (int64_t j = 0; j < n; ++j) colptr[j + 1] += colptr[j];
  int64_t* rowval = xmalloc((size_t)nnz * sizeof(int64_t));
  double* nzval = xmalloc((size_t)nnz * sizeof(double));
  int64_t* cur = xmalloc((size_t)n * sizeof(int64_t));
  memcpy(cur, colptr, (size_t)n * sizeof(int64_t));
  for (int64_t r = 0; r < n; ++r) { /* rows visited ascending → rows ascending per column */
    int k = row_entries(r, cols, vals);
    for (int t = 0; t < k; ++t) {
      int64_t p = cur[cols[t]]++;
      rowval[p] = r + 1; /* 1-based as Julia */
      nzval[p] = vals[t];
    }
  }
  free(cur);
  for (int64_t j = 0; j <= n; ++j) colptr[j] += 1;
  int32_t* invrows = xmalloc((size_t)n * sizeof(int32_t)); /* lid_to_ohid: owned rows 1..n */
  for (int64_t i = 0; i < n; ++i) invrows[i] = (int32_t)(i + 1);
  if (dt != 0) {  /* Float32 / ComplexF64: one literal pass, x from --xin */
    if (!xin || !yout) { fprintf(stderr, "--dtype f32|c128 needs --xin and --yout\n"); return 2; }
    const size_t es = dt == 1 ? sizeof(float) : sizeof(cplx);
    void* Bx = read_bytes(xin, (size_t)n * es);
    void* Cx = xmalloc((size_t)n * es);
    double t0 = now();
    if (dt == 1) onepart_f32(n, colptr, rowval, nzval, invrows, (const float*)Bx, (float*)Cx);
    else onepart_c128(n, colptr, rowval, nzval, invrows, (const cplx*)Bx, (cplx*)Cx);
    write_bytes(yout, Cx, (size_t)n * es);
    printf("{\"mode\": \"one-part\", \"dtype\": \"%s\", \"kind\": %d, \"n_per_dim\": %lld, \"nnz\": %lld, "
           "\"seconds\": %.3f}\n", dtype, kind, (long long)N3[0], (long long)nnz, now() - t0);
    return 0;
  }
  double* B = xin ? read_vec(xin, n) : xmalloc((size_t)n * sizeof(double));
  if (!xin) seeded_vec(B, n);
  double* Cv = xmalloc((size_t)n * sizeof(double));
  const double alpha = 1.0;
  const int rflag = 1;
  int done = 0;
  double t0 = now(), t1 = t0;
  do {
    /* mul!(co, aoo, bo, α, β=0): fill!(C, 0) then the column loop */
    memset(Cv, 0, (size_t)n * sizeof(double));
    for (int64_t j = 0; j < n; ++j) {
      const double axj = B[j] * alpha;
      for (int64_t p = colptr[j] - 1; p < colptr[j + 1] - 1; ++p) {
        const int64_t I = rowval[p];
        const int32_t i = invrows[I - 1] * rflag;
        if (i > 0) Cv[i - 1] += nzval[p] * axj;
      }
    }
    ++done;
    t1 = now();
  } while (reps > 0 ? done < reps : (t1 - t0) < seconds);
  const double per = (t1 - t0) / done;
  const double bytes = (double)nnz * 12.0 + (double)(n + 1) * 4.0 + (double)n * 16.0;
  if (yout) write_vec(yout, Cv, n);
  double cs = 0.0;
  for (int64_t i = 0; i < n; ++i) cs += Cv[i];
  printf("{\"kind\": %d, \"n_per_dim\": %lld, \"rows\": %lld, \"nnz\": %lld, \"ranks\": 1, \"reps\": %d, "
         "\"sec_per_spmv\": %.9g, \"gbps\": %.6g, \"bytes_per_spmv\": %.0f, \"checksum\": %.17g}\n",
         kind, (long long)N3[0], (long long)n, (long long)nnz, done, per, bytes / per / 1e9, bytes, cs);
  return 0;
}
