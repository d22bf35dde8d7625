/*
 * spmv_ref.c — TEST INFRASTRUCTURE (oracle).  Plain-C restatement of the
 * reference's CPU hot path, used as the CPU baseline of bench.py
 * (cpu_baseline.kind = "port") and as a checker at sizes where the Python
 * oracle is slow.  Never linked into the product.
 *
 * Restated (reference paths relative to /root/reference):
 *  - the local kernel mul!(C, A::SubSparseMatrix{SparseMatrixCSC}, B, α, β)
 *    SparseUtils.jl:157-187: column loop over the owned columns, Int64
 *    colptr/rowval, `i = invrows[I]*rflag; if i>0: C[i] += nzv[p]*αxj`,
 *    after `fill!(C, 0)` for β = 0 (Interfaces.jl:2261-2266);
 *  - the single-part operator of the benchmark: the 27-point Q1-hex FE
 *    operator of test_fem_sa.jl's pattern in 3D (Dirichlet rows keep their
 *    diagonal, one per touching cell; entries summed over the cells holding
 *    both nodes in ascending cell order), or test_fdm.jl's 7-point operator,
 *    assembled as `sparse` does (CSC, rows ascending in each column).
 *
 * Usage: spmv_ref --kind 27|7 --n N [--seconds S] [--reps R] [--ranks P]
 *                 [--xin file --yout file]   (raw float64 in/out, length N^3)
 * --ranks P (P > 1) restates MPIBackend with P ranks on P host threads: the
 * rows are split into P contiguous blocks (PRange(parts, n), Interfaces.jl:
 * 1014-1030); each rank holds the CSC of its owned rows over its local
 * columns (owned + ghost, ghosts appended) and runs the same column loop on
 * its own copy of x, then all ranks meet at a barrier (the halo exchange and
 * the max-over-ranks timing of PTimer).
 * Prints one JSON line {"rows","nnz","reps","sec_per_spmv","gbps",...}.
 * Bytes per SpMV use the same algorithmic formula as bench.py (SURVEY.md
 * §8d, Int32 index width): nnz*(8+4) + (n+1)*4 + n*8 (x) + n*8 (y).
 */
#define _POSIX_C_SOURCE 200809L
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

static double Ke[64];

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

static int64_t N;
static int kind;
static double fd_diag, fd_off;

static int dirichlet(int64_t x, int64_t y, int64_t z) {
  return x == 0 || y == 0 || z == 0 || x == N - 1 || y == N - 1 || z == N - 1;
}

static double fe_value(int64_t gx, int64_t gy, int64_t gz, int dx, int dy, int dz) {
  double acc = 0.0;
  int first = 1;
  for (int cz = -1; cz <= 0; ++cz) {
    int64_t c2 = gz + cz;
    int bz = (int)(gz + dz - c2);
    if (c2 < 0 || c2 > N - 2 || bz < 0 || bz > 1) continue;
    for (int cy = -1; cy <= 0; ++cy) {
      int64_t c1 = gy + cy;
      int by = (int)(gy + dy - c1);
      if (c1 < 0 || c1 > N - 2 || by < 0 || by > 1) continue;
      for (int cx = -1; cx <= 0; ++cx) {
        int64_t c0 = gx + cx;
        int bx = (int)(gx + dx - c0);
        if (c0 < 0 || c0 > N - 2 || bx < 0 || bx > 1) continue;
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
    if (gz + cz < 0 || gz + cz > N - 2) continue;
    for (int cy = -1; cy <= 0; ++cy) {
      if (gy + cy < 0 || gy + cy > N - 2) continue;
      for (int cx = -1; cx <= 0; ++cx) {
        if (gx + cx < 0 || gx + cx > N - 2) continue;
        acc = first ? 1.0 : acc + 1.0;
        first = 0;
      }
    }
  }
  return acc;
}

/* row r's entries (ascending column) */
static int row_entries(int64_t r, int64_t* cols, double* vals) {
  int64_t x = r % N, y = (r / N) % N, z = r / (N * N);
  if (dirichlet(x, y, z)) {
    cols[0] = r;
    vals[0] = kind == 7 ? 1.0 : ncells(x, y, z);
    return 1;
  }
  int k = 0;
  for (int dz = -1; dz <= 1; ++dz)
    for (int dy = -1; dy <= 1; ++dy)
      for (int dx = -1; dx <= 1; ++dx) {
        int nz = (dx != 0) + (dy != 0) + (dz != 0);
        if (kind == 7 && nz > 1) continue;
        cols[k] = (x + dx) + N * ((y + dy) + N * (z + dz));
        vals[k] = kind == 7 ? (nz == 0 ? fd_diag : fd_off) : fe_value(x, y, z, dx, dy, dz);
        ++k;
      }
  return k;
}

/* ---- MPIBackend-like ranks on threads -------------------------------- */
typedef struct {
  int64_t r0, r1;          /* owned global rows [r0, r1) */
  int64_t c0, nc;          /* local columns: global c0 .. c0+nc-1 (owned + ghosts) */
  int64_t *colptr, *rowval;
  double *nzval, *x, *y;
  int32_t* invrows;        /* local row lid → ohid (all owned here) */
} Rank;

static pthread_barrier_t g_bar;
static volatile int g_stop;
static int g_reps_target;
static double g_seconds;
static int g_done;

static void rank_build(Rank* R, const double* B) {
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
  for (int64_t j = 0; j < R->nc; ++j) R->colptr[j + 1] += R->colptr[j];
  R->rowval = malloc((size_t)(nnz > 0 ? nnz : 1) * sizeof(int64_t));
  R->nzval = malloc((size_t)(nnz > 0 ? nnz : 1) * sizeof(double));
  int64_t* cur = malloc((size_t)R->nc * sizeof(int64_t));
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
  R->invrows = malloc((size_t)(nrow > 0 ? nrow : 1) * sizeof(int32_t));
  for (int64_t i = 0; i < nrow; ++i) R->invrows[i] = (int32_t)(i + 1);
  R->x = malloc((size_t)R->nc * sizeof(double));
  memcpy(R->x, B + lo, (size_t)R->nc * sizeof(double));
  R->y = malloc((size_t)(nrow > 0 ? nrow : 1) * sizeof(double));
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

int main(int argc, char** argv) {
  N = 64;
  kind = 27;
  double seconds = 10.0;
  int reps = 0, ranks = 1;
  const char *xin = NULL, *yout = NULL;
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "--n") && i + 1 < argc) N = atoll(argv[++i]);
    else if (!strcmp(argv[i], "--kind") && i + 1 < argc) kind = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--seconds") && i + 1 < argc) seconds = atof(argv[++i]);
    else if (!strcmp(argv[i], "--reps") && i + 1 < argc) reps = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--ranks") && i + 1 < argc) ranks = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--xin") && i + 1 < argc) xin = argv[++i];
    else if (!strcmp(argv[i], "--yout") && i + 1 < argc) yout = argv[++i];
    else { fprintf(stderr, "unknown argument %s\n", argv[i]); return 2; }
  }
  if (kind != 7 && kind != 27) { fprintf(stderr, "kind must be 7 or 27\n"); return 2; }
  const double h = 2.0 / (double)(N - 1);
  q1_hex_ke(h);
  fd_diag = -((-6.0) / (h * h));
  fd_off = -(1.0 / (h * h));
  const int64_t n = N * N * N;
  const int maxk = kind;
  /* CSC via a counting transpose of the row lists (sparse(): rows ascending) */
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
  int64_t* rowval = malloc((size_t)nnz * sizeof(int64_t));
  double* nzval = malloc((size_t)nnz * sizeof(double));
  int64_t* cur = malloc((size_t)n * sizeof(int64_t));
  memcpy(cur, colptr, (size_t)n * sizeof(int64_t));
  for (int64_t r = 0; r < n; ++r) { /* rows visited ascending → rows ascending per column */
    int k = row_entries(r, cols, vals);
    for (int t = 0; t < k; ++t) {
      int64_t p = cur[cols[t]]++;
      rowval[p] = r + 1; /* 1-based as Julia */
      nzval[p] = vals[t];
    }
  }
  for (int64_t j = 0; j <= n; ++j) colptr[j] += 1;
  (void)maxk;
  int32_t* invrows = malloc((size_t)n * sizeof(int32_t)); /* lid_to_ohid: owned rows 1..n */
  for (int64_t i = 0; i < n; ++i) invrows[i] = (int32_t)(i + 1);
  double* B = malloc((size_t)n * sizeof(double));
  double* Cv = malloc((size_t)n * sizeof(double));
  if (xin) {
    FILE* f = fopen(xin, "rb");
    if (!f || fread(B, sizeof(double), (size_t)n, f) != (size_t)n) { fprintf(stderr, "bad --xin\n"); return 1; }
    fclose(f);
  } else {
    uint64_t s = 20250114u;
    for (int64_t i = 0; i < n; ++i) {
      s = s * 6364136223846793005ull + 1442695040888963407ull;
      B[i] = ((double)(s >> 11) / 9007199254740992.0) * 2.0 - 1.0;
    }
  }
  if (ranks > 1) {
    Rank* Rk = calloc((size_t)ranks, sizeof(Rank));
    pthread_t* th = malloc((size_t)ranks * sizeof(pthread_t));
    for (int q = 0; q < ranks; ++q) { /* _oid_to_gid (Interfaces.jl:1307-1319), 0-based */
      const int64_t ol = n / ranks, rem = n % ranks;
      const int p = q + 1;
      int64_t len = ol, off = ol * (p - 1);
      if (!(rem < (ranks - p + 1))) { len = ol + 1; off = ol * (p - 1) + p - (ranks - rem) - 1; }
      Rk[q].r0 = off;
      Rk[q].r1 = off + len;
      rank_build(&Rk[q], B);
    }
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
      for (int64_t i = 0; i < Rk[q].r1 - Rk[q].r0; ++i) {
        cs += Rk[q].y[i];
        Cv[Rk[q].r0 + i] = Rk[q].y[i];
      }
    if (yout) {
      FILE* f = fopen(yout, "wb");
      fwrite(Cv, sizeof(double), (size_t)n, f);
      fclose(f);
    }
    printf("{\"kind\": %d, \"n_per_dim\": %lld, \"rows\": %lld, \"nnz\": %lld, \"ranks\": %d, \"reps\": %d, "
           "\"sec_per_spmv\": %.9g, \"gbps\": %.6g, \"bytes_per_spmv\": %.0f, \"checksum\": %.17g}\n",
           kind, (long long)N, (long long)n, (long long)nnz, ranks, g_done, per, bytes / per / 1e9, bytes, cs);
    return 0;
  }
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
  if (yout) {
    FILE* f = fopen(yout, "wb");
    fwrite(Cv, sizeof(double), (size_t)n, f);
    fclose(f);
  }
  double cs = 0.0;
  for (int64_t i = 0; i < n; ++i) cs += Cv[i];
  printf("{\"kind\": %d, \"n_per_dim\": %lld, \"rows\": %lld, \"nnz\": %lld, \"ranks\": 1, \"reps\": %d, "
         "\"sec_per_spmv\": %.9g, \"gbps\": %.6g, \"bytes_per_spmv\": %.0f, \"checksum\": %.17g}\n",
         kind, (long long)N, (long long)n, (long long)nnz, done, per, bytes / per / 1e9, bytes, cs);
  return 0;
}
