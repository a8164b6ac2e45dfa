/* oracle.c — CPU restatement of the kmldpc per-codeword hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Plain C, compiled -O2
 * -ffp-contract=off so that every floating-point operation is the IEEE
 * operation the reference's x86-64 build performs.  Complex division uses C99
 * `double complex` division (GCC lowers it to libgcc __divdc3, exactly what the
 * reference's std::complex<double> division calls), |z| uses hypot (what
 * std::abs(std::complex<double>) calls), exp/log/sqrt/pow come from the same
 * glibc libm as the reference.
 *
 * File:line citations are relative to /root/reference/kmldpc.
 */
#define _GNU_SOURCE
#include "oracle.h"

#include <complex.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* lib/lab/include/utility.h:10-16 */
static const double kPi = 3.14159265358979;
static const double kSmallestProb = 1.0e-12;
static const double kSqrt2 = 1.4142135623730950488016;

struct orc_code {
  int M, N, K, cc_len, Z, E, chk, is5g, max_iter;
  int32_t *perm;     /* tempP */
  int32_t *row_ptr;  /* M+1 */
  int32_t *row_col;  /* E: column of slot */
  int32_t *col_ptr;  /* N+1 */
  int32_t *col_slot; /* E: slot ids in column-list order */
  uint64_t *enc;     /* reduced matrix enc_h_, M rows x W words */
  int W;
};

struct orc_modem {
  int m, Kc;
  double *pts; /* 2*Kc normalised */
};

/* ------------------------------------------------------------------ H load */

static int read_token(FILE *f, char *buf, int n) { return fscanf(f, "%1023s", buf) == 1 && n > 0; }

typedef struct {
  int32_t *cols; /* per row, file order */
  int32_t *ptr;
} raw_rows;

static inline int getbit(const uint64_t *row, int j) { return (int)((row[j >> 6] >> (j & 63)) & 1u); }
static inline void flipbit(uint64_t *row, int j) { row[j >> 6] ^= (1ull << (j & 63)); }

/* Column swap of the dense bit matrix (both columns in every row). */
static void swap_cols(uint64_t *A, int M, int W, int a, int b) {
  for (int m = 0; m < M; m++) {
    uint64_t *r = A + (size_t)m * W;
    int x = getbit(r, a), y = getbit(r, b);
    if (x != y) {
      flipbit(r, a);
      flipbit(r, b);
    }
  }
}

static void swap_rows(uint64_t *A, int W, int a, int b) {
  uint64_t *ra = A + (size_t)a * W, *rb = A + (size_t)b * W;
  for (int w = 0; w < W; w++) {
    uint64_t t = ra[w];
    ra[w] = rb[w];
    rb[w] = t;
  }
}

/* binaryldpccodec.cc:386-431: forward Gauss-Jordan with column pivoting. */
static int eliminate_forward(uint64_t *A, int M, int N, int W, int32_t *perm) {
  int chk = 0;
  for (int i = 0; i < M; i++) {
    int found = 0, ii = 0, jj;
    for (jj = i; jj < N; jj++) {
      for (ii = i; ii < M; ii++)
        if (getbit(A + (size_t)ii * W, jj)) {
          found = 1;
          break;
        }
      if (found) {
        chk++;
        break;
      }
    }
    if (!found) break;
    if (ii != i) swap_rows(A, W, i, ii);
    if (jj != i) {
      int t = perm[i];
      perm[i] = perm[jj];
      perm[jj] = t;
      swap_cols(A, M, W, i, jj);
    }
    const uint64_t *ri = A + (size_t)i * W;
    for (int m = 0; m < M; m++) {
      uint64_t *rm = A + (size_t)m * W;
      if (m != i && getbit(rm, i))
        for (int w = 0; w < W; w++) rm[w] ^= ri[w];
    }
  }
  return chk;
}

/* binary5gldpccodec.cc:281-325: backward Gauss-Jordan, pivots at the right. */
static int eliminate_backward(uint64_t *A, int M, int N, int W, int32_t *perm) {
  int chk = 0;
  for (int i = M - 1; i >= 0; --i) {
    const int c = i + N - M;
    int found = 0, ii = 0, jj;
    for (jj = c; jj >= 0; --jj) {
      for (ii = i; ii >= 0; --ii)
        if (getbit(A + (size_t)ii * W, jj)) {
          found = 1;
          break;
        }
      if (found) {
        chk++;
        break;
      }
    }
    if (!found) break;
    if (ii != i) swap_rows(A, W, i, ii);
    if (jj != c) {
      int t = perm[c];
      perm[c] = perm[jj];
      perm[jj] = t;
      swap_cols(A, M, W, c, jj);
    }
    const uint64_t *ri = A + (size_t)i * W;
    for (int m = M - 1; m >= 0; --m) {
      uint64_t *rm = A + (size_t)m * W;
      if (m != i && getbit(rm, c))
        for (int w = 0; w < W; w++) rm[w] ^= ri[w];
    }
  }
  return chk;
}

orc_code *orc_code_load(const char *path, int is5g, int active, int reversed_rows, int max_iter) {
  FILE *f = fopen(path, "r");
  if (!f) return NULL;
  char tok[1024];
  int M = 0, N = 0, rank = 0, Z = 0;
  if (!read_token(f, tok, 1024)) goto fail_f;
  if (is5g) {
    if (fscanf(f, "%d %d %d %d", &M, &N, &rank, &Z) != 4) goto fail_f;
  } else {
    if (fscanf(f, "%d %d %d", &M, &N, &rank) != 3) goto fail_f;
  }
  if (!read_token(f, tok, 1024)) goto fail_f;
  raw_rows rr;
  rr.ptr = (int32_t *)calloc(M + 1, sizeof(int32_t));
  size_t cap = (size_t)M * 8 + 16, used = 0;
  rr.cols = (int32_t *)malloc(cap * sizeof(int32_t));
  for (int i = 0; i < M; i++) {
    int row_no, deg;
    if (fscanf(f, "%d %d", &row_no, &deg) != 2) goto fail_rr;
    for (int j = 0; j < deg; j++) {
      int col;
      if (fscanf(f, "%d", &col) != 1) goto fail_rr;
      if (used == cap) {
        cap *= 2;
        rr.cols = (int32_t *)realloc(rr.cols, cap * sizeof(int32_t));
      }
      rr.cols[used++] = col;
    }
    rr.ptr[i + 1] = (int32_t)used;
  }
  fclose(f);

  orc_code *c = (orc_code *)calloc(1, sizeof(orc_code));
  c->M = M;
  c->N = N;
  c->Z = is5g ? Z : 0;
  c->is5g = is5g;
  c->max_iter = max_iter;
  c->W = (N + 63) / 64;
  c->perm = (int32_t *)malloc(sizeof(int32_t) * N);
  for (int j = 0; j < N; j++) c->perm[j] = j;
  c->chk = rank;
  const int W = c->W;
  /* dense H from the file rows (dec_h_, binaryldpccodec.cc:360-366) */
  uint64_t *H = (uint64_t *)calloc((size_t)M * W, sizeof(uint64_t));
  for (int i = 0; i < M; i++)
    for (int k = rr.ptr[i]; k < rr.ptr[i + 1]; k++) H[(size_t)i * W + (rr.cols[k] >> 6)] |= 1ull << (rr.cols[k] & 63);

  c->E = (int)used;
  c->row_ptr = (int32_t *)malloc(sizeof(int32_t) * (M + 1));
  c->row_col = (int32_t *)malloc(sizeof(int32_t) * c->E);
  if (active) {
    c->enc = (uint64_t *)malloc((size_t)M * W * sizeof(uint64_t));
    memcpy(c->enc, H, (size_t)M * W * sizeof(uint64_t));
    c->chk = is5g ? eliminate_backward(c->enc, M, N, W, c->perm) : eliminate_forward(c->enc, M, N, W, c->perm);
    /* Rebuilt graph from dec_h[i][j] = H[i][perm[j]] (binaryldpccodec.cc:441-481):
     * row list = descending new column; column list = descending row. */
    int e = 0;
    c->row_ptr[0] = 0;
    int32_t *inv = (int32_t *)malloc(sizeof(int32_t) * N);
    for (int j = 0; j < N; j++) inv[c->perm[j]] = j;
    int32_t *tmp = (int32_t *)malloc(sizeof(int32_t) * 64);
    int tcap = 64;
    for (int i = 0; i < M; i++) {
      int n = 0;
      int deg = rr.ptr[i + 1] - rr.ptr[i];
      if (deg > tcap) {
        tcap = deg * 2;
        tmp = (int32_t *)realloc(tmp, sizeof(int32_t) * tcap);
      }
      for (int k = rr.ptr[i]; k < rr.ptr[i + 1]; k++) tmp[n++] = inv[rr.cols[k]];
      /* sort descending */
      for (int a = 1; a < n; a++) {
        int v = tmp[a], b = a - 1;
        while (b >= 0 && tmp[b] < v) {
          tmp[b + 1] = tmp[b];
          b--;
        }
        tmp[b + 1] = v;
      }
      for (int a = 0; a < n; a++) c->row_col[e++] = tmp[a];
      c->row_ptr[i + 1] = e;
    }
    free(tmp);
    free(inv);
  } else {
    /* file-order graph (binaryldpccodec.cc:105-123): row list = reverse file order */
    c->row_ptr[0] = 0;
    int e = 0;
    for (int i = 0; i < M; i++) {
      for (int k = rr.ptr[i + 1] - 1; k >= rr.ptr[i]; k--) c->row_col[e++] = rr.cols[k];
      c->row_ptr[i + 1] = e;
    }
    c->enc = NULL;
  }
  if (reversed_rows) {
    for (int i = 0; i < M; i++) {
      int a = c->row_ptr[i], b = c->row_ptr[i + 1] - 1;
      while (a < b) {
        int t = c->row_col[a];
        c->row_col[a] = c->row_col[b];
        c->row_col[b] = t;
        a++;
        b--;
      }
    }
  }
  /* column lists: descending row index */
  c->col_ptr = (int32_t *)calloc(N + 1, sizeof(int32_t));
  c->col_slot = (int32_t *)malloc(sizeof(int32_t) * c->E);
  for (int e = 0; e < c->E; e++) c->col_ptr[c->row_col[e] + 1]++;
  for (int j = 0; j < N; j++) c->col_ptr[j + 1] += c->col_ptr[j];
  int32_t *fill = (int32_t *)malloc(sizeof(int32_t) * N);
  for (int j = 0; j < N; j++) fill[j] = c->col_ptr[j + 1];
  for (int i = 0; i < M; i++) /* ascending rows, fill from the back => descending */
    for (int e = c->row_ptr[i]; e < c->row_ptr[i + 1]; e++) c->col_slot[--fill[c->row_col[e]]] = e;
  free(fill);

  c->K = N - c->chk;
  c->cc_len = is5g ? N - 2 * Z : N;
  free(H);
  free(rr.cols);
  free(rr.ptr);
  return c;
fail_rr:
  free(rr.cols);
  free(rr.ptr);
fail_f:
  fclose(f);
  return NULL;
}

void orc_code_free(orc_code *c) {
  if (!c) return;
  free(c->perm);
  free(c->row_ptr);
  free(c->row_col);
  free(c->col_ptr);
  free(c->col_slot);
  free(c->enc);
  free(c);
}

void orc_code_dims(const orc_code *c, int32_t *d) {
  d[0] = c->M;
  d[1] = c->N;
  d[2] = c->K;
  d[3] = c->cc_len;
  d[4] = c->Z;
  d[5] = c->E;
  d[6] = c->chk;
  d[7] = c->max_iter;
}

void orc_code_perm(const orc_code *c, int32_t *perm) { memcpy(perm, c->perm, sizeof(int32_t) * c->N); }

void orc_code_graph(const orc_code *c, int32_t *row_ptr, int32_t *row_col, int32_t *col_ptr, int32_t *col_slot) {
  memcpy(row_ptr, c->row_ptr, sizeof(int32_t) * (c->M + 1));
  memcpy(row_col, c->row_col, sizeof(int32_t) * c->E);
  memcpy(col_ptr, c->col_ptr, sizeof(int32_t) * (c->N + 1));
  memcpy(col_slot, c->col_slot, sizeof(int32_t) * c->E);
}

/* ------------------------------------------------------------- Encoder */

void orc_encode(const orc_code *c, int32_t *uu, int32_t *cc) {
  const int N = c->N, chk = c->chk, K = c->K, W = c->W;
  if (!c->enc) { /* binaryldpccodec.cc:156-161, binary5gldpccodec.cc:103-108: the inactive
                    encoder zeroes uu (an in/out argument) and the codeword */
    for (int i = 0; i < K; i++) uu[i] = 0;
    for (int i = 0; i < c->cc_len; i++) cc[i] = 0;
    return;
  }
  if (!c->is5g) { /* binaryldpccodec.cc:148-155: cc = [parity | info] */
    for (int t = chk; t < N; t++) cc[t] = uu[t - chk];
    for (int t = 0; t < chk; t++) {
      const uint64_t *r = c->enc + (size_t)t * W;
      int acc = 0;
      for (int j = chk; j < N; j++) acc ^= (cc[j] & getbit(r, j));
      cc[t] = acc;
    }
  } else { /* binary5gldpccodec.cc:92-102: [info | parity], drop first 2Z */
    int32_t *full = (int32_t *)malloc(sizeof(int32_t) * N);
    for (int t = 0; t < K; t++) full[t] = uu[t];
    for (int t = 0; t < chk; t++) {
      const uint64_t *r = c->enc + (size_t)t * W;
      int acc = 0;
      for (int j = 0; j < K; j++) acc ^= (full[j] & getbit(r, j));
      full[K + t] = acc;
    }
    for (int t = 0; t < c->cc_len; t++) cc[t] = full[t + 2 * c->Z];
    free(full);
  }
}

/* ------------------------------------------------------------------- BP */

int orc_bp_decode(const orc_code *c, const double *p0, int iter_count, uint8_t *uu_hat, uint8_t *cc_hat_out,
                  double *syn) {
  const int M = c->M, N = c->N, E = c->E, K = c->K;
  double *buf = (double *)malloc(sizeof(double) * 6 * (size_t)E);
  double *c2v0 = buf, *c2v1 = buf + E, *v2c0 = buf + 2 * E, *v2c1 = buf + 3 * E, *al0 = buf + 4 * E,
         *al1 = buf + 5 * E;
  uint8_t *cc_hat = (uint8_t *)malloc(N);
  const int punct = c->is5g ? 2 * c->Z : 0;
  /* InitMsg: binaryldpccodec.cc:302-314 */
  for (int e = 0; e < E; e++) c2v0[e] = c2v1[e] = 0.5;
  int iter;
  for (iter = 0; iter < iter_count; iter++) {
    /* VN phase: binaryldpccodec.cc:177-213 */
    for (int v = 0; v < N; v++) {
      double a0, a1;
      if (v < punct) { /* binary5gldpccodec.cc:126-129 */
        a0 = 0.5;
        a1 = 1.0 - 0.5;
      } else {
        a0 = p0[v - punct];
        a1 = 1.0 - p0[v - punct];
      }
      const int b = c->col_ptr[v], en = c->col_ptr[v + 1];
      for (int k = b; k < en; k++) {
        const int e = c->col_slot[k];
        al0[e] = a0;
        al1[e] = a1;
        double n0 = a0 * c2v0[e];
        double n1 = a1 * c2v1[e];
        double s = n0 + n1;
        a0 = n0 / s;
        a1 = n1 / s;
      }
      cc_hat[v] = (a0 > a1) ? 0 : 1;
      double b0 = 1.0, b1 = 1.0;
      for (int k = en - 1; k >= b; k--) {
        const int e = c->col_slot[k];
        double t0 = al0[e] * b0;
        double t1 = al1[e] * b1;
        double s = t0 + t1;
        v2c0[e] = t0 / s;
        v2c1[e] = t1 / s;
        double n0 = b0 * c2v0[e];
        double n1 = b1 * c2v1[e];
        s = n0 + n1;
        b0 = n0 / s;
        b1 = n1 / s;
      }
    }
    /* binaryldpccodec.cc:214-216 / binary5gldpccodec.cc:167-170 */
    for (int i = 0; i < K; i++) uu_hat[i] = c->is5g ? cc_hat[i] : cc_hat[i + c->chk];
    /* parity check: binaryldpccodec.cc:218-232 */
    int ok = 1;
    for (int r = 0; r < M && ok; r++) {
      int p = 0;
      for (int e = c->row_ptr[r]; e < c->row_ptr[r + 1]; e++) p ^= cc_hat[c->row_col[e]];
      if (p) ok = 0;
    }
    if (ok) break;
    /* CN phase: binaryldpccodec.cc:235-275 */
    for (int r = 0; r < M; r++) {
      const int b = c->row_ptr[r], en = c->row_ptr[r + 1];
      double a0 = 1.0, a1 = 0.0;
      for (int e = b; e < en; e++) {
        al0[e] = a0;
        al1[e] = a1;
        double n0 = a0 * v2c0[e] + a1 * v2c1[e];
        double n1 = a0 * v2c1[e] + a1 * v2c0[e];
        double s = n0 + n1;
        a0 = n0 / s;
        a1 = n1 / s;
      }
      double b0 = 1.0, b1 = 0.0;
      for (int e = en - 1; e >= b; e--) {
        double t0 = al0[e] * b0 + al1[e] * b1;
        double t1 = al0[e] * b1 + al1[e] * b0;
        double s = t0 + t1;
        double q = t0 / s;
        if (q > 1.0 - kSmallestProb) q = 1.0 - kSmallestProb;
        if (q < kSmallestProb) q = kSmallestProb;
        c2v0[e] = q;
        c2v1[e] = 1.0 - q;
        double n0 = b0 * v2c0[e] + b1 * v2c1[e];
        double n1 = b0 * v2c1[e] + b1 * v2c0[e];
        s = n0 + n1;
        b0 = n0 / s;
        b1 = n1 / s;
      }
      if (syn) syn[r] = a0; /* binaryldpccodec.cc:274 */
    }
  }
  if (cc_hat_out) memcpy(cc_hat_out, cc_hat, N);
  free(cc_hat);
  free(buf);
  return iter + (iter < c->max_iter); /* binaryldpccodec.cc:277 */
}

int orc_parity_count(const orc_code *c, const uint8_t *bits) {
  int count = 0;
  for (int r = 0; r < c->M; r++) {
    int p = 0;
    for (int e = c->row_ptr[r]; e < c->row_ptr[r + 1]; e++) p ^= bits[c->row_col[e]];
    count += (p != 0);
  }
  return count;
}

/* ----------------------------------------------------------------- Modem */

orc_modem *orc_modem_load(const char *path) {
  FILE *f = fopen(path, "r");
  if (!f) return NULL;
  char tok[1024];
  int m = 0, dims = 0;
  if (!read_token(f, tok, 1024) || fscanf(f, "%d", &m) != 1 || !read_token(f, tok, 1024) || fscanf(f, "%d", &dims) != 1 ||
      !read_token(f, tok, 1024)) {
    fclose(f);
    return NULL;
  }
  orc_modem *md = (orc_modem *)calloc(1, sizeof(orc_modem));
  md->m = m;
  md->Kc = 1 << m;
  md->pts = (double *)malloc(sizeof(double) * 2 * md->Kc);
  double energies = 0;
  for (int i = 0; i < md->Kc; i++) {
    int dec, acc = 0;
    if (fscanf(f, "%d", &dec) != 1) goto bad;
    for (int j = 0; j < m; j++) {
      int b;
      if (fscanf(f, "%d", &b) != 1) goto bad;
      acc = (acc << 1) + b;
    }
    if (dec != acc || dec != i) goto bad; /* modem.cc:113-118 */
    double re, im;
    if (fscanf(f, "%lf %lf", &re, &im) != 2) goto bad;
    md->pts[2 * i] = re;
    md->pts[2 * i + 1] = im;
    energies += pow(hypot(re, im), 2); /* modem.cc:122: pow(abs(s), 2) */
  }
  fclose(f);
  energies /= md->Kc;
  {
    double sc = sqrt(energies);
    for (int i = 0; i < md->Kc; i++) { /* complex /= real: component-wise */
      md->pts[2 * i] /= sc;
      md->pts[2 * i + 1] /= sc;
    }
  }
  return md;
bad:
  fclose(f);
  free(md->pts);
  free(md);
  return NULL;
}

void orc_modem_free(orc_modem *m) {
  if (!m) return;
  free(m->pts);
  free(m);
}

int orc_modem_bits(const orc_modem *m) { return m->m; }

void orc_modem_points(const orc_modem *m, double *cons) { memcpy(cons, m->pts, sizeof(double) * 2 * m->Kc); }

/* modem.cc:12-21, MSB-first label */
void orc_map(const orc_modem *md, const int32_t *cc, int S, double *x) {
  for (int i = 0; i < S; i++) {
    int idx = 0;
    for (int j = 0; j < md->m; j++) idx = (idx << 1) + cc[j + i * md->m];
    x[2 * i] = md->pts[2 * idx];
    x[2 * i + 1] = md->pts[2 * idx + 1];
  }
}

static inline double clipp(double v) { /* utility.cc:18-26 */
  if (v < kSmallestProb)
    return kSmallestProb;
  else if (v > 1.0 - kSmallestProb)
    return 1.0 - kSmallestProb;
  return v;
}

void orc_demap(const orc_modem *md, const double *y, int S, double hr, double hi, double var, double *p0) {
  const int Kc = md->Kc, m = md->m;
  double *sp = (double *)malloc(sizeof(double) * Kc);
  double *pr = (double *)malloc(sizeof(double) * Kc);
  const double bitlin = 0.5;
  for (int i = 0; i < S; i++) {
    const double yr = y[2 * i], yi = y[2 * i + 1];
    /* SoftAWGNDemodulation: modemlinearsystem.cc:51-79 */
    for (int k = 0; k < Kc; k++) {
      const double cr = md->pts[2 * k], ci = md->pts[2 * k + 1];
      double sr = cr * hr - ci * hi; /* symbol *= theta_h (naive complex mul) */
      double si = cr * hi + ci * hr;
      sr = sr - yr;
      si = si - yi;
      double d = (sr * sr + si * si) / var;
      pr[k] = -d;
    }
    double mx = pr[0];
    for (int k = 1; k < Kc; k++)
      if (mx < pr[k]) mx = pr[k];
    for (int k = 0; k < Kc; k++) pr[k] = exp(pr[k] - mx);
    double sum = 0.0;
    for (int k = 0; k < Kc; k++) sum += pr[k];
    for (int k = 0; k < Kc; k++) pr[k] = clipp(clipp(pr[k] / sum)); /* ProbClip twice (:246, modem.cc:27) */
    /* Modem::DeMapping: modem.cc:30-77 with bitLin = 0.5 */
    for (int k = 0; k < Kc; k++) sp[k] = 1.0;
    for (int j = 0; j < m; j++)
      for (int k = 0; k < Kc; k++) sp[k] *= (((k >> (m - 1 - j)) & 1) == 0) ? bitlin : 1.0 - bitlin;
    sum = 0.0;
    for (int k = 0; k < Kc; k++) {
      sp[k] *= pr[k];
      sum += sp[k];
    }
    for (int k = 0; k < Kc; k++) sp[k] /= sum;
    for (int j = 0; j < m; j++) {
      double q0 = 0.0, q1 = 0.0;
      for (int k = 0; k < Kc; k++) {
        if (((k >> (m - 1 - j)) & 1) == 0)
          q0 += sp[k];
        else
          q1 += sp[k];
      }
      q0 /= bitlin;
      q1 /= (1.0 - bitlin);
      p0[i * m + j] = clipp(q0 / (q0 + q1));
    }
  }
  free(sp);
  free(pr);
}

/* -------------------------------------------------------------- k-means */

void orc_cdiv(double a, double b, double c, double d, double *re, double *im) {
  double complex z = CMPLX(a, b) / CMPLX(c, d);
  *re = creal(z);
  *im = cimag(z);
}

double orc_hypot(double x, double y) { return hypot(x, y); }

/* KMeans::Run (src/kmeans.cc:15-84).  h_hat (optional) = clusters[0]/c[0]
 * (simulator.cc:145); clusters (optional, [Kc] interleaved) = KMeans::clusters();
 * idx (optional, [S]) = KMeans::idx(), the closing assignment (kmeans.cc:76-83). */
void orc_kmeans_state(const double *y, int S, const double *cons, int Kc, int iters, double *h_hat, double *clusters,
                      int *idx) {
  /* kmeans.cc:17-22: first max of |y| */
  int maxIndex = 0;
  double best = hypot(y[0], y[1]);
  for (int i = 1; i < S; i++) {
    double a = hypot(y[2 * i], y[2 * i + 1]);
    if (best < a) {
      best = a;
      maxIndex = i;
    }
  }
  double complex c0 = CMPLX(cons[0], cons[1]);
  double complex hatH = CMPLX(y[2 * maxIndex], y[2 * maxIndex + 1]) / c0;
  double complex *cl = (double complex *)malloc(sizeof(double complex) * Kc);
  double complex *tmp = (double complex *)malloc(sizeof(double complex) * Kc);
  int *cnt = (int *)calloc(Kc, sizeof(int));
  double complex *sum = (double complex *)calloc(Kc, sizeof(double complex));
  double *dist = (double *)malloc(sizeof(double) * Kc);
  for (int k = 0; k < Kc; k++) {
    cl[k] = CMPLX(cons[2 * k], cons[2 * k + 1]) * hatH;
    tmp[k] = CMPLX(0.0, 0.0);
  }
  for (int it = 0; it < iters; it++) {
    /* cnt/sum are NOT reset: clear() + operator[] keeps the old storage
     * (kmeans.cc:33-34), so the counts accumulate across iterations. */
    for (int j = 0; j < S; j++) {
      for (int k = 0; k < Kc; k++) dist[k] = hypot(creal(cl[k]) - y[2 * j], cimag(cl[k]) - y[2 * j + 1]);
      int mi = 0;
      for (int k = 1; k < Kc; k++)
        if (dist[k] < dist[mi]) mi = k;
      cnt[mi]++;
      sum[mi] = CMPLX(creal(sum[mi]) + y[2 * j], cimag(sum[mi]) + y[2 * j + 1]);
    }
    int same = 1;
    for (int k = 0; k < Kc; k++)
      if (!(creal(cl[k]) == creal(tmp[k]) && cimag(cl[k]) == cimag(tmp[k]))) {
        same = 0;
        break;
      }
    if (same) break;
    for (int k = 0; k < Kc; k++) tmp[k] = cl[k];
    for (int k = 0; k < Kc; k++) cl[k] = sum[k] / CMPLX((double)cnt[k], 0.0);
    /* absValues was cleared (kmeans.cc:65) -> max over an empty range -> index 0 */
    hatH = cl[0] / c0;
    for (int k = 0; k < Kc; k++) cl[k] = CMPLX(cons[2 * k], cons[2 * k + 1]) * hatH;
  }
  if (h_hat) {
    double complex hh = cl[0] / c0; /* simulator.cc:145 */
    h_hat[0] = creal(hh);
    h_hat[1] = cimag(hh);
  }
  if (clusters)
    for (int k = 0; k < Kc; k++) {
      clusters[2 * k] = creal(cl[k]);
      clusters[2 * k + 1] = cimag(cl[k]);
    }
  if (idx) /* kmeans.cc:76-83: min_element = the first minimum */
    for (int j = 0; j < S; j++) {
      for (int k = 0; k < Kc; k++) dist[k] = hypot(creal(cl[k]) - y[2 * j], cimag(cl[k]) - y[2 * j + 1]);
      int mi = 0;
      for (int k = 1; k < Kc; k++)
        if (dist[k] < dist[mi]) mi = k;
      idx[j] = mi;
    }
  free(cl);
  free(tmp);
  free(cnt);
  free(sum);
  free(dist);
}

void orc_kmeans_hhat(const double *y, int S, const double *cons, int Kc, int iters, double *h_hat) {
  orc_kmeans_state(y, S, cons, Kc, iters, h_hat, NULL, NULL);
}

void orc_rotations(const double *h_hat, double *h4) {
  double complex h = CMPLX(h_hat[0], h_hat[1]);
  for (int j = 0; j < 4; j++) {
    double complex r = cexp(CMPLX(0.0, (kPi / 2) * (double)j));
    double complex z = h * r;
    h4[2 * j] = creal(z);
    h4[2 * j + 1] = cimag(z);
  }
}

/* ------------------------------------------------------------------ RNG */

void orc_rng_seed(orc_rng *r, long state) { r->state = state; }

/* randnum.cc:36-45 (A=48271, M=2^31-1, Schrage) */
double orc_uniform(orc_rng *r) {
  const int A = 48271;
  const long Mm = 2147483647;
  const int Q = (int)(Mm / A), R = (int)(Mm % A);
  int tmp = (int)(A * (r->state % Q) - R * (r->state / Q));
  if (tmp >= 0)
    r->state = tmp;
  else
    r->state = tmp + Mm;
  return r->state / (double)Mm;
}

/* randnum.cc:48-72 polar method, one pair */
void orc_normal_pair(orc_rng *r, double *a, double *b) {
  double x1 = 0, x2 = 0, w = 2.0;
  while (w > 1.0) {
    x1 = 2.0 * orc_uniform(r) - 1.0;
    x2 = 2.0 * orc_uniform(r) - 1.0;
    w = x1 * x1 + x2 * x2;
  }
  w = sqrt(-2.0 * log(w) / w);
  *a = x1 * w;
  *b = x2 * w;
}

/* ------------------------------------------------------ per-codeword loop */

void orc_gen_frame(const orc_code *c, const orc_modem *m, orc_rng *r, double snr, int32_t *uu, int32_t *cc,
                   double *true_h, double *y) {
  const int K = c->K, S = c->cc_len / m->m;
  for (int t = 0; t < K; t++) uu[t] = (orc_uniform(r) < 0.5 ? 0 : 1); /* sourcesink.cc:5-10 */
  orc_encode(c, uu, cc);
  double hr, hi;
  orc_normal_pair(r, &hr, &hi); /* simulator.cc:121-123 */
  const double s5 = sqrt(0.5);
  hr = hr * s5;
  hi = hi * s5;
  true_h[0] = hr;
  true_h[1] = hi;
  const double var = pow(10.0, -0.1 * (snr)); /* simulator.cc:74-75 */
  const double sigma = sqrt(var);
  const double ns = sigma / kSqrt2;
  double *x = (double *)malloc(sizeof(double) * 2 * S);
  orc_map(m, cc, S, x);
  for (int j = 0; j < S; j++) { /* modemlinearsystem.cc:38-48 */
    double nr, ni;
    orc_normal_pair(r, &nr, &ni);
    double tr = x[2 * j] * hr - x[2 * j + 1] * hi;
    double ti = x[2 * j] * hi + x[2 * j + 1] * hr;
    double sr = nr * ns - ni * 0.0;
    double si = nr * 0.0 + ni * ns;
    y[2 * j] = tr + sr;
    y[2 * j + 1] = ti + si;
  }
  free(x);
}

void orc_receive(const orc_code *c, const orc_modem *m, const double *y, const double *true_h, double snr, int blind,
                 int metric_soft, int metric_iter, uint8_t *uu_hat, double *p0_out, double *metrics_out,
                 int32_t *chosen_out, double *h_hat_out, int32_t *ret_out, double *syn) {
  const int S = c->cc_len / m->m;
  const double var = pow(10.0, -0.1 * (snr));
  double *p0 = (double *)malloc(sizeof(double) * c->cc_len);
  uint8_t *rr = (uint8_t *)malloc(c->N);
  uint8_t *cch = (uint8_t *)malloc(c->N);
  double h[2] = {true_h ? true_h[0] : 0.0, true_h ? true_h[1] : 0.0};
  int chosen = 0;
  double metrics[4] = {0, 0, 0, 0};
  double hh[2] = {0, 0};
  if (blind) {
    orc_kmeans_hhat(y, S, m->pts, m->Kc, 20, hh); /* simulator.cc:140-145 */
    double h4[8];
    orc_rotations(hh, h4);
    for (int j = 0; j < 4; j++) { /* kmcodec.cc:122-142 */
      orc_demap(m, y, S, h4[2 * j], h4[2 * j + 1], var, p0);
      double mt;
      if (metric_soft) { /* kmcodec.cc:147-156 */
        orc_bp_decode(c, p0, metric_iter, uu_hat, cch, syn);
        mt = 0.0;
        for (int r = 0; r < c->M; r++) mt += log(syn[r]);
      } else if (c->is5g) { /* kmcodec.cc:157-160, 105-107 */
        orc_bp_decode(c, p0, metric_iter, uu_hat, cch, syn);
        mt = orc_parity_count(c, cch);
      } else { /* kmcodec.cc:109-117: rr = P0 > 0.5 */
        for (int i = 0; i < c->cc_len; i++) rr[i] = p0[i] > 0.5 ? 1 : 0;
        mt = orc_parity_count(c, rr);
      }
      metrics[j] = fabs(mt);
    }
    chosen = 0;
    for (int j = 1; j < 4; j++)
      if (metrics[j] < metrics[chosen]) chosen = j;
    h[0] = h4[2 * chosen];
    h[1] = h4[2 * chosen + 1];
  }
  orc_demap(m, y, S, h[0], h[1], var, p0);
  int ret = orc_bp_decode(c, p0, c->max_iter, uu_hat, NULL, syn);
  if (p0_out) memcpy(p0_out, p0, sizeof(double) * c->cc_len);
  if (metrics_out) memcpy(metrics_out, metrics, sizeof(metrics));
  if (chosen_out) *chosen_out = chosen;
  if (h_hat_out) {
    h_hat_out[0] = hh[0];
    h_hat_out[1] = hh[1];
  }
  if (ret_out) *ret_out = ret;
  free(p0);
  free(rr);
  free(cch);
}
