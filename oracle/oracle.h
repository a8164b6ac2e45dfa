/* oracle.h — CPU restatement of the kmldpc hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this; the product (libkmldpc_amd.so) never does.
 *
 * Parity status: PINNED.  Every function below is checked against golden
 * vectors generated from the reference itself (oracle/_ref/ref_harness, built
 * from /root/reference sources; fixtures in tests/golden/ (npz),
 * tests/golden/counters.json) by tests/test_oracle.py.
 *
 * Each function cites the reference file:line it restates (paths relative to
 * /root/reference/kmldpc).
 */
#ifndef KMLDPC_ORACLE_H
#define KMLDPC_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_code orc_code;
typedef struct orc_modem orc_modem;

/* --- LDPC code: lib/lab/src/binaryldpccodec.cc:62-129 (+SystemMatrixH :346-492),
 *     lib/lab/src/binary5gldpccodec.cc:11-78 (+SystemMatrixH :240-391).
 * reversed_rows=1 reproduces the row-list order of a copy-constructed codec
 * (binaryldpccodec.cc:31-46). */
orc_code *orc_code_load(const char *path, int is5g, int active, int reversed_rows, int max_iter);
void orc_code_free(orc_code *c);
/* dims[0]=M rows, [1]=Ncol internal columns, [2]=K info bits (code_dim),
 * [3]=cc_len transmitted bits, [4]=Z lifting (0 for PEG), [5]=E edges,
 * [6]=code_chk (rank), [7]=max_iter */
void orc_code_dims(const orc_code *c, int32_t *dims);
/* column permutation tempP (new column j = original column perm[j]) */
void orc_code_perm(const orc_code *c, int32_t *perm);
/* graph in reference traversal order: row_ptr[M+1], row_col[E] (column of each
 * slot, row-list order from row_head.right); col_ptr[Ncol+1], col_slot[E]
 * (slot ids in column-list order from col_head.down). */
void orc_code_graph(const orc_code *c, int32_t *row_ptr, int32_t *row_col, int32_t *col_ptr, int32_t *col_slot);

/* Encoder: binaryldpccodec.cc:144-162 / binary5gldpccodec.cc:86-109.
 * uu[K] -> cc[cc_len]; values 0/1. */
void orc_encode(const orc_code *c, int32_t *uu, int32_t *cc);

/* Sum-product BP: binaryldpccodec.cc:165-278 / binary5gldpccodec.cc:112-232.
 * p0[cc_len] = P(bit=0).  Writes uu_hat[K], cc_hat[Ncol] (may be NULL) and
 * syn[M] (syndrom_soft; only overwritten when a CN phase runs, like the
 * reference's member array).  Returns iter + (iter < max_iter). */
int orc_bp_decode(const orc_code *c, const double *p0, int iter_count, uint8_t *uu_hat, uint8_t *cc_hat, double *syn);
/* ParityCheck: binaryldpccodec.cc:281-300 — number of unsatisfied rows. */
int orc_parity_count(const orc_code *c, const uint8_t *bits);

/* --- Modem: lib/lab/src/modem.cc:87-129 (init), :12-21 (Mapping),
 *     :23-79 (DeMapping); modemlinearsystem.cc:51-79 (SoftAWGNDemodulation). */
orc_modem *orc_modem_load(const char *path);
void orc_modem_free(orc_modem *m);
int orc_modem_bits(const orc_modem *m);
/* normalised constellation, cons[2*Kc] */
void orc_modem_points(const orc_modem *m, double *cons);
void orc_map(const orc_modem *m, const int32_t *cc, int S, double *x);
/* y[2*S], h=(hr,hi), var -> p0[S*bits] */
void orc_demap(const orc_modem *m, const double *y, int S, double hr, double hi, double var, double *p0);

/* --- k-means: src/kmeans.cc:15-84 (with its cumulative-count semantics),
 * followed by h_hat = clusters[0]/c[0] (src/simulator.cc:145). */
void orc_kmeans_hhat(const double *y, int S, const double *cons, int Kc, int iters, double *h_hat);
void orc_kmeans_state(const double *y, int S, const double *cons, int Kc, int iters, double *h_hat, double *clusters,
                      int *idx);
/* candidates h_hat*exp(i*kPi/2*j), j=0..3 (src/simulator.cc:146-148) */
void orc_rotations(const double *h_hat, double *h4);

/* --- RNG: lib/lab/src/randnum.cc:9-79 (Park-Miller / Schrage, polar normal). */
typedef struct {
  long state;
} orc_rng;
void orc_rng_seed(orc_rng *r, long state); /* SetSeed(-1) == state 17 */
double orc_uniform(orc_rng *r);
void orc_normal_pair(orc_rng *r, double *a, double *b);

/* --- One codeword of Simulator::run_blocks (src/simulator.cc:116-167):
 * frame generation (GetBitStr, Encoder, true_h, PartitionModemLSystem). */
void orc_gen_frame(const orc_code *c, const orc_modem *m, orc_rng *r, double snr, int32_t *uu, int32_t *cc, double *true_h,
                   double *y);
/* KmCodec::Decoder (src/kmcodec.cc:54-72) for one codeword.  blind=0 uses
 * true_h; blind=1 runs k-means + the 4-candidate metric.  metric_iter is the
 * 5G/soft metric BP iteration count.  Writes uu_hat[K]; optional outputs:
 * p0 (chosen, cc_len), metrics[4], chosen, h_hat[2], ret (BP return), syn
 * (persistent syndrom_soft state, M doubles, required). */
void orc_receive(const orc_code *c, const orc_modem *m, const double *y, const double *true_h, double snr, int blind,
                 int metric_soft, int metric_iter, uint8_t *uu_hat, double *p0, double *metrics, int32_t *chosen,
                 double *h_hat, int32_t *ret, double *syn);

/* glibc-compatible complex division (__divdc3) and hypot, exported so the
 * tests can pin the device restatements against them. */
void orc_cdiv(double a, double b, double c, double d, double *re, double *im);
double orc_hypot(double x, double y);

#ifdef __cplusplus
}
#endif
#endif
