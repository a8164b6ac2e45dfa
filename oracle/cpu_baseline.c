/* cpu_baseline.c — the reported CPU baseline for bench.py (TEST/BENCH
 * INFRASTRUCTURE ONLY; never part of the product path).
 *
 * Times the oracle's restatement of the reference receive path
 * (KmCodec::Decoder = [k-means + 4-candidate metric] + demap + sum-product BP,
 * src/kmcodec.cc:54-72, plus SourceSink::CntErr, lib/lab/src/sourcesink.cc:29-47)
 * on T host threads, one std-thread-equivalent pthread per core, each with its
 * own frames from its own Park-Miller stream (seed 17 + thread id).  Frame
 * generation (source, encoder, channel) happens before the timed region, as in
 * the GPU measurement where the frames are resident in HBM; it is timed
 * separately, so the full loop (source + encoder + channel + receive) rate is
 * reported beside the decode-only rate.
 *
 * usage: cpu_baseline H.txt modem.txt is5g snr max_iter blind n_per_thread threads
 * prints one JSON object.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "oracle.h"

typedef struct {
  const orc_code *c;
  const orc_modem *m;
  double snr;
  int blind, n, tid;
  int32_t *uu;
  double *y, *h;
  long err_bits, err_blk;
  double sum_e2;
  double syn_dummy;
} job;

static double now(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

static void *gen(void *p) {
  job *j = (job *)p;
  int32_t d[8];
  orc_code_dims(j->c, d);
  const int K = d[2], cc_len = d[3], S = cc_len / orc_modem_bits(j->m);
  int32_t *cc = (int32_t *)malloc(sizeof(int32_t) * cc_len);
  orc_rng r;
  orc_rng_seed(&r, 17 + j->tid);
  for (int i = 0; i < j->n; i++)
    orc_gen_frame(j->c, j->m, &r, j->snr, j->uu + (size_t)i * K, cc, j->h + 2 * i, j->y + (size_t)i * 2 * S);
  free(cc);
  return NULL;
}

static void *dec(void *p) {
  job *j = (job *)p;
  int32_t d[8];
  orc_code_dims(j->c, d);
  const int M = d[0], K = d[2], cc_len = d[3], S = cc_len / orc_modem_bits(j->m);
  uint8_t *uh = (uint8_t *)malloc(K);
  double *syn = (double *)calloc(M, sizeof(double));
  j->err_bits = 0;
  j->err_blk = 0;
  j->sum_e2 = 0;
  for (int i = 0; i < j->n; i++) {
    orc_receive(j->c, j->m, j->y + (size_t)i * 2 * S, j->h + 2 * i, j->snr, j->blind, 0, 5, uh, NULL, NULL, NULL,
                NULL, NULL, syn);
    int e = 0;
    const int32_t *u = j->uu + (size_t)i * K;
    for (int t = 0; t < K; t++) e += (u[t] != uh[t]);
    j->err_bits += e;
    j->err_blk += (e > 0);
    j->sum_e2 += (double)e * e;
  }
  free(uh);
  free(syn);
  return NULL;
}

int main(int argc, char **argv) {
  if (argc < 9) {
    fprintf(stderr, "usage: %s H modem is5g snr max_iter blind n_per_thread threads\n", argv[0]);
    return 2;
  }
  const int is5g = atoi(argv[3]);
  const double snr = atof(argv[4]);
  const int max_iter = atoi(argv[5]);
  const int blind = atoi(argv[6]);
  const int n = atoi(argv[7]);
  const int T = atoi(argv[8]);
  orc_code *c = orc_code_load(argv[1], is5g, 1, 0, max_iter);
  orc_modem *m = orc_modem_load(argv[2]);
  if (!c || !m) {
    fprintf(stderr, "load failed\n");
    return 1;
  }
  int32_t d[8];
  orc_code_dims(c, d);
  const int K = d[2], S = d[3] / orc_modem_bits(m);
  job *jobs = (job *)calloc(T, sizeof(job));
  pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * T);
  for (int t = 0; t < T; t++) {
    jobs[t].c = c;
    jobs[t].m = m;
    jobs[t].snr = snr;
    jobs[t].blind = blind;
    jobs[t].n = n;
    jobs[t].tid = t;
    jobs[t].uu = (int32_t *)malloc(sizeof(int32_t) * (size_t)n * K);
    jobs[t].y = (double *)malloc(sizeof(double) * (size_t)n * 2 * S);
    jobs[t].h = (double *)malloc(sizeof(double) * 2 * n);
  }
  double tg = now();
  for (int t = 0; t < T; t++) pthread_create(&th[t], NULL, gen, &jobs[t]);
  for (int t = 0; t < T; t++) pthread_join(th[t], NULL);
  double t0 = now();
  const double gen_s = t0 - tg;
  for (int t = 0; t < T; t++) pthread_create(&th[t], NULL, dec, &jobs[t]);
  for (int t = 0; t < T; t++) pthread_join(th[t], NULL);
  double el = now() - t0;
  long eb = 0, ek = 0;
  double e2 = 0;
  for (int t = 0; t < T; t++) {
    eb += jobs[t].err_bits;
    ek += jobs[t].err_blk;
    e2 += jobs[t].sum_e2;
  }
  long tot = (long)n * T;
  printf("{\"codewords\": %ld, \"threads\": %d, \"seconds\": %.6f, \"cw_per_s\": %.3f, \"gen_seconds\": %.6f, "
         "\"full_loop_cw_per_s\": %.3f, \"err_blk\": %ld, \"err_bit\": %ld, \"sum_e2\": %.1f, \"K\": %d, "
         "\"fer\": %.6f, \"ber\": %.8f}\n",
         tot, T, el, tot / el, gen_s, tot / (el + gen_s), ek, eb, e2, K, (double)ek / tot, (double)eb / ((double)tot * K));
  return 0;
}
