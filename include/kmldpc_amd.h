/* kmldpc_amd.h — C ABI of the MI355X-native kmldpc hot path.
 *
 * Drop-in boundary for the per-codeword receive loop of trganda/kmldpc
 * (paths relative to /root/reference/kmldpc).  The reference has no FFI; its
 * boundary is a set of C++ classes.  Each entry point below replaces one of
 * them, batched over B codewords:
 *
 *   kml_create                lab::BinaryLDPCCodec(const toml::value&)            lib/lab/include/binaryldpccodec.h:16
 *                             lab::Binary5GLDPCCodec(const toml::value&)           lib/lab/include/binary5gldpccodec.h:12
 *                             lab::Modem(const toml::value&)                       lib/lab/include/modem.h:13
 *                             KmCodec(toml::value)                                 include/kmcodec.h:16
 *   kml_bp_decode             virtual int BinaryLDPCCodec::Decoder(const double *M2V, int *uu_hat, int iter_count)
 *                                                                                  lib/lab/include/binaryldpccodec.h:20
 *                                                                                  (override binary5gldpccodec.h:17)
 *   kml_demap                 void ModemLinearSystem::DeMapping(thetaList, double *bitLin, double *bitLout)
 *                                                                                  lib/lab/include/modemlinearsystem.h:20-22
 *   kml_kmeans                kmldpc::KMeans(data, constellations, iter); Run(); clusters()
 *                                                                                  include/kmeans.h:14-22
 *                             + h_hat = clusters[0]/c[0] and its 4 rotations       src/simulator.cc:145-148
 *   kml_kmeans_state          KMeans::clusters(), KMeans::idx() after Run()          include/kmeans.h:18-19
 *                                                                                  (src/kmeans.cc:72-83, 86-94)
 *   kml_kmeans_dump_mat       void KMeans::DumpToMat(std::string&, std::vector<complex>& append)
 *                                                                                  include/kmeans.h:21, src/kmeans.cc:99-109
 *                             (host only; the reference needs matio, this writes the level-5 file itself)
 *   kml_decode_frames         void KmCodec::Decoder(ModemLinearSystem&, const std::vector<complex>& h_hats, int *uu_hat)
 *                                                                                  include/kmcodec.h:23-25
 *   kml_decode_candidates     the same KmCodec::Decoder with the caller's h_hats (any 1..4 estimates)
 *                                                                                  include/kmcodec.h:23-25
 *   kml_count_errors          void SourceSink::CntErr(const int*, const int*, int, int)  lib/lab/include/sourcesink.h:15
 *   kml_sim_*                 the throughput driver: frame generation + receive + counting for one
 *                             SNR point of Simulator::run_blocks (src/simulator.cc:112-168)
 *
 * Conventions
 *   - Every call returns 0 on success or a negative KML_E* code and never exits
 *     the process (the reference logs and exit(-1)s).  kml_last_error() holds
 *     the message of the last failure on that context (with a NULL context: the
 *     last failure of a context-free call, kml_comm_unique_id, on this thread).
 *   - Bits (uu, uu_hat, cc_hat) are one byte per bit (0/1) unless a name says
 *     "_bits" (packed little-endian uint64 words).  Complex numbers are
 *     interleaved (re, im) doubles.
 *   - Pointers are host pointers unless KML_DEVICE_PTRS is set in `flags`, in
 *     which case they must be device pointers on the context's GPU; results are
 *     complete when the call returns (the context's HIP stream is synchronised).
 *   - A context is bound to one GPU and one HIP stream and is not thread-safe;
 *     use one context per GPU / per thread.
 */
#ifndef KMLDPC_AMD_H
#define KMLDPC_AMD_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KML_ABI_VERSION 2  /* 2: KML_DIM_PART_G (KML_DIM_COUNT 13) */

enum {
  KML_OK = 0,
  KML_E_ARG = -1,    /* bad argument */
  KML_E_IO = -2,     /* cannot open / parse a config, H-matrix or constellation file */
  KML_E_HIP = -3,    /* HIP runtime failure */
  KML_E_UNSUP = -4,  /* configuration not supported */
  KML_E_NOMEM = -5
};

enum {
  KML_DEVICE_PTRS = 1,
  /* kml_decode_frames: KmCodec::GetHistogramData instead of Decoder — the
   * candidate metrics only, no final decode; uu_hat is what the last metric
   * decode left (BP-based metrics) or zeros (hard PEG metric). */
  KML_HISTOGRAM = 2
};

typedef struct kml_ctx kml_ctx;

/* dims[]: index names for kml_dims */
enum {
  KML_DIM_M = 0,        /* check rows */
  KML_DIM_NCOL = 1,     /* internal columns (incl. punctured) */
  KML_DIM_K = 2,        /* info bits (code_dim) */
  KML_DIM_CCLEN = 3,    /* transmitted bits */
  KML_DIM_Z = 4,        /* 5G lifting factor */
  KML_DIM_E = 5,        /* edges */
  KML_DIM_CHK = 6,      /* GF(2) rank (code_chk) */
  KML_DIM_MAXITER = 7,  /* [ldpc] max_iter */
  KML_DIM_BITS = 8,     /* bits per symbol */
  KML_DIM_KC = 9,       /* constellation points */
  KML_DIM_S = 10,       /* symbols per codeword */
  KML_DIM_BP_LDS = 11,  /* 1 if the decoder keeps messages in LDS */
  KML_DIM_PART_G = 12,  /* workgroups per codeword of the partitioned decoder (4), 0 when not used */
  KML_DIM_COUNT = 13
};

/* Create a context from a reference config.toml.  Relative matrix_file /
 * modem_file paths are resolved against data_dir (NULL or "" = the CWD, as
 * the reference does).  device = HIP device ordinal; device < 0 creates a
 * host-only context (planner, encoder, constellation; no GPU calls). */
int kml_create(const char *config_toml, const char *data_dir, int device, kml_ctx **out);
/* Same without a config file: the [ldpc]/[modem]/[xcodec] keys given directly. */
int kml_create_explicit(const char *matrix_file, const char *modem_file, int is5g, int active, int max_iter,
                        int metric_soft, int metric_iter, int device, kml_ctx **out);
void kml_destroy(kml_ctx *ctx);
const char *kml_last_error(const kml_ctx *ctx);
int kml_abi_version(void);
/* Name of the BP kernel family the context last launched ("bp_regular_kernel",
 * "bp_irregular_kernel", "bp_part_kernel" (the partitioned cooperative kernel,
 * PEG8064), "bp_kernel"; "" before any decode). */
const char *kml_bp_kernel(const kml_ctx *ctx);

int kml_dims(const kml_ctx *ctx, int32_t *dims /* [KML_DIM_COUNT] */);
/* Host-side code plan, for inspection and parity tests. */
int kml_code_perm(const kml_ctx *ctx, int32_t *perm /* [Ncol] */);
int kml_code_graph(const kml_ctx *ctx, int32_t *row_ptr /* [M+1] */, int32_t *row_col /* [E] */,
                   int32_t *col_ptr /* [Ncol+1] */, int32_t *col_slot /* [E] */);
int kml_constellation(const kml_ctx *ctx, double *points /* [2*Kc] */);
/* Host encoder (BinaryLDPCCodec::Encoder), uu[K] -> cc[cc_len], bytes. */
int kml_encode(const kml_ctx *ctx, const uint8_t *uu, uint8_t *cc, int B);

/* BinaryLDPCCodec::Decoder, batched.  p0[B][cc_len] = P(bit = 0) (the
 * reference's M2V).  Outputs (any may be NULL): uu_hat[B][K], ret[B] (the
 * reference return value iter + (iter < max_iter)), cc_hat[B][Ncol],
 * syn[B][M] (syndrom_soft; rows are only written when a CN phase runs, like
 * the reference's member array).  iter_count = 0 runs no iteration and, like
 * the reference (uu_hat is written inside its loop), leaves uu_hat and cc_hat
 * as the caller passed them. */
int kml_bp_decode(kml_ctx *ctx, const double *p0, int B, int iter_count, uint8_t *uu_hat, int32_t *ret,
                  uint8_t *cc_hat, double *syn, int flags);

/* ModemLinearSystem::DeMapping with bitLin = 0.5 and one channel estimate per
 * codeword: y[B][S][2], h[B][2], var = 10^(-snr/10) -> p0[B][cc_len]. */
int kml_demap(kml_ctx *ctx, const double *y, const double *h, double var, int B, double *p0, int flags);

/* KMeans(y, constellation, iters).Run(); h_hat = clusters[0]/c[0];
 * h4[j] = h_hat * exp(i*kPi/2*j).  h_hat[B][2], h4[B][4][2] (either may be NULL). */
int kml_kmeans(kml_ctx *ctx, const double *y, int B, int iters, double *h_hat, double *h4, int flags);

/* The same Run, then KMeans::clusters() = c[k] * hatH -> clusters[B][Kc][2] and
 * KMeans::idx() (the closing assignment, first minimum of glibc hypot,
 * kmeans.cc:76-83) -> idx[B][S].  Either output may be NULL. */
int kml_kmeans_state(kml_ctx *ctx, const double *y, int B, int iters, double *clusters, int32_t *idx, int flags);

/* KMeans::DumpToMat(filename, append) of ONE codeword (host only, no context):
 * a MAT-file level 5 with the reference's variables, each an n x 1 column,
 * uncompressed as lab::Mat writes them (lib/lab/src/mat.cc): data[S] complex,
 * cluster[Kc] complex, idx[S] int32, constellations[Kc] complex, hHats =
 * append[0..3] complex, realH = append[4] (1 x 1 complex).  Complex inputs
 * are interleaved (re, im); append holds 5 complex values.  Returns 0,
 * KML_E_ARG or KML_E_IO. */
int kml_kmeans_dump_mat(const char *path, const double *data, int S, const double *clusters, const int32_t *idx,
                        const double *constellations, int Kc, const double *append);

/* KmCodec::Decoder for B codewords at Es/N0 = snr dB.  true_h[B][2] selects
 * the known-channel path ([decoder] true_h_arg = true); true_h == NULL runs the
 * blind path (k-means, 4 candidates, syndrome metric).  Optional outputs:
 * chosen[B], metrics[B][4], ret[B], h_hat[B][2]. */
int kml_decode_frames(kml_ctx *ctx, const double *y, const double *true_h, double snr, int B, uint8_t *uu_hat,
                      int32_t *chosen, double *metrics, int32_t *ret, double *h_hat, int flags);

/* KmCodec::Decoder(mls, h_hats, uu_hat) (include/kmcodec.h:23-25,
 * src/kmcodec.cc:54-72) with the caller's channel estimates h_hats[B][nc][2],
 * 1 <= nc <= 4: nc == 1 demaps with h_hats[b][0] and decodes (no metric);
 * nc > 1 computes every candidate's syndrome metric (hard PEG count, 5G
 * metric_iter BP count, or the soft metric, as configured), takes the first
 * minimum, demaps with it and decodes.  chosen[B], metrics[B][4] (entries
 * >= nc are 0), ret[B] may be NULL.  KML_HISTOGRAM: metrics only
 * (KmCodec::GetHistogramData, kmcodec.cc:75-79), for nc == 1 too: the single
 * candidate's metric, no final decode, ret zeroed. */
int kml_decode_candidates(kml_ctx *ctx, const double *y, const double *h_hats, int nc, double snr, int B,
                          uint8_t *uu_hat, int32_t *chosen, double *metrics, int32_t *ret, int flags);

/* SourceSink::CntErr over B codewords; counters[4] += {err_bit, err_blk, tot_bit, tot_blk}. */
int kml_count_errors(kml_ctx *ctx, const uint8_t *uu, const uint8_t *uu_hat, int B, uint64_t *counters, int flags);

/* --- throughput driver (GPU-resident frames) ----------------------------- */
/* Generate B frames for codeword indices [first_cw, first_cw + B) at Es/N0 =
 * snr into the context's resident buffers (Philox stream keyed by seed). */
int kml_sim_generate(kml_ctx *ctx, double snr, uint64_t seed, uint64_t first_cw, int B);
/* Receive the resident batch (blind or known-H) and accumulate the counters.
 * counters[8] (may be NULL) receives {err_bit, err_blk, tot_bit, tot_blk,
 * vn_phases, cn_phases, converged, redone} of this call (redone: codewords a
 * FAST kernel deferred mid-decode to the exact kernel.  Unproven FAST
 * quotients are settled in place (exact_div.hpp dd_fix), so this is 0 unless
 * KML_FORCE_REDO=1 forces the path; see DESIGN.md "Bit-exactness strategy").  If sync == 0 the call
 * returns after enqueueing the work (counters must then be NULL); use
 * kml_sync to wait. */
int kml_sim_decode(kml_ctx *ctx, double snr, int blind, uint64_t *counters, int sync);
int kml_sync(kml_ctx *ctx);
/* Synchronous form with the per-codeword view the simulator's stop rule needs:
 * cw_err[B] (may be NULL) = error bits of each resident codeword, metrics[B][4]
 * (may be NULL) = the candidate metrics.  histogram != 0 runs
 * KmCodec::GetHistogramData instead of Decoder (simulator.cc:154-162): metrics
 * only, no final decode, and the error count then sees the uu_hat the last
 * metric decode left (5G metric) or all-zero decisions (hard PEG metric, whose
 * reference buffer is uninitialised).  counters[8] as kml_sim_decode. */
int kml_sim_decode_ex(kml_ctx *ctx, double snr, int blind, int histogram, int32_t *cw_err, double *metrics,
                      uint64_t *counters);

/* --- simulator driver (Simulator::Simulate / run / run_blocks) ------------ */
/* The parsed config.toml: f[3] = {minimum_snr, maximum_snr, step_snr};
 * n[10] = {maximum_error_number, maximum_block_number, thread_block_number,
 * true_h_arg, 5gldpc, metric_type, metric_iter, histogram.enable, max_iter,
 * active}. */
int kml_run_config(const kml_ctx *ctx, double *f, int64_t *n);

/* In-place sum of n counters over all ranks (RCCL / gloo / MPI in the caller). */
typedef int (*kml_allreduce_fn)(uint64_t *vals, int n, void *user);
/* Decode `count` frames with global codeword indices [first_cw, first_cw+count):
 * cw_err[count] error bits per codeword, metrics[count][4] (histogram mode). */
typedef int (*kml_batch_fn)(uint64_t first_cw, int count, int32_t *cw_err, double *metrics, void *user);
/* Progress: counters {err_bit, err_blk, tot_bit, tot_blk} (SourceSink::PrintResult). */
typedef void (*kml_report_fn)(const uint64_t *counters, void *user);

typedef struct {
  double snr;
  int rank, world;       /* this process's shard of the codeword index space */
  int batch;             /* codewords per rank per round */
  uint64_t max_blocks;   /* maximum_block_number */
  uint64_t max_err;      /* maximum_error_number */
  int K;                 /* info bits per codeword (tot_bit += K) */
  int ncand;             /* histogram: metrics per codeword (1 known-H, 4 blind) */
  const char *hist_path; /* histogram output file of this rank, NULL = none */
  int report_every;      /* PrintResult period in codewords (reference: 100) */
} kml_point_cfg;

/* One SNR point of Simulator::run with the stop rule of run_blocks
 * (simulator.cc:117): codewords are taken in global index order until
 * maximum_block_number are counted or maximum_error_number block errors
 * reached, exactly as a single sequential stream would, whatever world and
 * batch are.  Rank r decodes indices [t*world*batch + r*batch, ...) of round t;
 * per round the ranks exchange world + 4 counters through `reduce` (no
 * per-codeword data moves between ranks).  counters[4] = the point's totals
 * {err_bit, err_blk, tot_bit, tot_blk}. */
int kml_sweep_point(const kml_point_cfg *cfg, kml_batch_fn decode, void *decode_user, kml_allreduce_fn reduce,
                    void *reduce_user, kml_report_fn report, void *report_user, uint64_t *counters);
/* kml_sweep_point with the context's GPU frame generator (Philox keyed by
 * seed and global codeword index) and receive path ([decoder] true_h_arg,
 * [histogram] enable from the config). */
int kml_sim_point(kml_ctx *ctx, const kml_point_cfg *cfg, uint64_t seed, kml_allreduce_fn reduce, void *reduce_user,
                  kml_report_fn report, void *report_user, uint64_t *counters);
/* Load B host frames (uu[B][K] source-bit bytes, y[B][S][2], true h[B][2])
 * into the resident batch in place of kml_sim_generate, e.g. the reference's
 * own seed-17 stream from kml_ref_frames, so kml_sim_decode's counters can be
 * compared with SourceSink::CntErr's (sourcesink.cc:29-47) on identical frames. */
int kml_sim_load(kml_ctx *ctx, double snr, const uint8_t *uu, const double *y, const double *h, int B,
                 uint64_t first_cw);
/* Copy the resident frames out (for checks): uu[B][K] bytes, y[B][S][2], h[B][2]. */
int kml_sim_frames(kml_ctx *ctx, uint8_t *uu, double *y, double *h);

/* --- multi-GPU counter reduction: RCCL over xGMI ------------------------- */
/* The reference sums its worker threads' counters under a mutex
 * (lib/lab/src/threadsafe_sourcesink.cc); across GPUs that is one RCCL
 * all-reduce, issued by this library on the context's stream.  Rank 0 calls
 * kml_comm_unique_id, the caller distributes the 128 bytes (any CPU channel,
 * e.g. torch.distributed gloo), and every rank calls kml_comm_init (a
 * collective).  librccl.so.1 is loaded on first use. */
#define KML_COMM_ID_BYTES 128
int kml_comm_unique_id(uint8_t *id /* [KML_COMM_ID_BYTES] */);
int kml_comm_init(kml_ctx *ctx, const uint8_t *id, int world, int rank);
/* Ranks of the context's communicator (0 = none). */
int kml_comm_size(const kml_ctx *ctx);
/* In-place sum over the ranks of n host values (staged through the GPU;
 * synchronous). */
int kml_comm_allreduce_u64(kml_ctx *ctx, uint64_t *vals, int n);
int kml_comm_allreduce_f64(kml_ctx *ctx, double *vals, int n);

/* --- the reference's host random sources (parity runs) ------------------ */
/* lab::CLCRandNum (randnum.cc:4-92): Park-Miller minimal standard with
 * Schrage's method; *state = 17 is SetSeed(-1).  Normal(): polar method. */
double kml_lcg_uniform(int64_t *state);
void kml_lcg_normal(int64_t *state, double *nn, int len);
/* lab::CWHRandNum (randnum.cc:95-166): Wichmann-Hill; xyz = {13, 37, 91} is SetSeed(-1). */
double kml_wh_uniform(int32_t *xyz);
void kml_wh_normal(int32_t *xyz, double *nn, int len);
/* lab::SourceSink::GetBitStr / GetSymStr (sourcesink.cc:5-19) on a CLCRandNum state. */
void kml_get_bit_str(int64_t *state, uint8_t *uu, int len);
void kml_get_sym_str(int64_t *state, int32_t *uu, int qary, int len);
/* n frames of Simulator::run_blocks' sequential stream (simulator.cc:118-130)
 * from a CLCRandNum state (advanced in place): uu[n][K] bytes, true_h[n][2],
 * y[n][S][2].  Host-side; also works on a host-only context. */
int kml_ref_frames(const kml_ctx *ctx, int64_t *state, double snr, int n, uint8_t *uu, double *true_h, double *y);

/* --- profiling ----------------------------------------------------------- */
/* When enabled, every kernel launch of the context is bracketed by HIP events
 * on the context's stream.  kml_prof_read returns, for the named stage
 * ("bp", "demap", "kmeans", "metric", "framegen"), the number of launches,
 * their summed device time in ms and the summed algorithmic bytes
 * (SURVEY §8d accounting for "bp"). */
int kml_prof_enable(kml_ctx *ctx, int on);
int kml_prof_reset(kml_ctx *ctx);
int kml_prof_read(kml_ctx *ctx, const char *stage, int64_t *launches, double *total_ms, double *alg_bytes);
/* Summed algorithmic fp64 flops of the stage's launches ("bp" only). */
int kml_prof_read_flops(kml_ctx *ctx, const char *stage, double *alg_flops);

/* Device-side probe of the exact-math helpers: in[n][4] = (a, b, c, d) ->
 * out[n][4] = (hypot(a,b), re((a+ib)/(c+id)), im(...), exp(a)) with the
 * glibc-exact restatements the kernels use. */
int kml_math_probe(kml_ctx *ctx, const double *in, int n, double *out);
/* Device-side probe of the soft metric's log (kml_log, glibc-exact): out[i] = log(in[i]). */
int kml_log_probe(kml_ctx *ctx, const double *in, int n, double *out);
/* Device-side probe of the decoder's divisions (exact_div.hpp, bp_common.hpp):
 * in[n][3] = (n0, n1, s) -> out[n][12] = (FAST VN quotients n0/s, n1/s
 * (dd_quot), div_rn n0/s, n1/s (correctly rounded, any operands), the CN
 * phase's near-one quotients n0/s, n1/s, the near-one reciprocal formula of s,
 * hipcc's refined reciprocal of s, hipcc's '/' n0/s, n1/s, flags: bit 0 / 1 =
 * dd_check could not prove the FAST quotient of n0 / n1, bit 2 = div2's
 * suspect flag, |1 - s v_rcp_f64(s)|: the hardware reciprocal's error). */
int kml_div_probe(kml_ctx *ctx, const double *in, int n, double *out);
/* Test hook: after the nth (0-based) cooperative BP launch from now, set that
 * kernel's abort word as a timed-out group barrier would (nth < 0: off).  The
 * call that owns the launch must then fail with KML_E_HIP, even when later
 * launches of the same call (chunks of a host-buffer decode) follow it.
 * nth = -2: raise the abort after the next cooperative launch AND fail that
 * call at once, before its sync (the error-return path: the next call must
 * start clean, not inherit the abort). */
int kml_debug_inject_abort(kml_ctx *ctx, int nth);

#ifdef __cplusplus
}
#endif
#endif
