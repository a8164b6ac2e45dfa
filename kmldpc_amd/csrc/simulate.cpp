// simulate.cpp — the Monte-Carlo driver around the receive path:
// Simulator::run / run_blocks (src/simulator.cc:72-168) as a batched,
// rank-sharded loop over one SNR point.
//
// The reference runs ceil(maximum_block_number / thread_block_number) tasks on
// a thread pool; each task checks `tot_blk >= maximum_block_number ||
// err_blk >= maximum_error_number` before every codeword (simulator.cc:117).
// A single sequential stream therefore counts codewords 0, 1, 2, ... and stops
// right after the codeword that brings err_blk to the limit.  Here codewords
// are identified by a global index (the GPU frame generator is keyed by it), a
// round decodes world*batch consecutive indices, and the prefix rule is applied
// exactly after each round: the ranks all-reduce their per-rank block-error
// counts (world numbers), each rank truncates its own slice where the running
// total reaches the limit, and the four counters are all-reduced.  The totals
// equal the sequential stream's for any world and batch.
#include <algorithm>
#include <cstdio>
#include <vector>

#include "../../include/kmldpc_amd.h"

extern "C" int kml_sweep_point(const kml_point_cfg *cfg, kml_batch_fn decode, void *duser, kml_allreduce_fn reduce,
                               void *ruser, kml_report_fn report, void *puser, uint64_t *counters) {
  if (!cfg || !decode || !counters || cfg->batch <= 0 || cfg->world < 1 || cfg->rank < 0 ||
      cfg->rank >= cfg->world || cfg->K < 0 || (cfg->world > 1 && !reduce))
    return KML_E_ARG;
  const int W = cfg->world, r = cfg->rank, B = cfg->batch;
  const int nc = cfg->ncand < 1 ? 1 : (cfg->ncand > 4 ? 4 : cfg->ncand);
  const uint64_t K = (uint64_t)cfg->K;
  FILE *hf = nullptr;
  if (cfg->hist_path) {
    hf = fopen(cfg->hist_path, "w");
    if (!hf) return KML_E_IO;
  }
  std::vector<int32_t> err(B, 0);
  std::vector<double> met(cfg->hist_path ? (size_t)B * 4 : 0);
  std::vector<uint64_t> v(W);
  uint64_t ebit = 0, eblk = 0, tbit = 0, tot = 0;
  int rc = KML_OK;
  while (tot < cfg->max_blocks && eblk < cfg->max_err) {
    const uint64_t R = std::min<uint64_t>((uint64_t)W * B, cfg->max_blocks - tot);
    const long long mine = std::max<long long>(0, std::min<long long>(B, (long long)R - (long long)r * B));
    if (mine > 0) {
      rc = decode(tot + (uint64_t)r * B, (int)mine, err.data(), cfg->hist_path ? met.data() : nullptr, duser);
      if (rc != KML_OK) break;
    }
    uint64_t my_eb = 0;
    for (long long j = 0; j < mine; j++) my_eb += err[j] > 0;
    std::fill(v.begin(), v.end(), 0);
    v[r] = my_eb;
    // a 1-rank world still reduces when the caller passes a reducer (an identity
    // all-reduce; exercises a 1-rank RCCL process group)
    if (reduce && (rc = reduce(v.data(), W, ruser)) != KML_OK) break;
    uint64_t before = eblk;
    for (int q = 0; q < r; q++) before += v[q];
    // this rank's codewords in global order, with the per-codeword stop check
    uint64_t l_eb = 0, l_ebit = 0, take = 0;
    for (long long j = 0; j < mine; j++) {
      if (before + l_eb >= cfg->max_err) break;
      take++;
      if (err[j] > 0) {
        l_eb++;
        l_ebit += (uint64_t)err[j];
      }
      if (hf) {  // metrics rotated to start at the first minimum (simulator.cc:156-161)
        const double *m = &met[(size_t)j * 4];
        int best = 0;
        for (int q = 1; q < nc; q++)
          if (m[q] < m[best]) best = q;
        for (int q = best; q < best + nc; q++) fprintf(hf, "%g ", m[q % nc]);
        fputc('\n', hf);
      }
      if (W == 1 && report && cfg->report_every > 0 && (tot + take) % (uint64_t)cfg->report_every == 0) {
        const uint64_t c[4] = {ebit + l_ebit, eblk + l_eb, (tot + take) * K, tot + take};
        report(c, puser);
      }
    }
    uint64_t loc[4] = {l_ebit, l_eb, take * K, take};
    if (reduce && (rc = reduce(loc, 4, ruser)) != KML_OK) break;
    ebit += loc[0];
    eblk += loc[1];
    tbit += loc[2];
    tot += loc[3];
    if (W > 1 && report) {
      const uint64_t c[4] = {ebit, eblk, tbit, tot};
      report(c, puser);
    }
    if (loc[3] == 0) break;  // nothing counted (every rank hit the error limit)
  }
  if (hf) fclose(hf);
  counters[0] = ebit;
  counters[1] = eblk;
  counters[2] = tbit;
  counters[3] = tot;
  return rc;
}

namespace {
struct GpuBatch {
  kml_ctx *ctx;
  double snr;
  uint64_t seed;
  int blind, histogram;
};

int gpu_batch(uint64_t first, int count, int32_t *cw_err, double *metrics, void *user) {
  GpuBatch *g = static_cast<GpuBatch *>(user);
  int rc = kml_sim_generate(g->ctx, g->snr, g->seed, first, count);
  if (rc != KML_OK) return rc;
  return kml_sim_decode_ex(g->ctx, g->snr, g->blind, g->histogram, cw_err, metrics, nullptr);
}
}  // namespace

extern "C" int kml_sim_point(kml_ctx *ctx, const kml_point_cfg *cfg, uint64_t seed, kml_allreduce_fn reduce,
                             void *ruser, kml_report_fn report, void *puser, uint64_t *counters) {
  if (!ctx || !cfg) return KML_E_ARG;
  int64_t n[10];
  int rc = kml_run_config(ctx, nullptr, n);
  if (rc != KML_OK) return rc;
  GpuBatch g{ctx, cfg->snr, seed, n[3] ? 0 : 1, cfg->hist_path ? 1 : 0};
  kml_point_cfg c = *cfg;
  int32_t d[KML_DIM_COUNT];
  kml_dims(ctx, d);
  c.K = d[KML_DIM_K];
  c.ncand = n[3] ? 1 : 4;
  // soft metric: the reference restarts the codec (and its stale syndrome
  // state) every thread_block_number codewords; batches that start on those
  // boundaries keep every stale chain inside one batch of one rank
  const long long T = n[2];
  if (n[5] && T > 0) {
    if (T <= c.batch)
      c.batch -= (int)(c.batch % T);
    else if (T <= (1 << 20))
      c.batch = (int)T;
  }
  return kml_sweep_point(&c, gpu_batch, &g, reduce, ruser, report, puser, counters);
}
