"""GPU tests of the measurement path (SURVEY §8 rows d/e, a13, cfg5):

* the sim path's CntErr (the BP epilogue's packed-bit error count,
  bp_common.hpp) against an independent count of uu_hat != uu for every
  codeword, on all three kernel families;
* the bench's BER match: the reference's own seed-17 stream decoded through
  the resident-batch path reproduces the reference's per-codeword error bits
  (tests/golden/bench, made by oracle/_ref = the reference's sources);
* Monte-Carlo BER of GPU (Philox) frames within 1 sigma of the reference BER;
* `bench.py --gpus 2` really runs 2 ranks (gloo here, RCCL on a multi-GPU node)
  and sums their counters;
* cfg5: the PEG8064 + 64QAM-Gray blind Eb/N0 0..4 dB sweep through the
  simulator driver, sharded over 2 ranks, equals the 1-rank run and matches
  the reference's sweep counters statistically.
"""
import json
import math
import os
import re
import subprocess
import sys

import numpy as np
import pytest

from conftest import GOLDEN, REPO, write_config

import kmldpc_amd as K

pytestmark = pytest.mark.gpu


def _ctx(data_dir, tmp_path, matrix, modem, is5g=False, known=True, max_iter=20, snr=2.0, **kw):
    cfg = str(tmp_path / f"c_{matrix}_{known}.toml")
    write_config(cfg, data_dir, matrix, modem, is5g=is5g, known=known, max_iter=max_iter, snr=snr, **kw)
    return K.Context(cfg, data_dir=data_dir, device=0)


def _bench_fixture(name):
    z = np.load(os.path.join(GOLDEN, "bench", name + ".npz"))
    return json.loads(bytes(z["hdr_json"]).decode()), z["errs"].astype(np.int64)


def _ber_sigma(errs, Kb):
    e = np.asarray(errs, np.float64)
    return e.std(ddof=1) / math.sqrt(len(e)) / Kb


# (matrix, modem, is5g, max_iter, snr, known, B): one per kernel family, plus blind
SIM_CASES = [
    ("PEG2304regular0.5.txt", "2bits_QPSK.txt", False, 20, 2.0, True, 4096),      # bp_regular_kernel (fused demap)
    ("PEG2304regular0.5.txt", "2bits_QPSK.txt", False, 20, 2.0, False, 2048),     # blind: k-means + metric + BP
    ("5GLDPCBG2a3_R12_K960.txt", "4bit_16QAM_Gray.txt", True, 50, 5.01, True, 2048),  # bp_irregular_kernel
    ("PEG8064regular0.5.txt", "6bits_64QAM_Gray.txt", False, 20, 6.77, True, 512),    # bp_part_kernel
]


@pytest.mark.parametrize("matrix,modem,is5g,max_iter,snr,known,B", SIM_CASES)
def test_sim_cnterr_matches_independent_count(data_dir, tmp_path, matrix, modem, is5g, max_iter, snr, known, B):
    """kml_sim_decode_ex's per-codeword error bits (the BP epilogue's
    ballot/popcount CntErr) equal (uu_hat != uu).sum() with uu_hat from
    kml_decode_frames on the same frames and uu from the frame generator."""
    ctx = _ctx(data_dir, tmp_path, matrix, modem, is5g=is5g, known=known, max_iter=max_iter, snr=snr)
    ctx.sim_generate(snr, B, seed=123, first_cw=5000)
    uu, y, h = ctx.sim_frames(B)
    cw_err, _, c = ctx.sim_decode_ex(snr, blind=not known)
    r = ctx.decode_frames(y, snr, h if known else None)
    indep = (r["uu_hat"] != uu).sum(axis=1)
    assert np.array_equal(cw_err, indep)
    assert c["err_bit"] == int(indep.sum()) and c["err_blk"] == int((indep > 0).sum())
    assert c["tot_blk"] == B and c["tot_bit"] == B * ctx.K
    assert 0 < c["err_blk"] < B or snr > 6  # a non-trivial mix of right and wrong codewords
    ctx.close()


@pytest.mark.parametrize("name,n", [("peg2304_qpsk_known_32768", 32768), ("peg2304_qpsk_blind_32768", 8192),
                                    ("bg2_16qam_known_16384", 16384), ("peg8064_64qam_blind_2048", 2048),
                                    ("peg8064_64qam_blind_s477_1024", 1024), ("peg8064_64qam_blind_s577_1024", 1024),
                                    ("peg8064_64qam_blind_s777_1024", 1024), ("peg8064_64qam_blind_s877_1024", 1024)])
def test_bench_reference_stream_is_exact(data_dir, tmp_path, name, n):
    """The bench's ber_match leg: the first n codewords of the reference's
    seed-17 stream loaded as the resident batch (kml_sim_load) give, codeword by
    codeword, the error bits the reference's SourceSink::CntErr counted."""
    hdr, ref = _bench_fixture(name)
    ctx = _ctx(data_dir, tmp_path, hdr["matrix"], hdr["modem"], is5g=hdr["is5g"], known=hdr["known"],
               max_iter=hdr["max_iter"], snr=hdr["snr"])
    uu, th, y = ctx.ref_frames(K.CLCRandNum(hdr["seed"]), hdr["snr"], n)
    ctx.sim_load(hdr["snr"], uu, y, th)
    cw_err, _, c = ctx.sim_decode_ex(hdr["snr"], blind=not hdr["known"])
    assert np.array_equal(cw_err, ref[:n])
    assert c["err_bit"] == int(ref[:n].sum()) and c["err_blk"] == int((ref[:n] > 0).sum())
    if n == hdr["n"]:
        assert (c["err_bit"], c["err_blk"]) == (hdr["err_bit"], hdr["err_blk"])
    ctx.close()


@pytest.mark.parametrize("name,B", [("peg2304_qpsk_known", 16384), ("peg2304_qpsk_blind", 8192),
                                    ("bg2_16qam_known", 4096), ("peg8064_64qam_blind", 1024)])
def test_gpu_monte_carlo_ber_matches_reference(data_dir, tmp_path, name, B):
    """north_star: BER within Monte-Carlo confidence of the reference, on GPU
    (Philox) frames, against the reference statistic of the same point
    (bench/large_oracle.json: the oracle restatement, bit-exact vs the
    reference, over 8 seed streams of the reference's generator).  Eight
    independent Philox seeds of B codewords each:
      * the pooled BER within 3 sigma of the reference (sigma combines both
        standard errors, the codeword as the unit — the bit errors of one
        codeword are dependent);
      * the eight per-seed BERs scatter as their standard errors say (chi-square
        of their deviations from the pooled mean, 7 dof, below its 99.9% point).
    A single fixed-seed draw at 1 sigma would pass only ~68% of the time for an
    identical distribution, so it is printed (and carried by the bench line as
    ber_within_1sigma) but not asserted.  The exact form of "BER match" —
    identical frames, identical counters — is test_bench_reference_stream_is_exact."""
    ref = json.load(open(os.path.join(GOLDEN, "bench", "large_oracle.json")))[name]
    Kb, n_ref = ref["K"], ref["codewords"]
    ctx = _ctx(data_dir, tmp_path, ref["matrix"], ref["modem"], is5g=ref["is5g"], known=ref["known"],
               max_iter=ref["max_iter"], snr=ref["snr"])
    g, sg, errs = [], [], []
    for seed in range(8):
        ctx.sim_generate(ref["snr"], B, seed=1000 + seed, first_cw=0)
        cw_err, _, c = ctx.sim_decode_ex(ref["snr"], blind=not ref["known"])
        g.append(c["err_bit"] / c["tot_bit"])
        sg.append(_ber_sigma(cw_err, Kb))
        errs.append(cw_err)
    ctx.close()
    allerr = np.concatenate(errs)
    ber = float(allerr.sum()) / (len(allerr) * Kb)
    ber_ref = ref["err_bit"] / (n_ref * Kb)
    m = ref["err_bit"] / n_ref
    sig_ref = math.sqrt((ref["sum_e2"] / n_ref - m * m) * n_ref / (n_ref - 1) / n_ref) / Kb
    sig = math.hypot(_ber_sigma(allerr, Kb), sig_ref)
    z = (ber - ber_ref) / sig
    chi2 = sum(((gi - ber) / si) ** 2 for gi, si in zip(g, sg))
    zs = [(gi - ber_ref) / math.hypot(si, sig_ref) for gi, si in zip(g, sg)]
    print(f"{name}: GPU BER {ber:.6f} ({len(allerr)} cw, 8 seeds) vs reference {ber_ref:.6f} ({n_ref} cw): "
          f"z {z:+.3f}; per-seed z {[round(v, 2) for v in zs]} ({sum(abs(v) <= 1 for v in zs)}/8 within 1 sigma); "
          f"chi2 {chi2:.2f}")
    assert abs(z) <= 3
    assert chi2 <= 24.32  # chi-square, 7 dof, 99.9%


def _bench(args, timeout=300):
    env = dict(os.environ, PYTHONPATH=REPO)
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, capture_output=True, text=True,
                       timeout=timeout, env=env, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{"metric"')]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_two_ranks_gloo(data_dir, tmp_path):
    """`bench.py --gpus 2` launches 2 rank processes itself (torch.distributed.run
    as a child), both decode their shard of global codeword indices, and the
    counters of rank 0's line are the sum over both shards — equal to one
    decode of the whole index range."""
    B = 2048
    line = _bench(["--gpus", "2", "--dist-backend", "gloo", "--steps", "2", "--warmup", "1", "--batch", str(B),
                   "--no-cpu-baseline", "--no-ber-match", "--full-loop-batches", "1"])
    assert line["n_gpus"] == 2 and line["ranks"] == 2 and line["dist_backend"].startswith("gloo counters")
    assert len(line["rank_ms_per_step"]) == 2 and line["config"]["global_batch"] == 2 * B
    st = line["stats"]
    assert st["codewords"] == 2 * B
    ctx = _ctx(data_dir, tmp_path, "PEG2304regular0.5.txt", "2bits_QPSK.txt")
    ctx.sim_generate(2.0, 2 * B, seed=17, first_cw=0)
    c = ctx.sim_decode(2.0, blind=False)
    assert round(st["fer"] * 2 * B) == c["err_blk"]
    assert round(st["ber"] * c["tot_bit"]) == c["err_bit"]
    assert line["full_loop"]["value"] > 0 and line["value"] > 0
    ctx.close()


@pytest.mark.timeout(400)
def test_bench_eight_ranks_gloo(data_dir, tmp_path):
    """`bench.py --gpus 8` with 8 rank processes sharing this GPU (gloo
    counters): the N = 8 rank logic of the driver's scaling run (child
    torchrun, shard offsets rank * B, barrier, max-over-ranks timing, counter
    all-reduce) with only the RCCL transport left out.  Rank 0's counters equal
    one decode of the whole index range [0, 8 B) (simulator.cc:35-42, 86-100)."""
    B, W = 512, 8
    line = _bench(["--gpus", str(W), "--dist-backend", "gloo", "--steps", "2", "--warmup", "1", "--batch", str(B),
                   "--no-cpu-baseline", "--no-ber-match", "--full-loop-batches", "1"], timeout=380)
    assert line["n_gpus"] == W and line["ranks"] == W and line["dist_backend"].startswith("gloo counters")
    assert len(line["rank_ms_per_step"]) == W and line["config"]["global_batch"] == W * B
    assert line["ms_per_step"] == pytest.approx(max(line["rank_ms_per_step"]), rel=1e-6)
    st = line["stats"]
    assert st["codewords"] == W * B
    ctx = _ctx(data_dir, tmp_path, "PEG2304regular0.5.txt", "2bits_QPSK.txt")
    ctx.sim_generate(2.0, W * B, seed=17, first_cw=0)
    c = ctx.sim_decode(2.0, blind=False)
    assert round(st["fer"] * W * B) == c["err_blk"]
    assert round(st["ber"] * c["tot_bit"]) == c["err_bit"]
    ctx.close()


@pytest.mark.timeout(400)
def test_simulate_eight_ranks_gloo_matches_single_rank(data_dir, tmp_path):
    """kmldpc_amd.simulate under torchrun --nproc-per-node 8 (ranks sharing this
    GPU, gloo counters): blind PEG2304 at two SNR points with an error limit
    that lands inside a round and a block limit no round size divides.  The
    BER / FER tables equal the single-process run's (the stop rule is exact for
    any world, simulate.cpp kml_sweep_point; simulator.cc:117)."""
    cfg = tmp_path / "config.toml"
    write_config(str(cfg), data_dir, "PEG2304regular0.5.txt", "2bits_QPSK.txt", known=False, snr=1.0, snr_max=2.0,
                 snr_step=1.0, max_blocks=2900, max_err=333, thread_blocks=1000)
    env = dict(os.environ, PYTHONPATH=REPO, KML_BATCH="96", KML_SEED="5", KML_DIST_BACKEND="gloo",
               OMP_NUM_THREADS="1")
    r1 = subprocess.run([sys.executable, "-m", "kmldpc_amd.simulate", str(cfg)], cwd=tmp_path, env=env,
                        capture_output=True, text=True, timeout=300)
    assert r1.returncode == 0, r1.stderr[-3000:]
    r8 = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=8",
                         "--master-addr=127.0.0.1", "--master-port=29547", "-m", "kmldpc_amd.simulate", str(cfg)],
                        cwd=tmp_path, env=env, capture_output=True, text=True, timeout=360)
    assert r8.returncode == 0, r8.stderr[-3000:]
    b1, f1 = _tables(r1.stdout)
    b8, f8 = _tables(r8.stdout)
    assert b1 == b8 and f1 == f8 and len(b1) == 2


def test_bench_one_rank_rccl_group(data_dir):
    """The RCCL leg on hardware: `bench.py --gpus 1 --force-dist` runs one rank
    under torch.distributed.run (gloo rendezvous), builds the library's RCCL
    communicator (kml_comm_unique_id / kml_comm_init) and all-reduces the
    counters through it (kml_comm_allreduce_f64, on the context's stream); its
    counters equal the plain single-process run on the same frames."""
    args = ["--steps", "2", "--warmup", "1", "--batch", "2048", "--no-cpu-baseline", "--no-ber-match",
            "--full-loop-batches", "1"]
    plain = _bench(args)
    line = _bench(args + ["--gpus", "1", "--force-dist"])
    assert line["rccl_ranks"] == 1 and line["dist_backend"].startswith("rccl counters") and line["ranks"] == 1
    assert len(line["rank_ms_per_step"]) == 1
    for k in ("fer", "ber", "codewords", "mean_cn_phases"):
        assert line["stats"][k] == plain["stats"][k], k


def test_simulate_one_rank_rccl_group(data_dir, tmp_path):
    """kmldpc_amd.simulate under torchrun --nproc-per-node 1 with a forced
    1-rank process group (KML_FORCE_DIST=1, --dist-backend nccl): the
    per-round stop-rule and counter all-reduces of kml_sim_point run through
    the library's RCCL communicator, and the BER / FER tables equal the run
    without a process group."""
    cfg = tmp_path / "config.toml"
    write_config(str(cfg), data_dir, "PEG2304regular0.5.txt", "2bits_QPSK.txt", known=False, snr=1.0, snr_max=2.0,
                 snr_step=1.0, max_blocks=3000, max_err=700, thread_blocks=1000)
    env = dict(os.environ, PYTHONPATH=REPO, KML_BATCH="1024", KML_SEED="3", OMP_NUM_THREADS="1")
    r1 = subprocess.run([sys.executable, "-m", "kmldpc_amd.simulate", str(cfg)], cwd=tmp_path, env=env,
                        capture_output=True, text=True, timeout=300)
    assert r1.returncode == 0, r1.stderr[-3000:]
    r2 = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
                         "--master-addr=127.0.0.1", "--master-port=29541", "-m", "kmldpc_amd.simulate", str(cfg)],
                        cwd=tmp_path, env=dict(env, KML_FORCE_DIST="1", KML_DIST_BACKEND="nccl"),
                        capture_output=True, text=True, timeout=300)
    assert r2.returncode == 0, r2.stderr[-3000:]
    assert _tables(r1.stdout) == _tables(r2.stdout)


def test_bench_single_rank_line(data_dir):
    """The N=1 line carries the roofline (fp64-valu), the exact BER match on
    the reference stream and the 1-sigma statistic."""
    line = _bench(["--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--full-loop-batches", "1"])
    assert line["n_gpus"] == 1 and line["rccl_ranks"] == 0 and line["dist_backend"] is None
    rf = line["roofline"]
    assert rf["bound"] == "fp64-valu" and 0 < rf["frac"] < 1
    bm = line["stats"]["ber_match"]
    assert bm["exact"] and bm["per_codeword_equal"]
    assert isinstance(line["stats"]["ber_within_1sigma"], bool)


CFG5_SNRS = [4.77, 5.77, 6.77, 7.77, 8.77]
_PAT = re.compile(r"^(\d\.\d{3}) (\d\.\d{14})$")


def _tables(out):
    """The BER / FER result tables of the driver's console output."""
    msgs = [ln.split("[INFO]\x1b[0m ", 1)[1] for ln in out.splitlines() if "[INFO]" in ln]
    i, j = msgs.index("BER Result"), msgs.index("FER Result")
    ber = {m.group(1): float(m.group(2)) for m in map(_PAT.match, msgs[i + 1:j]) if m}
    fer = {m.group(1): float(m.group(2)) for m in map(_PAT.match, msgs[j + 1:j + 1 + len(ber)]) if m}
    return ber, fer


def test_cfg5_sweep_sharded_matches_single_rank_and_reference(data_dir, tmp_path):
    """cfg5 (BASELINE configs[4]): PEG8064 + 64QAM-Gray, blind k-means, Eb/N0
    0..4 dB (snr 4.77..8.77), through the simulator driver
    (Simulator::Simulate, simulator.cc:25-67), 4096 codewords per point (the
    bench's batch).  Two ranks sharing this GPU (gloo counters) print the same
    BER/FER tables as one rank — codeword indices, not ranks, key the frames.
    Against the reference statistic of each point (bench/large_oracle.json:
    8192 codewords of the oracle restatement, bit-exact vs the reference, over
    8 seed streams): every point within 3 sigma, and the five z-scores jointly
    consistent with N(0, 1) (sum z^2 below the 99% chi-square quantile, 5 dof).
    The bit-exact parity of the same points is test_decode_frames_vs_reference_stream
    on the peg8064_64qam_blind_s* fixtures and test_bench_reference_stream_is_exact."""
    large = json.load(open(os.path.join(GOLDEN, "bench", "large_oracle.json")))
    cfg = tmp_path / "config.toml"
    nblk = 4096
    write_config(str(cfg), data_dir, "PEG8064regular0.5.txt", "6bits_64QAM_Gray.txt", known=False, snr=4.77,
                 snr_max=8.77, snr_step=1.0, max_blocks=nblk, max_err=10 ** 9, thread_blocks=nblk)
    env = dict(os.environ, PYTHONPATH=REPO, KML_BATCH="1024", KML_SEED="7", KML_DIST_BACKEND="gloo",
               OMP_NUM_THREADS="1")
    r1 = subprocess.run([sys.executable, "-m", "kmldpc_amd.simulate", str(cfg)], cwd=tmp_path, env=env,
                        capture_output=True, text=True, timeout=300)
    assert r1.returncode == 0, r1.stderr[-3000:]
    r2 = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                         "--master-addr=127.0.0.1", "--master-port=29533", "-m", "kmldpc_amd.simulate", str(cfg)],
                        cwd=tmp_path, env=env, capture_output=True, text=True, timeout=300)
    assert r2.returncode == 0, r2.stderr[-3000:]
    b1, f1 = _tables(r1.stdout)
    b2, f2 = _tables(r2.stdout)
    assert b1 == b2 and f1 == f2 and len(b1) == 5
    from kmldpc_amd.simulate import point_seed
    ctx = _ctx(data_dir, tmp_path, "PEG8064regular0.5.txt", "6bits_64QAM_Gray.txt", known=False, snr=4.77)
    Kb = ctx.K
    zs = []
    for p, snr in enumerate(CFG5_SNRS):
        key = f"{snr:.3f}"
        # the driver's frames of this point, decoded directly: same counters, plus the per-codeword spread
        s = 4.77 + 1.0 * p
        ctx.sim_generate(s, nblk, seed=point_seed(7, p), first_cw=0)
        cw_err, _, c = ctx.sim_decode_ex(s, blind=True)
        assert abs(b1[key] - c["err_bit"] / c["tot_bit"]) < 1e-13 and abs(f1[key] - c["err_blk"] / nblk) < 1e-13
        ref = large["peg8064_64qam_blind" + ("" if snr == 6.77 else f"_s{int(round(snr * 100))}")]
        assert abs(ref["snr"] - snr) < 1e-12 and ref["K"] == Kb
        n_ref = ref["codewords"]
        ber_ref = ref["err_bit"] / (n_ref * Kb)
        m = ref["err_bit"] / n_ref
        sig_ref = math.sqrt((ref["sum_e2"] / n_ref - m * m) * n_ref / (n_ref - 1) / n_ref) / Kb
        sig = math.hypot(sig_ref, _ber_sigma(cw_err, Kb))
        z_p = (b1[key] - ber_ref) / sig
        zs.append(z_p)
        print(f"cfg5 snr {snr}: GPU BER {b1[key]:.6f} FER {f1[key]:.4f} ({nblk} cw) vs reference BER {ber_ref:.6f} "
              f"FER {ref['fer']:.4f} ({n_ref} cw): sigma {sig:.6f}, z {z_p:+.2f}")
        assert abs(z_p) <= 3, snr
    print(f"cfg5: {sum(abs(z) <= 1 for z in zs)}/5 points within 1 sigma, sum z^2 = {sum(z * z for z in zs):.2f}")
    assert sum(z * z for z in zs) <= 15.09  # chi-square, 5 dof, 99%
    ctx.close()
    bers = [b1[f"{s:.3f}"] for s in CFG5_SNRS]
    assert all(a >= b for a, b in zip(bers, bers[1:]))  # BER falls with SNR
