"""GPU tests of the simulator driver (f2/f3 rows): kml_sim_point's stop rule on
real GPU decodes, histogram mode (KmCodec::GetHistogramData), and the two
front ends — the `kmldpc_sim` executable and `python -m kmldpc_amd.simulate` —
which must print the reference's lines and agree with each other."""
import os
import re
import subprocess
import sys

import numpy as np
import pytest

from conftest import REPO, write_config

import kmldpc_amd as K

pytestmark = pytest.mark.gpu


def _sequential(errs, max_blocks, max_err, Kb):
    eb = ebit = tot = 0
    while tot < max_blocks and eb < max_err:
        e = int(errs[tot])
        tot += 1
        if e:
            eb += 1
            ebit += e
    return dict(err_bit=ebit, err_blk=eb, tot_bit=tot * Kb, tot_blk=tot)


@pytest.mark.parametrize("known", [True, False])
def test_sim_point_stop_rule_on_gpu(data_dir, tmp_path, known):
    cfg = str(tmp_path / "c.toml")
    write_config(cfg, data_dir, "PEG2304regular0.5.txt", "2bits_QPSK.txt", known=known, snr=1.5)
    ctx = K.Context(cfg, data_dir=data_dir, device=0)
    N, seed = 3000, 99
    ctx.sim_generate(1.5, N, seed=seed, first_cw=0)
    errs, _, c = ctx.sim_decode_ex(1.5, blind=not known)
    assert c["tot_blk"] == N and int((errs > 0).sum()) == c["err_blk"] and int(errs.sum()) == c["err_bit"]
    for max_blocks, max_err, batch in [(3000, 10 ** 9, 1024), (2500, 300, 700), (3000, 1, 256), (777, 10 ** 9, 100)]:
        got = ctx.sim_point(1.5, seed, batch=batch, max_blocks=max_blocks, max_err=max_err)
        assert got == _sequential(errs, max_blocks, max_err, ctx.K), (max_blocks, max_err, batch)
    ctx.close()


def test_histogram_mode_peg_hard_metric(data_dir, tmp_path):
    cfg = str(tmp_path / "c.toml")
    write_config(cfg, data_dir, "PEG2304regular0.5.txt", "2bits_QPSK.txt", known=False, snr=3.0, histogram=True)
    ctx = K.Context(cfg, data_dir=data_dir, device=0)
    B = 512
    ctx.sim_generate(3.0, B, seed=5)
    uu, y, h = ctx.sim_frames(B)
    errs, met, c = ctx.sim_decode_ex(3.0, blind=True, histogram=True)
    # metrics = GetMetrics of the decode path; no final decode was run
    out = ctx.decode_frames(y, 3.0)
    assert np.array_equal(met, out["metrics"])
    assert c["vn_phases"] == 0 and c["cn_phases"] == 0
    # hard PEG metric: the error count sees all-zero decisions
    assert np.array_equal(errs, uu.sum(axis=1))
    ctx.close()


def test_histogram_mode_5g_metric_uses_last_candidate_decode(data_dir, tmp_path):
    cfg = str(tmp_path / "c.toml")
    write_config(cfg, data_dir, "5GLDPCBG2a3_R12_K960.txt", "4bit_16QAM_Gray.txt", is5g=True, known=False, snr=6.0,
                 histogram=True, max_iter=50, metric_iter=5)
    ctx = K.Context(cfg, data_dir=data_dir, device=0)
    B = 256
    ctx.sim_generate(6.0, B, seed=8)
    uu, y, h = ctx.sim_frames(B)
    errs, met, c = ctx.sim_decode_ex(6.0, blind=True, histogram=True)
    out = ctx.decode_frames(y, 6.0)
    assert np.array_equal(met, out["metrics"])
    _, h4 = ctx.kmeans(y)
    var = 10 ** (-6.0 / 10)
    p0 = ctx.demap(y, h4[:, 3], var)
    r = ctx.bp_decode(p0, iter_count=5)
    assert np.array_equal(errs, (r["uu_hat"] != uu).sum(axis=1))
    ctx.close()


def test_histogram_file_from_sim_point(data_dir, tmp_path):
    cfg = str(tmp_path / "c.toml")
    write_config(cfg, data_dir, "PEG2304regular0.5.txt", "2bits_QPSK.txt", known=False, snr=2.0, histogram=True)
    ctx = K.Context(cfg, data_dir=data_dir, device=0)
    ctx.sim_generate(2.0, 300, seed=21)
    _, met, _ = ctx.sim_decode_ex(2.0, blind=True, histogram=True)
    hp = str(tmp_path / "hist.txt")
    ctx.sim_point(2.0, 21, batch=128, max_blocks=300, max_err=10 ** 9, hist_path=hp)
    lines = open(hp).read().splitlines()
    assert len(lines) == 300
    for j in (0, 17, 299):
        best = int(np.argmin(met[j]))
        assert lines[j] == " ".join("%g" % met[j][q % 4] for q in range(best, best + 4)) + " "
    ctx.close()


_LINE = re.compile(r"^\[\d{4}-\d\d-\d\d \d\d:\d\d:\d\d\] \x1b\[32;1m\[INFO\]\x1b\[0m (.*)$")


def _messages(out):
    msgs = []
    for ln in out.splitlines():
        m = _LINE.match(ln)
        assert m, repr(ln)
        msgs.append(m.group(1))
    return msgs


def test_driver_executable_and_python_driver_agree(data_dir, tmp_path):
    cfg = tmp_path / "config.toml"
    write_config(str(cfg), data_dir, "PEG2304regular0.5.txt", "2bits_QPSK.txt", known=True, snr=1.0, snr_max=2.0,
                 snr_step=1.0, max_blocks=1000, max_err=150)
    env = dict(os.environ, KML_BATCH="384", KML_SEED="4")
    exe = os.path.join(REPO, "kmldpc_amd", "bin", "kmldpc_sim")
    r1 = subprocess.run([exe, str(cfg)], cwd=tmp_path, env=env, capture_output=True, text=True, timeout=300)
    assert r1.returncode == 0, r1.stderr
    r2 = subprocess.run([sys.executable, "-m", "kmldpc_amd.simulate", str(cfg)], cwd=tmp_path,
                        env=dict(env, PYTHONPATH=REPO), capture_output=True, text=True, timeout=300)
    assert r2.returncode == 0, r2.stderr
    m1, m2 = _messages(r1.stdout), _messages(r2.stdout)
    assert m1[0] == "Start simulation" and m1[1] == "Using traditional LDPC."
    assert m1[2] == "[1.000,1.000,2.000]" and m1[3] == "[MAX_ERROR_BLK = 150,MAX_BLK = 1000]"
    assert m1[-2] == "Simulation done" and m1[-1].startswith("Total time cost: ")
    assert m1[:-1] == m2[:-1]  # identical frames (same seed) -> identical counters and lines
    res = [m for m in m1 if m.startswith("SNR = ")]
    # the error limit (150) stops the 1 dB point early; progress lines every 100 blocks
    pat = re.compile(r"SNR = (\d\.\d{3}) Total blk = (\d{7}) Error blk = (\d{7}) Error bit = (\d{7}) "
                     r"BER = (\d\.\d{14}) FER = (\d\.\d{14})")
    finals = {}
    for m in res:
        g = pat.match(m)
        assert g, m
        finals[g.group(1)] = (int(g.group(2)), int(g.group(3)))
    assert finals["1.000"][1] == 150 and finals["1.000"][0] < 1000
    assert finals["2.000"][0] <= 1000
    i = m1.index("BER Result")
    assert re.match(r"^1\.000 0\.\d{14}$", m1[i + 1]) and m1[i + 3] == "FER Result"


def test_soft_metric_sim_path_statistics(data_dir, tmp_path):
    """The soft-metric blind path on GPU frames (sim path, per-task stale-state
    restarts) has the reference's FER within Monte-Carlo confidence (reference:
    the Decoder-only soft stream of tests/golden/soft, 300 cw)."""
    from conftest import load_soft_case
    hdr, z = load_soft_case("peg2304_qpsk_soft")
    ref = float(np.mean(z["errs"] > 0))
    cfg = str(tmp_path / "c.toml")
    write_config(cfg, data_dir, hdr["matrix"], hdr["modem"], known=False, snr=hdr["snr"], metric_type=True,
                 metric_iter=hdr["metric_iter"], thread_blocks=100000)
    ctx = K.Context(cfg, data_dir=data_dir, device=0)
    B = 4000
    ctx.sim_generate(hdr["snr"], B, seed=31)
    errs, met, c = ctx.sim_decode_ex(hdr["snr"], blind=True)
    fer = c["err_blk"] / c["tot_blk"]
    sigma = np.sqrt(ref * (1 - ref) / len(z["errs"]) + ref * (1 - ref) / B)
    print(f"soft-metric GPU FER {fer:.4f} vs reference {ref:.4f} (sigma {sigma:.4f})")
    assert abs(fer - ref) < 4 * sigma
    ctx.close()
