"""Pin the CPU oracle (oracle/oracle.c) against the reference's own outputs.

The golden fixtures were produced by running the reference sources
(/root/reference, compiled by oracle/Makefile into oracle/_ref/ref_harness) with
seed 17; see tests/golden/make_golden.py.  These tests need no GPU.
"""
import json
import math
import os
import zlib

import numpy as np
import pytest

from conftest import GOLDEN, case_names, load_case
from oracle import oracle as O

CASES = case_names()


def crc(a):
    return zlib.crc32(np.ascontiguousarray(a).tobytes()) & 0xFFFFFFFF


_codes = {}


def get_code(data_dir, hdr):
    key = (hdr["matrix"], hdr["is5g"], hdr["active"], hdr["max_iter"])
    if key not in _codes:
        _codes[key] = O.Code(os.path.join(data_dir, hdr["matrix"]), bool(hdr["is5g"]), bool(hdr["active"]), False,
                             hdr["max_iter"])
    return _codes[key]


def n_for(hdr, cap):
    return min(hdr["ncw"], cap)


@pytest.mark.parametrize("case", CASES)
def test_frames_and_receive_match_reference(case, data_dir):
    """Frame generation (RNG, encoder, channel) and the receive chain
    (k-means, metrics, demap, BP, counts) are bit-exact vs the reference."""
    hdr, z = load_case(case)
    code = get_code(data_dir, hdr)
    modem = O.Modem(os.path.join(data_dir, hdr["modem"]))
    assert np.array_equal(modem.points.reshape(-1, 2), z["cons"])
    n = n_for(hdr, 40 if code.N > 5000 else 120)
    uu, cc, th, y = O.gen_frames(code, modem, hdr["snr"], n)
    nv = z["v_y"].shape[0]
    for i in range(n):
        assert crc(uu[i].astype(np.uint8)) == z["s_crc_uu"][i]
        assert np.array_equal(th[i], z["s_true_h"][i])
        assert crc(y[i]) == z["s_crc_y"][i], f"y mismatch at cw {i}"
        if i < nv:
            assert np.array_equal(cc[i].astype(np.uint8), z["v_cc"][i])
    syn = np.zeros(code.M)
    blind = not hdr["known"]
    for i in range(n):
        r = O.receive(code, modem, y[i], th[i], hdr["snr"], blind, syn=syn)
        assert r["chosen"] == z["s_chosen"][i], f"cw {i}"
        if blind:
            assert np.array_equal(r["h_hat"], z["s_hhat"][i]), f"cw {i}"
            assert np.array_equal(r["metrics"], z["s_metrics"][i]), f"cw {i}"
        assert crc(r["p0"]) == z["s_crc_p0"][i], f"p0 cw {i}"
        assert r["ret"] == z["s_ret"][i]
        assert crc(r["uu_hat"]) == z["s_crc_uuhat"][i]
        errs = int(np.sum(r["uu_hat"] != uu[i].astype(np.uint8)))
        assert errs == z["s_errs"][i]


@pytest.mark.parametrize("case", CASES)
def test_bp_internals_match_reference(case, data_dir):
    """Direct decode of the reference's P0 vectors: cc_hat and syndrom_soft
    (every CN-phase message enters it) are bit-exact."""
    hdr, z = load_case(case)
    code = get_code(data_dir, hdr)
    for i in range(z["v_p0"].shape[0]):
        ret, uh, cch, syn = code.bp_decode(z["v_p0"][i])
        assert ret == z["s_ret"][i]
        assert np.array_equal(cch, z["v_cc_hat"][i])
        if ret > 1:  # syndrom_soft is only written when a CN phase ran
            assert np.array_equal(syn, z["v_syn"][i])
        assert np.array_equal(uh, z["v_uu_hat"][i])


def test_end_to_end_counters(data_dir):
    """SourceSink counters of the reference's own loop (2000 cw, seed 17)."""
    ctr = json.load(open(os.path.join(GOLDEN, "counters.json")))
    c = ctr["peg2304_qpsk_known_2000"]
    code = O.Code(os.path.join(data_dir, c["matrix"]), False, True, False, c["max_iter"])
    modem = O.Modem(os.path.join(data_dir, c["modem"]))
    n = 300  # prefix of the same stream; full 2000 in the slow variant
    uu, cc, th, y = O.gen_frames(code, modem, c["snr"], n)
    eb = ek = 0
    for i in range(n):
        r = O.receive(code, modem, y[i], th[i], c["snr"], False)
        e = int(np.sum(r["uu_hat"] != uu[i].astype(np.uint8)))
        eb += e
        ek += e > 0
    hdr, z = load_case("peg2304_qpsk_known")
    assert ek == int(np.sum(z["s_errs"][:n] > 0))
    assert eb == int(np.sum(z["s_errs"][:n]))


@pytest.mark.slow
def test_end_to_end_counters_full(data_dir):
    ctr = json.load(open(os.path.join(GOLDEN, "counters.json")))
    c = ctr["peg2304_qpsk_known_2000"]
    code = O.Code(os.path.join(data_dir, c["matrix"]), False, True, False, c["max_iter"])
    modem = O.Modem(os.path.join(data_dir, c["modem"]))
    uu, cc, th, y = O.gen_frames(code, modem, c["snr"], c["n"])
    eb = ek = 0
    for i in range(c["n"]):
        r = O.receive(code, modem, y[i], th[i], c["snr"], False)
        e = int(np.sum(r["uu_hat"] != uu[i].astype(np.uint8)))
        eb += e
        ek += e > 0
    assert (ek, eb) == (c["err_blk"], c["err_bit"])


def test_copy_constructed_row_order_same_decisions(data_dir):
    """binaryldpccodec.cc:31-46 reverses each row list in a copy; hard decisions
    are unchanged on the golden P0 vectors (messages may differ in the ulp)."""
    hdr, z = load_case("peg2304_qpsk_known")
    a = get_code(data_dir, hdr)
    b = O.Code(os.path.join(data_dir, hdr["matrix"]), False, True, True, hdr["max_iter"])
    for i in range(z["v_p0"].shape[0]):
        ra, ua, _, _ = a.bp_decode(z["v_p0"][i])
        rb, ub, _, _ = b.bp_decode(z["v_p0"][i])
        assert ra == rb and np.array_equal(ua, ub)


# ---------------------------------------------------------------- soft metric
from conftest import load_soft_case, soft_case_names  # noqa: E402


def oracle_soft_stream(code, modem, hdr, y, n):
    """The oracle run the way the reference's codec instance sees it: one
    syndrom_soft buffer carried across every decode of the stream (initially
    zeros), KmCodec::Decoder (mode soft) or GetHistogramData only (softhist)."""
    syn = np.zeros(code.M)
    var = 10 ** (-0.1 * hdr["snr"])
    out = []
    for i in range(n):
        if hdr["mode"] == "soft":
            r = O.receive(code, modem, y[i], np.zeros(2), hdr["snr"], True, metric_soft=True,
                          metric_iter=hdr["metric_iter"], syn=syn)
            out.append((r["metrics"], r["chosen"], r["uu_hat"]))
        else:
            hh = O.kmeans_hhat(y[i], modem.points)
            h4 = O.rotations(hh)
            met = np.zeros(4)
            uh = None
            for j in range(4):
                p0 = modem.demap(y[i], h4[j], var)
                _, uh, _, syn = code.bp_decode(p0, hdr["metric_iter"], syn=syn)
                mt = 0.0
                for v in syn:
                    mt += math.log(v)  # glibc log, like the reference
                met[j] = abs(mt)
            out.append((met, int(np.argmin(met)), uh))
    return out


def soft_frames(code, modem, hdr, z, n):
    """The fixture stream's frames, regenerated by the oracle (seed 17) and
    checked against the reference's CRCs."""
    uu, cc, th, y = O.gen_frames(code, modem, hdr["snr"], n)
    for i in range(n):
        assert crc(y[i]) == z["crc_y"][i] and crc(uu[i].astype(np.uint8)) == z["crc_uu"][i], i
    return uu, y


def soft_uu_hat(z, n, K):
    return np.unpackbits(z["uu_hat_bits"][:n], axis=1)[:, :K]


@pytest.mark.parametrize("case", soft_case_names())
def test_soft_metric_stream_matches_reference(case, data_dir):
    hdr, z = load_soft_case(case)
    code = O.Code(os.path.join(data_dir, hdr["matrix"]), bool(hdr["is5g"]), True, False, hdr["max_iter"])
    modem = O.Modem(os.path.join(data_dir, hdr["modem"]))
    n = min(len(z["chosen"]), 60)
    uu, y = soft_frames(code, modem, hdr, z, n)
    want_uh = soft_uu_hat(z, n, hdr["K"])
    res = oracle_soft_stream(code, modem, hdr, y, n)
    for i, (met, ch, uh) in enumerate(res):
        assert ch == z["chosen"][i], (case, i)
        assert np.array_equal(uh, want_uh[i]), (case, i)
        if hdr["mode"] == "softhist":  # returned exactly by GetHistogramData
            assert np.array_equal(met, z["metrics"][i]), (case, i)
        else:  # parsed from the codec's "%.14f" log records
            assert np.allclose(met, z["metrics"][i], rtol=0, atol=6e-15 * np.maximum(1, np.abs(met))), (case, i)


# --- the bench workload's and cfg5's reference counters (tests/golden/bench, sweep)

def _oracle_errs(data_dir, matrix, modem, is5g, known, max_iter, snr, n):
    code = O.Code(os.path.join(data_dir, matrix), bool(is5g), True, False, max_iter)
    md = O.Modem(os.path.join(data_dir, modem))
    uu, _, th, y = O.gen_frames(code, md, snr, n)
    syn = np.zeros(code.M)
    out = []
    for i in range(n):
        r = O.receive(code, md, y[i], th[i], snr, not known, syn=syn)
        out.append(int(np.sum(r["uu_hat"] != uu[i].astype(np.uint8))))
    return np.array(out)


@pytest.mark.parametrize("name,n", [("peg2304_qpsk_known_32768", 300), ("peg2304_qpsk_blind_32768", 120)])
def test_oracle_reproduces_bench_fixture(name, n, data_dir):
    """The bench's BER-match reference (the reference's own SourceSink counters
    over the first 32768 seed-17 codewords): self-consistent, and its first n
    per-codeword error counts are reproduced by the oracle."""
    z = np.load(os.path.join(GOLDEN, "bench", name + ".npz"))
    hdr = json.loads(bytes(z["hdr_json"]).decode())
    errs = z["errs"].astype(np.int64)
    assert len(errs) == hdr["n"] == hdr["tot_blk"]
    assert int(errs.sum()) == hdr["err_bit"] and int((errs > 0).sum()) == hdr["err_blk"]
    assert abs(hdr["ber"] - hdr["err_bit"] / (hdr["K"] * hdr["n"])) < 1e-15
    got = _oracle_errs(data_dir, hdr["matrix"], hdr["modem"], hdr["is5g"], hdr["known"], hdr["max_iter"], hdr["snr"],
                       n)
    assert np.array_equal(got, errs[:n])
    # the 2000-codeword counters of counters.json are a prefix of this stream
    ctr = json.load(open(os.path.join(GOLDEN, "counters.json")))
    c2k = ctr["peg2304_qpsk_known_2000" if hdr["known"] else "peg2304_qpsk_blind_2000"]
    assert int(errs[:2000].sum()) == c2k["err_bit"] and int((errs[:2000] > 0).sum()) == c2k["err_blk"]


def test_oracle_reproduces_cfg5_sweep_fixture(data_dir):
    """cfg5 sweep counters (PEG8064 + 64QAM-Gray blind, snr 4.77..8.77, the
    reference's simulate mode): the oracle reproduces each point's first
    codewords of the seed-17 stream."""
    z = np.load(os.path.join(GOLDEN, "sweep", "cfg5.npz"))
    assert z["errs"].shape == (5, 400)
    for p, snr in enumerate(z["snr"]):
        e = z["errs"][p].astype(np.int64)
        assert int(e.sum()) == z["counters"][p][0] and int((e > 0).sum()) == z["counters"][p][1]
        got = _oracle_errs(data_dir, "PEG8064regular0.5.txt", "6bits_64QAM_Gray.txt", False, False, 20, float(snr), 6)
        assert np.array_equal(got, e[:6]), snr


KMSTATE = sorted(f[:-4] for f in os.listdir(os.path.join(os.path.dirname(__file__), "golden", "kmstate")))


@pytest.mark.parametrize("name", KMSTATE)
def test_oracle_kmeans_state_matches_reference(name, data_dir):
    """KMeans::clusters() and idx() after Run, from the reference itself
    (golden/kmstate, ref_harness mode kmstate): the oracle restatement
    (orc_kmeans_state) reproduces them bit for bit."""
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "kmstate", name + ".npz"))
    hdr = json.loads(bytes(z["hdr_json"]).decode())
    om = O.Modem(os.path.join(data_dir, hdr["modem"]))
    for b in range(hdr["n"]):
        cl, idx = O.kmeans_state(z["y"][b], om.points, hdr["iters"])
        assert np.array_equal(cl, z["clusters"][b]), b
        assert np.array_equal(idx, z["idx"][b]), b
