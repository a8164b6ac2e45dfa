"""GPU parity tests: the HIP path (through the C ABI) against the oracle and
the reference-generated golden fixtures.  Run on an MI355X with -m gpu.

Bars:
  * BP decoder (pure IEEE + - * /): bit-exact — uu_hat, return value, cc_hat
    and syndrom_soft (which depends on every CN-phase message).
  * k-means (hypot, Smith division, complex products): bit-exact h_hat.
  * demapper (exp = kml_exp, the glibc-exact restatement): bit-exact P0.
  * full KmCodec::Decoder path vs the reference stream fixtures: chosen
    candidate, metrics, h_hat, BP return value and uu_hat, bit-exact.
"""
import json
import os
import zlib

import numpy as np
import pytest

from conftest import GOLDEN, case_names, load_case
from oracle import oracle as O

import kmldpc_amd as K

pytestmark = pytest.mark.gpu

CASES = case_names()
_ctx = {}


def crc(a):
    return zlib.crc32(np.ascontiguousarray(a).tobytes()) & 0xFFFFFFFF


def ctx_for(data_dir, matrix, modem, is5g, max_iter=20, active=True):
    key = (matrix, modem, is5g, max_iter, active)
    if key not in _ctx:
        _ctx[key] = K.Context(matrix_file=os.path.join(data_dir, matrix), modem_file=os.path.join(data_dir, modem),
                              is5g=is5g, active=active, max_iter=max_iter, device=0)
    return _ctx[key]


_oc = {}


def oracle_for(data_dir, matrix, is5g, max_iter=20, active=True):
    key = (matrix, is5g, max_iter, active)
    if key not in _oc:
        _oc[key] = O.Code(os.path.join(data_dir, matrix), is5g, active, False, max_iter)
    return _oc[key]


def ulp_diff(a, b):
    ia = a.view(np.int64)
    ib = b.view(np.int64)
    return np.abs(ia - ib)


def test_device_exact_math_matches_host(data_dir):
    ctx = ctx_for(data_dir, "PEG2304regular0.5.txt", "2bits_QPSK.txt", False)
    rng = np.random.default_rng(1)
    n = 400000
    x = np.empty((n, 4))
    s = 2.0 ** rng.uniform(-20, 20, n)
    x[:, 0] = rng.normal(size=n) * s
    x[:, 1] = rng.normal(size=n) * np.where(np.arange(n) % 3 == 0, s, 1.0)
    x[:, 2] = rng.normal(size=n)
    x[:, 3] = rng.normal(size=n) * (np.arange(n) % 5 != 0)
    x[::17, 2] = np.arange(n)[::17] % 300 + 1.0
    x[::17, 3] = 0.0
    out = ctx.math_probe(x)
    h_ref = np.array([O.lib().orc_hypot(a, b) for a, b in x[:, :2]])
    assert np.array_equal(out[:, 0], h_ref)
    q = np.array([O.cdiv(*r) for r in x[:20000]])
    assert np.array_equal(out[:20000, 1:3], q)


def test_device_log_vs_glibc(data_dir):
    """The soft metric's log (kml_log) equals glibc's log bit for bit on device:
    probabilities, the close-to-1 branch, every exponent, special values."""
    import math
    ctx = ctx_for(data_dir, "PEG2304regular0.5.txt", "2bits_QPSK.txt", False)
    rng = np.random.default_rng(3)
    n = 300000
    x = np.concatenate([2.0 ** rng.uniform(-45, 0, n // 3), 1.0 + rng.uniform(-0.0625, 0.0647, n // 3),
                        2.0 ** rng.uniform(-1074, 1023, n // 3),
                        np.array([0.0, -0.0, 1.0, np.inf, -1.0, np.nan, 5e-324, 1e-12, 1 - 1e-12])])
    out = ctx.log_probe(x)
    with np.errstate(all="ignore"):
        ref = np.array([math.log(v) if v > 0 else (-np.inf if v == 0 else np.nan) for v in x])
    ref[x == np.inf] = np.inf
    same = (out.view(np.int64) == ref.view(np.int64)) | (np.isnan(out) & np.isnan(ref))
    assert same.all(), x[~same][:5]


def test_device_exp_vs_glibc(data_dir):
    """The demapper's exp (kml_exp) equals glibc's exp bit for bit on device."""
    import math
    ctx = ctx_for(data_dir, "PEG2304regular0.5.txt", "2bits_QPSK.txt", False)
    rng = np.random.default_rng(2)
    n = 200000
    x = np.zeros((n, 4))
    x[:, 0] = -rng.exponential(8.0, n)
    x[:, 2] = 1.0
    out = ctx.math_probe(x)[:, 3]
    ref = np.array([math.exp(v) for v in x[:, 0]])
    assert np.array_equal(out, ref)


def _same(a, b):
    """bitwise equality, any NaN equal to any NaN"""
    return (a.view(np.int64) == b.view(np.int64)) | (np.isnan(a) & np.isnan(b))


def test_fast_division_proven_or_flagged(data_dir):
    """The decoder's FAST VN division (exact_div.hpp dd_quot + dd_check, used
    by bp_common.hpp div2) over the value domain it runs on: numerators in
    {0} U [2^-961, 1] (bp_common.hpp fast_prior_ok), s = RN(n0 + n1) (the
    normalisations of the BP chains).
    Every quotient the check passes equals IEEE division; the check flags a
    quotient only near a rounding midpoint (the decoder then redoes the
    codeword on the exact path), which random operands almost never are; and
    div_rn equals IEEE division on all of them."""
    ctx = ctx_for(data_dir, "PEG2304regular0.5.txt", "2bits_QPSK.txt", False)
    rng = np.random.default_rng(7)
    flagged = total = 0
    for scale_exp in (1, 8, 40, 200, 840, 961):
        n = 400000
        n0 = rng.random(n) * 2.0 ** -rng.uniform(0, scale_exp, n)
        n1 = rng.random(n) * 2.0 ** -rng.uniform(0, scale_exp, n)
        n0[::97] = 0.0
        n1[1::89] = 0.0
        n0 = np.where(n0 < 2.0 ** -961, 0.0, n0)
        n1 = np.where(n1 < 2.0 ** -961, 0.0, n1)
        s = n0 + n1
        keep = s > 0
        x = np.stack([n0[keep], n1[keep], s[keep]], axis=1)
        out = ctx.div_probe(x)
        ref0, ref1 = x[:, 0] / x[:, 2], x[:, 1] / x[:, 2]
        f = out[:, 10].astype(np.int64)
        assert np.array_equal(out[f & 1 == 0, 0], ref0[f & 1 == 0]), scale_exp
        assert np.array_equal(out[f & 2 == 0, 1], ref1[f & 2 == 0]), scale_exp
        assert np.array_equal((f & 4) != 0, (f & 3) != 0)  # div2's suspect flag is the OR of the two
        assert np.array_equal(out[:, 2], ref0) and np.array_equal(out[:, 3], ref1), scale_exp  # div_rn
        flagged += int(np.count_nonzero(f & 3))
        total += 2 * x.shape[0]
    print(f"FAST quotients flagged: {flagged} of {total}")
    assert flagged <= total * 1e-6


def test_hardware_reciprocal_error(data_dir):
    """The FAST division's proof (exact_div.hpp) takes v_rcp_f64's relative
    error e0 <= 2^-23 as its premise (the ISA's 2^29 ulp; the argument holds
    up to 2^-20.1 for the shipped Newton form, 2^-22.3 Newton-free).  Measured here over
    every 20-bit leading significand pattern (random low bits) and 2 M random
    operands across the exponent range the decoders divide by."""
    ctx = ctx_for(data_dir, "PEG2304regular0.5.txt", "2bits_QPSK.txt", False)
    rng = np.random.default_rng(13)
    m = (np.arange(1 << 20, dtype=np.uint64) << np.uint64(32)) | rng.integers(0, 1 << 32, 1 << 20, dtype=np.uint64)
    sweep = ((np.uint64(1023) << np.uint64(52)) | m).view(np.float64)  # [1, 2), every 20-bit leading pattern
    rand = (rng.random(1 << 21) + 1.0) * 2.0 ** rng.integers(-962, 2, 1 << 21).astype(np.float64)
    worst = 0.0
    for s in (sweep, rand):
        x = np.stack([np.ones_like(s), np.ones_like(s), s], axis=1)
        e0 = ctx.div_probe(x)[:, 11]
        worst = max(worst, float(e0.max()))
    print(f"max |1 - s rcp(s)| = 2^{np.log2(worst):.2f}")
    assert worst <= 2.0 ** -23


def test_exact_division_any_operands(data_dir):
    """div_rn (exact_div.hpp: every division off the FAST path, the demapper's
    and k-means') equals x86 IEEE division bit for bit on any operands: every
    exponent incl. subnormal and overflowing quotients, signs, zeros,
    infinities and NaN (NaN equal to NaN)."""
    ctx = ctx_for(data_dir, "PEG2304regular0.5.txt", "2bits_QPSK.txt", False)
    rng = np.random.default_rng(11)
    n = 600000
    a = (rng.random(n) + 0.5) * 2.0 ** rng.integers(-1074, 1024, n).astype(np.float64)
    b = (rng.random(n) + 0.5) * 2.0 ** rng.integers(-1074, 1024, n).astype(np.float64)
    a *= np.where(rng.random(n) < 0.5, -1.0, 1.0)
    bits = rng.integers(0, 2 ** 63, n, dtype=np.int64)  # raw patterns: subnormals, NaNs, infinities
    a[::7] = bits[::7].view(np.float64)
    b[3::11] = bits[3::11][::-1].view(np.float64)
    special = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 5e-324, -5e-324, 2.2250738585072014e-308,
                        1.7976931348623157e308, 1.0, -1.0, 3.0])
    sa, sb = np.meshgrid(special, special)
    a = np.concatenate([a, sa.ravel()])
    b = np.concatenate([b, sb.ravel()])
    x = np.stack([a, a, b], axis=1)
    out = ctx.div_probe(x)
    with np.errstate(all="ignore"):
        ref = a / b
    bad = ~_same(out[:, 2], ref)
    assert not bad.any(), (a[bad][:4], b[bad][:4], out[bad, 2][:4], ref[bad][:4])


def _near_midpoint_significands(K, width):
    """Significands N in [2^52, 2^53) with (K N) mod 2^53 within width + 8 below
    / 8 above 2^52, and N near the ends of the binade: the only n for which
    n / s, s = 1 - K 2^-53, can be rounded wrongly by the CN division's last
    fma (tools/verify_cn_division.py derives and checks this exactly)."""
    two52, two53 = 2 ** 52, 2 ** 53
    out = set(range(two53 - 256, two53)) | set(range(two52, two52 + 256))
    t = 0
    while K % 2 == 0:
        K //= 2
        t += 1
    mod = two53 >> t
    inv = pow(K % mod, -1, mod)
    for B in range(two52 - width - 8, two52 + 9):
        if B % (1 << t) == 0:
            n0 = (inv * (B >> t)) % mod
            out.update(n for n in (n0 + i * mod for i in range(1 << t)) if two52 <= n < two53)
    return sorted(out)


def test_cn_reciprocal_exhaustive(data_dir):
    """The CN phases' near-one reciprocal (bp_common.hpp rcp_near1) is RN(1/s)
    on every double s with |s - 1| <= 2^-40 (1 + j 2^-52, j <= 2^12, and
    1 - k 2^-53, k <= 2^13).  hipcc's refined reciprocal is not (one ulp low on
    s = 1 - k 2^-53, k = 3, 5, ..., 13), and its '/' then misrounds a few n / s:
    on every near-midpoint candidate n the CN division equals IEEE division
    and '/' is reported; random normalisation-like pairs are checked too."""
    ctx = ctx_for(data_dir, "PEG2304regular0.5.txt", "2bits_QPSK.txt", False)
    j = np.arange(0, 2 ** 12 + 1, dtype=np.float64)
    k = np.arange(1, 2 ** 13 + 1, dtype=np.float64)
    s = np.concatenate([1.0 + j * 2.0 ** -52, 1.0 - k * 2.0 ** -53])
    assert s.size == 12289 and np.all(np.abs(s - 1.0) <= 2.0 ** -40)
    rng = np.random.default_rng(3)
    n0 = rng.random(s.size) * s
    x = np.stack([n0, s - n0, s], axis=1)
    out = ctx.div_probe(x)
    assert np.array_equal(out[:, 6], 1.0 / s)  # near-one formula == RN(1/s) for every s
    print(f"hipcc's refinement != RN(1/s) on {int(np.sum(out[:, 7] != 1.0 / s))} of {s.size} s")
    assert np.array_equal(out[:, 4], x[:, 0] / x[:, 2]) and np.array_equal(out[:, 5], x[:, 1] / x[:, 2])
    # near-midpoint candidates: s = 1 - K 2^-53 for K in [-32, 16] (K = -2j: s = 1 + j 2^-52)
    rows = []
    for K in [kk for kk in range(-32, 17) if kk and (kk > 0 or kk % 2 == 0)]:
        sv = 1.0 - K * 2.0 ** -53
        for N in _near_midpoint_significands(K, K * K):
            rows.append((N * 2.0 ** -53, sv))
    x = np.array([(n, 0.0, sv) for n, sv in rows])
    out = ctx.div_probe(x)
    ref = x[:, 0] / x[:, 2]
    assert np.array_equal(out[:, 4], ref)
    assert np.array_equal(out[:, 2], ref)  # div_rn
    f = out[:, 10].astype(np.int64)
    assert np.array_equal(out[f & 1 == 0, 0], ref[f & 1 == 0])  # the FAST VN form: proven, or flagged
    miss = int(np.sum(out[:, 8] != ref))
    print(f"near-midpoint candidates: {len(rows)}; hipcc '/' misrounds {miss}; "
          f"FAST VN form flags {int(np.count_nonzero(f & 1))}")
    assert miss > 0  # the finding that motivates exact_div.hpp (hipcc's '/' is not RN everywhere)
    # random normalisation-like pairs (products of normalised pairs), the CN
    # phases' operands (their sums are within 2^-49 of 1: bp_common.hpp rcp_cn_rows)
    n = 400000
    a = rng.random(n)
    b = rng.random(n)
    a0, a1 = a / (a + (1 - a)), (1 - a) / (a + (1 - a))
    b0, b1 = b / (b + (1 - b)), (1 - b) / (b + (1 - b))
    m0 = a0 * b0 + a1 * b1
    m1 = a0 * b1 + a1 * b0
    x = np.stack([m0, m1, m0 + m1], axis=1)
    assert np.all(np.abs(x[:, 2] - 1.0) <= 2.0 ** -49)
    out = ctx.div_probe(x)
    assert np.array_equal(out[:, 4], x[:, 0] / x[:, 2]) and np.array_equal(out[:, 5], x[:, 1] / x[:, 2])


@pytest.mark.parametrize("case", CASES)
def test_bp_golden_vectors(case, data_dir):
    """Decode the reference's own P0 vectors: every output bit-exact."""
    hdr, z = load_case(case)
    ctx = ctx_for(data_dir, hdr["matrix"], hdr["modem"], bool(hdr["is5g"]), hdr["max_iter"], bool(hdr["active"]))
    p0 = z["v_p0"]
    B = p0.shape[0]
    syn0 = np.full((B, ctx.M), -1.0)
    r = ctx.bp_decode(p0, cc_hat=True, syn=syn0)
    assert np.array_equal(r["ret"], z["s_ret"][:B])
    assert np.array_equal(r["uu_hat"], z["v_uu_hat"])
    assert np.array_equal(r["cc_hat"], z["v_cc_hat"])
    for i in range(B):
        if r["ret"][i] > 1:
            assert np.array_equal(r["syn"][i], z["v_syn"][i]), f"syndrom_soft cw {i}"


@pytest.mark.parametrize("matrix,modem,is5g,snr,max_iter,n", [
    ("PEG2304regular0.5.txt", "2bits_QPSK.txt", False, 2.0, 20, 300),
    ("PEG2304regular0.5.txt", "4bit_16QAM_Gray.txt", False, 4.0, 20, 200),
    ("5GLDPCBG2a3_R12_K960.txt", "4bit_16QAM_Gray.txt", True, 5.01, 50, 200),
    ("PEG8064regular0.5.txt", "6bits_64QAM_Gray.txt", False, 8.5, 20, 48),
    ("PEG8064regular0.5.txt", "2bits_QPSK.txt", False, 1.8, 20, 40),
    ("5GLDPCBG2a3_R12_K960.txt", "2bits_QPSK.txt", True, 1.5, 50, 100),
    ("5GLDPCBG2a3_R12_K960.txt", "6bits_64QAM_Gray.txt", True, 10.0, 50, 60),
])
def test_bp_vs_oracle_stream(data_dir, matrix, modem, is5g, snr, max_iter, n):
    """Oracle frames -> oracle P0 -> GPU BP vs oracle BP, bit-exact incl. the
    syndrome messages, plus a short iteration budget (the metric BP)."""
    ctx = ctx_for(data_dir, matrix, modem, is5g, max_iter)
    oc = oracle_for(data_dir, matrix, is5g, max_iter)
    om = O.Modem(os.path.join(data_dir, modem))
    uu, cc, th, y = O.gen_frames(oc, om, snr, n)
    var = 10.0 ** (-0.1 * snr)
    p0 = np.stack([om.demap(y[i], th[i], var) for i in range(n)])
    for it in (max_iter, 5, 1):
        r = ctx.bp_decode(p0, iter_count=it, cc_hat=True, syn=np.zeros((n, ctx.M)))
        for i in range(n):
            ret, uh, cch, syn = oc.bp_decode(p0[i], it)
            assert r["ret"][i] == ret, (it, i)
            assert np.array_equal(r["uu_hat"][i], uh), (it, i)
            assert np.array_equal(r["cc_hat"][i], cch), (it, i)
            assert np.array_equal(r["syn"][i], syn), (it, i)


@pytest.mark.parametrize("matrix,modem,is5g,snr,n", [
    ("PEG2304regular0.5.txt", "2bits_QPSK.txt", False, 2.0, 200),
    ("PEG2304regular0.5.txt", "2bits_4PSK.txt", False, 2.0, 100),
    ("PEG2304regular0.5.txt", "4bit_16QAM_Gray.txt", False, 5.0, 100),
    ("PEG8064regular0.5.txt", "6bits_64QAM_Gray.txt", False, 6.77, 40),
    ("PEG8064regular0.5.txt", "2bits_QPSK.txt", False, 2.0, 40),
    ("PEG8064regular0.5.txt", "4bit_16QAM_Gray.txt", False, 6.0, 40),
    ("5GLDPCBG2a3_R12_K960.txt", "6bits_64QAM_Gray.txt", True, 10.0, 100),
    ("5GLDPCBG2a3_R12_K960.txt", "2bits_QPSK.txt", True, 2.0, 100),
])
def test_demap_vs_oracle(data_dir, matrix, modem, is5g, snr, n):
    ctx = ctx_for(data_dir, matrix, modem, is5g)
    oc = oracle_for(data_dir, matrix, is5g)
    om = O.Modem(os.path.join(data_dir, modem))
    uu, cc, th, y = O.gen_frames(oc, om, snr, n)
    var = 10.0 ** (-0.1 * snr)
    ref = np.stack([om.demap(y[i], th[i], var) for i in range(n)])
    got = ctx.demap(y, th, var)
    d = ulp_diff(got.reshape(-1), ref.reshape(-1))
    print(f"demap: {np.mean(d != 0):.2e} of P0 differ, max {int(d.max())} ulp")
    assert np.array_equal(got, ref)


def _adversarial_symbols(pts, S, B, rng):
    """Received symbols that stress the demapper's fast-division ranges and the
    metric's single-precision screen: exactly on a point (distance 0), on the
    midpoint of two points and at 0 (P0 = 0.5 ties), tiny offsets, far outside
    the constellation (exp underflow), with unit, rotated, tiny and huge
    channels."""
    y = np.zeros((B, S, 2))
    th = np.zeros((B, 2))
    for b in range(B):
        h = [[1.0, 0.0], [0.0, 1.0], [0.6, -0.8], [1e-3, 2e-3], [40.0, 3.0]][b % 5] if b < 10 else rng.normal(size=2)
        th[b] = h
        hc = complex(h[0], h[1])
        kinds = rng.integers(0, 6, S)
        i1 = rng.integers(0, len(pts), S)
        i2 = rng.integers(0, len(pts), S)
        p1 = pts[i1, 0] + 1j * pts[i1, 1]
        p2 = pts[i2, 0] + 1j * pts[i2, 1]
        noise = rng.normal(size=S) + 1j * rng.normal(size=S)
        z = np.select([kinds == 0, kinds == 1, kinds == 2, kinds == 3, kinds == 4],
                      [p1 * hc, (p1 + p2) / 2 * hc, 0.0, p1 * hc + 1e-9 * noise, 30.0 * noise],
                      p1 * hc + 0.3 * noise)
        y[b, :, 0] = z.real
        y[b, :, 1] = z.imag
    return y, th


@pytest.mark.parametrize("matrix,modem,snr", [
    ("PEG2304regular0.5.txt", "2bits_QPSK.txt", 2.0),
    ("PEG2304regular0.5.txt", "4bit_16QAM_Gray.txt", 5.01),
    ("PEG8064regular0.5.txt", "6bits_64QAM_Gray.txt", 6.77),
    ("PEG8064regular0.5.txt", "6bits_64QAM_Gray.txt", 40.0),
])
def test_demap_and_metric_adversarial(data_dir, matrix, modem, snr):
    """Bit-exact P0 (fast shared-reciprocal divisions with IEEE fallback) and
    bit-exact hard metrics (single-precision screen with exact fallback) on
    adversarial symbols, against the oracle demapper + parity count."""
    ctx = ctx_for(data_dir, matrix, modem, False)
    oc = oracle_for(data_dir, matrix, False)
    om = O.Modem(os.path.join(data_dir, modem))
    pts = om.points.reshape(-1, 2)
    rng = np.random.default_rng(5)
    B = 20
    y, th = _adversarial_symbols(pts, ctx.S, B, rng)
    var = 10.0 ** (-0.1 * snr)
    ref = np.stack([om.demap(y[i], th[i], var) for i in range(B)])
    got = ctx.demap(y, th, var)
    assert np.array_equal(got, ref, equal_nan=True)
    out = ctx.decode_frames(y, snr, true_h=th, histogram=True)
    for i in range(B):
        rr = (ref[i] > 0.5).astype(np.uint8)
        assert out["metrics"][i][0] == abs(oc.parity_count(rr)), i
    # GetHistogramData with one caller estimate (kml_decode_candidates, nc = 1):
    # the same single-candidate metric, no final decode
    c1 = ctx.decode_candidates(y, th.reshape(B, 1, 2), snr, histogram=True)
    assert np.array_equal(c1["metrics"], out["metrics"]) and not c1["ret"].any()


@pytest.mark.parametrize("blind", [False, True])
def test_fused_demap_matches_separate(data_dir, blind, monkeypatch):
    """Known-channel and chosen-candidate QPSK decodes on the regular code run
    the demap in the BP kernel's prologue; KML_FUSED_DEMAP=0 runs the separate
    demap kernel: every output is identical (and the oracle agrees)."""
    ctx = ctx_for(data_dir, "PEG2304regular0.5.txt", "2bits_QPSK.txt", False)
    oc = oracle_for(data_dir, "PEG2304regular0.5.txt", False)
    om = O.Modem(os.path.join(data_dir, "2bits_QPSK.txt"))
    uu, cc, th, y = O.gen_frames(oc, om, 2.0, 96, state=23)
    r1 = ctx.decode_frames(y, 2.0, None if blind else th)
    monkeypatch.setenv("KML_FUSED_DEMAP", "0")
    r0 = ctx.decode_frames(y, 2.0, None if blind else th)
    for k in ("uu_hat", "chosen", "ret", "metrics"):
        assert np.array_equal(r1[k], r0[k]), k
    for i in range(0, 96, 8):
        ref = O.receive(oc, om, y[i], th[i], 2.0, blind)
        assert np.array_equal(r1["uu_hat"][i], ref["uu_hat"]) and r1["ret"][i] == ref["ret"], i


@pytest.mark.parametrize("matrix,modem,is5g,snr,n", [
    ("PEG2304regular0.5.txt", "2bits_QPSK.txt", False, 2.0, 1000),
    ("PEG2304regular0.5.txt", "2bits_QPSK.txt", False, -1.0, 500),
    ("PEG2304regular0.5.txt", "2bits_QPSK.txt", False, 8.0, 300),
    ("PEG2304regular0.5.txt", "2bits_4PSK.txt", False, 2.0, 200),
    ("PEG2304regular0.5.txt", "4bit_16QAM_Gray.txt", False, 5.01, 100),
    ("PEG2304regular0.5.txt", "4bit_16QAM_phi1.txt", False, 8.0, 50),
    ("PEG2304regular0.5.txt", "6bits_64QAM_Gray.txt", False, 10.5, 60),
    ("PEG8064regular0.5.txt", "6bits_64QAM_Gray.txt", False, 6.77, 30),
    # S = 4032: 63 of the 64 lane-words km_wave_kernel holds (kmeans.hip kMaxS)
    ("PEG8064regular0.5.txt", "2bits_QPSK.txt", False, 2.0, 60),
    ("PEG8064regular0.5.txt", "2bits_QPSK.txt", False, -2.0, 30),
    ("PEG8064regular0.5.txt", "4bit_16QAM_Gray.txt", False, 6.4, 40),
    # 5G BG2: S = 320 (64QAM, a partial fifth word), 480 (16QAM), 960 (QPSK)
    ("5GLDPCBG2a3_R12_K960.txt", "6bits_64QAM_Gray.txt", True, 11.0, 200),
    ("5GLDPCBG2a3_R12_K960.txt", "4bit_16QAM_phi1.txt", True, 11.0, 100),
    ("5GLDPCBG2a3_R12_K960.txt", "2bits_QPSK.txt", True, 2.0, 200),
])
@pytest.mark.parametrize("kernel", ["wave", "split"])
def test_kmeans_vs_oracle(data_dir, matrix, modem, is5g, snr, n, kernel, monkeypatch):
    monkeypatch.setenv("KML_KMEANS", kernel)
    ctx = ctx_for(data_dir, matrix, modem, is5g)
    oc = oracle_for(data_dir, matrix, is5g)
    om = O.Modem(os.path.join(data_dir, modem))
    uu, cc, th, y = O.gen_frames(oc, om, snr, n)
    hh, h4 = ctx.kmeans(y)
    for i in range(n):
        ref = O.kmeans_hhat(y[i], om.points)
        assert np.array_equal(hh[i], ref), i
        assert np.array_equal(h4[i], O.rotations(ref)), i


@pytest.mark.parametrize("modem", ["2bits_QPSK.txt", "4bit_16QAM_Gray.txt", "6bits_64QAM_Gray.txt"])
def test_kmeans_adversarial_ties(data_dir, modem):
    """Symbols exactly on constellation points, on midpoints between points
    (distance ties) and at zero, under exact and rotated channels: the
    squared-norm screening + exact-hypot tie band must reproduce the
    reference's first-minimum decisions bit for bit."""
    matrix = "PEG8064regular0.5.txt" if "64QAM" in modem else "PEG2304regular0.5.txt"
    ctx = ctx_for(data_dir, matrix, modem, False)
    om = O.Modem(os.path.join(data_dir, modem))
    pts = om.points.reshape(-1, 2)
    rng = np.random.default_rng(11)
    S = ctx.S
    B = 24
    y = np.zeros((B, S, 2))
    for b in range(B):
        h = [1.0, 0.0] if b % 3 == 0 else ([0.0, 1.0] if b % 3 == 1 else rng.normal(size=2))
        hc = complex(h[0], h[1])
        kinds = rng.integers(0, 4, S)
        i1 = rng.integers(0, len(pts), S)
        i2 = rng.integers(0, len(pts), S)
        p1 = pts[i1, 0] + 1j * pts[i1, 1]
        p2 = pts[i2, 0] + 1j * pts[i2, 1]
        z = np.where(kinds == 0, p1 * hc, np.where(kinds == 1, (p1 + p2) / 2 * hc,
                     np.where(kinds == 2, 0.0, p1 * hc + 1e-3 * (rng.normal(size=S) + 1j * rng.normal(size=S)))))
        y[b, :, 0] = z.real
        y[b, :, 1] = z.imag
    hh, h4 = ctx.kmeans(y)
    for b in range(B):
        ref = O.kmeans_hhat(y[b], om.points)
        assert np.array_equal(hh[b], ref, equal_nan=True), b


@pytest.mark.parametrize("mode", ["wave", "wave_sequential_sum", "wave_every_word", "split"])
@pytest.mark.parametrize("modem", ["2bits_QPSK.txt", "4bit_16QAM_Gray.txt", "6bits_64QAM_Gray.txt"])
def test_kmeans_cumulative_sum_adversarial(data_dir, modem, mode, monkeypatch):
    """The k-means kernels' cumulative cluster-0 sums (kmeans.hip
    ordered_sum_vals1: binade-segmented grid scans, tie
    parities, binade exits) and their incremental assignment against the
    oracle's sequential kmeans.cc:33-46, on inputs built to hit their corner
    cases: noise on a coarse dyadic grid (ties), a cluster-0 centre on an axis
    (sums that change sign), tiny and huge channels (extreme binades;
    thresholds past the float range; |h| ~ 1e-31, thresholds below FLT_MIN), NaN / inf symbols (the complex products'
    infinity recovery) and realistic frames; with the one-wave kernel
    (KML_KMEANS=wave: the members' values in LDS) with and without its scans
    and with every word re-assigned every iteration (KML_KM_INCR=0), and the
    two-launch form (KML_KMEANS=split, the path of S > 4096)."""
    monkeypatch.setenv("KML_KMEANS", mode.split("_")[0])
    monkeypatch.setenv("KML_KM_SCAN", "0" if mode.endswith("sequential_sum") else "1")
    monkeypatch.setenv("KML_KM_INCR", "0" if mode.endswith("every_word") else "1")
    matrix = "PEG8064regular0.5.txt" if "64QAM" in modem else "PEG2304regular0.5.txt"
    ctx = ctx_for(data_dir, matrix, modem, False)
    om = O.Modem(os.path.join(data_dir, modem))
    pts = om.points.reshape(-1, 2) @ [1, 1j]
    rng = np.random.default_rng(41)
    S, B = ctx.S, 24
    y = np.zeros((B, S, 2))
    for b in range(B):
        kind = b % 6
        # kind 5: |h| ~ 1e-31, drift thresholds below FLT_MIN (kmeans.hip: clamped to 0)
        hc = [1.0, 1j, 1e-200 * complex(*rng.normal(size=2)), 1e150 * complex(*rng.normal(size=2)),
              complex(*rng.normal(size=2)), 1e-31 * complex(*rng.normal(size=2))][kind]
        sym = pts[rng.integers(0, len(pts), S)]
        if kind == 0:  # dyadic noise: the grid sums hit exact ties
            noise = (rng.integers(-40, 40, S) + 1j * rng.integers(-40, 40, S)) * 2.0 ** -7
        else:
            noise = 0.3 * abs(hc) * (rng.normal(size=S) + 1j * rng.normal(size=S))
        zz = sym * hc + noise
        if b == 9:
            zz[rng.integers(0, S, 3)] = np.nan
        if b == 14:
            zz[rng.integers(0, S, 2)] = np.inf
        y[b, :, 0], y[b, :, 1] = zz.real, zz.imag
    hh, h4 = ctx.kmeans(y)
    for b in range(B):
        ref = O.kmeans_hhat(y[b], om.points)
        assert np.array_equal(hh[b], ref, equal_nan=True), b
    oc = oracle_for(data_dir, matrix, False)
    _, _, _, yr = O.gen_frames(oc, om, 6.77 if "64QAM" in modem else 2.0, 12, state=77)
    hh, _ = ctx.kmeans(yr)
    for b in range(yr.shape[0]):
        assert np.array_equal(hh[b], O.kmeans_hhat(yr[b], om.points)), b


@pytest.mark.parametrize("case", CASES)
def test_decode_frames_vs_reference_stream(case, data_dir):
    """KmCodec::Decoder on the reference's own frames (regenerated bit-exactly
    by the oracle, pinned by the y CRCs): chosen candidate, BP return value,
    decoded bits and error counts equal the reference's."""
    hdr, z = load_case(case)
    ctx = ctx_for(data_dir, hdr["matrix"], hdr["modem"], bool(hdr["is5g"]), hdr["max_iter"], bool(hdr["active"]))
    oc = oracle_for(data_dir, hdr["matrix"], bool(hdr["is5g"]), hdr["max_iter"], bool(hdr["active"]))
    om = O.Modem(os.path.join(data_dir, hdr["modem"]))
    n = hdr["ncw"]
    uu, cc, th, y = O.gen_frames(oc, om, hdr["snr"], n)
    assert all(crc(y[i]) == z["s_crc_y"][i] for i in range(n))
    r = ctx.decode_frames(y, hdr["snr"], None if not hdr["known"] else th)
    bad = [i for i in range(n) if crc(r["uu_hat"][i]) != z["s_crc_uuhat"][i]]
    assert not bad, f"{len(bad)}/{n} codewords differ: {bad[:10]}"
    assert np.array_equal(r["ret"], z["s_ret"][:n])
    if not hdr["known"]:
        assert np.array_equal(r["chosen"], z["s_chosen"][:n])
        assert np.array_equal(r["metrics"], z["s_metrics"][:n])
        assert np.array_equal(r["h_hat"], z["s_hhat"][:n])
    cnt = ctx.count_errors(uu.astype(np.uint8), r["uu_hat"])
    assert cnt["err_bit"] == int(z["s_errs"][:n].sum())
    assert cnt["err_blk"] == int((z["s_errs"][:n] > 0).sum())
    assert cnt["tot_blk"] == n


def test_reference_counters_2000(data_dir):
    """End-to-end SourceSink counters of the reference (2000 cw, seed 17),
    reproduced by the product alone: the reference's frame stream from
    kml_ref_frames (CLCRandNum state 17), the GPU receive path, CntErr."""
    ctr = json.load(open(os.path.join(GOLDEN, "counters.json")))
    for name, c in ctr.items():
        ctx = ctx_for(data_dir, c["matrix"], c["modem"], c["is5g"], c["max_iter"])
        uu, th, y = ctx.ref_frames(K.CLCRandNum(17), c["snr"], c["n"])
        r = ctx.decode_frames(y, c["snr"], th if c["known"] else None)
        cnt = ctx.count_errors(uu, r["uu_hat"])
        assert (cnt["err_blk"], cnt["err_bit"], cnt["tot_blk"]) == (c["err_blk"], c["err_bit"], c["tot_blk"]), name


def test_gpu_frames_are_codewords_and_channel_consistent(data_dir):
    """GPU frame generation: at very high SNR the known-H path decodes every
    codeword without error at iteration 0, and the frames are reproducible."""
    ctx = ctx_for(data_dir, "PEG2304regular0.5.txt", "2bits_QPSK.txt", False)
    ctx.sim_generate(60.0, 256, seed=3, first_cw=1000)
    c = ctx.sim_decode(60.0, blind=False)
    assert c["tot_blk"] == 256 and c["err_blk"] == 0 and c["converged"] == 256 and c["cn_phases"] == 0
    uu1, y1, h1 = ctx.sim_frames(256)
    ctx.sim_generate(60.0, 128, seed=3, first_cw=1128)  # a sub-range regenerates identical frames
    uu2, y2, h2 = ctx.sim_frames(128)
    assert np.array_equal(uu1[128:], uu2) and np.array_equal(y1[128:], y2) and np.array_equal(h1[128:], h2)
    # transmitted bits are codewords: hard-decode y/h at 60 dB and check
    x = (y1[:, :, 0] + 1j * y1[:, :, 1]) / (h1[:, 0] + 1j * h1[:, 1])[:, None]
    assert abs(np.mean(np.abs(x) ** 2) - 1.0) < 1e-3


CODES = [("PEG2304regular0.5.txt", "2bits_QPSK.txt", False, 20),   # bp_regular_kernel (LDS)
         ("5GLDPCBG2a3_R12_K960.txt", "4bit_16QAM_Gray.txt", True, 50),  # bp_irregular_kernel (LDS)
         ("PEG8064regular0.5.txt", "6bits_64QAM_Gray.txt", False, 20)]  # bp_part_kernel (partitioned LDS slots)
FAMILY = {"PEG2304regular0.5.txt": "bp_regular_kernel", "5GLDPCBG2a3_R12_K960.txt": "bp_irregular_kernel",
          "PEG8064regular0.5.txt": "bp_part_kernel"}


@pytest.mark.parametrize("matrix,modem,is5g,max_iter", CODES)
def test_dispatch_takes_the_specialised_kernel(data_dir, matrix, modem, is5g, max_iter):
    """Each code runs on its own kernel family (so the parity tests below cover
    all three), not on the generic fallback."""
    ctx = ctx_for(data_dir, matrix, modem, is5g, max_iter)
    ctx.bp_decode(np.full((2, ctx.cc_len), 0.3), iter_count=2)
    assert ctx.bp_kernel() == FAMILY[matrix]


@pytest.mark.parametrize("tagged", ["1", "0"])
def test_partitioned_kernel_tagged_exchange_and_deferral(data_dir, monkeypatch, tagged):
    """The partitioned kernel's tagged exchange (FAST codewords: direct mailbox
    stores, tag polling, per-iteration early-stop flags; groups of 4) and the
    barrier-exchange launch it defers the other codewords to: a PEG8064 batch
    with two codewords outside the fast-division domain (-0.0 / subnormal
    priors) among FAST ones, iteration budgets 20, 1 and 0, bit-exact against
    the oracle on ret, cc_hat and the soft syndromes; KML_PART_TAGGED=0
    (barrier exchange only) gives the same."""
    monkeypatch.setenv("KML_PART_TAGGED", tagged)
    ctx = K.Context(matrix_file=os.path.join(data_dir, "PEG8064regular0.5.txt"),
                    modem_file=os.path.join(data_dir, "6bits_64QAM_Gray.txt"), is5g=False, active=True,
                    max_iter=20, device=0)
    assert ctx.dims["part_group"] == 4
    oc = oracle_for(data_dir, "PEG8064regular0.5.txt", False, 20)
    rng = np.random.default_rng(33)
    B = 300
    p0 = np.clip(rng.normal(0.5, 0.28, (B, ctx.cc_len)), 0.02, 0.98)
    p0[7, ::5] = -0.0
    p0[23, 1::7] = 5e-320
    for it in (20, 1, 0):
        r = ctx.bp_decode(p0, iter_count=it, cc_hat=True, syn=np.zeros((B, ctx.M)))
        assert ctx.bp_kernel() == "bp_part_kernel"
        for i in list(range(0, B, 13)) + [7, 23, B - 1]:
            ret, uh, cch, syn = oc.bp_decode(p0[i], it)
            assert r["ret"][i] == ret, (it, i)
            assert np.array_equal(r["uu_hat"][i], uh), (it, i)  # it = 0: untouched (zeros) on both sides
            if it > 0:  # with no iteration the reference's cc_hat_ is whatever its array held: undefined
                assert np.array_equal(r["cc_hat"][i], cch), (it, i)
            assert np.array_equal(r["syn"][i], syn, equal_nan=True), (it, i)
        if it == 0:
            assert not r["cc_hat"].any()  # the caller's (zero) array, untouched
    ctx.close()


def test_partitioned_kernel_deferral_liveness(data_dir, monkeypatch):
    """Liveness of the partitioned kernel around deferred codewords: 150 rounds
    of the decodes above (FAST codewords beside two deferred ones, budgets 20, 1
    and 0, batches of 300, 1024 and 4096) never abort.  Before the not-FAST
    vote travelled through the group barrier's flag count, member 0 cleared a
    group word after a deferred codeword that a slower member might not have
    read yet; the members then took different paths and a group barrier timed
    out (tools/stress_part.py: the 42nd round)."""
    monkeypatch.setenv("KML_PART_TAGGED", "1")
    ctx = K.Context(matrix_file=os.path.join(data_dir, "PEG8064regular0.5.txt"),
                    modem_file=os.path.join(data_dir, "6bits_64QAM_Gray.txt"), is5g=False, active=True,
                    max_iter=20, device=0)
    assert ctx.dims["part_group"] == 4
    rng = np.random.default_rng(33)
    for r in range(150):
        B = (300, 1024, 4096)[r % 3]
        p0 = np.clip(rng.normal(0.5, 0.28, (B, ctx.cc_len)), 0.02, 0.98)
        p0[7, ::5] = -0.0
        p0[23, 1::7] = 5e-320
        for it in (20, 1, 0):
            ctx.bp_decode(p0, iter_count=it, cc_hat=True, syn=np.zeros((B, ctx.M)))
    ctx.close()


@pytest.mark.parametrize("matrix,modem,is5g,max_iter", CODES)
def test_empty_and_ragged_batches(data_dir, matrix, modem, is5g, max_iter):
    ctx = ctx_for(data_dir, matrix, modem, is5g, max_iter)
    r = ctx.bp_decode(np.zeros((0, ctx.cc_len)))
    assert r["uu_hat"].shape == (0, ctx.K)
    # odd batch sizes around the grid size
    rng = np.random.default_rng(9)
    oc = oracle_for(data_dir, matrix, is5g, max_iter)
    for B in (1, 3, 257, 513):
        p0 = rng.uniform(0.05, 0.95, (B, ctx.cc_len))
        r = ctx.bp_decode(p0, iter_count=3)
        for i in (0, B - 1):
            ret, uh, _, _ = oc.bp_decode(p0[i], 3)
            assert r["ret"][i] == ret and np.array_equal(r["uu_hat"][i], uh)


@pytest.mark.parametrize("matrix,modem,is5g,max_iter", CODES)
def test_extreme_inputs_match_oracle(data_dir, matrix, modem, is5g, max_iter):
    """Saturated / tie / NaN-free edge inputs: P0 at the clip bounds, exactly
    0.5 everywhere (every hard decision is a tie -> 1), 0/1 extremes, and -0.0
    and subnormal priors (outside the fast-division domain: the IEEE path)."""
    ctx = ctx_for(data_dir, matrix, modem, is5g, max_iter)
    oc = oracle_for(data_dir, matrix, is5g, max_iter)
    n = ctx.cc_len
    rng = np.random.default_rng(4)
    cases = [np.full(n, 0.5), np.full(n, 1e-12), np.full(n, 1 - 1e-12),
             np.where(rng.random(n) < 0.5, 1e-12, 1 - 1e-12), rng.choice([0.0, 1.0, 0.5], n),
             np.where(rng.random(n) < 0.3, -0.0, rng.uniform(0.2, 0.8, n)),
             np.where(rng.random(n) < 0.3, 5e-320, rng.uniform(0.2, 0.8, n))]
    p0 = np.stack(cases)
    r = ctx.bp_decode(p0, cc_hat=True, syn=np.zeros((len(cases), ctx.M)))
    for i in range(len(cases)):
        ret, uh, cch, syn = oc.bp_decode(p0[i])
        assert r["ret"][i] == ret, i
        assert np.array_equal(r["cc_hat"][i], cch), i
        assert np.array_equal(r["syn"][i], syn, equal_nan=True), i


@pytest.mark.parametrize("matrix,modem,is5g,max_iter", CODES)
def test_nan_and_inf_priors_match_oracle(data_dir, matrix, modem, is5g, max_iter):
    """NaN and +-inf priors (the IEEE path): the messages then carry NaNs, whose
    sign bits the decision-in-sign-bit parity (bp_regular / bp_irregular) must
    not confuse with a column's decision; the outputs equal the oracle's."""
    ctx = ctx_for(data_dir, matrix, modem, is5g, max_iter)
    oc = oracle_for(data_dir, matrix, is5g, max_iter)
    n = ctx.cc_len
    rng = np.random.default_rng(9)
    base = rng.uniform(0.05, 0.95, n)
    cases = [np.where(rng.random(n) < 0.01, np.nan, base), np.where(rng.random(n) < 0.01, -np.nan, base),
             np.where(rng.random(n) < 0.01, np.inf, base), np.where(rng.random(n) < 0.01, -np.inf, base)]
    p0 = np.stack(cases)
    r = ctx.bp_decode(p0, cc_hat=True, syn=np.zeros((len(cases), ctx.M)))
    for i in range(len(cases)):
        ret, uh, cch, syn = oc.bp_decode(p0[i])
        assert r["ret"][i] == ret, i
        assert np.array_equal(r["cc_hat"][i], cch), i
        assert np.array_equal(r["syn"][i], syn, equal_nan=True), i


# ---------------------------------------------------------------- soft metric
from conftest import load_soft_case, soft_case_names  # noqa: E402


def _soft_setup(case, data_dir):
    hdr, z = load_soft_case(case)
    code = O.Code(os.path.join(data_dir, hdr["matrix"]), bool(hdr["is5g"]), True, False, hdr["max_iter"])
    modem = O.Modem(os.path.join(data_dir, hdr["modem"]))
    n = len(z["chosen"])
    uu, cc, th, y = O.gen_frames(code, modem, hdr["snr"], n)
    for i in range(n):
        assert crc(y[i]) == z["crc_y"][i]
    uh = np.unpackbits(z["uu_hat_bits"], axis=1)[:, :hdr["K"]]
    return hdr, z, y, uh


def _soft_ctx(hdr, data_dir):
    return K.Context(matrix_file=os.path.join(data_dir, hdr["matrix"]), modem_file=os.path.join(data_dir, hdr["modem"]),
                     is5g=bool(hdr["is5g"]), max_iter=hdr["max_iter"], metric_soft=True,
                     metric_iter=hdr["metric_iter"], device=0)


@pytest.mark.parametrize("case", [c for c in soft_case_names() if not c.endswith("softhist")])
def test_soft_metric_decode_matches_reference_stream(case, data_dir):
    """KmCodec::Decoder with metric_type = true over the reference's stream: the
    chosen candidate, the metrics and uu_hat bit-exact, including the stale
    syndrom_soft reads, whether the stream is decoded in one batch or split
    across calls (the context carries the codec state like one instance)."""
    hdr, z, y, uh = _soft_setup(case, data_dir)
    n = len(z["chosen"])
    ctx = _soft_ctx(hdr, data_dir)
    out = ctx.decode_frames(y, hdr["snr"])
    assert np.array_equal(out["chosen"], z["chosen"])
    assert np.array_equal(out["uu_hat"], uh)
    ref = z["metrics"]
    assert np.allclose(out["metrics"], ref, rtol=0, atol=6e-15 * np.maximum(1, np.abs(ref)))
    ctx.close()
    ctx = _soft_ctx(hdr, data_dir)
    cut = n // 3 + 1
    o1 = ctx.decode_frames(y[:cut], hdr["snr"])
    o2 = ctx.decode_frames(y[cut:], hdr["snr"])
    assert np.array_equal(np.concatenate([o1["chosen"], o2["chosen"]]), z["chosen"])
    assert np.array_equal(np.concatenate([o1["uu_hat"], o2["uu_hat"]]), uh)
    assert np.array_equal(np.concatenate([o1["metrics"], o2["metrics"]]), out["metrics"])
    ctx.close()


def test_soft_metric_histogram_matches_reference(data_dir):
    """GetHistogramData with the soft metric (histogram mode, no final decode):
    metrics exact, uu_hat = what the last candidate's metric decode left."""
    hdr, z, y, uh = _soft_setup("peg2304_qpsk_softhist", data_dir)
    ctx = _soft_ctx(hdr, data_dir)
    out = ctx.decode_frames(y, hdr["snr"], histogram=True)
    assert np.array_equal(out["metrics"], z["metrics"])
    assert np.array_equal(out["chosen"], z["chosen"])
    assert np.array_equal(out["uu_hat"], uh)
    ctx.close()


KMSTATE = sorted(f[:-4] for f in os.listdir(os.path.join(os.path.dirname(__file__), "golden", "kmstate")))


@pytest.mark.gpu
@pytest.mark.parametrize("name", KMSTATE)
def test_kmeans_state_vs_reference(name, data_dir):
    """kml_kmeans_state = KMeans::clusters() and idx() after Run, on the
    reference's own frames and outputs (golden/kmstate, ref_harness), plus the
    oracle on fresh frames of the same configuration."""
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "kmstate", name + ".npz"))
    hdr = json.loads(bytes(z["hdr_json"]).decode())
    ctx = ctx_for(data_dir, hdr["matrix"], hdr["modem"], False)
    cl, idx = ctx.kmeans_state(z["y"], hdr["iters"])
    assert np.array_equal(cl, z["clusters"])
    assert np.array_equal(idx, z["idx"])
    oc = oracle_for(data_dir, hdr["matrix"], False)
    om = O.Modem(os.path.join(data_dir, hdr["modem"]))
    _, _, _, y = O.gen_frames(oc, om, hdr["snr"], 3 * hdr["n"], state=5)
    cl, idx = ctx.kmeans_state(y)
    for b in range(y.shape[0]):
        rc, ri = O.kmeans_state(y[b], om.points)
        assert np.array_equal(cl[b], rc) and np.array_equal(idx[b], ri), b


@pytest.mark.gpu
@pytest.mark.parametrize("modem", ["2bits_QPSK.txt", "4bit_16QAM_Gray.txt", "6bits_64QAM_Gray.txt"])
def test_kmeans_cluster0_majority(data_dir, modem):
    """Frames that put more than S/2 symbols into cluster 0, past the member
    list's capacity L.cap = S/3 (km_wave_kernel then sums cluster 0 straight
    from the membership words instead of its LDS value list): an all-zero codeword (every distance ties, the
    first minimum wins), every symbol on point 0 times h, and 60-95 % of the
    symbols near point 0 times h with the rest random.  h_hat, clusters and
    idx bit-exact against the oracle (kmeans.cc:15-84)."""
    matrix = "PEG8064regular0.5.txt" if "64QAM" in modem else "PEG2304regular0.5.txt"
    ctx = ctx_for(data_dir, matrix, modem, False)
    om = O.Modem(os.path.join(data_dir, modem))
    pts = om.points.reshape(-1, 2) @ [1, 1j]
    rng = np.random.default_rng(29)
    S, B = ctx.S, 10
    y = np.zeros((B, S, 2))
    for b in range(1, B):
        hc = complex(1.0, 0.0) if b % 3 == 1 else complex(*rng.normal(size=2))
        frac = 1.0 if b < 3 else 0.6 + 0.35 * rng.random()
        near = rng.random(S) < frac
        noise = (0.0 if b < 3 else 0.05) * (rng.normal(size=S) + 1j * rng.normal(size=S))
        zz = np.where(near, pts[0] * hc + noise, pts[rng.integers(0, len(pts), S)] * hc)
        y[b, :, 0], y[b, :, 1] = zz.real, zz.imag
    hh, h4 = ctx.kmeans(y)
    cl, idx = ctx.kmeans_state(y)
    for b in range(B):
        ref = O.kmeans_hhat(y[b], om.points)
        assert np.array_equal(hh[b], ref, equal_nan=True), b
        rc, ri = O.kmeans_state(y[b], om.points)
        assert np.array_equal(cl[b], rc, equal_nan=True), b
        assert np.array_equal(idx[b], ri), b
        if b < 3:
            assert (ri == 0).sum() > S // 2, b  # the case under test is reached


@pytest.mark.gpu
@pytest.mark.parametrize("modem", ["2bits_QPSK.txt", "4bit_16QAM_Gray.txt", "6bits_64QAM_Gray.txt"])
def test_kmeans_state_adversarial_ties(data_dir, modem):
    """Final assignment with exact distance ties (symbols on midpoints between
    clusters, at zero, on points): idx is the FIRST minimum (min_element)."""
    matrix = "PEG8064regular0.5.txt" if "64QAM" in modem else "PEG2304regular0.5.txt"
    ctx = ctx_for(data_dir, matrix, modem, False)
    om = O.Modem(os.path.join(data_dir, modem))
    pts = om.points.reshape(-1, 2)
    rng = np.random.default_rng(23)
    S, B = ctx.S, 12
    y = np.zeros((B, S, 2))
    for b in range(B):
        hc = complex(1.0, 0.0) if b % 2 == 0 else complex(*rng.normal(size=2))
        p1 = pts[rng.integers(0, len(pts), S)] @ [1, 1j]
        p2 = pts[rng.integers(0, len(pts), S)] @ [1, 1j]
        kinds = rng.integers(0, 4, S)
        zz = np.where(kinds == 0, p1 * hc, np.where(kinds == 1, (p1 + p2) / 2 * hc,
                      np.where(kinds == 2, 0.0, p1 * hc + 1e-3 * (rng.normal(size=S) + 1j * rng.normal(size=S)))))
        y[b, :, 0], y[b, :, 1] = zz.real, zz.imag
    cl, idx = ctx.kmeans_state(y)
    for b in range(B):
        rc, ri = O.kmeans_state(y[b], om.points)
        assert np.array_equal(cl[b], rc, equal_nan=True), b
        assert np.array_equal(idx[b], ri), b


@pytest.mark.gpu
@pytest.mark.parametrize("matrix,modem,is5g", [
    ("PEG2304regular0.5.txt", "2bits_QPSK.txt", False),
    ("5GLDPCBG2a3_R12_K960.txt", "4bit_16QAM_Gray.txt", True),
    ("PEG8064regular0.5.txt", "6bits_64QAM_Gray.txt", False),
])
def test_gpu_encoder_equals_host_encoder(data_dir, matrix, modem, is5g):
    """The GPU frame generator's encoder (framegen.hip) equals the host encoder
    (BinaryLDPCCodec::Encoder restated, kml_encode) bit for bit: at 60 dB the
    nearest constellation point of y / h gives back the transmitted label
    bits (MSB first, modem.cc:12-21), which must be encode(uu)."""
    ctx = ctx_for(data_dir, matrix, modem, is5g)
    B = 200
    ctx.sim_generate(60.0, B, seed=9, first_cw=77)
    uu, y, h = ctx.sim_frames(B)
    pts = ctx.constellation().reshape(-1, 2)
    pc = pts[:, 0] + 1j * pts[:, 1]
    x = (y[:, :, 0] + 1j * y[:, :, 1]) / (h[:, 0] + 1j * h[:, 1])[:, None]
    lab = np.abs(x[:, :, None] - pc[None, None, :]).argmin(axis=2)
    bits = ctx.bits
    cc_gpu = ((lab[:, :, None] >> np.arange(bits - 1, -1, -1)) & 1).reshape(B, -1).astype(np.uint8)
    cc_host = ctx.encode(uu)
    assert np.array_equal(cc_gpu, cc_host)


@pytest.mark.parametrize("blind", [False, True])
@pytest.mark.parametrize("matrix,modem,is5g", [("PEG2304regular0.5.txt", "2bits_QPSK.txt", False),
                                               ("5GLDPCBG2a3_R12_K960.txt", "4bit_16QAM_Gray.txt", True),
                                               ("PEG8064regular0.5.txt", "6bits_64QAM_Gray.txt", False)])
def test_host_buffer_chunked_decode_matches_one_piece(data_dir, matrix, modem, is5g, blind, monkeypatch):
    """kml_decode_frames with host buffers (known channel, or blind with the
    hard metric) uploads the frames in chunks on a copy stream while the
    previous chunk decodes (KML_HOST_CHUNK codewords per chunk): with small
    chunks and a ragged last chunk every output equals the one-piece call
    (KML_HOST_CHUNK=0), and sampled codewords equal the oracle."""
    ctx = ctx_for(data_dir, matrix, modem, is5g, max_iter=50 if is5g else 20)
    oc = oracle_for(data_dir, matrix, is5g, max_iter=50 if is5g else 20)
    om = O.Modem(os.path.join(data_dir, modem))
    B = 61
    uu, cc, th, y = O.gen_frames(oc, om, 5.0 if is5g else 2.0, B, state=31)
    snr = 5.0 if is5g else 2.0
    monkeypatch.setenv("KML_HOST_CHUNK", "0")
    r0 = ctx.decode_frames(y, snr, None if blind else th)
    monkeypatch.setenv("KML_HOST_CHUNK", "16")
    r1 = ctx.decode_frames(y, snr, None if blind else th)
    for k in ("uu_hat", "chosen", "ret", "metrics", "h_hat"):
        assert np.array_equal(r1[k], r0[k]), k
    for i in (0, 15, 16, 47, 48, 60):
        ref = O.receive(oc, om, y[i], th[i], snr, blind)
        assert np.array_equal(r1["uu_hat"][i], ref["uu_hat"]) and r1["ret"][i] == ref["ret"], i
        if blind:
            assert r1["chosen"][i] == ref["chosen"], i


@pytest.mark.parametrize("blind", [False, True])
def test_chunked_decode_reports_abort_of_an_early_chunk(data_dir, blind, monkeypatch):
    """A cooperative launch that aborts (as if a poll had timed out) in chunk 0
    of a chunked host-buffer call must fail the call: later chunks' launches
    must not clear the abort word before the call's single sync reads it
    (capi.cpp run_bp / sync).  The abort is injected after the first
    cooperative launch (kml_debug_inject_abort); the next call is clean."""
    matrix, modem = "PEG8064regular0.5.txt", "6bits_64QAM_Gray.txt"
    ctx = ctx_for(data_dir, matrix, modem, False)
    oc = oracle_for(data_dir, matrix, False)
    om = O.Modem(os.path.join(data_dir, modem))
    B = 40
    uu, cc, th, y = O.gen_frames(oc, om, 6.0, B, state=33)
    monkeypatch.setenv("KML_HOST_CHUNK", "16")  # 3 chunks
    r0 = ctx.decode_frames(y, 6.0, None if blind else th)
    ctx.debug_inject_abort(0)
    with pytest.raises(K.KmlError, match="aborted: raised by the host"):  # no poll timed out
        ctx.decode_frames(y, 6.0, None if blind else th)
    r1 = ctx.decode_frames(y, 6.0, None if blind else th)  # the abort was reported and cleared
    for k in ("uu_hat", "ret"):
        assert np.array_equal(r1[k], r0[k]), k


def test_error_return_after_coop_launch_leaves_next_call_clean(data_dir):
    """A call that fails after a cooperative launch but before its sync (any
    error return between them) must settle that launch's abort word: the
    next call starts clean instead of inheriting a timeout (capi.cpp fail(),
    coop_this_call).  Injected: the abort is raised after the launch and the
    call fails at once (kml_debug_inject_abort(-2))."""
    matrix, modem = "PEG8064regular0.5.txt", "6bits_64QAM_Gray.txt"
    ctx = ctx_for(data_dir, matrix, modem, False)
    oc = oracle_for(data_dir, matrix, False)
    om = O.Modem(os.path.join(data_dir, modem))
    B = 24
    uu, cc, th, y = O.gen_frames(oc, om, 6.0, B, state=35)
    r0 = ctx.decode_frames(y, 6.0, th)
    ctx.debug_inject_abort(-2)
    with pytest.raises(K.KmlError, match="injected failure"):
        ctx.decode_frames(y, 6.0, th)
    r1 = ctx.decode_frames(y, 6.0, th)
    for k in ("uu_hat", "ret"):
        assert np.array_equal(r1[k], r0[k]), k


def test_pending_abort_survives_a_later_argument_error(data_dir):
    """kml_sim_decode(sync=0) leaves its cooperative launch pending for
    kml_sync.  A later call that fails on its arguments, before any GPU work,
    must not settle (and drop) that launch's abort: kml_sync still reports it
    (capi.cpp call_begin / fail()).  Then the context is clean again."""
    ctx = ctx_for(data_dir, "PEG8064regular0.5.txt", "6bits_64QAM_Gray.txt", False)
    ctx.sim_generate(6.0, 64, seed=5)
    c0 = ctx.sim_decode(6.0, blind=False)
    ctx.debug_inject_abort(0)
    ctx.sim_decode(6.0, blind=False, sync=False)
    cnt = np.zeros(8, np.uint64)
    rc = K.lib().kml_sim_decode(ctx._h, 6.0, 0, K._p(cnt), 0)  # KML_E_ARG: counters need sync != 0
    assert rc == -1
    # the counter all-reduce's argument errors likewise (comm_allreduce
    # starts a call too): a null buffer, then no communicator on this context
    assert K.lib().kml_comm_allreduce_u64(ctx._h, None, 4) == -1
    assert K.lib().kml_comm_allreduce_f64(ctx._h, K._p(np.zeros(2)), 2) == -1
    with pytest.raises(K.KmlError, match="aborted: raised by the host"):
        ctx.sync()
    assert ctx.sim_decode(6.0, blind=False) == c0


# The exact path and the redo machinery (exact_div.hpp, DESIGN.md "Exact
# division"): KML_NO_FAST=1 decodes every codeword on the exact path (div_rn
# everywhere); KML_FORCE_REDO=1 treats every FAST decode as suspect, so each
# codeword is decoded on the FAST path, deferred at its first CN barrier and
# redone by the exact kernel (regular / irregular: the second launch; the
# partitioned kernel: tagged -> barrier-exchange FAST -> exact).  Both must
# reproduce the reference bit for bit, syndromes included.
EXACT_MODES = ["KML_NO_FAST", "KML_FORCE_REDO"]


@pytest.mark.parametrize("mode", EXACT_MODES)
@pytest.mark.parametrize("case", ["peg2304_qpsk_known", "bg2_16qam_known", "peg8064_64qam_known",
                                  "peg2304_4psk_known_lowsnr"])
def test_exact_path_golden_vectors(case, data_dir, mode, monkeypatch):
    hdr, z = load_case(case)
    monkeypatch.setenv(mode, "1")
    ctx = ctx_for(data_dir, hdr["matrix"], hdr["modem"], bool(hdr["is5g"]), hdr["max_iter"], bool(hdr["active"]))
    p0 = z["v_p0"]
    B = p0.shape[0]
    syn0 = np.full((B, ctx.M), -1.0)
    r = ctx.bp_decode(p0, cc_hat=True, syn=syn0)
    assert np.array_equal(r["ret"], z["s_ret"][:B])
    assert np.array_equal(r["uu_hat"], z["v_uu_hat"])
    assert np.array_equal(r["cc_hat"], z["v_cc_hat"])
    for i in range(B):
        if r["ret"][i] > 1:
            assert np.array_equal(r["syn"][i], z["v_syn"][i]), f"syndrom_soft cw {i}"
        else:  # no CN phase ran: the rows the caller passed in stay (the reference's member array)
            assert np.array_equal(r["syn"][i], syn0[i]), f"syndrom_soft cw {i} written without a CN phase"


@pytest.mark.parametrize("mode", EXACT_MODES)
@pytest.mark.parametrize("case", ["peg2304_qpsk_known", "peg2304_qpsk_blind", "bg2_16qam_blind", "peg8064_64qam_blind"])
def test_exact_path_reference_stream(case, data_dir, mode, monkeypatch):
    """KmCodec::Decoder on the reference's frames through the exact path and
    through forced redos (fused QPSK demap prologue included): chosen
    candidate, return values and decoded bits equal the reference's."""
    monkeypatch.setenv(mode, "1")
    test_decode_frames_vs_reference_stream(case, data_dir)


def test_forced_redo_counts_and_counters(data_dir, monkeypatch):
    """Every FAST decode of a forced-redo run is counted as redone (and once
    only), and the sim path's counters equal the normal run's."""
    ctx = ctx_for(data_dir, "PEG2304regular0.5.txt", "2bits_QPSK.txt", False)
    ctx.sim_generate(2.0, 1024, seed=5, first_cw=0)
    c0 = ctx.sim_decode(2.0, blind=False)
    # an unproven FAST quotient is settled in place (dd_fix; bp_regular reruns
    # the column settled), so no codeword is redone unless forced
    assert c0["redone"] == 0
    monkeypatch.setenv("KML_FORCE_REDO", "1")
    c1 = ctx.sim_decode(2.0, blind=False)
    assert c1["redone"] == 1024
    for k in ("err_bit", "err_blk", "tot_bit", "tot_blk", "vn_phases", "cn_phases", "converged"):
        assert c1[k] == c0[k], k


@pytest.mark.parametrize("modem", ["2bits_QPSK.txt", "4bit_16QAM_Gray.txt", "6bits_64QAM_Gray.txt"])
def test_candidate_metric_screen_equals_exact_demap(data_dir, modem, monkeypatch):
    """The candidate metric's single-precision screen (demap_common.hpp
    hard_bits_screen: v_exp_f32, fma ordering, fminf, the fmin <= 64 and
    2^20 gates) decides a hard bit only where the exact demapper agrees.  On
    frames built to sit at its edges — symbols on decision boundaries (midpoints
    of constellation points, tiny offsets), channels of |h| from 1e-3 to 1e4 —
    the metrics and chosen candidates with the screen on equal those with every
    symbol on the exact demapper (KML_CM_NOSCREEN=1)."""
    matrix = "PEG8064regular0.5.txt" if "64QAM" in modem else "PEG2304regular0.5.txt"
    ctx = ctx_for(data_dir, matrix, modem, False)
    om = O.Modem(os.path.join(data_dir, modem))
    pts = om.points.reshape(-1, 2) @ [1, 1j]
    rng = np.random.default_rng(57)
    S, B = ctx.S, 12
    y = np.zeros((B, S, 2))
    hh = np.zeros((B, 4, 2))
    for b in range(B):
        hc = complex(*rng.normal(size=2)) * [1e-3, 0.3, 1.0, 30.0, 1e4][b % 5]
        i1, i2 = rng.integers(0, len(pts), S), rng.integers(0, len(pts), S)
        mid = (pts[i1] + pts[i2]) / 2
        off = rng.choice([0.0, 1e-12, -1e-9, 1e-6, 3e-4], S) * (rng.normal(size=S) + 1j * rng.normal(size=S))
        zz = (np.where(rng.random(S) < 0.7, mid, pts[i1]) + off) * hc
        y[b, :, 0], y[b, :, 1] = zz.real, zz.imag
        h4 = O.rotations(np.array([hc.real, hc.imag]) * (1 + 1e-7 * rng.normal()))
        hh[b] = np.asarray(h4).reshape(4, 2)
    snr = 6.77 if "64QAM" in modem else 4.0
    r_on = ctx.decode_candidates(y, hh, snr)
    monkeypatch.setenv("KML_CM_NOSCREEN", "1")
    r_off = ctx.decode_candidates(y, hh, snr)
    assert np.array_equal(r_on["metrics"], r_off["metrics"])
    assert np.array_equal(r_on["chosen"], r_off["chosen"])
    assert np.array_equal(r_on["uu_hat"], r_off["uu_hat"])


@pytest.mark.parametrize("matrix,modem,is5g,snr,n", [
    ("PEG8064regular0.5.txt", "2bits_QPSK.txt", False, 2.2, 120),
    ("PEG8064regular0.5.txt", "4bit_16QAM_Gray.txt", False, 6.4, 60),
    ("PEG2304regular0.5.txt", "2bits_4PSK.txt", False, 2.0, 300),
    ("PEG2304regular0.5.txt", "6bits_64QAM_Gray.txt", False, 10.5, 200),
    ("5GLDPCBG2a3_R12_K960.txt", "6bits_64QAM_Gray.txt", True, 11.0, 200),
    ("5GLDPCBG2a3_R12_K960.txt", "2bits_QPSK.txt", True, 2.0, 200),
])
def test_cross_product_blind_streams_vs_oracle(data_dir, matrix, modem, is5g, snr, n):
    """The (code x constellation) pairs beyond the reference fixtures' 40-100
    codewords: fresh oracle streams (another seed) through the whole blind
    KmCodec::Decoder path — k-means with the threshold tiers and, for <= 4
    points, the segmented member list; the candidate metric; the rotated-point
    64QAM demapper — chosen candidate, h_hat, metrics, BP return value and
    uu_hat bit-exact against the oracle's receive()."""
    max_iter = 50 if is5g else 20
    ctx = ctx_for(data_dir, matrix, modem, is5g, max_iter)
    oc = oracle_for(data_dir, matrix, is5g, max_iter)
    om = O.Modem(os.path.join(data_dir, modem))
    uu, cc, th, y = O.gen_frames(oc, om, snr, n, state=61)
    r = ctx.decode_frames(y, snr, None)
    for i in range(n):
        ref = O.receive(oc, om, y[i], th[i], snr, True)
        assert r["chosen"][i] == ref["chosen"], i
        assert np.array_equal(r["h_hat"][i], ref["h_hat"]), i
        assert np.array_equal(r["metrics"][i], ref["metrics"]), i
        assert r["ret"][i] == ref["ret"], i
        assert np.array_equal(r["uu_hat"][i], ref["uu_hat"]), i
