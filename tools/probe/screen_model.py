"""CPU model of demap_common.hpp hard_bits_screen (the blind metric's
single-precision screen): the same steps in numpy float32 / float64, checked
against the oracle demapper's hard decisions (P0 > 0.5).  A decided bit that
disagrees with the oracle is a screen bug; undecided symbols go to the exact
demapper on the GPU and are only counted here.
Run: python tools/probe/screen_model.py [modem] [n_symbols]"""
import gzip
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402

LOG2E = 1.4426950408889634


def screen(pts, y, h, var):
    """bits [S] (bit j of the label set: P0_j > 0.5), ok [S]."""
    KC = pts.shape[0]
    MB = KC.bit_length() - 1
    cr, ci = pts[:, 0], pts[:, 1]
    yr, yi = y[:, 0:1], y[:, 1:2]
    hr, hi = h
    iv = (1.0 / var) * LOG2E
    ok = np.ones(y.shape[0], bool)
    if MB >= 4:
        A = (hr * hr + hi * hi) * iv
        Br = (hr * yr + hi * yi) * iv
        Bi = (hi * yr - hr * yi) * iv
        Y = (yr * yr + yi * yi) * iv
        cb = max(np.max(cr * cr + ci * ci), 2 * max(np.max(np.abs(cr)), np.max(np.abs(ci)))) * (1 + 2.0 ** -40)
        ok &= (cb * (A + np.abs(Br) + np.abs(Bi)) + Y <= 2.0 ** 20)[:, 0]
        s0, s1, s2 = cr * cr + ci * ci, 2 * cr, 2 * ci
        d = s0 * A + (-s1 * Br + (s2 * Bi + Y))  # fma order; double rounding differences are < 2^-30 here
    else:
        sr = cr * hr - ci * hi - yr
        si = cr * hi + ci * hr - yi
        d = (sr * sr + si * si) * iv
    f = d.astype(np.float32)
    fmin = np.min(f, axis=1)
    ok &= fmin <= np.float32(64)
    with np.errstate(over="ignore", invalid="ignore"):
        e = np.exp2((fmin[:, None] - f).astype(np.float32)).astype(np.float32)
    bits = np.zeros(y.shape[0], np.int64)
    g = np.float32(1 + 2.0 ** -12)
    lab = np.arange(KC)
    tot = np.zeros(y.shape[0], np.float32)
    q0 = np.zeros((y.shape[0], MB), np.float32)
    q1 = np.zeros((y.shape[0], MB), np.float32)
    for k in range(KC):  # sequential float sums, the kernel's order
        tot = (tot + e[:, k]).astype(np.float32)
        for j in range(MB):
            if ((lab[k] >> (MB - 1 - j)) & 1) == 0:
                q0[:, j] = (q0[:, j] + e[:, k]).astype(np.float32)
            elif MB < 4:
                q1[:, j] = (q1[:, j] + e[:, k]).astype(np.float32)
    if MB >= 4:
        q1 = (tot[:, None] - q0).astype(np.float32)
    for j in range(MB):
        one = q0[:, j] > q1[:, j] * g
        zero = q1[:, j] > q0[:, j] * g
        ok &= one | zero
        bits |= one.astype(np.int64) << j
    return bits, ok


def main():
    modem = sys.argv[1] if len(sys.argv) > 1 else "6bits_64QAM_Gray.txt"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, modem)
        with gzip.open(os.path.join(ROOT, "tests", "golden", "data", modem + ".gz"), "rb") as gz:
            open(p, "wb").write(gz.read())
        om = O.Modem(p)
    pts = om.points.reshape(-1, 2)
    MB = om.m
    rng = np.random.default_rng(11)
    bad = und = tot = 0
    for snr in (0.0, 2.0, 6.77, 12.0, 25.0):
        var = 10.0 ** (-0.1 * snr)
        for trial in range(8):
            h = rng.normal(size=2) * (1.0 if trial < 6 else 30.0 ** (trial - 6.5))
            hc = complex(h[0], h[1])
            idx = rng.integers(0, len(pts), n // 40)
            z = (pts[idx, 0] + 1j * pts[idx, 1]) * hc
            # the blind candidates: the channel rotated by k * 90 degrees
            z = z * (1j ** rng.integers(0, 4))
            z = z + np.sqrt(var / 2) * (rng.normal(size=z.size) + 1j * rng.normal(size=z.size))
            y = np.stack([z.real, z.imag], axis=1)
            p0 = om.demap(y, h, var).reshape(-1, MB)
            ref = np.zeros(y.shape[0], np.int64)
            for j in range(MB):
                ref |= (p0[:, j] > 0.5).astype(np.int64) << j
            bits, ok = screen(pts, y, h, var)
            bad += int(np.sum(ok & (bits != ref)))
            und += int(np.sum(~ok))
            tot += y.shape[0]
    print(f"{modem}: {tot} symbols, {und} undecided ({und / tot:.2%}), {bad} wrong decisions")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
