"""CPU checks of two exactness arguments in demap_common.hpp (no GPU):

* the blind metric's single-precision screen (hard_bits_screen): replayed in
  numpy by tools/probe/screen_model.py, every bit it decides must equal the
  oracle demapper's hard decision (P0 > 0.5, kmcodec.cc:111-115);
* the LEAN FAST demapper sums the clipped terms without the prior weight
  w = 2^-MB: scaling by a power of two commutes with every rounding of the sum
  and of the quotients (modemlinearsystem.cc:240-246, modem.cc:58-70), so the
  probabilities are the same bits."""
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools", "probe"))


@pytest.mark.parametrize("modem", ["2bits_QPSK.txt", "4bit_16QAM_Gray.txt", "6bits_64QAM_Gray.txt"])
def test_metric_screen_never_contradicts_the_oracle(data_dir, modem):
    import screen_model as SM
    from oracle import oracle as O

    om = O.Modem(os.path.join(data_dir, modem))
    pts = om.points.reshape(-1, 2)
    MB = om.m
    rng = np.random.default_rng(3)
    decided = 0
    for snr in (0.0, 6.77, 25.0):
        var = 10.0 ** (-0.1 * snr)
        for trial in range(4):
            h = rng.normal(size=2) * (1.0 if trial < 3 else 20.0)
            idx = rng.integers(0, len(pts), 400)
            z = (pts[idx, 0] + 1j * pts[idx, 1]) * complex(h[0], h[1]) * (1j ** rng.integers(0, 4))
            z = z + np.sqrt(var / 2) * (rng.normal(size=z.size) + 1j * rng.normal(size=z.size))
            y = np.stack([z.real, z.imag], axis=1)
            p0 = om.demap(y, h, var).reshape(-1, MB)
            ref = np.zeros(y.shape[0], np.int64)
            for j in range(MB):
                ref |= (p0[:, j] > 0.5).astype(np.int64) << j
            bits, ok = SM.screen(pts, y, h, var)
            assert np.array_equal(bits[ok], ref[ok])
            decided += int(ok.sum())
    assert decided > 0.95 * 4800  # the screen decides nearly every symbol


@pytest.mark.parametrize("MB", [2, 4, 6])
def test_unweighted_sum_gives_the_same_quotients(MB):
    rng = np.random.default_rng(MB)
    w = 0.5 ** MB
    for _ in range(200):
        KC = 1 << MB
        # clipped terms in [1e-12, 1 - 1e-12], many at the clip floor like a real symbol
        c = np.exp(-rng.exponential(8.0, KC))
        c[rng.random(KC) < 0.5] = 1e-12
        c = np.clip(c, 1e-12, 1 - 1e-12)
        s_w = 0.0
        s_u = 0.0
        for k in range(KC):  # the reference's ascending order
            s_w = s_w + w * c[k]
            s_u = s_u + c[k]
        assert s_w == w * s_u
        assert np.array_equal((w * c) / s_w, c / s_u)
