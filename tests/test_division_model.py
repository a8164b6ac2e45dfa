"""Host model of the FAST division (kmldpc_amd/csrc/exact_div.hpp dd_rcp /
dd_quot / dd_check) in exact rational arithmetic.

The reference divides with x86 `divsd` (binaryldpccodec.cc:186-187, 207-208,
214-215); the GPU's FAST VN division must give RN(n / s) or flag the quotient.
Here v_rcp_f64 is modelled as 1/s with an adversarial relative error up to the
ISA's documented 2^-23 (the GPU test test_hardware_reciprocal_error measures the
device's), every fma / multiply rounds once (float(Fraction) is
round-to-nearest-even), and the properties the proof claims are asserted:
q is faithful, and an unflagged q equals RN(n / s).  Operands include
near-midpoint quotients built on purpose.
"""
import random
from fractions import Fraction as F

import pytest


def rn(x):
    return float(x)


def fma(a, b, c):
    return rn(F(a) * F(b) + F(c))


def mul(a, b):
    return rn(F(a) * F(b))


NEWTON = True  # the shipped form (exact_div.hpp KML_DD_NEWTON); False: the Newton-free form


def model(n, s, rel):
    y0 = rn(F(1) / F(s) * (1 + rel))  # v_rcp_f64 with relative error rel
    if NEWTON:
        hi = fma(y0, fma(-y0, s, 1.0), y0)
        lo = mul(fma(-hi, s, 1.0), hi)
        k = mul(hi, 1.0 + 2.0 ** -40)
    else:
        hi = y0
        e = fma(-y0, s, 1.0)
        lo = mul(y0, fma(e, e, e))
        k = fma(y0, 1.0 + 2.0 ** -40, lo)
    q = fma(n, hi, mul(n, lo))
    t = fma(fma(-q, s, n), k, q)
    return q, t == q


def neighbours(x):
    import math
    return math.nextafter(x, -math.inf), math.nextafter(x, math.inf)


def check(n, s, rel):
    global NEWTON
    q, proven = model(n, s, rel)
    NEWTON = not NEWTON  # both forms on every case
    q2, proven2 = model(n, s, rel)
    NEWTON = not NEWTON
    assert not proven2 or q2 == rn(F(n) / F(s))
    exact = F(n) / F(s)
    r = rn(exact)
    lo, hi = neighbours(r)
    # faithful: q is RN(n/s) or the other grid neighbour of n/s
    assert q in (r, lo, hi)
    if q != r:
        assert (F(q) - exact) * (F(r) - exact) < 0, "q is not a neighbour of n/s"
    if proven:
        assert q == r, (n.hex(), s.hex(), rel)
    return proven


@pytest.mark.parametrize("seed", range(4))
def test_fast_division_model_random(seed):
    rng = random.Random(seed)
    flagged = 0
    for _ in range(3000):
        s = rng.uniform(1e-12, 1.0) * 2.0 ** rng.randint(-40, 0)
        n = s * rng.uniform(0.0, 1.0)
        rel = rng.choice([-1, 1]) * rng.uniform(0, 2.0 ** -23)
        flagged += not check(n, s, rel)
    assert flagged < 5


def near_midpoint_cases(kmax=120):
    """s = 1 - k 2^-53 and a 54-bit odd midpoint significand J with J k within
    a few units of t 2^53 (t odd): n = RN(s m) makes n / s lie within ~2^-105
    of the midpoint m = J 2^-54 (the hardest inputs for any division tail)."""
    out = []
    for k in range(1, kmax):
        s = 1.0 - k * 2.0 ** -53
        for t in range(k | 1, 2 * k, 2):
            J0 = (t << 53) // k
            for J in range(J0 - 3, J0 + 4):
                if J % 2 == 0 or not (1 << 53) <= J < (1 << 54):
                    continue
                n = rn(F(s) * F(J, 1 << 54))
                out.append((n, s))
    return out


def test_fast_division_model_near_midpoints():
    """Quotients within ~2^-105 of a rounding midpoint: the proof must flag
    them or they must be exact; never an unflagged misrounding."""
    cases = near_midpoint_cases()
    assert len(cases) > 1000
    flagged = 0
    for n, s in cases:
        for rel in (2.0 ** -23, -(2.0 ** -23), 0.0, 2.0 ** -30):
            for scale in (1.0, 2.0 ** -300):
                flagged += not check(n * scale, s, rel)
    # the check's window is 2^-39: flagged (and settled by dd_fix), never wrong
    assert flagged > 0


def test_fast_division_model_saturated_case():
    """The recurring BP case DESIGN.md cites: n0 = 1/4 + 3 ulp, s = 1/2 - 2^-55."""
    s = 0.5 - 2.0 ** -55
    n = 0.25 + 3 * 2.0 ** -54
    for rel in (2.0 ** -23, -(2.0 ** -23), 1e-9, 0.0):
        check(n, s, rel)
