"""Exact check of the CN phases' division n / s for sums s near 1.

The CN kernels form q = fma(fma(-s, m, n), r, m), m = RN(n * r), with r the
near-one reciprocal rcp_near1(s) = RN(1/s) (bp_common.hpp).  On the GPU,
rcp_near1 equals hipcc's refined reciprocal for every s with |s - 1| <= 2^-40
except s = 1 - k 2^-53, k in {3, 5, ..., 13} (tests/test_gpu_parity.py
test_cn_reciprocal_exhaustive measures it), where hipcc's is one ulp lower.

The result depends only on the significand N of n (n = N 2^a; no under- or
overflow in the FAST domain).  q - Q = (Q - m)(s r - 1) is below 2^-51 ulp(Q),
so q can differ from RN(Q) only when Q lies within 2^-51 ulp of a rounding
midpoint.  For s = 1 - k 2^-53, Q / 2^a = N + k N 2^-53 + k^2 N 2^-106 + ...,
so that happens only for the N whose k N mod 2^53 lies within k^2 + 8 of 2^52,
or for N within 256 of either end of the binade (Q may leave n's binade).
The s > 1 side, s = 1 + j 2^-52, is the same with k = -2j.  This script
enumerates all of those N for every k, j <= 64 and evaluates the sequence
exactly in rational arithmetic (each fma one rounding), for both
reciprocals: the near-one one must round to RN(Q) on every candidate (hipcc's
refinement does not on three).  CPU only; exits non-zero when the near-one
reciprocal misses.
"""
from fractions import Fraction as F
import sys

TWO52, TWO53 = 2 ** 52, 2 ** 53


def rn(x):
    return F(float(x))  # CPython: Fraction -> float is correctly rounded


def tail(n, s, r):
    """m = RN(n r); f = fma(-s, m, n); q = fma(f, r, m), each fma one rounding."""
    m = rn(n * r)
    f = rn(n - s * m)
    return rn(m + f * r)


def candidates(K, width):
    """Significands N in [2^52, 2^53) with (K N) mod 2^53 in
    [2^52 - width - 8, 2^52 + 8] (K may be even or negative), plus the N near
    either end of the binade (Q may leave the binade of n)."""
    out = set(range(TWO53 - 256, TWO53)) | set(range(TWO52, TWO52 + 256))
    t = 0
    while K % 2 == 0:
        K //= 2
        t += 1
    mod = TWO53 >> t
    inv = pow(K % mod, -1, mod)
    for B in range(TWO52 - width - 8, TWO52 + 9):
        if B % (1 << t):
            continue
        n0 = (inv * (B >> t)) % mod
        for i in range(1 << t):
            N = n0 + i * mod
            if TWO52 <= N < TWO53:
                out.add(N)
    return out


def main():
    bad = 0
    checked = 0
    cases = [(F(1) - F(k, TWO53), k) for k in range(1, 65)] + [(F(1) + F(j, TWO52), -j) for j in range(1, 65)]
    for s, k in cases:
        r_rn = rn(1 / s)
        rs = [r_rn]
        if 3 <= k <= 13 and k % 2:
            rs.append(r_rn - F(1, TWO52))  # hipcc's refinement on these s
        K = k if k > 0 else -2 * (-k)  # s = 1 - K 2^-53
        for N in sorted(candidates(K, K * K)):
            n = F(N, TWO52)
            want = rn(n / s)
            for i, r in enumerate(rs):
                got = tail(n, s, r)
                checked += 1
                if got != want:
                    which = "near-one" if i == 0 else "hipcc refinement"
                    bad += i == 0
                    print(f"{which} misses: s = 1{'-' if k > 0 else '+'}{abs(k)} ulp, N = {N}, r = {float(r).hex()}")
    print(f"checked {checked} (s, N, r) cases; near-one reciprocal misses: {bad}")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
