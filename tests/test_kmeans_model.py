"""CPU checks of the algorithms behind the k-means kernel's shortcuts
(kmeans.hip): the binade-segmented scan that replaces the sequential
cluster-0 sum must equal the left-to-right fp64 sum bit for bit, including
signed zeros, ties, binade and sign changes, huge/tiny/non-finite values."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools", "probe"))

import km_scan_model as M  # noqa: E402


def test_wave_scan_sum_equals_sequential_sum():
    for seed in (1, 2):
        cases, st = M.check(seed=seed, trials=600)
        assert cases == 600 and st["exits"] > 0 and st["seq"] > 0


def test_segment_fillers_are_the_sum_identity():
    """kmeans.hip KML_KM_SEG: the member list holds -0.0 fillers between the
    words' members; x + (-0.0) == x for every double x (signed zeros,
    infinities, NaN payloads), so both the sequential sum and the wave scan
    over the filled list equal the sum over the members alone, bit for bit."""
    import math
    import random
    import struct

    def bits(v):
        return struct.pack("<d", v)

    rnd = random.Random(7)
    specials = [0.0, -0.0, math.inf, -math.inf, float("nan"), 5e-324, -5e-324, 1e308, -1e308]
    for x in specials + [rnd.uniform(-1, 1) * 2.0 ** rnd.randint(-1074, 1023) for _ in range(2000)]:
        assert bits(x + -0.0) == bits(x), x
    for trial in range(300):
        n = rnd.randint(1, 400)
        members = [rnd.gauss(0.0, 1.0) * 2.0 ** rnd.randint(-30, 30) for _ in range(n)]
        if trial % 10 == 0:
            members[rnd.randrange(n)] = rnd.choice(specials)
        # words of up to 16 members, each followed by one or two fillers
        filled, i = [], 0
        while i < n:
            k = rnd.randint(0, 16)
            filled += members[i:i + k] + [-0.0] * rnd.randint(1, 2)
            i += k
        acc0 = rnd.choice([0.0, rnd.gauss(0.0, 1e3)])
        ref = M.seq_sum(acc0, members)
        assert bits(M.seq_sum(acc0, filled)) == bits(ref) or (math.isnan(ref) and math.isnan(M.seq_sum(acc0, filled)))
        got = M.wave_sum(acc0, filled, {"exits": 0, "seq": 0, "steps": 0, "ties": 0})
        assert bits(got) == bits(ref) or (math.isnan(ref) and math.isnan(got)), trial
