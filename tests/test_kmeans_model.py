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
