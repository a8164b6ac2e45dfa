"""FAST-division diagnostics (GPU): run one bench workload through a
KML_DIV_STATS=1 build and report how often the VN divisions' reciprocal premise
(|e1| <= 2^-46) and per-quotient checks fail, the largest |e1| seen, and the
first failing operands with their distance to the rounding midpoint (exact
rational arithmetic).

    make variant V=divstats VFLAGS="-DKML_DIV_STATS=1"
    KML_LIB=kmldpc_amd/libkmldpc_amd_divstats.so python tools/div_stats.py [bench workload args]
"""
import argparse
import ctypes as C
import json
import os
import struct
import sys
from fractions import Fraction

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import kmldpc_amd as K  # noqa: E402


def as_f(u):
    return struct.unpack("<d", struct.pack("<Q", u))[0]


def midpoint_gap(n, s, q):
    """(n/s - q) / half-gap towards n/s, exactly (1.0 = at the midpoint)."""
    import math
    if not all(math.isfinite(v) for v in (n, s, q)) or s == 0:
        return None
    x = Fraction(n) / Fraction(s)
    fq = Fraction(q)
    import math
    nb = math.nextafter(q, math.inf if x > fq else -math.inf)
    half = abs(Fraction(nb) - fq) / 2
    return float((x - fq) / half) if half else float("nan")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--matrix", default="PEG2304regular0.5.txt")
    ap.add_argument("--modem", default="2bits_QPSK.txt")
    ap.add_argument("--snr", type=float, default=2.0)
    ap.add_argument("--is5g", action="store_true")
    ap.add_argument("--blind", action="store_true")
    ap.add_argument("--max-iter", type=int, default=20)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--out")
    a = ap.parse_args()
    bargs = bench.argparse.Namespace(matrix=a.matrix, modem=a.modem, snr=a.snr, is5g=a.is5g, max_iter=a.max_iter,
                                     blind=a.blind, batch=a.batch, seed=1)
    d = bench.data_dir()
    cfg = bench.write_config(d, bargs)
    ctx = K.Context(cfg, data_dir=d, device=0)
    L = K.lib()
    names = [n for n in ("kml_debug_div_stats_reg", "kml_debug_div_stats_irr", "kml_debug_div_stats_coop")
             if hasattr(L, n)]
    buf = (C.c_ulonglong * (8 + 5 * 64))()
    for n in names:
        getattr(L, n)(buf, 1)
    ctx.sim_generate(a.snr, a.batch, seed=1, first_cw=0)
    cnt = ctx.sim_decode(a.snr, blind=a.blind)
    out = {"workload": vars(a), "counters": cnt, "kernel": ctx.bp_kernel(), "tu": {}}
    for n in names:
        getattr(L, n)(buf, 0)
        v = list(buf)
        if v[0] == 0:
            continue
        samples = []
        for i in range(min(64, v[5])):
            n0, n1, s, q0, q1 = (as_f(x) for x in v[8 + 5 * i: 13 + 5 * i])
            ok0 = s != 0 and q0 == n0 / s
            ok1 = s != 0 and q1 == n1 / s
            samples.append({"n0": n0.hex(), "n1": n1.hex(), "s": s.hex(), "q0_ok": ok0, "q1_ok": ok1,
                            "g0": midpoint_gap(n0, s, q0), "g1": midpoint_gap(n1, s, q1)})
        out["tu"][n] = {"pairs": v[0], "rcp_premise_failed": v[1], "q0_unproven": v[2], "q1_unproven": v[3],
                        "max_abs_e1": as_f(v[4]), "failures": v[5], "samples": samples[:16]}
    ctx.close()
    s = json.dumps(out, indent=1)
    print(s)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
