"""CPU model of the k-means incremental assignment's word flagging
(kmeans.hip km_wave_kernel), TEST/ANALYSIS INFRASTRUCTURE ONLY.

Runs the reference's k-means (kmeans.cc:15-84: cumulative cluster-0 sums,
re-projection from cluster 0) on oracle frames and counts, per iteration, how
many 64-symbol words the drift rule re-assigns whole:
  * K = 0 (round 5): a word is re-assigned when the accumulated drift D reaches
    the smallest threshold D_ref + g / (2 Cmax) of its symbols (g: the margin
    between the symbol's distances to cluster 0 and to the nearest other
    cluster);
  * K > 0 (KML_KM_WEAK, kKmWeak = 3): the K smallest thresholds are the word's
    weak symbols, re-assigned on their own (gathered) when D reaches their
    minimum, and the word is re-assigned whole only when D reaches the minimum
    of the others.
Exact margins here (the kernel uses conservative lower bounds), so the counts
are a model, not the kernel's.

    python tools/probe/km_weak_model.py [n_codewords] [snr]
"""
import gzip
import os
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
from oracle import oracle as O  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    snr = float(sys.argv[2]) if len(sys.argv) > 2 else 2.0
    d = tempfile.mkdtemp(prefix="kml_kmw_")
    for fn in ("PEG2304regular0.5.txt", "2bits_QPSK.txt"):
        with gzip.open(os.path.join(REPO, "tests", "golden", "data", fn + ".gz")) as g, open(os.path.join(d, fn), "wb") as f:
            f.write(g.read())
    oc = O.Code(os.path.join(d, "PEG2304regular0.5.txt"), False, True, False, 20)
    om = O.Modem(os.path.join(d, "2bits_QPSK.txt"))
    pts = om.points.reshape(-1, 2) @ [1, 1j]
    _, _, _, y = O.gen_frames(oc, om, snr, n)
    cmax = np.abs(pts).max()
    for K in (0, 1, 2, 3, 4, 8):
        tot = dict(full=0, weakw=0, weaks=0, iters=0, maxs=0)
        for b in range(n):
            z = y[b, :, 0] + 1j * y[b, :, 1]
            S = len(z)
            Sw = (S + 63) // 64
            hat = z[np.argmax(np.abs(z))] / pts[0]
            prev = None
            s0, c0, D, hprev = 0, 0, 0.0, hat
            t1, t2 = np.zeros(Sw), np.zeros(Sw)
            weak = [np.zeros(0, int)] * Sw
            for it in range(20):
                cl = pts * hat
                if prev is not None and np.array_equal(cl, prev):
                    break
                D += abs(hat - hprev)
                dist = np.abs(cl[None, :] - z[:, None])
                m = np.argmin(dist, axis=1) == 0
                g = np.abs(dist[:, 0] - dist[:, 1:].min(axis=1))
                nw = 0
                for w in range(Sw):
                    sl = np.arange(w * 64, min(S, w * 64 + 64))
                    thr = D + g[sl] / (2 * cmax)
                    if it == 0 or not (D < t2[w]):
                        tot["full"] += 1
                        o = np.argsort(thr, kind="stable")
                        weak[w] = sl[o[:K]]
                        t1[w] = thr[o[0]]
                        t2[w] = thr[o[K]] if K < len(sl) else np.inf
                    elif K and not (D < t1[w]):
                        tot["weakw"] += 1
                        tot["weaks"] += len(weak[w])
                        nw += len(weak[w])
                        t1[w] = (D + g[weak[w]] / (2 * cmax)).min()
                tot["iters"] += 1
                tot["maxs"] = max(tot["maxs"], nw)
                prev, hprev = cl, hat
                s0 += z[m].sum()
                c0 += m.sum()
                hat = (s0 / c0) / pts[0]
        it = tot["iters"]
        print(f"K={K}: whole words per iteration {tot['full'] / it:.2f} of {Sw}, weak-flagged words {tot['weakw'] / it:.2f}, "
              f"weak symbols {tot['weaks'] / it:.2f} (max {tot['maxs']} in one iteration)")


if __name__ == "__main__":
    main()
