"""CPU model of the k-means member-list rebuilds (kmeans.hip km_wave_kernel),
ANALYSIS INFRASTRUCTURE ONLY.  On the reference's k-means trajectories
(kmeans.cc:15-84) for PEG2304 / QPSK frames it counts, per iteration, the
64-symbol words whose member values are reloaded into the LDS list:
  * compacted list (KML_KM_SEG=0): every word whose members or list offset
    changed (a count change shifts every later word);
  * per-word segments (KML_KM_SEG=1) of capacity members + slack: only the
    changed words, plus a full relayout when a word outgrows its segment;
and the scanned list length (members + fillers).

    python tools/probe/km_seg_model.py
"""
import gzip
import os
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
from oracle import oracle as O  # noqa: E402

d = tempfile.mkdtemp(prefix="kml_kmseg_")
for fn in ("PEG2304regular0.5.txt", "2bits_QPSK.txt"):
    with gzip.open(os.path.join(REPO, "tests", "golden", "data", fn + ".gz")) as g, open(os.path.join(d, fn), "wb") as f:
        f.write(g.read())
oc = O.Code(os.path.join(d, 'PEG2304regular0.5.txt'), False, True, False, 20)
om = O.Modem(os.path.join(d, '2bits_QPSK.txt'))
pts = om.points.reshape(-1, 2) @ [1, 1j]
n = 150
uu, cc, th, y = O.gen_frames(oc, om, 2.0, n)
for slack in (0, 1, 2, 4, 6, 8):
    tot = dict(full=0, wordw=0, iters=0, chgit=0, cur_words=0, elems=0, members=0)
    for b in range(n):
        z = y[b, :, 0] + 1j * y[b, :, 1]
        S = len(z); Sw = (S + 63) // 64
        hat = z[np.argmax(np.abs(z))] / pts[0]
        prev = None; s0 = 0; c0 = 0
        cap = None; bits_prev = None
        for it in range(20):
            cl = pts * hat
            if prev is not None and np.array_equal(cl, prev): break
            dist = np.abs(cl[None, :] - z[:, None])
            m = np.argmin(dist, axis=1) == 0
            words = [m[w*64:(w+1)*64] for w in range(Sw)]
            cnt = np.array([w.sum() for w in words])
            tot['iters'] += 1
            if bits_prev is None or any(not np.array_equal(a, b2) for a, b2 in zip(words, bits_prev)):
                tot['chgit'] += 1
                # current scheme: words whose bits or offset changed
                excl = np.concatenate([[0], np.cumsum(cnt)[:-1]])
                if bits_prev is None:
                    tot['cur_words'] += Sw
                else:
                    excl_p = np.concatenate([[0], np.cumsum([w.sum() for w in bits_prev])[:-1]])
                    tot['cur_words'] += sum(1 for w in range(Sw) if not np.array_equal(words[w], bits_prev[w]) or excl[w] != excl_p[w])
                # segment scheme
                if cap is None or np.any(cnt > cap):
                    tot['full'] += 1
                    cap = cnt + slack
                else:
                    tot['wordw'] += sum(1 for w in range(Sw) if not np.array_equal(words[w], bits_prev[w]))
            tot['elems'] += cap.sum(); tot['members'] += cnt.sum()
            bits_prev = words
            prev = cl
            s0 += z[m].sum(); c0 += m.sum()
            hat = (s0 / c0) / pts[0]
    it = tot['iters']
    print(f"slack {slack}: iterations with changes {tot['chgit']/it:.3f}; current words reloaded/iter {tot['cur_words']/it:.2f}; "
          f"segment: full rebuilds/iter {tot['full']/it:.3f}, word rewrites/iter {tot['wordw']/it:.2f}, scan elems {tot['elems']/it:.0f} vs members {tot['members']/it:.0f}")
