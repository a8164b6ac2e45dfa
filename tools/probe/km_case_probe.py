"""GPU probe (diagnostics): h_hat of the fused k-means on the adversarial
frames of tests/test_gpu_parity.py::test_kmeans_word_scan_adversarial (QPSK),
printed beside the oracle's, for the library KML_LIB names."""
import gzip
import os
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import kmldpc_amd as K  # noqa: E402
from oracle import oracle as O  # noqa: E402

d = tempfile.mkdtemp()
for fn in ("PEG2304regular0.5.txt", "2bits_QPSK.txt"):
    open(os.path.join(d, fn), "wb").write(gzip.open(os.path.join(REPO, "tests/golden/data", fn + ".gz")).read())
ctx = K.Context(matrix_file=os.path.join(d, "PEG2304regular0.5.txt"), modem_file=os.path.join(d, "2bits_QPSK.txt"),
                device=0)
om = O.Modem(os.path.join(d, "2bits_QPSK.txt"))
pts = om.points.reshape(-1, 2) @ [1, 1j]
rng = np.random.default_rng(41)
S, B = ctx.S, 20
y = np.zeros((B, S, 2))
for b in range(B):
    kind = b % 5
    hc = [1.0, 1j, 1e-200 * complex(*rng.normal(size=2)), 1e150 * complex(*rng.normal(size=2)),
          complex(*rng.normal(size=2))][kind]
    sym = pts[rng.integers(0, len(pts), S)]
    if kind == 0:
        noise = (rng.integers(-40, 40, S) + 1j * rng.integers(-40, 40, S)) * 2.0 ** -7
    else:
        noise = 0.3 * abs(hc) * (rng.normal(size=S) + 1j * rng.normal(size=S))
    zz = sym * hc + noise
    if b == 9:
        zz[rng.integers(0, S, 3)] = np.nan
    if b == 14:
        zz[rng.integers(0, S, 2)] = np.inf
    y[b, :, 0], y[b, :, 1] = zz.real, zz.imag
for it in (1, 2, 3, 5, 20):
    hh, _ = ctx.kmeans(y[[9, 14]], iters=it)
    print("iters", it, "gpu", hh.tolist(), "ref", [O.kmeans_hhat(y[b], om.points, it).tolist() for b in (9, 14)])
hh, _ = ctx.kmeans(y)
bad = [b for b in range(B) if not np.array_equal(hh[b], O.kmeans_hhat(y[b], om.points), equal_nan=True)]
print("lib", os.environ.get("KML_LIB", "default"), "mismatching codewords", bad)
