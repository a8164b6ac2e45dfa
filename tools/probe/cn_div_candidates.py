"""GPU check of the near-midpoint candidates of tools/verify_cn_division.py:
hipcc's '/', the FAST division (hipcc's refinement) and the CN near-one
division against numpy's IEEE division."""
import gzip, os, sys, tempfile
from fractions import Fraction as F
import numpy as np
R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "tools"))
import kmldpc_amd as K
import verify_cn_division as V
G = os.path.join(R, "tests", "golden", "data")
D = tempfile.mkdtemp()
for fn in ("PEG2304regular0.5.txt.gz", "2bits_QPSK.txt.gz"):
    open(os.path.join(D, fn[:-3]), "wb").write(gzip.open(os.path.join(G, fn)).read())
ctx = K.Context(matrix_file=os.path.join(D, "PEG2304regular0.5.txt"), modem_file=os.path.join(D, "2bits_QPSK.txt"))
rows = []
for k in list(range(1, 65)) + [-j for j in range(1, 65)]:
    s = 1.0 - k * 2.0 ** -53 if k > 0 else 1.0 + (-k) * 2.0 ** -52
    mult = k if k > 0 else 1
    for N in V.candidates(abs(mult), mult * mult):
        for sc in (2.0 ** -53, 2.0 ** -60, 2.0 ** -200):
            rows.append((N * sc, s))
x = np.array([(n, 0.0, s) for n, s in rows])
out = ctx.div_probe(x)
ref = x[:, 0] / x[:, 2]
for name, col in (("hipcc '/'", 2), ("FAST (refine)", 0), ("CN near-one", 4)):
    bad = np.where(out[:, col] != ref)[0]
    print(f"{name}: {bad.size} of {len(rows)} differ from IEEE")
    for i in bad[:6]:
        print(f"   n={x[i,0].hex()} s={x[i,2].hex()} got={out[i,col].hex()} ieee={ref[i].hex()}")
