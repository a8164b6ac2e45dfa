"""Where does the near-one reciprocal formula differ from hipcc's refinement?"""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import kmldpc_amd as K
import gzip, tempfile
G = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests", "golden", "data")
D = tempfile.mkdtemp()
for fn in ("PEG2304regular0.5.txt.gz", "2bits_QPSK.txt.gz"):
    open(os.path.join(D, fn[:-3]), "wb").write(gzip.open(os.path.join(G, fn)).read())
ctx = K.Context(matrix_file=os.path.join(D, "PEG2304regular0.5.txt"), modem_file=os.path.join(D, "2bits_QPSK.txt"))
j = np.arange(0, 2 ** 12 + 1, dtype=np.float64)
k = np.arange(1, 2 ** 13 + 1, dtype=np.float64)
s = np.concatenate([1.0 + j * 2.0 ** -52, 1.0 - k * 2.0 ** -53])
x = np.stack([s * 0.3, s * 0.7, s], axis=1)
out = ctx.div_probe(x)
rn = 1.0 / s
bad = out[:, 6] != out[:, 7]
print("mismatch", bad.sum(), "near==RN", np.sum(out[:, 6] == rn), "refine==RN", np.sum(out[:, 7] == rn), "of", s.size)
idx = np.where(bad)[0]
for i in idx[:20]:
    print(f"s=1{'+' if s[i]>=1 else '-'}{abs(s[i]-1)/2**-53:.0f}*2^-53 near={out[i,6].hex()} refine={out[i,7].hex()} RN={rn[i].hex()}")
