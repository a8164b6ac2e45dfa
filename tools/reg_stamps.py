"""Phase timing of bp_regular_kernel (the headline BP kernel) from its
s_memtime stamps.  Needs the stamps build:

    make stamps
    KML_LIB=kmldpc_amd/libkmldpc_amd_stamps.so python tools/reg_stamps.py

Decodes the headline workload (PEG2304 + QPSK, Es/N0 2 dB, known H, fused
demap) once and prints thread 0's cycles per codeword for each phase."""
import ctypes as C
import gzip
import os
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
os.environ.setdefault("KML_LIB", os.path.join(REPO, "kmldpc_amd", "libkmldpc_amd_stamps.so"))
import kmldpc_amd as K  # noqa: E402

NAMES = ["queue + barriers", "demap / P0", "InitMsg + barrier", "iterations", "epilogue + barrier", "result atomics"]


def main():
    d = tempfile.mkdtemp(prefix="kml_st_")
    src = os.path.join(REPO, "tests", "golden", "data")
    for fn in ("PEG2304regular0.5.txt.gz", "2bits_QPSK.txt.gz"):
        with gzip.open(os.path.join(src, fn), "rb") as g, open(os.path.join(d, fn[:-3]), "wb") as f:
            f.write(g.read())
    ctx = K.Context(matrix_file=os.path.join(d, "PEG2304regular0.5.txt"), modem_file=os.path.join(d, "2bits_QPSK.txt"),
                    max_iter=int(os.environ.get("ITERS", "20")), device=0)
    B = int(os.environ.get("B", "32768"))
    ctx.sim_generate(2.0, B, seed=3)
    fn = K.lib().kml_debug_reg_stamps
    fn.argtypes = [C.c_void_p, C.c_int]
    buf = np.zeros(8 + 64, np.uint64)
    ctx.sim_decode(2.0)  # warm-up
    fn(buf.ctypes.data, 1)
    ctx.sim_decode(2.0)
    fn(buf.ctypes.data, 0)
    st = buf[:8].astype(np.float64)
    ws = buf[8:].reshape(16, 4).astype(np.float64)
    ncw, its = st[6], st[7]
    print(f"bp_regular_kernel: {int(ncw)} codewords, {its / ncw:.2f} CN phases per codeword")
    tot = st[:6].sum() / ncw
    for i, n in enumerate(NAMES):
        print(f"  {n:24s} {st[i] / ncw:9.0f} cycles/cw  {100 * st[i] / ncw / tot:5.1f}%")
    print(f"  {'total':24s} {tot:9.0f} cycles/cw; iterations {st[3] / max(its, 1):.0f} cycles per CN phase")
    print("  per wave, cycles per CN phase: VN compute, VN barrier, CN compute, CN barrier")
    for w in range(12):
        print(f"    wave {w:2d}: " + " ".join(f"{x / max(its, 1):7.0f}" for x in ws[w]))


if __name__ == "__main__":
    main()
