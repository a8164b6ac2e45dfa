"""Phase timing of the k-means kernel (kmeans.hip, km_wave_kernel) from
its s_memtime stamps.  Needs the stamps build:

    make stamps
    KML_LIB=kmldpc_amd/libkmldpc_amd_stamps.so python tools/km_stamps.py

Runs the blind PEG2304/QPSK k-means on one batch of GPU frames and prints
thread 0's cycles per codeword and per iteration for each phase, and the
incremental-assignment counters."""
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

NAMES = ["prologue (load + first max)", "clusters + convergence", "assignment", "compaction", "sum", "update + barrier"]
SLOT = [0, 1, 2, 3, 4, 9]


def main():
    matrix = os.environ.get("MATRIX", "PEG2304regular0.5.txt")
    modem = os.environ.get("MODEM", "2bits_QPSK.txt")
    snr = float(os.environ.get("SNR", "2.0"))
    d = tempfile.mkdtemp(prefix="kml_st_")
    src = os.path.join(REPO, "tests", "golden", "data")
    for fn in (matrix + ".gz", modem + ".gz"):
        with gzip.open(os.path.join(src, fn), "rb") as g, open(os.path.join(d, fn[:-3]), "wb") as f:
            f.write(g.read())
    ctx = K.Context(matrix_file=os.path.join(d, matrix), modem_file=os.path.join(d, modem), max_iter=20, device=0)
    B = int(os.environ.get("B", "32768"))
    ctx.sim_generate(snr, B, seed=3)
    fn = K.lib().kml_debug_km_stamps
    fn.argtypes = [C.c_void_p, C.c_int]
    buf = np.zeros(16, np.uint64)
    ctx.sim_decode(snr, blind=True)  # warm-up
    fn(buf.ctypes.data, 1)
    ctx.sim_decode(snr, blind=True)
    fn(buf.ctypes.data, 0)
    st = buf.astype(np.float64)
    ncw, iters, words, comp = st[8], st[5], st[6], st[7]
    sw = (ctx.S + 63) // 64
    print(f"{matrix} + {modem}, snr {snr}: {int(ncw)} codewords, {iters / ncw:.2f} iterations per codeword")
    print(f"  words assigned per iteration {words / iters:.2f} of {sw}; compactions per iteration {comp / iters:.3f}")
    tot = st[SLOT].sum() / ncw
    for n, i in zip(NAMES, SLOT):
        print(f"  {n:30s} {st[i] / ncw:9.0f} cycles/cw  {st[i] / max(iters, 1):7.0f} /iter  {100 * st[i] / ncw / tot:5.1f}%")
    print(f"  {'total':30s} {tot:9.0f} cycles/cw")
    print(f"  wave-sum steps per iteration (real chain) {st[10] / max(iters, 1):.2f}")
    print(f"  gathered weak-symbol passes per iteration {st[11] / max(iters, 1):.2f} (KML_KM_WEAK)")


if __name__ == "__main__":
    main()
