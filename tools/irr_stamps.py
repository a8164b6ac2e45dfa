"""Per-wave phase timing of bp_irregular_kernel (5G BG2) from its s_memtime
stamps.  Needs the stamps build:

    make stamps
    KML_LIB=kmldpc_amd/libkmldpc_amd_stamps.so python tools/irr_stamps.py

Decodes the BG2 bench workload (K960 + 16QAM, Es/N0 5.01 dB, 50 iterations,
known H) once and prints, for each of the 12 waves, its cycles per iteration
in each phase: the VN phase ends at the slowest wave's VN work, the CN phase
at the slowest wave's CN work, so the per-wave spread is the cost of the plan."""
import argparse
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
os.environ.setdefault("KML_LIB", os.path.join(REPO, "kmldpc_amd", "libkmldpc_amd_stamps.so"))
import bench  # noqa: E402
import kmldpc_amd as K  # noqa: E402

NAMES = ["VN pair", "VN single", "VN barrier", "parity", "CN pair", "CN single", "CN barrier"]


def main():
    args = argparse.Namespace(snr=5.01, batch=int(os.environ.get("B", "16384")), blind=False, is5g=True,
                              max_iter=int(os.environ.get("ITERS", "50")),
                              matrix="5GLDPCBG2a3_R12_K960.txt", modem="4bit_16QAM_Gray.txt")
    d = bench.data_dir()
    ctx = K.Context(bench.write_config(d, args), data_dir=d, device=0)
    ctx.sim_generate(args.snr, args.batch, seed=1)
    fn = K.lib().kml_debug_irr_stamps
    fn.argtypes = [C.c_void_p, C.c_int]
    buf = np.zeros((12, 8), np.uint64)
    ctx.sim_decode(args.snr)  # warm-up
    fn(buf.ctypes.data, 1)
    ctx.sim_decode(args.snr)
    fn(buf.ctypes.data, 0)
    print("kernel:", ctx.bp_kernel())
    st = buf.astype(np.float64)
    its = st[0, 7]
    per = st[:, :7] / its
    print(f"iterations run {its:.0f} ({its / args.batch:.2f} per codeword); cycles per iteration, per wave:")
    print("  wave " + " ".join(f"{n:>10s}" for n in NAMES) + "      total")
    for w in range(12):
        print(f"  {w:4d} " + " ".join(f"{x:10.0f}" for x in per[w]) + f" {per[w].sum():10.0f}")
    vn = per[:, 0] + per[:, 1]
    cn = per[:, 4] + per[:, 5]
    print(f"  VN work: max {vn.max():.0f} mean {vn.mean():.0f}; CN work (+parity): max {(cn + per[:, 3]).max():.0f} "
          f"mean {(cn + per[:, 3]).mean():.0f}; iteration {per[0].sum():.0f}")
    for s in range(4):
        ws = [w for w in range(12) if w % 4 == s]
        print(f"  SIMD {s} (waves {ws}): VN sum {vn[ws].sum():.0f}, CN sum {cn[ws].sum():.0f}")


if __name__ == "__main__":
    main()
