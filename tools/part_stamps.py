"""Phase timing of the partitioned cooperative BP kernel (bp_coop.hip,
bp_part_kernel) from its s_memtime stamps.  Needs the stamps build:

    make stamps
    KML_LIB=kmldpc_amd/libkmldpc_amd_stamps.so python tools/part_stamps.py

Decodes one known-H batch of PEG8064/64QAM frames and prints, per phase of an
iteration, wave 0's average cycles (mean over workgroups)."""
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

# the tagged exchange (default) stamps: 0 loop top, 2 VN compute, 4 v2c poll,
# 5 previous flags poll + sync, 6 parity + CN compute, 7 flag post (last wave), 8 c2v poll + sync
TAGGED_NAMES = ["iteration boundary", "-", "VN compute (wave 0)", "-", "poll v2c (wave 0)",
                "prev. flags poll + sync", "CN compute + parity (wave 0)", "flag post", "c2v poll + sync", "-"]
NAMES = ["iteration boundary", "receive c2v (+sync)", "VN compute (wave 0)", "VN drain (sync)",
         "send v2c + group barrier", "receive v2c + decisions (+sync)", "parity + CN compute (wave 0)",
         "CN drain (sync)", "send c2v + group barrier (+flags)", "-"]


def main():
    d = tempfile.mkdtemp(prefix="kml_st_")
    src = os.path.join(REPO, "tests", "golden", "data")
    for fn in ("PEG8064regular0.5.txt.gz", "6bits_64QAM_Gray.txt.gz"):
        with gzip.open(os.path.join(src, fn), "rb") as g, open(os.path.join(d, fn[:-3]), "wb") as f:
            f.write(g.read())
    ctx = K.Context(matrix_file=os.path.join(d, "PEG8064regular0.5.txt"),
                    modem_file=os.path.join(d, "6bits_64QAM_Gray.txt"), max_iter=20, device=0)
    B = int(os.environ.get("B", "4096"))
    ctx.sim_generate(6.77, B, seed=3)
    L = K.lib()
    fn = L.kml_debug_part_stamps
    fn.argtypes = [C.c_void_p, C.c_int]
    buf = np.zeros(256 * 10, np.uint64)
    ctx.sim_decode(6.77)  # warm-up
    fn(buf.ctypes.data, 1)
    c = ctx.sim_decode(6.77)
    fn(buf.ctypes.data, 0)
    print("kernel:", ctx.bp_kernel())
    st = buf.reshape(256, 10).astype(np.float64)
    groups = 64
    iters_per_group = float(c["vn_phases"]) / groups
    per_iter = st.mean(axis=0) / iters_per_group
    tot = per_iter[:9].sum()
    print(f"codewords {B}, mean VN phases {c['vn_phases'] / B:.2f}, iterations per group {iters_per_group:.0f}")
    names = NAMES if os.environ.get("KML_PART_TAGGED", "1") == "0" else TAGGED_NAMES
    for i in range(9):
        print(f"  {names[i]:36s} {per_iter[i]:9.0f} cycles  {100 * per_iter[i] / tot:5.1f}%")
    print(f"  {'total per iteration':36s} {tot:9.0f} cycles")
    # per member (workgroup w is member (w >> 3) % 4): a member that computes
    # longer makes the others wait at the exchange
    member = (np.arange(256) >> 3) % 4
    for m in range(4):
        row = st[member == m].mean(axis=0) / iters_per_group
        print(f"  member {m}: " + " ".join(f"{row[i]:6.0f}" for i in range(9)))
    spread = st[:, 4] / iters_per_group
    print(f"  barrier-1 per-WG spread: min {spread.min():.0f} max {spread.max():.0f}")


if __name__ == "__main__":
    main()
