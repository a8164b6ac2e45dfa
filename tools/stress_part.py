"""Liveness stress of the partitioned cooperative kernel (bp_part_kernel):
repeats tests/test_gpu_parity.py::test_partitioned_kernel_tagged_exchange_and_
deferral's decodes (PEG8064, groups of 4, FAST codewords among two deferred
ones, iteration budgets 20, 1 and 0) with fresh priors, and stops at the first
abort, printing the site the library reports (group barrier / v2c / c2v mailbox
poll / early-stop flag poll) and the workgroup.

    python tools/stress_part.py [rounds] [tagged (1) | barrier exchange only (0)]
"""
import gzip
import os
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import kmldpc_amd as K  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    tagged = sys.argv[2] if len(sys.argv) > 2 else "1"
    d = tempfile.mkdtemp(prefix="kml_stress_")
    src = os.path.join(REPO, "tests", "golden", "data")
    for fn in ("PEG8064regular0.5.txt.gz", "6bits_64QAM_Gray.txt.gz"):
        with gzip.open(os.path.join(src, fn), "rb") as g, open(os.path.join(d, fn[:-3]), "wb") as f:
            f.write(g.read())
    os.environ["KML_PART_TAGGED"] = tagged
    ctx = K.Context(matrix_file=os.path.join(d, "PEG8064regular0.5.txt"),
                    modem_file=os.path.join(d, "6bits_64QAM_Gray.txt"), max_iter=20, device=0)
    assert ctx.dims["part_group"] == 4
    rng = np.random.default_rng(33)
    t0 = time.time()
    n = 0
    for r in range(rounds):
        B = (300, 1024, 4096)[r % 3]
        p0 = np.clip(rng.normal(0.5, 0.28, (B, ctx.cc_len)), 0.02, 0.98)
        p0[7, ::5] = -0.0
        p0[23, 1::7] = 5e-320
        for it in (20, 1, 0):
            try:
                ctx.bp_decode(p0, iter_count=it, cc_hat=True, syn=np.zeros((B, ctx.M)))
            except K.KmlError as e:
                print(f"ABORT round {r} B {B} iter_count {it}: {e}", flush=True)
                return 1
            n += 1
        if r % 20 == 0:
            print(f"round {r}: {n} decodes, {time.time() - t0:.1f} s", flush=True)
    print(f"no abort in {n} decodes ({time.time() - t0:.1f} s)")
    return 0


if __name__ == "__main__":
    sys.exit(main())
