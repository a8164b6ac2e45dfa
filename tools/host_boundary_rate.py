"""PCIe-inclusive throughput of the C-ABI boundary with HOST buffers: the
reference-side integration hands kml_decode_frames host arrays (y, true_h in,
uu_hat out), so every call moves the frames over PCIe.  bench.py's `value` is
the HBM-resident rate; this is the number a host-driven caller sees.

    python tools/host_boundary_rate.py [--batch 32768] [--reps 5]
"""
import argparse
import gzip
import json
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import kmldpc_amd as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32768)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--snr", type=float, default=2.0)
    ap.add_argument("--blind", action="store_true", help="blind path (k-means + 4-candidate metric): y only")
    args = ap.parse_args()
    d = tempfile.mkdtemp()
    for fn in ["PEG2304regular0.5.txt", "2bits_QPSK.txt"]:
        with gzip.open(os.path.join(REPO, "tests", "golden", "data", fn + ".gz")) as g, open(os.path.join(d, fn), "wb") as f:
            f.write(g.read())
    ctx = K.Context(matrix_file=os.path.join(d, "PEG2304regular0.5.txt"), modem_file=os.path.join(d, "2bits_QPSK.txt"),
                    max_iter=20, device=0)
    B = args.batch
    ctx.sim_generate(args.snr, B, seed=5)
    uu, y, h = ctx.sim_frames(B)  # host copies of GPU-generated frames
    th = None if args.blind else h
    ctx.decode_frames(y, args.snr, th)  # warm-up (allocations)
    t0 = time.perf_counter()
    for _ in range(args.reps):
        ctx.decode_frames(y, args.snr, th)
    dt = (time.perf_counter() - t0) / args.reps
    bytes_in = y.nbytes + (0 if args.blind else h.nbytes)
    print(json.dumps({"metric": "codewords/s through kml_decode_frames with host buffers (PCIe-inclusive)",
                      "path": "blind" if args.blind else "known channel",
                      "value": round(B / dt, 1), "batch": B, "ms_per_call": round(dt * 1e3, 3),
                      "host_to_device_bytes_per_cw": bytes_in // B, "device_to_host_bytes_per_cw": ctx.K}))


if __name__ == "__main__":
    main()
