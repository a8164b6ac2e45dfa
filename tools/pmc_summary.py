"""Summarise rocprofv3 counter-collection CSVs for one kernel.

    python tools/pmc_summary.py <dir-with-*_counter_collection.csv> <kernel-substring> [--json out.json]
        [--batch B] [--workload NAME] [--calib-kernel demap_kernel --calib-bytes-per-dispatch N]

Prints per-counter averages per dispatch of the matching kernel.  FETCH_SIZE /
WRITE_SIZE are in KiB (rocprofv3 derived counters).  Per MI355X_MICROARCH.md
"HBM": on gfx950 FETCH_SIZE reads exactly half the bytes of a wide (16 B/lane)
coalesced stream; WRITE_SIZE is exact for 16 B/lane stores; other widths must
be calibrated on a known byte count, which --calib-kernel does (the demapper
reads y and writes P0 with 16 B per lane, its bytes are known exactly).
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def load(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            rows.extend(csv.DictReader(fh))
    return rows


def per_dispatch(rows, sub):
    acc = defaultdict(lambda: defaultdict(float))
    for r in rows:
        name = r.get("Kernel_Name", "")
        if sub not in name:
            continue
        did = r.get("Dispatch_Id") or r.get("Correlation_Id")
        acc[r["Counter_Name"]][did] += float(r["Counter_Value"])
    return {k: (sum(v.values()) / len(v), len(v)) for k, v in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--json")
    ap.add_argument("--batch", type=int)
    ap.add_argument("--workload")
    ap.add_argument("--alg-bytes-per-launch", type=float)
    ap.add_argument("--waves-per-simd", type=float, help="resident waves per SIMD of the kernel (issue view)")
    ap.add_argument("--round", help="evidence label (e.g. r02_v1)")
    ap.add_argument("--src-sha", help="bench.src_sha() of the kernel sources the counters were taken at")
    args = ap.parse_args()
    rows = []
    for d in args.dirs:
        rows.extend(load(d))
    res = per_dispatch(rows, args.kernel)
    for k, (v, n) in sorted(res.items()):
        print(f"{args.kernel}: {k} = {v:.1f} per dispatch over {n} dispatches")
    if args.json:
        fetch = res.get("FETCH_SIZE", (None, 0))[0]
        write = res.get("WRITE_SIZE", (None, 0))[0]
        out = {
            "kernel": args.kernel, "batch": args.batch, "workload": args.workload,
            "fetch_kib_raw": fetch, "write_kib_raw": write,
            "note": "FETCH_SIZE/WRITE_SIZE KiB per dispatch from rocprofv3 --pmc (separate passes); "
                    "hbm_bytes_per_launch = (2*FETCH_SIZE + WRITE_SIZE) * 1024 per the gfx950 FETCH_SIZE "
                    "half-count correction of MI355X_MICROARCH.md (an upper bound for narrower reads)",
        }
        if fetch is not None and write is not None:
            out["hbm_bytes_per_launch"] = (2 * fetch + write) * 1024
            out["hbm_bytes_per_launch_uncorrected"] = (fetch + write) * 1024
        if args.round:
            out["round"] = args.round
        if args.src_sha:
            out["src_sha"] = args.src_sha
        flops = res.get("SQ_INSTS_VALU_FLOPS_FP64", (None, 0))[0]
        if flops:
            # per-wave flop count (FMA 2, add/mul/trans 1) x 64 lanes: every lane of
            # the BP kernels' waves is active in the fp64 phases
            out["fp64_flops_executed_per_launch"] = 64 * flops
        if args.alg_bytes_per_launch:
            out["alg_bytes_per_launch"] = args.alg_bytes_per_launch
        # VALU issue view: every wave64 VALU instruction holds a SIMD for 4
        # cycles, v_rcp_f64 (TRANS) for 16; the wave's lifetime in cycles is
        # 4 x SQ_WAVE_CYCLES (quad-cycles); waves per CU = 4 per SIMD here.
        valu = res.get("SQ_INSTS_VALU", (None, 0))[0]
        trans = res.get("SQ_INSTS_VALU_TRANS_F64", (None, 0))[0]
        wave_q = res.get("SQ_WAVE_CYCLES", (None, 0))[0]
        if valu and trans is not None and wave_q and args.waves_per_simd:
            issue = (valu - trans) * 4 + trans * 16
            simd_cycles = wave_q * 4 / args.waves_per_simd  # waves share a SIMD
            out["valu_wave_instr_per_launch"] = valu
            out["trans_f64_per_launch"] = trans
            out["valu_issue_cycles_per_launch"] = issue
            out["simd_cycles_per_launch"] = simd_cycles
            out["valu_issue_busy_frac"] = round(issue / simd_cycles, 4)
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)
        print(json.dumps(out))


if __name__ == "__main__":
    main()
