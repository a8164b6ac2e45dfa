"""Per-kernel evidence of one bench workload from tools/pmc_workload.sh output:
rocprofv3 --kernel-trace --stats averages and the PMC counters per dispatch.

    python tools/kernel_evidence.py gpurun_out/pmc_<name> [--out profiles/<prefix>_kernels_<name>.json]

Per kernel: average duration, HBM bytes per dispatch ((2*FETCH_SIZE +
WRITE_SIZE) KiB x 1024, the gfx950 FETCH_SIZE half-count correction of
MI355X_MICROARCH.md) and the GB/s they mean over that duration, executed fp64
flops (64 x SQ_INSTS_VALU_FLOPS_FP64) and TFLOP/s, VALU wave-instructions,
the VALU issue-busy fraction (4 SIMD cycles per wave64 VALU instruction, 16
per v_rcp_f64, over SQ_WAVE_CYCLES x 4 / waves per SIMD), and the LDS bank
conflict share (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE).
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

HBM_PEAK_GBS = 8000.0
FP64_PEAK_TFLOPS = 78.6
# resident waves per SIMD of each kernel family (block size / LDS limits)
WAVES_PER_SIMD = {"bp_regular_kernel": 3, "bp_irregular_kernel": 3, "bp_part_kernel[tagged]": 4, "km_fused_kernel": None,
                  "cand_metric_kernel": None, "demap_kernel": None}


def short(name):
    n = name.replace("kml::(anonymous namespace)::", "").replace("void ", "")
    base = n.split("(")[0].split("<")[0].strip()
    if base == "bp_part_kernel":  # its last template argument: the tagged launch or the deferred barrier launch
        base += "[tagged]" if n.split(">")[0].rstrip().endswith("true") else "[barrier]"
    return base


def counters(d):
    acc = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
    for f in glob.glob(os.path.join(d, "*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            acc[short(r["Kernel_Name"])][r["Counter_Name"]][r.get("Dispatch_Id") or r["Correlation_Id"]] += float(
                r["Counter_Value"])
    return {k: {c: sum(v.values()) / len(v) for c, v in cs.items()} for k, cs in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out")
    a = ap.parse_args()
    stats = {}
    for r in csv.DictReader(open(os.path.join(a.dir, "t", "run_kernel_stats.csv"))):
        k = short(r["Name"])
        if k.startswith("__amd"):
            continue
        prev = stats.get(k)
        calls, tot = int(r["Calls"]), float(r["TotalDurationNs"])
        if prev:  # template instantiations of one family
            calls += prev["calls"]
            tot += prev["total_ns"]
        stats[k] = {"calls": calls, "total_ns": tot}
    pmc = counters(a.dir)
    out = {}
    for k, st in sorted(stats.items(), key=lambda kv: -kv[1]["total_ns"]):
        ms = st["total_ns"] / st["calls"] / 1e6
        e = {"calls": st["calls"], "avg_ms": round(ms, 4)}
        c = pmc.get(k, {})
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            b = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024
            e["hbm_bytes_per_dispatch"] = round(b)
            e["hbm_GBs"] = round(b / (ms * 1e-3) / 1e9, 1)
            e["hbm_frac"] = round(b / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
        if "SQ_INSTS_VALU_FLOPS_FP64" in c:
            fl = 64 * c["SQ_INSTS_VALU_FLOPS_FP64"]
            e["fp64_flops_executed"] = round(fl)
            e["fp64_TFLOPs"] = round(fl / (ms * 1e-3) / 1e12, 2)
            e["fp64_frac"] = round(fl / (ms * 1e-3) / 1e12 / FP64_PEAK_TFLOPS, 4)
        if "SQ_INSTS_VALU" in c:
            e["valu_wave_instr"] = round(c["SQ_INSTS_VALU"])
            w = WAVES_PER_SIMD.get(k)
            if w and "SQ_WAVE_CYCLES" in c and "SQ_INSTS_VALU_TRANS_F64" in c:
                issue = (c["SQ_INSTS_VALU"] - c["SQ_INSTS_VALU_TRANS_F64"]) * 4 + c["SQ_INSTS_VALU_TRANS_F64"] * 16
                e["valu_issue_busy_frac"] = round(issue / (c["SQ_WAVE_CYCLES"] * 4 / w), 4)
        if "SQ_LDS_BANK_CONFLICT" in c and c.get("SQ_LDS_IDX_ACTIVE"):
            e["lds_bank_conflict_frac"] = round(c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"], 4)
        if "SQ_ACTIVE_INST_VALU" in c and "SQ_BUSY_CYCLES" in c:
            e["sq_active_inst_valu_per_busy_cycle"] = round(c["SQ_ACTIVE_INST_VALU"] / c["SQ_BUSY_CYCLES"], 3)
        out[k] = e
    s = json.dumps({"source": a.dir, "kernels": out}, indent=1)
    print(s)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
