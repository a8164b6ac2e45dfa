"""Per-kernel evidence of one bench workload from tools/pmc_workload.sh output:
rocprofv3 --kernel-trace --stats averages and the PMC counters, per LAUNCH.

    python tools/kernel_evidence.py gpurun_out/pmc_<name> [--out profiles/<prefix>_kernels_<name>.json]
        [--merge profiles/pmc_bp.json --name <name> --matrix M --batch B [--blind] --round R --src-sha S]

A BP decode is a chain of dispatches of one kernel family: the FAST kernel
(the partitioned PEG8064 kernel: its tagged and barrier launches) and the
EXACT kernel over the codewords the FAST one deferred (kernels.hpp; one EXACT
dispatch per chain, usually with no work).  bench.py's avg_launch_ms times the
whole chain (one kml run_bp), so every BP figure here is per chain: the
family's total duration and counter totals over the run / its EXACT dispatches.
demap_kernel and cand_metric_kernel are FAST + EXACT pairs too.  Other kernels:
per dispatch.

Per kernel: average duration, HBM bytes ((2*FETCH_SIZE + WRITE_SIZE) KiB x
1024, the gfx950 FETCH_SIZE half-count correction of MI355X_MICROARCH.md) and
the GB/s they mean over that duration, executed fp64 flops (64 x
SQ_INSTS_VALU_FLOPS_FP64) and TFLOP/s, VALU wave-instructions, the VALU
issue-busy fraction (4 SIMD cycles per wave64 VALU instruction, 16 per
v_rcp_f64, over SQ_WAVE_CYCLES x 4 / waves per SIMD), and the LDS bank conflict
share (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE).

--merge adds (or replaces) this workload's entry in the PMC map bench.py reads:
{"entries": [{"name", "matrix", "blind", "batch", "round", "src_sha", "kernels": {...}}]}.
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

HBM_PEAK_GBS = 8000.0
FP64_PEAK_TFLOPS = 78.6
BP_FAMILIES = ("bp_regular_kernel", "bp_irregular_kernel", "bp_part_kernel")
# kernels launched as a FAST dispatch + an EXACT dispatch over its deferrals (last template argument EXACT)
CHAIN_FAMILIES = BP_FAMILIES + ("demap_kernel", "cand_metric_kernel")
# resident waves per SIMD of each kernel family (block size / register limits)
WAVES_PER_SIMD = {"bp_regular_kernel": 3, "bp_irregular_kernel": 3, "bp_part_kernel": 4}


def parse(name):
    """(family, variant) of a rocprofv3 kernel name; variant 'exact' marks a chain's last dispatch."""
    n = name.replace("kml::(anonymous namespace)::", "").replace("void ", "")
    fam = n.split("(")[0].split("<")[0].strip()
    if fam not in CHAIN_FAMILIES or "<" not in n:
        return fam, ""
    targs = [t.strip() for t in n.split("<", 1)[1].split(">")[0].split(",")]
    # the EXACT flag: demap_kernel<MB, EXACT, ROT>, the others' last argument
    exact = (targs[1] if fam == "demap_kernel" and len(targs) > 2 else targs[-1]) == "true"
    if fam == "bp_part_kernel":
        return fam, "exact" if exact else ("fast_tagged" if targs[-2] == "true" else "fast_barrier")
    return fam, "exact" if exact else "fast"


def durations(d):
    tot = defaultdict(lambda: defaultdict(lambda: [0, 0.0]))
    for f in glob.glob(os.path.join(d, "t", "*kernel_stats.csv")):
        for r in csv.DictReader(open(f)):
            fam, var = parse(r["Name"])
            if fam.startswith("__amd"):
                continue
            tot[fam][var][0] += int(r["Calls"])
            tot[fam][var][1] += float(r["TotalDurationNs"])
    return tot


def counters(d):
    """family -> variant -> counter -> (total over dispatches, dispatches)"""
    acc = defaultdict(lambda: defaultdict(lambda: defaultdict(lambda: defaultdict(float))))
    for f in glob.glob(os.path.join(d, "*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            fam, var = parse(r["Kernel_Name"])
            acc[fam][var][r["Counter_Name"]][r.get("Dispatch_Id") or r["Correlation_Id"]] += float(r["Counter_Value"])
    return {f: {v: {c: (sum(x.values()), len(x)) for c, x in cs.items()} for v, cs in vs.items()}
            for f, vs in acc.items()}


def per_launch(cnt, fam):
    """counter -> value per launch (per chain for the BP families)"""
    vs = cnt.get(fam, {})
    names = set(c for v in vs.values() for c in v)
    out = {}
    for c in names:
        tot = sum(v[c][0] for v in vs.values() if c in v)
        if fam in CHAIN_FAMILIES and "exact" in vs:
            n = vs["exact"].get(c, (0, 0))[1]
        else:
            n = sum(v[c][1] for v in vs.values() if c in v)
        if n:
            out[c] = tot / n
    return out


def evidence(d):
    dur = durations(d)
    cnt = counters(d)
    out = {}
    for fam, vs in sorted(dur.items(), key=lambda kv: -sum(x[1] for x in kv[1].values())):
        total_ns = sum(x[1] for x in vs.values())
        if fam in CHAIN_FAMILIES:
            launches = vs.get("exact", [0, 0.0])[0] or sum(x[0] for x in vs.values())
        else:
            launches = sum(x[0] for x in vs.values())
        ms = total_ns / max(launches, 1) / 1e6
        e = {"launches": launches, "avg_ms": round(ms, 4)}
        if fam in CHAIN_FAMILIES:
            e["per"] = "launch chain (FAST dispatches + the EXACT dispatch)"
            e["dispatches"] = {v: {"calls": x[0], "avg_ms": round(x[1] / max(x[0], 1) / 1e6, 4)} for v, x in vs.items()}
        c = per_launch(cnt, fam)
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            b = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024
            e["hbm_bytes_per_launch"] = round(b)
            e["fetch_kib_raw"] = round(c["FETCH_SIZE"], 1)
            e["write_kib_raw"] = round(c["WRITE_SIZE"], 1)
            e["hbm_GBs"] = round(b / (ms * 1e-3) / 1e9, 1)
            e["hbm_frac"] = round(b / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
        if "SQ_INSTS_VALU_FLOPS_FP64" in c:
            fl = 64 * c["SQ_INSTS_VALU_FLOPS_FP64"]
            e["fp64_flops_executed_per_launch"] = round(fl)
            e["fp64_TFLOPs"] = round(fl / (ms * 1e-3) / 1e12, 2)
            e["fp64_frac"] = round(fl / (ms * 1e-3) / 1e12 / FP64_PEAK_TFLOPS, 4)
        if "SQ_INSTS_VALU" in c:
            e["valu_wave_instr_per_launch"] = round(c["SQ_INSTS_VALU"])
            w = WAVES_PER_SIMD.get(fam)
            if w and "SQ_WAVE_CYCLES" in c and "SQ_INSTS_VALU_TRANS_F64" in c:
                issue = (c["SQ_INSTS_VALU"] - c["SQ_INSTS_VALU_TRANS_F64"]) * 4 + c["SQ_INSTS_VALU_TRANS_F64"] * 16
                e["valu_issue_busy_frac"] = round(issue / (c["SQ_WAVE_CYCLES"] * 4 / w), 4)
        if "SQ_LDS_BANK_CONFLICT" in c and c.get("SQ_LDS_IDX_ACTIVE"):
            e["lds_bank_conflict_frac"] = round(c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"], 4)
        if "SQ_ACTIVE_INST_VALU" in c and "SQ_BUSY_CYCLES" in c:
            e["sq_active_inst_valu_per_busy_cycle"] = round(c["SQ_ACTIVE_INST_VALU"] / c["SQ_BUSY_CYCLES"], 3)
        out[fam] = e
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out")
    ap.add_argument("--merge", help="PMC map to add this workload's entry to (profiles/pmc_bp.json)")
    ap.add_argument("--name")
    ap.add_argument("--matrix")
    ap.add_argument("--batch", type=int)
    ap.add_argument("--blind", action="store_true")
    ap.add_argument("--round")
    ap.add_argument("--src-sha")
    a = ap.parse_args()
    ev = evidence(a.dir)
    s = json.dumps({"source": a.dir, "kernels": ev}, indent=1)
    print(s)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")
    if a.merge:
        m = json.load(open(a.merge)) if os.path.exists(a.merge) else {}
        if "entries" not in m:
            m = {"entries": []}
        m["rule"] = ("per workload (matrix, blind, batch per GPU) and kernel family, taken at the kernel sources "
                     "src_sha (bench.src_sha()); BP families per launch chain; HBM bytes = (2*FETCH_SIZE + "
                     "WRITE_SIZE) KiB x 1024 (gfx950 correction); fp64 flops executed = 64 x SQ_INSTS_VALU_FLOPS_FP64")
        m["entries"] = [e for e in m["entries"]
                        if not (e["matrix"] == a.matrix and e["blind"] == a.blind and e["batch"] == a.batch)]
        m["entries"].append({"name": a.name, "matrix": a.matrix, "blind": a.blind, "batch": a.batch,
                             "round": a.round, "src_sha": a.src_sha, "kernels": ev})
        with open(a.merge, "w") as f:
            json.dump(m, f, indent=1)
            f.write("\n")


if __name__ == "__main__":
    main()
