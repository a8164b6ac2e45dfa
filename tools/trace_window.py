"""Average duration of the TIMED dispatches of one kernel in a rocprofv3
--kernel-trace CSV of a bench.py run.

    python tools/trace_window.py <run_kernel_trace.csv> <bench line json> [--out summary.json]

bench.py's line carries roofline.timed_dispatches = {"kernel", "first", "count"}:
the ordinal range of that kernel's dispatches inside the timed region (warm-up
launches precede it; the untimed statistics / full-loop / BER-match launches
follow it and decode other frames).  rocprofv3's --stats average covers every
dispatch of the process, so it is not the number the bench line's
avg_launch_ms describes; this window is.

A BP decode is a launch chain (FAST dispatches, then one EXACT dispatch over
the deferred codewords; tools/kernel_evidence.py): dispatches are grouped into
chains at each EXACT dispatch, and a chain's duration is the span from its
first dispatch's start to its EXACT dispatch's end (what the bench's HIP
events around the chain see), with the summed kernel time beside it.
"""
import argparse
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kernel_evidence import parse  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("bench")
    ap.add_argument("--out")
    a = ap.parse_args()
    line = json.loads(open(a.bench).read().strip().splitlines()[-1])
    w = line["roofline"]["timed_dispatches"]
    rows = [r for r in csv.DictReader(open(a.trace)) if parse(r["Kernel_Name"])[0] == w["kernel"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    chains, cur = [], []
    for r in rows:
        cur.append(r)
        if parse(r["Kernel_Name"])[1] in ("exact", ""):
            chains.append(cur)
            cur = []
    span = [(int(c[-1]["End_Timestamp"]) - int(c[0]["Start_Timestamp"])) / 1e6 for c in chains]
    busy = [sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in c) / 1e6 for c in chains]
    durs = span
    sel = durs[w["first"]: w["first"] + w["count"]]
    selb = busy[w["first"]: w["first"] + w["count"]]
    out = {
        "kernel": w["kernel"],
        "dispatches_in_trace": len(rows),
        "chains_in_trace": len(chains),
        "timed_avg_kernel_busy_ms": sum(selb) / len(selb),
        "timed_window": [w["first"], w["first"] + w["count"]],
        "timed_avg_ms": sum(sel) / len(sel),
        "timed_min_ms": min(sel),
        "timed_max_ms": max(sel),
        "all_dispatch_avg_ms": sum(durs) / len(durs),
        "bench_avg_launch_ms": line["roofline"]["avg_launch_ms"],
        "rel_diff_vs_bench": sum(sel) / len(sel) / line["roofline"]["avg_launch_ms"] - 1.0,
        "source": "rocprofv3 --kernel-trace of the bench command whose line is 'bench'",
    }
    s = json.dumps(out, indent=1)
    print(s)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
