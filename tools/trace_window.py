"""Average duration of the TIMED dispatches of one kernel in a rocprofv3
--kernel-trace CSV of a bench.py run.

    python tools/trace_window.py <run_kernel_trace.csv> <bench line json> [--out summary.json]

bench.py's line carries roofline.timed_dispatches = {"kernel", "first", "count"}:
the ordinal range of that kernel's dispatches inside the timed region (warm-up
launches precede it; the untimed statistics / full-loop / BER-match launches
follow it and decode other frames).  rocprofv3's --stats average covers every
dispatch of the process, so it is not the number the bench line's
avg_launch_ms describes; this window is.
"""
import argparse
import csv
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("bench")
    ap.add_argument("--out")
    a = ap.parse_args()
    line = json.loads(open(a.bench).read().strip().splitlines()[-1])
    w = line["roofline"]["timed_dispatches"]
    rows = [r for r in csv.DictReader(open(a.trace)) if w["kernel"] in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
    sel = durs[w["first"]: w["first"] + w["count"]]
    out = {
        "kernel": w["kernel"],
        "dispatches_in_trace": len(durs),
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
