"""Copy the judged evidence of a tools/gpu_round.sh + tools/gpu_pmc_all.sh run into profiles/.

    python tools/collect_round.py <prefix> [--bench] [--pmc]      # e.g. r03_v1

--bench (gpurun_out/round/): profiles/<prefix>_bench*.json (bench lines) and
<prefix>_gpu_tests.log.
--pmc (gpurun_out/pmc_<workload>/): per workload <prefix>_kernel_stats_<w>.csv
(rocprofv3 --kernel-trace --stats), <prefix>_kernels_<w>.json (per-kernel PMC
evidence, tools/kernel_evidence.py), <prefix>_bp_timed_window_<w>.json (the
traced bench's timed launch chains, tools/trace_window.py), and the workload's
entry in profiles/pmc_bp.json (the map bench.py reads), tagged with this
source tree's src_sha.
"""
import argparse
import json
import os
import shutil
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "gpurun_out")
# workload -> (matrix, blind, batch per GPU): the bench arguments of tools/gpu_pmc_all.sh
WORKLOADS = {
    "headline": ("PEG2304regular0.5.txt", False, 32768),
    "blind": ("PEG2304regular0.5.txt", True, 32768),
    "bg2": ("5GLDPCBG2a3_R12_K960.txt", False, 16384),
    "peg8064": ("PEG8064regular0.5.txt", True, 4096),
}
BENCH = {"headline": "bench", "blind": "bench_blind", "bg2": "bench_bg2", "peg8064": "bench_peg8064"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prefix")
    ap.add_argument("--bench", action="store_true")
    ap.add_argument("--pmc", action="store_true")
    a = ap.parse_args()
    dst = os.path.join(REPO, "profiles")
    pre = a.prefix
    if a.bench:
        src = os.path.join(OUT, "round")
        for name in BENCH.values():
            line = open(os.path.join(src, name + ".json")).read().strip().splitlines()[-1]
            with open(os.path.join(dst, f"{pre}_{name}.json"), "w") as f:
                f.write(line + "\n")
        shutil.copy(os.path.join(src, "gpu_tests.log"), os.path.join(dst, f"{pre}_gpu_tests.log"))
    if a.pmc:
        sys.path.insert(0, REPO)
        import bench

        sha = bench.src_sha()
        for w, (matrix, blind, batch) in WORKLOADS.items():
            d = os.path.join(OUT, f"pmc_{w}")
            if not os.path.isdir(d):
                print("no", d)
                continue
            shutil.copy(os.path.join(d, "t", "run_kernel_stats.csv"), os.path.join(dst, f"{pre}_kernel_stats_{w}.csv"))
            cmd = [sys.executable, os.path.join(REPO, "tools", "kernel_evidence.py"), d,
                   "--out", os.path.join(dst, f"{pre}_kernels_{w}.json"), "--merge", os.path.join(dst, "pmc_bp.json"),
                   "--name", w, "--matrix", matrix, "--batch", str(batch), "--round", pre, "--src-sha", sha]
            if blind:
                cmd.append("--blind")
            subprocess.run(cmd, check=True, capture_output=True)
            subprocess.run([sys.executable, os.path.join(REPO, "tools", "trace_window.py"),
                            os.path.join(d, "t", "run_kernel_trace.csv"), os.path.join(d, "t.json"),
                            "--out", os.path.join(dst, f"{pre}_bp_timed_window_{w}.json")], check=True, capture_output=True)
            shutil.copy(os.path.join(d, "t.json"), os.path.join(dst, f"{pre}_trace_bench_{w}.json"))
    print("wrote", pre, "evidence to profiles/")


if __name__ == "__main__":
    main()
