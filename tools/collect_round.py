"""Copy the judged evidence of a tools/gpu_round.sh run into profiles/.

    python tools/collect_round.py <prefix>      # e.g. r01_v6

Writes profiles/<prefix>_bench*.json (bench lines), <prefix>_kernel_stats.csv
(rocprofv3 --kernel-trace --stats of the headline bench),
<prefix>_gpu_tests.log, and <prefix>_pmc_bp.txt (per-dispatch PMC averages of
the BP kernel, every counter group).
"""
import os
import shutil
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "gpurun_out", "round")


def main():
    pre = sys.argv[1]
    dst = os.path.join(REPO, "profiles")
    for name in ["bench", "bench_blind", "bench_bg2", "bench_peg8064"]:
        line = open(os.path.join(SRC, name + ".json")).read().strip().splitlines()[-1]
        with open(os.path.join(dst, f"{pre}_{name}.json"), "w") as f:
            f.write(line + "\n")
    shutil.copy(os.path.join(SRC, "trace", "run_kernel_stats.csv"), os.path.join(dst, f"{pre}_kernel_stats.csv"))
    shutil.copy(os.path.join(SRC, "gpu_tests.log"), os.path.join(dst, f"{pre}_gpu_tests.log"))
    # the timed-window average of the traced bench command (what avg_launch_ms describes)
    subprocess.run([sys.executable, os.path.join(REPO, "tools", "trace_window.py"),
                    os.path.join(SRC, "trace", "run_kernel_trace.csv"), os.path.join(SRC, "trace_bench.json"),
                    "--out", os.path.join(dst, f"{pre}_bp_timed_window.json")], check=True, capture_output=True)
    shutil.copy(os.path.join(SRC, "trace_bench.json"), os.path.join(dst, f"{pre}_trace_bench.json"))
    dirs = [os.path.join(SRC, d) for d in ["pmc_fetch", "pmc_write", "pmc_a", "pmc_b", "pmc_c"]]
    out = subprocess.run([sys.executable, os.path.join(REPO, "tools", "pmc_summary.py"), *dirs, "--kernel",
                          "bp_regular_kernel"], capture_output=True, text=True, check=True).stdout
    with open(os.path.join(dst, f"{pre}_pmc_bp.txt"), "w") as f:
        f.write(out)
    # the summary bench.py reads (headline kernel/workload, this source tree's src_sha)
    sys.path.insert(0, REPO)
    import bench

    subprocess.run([sys.executable, os.path.join(REPO, "tools", "pmc_summary.py"), *dirs, "--kernel",
                    "bp_regular_kernel", "--json", os.path.join(dst, "pmc_bp.json"), "--batch", "32768",
                    "--workload", "PEG2304regular0.5.txt", "--waves-per-simd", "3", "--round", pre,
                    "--src-sha", bench.src_sha()], capture_output=True, text=True, check=True)
    print("wrote", pre, "evidence to profiles/")


if __name__ == "__main__":
    main()
