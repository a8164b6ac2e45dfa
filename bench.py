"""Throughput benchmark of the kmldpc receive path on MI355X.

Workload (BASELINE.json configs[1]): PEG2304 R=1/2 + QPSK, Es/N0 = 2.0 dB
(= Eb/N0 2 dB), max 20 BP iterations, known-channel ("ideal") demap, a batch of
B synthetic y = h*x + w frames per GPU generated on the GPU before the timed
region (resident in HBM).  One step = demap + sum-product BP (+ error
counting) over the whole resident batch, i.e. KmCodec::Decoder + SourceSink::CntErr
(src/kmcodec.cc:54-72, lib/lab/src/sourcesink.cc:29-47) for B codewords.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--blind]

--gpus N > 1 without a torch.distributed environment starts
`python -m torch.distributed.run --nproc-per-node N bench.py ...` as a child
process (before anything here touches the GPU), forwards rank 0's JSON line
and exits with the child's status.  Each rank is one process on one GPU;
frames are sharded by global codeword index (weak scaling, no data-path
collective) and the error counters are summed with one RCCL all-reduce at the
end (simulator.cc:35-42, :86-100 run SNR points / codeword chunks as
independent tasks the same way).  Rank 0 prints ONE JSON line.

Besides the timed region the line carries, all untimed:
  * stats.ber_match: the first B_ref codewords of the reference's own seed-17
    stream (CLCRandNum::SetSeed(-1)) decoded on the GPU, compared codeword by
    codeword with the reference's SourceSink::CntErr counters for the same
    codewords (tests/golden/bench/*.npz, made by running the reference itself);
    and the timed Philox batch's BER against the reference BER with its
    standard error (ber_within_1sigma);
  * full_loop: GPU frame generation + decode rate (kml_sim_generate + decode);
  * cpu_baseline: the bit-exact C restatement on the host cores (rank 0, N=1).
"""
import argparse
import gzip
import hashlib
import json
import math
import os
import socket
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

K = None  # kmldpc_amd, imported only in a rank process (after the launch decision)

KERNEL_NOTES = {
    "bp_regular_kernel": "sum-product BP, messages LDS-resident",
    "bp_irregular_kernel": "sum-product BP, irregular degrees, messages LDS-resident",
    "bp_part_kernel": "sum-product BP, partitioned LDS slots + cut-edge mailboxes: 4 workgroups on one XCD per "
                      "codeword, tagged mailbox exchange",
    "bp_kernel": "sum-product BP, generic",
}
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8 TB/s spec
FP64_PEAK_TFLOPS = 78.6  # MI355X fp64 dense peak (vector = matrix rate, AMD spec)
# sources whose code the PMC summary describes (profiles/pmc_bp.json src_sha)
# every kernel and launcher source: a PMC map entry is current only at the sources it was taken at
PMC_SOURCES = sorted(f for f in os.listdir(os.path.join(REPO, "kmldpc_amd", "csrc"))
                     if f.endswith((".hip", ".hpp", ".cpp")))


def src_sha():
    h = hashlib.sha256()
    for fn in PMC_SOURCES:
        with open(os.path.join(REPO, "kmldpc_amd", "csrc", fn), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def data_dir():
    d = tempfile.mkdtemp(prefix="kml_bench_")
    src = os.path.join(REPO, "tests", "golden", "data")
    for fn in os.listdir(src):
        if fn.endswith(".gz"):
            with gzip.open(os.path.join(src, fn), "rb") as g, open(os.path.join(d, fn[:-3]), "wb") as f:
                f.write(g.read())
    return d


def write_config(d, args):
    cfg = os.path.join(d, "config.toml")
    with open(cfg, "w") as f:
        f.write(f"""[range]
    minimum_snr = {args.snr!r}
    maximum_snr = {args.snr!r}
    step_snr = 1.0
    maximum_error_number = 1000000000
    maximum_block_number = 1000000000
    thread_block_number = {args.batch}
[decoder]
    true_h_arg = {"false" if args.blind else "true"}
[xcodec]
    5gldpc = {"true" if args.is5g else "false"}
    metric_type = false
    metric_iter = 5
[histogram]
    enable = false
[ldpc]
    max_iter = {args.max_iter}
    active = true
    matrix_file = "{args.matrix}"
[modem]
    modem_file = "{args.modem}"
""")
    return cfg


def cgroup_cpu_quota():
    """CPUs' worth of quota from cgroup v2 cpu.max (None = unlimited / unknown)."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else float(q) / float(p)
    except (OSError, ValueError):
        return None


def cpu_baseline(d, args):
    """The oracle restatement of the same receive path timed on host cores
    (reported baseline; test infrastructure, never the measured product).
    T = every CPU in sched_getaffinity (BASELINE.md's plan), lowered to the
    cgroup CPU quota when one is set (threads beyond it only time-slice)."""
    exe = os.path.join(REPO, "oracle", "cpu_baseline")
    if not os.path.exists(exe):
        return None
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count() or 1
    quota = cgroup_cpu_quota()
    threads = affinity if quota is None else max(1, min(affinity, int(math.ceil(quota))))
    # bounded sample: ~args.cpu_seconds of decode at ~1000 cw/s per thread (known H; blind ~1/2)
    per_thread_rate = 500.0 if args.blind else 1000.0
    if args.matrix.startswith("PEG8064") or args.is5g:
        per_thread_rate /= 8.0
    n = args.cpu_cw_per_thread or max(50, int(args.cpu_seconds * per_thread_rate))
    cmd = [exe, os.path.join(d, args.matrix), os.path.join(d, args.modem), str(int(args.is5g)), repr(args.snr),
           str(args.max_iter), str(int(args.blind)), str(n), str(threads)]
    try:
        out = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
        r = json.loads(out.stdout.strip().splitlines()[-1])
    except Exception as e:  # pragma: no cover
        print(f"cpu_baseline failed: {e}", file=sys.stderr)
        return None
    cpu_model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    ncw = r["codewords"]
    fer, ber = r["fer"], r["ber"]
    mean_e = r["err_bit"] / ncw
    ber_sig = (math.sqrt(max(r["sum_e2"] / ncw - mean_e * mean_e, 0.0) * ncw / max(ncw - 1, 1) / ncw) / r["K"]
               if ncw > 1 else None)
    out = {"value": round(r["cw_per_s"], 3), "unit": "codewords/s", "cores": threads, "kind": "port",
           "affinity_cpus": affinity, "cgroup_cpu_quota": quota,
           "full_loop_value": round(r["full_loop_cw_per_s"], 3),
           "sample": f"{ncw} codewords ({n}/thread x {threads} threads, one Park-Miller stream per "
                     f"thread) of the same workload through oracle/ (C restatement of KmCodec::Decoder + CntErr, "
                     f"bit-exact vs reference): decode {r['seconds']:.1f} s (value), + frame generation "
                     f"{r['gen_seconds']:.1f} s (full_loop_value)",
           # the baseline's BER/FER with 1 sigma (FER binomial; BER over codewords, whose bit
           # errors are dependent)
           "fer": round(fer, 6), "fer_sigma": round(math.sqrt(fer * (1 - fer) / ncw), 6),
           "ber": round(ber, 8), "ber_sigma": round(ber_sig, 8) if ber_sig is not None else None,
           "cpu_model": cpu_model}
    out["single_core"] = single_core_rates(d, args, exe)
    return out


def single_core_rates(d, args, exe):
    """One core: the reference itself (oracle/_ref/ref_harness: the reference's
    own sources, its sequential seed-17 stream, construction excluded) beside
    the restatement (oracle/cpu_baseline, 1 thread) on the same workload; both
    decode-only (frames generated outside the timed loop) and full-loop rates.
    A bounded sample of about args.ref_seconds each."""
    harness = os.path.join(REPO, "oracle", "_ref", "ref_harness")
    per_core = 250.0 if args.blind else 500.0
    if args.matrix.startswith("PEG8064") or args.is5g:
        per_core = 30.0 if args.matrix.startswith("PEG8064") else 130.0
    n = max(20, int(args.ref_seconds * per_core))
    res = {"codewords": n}
    try:
        cmd = [exe, os.path.join(d, args.matrix), os.path.join(d, args.modem), str(int(args.is5g)), repr(args.snr),
               str(args.max_iter), str(int(args.blind)), str(n), "1"]
        pr = json.loads(subprocess.run(cmd, capture_output=True, text=True, timeout=600).stdout.strip().splitlines()[-1])
        res["port"] = {"value": round(pr["cw_per_s"], 3), "full_loop_value": round(pr["full_loop_cw_per_s"], 3),
                       "what": "oracle/cpu_baseline, 1 thread, own Park-Miller stream"}
    except Exception as e:  # pragma: no cover
        res["port"] = f"failed: {e}"
    if not os.path.exists(harness):
        res["reference"] = "oracle/_ref/ref_harness not built (needs /root/reference at build time)"
        return res
    try:
        out = os.path.join(d, "ref_sim.bin")
        rr = subprocess.run([harness, os.path.join(d, "config.toml"), repr(args.snr), str(n), out, "simulate"],
                            capture_output=True, text=True, timeout=900, cwd=d)
        t = json.loads([ln for ln in rr.stderr.splitlines() if ln.startswith('{"codewords"')][-1])
        rx, gen = t["receive_seconds"], t["gen_seconds"]
        res["reference"] = {"value": round(n / rx, 3), "full_loop_value": round(n / (rx + gen), 3),
                            "what": "oracle/_ref/ref_harness simulate mode: the reference's KmCodec::Decoder + "
                                    "k-means + SourceSink::CntErr on its own seed-17 stream, 1 core, construction "
                                    "excluded; value = receive only, full_loop_value = + source/encoder/channel"}
        if isinstance(res.get("port"), dict):
            res["port_over_reference"] = round(res["port"]["value"] / res["reference"]["value"], 3)
    except Exception as e:  # pragma: no cover
        res["reference"] = f"failed: {e}"
    return res


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n):
    """Run this script under torch.distributed.run with n ranks as a CHILD
    process (no exec: nothing in this process has touched the GPU), forward
    rank 0's JSON line to stdout and return the child's exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    p = subprocess.run(cmd, stdout=subprocess.PIPE, text=True, env=env)
    for line in p.stdout.splitlines():
        if line.startswith('{"metric"'):
            print(line, flush=True)
        elif line.strip():
            print(line, file=sys.stderr)
    return p.returncode


def bench_fixture(args):
    """The reference's counters for the first B_ref seed-17 codewords of this
    workload (tests/golden/bench/, generated by oracle/_ref), or None."""
    import numpy as np

    d = os.path.join(REPO, "tests", "golden", "bench")
    if not os.path.isdir(d):
        return None
    for fn in sorted(os.listdir(d)):
        if not fn.endswith(".npz"):
            continue
        z = np.load(os.path.join(d, fn))
        hdr = json.loads(bytes(z["hdr_json"]).decode())
        if (hdr["matrix"] == args.matrix and hdr["modem"] == args.modem and hdr["is5g"] == args.is5g
                and hdr["known"] == (not args.blind) and hdr["max_iter"] == args.max_iter
                and abs(hdr["snr"] - args.snr) < 1e-12):
            return fn, hdr, z["errs"].astype(np.int64)
    return None


def large_reference(args):
    """tests/golden/bench/large_oracle.json entry for this workload, or None."""
    fn = os.path.join(REPO, "tests", "golden", "bench", "large_oracle.json")
    if not os.path.exists(fn):
        return None
    for v in json.load(open(fn)).values():
        if (v["matrix"] == args.matrix and v["modem"] == args.modem and v["is5g"] == args.is5g
                and v["known"] == (not args.blind) and v["max_iter"] == args.max_iter
                and abs(v["snr"] - args.snr) < 1e-12):
            return v
    return None


def ber_sigma(sum_e, sum_e2, n, Kbits):
    """Standard error of a BER estimate from per-codeword error counts (the
    bit errors of one codeword are not independent, so the codeword is the unit)."""
    if n < 2:
        return float("nan")
    mean = sum_e / n
    var = max(sum_e2 / n - mean * mean, 0.0) * n / (n - 1)
    return math.sqrt(var / n) / Kbits


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=32768, help="codewords per GPU per step")
    ap.add_argument("--snr", type=float, default=2.0, help="Es/N0 in dB (reference 'snr')")
    ap.add_argument("--max-iter", type=int, default=20)
    ap.add_argument("--matrix", default="PEG2304regular0.5.txt")
    ap.add_argument("--modem", default="2bits_QPSK.txt")
    ap.add_argument("--is5g", action="store_true")
    ap.add_argument("--blind", action="store_true")
    ap.add_argument("--seed", type=int, default=17)
    ap.add_argument("--cpu-cw-per-thread", type=int, default=0, help="0: sized for --cpu-seconds")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--ref-seconds", type=float, default=6.0,
                    help="single-core samples (reference and restatement) of about this many seconds each")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-ber-match", action="store_true")
    ap.add_argument("--full-loop-batches", type=int, default=3)
    ap.add_argument("--force-dist", action="store_true",
                    help="run under torch.distributed.run and build the process group (init, all_reduce, "
                         "all_gather) even for --gpus 1: a 1-rank RCCL group")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (RCCL over xGMI, the production path) or gloo (CPU counters; lets N ranks share "
                         "fewer GPUs for testing)")
    args = ap.parse_args()

    if (args.gpus > 1 or args.force_dist) and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))

    global K
    import kmldpc_amd as K  # noqa: E402

    K.lib()  # load the HIP library (and its ROCm runtime) before torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus > 1 and world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    dist = None
    device = local
    ranks_seen = 1
    if world > 1 or args.force_dist:
        # torch.distributed (gloo) is the rendezvous and CPU control channel only
        # (barriers, the RCCL id broadcast, the timing gather).  The counters'
        # all-reduce is the library's own RCCL communicator (kml_comm_*) on the
        # context's stream: torch never initialises a HIP runtime of its own in
        # this process (its bundled runtime beside the library's is two ROCm
        # runtimes in one process, and the second to start finds no device).
        import torch.distributed as dist_mod

        dist_mod.init_process_group(backend="gloo")
        if args.dist_backend == "gloo":  # counters reduced on the CPU; ranks may share a GPU (tests on a 1-GPU box)
            import torch
            device = local % max(torch.cuda.device_count(), 1)
        dist = dist_mod
        ranks_seen = dist.get_world_size()

    import numpy as np

    d = data_dir()
    cfg = write_config(d, args)
    ctx = K.Context(cfg, data_dir=d, device=device)
    comm_ranks = 0
    if dist is not None and args.dist_backend == "nccl":
        uid = [K.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        ctx.comm_init(uid[0], ranks_seen, rank)  # RCCL communicator over the ranks' GPUs (xGMI)
        comm_ranks = ctx.comm_size()
    B = args.batch
    # frames for global codeword indices [rank*B, (rank+1)*B): resident in HBM
    ctx.sim_generate(args.snr, B, seed=args.seed, first_cw=rank * B)

    def barrier():
        ctx.sync()
        if dist is not None:
            dist.barrier()

    for _ in range(args.warmup):
        ctx.sim_decode(args.snr, blind=args.blind, sync=False)
    barrier()
    ctx.prof_reset()
    ctx.prof_enable(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ctx.sim_decode(args.snr, blind=args.blind, sync=False)
    barrier()
    t1 = time.perf_counter()
    ctx.prof_enable(False)
    elapsed = t1 - t0
    bp = ctx.prof_read("bp")
    bp_kernel = ctx.bp_kernel()
    stages = {s: ctx.prof_read(s) for s in ("demap", "kmeans", "metric")}
    # one more (untimed) pass for the statistical counters and per-codeword errors
    cw_err, _, c = ctx.sim_decode_ex(args.snr, blind=args.blind)
    e64 = cw_err.astype(np.float64)
    vals = np.array([c["err_bit"], c["err_blk"], c["tot_bit"], c["tot_blk"], c["vn_phases"], c["cn_phases"],
                     e64.sum(), (e64 * e64).sum(), c.get("redone", 0)], dtype=np.float64)

    # full loop (untimed by the headline): GPU frame generation + decode, fresh frames per batch
    fl_n = max(0, args.full_loop_batches)
    fl_t = 0.0
    if fl_n:
        barrier()
        tf = time.perf_counter()
        for i in range(fl_n):
            ctx.sim_generate(args.snr, B, seed=args.seed + 1, first_cw=(i * world + rank) * B)
            ctx.sim_decode(args.snr, blind=args.blind, sync=False)
        barrier()
        fl_t = time.perf_counter() - tf

    t_max, fl_max, per_rank = elapsed, fl_t, [elapsed]
    if dist is not None:
        import torch
        if comm_ranks:
            vals = ctx.comm_allreduce(np.ascontiguousarray(vals, np.float64))  # RCCL over xGMI: the only collective
        else:
            tv = torch.tensor(vals)
            dist.all_reduce(tv)  # gloo (CPU counters)
            vals = tv.numpy()
        tt = torch.tensor([elapsed, fl_t], dtype=torch.float64)
        gathered = [torch.zeros_like(tt) for _ in range(ranks_seen)]
        dist.all_gather(gathered, tt)  # timing: CPU control channel
        per_rank = [float(g[0].item()) for g in gathered]
        t_max = max(per_rank)
        fl_max = max(float(g[1].item()) for g in gathered)

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return
    total_cw = B * args.steps * world
    value = total_cw / t_max
    err_bit, err_blk, tot_bit, tot_blk, vn, cn, sum_e, sum_e2, redone = vals
    Kbits = tot_bit / max(tot_blk, 1)
    bp_avg_ms = bp["ms"] / max(bp["launches"], 1)
    bp_bytes = bp["bytes"] / max(bp["launches"], 1)
    bp_flops = bp["flops"] / max(bp["launches"], 1)
    achieved_gbs = bp_bytes / (bp_avg_ms * 1e-3) / 1e9 if bp_avg_ms > 0 else 0.0
    achieved_tf = bp_flops / (bp_avg_ms * 1e-3) / 1e12 if bp_avg_ms > 0 else 0.0

    # PMC map entry of the same workload and kernel family (profiles/pmc_bp.json, tools/kernel_evidence.py)
    traffic, issue_view, frac_exec, pmc_note, pmc_others = None, None, None, "no PMC entry for this kernel/workload", None
    pmc = os.path.join(REPO, "profiles", "pmc_bp.json")
    fam = bp_kernel.split()[0]
    if os.path.exists(pmc):
        try:
            pm = json.load(open(pmc))
            ent = [e for e in pm.get("entries", []) if e.get("matrix") == args.matrix
                   and bool(e.get("blind")) == bool(args.blind) and e.get("batch") == B and fam in e.get("kernels", {})]
            if ent:
                e = ent[-1]
                k = e["kernels"][fam]
                current = e.get("src_sha") == src_sha()
                pmc_note = (f"profiles/pmc_bp.json entry {e.get('name')} ({e.get('round', '?')}), "
                            + ("taken at these kernel sources" if current else
                               "STALE: taken at other kernel sources (src_sha differs)")
                            + f"; rocprofv3 avg per launch chain {k.get('avg_ms')} ms")
                traffic = k.get("hbm_bytes_per_launch")
                if k.get("fp64_flops_executed_per_launch"):
                    fe = k["fp64_flops_executed_per_launch"]
                    frac_exec = {"fp64_flops_executed_per_launch": fe,
                                 "achieved": round(fe / (bp_avg_ms * 1e-3) / 1e12, 2),
                                 "frac": round(fe / (bp_avg_ms * 1e-3) / 1e12 / FP64_PEAK_TFLOPS, 4),
                                 "rule": "64 x SQ_INSTS_VALU_FLOPS_FP64 per launch (PMC) / this run's avg launch time"}
                if k.get("valu_issue_busy_frac") is not None:
                    issue_view = {"valu_issue_busy_frac": k["valu_issue_busy_frac"],
                                  "valu_wave_instr_per_launch": k.get("valu_wave_instr_per_launch"),
                                  "lds_bank_conflict_frac": k.get("lds_bank_conflict_frac"),
                                  "rule": "SIMD cycles the VALU instruction stream occupies (4 per wave64 "
                                          "instruction, 16 per v_rcp_f64) / SIMD cycles of the launch"}
                # the workload's other kernels (k-means, candidate metric, demap), same PMC runs
                pmc_others = {n: {x: v[x] for x in ("avg_ms", "hbm_GBs", "hbm_frac", "fp64_TFLOPs", "fp64_frac",
                                                    "lds_bank_conflict_frac") if x in v}
                              for n, v in e["kernels"].items() if n != fam and v.get("avg_ms", 0) >= 0.05}
        except Exception as ex:  # a malformed map is reported, never fatal
            pmc_note = f"profiles/pmc_bp.json unreadable: {ex}"

    stats = {
        "fer": err_blk / max(tot_blk, 1),
        "ber": err_bit / max(tot_bit, 1),
        "ber_sigma": ber_sigma(sum_e, sum_e2, tot_blk, Kbits),
        "codewords": int(tot_blk),
        "mean_cn_phases": cn / max(tot_blk, 1),
        "mean_vn_phases": vn / max(tot_blk, 1),
        # codewords the FAST kernel could not prove correctly rounded and the EXACT kernel redid
        "redone": int(redone),
        "stage_ms_per_step": {s: round(v["ms"] / max(args.steps, 1), 4) for s, v in stages.items() if v["launches"]},
        "bp_ms_per_step": round(bp["ms"] / max(args.steps, 1), 4),
    }
    fx = None if args.no_ber_match else bench_fixture(args)
    if fx is not None:
        fn, hdr, ref_errs = fx
        n_ref = int(hdr["n"])
        # (1) the reference's own stream through the GPU path, codeword by codeword
        rng = K.CLCRandNum(hdr.get("seed", 17))
        uu, th, y = ctx.ref_frames(rng, args.snr, n_ref)
        ctx.sim_load(args.snr, uu, y, th)
        del y
        g_err, _, gc = ctx.sim_decode_ex(args.snr, blind=args.blind)
        same = bool(np.array_equal(g_err.astype(np.int64), ref_errs))
        ref_bit, ref_blk = int(ref_errs.sum()), int((ref_errs > 0).sum())
        r_e = ref_errs.astype(np.float64)
        ber_ref = ref_bit / (n_ref * hdr["K"])
        sig_ref = ber_sigma(r_e.sum(), (r_e * r_e).sum(), n_ref, hdr["K"])
        ref_src = f"reference seed-17 run, {n_ref} codewords"
        # the larger reference sample (oracle restatement, bit-exact vs the reference, 8 streams) when present
        lg = large_reference(args)
        if lg is not None:
            ber_ref = lg["err_bit"] / (lg["codewords"] * lg["K"])
            sig_ref = ber_sigma(lg["err_bit"], lg["sum_e2"], lg["codewords"], lg["K"])
            ref_src = f"{lg['codewords']} codewords, {lg['streams']} reference streams (seeds {lg['seeds']}), {lg['source']}"
        # (2) the timed (Philox) batch vs the reference, Monte-Carlo standard errors
        sig = math.hypot(sig_ref, stats["ber_sigma"])
        z = (stats["ber"] - ber_ref) / sig if sig > 0 else float("nan")
        stats.update({
            "ber_ref": ber_ref, "ber_ref_sigma": sig_ref, "ber_ref_sample": ref_src,
            "ber_z": z, "ber_sigma_combined": sig, "ber_within_1sigma": bool(abs(z) <= 1.0),
            "ber_match": {
                "frames": f"reference stream CLCRandNum seed 17, first {n_ref} codewords (kml_ref_frames)",
                "reference": f"tests/golden/bench/{fn} (oracle/_ref: the reference's own sources, SourceSink::CntErr)",
                "ref_err_bit": ref_bit, "ref_err_blk": ref_blk,
                "gpu_err_bit": int(gc["err_bit"]), "gpu_err_blk": int(gc["err_blk"]),
                "per_codeword_equal": same,
                "exact": same and ref_bit == int(gc["err_bit"]) and ref_blk == int(gc["err_blk"]),
            },
        })
    line = {
        "metric": "decoded codewords/sec (N=2304 R=1/2, 20 BP iters) at 1/2/4/8 GPUs; BER match",
        "value": round(value, 1),
        "unit": "codewords/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(t_max / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic y=h*x+w frames generated on the GPU (Philox), resident in HBM before timing",
        "config": {
            "workload": f"{args.matrix.split('.txt')[0]} + {args.modem.split('.txt')[0]}, Es/N0 {args.snr} dB, "
                        f"max {args.max_iter} BP iters, {'blind k-means' if args.blind else 'known-H ideal'} demap",
            "batch_per_gpu": B,
            "global_batch": B * world,
            "parallelism": f"codeword-sharded x{world}",
        },
        "dist_backend": (("rccl" if comm_ranks else "gloo") + " counters, gloo control") if dist is not None else None,
        # ranks of the library's RCCL communicator (0: none — one process, or gloo counters)
        "rccl_ranks": comm_ranks,
        "ranks": ranks_seen,
        "rank_ms_per_step": [round(t / args.steps * 1e3, 3) for t in per_rank],
        "full_loop": {
            "value": round(fl_n * B * world / fl_max, 1) if fl_max > 0 else None,
            "unit": "codewords/s",
            "batches": fl_n,
            "what": "kml_sim_generate (Philox source + encoder + channel) + receive, fresh frames per batch",
        },
        "roofline": {
            # Messages are LDS-resident; the kernel is bound by the fp64 vector
            # pipes (no matrix instructions): the roof is MI355X's fp64 peak.
            "bound": "fp64-valu",
            "achieved": round(achieved_tf, 2),
            "peak": FP64_PEAK_TFLOPS,
            "unit": "TFLOP/s",
            "frac": round(achieved_tf / FP64_PEAK_TFLOPS, 4),
            "traffic": traffic,
            "kernel": f"{bp_kernel} ({KERNEL_NOTES.get(bp_kernel, 'sum-product BP')})",
            "avg_launch_ms": round(bp_avg_ms, 4),
            # ordinal range of this kernel's dispatches inside the timed region
            # (tools/trace_window.py reads it against a rocprofv3 kernel trace)
            "timed_dispatches": {"kernel": bp_kernel.split()[0], "count": int(bp["launches"]),
                                 "first": int(bp["launches"]) // max(args.steps, 1) * args.warmup},
            "alg_flops_per_launch": round(bp_flops),
            "alg_flops_rule": "per executed VN phase sum_cols (68*d-23), per CN phase sum_rows (73*d-52) fp64 flops "
                              "(DESIGN.md: Roofline); known-channel QPSK launches also run the demap in their "
                              "prologue, whose work is not counted",
            "frac_executed": frac_exec,
            "issue_view": issue_view,
            "pmc": pmc_note,
            "pmc_other_kernels": pmc_others,
            "hbm_view": {
                "counter_bytes_per_launch": traffic,
                "counter_GBs": round(traffic / (bp_avg_ms * 1e-3) / 1e9, 1) if traffic and bp_avg_ms > 0 else None,
                "peak_GBs": HBM_PEAK_GBS,
                "frac": round(traffic / (bp_avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)
                if traffic and bp_avg_ms > 0 else None,
                "flooding_model_bytes_per_launch": round(bp_bytes),
                "bytes_avoided_vs_flooding_model": round(bp_bytes - traffic) if traffic else None,
                "rule": "counter bytes = (2*FETCH_SIZE + WRITE_SIZE) per launch (gfx950 correction, "
                        "MI355X_MICROARCH.md); the flooding model (SURVEY 8d: VN 24E+9N, CN 24E bytes per phase) "
                        "is what an HBM-resident decoder would move; LDS residency avoids it",
            },
        },
        "stats": stats,
    }
    if world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(d, args)
    print(json.dumps(line), flush=True)
    ctx.close()  # release the device buffers while the runtime is fully up
    if os.environ.get("KML_DUMP_MAPS"):  # diagnostics: map a crash at exit to its library
        with open("/proc/self/maps") as src, open(os.environ["KML_DUMP_MAPS"], "w") as dst:
            dst.write(src.read())
    if os.environ.get("KML_EXIT_RESET") == "1":  # diagnostics (W3): tear the device down before exit()
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so")  # the library's runtime (torch's is never started here)
        print("hipDeviceSynchronize:", hip.hipDeviceSynchronize(), "hipDeviceReset:", hip.hipDeviceReset(),
              file=sys.stderr, flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
