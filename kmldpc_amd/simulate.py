"""Simulator: the reference's `kmldpc` run (kmldpc/kmldpc.cpp + src/simulator.cc)
over one or more MI355X GPUs, one process per GPU.

    python -m kmldpc_amd.simulate [config.toml]                     # 1 GPU
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        -m kmldpc_amd.simulate config.toml                          # 8 GPUs

Each SNR point of the sweep (Simulator::Simulate, simulator.cc:24-67) runs
through kml_sim_point: rank r decodes its slice of every round of global
codeword indices on its own GPU (frames generated in HBM, Philox keyed by seed
and index), and the per-round stop rule of run_blocks (simulator.cc:117) is
applied exactly through an all-reduce of world + 4 counters (RCCL over xGMI when
the process group is NCCL).  Rank 0 prints the reference's console lines
(SourceSink::PrintResult progress, the BER / FER tables).  With world > 1 the
progress is printed once per round instead of every 100 blocks, and histogram
files are per rank (histogram_<snr>.rank<r>.txt).
"""
import argparse
import os
import sys
import time

import numpy as np

from . import Context, lib

INFO = " \x1b[32;1m[INFO]\x1b[0m "
ERROR = " \x1b[31;1m[ERROR]\x1b[0m "


def _stamp():
    return time.strftime("%Y-%m-%d %H:%M:%S", time.localtime())


class Logger:
    """lab::logger (log.cc): `[time] [INFO] message`, tee'd to logs/<time>-kmldpc.logger."""

    def __init__(self, enabled=True, log_dir="logs"):
        self.enabled = enabled
        self.f = None
        if enabled and os.path.isdir(log_dir):
            self.f = open(os.path.join(log_dir, _stamp() + "-kmldpc.logger"), "w")

    def _emit(self, tag, msg):
        if not self.enabled:
            return
        line = "[" + _stamp() + "]" + tag + msg + "\n"
        sys.stdout.write(line)
        sys.stdout.flush()
        if self.f:
            self.f.write(line)
            self.f.flush()

    def info(self, msg):
        self._emit(INFO, msg)

    def error(self, msg):
        self._emit(ERROR, msg)


def result_line(snr, c):
    """SourceSink::PrintResult (sourcesink.cc:50-65)."""
    err_bit, err_blk, tot_bit, tot_blk = c
    ber = err_bit / tot_bit if tot_bit else 0.0
    fer = err_blk / tot_blk if tot_blk else 0.0
    return (f"SNR = {snr:03.3f} Total blk = {tot_blk:07d} Error blk = {err_blk:07d} Error bit = {err_bit:07d} "
            f"BER = {ber:.14f} FER = {fer:.14f}")


def point_seed(seed, i):
    """Frame seed of SNR point i (same rule as kmldpc_sim)."""
    return (int(seed) ^ ((0x9E3779B97F4A7C15 * (i + 1)) & 0xFFFFFFFFFFFFFFFF)) & 0xFFFFFFFFFFFFFFFF


class Simulator:
    """Simulator (include/simulator.h): constructed from config.toml, Simulate() runs the sweep."""

    def __init__(self, config, data_dir=None, device=0, batch=32768, seed=0, dist=None, log=None, comm_backend="nccl"):
        self.ctx = Context(config, data_dir=data_dir or os.path.dirname(os.path.abspath(config)), device=device)
        self.rc = self.ctx.run_config()
        self.batch = int(batch)
        self.seed = int(seed)
        self.dist = dist
        self.rank = dist.get_rank() if dist else 0
        self.world = dist.get_world_size() if dist else 1
        self.log = log or Logger(enabled=self.rank == 0)
        if dist is not None and comm_backend == "nccl":  # RCCL communicator for the counter all-reduces
            from . import comm_unique_id
            uid = [comm_unique_id() if self.rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            self.ctx.comm_init(uid[0], self.world, self.rank)
        rc = self.rc
        self.log.info("Using 5G LDPC." if rc["5gldpc"] else "Using traditional LDPC.")
        self.log.info(f"[{rc['minimum_snr']:.3f},{rc['step_snr']:.3f},{rc['maximum_snr']:.3f}]")
        self.log.info(f"[MAX_ERROR_BLK = {rc['maximum_error_number']},MAX_BLK = {rc['maximum_block_number']}]")

    def _reduce(self, a):
        if self.ctx.comm_size():  # the library's RCCL communicator (xGMI), on the context's stream
            return self.ctx.comm_allreduce(np.ascontiguousarray(a, np.uint64))
        import torch
        t = torch.from_numpy(a.astype(np.int64))
        self.dist.all_reduce(t)  # gloo
        return t.numpy().astype(np.uint64)

    def run(self, snr, i):
        """Simulator::run for one SNR point -> (ber, fer, counters)."""
        rc = self.rc
        hist = None
        if rc["histogram"]:
            hist = f"histogram_{snr:f}.txt" if self.world == 1 else f"histogram_{snr:f}.rank{self.rank}.txt"
        c = self.ctx.sim_point(snr, point_seed(self.seed, i), rank=self.rank, world=self.world, batch=self.batch,
                               max_blocks=max(rc["maximum_block_number"], 0), max_err=max(rc["maximum_error_number"], 0),
                               hist_path=hist, reduce=self._reduce if self.dist is not None else None,
                               report=lambda v: self.log.info(result_line(snr, v)))
        v = [c["err_bit"], c["err_blk"], c["tot_bit"], c["tot_blk"]]
        self.log.info(result_line(snr, v))
        ber = v[0] / v[2] if v[2] else 0.0
        fer = v[1] / v[3] if v[3] else 0.0
        return ber, fer, v

    def Simulate(self):
        rc = self.rc
        n = int((rc["maximum_snr"] - rc["minimum_snr"]) / rc["step_snr"] + 1)
        res = []
        for i in range(n):
            snr = rc["minimum_snr"] + rc["step_snr"] * i
            ber, fer, v = self.run(snr, i)
            res.append((snr, ber, fer, v))
        self.log.info("BER Result")
        for snr, ber, _, _ in res:
            self.log.info(f"{snr:03.3f} {ber:.14f}")
        self.log.info("FER Result")
        for snr, _, fer, _ in res:
            self.log.info(f"{snr:03.3f} {fer:.14f}")
        return res


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("config", nargs="?", default="config.toml")
    ap.add_argument("--batch", type=int, default=int(os.environ.get("KML_BATCH", "32768")))
    ap.add_argument("--seed", type=int, default=int(os.environ.get("KML_SEED", "0")))
    ap.add_argument("--dist-backend", default=os.environ.get("KML_DIST_BACKEND", "nccl"),
                    help="nccl (RCCL over xGMI, one GPU per rank) or gloo (CPU counters; ranks may share a GPU)")
    ap.add_argument("--force-dist", action="store_true", default=os.environ.get("KML_FORCE_DIST", "") == "1",
                    help="build the process group (and run its all-reduces) even when WORLD_SIZE is 1, "
                         "e.g. a 1-rank RCCL group under torchrun --nproc-per-node 1")
    args = ap.parse_args(argv)
    t0 = time.monotonic()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    log = Logger(enabled=rank == 0)
    log.info("Start simulation")
    if not os.path.exists(args.config):
        log.error("Encouter error while opening config.toml")
        log.info("Simulation done")
        return 0
    lib()  # the HIP library (and its ROCm runtime) before torch
    dist = None
    if world > 1 or (args.force_dist and "WORLD_SIZE" in os.environ):
        # gloo: rendezvous and CPU control; the counters' all-reduce is the
        # library's own RCCL communicator with --dist-backend nccl (see bench.py)
        import torch.distributed as dist_mod
        dist_mod.init_process_group(backend="gloo")
        if args.dist_backend != "nccl":  # gloo counters: ranks may share a GPU
            import torch
            local = local % max(torch.cuda.device_count(), 1)
        dist = dist_mod
    sim = Simulator(args.config, device=local, batch=args.batch, seed=args.seed, dist=dist, log=log,
                    comm_backend=args.dist_backend)
    sim.Simulate()
    sim.ctx.close()
    if dist is not None:
        dist.destroy_process_group()
    log.info("Simulation done")
    ms = int((time.monotonic() - t0) * 1000)
    mins = ms // 60000
    secs = ms // 1000 - mins * 60
    log.info(f"Total time cost: {mins}min:{secs}sec:{ms - mins * 60000}ms")
    return 0


if __name__ == "__main__":
    sys.exit(main())
