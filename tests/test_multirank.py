"""N > 1 path on the CPU: world_size-2 gloo runs of the simulator driver's
sharding + stop rule (kml_sweep_point, the code kml_sim_point and
kmldpc_amd.simulate run on the GPUs), checked against a sequential restatement
of Simulator::run_blocks (src/simulator.cc:116-167).

The per-codeword outcomes fed to the driver are the reference's own: the error
bits and candidate metrics of its seed-17 stream (tests/golden fixtures), so the
counters are the ones a single-threaded reference run would print.  The only
collective is the per-round all-reduce of world + 4 counters.
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import load_case

import kmldpc_amd as K


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _sequential(errs, max_blocks, max_err, Kb):
    """run_blocks' loop on one thread: stop check before every codeword (:117)."""
    eb = ebit = tot = 0
    reports = []
    while tot < max_blocks and eb < max_err and tot < len(errs):
        e = int(errs[tot])
        tot += 1
        if e:
            eb += 1
            ebit += e
        if tot % 100 == 0:
            reports.append([ebit, eb, tot * Kb, tot])
    return dict(err_bit=ebit, err_blk=eb, tot_bit=tot * Kb, tot_blk=tot), reports


def _hist_line(m, nc):
    best = int(np.argmin(m[:nc]))
    return " ".join("%g" % m[q % nc] for q in range(best, best + nc)) + " "


def _worker(rank, world, port, case, cases, outdir, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch
    hdr, z = load_case(case)
    errs = z["s_errs"].astype(np.int64)
    mets = z["s_metrics"].astype(np.float64)

    def decode(first, count):
        assert first + count <= len(errs), "driver asked past the fixture stream"
        return errs[first:first + count], mets[first:first + count]

    def reduce(a):
        t = torch.from_numpy(a.astype(np.int64))
        dist.all_reduce(t)
        return t.numpy().astype(np.uint64)

    out = []
    for (max_blocks, max_err, batch) in cases:
        reports = []
        hp = os.path.join(outdir, f"h_{max_blocks}_{max_err}_{batch}_r{rank}.txt")
        r = K.sweep_point(2.0, decode, K=hdr["K"], batch=batch, max_blocks=max_blocks, max_err=max_err, rank=rank,
                          world=world, reduce=reduce, report=reports.append, hist_path=hp, ncand=4)
        out.append((r, reports))
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


CASES = [
    (600, 10 ** 9, 64),  # block limit only, ragged last round
    (600, 57, 50),  # error limit lands inside a round
    (599, 300, 7),  # odd batch
    (450, 1, 16),  # stop after the first block error
    (0, 5, 8),  # nothing to do
    (40, 0, 8),  # maximum_error_number = 0: stop before the first codeword
]


@pytest.mark.parametrize("case,world", [("peg2304_qpsk_blind", 2), ("peg2304_qpsk_known", 2), ("peg2304_qpsk_known", 8),
                                        ("peg2304_qpsk_blind", 5)])
def test_multi_rank_gloo_sweep_matches_sequential(case, world, tmp_path):
    """world 2, 5 and 8 over gloo: the driver's first 8-GPU run then exercises
    only the RCCL transport, not untested rank logic (the batches 64, 50, 7, 16
    and 8 do not divide the block limits, so the last round is ragged and the
    error limit lands inside a round on some rank other than 0)."""
    hdr, z = load_case(case)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, case, CASES, str(tmp_path), q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=600) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    errs = z["s_errs"]
    mets = z["s_metrics"]
    for i, (max_blocks, max_err, batch) in enumerate(CASES):
        want, _ = _sequential(errs, max_blocks, max_err, hdr["K"])
        for r in range(world):
            got, reports = res[r][i]
            assert got == want, (case, max_blocks, max_err, batch, r)
            # one progress record per round, cumulative and monotone, ending at the totals
            if want["tot_blk"]:
                assert reports[-1] == [want["err_bit"], want["err_blk"], want["tot_bit"], want["tot_blk"]]
                assert all(a[3] <= b[3] for a, b in zip(reports, reports[1:]))
        # histogram lines: the ranks' files interleave per round into the sequential order
        lines = {r: open(tmp_path / f"h_{max_blocks}_{max_err}_{batch}_r{r}.txt").read().splitlines()
                 for r in range(world)}
        merged = []
        pos = {r: 0 for r in range(world)}
        while any(pos[r] < len(lines[r]) for r in range(world)):
            for r in range(world):
                merged += lines[r][pos[r]:pos[r] + batch]
                pos[r] += batch
        n = want["tot_blk"]
        assert merged == [_hist_line(mets[j], 4) for j in range(n)]


def test_single_rank_reports_every_100_blocks():
    hdr, z = load_case("peg2304_qpsk_known")
    errs = z["s_errs"]

    def decode(first, count):
        return errs[first:first + count], None

    for batch in (64, 256, 1000):
        reports = []
        got = K.sweep_point(2.0, decode, K=hdr["K"], batch=batch, max_blocks=600, max_err=10 ** 9,
                            report=reports.append)
        want, want_reports = _sequential(errs, 600, 10 ** 9, hdr["K"])
        assert got == want
        assert reports == want_reports  # SourceSink::PrintResult at tot_blk % 100 == 0 (:167)


def test_sweep_point_rejects_bad_arguments():
    with pytest.raises(K.KmlError):
        K.sweep_point(2.0, lambda f, c: (np.zeros(c), None), K=10, batch=0, max_blocks=10, max_err=1)
    with pytest.raises(K.KmlError):  # world > 1 needs a reduce callback
        K.sweep_point(2.0, lambda f, c: (np.zeros(c), None), K=10, batch=4, max_blocks=10, max_err=1, rank=0,
                      world=2)
    with pytest.raises(K.KmlError):  # a failing decode callback stops the point with an error
        K.sweep_point(2.0, lambda f, c: 1 / 0, K=10, batch=4, max_blocks=10, max_err=1)
