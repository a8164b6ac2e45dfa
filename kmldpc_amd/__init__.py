"""kmldpc_amd — MI355X-native kmldpc receive path (BP decoder + k-means blind demap).

Python face of the C ABI in include/kmldpc_amd.h (libkmldpc_amd.so, built for
gfx950 by `make lib` / __graft_entry__.build()).  There is no CPU fallback: if
the shared library is missing or the GPU is unavailable, every GPU entry point
raises.  The class names mirror the reference's C++ interface
(/root/reference/kmldpc):

    Context                    config.toml + H-matrix + constellation (KmCodec / BinaryLDPCCodec / Modem ctors)
    Context.bp_decode          lab::BinaryLDPCCodec::Decoder            lib/lab/src/binaryldpccodec.cc:165-278
    Context.demap              lab::ModemLinearSystem::DeMapping         lib/lab/src/modemlinearsystem.cc:93-98
    Context.kmeans             kmldpc::KMeans::Run + simulator.cc:145-148
    Context.decode_frames      KmCodec::Decoder                          src/kmcodec.cc:54-72
    Context.count_errors       lab::SourceSink::CntErr                   lib/lab/src/sourcesink.cc:29-47
    Context.sim_generate/decode  one SNR point of Simulator::run_blocks   src/simulator.cc:112-168
    Context.sim_point          Simulator::run (stop rule, rank sharding) src/simulator.cc:72-110
    sweep_point                the same driver logic with caller-supplied decode / all-reduce
    kmldpc_amd.simulate        Simulator::Simulate + main (SNR sweep, console / log output)
"""
import ctypes as C
import os

import numpy as np

__all__ = ["Context", "KmlError", "lib", "LIB_PATH", "BinaryLDPCCodec", "KMeans", "KmCodec", "dump_kmeans_mat"]

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("KML_LIB") or os.path.join(HERE, "libkmldpc_amd.so")  # KML_LIB: A/B builds
INCLUDE = os.path.join(os.path.dirname(HERE), "include", "kmldpc_amd.h")

KML_DEVICE_PTRS = 1
KML_HISTOGRAM = 2
DIM_NAMES = ["M", "Ncol", "K", "cc_len", "Z", "E", "chk", "max_iter", "bits", "Kc", "S", "bp_lds", "part_group"]


def comm_unique_id():
    """A fresh RCCL unique id (128 bytes) for kml_comm_init (rank 0 calls it)."""
    u = np.zeros(128, np.uint8)
    r = lib().kml_comm_unique_id(_p(u))
    if r != 0:
        raise KmlError(f"{lib().kml_last_error(None).decode()} (code {r})")
    return u.tobytes()


class KmlError(RuntimeError):
    pass


# kml_point_cfg and the driver callbacks (include/kmldpc_amd.h)
class PointCfg(C.Structure):
    _fields_ = [("snr", C.c_double), ("rank", C.c_int), ("world", C.c_int), ("batch", C.c_int),
                ("max_blocks", C.c_uint64), ("max_err", C.c_uint64), ("K", C.c_int), ("ncand", C.c_int),
                ("hist_path", C.c_char_p), ("report_every", C.c_int)]


ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.POINTER(C.c_uint64), C.c_int, C.c_void_p)
BATCH_FN = C.CFUNCTYPE(C.c_int, C.c_uint64, C.c_int, C.POINTER(C.c_int32), C.POINTER(C.c_double), C.c_void_p)
REPORT_FN = C.CFUNCTYPE(None, C.POINTER(C.c_uint64), C.c_void_p)
RUN_CONFIG_KEYS = ["maximum_error_number", "maximum_block_number", "thread_block_number", "true_h_arg", "5gldpc",
                   "metric_type", "metric_iter", "histogram", "max_iter", "active"]


_lib = None


def lib():
    """Load libkmldpc_amd.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise KmlError(f"{LIB_PATH} not built: run `make lib` (or __graft_entry__.build())")
    L = C.CDLL(LIB_PATH)
    P, I, D = C.c_void_p, C.c_int, C.c_double
    PP = C.POINTER(C.c_void_p)
    sig = {
        "kml_abi_version": (I, []),
        "kml_bp_kernel": (C.c_char_p, [P]),
        "kml_create": (I, [C.c_char_p, C.c_char_p, I, PP]),
        "kml_create_explicit": (I, [C.c_char_p, C.c_char_p, I, I, I, I, I, I, PP]),
        "kml_destroy": (None, [P]),
        "kml_last_error": (C.c_char_p, [P]),
        "kml_dims": (I, [P, P]),
        "kml_code_perm": (I, [P, P]),
        "kml_code_graph": (I, [P, P, P, P, P]),
        "kml_constellation": (I, [P, P]),
        "kml_encode": (I, [P, P, P, I]),
        "kml_bp_decode": (I, [P, P, I, I, P, P, P, P, I]),
        "kml_demap": (I, [P, P, P, D, I, P, I]),
        "kml_kmeans": (I, [P, P, I, I, P, P, I]),
        "kml_kmeans_state": (I, [P, P, I, I, P, P, I]),
        "kml_kmeans_dump_mat": (I, [C.c_char_p, P, I, P, P, P, I, P]),
        "kml_decode_frames": (I, [P, P, P, D, I, P, P, P, P, P, I]),
        "kml_count_errors": (I, [P, P, P, I, P, I]),
        "kml_decode_candidates": (I, [P, P, P, I, D, I, P, P, P, P, I]),
        "kml_sim_generate": (I, [P, D, C.c_uint64, C.c_uint64, I]),
        "kml_sim_decode": (I, [P, D, I, P, I]),
        "kml_sync": (I, [P]),
        "kml_sim_frames": (I, [P, P, P, P]),
        "kml_sim_load": (I, [P, D, P, P, P, I, C.c_uint64]),
        "kml_prof_enable": (I, [P, I]),
        "kml_prof_reset": (I, [P]),
        "kml_prof_read": (I, [P, C.c_char_p, P, P, P]),
        "kml_prof_read_flops": (I, [P, C.c_char_p, P]),
        "kml_math_probe": (I, [P, P, I, P]),
        "kml_div_probe": (I, [P, P, I, P]),
        "kml_debug_inject_abort": (I, [P, I]),
        "kml_comm_unique_id": (I, [P]),
        "kml_comm_init": (I, [P, P, I, I]),
        "kml_comm_size": (I, [P]),
        "kml_comm_allreduce_u64": (I, [P, P, I]),
        "kml_comm_allreduce_f64": (I, [P, P, I]),
        "kml_log_probe": (I, [P, P, I, P]),
        "kml_lcg_uniform": (D, [P]),
        "kml_lcg_normal": (None, [P, P, I]),
        "kml_wh_uniform": (D, [P]),
        "kml_wh_normal": (None, [P, P, I]),
        "kml_get_bit_str": (None, [P, P, I]),
        "kml_get_sym_str": (None, [P, P, I, I]),
        "kml_ref_frames": (I, [P, P, D, I, P, P, P]),
        "kml_sim_decode_ex": (I, [P, D, I, I, P, P, P]),
        "kml_run_config": (I, [P, P, P]),
        "kml_sweep_point": (I, [C.POINTER(PointCfg), BATCH_FN, P, ALLREDUCE_FN, P, REPORT_FN, P, P]),
        "kml_sim_point": (I, [P, C.POINTER(PointCfg), C.c_uint64, ALLREDUCE_FN, P, REPORT_FN, P, P]),
    }
    ab_build = "KML_LIB" in os.environ  # an A/B build of other sources may predate newer entry points
    for name, (res, args) in sig.items():
        if ab_build and not hasattr(L, name):
            continue
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def header_symbols():
    """Function names declared by include/kmldpc_amd.h."""
    import re
    txt = open(INCLUDE).read()
    return sorted(set(re.findall(r"\b(kml_[a-z0-9_]+)\s*\(", txt)))


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def _f64(a, shape=None):
    a = np.ascontiguousarray(a, dtype=np.float64)
    if shape is not None:
        a = a.reshape(shape)
    return a


class Context:
    """One code + modem on one GPU (device < 0: host-only planner context)."""

    def __init__(self, config=None, data_dir=None, device=0, *, matrix_file=None, modem_file=None, is5g=False,
                 active=True, max_iter=20, metric_soft=False, metric_iter=5):
        L = lib()
        h = C.c_void_p()
        if config is not None:
            r = L.kml_create(os.fsencode(config), os.fsencode(data_dir) if data_dir else None, int(device),
                             C.byref(h))
        else:
            if matrix_file is None or modem_file is None:
                raise ValueError("need a config path or matrix_file + modem_file")
            r = L.kml_create_explicit(os.fsencode(matrix_file), os.fsencode(modem_file), int(is5g), int(active),
                                      int(max_iter), int(metric_soft), int(metric_iter), int(device), C.byref(h))
        self._h = h
        if r != 0:
            msg = L.kml_last_error(h).decode() if h.value else "kml_create failed"
            if h.value:
                L.kml_destroy(h)
            self._h = None
            raise KmlError(f"kml_create: {msg} (code {r})")
        d = np.zeros(len(DIM_NAMES), np.int32)
        L.kml_dims(h, _p(d))
        self.dims = {k: int(v) for k, v in zip(DIM_NAMES, d)}
        for k, v in self.dims.items():
            setattr(self, k, v)
        self.device = device
        self._sim_B = 0

    def close(self):
        if getattr(self, "_h", None):
            lib().kml_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _chk(self, r, what):
        if r != 0:
            raise KmlError(f"{what}: {lib().kml_last_error(self._h).decode()} (code {r})")

    # ---- planner / host side
    def perm(self):
        p = np.zeros(self.Ncol, np.int32)
        self._chk(lib().kml_code_perm(self._h, _p(p)), "kml_code_perm")
        return p

    def graph(self):
        rp = np.zeros(self.M + 1, np.int32)
        rc = np.zeros(self.E, np.int32)
        cp = np.zeros(self.Ncol + 1, np.int32)
        cs = np.zeros(self.E, np.int32)
        self._chk(lib().kml_code_graph(self._h, _p(rp), _p(rc), _p(cp), _p(cs)), "kml_code_graph")
        return rp, rc, cp, cs

    def constellation(self):
        pts = np.zeros(2 * self.Kc)
        self._chk(lib().kml_constellation(self._h, _p(pts)), "kml_constellation")
        return pts.reshape(-1, 2)

    def encode(self, uu):
        uu = np.ascontiguousarray(uu, np.uint8).reshape(-1, self.K)
        cc = np.zeros((uu.shape[0], self.cc_len), np.uint8)
        self._chk(lib().kml_encode(self._h, _p(uu), _p(cc), uu.shape[0]), "kml_encode")
        return cc

    # ---- GPU entry points
    def bp_decode(self, p0, iter_count=None, cc_hat=False, syn=None):
        """BinaryLDPCCodec::Decoder over a batch; returns dict(uu_hat, ret[, cc_hat, syn])."""
        p0 = _f64(p0).reshape(-1, self.cc_len)
        B = p0.shape[0]
        it = self.max_iter if iter_count is None else int(iter_count)
        uh = np.zeros((B, self.K), np.uint8)
        ret = np.zeros(B, np.int32)
        cch = np.zeros((B, self.Ncol), np.uint8) if cc_hat else None
        if syn is not None:
            syn = _f64(syn).reshape(B, self.M).copy()
        self._chk(lib().kml_bp_decode(self._h, _p(p0), B, it, _p(uh), _p(ret), _p(cch), _p(syn), 0), "kml_bp_decode")
        out = dict(uu_hat=uh, ret=ret)
        if cc_hat:
            out["cc_hat"] = cch
        if syn is not None:
            out["syn"] = syn
        return out

    def demap(self, y, h, var):
        y = _f64(y).reshape(-1, self.S, 2)
        B = y.shape[0]
        h = _f64(h).reshape(B, 2)
        p0 = np.zeros((B, self.cc_len))
        self._chk(lib().kml_demap(self._h, _p(y), _p(h), float(var), B, _p(p0), 0), "kml_demap")
        return p0

    def kmeans(self, y, iters=20):
        y = _f64(y).reshape(-1, self.S, 2)
        B = y.shape[0]
        hh = np.zeros((B, 2))
        h4 = np.zeros((B, 4, 2))
        self._chk(lib().kml_kmeans(self._h, _p(y), B, int(iters), _p(hh), _p(h4), 0), "kml_kmeans")
        return hh, h4

    def kmeans_state(self, y, iters=20):
        """KMeans(y, constellations, iters).Run(); clusters() -> [B, Kc, 2], idx() -> [B, S] int32."""
        y = _f64(y).reshape(-1, self.S, 2)
        B = y.shape[0]
        cl = np.zeros((B, self.Kc, 2))
        idx = np.zeros((B, self.S), np.int32)
        self._chk(lib().kml_kmeans_state(self._h, _p(y), B, int(iters), _p(cl), _p(idx), 0), "kml_kmeans_state")
        return cl, idx

    def decode_frames(self, y, snr, true_h=None, histogram=False):
        """KmCodec::Decoder: known channel if true_h is given, else the blind path.
        histogram=True runs KmCodec::GetHistogramData instead (metrics, no final decode)."""
        y = _f64(y).reshape(-1, self.S, 2)
        B = y.shape[0]
        th = None if true_h is None else _f64(true_h).reshape(B, 2)
        uh = np.zeros((B, self.K), np.uint8)
        ch = np.zeros(B, np.int32)
        met = np.zeros((B, 4))
        ret = np.zeros(B, np.int32)
        hh = np.zeros((B, 2))
        self._chk(lib().kml_decode_frames(self._h, _p(y), _p(th), float(snr), B, _p(uh), _p(ch), _p(met), _p(ret),
                                          _p(hh), KML_HISTOGRAM if histogram else 0), "kml_decode_frames")
        return dict(uu_hat=uh, chosen=ch, metrics=met, ret=ret, h_hat=hh)

    def decode_candidates(self, y, h_hats, snr, histogram=False):
        """KmCodec::Decoder with explicit estimates h_hats[B][nc][2] (kml_decode_candidates)."""
        y = _f64(y, (-1, self.S, 2))
        B = y.shape[0]
        hh = _f64(h_hats, (B, -1, 2))
        nc = hh.shape[1]
        uh = np.zeros((B, self.K), np.uint8)
        ch = np.zeros(B, np.int32)
        met = np.zeros((B, 4))
        ret = np.zeros(B, np.int32)
        self._chk(lib().kml_decode_candidates(self._h, _p(y), _p(hh), nc, float(snr), B, _p(uh), _p(ch), _p(met),
                                              _p(ret), KML_HISTOGRAM if histogram else 0), "kml_decode_candidates")
        return dict(uu_hat=uh, chosen=ch, metrics=met, ret=ret)

    def count_errors(self, uu, uu_hat):
        uu = np.ascontiguousarray(uu, np.uint8).reshape(-1, self.K)
        uh = np.ascontiguousarray(uu_hat, np.uint8).reshape(-1, self.K)
        cnt = np.zeros(4, np.uint64)
        self._chk(lib().kml_count_errors(self._h, _p(uu), _p(uh), uu.shape[0], _p(cnt), 0), "kml_count_errors")
        return dict(zip(["err_bit", "err_blk", "tot_bit", "tot_blk"], [int(x) for x in cnt]))

    def sim_generate(self, snr, B, seed=17, first_cw=0):
        self._chk(lib().kml_sim_generate(self._h, float(snr), int(seed), int(first_cw), int(B)), "kml_sim_generate")
        self._sim_B = int(B)

    def sim_decode(self, snr, blind=False, sync=True):
        if not sync:
            self._chk(lib().kml_sim_decode(self._h, float(snr), int(blind), None, 0), "kml_sim_decode")
            return None
        cnt = np.zeros(8, np.uint64)
        self._chk(lib().kml_sim_decode(self._h, float(snr), int(blind), _p(cnt), 1), "kml_sim_decode")
        return dict(zip(["err_bit", "err_blk", "tot_bit", "tot_blk", "vn_phases", "cn_phases", "converged", "redone"],
                        [int(x) for x in cnt[:8]]))

    def bp_kernel(self):
        """Name of the BP kernel family the last decode launched."""
        return lib().kml_bp_kernel(self._h).decode()

    def sync(self):
        self._chk(lib().kml_sync(self._h), "kml_sync")

    def sim_decode_ex(self, snr, blind=False, histogram=False):
        """Synchronous sim decode with per-codeword error bits and metrics."""
        B = self._sim_B
        err = np.zeros(B, np.int32)
        met = np.zeros((B, 4))
        cnt = np.zeros(8, np.uint64)
        self._chk(lib().kml_sim_decode_ex(self._h, float(snr), int(blind), int(histogram), _p(err), _p(met), _p(cnt)),
                  "kml_sim_decode_ex")
        return err, met, dict(zip(["err_bit", "err_blk", "tot_bit", "tot_blk", "vn_phases", "cn_phases",
                                   "converged", "redone"], [int(x) for x in cnt[:8]]))

    def run_config(self):
        """The parsed config.toml ([range], [decoder], [xcodec], [histogram], [ldpc])."""
        f = np.zeros(3)
        n = np.zeros(10, np.int64)
        self._chk(lib().kml_run_config(self._h, _p(f), _p(n)), "kml_run_config")
        d = dict(minimum_snr=float(f[0]), maximum_snr=float(f[1]), step_snr=float(f[2]))
        d.update({k: int(v) for k, v in zip(RUN_CONFIG_KEYS, n)})
        return d

    def sim_point(self, snr, seed, *, rank=0, world=1, batch=32768, max_blocks, max_err, hist_path=None,
                  reduce=None, report=None, report_every=100):
        """One SNR point of Simulator::run on this GPU (kml_sim_point); see sweep_point for reduce/report."""
        cfg = point_cfg(snr, rank, world, batch, max_blocks, max_err, self.K, 4, hist_path, report_every)
        cnt = np.zeros(4, np.uint64)
        rf, pf = _reduce_cb(reduce), _report_cb(report)
        self._chk(lib().kml_sim_point(self._h, C.byref(cfg), int(seed), rf, None, pf, None, _p(cnt)),
                  "kml_sim_point")
        return dict(zip(["err_bit", "err_blk", "tot_bit", "tot_blk"], [int(x) for x in cnt]))

    def sim_load(self, snr, uu, y, h, first_cw=0):
        """Make host frames (uu[B][K] bytes, y[B][S][2], true h[B][2]) the resident batch (kml_sim_load)."""
        uu = np.ascontiguousarray(uu, np.uint8).reshape(-1, self.K)
        B = uu.shape[0]
        y = _f64(y, (B, self.S, 2))
        h = _f64(h, (B, 2))
        self._chk(lib().kml_sim_load(self._h, float(snr), _p(uu), _p(y), _p(h), B, int(first_cw)), "kml_sim_load")
        self._sim_B = B

    def sim_frames(self, B):
        uu = np.zeros((B, self.K), np.uint8)
        y = np.zeros((B, self.S, 2))
        h = np.zeros((B, 2))
        self._chk(lib().kml_sim_frames(self._h, _p(uu), _p(y), _p(h)), "kml_sim_frames")
        return uu, y, h

    def prof_enable(self, on=True):
        self._chk(lib().kml_prof_enable(self._h, int(on)), "kml_prof_enable")

    def prof_reset(self):
        self._chk(lib().kml_prof_reset(self._h), "kml_prof_reset")

    def prof_read(self, stage):
        n = np.zeros(1, np.int64)
        ms = np.zeros(1)
        by = np.zeros(1)
        fl = np.zeros(1)
        self._chk(lib().kml_prof_read(self._h, stage.encode(), _p(n), _p(ms), _p(by)), "kml_prof_read")
        self._chk(lib().kml_prof_read_flops(self._h, stage.encode(), _p(fl)), "kml_prof_read_flops")
        return dict(launches=int(n[0]), ms=float(ms[0]), bytes=float(by[0]), flops=float(fl[0]))

    def div_probe(self, x):
        x = _f64(x).reshape(-1, 3)
        out = np.zeros((x.shape[0], 12))
        self._chk(lib().kml_div_probe(self._h, _p(x), x.shape[0], _p(out)), "kml_div_probe")
        return out

    # ---- multi-GPU counter reduction (RCCL over xGMI, kml_comm_*)
    def comm_init(self, uid, world, rank):
        """Join the RCCL communicator of `world` ranks (a collective); uid from
        comm_unique_id() on rank 0, distributed over any CPU channel."""
        u = np.frombuffer(bytes(uid), np.uint8).copy()
        if u.size != 128:
            raise ValueError("RCCL unique id must be 128 bytes")
        self._chk(lib().kml_comm_init(self._h, _p(u), int(world), int(rank)), "kml_comm_init")

    def comm_size(self):
        return int(lib().kml_comm_size(self._h))

    def comm_allreduce(self, vals):
        """In-place sum over the ranks of a uint64 or float64 numpy array (RCCL)."""
        if vals.dtype == np.uint64:
            self._chk(lib().kml_comm_allreduce_u64(self._h, _p(vals), vals.size), "kml_comm_allreduce_u64")
        elif vals.dtype == np.float64:
            self._chk(lib().kml_comm_allreduce_f64(self._h, _p(vals), vals.size), "kml_comm_allreduce_f64")
        else:
            raise TypeError("comm_allreduce: uint64 or float64")
        return vals

    def debug_inject_abort(self, nth):
        """Test hook: raise the abort word after the nth cooperative BP launch."""
        self._chk(lib().kml_debug_inject_abort(self._h, int(nth)), "kml_debug_inject_abort")

    def ref_frames(self, rng, snr, n):
        """n frames of the reference's sequential stream (Simulator::run_blocks)
        from rng (a CLCRandNum); returns uu[n][K], true_h[n][2], y[n][S][2]."""
        uu = np.zeros((n, self.K), np.uint8)
        th = np.zeros((n, 2))
        y = np.zeros((n, self.S, 2))
        self._chk(lib().kml_ref_frames(self._h, _p(rng.state), float(snr), int(n), _p(uu), _p(th), _p(y)),
                  "kml_ref_frames")
        return uu, th, y

    def log_probe(self, x):
        x = _f64(x).reshape(-1)
        out = np.zeros_like(x)
        self._chk(lib().kml_log_probe(self._h, _p(x), x.shape[0], _p(out)), "kml_log_probe")
        return out

    def math_probe(self, x):
        x = _f64(x).reshape(-1, 4)
        out = np.zeros_like(x)
        self._chk(lib().kml_math_probe(self._h, _p(x), x.shape[0], _p(out)), "kml_math_probe")
        return out


# ---------------------------------------------------------------------------
# The reference's host random sources (lib/lab/src/randnum.cc, sourcesink.cc)

class CLCRandNum:
    """lab::CLCRandNum: Park-Miller (A = 48271) + polar normals; SetSeed(-1) -> state 17."""

    def __init__(self, state=17):
        self.state = np.array([state], np.int64)

    def Uniform(self):
        return lib().kml_lcg_uniform(_p(self.state))

    def Normal(self, n):
        out = np.zeros(n)
        lib().kml_lcg_normal(_p(self.state), _p(out), int(n))
        return out

    def GetBitStr(self, n):
        out = np.zeros(n, np.uint8)
        lib().kml_get_bit_str(_p(self.state), _p(out), int(n))
        return out

    def GetSymStr(self, qary, n):
        out = np.zeros(n, np.int32)
        lib().kml_get_sym_str(_p(self.state), _p(out), int(qary), int(n))
        return out


class CWHRandNum:
    """lab::CWHRandNum: Wichmann-Hill + polar normals; SetSeed(-1) -> (13, 37, 91)."""

    def __init__(self, xyz=(13, 37, 91)):
        self.xyz = np.array(xyz, np.int32)

    def Uniform(self):
        return lib().kml_wh_uniform(_p(self.xyz))

    def Normal(self, n):
        out = np.zeros(n)
        lib().kml_wh_normal(_p(self.xyz), _p(out), int(n))
        return out


# ---------------------------------------------------------------------------
# Simulator driver host logic (kml_sweep_point): stop rule + rank sharding.

def point_cfg(snr, rank, world, batch, max_blocks, max_err, K, ncand=4, hist_path=None, report_every=100):
    return PointCfg(float(snr), int(rank), int(world), int(batch), int(max_blocks), int(max_err), int(K),
                    int(ncand), os.fsencode(hist_path) if hist_path else None, int(report_every))


def _reduce_cb(fn):
    """fn(np.ndarray[uint64]) -> summed array over ranks (in place or returned)."""
    if fn is None:
        return ALLREDUCE_FN()

    def cb(vals, n, _user):
        try:
            a = np.ctypeslib.as_array(vals, shape=(n,))
            r = fn(a.copy())
            a[:] = np.asarray(r if r is not None else a, dtype=np.uint64)
            return 0
        except Exception:  # never let a Python exception unwind through C
            import traceback
            traceback.print_exc()
            return -1
    return ALLREDUCE_FN(cb)


def _report_cb(fn):
    if fn is None:
        return REPORT_FN()

    def cb(c, _user):
        try:
            fn([int(c[i]) for i in range(4)])
        except Exception:
            import traceback
            traceback.print_exc()
    return REPORT_FN(cb)


def sweep_point(snr, decode, *, K, batch, max_blocks, max_err, rank=0, world=1, reduce=None, report=None,
                hist_path=None, ncand=4, report_every=100):
    """kml_sweep_point with Python callbacks: decode(first_cw, count) ->
    (err[count] int, metrics[count][4] or None); reduce(np.uint64 array) -> sum
    over ranks; report([err_bit, err_blk, tot_bit, tot_blk])."""
    def dcb(first, count, err, met, _user):
        try:
            e, m = decode(int(first), int(count))
            np.ctypeslib.as_array(err, shape=(count,))[:] = np.asarray(e, np.int32)
            if met and m is not None:
                np.ctypeslib.as_array(met, shape=(count, 4))[:] = np.asarray(m, np.float64)
            return 0
        except Exception:
            import traceback
            traceback.print_exc()
            return -1
    cfg = point_cfg(snr, rank, world, batch, max_blocks, max_err, K, ncand, hist_path, report_every)
    cnt = np.zeros(4, np.uint64)
    bf, rf, pf = BATCH_FN(dcb), _reduce_cb(reduce), _report_cb(report)
    r = lib().kml_sweep_point(C.byref(cfg), bf, None, rf, None, pf, None, _p(cnt))
    if r != 0:
        raise KmlError(f"kml_sweep_point failed (code {r})")
    return dict(zip(["err_bit", "err_blk", "tot_bit", "tot_blk"], [int(x) for x in cnt]))


# ---------------------------------------------------------------------------
# Reference-shaped facades (same method names and argument meaning as the C++
# classes, batched along a leading axis).

class BinaryLDPCCodec:
    """lab::BinaryLDPCCodec / lab::Binary5GLDPCCodec (lib/lab/include/binaryldpccodec.h:11-56)."""

    def __init__(self, ctx):
        self.ctx = ctx

    def Decoder(self, M2V, uu_hat, iter_count):
        """Decodes M2V[B, cc_len]; fills uu_hat[B, K]; returns the per-codeword return values."""
        r = self.ctx.bp_decode(M2V, iter_count)
        uu_hat[...] = r["uu_hat"].reshape(uu_hat.shape)
        return r["ret"]

    def Encoder(self, uu, cc):
        cc[...] = self.ctx.encode(uu).reshape(cc.shape)

    def code_dim(self):
        return self.ctx.K

    def code_len(self):
        return self.ctx.cc_len

    def num_row(self):
        return self.ctx.M

    def max_iter(self):
        return self.ctx.max_iter


class KMeans:
    """kmldpc::KMeans (include/kmeans.h:12-32), batched: data[B, S, 2]."""

    def __init__(self, ctx, data, iters=20):
        self.ctx, self.data, self.iters = ctx, data, iters
        self._hh = None

    def Run(self):
        self._hh, self._h4 = self.ctx.kmeans(self.data, self.iters)

    def h_hat(self):
        """clusters()[0] / constellations[0] (src/simulator.cc:145)."""
        return self._hh

    def h_hats(self):
        """the 4 phase candidates (src/simulator.cc:146-148)."""
        return self._h4

    def clusters(self):
        """KMeans::clusters() per codeword, [B, Kc, 2] (include/kmeans.h:18)."""
        self._state()
        return self._cl

    def idx(self):
        """KMeans::idx() per codeword, [B, S] int32 (include/kmeans.h:19)."""
        self._state()
        return self._idx

    def _state(self):
        if getattr(self, "_cl", None) is None:
            self._cl, self._idx = self.ctx.kmeans_state(self.data, self.iters)

    def DumpToMat(self, filename, append, b=0):
        """KMeans::DumpToMat (src/kmeans.cc:99-109) of codeword b: append = the 4
        candidates and the true H (5 complex values, [5, 2] or complex[5])."""
        self._state()
        dump_kmeans_mat(filename, np.asarray(self.data).reshape(-1, self.ctx.S, 2)[b], self._cl[b], self._idx[b],
                        self.ctx.constellation(), append)


def dump_kmeans_mat(filename, data, clusters, idx, constellations, append):
    """kml_kmeans_dump_mat: one codeword's k-means state as a MAT-file level 5
    (data, cluster, idx, constellations, hHats, realH; lib/lab/src/mat.cc)."""
    def cplx(a, n=None):
        a = np.asarray(a)
        if np.iscomplexobj(a):
            a = np.stack([a.real, a.imag], -1)
        a = np.ascontiguousarray(a, np.float64).reshape(-1, 2)
        assert n is None or a.shape[0] == n
        return a
    d, c, k = cplx(data), cplx(clusters), cplx(constellations)
    ap = cplx(append, 5)
    ix = np.ascontiguousarray(idx, np.int32).reshape(-1)
    assert ix.size == d.shape[0] and c.shape[0] == k.shape[0]
    rc = lib().kml_kmeans_dump_mat(os.fsencode(filename), _p(d), d.shape[0], _p(c), _p(ix), _p(k), k.shape[0], _p(ap))
    if rc != 0:
        raise KmlError(f"kml_kmeans_dump_mat: error {rc}")


class KmCodec:
    """KmCodec (include/kmcodec.h:16-53): blind or known-channel decode."""

    def __init__(self, ctx):
        self.ctx = ctx

    def Decoder(self, y, snr, uu_hat, true_h=None):
        r = self.ctx.decode_frames(y, snr, true_h)
        uu_hat[...] = r["uu_hat"].reshape(uu_hat.shape)
        return r

    def uu_len(self):
        return self.ctx.K

    def cc_len(self):
        return self.ctx.cc_len
