"""ctypes wrapper over oracle/liboracle.so.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() (as the
checker) and bench.py's cpu_baseline leg.  The product package kmldpc_amd never
imports this module.
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_lib = None


def lib():
    global _lib
    if _lib is None:
        path = os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError("oracle/liboracle.so missing: run `make -C oracle`")
        L = C.CDLL(path)
        P = C.c_void_p
        D = C.c_double
        I = C.c_int
        L.orc_code_load.restype = P
        L.orc_code_load.argtypes = [C.c_char_p, I, I, I, I]
        L.orc_code_free.argtypes = [P]
        L.orc_code_dims.argtypes = [P, P]
        L.orc_code_perm.argtypes = [P, P]
        L.orc_code_graph.argtypes = [P, P, P, P, P]
        L.orc_encode.argtypes = [P, P, P]
        L.orc_bp_decode.restype = I
        L.orc_bp_decode.argtypes = [P, P, I, P, P, P]
        L.orc_parity_count.restype = I
        L.orc_parity_count.argtypes = [P, P]
        L.orc_modem_load.restype = P
        L.orc_modem_load.argtypes = [C.c_char_p]
        L.orc_modem_free.argtypes = [P]
        L.orc_modem_bits.restype = I
        L.orc_modem_bits.argtypes = [P]
        L.orc_modem_points.argtypes = [P, P]
        L.orc_map.argtypes = [P, P, I, P]
        L.orc_demap.argtypes = [P, P, I, D, D, D, P]
        L.orc_kmeans_hhat.argtypes = [P, I, P, I, I, P]
        L.orc_kmeans_state.argtypes = [P, I, P, I, I, P, P, P]
        L.orc_rotations.argtypes = [P, P]
        L.orc_rng_seed.argtypes = [P, C.c_long]
        L.orc_uniform.restype = D
        L.orc_uniform.argtypes = [P]
        L.orc_normal_pair.argtypes = [P, P, P]
        L.orc_gen_frame.argtypes = [P, P, P, D, P, P, P, P]
        L.orc_receive.argtypes = [P, P, P, P, D, I, I, I, P, P, P, P, P, P, P]
        L.orc_cdiv.argtypes = [D, D, D, D, P, P]
        L.orc_hypot.restype = D
        L.orc_hypot.argtypes = [D, D]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


class Code:
    """Oracle LDPC code (binaryldpccodec.cc / binary5gldpccodec.cc)."""

    def __init__(self, path, is5g=False, active=True, reversed_rows=False, max_iter=20):
        self.h = lib().orc_code_load(path.encode(), int(is5g), int(active), int(reversed_rows), int(max_iter))
        if not self.h:
            raise RuntimeError(f"oracle: cannot load {path}")
        d = np.zeros(8, np.int32)
        lib().orc_code_dims(self.h, _p(d))
        self.M, self.N, self.K, self.cc_len, self.Z, self.E, self.chk, self.max_iter = [int(x) for x in d]
        self.is5g = bool(is5g)

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_code_free(self.h)
            self.h = None

    def perm(self):
        p = np.zeros(self.N, np.int32)
        lib().orc_code_perm(self.h, _p(p))
        return p

    def graph(self):
        rp = np.zeros(self.M + 1, np.int32)
        rc = np.zeros(self.E, np.int32)
        cp = np.zeros(self.N + 1, np.int32)
        cs = np.zeros(self.E, np.int32)
        lib().orc_code_graph(self.h, _p(rp), _p(rc), _p(cp), _p(cs))
        return rp, rc, cp, cs

    def encode(self, uu):
        uu = np.array(uu, np.int32)  # a copy: the inactive encoder zeroes its uu (binaryldpccodec.cc:157-158)
        cc = np.zeros(self.cc_len, np.int32)
        lib().orc_encode(self.h, _p(uu), _p(cc))
        return cc

    def bp_decode(self, p0, iter_count=None, syn=None):
        p0 = np.ascontiguousarray(p0, np.float64)
        uh = np.zeros(self.K, np.uint8)
        cch = np.zeros(self.N, np.uint8)
        if syn is None:
            syn = np.zeros(self.M, np.float64)
        ret = lib().orc_bp_decode(self.h, _p(p0), int(iter_count if iter_count is not None else self.max_iter),
                                  _p(uh), _p(cch), _p(syn))
        return ret, uh, cch, syn

    def parity_count(self, bits):
        b = np.ascontiguousarray(bits, np.uint8)
        return lib().orc_parity_count(self.h, _p(b))


class Modem:
    def __init__(self, path):
        self.h = lib().orc_modem_load(path.encode())
        if not self.h:
            raise RuntimeError(f"oracle: cannot load {path}")
        self.m = lib().orc_modem_bits(self.h)
        self.Kc = 1 << self.m
        self.points = np.zeros(2 * self.Kc)
        lib().orc_modem_points(self.h, _p(self.points))

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_modem_free(self.h)
            self.h = None

    def demap(self, y, h, var):
        y = np.ascontiguousarray(y, np.float64).reshape(-1)
        S = y.size // 2
        p0 = np.zeros(S * self.m)
        lib().orc_demap(self.h, _p(y), S, float(h[0]), float(h[1]), float(var), _p(p0))
        return p0


class Rng:
    def __init__(self, state=17):
        self.buf = np.zeros(1, np.int64)
        lib().orc_rng_seed(_p(self.buf), state)


def kmeans_hhat(y, cons, iters=20):
    y = np.ascontiguousarray(y, np.float64).reshape(-1)
    cons = np.ascontiguousarray(cons, np.float64).reshape(-1)
    out = np.zeros(2)
    lib().orc_kmeans_hhat(_p(y), y.size // 2, _p(cons), cons.size // 2, iters, _p(out))
    return out


def kmeans_state(y, cons, iters=20):
    """KMeans::clusters() [Kc, 2] and idx() [S] after Run (kmeans.cc:72-83)."""
    y = np.ascontiguousarray(y, np.float64).reshape(-1)
    cons = np.ascontiguousarray(cons, np.float64).reshape(-1)
    cl = np.zeros(cons.size)
    idx = np.zeros(y.size // 2, np.int32)
    lib().orc_kmeans_state(_p(y), y.size // 2, _p(cons), cons.size // 2, iters, None, _p(cl), _p(idx))
    return cl.reshape(-1, 2), idx


def rotations(hh):
    hh = np.ascontiguousarray(hh, np.float64)
    out = np.zeros(8)
    lib().orc_rotations(_p(hh), _p(out))
    return out.reshape(4, 2)


def gen_frames(code, modem, snr, n, state=17):
    """n codewords of the reference's sequential per-codeword stream (seed 17)."""
    r = Rng(state)
    S = code.cc_len // modem.m
    uu = np.zeros((n, code.K), np.int32)
    cc = np.zeros((n, code.cc_len), np.int32)
    th = np.zeros((n, 2))
    y = np.zeros((n, S, 2))
    for i in range(n):
        lib().orc_gen_frame(code.h, modem.h, _p(r.buf), float(snr), _p(uu[i]), _p(cc[i]), _p(th[i]), _p(y[i]))
    return uu, cc, th, y


def receive(code, modem, y, true_h, snr, blind, metric_soft=False, metric_iter=5, syn=None):
    y = np.ascontiguousarray(y, np.float64)
    th = np.ascontiguousarray(true_h, np.float64)
    uh = np.zeros(code.K, np.uint8)
    p0 = np.zeros(code.cc_len)
    met = np.zeros(4)
    ch = np.zeros(1, np.int32)
    hh = np.zeros(2)
    ret = np.zeros(1, np.int32)
    if syn is None:
        syn = np.zeros(code.M)
    lib().orc_receive(code.h, modem.h, _p(y), _p(th), float(snr), int(blind), int(metric_soft), int(metric_iter),
                      _p(uh), _p(p0), _p(met), _p(ch), _p(hh), _p(ret), _p(syn))
    return dict(uu_hat=uh, p0=p0, metrics=met, chosen=int(ch[0]), h_hat=hh, ret=int(ret[0]), syn=syn)


def cdiv(a, b, c, d):
    re = np.zeros(1)
    im = np.zeros(1)
    lib().orc_cdiv(a, b, c, d, _p(re), _p(im))
    return re[0], im[0]
