"""ctypes binding of the C oracle — TEST INFRASTRUCTURE ONLY.

Loaded by tests/, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg to check /
time the MI355X backend. The product package ``plssvm_sparse_fp22_amd`` never imports this.
The C sources restate the reference OpenMP hot path (see oracle/oracle.h for the file:line map
and the fixtures that pin it).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
KERNELS = {"linear": 0, "polynomial": 1, "poly": 1, "rbf": 2}

_libs: dict = {}


def build() -> None:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib(fast: bool = False) -> ctypes.CDLL:
    name = "liboracle_fast.so" if fast else "liboracle.so"
    if name not in _libs:
        path = os.path.join(_HERE, "build", name)
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        _declare(L)
        _libs[name] = L
    return _libs[name]


_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_INT = ctypes.c_int


def _declare(L):
    for suf, R in (("f64", ctypes.c_double), ("f32", ctypes.c_float)):
        f = getattr(L, f"orc_kernel_{suf}")
        f.argtypes = [_INT, _INT, R, R, _P, _P, _I64]
        f.restype = R
        f = getattr(L, f"orc_q_{suf}")
        f.argtypes = [_INT, _INT, R, R, _P, _I64, _I64, _P]
        f = getattr(L, f"orc_kp_{suf}")
        f.argtypes = [_INT, _INT, R, R, _P, _I64, _I64, _P, R, R, R, _P, _P, _INT]
        f = getattr(L, f"orc_q_csr_{suf}")
        f.argtypes = [_INT, _INT, R, R, _P, _P, _P, _I64, _I64, _P]
        f = getattr(L, f"orc_kp_csr_{suf}")
        f.argtypes = [_INT, _INT, R, R, _P, _P, _P, _I64, _I64, _P, R, R, R, _P, _P, _INT]
        f = getattr(L, f"orc_kp_csr_factored_{suf}")
        f.argtypes = [_P, _P, _P, _I64, _I64, _P, R, R, R, _P, _P, _INT]
        f = getattr(L, f"orc_cg_{suf}")
        f.argtypes = [_INT, _INT, R, R, _P, _P, _P, _I64, _I64, _P, _I64, R, _P, R, R, _P, _P, _INT]
        f.restype = _I64
        f = getattr(L, f"orc_learn_{suf}")
        f.argtypes = [_INT, _INT, R, R, R, R, _I64, _P, _P, _P, _P, _I64, _I64, _P, _P, _P, _P, _INT]
        f.restype = _I64
        f = getattr(L, f"orc_predict_{suf}")
        f.argtypes = [_INT, _INT, R, R, _P, _P, _I64, _I64, R, _P, _I64, _P]
    L.orc_fp22_encode.argtypes = [ctypes.c_float]
    L.orc_fp22_encode.restype = ctypes.c_uint32
    L.orc_fp22_decode.argtypes = [ctypes.c_uint32]
    L.orc_fp22_decode.restype = ctypes.c_float
    L.orc_fp22_pack.argtypes = [_P, _I64, _P]
    L.orc_fp22_unpack.argtypes = [_P, _I64, _P]
    L.orc_fp22_words.argtypes = [_I64]
    L.orc_fp22_words.restype = _I64


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _suf(dtype):
    return "f64" if np.dtype(dtype) == np.float64 else "f32"


class Data:
    """Dense (row-major [n][d]) or CSR view handed to the C oracle."""

    def __init__(self, X=None, rowptr=None, col=None, val=None, n=None, d=None, dtype=np.float64):
        self.dtype = np.dtype(dtype)
        if X is not None:
            self.X = np.ascontiguousarray(X, dtype=self.dtype)
            self.n, self.d = self.X.shape
            self.rowptr = self.col = None
        else:
            self.X = np.ascontiguousarray(val, dtype=self.dtype)
            self.rowptr = np.ascontiguousarray(rowptr, dtype=np.int64)
            self.col = np.ascontiguousarray(col, dtype=np.int32)
            self.n, self.d = int(n), int(d)

    @property
    def csr(self):
        return self.rowptr is not None


def kernel_value(kernel, a, b, degree=3, gamma=1.0, coef0=0.0, fast=False):
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b, dtype=a.dtype)
    f = getattr(lib(fast), f"orc_kernel_{_suf(a.dtype)}")
    return f(KERNELS[kernel], degree, gamma, coef0, _ptr(a), _ptr(b), a.shape[0])


def generate_q(kernel, data: Data, degree=3, gamma=1.0, coef0=0.0, fast=False):
    q = np.zeros(max(data.n - 1, 0), dtype=data.dtype)
    s = _suf(data.dtype)
    if data.csr:
        getattr(lib(fast), f"orc_q_csr_{s}")(KERNELS[kernel], degree, gamma, coef0, _ptr(data.rowptr),
                                              _ptr(data.col), _ptr(data.X), data.n, data.d, _ptr(q))
    else:
        getattr(lib(fast), f"orc_q_{s}")(KERNELS[kernel], degree, gamma, coef0, _ptr(data.X), data.n, data.d,
                                          _ptr(q))
    return q


def kp(kernel, data: Data, q, QA_cost, cost, add, p, ret=None, degree=3, gamma=1.0, coef0=0.0, nthreads=0,
       fast=False):
    """ret += add * Q~ p  (reference run_device_kernel semantics; cost is C, 1/C is passed down)."""
    dt = data.dtype
    q = np.ascontiguousarray(q, dtype=dt)
    p = np.ascontiguousarray(p, dtype=dt)
    ret = np.zeros(data.n - 1, dtype=dt) if ret is None else ret
    s = _suf(dt)
    cost_inv = dt.type(1) / dt.type(cost)
    if data.csr:
        getattr(lib(fast), f"orc_kp_csr_{s}")(KERNELS[kernel], degree, gamma, coef0, _ptr(data.rowptr),
                                               _ptr(data.col), _ptr(data.X), data.n, data.d, _ptr(q), QA_cost,
                                               cost_inv, add, _ptr(p), _ptr(ret), nthreads)
    else:
        getattr(lib(fast), f"orc_kp_{s}")(KERNELS[kernel], degree, gamma, coef0, _ptr(data.X), data.n, data.d,
                                           _ptr(q), QA_cost, cost_inv, add, _ptr(p), _ptr(ret), nthreads)
    return ret


def kp_csr_factored(data: Data, q, QA_cost, cost, add, p, ret=None, nthreads=0, fast=True):
    """CPU baseline only: the linear K·p of CSR data in the O(nnz) factored form."""
    assert data.csr
    dt = data.dtype
    q = np.ascontiguousarray(q, dtype=dt)
    p = np.ascontiguousarray(p, dtype=dt)
    ret = np.zeros(data.n - 1, dtype=dt) if ret is None else ret
    getattr(lib(fast), f"orc_kp_csr_factored_{_suf(dt)}")(_ptr(data.rowptr), _ptr(data.col), _ptr(data.X), data.n,
                                                          data.d, _ptr(q), QA_cost, dt.type(1) / dt.type(cost), add,
                                                          _ptr(p), _ptr(ret), nthreads)
    return ret


def solve_cg(kernel, data: Data, b, imax, eps, q, QA_cost, cost, degree=3, gamma=1.0, coef0=0.0, nthreads=0,
             fast=False):
    dt = data.dtype
    m = data.n - 1
    x = np.zeros(m, dtype=dt)
    trace = np.full(imax + 1, np.nan)
    b = np.ascontiguousarray(b, dtype=dt)
    q = np.ascontiguousarray(q, dtype=dt)
    it = getattr(lib(fast), f"orc_cg_{_suf(dt)}")(
        KERNELS[kernel], degree, gamma, coef0, _ptr(data.X), _ptr(data.rowptr), _ptr(data.col), data.n, data.d,
        _ptr(b), imax, eps, _ptr(q), QA_cost, dt.type(1) / dt.type(cost), _ptr(x), _ptr(trace), nthreads)
    return x, trace[: it + 1], it


def learn(kernel, data: Data, y, cost=1.0, eps=1e-3, imax=-1, degree=3, gamma=None, coef0=0.0, nthreads=0,
          fast=False):
    """csvm<T>::learn(); returns dict(alpha[n], bias, rho, QA_cost, trace, iters)."""
    dt = data.dtype
    if gamma is None:
        gamma = dt.type(1) / dt.type(data.d)
    y = np.ascontiguousarray(y, dtype=dt)
    alpha = np.zeros(data.n, dtype=dt)
    bias = np.zeros(1, dtype=dt)
    qa = np.zeros(1, dtype=dt)
    im = data.d if imax < 0 else imax
    trace = np.full(im + 1, np.nan)
    it = getattr(lib(fast), f"orc_learn_{_suf(dt)}")(
        KERNELS[kernel], degree, gamma, coef0, cost, eps, im, _ptr(data.X), _ptr(data.rowptr), _ptr(data.col),
        _ptr(y), data.n, data.d, _ptr(alpha), _ptr(bias), _ptr(qa), _ptr(trace), nthreads)
    return dict(alpha=alpha, bias=dt.type(bias[0]), rho=-dt.type(bias[0]), QA_cost=dt.type(qa[0]),
                trace=trace[: it + 1], iters=it)


def predict(kernel, SV, alpha, rho, Z, degree=3, gamma=1.0, coef0=0.0):
    SV = np.ascontiguousarray(SV)
    dt = SV.dtype
    alpha = np.ascontiguousarray(alpha, dtype=dt)
    Z = np.ascontiguousarray(Z, dtype=dt)
    out = np.zeros(Z.shape[0], dtype=dt)
    getattr(lib(), f"orc_predict_{_suf(dt)}")(KERNELS[kernel], degree, gamma, coef0, _ptr(SV), _ptr(alpha),
                                                SV.shape[0], SV.shape[1], -rho, _ptr(Z), Z.shape[0], _ptr(out))
    return out


def fp22_pack(v):
    v = np.ascontiguousarray(v, dtype=np.float32)
    L = lib()
    w = np.zeros(L.orc_fp22_words(v.size), dtype=np.uint32)
    L.orc_fp22_pack(_ptr(v), v.size, _ptr(w))
    return w


def fp22_unpack(words, n):
    words = np.ascontiguousarray(words, dtype=np.uint32)
    v = np.zeros(n, dtype=np.float32)
    lib().orc_fp22_unpack(_ptr(words), n, _ptr(v))
    return v
