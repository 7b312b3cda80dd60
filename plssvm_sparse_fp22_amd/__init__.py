"""plssvm_sparse_fp22_amd — MI355X-native PLSSVM CG hot path (implicit Q~·p), host-side mirror.

Mirrors the reference's C++ surface for this path so tests read like the reference's own:

* :class:`Parameter` ~ ``plssvm::parameter<T>`` (include/plssvm/parameter.hpp:181-194 defaults:
  C = 1, epsilon = 1e-3, degree = 3, gamma = 1/d, coef0 = 0);
* :class:`CSVM` ~ ``plssvm::hip::csvm<T>`` / ``detail::gpu_csvm<T, ...>``
  (include/plssvm/csvm.hpp:33-278, include/plssvm/backends/gpu_csvm.hpp:37-190) including the
  protected-for-mock hooks of ``mock_hip_csvm`` (tests/backends/HIP/mock_hip_csvm.hpp:24-51):
  ``setup_data_on_device``, ``generate_q``, ``run_device_kernel`` (+ reduction), ``solver_CG``,
  ``set_cost``, ``set_QA_cost``.

Everything computes in libplssvm_mi355x.so (hand-written gfx950 HIP kernels) through the C ABI
``include/plssvm_mi355x.h``; this module only marshals host buffers.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _abi
from ._abi import BackendError, KERNELS
from . import io as _io
from .io import parse_libsvm, parse_model, read_binary, write_binary

__all__ = ["Parameter", "CSVM", "BackendError", "parse_libsvm", "parse_model", "read_binary", "write_binary",
           "device_count", "unique_id", "partition", "torch_exchange"]


def device_count() -> int:
    return int(_abi.lib().plssvm_mi_device_count())


def unique_id() -> bytes:
    """RCCL unique id for a row-block group (rank 0 creates it and shares it out of band)."""
    buf = ctypes.create_string_buffer(_abi.UNIQUE_ID_BYTES)
    _abi.check(_abi.lib().plssvm_mi_get_unique_id(buf))
    return buf.raw


def partition(m, rank, world_size):
    """Work split of the implicit matrix (host-only): (first super-block, end super-block,
    total tiles, tiles owned by rank); see plssvm_mi_partition in include/plssvm_mi355x.h."""
    out = (ctypes.c_int64 * 4)()
    _abi.check(_abi.lib().plssvm_mi_partition(m, rank, world_size, out))
    return tuple(out)


def torch_exchange(dist, group=None):
    """Host-staged exchange (plssvm_mi_comm_init_host) over torch.distributed, e.g. gloo: every rank
    all-gathers the buffers and sums them in rank order 0..G-1, so all ranks get the same bits — the
    reference's device_reduction, which sums devices 0..G-1 on the host (gpu_csvm.cpp:366-386).

    Failure protocol: each payload carries one status element. A rank whose local step fails still
    takes part in the collective (sending the failure flag), and then every rank raises, so the whole
    group returns PLSSVM_MI_ERR_RCCL together instead of the peers waiting forever in the collective."""
    import torch

    def fn(buf, op, local_error=None):
        world = dist.get_world_size(group)
        rank = dist.get_rank(group)
        count = buf.size // world if op == _abi.XCHG_ALLGATHER else buf.size
        dt = torch.from_numpy(buf[:0]).dtype
        payload = torch.zeros(count + 1, dtype=dt)
        try:
            if local_error is not None:
                raise local_error
            src = buf[rank * count:(rank + 1) * count] if op == _abi.XCHG_ALLGATHER else buf
            payload[:count] = torch.from_numpy(src.copy())
        except Exception as e:  # noqa: BLE001 — still join the collective, flagged
            payload.zero_()
            payload[count] = 1
            err = e
        else:
            err = None
        parts = [torch.empty(count + 1, dtype=dt) for _ in range(world)]
        dist.all_gather(parts, payload, group=group)
        failed = [r for r in range(world) if float(parts[r][count]) != 0.0]
        if failed:
            raise RuntimeError(f"host exchange failed on rank(s) {failed}") from err
        if op == _abi.XCHG_ALLGATHER:
            for r in range(world):
                buf[r * count:(r + 1) * count] = parts[r][:count].numpy()
        else:
            acc = parts[0][:count].numpy().copy()
            for r in range(1, world):
                acc += parts[r][:count].numpy()
            buf[:] = acc

    return fn


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


class Parameter:
    """plssvm::parameter<T> subset used by the hot path."""

    def __init__(self, kernel="linear", degree=3, gamma=0.0, coef0=0.0, cost=1.0, epsilon=1e-3,
                 real_type=np.float64, print_info=False):
        if kernel not in KERNELS:
            raise ValueError(f"Unknown kernel type {kernel!r}")
        self.kernel = kernel
        self.degree = int(degree)
        self.gamma = gamma
        self.coef0 = coef0
        self.cost = cost
        self.epsilon = epsilon
        self.real_type = np.dtype(real_type)
        self.print_info = print_info
        self.data = None  # dense [n][d]
        self.csr = None  # (rowptr, col, val, n, d); val real or packed FP22 words
        self.coo = None  # (row, col, val, n, d) triplets in any order; val real or packed FP22 words
        self.val_fmt = _abi.VAL_REAL
        self.labels = None

    def parse_train_file(self, path, sparse=False):
        try:
            with open(path, "rb") as f:
                binary = f.read(8) == _io.BIN_MAGIC
        except FileNotFoundError:  # file_not_found_exception (src/plssvm/detail/file_reader.cpp:104-108)
            raise FileNotFoundError(f"Couldn't find file: '{path}'!") from None
        if binary:  # PLSSVMB1 binary CSR / FP22 file (io.write_binary): always sparse
            csr, y, fmt = _io.read_binary(path, dtype=self.real_type)
            self.csr, self.data, self.labels = csr, None, y
            self.val_fmt = _abi.VAL_FP22 if fmt == _io.BIN_FP22 else _abi.VAL_REAL
            if self.gamma == 0:
                self.gamma = float(self.real_type.type(1) / self.real_type.type(csr[4]))
            return self
        X, y = parse_libsvm(path, dtype=self.real_type, sparse=sparse)
        if sparse:
            self.csr, self.data = X, None
            d = X[4]
        else:
            self.data, self.csr = X, None
            d = X.shape[1]
        self.labels = y
        if self.gamma == 0:  # parameter.cpp:150-152
            self.gamma = float(self.real_type.type(1) / self.real_type.type(d))
        return self

    @property
    def num_features(self):
        if self.data is not None:
            return self.data.shape[1]
        return int((self.csr if self.csr is not None else self.coo)[4])

    @property
    def num_data_points(self):
        if self.data is not None:
            return self.data.shape[0]
        return int((self.csr if self.csr is not None else self.coo)[3])


class CSVM:
    """One MI355X context (one GPU, one HIP stream). ``world_size > 1`` joins a row-block group."""

    def __init__(self, params: Parameter, device=0, rank=0, world_size=1, uid=None, kp_mode="auto",
                 sim_rank=None, rbf_form=0, exchange=None, sparse_algo="auto", cg_variant=None):
        if params.data is None and params.csr is None and params.coo is None:
            raise ValueError("No data points provided!")
        if params.data is not None:
            if params.data.ndim != 2 or params.data.shape[0] == 0:
                raise ValueError("Data set is empty!")
            if params.data.shape[1] == 0:
                raise ValueError("No features provided for the data points!")
        self.params = params
        self.dtype = params.real_type
        self.num_data_points = params.num_data_points
        self.num_features = params.num_features
        gamma = params.gamma if params.gamma != 0 else 1.0 / self.num_features
        self._ctx = ctypes.c_void_p()
        L = _abi.lib()
        _abi.check(L.plssvm_mi_create(self.dtype.itemsize, KERNELS[params.kernel], params.degree, float(gamma),
                                      float(params.coef0), float(params.cost), device, ctypes.byref(self._ctx)))
        mode = {"auto": _abi.KP_AUTO, "pairwise": _abi.KP_PAIRWISE, "factored": _abi.KP_FACTORED}[kp_mode]
        if mode != _abi.KP_AUTO:
            self._check(L.plssvm_mi_set_option(self._ctx, _abi.OPT_KP_MODE, mode))
        if rbf_form:  # 1 = direct RBF pair form on sparse data, see PLSSVM_MI_OPT_RBF_FORM
            self._check(L.plssvm_mi_set_option(self._ctx, _abi.OPT_RBF_FORM, rbf_form))
        algo = {"auto": _abi.SPARSE_AUTO, "pattern": _abi.SPARSE_PATTERN, "expansion": _abi.SPARSE_EXPANSION,
                "dense": _abi.SPARSE_DENSE, "onthefly": _abi.SPARSE_ONTHEFLY}[sparse_algo]
        if algo != _abi.SPARSE_AUTO:  # sparse poly/rbf K·p algorithm, see PLSSVM_MI_OPT_SPARSE_ALGO
            self._check(L.plssvm_mi_set_option(self._ctx, _abi.OPT_SPARSE_ALGO, algo))
        if cg_variant is not None:  # "reference" | "one_reduction" | "auto", see PLSSVM_MI_OPT_CG_VARIANT
            v = {"reference": 0, "one_reduction": 1, "auto": 2}[cg_variant]
            self._check(L.plssvm_mi_set_option(self._ctx, _abi.OPT_CG_VARIANT, v))
        if sim_rank is not None:  # (rank, world): single-GPU test hook, see PLSSVM_MI_OPT_SIM_RANK
            self._check(L.plssvm_mi_set_option(self._ctx, _abi.OPT_SIM_RANK, sim_rank[0] | (sim_rank[1] << 16)))
        if exchange is not None:  # host-staged group: fn(numpy buffer, op) combines in place (torch_exchange)
            self._xchg = _abi.EXCHANGE_FN(self._exchange_cb(exchange, world_size))
            self._check(L.plssvm_mi_comm_init_host(self._ctx, rank, world_size, self._xchg, None))
        elif world_size > 1 or uid is not None:  # a single-rank group (uid given) also runs its collectives on RCCL
            if uid is None:
                raise ValueError("world_size > 1 needs the group's unique id (rank 0: plssvm_sparse_fp22_amd.unique_id())")
            self._uid = ctypes.create_string_buffer(uid, _abi.UNIQUE_ID_BYTES)
            self._check(L.plssvm_mi_comm_init(self._ctx, rank, world_size, self._uid))
        self.world_size = world_size
        self.rank = rank
        self.QA_cost = None
        self.w = None
        self.alpha = None
        self.bias = None
        self.trace = None
        self.iters = None
        self._on_device = False

    @staticmethod
    def _exchange_cb(exchange, world_size):
        # exchange(buf, op) must be collective even when it fails: torch_exchange flags a local failure
        # inside its collective so every rank raises (a custom exchange that raises before its collective
        # leaves the peers waiting in theirs)
        def cb(ptr, count, real_bytes, op, user):
            try:
                n = count * (world_size if op == _abi.XCHG_ALLGATHER else 1)
                ct = ctypes.c_float if real_bytes == 4 else ctypes.c_double
                buf = np.ctypeslib.as_array((ct * n).from_address(ptr))
                exchange(buf, op)
                return 0
            except Exception:  # noqa: BLE001 — reported as PLSSVM_MI_ERR_RCCL by the library
                import traceback

                traceback.print_exc()
                return -1

        return cb

    # ---- lifetime ----
    def close(self):
        if getattr(self, "_ctx", None) and self._ctx.value:
            _abi.lib().plssvm_mi_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _check(self, code):
        _abi.check(code, self._ctx)

    @property
    def m(self):
        return self.num_data_points - 1

    # ---- gpu_csvm hot-path surface ----
    def setup_data_on_device(self):
        L = _abi.lib()
        p = self.params
        if p.data is not None:
            X = np.ascontiguousarray(p.data, dtype=self.dtype)
            self._check(L.plssvm_mi_setup_dense(self._ctx, _ptr(X), X.shape[0], X.shape[1]))
        elif p.csr is not None:
            rowptr, col, val, n, d = p.csr
            rowptr = np.ascontiguousarray(rowptr, dtype=np.int64)
            col = np.ascontiguousarray(col, dtype=np.int32)
            val = np.ascontiguousarray(val, dtype=np.uint32 if p.val_fmt == _abi.VAL_FP22 else self.dtype)
            self._check(L.plssvm_mi_setup_csr(self._ctx, _ptr(rowptr), _ptr(col), _ptr(val), p.val_fmt, n, d))
        else:
            row, col, val, n, d = p.coo
            row = np.ascontiguousarray(row, dtype=np.int64)
            col = np.ascontiguousarray(col, dtype=np.int32)
            val = np.ascontiguousarray(val, dtype=np.uint32 if p.val_fmt == _abi.VAL_FP22 else self.dtype)
            self._check(L.plssvm_mi_setup_coo(self._ctx, _ptr(row), _ptr(col), _ptr(val), p.val_fmt, row.size, n, d))
        self._on_device = True

    def generate_q(self):
        q = np.zeros(max(self.m, 1), dtype=self.dtype)
        qa = ctypes.c_double()
        self._check(_abi.lib().plssvm_mi_generate_q(self._ctx, _ptr(q), ctypes.byref(qa)))
        self.QA_cost = self.dtype.type(qa.value)
        return q[: self.m]

    def set_cost(self, cost):
        self._check(_abi.lib().plssvm_mi_set_cost(self._ctx, float(cost)))

    def set_QA_cost(self, qa):
        self._check(_abi.lib().plssvm_mi_set_qa_cost(self._ctx, float(qa)))
        self.QA_cost = self.dtype.type(qa)

    def run_device_kernel(self, q, ret, d, add):
        """ret += add * Q~ d (run_device_kernel + device_reduction); q=None uses the device q."""
        assert ret.dtype == self.dtype and ret.flags.c_contiguous
        qq = None if q is None else np.ascontiguousarray(q, dtype=self.dtype)
        dd = np.ascontiguousarray(d, dtype=self.dtype)
        self._check(_abi.lib().plssvm_mi_kp(self._ctx, _ptr(qq), _ptr(dd), _ptr(ret), float(add)))
        return ret

    def kp_part(self, p, part="kernel"):
        """Test hook (plssvm_mi_kp_part): 'kernel' = sum_j k(x_i, x_j) p_j; 'overlap' = the sparse
        poly/rbf overlap sum (the per-pair work of the sparse kernels only); 'remainder' = the kernel
        expansion's stored remainder stream alone (pairs sharing >= 2 features, in the stored layout)."""
        pp = np.ascontiguousarray(p, dtype=self.dtype)
        out = np.zeros(max(self.m, 1), dtype=self.dtype)
        code = {"kernel": _abi.PART_KERNEL, "overlap": _abi.PART_OVERLAP, "remainder": _abi.PART_REMAINDER}[part]
        self._check(_abi.lib().plssvm_mi_kp_part(self._ctx, _ptr(pp), _ptr(out), code))
        return out[: self.m]

    def solver_CG(self, b, imax, eps, q=None):
        b = np.ascontiguousarray(b, dtype=self.dtype)
        qq = None if q is None else np.ascontiguousarray(q, dtype=self.dtype)
        x = np.zeros(max(self.m, 1), dtype=self.dtype)
        trace = np.full(imax + 1, np.nan)
        it = ctypes.c_int64()
        self._check(_abi.lib().plssvm_mi_solve_cg(self._ctx, _ptr(b), _ptr(qq), imax, float(eps), _ptr(x),
                                                  _ptr(trace), ctypes.byref(it)))
        self.iters = it.value
        self.trace = trace[: it.value + 1]
        return x[: self.m]

    def learn(self, imax=-1):
        """csvm<T>::learn(): setup, q, QA_cost, CG with imax = num_features, bias, alpha[m] = -sum."""
        if self.params.labels is None:
            raise ValueError("No labels given for training! Maybe the data is only usable for prediction?")
        if not self._on_device:
            self.setup_data_on_device()
        y = np.ascontiguousarray(self.params.labels, dtype=self.dtype)
        alpha = np.zeros(self.num_data_points, dtype=self.dtype)
        bias = ctypes.c_double()
        im = self.num_features if imax < 0 else imax
        trace = np.full(im + 1, np.nan)
        it = ctypes.c_int64()
        self._check(_abi.lib().plssvm_mi_learn(self._ctx, _ptr(y), im, float(self.params.epsilon), _ptr(alpha),
                                               ctypes.byref(bias), _ptr(trace), ctypes.byref(it)))
        self.alpha = alpha
        self.bias = self.dtype.type(bias.value)
        self.rho = -self.bias
        self.iters = it.value
        self.trace = trace[: it.value + 1]
        return self

    # ---- model use: update_w / predict / accuracy (csvm.hpp:123-178, gpu_csvm.cpp:52-127,327-350) ----
    def _model(self, alpha, bias):
        alpha = self.alpha if alpha is None else alpha
        bias = self.bias if bias is None else bias
        if alpha is None:
            raise ValueError("No alphas provided for prediction!")
        alpha = np.ascontiguousarray(alpha, dtype=self.dtype)
        if alpha.shape != (self.num_data_points,):
            raise ValueError(f"alpha must have {self.num_data_points} entries")
        if not self._on_device:
            self.setup_data_on_device()
        return alpha, float(0.0 if bias is None else bias)

    def update_w(self, alpha=None):
        """w = sum_i alpha_i x_i over all points (the linear kernel's model vector)."""
        alpha, _ = self._model(alpha, 0.0)
        w = np.zeros(max(self.num_features, 1), dtype=self.dtype)
        self._check(_abi.lib().plssvm_mi_update_w(self._ctx, _ptr(alpha), _ptr(w)))
        self.w = w[: self.num_features]
        return self.w

    def predict_values(self, points, alpha=None, bias=None, val_fmt=None):
        """Decision values bias + sum_i alpha_i k(x_i, z) for dense points [np][d] or a CSR tuple
        (rowptr, col, val, np, d); defaults to the learned alpha and bias."""
        alpha, b = self._model(alpha, bias)
        L = _abi.lib()
        if isinstance(points, tuple):
            rowptr, col, val, npts, d = points
            fmt = _abi.VAL_REAL if val_fmt is None else val_fmt
            rowptr = np.ascontiguousarray(rowptr, dtype=np.int64)
            col = np.ascontiguousarray(col, dtype=np.int32)
            val = np.ascontiguousarray(val, dtype=np.uint32 if fmt == _abi.VAL_FP22 else self.dtype)
            out = np.zeros(max(npts, 1), dtype=self.dtype)
            self._check(L.plssvm_mi_predict_csr(self._ctx, _ptr(alpha), b, _ptr(rowptr), _ptr(col), _ptr(val), fmt,
                                                npts, d, _ptr(out)))
            return out[:npts]
        Z = np.ascontiguousarray(points, dtype=self.dtype)
        if Z.ndim != 2:
            raise ValueError("points must be a 2-D array [np][d]")
        out = np.zeros(max(Z.shape[0], 1), dtype=self.dtype)
        self._check(L.plssvm_mi_predict_dense(self._ctx, _ptr(alpha), b, _ptr(Z), Z.shape[0], Z.shape[1], _ptr(out)))
        return out[: Z.shape[0]]

    def predict(self, points, alpha=None, bias=None, val_fmt=None):
        """Predicted labels (+-1): plssvm::operators::sign of the decision values (operators.hpp:174-177)."""
        v = self.predict_values(points, alpha, bias, val_fmt)
        return np.where(v > 0, self.dtype.type(1), self.dtype.type(-1))

    def accuracy(self, points=None, labels=None):
        """csvm::accuracy: fraction of correctly predicted labels (defaults: the training data)."""
        if points is None:
            points = self.params.data if self.params.data is not None else self.params.csr
            labels = self.params.labels
        if labels is None:
            raise ValueError("No labels given for the accuracy calculation!")
        pred = self.predict(points)
        if pred.shape[0] != len(labels):
            raise ValueError("the number of points to predict and correct labels mismatch")
        return float(np.mean(pred == np.asarray(labels, dtype=self.dtype)))

    # ---- stepwise CG + timing (bench.py) ----
    def cg_begin(self, b, q=None, eps=None):
        b = np.ascontiguousarray(b, dtype=self.dtype)
        qq = None if q is None else np.ascontiguousarray(q, dtype=self.dtype)
        d0 = ctypes.c_double()
        e = self.params.epsilon if eps is None else eps
        self._check(_abi.lib().plssvm_mi_cg_begin(self._ctx, _ptr(b), _ptr(qq), float(e), ctypes.byref(d0)))
        return d0.value

    def cg_step(self, n, force=False):
        it = ctypes.c_int64()
        conv = ctypes.c_int()
        self._check(_abi.lib().plssvm_mi_cg_step(self._ctx, n, 1 if force else 0, ctypes.byref(it),
                                                 ctypes.byref(conv)))
        return it.value, bool(conv.value)

    def cg_result(self, trace_len=0):
        x = np.zeros(max(self.m, 1), dtype=self.dtype)
        trace = np.full(max(trace_len, 1), np.nan)
        it = ctypes.c_int64()
        self._check(_abi.lib().plssvm_mi_cg_result(self._ctx, _ptr(x), _ptr(trace), trace_len, ctypes.byref(it)))
        return x[: self.m], trace[: min(trace_len, it.value + 1)], it.value

    def time_kp(self, reps=5):
        a, b = ctypes.c_double(), ctypes.c_double()
        self._check(_abi.lib().plssvm_mi_time_kp(self._ctx, reps, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    def info(self):
        inf = _abi.Info()
        self._check(_abi.lib().plssvm_mi_get_info(self._ctx, ctypes.byref(inf)))
        return {k: getattr(inf, k) for k, _ in _abi.Info._fields_}

    def get_num_devices(self):
        return self.world_size
