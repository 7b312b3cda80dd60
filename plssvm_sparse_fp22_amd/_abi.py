"""ctypes binding of libplssvm_mi355x.so (C ABI: include/plssvm_mi355x.h).

The shared library is built in-tree by ``__graft_entry__.build()`` (``make -C
plssvm_sparse_fp22_amd/csrc``). There is no fallback: if the library is missing or cannot be
loaded, :func:`lib` raises, so nothing silently runs on the CPU.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# PLSSVM_MI_LIB: an alternative build of the same library (A/B measurements of compile-time variants,
# tools/variants.sh); never a CPU stand-in — every build behind this name is the gfx950 HIP path
LIB_PATH = os.environ.get("PLSSVM_MI_LIB") or os.path.join(_HERE, "libplssvm_mi355x.so")

OK = 0
ERR = {-1: "ERR_ARG", -2: "ERR_HIP", -3: "ERR_RCCL", -4: "ERR_OOM", -5: "ERR_UNSUPPORTED", -6: "ERR_STATE",
       -7: "ERR_NODEV"}
KERNELS = {"linear": 0, "polynomial": 1, "poly": 1, "rbf": 2}
VAL_REAL, VAL_FP22 = 0, 1
KP_AUTO, KP_PAIRWISE, KP_FACTORED = 0, 1, 2
OPT_KP_MODE = 1
UNIQUE_ID_BYTES = 128

# every symbol include/plssvm_mi355x.h declares (checked by tests/test_abi.py)
EXPORTS = (
    "plssvm_mi_device_count", "plssvm_mi_create", "plssvm_mi_destroy", "plssvm_mi_last_error",
    "plssvm_mi_set_option", "plssvm_mi_set_cost", "plssvm_mi_set_qa_cost", "plssvm_mi_get_unique_id",
    "plssvm_mi_comm_init", "plssvm_mi_setup_dense", "plssvm_mi_setup_csr", "plssvm_mi_generate_q", "plssvm_mi_kp",
    "plssvm_mi_solve_cg", "plssvm_mi_cg_begin", "plssvm_mi_cg_step", "plssvm_mi_cg_result", "plssvm_mi_learn",
    "plssvm_mi_time_kp", "plssvm_mi_get_info", "plssvm_mi_partition",
    "plssvm_mi_update_w", "plssvm_mi_predict_dense", "plssvm_mi_predict_csr", "plssvm_mi_setup_coo",
    "plssvm_mi_comm_init_host", "plssvm_mi_kp_part", "plssvm_mi_set_progress", "plssvm_mi_comm_abort",
)
OPT_SIM_RANK = 2
OPT_RBF_FORM = 3
OPT_SPARSE_ALGO = 4
OPT_CG_VARIANT = 5
SPARSE_AUTO, SPARSE_PATTERN, SPARSE_EXPANSION, SPARSE_DENSE, SPARSE_ONTHEFLY = 0, 1, 2, 3, 4
PART_KERNEL, PART_OVERLAP, PART_REMAINDER = 0, 1, 2
XCHG_ALLREDUCE, XCHG_ALLGATHER = 0, 1
# int fn(void *buf, int64_t count, int real_bytes, int op, void *user)   (plssvm_mi_exchange_fn)
EXCHANGE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                               ctypes.c_void_p)
# void fn(int64_t first, int64_t count, const double *deltas, double target, double batch_ms, void *user)
PROGRESS_FN = ctypes.CFUNCTYPE(None, ctypes.c_int64, ctypes.c_int64, ctypes.POINTER(ctypes.c_double), ctypes.c_double,
                               ctypes.c_double, ctypes.c_void_p)


class Info(ctypes.Structure):
    _fields_ = [(k, ctypes.c_int64) for k in ("n", "d", "m", "n_pad", "d_pad", "nnz", "tiles_total", "tiles_local",
                                              "tile_rows", "tile_cols", "device_bytes", "pairs")] + \
               [(k, ctypes.c_int) for k in ("kp_mode", "rank", "world_size", "real_bytes", "kernel", "is_sparse",
                                            "val_fmt", "rbf_factored")] + [("pair_slots", ctypes.c_int64), ("spmv_bytes", ctypes.c_int64)] + \
               [("rbf_small_args", ctypes.c_int), ("sparse_algo", ctypes.c_int), ("exp_terms", ctypes.c_int),
                ("exp_waves", ctypes.c_int), ("exp_chunks", ctypes.c_int64), ("exp_hbytes", ctypes.c_int),
                ("exp_layout", ctypes.c_int), ("exp_dot2", ctypes.c_int), ("centered", ctypes.c_int),
                ("exp_lt", ctypes.c_int)]


class BackendError(RuntimeError):
    """plssvm::hip::backend_exception equivalent raised for a non-zero ABI return code."""

    def __init__(self, code, msg):
        super().__init__(f"{ERR.get(code, code)}: {msg}")
        self.code = code


_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: build it with __graft_entry__.build() "
                              "(make -C plssvm_sparse_fp22_amd/csrc); there is no CPU fallback")
        L = ctypes.CDLL(LIB_PATH)
        _declare(L)
        _lib = L
    return _lib


def _declare(L):
    P, I64, I, D = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_double
    PP = ctypes.POINTER(ctypes.c_void_p)
    PD, PI64, PI = ctypes.POINTER(D), ctypes.POINTER(I64), ctypes.POINTER(I)
    sig = {
        "plssvm_mi_device_count": ([], I),
        "plssvm_mi_create": ([I, I, I, D, D, D, I, PP], I),
        "plssvm_mi_destroy": ([P], None),
        "plssvm_mi_last_error": ([P], ctypes.c_char_p),
        "plssvm_mi_set_option": ([P, I, I64], I),
        "plssvm_mi_set_cost": ([P, D], I),
        "plssvm_mi_set_qa_cost": ([P, D], I),
        "plssvm_mi_get_unique_id": ([P], I),
        "plssvm_mi_comm_init": ([P, I, I, P], I),
        "plssvm_mi_setup_dense": ([P, P, I64, I64], I),
        "plssvm_mi_setup_csr": ([P, P, P, P, I, I64, I64], I),
        "plssvm_mi_setup_coo": ([P, P, P, P, I, I64, I64, I64], I),
        "plssvm_mi_generate_q": ([P, P, PD], I),
        "plssvm_mi_kp": ([P, P, P, P, D], I),
        "plssvm_mi_solve_cg": ([P, P, P, I64, D, P, P, PI64], I),
        "plssvm_mi_cg_begin": ([P, P, P, D, PD], I),
        "plssvm_mi_cg_step": ([P, I64, I, PI64, PI], I),
        "plssvm_mi_cg_result": ([P, P, P, I64, PI64], I),
        "plssvm_mi_learn": ([P, P, I64, D, P, PD, P, PI64], I),
        "plssvm_mi_update_w": ([P, P, P], I),
        "plssvm_mi_predict_dense": ([P, P, D, P, I64, I64, P], I),
        "plssvm_mi_predict_csr": ([P, P, D, P, P, P, I, I64, I64, P], I),
        "plssvm_mi_time_kp": ([P, I, PD, PD], I),
        "plssvm_mi_get_info": ([P, ctypes.POINTER(Info)], I),
        "plssvm_mi_partition": ([I64, I, I, PI64], I),
        "plssvm_mi_comm_init_host": ([P, I, I, EXCHANGE_FN, P], I),
        "plssvm_mi_kp_part": ([P, P, P, I], I),
        "plssvm_mi_comm_abort": ([P], I),
        "plssvm_mi_set_progress": ([P, PROGRESS_FN, P], I),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res


def check(code, ctx=None):
    if code != OK:
        msg = lib().plssvm_mi_last_error(ctx)
        raise BackendError(code, msg.decode() if msg else "")
