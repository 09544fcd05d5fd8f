"""ctypes binding of libgnot_hip.so (C ABI: include/gnot_hip.h).

This is the reference-side binding a maintainer adds to aloe101/GNOT-Replication (see
INTEGRATION.md): plain pointers and sizes, one `gnot_plan` per model.  There is deliberately no
fallback: if the shared library is missing or cannot be loaded, importing the product path fails.
"""
import ctypes
import hashlib
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(_HERE)                      # gnot-replication_amd/
LIB_PATH = os.path.join(PKG_ROOT, "lib", "libgnot_hip.so")
CSRC = os.path.join(PKG_ROOT, "csrc")


class GnotConfig(ctypes.Structure):
    """gnot_config: the 12 GNOT constructor arguments (reference model.py:143)."""
    _fields_ = [(n, ctypes.c_int) for n in (
        "input_dim", "theta_dim", "input_func_dim", "out_dim", "n_attn_layers", "n_attn_hidden_dim",
        "n_mlp_num_layers", "n_mlp_hidden_dim", "n_input_hidden_dim", "n_expert", "n_head",
        "n_input_functions")]


EXPORTS = [
    "gnot_plan_create", "gnot_plan_destroy", "gnot_plan_num_linears", "gnot_plan_linear_dims",
    "gnot_plan_bind_params", "gnot_plan_set_batch", "gnot_plan_workspace_bytes",
    "gnot_plan_bind_workspace", "gnot_plan_bind_workspace_async", "gnot_plan_set_moe_recompute", "gnot_plan_set_precision",
    "gnot_plan_set_input_grads", "gnot_input_grads", "gnot_plan_grad_offsets", "gnot_pack_weights", "gnot_forward",
    "gnot_backward", "gnot_profile_enable", "gnot_profile_read", "gnot_debug_buffer", "gnot_last_error",
    "gnot_version", "gnot_plan_set_shard", "gnot_plan_set_grad_comm", "gnot_shard_range", "gnot_shard_exchange",
    "gnot_rel_l2_work_floats", "gnot_rel_l2_loss", "gnot_adamw_step",
]

# gnot_comm callbacks (include/gnot_hip.h)
ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p)
ALLTOALLV_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64),
                                ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64), ctypes.c_void_p)


class GnotComm(ctypes.Structure):
    _fields_ = [("user", ctypes.c_void_p), ("allreduce_sum", ALLREDUCE_FN), ("alltoallv", ALLTOALLV_FN)]


def build(jobs=8, quiet=True):
    """Compile the HIP sources for gfx950 into lib/libgnot_hip.so (hipcc cross-compiles, no GPU)."""
    cmd = ["make", "-C", CSRC, f"-j{jobs}"]
    res = subprocess.run(cmd, capture_output=quiet, text=True)
    if res.returncode != 0:
        raise RuntimeError("building libgnot_hip.so failed:\n" + (res.stdout or "") + (res.stderr or ""))
    return LIB_PATH


# every file the library's code depends on (csrc/Makefile's SRCS, its headers and its flags)
SOURCES = ["Makefile", "gnot_common.h", "gnot_kernels.h", "x6_core.h", "pack.hip", "linear.hip", "linear2.hip",
           "chain.hip", "chain2.hip", "chainw.hip", "wgrad.hip", "state.hip", "attn.hip", "attn_mfma.hip", "misc.hip",
           "train.hip", "engine.cpp"]


def source_hash():
    """16 hex digits of sha256 over the library's sources (SOURCES + include/gnot_hip.h): the identity of
    the kernels a measurement was taken on.  profiles/pmc_traffic.json stores it per entry, and bench.py
    reports an entry's traffic only for the same hash (a changed kernel or launch sequence prints null).
    None when an experiment build is loaded instead (GNOT_LIB)."""
    if os.environ.get("GNOT_LIB"):
        return None
    h = hashlib.sha256()
    for f in [os.path.join(CSRC, n) for n in SOURCES] + [os.path.join(os.path.dirname(PKG_ROOT), "include", "gnot_hip.h")]:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def _declare(lib):
    P = ctypes.c_void_p
    i32, i64, sz = ctypes.c_int, ctypes.c_int64, ctypes.c_size_t
    lib.gnot_plan_create.argtypes = [ctypes.POINTER(GnotConfig), ctypes.POINTER(P)]
    lib.gnot_plan_destroy.argtypes = [P]
    lib.gnot_plan_destroy.restype = None
    lib.gnot_plan_num_linears.argtypes = [P]
    lib.gnot_plan_linear_dims.argtypes = [P, ctypes.POINTER(ctypes.c_int32)]
    lib.gnot_plan_bind_params.argtypes = [P, ctypes.POINTER(P), ctypes.POINTER(P)]
    lib.gnot_plan_set_batch.argtypes = [P, i32, ctypes.POINTER(i64), ctypes.POINTER(i64), i32]
    lib.gnot_plan_workspace_bytes.argtypes = [P]
    lib.gnot_plan_workspace_bytes.restype = sz
    lib.gnot_plan_bind_workspace.argtypes = [P, P, sz]
    lib.gnot_plan_bind_workspace_async.argtypes = [P, P, sz, P]
    lib.gnot_plan_set_moe_recompute.argtypes = [P, ctypes.c_int]
    lib.gnot_plan_set_precision.argtypes = [P, ctypes.c_int]
    lib.gnot_plan_set_input_grads.argtypes = [P, ctypes.c_int]
    lib.gnot_input_grads.argtypes = [P, P, P, ctypes.POINTER(P), P]
    lib.gnot_plan_grad_offsets.argtypes = [P, ctypes.POINTER(i64)]
    lib.gnot_pack_weights.argtypes = [P, P]
    lib.gnot_forward.argtypes = [P, P, P, ctypes.POINTER(P), P, P]
    lib.gnot_backward.argtypes = [P, P, P]
    lib.gnot_profile_enable.argtypes = [P, ctypes.c_char_p]
    lib.gnot_profile_read.argtypes = [P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(i64),
                                      ctypes.POINTER(ctypes.c_double)]
    lib.gnot_debug_buffer.argtypes = [P, ctypes.c_char_p, ctypes.POINTER(P), ctypes.POINTER(i64)]
    lib.gnot_plan_set_shard.argtypes = [P, i32, i32, i32, ctypes.POINTER(i64), ctypes.POINTER(GnotComm)]
    lib.gnot_plan_set_grad_comm.argtypes = [P, ctypes.POINTER(GnotComm)]
    lib.gnot_shard_range.argtypes = [i64, i32, i32, ctypes.POINTER(i64), ctypes.POINTER(i64)]
    lib.gnot_shard_exchange.argtypes = [i32, ctypes.POINTER(i64), i32, i32, i32, i32, ctypes.POINTER(i64),
                                        ctypes.POINTER(i64), ctypes.POINTER(i64), i64, ctypes.POINTER(i64)]
    lib.gnot_rel_l2_work_floats.argtypes = [ctypes.POINTER(i64), i32, i32]
    lib.gnot_rel_l2_work_floats.restype = sz
    lib.gnot_rel_l2_loss.argtypes = [P, P, P, ctypes.POINTER(i64), i32, i32, P, P, P, P]
    lib.gnot_adamw_step.argtypes = [P, P, P, P, i64, P, P]
    lib.gnot_last_error.restype = ctypes.c_char_p
    lib.gnot_last_error.argtypes = []
    lib.gnot_version.restype = ctypes.c_char_p
    lib.gnot_version.argtypes = []
    return lib


_LIB = None


def load():
    """Load libgnot_hip.so (raises if it is missing: there is no CPU fallback)."""
    global _LIB
    if _LIB is None:
        path = os.environ.get("GNOT_LIB", LIB_PATH)      # experiment builds of the same library
        if not os.path.exists(path):
            raise ImportError(f"{path} not found: build it with `make -C {CSRC}` "
                              "(gnot_amd has no CPU fallback)")
        _LIB = _declare(ctypes.CDLL(path))
    return _LIB


def check(rc):
    if rc != 0:
        raise RuntimeError(f"libgnot_hip error {rc}: {load().gnot_last_error().decode()}")
