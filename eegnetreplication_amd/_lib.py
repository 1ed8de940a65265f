"""ctypes binding of libeegnet_hip.so (C-ABI declared in include/eegnet_abi.h).

The library is built in-tree by ``__graft_entry__.build()`` (hipcc --offload-arch=gfx950).  There is
no fallback: if the library is missing or a call fails, a RuntimeError says so.
"""

from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# EEGNET_LIB selects a variant built beside it (e.g. libeegnet_hip_trace.so for tools/trace_step.py)
LIB_PATH = os.path.join(_HERE, os.environ.get("EEGNET_LIB", "libeegnet_hip.so"))

_lock = threading.Lock()
_lib = None


class Fold(ctypes.Structure):
    """Mirror of ``eegnet_fold`` (include/eegnet_abi.h): one model of a fold-indexed step."""
    _fields_ = [(n, ctypes.c_void_p) for n in ("params", "bn_buffers", "num_batches_tracked", "x", "labels",
                                              "grads", "adam_state", "step", "losses", "ws", "perm")] + \
               [("seed", ctypes.c_uint64), ("xstat", ctypes.c_void_p)]


ABI_VERSION = 5     # include/eegnet_abi.h EEGNET_ABI_VERSION: the struct layouts these mirrors follow


class Dims(ctypes.Structure):
    """Mirror of ``eegnet_dims`` (include/eegnet_abi.h)."""
    _fields_ = [
        ("B", ctypes.c_int), ("C", ctypes.c_int), ("T", ctypes.c_int),
        ("F1", ctypes.c_int), ("D", ctypes.c_int), ("K1", ctypes.c_int),
        ("p_drop", ctypes.c_float), ("bn_eps", ctypes.c_float), ("bn_momentum", ctypes.c_float),
        ("x_pitch", ctypes.c_int),
    ]


_vp = ctypes.c_void_p
_SIGS = {
    "eegnet_param_count": (ctypes.c_int, [ctypes.POINTER(Dims), ctypes.POINTER(ctypes.c_int64)]),
    "eegnet_workspace_bytes": (ctypes.c_int, [ctypes.POINTER(Dims), ctypes.POINTER(ctypes.c_size_t)]),
    "eegnet_forward_train": (ctypes.c_int, [ctypes.POINTER(Dims), _vp, _vp, _vp, _vp, _vp,
                                            ctypes.c_uint64, ctypes.c_uint64, _vp, _vp, _vp, _vp]),
    "eegnet_backward": (ctypes.c_int, [ctypes.POINTER(Dims), _vp, _vp, _vp, _vp, _vp, _vp,
                                       ctypes.c_uint64, ctypes.c_uint64, _vp, _vp, _vp, _vp,
                                       ctypes.c_int]),
    "eegnet_clamp_grads": (ctypes.c_int, [ctypes.POINTER(Dims), _vp, _vp]),
    "eegnet_forward_eval": (ctypes.c_int, [ctypes.POINTER(Dims), _vp, _vp, _vp, _vp, _vp]),
    "eegnet_forward_eval_bf16": (ctypes.c_int, [ctypes.POINTER(Dims), _vp, _vp, _vp, _vp, _vp]),
    "eegnet_adam_step": (ctypes.c_int, [ctypes.c_int64, _vp, _vp, _vp, _vp, _vp, ctypes.c_float,
                                        ctypes.c_float, ctypes.c_float, ctypes.c_float, _vp]),
    "eegnet_train_step": (ctypes.c_int, [ctypes.POINTER(Dims), _vp, _vp, _vp, _vp, ctypes.c_uint64,
                                         ctypes.c_uint64, _vp, _vp, _vp, ctypes.c_float,
                                         ctypes.c_float, ctypes.c_float, ctypes.c_float, _vp, _vp,
                                         _vp, _vp, ctypes.c_int, _vp]),
    "eegnet_train_stage": (ctypes.c_int, [ctypes.POINTER(Dims), ctypes.c_int, ctypes.c_int64, _vp, _vp, _vp,
                                          _vp, ctypes.c_uint64, ctypes.c_uint64, _vp, _vp, _vp,
                                          ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                          _vp, _vp, _vp, ctypes.c_int, _vp]),
    "eegnet_stage_sums": (ctypes.c_int, [ctypes.POINTER(Dims), ctypes.c_int, ctypes.POINTER(ctypes.c_size_t),
                                         ctypes.POINTER(ctypes.c_int)]),
    "eegnet_train_step_folds": (ctypes.c_int, [ctypes.POINTER(Dims), ctypes.c_int, _vp, ctypes.c_int64,
                                               ctypes.c_int64, ctypes.c_uint64, ctypes.c_float,
                                               ctypes.c_float, ctypes.c_float, ctypes.c_float, _vp]),
    "eegnet_profile_enable": (ctypes.c_int, [ctypes.c_int]),
    "eegnet_profile_collect": (ctypes.c_int, [ctypes.c_char_p, _vp, _vp, ctypes.c_int, _vp]),
    "eegnet_trace_enable": (ctypes.c_int, [_vp]),
    "eegnet_trace_bytes": (ctypes.c_size_t, []),
    "eegnet_dims_bytes": (ctypes.c_size_t, []),
    "eegnet_wide_spec": (ctypes.c_int, [ctypes.POINTER(Dims)]),
    "eegnet_x_pitch": (ctypes.c_int, [ctypes.POINTER(Dims)]),
    "eegnet_x_stats_width": (ctypes.c_int, [ctypes.POINTER(Dims)]),
    "eegnet_x_stats": (ctypes.c_int, [ctypes.POINTER(Dims), ctypes.c_int64, _vp, _vp, _vp]),
    "eegnet_fold_bytes": (ctypes.c_size_t, []),
    "eegnet_abi_version": (ctypes.c_int, []),
    "eegnet_last_error": (ctypes.c_char_p, []),
    "eegnet_build_info": (ctypes.c_char_p, []),
}
EXPORTED_SYMBOLS = tuple(_SIGS)


def load(path: str | None = None):
    """Load (once) and return the ctypes handle.  Raises RuntimeError when the .so is missing."""
    global _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise RuntimeError(
                f"libeegnet_hip.so not found at {p}: build it with `python -c 'import "
                f"__graft_entry__ as g; g.build()'` (hipcc --offload-arch=gfx950). There is no "
                f"CPU fallback for the EEGNet HIP path.")
        lib = ctypes.CDLL(p)
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.eegnet_abi_version() != ABI_VERSION:
            raise RuntimeError(f"{p} has struct ABI {lib.eegnet_abi_version()}, this binding {ABI_VERSION}: "
                               f"rebuild it")
        for name, mirror in (("eegnet_dims_bytes", Dims), ("eegnet_fold_bytes", Fold)):
            if getattr(lib, name)() != ctypes.sizeof(mirror):
                raise RuntimeError(f"{p} was built with another {mirror.__name__} layout ({name}() = "
                                   f"{getattr(lib, name)()}, binding {ctypes.sizeof(mirror)}): rebuild it")
        if path is None:
            _lib = lib
        return lib


def check(rc: int, what: str):
    if rc != 0:
        msg = load().eegnet_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed (rc={rc}): {msg}")


def dims(B, C, T, F1=8, D=2, K1=32, p=0.5, eps=1e-5, momentum=0.1, x_pitch=0) -> Dims:
    return Dims(int(B), int(C), int(T), int(F1), int(D), int(K1), float(p), float(eps),
                float(momentum), int(x_pitch))


def param_count(d: Dims) -> int:
    out = ctypes.c_int64(0)
    check(load().eegnet_param_count(ctypes.byref(d), ctypes.byref(out)), "eegnet_param_count")
    return int(out.value)


def workspace_bytes(d: Dims) -> int:
    out = ctypes.c_size_t(0)
    check(load().eegnet_workspace_bytes(ctypes.byref(d), ctypes.byref(out)),
          "eegnet_workspace_bytes")
    return int(out.value)


KERNEL_IDS = ("k_pass_a", "k_pass_b", "k_pass_c", "k_pass_d", "k_pass_e", "k_adam", "k_infer",
              "memset_tickets", "k_infer_bf16", "k_wpass_a", "k_wpass_b", "k_wpass_b2", "k_wpass_c",
              "k_wpass_d", "k_wpass_e", "k_winfer", "k_coltail", "k_xstats")


def profile_enable(on: bool = True, kernels=None):
    """Bracket launches with hipEvents: every kernel (``kernels=None``) or only the named ones."""
    mask = 0
    if on:
        mask = -1 if kernels is None else sum(1 << KERNEL_IDS.index(k) for k in kernels)
    check(load().eegnet_profile_enable(mask), "eegnet_profile_enable")


def profile_collect() -> dict:
    """{kernel name: (launches, total device ms)} since the last collect."""
    cap = 32
    names = ctypes.create_string_buffer(32 * cap)
    counts = (ctypes.c_int * cap)()
    tot = (ctypes.c_double * cap)()
    n = ctypes.c_int(0)
    check(load().eegnet_profile_collect(names, ctypes.cast(counts, ctypes.c_void_p),
                                        ctypes.cast(tot, ctypes.c_void_p), cap,
                                        ctypes.cast(ctypes.pointer(n), ctypes.c_void_p)),
          "eegnet_profile_collect")
    out = {}
    for i in range(n.value):
        nm = names.raw[32 * i:32 * i + 32].split(b"\0", 1)[0].decode()
        out[nm] = (int(counts[i]), float(tot[i]))
    return out
