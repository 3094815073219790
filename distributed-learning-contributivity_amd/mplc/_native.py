"""ctypes binding of libmplc_hip.so (the C ABI declared in include/mplc_hip.h).

The HIP library is the product path: every coalition-evaluation kernel runs through it.  There is no
CPU fallback; if the library is missing or fails to load, calls raise RuntimeError.
"""
import ctypes
import os
import threading

# MPLC_LIB_PATH: another build of the same library (tests/test_native_sanitize.py loads the host-ASan build)
_LIB_PATH = os.environ.get("MPLC_LIB_PATH") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib",
                                                            "libmplc_hip.so")
_lock = threading.Lock()
_lib = None

c_int, c_int64, c_uint64, c_size_t, c_void_p = (ctypes.c_int, ctypes.c_int64, ctypes.c_uint64, ctypes.c_size_t,
                                                ctypes.c_void_p)

# name -> (restype, argtypes).  Must list every symbol include/*.h declares (tests check both ways).
SIGNATURES = {
    "mplc_abi_version": (c_int, []),
    "mplc_shapley_workspace_bytes": (c_size_t, [c_int, c_uint64]),
    "mplc_shapley_partial": (c_int, [c_void_p, c_uint64, c_uint64, c_int, c_void_p, c_void_p, c_size_t, c_void_p]),
    "mplc_shapley_finalize": (c_int, [c_void_p, c_int, c_void_p, c_void_p]),
    "mplc_shapley_exact": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_size_t, c_void_p]),
    "mplc_fedavg_aggregate": (c_int, [c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_int, c_int64, c_void_p,
                                      c_int64, c_int, c_void_p]),
    "mplc_fedavg_aggregate_bcast_skip": (c_int, [c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_int, c_int64,
                                                 c_void_p, c_int64, c_int64, c_int64, c_void_p]),
    "mplc_fedavg_aggregate_skip": (c_int, [c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_int, c_int64, c_void_p,
                                           c_int64, c_int64, c_int64, c_void_p]),
    # Monte-Carlo Shapley permutation walks over a dense table (csrc/mc_shapley.hip)
    "mplc_tmc_walk": (c_int, [c_void_p, c_int, c_void_p, c_int, ctypes.c_double, ctypes.c_double, c_int, c_void_p,
                              c_void_p, c_void_p, c_void_p, c_void_p]),
    "mplc_tmc_moments_workspace_bytes": (c_size_t, [c_int, c_int]),
    "mplc_tmc_moments": (c_int, [c_void_p, c_int, c_void_p, c_uint64, c_uint64, c_int, ctypes.c_double,
                                 ctypes.c_double, c_int, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    # batched CNN trainer (include/mplc_hip_cnn.h); mplc.cnn re-binds train_step with its struct type
    "mplc_cnn_stride": (c_int, []),
    "mplc_cnn_wgrad_split_samples": (c_int, []),
    "mplc_cnn_layout": (c_int64, [c_int]),
    "mplc_cnn_init_params": (c_int, [c_void_p, c_int64, c_void_p, c_int, c_void_p]),
    "mplc_cnn_copy_rows": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_int, c_void_p]),
    "mplc_cnn_train_step": (c_int, [c_void_p, c_void_p]),
    "mplc_seq_snapshot": (c_int, [c_void_p, c_int64, c_int64, c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int,
                                  c_int, c_void_p, c_void_p, c_void_p]),
    "mplc_cnn_evaluate": (c_int, [c_void_p, c_int64, c_int, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p,
                                  c_void_p, c_void_p, c_void_p, c_void_p]),
    # batched CIFAR10 CNN trainer (include/mplc_hip_cifar.h); mplc.cifar re-binds train_step with its struct
    "mplc_cifar_stride": (c_int, []),
    "mplc_cifar_wgrad_split_samples": (c_int, []),
    "mplc_cifar_layout": (c_int64, [c_int]),
    "mplc_cifar_init_params": (c_int, [c_void_p, c_int64, c_void_p, c_int, c_void_p]),
    "mplc_cifar_train_step": (c_int, [c_void_p, c_void_p]),
    "mplc_cifar_eval_workspace_floats": (c_int64, [c_int, c_int]),
    "mplc_cifar_evaluate": (c_int, [c_void_p, c_int64, c_int, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p,
                                    c_void_p, c_void_p]),
    # batched FedAvg logistic regression (Titanic)
    "mplc_lr_fedavg": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p,
                               c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_int,
                               c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int64,
                               c_void_p]),
}

ABI_VERSION = 4  # include/mplc_hip.h MPLC_ABI_VERSION


def check_layout(query, expected, what):
    """Compare the library's layout items (query(i) for i, value in expected) with the host's constants."""
    bad = {name: (int(query(i)), v) for name, (i, v) in expected.items() if int(query(i)) != int(v)}
    if bad:
        raise RuntimeError(f"libmplc_hip.so {what} layout mismatch (library, host): {bad}; rebuild the library")


def lib_path():
    return _LIB_PATH


def lib():
    """Load (once) and return the ctypes handle; raise RuntimeError if the HIP library is unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(_LIB_PATH):
            raise RuntimeError(f"libmplc_hip.so not found at {_LIB_PATH}: run __graft_entry__.build() "
                               "(or distributed-learning-contributivity_amd/build_native.py) first")
        try:
            h = ctypes.CDLL(_LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        except OSError as e:
            raise RuntimeError(f"failed to load {_LIB_PATH}: {e}") from e
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(h, name, None)
            if fn is None:
                raise RuntimeError(f"{_LIB_PATH} does not export {name}")
            fn.restype = res
            fn.argtypes = args
        if h.mplc_abi_version() != ABI_VERSION:
            raise RuntimeError("libmplc_hip.so ABI version mismatch; rebuild")
        _lib = h
        return _lib


def register(name, restype, argtypes):
    """Add a signature (used by modules that bind further entry points)."""
    SIGNATURES[name] = (restype, argtypes)
    if _lib is not None:
        fn = getattr(_lib, name)
        fn.restype = restype
        fn.argtypes = argtypes


def check(status, what):
    if status != 0:
        kinds = {-1: "invalid argument", -2: "workspace too small", -3: "unsupported shape"}
        msg = kinds.get(status, f"hipError_t {status}")
        raise RuntimeError(f"{what} failed: {msg}")


def ptr(t):
    """Raw device pointer of a torch tensor (None -> NULL)."""
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream_handle(device=None):
    """hipStream_t of torch's current stream on `device` as a void* for the C ABI."""
    import torch
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
