"""CPU: the C ABI's host code under AddressSanitizer + UndefinedBehaviorSanitizer.

build_native.py --sanitize compiles every csrc/*.hip with -fsanitize=address,undefined on the host pass only
(device code unchanged; GPU sanitizers are not available) into build/asan/libmplc_hip.so.  A child Python
with the ASan runtime preloaded loads that library (MPLC_LIB_PATH) and drives every entry point through its
argument validation and the host-side sizing arithmetic - null pointers, zero / negative / oversized
counts, misaligned shard ranges, short workspaces, inconsistent step structs - each of which must return its
error code before any HIP call.  Any heap/stack overflow, use-after-free, signed overflow, invalid shift or
misaligned access in that host code aborts the child (-fno-sanitize-recover)."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "distributed-learning-contributivity_amd")

CHILD = r'''
import ctypes, sys
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[2])
from mplc import _native
h = _native.lib()
assert _native.lib_path().endswith("build/asan/libmplc_hip.so"), _native.lib_path()
E_ARG, E_WS, E_SHAPE = -1, -2, -3
vp = ctypes.c_void_p
buf = (ctypes.c_double * 64)()
P = ctypes.cast(buf, vp)
# exact Shapley: sizing for every n and shard size, then every invalid call
for n in range(0, 42):
    for cnt in (0, 1, 1 << 16, 1 << min(n, 40), (1 << 40) + 65536):
        h.mplc_shapley_workspace_bytes(n, cnt)
assert h.mplc_shapley_partial(None, 0, 16, 4, P, None, 0, None) == E_ARG
assert h.mplc_shapley_partial(P, 0, 0, 4, P, None, 0, None) == E_ARG
assert h.mplc_shapley_partial(P, 0, 17, 4, P, None, 0, None) == E_ARG          # beyond 2^n
assert h.mplc_shapley_partial(P, 16, 1, 4, P, None, 0, None) == E_ARG          # begin beyond 2^n
assert h.mplc_shapley_partial(P, 0, 1 << 16, 41, P, None, 0, None) == E_ARG    # n > MAX_N
assert h.mplc_shapley_partial(P, 100, 1 << 16, 20, P, P, 8, None) == E_ARG     # not span-aligned
assert h.mplc_shapley_partial(P, 0, 1 << 16, 20, P, P, 8, None) == E_WS        # workspace too small
assert h.mplc_shapley_partial(P, 0, 1 << 16, 20, P, None, 1 << 20, None) == E_WS
assert h.mplc_shapley_finalize(None, 4, P, None) == E_ARG
assert h.mplc_shapley_finalize(P, 0, P, None) == E_ARG
assert h.mplc_shapley_exact(P, 0, P, P, 64, None) == E_ARG
assert h.mplc_shapley_exact(P, 20, P, P, 64, None) == E_WS
# FedAvg aggregation
assert h.mplc_fedavg_aggregate_bcast_skip(P, 64, P, P, P, 1, 16, None, 64, 0, 8, None) == E_ARG
# Monte-Carlo walks
for n in range(0, 34):
    for k in (0, 1, 1000):
        h.mplc_tmc_moments_workspace_bytes(n, k)
assert h.mplc_tmc_walk(None, 4, P, 1, 1.0, 0.05, 0, P, P, P, P, None) == E_ARG
assert h.mplc_tmc_walk(P, 0, P, 1, 1.0, 0.05, 0, P, P, P, P, None) == E_ARG
assert h.mplc_tmc_walk(P, 4, P, 0, 1.0, 0.05, 0, P, P, P, P, None) == E_ARG
assert h.mplc_tmc_walk(P, 4, P, 1, 1.0, 0.05, 1, None, P, P, P, None) == E_ARG
assert h.mplc_tmc_moments(P, 4, P, 0, 0, 4, 1.0, 0.05, 0, None, None, P, 0, None) == E_ARG  # no output
assert h.mplc_tmc_moments(P, 4, P, 0, 0, 4, 1.0, 0.05, 0, None, P, P, 1, None) == E_WS
# MNIST CNN
assert h.mplc_cnn_stride() == 1199936
assert h.mplc_cnn_init_params(None, 1199936, P, 1, None) == E_ARG
assert h.mplc_cnn_init_params(P, 1199936, P, 0, None) == E_ARG
assert h.mplc_cnn_init_params(P, 1199936, P, 70000, None) == E_ARG
assert h.mplc_cnn_init_params(P, 100, P, 1, None) == E_ARG
assert h.mplc_cnn_copy_rows(P, P, 1199937, P, 1, None) == E_ARG
assert h.mplc_cnn_copy_rows(P, P, 1199936, P, 0, None) == E_ARG
assert h.mplc_cnn_evaluate(P, 1199936, 1, P, P, 10, 10, P, P, P, P, None, None) == E_ARG
assert h.mplc_cnn_evaluate(P, 1199936, 0, P, P, 10, 10, P, P, P, P, P, None) == E_ARG
assert h.mplc_cnn_evaluate(P, 1199936, 1, P, P, 10, 70000, P, P, P, P, P, None) == E_ARG
from mplc import cnn, cifar
cnn._bind()
t = cnn.TrainT()
assert h.mplc_cnn_train_step(ctypes.byref(t), None) == E_ARG                 # n_rep = 0
t.n_rep, t.bmax, t.w2_splits = 1, 27, 1
assert h.mplc_cnn_train_step(ctypes.byref(t), None) == E_SHAPE             # 27 samples need 3 wgrad splits
t.w2_splits = 3
assert h.mplc_cnn_train_step(ctypes.byref(t), None) == E_ARG               # null buffers
assert h.mplc_cnn_train_step(None, None) == E_ARG
# CIFAR10 CNN
cifar._bind()
assert h.mplc_cifar_init_params(P, 5, P, 1, None) == E_ARG
for m in (0, 1, 1000, 65535):
    for c in (0, 1, 500, 65535):
        h.mplc_cifar_eval_workspace_floats(m, c)
assert h.mplc_cifar_evaluate(P, 1251008, 1, P, P, 10, 10, None, P, P, None) == E_ARG
ct = cifar.CifarTrainT()
assert h.mplc_cifar_train_step(ctypes.byref(ct), None) == E_ARG
ct.n_rep, ct.bmax, ct.wg_splits = 1, 11, 1
assert h.mplc_cifar_train_step(ctypes.byref(ct), None) == E_SHAPE
# sequential snapshots, logistic regression
assert h.mplc_seq_snapshot(P, 64, 16, P, 0, P, P, 0, 1, 1, 1, P, P, None) == E_ARG
assert h.mplc_seq_snapshot(P, 8, 16, P, 1, P, P, 0, 1, 1, 1, P, P, None) == E_ARG
args = [None] * 27
args[2], args[7], args[12], args[13], args[14], args[17], args[20], args[25] = 27, 1, 1, 1, 0, 0, 0, 0
assert h.mplc_lr_fedavg(*args) == E_ARG
print("SANITIZE_OK")
'''


def _runtime():
    clang = "/opt/rocm/lib/llvm/bin/clang++"
    if not os.path.exists(clang):
        return None
    rt = subprocess.run([clang, "--print-file-name=libclang_rt.asan-x86_64.so"], capture_output=True,
                        text=True).stdout.strip()
    return rt if os.path.isfile(rt) else None


def test_c_abi_host_code_under_asan_ubsan():
    rt = _runtime()
    if rt is None:
        pytest.skip("clang ASan runtime not found")
    sys.path.insert(0, PKG)
    import build_native
    lib = build_native.build(sanitize=True)
    nm = subprocess.run(["nm", "-D", lib], capture_output=True, text=True).stdout
    assert "__asan_report" in nm and "__ubsan_handle" in nm  # instrumented host code
    env = dict(os.environ, LD_PRELOAD=rt, MPLC_LIB_PATH=lib, HIP_VISIBLE_DEVICES="",
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([sys.executable, "-c", CHILD, REPO, PKG], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "SANITIZE_OK" in r.stdout, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
