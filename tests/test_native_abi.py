"""CPU: the C-ABI library builds/loads and exports exactly what include/*.h declares (no compute calls)."""
import glob
import os
import re
import subprocess

import pytest

from mplc import _native

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    syms = set()
    for h in glob.glob(os.path.join(REPO, "include", "*.h")):
        text = open(h).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"\b(mplc_[a-z0-9_]+)\s*\(", text):
            syms.add(m.group(1))
    return syms


def exported_symbols(path):
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if " T " in line and line.split()[-1].startswith("mplc_")}


def test_library_exists_and_loads():
    if not os.path.exists(_native.lib_path()):
        import __graft_entry__
        __graft_entry__.build()
    h = _native.lib()
    assert h.mplc_abi_version() == _native.ABI_VERSION


def test_exports_match_headers():
    decl = declared_symbols()
    assert "mplc_shapley_exact" in decl and "mplc_fedavg_aggregate" in decl
    exp = exported_symbols(_native.lib_path())
    assert decl <= exp, f"declared but not exported: {decl - exp}"
    assert exp <= decl, f"exported but not declared: {exp - decl}"
    assert set(_native.SIGNATURES) == decl


def test_argument_errors_without_gpu():
    h = _native.lib()
    # argument validation happens before any HIP call
    assert h.mplc_shapley_partial(None, 0, 0, 5, None, None, 0, None) == -1
    assert h.mplc_shapley_finalize(None, 0, None, None) == -1
    assert h.mplc_shapley_workspace_bytes(10, 1024) == 0
    assert h.mplc_shapley_workspace_bytes(20, 1 << 20) == 16 * 8 * 18 * 8  # 16 spans x 8 pass-group blocks
    assert h.mplc_shapley_workspace_bytes(28, 1 << 28) == 4096 * 18 * 8  # >= 256 spans: one block each
    with pytest.raises(RuntimeError):
        _native.check(-2, "x")


def test_abi_version_bumped_with_the_cifar_layout():
    # version 2: MPLC_CIFAR_WT grew to 114688 (Winograd weights) and the layout queries were added; version 3: the
    # pooled-gradient slots dz4 / dz2 shrank to their pooled sizes; version 4: mplc_cnn_train_t's fused W3 average
    # (avg_*) and mplc_fedavg_aggregate_skip
    assert _native.ABI_VERSION == 4
    text = open(os.path.join(REPO, "include", "mplc_hip.h")).read()
    assert re.search(r"#define MPLC_ABI_VERSION 4\b", text)
    assert "mplc_fedavg_aggregate_skip" in text
    cnn = open(os.path.join(REPO, "include", "mplc_hip_cnn.h")).read()
    assert all(f in cnn for f in ("avg_first", "avg_w", "avg_scale", "avg_glob", "avg_out", "avg_rep"))
    defs = _header_defines("mplc_hip_cifar.h")
    assert (defs["MPLC_CIFAR_DZ4"], defs["MPLC_CIFAR_DZ2"]) == (6 * 6 * 64, 15 * 15 * 32)


def _header_defines(name):
    text = open(os.path.join(REPO, "include", name)).read()
    return {m.group(1): int(m.group(2)) for m in re.finditer(r"#define (MPLC_\w+) \(?(-?\d+)\)?", text)}


@pytest.mark.parametrize("model", ["cnn", "cifar"])
def test_layout_queries_match_host_constants_and_headers(model):
    """Every layout item the library reports equals the host's constant (which the host checks at bind time, so
    a mismatched library/host pair refuses to load) and the header's #define; unknown items return -1."""
    import ctypes
    from mplc import cifar, cnn
    mod, prefix, header = (cnn, "MPLC_CNN_Q_", "mplc_hip_cnn.h") if model == "cnn" else \
        (cifar, "MPLC_CIFAR_Q_", "mplc_hip_cifar.h")
    query = getattr(_native.lib(), f"mplc_{model}_layout")
    items = mod.layout_items()
    defs = _header_defines(header)
    qids = {k[len(prefix):]: v for k, v in defs.items() if k.startswith(prefix) and k != prefix + "COUNT"}
    assert set(qids) == set(items), "host and header list different layout items"
    assert defs[prefix + "COUNT"] == len(items)
    for name, (qid, value) in items.items():
        assert qids[name] == qid
        assert query(qid) == value, (name, query(qid), value)
    assert query(len(items)) == -1 and query(-1) == -1
    # the value constants the host hard-codes equal the header's
    hdr_prefix = "MPLC_CNN_" if model == "cnn" else "MPLC_CIFAR_"
    for name, (_, value) in items.items():
        if hdr_prefix + name in defs:
            assert defs[hdr_prefix + name] == value, name
    # _bind() runs the same comparison: a mismatch raises instead of loading silently
    with pytest.raises(RuntimeError, match="layout mismatch"):
        bad = dict(items)
        bad["STRIDE"] = (items["STRIDE"][0], items["STRIDE"][1] + 64)
        _native.check_layout(query, bad, model)
    assert ctypes.sizeof(cnn.TrainT) == query(items["TRAIN_T_BYTES"][0]) if model == "cnn" else True


def test_experiment_switches_refuse_product_builds(tmp_path):
    """A *_EXP_* timing switch (wrong results by design) is an #error unless MPLC_EXPERIMENT is defined."""
    csrc = os.path.join(REPO, "distributed-learning-contributivity_amd", "csrc")
    src = os.path.join(csrc, "mnist_cnn.hip")
    text = "".join(open(os.path.join(csrc, f)).read() for f in ("mnist_cnn.hip", "mnist_wgrad.hip"))
    switches = set(re.findall(r"#if(?:n?def)?\s*!?\s*(?:defined\()?(\w+_EXP_\w+)", text))
    assert switches, "no experiment switches found"
    common = open(os.path.join(csrc, "mnist_common.h")).read()  # both sources include it first
    guard = common[:common.index("namespace {")]
    for sw in switches:
        assert f"defined({sw})" in guard, f"{sw} is not covered by the #error guard"
    hipcc = "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    r = subprocess.run([hipcc, "-E", "-DWG_EXP_NOGEMM", "-I", os.path.join(REPO, "include"), "--offload-arch=gfx950",
                        "--cuda-host-only", src, "-o", str(tmp_path / "x.i")], capture_output=True, text=True)
    assert r.returncode != 0 and "MPLC_EXPERIMENT" in r.stderr
