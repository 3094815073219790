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
