"""GPU: the alternate kernel forms kept in the source are bit-identical to the product kernels.

build_native.build_variants() links mplc/lib/variants/libmplc_hip_alt.so with the MFMA form of MNIST's
dense1_bwd_adam (MPLC_D1_MFMA=1; DESIGN.md 7e: bit-identical, +1.9 % at 5120 replicas so not the default) and
the VALU form of CIFAR10's dense5_bwd (MPLC_D5_MFMA=0; bit-identical under the RMSprop no-contraction rule) and
the 32-row form of its dense5_fwd at every batch size (MPLC_D5F16_MAX=0; the product runs the 16-row form up to 16
samples per replica, exercised by the probe's small-batch CIFAR scenario) and conv4_fwd's 4-tile remainder group as a
padded 16-tile group (MPLC_WINO_QUAD=0; the product runs it on v_mfma_f32_4x4x1f32).
tests/variant_probe.py trains two epochs of small FedAvg / singleton coalitions of both models in a child process
per library (MPLC_LIB_PATH); every final model row must hash the same."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_DIR = os.path.join(REPO, "distributed-learning-contributivity_amd", "mplc", "lib")


def _probe(lib):
    env = dict(os.environ, MPLC_LIB_PATH=lib)
    r = subprocess.run([sys.executable, os.path.join(REPO, "tests", "variant_probe.py")], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = next(ln for ln in r.stdout.splitlines() if ln.startswith("VARIANT_PROBE "))
    return json.loads(line[len("VARIANT_PROBE "):])


def test_alternate_dense_forms_bit_identical():
    alt = os.path.join(LIB_DIR, "variants", "libmplc_hip_alt.so")
    assert os.path.exists(alt), "variant library missing: run __graft_entry__.build()"
    base = _probe(os.path.join(LIB_DIR, "libmplc_hip.so"))
    var = _probe(alt)
    print(base, var)
    assert base["lib"] != var["lib"]
    for model in ("mnist", "cifar10", "cifar10_smallb"):
        assert var[model] == base[model], (model, base[model], var[model])
        assert max(base[model]["scores"]) > 0.35  # the models learned: the dense backward passes did real work
