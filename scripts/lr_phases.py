"""Where the Titanic LR kernel's time goes: build a timing copy of libmplc_hip.so whose csrc/logreg.hip force-includes
scripts/lr_phase.h (wall-clock marks between the phases of every Newton iteration), run the config #2 sweep through
it, and print each phase's share and the per-fit iteration counts.

    python scripts/lr_phases.py build      # here (hipcc): scripts/_lrphase/libmplc_hip.so
    python scripts/lr_phases.py run OUT    # on the GPU box: OUT.json
"""
import ctypes
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "distributed-learning-contributivity_amd")
OUT_DIR = os.path.join(REPO, "scripts", "_lrphase")
LIB = os.path.join(OUT_DIR, "libmplc_hip.so")
PHASES = {10: "between fits (FedAvg bookkeeping, next partner's set-up)", 9: "stage rows", 1: "start objective", 2: "sigma + Hessian + gradient", 3: "convergence test",
          4: "Cholesky", 5: "triangular solves", 6: "line search", 8: "FedAvg average (+ hist)",
          7: "final test accuracy"}


def build():
    sys.path.insert(0, PKG)
    import build_native as bn
    bn.build()
    os.makedirs(OUT_DIR, exist_ok=True)
    obj = os.path.join(OUT_DIR, "logreg.o")
    subprocess.run([bn.HIPCC] + bn.CFLAGS + ["-include", os.path.join(REPO, "scripts", "lr_phase.h"), "-c",
                    os.path.join(bn.CSRC, "logreg.hip"), "-o", obj], check=True)
    others = [os.path.join(bn.BUILD, f[:-4] + ".o") for f in sorted(os.listdir(bn.CSRC))
              if f.endswith(".hip") and f != "logreg.hip"]
    subprocess.run([bn.HIPCC, "-shared", "-fPIC", f"--offload-arch={bn.ARCH}", "-o", LIB, obj] + others, check=True)
    print(LIB)


def run(out):
    os.environ["MPLC_LIB_PATH"] = LIB
    sys.path.insert(0, REPO)
    sys.path.insert(0, PKG)
    import time

    import torch
    import bench
    from mplc import _native
    from mplc.contributivity import Contributivity
    from mplc.engine import CoalitionEngine
    sc = bench.build_titanic_scenario()
    sc.engine = CoalitionEngine.for_scenario(sc)
    h = ctypes.CDLL(LIB)
    ticks, calls, khz = (ctypes.c_ulonglong * 16)(), (ctypes.c_ulonglong * 16)(), ctypes.c_int()
    res = {}
    for run_i in range(2):  # the first run loads the code object
        sc.coalition_values = {}
        h.lr_phase_read(ticks, calls, ctypes.byref(khz))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        Contributivity(scenario=sc).compute_contributivity("Shapley values")
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        assert h.lr_phase_read(ticks, calls, ctypes.byref(khz)) == 0
    assert _native.lib_path() == LIB
    import numpy as np
    sp = (ctypes.c_ulonglong * (4096 * 3))()
    assert h.lr_phase_spans(sp) == 0
    sp = np.array(sp, dtype=np.uint64).reshape(4096, 3)[:1023].astype(np.int64)
    t0s = sp[:, 0] - sp[:, 0].min()
    dur = sp[:, 1] - sp[:, 0]
    to_us = 1e3 / khz.value
    order = np.argsort(t0s)
    spans = {"first_start_to_last_end_us": round(float((sp[:, 1].max() - sp[:, 0].min()) * to_us), 1),
             "start_offsets_us_pct": [round(float(np.percentile(t0s, q) * to_us), 1) for q in (0, 25, 50, 75, 90, 100)],
             "durations_us_pct": [round(float(np.percentile(dur, q) * to_us), 1) for q in (0, 25, 50, 75, 90, 100)],
             "longest_wave_us": round(float(dur.max() * to_us), 1),
             "longest": [[int(i), round(float(dur[i] * to_us), 1), int(sp[i, 2] >> 32), int(sp[i, 2] & 0xffffffff)]
                         for i in np.argsort(dur)[-12:]],
             "iterations_per_fit_pct": [round(float(np.percentile((sp[:, 2] & 0xffffffff) / np.maximum(1, sp[:, 2] >> 32), q)), 2)
                                        for q in (0, 50, 90, 99, 100)]}
    tot = sum(ticks[i] for i in PHASES)
    res = {"wall_ms_with_marks": round(wall * 1e3, 2), "wall_clock_khz": khz.value,
           "newton_iterations": calls[3], "fits": calls[1], "spans": spans,
           "phases": {PHASES[i]: {"share": round(ticks[i] / tot, 4), "calls": calls[i],
                                  "us_per_call": round(ticks[i] / max(1, calls[i]) / khz.value * 1e3, 3)}
                      for i in PHASES}}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    build() if sys.argv[1] == "build" else run(sys.argv[2])
