"""Probe: two replica halves on two HIP streams with their step phases interleaved (MFMA-bound convolutions of
one half beside the HBM-bound dense layer of the other), against the one-stream lockstep step.
python scripts/probe_overlap.py [steps] [n_coalitions] [mode ...]   modes: single, split, lag
Timing only: the FedAvg aggregation is left out (both modes equally)."""
import ctypes
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "distributed-learning-contributivity_amd"))

import numpy as np
import torch

from mplc import _native
from mplc import cnn
from mplc.dataset import Mnist
from mplc.engine import CoalitionEngine
from mplc.scenario import Scenario

PER_REP = {  # field -> bytes per replica (arrays that are replica-major)
}


def sub_struct(st, r0, r1):
    t = cnn.TrainT()
    ctypes.pointer(t)[0] = st.t  # copy
    B, S = st.bmax, cnn.STRIDE
    splits = st.t.w2_splits
    per = {"reps": 32, "params": 4 * S, "adam_m": 4 * S, "adam_v": 4 * S, "idx": 4 * B, "cnt": 4, "adam_t": 4,
           "pooled": 4 * B * cnn.FEAT, "code": B * cnn.FEAT, "hidden": 4 * B * cnn.HID, "dhidden": 4 * B * cnn.HID,
           "dpooled": 4 * B * cnn.FEAT, "w1_part": 4 * B * cnn.W1_BANDS * cnn.W1P, "w2_part": 4 * splits * cnn.W2P,
           "w2t": 4 * cnn.W2T, "w3src": 4, "rep_glob": 4}
    for f, b in per.items():
        v = getattr(st.t, f)
        if v:
            setattr(t, f, v + r0 * b)
    t.n_rep = r1 - r0
    return t


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1023
    modes = sys.argv[3:] or ["single", "split", "lag"]
    sc = Scenario(10, [0.1] * 10, dataset=Mnist(synthetic=True), minibatch_count=20, epoch_count=1,
                  is_early_stopping=False).provision()
    eng = CoalitionEngine.for_scenario(sc)
    from itertools import combinations
    coals = [c for r in range(2, 11) for c in combinations(range(10), r)][:n]
    st = eng.trainer.prepare(coals, 1)
    lib = _native.lib()
    R = st.R
    # split at a coalition boundary near R / 2
    half = min(st.coal_first, key=lambda f: abs(f - R // 2))
    tA, tB = sub_struct(st, 0, half), sub_struct(st, half, R)
    sA, sB = torch.cuda.Stream(), torch.cuda.Stream()
    main_s = torch.cuda.current_stream()
    hA, hB = ctypes.c_void_p(sA.cuda_stream), ctypes.c_void_p(sB.cuda_stream)
    print(f"R={R} replicas, halves {half} / {R - half}, bmax {st.bmax}", flush=True)

    def call(t, s, ph, h):
        t.step, t.phases = s, ph
        _native.check(lib.mplc_cnn_train_step(ctypes.byref(t), h), "train_step")

    for mode in modes:
        torch.cuda.synchronize()
        # warm
        st.t.phases = 0
        st.step(0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if mode == "single":
            for s in range(steps):
                st.t.phases = 0
                st.step(s)
        elif mode == "split":  # both halves, whole steps, two streams, no ordering between them
            sA.wait_stream(main_s)
            sB.wait_stream(main_s)
            for s in range(steps):
                call(tA, s, 0, hA)
                call(tB, s, 0, hB)
        else:  # lag: half B runs one phase behind half A
            sA.wait_stream(main_s)
            sB.wait_stream(main_s)
            for s in range(steps):
                for ph in (1, 2, 4):
                    call(tA, s, ph, hA)
                    ev = torch.cuda.Event()
                    ev.record(sA)
                    sB.wait_event(ev)
                    call(tB, s, ph, hB)
            main_s.wait_stream(sA)
            main_s.wait_stream(sB)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"{mode}: {steps} steps {dt:.3f}s = {1000 * dt / steps:.2f} ms/step", flush=True)


if __name__ == "__main__":
    main()
