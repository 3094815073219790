"""Config #3 diagnosis: is coalition (2, 9)'s 0.9151 at E=1 (fp32 oracle 0.877 .. 0.887 over
eight CPU thread counts, fp64 0.9035) and partner 9's fp64 / fp32 disagreement ((9,): 0.636 fp64, 0.724 .. 0.751
fp32) summation-order forking or a kernel defect?

Scenario: tests/test_workload_gpu.py's config #3 (10 partners x 0.1 of synthetic MNIST signal 0.2, E=1, M=20, G=8,
4374 rows per partner at bs 27).  For each coalition given (default (2, 9) and (9,)):
  (1) per-round trajectories (FedAvg): each of the 20 rounds of epoch 0 started from the DEVICE's global model at
      that round's start, device vs oracle/cnn.py fedavg_round(precise=True) (fp64), per tensor
      ||dev - ref64|| / ||ref64 - start||, beside the fp32 oracle's own error (largest over 1, 2, 3, 8 and the
      box's CPU threads) - as scripts/diag_config1.py did for config #1's (0, 1);
  (2) free trajectories: device, fp64 and fp32 oracle (1, 3 and the box's threads) each trained from the same keyed
      initial model with no restart, the parameter distance to the fp64 trajectory every `--every` steps (FedAvg:
      at every round end), and each trajectory's test accuracy at the end.  A fork shows as a distance that jumps
      by orders of magnitude at one step and then grows, in the fp32 oracle as well as on the device.
Writes gpurun_out/diag_config3.json and prints a summary."""
import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, HERE, os.path.join(ROOT, "tests"), os.path.join(ROOT, "distributed-learning-contributivity_amd")):
    sys.path.insert(0, p)
from diag_config1 import tensor_errors  # noqa: E402


def rel_dist(a, ref64, start):
    """||a - ref64|| / ||ref64 - start|| over the whole parameter row (fp64)."""
    ref = ref64.astype(np.float64)
    return float(np.linalg.norm(a.astype(np.float64) - ref) / np.linalg.norm(ref - start.astype(np.float64)))


def oracle_single_traj(ocnn, data, prow, bs, p_id, mask, seed, every, dtype):
    """The oracle's singleton epoch (coalition_value's loop) with the parameter row kept every `every` steps."""
    import torch
    glob = ocnn.unpack(ocnn.init_params(ocnn.init_key(seed, mask)))
    precise = dtype == torch.float64
    params = {k: (v.to(torch.float64) if precise else v).clone() for k, v in glob.items()}
    opt = ocnn.KerasAdam(params, precise=precise)
    key = ocnn.shuffle_key(seed, mask, p_id)
    rows_all = ocnn.single_epoch_rows(key, prow[p_id], bs[p_id], 0)
    out = []
    for t, rows in enumerate(rows_all):
        g, _ = ocnn.gradients(params, data.x_train[rows], data.y_train[rows], dtype=torch.float64 if precise else None)
        opt.step(params, g)
        if (t + 1) % every == 0 or t + 1 == len(rows_all):
            out.append((t + 1, np.concatenate([params[k].detach().double().numpy().reshape(-1)
                                               for k in ocnn.OFF])))
    _, acc = ocnn.evaluate(params, data.x_test, data.y_test)
    return out, acc


def flat(row, ocnn):
    return np.concatenate([row[off:off + int(np.prod(shape))].astype(np.float64) for off, shape in ocnn.OFF.values()])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--coalitions", default="2,9;9")
    ap.add_argument("--every", type=int, default=9)
    args = ap.parse_args()
    import torch
    from oracle import cnn as ocnn
    from spread_fixtures import config3_scenario, load_spread
    from mplc.engine import CoalitionEngine
    t0 = time.time()
    sc = config3_scenario()
    eng = CoalitionEngine.for_scenario(sc, memory_budget_bytes=8 << 30, eval_budget_bytes=1 << 30)
    ds = sc.dataset
    data = ocnn.Data(ds.x_train, ds.y_train, ds.x_val, ds.y_val, ds.x_test, ds.y_test)
    prow = [p.train_idx for p in sc.partners_list]
    bs = [p.batch_size for p in sc.partners_list]
    M = sc.minibatch_count
    threads0 = torch.get_num_threads()
    traj_threads = sorted({1, 2, 3, 8, threads0})
    free_threads = sorted({1, 3, threads0})
    spread = load_spread("config3", sc)
    coals = [tuple(int(v) for v in c.split(",")) for c in args.coalitions.split(";")]
    report = {"seed": eng.seed, "M": M, "threads": threads0, "coalitions": {}}
    for coal in coals:
        mask = sum(1 << p for p in coal)
        rec = {}
        dev_v = float(eng.evaluate([coal])[0])
        key = str(list(coal))
        i = [list(c) for c in spread["coalitions"]].index(list(coal)) if list(coal) in spread["coalitions"] else None
        rec["accuracy"] = {"device": dev_v,
                           "fp32_by_threads": ({t: spread["fp32"][str(t)][i] for t in spread["threads"]}
                                               if i is not None else None),
                           "fp64": spread["fp64"][i] if i is not None else None}
        print(coal, "device %.4f" % dev_v, rec["accuracy"], flush=True)
        start = ocnn.init_params(ocnn.init_key(eng.seed, mask))
        if len(coal) > 1:
            # (1) per-round restarts from the device's global model
            st = eng.trainer.prepare([coal], 1)
            rounds, dev_ends = [], []
            for m in range(M):
                g0 = st.glob[0].cpu().numpy().copy()
                for s in range(m * st.round_len, (m + 1) * st.round_len):
                    st.step(s)
                st.aggregate(epoch_end=(m == M - 1))
                torch.cuda.synchronize()
                dev = st.glob[0].cpu().numpy().copy()
                dev_ends.append(flat(dev, ocnn))
                glob = ocnn.unpack(g0)
                g64 = ocnn.fedavg_round(data, prow, bs, coal, glob, seed=eng.seed, M=M, e=0, m=m, precise=True)
                g32s = []
                for th in traj_threads:
                    torch.set_num_threads(th)
                    g32s.append(ocnn.fedavg_round(data, prow, bs, coal, glob, seed=eng.seed, M=M, e=0, m=m))
                torch.set_num_threads(threads0)
                errs = tensor_errors(dev, g64, g32s, g0, ocnn.OFF)
                worst = max(errs[k][0] / errs[k][1] for k in errs)
                rounds.append({"round": m, "errors": errs, "worst_ratio": float(worst)})
                print(coal, "round", m, "worst dev/cpu %.2f" % worst,
                      {k: "%.1e/%.1e" % v for k, v in errs.items()}, flush=True)
            del st
            rec["rounds"] = rounds
            # (2) free trajectories at round ends
            trajs = {}
            for name, th, precise in [("fp64", 8, True)] + [(f"fp32_t{t}", t, False) for t in free_threads]:
                torch.set_num_threads(th)
                glob = ocnn.unpack(start)
                if precise:
                    glob = {k: v.to(torch.float64) for k, v in glob.items()}
                ends = []
                for m in range(M):
                    glob = ocnn.fedavg_round(data, prow, bs, coal, glob, seed=eng.seed, M=M, e=0, m=m, precise=precise)
                    ends.append(np.concatenate([glob[k].double().numpy().reshape(-1) for k in ocnn.OFF]))
                _, acc = ocnn.evaluate(glob, data.x_test, data.y_test)
                trajs[name] = (ends, acc)
            torch.set_num_threads(threads0)
            trajs["device"] = (dev_ends, dev_v)
            ref = trajs["fp64"][0]
            s0 = flat(start, ocnn)
            rec["free"] = {n: {"acc": float(a), "dist_to_fp64": [rel_dist(e, r, s0) for e, r in zip(ends, ref)]}
                           for n, (ends, a) in trajs.items()}
        else:
            p_id = coal[0]
            st = eng.trainer.prepare([coal], 1)
            dev_pts = []
            for s in range(st.total_steps):
                st.step(s)
                if (s + 1) % args.every == 0 or s + 1 == st.total_steps:
                    torch.cuda.synchronize()
                    dev_pts.append((s + 1, flat(st.params[0].cpu().numpy(), ocnn)))
            del st
            trajs = {"device": (dev_pts, dev_v)}
            for name, th, dt in [("fp64", 8, torch.float64)] + [(f"fp32_t{t}", t, torch.float32) for t in free_threads]:
                torch.set_num_threads(th)
                trajs[name] = oracle_single_traj(ocnn, data, prow, bs, p_id, mask, eng.seed, args.every, dt)
            torch.set_num_threads(threads0)
            ref = [r for _, r in trajs["fp64"][0]]
            s0 = flat(start, ocnn)
            rec["free"] = {n: {"acc": float(a), "steps": [t for t, _ in pts],
                               "dist_to_fp64": [rel_dist(r, f, s0) for (_, r), f in zip(pts, ref)]}
                           for n, (pts, a) in trajs.items()}
        for n, f in rec["free"].items():
            d = f["dist_to_fp64"]
            print(coal, n, "acc %.4f" % f["acc"], "dist to fp64:", " ".join("%.1e" % v for v in d), flush=True)
        report["coalitions"][key] = rec
    report["wall_s"] = time.time() - t0
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "diag_config3.json"), "w") as f:
        json.dump(report, f, indent=1)
    print("wall %.0fs" % report["wall_s"])


if __name__ == "__main__":
    main()
