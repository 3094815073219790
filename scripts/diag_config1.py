"""Config #1 3-partner diagnosis: is the (0, 1) coalition's gap to the fp32 oracle summation-
order noise or a defect of the bs-10 / ragged-minibatch path?

The partition is the reference's own split of the contrib yml's 3-partner variant ([0.2, 0.5, 0.3], MNIST,
dataset_proportion 0.1, E=1, M=10, G=8): 874 / 2186 / 1312 rows at bs 10 / 27 / 16, so every partner's round
ends with a short batch (87-88 rows at bs 10: 8 x 10 + 7 or 8; 218-219 at bs 27: 8 x 27 + 2 or 3; 131 at bs 16:
8 x 16 + 3).  Data: the learnable synthetic MNIST of tests/test_config1_gpu.py (signal 0.3, quantised to uint8).

For every coalition of the 3 partners:
  (1) one-round trajectories: each of the 10 FedAvg rounds of epoch 0 started from the DEVICE's global model at
      that round's start; device vs oracle/cnn.py fedavg_round(precise=True) (fp64), per tensor
      ||dev - ref64|| / ||ref64 - start||, beside the fp32 oracle's own error (the largest over 1, 2, 3, 8 and
      the box's CPU threads).  Singletons: the whole one-epoch fit (persistent Adam) the same way.
  (2) accuracies: the device's v(S), the fp64 oracle's (the same algorithm with every tensor operation in fp64)
      and the fp32 oracle's at 1, 2, 3, 4, 6, 8, 12 and 16 CPU threads.

Writes gpurun_out/diag_config1.json (GPU box) and prints a summary."""
import json
import os
import sys
import tempfile
import time
from itertools import combinations

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "distributed-learning-contributivity_amd"))


def scenario_3p(signal=0.3):
    from mplc.dataset import _synthetic_images
    from mplc.scenario import Scenario
    d = tempfile.mkdtemp(prefix="cfg1_")
    x, y, xt, yt = _synthetic_images((28, 28, 1), 60000, 10000, 0, signal)
    q = lambda a: np.round(a[..., 0] * 255).astype(np.uint8)  # noqa: E731
    np.savez(os.path.join(d, "mnist.npz"), x_train=q(x), y_train=np.argmax(y, 1).astype(np.uint8), x_test=q(xt),
             y_test=np.argmax(yt, 1).astype(np.uint8))
    os.environ["MPLC_DATA_DIR"] = d
    sc = Scenario(3, [0.2, 0.5, 0.3], dataset_name="mnist", dataset_proportion=0.1,
                  samples_split_option=["basic", "random"], epoch_count=1, minibatch_count=10,
                  gradient_updates_per_pass_count=8, methods=["Shapley values"])
    return sc.provision()


def tensor_errors(dev_row, ref64, g32s, start_row, OFF):
    out = {}
    for name, (off, shape) in OFF.items():
        n = int(np.prod(shape))
        ref = ref64[name].numpy().reshape(-1).astype(np.float64)
        upd = np.linalg.norm(ref - start_row[off:off + n].astype(np.float64))
        e_dev = np.linalg.norm(dev_row[off:off + n].astype(np.float64) - ref) / upd
        e_cpu = max(np.linalg.norm(g[name].numpy().reshape(-1).astype(np.float64) - ref) / upd for g in g32s)
        out[name] = (float(e_dev), float(e_cpu))
    return out


def main():
    import torch
    from oracle import cnn as ocnn
    from mplc.engine import CoalitionEngine
    t0 = time.time()
    sc = scenario_3p()
    eng = CoalitionEngine.for_scenario(sc, memory_budget_bytes=8 << 30, eval_budget_bytes=1 << 30)
    ds = sc.dataset
    data = ocnn.Data(ds.x_train, ds.y_train, ds.x_val, ds.y_val, ds.x_test, ds.y_test)
    prow = [p.train_idx for p in sc.partners_list]
    bs = [p.batch_size for p in sc.partners_list]
    M = sc.minibatch_count
    report = {"rows": [len(r) for r in prow], "batch_sizes": bs, "M": M, "seed": eng.seed}
    print("rows", report["rows"], "bs", bs, flush=True)
    threads0 = torch.get_num_threads()
    traj_threads = sorted({1, 2, 3, 8, threads0})
    coals = [k for r in range(1, 4) for k in combinations(range(3), r)]
    report["trajectory"] = {}
    for coal in coals:
        mask = sum(1 << p for p in coal)
        rows = []
        if len(coal) > 1:
            st = eng.trainer.prepare([coal], 1)
            for m in range(M):
                start = st.glob[0].cpu().numpy().copy()
                for s in range(m * st.round_len, (m + 1) * st.round_len):
                    st.step(s)
                st.aggregate(epoch_end=(m == M - 1))
                torch.cuda.synchronize()
                dev = st.glob[0].cpu().numpy().copy()
                glob = ocnn.unpack(start)
                g64 = ocnn.fedavg_round(data, prow, bs, coal, glob, seed=eng.seed, M=M, e=0, m=m, precise=True)
                g32s = []
                for th in traj_threads:
                    torch.set_num_threads(th)
                    g32s.append(ocnn.fedavg_round(data, prow, bs, coal, glob, seed=eng.seed, M=M, e=0, m=m))
                torch.set_num_threads(threads0)
                errs = tensor_errors(dev, g64, g32s, start, ocnn.OFF)
                worst = max(errs[k][0] / errs[k][1] for k in errs)
                rows.append({"round": m, "errors": errs, "worst_ratio": float(worst)})
                print(coal, "round", m, "worst dev/cpu ratio %.2f" % worst,
                      {k: "%.1e/%.1e" % v for k, v in errs.items()}, flush=True)
            del st
        else:
            # the singleton's whole epoch (persistent Adam, ragged last batch) from the keyed initial model
            p = coal[0]
            _, _ = eng.trainer.run([coal], 1, False, keep_models=True)
            dev = eng.trainer.last_models[0]
            start = ocnn.init_params(ocnn.init_key(eng.seed, mask))
            _, _, m64 = ocnn.coalition_value(data, prow, bs, coal, seed=eng.seed, epochs=1, M=M, return_model=True,
                                             precise=True)
            g32s = []
            for th in traj_threads:
                torch.set_num_threads(th)
                g32s.append(ocnn.unpack(ocnn.coalition_value(data, prow, bs, coal, seed=eng.seed, epochs=1, M=M,
                                                             return_model=True)[2]))
            torch.set_num_threads(threads0)
            errs = tensor_errors(dev, m64, g32s, start, ocnn.OFF)
            worst = max(errs[k][0] / errs[k][1] for k in errs)
            rows.append({"round": "epoch", "errors": errs, "worst_ratio": float(worst)})
            print(coal, "epoch fit", "worst dev/cpu ratio %.2f" % worst,
                  {k: "%.1e/%.1e" % v for k, v in errs.items()}, flush=True)
        report["trajectory"][str(coal)] = rows
    # accuracies
    acc_threads = [1, 2, 3, 4, 6, 8, 12, 16]
    dev_v = eng.evaluate(coals)
    report["accuracy"] = {}
    for i, coal in enumerate(coals):
        v64 = ocnn.coalition_value(data, prow, bs, coal, seed=eng.seed, epochs=1, M=M, precise=True)[0]
        v32 = []
        for th in acc_threads:
            torch.set_num_threads(th)
            v32.append(ocnn.coalition_value(data, prow, bs, coal, seed=eng.seed, epochs=1, M=M)[0])
        torch.set_num_threads(threads0)
        report["accuracy"][str(coal)] = {"device": float(dev_v[i]), "fp64": float(v64),
                                         "fp32_by_threads": dict(zip(map(str, acc_threads), map(float, v32)))}
        print(coal, "device %.4f fp64 %.4f fp32 %s" % (dev_v[i], v64, " ".join("%.4f" % v for v in v32)), flush=True)
    report["wall_s"] = time.time() - t0
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "diag_config1.json"), "w") as f:
        json.dump(report, f, indent=1)


if __name__ == "__main__":
    main()
