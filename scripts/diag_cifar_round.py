"""Diagnostic: one CIFAR10 FedAvg round step by step, device replicas vs the fp64 / fp32 oracle fits.
python scripts/diag_cifar_round.py  (GPU)"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "distributed-learning-contributivity_amd"))
from mplc.dataset import Cifar10  # noqa: E402
from mplc.engine import CoalitionEngine  # noqa: E402
from mplc.scenario import Scenario  # noqa: E402
from oracle import cifar_cnn as occ  # noqa: E402
from oracle import cnn as ocnn  # noqa: E402

amounts = [0.05] * 19 + [float(1 - np.sum([0.05] * 19))]
sc = Scenario(20, amounts, dataset=Cifar10(synthetic=True, signal=0.4), minibatch_count=20,
              gradient_updates_per_pass_count=8, epoch_count=1, is_early_stopping=False).provision()
eng = CoalitionEngine.for_scenario(sc, memory_budget_bytes=8 << 30, eval_budget_bytes=1 << 30)
coal = tuple(int(a) for a in (sys.argv[1].split(",") if len(sys.argv) > 1 else (2, 9, 17)))
st = eng.trainer.prepare([coal], 1)
ds = sc.dataset
data = occ.Data(ds.x_train, ds.y_train, ds.x_val, ds.y_val, ds.x_test, ds.y_test)
prow = [p.train_idx for p in sc.partners_list]
bs = [p.batch_size for p in sc.partners_list]
mask = sum(1 << p for p in coal)
print("R", st.R, "round_len", st.round_len, "bs", [bs[p] for p in coal], "rows", [len(prow[p]) for p in coal])
start = st.glob[0].cpu().numpy().copy()
glob = occ.unpack(start)
fits = {}
for prec in (True, False):
    out = []
    for p_id in coal:
        key = ocnn.shuffle_key(eng.seed, mask, p_id)
        dt = torch.float64 if prec else torch.float32
        params = {k: v.to(dt).clone() for k, v in glob.items()}
        opt = occ.KerasRMSprop(params, precise=prec)
        traj = []
        for t, rows in enumerate(ocnn.fedavg_round_rows(key, prow[p_id], bs[p_id], 20, 0, 0)):
            masks = occ.step_masks(occ.fedavg_drop_key(key, 0, 0, t), len(rows))
            g, _ = occ.gradients(params, data.x_train[rows], data.y_train[rows], masks, dtype=dt if prec else None)
            opt.step(params, g)
            traj.append({k: v.detach().clone().to(torch.float64) for k, v in params.items()})
        out.append(traj)
    fits[prec] = out
cnt_hist = []
for s in range(st.round_len):
    st.step(s)
    torch.cuda.synchronize()
    cnt_hist.append(st.ws["cnt"].cpu().numpy()[:st.R].tolist())
    P = st.params.cpu().numpy()
    for r, p_id in enumerate(coal):
        if s >= len(fits[True][r]):
            continue
        ref = fits[True][r][s]
        f32 = fits[False][r][s]
        line = []
        for name, (off, shape) in occ.OFF.items():
            n = int(np.prod(shape))
            rv = ref[name].numpy().reshape(-1)
            upd = np.linalg.norm(rv - start[off:off + n].astype(np.float64))
            e_dev = np.linalg.norm(P[r, off:off + n].astype(np.float64) - rv) / upd
            e_cpu = np.linalg.norm(f32[name].numpy().reshape(-1) - rv) / upd
            line.append(f"{name} {e_dev:.1e}/{e_cpu:.1e}")
        print(f"step {s} rep {r} cnt {cnt_hist[-1][r]}: " + "  ".join(line))
