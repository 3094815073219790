"""GPU parity of the batched CIFAR10-CNN trainer (csrc/cifar_cnn.hip) against the torch-CPU oracle
(oracle/cifar_cnn.py).

Integer/index work must be bit-exact: initial weights, the sample schedule, the per-step dropout keys and
masks (keep bits of the stored codes).  Floating point: one step's gradients within 1e-4 relative (L2, vs an
fp64 reference on the same masks), forward activations within 1e-4, one RMSprop step against the Keras
2.3.1 update; trained coalition accuracies within +-1 point on average of the oracle (the reference's own
"accuracies within 1 pt" bar), each within 3 points.
Data: sklearn's bundled digits upsampled to 32x32x3 (mplc.dataset.digits_as_cifar) - real, learnable,
CIFAR-shaped, no network."""
import numpy as np
import pytest

from oracle import cifar_cnn as occ
from oracle import cnn as ocnn

pytestmark = pytest.mark.gpu


def make_scenario(partners=3, amounts=(0.2, 0.5, 0.3), M=2, G=4, E=2, es=False):
    from mplc.dataset import ArrayDataset, digits_as_cifar
    from mplc.scenario import Scenario
    x, y = digits_as_cifar()
    ds = ArrayDataset(x[:1500], y[:1500], x[1500:], y[1500:], name="cifar10")
    sc = Scenario(partners, list(amounts), dataset=ds, minibatch_count=M, gradient_updates_per_pass_count=G,
                  epoch_count=E, is_early_stopping=es)
    return sc.provision()


@pytest.fixture(scope="module")
def scenario():
    return make_scenario()


@pytest.fixture(scope="module")
def engine(scenario):
    from mplc.engine import CoalitionEngine
    return CoalitionEngine.for_scenario(scenario, memory_budget_bytes=16 << 30, eval_budget_bytes=1 << 30)


@pytest.fixture(scope="module")
def odata(scenario):
    ds = scenario.dataset
    return occ.Data(ds.x_train, ds.y_train, ds.x_val, ds.y_val, ds.x_test, ds.y_test)


def rows(scenario):
    return [p.train_idx for p in scenario.partners_list], [p.batch_size for p in scenario.partners_list]


def test_engine_selects_cifar_kernels(engine):
    assert engine.model_impl.name == "cifar10_cnn"
    assert engine.x_train_d.shape[1:] == (32, 32, 3)


def test_init_params_bit_exact(engine):
    st = engine.trainer.prepare([(0, 2), (1,)], 1)
    g = st.glob.cpu().numpy()
    for ci, c in enumerate([(0, 2), (1,)]):
        ref = occ.init_params(ocnn.init_key(engine.seed, sum(1 << p for p in c)))
        assert np.array_equal(g[ci], ref)
    p = st.params.cpu().numpy()
    assert np.array_equal(p[0], g[0]) and np.array_equal(p[1], g[0]) and np.array_equal(p[2], g[1])


def test_schedule_and_dropout_masks_bit_exact(scenario, engine):
    import torch
    prow, bs = rows(scenario)
    coal = [(0, 1, 2), (2,)]
    st = engine.trainer.prepare(coal, 2)
    M = engine.minibatch_count
    for s in (0, 1, st.round_len * M + 3):
        st.step(s)
        torch.cuda.synchronize()
        idx, cnt = st.ws["idx"].cpu().numpy(), st.ws["cnt"].cpu().numpy()
        dkeys = st.ws["drop_key"].cpu().numpy().view(np.uint64)
        code2, code4, code5 = (st.ws[k].cpu().numpy() for k in ("code2", "code4", "code5"))
        e, rem = divmod(s, M * st.round_len)
        m, t = divmod(rem, st.round_len)
        for r, p in enumerate((0, 1, 2)):
            key = ocnn.shuffle_key(engine.seed, 0b111, p)
            steps = ocnn.fedavg_round_rows(key, prow[p], bs[p], M, e, m)
            expect = steps[t] if t < len(steps) else np.array([], dtype=np.int64)
            assert cnt[r] == len(expect)
            assert idx[r, :cnt[r]].tolist() == [int(v) for v in expect]
            if cnt[r]:
                dk = occ.fedavg_drop_key(key, e, m, t)
                assert int(dkeys[r]) == dk
                c = int(cnt[r])
                assert np.array_equal((code2[r, :c] & 0x40) != 0, occ.dropout_keep(dk, "L2", c, 7200))
                assert np.array_equal((code4[r, :c] & 0x40) != 0, occ.dropout_keep(dk, "L4", c, 2304))
                assert np.array_equal((code5[r, :c] & 0x40) != 0, occ.dropout_keep(dk, "L5", c, 512))
        key = ocnn.shuffle_key(engine.seed, 0b100, 2)
        spe = -(-len(prow[2]) // bs[2])
        es_, ts = divmod(s, spe)
        srows = ocnn.single_epoch_rows(key, prow[2], bs[2], es_)[ts]
        assert idx[3, :cnt[3]].tolist() == [int(v) for v in srows]
        assert int(dkeys[3]) == occ.single_drop_key(key, es_, ts)


def _one_step(engine, coal):
    import torch
    st = engine.trainer.prepare(coal, 1)
    p0 = st.params.cpu().numpy().copy()
    st.step(0)
    torch.cuda.synchronize()
    return st, p0


def test_one_step_gradients_and_activations(scenario, engine, odata):
    """Step 1 of a fresh RMSprop: a = 0.1 g^2 gives |g|, the update's direction gives sign(g)."""
    import torch
    st, p0 = _one_step(engine, [(0, 1), (1, 2)])
    idx, cnt = st.ws["idx"].cpu().numpy(), st.ws["cnt"].cpu().numpy()
    dkeys = st.ws["drop_key"].cpu().numpy().view(np.uint64)
    p1 = st.params.cpu().numpy()
    a = st.rms.cpu().numpy()
    acts = {k: st.ws[k].cpu().numpy() for k in ("a1", "d2", "a3", "d4", "d5")}
    report, bad = [], []
    for r in range(st.R):
        c = int(cnt[r])
        rws = idx[r, :c]
        P = occ.unpack(p0[r])
        x, y = odata.x_train[rws], odata.y_train[rws]
        masks = occ.step_masks(int(dkeys[r]), c)
        g32, _ = occ.gradients(P, x, y, masks)
        g64, _ = occ.gradients(P, x, y, masks, dtype=torch.float64)
        g_dev = np.sign(p0[r] - p1[r]).astype(np.float64) * np.sqrt(a[r].astype(np.float64) / np.float32(0.1))
        for name, (off, shape) in occ.OFF.items():
            n = int(np.prod(shape))
            ref = g64[name].numpy().reshape(-1)
            scale = max(np.linalg.norm(ref), 1e-12)
            err_dev = np.linalg.norm(g_dev[off:off + n] - ref) / scale
            err_cpu = np.linalg.norm(g32[name].numpy().reshape(-1) - ref) / scale
            allow = max(4 * err_cpu, 1e-4)
            report.append((r, name, float(err_dev), float(err_cpu), float(allow)))
            if not err_dev < allow:
                bad.append(report[-1])
        with torch.no_grad():
            _, ref_acts = occ.forward(P, x, masks, return_acts=True)
        for k, v in ref_acts.items():
            v = v.reshape(c, -1).numpy()
            assert np.max(np.abs(acts[k][r, :c] - v)) <= 1e-4 * max(1.0, np.max(np.abs(v))), k
    print(report)
    assert not bad, (bad, report)


def test_one_rmsprop_step_matches_keras(scenario, engine, odata):
    st, p0 = _one_step(engine, [(0, 2)])
    idx, cnt = st.ws["idx"].cpu().numpy(), st.ws["cnt"].cpu().numpy()
    dkeys = st.ws["drop_key"].cpu().numpy().view(np.uint64)
    p1 = st.params.cpu().numpy()
    for r in range(st.R):
        c = int(cnt[r])
        P = occ.unpack(p0[r])
        rws = idx[r, :c]
        g, _ = occ.gradients(P, odata.x_train[rws], odata.y_train[rws], occ.step_masks(int(dkeys[r]), c))
        opt = occ.KerasRMSprop(P)
        opt.step(P, g)
        d_dev = p1[r] - p0[r]
        d_ref = occ.pack(P) - p0[r]
        # the first RMSprop step moves every weight by ~lr/sqrt(0.1) * sign(g): sign flips only where |g| ~ noise
        diff = np.abs(d_dev - d_ref)
        assert np.mean(diff) < 2e-6
        assert np.mean(diff > 1e-5) < 2e-3


def test_fedavg_aggregation_inside_training_is_np_average(engine):
    import torch
    st = engine.trainer.prepare([(0, 1, 2)], 1)
    for s in range(st.round_len):
        st.step(s)
    before = st.params.cpu().numpy().copy()
    st.aggregate()
    torch.cuda.synchronize()
    sizes = [engine.partner_sizes[p] for p in (0, 1, 2)]
    ref = np.average(before[:, :occ.STRIDE], axis=0, weights=np.asarray(sizes) / np.sum(sizes)).astype(np.float32)
    assert np.array_equal(st.glob.cpu().numpy()[0], ref)
    after = st.params.cpu().numpy()
    lo, hi = st.model.BCAST_SKIP  # W5: not broadcast, the next round's first step reads the coalition row
    for r in range(3):  # broadcast: every partner starts the next round from the average
        assert np.array_equal(after[r][:lo], ref[:lo]) and np.array_equal(after[r][hi:], ref[hi:])
        assert np.array_equal(after[r][lo:hi], before[r][lo:hi])
    st.step(st.round_len)  # first step of round 2: every replica sources W5 from coalition row 0
    torch.cuda.synchronize()
    assert st.ws["w5src"].cpu().tolist() == [0, 0, 0]


def test_eval_loss_independent_of_models_sharing_the_evaluation(engine):
    """the summed loss of a model (the val loss the early-stopping rule compares) must not depend on how
    many models share the evaluation or on the workspace budget - the chunk size follows both.  One model alone
    with a budget for a single chunk, against the same model among 7 others with a budget of a few 256-sample
    chunks (eval_plan then also splits the models into groups): bit-identical loss and hits."""
    from mplc.cnn import eval_plan
    st = engine.trainer.prepare([(0,), (1,), (2,), (0, 1), (0, 2), (1, 2), (0, 1, 2)], 1)
    rows = st.glob.contiguous()
    model = engine.model_impl
    x, y = engine.x_train_d, engine.y_train_d
    n = int(y.numel())
    assert n > 1024
    keep = engine.eval_budget_bytes
    try:
        engine.eval_budget_bytes = 8 << 30
        c1, l1 = model.evaluate(engine, rows[3:4].contiguous(), x, y)
        small = 150 << 20 if model.name == "cifar10_cnn" else 40 << 20
        engine.eval_budget_bytes = small
        chunk, group = eval_plan(n, 7, model.EVAL_SAMPLE_BYTES, model.EVAL_MODEL_BYTES, small)
        assert chunk % 256 == 0 and chunk < n and group < 7, (chunk, group)
        c7, l7 = model.evaluate(engine, rows, x, y)
    finally:
        engine.eval_budget_bytes = keep
    assert c7[3] == c1[0] and l7[3] == l1[0], (c7[3], c1[0], l7[3], l1[0])


def test_values_independent_of_batch_composition(engine):
    all7 = [(0,), (1,), (2,), (0, 1), (0, 2), (1, 2), (0, 1, 2)]
    together = engine.evaluate(all7)
    alone = [engine.evaluate([c])[0] for c in ((1, 2), (2,))]
    assert together[5] == alone[0] and together[2] == alone[1]


def test_coalition_accuracies_vs_oracle(scenario, engine, odata):
    prow, bs = rows(scenario)
    coals = [(0,), (1,), (0, 1), (0, 1, 2)]
    dev = engine.evaluate(coals)
    ref = np.array([occ.coalition_value(odata, prow, bs, c, seed=engine.seed, epochs=engine.epoch_count,
                                        M=engine.minibatch_count)[0] for c in coals])
    diff = np.abs(dev - ref)
    assert np.mean(diff) <= 0.01, (dev, ref)
    assert np.max(diff) <= 0.03, (dev, ref)
    # the models learn (10 classes: chance = 0.1).  RMSprop at lr 1e-4 for 2 epochs: the 270-sample singleton
    # (0,) is still near chance, the larger training sets are well above it
    assert np.all(dev[1:] > 0.3), dev


def test_contributivity_tmcs_on_cifar():
    """TMCS (BASELINE config #4's method) end to end through the batched CIFAR engine."""
    from mplc.contributivity import Contributivity
    sc = make_scenario(partners=3, amounts=(0.2, 0.5, 0.3), M=2, G=4, E=1)
    c = Contributivity(scenario=sc)
    c.compute_contributivity("TMCS", sv_accuracy=0.05)
    assert c.name == "TMC Shapley"
    assert np.all(np.isfinite(c.contributivity_scores))
    assert c.first_charac_fct_calls_count >= 1


def test_empty_minibatch_partner_restarts_from_global_model():
    """a FedAvg partner with fewer rows than minibatch_count has empty minibatches; in those rounds
    it trains nothing and enters the average with the round's global model (the reference builds it fresh
    from the global weights, mplc/multi_partner_learning.py:319).  Scenario refuses such a split
    (mplc/scenario.py's minibatch_count <= min(amounts) * n check), but the engine accepts any partner rows:
    the dense-layer broadcast skip must not leave that partner a stale copy.  Values and final models equal
    the plain copy-back path bit for bit."""
    from mplc.engine import CoalitionEngine
    sc = make_scenario(partners=2, amounts=(0.3, 0.7), M=2, G=2, E=1)
    d = sc.dataset
    rows0 = list(sc.partners_list[0].train_idx[:13])  # 13 rows, 20 minibatches: 7 empty ones
    rows1 = list(sc.partners_list[1].train_idx)
    eng = CoalitionEngine(x_train=d.x_train, y_train=d.y_train, x_val=d.x_val, y_val=d.y_val, x_test=d.x_test,
                          y_test=d.y_test, partner_rows=[rows0, rows1], batch_sizes=[1, 24], epoch_count=1,
                          minibatch_count=20, is_early_stopping=False, model="cifar10_cnn",
                          memory_budget_bytes=4 << 30, eval_budget_bytes=1 << 30)
    assert any(b[m + 1] == b[m] for b in [eng.bounds[0]] for m in range(20))
    coals = [(0, 1), (0,), (1,)]
    skip = eng.evaluate(coals, return_models=True, return_details=True)
    eng.bcast_skip = False
    full = eng.evaluate(coals, return_models=True, return_details=True)
    assert np.array_equal(skip["scores"], full["scores"])
    for a, b in zip(skip["models"][0], full["models"][0]):
        assert np.array_equal(a, b)


def test_all_kernel_timer_is_result_neutral(engine):
    """bench.py's config #4 line times every launch of the CIFAR step in stream (prof_kernel = MPLC_PROF_ALL, event
    arrays): v(S) unchanged, every kernel timed once per step, the stashed schedules count every sample."""
    from mplc.cifar import KERNEL_IDS, CifarModel
    from mplc.profiling import KernelTimer
    coals = [(0,), (1, 2), (0, 1, 2)]
    timer = KernelTimer("all", list(KERNEL_IDS), stash=True)
    engine.profiler = timer
    try:
        timed = engine.evaluate(coals)
    finally:
        engine.profiler = None
    plain = engine.evaluate(coals)
    assert np.array_equal(timed, plain)
    steps = len(timer.stash)
    assert steps > 0
    for k in KERNEL_IDS:
        assert timer.launches(k) == steps and timer.total_ms(k) > 0.0, k
    units = CifarModel.algorithmic_units(timer.stash)
    sizes = engine.partner_sizes
    assert units["samples"] == engine.epoch_count * sum(sizes[p] for c in coals for p in c)
    assert units["dense5_bwd_bytes"] > units["dense5_fwd_bytes"] > 0
