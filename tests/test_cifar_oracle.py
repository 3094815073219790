"""CPU: the CIFAR10 oracle (oracle/cifar_cnn.py) restates the reference model/optimizer semantics.

The Keras arithmetic itself cannot run here (no TF): these pin the restatement's own pieces - layer
shapes/parameter count (mplc/dataset.py:167-200: 1,250,858 parameters), glorot limits, the Keras 2.3.1
RMSprop update written out by hand, dropout mask rates and inverted scaling, and fp32-vs-fp64 gradients."""
import numpy as np
import pytest

from oracle import cifar_cnn as occ


def test_layout_matches_keras_parameter_count():
    total = sum(int(np.prod(shape)) for _, shape in occ.OFF.values())
    assert total == 1250858  # Keras model.count_params() of the reference architecture
    ends = sorted((off, off + int(np.prod(shape))) for off, shape in occ.OFF.values())
    assert all(a[1] <= b[0] for a, b in zip(ends, ends[1:]))  # no overlap
    assert ends[-1][1] <= occ.STRIDE and occ.STRIDE % 64 == 0


@pytest.mark.parametrize("name,fan", [("W1", 27 + 288), ("W2", 576), ("W3", 288 + 576), ("W4", 1152),
                                      ("W5", 2304 + 512), ("W6", 512 + 10)])
def test_glorot_limits(name, fan):
    assert occ.LIMITS[name] == np.float32(np.sqrt(6.0 / fan))


def test_init_params_range_and_zero_biases():
    row = occ.init_params(12345)
    for name, (off, shape) in occ.OFF.items():
        v = row[off:off + int(np.prod(shape))]
        if name.startswith("b"):
            assert not v.any()
        else:
            assert np.max(np.abs(v)) <= occ.LIMITS[name] and np.std(v) > 0.5 * occ.LIMITS[name] / np.sqrt(3)
    gaps = np.ones(occ.STRIDE, dtype=bool)
    for off, shape in occ.OFF.values():
        gaps[off:off + int(np.prod(shape))] = False
    assert not row[gaps].any()


def test_dropout_masks_rates_and_keys():
    k = occ.fedavg_drop_key(99, 1, 2, 3)
    assert k != occ.fedavg_drop_key(99, 1, 2, 4) and k != occ.single_drop_key(99, 1, 3)
    m2 = occ.dropout_keep(k, "L2", 11, 7200)
    m5 = occ.dropout_keep(k, "L5", 11, 512)
    assert abs(m2.mean() - 0.75) < 0.01 and abs(m5.mean() - 0.5) < 0.02
    assert np.array_equal(m2, occ.dropout_keep(k, "L2", 11, 7200))  # deterministic
    assert not np.array_equal(m2[0], m2[1])                          # per-slot


def test_dropout_is_inverted_and_scaled_in_fp32():
    import torch
    x = torch.full((2, 15, 15, 32), 3.0)
    keep = torch.ones_like(x)
    keep[0, 0, 0, 0] = 0.0
    y = occ._dropout(x, keep, 0.25)
    assert float(y[0, 0, 0, 0]) == 0.0
    assert float(y[0, 0, 0, 1]) == float(np.float32(3.0) * (np.float32(1) / np.float32(0.75)))


def test_keras_rmsprop_update_by_hand():
    import torch
    p = {"w": torch.tensor([1.0, -2.0, 0.5], dtype=torch.float32)}
    g1 = {"w": torch.tensor([0.1, -0.3, 0.0], dtype=torch.float32)}
    g2 = {"w": torch.tensor([0.2, 0.1, -0.4], dtype=torch.float32)}
    opt = occ.KerasRMSprop(p)
    w = p["w"].numpy().astype(np.float32).copy()
    a = np.zeros(3, dtype=np.float32)
    for it, g in enumerate((g1, g2)):
        opt.step(p, g)
        gn = g["w"].numpy()
        lr_t = np.float32(1e-4) * (np.float32(1) / (np.float32(1) + np.float32(1e-6) * np.float32(it)))
        a = np.float32(0.9) * a + np.float32(0.1) * (gn * gn)
        w = w - lr_t * gn / (np.sqrt(a) + np.float32(1e-7))
        np.testing.assert_allclose(p["w"].numpy(), w, rtol=0, atol=1e-7)
    assert opt.iterations == 2


def test_forward_shapes_and_gradients_fp32_vs_fp64():
    import torch
    rng = np.random.default_rng(0)
    P = occ.unpack(occ.init_params(7))
    x = torch.from_numpy(rng.random((3, 32, 32, 3), dtype=np.float32))
    y = torch.tensor([1, 4, 9])
    masks = occ.step_masks(occ.single_drop_key(5, 0, 0), 3)
    logits, acts = occ.forward(P, x, masks, return_acts=True)
    assert logits.shape == (3, 10)
    assert acts["a1"].shape == (3, 32, 32, 32) and acts["d2"].shape == (3, 15, 15, 32)
    assert acts["a3"].shape == (3, 15, 15, 64) and acts["d4"].shape == (3, 2304) and acts["d5"].shape == (3, 512)
    g32, _ = occ.gradients(P, x, y, masks)
    g64, _ = occ.gradients(P, x, y, masks, dtype=torch.float64)
    for k in g32:
        ref = g64[k].numpy().ravel()
        assert np.linalg.norm(g32[k].numpy().ravel() - ref) <= 1e-4 * max(np.linalg.norm(ref), 1e-12)
