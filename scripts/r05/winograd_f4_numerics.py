"""Numerics of Winograd F(4x4,3x3) against F(2x2,3x3) for the MNIST conv2 layer (32 -> 64 channels, 26x26 -> 24x24),
all arithmetic in fp32 as a kernel would do it (transforms in fp32, the per-transform-point GEMM accumulated over the
input channels in order, as the matrix core's fma chain), against the fp64 direct convolution.  DESIGN.md names
F(4x4,3x3) (1.78x fewer multiply-adds than F(2x2,3x3)) as the remaining lever of the conv kernels, "a numerics
question before it is a kernel": this answers the per-layer part of it.

    python scripts/r05/winograd_f4_numerics.py
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "distributed-learning-contributivity_amd"))

F32 = np.float32

# F(2x2,3x3)
BT2 = np.array([[1, 0, -1, 0], [0, 1, 1, 0], [0, -1, 1, 0], [0, 1, 0, -1]], dtype=np.float64)
G2 = np.array([[1, 0, 0], [0.5, 0.5, 0.5], [0.5, -0.5, 0.5], [0, 0, 1]], dtype=np.float64)
AT2 = np.array([[1, 1, 1, 0], [0, 1, -1, -1]], dtype=np.float64)
# F(4x4,3x3) (Lavin & Gray 2016)
BT4 = np.array([[4, 0, -5, 0, 1, 0], [0, -4, -4, 1, 1, 0], [0, 4, -4, -1, 1, 0], [0, -2, -1, 2, 1, 0],
                [0, 2, -1, -2, 1, 0], [0, 4, 0, -5, 0, 1]], dtype=np.float64)
G4 = np.array([[1 / 4, 0, 0], [-1 / 6, -1 / 6, -1 / 6], [-1 / 6, 1 / 6, -1 / 6], [1 / 24, 1 / 12, 1 / 6],
               [1 / 24, -1 / 12, 1 / 6], [0, 0, 1]], dtype=np.float64)
AT4 = np.array([[1, 1, 1, 1, 1, 0], [0, 1, -1, 2, -2, 0], [0, 1, 1, 4, 4, 0], [0, 1, -1, 8, -8, 1]],
               dtype=np.float64)


def direct64(x, w):
    """x [H][W][CI], w [3][3][CI][CO] -> valid conv [H-2][W-2][CO] in fp64."""
    H, W, _ = x.shape
    out = np.zeros((H - 2, W - 2, w.shape[3]))
    for ky in range(3):
        for kx in range(3):
            out += np.einsum("hwc,cd->hwd", x[ky:ky + H - 2, kx:kx + W - 2].astype(np.float64), w[ky, kx])
    return out


def winograd32(x, w, BT, G, AT):
    """fp32 Winograd: U = G g G^T per (ci, co) in fp32, V = B^T d B per tile and ci in fp32, M = sum_ci V U
    accumulated over ci in order in fp32 (an fma chain), Y = A^T M A in fp32."""
    m = AT.shape[0]
    a = BT.shape[0]
    H, W, CI = x.shape
    CO = w.shape[3]
    th, tw = (H - 2) // m, (W - 2) // m
    BT, G, AT = BT.astype(F32), G.astype(F32), AT.astype(F32)
    U = np.einsum("ik,klcd,jl->ijcd", G, w.astype(F32), G).astype(F32)  # [a][a][CI][CO]
    out = np.zeros((th * m, tw * m, CO), dtype=F32)
    for ty in range(th):
        for tx in range(tw):
            d = x[ty * m:ty * m + a, tx * m:tx * m + a].astype(F32)  # [a][a][CI]
            V = np.einsum("ik,klc,jl->ijc", BT, d, BT).astype(F32)
            M = np.zeros((a, a, CO), dtype=F32)
            for ci in range(CI):  # the fma chain over K
                M = (M + V[:, :, ci:ci + 1] * U[:, :, ci, :]).astype(F32)
            Y = np.einsum("ik,klc,jl->ijc", AT, M, AT).astype(F32)
            out[ty * m:ty * m + m, tx * m:tx * m + m] = Y
    return out


def main():
    import torch
    from mplc.dataset import digits_as_mnist
    rng = np.random.default_rng(0)
    x, _ = digits_as_mnist()
    # conv1 (3x3, 1 -> 32, glorot uniform, ReLU) on real digit images: conv2's input
    lim1 = np.sqrt(6 / (9 + 9 * 32))
    w1 = rng.uniform(-lim1, lim1, size=(3, 3, 1, 32))
    lim2 = np.sqrt(6 / (9 * 32 + 9 * 64))
    w2 = rng.uniform(-lim2, lim2, size=(3, 3, 32, 64)).astype(F32)
    rows = []
    for n in range(8):
        img = x[n].reshape(28, 28, 1).astype(np.float64)
        a1 = np.maximum(direct64(img, w1), 0).astype(F32)  # [26][26][32]
        a1 = a1[:24 + 2, :24 + 2]  # both tilings cover 24 x 24
        ref = direct64(a1, w2.astype(np.float64))  # [24][24][64]
        for name, (BT, G, AT) in (("F(2x2,3x3)", (BT2, G2, AT2)), ("F(4x4,3x3)", (BT4, G4, AT4))):
            y = winograd32(a1, w2, BT, G, AT).astype(np.float64)
            err = np.abs(y - ref)
            scale = np.abs(ref).max()
            rows.append((name, n, err.max() / scale, err.mean() / np.abs(ref).mean()))
        # fp32 direct (torch conv2d, the reference's arithmetic class) for scale
        t = torch.nn.functional.conv2d(torch.from_numpy(a1.transpose(2, 0, 1)[None]),
                                       torch.from_numpy(w2.transpose(3, 2, 0, 1).copy())).numpy()[0].transpose(1, 2, 0)
        err = np.abs(t.astype(np.float64) - ref)
        rows.append(("direct fp32", n, err.max() / np.abs(ref).max(), err.mean() / np.abs(ref).mean()))
    for name in ("direct fp32", "F(2x2,3x3)", "F(4x4,3x3)"):
        r = [(a, b) for (nm, _, a, b) in rows if nm == name]
        print(f"{name:12s} max |err| / max |ref|: {max(a for a, _ in r):.2e}   mean |err| / mean |ref|: "
              f"{np.mean([b for _, b in r]):.2e}")


if __name__ == "__main__":
    main()
