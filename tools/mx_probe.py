#!/usr/bin/env python3
"""Determine the operand/scale lane maps of v_mfma_scale_f32_16x16x128_f8f6f4 on the GPU with
one-hot probes (prints which (row, k) each (lane, byte) of an operand feeds, and how scales bind)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tensorflow_k8s_amd.ops._lib import lib  # noqa: E402

ONE = 0x38  # e4m3 1.0


def run(xb, yb, sx, sy):
    X = torch.from_numpy(xb.view('<i4').reshape(64, 8).copy()).cuda()
    Y = torch.from_numpy(yb.view('<i4').reshape(64, 8).copy()).cuda()
    D = torch.zeros(64, 4, device="cuda")
    lib().mx_probe(X, Y, torch.tensor(sx, dtype=torch.int32).cuda(), torch.tensor(sy, dtype=torch.int32).cuda(), D)
    return D.cpu()


def main():
    import numpy as np
    res = {}
    # Y = all ones -> D[i][j] = sum_k X[i][k]: one-hot X at (lane, byte) lights row i everywhere.
    yb = np.full((64, 32), ONE, dtype=np.uint8)
    rows = {}
    for lane in (0, 1, 15, 16, 17, 31, 32, 48, 63):
        for byte in (0, 1, 7, 8, 15, 16, 31):
            xb = np.zeros((64, 32), dtype=np.uint8)
            xb[lane, byte] = ONE
            D = run(xb, yb, [127] * 64, [127] * 64)
            nz = (D != 0).nonzero().tolist()
            # output lane l, reg r -> (i = 4*(l>>4) + r, j = l & 15)
            ij = sorted({(4 * (l >> 4) + r, l & 15) for l, r in nz})
            rows[f"{lane},{byte}"] = sorted({i for i, _ in ij})
    res["x_onehot_rows"] = rows
    # k pairing: X one-hot at (lane 0, byte b); Y one-hot at (lane L, byte c): D != 0 iff same k
    pair = {}
    for b in (0, 1, 8, 16, 31):
        xb = np.zeros((64, 32), dtype=np.uint8)
        xb[0, b] = ONE
        hits = []
        for L in range(0, 64, 16):
            for c in range(32):
                yb2 = np.zeros((64, 32), dtype=np.uint8)
                yb2[L, c] = ONE
                if float(run(xb, yb2, [127] * 64, [127] * 64).abs().sum()) != 0:
                    hits.append((L, c))
        pair[str(b)] = hits
    res["k_pairs_for_x_lane0"] = pair
    # scales: all-ones X,Y (sum = 128), scale of X lane 0 set to 128 (x2)
    xb = np.full((64, 32), ONE, dtype=np.uint8)
    sx = [127] * 64
    sx[0] = 128
    D = run(xb, yb, sx, [127] * 64)
    res["scale_x_lane0_effect"] = sorted({(4 * (l >> 4) + r, l & 15, float(D[l, r])) for l in range(64) for r in range(4)
                                          if float(D[l, r]) != 128.0})[:16]
    sx = [127] * 64
    sx[16] = 128
    D = run(xb, yb, sx, [127] * 64)
    res["scale_x_lane16_effect"] = sorted({(4 * (l >> 4) + r, l & 15, float(D[l, r])) for l in range(64) for r in range(4)
                                           if float(D[l, r]) != 128.0})[:16]
    print(json.dumps(res))


if __name__ == "__main__":
    main()
