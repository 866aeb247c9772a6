"""Which lane / byte of the scale VGPRs of v_mfma_scale_f32_16x16x128_f8f6f4
scales which (row, K-block) of each operand? (tools/micro/mfma_scale_probe.hip)

Operand data: every byte of lane l is fp8 e4m3 v(l // 16) with v = 1, 2, 4, 8,
the other operand all 1.0; neutral scales 127 (2^0) everywhere but one lane
whose four scale bytes are 128 (2^1). Output element D[i][j] (lane l holds
D[4 (l // 16) + r][l % 16]) = 32 (1 + 2 + 4 + 8) + 32 v(g) if (row i, block g)
took the doubled scale: the probe prints, per lane, the rows it scaled and the
data value of the block (hence which lane group's K-bytes the block is), for
the first operand (scale_a, rows = D rows) and the second (scale_b, columns =
D columns). A byte-select run then sets only byte k of one lane to 128 and
tries opsel 0..3."""
import ctypes
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, "micro", "mfma_scale_probe.so"))
lib.probe_run.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 5
dev = torch.device("cuda:0")
E4 = {1: 0x38, 2: 0x40, 4: 0x48, 8: 0x50}


def words(val_of_lane):
    w = torch.empty(64, 8, dtype=torch.int32)
    for l in range(64):
        b = val_of_lane(l)
        w[l, :] = b | (b << 8) | (b << 16) | (b << 24)
    return w.to(dev)


def run(oa, ob, a, b, sa, sb):
    out = torch.zeros(64, 4, device=dev)
    sa_t = torch.tensor(sa, dtype=torch.int64).to(torch.int32).to(dev)
    sb_t = torch.tensor(sb, dtype=torch.int64).to(torch.int32).to(dev)
    rc = lib.probe_run(oa, ob, a.data_ptr(), b.data_ptr(), sa_t.data_ptr(), sb_t.data_ptr(), out.data_ptr())
    assert rc == 0, rc
    D = torch.empty(16, 16)
    o = out.cpu()
    for l in range(64):
        for r in range(4):
            D[4 * (l // 16) + r, l % 16] = o[l, r]
    return D


NEUT = 0x7F7F7F7F
DBL = 0x80808080
res = {"scale_a": {}, "scale_b": {}, "opsel_a": {}, "opsel_b": {}}
vals = lambda l: E4[[1, 2, 4, 8][l // 16]]
ones = words(lambda l: 0x38)
var = words(vals)
base = run(0, 0, var, ones, [NEUT] * 64, [NEUT] * 64)
print("neutral D[0][0] =", base[0, 0].item(), "(expect 480)")
for L in range(64):
    sa = [NEUT] * 64
    sa[L] = DBL
    D = run(0, 0, var, ones, sa, [NEUT] * 64)
    rows = sorted({i for i in range(16) if (D[i, :] != 480).any()})
    extra = sorted({(D[i, 0] - base[i, 0]).item() / 32 for i in rows})
    res["scale_a"][L] = (rows, extra)
for L in range(64):
    sb = [NEUT] * 64
    sb[L] = DBL
    D = run(0, 0, ones, var, [NEUT] * 64, sb)
    cols = sorted({j for j in range(16) if (D[:, j] != 480).any()})
    extra = sorted({(D[0, j] - 480).item() / 32 for j in cols})
    res["scale_b"][L] = (cols, extra)
for k in range(4):
    for op in range(4):
        sa = [NEUT] * 64
        sa[5] = (NEUT & ~(0xFF << (8 * k))) | (0x80 << (8 * k))
        D = run(op, 0, var, ones, sa, [NEUT] * 64)
        res["opsel_a"][f"byte{k}_opsel{op}"] = bool((D != 480).any())
        sb = [NEUT] * 64
        sb[5] = (NEUT & ~(0xFF << (8 * k))) | (0x80 << (8 * k))
        D = run(0, op, ones, var, [NEUT] * 64, sb)
        res["opsel_b"][f"byte{k}_opsel{op}"] = bool((D != 480).any())
for k in ("scale_a", "scale_b"):
    print(k)
    for L, v in res[k].items():
        print(f"  lane {L:2d}: {'rows' if k == 'scale_a' else 'cols'} {v[0]} block value {v[1]}")
print("opsel_a", res["opsel_a"])
print("opsel_b", res["opsel_b"])
if len(sys.argv) > 1:
    json.dump({k: {str(kk): vv for kk, vv in v.items()} for k, v in res.items()}, open(sys.argv[1], "w"), indent=1)
