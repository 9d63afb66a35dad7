"""Probe: the front-end intermediates of one masked-batch call (max_layers 0) read back from the
workspace tail (feA / feB / feC, model.hip carve order), fe_fuse_dw2 on vs off, for bf16 and fp16:
which stage first differs.   python tools/dw2_probe2.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from chunkformer_amd.config import LARGE  # noqa: E402
from chunkformer_amd.encoder import ChunkFormerEncoder  # noqa: E402
from chunkformer_amd.weights import synthetic_features, synthetic_state_dict  # noqa: E402


def au(x):
    return (x + 255) // 256 * 256


def main():
    sd = synthetic_state_dict(LARGE, 0)
    xs = synthetic_features([3000, 1234, 6000], 5)
    lens = torch.tensor([x.shape[0] for x in xs], dtype=torch.int32)
    d, T2, T3 = 512, 129, 64
    for dt in ("bf16", "fp16"):
        enc = ChunkFormerEncoder(LARGE, sd, dtype=dt)
        enc.set_option("max_layers", 0)
        res = {}
        for fuse in (0, 1):
            enc.set_option("fe_fuse_dw2", fuse)
            out, _, nch, _, _, _ = enc.forward_parallel_chunk(xs, lens, 64, 128, 128)
            torch.cuda.synchronize()
            nwin = sum(nch)
            ws = enc._ws
            total = ws.numel() - 4096
            c_sz, b_sz = nwin * T3 * 9 * d * 2, nwin * T2 * 19 * d * 2
            c0 = total - au(c_sz)
            b0 = c0 - au(b_sz)
            a0 = b0 - au(b_sz)
            v = torch.float16 if dt == "fp16" else torch.bfloat16
            res[fuse] = {"A": ws[a0:a0 + b_sz].view(v).clone(), "B": ws[b0:b0 + b_sz].view(v).clone(),
                         "C": ws[c0:c0 + c_sz].view(v).clone(), "out": out.clone()}
        u, f = res[0], res[1]
        n3 = nwin * T3 * 9 * d
        # unfused: A = dw2 out (first nwin*T3*9*d), B = pw1 out; fused: A = conv0+dw1 out, B = dw2 out
        dw2_u, dw2_f = u["A"][:n3], f["B"][:n3]
        def cmp(a, b):
            ne = (a != b)
            return int(ne.sum()), float((a.float() - b.float()).abs().max())
        print(dt, "nwin", nwin, "dw2 out differ", cmp(dw2_u, dw2_f), "pw2 out differ", cmp(u["C"], f["C"]),
              "final", cmp(u["out"], f["out"]), flush=True)
        if cmp(dw2_u, dw2_f)[0]:
            ne = (dw2_u != dw2_f).nonzero().flatten()[:10]
            print("  first idx", ne.tolist(), "unfused", dw2_u[ne].float().tolist(), "fused", dw2_f[ne].float().tolist())
            idx = ne[0].item()
            row, ch = idx // d, idx % d
            print("  row", row, "ch", ch, "window", row // (T3 * 9), "t3", (row % (T3 * 9)) // 9, "f3", row % 9)
            # dw2 of the unfused pw1 rows in float64, at the differing outputs
            pw1 = u["B"][: nwin * T2 * 19 * d].view(nwin, T2, 19, d).double()
            wk = sd["encoder.embed.conv.5.weight"].double().view(d, 3, 3).cuda()
            bk = sd["encoder.embed.conv.5.bias"].double().cuda()
            for k in ne.tolist()[:10]:
                r, c = k // d, k % d
                wn, t3, f3 = r // (T3 * 9), (r % (T3 * 9)) // 9, r % 9
                acc = bk[c] + sum(wk[c, i, v] * pw1[wn, 2 * t3 + i, 2 * f3 + v, c] for i in range(3) for v in range(3))
                print("   f64", float(acc), "-> f16", float(torch.tensor(float(acc)).half()), "unfused", float(dw2_u[k]),
                      "fused", float(dw2_f[k]))


if __name__ == "__main__":
    main()
