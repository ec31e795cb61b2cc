"""A/B timing of the fused x3 Swin MLP (mmr_x3_swin_mlp) workgroup forms at the Swin-T stage-1 / stage-2 shapes (B = 256):
8-wave vs 4-wave workgroups (mmr_pin_variant MMR_PIN_X3_MLP; C = 96 only), alternated over several rounds on
one box, each output checked bit-identical.  Diagnostic only.
usage: python tools/x3_mlp_ab.py [B] [rounds]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mmr_amd import ops  # noqa: E402


def timeit(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    for C, T in ((96, B * 3136), (192, B * 784)):
        g = torch.Generator().manual_seed(C)
        x = (torch.randn(T, C, generator=g) * 1.5).to("cuda")
        gm, bt = (1 + 0.1 * torch.randn(C, generator=g)).to("cuda"), (0.1 * torch.randn(C, generator=g)).to("cuda")
        w1 = (torch.randn(4 * C, C, generator=g) * C ** -0.5).to("cuda")
        w2 = (torch.randn(C, 4 * C, generator=g) * (4 * C) ** -0.5).to("cuda")
        b1, b2 = (0.1 * torch.randn(4 * C, generator=g)).to("cuda"), (0.1 * torch.randn(C, generator=g)).to("cuda")
        pack = ops.x3_swin_mlp_pack(w1, w2)
        forms = (0, 1) if C == 96 else (-1,)
        outs, res = {}, {w: [] for w in forms}
        for _ in range(rounds):
            for w in forms:
                with ops.pinned(ops.PIN_X3_MLP, w):
                    res[w].append(timeit(lambda: ops.x3_swin_mlp(x, gm, bt, pack, b1, b2, 1e-5)))
                    outs[w] = ops.x3_swin_mlp(x, gm, bt, pack, b1, b2, 1e-5)
        same = all(torch.equal(outs[w], outs[forms[0]]) for w in forms)
        line = "  ".join(f"form {w}: " + " ".join(f"{t:7.1f}" for t in res[w]) + " us" for w in forms)
        print(f"C={C:3d} T={T:7d}  {line}  bit-identical={same}", flush=True)


if __name__ == "__main__":
    main()
