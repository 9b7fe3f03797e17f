"""Which rounding order does the public mmad_adam reproduce?  One flat Adam step
from a seeded state on the GPU (mmad_adam), against torch CPU single-tensor
Adam, torch GPU single-tensor / foreach Adam, and numpy float32 emulations of
the candidate orders.  Prints the fraction of bit-equal p per pair and the
largest difference in units of 2^-23 * max(|p0|, |p|).
Usage (GPU box): python tools/adam_probe.py"""
import sys

sys.path.insert(0, ".")
import numpy as np
import torch

from icra2021_multimodal_ad_amd import _native
from icra2021_multimodal_ad_amd._native import call, ptr, stream_ptr


def state(step, n=4099):
    g_ = torch.Generator().manual_seed(step)
    p0 = torch.randn(n, generator=g_) * 0.05
    g = torch.randn(n, generator=g_) * 1e-2
    m0 = torch.randn(n, generator=g_) * 1e-3 if step > 1 else torch.zeros(n)
    v0 = torch.rand(n, generator=g_) * 1e-5 if step > 1 else torch.zeros(n)
    return p0, g, m0, v0


def torch_adam(p0, g, m0, v0, step, lr, betas, dev, foreach):
    prm = torch.nn.Parameter(p0.clone().to(dev))
    opt = torch.optim.Adam([prm], lr=lr, betas=betas, eps=1e-8, foreach=foreach)
    opt.state[prm] = {"step": torch.tensor(float(step - 1)), "exp_avg": m0.clone().to(dev),
                      "exp_avg_sq": v0.clone().to(dev)}
    prm.grad = g.clone().to(dev)
    opt.step()
    st = opt.state[prm]
    return prm.detach().cpu(), st["exp_avg"].cpu(), st["exp_avg_sq"].cpu()


def cmp(name, a, b, p0):
    a, b = a.double(), b.double()
    scale = torch.maximum(p0.double().abs(), b.abs())
    d = ((a - b).abs() / scale * 2 ** 23).max().item()
    print(f"  {name:40s} equal {float((a == b).double().mean()):.5f}  max diff {d:.2f} ulp(scale)")


def main():
    lib = _native.load()
    for betas, step, lr in (((0.9, 0.999), 1, 1e-3), ((0.9, 0.999), 3, 1e-3), ((0.8, 0.95), 2, 3e-4)):
        p0, g, m0, v0 = state(step)
        b1, b2 = betas
        step_size = lr / (1.0 - b1 ** step)
        bc2_sqrt = (1.0 - b2 ** step) ** 0.5
        dp, dg, dm, dv = (t.clone().cuda() for t in (p0, g, m0, v0))
        call("mmad_adam", p0.numel(), ptr(dp), ptr(dg), ptr(dm), ptr(dv), b1, b2, 1e-8, step_size, bc2_sqrt,
             None, 0, stream_ptr())
        torch.cuda.synchronize()
        gp, gm, gv = dp.cpu(), dm.cpu(), dv.cpu()
        cp, cm, cv = torch_adam(p0, g, m0, v0, step, lr, betas, "cpu", False)
        tp, tm, tv = torch_adam(p0, g, m0, v0, step, lr, betas, "cuda", False)
        fp, fm, fv = torch_adam(p0, g, m0, v0, step, lr, betas, "cuda", True)
        print(f"betas {betas} step {step} lr {lr}: m==cpu {torch.equal(gm, cm)} v==cpu {torch.equal(gv, cv)}")
        f = np.float32
        M, V = gm.numpy(), gv.numpy()
        ss, bc2, eps = f(step_size), f(bc2_sqrt), f(1e-8)
        sq = np.sqrt(V.astype(np.float64)).astype(f)
        den = (sq / bc2 + eps).astype(f)
        e1 = torch.from_numpy((p0.numpy() + (f(-ss) * M) / den).astype(f))
        e2 = torch.from_numpy((p0.numpy() + f(-ss) * (M / den)).astype(f))
        cmp("mmad_adam vs torch cpu single", gp, cp, p0)
        cmp("mmad_adam vs torch gpu single", gp, tp, p0)
        cmp("mmad_adam vs torch gpu foreach", gp, fp, p0)
        cmp("mmad_adam vs emul p+(-s*m)/d", gp, e1, p0)
        cmp("mmad_adam vs emul p+(-s)*(m/d)", gp, e2, p0)
        cmp("torch cpu vs emul p+(-s*m)/d", cp, e1, p0)
        cmp("torch gpu single vs emul p+(-s)*(m/d)", tp, e2, p0)
        d_den = (torch.from_numpy(den))
        print("  denom emul vs torch cpu:",
              float(((v0 if False else torch.from_numpy(V)).sqrt() / bc2_sqrt + 1e-8 == d_den).double().mean()))
        _ = lib


if __name__ == "__main__":
    main()
