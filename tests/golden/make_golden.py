"""Generate the golden fixtures in tests/golden/*.npz from the CPU oracle.

    python tests/golden/make_golden.py          # rewrites the .npz files

The reference itself may not be executed in this environment,
so these vectors are produced by the oracle restatement (oracle/cai_oracle.py)
on seeded inputs with injected quantisation noise.  They freeze the oracle's
outputs so that (a) a CPU test notices any drift of the restatement and (b)
the GPU tests can compare the HIP path with stored numbers.  Files are plain
npz (loaded with allow_pickle=False); each holds inputs, injected noise,
upstream gradients and expected outputs/gradients.
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import cai_oracle as O  # noqa: E402


def _np(d):
    return {k: v.detach().cpu().numpy().astype(np.float32) if v.dtype.is_floating_point else v.detach().cpu().numpy()
            for k, v in d.items()}


def gaussian_conditional():
    g = torch.Generator().manual_seed(11)
    x = torch.randn(4, 8, 8, 8, generator=g) * 3
    scales = torch.rand(4, 8, 8, 8, generator=g) * 4 + 0.01
    means = torch.randn(4, 8, 8, 8, generator=g)
    noise = torch.rand(4, 8, 8, 8, generator=g) - 0.5
    gq = torch.randn(4, 8, 8, 8, generator=g)
    glik = torch.randn(4, 8, 8, 8, generator=g)
    gc = O.GaussianConditional(None)
    out = {"x": x, "scales": scales, "means": means, "noise": noise, "gq": gq, "glik": glik}
    for training in (True, False):
        xx, ss, mm = (t.clone().requires_grad_() for t in (x, scales, means))
        with O.NoiseFeed(tensors=[noise]):
            q, lik = gc(xx, ss, mm, training=training)
        ((q * gq).sum() + (lik * glik).sum()).backward()
        tag = "train" if training else "eval"
        out.update({f"{tag}_q": q, f"{tag}_lik": lik, f"{tag}_dx": xx.grad, f"{tag}_dscales": ss.grad,
                    f"{tag}_dmeans": mm.grad})
    return out


def entropy_bottleneck():
    torch.manual_seed(12)
    eb = O.EntropyBottleneck(8)
    g = torch.Generator().manual_seed(13)
    with torch.no_grad():   # move off the init point so every parameter matters
        for p in eb.parameters():
            p.add_(torch.randn(p.shape, generator=g) * 0.1)
    x = torch.randn(4, 8, 8, 8, generator=g) * 2
    noise = torch.rand(4, 8, 8, 8, generator=g) - 0.5
    gq = torch.randn(4, 8, 8, 8, generator=g)
    glik = torch.randn(4, 8, 8, 8, generator=g)
    out = {"x": x, "noise": noise, "gq": gq, "glik": glik}
    out.update({f"param.{k}": v.detach().clone() for k, v in eb.state_dict().items()})
    for training in (True, False):
        eb.zero_grad()
        xx = x.clone().requires_grad_()
        with O.NoiseFeed(tensors=[noise]):
            q, lik = eb(xx, training=training)
        ((q * gq).sum() + (lik * glik).sum()).backward()
        tag = "train" if training else "eval"
        out.update({f"{tag}_q": q, f"{tag}_lik": lik, f"{tag}_dx": xx.grad})
        out.update({f"{tag}_grad.{n}": p.grad.clone() for n, p in eb.named_parameters() if p.grad is not None})
    eb.zero_grad()
    aux = eb.loss()
    aux.backward()
    out["aux_loss"] = aux.reshape(1)
    out["aux_dquantiles"] = eb.quantiles.grad
    return out


def gdn():
    out = {}
    g = torch.Generator().manual_seed(14)
    x = torch.randn(2, 32, 8, 8, generator=g)
    gy = torch.randn(2, 32, 8, 8, generator=g)
    out.update({"x": x, "gy": gy})
    for inverse in (False, True):
        m = O.GDN(32, inverse=inverse)
        with torch.no_grad():
            m.beta.add_(torch.rand(m.beta.shape, generator=g) * 0.5)
            m.gamma.add_(torch.rand(m.gamma.shape, generator=g) * 0.05)
        xx = x.clone().requires_grad_()
        y = m(xx)
        (y * gy).sum().backward()
        tag = "igdn" if inverse else "gdn"
        out.update({f"{tag}_beta": m.beta.detach().clone(), f"{tag}_gamma": m.gamma.detach().clone(),
                    f"{tag}_y": y, f"{tag}_dx": xx.grad, f"{tag}_dbeta": m.beta.grad, f"{tag}_dgamma": m.gamma.grad})
    return out


def scale_hyperprior():
    torch.manual_seed(15)
    net = O.ScaleHyperprior(32, 48)
    x = torch.rand(2, 3, 64, 64, generator=torch.Generator().manual_seed(16))
    feed = O.NoiseFeed(record=torch.Generator().manual_seed(17))
    with feed:
        res = net(x)
    crit = O.RateDistortionLoss(3)(res, x)
    crit["loss"].backward()
    out = {"x": x, "x_hat": res["x_hat"], "lik_y": res["likelihoods"]["y"], "lik_z": res["likelihoods"]["z"],
           "loss": crit["loss"].reshape(1), "bpp_loss": crit["bpp_loss"].reshape(1),
           "mse_loss": crit["mse_loss"].reshape(1)}
    out.update({f"noise{i}": n for i, n in enumerate(feed.drawn)})
    out.update({f"param.{k}": v.detach().clone() for k, v in net.state_dict().items()})
    keep = ("g_a.0.weight", "g_a.1.beta", "g_a.1.gamma", "g_a.6.bias", "g_s.1.gamma", "g_s.6.weight", "g_s.6.bias",
            "h_a.0.weight", "h_s.4.bias", "entropy_bottleneck._matrix0", "entropy_bottleneck._factor3")
    named = dict(net.named_parameters())
    out.update({f"grad.{n}": named[n].grad for n in keep})
    net.eval()
    ev = O.entropy_estimation(net, x)
    out["eval_bpp"] = torch.tensor([ev["bpp"]])
    out["eval_psnr"] = torch.tensor([ev["psnr"]])
    return out


GENERATORS = {"gaussian_conditional": gaussian_conditional, "entropy_bottleneck": entropy_bottleneck, "gdn": gdn,
              "scale_hyperprior": scale_hyperprior}


def load(name):
    with np.load(os.path.join(HERE, f"{name}.npz"), allow_pickle=False) as f:
        return {k: torch.from_numpy(f[k]) for k in f.files}


def main():
    torch.set_num_threads(1)
    for name, fn in GENERATORS.items():
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **_np(fn()))
        print("wrote", name)


if __name__ == "__main__":
    main()
