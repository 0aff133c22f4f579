"""bench.py's own step at its own config, checked against the oracle.

The timed region of bench.py (BASELINE.json configs[1]: bmshj2018-hyperprior q1 (128, 192), 256x256, B=16,
bf16) differs from the model-level parity tests in how it runs, not in what it computes: the gradients land
straight in FusedAdam's flat buffer (the kernels accumulate into it), the parameter-gradient reduces are
deferred to one batched launch at the end of the backward, and forward + backward are replayed from a captured
HIP graph.  This test builds that step the way bench.py does (configure_optimizers with zero_grad_in_step,
warm-up on a side stream, torch.cuda.graph capture, the persistent loss seed) with the oracle's noise injected,
replays it once and compares the flat gradient buffer with the oracle's fp32 CPU gradients (bf16 bars of
test_production_mix_gpu.py); then the fused clip + Adam step is compared with torch's clip_grad_norm_ +
torch.optim.Adam applied to the same gradients (train.py:176-180).
"""
import math

import pytest
import torch

import cai_oracle as O

pytestmark = pytest.mark.gpu

GRAD_COS, TENSOR_COS, BF16_LOSS = 0.9999, 0.98, 1e-3


def test_bench_step_matches_oracle(cuda):
    from compressai._ops import loss_seed
    from compressai.entropy_models import set_noise_source
    from compressai.losses import RateDistortionLoss
    from compressai.optim import configure_optimizers
    from compressai.zoo import model_architectures

    torch.manual_seed(0)
    ref = O.ARCHS["bmshj2018-hyperprior"](128, 192)
    net = model_architectures["bmshj2018-hyperprior"](128, 192)
    net.load_state_dict(ref.state_dict())
    net = net.to(cuda).train()
    x = torch.rand(16, 3, 256, 256, generator=torch.Generator().manual_seed(90))
    feed = O.NoiseFeed(record=torch.Generator().manual_seed(91))
    with feed:
        out_r = ref(x)
    cr = O.RateDistortionLoss(1)(out_r, x)
    cr["loss"].backward()
    drawn = [n.to(cuda) for n in feed.drawn]

    opt, aux_opt = configure_optimizers(net, zero_grad_in_step=True)
    criterion = RateDistortionLoss(1)
    xd = x.to(cuda)
    state = {"i": 0}

    def source(t):      # the same buffers every call: the captured graph reads them by address
        n = drawn[state["i"] % len(drawn)]
        state["i"] += 1
        return n

    def fwd_bwd():      # bench.py fwd(): zero_grad launches nothing, the Adam kernels clear the gradients
        opt.zero_grad()
        aux_opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = net(xd)
            crit = criterion(out, xd)
        state["loss"] = crit["loss"].detach()
        crit["loss"].backward(loss_seed(crit["loss"]))

    set_noise_source(source)
    try:
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            fwd_bwd()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            fwd_bwd()
        opt.flat_grad.zero_()
        aux_opt.flat_grad.zero_()
        graph.replay()
        torch.cuda.synchronize()
    finally:
        set_noise_source(None)

    eloss = abs(state["loss"].item() - cr["loss"].item()) / abs(cr["loss"].item())
    pr = dict(ref.named_parameters())
    tcos, dots, na, nb = {}, 0.0, 0.0, 0.0
    grads = {}
    for n, p in net.named_parameters():
        gr = pr[n].grad
        if gr is None or n.endswith(".quantiles"):
            continue
        g = p.grad.detach().double().cpu()
        grads[n] = p.grad.detach().clone()
        assert torch.isfinite(g).all(), n
        tcos[n] = float(torch.nn.functional.cosine_similarity(g.flatten(), gr.double().flatten(), dim=0))
        dots += float((g * gr.double()).sum())
        na += float((g ** 2).sum())
        nb += float((gr.double() ** 2).sum())
    cos = dots / math.sqrt(na * nb)
    low = sorted(tcos.items(), key=lambda kv: kv[1])[:3]
    print(f"\nbench step (graph, FusedAdam direct gradients, deferred reduces): loss {eloss:.3e} grad cos {cos:.6f} "
          f"lowest {low}; {len(tcos)} tensors")
    assert len(tcos) == sum(1 for n, p in net.named_parameters() if not n.endswith(".quantiles"))
    assert eloss < BF16_LOSS
    assert cos > GRAD_COS
    assert low[0][1] > TENSOR_COS, low

    # the fused clip_grad_norm_(1.0) + Adam step on these gradients == torch's on a copy
    before = {n: p.detach().clone() for n, p in net.named_parameters()}
    opt.step(max_norm=1.0)
    torch.cuda.synchronize()
    names = sorted(grads)
    tw = [torch.nn.Parameter(before[n].clone()) for n in names]
    for t, n in zip(tw, names):
        t.grad = grads[n].clone()
    torch.nn.utils.clip_grad_norm_(tw, 1.0)
    torch.optim.Adam(tw, lr=1e-4).step()
    for t, n in zip(tw, names):
        p = dict(net.named_parameters())[n]
        d = (p.detach() - t.detach()).abs().max().item()
        assert d <= 1e-3 * 1e-4 + 1e-6 * before[n].abs().max().item(), (n, d)
    assert torch.count_nonzero(opt.flat_grad).item() == 0     # zero_grad_in_step: the step cleared them
