"""Early parameter-gradient reduces (compressai/_ops.py CAI_EARLY_REDUCE_MB): the queued reduce jobs run on a
side stream once their partials pass a byte threshold, while the backward goes on; the final flush joins that
stream.  Same kernels, same jobs, same order per gradient: the flat gradient buffer must be BIT-identical to
the all-at-the-end flush, eager and inside a captured HIP graph (bench.py's form), for a zoo model (C2), a
context model whose hyper branch runs on its own stream (mbt2018-mean, C3) and cheng2020-attn (C4: ResidualUnit
weight-gradient batches, two-stream attention branches); also with the early launches' grid capped
(cai_reduce_jobs_grid: each block walks the batch's blocks)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _step_grads(cuda, name, quality, batch, early_mb, graph, early_blocks=0):
    from compressai import _ops
    from compressai._ops import loss_seed
    from compressai.entropy_models import set_noise_source
    from compressai.losses import RateDistortionLoss
    from compressai.optim import configure_optimizers
    from compressai.zoo import image_models

    torch.manual_seed(0)
    net = image_models[name](quality).to(cuda).train()
    x = torch.rand(batch, 3, 256, 256, device=cuda, generator=torch.Generator(cuda).manual_seed(3))
    opt, aux_opt = configure_optimizers(net, zero_grad_in_step=True)
    crit = RateDistortionLoss(quality)
    cnt, bufs = [0], []

    def source(t):      # fixed noise per call index: the same buffers in every run and replay
        i = cnt[0]
        cnt[0] += 1
        if i == len(bufs):
            g = torch.Generator(cuda).manual_seed(i + 11)
            bufs.append(torch.rand(t.shape, device=cuda, generator=g) - 0.5)
        return bufs[i]

    def fwd_bwd():
        cnt[0] = 0
        opt.zero_grad()
        aux_opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = crit(net(x), x)["loss"]
        loss.backward(loss_seed(loss))

    old = _ops._EARLY_BYTES, _ops._EARLY_BLOCKS
    _ops._EARLY_BYTES, _ops._EARLY_BLOCKS = early_mb * 1e6, early_blocks
    set_noise_source(source)
    try:
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            fwd_bwd()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        opt.flat_grad.zero_()
        if graph:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                fwd_bwd()
            opt.flat_grad.zero_()
            g.replay()
        else:
            fwd_bwd()
        torch.cuda.synchronize()
        return opt.flat_grad.clone()
    finally:
        set_noise_source(None)
        _ops._EARLY_BYTES, _ops._EARLY_BLOCKS = old


@pytest.mark.parametrize("name,quality,batch", [("bmshj2018-hyperprior", 1, 16), ("mbt2018-mean", 1, 8),
                                                ("cheng2020-attn", 6, 2)])
@pytest.mark.parametrize("graph", [False, True])
def test_early_reduce_bit_identical(cuda, name, quality, batch, graph):
    base = _step_grads(cuda, name, quality, batch, 0, graph)
    for mb, blocks in ((16, 0), (64, 0), (64, 24)):
        early = _step_grads(cuda, name, quality, batch, mb, graph, blocks)
        assert torch.isfinite(base).all()
        assert base.abs().sum() > 0
        assert torch.equal(base, early), (mb, blocks, (base - early).abs().max().item())
