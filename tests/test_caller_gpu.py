"""The reference's caller sequence on the product models (examples/train.py:155-186):

    optimizer.zero_grad(); aux_optimizer.zero_grad()
    with autocast(): out = model(d); crit = criterion(out, d)
    scaler.scale(crit["loss"]).backward(); scaler.unscale_(optimizer)
    clip_grad_norm_(model.parameters(), clip_max_norm); scaler.step(optimizer)
    with autocast(): aux_loss = model.aux_loss()
    scaler.scale(aux_loss).backward(); scaler.unscale_(aux_optimizer); scaler.step(aux_optimizer); scaler.update()

run with torch.optim.Adam (the reference's optimizer) and with FusedAdam as a drop-in torch Optimizer, plus
FusedAdam's checkpoint format (torch.optim.Adam.state_dict, train.py:407,419,475), its handling of gradients a
caller detached (model.zero_grad()), GradScaler's non-finite skip rule, and the autocast dtype policy.
"""
import math

import pytest
import torch

import cai_oracle as O

pytestmark = pytest.mark.gpu


def _pair(name, args, dev):
    from compressai.zoo import model_architectures

    torch.manual_seed(0)
    ref = O.ARCHS[name](*args)
    net = model_architectures[name](*args)
    net.load_state_dict(ref.state_dict())
    return ref, net.to(dev)


def _torch_optimizers(net, lr, aux_lr):
    """train.py:111-142 verbatim in structure: torch.optim.Adam over sorted names."""
    named = dict(net.named_parameters())
    main = sorted(n for n, p in named.items() if not n.endswith(".quantiles") and p.requires_grad)
    aux = sorted(n for n, p in named.items() if n.endswith(".quantiles") and p.requires_grad)
    return (torch.optim.Adam((named[n] for n in main), lr=lr), torch.optim.Adam((named[n] for n in aux), lr=aux_lr))


def _reference_step(net, criterion, d, optimizer, aux_optimizer, scaler, clip_max_norm, dtype=None):
    optimizer.zero_grad()
    aux_optimizer.zero_grad()
    with torch.autocast("cuda", dtype=dtype or torch.bfloat16, enabled=dtype is not None):
        out_net = net(d)
        out_criterion = criterion(out_net, d)
    scaler.scale(out_criterion["loss"]).backward()
    scaler.unscale_(optimizer)
    torch.nn.utils.clip_grad_norm_(net.parameters(), clip_max_norm)
    scaler.step(optimizer)
    with torch.autocast("cuda", dtype=dtype or torch.bfloat16, enabled=dtype is not None):
        aux_loss = net.aux_loss()
    scaler.scale(aux_loss).backward()
    scaler.unscale_(aux_optimizer)
    scaler.step(aux_optimizer)
    scaler.update()
    return out_criterion


def _params_close(net, ref, lr):
    pr = dict(ref.named_parameters())
    diffs = torch.cat([(p.detach().cpu() - pr[n].detach()).abs().flatten() for n, p in net.named_parameters()])
    # Adam moves every element by ~lr early on; an element whose gradient is within rounding of zero may flip
    assert (diffs > 0.1 * lr).float().mean().item() < 1e-3
    assert diffs.median().item() < 1e-3 * lr


@pytest.mark.parametrize("opt_kind", ["torch.optim.Adam", "FusedAdam"])
def test_reference_caller_sequence_fp32(cuda, opt_kind):
    """train.py:155-186 with GradScaler + clip_grad_norm_ on the product model == the oracle's fp32 step."""
    from compressai.entropy_models import set_noise_source
    from compressai.losses import RateDistortionLoss
    from compressai.optim import configure_optimizers

    ref, net = _pair("bmshj2018-hyperprior", (32, 48), cuda)
    lr, aux_lr = 1e-2, 1e-1
    opt_r, aux_r = O.configure_optimizers(ref, lr=lr, aux_lr=aux_lr)
    if opt_kind == "FusedAdam":
        opt, aux = configure_optimizers(net, lr=lr, aux_lr=aux_lr)
    else:
        opt, aux = _torch_optimizers(net, lr, aux_lr)
    scaler = torch.amp.GradScaler("cuda")
    x = torch.rand(2, 3, 64, 64, generator=torch.Generator().manual_seed(3))
    for it in range(2):
        feed = O.NoiseFeed(record=torch.Generator().manual_seed(20 + it))
        with feed:
            O.train_step(ref, O.RateDistortionLoss(1), x, opt_r, aux_r)
        q = [n.to(cuda) for n in feed.drawn]
        set_noise_source(lambda t: q.pop(0))
        try:
            _reference_step(net, RateDistortionLoss(1), x.to(cuda), opt, aux, scaler, 1.0)
        finally:
            set_noise_source(None)
    _params_close(net, ref, lr)


def test_reference_caller_sequence_bf16_autocast(cuda):
    """The same sequence under bf16 autocast: runs, stays finite, and the loss tracks the fp32 oracle."""
    from compressai.entropy_models import set_noise_source
    from compressai.losses import RateDistortionLoss
    from compressai.optim import configure_optimizers

    ref, net = _pair("bmshj2018-hyperprior", (128, 192), cuda)
    opt, aux = configure_optimizers(net)
    scaler = torch.amp.GradScaler("cuda")
    x = torch.rand(2, 3, 128, 128, generator=torch.Generator().manual_seed(7))
    feed = O.NoiseFeed(record=torch.Generator().manual_seed(8))
    with feed:
        cr = O.RateDistortionLoss(1)(ref(x), x)
    q = [n.to(cuda) for n in feed.drawn]
    set_noise_source(lambda t: q.pop(0))
    try:
        c = _reference_step(net, RateDistortionLoss(1), x.to(cuda), opt, aux, scaler, 1.0, dtype=torch.bfloat16)
    finally:
        set_noise_source(None)
    assert abs(c["loss"].item() - cr["loss"].item()) < 1e-2 * abs(cr["loss"].item())
    assert all(torch.isfinite(p).all() for p in net.parameters())
    assert float(opt.step_count.item()) == 1.0


def test_fp16_autocast_policy(cuda):
    """fp16 autocast (the reference's torch.cuda.amp.autocast()) runs the bf16 kernels by default, identical to
    an explicit bf16 autocast; the opt-in "error" policy raises."""
    import compressai
    from compressai.entropy_models import set_noise_source

    _, net = _pair("bmshj2018-hyperprior", (32, 48), cuda)
    x = torch.rand(1, 3, 64, 64, generator=torch.Generator().manual_seed(1)).to(cuda)
    compressai.set_fp16_autocast_policy("error")
    try:
        with pytest.raises(RuntimeError, match="bf16"):
            with torch.autocast("cuda", dtype=torch.float16):
                net(x)
    finally:
        compressai.set_fp16_autocast_policy("bf16")
    outs = []
    for dt in (torch.float16, torch.bfloat16):
        noise = [torch.zeros(1, 32, 1, 1, device=cuda), torch.zeros(1, 48, 4, 4, device=cuda)]
        set_noise_source(lambda t: noise.pop(0))
        try:
            with torch.autocast("cuda", dtype=dt):
                outs.append(net(x)["x_hat"].detach().clone())
        finally:
            set_noise_source(None)
    assert torch.equal(outs[0], outs[1])


def test_train_one_epoch_as_written_fp16(cuda):
    """examples/train.py:145-206 (train_one_epoch_guided's body) as written: DataLoader batches,
    torch.cuda.amp.autocast() (fp16) around forward + criterion and around aux_loss, GradScaler scale / unscale_ /
    clip_grad_norm_ / step / update, torch.optim.Adam from the reference's configure_optimizers (train.py:111-142),
    on the product ScaleHyperprior.  Runs with no policy call: the fp16 regions compute in bf16 (one warning), the
    losses stay finite and track the same steps under an explicit bf16 autocast, and the scaler never skips.
    Parity caveat: the reference's fp16 autocast carries 11 mantissa bits, this path bf16's 8;
    no reference-held fixture pins either.  The first step's loss (before any update) is checked against the
    fp32 CPU oracle on the same weights, batch and quantisation noise within the bf16 model-level bound."""
    import warnings

    from torch.cuda.amp import GradScaler, autocast
    from torch.utils.data import DataLoader, TensorDataset

    from compressai.entropy_models import set_noise_source
    from compressai.losses import RateDistortionLoss

    first = {}

    def run(fp16):
        ref, model = _pair("bmshj2018-hyperprior", (64, 96), cuda)
        first.setdefault("ref", ref)
        optimizer, aux_optimizer = _torch_optimizers(model, 1e-4, 1e-3)
        scaler = GradScaler()
        criterion = RateDistortionLoss(1)
        data = torch.rand(8, 3, 64, 64, generator=torch.Generator().manual_seed(5))
        loader = DataLoader(TensorDataset(data), batch_size=2, shuffle=False)
        gen = torch.Generator().manual_seed(6)
        drawn = []

        def source(t):
            n = torch.empty(t.shape).uniform_(-0.5, 0.5, generator=gen)
            drawn.append(n)
            return n.to(cuda)

        set_noise_source(source)
        losses, auxes, scales = [], [], []
        try:
            model.train()
            device = next(model.parameters()).device
            for i, (d,) in enumerate(loader):
                d = d.to(device)
                optimizer.zero_grad()
                aux_optimizer.zero_grad()
                with (autocast() if fp16 else torch.autocast("cuda", dtype=torch.bfloat16)):
                    out_net = model(d)
                    out_criterion = criterion(out_net, d)
                scaler.scale(out_criterion["loss"]).backward()
                scaler.unscale_(optimizer)
                torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
                scaler.step(optimizer)
                with (autocast() if fp16 else torch.autocast("cuda", dtype=torch.bfloat16)):
                    aux_loss = model.aux_loss()
                scaler.scale(aux_loss).backward()
                scaler.unscale_(aux_optimizer)
                scaler.step(aux_optimizer)
                scaler.update()
                losses.append(out_criterion["loss"].item())
                auxes.append(aux_loss.item())
                if i == 0:
                    first.setdefault("noise", list(drawn))
                    first.setdefault("x", d.cpu())
                scales.append(scaler.get_scale())
        finally:
            set_noise_source(None)
        return losses, auxes, scales

    with warnings.catch_warnings(record=True) as caught:
        warnings.simplefilter("always")
        l16, a16, s16 = run(True)
    ours = [w for w in caught if "fp16 autocast regions run the bf16 kernels" in str(w.message)]
    import compressai._ops as ops
    assert len(ours) == 1 or ops._FP16_WARNED, [str(w.message) for w in caught]
    lbf, abf, _ = run(False)
    assert len(l16) == 4 and all(math.isfinite(v) for v in l16 + a16)
    assert s16 == sorted(s16) and s16[0] == 65536.0        # no inf / nan step was skipped
    for a, b in zip(l16, lbf):
        assert abs(a - b) <= 1e-2 * abs(b), (l16, lbf)
    # step 0 against the fp32 oracle (same initial weights, batch and noise): the bf16 model-level loss bound
    with O.NoiseFeed(list(first["noise"])):
        out_r = first["ref"](first["x"])
    l_ref = O.RateDistortionLoss(1)(out_r, first["x"])["loss"].item()
    assert abs(l16[0] - l_ref) <= 1e-2 * abs(l_ref), (l16[0], l_ref)


def _param_set(dev, seed=9, large=False):
    """large: > 65536 parameters in all (cai_adam_step's two-launch path instead of the one-block one)."""
    torch.manual_seed(seed)
    shapes = [(16, 3, 5, 5), (16,), (7,), (24, 24)] + ([(192, 128, 3, 3)] if large else [])
    base = [torch.randn(s) for s in shapes]
    return shapes, [torch.nn.Parameter(b.clone().to(dev)) for b in base], [torch.nn.Parameter(b.clone().to(dev))
                                                                           for b in base]


def test_fused_adam_state_dict_is_torch_adam_format(cuda):
    """FusedAdam.state_dict() has torch.optim.Adam's layout and values; a torch Adam checkpoint loads into
    FusedAdam and training continues identically."""
    from compressai.optim import FusedAdam

    shapes, pa, pb = _param_set(cuda)
    opt_t = torch.optim.Adam(pa, lr=1e-3)
    opt_f = FusedAdam(pb, lr=1e-3)
    g = torch.Generator().manual_seed(2)
    grads = [[torch.randn(s, generator=g).to(cuda) for s in shapes] for _ in range(6)]
    for it in range(3):
        for p, gg in zip(pa, grads[it]):
            p.grad = gg.clone()
        opt_f.zero_grad()
        for p, gg in zip(pb, grads[it]):
            p.grad.copy_(gg)
        opt_t.step()
        opt_f.step()
    st, sf = opt_t.state_dict(), opt_f.state_dict()
    assert set(sf) == {"state", "param_groups"}
    assert sf["param_groups"][0]["params"] == st["param_groups"][0]["params"]
    for k in ("lr", "betas", "eps", "weight_decay", "amsgrad"):
        assert sf["param_groups"][0][k] == st["param_groups"][0][k], k
    for i in st["state"]:
        assert float(sf["state"][i]["step"]) == float(st["state"][i]["step"])
        for k in ("exp_avg", "exp_avg_sq"):
            assert sf["state"][i][k].shape == st["state"][i][k].shape
            assert (sf["state"][i][k].cpu() - st["state"][i][k].cpu()).abs().max().item() < 1e-6
    # resume: a fresh FusedAdam from torch's checkpoint continues exactly like torch
    _, _, pc = _param_set(cuda)
    with torch.no_grad():
        for a, c in zip(pa, pc):
            c.copy_(a)
    opt_c = FusedAdam(pc, lr=5.0)
    opt_c.load_state_dict(st)
    assert opt_c.param_groups[0]["lr"] == 1e-3
    for it in range(3, 6):
        for p, gg in zip(pa, grads[it]):
            p.grad = gg.clone()
        opt_c.zero_grad()
        for p, gg in zip(pc, grads[it]):
            p.grad.copy_(gg)
        opt_t.step()
        opt_c.step()
    for a, c in zip(pa, pc):
        assert (a.detach() - c.detach()).abs().max().item() < 1e-6
    # and torch Adam accepts FusedAdam's checkpoint
    _, pd, _ = _param_set(cuda)
    opt_d = torch.optim.Adam(pd, lr=1.0)
    opt_d.load_state_dict(opt_c.state_dict())
    assert opt_d.param_groups[0]["lr"] == 1e-3


def test_fused_adam_survives_detached_grads(cuda):
    """model.zero_grad() (set_to_none=True) unlinks p.grad from the flat buffer: step() must re-home the fresh
    gradients instead of stepping on stale ones."""
    from compressai.optim import FusedAdam

    shapes, pa, pb = _param_set(cuda)
    opt_t = torch.optim.Adam(pa, lr=1e-2)
    opt_f = FusedAdam(pb, lr=1e-2)
    g = torch.Generator().manual_seed(4)
    for it in range(3):
        gr = [torch.randn(s, generator=g).to(cuda) for s in shapes]
        for p, gg in zip(pa, gr):
            p.grad = gg.clone()
        for p in pb:            # what Module.zero_grad() does by default
            p.grad = None
        for p, gg in zip(pb, gr):
            if it == 1 and p is pb[2]:
                continue        # an unused parameter this step: grad stays None -> zero
            p.grad = gg.clone()
        if it == 1:
            pa[2].grad = torch.zeros_like(pa[2])
        opt_t.step()
        opt_f.step()
        assert all(p.grad.data_ptr() == v.data_ptr() for p, v in zip(pb, opt_f._grad_views))
    for a, b in zip(pa, pb):
        assert (a.detach() - b.detach()).abs().max().item() < 1e-6


@pytest.mark.parametrize("large", [False, True], ids=["one-block", "two-launch"])
def test_fused_adam_skips_nonfinite_step(cuda, large):
    """An inf / NaN gradient skips the update on the device (GradScaler's rule) and leaves the step count."""
    from compressai.optim import FusedAdam

    shapes, _, pb = _param_set(cuda, large=large)
    opt = FusedAdam(pb, lr=1e-2)
    for p in pb:
        p.grad.fill_(0.5)
    opt.step(max_norm=1.0)
    before = [p.detach().clone() for p in pb]
    m_before = opt.exp_avg.clone()
    for bad in (float("inf"), float("nan")):
        opt.zero_grad()
        for p in pb:
            p.grad.fill_(0.5)
        pb[1].grad[3] = bad
        opt.step(max_norm=1.0)
        opt.zero_grad()
        for p in pb:
            p.grad.fill_(0.5)
        pb[0].grad[0, 0, 0, 0] = bad
        opt.step()                       # no clipping: the finiteness check still applies
    torch.cuda.synchronize()
    for a, b in zip(pb, before):
        assert torch.equal(a.detach(), b)
    assert torch.equal(opt.exp_avg, m_before)
    assert float(opt.step_count.item()) == 1.0


@pytest.mark.parametrize("large", [False, True], ids=["one-block", "two-launch"])
def test_fused_adam_skipped_step_consumes_grads(cuda, large):
    """zero_grad_in_step: a skipped (non-finite) step still leaves the gradient buffer zeroed, so the next
    zero_grad() (which then launches nothing) starts the following backward from zero."""
    from compressai.optim import FusedAdam

    shapes, _, pb = _param_set(cuda, large=large)
    opt = FusedAdam(pb, lr=1e-2, zero_grad_in_step=True)
    opt.zero_grad()
    for p in pb:
        p.grad.fill_(0.5)
    pb[1].grad[3] = float("nan")
    before = [p.detach().clone() for p in pb]
    opt.step(max_norm=1.0)
    opt.zero_grad()
    torch.cuda.synchronize()
    assert float(opt.step_count.item()) == 0.0
    assert all(torch.equal(a.detach(), b) for a, b in zip(pb, before))
    assert float(opt.flat_grad.abs().max()) == 0.0
