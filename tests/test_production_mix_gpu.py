"""Model-level checks at the BASELINE configs' own sizes, so the kernels the bench runs are the kernels
under test (the 192-channel conv tiles are gated on grid size: conv_halo_s1_kernel<192> needs >= 128 tiles,
conv_halo_phase_kernel<192> >= 512 blocks, so the 64-128 px model tests never dispatch them).

* C4 cheng2020-attn q6 at 256x256: fp32 parity against the float64 oracle at B=1, and bf16 bounds at the
  per-GPU batch B=4 with conv_halo_s1_kernel<192> asserted in the step's launches;
* C2 bmshj2018-hyperprior q1 (128, 192) -- the bench's own config -- and C3 mbt2018-mean q1 at 256x256, B=16,
  bf16, with the kernels that only full-size C2 grids take asserted (lane GDN <128> forward / backward, the
  halo gather / s^2-phase convs, the halo weight gradient, the image-side edge kernels); C2 also in fp32 at
  B=2 against the float64 oracle;
* C2' bmshj2018-hyperprior q6 (192, 320) at 256x256, B=16, bf16, with conv_halo_phase_kernel<192> asserted;
* C5 at paper resolution (master.py:708-742, 158-210): Spatial_aligner on its three token
  grids (32x40, 64x80, 128x160) against the CPU oracle, Channel_aligner on 512x640 features against the
  oracle module run on the GPU in fp32 (torch's own convolutions: the CPU would take minutes for its ~7
  TFLOP), and one full training step of Master_compresser(512, 640) guided by Guided_compresser on
  1024x1280 RGB, B=2: bf16 loss within 2 % of the HIP fp32 step, finite gradients.

Bars as in test_models_wide_gpu.py (fp32: 1e-4 outputs / 2e-3 gradients against float64, or 2x the fp32
oracle's own error; bf16: x_hat 1e-2, loss 1e-3, gradient cosine), with two additions that production sizes
force, both measured on MI355X (profiles/r03_graddiff_*.log):
* ReLU / LeakyReLU mask flips.  A pre-activation within fp32 round-off of 0 takes the other branch in one fp32
  path and not in the other; its gradient element then differs by the whole incoming gradient.  At 256x256
  this happens in BOTH fp32 paths: with seed 32 the CPU fp32 oracle itself misses a cheng2020 attention-unit
  weight gradient by 4.8e-3 (max norm) against float64, with seed 31 the HIP path misses another by 4.9e-3
  while the CPU does not.  A tensor whose max-norm error exceeds the bar therefore passes on its relative L2
  error (<= 5e-3: the flipped element is one term of the sum), and at most 2 % of the tensors may use that
  allowance.
* bf16 likelihoods: the max-norm error grows with the element count (196K y elements at B=4 vs 6K in the
  64x64 tests: 2.2e-2 measured); bounded at 5e-2 max and 5e-3 relative L2.
"""
import math

import pytest
import torch

import cai_oracle as O
import cai_oracle_master as OM

pytestmark = pytest.mark.gpu


def relerr(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    d = b.abs().max().item()
    return (a - b).abs().max().item() / (d if d > 0 else 1.0)


def rel_l2(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    d = b.norm().item()
    return (a - b).norm().item() / (d if d > 0 else 1.0)


def _pair(name, args, dev):
    from compressai.zoo import model_architectures

    torch.manual_seed(0)
    ref = O.ARCHS[name](*args)
    net = model_architectures[name](*args)
    net.load_state_dict(ref.state_dict())
    return ref, net.to(dev)


def _run(name, args, size, batch, cuda, bf16, quality, seed):
    """Oracle (fp32 CPU) and HIP step on the same weights / input / noise; the HIP step under the ledger,
    so the kernels it launched are known."""
    from compressai import _ledger
    from compressai.entropy_models import set_noise_source
    from compressai.losses import RateDistortionLoss

    ref, net = _pair(name, args, cuda)
    x = torch.rand(batch, 3, size, size, generator=torch.Generator().manual_seed(seed))
    feed = O.NoiseFeed(record=torch.Generator().manual_seed(seed + 1))
    with feed:
        out_r = ref(x)
    cr = O.RateDistortionLoss(quality)(out_r, x)
    cr["loss"].backward()
    q = [n.to(cuda) for n in feed.drawn]
    set_noise_source(lambda t: q.pop(0))
    try:
        with _ledger.recording(keep_replay=False) as led:
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=bf16):
                out = net(x.to(cuda))
                c = RateDistortionLoss(quality)(out, x.to(cuda))
            c["loss"].backward()
            torch.cuda.synchronize()
    finally:
        set_noise_source(None)
    assert not q
    kernels = {e.kernel for e in led.entries}
    return ref, net, out_r, out, cr, c, feed.drawn, x, kernels


@pytest.mark.parametrize("name,args,batch,quality,seed", [
    ("cheng2020-attn", (192,), 1, 6, 31),                 # C4 at 256x256
    ("bmshj2018-hyperprior", (128, 192), 2, 1, 33),       # C2 (the bench's model) at 256x256
], ids=["cheng2020-attn-q6-B1", "hyperprior-q1-B2"])
def test_fp32_parity_256(cuda, name, args, batch, quality, seed):
    ref, net, out_r, out, cr, c, drawn, x, _ = _run(name, args, 256, batch, cuda, False, quality, seed=seed)
    import copy

    r64 = copy.deepcopy(ref).double()
    for p in r64.parameters():
        p.grad = None
    with O.NoiseFeed([n.double() for n in drawn]):
        out64 = r64(x.double())
    O.RateDistortionLoss(quality)(out64, x.double())["loss"].backward()

    def check(a, a32, a64, bar, what):
        e, e32 = relerr(a, a64), relerr(a32, a64)
        assert e < max(bar, 2 * e32), (what, e, e32)

    check(out["x_hat"], out_r["x_hat"], out64["x_hat"], 1e-4, "x_hat")
    for k in out_r["likelihoods"]:
        check(out["likelihoods"][k], out_r["likelihoods"][k], out64["likelihoods"][k], 1e-4, k)
    for k in ("loss", "bpp_loss", "mse_loss"):
        assert abs(c[k].item() - cr[k].item()) <= 1e-4 * max(1.0, abs(cr[k].item())), k
    pr, p64 = dict(ref.named_parameters()), dict(r64.named_parameters())
    flips, total = [], 0
    for n, p in net.named_parameters():
        gr = pr[n].grad
        if gr is None:
            assert p.grad is None or p.grad.abs().max().item() == 0, n
            continue
        total += 1
        e, e32 = relerr(p.grad, p64[n].grad), relerr(gr, p64[n].grad)
        if e < max(2e-3, 2 * e32):
            continue
        el2 = rel_l2(p.grad, p64[n].grad)          # a mask flip: one term of the sum (module docstring)
        assert el2 < 5e-3, (n, e, e32, el2)
        flips.append((n, round(e, 6), round(el2, 6)))
    print(f"\nfp32 {name} 256 B={batch}: mask-flip allowance used by {len(flips)} of {total} tensors: {flips}")
    assert len(flips) <= 0.02 * total, flips


BF16_XHAT, BF16_LIK, BF16_LIK_L2, BF16_LOSS, GRAD_COS, TENSOR_COS = 1e-2, 5e-2, 5e-3, 1e-3, 0.9999, 0.98


# the kernels the bench's C2 / C3 step launches at 256x256 B=16 (none of them is taken at the 64-128 px model
# test sizes: the lane GDN kernels need >= 32768 pixels, the halo / phase / edge kernels full-size grids)
C2_MIX = ("gdn_fwd_lane_kernel<128>", "gdn_bwd_lane_kernel<128>", "conv_halo_kernel<5>", "conv_halo_phase_kernel",
          "conv_halo_quad_kernel",
          "wgrad_halo_kernel<5>", "edge_s2d_kernel (conv fwd)", "edge_d2s_kernel (deconv fwd)",
          "edge_wgrad_dma_kernel (+pack, reduce)")


@pytest.mark.parametrize("name,args,batch,quality,gated", [
    ("cheng2020-attn", (192,), 4, 6, ("conv_halo_s1_kernel<192>",)),                 # C4, per-GPU batch
    ("bmshj2018-hyperprior", (192, 320), 16, 6, ("conv_halo_phase_kernel<192>",)),   # C2' at C2's batch
    ("bmshj2018-hyperprior", (128, 192), 16, 1, C2_MIX),                             # C2: BASELINE configs[1]
    ("mbt2018-mean", (128, 192), 16, 1, C2_MIX),                                     # C3: configs[2]
], ids=["cheng2020-attn-q6-B4", "hyperprior-q6-B16", "hyperprior-q1-B16", "mbt2018-mean-q1-B16"])
def test_bf16_production_mix_256(cuda, name, args, batch, quality, gated):
    ref, net, out_r, out, cr, c, _, _, kernels = _run(name, args, 256, batch, cuda, True, quality, seed=41)
    missing = [k for k in gated if k not in kernels]
    assert not missing, (missing, sorted(kernels))
    ex = relerr(out["x_hat"], out_r["x_hat"])
    el = {k: relerr(out["likelihoods"][k], out_r["likelihoods"][k]) for k in out_r["likelihoods"]}
    el2 = {k: rel_l2(out["likelihoods"][k], out_r["likelihoods"][k]) for k in out_r["likelihoods"]}
    eloss = abs(c["loss"].item() - cr["loss"].item()) / abs(cr["loss"].item())
    pr = dict(ref.named_parameters())
    tcos, dots, na, nb = {}, 0.0, 0.0, 0.0
    for n, p in net.named_parameters():
        gr = pr[n].grad
        if gr is None or p.grad is None:
            continue
        g = p.grad.detach().float().cpu()
        assert torch.isfinite(g).all(), n
        tcos[n] = float(torch.nn.functional.cosine_similarity(g.double().flatten(), gr.double().flatten(), dim=0))
        dots += float((g.double() * gr.double()).sum())
        na += float((g.double() ** 2).sum())
        nb += float((gr.double() ** 2).sum())
    cos = dots / math.sqrt(na * nb)
    low = sorted(tcos.items(), key=lambda kv: kv[1])[:3]
    print(f"\nbf16 {name} B={batch}: x_hat {ex:.3e} lik {el} (L2 {el2}) loss {eloss:.3e} grad cos {cos:.6f} "
          f"lowest {low}")
    assert ex < BF16_XHAT
    for k, v in el.items():
        assert v < BF16_LIK and el2[k] < BF16_LIK_L2, k
    assert eloss < BF16_LOSS
    assert cos > GRAD_COS
    assert low[0][1] > TENSOR_COS, low


# ---------------------------------------------------------------------------------------------------------
# C5 at paper resolution: IR 512x640 (channel 1, master stride 1), RGB 1024x1280 guide
# ---------------------------------------------------------------------------------------------------------

def _copy(ref, mod, cuda):
    mod.load_state_dict(ref.state_dict())
    return mod.to(cuda)


@pytest.mark.parametrize("res", [(64, 80), (128, 160), (256, 320)], ids=["tokens32x40", "tokens64x80",
                                                                       "tokens128x160"])
def test_spatial_aligner_paper_grids(cuda, res):
    """Master_decoder(width=512, height=640).sp_aligner{1,2,3}: inputs (64, 80), (128, 160), (256, 320),
    i.e. Swin token grids 32x40, 64x80, 128x160 (window 4, shift 0 / 2), fp32 B=1 vs the CPU oracle."""
    from compressai.models.master import Spatial_aligner

    torch.manual_seed(50 + res[0])
    ref = OM.Spatial_aligner(input_resolution=res)
    with torch.no_grad():
        for blk in ref.blocks:
            blk.attn.relative_position_bias_table.normal_(0, 0.5)
    mod = _copy(ref, Spatial_aligner(input_resolution=res), cuda)
    gen = torch.Generator().manual_seed(60 + res[0])
    x = torch.randn(1, 192, *res, generator=gen)
    gd = torch.randn(1, 192, *res, generator=gen)
    xr, gr = x.clone().requires_grad_(), gd.clone().requires_grad_()
    yr = ref(xr, gr)
    g = torch.randn(yr.shape, generator=gen)
    yr.backward(g)
    xd = x.to(cuda).contiguous(memory_format=torch.channels_last).requires_grad_()
    gdd = gd.to(cuda).contiguous(memory_format=torch.channels_last).requires_grad_()
    y = mod(xd, gdd)
    y.backward(g.to(cuda))
    assert relerr(y, yr) < 1e-4
    assert relerr(xd.grad, xr.grad) < 2e-3
    assert relerr(gdd.grad, gr.grad) < 2e-3
    pr = dict(ref.named_parameters())
    for n, p in mod.named_parameters():
        assert relerr(p.grad, pr[n].grad) < 2e-3, n


@pytest.mark.parametrize("bf16", [False, True], ids=["fp32", "bf16"])
def test_channel_aligner_512x640(cuda, bf16):
    """Channel_aligner (4 x conv3x3(256) trunk per branch, conv5/conv6 heads, global pools) on the IR
    config's 64-channel 512x640 features, B=1, against the oracle module run on the GPU in fp32 (torch's
    convolutions, TF32 off).  fp32: outputs within 1e-4 (max norm); gradients within 5e-3 relative L2 --
    84M pre-activations per LeakyReLU layer put some within round-off of 0 (module docstring), and the beta
    branch's input gradient is the trunk's backward of a spatially uniform gradient, a sum with heavy
    cancellation (measured: d1 1.3e-3 L2, everything else <= 2e-4).  bf16 (the production kernels: the
    256-channel convs take conv_halo_s1_kernel): outputs 1e-2, every gradient's cosine >= 0.999 or within 2x
    the distance of torch's own bf16 autocast of the same module (d1's cancelling sum: ~0.995 in bf16)."""
    from compressai import _ledger
    from compressai.models.master import Channel_aligner

    prev = (torch.backends.cuda.matmul.allow_tf32, torch.backends.cudnn.allow_tf32, torch.backends.cudnn.enabled)
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cudnn.enabled = False     # the oracle's convs on torch's native path (no MIOpen kernel builds)
    try:
        torch.manual_seed(70)
        ref = OM.Channel_aligner()
        mod = _copy(ref, Channel_aligner(), cuda)
        ref = ref.to(cuda)
        gen = torch.Generator().manual_seed(71)
        f1 = torch.randn(1, 64, 512, 640, generator=gen)
        f2 = torch.randn(1, 64, 512, 640, generator=gen)
        g = torch.randn(1, 64, 512, 640, generator=gen).to(cuda)
        r1, r2 = f1.to(cuda).requires_grad_(), f2.to(cuda).requires_grad_()
        tcos = {}
        if bf16:
            # torch's own bf16 autocast of the same module: the bf16 error the HIP path is measured against
            t1, t2 = f1.to(cuda).requires_grad_(), f2.to(cuda).requires_grad_()
            with torch.autocast("cuda", dtype=torch.bfloat16):
                ot = ref(t1, t2)[0]
            (ot.float() * g).sum().backward()
            tgr = {"d1": t1.grad, "d2": t2.grad, **{n: p.grad.clone() for n, p in ref.named_parameters()}}
            ref.zero_grad(set_to_none=True)
        out_r, beta_r, gamma_r = ref(r1, r2)
        (out_r * g).sum().backward()
        d1 = f1.to(cuda).contiguous(memory_format=torch.channels_last).requires_grad_()
        d2 = f2.to(cuda).contiguous(memory_format=torch.channels_last).requires_grad_()
        with _ledger.recording(keep_replay=False) as led:
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=bf16):
                out, beta, gamma = mod(d1, d2)
            (out.float() * g).sum().backward()
            torch.cuda.synchronize()
        kernels = {e.kernel for e in led.entries}
        outs = {"out": (out, out_r), "beta": (beta, beta_r), "gamma": (gamma, gamma_r)}
        grads = {"d1": (d1.grad, r1.grad), "d2": (d2.grad, r2.grad)}
        pr = dict(ref.named_parameters())
        for n, p in mod.named_parameters():
            grads[n] = (p.grad, pr[n].grad)
        errs = {k: (relerr(a, b), rel_l2(a, b)) for k, (a, b) in {**outs, **grads}.items()}
        cos = {k: float(torch.nn.functional.cosine_similarity(a.double().flatten(), b.double().flatten(), dim=0))
               for k, (a, b) in grads.items()}
        print(f"\nChannel_aligner 512x640 {'bf16' if bf16 else 'fp32'} (max, rel-L2):",
              {k: (f"{a:.2e}", f"{b:.2e}") for k, (a, b) in errs.items()}, "lowest cos", min(cos.values()))
        for k in outs:
            assert errs[k][0] < (1e-2 if bf16 else 1e-4), (k, errs[k])
        if bf16:
            assert "conv_halo_s1_kernel<128>" in kernels or "conv_halo_s1_kernel<192>" in kernels, sorted(kernels)
            tcos = {k: float(torch.nn.functional.cosine_similarity(tgr[k].double().flatten(), b.double().flatten(),
                                                                    dim=0)) for k, (_, b) in grads.items()}
            print("torch bf16 autocast lowest cos", min(tcos.values()), "d1", tcos["d1"], "HIP d1", cos["d1"])
            for k, v in cos.items():        # >= 0.999, or no more than 2x torch's own bf16 distance
                assert v >= min(0.999, 1 - 2 * (1 - tcos[k])), (k, v, tcos[k])
        else:
            for k in grads:
                assert errs[k][1] < 5e-3, (k, errs[k])
    finally:
        torch.backends.cuda.matmul.allow_tf32, torch.backends.cudnn.allow_tf32, torch.backends.cudnn.enabled = prev


def test_master_guided_full_resolution_step(cuda):
    """BASELINE configs[4] per GPU: Master_compresser(width=512, height=640, channel=1) on IR 512x640 guided
    by Guided_compresser(channel=3) on RGB 1024x1280 (no_grad, training mode), B=2, one RD-loss training
    step in bf16 autocast and in the HIP fp32 mode on the same weights and noise: shapes, finite loss and
    gradients, bf16 loss within 2 % of fp32, bf16 gradient cosine against fp32."""
    from compressai.entropy_models import set_noise_source
    from compressai.losses import RateDistortionLoss
    from compressai.models import Guided_compresser, Master_compresser

    torch.manual_seed(80)
    net = Master_compresser(width=512, height=640, channel=1).to(cuda).train()
    guide = Guided_compresser(channel=3).to(cuda).train()
    gen = torch.Generator().manual_seed(81)
    x = torch.rand(2, 1, 512, 640, generator=gen).to(cuda)
    gx = torch.rand(2, 3, 1024, 1280, generator=gen).to(cuda)
    drawn = []
    ngen = torch.Generator().manual_seed(82)

    def record(t):
        n = torch.empty(t.shape).uniform_(-0.5, 0.5, generator=ngen).to(cuda)
        drawn.append(n)
        return n

    def step(bf16, source):
        net.zero_grad(set_to_none=True)
        set_noise_source(source)
        try:
            with torch.no_grad():
                hidden = guide(gx)["hidden"]
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=bf16):
                out = net(x, gx, hidden)
                c = RateDistortionLoss(1)(out, x)
            c["loss"].backward()
        finally:
            set_noise_source(None)
        torch.cuda.synchronize()
        grads = {n: p.grad.detach().float().clone() for n, p in net.named_parameters() if p.grad is not None}
        return out, c, hidden, grads

    out32, c32, hidden, g32 = step(False, record)
    assert out32["x_hat"].shape == (2, 1, 512, 640)
    assert out32["likelihoods"]["y"].shape == (2, 192, 32, 40)
    assert out32["likelihoods"]["z"].shape == (2, 192, 8, 10)
    assert hidden["gs1"].shape == (2, 192, 128, 160) and hidden["gs3"].shape == (2, 192, 512, 640)
    replay = list(drawn)
    out16, c16, _, g16 = step(True, lambda t: replay.pop(0))
    assert not replay
    l32, l16 = c32["loss"].item(), c16["loss"].item()
    assert math.isfinite(l32) and math.isfinite(l16)
    assert abs(l16 - l32) < 0.02 * abs(l32), (l16, l32)
    assert set(g16) == set(g32) and not any(n.startswith("g_s.") for n in g32)   # inherited g_s unused
    dots = na = nb = 0.0
    for n in g32:
        assert torch.isfinite(g16[n]).all() and torch.isfinite(g32[n]).all(), n
        dots += float((g16[n].double() * g32[n].double()).sum())
        na += float((g16[n].double() ** 2).sum())
        nb += float((g32[n].double() ** 2).sum())
    cos = dots / math.sqrt(na * nb)
    print(f"\nC5 full resolution: loss fp32 {l32:.5f} bf16 {l16:.5f}, gradient cosine {cos:.6f}")
    assert cos > 0.999


def test_master_guided_paper_resolution_vs_oracle(cuda):
    """C5 end to end at paper resolution against the oracle (master.py:904-951,
    1269-1295; train.py:208-246): Guided_compresser(channel=3) on RGB 1024x1280 in training mode under no_grad,
    then Master_compresser(width=512, height=640, channel=1) on IR 512x640 + RD loss + backward, B=1, the HIP
    fp32 path against the oracle modules run on the GPU in fp32 torch (TF32 off: the CPU would take many
    minutes for this step), with the same injected quantisation noise (guided's draws first, then the
    master's).  x_hat, both likelihoods, the guided hidden maps and the loss within 1e-4; every parameter
    gradient within 2e-3 (max norm) or, for a mask flip at a pre-activation within round-off of 0, 5e-3
    relative L2, on at most 2 % of the tensors (module docstring)."""
    from compressai.entropy_models import set_noise_source
    from compressai.losses import RateDistortionLoss
    from compressai.models import Guided_compresser, Master_compresser

    import time

    t0 = time.time()

    def stage(what):   # progress lines: the GPU box kills a run that writes nothing for 3 minutes
        print(f"[C5 paper resolution] {what} at {time.time() - t0:.1f} s", flush=True)

    prev = (torch.backends.cuda.matmul.allow_tf32, torch.backends.cudnn.allow_tf32, torch.backends.cudnn.enabled)
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False
    # the oracle's convolutions through torch's native im2col + GEMM path: MIOpen compiles a kernel per new
    # convolution shape on a fresh box (~200 s for this model)
    torch.backends.cudnn.enabled = False
    try:
        torch.manual_seed(90)
        ref = OM.Master_compresser(width=512, height=640, channel=1)
        refG = OM.Guided_compresser(channel=3)
        net = _copy(ref, Master_compresser(width=512, height=640, channel=1), cuda).train()
        guide = _copy(refG, Guided_compresser(channel=3), cuda).train()
        ref, refG = ref.to(cuda).train(), refG.to(cuda).train()
        gen = torch.Generator().manual_seed(91)
        x = torch.rand(1, 1, 512, 640, generator=gen).to(cuda)
        gx = torch.rand(1, 3, 1024, 1280, generator=gen).to(cuda)
        feed = O.NoiseFeed(record=torch.Generator().manual_seed(92))
        stage("models built")
        with feed:
            with torch.no_grad():
                hid_r = refG(gx)["hidden"]
            stage("oracle guided forward")
            out_r = ref(x, gx, hid_r)
        stage("oracle master forward")
        cr = O.RateDistortionLoss(1)(out_r, x)
        cr["loss"].backward()
        torch.cuda.synchronize()
        stage("oracle backward")
        q = [n.to(cuda) for n in feed.drawn]
        set_noise_source(lambda t: q.pop(0))
        try:
            with torch.no_grad():
                hid = guide(gx)["hidden"]
            out = net(x, gx, hid)
            c = RateDistortionLoss(1)(out, x)
            c["loss"].backward()
            torch.cuda.synchronize()
        finally:
            set_noise_source(None)
        stage("HIP step")
        assert not q
        errs = {"x_hat": relerr(out["x_hat"], out_r["x_hat"])}
        errs.update({f"lik_{k}": relerr(out["likelihoods"][k], out_r["likelihoods"][k]) for k in out_r["likelihoods"]})
        errs.update({f"hidden_{k}": relerr(hid[k], hid_r[k]) for k in hid_r})
        print("\nC5 paper resolution vs oracle:", {k: f"{v:.2e}" for k, v in errs.items()},
              f"loss {c['loss'].item():.6f} / {cr['loss'].item():.6f}")
        for k, v in errs.items():
            assert v < 1e-4, (k, v)
        for k in ("loss", "bpp_loss", "mse_loss"):
            assert abs(c[k].item() - cr[k].item()) <= 1e-4 * max(1.0, abs(cr[k].item())), k
        pr = dict(ref.named_parameters())
        flips, total = [], 0
        for n, p in net.named_parameters():
            gr = pr[n].grad
            if gr is None:
                assert p.grad is None or p.grad.abs().max().item() == 0, n     # the inherited, unused g_s
                continue
            total += 1
            e = relerr(p.grad, gr)
            if e < 2e-3:
                continue
            el2 = rel_l2(p.grad, gr)
            assert el2 < 5e-3, (n, e, el2)
            flips.append((n, round(e, 6), round(el2, 6)))
        print(f"mask-flip allowance used by {len(flips)} of {total} tensors: {flips}")
        assert total > 0 and len(flips) <= 0.02 * total, flips
    finally:
        torch.backends.cuda.matmul.allow_tf32, torch.backends.cudnn.allow_tf32, torch.backends.cudnn.enabled = prev


@pytest.mark.parametrize("name,quality,batch,only", [
    ("bmshj2018-hyperprior", 1, 16, None),
    ("cheng2020-attn", 6, 4, ("Functor_add", "CatArray")),
], ids=["C2", "C4"])
def test_step_launches_no_aten_kernels(cuda, name, quality, batch, only):
    """The training step (C2: bmshj2018-hyperprior q1, B=16; C4: cheng2020-attn q6, B=4; 256^2, bf16 autocast;
    bench.py's step: FusedAdam with zero_grad_in_step, the persistent loss seeds, clip + Adam + aux loss).
    C2 launches only libcai kernels: no ATen elementwise / fill / reduce kernel -- y's two gradients meet in h_a's
    first dgrad epilogue, the aux loss's quantile gradient accumulates through cai_axpy_dev.  C4 launches no ATen
    gradient sum (`only`): the residual blocks' inputs and the context model's y / y_hat are read through FanOutFn,
    whose native add sums their gradients, and no ATen concatenation (the entropy parameters' input is CatFn's
    native copy).  C4 still has three ATen launches: the masked conv's in-place weight mask (the reference's
    `weight.data *= mask`), one layout copy and one fill.
    Device kernels of the third eager step, from torch.profiler."""
    from torch.profiler import ProfilerActivity, profile

    from compressai._ops import loss_seed
    from compressai.losses import RateDistortionLoss
    from compressai.optim import configure_optimizers
    from compressai.zoo import image_models

    torch.manual_seed(0)
    net = image_models[name](quality).to(cuda).train()
    x = torch.rand(batch, 3, 256, 256, device=cuda)
    opt, aux_opt = configure_optimizers(net, zero_grad_in_step=True)
    crit = RateDistortionLoss(quality)

    def step():
        opt.zero_grad()
        aux_opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = crit(net(x), x)["loss"]
        loss.backward(loss_seed(loss))
        opt.step(max_norm=1.0)
        aux = net.aux_loss()
        aux.backward(loss_seed(aux))
        aux_opt.step()

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        step()
        torch.cuda.synchronize()
    names = sorted({e.name for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA})
    print(f"\n{name} step: {len(names)} distinct device kernels / copies")
    assert len(names) > 20, names               # the profiler saw the step's kernels
    aten = [n for n in names if ("at::" in n or "aten::" in n) and (only is None or any(o in n for o in only))]
    assert not aten, aten
    if only is None:
        # nor runtime copies / fills (HIP's blit kernels: __amd_rocclr_copyBuffer / fillBuffer, which carry no
        # ATen name; the profiler lists them as Memcpy / Memset)
        blits = [n for n in names if any(k in n for k in ("Memcpy", "Memset", "copyBuffer", "fillBuffer"))]
        assert not blits, blits
