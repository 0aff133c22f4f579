"""Data parallelism on the product path: two ranks on cuda:0 (gloo over CUDA
tensors -- RCCL needs one GPU per rank), each running the graph-captured forward + backward of a product model
+ FusedAdam on its half of the batch, then the gradient exchange.  The averaged flat gradient must equal the
oracle's gradient of the concatenated batch: the RD loss of equal halves is the mean of the per-half losses
(bpp and mse are per-batch means), so its gradient is the mean of the halves'.

Models: C2's ScaleHyperprior (small widths), the two configs BASELINE.json runs as 8-GPU DDP -- C4
cheng2020-attn at its q6 width N=192 (hyper branch on its side stream) and C5 Master_compresser (IR) guided by
a replicated frozen Guided_compresser (RGB) under no_grad in training mode (train.py:208-246): its cut is the
feature-encoder / channel-aligner outputs, and the inherited, unused g_s keeps zero gradients."""
import os
import socket
import subprocess
import sys

import pytest
import torch

import cai_oracle as O
import cai_oracle_master as OM

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _oracle_case(kind):
    """Oracle model(s), inputs, recorded noise and the oracle gradient of the whole batch."""
    gen = torch.Generator().manual_seed(11)
    feed = O.NoiseFeed(record=torch.Generator().manual_seed(12))
    case = {"quality": 1}
    if kind == "c2":
        torch.manual_seed(0)
        ref = O.ScaleHyperprior(32, 48)
        x = torch.rand(4, 3, 64, 64, generator=gen)
        sd = {k: v.clone() for k, v in ref.state_dict().items()}
        with feed:
            out = ref(x)
    elif kind == "cheng2020-attn":
        torch.manual_seed(1)
        ref = O.Cheng2020Attention(192)
        x = torch.rand(2, 3, 64, 64, generator=gen)
        sd = {k: v.clone() for k, v in ref.state_dict().items()}
        case["quality"] = 6
        with feed:
            out = ref(x)
    else:
        torch.manual_seed(2)
        ref = OM.Master_compresser(width=64, height=64, channel=1)
        refG = OM.Guided_compresser(channel=3)
        x = torch.rand(2, 1, 64, 64, generator=gen)
        gx = torch.rand(2, 3, 128, 128, generator=gen)
        sd = {k: v.clone() for k, v in ref.state_dict().items()}
        case["guide_state_dict"] = {k: v.clone() for k, v in refG.state_dict().items()}
        case["guide_x"] = gx
        with feed:
            with torch.no_grad():
                hidden = refG.train()(gx)["hidden"]
            out = ref(x, gx, hidden)
    O.RateDistortionLoss(case["quality"])(out, x)["loss"].backward()
    case.update(state_dict=sd, x=x, noise=[n.clone() for n in feed.drawn])
    return ref, case


@pytest.mark.parametrize("kind,mode", [("c2", "serial"), ("c2", "overlap"), ("c2", "overlap-eager"),
                                       ("cheng2020-attn", "serial"), ("cheng2020-attn", "overlap"),
                                       ("cheng2020-attn", "overlap-eager"),
                                       ("multimodal", "serial"), ("multimodal", "overlap"),
                                       ("multimodal", "overlap-eager")])
def test_world2_allreduced_flat_grad_matches_oracle(cuda, tmp_path, kind, mode):
    """serial: one all-reduce after the graph replay (bench.py --serial-allreduce); overlap: the bucketed
    exchange of compressai.distributed.OverlappedAllReduce over the model's phase plan (CompressionModel.
    dp_phases(): bucket i all-reduced on a side stream while the captured graph of backward phase i + 1
    replays -- C2: g_s, the hyper path, g_a in 3 pieces; cheng2020-attn: g_s in 2 pieces, the context /
    entropy-parameter stack, the hyper path, g_a in 4 pieces; C5: the synthesis, the context stack, the hyper
    path, g_a, the feature encoders + channel aligner); overlap-eager: the same without graphs."""
    from compressai.models.master import Master_compresser
    from compressai.zoo import image_models

    ref, case = _oracle_case(kind)
    inp, outp = tmp_path / "in.pt", tmp_path / "out.pt"
    torch.save(case, inp)
    port = str(_port())
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK="0", WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=port, CAI_DIST_IN=str(inp), CAI_DIST_OUT=str(outp), CAI_DIST_MODE=mode,
                   CAI_DIST_MODEL=kind)
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "dist_worker_product.py")], env=env))
    codes = []
    for p in procs:
        try:
            codes.append(p.wait(timeout=240))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    assert codes == [0, 0], codes
    res = torch.load(outp, weights_only=True)
    pr = dict(ref.named_parameters())
    flat = res["flat_grad"]
    gmax = max(p.grad.abs().max().item() for p in ref.parameters() if p.grad is not None)
    tail = tuple(("g_a.",) if kind != "multimodal" else ("fencoder1.", "fencoder2.", "ch_aligner."))
    plan = {"c2": lambda: image_models["bmshj2018-hyperprior"](1),
            "cheng2020-attn": lambda: image_models["cheng2020-attn"](6),
            "multimodal": lambda: Master_compresser(width=64, height=64, channel=1)}[kind]().dp_phases()
    n_tail = 0
    if mode.startswith("overlap"):
        assert res["nphases"] == len(plan) == len(res["bounds"]) - 1, (res["nphases"], res["bounds"])
        mb = [4 * (res["bounds"][i + 1] - res["bounds"][i]) / 1e6 for i in range(len(plan))]
        print(f"\n{kind} buckets (MB, backward order): {[round(v, 2) for v in mb]}")
        if kind == "cheng2020-attn":
            assert max(mb) <= 40.0, mb      # the head's single 95.8 MB bucket, split
    for name, off, n, st in zip(res["names"], res["offsets"], res["numels"], res["stage"]):
        g = flat[off:off + n]
        if mode.startswith("overlap"):
            # the bucket layout: each parameter inside its phase's bucket, the tail's in the last phases
            assert res["bounds"][st] <= off and off + n <= res["bounds"][st + 1], (name, st, off, res["bounds"])
            assert (plan[st][0] is not None and any(name.startswith(p) for p in plan[st][0])) or \
                (plan[st][0] is None and not name.startswith(tail)), (name, st)
            n_tail += name.startswith(tail)
        gr = pr[name].grad
        if gr is None:
            assert g.abs().max().item() == 0, name       # e.g. Master's inherited, unused g_s
            continue
        gr = gr.flatten()
        # denominator floored at 1e-6 of the model's largest gradient (tensors whose true gradient is round-off)
        err = (g - gr).abs().max().item() / max(gr.abs().max().item(), 1e-6 * gmax)
        assert err < 2e-3, (name, err)
    if mode.startswith("overlap"):
        assert n_tail > 0
    if kind == "multimodal":
        assert any(n.startswith("g_s.") for n in res["names"]) and all(
            pr[n].grad is None for n in res["names"] if n.startswith("g_s."))
