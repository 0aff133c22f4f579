"""Data parallelism on the product path: two ranks on cuda:0 (gloo over CUDA
tensors -- RCCL needs one GPU per rank), each running the graph-captured forward + backward of the product
ScaleHyperprior + FusedAdam on its half of the batch, then allreduce_mean_(opt.flat_grad).  The averaged flat
gradient must equal the oracle's gradient of the concatenated batch: the RD loss of equal halves is the mean
of the per-half losses (bpp and mse are per-batch means), so its gradient is the mean of the halves'."""
import os
import socket
import subprocess
import sys

import pytest
import torch

import cai_oracle as O

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("mode", ["serial", "overlap", "overlap-eager"])
def test_world2_allreduced_flat_grad_matches_oracle(cuda, tmp_path, mode):
    """serial: one all-reduce after the graph replay (bench.py --serial-allreduce); overlap: the two-bucket
    exchange of compressai.distributed.OverlappedAllReduce, the head bucket issued behind the graph's event
    node while g_a's backward runs; overlap-eager: the same with the head bucket issued from the hook."""
    torch.manual_seed(0)
    ref = O.ScaleHyperprior(32, 48)
    x = torch.rand(4, 3, 64, 64, generator=torch.Generator().manual_seed(11))
    feed = O.NoiseFeed(record=torch.Generator().manual_seed(12))
    sd = {k: v.clone() for k, v in ref.state_dict().items()}
    with feed:
        out = ref(x)
    O.RateDistortionLoss(1)(out, x)["loss"].backward()
    inp, outp = tmp_path / "in.pt", tmp_path / "out.pt"
    torch.save({"state_dict": sd, "x": x, "noise": [n.clone() for n in feed.drawn]}, inp)
    port = str(_port())
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK="0", WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=port, CAI_DIST_IN=str(inp), CAI_DIST_OUT=str(outp), CAI_DIST_MODE=mode)
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
    for name, off, n in zip(res["names"], res["offsets"], res["numels"]):
        g = flat[off:off + n]
        gr = pr[name].grad
        if gr is None:
            assert g.abs().max().item() == 0, name
            continue
        gr = gr.flatten()
        err = (g - gr).abs().max().item() / max(gr.abs().max().item(), 1e-30)
        assert err < 2e-3, (name, err)
