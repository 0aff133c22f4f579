"""Two host threads through the library at once ("The library must be reentrant with no global
mutable state, because DataParallel-style callers run one host thread per device").

Two independent replicas -- own weights, own FusedAdam pair, own CUDA stream, own training noise -- each take
two full training steps (bf16 forward, RD loss, backward with the deferred parameter-gradient reduces, fused
clip + Adam, aux loss + aux Adam: examples/train.py:155-186) concurrently from two host threads on cuda:0.  Every
kernel is deterministic (fixed-order reductions), so each replica must end bit-identical to the same two steps
run serially on the main thread.  A shared hand-off buffer, a deferred-reduce queue joined across the two
backwards, or any other shared mutable state shows up as a mismatch.  nn.DataParallel replicas themselves are
rejected (tests/test_api_cpu.py::test_dataparallel_replica_rejected).
"""
import threading

import pytest
import torch

pytestmark = pytest.mark.gpu

_tl = threading.local()


def _thread_noise(t):
    # the injected source is process-global; each thread draws from its own replica's generator
    return torch.empty(t.shape).uniform_(-0.5, 0.5, generator=_tl.gen).to(t.device)


class _Replica:
    def __init__(self, name, quality, seed, size, batch, dev):
        from compressai.losses import RateDistortionLoss
        from compressai.optim import configure_optimizers
        from compressai.zoo import image_models

        torch.manual_seed(seed)
        self.net = image_models[name](quality).to(dev).train()
        self.opt, self.aux_opt = configure_optimizers(self.net, zero_grad_in_step=True)
        self.crit = RateDistortionLoss(quality)
        self.x = torch.rand(batch, 3, size, size, generator=torch.Generator().manual_seed(seed + 1)).to(dev)
        self.seed = seed
        self.stream = torch.cuda.Stream(device=dev)
        self.losses = []

    def steps(self, n):
        _tl.gen = torch.Generator().manual_seed(self.seed + 2)
        self.stream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self.stream):
            for _ in range(n):
                self.opt.zero_grad()
                self.aux_opt.zero_grad()
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    out = self.net(self.x)
                    c = self.crit(out, self.x)
                c["loss"].backward()
                self.opt.step(max_norm=1.0)
                aux = self.net.aux_loss()
                aux.backward()
                self.aux_opt.step()
                self.losses.append(c["loss"].detach().clone())
        self.stream.synchronize()

    def state(self):
        return {n: p.detach().clone() for n, p in self.net.named_parameters()}


@pytest.mark.parametrize("name,quality,size,batch", [
    ("bmshj2018-hyperprior", 1, 256, 4),     # lane GDN, halo / phase / edge kernels, deferred reduces
    ("cheng2020-attn", 6, 128, 1),           # residual chains, attention gates, context model
], ids=["hyperprior-q1", "cheng2020-attn-q6"])
def test_two_threads_match_serial(cuda, name, quality, size, batch):
    from compressai.entropy_models import set_noise_source

    set_noise_source(_thread_noise)
    try:
        serial = [_Replica(name, quality, s, size, batch, cuda) for s in (10, 20)]
        for r in serial:
            r.steps(2)
        conc = [_Replica(name, quality, s, size, batch, cuda) for s in (10, 20)]
        errors = []

        def run(r):
            try:
                r.steps(2)
            except BaseException as e:   # surfaced below
                errors.append(e)

        threads = [threading.Thread(target=run, args=(r,)) for r in conc]
        for t in threads:
            t.start()
        for t in threads:
            t.join(timeout=100)
        assert not any(t.is_alive() for t in threads), "a replica thread did not finish"
        assert not errors, errors
    finally:
        set_noise_source(None)
    torch.cuda.synchronize()
    for a, b in zip(serial, conc):
        for la, lb in zip(a.losses, b.losses):
            assert torch.equal(la, lb), (la.item(), lb.item())
        sa, sb = a.state(), b.state()
        bad = [n for n in sa if not torch.equal(sa[n], sb[n])]
        assert not bad, bad[:5]
