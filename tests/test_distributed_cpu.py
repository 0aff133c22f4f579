"""Data-parallel path at world_size 2 over gloo on CPU.

One process per rank, as torchrun launches bench.py: ranks start from rank 0's
weights (broadcast_parameters_), each computes gradients on its own patches,
and ONE all-reduce (mean) of the flat gradient buffer makes every rank hold
the gradient of the global batch.  Checked against the single-process
gradient of the concatenated batch, computed with the CPU oracle.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out_dir):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "165-learning-based-multi-modality-image-and-video-compression_amd"),
              os.path.join(root, "oracle")):
        sys.path.insert(0, p)
    import cai_oracle as O
    from compressai.distributed import allreduce_mean_, broadcast_parameters_, init_from_env

    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    r, w = init_from_env(backend="gloo")
    assert (r, w) == (rank, world)
    torch.manual_seed(100 + rank)          # deliberately different init per rank
    net = O.build("bmshj2018-hyperprior", 1)
    broadcast_parameters_(net)
    x = torch.rand(2, 3, 64, 64, generator=torch.Generator().manual_seed(rank))
    feed = O.NoiseFeed(record=torch.Generator().manual_seed(50 + rank))
    with feed:
        out = net(x)
    O.RateDistortionLoss(1)(out, x)["loss"].backward()
    params = [p for p in net.parameters() if p.grad is not None]
    flat = torch.cat([p.grad.flatten() for p in params])
    allreduce_mean_(flat)
    torch.save({"flat": flat, "state": net.state_dict(), "noise": feed.drawn, "x": x},
               os.path.join(out_dir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_gradient_allreduce_world2(tmp_path):
    import cai_oracle as O

    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    res = [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(world)]
    # identical replicated weights and identical averaged gradients on every rank
    for k, v in res[0]["state"].items():
        assert torch.equal(v, res[1]["state"][k]), k
    assert torch.equal(res[0]["flat"], res[1]["flat"])
    # mean of per-rank gradients == gradient of the mean of per-rank losses
    net = O.build("bmshj2018-hyperprior", 1)
    net.load_state_dict(res[0]["state"])
    total = 0.0
    for r in range(world):
        with O.NoiseFeed(tensors=list(res[r]["noise"])):
            out = net(res[r]["x"])
        total = total + O.RateDistortionLoss(1)(out, res[r]["x"])["loss"] / world
    total.backward()
    ref = torch.cat([p.grad.flatten() for p in net.parameters() if p.grad is not None])
    assert torch.allclose(res[0]["flat"], ref, rtol=1e-4, atol=1e-6)


# ---------------------------------------------------------------------------------------------------------
# The bucketed exchange's phase logic (compressai.distributed.OverlappedAllReduce) on CPU tensors: a toy model
# shaped like the zoo models (a Sequential analysis transform g_a whose output is the model's cut, further cut at
# the inputs of g_a[4] and g_a[2]; a head consuming y twice), FusedAdam-style flat gradients laid out by
# configure_optimizers(tail=("g_a.",), tail_cuts=...).  Each rank runs the phased backward + per-bucket
# all-reduce; the result must equal the all-reduced plain backward, bucket by bucket.
# ---------------------------------------------------------------------------------------------------------

def _toy_model():
    import torch.nn as nn

    class Toy(nn.Module):
        dp_tail = ("g_a.",)
        dp_tail_cuts = ("g_a.4", "g_a.2")
        _dp_cut_fn = None

        def __init__(self):
            super().__init__()
            self.g_a = nn.Sequential(nn.Conv2d(3, 8, 3, padding=1), nn.Tanh(), nn.Conv2d(8, 8, 3, padding=1),
                                     nn.Tanh(), nn.Conv2d(8, 8, 3, stride=2, padding=1), nn.Tanh(),
                                     nn.Conv2d(8, 6, 3, padding=1))
            self.h = nn.Conv2d(6, 6, 1)
            self.g_s = nn.Conv2d(6, 3, 3, padding=1)

        def _dp_cut(self, *ts):
            if self._dp_cut_fn is not None:
                ts = self._dp_cut_fn(*ts)
            return ts[0] if len(ts) == 1 else ts

        def forward(self, x):
            y = self._dp_cut(self.g_a(x))
            return (self.g_s(y) ** 2).mean() + (self.h(y).sigmoid() * y).mean()

    return Toy()


def _phase_worker(rank, world, port, out_dir, micro):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "165-learning-based-multi-modality-image-and-video-compression_amd"))
    from compressai.distributed import OverlappedAllReduce, allreduce_mean_, init_from_env
    from compressai.optim import dp_stage, parameter_groups

    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    init_from_env(backend="gloo")
    torch.manual_seed(0)
    net = _toy_model()
    main, _ = parameter_groups(net)
    named = dict(net.named_parameters())
    stage = [dp_stage(n, net.dp_tail, net.dp_tail_cuts) for n in main]
    order = [i for s in range(4) for i, t in enumerate(stage) if t == s]
    sizes = [named[main[i]].numel() for i in order]
    offs = [sum(sizes[:k]) for k in range(len(sizes))]
    bounds = [0] + [min([o for o, i in zip(offs, order) if stage[i] >= s] or [sum(sizes)]) for s in (1, 2, 3)]
    bounds.append(sum(sizes))
    flat = torch.zeros(sum(sizes))
    for o, i, n in zip(offs, order, sizes):     # parameters' .grad as views of the flat buffer (FusedAdam)
        named[main[i]].grad = flat[o:o + n].view_as(named[main[i]])
    head = [named[main[i]] for i in order if stage[i] == 0]
    stages = [[named[main[i]] for i in order if stage[i] == s] for s in (1, 2, 3)]
    sync = OverlappedAllReduce(flat, bounds, net, head, [net.get_submodule(c) for c in net.dp_tail_cuts], stages)
    assert sync.nphases == 4
    xs = [torch.rand(2, 3, 16, 16, generator=torch.Generator().manual_seed(10 * rank + k)) for k in range(micro)]
    # reference: the plain backward of the same loss, one all-reduce
    loss = sum(net(x) for x in xs)
    sync._cuts = {k: [] for k in sync._cuts}
    ref_flat = torch.autograd.grad(loss, [named[main[i]] for i in order])
    ref_local = torch.cat([g.flatten() for g in ref_flat])
    ref_flat = allreduce_mean_(ref_local.clone())
    # phased: micro-batch forwards accumulate their cuts; every bucket is final after its phase
    flat.zero_()
    loss = sum(net(x) for x in xs)
    assert [len(c) for c in sync._cuts.values()] == [micro] * 3
    sync.backward_head(loss)
    done = [flat[bounds[0]:bounds[1]].clone()]
    for i in range(1, sync.nphases):
        sync.reduce_bucket(i - 1)
        sync.backward_phase(i)
        done.append(flat[bounds[i]:bounds[i + 1]].clone())
    sync.finish()
    assert all(len(c) == 0 for c in sync._cuts.values())
    torch.save({"flat": flat, "ref": ref_flat, "ref_local": ref_local, "bounds": bounds, "done": done},
               os.path.join(out_dir, f"r{rank}.pt"))
    # a plain backward outside the phases releases its cuts: nothing leaks into the next step
    net(xs[0]).backward()
    assert all(len(c) == 0 for c in sync._cuts.values())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("micro", [1, 2])
def test_bucketed_phases_world2(tmp_path, micro):
    world = 2
    mp.spawn(_phase_worker, args=(world, _free_port(), str(tmp_path), micro), nprocs=world, join=True)
    res = [torch.load(tmp_path / f"r{r}.pt", weights_only=True) for r in range(world)]
    assert torch.equal(res[0]["flat"], res[1]["flat"])
    assert torch.allclose(res[0]["flat"], res[0]["ref"], rtol=1e-5, atol=1e-7)
    b = res[0]["bounds"]
    assert len(b) == 5 and all(b[i] < b[i + 1] for i in range(4))
    # each bucket was final when its phase ended (before its all-reduce): the rank's local gradient of the
    # whole loss, bucket by bucket
    for r in range(world):
        for i, d in enumerate(res[r]["done"]):
            assert torch.allclose(d, res[r]["ref_local"][b[i]:b[i + 1]], rtol=1e-5, atol=1e-7), (r, i)


def _toy_sync(net):
    from compressai.distributed import OverlappedAllReduce
    from compressai.optim import dp_stage, parameter_groups

    main, _ = parameter_groups(net)
    named = dict(net.named_parameters())
    stage = [dp_stage(n, net.dp_tail, net.dp_tail_cuts) for n in main]
    order = [i for s in range(4) for i, t in enumerate(stage) if t == s]
    sizes = [named[main[i]].numel() for i in order]
    offs = [sum(sizes[:k]) for k in range(len(sizes))]
    bounds = [0] + [min([o for o, i in zip(offs, order) if stage[i] >= s] or [sum(sizes)]) for s in (1, 2, 3)]
    bounds.append(sum(sizes))
    flat = torch.zeros(sum(sizes))
    for o, i, n in zip(offs, order, sizes):
        named[main[i]].grad = flat[o:o + n].view_as(named[main[i]])
    head = [named[main[i]] for i in order if stage[i] == 0]
    stages = [[named[main[i]] for i in order if stage[i] == s] for s in (1, 2, 3)]
    sync = OverlappedAllReduce(flat, bounds, net, head, [net.get_submodule(c) for c in net.dp_tail_cuts], stages)
    return sync, flat, [named[main[i]] for i in order]


def test_forward_without_backward_is_pruned():
    """a grad-enabled forward that is never backpropagated (a logging forward) must not keep its
    cuts (and graph) for the step, nor feed them to the phases: the phased gradient equals the plain one."""
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "165-learning-based-multi-modality-image-and-video-compression_amd"))
    torch.manual_seed(0)
    net = _toy_model()
    sync, flat, params = _toy_sync(net)
    x = torch.rand(2, 3, 16, 16, generator=torch.Generator().manual_seed(1))
    ref = torch.cat([g.flatten() for g in torch.autograd.grad(net(x), params)])
    sync._cuts = {k: [] for k in sync._cuts}
    sync._nfwd = 0
    flat.zero_()
    _ = net(torch.rand(2, 3, 16, 16))          # logging forward, no backward
    loss = net(x)
    assert [len(c) for c in sync._cuts.values()] == [2, 2, 2]
    sync.backward_head(loss)
    assert [len(c) for c in sync._cuts.values()] == [1, 1, 1]
    for i in range(1, sync.nphases):
        sync.backward_phase(i)
    sync.finish()
    assert torch.allclose(flat, ref, rtol=1e-5, atol=1e-7)
    sync.remove()


def test_tail_cuts_must_descend():
    """cuts of one parent listed in ascending order would leave the lower buckets zero; rejected."""
    import sys

    import pytest

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "165-learning-based-multi-modality-image-and-video-compression_amd"))
    from compressai.optim import check_tail_cuts, configure_optimizers

    assert check_tail_cuts(("g_a.4", "g_a.2")) == ("g_a.4", "g_a.2")
    assert check_tail_cuts(("g_a.5", "g_a.2", "g_a.1", "h.3")) == ("g_a.5", "g_a.2", "g_a.1", "h.3")
    for bad in (("g_a.2", "g_a.4"), ("g_a.2", "g_a.2"), ("g_a",)):
        with pytest.raises(ValueError):
            check_tail_cuts(bad)
    net = _toy_model()
    with pytest.raises(ValueError):
        configure_optimizers(net, tail=("g_a.",), tail_cuts=("g_a.2", "g_a.4"))


def _toy_plan_model():
    """A CPU stand-in shaped like the context models (JAHP / cheng2020): y = g_a(x) feeds the hyper path
    (h_a -> h_s -> "params"), the context model and the synthesis; the loss reads x_hat and two likelihoods."""
    import torch.nn as nn

    class ToyJ(nn.Module):
        _dp_mark_fn = None

        def __init__(self):
            super().__init__()
            self.g_a = nn.Sequential(nn.Conv2d(3, 8, 3, padding=1), nn.Tanh(), nn.Conv2d(8, 8, 3, padding=1),
                                     nn.Tanh(), nn.Conv2d(8, 6, 3, padding=1))
            self.h_a = nn.Conv2d(6, 6, 1)
            self.h_s = nn.Conv2d(6, 6, 1)
            self.ctx = nn.Conv2d(6, 6, 3, padding=1)
            self.ep = nn.Conv2d(6, 6, 1)
            self.g_s = nn.Sequential(nn.Conv2d(6, 8, 3, padding=1), nn.Tanh(), nn.Conv2d(8, 8, 3, padding=1),
                                     nn.Tanh(), nn.Conv2d(8, 3, 3, padding=1))

        def _dp_mark(self, name, *ts):
            if self._dp_mark_fn is not None:
                ts = self._dp_mark_fn(name, *ts)
            return ts[0] if len(ts) == 1 else ts

        def dp_phases(self):
            return [(["g_s.2.", "g_s.3.", "g_s.4."], ["loss"], ["g_s.2", "lik_y", "lik_z"]),
                    (["g_s.0.", "g_s.1."], ["g_s.2"], ["gs_in"]),
                    (["ep.", "ctx."], ["gs_in", "lik_y"], ["params", "yq"]),
                    (None, ["params", "lik_z"], ["y"]),
                    (["g_a.2.", "g_a.3.", "g_a.4."], ["y", "yq"], ["g_a.2"]),
                    (["g_a.0.", "g_a.1."], ["g_a.2"], [])]

        def forward(self, x):
            y = self._dp_mark("y", self.g_a(x))
            z = self.h_a(y)
            lik_z = torch.sigmoid(z) * 0.9 + 0.05
            params = self._dp_mark("params", self.h_s(z))
            yq = self._dp_mark("yq", y)
            g = self.ep(params + self.ctx(yq))
            lik_y = torch.sigmoid(g * yq) * 0.9 + 0.05
            x_hat = self.g_s(self._dp_mark("gs_in", yq))
            lik_y, lik_z = self._dp_mark("lik_y", lik_y), self._dp_mark("lik_z", lik_z)
            return (x_hat ** 2).mean() - torch.log(lik_y).mean() - 0.5 * torch.log(lik_z).mean()

    return ToyJ()


def test_phase_plan_buckets_final_in_order():
    """The plan-driven exchange (CompressionModel.dp_phases form: the synthesis in pieces, the context /
    entropy-parameter stack, the hyper path, g_a in pieces): after phase i, bucket i holds the plain backward's
    gradient and every later bucket is still untouched; y's gradient arrives in two parts (the hyper path's at
    y, the context path's at "yq", both roots of the first g_a phase); the likelihood cut lik_z waits two
    phases for its root.  (A phase whose inputs include y AND the "params" cut above the hyper path would
    pull that path into the phase: counted twice.)"""
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "165-learning-based-multi-modality-image-and-video-compression_amd"))
    from compressai.distributed import OverlappedAllReduce, _cut_site
    from compressai.optim import parameter_groups, phase_of

    torch.manual_seed(0)
    net = _toy_plan_model()
    plan = net.dp_phases()
    main, _ = parameter_groups(net)
    named = dict(net.named_parameters())
    stage = [phase_of(n, plan) for n in main]
    order = [i for s in range(len(plan)) for i, t in enumerate(stage) if t == s]
    sizes = [named[main[i]].numel() for i in order]
    offs = [sum(sizes[:k]) for k in range(len(sizes))]
    bounds = [0] + [min([o for o, i in zip(offs, order) if stage[i] >= s] or [sum(sizes)])
                    for s in range(1, len(plan))] + [sum(sizes)]
    assert all(bounds[i] < bounds[i + 1] for i in range(len(plan)))
    flat = torch.zeros(sum(sizes))
    for o, i, n in zip(offs, order, sizes):
        named[main[i]].grad = flat[o:o + n].view_as(named[main[i]])
    phases = [([named[main[i]] for i in order if stage[i] == k], r, inp) for k, (_, r, inp) in enumerate(plan)]
    names = {n for _, r, inp in plan for n in (*r, *inp) if n != "loss"}
    sync = OverlappedAllReduce(flat, bounds, phases=phases, sites={n: _cut_site(net, n) for n in names})
    assert sync.nphases == len(plan)
    xs = [torch.rand(2, 3, 12, 12, generator=torch.Generator().manual_seed(k)) for k in range(2)]
    loss = sum(net(x) for x in xs)
    ref = torch.cat([g.flatten() for g in torch.autograd.grad(loss, [named[main[i]] for i in order])])
    sync._cuts = {k: [] for k in sync._cuts}
    sync._nfwd = 0
    flat.zero_()
    loss = sum(net(x) for x in xs)            # two micro-batches: their cuts accumulate
    assert all(len(c) == 2 for c in sync._cuts.values())
    for i in range(sync.nphases):
        if i == 0:
            sync.backward_head(loss)
        else:
            sync.backward_phase(i)
        b0, b1 = bounds[i], bounds[i + 1]
        assert torch.allclose(flat[b0:b1], ref[b0:b1], rtol=1e-5, atol=1e-7), i
        assert not flat[b1:].any(), f"phase {i} wrote a later bucket"
    sync.finish()
    assert torch.allclose(flat, ref, rtol=1e-5, atol=1e-7)
    sync.remove()
    assert net._dp_mark_fn is None
