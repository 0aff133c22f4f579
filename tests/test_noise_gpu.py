"""Training noise on the device (cai_uniform_noise, csrc/entropy.hip) vs the Philox4x32-10 restatement
(oracle/philox_oracle.py, pinned by Random123 KATs in test_noise_cpu.py): bit-exact values, U(-1/2, 1/2)
moments, a new counter per call, and fresh noise on every replay of a captured graph."""
import pytest
import torch

import philox_oracle as P

pytestmark = pytest.mark.gpu


def _state(seed, draw=0):
    from compressai.entropy_models.entropy_models import _as_i64

    return torch.tensor([_as_i64(seed), _as_i64(draw), 0], dtype=torch.int64, device="cuda")


def _draw(n, st):
    from compressai._native import lib
    from compressai._ops import _p, _stream

    out = torch.empty(n, dtype=torch.float32, device="cuda")
    assert lib.cai_uniform_noise(_p(out), n, _p(st), _stream()) == 0
    return out


@pytest.mark.parametrize("seed,draw", [(0, 0), (123456789, 5), ((1 << 64) - 1, (1 << 40) + 3)])
def test_noise_matches_philox(cuda, seed, draw):
    st = _state(seed, draw)
    n = 4099                                     # ragged tail: the scalar store path
    out = _draw(n, st).cpu().numpy()
    for start in (0, 1024, n - 7):
        want = P.uniform_noise(min(64, n - start), seed, draw, start)
        assert (out[start:start + len(want)] == want).all()
    from compressai.entropy_models.entropy_models import _as_i64

    assert int(st[1].item()) == _as_i64(draw + 1) and int(st[2].item()) == 0   # advanced once, ticket reset


def test_noise_moments_and_fresh_draws(cuda):
    st = _state(7)
    a, b = _draw(1 << 22, st), _draw(1 << 22, st)   # > 2048 blocks' worth of quads: grid-stride loop
    for u in (a, b):
        assert float(u.min()) >= -0.5 and float(u.max()) < 0.5
        assert abs(float(u.mean())) < 1e-3
        assert abs(float(u.var()) - 1.0 / 12.0) < 1e-3
    assert not torch.equal(a, b)
    assert int(st[1].item()) == 2


def test_graph_replay_draws_fresh_noise(cuda):
    from compressai.entropy_models import seed_noise
    from compressai.entropy_models.entropy_models import _draw_noise

    x = torch.zeros(2, 8, 16, 16, device="cuda").contiguous(memory_format=torch.channels_last)
    seed_noise(99)
    e0, e1 = _draw_noise(x).clone(), _draw_noise(x).clone()
    assert e0.stride() == x.stride() and not torch.equal(e0, e1)
    seed_noise(99)
    static = torch.empty_like(x)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            static.copy_(_draw_noise(x))
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    r0 = static.clone()
    g.replay()
    r1 = static.clone()
    assert torch.equal(r0, e0) and torch.equal(r1, e1)


def test_manual_seed_reproducible(cuda):
    """torch.cuda.manual_seed(s) with a new seed value restarts the generator from s (seed_noise(s) restarts
    it unconditionally)."""
    from compressai.entropy_models import seed_noise
    from compressai.entropy_models.entropy_models import _draw_noise

    x = torch.zeros(3, 5, 7, 9, device="cuda")
    torch.cuda.manual_seed(2024)
    a = _draw_noise(x).clone()
    torch.cuda.manual_seed(2025)
    c = _draw_noise(x).clone()
    torch.cuda.manual_seed(2024)
    b = _draw_noise(x).clone()
    seed_noise(2024)
    d = _draw_noise(x).clone()
    assert torch.equal(a, b) and torch.equal(a, d) and not torch.equal(a, c)


@pytest.mark.parametrize("arch,draws", [("bmshj2018-hyperprior", 2), ("mbt2018", 3)])
def test_hyper_stream_device_noise_one_stream(cuda, monkeypatch, arch, draws):
    """The models' hyper branch on a side stream with the DEVICE generator (no injected noise): every draw
    of a step runs on the caller's stream (z's before the fork), so after N graph replays the draw index
    advanced by exactly N x the draws per step, the arrival ticket is back at 0, and z's noise, y's and
    (mbt2018) the likelihood's second draw come from distinct counter ranges."""
    import compressai.models.google as G
    from compressai.entropy_models import seed_noise
    from compressai.entropy_models.entropy_models import _as_i64, _noise_state
    from compressai.zoo import image_models

    monkeypatch.setattr(G, "_HYPER_STREAM", "1")
    drawn = []
    real = G._draw_noise

    def rec(t):
        n = real(t)
        drawn.append((torch.cuda.current_stream().cuda_stream, n.detach().clone()))
        return n

    monkeypatch.setattr(G, "_draw_noise", rec)
    import compressai.entropy_models.entropy_models as E

    monkeypatch.setattr(E, "_draw_noise", rec)
    real_for = G._noise_for
    handles = []

    def rec_for(t):      # y's draw: a DeviceDraw made inside the quantize kernel on the caller's stream
        n = real_for(t)
        handles.append(n)
        drawn.append((torch.cuda.current_stream().cuda_stream, None))
        return n

    monkeypatch.setattr(G, "_noise_for", rec_for)
    torch.manual_seed(0)
    net = image_models[arch](1).cuda().train()
    x = torch.rand(2, 3, 64, 64, generator=torch.Generator().manual_seed(1)).cuda()
    seed_noise(4321)
    st = _noise_state(x.device)
    main = torch.cuda.current_stream().cuda_stream

    def step():
        out = net(x)
        loss = sum(v.float().log().sum() for v in out["likelihoods"].values()) + out["x_hat"].float().sum()
        loss.backward()

    step()
    torch.cuda.synchronize()
    assert int(st[1].item()) == draws and int(st[2].item()) == 0
    assert len(drawn) == draws and all(s == main for s, _ in drawn)
    flat = [n.flatten() for _, n in drawn if n is not None]
    for i in range(len(flat)):
        for j in range(i + 1, len(flat)):
            k = min(flat[i].numel(), flat[j].numel())
            assert not torch.equal(flat[i][:k], flat[j][:k]), (i, j)
    # the in-kernel draws recorded their own draw indices: distinct, inside this step's range
    idx = [int(h.slot[1]) for h in handles if hasattr(h, "slot")]
    assert len(set(idx)) == len(idx) and all(0 <= i < draws for i in idx)
    # captured: the same invariants over replays
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    torch.cuda.synchronize()
    before = int(st[1].item())
    reps = 7
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    assert int(st[1].item()) == _as_i64(before + reps * draws) and int(st[2].item()) == 0


# ---------------------------------------------------------------------------------------------------------------
# in-kernel draws (cai_noise_src DRAW / REPLAY, _ops.DeviceDraw) vs the same kernels fed by cai_uniform_noise
# ---------------------------------------------------------------------------------------------------------------

def _full_state(seed, draw):
    from compressai._native import NOISE_STATE_WORDS
    from compressai.entropy_models.entropy_models import _as_i64

    st = torch.zeros(NOISE_STATE_WORDS, dtype=torch.int64, device="cuda")
    st[0], st[1] = _as_i64(seed), _as_i64(draw)
    return st


def _buf_for(x, st):
    """cai_uniform_noise's draw in x's (dense, pixel-major) layout: element (p, c) at storage index p*C + c."""
    from compressai._native import lib
    from compressai._ops import _p, _stream

    n = torch.empty_like(x, dtype=torch.float32)
    assert lib.cai_uniform_noise(_p(n), n.numel(), _p(st), _stream()) == 0
    return n


def _pair(shape, dtype, seed=77, draw=5):
    from compressai._ops import DeviceDraw

    g = torch.Generator().manual_seed(sum(shape))
    x = (torch.randn(*shape, generator=g) * 3).cuda().to(dtype).contiguous(memory_format=torch.channels_last)
    sa, sb = _full_state(seed, draw), _full_state(seed, draw)
    return x, _buf_for(x, sa), sa, DeviceDraw(x.shape, sb), sb


def _check_state(sa, sb, d):
    torch.cuda.synchronize()
    assert torch.equal(sa, sb), "generator states diverged"
    assert int(sb[1]) == d + 1 and int(sb[2:].abs().sum()) == 0      # advanced once, tickets and shards reset


# (B, C, H, W): one block (fewer than 8 shards), a ragged grid, a multiple of 8, the capped 1024-block grid
_EW_SHAPES = [(1, 3, 5, 7), (3, 20, 37, 29), (2, 192, 16, 16), (16, 192, 16, 16)]


@pytest.mark.parametrize("shape", _EW_SHAPES)
def test_quantize_draw_matches_buffer(cuda, shape):
    from compressai._native import Q_NOISE
    from compressai.entropy_models.entropy_models import _QuantizeFn

    x, nbuf, sa, draw, sb = _pair(shape, torch.float32)
    a = _QuantizeFn.apply(x, None, nbuf, Q_NOISE)
    b = _QuantizeFn.apply(x, None, draw, Q_NOISE)
    _check_state(sa, sb, 5)
    assert torch.equal(a, b)
    assert draw.slot.tolist() == [77, 5]


@pytest.mark.parametrize("shape", _EW_SHAPES)
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gaussian_draw_replay_matches_buffer(cuda, shape, dtype):
    """gc_fwd DRAW == gc_fwd on cai_uniform_noise's buffer, and gc_bwd REPLAY == gc_bwd on the buffer."""
    from compressai.entropy_models import GaussianConditional

    x, nbuf, sa, draw, sb = _pair(shape, dtype)
    gen = torch.Generator().manual_seed(3)
    scales = (torch.rand(*shape, generator=gen) * 4 + 0.05).cuda().to(dtype).contiguous(
        memory_format=torch.channels_last)
    means = (torch.randn(*shape, generator=gen)).cuda().to(dtype).contiguous(memory_format=torch.channels_last)
    gc = GaussianConditional(None).cuda().train()
    outs = []
    for noise in (nbuf, draw):
        xi, si, mi = (t.detach().clone().requires_grad_(True) for t in (x, scales, means))
        q, lik = gc(xi, si, means=mi, noise=noise)
        (q.float().sum() * 0.3 + lik.log().sum()).backward()
        outs.append((q, lik, xi.grad, si.grad, mi.grad))
    _check_state(sa, sb, 5)
    for u, v in zip(*outs):
        assert torch.equal(u, v)


@pytest.mark.parametrize("shape", [(16, 128, 4, 4), (1, 3, 5, 7), (16, 192, 16, 16), (2, 40, 33, 17)])
def test_bottleneck_draw_replay_matches_buffer(cuda, shape):
    """eb_fwd DRAW (its grid capped for the tickets on the large case) and eb_bwd REPLAY == the buffer path."""
    from compressai.entropy_models import EntropyBottleneck

    x, nbuf, sa, draw, sb = _pair(shape, torch.float32)
    torch.manual_seed(0)
    eb = EntropyBottleneck(shape[1]).cuda().train()
    outs = []
    for noise in (nbuf, draw):
        eb.zero_grad(set_to_none=True)
        xi = x.detach().clone().requires_grad_(True)
        q, lik = eb(xi, noise=noise)
        (q.sum() * 0.1 + lik.log().sum()).backward()
        outs.append((q, lik, xi.grad) + tuple(p.grad.clone() for p in eb.parameters()))
    _check_state(sa, sb, 5)
    for u, v in zip(*outs):
        assert torch.equal(u, v)


def test_device_draw_graph_replays_fresh(cuda):
    """A DeviceDraw made inside a captured region draws a new index on every replay (its slot lives in the
    graph's pool), and the backward inside the same graph replays that draw."""
    from compressai.entropy_models import GaussianConditional, seed_noise
    from compressai.entropy_models.entropy_models import _noise_state

    x = torch.randn(4, 64, 8, 8, device="cuda").contiguous(memory_format=torch.channels_last)
    scales = torch.full_like(x, 1.5)
    gc = GaussianConditional(None).cuda().train()
    xi = x.clone().requires_grad_(True)

    def step():
        q, lik = gc(xi, scales)
        lik.log().sum().backward()
        return q

    seed_noise(5)
    step()
    torch.cuda.synchronize()
    st = _noise_state(x.device)
    assert int(st[1]) == 1
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    xi.grad = None
    with torch.cuda.graph(g):
        q = step()
    qs = []
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        qs.append((q.detach() - x).clone())
    assert int(st[1]) == 2 + 3 and int(st[2:].abs().sum()) == 0
    for u in qs:
        assert float(u.min()) >= -0.5 - 1e-5 and float(u.max()) <= 0.5 + 1e-5   # (x + u) - x rounds
    assert not torch.equal(qs[0], qs[1]) and not torch.equal(qs[1], qs[2])
