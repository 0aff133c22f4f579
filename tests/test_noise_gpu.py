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
    flat = [n.flatten() for _, n in drawn]
    for i in range(draws):
        for j in range(i + 1, draws):
            k = min(flat[i].numel(), flat[j].numel())
            assert not torch.equal(flat[i][:k], flat[j][:k]), (i, j)
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
