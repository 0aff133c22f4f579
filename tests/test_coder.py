"""Entropy-coding side (libcai_coder.so via compressai._CXX / compressai.ans) vs the
pure-Python oracle (oracle/cai_coder_oracle.py).  Host code: runs on CPU.

Bar: bit-exact -- identical quantized CDF tables and identical stream bytes;
decode(encode(x)) == x including out-of-range symbols (bypass escapes).
Pins: the reference's KAT pmf_to_quantized_cdf([0.1, 0.2, 0, 0], 16)
(tests/test_ops.py:103-106) and its error cases (:108-118).
"""
import ctypes
import os
import re

import numpy as np
import pytest

import cai_coder_oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def coder():
    from compressai import _coder

    if not os.path.exists(_coder.LIB_PATH):
        pytest.skip("libcai_coder.so not built")
    _coder.lib.load()
    return _coder


def _declared():
    src = open(os.path.join(ROOT, "include", "cai_coder.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(cai_[a-z0-9_]+)\s*\(", src)))


def test_header_symbols_exported_and_bound(coder):
    raw = ctypes.CDLL(coder.LIB_PATH)
    decl = _declared()
    assert [f for f in decl if not hasattr(raw, f)] == []
    assert set(decl) == set(coder.SIGNATURES)
    assert coder.lib.cai_coder_abi_count() == len(decl)


def test_pmf_to_quantized_cdf_kat(coder):
    from compressai._CXX import pmf_to_quantized_cdf

    assert pmf_to_quantized_cdf([0.1, 0.2, 0, 0], 16) == [0, 21845, 65534, 65535, 65536]
    assert O.pmf_to_quantized_cdf([0.1, 0.2, 0, 0], 16) == [0, 21845, 65534, 65535, 65536]


@pytest.mark.parametrize("pmf", [[0.1, -0.2, 0.3], [0.1, float("nan")], [0.1, float("inf")], [0.0, 0.0]])
def test_pmf_to_quantized_cdf_errors(coder, pmf):
    """tests/test_ops.py:108-118: invalid pmfs raise ValueError."""
    from compressai._CXX import pmf_to_quantized_cdf

    with pytest.raises(ValueError):
        pmf_to_quantized_cdf(pmf, 16)
    with pytest.raises(ValueError):
        O.pmf_to_quantized_cdf(pmf, 16)


@pytest.mark.parametrize("seed", range(6))
def test_pmf_to_quantized_cdf_matches_oracle(coder, seed):
    from compressai._CXX import pmf_to_quantized_cdf

    rng = np.random.default_rng(seed)
    n = int(rng.integers(2, 300))
    p = rng.random(n).astype(np.float32) ** 6      # many near-zero slots: exercises the stealing loop
    p[rng.random(n) < 0.2] = 0
    p[0] = max(p[0], 1e-3)
    p = (p / p.sum()).astype(np.float32)
    assert pmf_to_quantized_cdf(p.tolist(), 16) == O.pmf_to_quantized_cdf(p.tolist(), 16)


def test_cdf_rows_match_single(coder):
    rng = np.random.default_rng(7)
    lengths = rng.integers(2, 40, size=24).astype(np.int32)
    pmf = np.zeros((24, 40), dtype=np.float32)
    for r, n in enumerate(lengths):
        q = rng.random(n).astype(np.float32)
        pmf[r, :n] = q / q.sum()
    tab = coder.pmf_to_quantized_cdf_rows(pmf, lengths, 16, 42)
    for r, n in enumerate(lengths):
        assert tab[r, :n + 1].tolist() == O.pmf_to_quantized_cdf(pmf[r, :n].tolist(), 16)
        assert not tab[r, n + 1:].any()


def _tables(rng, ncdf=5):
    cdfs, sizes, offs = [], [], []
    for _ in range(ncdf):
        n = int(rng.integers(1, 24))
        q = rng.random(n + 1).astype(np.float32)
        q[-1] = 1e-6                                  # tail mass slot
        c = O.pmf_to_quantized_cdf((q / q.sum()).tolist(), 16)
        cdfs.append(c)
        sizes.append(len(c))
        offs.append(-int(rng.integers(0, n + 1)))
    return cdfs, sizes, offs


@pytest.mark.parametrize("seed", range(5))
def test_rans_bytes_match_oracle(coder, seed):
    from compressai import ans

    rng = np.random.default_rng(100 + seed)
    cdfs, sizes, offs = _tables(rng)
    n = int(rng.integers(1, 700))
    syms = rng.integers(-60, 60, size=n)
    syms[rng.random(n) < 0.01] = 1 << 20           # long bypass escapes
    syms[rng.random(n) < 0.01] = -(1 << 20)
    idx = rng.integers(0, len(cdfs), size=n)
    s_ref = O.encode_with_indexes(syms.tolist(), idx.tolist(), cdfs, sizes, offs)
    s = ans.RansEncoder().encode_with_indexes(syms.tolist(), idx.tolist(), cdfs, sizes, offs)
    assert s == s_ref
    assert ans.RansDecoder().decode_with_indexes(s, idx.tolist(), cdfs, sizes, offs) == syms.tolist()
    assert O.decode_with_indexes(s, idx.tolist(), cdfs, sizes, offs) == syms.tolist()


def test_buffered_encoder_and_stream_decoder(coder):
    """BufferedRansEncoder + RansDecoder.set_stream/decode_stream (the AR models' pattern)."""
    from compressai import ans

    rng = np.random.default_rng(5)
    cdfs, sizes, offs = _tables(rng, 4)
    chunks = [(rng.integers(-10, 10, size=int(k)), rng.integers(0, 4, size=int(k))) for k in rng.integers(1, 30, 12)]
    enc, ref = ans.BufferedRansEncoder(), O.BufferedRansEncoder()
    for s, i in chunks:
        enc.encode_with_indexes(s.tolist(), i.tolist(), cdfs, sizes, offs)
        ref.encode_with_indexes(s.tolist(), i.tolist(), cdfs, sizes, offs)
    stream = enc.flush()
    assert stream == ref.flush()
    dec = ans.RansDecoder()
    dec.set_stream(stream)
    for s, i in chunks:
        assert dec.decode_stream(i.tolist(), cdfs, sizes, offs) == s.tolist()


def test_single_symbol_and_empty_streams(coder):
    from compressai import ans

    cdfs = [O.pmf_to_quantized_cdf([0.5, 0.5, 1e-9], 16)]
    sizes, offs = [len(cdfs[0])], [0]
    for syms in ([], [0], [1], [5], [-3]):
        s = ans.RansEncoder().encode_with_indexes(syms, [0] * len(syms), cdfs, sizes, offs)
        assert s == O.encode_with_indexes(syms, [0] * len(syms), cdfs, sizes, offs)
        assert ans.RansDecoder().decode_with_indexes(s, [0] * len(syms), cdfs, sizes, offs) == syms


def test_batch_streams_equal_single(coder):
    from compressai import ans

    rng = np.random.default_rng(11)
    cdfs, sizes, offs = _tables(rng)
    tabs = coder.Tables(cdfs, sizes, offs)
    sym = rng.integers(-30, 30, size=(6, 200))
    idx = rng.integers(0, len(cdfs), size=(6, 200))
    strings = coder.encode_streams(sym, idx, tabs, 6)
    for b in range(6):
        assert strings[b] == ans.RansEncoder().encode_with_indexes(sym[b].tolist(), idx[b].tolist(), cdfs, sizes, offs)
    assert (coder.decode_streams(strings, idx, tabs) == sym).all()


def test_invalid_arguments_raise(coder):
    from compressai import ans

    cdfs = [O.pmf_to_quantized_cdf([0.5, 0.5], 16)]
    with pytest.raises(ValueError, match="out of range"):
        ans.RansEncoder().encode_with_indexes([0], [3], cdfs, [3], [0])
    s = ans.RansEncoder().encode_with_indexes(list(range(2)) * 50, [0] * 100, cdfs, [3], [0])
    with pytest.raises(ValueError):
        ans.RansDecoder().decode_with_indexes(s[:5], [0] * 100, cdfs, [3], [0])   # not a whole word
    with pytest.raises(ValueError):
        ans.RansDecoder().decode_with_indexes(s[:8], [0] * 100, cdfs, [3], [0])   # truncated


def test_update_tables_cpu_exact(coder):
    """EntropyBottleneck / GaussianConditional.update() (entropy_models.py:396-441, 655-678) on CPU
    parameters: the pmfs are the reference's torch expressions, so the tables equal the oracle's
    pure-Python quantization of the same pmfs exactly."""
    import torch

    import cai_oracle as OR
    from compressai.entropy_models import EntropyBottleneck, GaussianConditional
    from compressai.models import get_scale_table

    torch.manual_seed(2)
    ref = OR.EntropyBottleneck(16)
    with torch.no_grad():
        ref.quantiles.add_(torch.randn(16, 1, 3))
    eb = EntropyBottleneck(16)
    eb.load_state_dict(ref.state_dict(), strict=False)
    assert eb.update() and not eb.update() and eb.update(force=True)
    with torch.no_grad():
        q = ref.quantiles
        med = q[:, 0, 1]
        mn = torch.clamp(torch.ceil(med - q[:, 0, 0]).int(), min=0)
        mx = torch.clamp(torch.ceil(q[:, 0, 2] - med).int(), min=0)
        length = mn + mx + 1
        samples = torch.arange(int(length.max()))[None, :] + (med - mn)[:, None, None]
        lo = ref._logits_cumulative(samples - 0.5, stop_gradient=True)
        up = ref._logits_cumulative(samples + 0.5, stop_gradient=True)
        sg = -torch.sign(lo + up)
        pmf = torch.abs(torch.sigmoid(sg * up) - torch.sigmoid(sg * lo))[:, 0, :]
        tail = torch.sigmoid(lo[:, 0, :1]) + torch.sigmoid(-up[:, 0, -1:])
    assert torch.equal(eb._offset, -mn) and torch.equal(eb._cdf_length, length + 2)
    for i, n in enumerate(length.tolist()):
        c = O.pmf_to_quantized_cdf(pmf[i, :n].tolist() + [float(tail[i, 0])], 16)
        assert eb._quantized_cdf[i, :len(c)].tolist() == c
        assert not eb._quantized_cdf[i, len(c):].any()

    gc = GaussianConditional(None)
    assert gc.update_scale_table(get_scale_table())
    st = get_scale_table().float()
    center = torch.ceil(st * float(-__import__("scipy.stats").stats.norm.ppf(1e-9 / 2))).int()
    assert torch.equal(gc._offset, -center)
    samples = torch.abs(torch.arange(int((2 * center + 1).max())).int() - center[:, None]).float()
    upper = 0.5 * torch.erfc(float(-(2 ** -0.5)) * ((0.5 - samples) / st[:, None]))
    lower = 0.5 * torch.erfc(float(-(2 ** -0.5)) * ((-0.5 - samples) / st[:, None]))
    pmf = upper - lower
    for i in (0, 9, 33, 63):
        n = int(2 * center[i] + 1)
        c = O.pmf_to_quantized_cdf(pmf[i, :n].tolist() + [float(2 * lower[i, 0])], 16)
        assert gc._quantized_cdf[i, :len(c)].tolist() == c
