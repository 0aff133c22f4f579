"""Phase timing of the fused ResidualUnit kernel from a diagnostic build: the stamps (RU_STAMP, cai_ru_probe_read)
are not in the product source -- re-apply commit 53c4b80's csrc/resunit.hip hunks, build with
tools/quick_variant.sh ruprobe resunit.hip -DCAI_RU_PROBE and run with CAI_LIB=<that lib> CAI_AB_STREAM=0.  One
AttentionBlock(192) step at B=4 per map size, then the per-block stamps of the last launch of each direction --
median / max of every phase in microseconds (profiles/r05_resunit_phase_probe.log).
usage: python tools/ru_probe.py"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "165-learning-based-multi-modality-image-and-video-compression_amd"))
import compressai.layers as L  # noqa: E402
from compressai import _native as native  # noqa: E402

names = ["staging", "phase A", "phase B taps", "epilogue B", "phase C mma", "epilogue C"]
lib = native.lib.load()
lib.cai_ru_probe_read.argtypes = [ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32]
dev = torch.device("cuda:0")
for H in (64, 16):
    torch.manual_seed(0)
    mod = L.AttentionBlock(192).to(dev)
    x0 = torch.randn(4, 192, H, H, device=dev).contiguous(memory_format=torch.channels_last)
    for _ in range(3):
        x = x0.clone().requires_grad_()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = mod(x)
        y.float().sum().backward()
    torch.cuda.synchronize()
    nblk = 4 * (H // 8) * (H // 8)
    for bwd in (0, 1):
        buf = np.zeros((nblk, 8), dtype=np.uint64)
        assert lib.cai_ru_probe_read(bwd, buf.ctypes.data, nblk) == 0
        t = buf[:, :7].astype(np.int64)
        t0 = t[:, 0].min()
        d = np.diff(t, axis=1) / 100.0   # 100 MHz ticks -> us
        print(f"{H}x{H} B=4 {'bwd' if bwd else 'fwd'}: {nblk} blocks, launch span {(t[:, 6].max() - t0) / 100:.2f} us, "
              f"block total median {np.median((t[:, 6] - t[:, 0]) / 100):.2f} us, start skew max {(t[:, 0].max() - t0) / 100:.2f} us")
        for k, n in enumerate(names):
            print(f"    {n:14s} median {np.median(d[:, k]):6.2f}  max {d[:, k].max():6.2f}")
