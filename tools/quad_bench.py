"""Per-launch timing of the C2 128-channel k5 s2 phase-direction layers through the C ABI (the launches
conv_halo_quad_kernel takes at B = 16): g_s[4] ConvTranspose2d 128->128 64^2 -> 128^2 forward and the g_a[2]
input gradient.  HIP events on the library's stream around N back-to-back launches; prints one line per layer.
usage: CAI_LIB=... python tools/quad_bench.py [--iters N] [--batch B]"""
import argparse
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "165-learning-based-multi-modality-image-and-video-compression_amd"))

from compressai import _native as native  # noqa: E402
from compressai._ops import _p, _stream  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--tag", default=os.path.basename(os.environ.get("CAI_LIB", "libcai.so")))
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    raw = native.lib.load()
    G = native.ConvGeom
    B = args.batch
    w = (torch.randn(128, 128, 5, 5, device=dev) * 0.05).contiguous()
    bias = torch.randn(128, device=dev)
    x = torch.randn(B, 64, 64, 128, device=dev).bfloat16().contiguous()
    y = torch.empty(B, 128, 128, 128, device=dev).bfloat16()
    cases = (("deconv_fwd", G(B, 128, 64, 64, 128, 128, 128, 5, 2, 2, 1, 1), 0),
             ("conv_dgrad", G(B, 128, 128, 128, 128, 64, 64, 5, 2, 2, 0, 0), 1))
    for rep, (kind, g, direction) in enumerate(cases + cases):   # the first round warms the clocks up
        name = raw.cai_conv_kernel_name(ctypes.byref(g), native.BF16, direction, 0).decode()
        wp = torch.empty(native.lib.cai_conv_packed_weight_bytes(ctypes.byref(g), native.BF16, direction),
                         dtype=torch.uint8, device=dev)
        native.lib.cai_conv_pack_weight(ctypes.byref(g), native.BF16, direction, _p(w), None, _p(wp), _stream())

        def launch():
            if direction == 0:
                native.lib.cai_conv_fwd(ctypes.byref(g), native.BF16, _p(x), 128, 0, _p(wp), _p(bias), 0, 0.0,
                                        _p(y), native.BF16, 128 * 128 * 128, 1, 128 * 128, 128, None, 0, _stream())
            else:
                native.lib.cai_conv_dgrad(ctypes.byref(g), native.BF16, _p(x), 128, _p(wp), _p(y), 128,
                                          native.MASK_NONE, 0.0, None, 0, None, 0, _stream())

        for _ in range(20):
            launch()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            launch()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / args.iters
        flop = 2.0 * B * 128 * 128 * 128 * 128 * 25 / 4
        if rep < len(cases):
            continue
        print(f"{args.tag:24s} {kind:10s} {name:26s} {us:8.2f} us  {flop / us / 1e6:7.1f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main()
