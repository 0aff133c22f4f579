"""Per-launch timing of the C2 GDN / IGDN layers at 16 x 128 x 128 x 128 (bf16) through the C ABI: the lane
forward (cai_gdn_fwd) and the lane backward kernel alone (cai_gdn_backward_deferred: the parameter-gradient
reduce left as a job, not run).  HIP events around N launches after a warm-up round.
usage: CAI_LIB=... python tools/gdn_bench.py [--iters N] [--npix P]"""
import argparse
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "165-learning-based-multi-modality-image-and-video-compression_amd"))

from compressai import _native as native  # noqa: E402
from compressai._native import ReduceJob  # noqa: E402
from compressai._ops import _p, _stream  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--npix", type=int, default=16 * 128 * 128)
    ap.add_argument("--tag", default=os.path.basename(os.environ.get("CAI_LIB", "libcai.so")))
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    C, P = 128, args.npix
    raw = native.lib.load()
    beta_raw = (torch.rand(C, device=dev) + 0.5).contiguous()
    gamma_raw = (torch.rand(C, C, device=dev) * 0.1).contiguous()
    beta = torch.empty(C, device=dev)
    gop = torch.empty(2 * C * C, dtype=torch.bfloat16, device=dev)
    native.lib.cai_gdn_reparam(_p(beta_raw), _p(gamma_raw), C, 1e-6, 2 ** -18, native.BF16, _p(beta), _p(gop),
                               _stream())
    x = torch.randn(P, C, device=dev).bfloat16().contiguous()
    dy = torch.randn(P, C, device=dev).bfloat16().contiguous()
    out = torch.empty(P, C, device=dev).bfloat16()
    dbr, dgr = torch.zeros(C, device=dev), torch.zeros(C, C, device=dev)
    nws = native.lib.cai_gdn_backward_workspace_bytes(P, C, native.BF16)
    ws = torch.empty(nws, dtype=torch.uint8, device=dev)
    job = ReduceJob()
    for inv in (0, 1):
        fname = raw.cai_gdn_kernel_name(native.BF16, P, C, C, C, 0).decode() if hasattr(raw, "cai_gdn_kernel_name") else "gdn"

        def fwd():
            native.lib.cai_gdn_fwd(native.BF16, _p(x), C, P, C, _p(gop), _p(beta), inv, _p(out), C, _stream())

        def bwd():
            native.lib.cai_gdn_backward_deferred(native.BF16, _p(x), C, _p(dy), C, P, C, _p(gop), _p(beta), inv,
                                                 _p(out), C, _p(beta_raw), _p(gamma_raw), 1e-6, 2 ** -18, _p(dbr),
                                                 _p(dgr), 0, _p(ws), nws, _stream(), ctypes.byref(job))

        for what, fn in (("fwd", fwd), ("bwd", bwd)):
            for rep in range(2):
                for _ in range(20):
                    fn()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.iters):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / args.iters
            nbytes = P * C * 2 * (2 if what == "fwd" else 3)
            print(f"{args.tag:22s} {'IGDN' if inv else 'GDN ':4s} {what} npix={P} {us:8.2f} us  "
                  f"{nbytes / us / 1e6:5.2f} TB/s (x{', dy' if what == 'bwd' else ''} in, {'dx' if what == 'bwd' else 'y'} out)",
                  flush=True)


if __name__ == "__main__":
    main()
