"""Replay timing of the deferred parameter-gradient reduces (cai_reduce_jobs) of a real training step.

Runs a few eager C2 steps (bmshj2018-hyperprior q1, B=16, 256^2, bf16, FusedAdam: deferred reduces on), records
every cai_reduce_jobs call (job list), keeps the step's tensors alive, then replays each recorded call N times
between HIP events and prints its time, job mix and the partial bytes it reads.
usage: CAI_LIB=... python tools/reduce_bench.py [--model ...] [--iters N]"""
import argparse
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "165-learning-based-multi-modality-image-and-video-compression_amd"))

from compressai import _ops  # noqa: E402
from compressai._native import ReduceJob  # noqa: E402
from compressai.losses import RateDistortionLoss  # noqa: E402
from compressai.optim import configure_optimizers  # noqa: E402
from compressai.zoo import image_models  # noqa: E402

KIND = {1: "WGRAD", 2: "GDN", 3: "EDGE"}


def job_bytes(j):
    if j.kind == 1:       # S splits x Ng x ncols fp32
        return 4.0 * j.i[0] * j.i[1] * j.i[2]
    if j.kind == 2:       # nblk x (C*C + C) fp32
        return 4.0 * j.i[0] * (j.i[1] * j.i[1] + j.i[1])
    return 0.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="bmshj2018-hyperprior")
    ap.add_argument("--quality", type=int, default=1)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--tag", default=os.path.basename(os.environ.get("CAI_LIB", "libcai.so")))
    ap.add_argument("-v", action="store_true", help="time every job alone as well")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    net = image_models[args.model](args.quality).to(dev).train()
    opt, aux_opt = configure_optimizers(net)
    x = torch.rand(args.batch, 3, 256, 256, device=dev)
    crit = RateDistortionLoss(args.quality)
    real = _ops.lib
    calls = []

    class Spy:
        def __getattr__(self, name):
            fn = getattr(real, name)
            if name != "cai_reduce_jobs":
                return fn

            def call(arr, n, st):
                calls.append((ReduceJob * n)(*[arr[i] for i in range(n)]))
                return fn(arr, n, st)
            return call

    keep = []
    for it in range(3):
        if it == 2:
            _ops.lib = Spy()
        opt.zero_grad()
        aux_opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = net(x)
            loss = crit(out, x)["loss"]
        loss.backward()
        keep.append((out, loss))
    _ops.lib = real
    torch.cuda.synchronize()
    # the recorded jobs read workspaces the caching allocator took back: hold every cached block (no allocation
    # below may reuse them while the replays read)
    total_b = 0.0
    for k, arr in enumerate(calls):
        jobs = list(arr)
        kinds = {}
        for j in jobs:
            kinds[KIND.get(j.kind, "?")] = kinds.get(KIND.get(j.kind, "?"), 0) + 1
        nbytes = sum(job_bytes(j) for j in jobs)
        for _ in range(5):
            real.cai_reduce_jobs(arr, len(jobs), _ops._stream())
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            real.cai_reduce_jobs(arr, len(jobs), _ops._stream())
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / args.iters
        total_b += nbytes
        print(f"{args.tag:20s} call {k}: {len(jobs):2d} jobs {kinds}  partials {nbytes / 1e6:7.1f} MB  "
              f"{us:7.2f} us  {nbytes / us / 1e6:6.2f} TB/s", flush=True)
        if args.v:       # each job alone
            for j in jobs:
                one = (ReduceJob * 1)(j)
                real.cai_reduce_jobs(one, 1, _ops._stream())
                e0.record()
                for _ in range(args.iters):
                    real.cai_reduce_jobs(one, 1, _ops._stream())
                e1.record()
                torch.cuda.synchronize()
                u1 = e0.elapsed_time(e1) * 1e3 / args.iters
                print(f"      {KIND.get(j.kind):5s} blocks {j.nblocks:5d} i={list(j.i)[:8]}  {job_bytes(j) / 1e6:6.1f} MB "
                      f"{u1:7.2f} us  {job_bytes(j) / u1 / 1e6:5.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
