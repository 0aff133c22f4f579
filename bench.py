#!/usr/bin/env python3
"""Headline benchmark: 256x256 patches/s of one RD-loss training step.

Workload (BASELINE.json configs[1]): bmshj2018-hyperprior (ScaleHyperprior,
quality 1 -> N=128, M=192), bf16 autocast, 16 synthetic U[0,1) 256x256 RGB
patches per GPU, one step = forward + RD loss + backward + clip_grad_norm(1.0)
+ Adam (main) + aux-loss backward + Adam (aux), i.e. examples/train.py:155-186.
Inputs live in HBM before the timed region; the whole step is replayed from
HIP graphs.

Multi-GPU: one process per GPU.  `python bench.py --gpus N` starts N rank
processes itself (before anything touches the GPU) with RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_ADDR=127.0.0.1 set; under torchrun the ranks come from its
environment.  Per-patch data parallelism with one RCCL all-reduce (average) of
the flat gradient per step; each rank seeds its training noise differently;
per-GPU batch is fixed (weak scaling) and `value` is the whole-job rate over
the max-over-ranks time.

Also reported (rank 0):
  roofline      -- the step's dominant launch (the instrumented call with the
                   largest GPU time in a profiled step, compressai/_ledger.py),
                   replayed alone and timed with HIP events on the stream it
                   runs on: algorithmic FLOPs (or bytes) / average launch time
                   vs the bf16 dense MFMA peak (or HBM peak); `traffic` from the
                   committed rocprofv3 PMC passes for that launch, if any;
  step_roofline -- SURVEY.md §8(d): roofline seconds per step = sum over the
                   step's launches of max(FLOP/P_mfma, bytes/BW_hbm), divided by
                   the measured seconds per step;
  cpu_baseline  -- the CPU oracle (op-for-op restatement of the reference path,
                   fp32) timed on this host on a bounded sample at the same
                   per-step batch: all available cores, plus one thread
                   (rank 0, N=1).
"""
import argparse
import ctypes
import json
import math
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "165-learning-based-multi-modality-image-and-video-compression_amd")
for _p in (PKG, os.path.join(ROOT, "oracle")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
MM_IR = (512, 640)          # FLIR IR frame (ResearchReport.pdf 4.2; image_rgbt_rgb.py:133-141)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=None, help="patches (pairs) per GPU; default 16 (2 for multimodal)")
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--model", default="bmshj2018-hyperprior",
                    help="a zoo name, or 'multimodal' (BASELINE configs[4]: Master_compresser on IR 512x640 "
                         "guided by Guided_compresser on RGB 1024x1280, train.py:208-274)")
    ap.add_argument("--quality", type=int, default=1)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--dist-backend", default=None, help="torch.distributed backend (default: nccl = RCCL)")
    ap.add_argument("--same-device", action="store_true",
                    help="rehearsal on a 1-GPU box: every rank on cuda:0 (needs --dist-backend gloo)")
    ap.add_argument("--serial-allreduce", action="store_true",
                    help="N > 1: one all-reduce after the backward instead of the two overlapped buckets")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="bounded CPU-baseline sample (0 = skip)")
    ap.add_argument("--cpu-batch", type=int, default=None, help="CPU baseline batch (default: the GPU per-step batch)")
    ap.add_argument("--no-profile", action="store_true", help="skip the profiled step (no roofline fields)")
    ap.add_argument("--keep-grads", action="store_true",
                    help="A/B: optimizers without zero_grad_in_step (zero_grad() fills the gradient buffers)")
    ap.add_argument("--ops-json", default=None, help="write the profiled step's per-launch table here")
    ap.add_argument("--roofline-only", action="store_true",
                    help="profile one step, then replay only its dominant launch --steps times "
                         "(for rocprofv3 --pmc passes)")
    ap.add_argument("--two-graphs", action="store_true",
                    help="one rank: capture the step as two graphs (forward+backward, then clip+Adam+aux) like N > 1 "
                         "(A/B of the single-graph step)")
    ap.add_argument("--replay", default=None,
                    help="with --roofline-only: replay this launch instead of the dominant one "
                         "('kind:index' of the ops table, e.g. conv_wgrad:3)")
    return ap.parse_args()


# --------------------------------------------------------------------------------------------------------
# launcher: N rank processes, started before anything touches the GPU
# --------------------------------------------------------------------------------------------------------

def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int) -> int:
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    for p in procs:
        c = p.wait()
        if c and not rc:
            rc = c
    return rc


# --------------------------------------------------------------------------------------------------------
# measurement helpers
# --------------------------------------------------------------------------------------------------------

def host_cores() -> int:
    """CPUs this process may use: affinity mask, capped by a cgroup v2 CPU quota when one is set."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) / int(period))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def profile_step(step_fn):
    """One step under the ledger with the GPU queue pre-filled (a sleep kernel holds the stream while the host
    enqueues the whole step), so each launch's event pair brackets GPU time only."""
    import torch

    from compressai import _ledger

    torch.cuda.synchronize()
    torch.cuda._sleep(int(1e9))        # ~0.4 s of GPU spin: the host runs ahead of the device
    with _ledger.recording() as led:
        step_fn()
    led.finish()
    return led


def replay_time(entry, reps: int) -> float:
    """Average ms of one launch, replayed alone `reps` times between two HIP events on the current stream."""
    import torch

    for _ in range(3):
        entry.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        entry.replay()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def lib_build() -> str:
    """sha256 prefix of the libcai.so this process runs: PMC records are only valid for the build they measured."""
    import hashlib

    from compressai._native import LIB_PATH

    with open(LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def pmc_traffic(workload: str, kernel: str, shape: str):
    """(HBM bytes per launch, note) from the committed rocprofv3 PMC passes (profiles/pmc_traffic.json, written by
    tools/pmc_traffic.sh + tools/pmc_traffic_update.py: 2 x FETCH_SIZE + WRITE_SIZE, MI355X_MICROARCH.md 'HBM').
    A record counts only for the libcai.so build it measured (its lib_sha256): bytes None when no record of this
    exact launch and build is committed."""
    try:
        recs = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))
    except (OSError, ValueError):
        return None, "no PMC record committed"
    if isinstance(recs, dict):
        recs = [recs]
    build = lib_build()
    stale = None
    for r in recs:
        if r.get("workload") == workload and r.get("kernel") == kernel and r.get("shape") == shape:
            if r.get("lib_sha256") == build:
                return r.get("hbm_bytes_per_launch"), f"rocprofv3 FETCH/WRITE passes of this launch, build {build}"
            stale = r.get("lib_sha256")
    if stale is not None or any(r.get("kernel") == kernel for r in recs):
        return None, f"PMC record of this launch is for another build ({stale}); this build {build}: re-measure"
    return None, "no PMC record of this launch"


def dominant_roofline(led, workload: str, reps: int = 20, pick=None):
    from compressai import _ledger

    ents = led.entries
    if pick is not None:
        kind, idx = pick.split(":")
        e = [x for x in ents if x.kind == kind][int(idx)]
        ms = replay_time(e, reps)
    else:
        # the single profiled step's per-launch times are noisy for short launches (a 15 us kernel can read 80 us
        # once): the three longest launches are re-timed by replay and the longest replay is the dominant launch
        cands = sorted(ents, key=lambda x: -x.ms)[:3]
        timed = [(replay_time(c, reps), i, c) for i, c in enumerate(cands)]
        ms, _, e = max(timed, key=lambda t: (t[0], -t[1]))
    bound = e.bound()
    if bound == "mfma":
        achieved, peak, unit = e.flops / (ms * 1e9), e.peak_tflops(), "TFLOP/s"
    else:
        achieved, peak, unit = e.nbytes / (ms * 1e6), _ledger.HBM_PEAK_GBS, "GB/s"
    # the replayed op's kernels as rocprofv3 lists them: weight gradients through the pixel-split kernels end
    # with their fixed-order slab reduce (reduce_jobs_kernel: compare the rocprof averages summed over both)
    kernels = [e.kernel]
    if e.kind == "conv_wgrad" and e.kernel.startswith(("wgrad_halo", "wgrad_glds")):
        kernels.append("reduce_jobs_kernel")
    traffic, tnote = pmc_traffic(workload, e.kernel, e.shape)
    return {"kernel": e.kernel, "op_kernels": kernels, "launch": f"{e.kind}: {e.shape}", "bound": bound,
            "achieved": round(achieved, 2),
            "peak": peak, "unit": unit, "frac": round(achieved / peak, 4),
            "traffic": traffic, "traffic_note": tnote, "lib_sha256": lib_build(),
            "avg_launch_ms": round(ms, 5), "in_step_ms": round(e.ms, 5),
            "algorithmic_flop_per_launch": e.flops, "algorithmic_bytes_per_launch": e.nbytes,
            "timing": f"HIP events on the launch's stream, {reps} back-to-back replays"}


def step_roofline(led, ms_per_step: float):
    rl = sum(e.roofline_ms() for e in led.entries)
    busy = sum(e.ms for e in led.entries)
    flops = sum(e.flops for e in led.entries)
    nbytes = sum(e.nbytes for e in led.entries)
    return {"roofline_ms_per_step": round(rl, 4), "measured_ms_per_step": round(ms_per_step, 4),
            "frac": round(rl / ms_per_step, 4), "launches_instrumented": len(led.entries),
            "instrumented_gpu_ms": round(busy, 4), "flop_per_step": flops, "bytes_per_step": nbytes,
            "achieved_tflops": round(flops / (ms_per_step * 1e9), 2),
            "note": "sum over the step's launches of max(FLOP/2.5 PF/s bf16 | 157 TF/s fp32, bytes/8 TB/s) "
                    "(SURVEY.md 8(d)); algorithmic FLOPs / bytes per launch from compressai/_ledger.py"}


def dominant_class(led):
    """The kernel class with the largest summed GPU time in the profiled step (all launches of one kernel
    name), with its summed algorithmic work and roofline fraction: for launch-bound configs (cheng2020, 467
    small convs) the time goes to a class of short launches, not to the single longest one."""
    by = {}
    for e in led.entries:
        k = by.setdefault(e.kernel, {"kernel": e.kernel, "launches": 0, "ms": 0.0, "roofline_ms": 0.0, "flops": 0.0,
                                     "bytes": 0.0})
        k["launches"] += 1
        k["ms"] += e.ms
        k["roofline_ms"] += e.roofline_ms()
        k["flops"] += e.flops
        k["bytes"] += e.nbytes
    top = max(by.values(), key=lambda k: k["ms"])
    total = sum(k["ms"] for k in by.values())
    return {"kernel": top["kernel"], "launches": top["launches"], "ms_per_step": round(top["ms"], 4),
            "share_of_instrumented": round(top["ms"] / total, 4), "frac": round(top["roofline_ms"] / top["ms"], 4),
            "achieved_tflops": round(top["flops"] / (top["ms"] * 1e9), 2),
            "achieved_gbs": round(top["bytes"] / (top["ms"] * 1e6), 1),
            "note": "frac = sum of max(FLOP/peak, bytes/BW) over the class's launches / their summed measured time"}


def ops_table(led):
    rows = [e.as_dict() for e in led.entries]
    by_kernel = {}
    for r in rows:
        k = by_kernel.setdefault(r["kernel"], {"kernel": r["kernel"], "launches": 0, "ms": 0.0, "flops": 0.0,
                                               "bytes": 0.0, "roofline_ms": 0.0})
        k["launches"] += 1
        k["ms"] += r["ms"]
        k["flops"] += r["flops"]
        k["bytes"] += r["bytes"]
        k["roofline_ms"] += r["roofline_ms"]
    kernels = sorted(by_kernel.values(), key=lambda k: -k["ms"])
    return {"launches": rows, "by_kernel": kernels}


def cpu_baseline(model_name, quality, batch, size, seconds):
    import torch

    import cai_oracle as O

    cores = host_cores()

    def run(threads, min_steps, budget):
        torch.set_num_threads(threads)
        torch.manual_seed(0)
        net = O.build(model_name, quality)
        opt, aux_opt = O.configure_optimizers(net)
        crit = O.RateDistortionLoss(quality)
        x = torch.rand(batch, 3, size, size, generator=torch.Generator().manual_seed(0))
        xw = x[: min(2, batch)]
        O.train_step(net, crit, xw, opt, aux_opt)           # warm-up (small batch)
        n, t0 = 0, time.perf_counter()
        while True:
            O.train_step(net, crit, x, opt, aux_opt)
            n += 1
            dt = time.perf_counter() - t0
            if n >= min_steps and (dt >= budget or n >= 50):
                break
        return n, dt

    n, dt = run(cores, 1, seconds)
    n1, dt1 = run(1, 1, 0.0)
    torch.set_num_threads(cores)
    return {"value": round(n * batch / dt, 4), "unit": "patches/s", "cores": cores, "kind": "port",
            "host_cpus": os.cpu_count(), "value_1thread": round(n1 * batch / dt1, 4),
            "sample": f"oracle {model_name} q{quality} fp32 train step (fwd+bwd+clip+Adam+aux), batch {batch} "
                      f"@ {size}x{size} (same per-step batch as the GPU), {n} timed steps after a batch-2 warm-up "
                      f"on {cores} threads (the CPUs this process may use: affinity / cgroup quota; "
                      f"os.cpu_count()={os.cpu_count()}); value_1thread: {n1} step(s) on 1 thread "
                      f"(the reference eval scripts' torch.set_num_threads(1), __main__t.py:61)"}


# --------------------------------------------------------------------------------------------------------
# the benchmark
# --------------------------------------------------------------------------------------------------------

def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    if args.batch is None:
        args.batch = 2 if args.model == "multimodal" else 16

    import torch
    import torch.distributed as dist

    from compressai.distributed import OverlappedAllReduce, allreduce_mean_, broadcast_parameters_, init_from_env
    from compressai._ops import loss_seed
    from compressai.losses import RateDistortionLoss
    from compressai.optim import configure_optimizers
    from compressai.zoo import image_models

    rank, world = init_from_env(backend=args.dist_backend)
    if world != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but the job has {world} ranks")
    local = 0 if args.same_device else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    torch.manual_seed(0)                     # identical initial weights (rank 0's are broadcast anyway)
    multimodal = args.model == "multimodal"
    gen = torch.Generator().manual_seed(1234 + rank)
    if multimodal:
        # train.py:208-246 / 379-382: IR master (channel 1, 512x640) guided by RGB (1024x1280);
        # the Guided codec runs under no_grad in training mode, in fp32 like the reference
        from compressai.models import Guided_compresser, Master_compresser

        H, W = MM_IR
        net = Master_compresser(width=H, height=W, channel=1).to(dev).train()
        net_g = Guided_compresser(channel=3).to(dev).train()
        broadcast_parameters_(net_g)
        x = torch.rand(args.batch, 1, H, W, generator=gen).to(dev)
        guide = torch.rand(args.batch, 3, 2 * H, 2 * W, generator=gen).to(dev)
    else:
        net = image_models[args.model](args.quality).to(dev).train()
        x = torch.rand(args.batch, 3, args.size, args.size, generator=gen).to(dev)
    broadcast_parameters_(net)
    torch.cuda.manual_seed(1000 + rank)      # per-rank training noise
    # N > 1: the gradient exchange in buckets, each all-reduced while the backward below it runs
    # (compressai.distributed.OverlappedAllReduce over the model's phase plan, CompressionModel.dp_phases():
    # g_s in pieces, the entropy path, then g_a in pieces for the zoo models)
    overlap = world > 1 and not args.serial_allreduce
    # the reference loop order (zero_grad, forward, backward, step): the Adam kernels consume the gradients
    # and zero_grad() launches nothing (FusedAdam zero_grad_in_step)
    opt, aux_opt = configure_optimizers(net, zero_grad_in_step=not args.keep_grads,
                                        phases=net.dp_phases() if overlap else None)
    sync = OverlappedAllReduce.for_model(net, opt) if overlap else None
    criterion = RateDistortionLoss(args.quality)
    state = {}

    def fwd(two_phase=False):
        opt.zero_grad()
        aux_opt.zero_grad()
        if multimodal:
            with torch.no_grad():
                hidden = net_g(guide)["hidden"]
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = net(x, guide, hidden) if multimodal else net(x)
            crit = criterion(out, x)
        state["loss"] = crit["loss"].detach()
        if two_phase:
            sync.backward_head(crit["loss"])    # phase 0 (the synthesis' outermost piece): bucket 0 is final
        else:
            crit["loss"].backward(loss_seed(crit["loss"]))   # a persistent 1.0 seed: no fill launch

    def fwd_bwd():
        fwd()

    def opt_part():
        opt.step(max_norm=1.0)
        aux = net.aux_loss()
        aux.backward(loss_seed(aux))
        aux_opt.step()

    def local_step():
        fwd_bwd()
        opt_part()

    def eager_step():
        if sync is None:
            fwd_bwd()
            allreduce_mean_(opt.flat_grad)
        else:
            fwd(two_phase=True)
            sync.reduce_head()      # side stream, overlapped with the next phase
            sync.backward_tail()
            sync.finish()
        opt_part()

    if multimodal:
        workload = ("multimodal paired codec: Master_compresser(IR 1x%dx%d) + Guided_compresser(RGB 3x%dx%d, "
                    "no_grad fp32) RD-loss training step (fwd+bwd+clip+Adam+aux), HIP-graph replay"
                    % (MM_IR[0], MM_IR[1], 2 * MM_IR[0], 2 * MM_IR[1]))
    else:
        workload = (f"{args.model} q{args.quality} B={args.batch} {args.size}x{args.size} RD-loss training step "
                    f"(fwd+bwd+clip+Adam+aux), HIP-graph replay")

    if args.roofline_only:
        for _ in range(2):
            local_step()
        led = profile_step(local_step)
        if rank == 0:
            print(json.dumps(dict(dominant_roofline(led, workload, reps=args.steps, pick=args.replay),
                                  workload=workload)), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return

    step = eager_step
    if not args.no_graph:
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(3):
                eager_step()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        gA, gB = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        # one rank: the whole step is ONE graph (the gap between two graph launches -- the backward's last reduce to
        # the clip's first kernel -- measured 8.7 us per C2 step); N > 1 needs the exchange between the two
        single = sync is None and world == 1 and not args.two_graphs
        if single:
            with torch.cuda.graph(gA):
                fwd_bwd()
                opt_part()
        elif sync is None:
            with torch.cuda.graph(gA):
                fwd_bwd()
        else:
            gT = [torch.cuda.CUDAGraph() for _ in range(1, sync.nphases)]   # the tail's backward phases
            with torch.cuda.graph(gA):
                fwd(two_phase=True)
            for i, g in enumerate(gT, 1):
                with torch.cuda.graph(g, pool=gA.pool()):
                    sync.backward_phase(i)
        if not single:
            with torch.cuda.graph(gB, pool=gA.pool()):
                opt_part()

        def step():
            gA.replay()
            if single:
                return
            if sync is None:
                allreduce_mean_(opt.flat_grad)
            else:
                for i, g in enumerate(gT, 1):
                    sync.reduce_bucket(i - 1)       # side stream, overlapped with phase i on the compute stream
                    g.replay()
                sync.finish()
            gB.replay()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    dt = dt.item()
    loss = float(state["loss"].item())
    if not math.isfinite(loss):
        raise RuntimeError(f"non-finite loss {loss}")
    ms_per_step = dt / args.steps * 1e3
    peak_gb = torch.cuda.max_memory_allocated(dev) / 1e9   # the timed steps' (and their graphs') peak

    roof = step_roof = dom_class = None
    if rank == 0 and not args.no_profile:
        led = profile_step(local_step)
        roof = dominant_roofline(led, workload)
        step_roof = step_roofline(led, ms_per_step)
        dom_class = dominant_class(led)
        if args.ops_json:
            with open(args.ops_json, "w") as f:
                json.dump(ops_table(led), f, indent=1)
    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0 and not multimodal:
        cpu = cpu_baseline(args.model, args.quality, args.cpu_batch or args.batch, args.size, args.cpu_seconds)
    if rank == 0:
        value = world * args.batch * args.steps / dt
        unit = "IR+RGB pairs/s" if multimodal else "patches/s"
        line = {
            "metric": METRIC, "value": round(value, 3), "unit": unit, "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
            "data": ("synthetic U[0,1) IR/RGB frame pairs, random-init weights" if multimodal else
                     "synthetic U[0,1) 256x256 RGB patches, random-init weights"),
            "config": {"workload": workload,
                       "model": args.model, "quality": args.quality, "global_batch": args.batch * world,
                       "per_gpu_batch": args.batch, "seq_len": None,
                       "patch": list(MM_IR) if multimodal else args.size, "parallelism": f"dp{world}",
                       "grad_exchange": (f"{sync.nphases}-bucket all-reduce in backward order (MB: "
                                         f"{' / '.join(f'{4 * b.numel() / 1e6:.1f}' for b in sync.buckets)}), "
                                         f"bucket i overlapped with backward phase i+1; exposed: the last" if sync else
                                         "1 all-reduce after backward") if world > 1 else None},
            "final_loss": round(loss, 5), "max_memory_allocated_gb": round(peak_gb, 3),
            "roofline": roof, "dominant_class": dom_class, "step_roofline": step_roof, "cpu_baseline": cpu,
        }
        if cpu:
            line["gpu_over_cpu"] = round(value / cpu["value"], 1)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
