"""Benchmark: MobileNetV2UNet fwd+bwd+Adam training throughput on MI355X.

Workload (BASELINE.json configs[1], the metric's config): MobileNetV2UNet,
10 classes, 256x512, batch 32 per GPU, fp32, synthetic device-resident
inputs (x ~ N(0,1), int64 labels), deterministic random-init weights (no
pretrained checkpoint offline).  One step = zero_grad + forward + fused
upsample/cross-entropy loss + backward (+ RCCL gradient all-reduce when N > 1)
+ torch.optim.Adam(lr=1.5e-4) step -- the reference loop of src/train.py:35-39.

    python bench.py [--gpus N] [--steps K] [--warmup W]
N > 1 runs under torch.distributed.run (one process per GPU, RCCL), per-GPU
batch fixed (weak scaling); value = all images / max-over-ranks time.

Also reported:
  roofline      -- the dense 3x3 conv family (forward + data gradient), timed with
                   HIP events around those launches inside the timed region:
                   achieved = their algorithmic FLOPs (f32, vs the f32 MFMA peak) or
                   bytes (bf16io, vs HBM) / their summed launch durations.
  step_roofline -- the whole step against SURVEY 8(d)'s algorithmic work per image.
  cpu_baseline  -- the CPU oracle (oracle/segref.py, torch-CPU restatement of
                   the reference) on a bounded sample, rank 0 at N = 1 only.
  bf16io        -- (default f32 run) the same workload in BASELINE configs[2]'s
                   arithmetic (bf16 MFMA operands + bf16 activation storage): its own
                   warm-up and timed region after the headline's, with its own
                   ms_per_step, HBM roofline and step roofline (--no-bf16io-block).
  infer         -- (default run, N = 1) BASELINE configs[3]: inference.py's per-frame
                   path as one hipGraph replay, fp16, 500 timed frames (--no-infer-block).
  unet_cfg5     -- (default run) BASELINE configs[4]: UNet 10-class 512x1024 bs=8/GPU, bf16io
                   and f32, each with its own warm-up, timed region, roofline and step
                   roofline (--no-unet-block).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "team02-objectdetection_amd")
for _p in (PKG, REPO):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402

F32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 matrix (= vector) peak, spec
BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: BF16 MFMA ~2.5 PF dense (no sparsity)
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--height", type=int, default=256)
    ap.add_argument("--width", type=int, default=512)
    ap.add_argument("--classes", type=int, default=10)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-timer", action="store_true", help="skip the per-launch HIP-event roofline timing")
    ap.add_argument("--no-infer-block", action="store_true",
                    help="skip the nested \"infer\" measurement (configs[3], 500 graph-replayed frames) of the default line")
    ap.add_argument("--no-bf16io-block", action="store_true",
                    help="skip the nested \"bf16io\" measurement (configs[2] math on the same workload) that follows "
                         "the f32 headline")
    ap.add_argument("--no-unet-block", action="store_true",
                    help="skip the nested \"unet_cfg5\" measurement (BASELINE configs[4]: UNet 10-class 512x1024 "
                         "bs=8/GPU, bf16io and f32) of the default line")
    ap.add_argument("--no-dp1-block", action="store_true",
                    help="skip the nested world-1 RCCL DataParallel overhead block (multi_gpu.world1_rccl) of the "
                         "default line")
    ap.add_argument("--workload", choices=("train", "infer"), default="train",
                    help="train: BASELINE configs[1] (the headline); infer: configs[3], inference.py's per-frame path")
    ap.add_argument("--frames", type=int, default=500, help="timed frames of --workload infer")
    ap.add_argument("--math", choices=("f32", "bf16", "bf16io", "f16"), default=None,
                    help="conv arithmetic. train: f32 = configs[1] (default, the headline); bf16 = the bf16 "
                         "configurations (configs[2]/[4]): bf16 MFMA operands, fp32 accumulation / activations / BN "
                         "/ Adam; bf16io = bf16 math + bf16 activation/gradient storage.  infer: f16 = configs[3] "
                         "(default), f32, bf16")
    ap.add_argument("--optimizer", choices=("seg", "torch"), default="seg",
                    help="seg: seg_amd.Adam (one-launch HIP step, csrc/adam.hip); torch: torch.optim.Adam (foreach)")
    ap.add_argument("--dist-backend", choices=("nccl", "gloo"), default="nccl",
                    help="nccl = RCCL over xGMI (the measurement); gloo = rehearsal of the N-rank path on fewer GPUs "
                         "(ranks share devices round-robin; not a throughput figure)")
    ap.add_argument("--model", choices=("MobileNetV2UNet", "UNet"), default="MobileNetV2UNet",
                    help="UNet = BASELINE configs[4] shape family (use --height 512 --width 1024 --batch 8)")
    return ap.parse_args()


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_baseline(args):
    """The oracle (torch CPU, all host cores) on a bounded sample of the same workload."""
    from oracle import segref
    import seg_amd
    from seg_amd import deterministic_init, synthetic_batch
    threads = os.cpu_count() or 1
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else threads
    threads = min(threads, aff, int(os.environ.get("OMP_NUM_THREADS", aff)))
    torch.set_num_threads(threads)
    model = deterministic_init(getattr(seg_amd, args.model)(args.classes), seed=0)
    p = segref.canonical_state(model.state_dict())
    bs = 4 if args.model == "MobileNetV2UNet" else 1
    x, y = synthetic_batch(bs, args.height, args.width, args.classes, seed=1)
    segref.adam_steps(args.model, p, [(x, y)])  # warm-up step
    t0 = time.perf_counter()
    steps = 0
    while True:
        segref.adam_steps(args.model, p, [(x, y)])
        steps += 1
        if time.perf_counter() - t0 > args.cpu_seconds:
            break
    dt = time.perf_counter() - t0
    return {"value": round(steps * bs / dt, 3), "unit": "images/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(),
            "sample": f"oracle/segref.py {args.model} fwd+bwd+Adam, bs={bs}, {args.height}x{args.width}, "
                      f"{steps} timed steps ({dt:.1f} s) after 1 warm-up, torch CPU fp32"}


def infer_measure(args, math, frames, cpu_baseline=True):
    """configs[3]: inference.py's per-frame path (preprocess_image -> model.eval() forward ->
    argmax + INTER_NEAREST mask) for a 720x1280 uint8 BGR frame resized to 128x256, bs=1,
    replayed as one HIP graph.  Returns per-frame latencies (graph / eager / graph with the
    H2D frame copy) and the CPU path's frames/s."""
    import numpy as np
    from seg_amd import MobileNetV2UNet, deterministic_init
    from seg_amd.infer import Predictor
    dev = torch.device("cuda", torch.cuda.current_device())
    model = deterministic_init(MobileNetV2UNet(args.classes), seed=0, random_running_stats=True).to(dev).eval()
    g = np.random.Generator(np.random.PCG64(0))
    frame = g.integers(0, 256, (720, 1280, 3), dtype=np.uint8)
    res = {}
    for mode in ("graph", "eager", "graph_h2d"):
        pred = Predictor(model, frame_hw=(720, 1280), graph=mode != "eager", math=math)
        pred.set_frame(frame)
        fn = (lambda: pred(frame)) if mode == "graph_h2d" else pred.step
        for _ in range(max(args.warmup, 3)):
            fn()
        torch.cuda.synchronize()
        n = frames if mode != "graph_h2d" else max(frames // 5, 20)
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        res[mode] = (time.perf_counter() - t0) / n
    cpu = None
    if cpu_baseline:
        from oracle import cvresize, segref
        threads = min(os.cpu_count() or 1, len(os.sched_getaffinity(0)))
        threads = min(threads, int(os.environ.get("OMP_NUM_THREADS", threads)))
        torch.set_num_threads(threads)
        p = segref.canonical_state(model.state_dict())
        def one():
            x, _ = cvresize.preprocess_image(frame)
            with torch.no_grad():
                lo = segref.mobilenet_unet_forward(p, torch.from_numpy(x), False)
            return cvresize.class_mask(lo.numpy(), (720, 1280))
        one()
        t0, k = time.perf_counter(), 0
        while time.perf_counter() - t0 < args.cpu_seconds:
            one()
            k += 1
        dt = time.perf_counter() - t0
        cpu = {"value": round(k / dt, 2), "unit": "frames/s", "cores": threads, "kind": "port", "cpu_model": cpu_model(),
               "sample": f"oracle cvresize.preprocess_image + segref eval forward (torch CPU fp32) + class_mask, "
                         f"{k} frames in {dt:.1f} s"}
    return {"value": round(1.0 / res["graph"], 1), "unit": "frames/s", "ms_per_frame": round(res["graph"] * 1e3, 4),
            "latency_ms": {"graph": round(res["graph"] * 1e3, 4), "eager": round(res["eager"] * 1e3, 4),
                           "graph_with_h2d_frame_copy": round(res["graph_h2d"] * 1e3, 4)},
            "frames": frames, "cpu_baseline": cpu}


INFER_MATH = {"f32": "fp32 everywhere", "f16": "folded conv operands fp16 (RNE) on the f16 MFMA, fp32 "
              "accumulation; depthwise, preprocess and argmax in fp32",
              "bf16": "folded conv operands bf16 on the bf16 MFMA, fp32 accumulation"}
INFER_WORKLOAD = ("inference.py per-frame path: cv2-style resize + normalise, BN-folded eval forward, argmax + "
                  "nearest mask, one hipGraph replay per frame")


def bench_infer(args):
    """configs[3] as the headline (--workload infer).  value = frames/s with the frame already in HBM."""
    torch.cuda.set_device(0)
    r = infer_measure(args, args.math, args.frames, not args.no_cpu_baseline)
    line = {"metric": "frames/sec inference MobileNetV2UNet 720x1280 frame -> 128x256, bs=1 (BASELINE configs[3])",
            "value": r["value"], "unit": "frames/s", "n_gpus": 1, "steps": args.frames,
            "warmup": args.warmup, "ms_per_step": r["ms_per_frame"], "higher_is_better": True,
            "scaling": "none", "vs_baseline": None, "dtype": args.math, "data": "synthetic",
            "math": INFER_MATH[args.math],
            "config": {"workload": INFER_WORKLOAD, "model": "MobileNetV2UNet", "global_batch": 1, "frame": [720, 1280],
                       "image": [128, 256], "parallelism": "none"},
            "latency_ms": r["latency_ms"], "roofline": None, "cpu_baseline": r["cpu_baseline"]}
    print(json.dumps(line), flush=True)


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launcher_command(argv, gpus: int, port: int):
    """The child command `bench.py --gpus N` (N > 1, no WORLD_SIZE in the environment)
    runs: one process per GPU under torch.distributed.run, the driver's own form."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *argv]


def check_world(world: int, gpus: int):
    """Every rank must see the world size it was asked for (--gpus)."""
    if world != gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {gpus}; launch with "
                         f"torch.distributed.run --nproc-per-node {gpus} or drop WORLD_SIZE")


def main():
    args = parse()
    if args.math is None:
        args.math = "f16" if args.workload == "infer" else "f32"
    if args.workload == "infer" and args.math == "bf16io":
        raise SystemExit("--math bf16io is a training configuration")
    if args.workload == "train" and args.math == "f16":
        raise SystemExit("--math f16 is the inference configuration (--workload infer)")
    if args.workload == "infer":
        return bench_infer(args)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # `python bench.py --gpus N`: start the N ranks as a CHILD process (nothing has touched
        # the GPU in this process; never exec) and forward its exit code
        import subprocess
        rc = subprocess.call(launcher_command(sys.argv[1:], args.gpus, _free_port()))
        sys.exit(rc)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    check_world(world, args.gpus)
    dist = world > 1
    if args.dist_backend == "gloo":
        local = local % torch.cuda.device_count()
    # bind the rank's GPU before the process group exists, so RCCL's communicators (and the
    # barriers below) are created on this rank's device, never on device 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if dist:
        if args.dist_backend == "nccl":
            torch.distributed.init_process_group(args.dist_backend, device_id=dev)
        else:
            torch.distributed.init_process_group(args.dist_backend)
        assert torch.distributed.get_world_size() == args.gpus

    head = train_workload(args, args.math, dev, world, rank, dist)
    nested = None
    default_line = args.math == "f32" and args.model == "MobileNetV2UNet"
    if default_line and not args.no_bf16io_block:
        # BASELINE configs[2]'s arithmetic on the same workload (the north-star HBM target):
        # its own model, warm-up and timed region after the headline's
        nested = train_workload(args, "bf16io", dev, world, rank, dist)
    unet = None
    if default_line and not args.no_unet_block:
        # BASELINE configs[4]: UNet 10-class, 512x1024, bs=8/GPU -- bf16 (bf16io storage) as the config
        # names it, and f32 beside it; each its own model, warm-up and timed region
        ua = argparse.Namespace(**vars(args))
        ua.model, ua.batch, ua.height, ua.width = "UNet", 8, 512, 1024
        ua.steps, ua.warmup = min(args.steps, 10), max(min(args.warmup, 3), 2)
        unet = {}
        for m in ("bf16io", "f32"):
            r = train_workload(ua, m, dev, world, rank, dist)
            unet[m] = {"value": r["value"], "unit": "images/s", "ms_per_step": r["ms_per_step"],
                       "steps": ua.steps, "warmup": ua.warmup, "final_loss": r["final_loss"],
                       "math": MATH_NOTE[m], "roofline": r["roofline"], "bn_bwd_roofline": r["bn_bwd_roofline"],
                       "step_roofline": r["step_roofline"],
                       **({"multi_gpu": r["multi_gpu"]} if r["multi_gpu"] is not None else {})}

    dp1 = None
    if default_line and world == 1 and not args.no_dp1_block:
        # the DataParallel host path at world size 1 over RCCL against the plain model, interleaved (VERDICT r5
        # item 7: what the bucket machinery -- tape stops, all-reduce launches, BN-buffer broadcast -- costs a step
        # when no 8-GPU node is at hand)
        dp1 = {m: dp_world1(args, m, dev) for m in ("f32", "bf16io")}
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(args)
        line = {"metric": f"images/sec fwd+bwd {args.model} {args.height}x{args.width} bs={args.batch}/GPU",
                "value": head["value"], "unit": "images/s", "n_gpus": world, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": head["ms_per_step"], "higher_is_better": True,
                "scaling": "weak", "vs_baseline": None, "dtype": args.math, "data": "synthetic",
                "config": {"workload": f"{args.model} {args.classes}-class fwd+bwd+Adam, "
                                       f"{args.height}x{args.width}, bs={args.batch}/GPU ({_cfg_name(args, args.math)})",
                           "model": args.model, "global_batch": args.batch * world,
                           "image": [args.height, args.width], "parallelism": f"dp{world}",
                           "collectives": "RCCL (torch.distributed nccl)" if args.dist_backend == "nccl" else
                                          "gloo REHEARSAL (ranks share GPUs; not a throughput figure)",
                           "optimizer": {"seg": "seg_amd.Adam (HIP, one launch)", "torch": "torch.optim.Adam (foreach)"}[args.optimizer]},
                "final_loss": head["final_loss"], "math": MATH_NOTE[args.math],
                "roofline": head["roofline"], "bn_bwd_roofline": head["bn_bwd_roofline"],
                "step_roofline": head["step_roofline"], "cpu_baseline": cpu}
        if head["multi_gpu"] is not None:
            line["multi_gpu"] = head["multi_gpu"]
        if nested is not None:
            line["bf16io"] = {"workload": f"same model, shape and step as the headline with bf16io math "
                                          f"({_cfg_name(args, 'bf16io')})", "dtype": "bf16io",
                              "math": MATH_NOTE["bf16io"], **nested}
        if unet is not None:
            line["unet_cfg5"] = {"workload": "BASELINE configs[4]: UNet 10-class fwd+bwd+Adam, 512x1024, "
                                             f"bs=8/GPU, dp{world} (bf16 = bf16io math; f32 beside it)",
                                 "model": "UNet", "global_batch": 8 * world, "image": [512, 1024],
                                 "scaling": "weak", **unet}
        if dp1 is not None:
            line["multi_gpu"] = {"world1_rccl": dp1}
        if world == 1 and args.model == "MobileNetV2UNet" and not args.no_infer_block:
            # BASELINE configs[3] on the same GPU after the training lines (its own timed loop)
            r = infer_measure(args, "f16", 500, cpu_baseline=False)
            line["infer"] = {"workload": f"BASELINE configs[3]: {INFER_WORKLOAD}", "dtype": "f16",
                             "math": INFER_MATH["f16"], "model": "MobileNetV2UNet", "frame": [720, 1280],
                             "image": [128, 256], **{k: v for k, v in r.items() if k != "cpu_baseline"}}
        print(json.dumps(line), flush=True)
    if dist:
        torch.distributed.destroy_process_group()


def dp_world1(args, math, dev, rounds=3):
    """The DataParallel path (seg_amd/ddp.py) on ONE rank over RCCL against the plain model, same workload, same
    process, interleaved rounds of args.steps timed steps each.  At world size 1 the all-reduces
    move no data between GPUs, so the difference is the bucket machinery itself: the tape's host-callback stops (one
    per gradient bucket, where the host leaves the replay, launches the bucket's all-reduce and resumes), RCCL's
    launches on its stream and the compute stream's waits for them, the BN-buffer broadcast and the copies of the
    averaged buckets handed to autograd.  Reports stops per step, host time per stop and the step-time overhead."""
    import seg_amd
    from seg_amd import Adam, deterministic_init, engine, synthetic_batch, tape
    from seg_amd.ddp import DataParallel
    own = not torch.distributed.is_initialized()
    if own:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ["MASTER_PORT"] = str(_free_port())
        torch.distributed.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    x, y = synthetic_batch(args.batch, args.height, args.width, args.classes, seed=1000)
    x, y = x.to(dev), y.to(dev)
    arms = {}
    for kind in ("plain", "dp"):
        core = deterministic_init(getattr(seg_amd, args.model)(args.classes), seed=0).to(dev).train()
        engine.set_conv_math(core, math)
        m = DataParallel(core) if kind == "dp" else core
        arms[kind] = (core, m, Adam(m.parameters(), lr=1.5e-4))

    def step(kind):
        _, m, opt = arms[kind]
        opt.zero_grad(set_to_none=True)
        m.forward_loss(x, y).backward()
        opt.step()

    for kind in arms:
        for _ in range(max(args.warmup, 2)):
            step(kind)
    ms = {"plain": [], "dp": []}
    stops = host = 0.0
    for _ in range(rounds):
        for kind in ("plain", "dp"):
            torch.cuda.synchronize()
            s0, h0 = tape.STOP_STATS["stops"], tape.STOP_STATS["host_s"]
            t0 = time.perf_counter()
            for _ in range(args.steps):
                step(kind)
            torch.cuda.synchronize()
            ms[kind].append((time.perf_counter() - t0) / args.steps * 1e3)
            if kind == "dp":
                stops += tape.STOP_STATS["stops"] - s0
                host += tape.STOP_STATS["host_s"] - h0
    nb = len(arms["dp"][1]._buckets or [])
    for core, m, opt in arms.values():
        engine.release_plans(core)
    del arms
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    if own:
        torch.distributed.destroy_process_group()
    n = rounds * args.steps
    plain, dp = sorted(ms["plain"])[rounds // 2], sorted(ms["dp"])[rounds // 2]
    return {"math": math, "buckets": nb, "tape_stops_per_step": round(stops / n, 2),
            "host_us_per_stop": round(host / max(stops, 1) * 1e6, 1),
            "host_us_in_stops_per_step": round(host / n * 1e6, 1),
            "ms_per_step_plain": round(plain, 3), "ms_per_step_dp": round(dp, 3),
            "overhead_frac": round(dp / plain - 1.0, 4),
            "rounds_ms": {k: [round(v, 3) for v in vs] for k, vs in ms.items()},
            "note": f"{rounds} interleaved rounds of {args.steps} steps each arm (medians); world size 1 over RCCL "
                    "(torch.distributed nccl): DataParallel = bucketed ncclAvg all-reduces launched at tape stops, "
                    "BN-buffer broadcast, bucket copies to autograd; plain = the same model without it"}


MATH_NOTE = {"f32": "fp32 everywhere",
             "bf16": "conv operands bf16 (RNE) on the bf16 MFMA, fp32 accumulation; activations, "
                     "BatchNorm, depthwise convs, loss and Adam in fp32",
             "bf16io": "conv operands bf16 on the bf16 MFMA, fp32 accumulation; activations and their "
                       "gradients stored bf16 in HBM (fp32 arithmetic inside every kernel); BN "
                       "statistics, parameter gradients, loss and Adam fp32"}


def _cfg_name(args, math):
    if args.model == "MobileNetV2UNet":
        return "BASELINE configs[1]" if math == "f32" else f"BASELINE configs[2] math ({math}) at N GPUs"
    return f"BASELINE configs[4] shape, {math} conv math"


def train_workload(args, math, dev, world, rank, dist):
    """Warm up, then time args.steps training steps of args.model with conv math `math`
    (barrier + synchronize on both sides, max over ranks), then the untimed roofline
    passes.  Returns value / ms_per_step / final_loss / roofline / step_roofline /
    multi_gpu; frees the model's plans afterwards."""
    import seg_amd
    from seg_amd import deterministic_init, synthetic_batch
    from seg_amd import engine
    core = deterministic_init(getattr(seg_amd, args.model)(args.classes), seed=0).to(dev).train()
    engine.set_conv_math(core, math)
    peak = F32_MFMA_PEAK_TFLOPS if math == "f32" else BF16_MFMA_PEAK_TFLOPS
    model = core
    if dist:
        from seg_amd.ddp import DataParallel
        model = DataParallel(core)
    if args.optimizer == "seg":
        from seg_amd import Adam
        opt = Adam(model.parameters(), lr=1.5e-4)
    else:
        opt = torch.optim.Adam(model.parameters(), lr=1.5e-4)
    x, y = synthetic_batch(args.batch, args.height, args.width, args.classes, seed=1000 + rank)
    x, y = x.to(dev), y.to(dev)

    def step():
        opt.zero_grad(set_to_none=True)
        loss = model.forward_loss(x, y)
        loss.backward()
        opt.step()
        return loss

    for _ in range(args.warmup):
        step()
    # live per-launch HIP events on the roofline family only (each event pair is a marker
    # packet on the queue: timing all ~130 conv launches costs ~3 % of the step)
    conv3 = {"igemm3_fwd", "igemm3_dgrad", "wino3_fwd", "wino3_dgrad"}
    timer = None if args.no_timer else engine.KernelTimer(kinds=conv3)
    if dist:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    engine.TIMER = timer
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    if dist:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    engine.TIMER = None
    final_loss = loss.item()
    per_rank = [dt]
    if dist:
        t = torch.zeros(world, device=dev, dtype=torch.float64)
        t[rank] = dt
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.SUM)
        per_rank = t.tolist()
    dt = max(per_rank)
    images = args.batch * args.steps * world
    value = images / dt
    scaling = None
    if dist:
        # same-run reference for the weak-scaling efficiency: the same K steps on every rank
        # with no communication at all (DataParallel.no_sync: no gradient all-reduce; the BN
        # buffer broadcast switched off too), max over ranks.  One untimed step first: the
        # no_sync plan is a different launch tape, recorded (and its buffers allocated) then.
        bcast = model.broadcast_buffers
        model.broadcast_buffers = False
        with model.no_sync():
            step()
            torch.distributed.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                step()
            torch.cuda.synchronize()
            solo = time.perf_counter() - t0
        model.broadcast_buffers = bcast
        t = torch.tensor([solo], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        solo = float(t)
        scaling = {"ranks_seen": world, "ms_per_step_per_rank": [round(v / args.steps * 1e3, 3) for v in per_rank],
                   "ms_per_step_without_communication": round(solo / args.steps * 1e3, 3),
                   "weak_scaling_eff_vs_no_communication": round(solo / dt, 4),
                   "note": "efficiency = same-run step time with no gradient all-reduce and no BN-buffer "
                           "broadcast (after one untimed no_sync step) / the timed step time (the driver "
                           "computes the cross-run N=1 efficiency itself)"}

    roof = bn_roof = None
    if timer is not None:
        roof, bn_roof = _roofline(args, math, model, core, engine, timer, conv3, step, dt, peak)
    step_roof = _step_roofline(args, math, core, engine, value, peak)
    res = {"value": round(value, 2), "ms_per_step": round(dt / args.steps * 1e3, 3),
           "final_loss": round(final_loss, 5), "roofline": roof, "bn_bwd_roofline": bn_roof,
           "step_roofline": step_roof, "multi_gpu": scaling}
    engine.release_plans(core)
    del model, core, opt
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return res


def _roofline(args, math, model, core, engine, timer, conv3, step, dt, peak):
    """The dominant kernel family's roofline: the dense 3x3 conv forward + data gradient,
    timed live inside the timed region (timer), plus the untimed re-timing passes."""
    def family(rec, kinds):
        sel = [(f, s) for k, f, s in rec if k in kinds]
        fl, sec = sum(f for f, _ in sel), sum(s for _, s in sel)
        return fl, sec, len(sel)

    def extra_pass(overlap):
        """3 untimed steps with every conv launch timed (after the timed region)."""
        saved = engine.OVERLAP
        engine.OVERLAP = overlap
        t = engine.KernelTimer()
        engine.TIMER = t
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        engine.TIMER = None
        engine.OVERLAP = saved
        return t.elapsed()

    rec = timer.elapsed()
    flops, secs, n = family(rec, conv3)
    pmc = {}
    wfl, wsec, wn = family(rec, {"wino3_fwd", "wino3_dgrad"})
    achieved = flops / secs / 1e12 if secs > 0 else 0.0
    traffic, traffic_src, mfma_busy = None, None, None
    prof = os.path.join(REPO, "profiles", "latest_roofline.json" if math == "f32" else f"latest_roofline_{math}.json")
    # the committed profile is of the default workload (MobileNetV2UNet bs=32 256x512): attach its
    # PMC figures only to that workload's line
    default_workload = (args.model, args.batch, args.height, args.width) == ("MobileNetV2UNet", 32, 256, 512)
    if os.path.exists(prof) and default_workload:
        with open(prof) as fh:
            rj = json.load(fh)
        c3 = rj["families"].get("conv3", {})
        traffic = c3.get("hbm_bytes_per_op")
        mfma_busy = c3.get("mfma_busy_frac")
        pmc = rj["families"]
        # the PMC figure is not measured in this run: name the profile and commit it came from
        traffic_src = {"file": os.path.relpath(prof, REPO), "profile": rj.get("profile"),
                       "commit": rj.get("commit"),
                       "counters": "rocprofv3 PMC (2*FETCH_SIZE+WRITE_SIZE)*1KiB of the conv3 family per step "
                                   f"/ {c3.get('ops_per_step', 17)} conv ops ({c3.get('calls_per_step')} launches per "
                                   "step, checked against the step's op count by tools/roofline_report.py), separate "
                                   "--pmc passes; SQ_VALU_MFMA_BUSY_CYCLES and GRBM_GUI_ACTIVE in a third pass"}
    # algorithmic bytes of the family: every 3x3 conv's input and output tensors once
    # (fwd: X + Y, dgrad: dY + dX) at the storage element size, averaged over its launches
    prog = engine.get_program(core, args.batch, args.height, args.width)
    sb = 2 if math == "bf16io" else 4
    abytes = []
    for op in prog.ops:
        if isinstance(op, engine.ConvOp) and op.kind == "igemm" and op.ks == 3:
            xy = sb * (op.inp.M * op.cin + op.y.M * op.cout)
            abytes.append(xy)
            if not op.first:
                abytes.append(xy)
    alg_bytes = sum(abytes) / max(len(abytes), 1)
    # the other conv families and the side-stream-free figure: separate untimed passes
    rec_all = extra_pass(engine.OVERLAP)
    wf, ws, wgn = family(rec_all, {"igemm3_wgrad", "wino3_wgrad"})
    af, as_, an = family(rec_all, {k for k, _, _ in rec_all if k.startswith(("igemm", "wino", "halo"))})
    rec_iso = extra_pass(False)
    ifl, isec, inn = family(rec_iso, conv3)
    bn_roof = _bn_roofline(args, math, family, rec_all, rec_iso, dt, pmc, traffic_src)
    # the family is graded against the resource its own arithmetic intensity makes binding:
    # roofline time = max(bytes / HBM, FLOPs / MFMA peak) (the bf16io 3x3 family,
    # ~420 FLOP/B, sits above the bf16 ridge of 2500 / 8 = 312 FLOP/B -- MFMA-bound, not HBM-bound)
    gbs = alg_bytes * n / secs / 1e9 if secs > 0 else 0.0
    ai = (flops / max(n, 1)) / alg_bytes if alg_bytes else 0.0
    ridge = peak * 1e12 / (HBM_PEAK_GBS * 1e9)
    grading = {"arithmetic_intensity_flop_per_byte": round(ai, 1), "ridge_flop_per_byte": round(ridge, 1)}
    if ai >= ridge:
        bound = {"bound": "mfma", "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
                 "frac": round(achieved / peak, 4), "hbm_gbs": round(gbs, 1),
                 "hbm_frac": round(gbs / HBM_PEAK_GBS, 4), **grading}
    else:
        bound = {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                 "frac": round(gbs / HBM_PEAK_GBS, 4), "mfma_tflops": round(achieved, 2),
                 "mfma_frac": round(achieved / peak, 4), **grading}
    return {**bound,
            "traffic": round(traffic) if traffic else None,
            "traffic_source": traffic_src,
            "traffic_over_algorithmic": round(traffic / alg_bytes, 3) if traffic else None,
            # same profile: SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 1024 SIMDs) over the family
            "mfma_busy_frac_pmc": round(mfma_busy, 4) if mfma_busy else None,
            "algorithmic_bytes_per_launch": round(alg_bytes),
            "kernel": ("dense 3x3 conv fwd + dgrad on f32 MFMA: igemm_conv_kernel<*,*,*,*,3,*> (implicit GEMM), "
                       "halo3x3_kernel (LDS-halo direct conv, narrow decoder convs) and, for the deep decoder "
                       "convs, wino_gemm_kernel + wino_out_kernel (Winograd F(2x2,3x3): 2.25x fewer executed "
                       "MFMA FLOPs than the algorithmic count used here)"
                       if math == "f32" else
                       "dense 3x3 conv fwd + dgrad on bf16 MFMA: igemm_conv_kernel<*,*,*,*,3,*,*,false,__bf16> "
                       "(implicit GEMM, v_mfma_f32_32x32x16_bf16, fp32 accumulation) and halo3x3_kernel "
                       "(LDS-halo direct conv, narrow convs)"),
            "winograd": {"launches": wn, "algorithmic_tflops": round(wfl / wsec / 1e12, 2) if wsec else None,
                         "executed_mfma_tflops": round(wfl / 2.25 / wsec / 1e12, 2) if wsec else None},
            "launches": n, "flops_per_launch": round(flops / max(n, 1)),
            "avg_launch_us": round(secs / max(n, 1) * 1e6, 2),
            "share_of_step": round(secs / dt, 4),
            "note": "live launches share the CUs with the weight-gradient side stream (engine.OVERLAP); "
                    "without_side_stream re-times the same launches in 3 untimed steps with it off",
            "without_side_stream": (
                {"achieved": round(ifl / isec / 1e12, 2) if isec else None, "unit": "TFLOP/s",
                 "frac": round(ifl / isec / 1e12 / peak, 4) if isec else None,
                 "avg_launch_us": round(isec / max(inn, 1) * 1e6, 2), "launches": inn}
                if bound["bound"] == "mfma" else
                {"achieved": round(alg_bytes * inn / isec / 1e9, 1) if isec else None, "unit": "GB/s",
                 "frac": round(alg_bytes * inn / isec / 1e9 / HBM_PEAK_GBS, 4) if isec else None,
                 "mfma_tflops": round(ifl / isec / 1e12, 2) if isec else None,
                 "avg_launch_us": round(isec / max(inn, 1) * 1e6, 2), "launches": inn}),
            "wgrad3": {"achieved": round(wf / ws / 1e12, 2) if ws else None, "launches": wgn,
                       "avg_launch_us": round(ws / max(wgn, 1) * 1e6, 2)},
            "all_mfma_convs": {"achieved": round(af / as_ / 1e12, 2) if as_ else None, "launches": an}}, bn_roof


def _bn_roofline(args, math, family, rec_all, rec_iso, dt, pmc, traffic_src):
    """The BatchNorm-backward family (in bf16io it is the largest share of the step), graded
    against HBM: algorithmic bytes = every BN layer's dA and y read once and dY written once (3 |Y| at the storage
    element size; seg_bn_backward / seg_bn_bwd_apply carry them, the tile finalizes none), divided by the summed
    durations of those launches (HIP events, the 3 untimed all-launch steps after the timed region)."""
    by, sec, n = family(rec_all, {"bn_bwd"})
    if not sec:
        return None
    iby, isec, inn = family(rec_iso, {"bn_bwd"})
    steps = 3
    gbs = by / sec / 1e9
    fam = pmc.get("bn_bwd", {}) if pmc else {}
    traffic = fam.get("hbm_bytes_per_step")
    default_workload = (args.model, args.batch, args.height, args.width) == ("MobileNetV2UNet", 32, 256, 512)
    return {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(gbs / HBM_PEAK_GBS, 4),
            "algorithmic_bytes_per_step": round(by / steps), "launch_entries_per_step": round(n / steps),
            "ms_per_step": round(sec / steps * 1e3, 3), "share_of_step": round(sec / steps / (dt / args.steps), 4),
            "traffic_per_step": round(traffic) if traffic and default_workload else None,
            "traffic_over_algorithmic": round(traffic / (by / steps), 3) if traffic and default_workload else None,
            "traffic_source": traffic_src if traffic and default_workload else None,
            "kernel": "BatchNorm backward (csrc/bn.hip): chan_partial_kernel<1> (sum dz, sum dz (y - mean)) + "
                      "bn_bwd_finalize_kernel + bn_bwd_apply_rt_kernel per layer (seg_bn_backward), or, where the "
                      "data gradient that completes dA wrote the partials (seg_conv_igemm_bnout*), "
                      "bn_bwd_finalize_tiles_kernel + the apply",
            "note": "durations from HIP events around each BN-backward launch entry in 3 untimed steps after the timed "
                    "region (every launch timed, side stream as configured); without_side_stream: the same with it off",
            "without_side_stream": {"achieved": round(iby / isec / 1e9, 1) if isec else None, "unit": "GB/s",
                                    "frac": round(iby / isec / 1e9 / HBM_PEAK_GBS, 4) if isec else None,
                                    "ms_per_step": round(isec / steps * 1e3, 3)}}


def _step_roofline(args, math, core, engine, value, peak):
    """Whole-step roofline (the north-star figure): algorithmic work of one
    training image under the fused-execution model -- FLOPs = 3 x the forward conv FLOPs
    (fwd, data and weight gradient); bytes = sum over convs of (3|X| + 5|Y|) * s plus the
    loss (2 C H W s + 8 H W), s = activation bytes (4 f32, 2 with bf16 storage)."""
    prog = engine.get_program(core, args.batch, args.height, args.width)
    sb = 2 if math == "bf16io" else 4
    fl_img = by_img = 0.0
    for op in prog.ops:
        if isinstance(op, engine.ConvOp):
            fl_img += 3 * op.flops() / args.batch
            by_img += (3 * op.inp.M * op.cin + 5 * op.y.M * op.cout) * sb / args.batch
    by_img += (2 * args.classes * args.height * args.width * sb + 8 * args.height * args.width)
    return {"flops_per_img": round(fl_img), "bytes_per_img": round(by_img),
            "achieved_tflops": round(fl_img * value / 1e12, 2), "achieved_gbs": round(by_img * value / 1e9, 1),
            "frac_mfma_peak": round(fl_img * value / 1e12 / peak, 4),
            "frac_hbm_peak": round(by_img * value / 1e9 / HBM_PEAK_GBS, 4),
            "bound_img_per_s": round(1.0 / max(fl_img / (peak * 1e12), by_img / (HBM_PEAK_GBS * 1e9)), 1)}


if __name__ == "__main__":
    main()
