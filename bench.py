#!/usr/bin/env python3
"""Benchmark: images/sec of the multimodal DFU fusion training step (ResNet50 RGB + ViT-B/16
thermal -> 2816->512->2 head; weighted CE; AdamW) at bs=64 per GPU on MI355X.

One "step" = forward + backward + AdamW over one batch of 64 synthetic 224x224 RGB+thermal
pairs already resident in HBM (BASELINE.json config C3; C4 = the same per GPU over N ranks,
launched by torch.distributed.run, RCCL gradient all-reduce).  Prints ONE JSON line on rank 0.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch 64] [--config fusion|thermal|rgb]
  python bench.py --config gradcam [--batch 32]   # C5: fusion predict + Grad-CAM maps per sample
  python bench.py --config pipeline [--batch 64]  # §8f row 3: GPU train transforms per pair
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "dfu-multimodal_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

# Algorithmic GEMM/conv FLOPs per unit of work (fwd + dgrad + wgrad), SURVEY.md §8(d)
FLOPS_PER_UNIT = {"fusion": 129.44e9, "thermal": 105.15e9, "rgb": 24.29e9, "gradcam": 173.20e9}
PEAK_BF16_TFLOPS = 2500.0
PEAK_HBM_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E ~8 TB/s
PRECISION_NOTE = {
    "parity": "the library default.  forward: ResNet50 bf16x3 (split-bf16 MFMA, fp32-accurate), "
              "ViT-B/16 Blocks fp16 MFMA inside the fusion model (fp32 accumulate / residual / "
              "LN / softmax), bf16x3 when the ViT classifies alone (C2); backward + AdamW: bf16 "
              "MFMA, fp32 master weights and optimizer state (DESIGN.md §4)",
    "bf16": "bf16 MFMA operands and activations, fp32 accumulate / statistics / master weights",
    "bf16x3": "forward fp32-accurate on split-bf16 MFMA everywhere; backward bf16"}  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md chip table)
RGB_MEAN = (0.485, 0.456, 0.406)
RGB_STD = (0.229, 0.224, 0.225)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=None, help="per GPU (default 64; gradcam 32)")
    ap.add_argument("--config", default="fusion", choices=["fusion", "thermal", "rgb", "gradcam",
                                                               "pipeline"])
    ap.add_argument("--graph", action="store_true",
                    help="replay the train step as one HIP graph (default: eager, measured faster: "
                         "the two encoder streams overlap better than the graph's branches)")
    ap.add_argument("--no-graph", action="store_true", help="eager (the default; kept for scripts)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=None,
                    help="CPU baseline threads (default: the host's physical cores, lscpu "
                         "sockets x cores per socket, BASELINE.md)")
    ap.add_argument("--precision", default=None, choices=["parity", "bf16", "bf16x3"],
                    help="forward precision of the timed step (value).  Default: the library's "
                         "own default (dfu_hip.functional.DEFAULT_PRECISION = parity: the ResNet "
                         "forward bf16x3, the ViT Blocks fp16 in the fusion model / bf16x3 when "
                         "the ViT classifies alone, backward bf16 -- the mode that meets "
                         "north_star's 1e-3 logits bar with margin, DESIGN.md §4), with no "
                         "set_precision call; the other modes are timed beside it")
    ap.add_argument("--no-alt-precision", action="store_true",
                    help="skip timing the other precision modes")
    ap.add_argument("--no-parity", action="store_true",
                    help="skip the in-run logits parity check against the CPU oracle")
    args = ap.parse_args()
    if args.batch is None:
        args.batch = 32 if args.config == "gradcam" else 64
    return args


def baseline_threads(args):
    """--cpu-threads, else the host's physical cores (lscpu), else os.cpu_count()."""
    if args.cpu_threads:
        return args.cpu_threads
    return host_cores().get("physical_cores") or os.cpu_count() or 1


def arithmetic_label(model):
    """What the timed step computes in, per encoder, under the current precision mode (the
    line's `dtype`): the forward stage modes (models.precision.stages), then the backward."""
    from dfu_hip import functional as Fn
    from models import precision as P
    fwd = {}
    for name, m in P.stages(model).items():
        enc = "ResNet50" if name.startswith("resnet") else "ViT-B/16 Blocks"
        fwd.setdefault(enc, set()).add(Fn.stage_mode(m))
    parts = [f"{enc} {'/'.join(sorted(ms))}" for enc, ms in fwd.items()]
    return (f"fwd {', '.join(parts)} (fp32 accumulate, residual stream, statistics); "
            f"bwd bf16 MFMA; fp32 master weights / AdamW")


def synthetic(B, device, seed):
    """uint8 U{0..255} images normalised as the reference transforms
    (train_multimodal_fusion.py:181, 198), labels U{0,1}; generated once on the device."""
    g = torch.Generator(device=device).manual_seed(seed)
    rgb = torch.randint(0, 256, (B, 3, 224, 224), generator=g, device=device, dtype=torch.uint8)
    th = torch.randint(0, 256, (B, 3, 224, 224), generator=g, device=device, dtype=torch.uint8)
    y = torch.randint(0, 2, (B,), generator=g, device=device, dtype=torch.int64)
    mean = torch.tensor(RGB_MEAN, device=device).view(1, 3, 1, 1)
    std = torch.tensor(RGB_STD, device=device).view(1, 3, 1, 1)
    rgb = ((rgb.float() / 255.0 - mean) / std).contiguous()
    th = ((th.float() / 255.0 - 0.5) / 0.5).contiguous()
    return rgb, th, y


def build(config, device):
    from models.fusion import MultimodalFusionModel
    from models.single import RGBOnlyModel, ThermalOnlyModel
    if config == "fusion":
        # DFU_SERIAL_BRANCHES=1: both encoders on one stream (measures the side-stream overlap)
        model = MultimodalFusionModel(
            num_classes=2, dropout=0.7,
            concurrent_branches=os.environ.get("DFU_SERIAL_BRANCHES", "0") != "1")
        fwd = lambda m, r, t: m(r, t)  # noqa: E731
    elif config == "thermal":  # train_thermal_only.py:188-205
        model = ThermalOnlyModel(num_classes=2)
        fwd = lambda m, r, t: m(t)  # noqa: E731
    else:  # train_rgb_only.py:200-217
        model = RGBOnlyModel(num_classes=2)
        fwd = lambda m, r, t: m(r)  # noqa: E731
    return model.to(device).train(), fwd


def host_cores():
    """Host CPU description for cpu_baseline: os.cpu_count() and lscpu's sockets x cores per
    socket x threads per core (the core count is stated)."""
    import subprocess
    info = {"os_cpu_count": os.cpu_count()}
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        keys = {"Socket(s)": "sockets", "Core(s) per socket": "cores_per_socket",
                "Thread(s) per core": "threads_per_core", "Model name": "model"}
        for line in out.splitlines():
            k, _, v = line.partition(":")
            if k.strip() in keys:
                v = v.strip()
                info[keys[k.strip()]] = int(v) if v.isdigit() else v
        if "sockets" in info and "cores_per_socket" in info:
            info["physical_cores"] = info["sockets"] * info["cores_per_socket"]
    except (OSError, subprocess.SubprocessError):
        pass
    return info


def cpu_baseline(config, threads, warmup=3, timed=10, B=8, sweep=True):
    """The oracle (plain PyTorch fp32, oracle/torch_ref.py) timed on the host cores on a bounded
    sample of the same workload, as BASELINE.md prescribes: the full train step (fwd + bwd +
    AdamW) at batch B, `warmup` untimed steps, then the median of `timed` steps.  `threads` is
    the host's physical core count; with `sweep` the count is halved until the step time rises
    (best of two steps per count after a warm-up; on the 2 x 64-core EPYC hosts all 128 threads
    ran the step 6.6x SLOWER than 16: cross-socket traffic and oneDNN's per-op thread start-up
    at batch 8) and the fastest count is used -- an interior minimum of the sweep, so the
    baseline is the best this host does, with every count tried reported."""
    import statistics
    from oracle import torch_ref as R
    torch.manual_seed(0)
    if config == "fusion":
        model = R.MultimodalFusionModel(num_classes=2, dropout=0.7)
        run = lambda r, t: model(r, t)  # noqa: E731
    elif config == "thermal":
        model = R.VisionTransformer(num_classes=2)
        run = lambda r, t: model(t)  # noqa: E731
    else:
        model = R.ResNet(num_classes=2)
        run = lambda r, t: model(r)  # noqa: E731
    model.train()
    rgb, th, y = R.synthetic_batch(B, seed=42)
    crit = torch.nn.CrossEntropyLoss(weight=torch.tensor([2.0, 2.0]))
    opt = torch.optim.AdamW(model.parameters(), lr=1e-4, weight_decay=1e-4)

    def step():
        opt.zero_grad()
        loss = crit(run(rgb, th), y)
        loss.backward()
        opt.step()

    tried = {}

    def probe(t):
        torch.set_num_threads(t)
        step()  # warm this thread count
        best = float("inf")
        for _ in range(2):
            t0 = time.perf_counter()
            step()
            best = min(best, time.perf_counter() - t0)
        tried[t] = best

    # halve the thread count from the physical cores until the step time rises (and at least
    # once past the fastest count), so the count used is an interior minimum of the sweep
    t = threads
    probe(t)
    while sweep and t > 1:
        t //= 2
        probe(t)
        if tried[t] > min(tried.values()):
            break
    use = min(tried, key=tried.get)
    torch.set_num_threads(use)
    for _ in range(warmup):
        step()
    times = []
    for _ in range(timed):
        t0 = time.perf_counter()
        step()
        times.append(time.perf_counter() - t0)
    med = statistics.median(times)
    cores = host_cores()
    return {"value": round(B / med, 3), "unit": "images/sec", "cores": use,
            "kind": "port", "host": cores,
            "thread_sweep_ms": {str(k): round(v * 1e3) for k, v in tried.items()},
            "sample": f"oracle fp32 eager {config} train step (fwd+bwd+AdamW), batch {B}: "
                      f"median of {timed} timed steps ({med * 1e3:.0f} ms/step, "
                      f"{sum(times):.1f} s) after {warmup} warm-up, "
                      f"torch.set_num_threads({use}), the fastest of {sorted(tried)} on a "
                      f"host with {cores.get('physical_cores', '?')} physical cores "
                      f"(os.cpu_count() {cores['os_cpu_count']}; best of two steps each, halved "
                      f"until the time rose)"}


def cpu_baseline_gradcam(threads, budget_s=10.0):
    """The oracle's restatement of the reference Grad-CAM (oracle/gradcam_ref.py) timed on the host
    cores, sample by sample as the reference runs it (bs=1, grad_cam_visualization.py:686): fusion
    forward under no_grad, the ResNet 'layer4' CAM and the ViT input saliency.  As cpu_baseline:
    one sample is timed at `threads` (the physical cores) and at 1/2 .. 1/16 of it, and the
    fastest count is used."""
    from oracle import gradcam_ref as G
    from oracle import torch_ref as R
    torch.manual_seed(0)
    model = R.MultimodalFusionModel(num_classes=2, dropout=0.7).eval()
    rgb, th, _ = R.synthetic_batch(4, seed=42)
    cam = G.GradCAMRef(model.resnet, ["layer4"])

    def sample(i):
        with torch.no_grad():
            torch.softmax(model(rgb[i:i + 1], th[i:i + 1]), 1).argmax(1)
        cam.generate_cam(rgb[i:i + 1])
        G.saliency_ref(model.vit, th[i:i + 1])

    tried = {}
    for t in dict.fromkeys(x for x in (threads, threads // 2, threads // 4, threads // 8,
                                       threads // 16) if x >= 1):
        torch.set_num_threads(t)
        sample(0)
        t0 = time.perf_counter()
        sample(1)
        tried[t] = time.perf_counter() - t0
    use = min(tried, key=tried.get)
    torch.set_num_threads(use)
    t0 = time.perf_counter()
    n = 0
    while n < 8 and (n == 0 or time.perf_counter() - t0 < budget_s):
        sample(n % 4)
        n += 1
    dt = time.perf_counter() - t0
    return {"value": round(n / dt, 3), "unit": "samples/sec", "cores": use, "kind": "port",
            "thread_sweep_ms": {str(k): round(v * 1e3) for k, v in tried.items()},
            "sample": f"oracle fp32 eager Grad-CAM (fusion predict + ResNet layer4 CAM + ViT "
                      f"input saliency), bs=1 as the reference, {n} samples ({dt:.1f} s), "
                      f"torch.set_num_threads({use}), the fastest of {sorted(tried)} (one sample "
                      f"each after a warm-up)"}


# The PMC traffic measurement this tree's bench line cites (tools/prof_summary.py output of the
# separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes; bench.py cannot read counters itself).
TRAFFIC_FILE = os.path.join("profiles", "r26_gemm_traffic.json")  # parity-mode step (round 6)


def gemm_traffic():
    """HBM bytes per GEMM launch from TRAFFIC_FILE (chosen by name, never by file time)."""
    path = os.path.join(ROOT, TRAFFIC_FILE)
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        t = json.load(f)
    return t["bytes_per_launch"], TRAFFIC_FILE


def gemm_roofline(fwd_bwd, tail, replays=3):
    """Dominant kernel: the MFMA GEMM template (dfu_gemm: every ViT linear and ResNet conv, fwd,
    dgrad and wgrad — all of the step's algorithmic GEMM/conv FLOPs except attention's QK^T/PV
    and the fp32 head).  One eager step records every dfu_gemm launch (descriptor + live
    buffers); the recorded launches are then replayed back-to-back on the same stream between
    two HIP events, `replays` times.  achieved = algorithmic FLOPs / measured duration; the
    per-launch average includes each launch's split-K slab reduction (rocprofv3 lists those as
    k_splitk_reduce) and is what profiles/*_kernel_stats.md checks against rocprof."""
    from dfu_hip import ops
    ops.gemm_record = []
    try:
        fwd_bwd()
        tail()
        rec = ops.gemm_record
    finally:
        ops.gemm_record = None
    torch.cuda.synchronize()
    ops.gemm_replay(rec)  # warm
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(replays):
        ops.gemm_replay(rec)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / replays  # per step
    flops = sum(r[1] for r in rec)
    # MFMA work executed (ops.gemm's record): a bf16x3 GEMM runs three products of the real K,
    # on the tripled K and on interleaved pairs alike (K = 2C: three 32-wide MFMAs per 64-wide
    # K-step)
    executed = sum(r[4] for r in rec)
    nbytes = sum(r[2] for r in rec)
    n = len(rec)
    # each launch priced at its OWN bound: the MFMA time of the work it executes at the dense
    # peak, or the HBM time of its compulsory bytes at 8 TB/s, whichever is longer (the layer-1
    # convolutions and the split-K weight gradients of small planes are HBM-bound, the ViT
    # linears MFMA-bound); their sum over the measured replay time is the family's fraction of
    # its per-launch roofline
    t_mfma = [r[4] / (PEAK_BF16_TFLOPS * 1e12) for r in rec]
    t_hbm = [r[2] / (PEAK_HBM_GBS * 1e9) for r in rec]
    bound_us = sum(max(a, b) for a, b in zip(t_mfma, t_hbm)) * 1e6
    per_launch = {"frac": round(bound_us / us, 4), "bound_us_per_step": round(bound_us, 1),
                  "measured_us_per_step": round(us, 1),
                  "mfma_bound_launches": sum(1 for a, b in zip(t_mfma, t_hbm) if a >= b),
                  "hbm_bound_launches": sum(1 for a, b in zip(t_mfma, t_hbm) if a < b),
                  "basis": f"sum over the step's launches of max(executed MFMA FLOPs / "
                           f"{PEAK_BF16_TFLOPS:.0f} TFLOP/s, algorithmic bytes / "
                           f"{PEAK_HBM_GBS:.0f} GB/s) / replay time"}
    return {"launches_per_step": n, "avg_launch_us": us / n, "flops_per_launch": flops / n,
            "per_launch_roofline": per_launch,
            "bytes_per_launch": nbytes / n, "gemm_ms_per_step": us / 1e3,
            "achieved": flops / (us * 1e-6) / 1e12,
            "mfma_executed": executed / (us * 1e-6) / 1e12,
            "x3_launches": sum(1 for r in rec if r[4] == 3.0 * r[1])}


def main_gradcam(args, rank, world, dev):
    """C5 (grad_cam_visualization.py visualize_multimodal :561-632, batched): per batch of B
    samples resident in HBM, one eval fusion forward under no_grad (softmax, argmax), then
    GradCAM(model.resnet, ['layer4']) -> (B, 7, 7) CAMs and GradCAM(model.vit, ['blocks']) ->
    (B, 224, 224) input saliency, each one forward + backward with input gradients.  Replicas
    over ranks (each its own samples; no data-path collective)."""
    from models.fusion import MultimodalFusionModel
    from models.gradcam import GradCAM
    from dfu_hip import functional as Fn
    if args.precision is not None:
        Fn.set_precision(args.precision)
    args.precision = Fn.get_precision()  # the library default unless --precision names one
    model = MultimodalFusionModel(num_classes=2, dropout=0.7).to(dev).eval()
    rgb, th, _ = synthetic(args.batch, dev, seed=42 + rank)
    cam_rgb = GradCAM(model.resnet, ["layer4"])
    cam_th = GradCAM(model.vit, ["blocks"])
    outs = {}

    def step():
        with torch.no_grad():
            probs = torch.softmax(model(rgb, th), dim=1)
        outs["pred"] = probs.argmax(1)
        outs["cam"] = cam_rgb.generate_cams(rgb)
        outs["sal"] = cam_th.generate_cams(th)

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(max(1, args.warmup)):
            step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    assert outs["cam"].shape == (args.batch, 7, 7) and outs["sal"].shape == (args.batch, 224, 224)
    ref_cam = outs["cam"].clone()
    graph = None
    choice = {}
    if not args.no_graph:
        from dfu_hip import graphs
        # the hooks' Python runs once, at capture; replays rewrite the same buffers
        graph = graphs.try_capture(step, log=None if rank == 0 else False)
        if graph is not None:
            graph.replay()
            torch.cuda.synchronize()
            if not torch.allclose(outs["cam"], ref_cam, atol=1e-2):
                if rank == 0:
                    print("[bench] graph replay changed the CAMs; eager", file=sys.stderr)
                graph = None
        if graph is not None:
            # keep whichever of eager and replay is faster on this box: a
            # few untimed rounds of each, same work
            def _ms(fn, n=5):
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(n):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                return e0.elapsed_time(e1) / n
            choice = {"graph_ms": round(_ms(graph.replay), 3), "eager_ms": round(_ms(step), 3)}
            if world > 1:  # every rank takes the same path
                t = torch.tensor([choice["graph_ms"], choice["eager_ms"]], device=dev)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                choice = {"graph_ms": round(t[0].item(), 3), "eager_ms": round(t[1].item(), 3)}
            if choice["eager_ms"] < choice["graph_ms"]:
                graph = None
    run = graph.replay if graph is not None else step
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(args.steps):
        run()
    ev1.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    gpu_ms = ev0.elapsed_time(ev1)
    if world > 1:
        t = torch.tensor([elapsed, gpu_ms / 1000.0], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, gpu_s = t.tolist()
        gpu_ms = gpu_s * 1000.0
    gr = gemm_roofline(step, lambda: None)
    value = args.batch * args.gpus * args.steps / elapsed
    per_step_s = gpu_ms / 1000.0 / args.steps
    achieved = args.batch * FLOPS_PER_UNIT["gradcam"] / per_step_s / 1e12
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            try:
                cpu = cpu_baseline_gradcam(baseline_threads(args))
            except Exception as e:
                cpu = {"error": f"{type(e).__name__}: {e}"}
        traffic, traffic_src = gemm_traffic()
        line = {
            "metric": "samples/sec (fusion predict + Grad-CAM maps, bs=32/GPU)",
            "value": round(value, 2), "unit": "samples/sec", "n_gpus": args.gpus,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed * 1000.0 / args.steps, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": arithmetic_label(model),
            "precision": args.precision,
            "precision_source": "library default (no set_precision call)"
            if args.precision == Fn.DEFAULT_PRECISION else "--precision",
            "data": "synthetic 224x224 RGB+thermal pairs (uint8 U{0..255}, reference "
                    "normalisation), random-init weights (seed 42), resident in HBM",
            "config": {"workload": "C5 fusion eval predict + ResNet 'layer4' Grad-CAM + ViT "
                                   "'blocks' input saliency (fwd+bwd with input grads)",
                       "model": "resnet50+vit_base_patch16_224 late fusion",
                       "global_batch": args.batch * args.gpus, "per_gpu_batch": args.batch,
                       "image": 224, "parallelism": f"replicas{args.gpus}",
                       "hip_graph": graph is not None, "graph_vs_eager_ms": choice or None,
                       "dist": args.dist},
            "roofline": {"bound": "mfma", "achieved": round(gr["achieved"], 1),
                         "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(gr["achieved"] / PEAK_BF16_TFLOPS, 4),
                         "traffic": None, "traffic_note": "PMC traffic measured on the C3 bench "
                                                          f"({traffic_src}: {traffic} B/launch)",
                         "algorithmic_bytes_per_launch": round(gr["bytes_per_launch"]),
                         "kernel": "dfu gemm_kernel (MFMA bf16 GEMM template)",
                         "launches_per_step": gr["launches_per_step"],
                         "avg_launch_us": round(gr["avg_launch_us"], 2),
                         "gemm_ms_per_step": round(gr["gemm_ms_per_step"], 3),
                         "step": {"achieved": round(achieved, 1),
                                  "frac": round(achieved / PEAK_BF16_TFLOPS, 4),
                                  "basis": f"173.20 GFLOP per sample (SURVEY 8d) x {args.batch} / "
                                           f"HIP-event step time {per_step_s * 1e3:.3f} ms"}},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def main_pipeline(args, rank, world, dev):
    """§8f row 3: the reference's train transforms (train_multimodal_fusion.py:172-205) for B
    decoded RGB + thermal pairs per step — resize 640x480 -> 224x224, flips, rotation, colour
    jitter (RGB), affine, ToTensor, Normalize — on the GPU (csrc/augment.hip).  Staged batches
    are resident in HBM before the timed region; the PCIe-inclusive rate (host packing + one
    H2D copy per modality) is reported beside it.  Replicas over ranks."""
    import numpy as np
    from data import gpu_transforms as GT
    H0, W0, NB = 480, 640, 3
    rng = np.random.default_rng(rank)
    g = torch.Generator().manual_seed(42 + rank)
    rgb_pre = GT.GpuPreprocessor(GT.rgb_train_transform, dev)
    th_pre = GT.GpuPreprocessor(GT.thermal_train_transform, dev)

    def host_batch():
        r = [rng.integers(0, 256, (H0, W0, 3), dtype=np.uint8) for _ in range(args.batch)]
        t = [rng.integers(0, 256, (H0, W0, 3), dtype=np.uint8) for _ in range(args.batch)]
        pr = [GT.sample_params(GT.rgb_train_transform, g) for _ in r]
        pt = [GT.sample_params(GT.thermal_train_transform, g) for _ in t]
        return r, pr, t, pt
    hosts = [host_batch() for _ in range(NB)]
    staged = [(rgb_pre.stage(r, pr), th_pre.stage(t, pt)) for r, pr, t, pt in hosts]
    torch.cuda.synchronize()

    def step(i):
        a, b = staged[i % NB]
        return rgb_pre.run(a), th_pre.run(b)
    for i in range(max(1, args.warmup)):
        step(i)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for i in range(args.steps):
        step(i)
    ev1.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    gpu_s = ev0.elapsed_time(ev1) / 1000.0
    if world > 1:
        t = torch.tensor([elapsed, gpu_s], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, gpu_s = t.tolist()
    # PCIe-inclusive: host packing + H2D + kernels, same batches
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for i in range(args.steps):
        r, pr, t, pt = hosts[i % NB]
        rgb_pre(r, pr), th_pre(t, pt)
    torch.cuda.synchronize()
    incl = args.batch * args.steps / (time.perf_counter() - t1)
    # algorithmic HBM bytes per pair (both modalities): source read, horizontal-pass rows
    # written + read, resized image written + read (+ once more by the contrast statistics when
    # drawn: not counted), fp32 NCHW output written
    OS = 224
    per_img = H0 * W0 * 3 + 2 * H0 * OS * 3 + 2 * OS * OS * 3 + OS * OS * 3 * 4
    per_pair = 2 * per_img
    achieved = args.batch * per_pair / (gpu_s / args.steps) / 1e9
    value = args.batch * args.gpus * args.steps / elapsed
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import transforms_ref as TR
            r, pr, t, pt = hosts[0]
            n, t0c = 0, time.perf_counter()
            while time.perf_counter() - t0c < 10.0:
                j = n % len(r)
                for im, p, spec in ((r[j], pr[j], GT.rgb_train_transform),
                                    (t[j], pt[j], GT.thermal_train_transform)):
                    TR.reference_transform(im, spec.size, spec.mean, spec.std, p.hflip, p.vflip,
                                           p.angle, p.ops, p.affine)
                n += 1
            cpu = {"value": round(n / (time.perf_counter() - t0c), 2), "unit": "pairs/sec",
                   "cores": 1, "kind": "port",
                   "sample": f"{n} pairs through the PIL/torch transforms torchvision runs "
                             "(oracle/transforms_ref.py), one core, same images and parameters"}
        line = {
            "metric": "pairs/sec (RGB+thermal train transforms on GPU, decoded 640x480 inputs)",
            "value": round(value, 2), "unit": "pairs/sec", "n_gpus": args.gpus,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed * 1000.0 / args.steps, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic decoded 640x480 RGB + thermal frames (uint8 uniform), "
                    "parameters drawn in torchvision's order (seeded)",
            "config": {"workload": "§8f row 3 input pipeline: Resize(224) + flips + "
                                   "RandomRotation(30) + ColorJitter (RGB, p 0.6) + RandomAffine "
                                   "(p 0.6) + ToTensor + Normalize, both modalities",
                       "per_gpu_batch": args.batch, "source": f"{W0}x{H0}",
                       "parallelism": f"replicas{args.gpus}", "dist": args.dist},
            "pcie_inclusive_pairs_per_sec": round(incl, 1),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS,
                         "unit": "GB/s", "frac": round(achieved / PEAK_HBM_GBS, 4), "traffic": None,
                         "kernel": "augment pipeline (8 launches per step: 2 resize passes, "
                                   "contrast statistics, gather/normalise, per modality)",
                         "algorithmic_bytes_per_pair": per_pair},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def timed_steps(step, steps, world, dev, per_step=True):
    """Run `steps` steps between barrier + synchronize brackets; returns the wall-clock seconds
    (max over ranks), the HIP-event window in ms (max over ranks) and the per-step HIP-event
    durations (ms, this rank) from an event recorded after every step."""
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    t0 = time.perf_counter()
    evs[0].record()
    for k in range(steps):
        step()
        if per_step or k == steps - 1:
            evs[k + 1].record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    gpu_ms = evs[0].elapsed_time(evs[-1])
    durs = [evs[k].elapsed_time(evs[k + 1]) for k in range(steps)] if per_step else []
    if world > 1:
        t = torch.tensor([elapsed, gpu_ms / 1000.0], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, gpu_s = t.tolist()
        gpu_ms = gpu_s * 1000.0
    return elapsed, gpu_ms, durs


def pct(xs, q):
    """q-th percentile (linear interpolation) of a non-empty list."""
    xs = sorted(xs)
    k = (len(xs) - 1) * q
    lo = int(k)
    hi = min(lo + 1, len(xs) - 1)
    return xs[lo] + (xs[hi] - xs[lo]) * (k - lo)


def parity_check(config, dev, B, threads):
    """Logits parity measured in this run (north_star: within 1e-3 abs of the reference CPU
    path): the fp32 CPU oracle (oracle/torch_ref.py, torchvision/timm restated) and the HIP
    model on the same seeded weights and synthetic batch, C3's own batch size, train-mode BN,
    dropout identity, forward only, in both precision modes."""
    from dfu_hip import functional as Fn
    from models.fusion import MultimodalFusionModel
    from models.single import RGBOnlyModel, ThermalOnlyModel
    from oracle import torch_ref as R
    torch.set_num_threads(threads)
    torch.manual_seed(0)
    rgb, th, _ = R.synthetic_batch(B, seed=42)
    if config == "fusion":
        ref = R.MultimodalFusionModel(num_classes=2, dropout=0.0)
        hip = MultimodalFusionModel(num_classes=2, dropout=0.0)
        run_ref, run_hip = (lambda m: m(rgb, th)), (lambda m: m(rgb.to(dev), th.to(dev)))
    elif config == "thermal":
        ref = R.VisionTransformer(num_classes=2)
        ref.head = torch.nn.Sequential(torch.nn.Dropout(0.0), torch.nn.Linear(768, 2))
        hip = ThermalOnlyModel(drop_rate=0.0)
        ref = _Wrap(ref)
        run_ref, run_hip = (lambda m: m(th)), (lambda m: m(th.to(dev)))
    else:
        ref = R.ResNet()
        ref.fc = torch.nn.Sequential(torch.nn.Dropout(0.0), torch.nn.Linear(2048, 2))
        hip = RGBOnlyModel(drop_rate=0.0)
        ref = _Wrap(ref)
        run_ref, run_hip = (lambda m: m(rgb)), (lambda m: m(rgb.to(dev)))
    hip.load_state_dict(ref.state_dict(), strict=True)
    hip = hip.to(dev).train()
    t0 = time.perf_counter()
    with torch.no_grad():
        want = run_ref(ref.train())
    t_ref = time.perf_counter() - t0
    out = {"batch": B, "bar": 1e-3, "max_abs_logit": round(want.abs().max().item(), 4),
           "oracle": "oracle/torch_ref.py fp32 on the host, train-mode BN, dropout identity",
           "oracle_forward_s": round(t_ref, 2)}
    for mode in ("bf16", "bf16x3", "parity"):
        with torch.no_grad(), Fn.precision(mode):
            got = run_hip(hip).float().cpu()
        d = (got - want).abs().max().item()
        out[mode] = {"max_abs_logits_vs_fp32_oracle": float(f"{d:.3e}"), "meets_bar": d <= 1e-3}
    del hip
    torch.cuda.empty_cache()
    return out


class _Wrap(torch.nn.Module):
    """The oracle encoder as the single-modality models' ``backbone`` (state-dict prefix)."""

    def __init__(self, m):
        super().__init__()
        self.backbone = m

    def forward(self, x):
        return self.backbone(x)


def free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n):
    """`--gpus N` (N > 1) without a launcher: this process, which has not touched the GPU
    (torch.cuda.device_count() does not initialise it), starts the N ranks as ONE child
    process -- torch.distributed.run, one rank per GPU, rendezvous on 127.0.0.1 -- and exits
    with its status.  It never times one process and multiplies by N.  Fails (exit 2) when the
    node has fewer than N GPUs, unless DFU_SHARE_DEVICE=1 (the gloo rehearsal that puts every
    rank on device 0)."""
    import subprocess
    have = torch.cuda.device_count()
    if have < n and os.environ.get("DFU_SHARE_DEVICE", "0") != "1":
        print(f"[bench] --gpus {n} needs {n} GPUs, this node has {have}; not running "
              f"(a one-process run is never reported as {n} GPUs)", file=sys.stderr)
        sys.exit(2)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr=127.0.0.1", f"--master-port={free_port()}",
           os.path.abspath(__file__)] + sys.argv[1:]
    print(f"[bench] launching {n} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    sys.exit(subprocess.call(cmd))


def main():
    args = parse()
    if args.gpus > 1 and int(os.environ.get("WORLD_SIZE", "1")) == 1:
        launch_ranks(args.gpus)
    from dfu_hip import parallel
    rank, world, local = parallel.init_from_env()
    if world != args.gpus:
        print(f"[bench] rank {rank}: --gpus {args.gpus} but WORLD_SIZE {world}: the line would "
              f"misreport the job; not running", file=sys.stderr)
        sys.exit(2)
    if world > 1 and dist.get_world_size() != args.gpus:
        print(f"[bench] process group has {dist.get_world_size()} ranks, --gpus {args.gpus}",
              file=sys.stderr)
        sys.exit(2)
    args.dist = {"ranks": world, "backend": dist.get_backend() if world > 1 else None,
                 "device_count": torch.cuda.device_count(),
                 "shared_device": os.environ.get("DFU_SHARE_DEVICE", "0") == "1"}
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    # per-rank torch seed (the dropout RNG is seeded per rank; dfu_hip.nn.Dropout
    # also mixes the rank into its key); the weights are broadcast from rank 0 below
    torch.manual_seed(42 + rank)
    if args.config == "gradcam":
        return main_gradcam(args, rank, world, dev)
    if args.config == "pipeline":
        return main_pipeline(args, rank, world, dev)

    from dfu_hip import functional as Fn
    from dfu_hip import nn as hnn
    from dfu_hip.optim import FusedAdamW
    precision_source = "library default (no set_precision call)"
    if args.precision is not None:
        Fn.set_precision(args.precision)
        precision_source = "--precision"
    args.precision = Fn.get_precision()
    model, fwd = build(args.config, dev)
    parallel.broadcast_parameters(model)
    opt = FusedAdamW(model.parameters(), lr=1e-4, weight_decay=1e-4)
    crit = hnn.CrossEntropyLoss(weight=torch.tensor([2.0, 2.0], device=dev))
    use_graph = args.graph and not args.no_graph
    # eager: bucketed all-reduce on a side stream, launched from the gradient-ready hooks while
    # backward runs; a captured graph issues every bucket after backward instead
    reducer = parallel.GradAllReducer(opt.flat, overlap=not use_graph) if world > 1 else None
    rgb, th, y = synthetic(args.batch, dev, seed=42 + rank)

    def fwd_bwd():
        opt.zero_grad()
        if reducer is not None and reducer.overlap:
            reducer.start()
        out = fwd(model, rgb, th)
        loss = crit(out, y)
        loss.backward()
        Fn.join_grad_streams()  # the thermal branch's side stream rejoins (graph capture needs it)
        return loss

    def tail():
        if reducer is not None:
            reducer.finish()
        opt.step()

    graph = None
    # warm-up (also builds every persistent buffer) on a side stream, as graph capture needs
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(max(1, args.warmup)):
            fwd_bwd()
            tail()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    if use_graph:
        from dfu_hip import graphs
        opt.check_grads = False

        def captured():
            fwd_bwd()
            if reducer is None:
                opt.step()
        graph = graphs.try_capture(captured, log=None if rank == 0 else False)
        if graph is None:  # graph capture is an optimisation: the failure was reported
            opt.check_grads = True
        else:
            for _ in range(2):
                graph.replay()
                if reducer is not None:
                    tail()
            torch.cuda.synchronize()

    def step():
        if graph is not None:
            graph.replay()
            if reducer is not None:
                tail()
        else:
            fwd_bwd()
            tail()

    elapsed, gpu_ms, durs = timed_steps(step, args.steps, world, dev)
    # the other precision modes, same model and batch, eager (reported beside `value`)
    alts = []
    if not args.no_alt_precision and graph is None:
        for other in [m for m in ("bf16", "bf16x3", "parity") if m != args.precision]:
            old = Fn.set_precision(other)
            try:
                for _ in range(2):
                    step()
                a_el, a_ms, a_durs = timed_steps(step, args.steps, world, dev)
            finally:
                Fn.set_precision(old)
            alts.append({"precision": other,
                         "value": round(args.batch * args.gpus * args.steps / a_el, 2),
                         "ms_per_step": round(a_el * 1000.0 / args.steps, 3),
                         "gpu_ms_per_step_median": round(pct(a_durs, 0.5), 3)})
    # every rank runs the instrumented steps (their all-reduces must pair up); rank 0 reports
    opt.check_grads = True
    gr = gemm_roofline(fwd_bwd, tail)
    imgs = args.batch * args.gpus * args.steps
    value = imgs / elapsed
    per_gpu_step_s = (gpu_ms / 1000.0) / args.steps
    achieved = args.batch * FLOPS_PER_UNIT[args.config] / per_gpu_step_s / 1e12
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            try:
                cpu = cpu_baseline(args.config, baseline_threads(args))
            except Exception as e:  # never lose the GPU line over the baseline
                cpu = {"error": f"{type(e).__name__}: {e}"}
        metric = {"fusion": "images/sec (fusion fwd+bwd, bs=64/GPU)",
                  "thermal": "images/sec (thermal ViT-B/16 fwd+bwd, bs=64/GPU)",
                  "rgb": "images/sec (RGB ResNet50 fwd+bwd, bs=64/GPU)"}[args.config]
        traffic, traffic_src = gemm_traffic()
        modes = {args.precision: {"value": round(value, 2),
                                  "ms_per_step": round(elapsed * 1000.0 / args.steps, 3)}}
        for alt in alts:
            modes[alt["precision"]] = {k: v for k, v in alt.items() if k != "precision"}
        parity = None
        if world == 1 and not args.no_parity:
            try:
                pthreads = (cpu or {}).get("cores") or min(16, baseline_threads(args))
                parity = parity_check(args.config, dev, args.batch, pthreads)
            except Exception as e:  # never lose the GPU line over the check
                parity = {"error": f"{type(e).__name__}: {e}"}
        if parity is not None and "error" not in parity:
            for m, v in modes.items():
                if m in parity:
                    v["meets_parity_bar"] = parity[m]["meets_bar"]
        line = {
            "metric": metric,
            "value": round(value, 2),
            "unit": "images/sec",
            "n_gpus": args.gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed * 1000.0 / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": arithmetic_label(model),
            "precision": args.precision,
            "precision_source": precision_source,
            "precision_note": PRECISION_NOTE.get(args.precision),
            "data": "synthetic 224x224 RGB+thermal pairs (uint8 U{0..255}, reference "
                    "normalisation), random-init weights (seed 42), resident in HBM",
            "config": {"workload": f"C3 {args.config} train step (fwd+bwd+AdamW) "
                                   f"ResNet50+ViT-B/16 -> 2816->512->2",
                       "model": "resnet50+vit_base_patch16_224 late fusion",
                       "global_batch": args.batch * args.gpus, "per_gpu_batch": args.batch,
                       "image": 224, "parallelism": f"dp{args.gpus}",
                       "hip_graph": graph is not None, "dist": args.dist},
            "gpu_step_ms": {"median": round(pct(durs, 0.5), 3), "p10": round(pct(durs, 0.1), 3),
                            "p90": round(pct(durs, 0.9), 3), "basis": "HIP events after every "
                            "step of the timed window (rank 0)"},
            "precision_modes": modes,
            "value_meets_parity_bar": None if parity is None or "error" in parity
            else parity[args.precision]["meets_bar"],
            "parity": parity,
            "roofline": {"bound": "mfma", "achieved": round(gr["achieved"], 1),
                         "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(gr["achieved"] / PEAK_BF16_TFLOPS, 4),
                         "traffic": None if traffic is None else round(traffic),
                         "traffic_unit": "bytes per launch (HBM, PMC)",
                         "algorithmic_bytes_per_launch": round(gr["bytes_per_launch"]),
                         "traffic_source": traffic_src,
                         "kernel": "dfu gemm_kernel / gemm_ps (MFMA GEMM template, bf16 "
                                   "operands; in the parity mode the ViT forward's on fp16 "
                                   "MFMA and the ResNet forward's split-bf16: all ViT linears "
                                   "and implicit-GEMM convs, fwd/dgrad/wgrad)",
                         "launches_per_step": gr["launches_per_step"],
                         "avg_launch_us": round(gr["avg_launch_us"], 2),
                         "gflop_per_launch": round(gr["flops_per_launch"] / 1e9, 4),
                         "flop_basis": "algorithmic 2MNK per GEMM (a bf16x3 GEMM's tripled K "
                                       "counted once; strided dgrad / s^2)",
                         "mfma_executed_tflops": round(gr["mfma_executed"], 1),
                         "x3_launches_per_step": gr["x3_launches"],
                         "gemm_ms_per_step": round(gr["gemm_ms_per_step"], 3),
                         "per_launch_roofline": gr["per_launch_roofline"],
                         "step": {"achieved": round(achieved, 1),
                                  "frac": round(achieved / PEAK_BF16_TFLOPS, 4),
                                  "basis": f"{FLOPS_PER_UNIT[args.config] / 1e9:.2f} GFLOP per "
                                           f"image pair (SURVEY 8d) x {args.batch} / HIP-event "
                                           f"step time {per_gpu_step_s * 1e3:.3f} ms"}},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
