#!/usr/bin/env python3
"""Benchmark: lego 800x800 (64 coarse + 128 fine) NeRF render on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

One step = one full 800x800 frame (640,000 rays, 64 coarse + 192 fine MLP
evaluations per ray) of a lego test view (views 0, 8, ..., 192 cycled), split
into row bands across the ranks, maps all-gathered over RCCL. Inputs (packed
weights, z tables) are resident in HBM before timing starts. Weights: the lego
checkpoint trained by tools/train_lego.py (checkpoints/lego) when present,
else the deterministic synthetic generator (--synthetic forces it).

The headline run uses the default MLP arithmetic (--precision f16x3: FP32
operands as 3-term FP16 splits on FP16 MFMA with FP32 accumulation, held to the
same parity gates as FP32); the same frames are then timed with
the FP32-MFMA kernel and reported under "fp32_mfma".

Prints one JSON line (rank 0) with, besides the contract keys:
  roofline        the fused MLP kernel's HIP-event-timed launches: executed MFMA
                  FLOP/s vs the dense peak of the type it runs on (+ algorithmic)
  parity          GPU vs the parity oracle (oracle/nerf_oracle.py) on a strip
  cpu_baseline    the reference's CPU path (torch-CPU restatement,
                  oracle/torch_render.py) timed on this host's cores on a strip
  psnr_vs_gt      evaluator PSNR/SSIM of the HIP render of the packed lego test
                  views vs ground truth (data/lego/test.npz), and |dPSNR| HIP vs
                  oracle on the strip
  c3_train_step   BASELINE configs[2]: the 1024-ray training step, timed
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "nerf-rep_for_test_amd"))

FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: dense FP32 matrix peak
FP16_MFMA_PEAK_TFLOPS = 16 * FP32_MFMA_PEAK_TFLOPS   # dense FP16/BF16 MFMA (1/16 rule, ~2.5 PF)
# FP16 MFMA FLOP the x3 kernel executes per sample: 65 slices of MFMA tiles
# (layer 0 2, layers 1-4/6/7 8 each, skip layer 10, views 4 x 2 K steps + the
# direction step, the feature layer folded into views) = 528 384 MACs, x3
# products, x2 FLOP. The algorithmic count (the reference's FLOPs) stays
# NerfPipeline.MLP_FLOP_PER_SAMPLE = 1 186 816.
X3_EXEC_FLOP_PER_SAMPLE = 2 * 3 * 528384
HBM_PEAK_BPS = 8.0e12          # MI355X_MICROARCH.md
METRIC = "Mrays/s + ms/frame, lego 800x800 (64c+128f); PSNR vs ref"


GT_STRIDE = 8          # tools/pack_lego.py: data/lego/test.npz = test frames 0, 8, ..., 192
DEFAULT_CKPT = os.path.join(REPO, "checkpoints", "lego")
GT_PATH = os.path.join(REPO, "data", "lego", "test.npz")


def lego_camera(H, W, idx):
    """Test view GT_STRIDE * (idx mod 25): the frames whose ground truth is packed."""
    cams = np.load(os.path.join(REPO, "tests", "golden", "lego_test_cameras.npz"))
    poses, angle = cams["poses"], float(cams["camera_angle_x"])
    focal = 0.5 * W / np.tan(0.5 * angle)            # blender.py:41-42
    K = np.array([[focal, 0, W / 2], [0, focal, H / 2], [0, 0, 1]], np.float32)
    return poses[(GT_STRIDE * idx) % len(poses)], K


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--H", type=int, default=800)
    ap.add_argument("--W", type=int, default=800)
    ap.add_argument("--cpu-rows", type=int, default=24,
                    help="rows of the frame the CPU oracle baseline renders")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--precision", default="f16x3", choices=["fp32", "f16x3"],
                    help="MLP arithmetic of the headline run: the 3-term FP16 split of the "
                         "FP32 operands on FP16 MFMA (default), or FP32 MFMA")
    ap.add_argument("--config", default="c2", choices=["c2", "c3", "c4"],
                    help="c2: lego 800x800 64c+128f (BASELINE configs[1], the headline); "
                         "c3: train step, 1024 rays/rank (configs[2]); "
                         "c4: c2 with ESS + ERT (configs[3], lego.yaml:96-99)")
    ap.add_argument("--checkpoint", default=None,
                    help="trained weights (a reference-format .pth or model dir); default: "
                         "checkpoints/lego (trained by tools/train_lego.py) when present")
    ap.add_argument("--synthetic", action="store_true",
                    help="synthetic generator weights even when the trained checkpoint exists")
    ap.add_argument("--no-gt", action="store_true",
                    help="skip the PSNR/SSIM-vs-ground-truth renders (profiling runs)")
    ap.add_argument("--no-c3", action="store_true",
                    help="skip the C3 train-step sub-record of the default run")
    ap.add_argument("--train-mlp", default="x3", choices=["x3", "torch"],
                    help="c3: the MLPs on the x3 MFMA training kernels (default) or as torch "
                         "modules (FP32 hipBLASLt GEMMs)")
    ap.add_argument("--train-launch", default="auto", choices=["auto", "eager", "graph"],
                    help="c3: how a step's kernels are launched: op by op (eager), one HIP "
                         "graph replay (graph), or (auto, 1 rank) whichever ran faster in a "
                         "5-step calibration of each on this box before the timed steps "
                         "(the step is GPU-bound on a fast host and launch-bound on a slow "
                         "one: 5.33 ms of kernels ran 5.71 ms eager on one box)")
    ap.add_argument("--train-graph", action="store_true",
                    help="c3: replay the step as one HIP graph (capturable Adam) instead of "
                         "launching it op by op; the step is GPU-bound (~5.5 ms of kernel "
                         "time), the graph measured 0.15 ms slower (5.46 vs 5.32 ms)")
    ap.add_argument("--ert-segment", type=int, default=8,
                    help="c4: depth-segment length of the ERT sample compaction (8: 1.94 "
                         "Mrays/s, 16: 1.92, 32: 1.86, 64: 1.70 measured)")
    ap.add_argument("--no-fp32-run", action="store_true",
                    help="skip the second, FP32-MFMA timing reported under 'fp32_mfma'")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    from nerfhip.dist import render_frame_sharded
    from nerfhip.render import NerfPipeline
    from nerfhip.synthetic import make_occupancy_grid, make_params

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE",
              file=sys.stderr)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    H, W = args.H, args.W
    ckpt = args.checkpoint
    if ckpt is None and not args.synthetic and os.path.exists(DEFAULT_CKPT):
        ckpt = DEFAULT_CKPT
    if ckpt:
        from nerfhip.checkpoint import load_checkpoint, network_params, resolve
        params = {k: v.numpy() for k, v in network_params(ckpt).items()}
        step = load_checkpoint(resolve(ckpt)).get("epoch")
        data = (f"lego checkpoint {os.path.relpath(resolve(ckpt), REPO)} (trained on the 100 "
                f"lego train views by tools/train_lego.py, {step} steps), lego test cameras")
    else:
        params = make_params(0, 2.0, 0.0)
        data = "synthetic weights (deterministic generator, seed 0, gain 2), lego test cameras"

    def barrier():
        if world > 1:
            dist.barrier()

    c4 = args.config == "c4"
    if args.config == "c3":
        return bench_train(args, world, rank, dev, params, data, barrier)

    def make_pipe(precision):
        pipe = NerfPipeline(dev, N_samples=64, N_importance=128, near=2.0, far=6.0,
                            mlp_precision=precision, enable_ess=c4, enable_ert=c4,
                            ert_threshold=0.01, ert_segment=args.ert_segment)
        pipe.set_weights(params)
        if c4:
            pipe.set_grid(make_occupancy_grid(0, 128, 1.2, 0.1))
        return pipe

    def measure(precision):
        """warmup + K timed frames (barrier + sync both sides, max over ranks)."""
        pipe = make_pipe(precision)

        def frame(i):
            pose, K = lego_camera(H, W, i)
            return render_frame_sharded(
                lambda p0, n: pipe.render_band(H, W, pose, K, p0, n),
                H, W, rank, world, dev, chunk_aligned=c4)

        for i in range(args.warmup):
            frame(i)
        torch.cuda.synchronize()
        barrier()
        pipe.timer = []
        pipe.stage_timer = []
        pipe.ert_stats = []
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.steps):
            frame(args.warmup + i)
        torch.cuda.synchronize()
        barrier()
        elapsed = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        timer, pipe.timer = pipe.timer, None
        stages, pipe.stage_timer = pipe.stage_timer, None
        roof = roofline(precision, timer, elapsed, world, H, W, pmc_workload=world == 1 and not c4)
        roof["byte_kernels"] = byte_kernels(stages, args.steps)
        return pipe, elapsed, roof

    pipe, elapsed, roof = measure(args.precision)
    rays = H * W * args.steps
    result = {
        "metric": METRIC,
        "value": rays / elapsed / 1e6,
        "unit": "Mrays/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": DTYPES[args.precision],
        "data": data,
        "config": {"workload": "lego 800x800, 64 coarse + 128 fine samples, 1 frame per step "
                               "(test poses cycled), " +
                               ("ESS + ERT on (threshold 0.01, synthetic occupancy grid, "
                                "2048-ray chunks)" if c4 else "ESS/ERT off") + ", perturb 0, eval",
                   "baseline_config": "configs[3]" if c4 else "configs[1]",
                   "H": H, "W": W, "N_samples": 64, "N_importance": 128,
                   "mlp_precision": args.precision,
                   "parallelism": f"row-band tiles x{world} + RCCL all-gather of pixels"},
        "roofline": roof,
    }
    if c4:
        ev, full = pipe.evaluated_samples()
        result["ert_compaction"] = {
            "evaluated_samples_per_ray": ev / (rays / world),
            "full_samples_per_ray": full / (rays / world),
            "evaluated_fraction": ev / max(1, full),
            "note": "MLP samples evaluated per ray (coarse 64 + fine 192 in full) with depth "
                    f"segments of {args.ert_segment} and rays retired at T < 0.01 (their later weights are "
                    "zeroed by _raw2outputs_with_ert, VR:1115-1123)"}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        if c4:
            result["cpu_baseline"], result["parity"] = cpu_baseline_c4(
                make_pipe(args.precision), H, W, params, args.cpu_rows)
        else:
            result["parity"] = oracle_parity(pipe, H, W, params, args.cpu_rows)
            result["cpu_baseline"] = torch_cpu_baseline(pipe, H, W, params, 2 * args.cpu_rows,
                                                        result["parity"])
        result["psnr_vs_ref"] = result["parity"]["psnr_fine_rgb"]
    if rank == 0 and world == 1 and not c4 and not args.no_gt and os.path.exists(GT_PATH):
        result["psnr_vs_gt"] = psnr_vs_gt(pipe, H, W, result.get("parity"))
    del pipe
    if args.precision != "fp32" and not args.no_fp32_run:
        _, el32, roof32 = measure("fp32")
        result["fp32_mfma"] = {"value": rays / el32 / 1e6, "ms_per_step": el32 / args.steps * 1e3,
                               "dtype": DTYPES["fp32"], "roofline": roof32}
    if world == 1 and not c4 and not args.no_c3:
        # the frames' multi-GB buffers are still cached by torch's allocator: give
        # them back before the 1024-ray step settles into its own working set
        torch.cuda.empty_cache()
        c3 = bench_train(args, world, rank, dev, params, data, barrier, steps=20, warmup=10,
                         emit=False)
        result["c3_train_step"] = {k: c3[k] for k in ("metric", "value", "unit", "ms_per_step",
                                                      "steps", "warmup", "dtype", "config",
                                                      "roofline", "loss_last")}
    if "parity" in result:
        result["parity"].pop("_maps", None)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


def bench_train(args, world, rank, dev, params, data, barrier, steps=None, warmup=None,
                emit=True):
    """C3: NerfTrainer.step on 1024 random lego-camera pixels per rank (synthetic
    targets), data parallel over ranks (weak scaling). emit=False: return the
    record (the default bench run's "c3_train_step" sub-record) instead of
    printing it."""
    import torch
    import torch.distributed as dist
    from nerfhip.render import NerfPipeline
    from nerfhip.train import NerfTrainer, camera_rays_at
    cams = np.load(os.path.join(REPO, "tests", "golden", "lego_test_cameras.npz"))
    H = W = 800
    focal = 0.5 * W / np.tan(0.5 * float(cams["camera_angle_x"]))
    poses = torch.from_numpy(cams["poses"].astype(np.float32)).to(dev)
    K = torch.tensor([[focal, 0, W / 2], [0, focal, H / 2], [0, 0, 1]], dtype=torch.float32,
                     device=dev)
    launch = "graph" if args.train_graph else args.train_launch
    if launch == "auto" and (world > 1 or args.train_mlp != "x3"):
        launch = "eager"   # the graph step is calibrated on one rank with the HIP ops only
    group = dist.group.WORLD if world > 1 else None
    gen = torch.Generator(device=dev).manual_seed(1000 + rank)
    nrays = 1024

    def batch():
        pix = torch.randint(0, H * W, (nrays,), device=dev, generator=gen)
        view = torch.randint(0, poses.shape[0], (nrays,), device=dev, generator=gen)
        ro, rd = camera_rays_at(poses, K, pix, view, W)
        target = torch.rand((nrays, 3), device=dev, generator=gen)
        return ro, rd, target

    n_steps = args.steps if steps is None else steps
    n_warm = max(3, args.warmup if warmup is None else warmup)   # the graph captures step 3
    batches = [batch() for _ in range(n_warm + n_steps)]

    def warmed(graph):
        tr = NerfTrainer(dev, params, mlp=args.train_mlp, graph=graph)
        for i in range(n_warm):
            tr.step(*batches[i], group=group)
        torch.cuda.synchronize()
        return tr

    calib = None
    if launch == "auto":
        # 5 steps of each launch mode on this box (same batches, separate trainers);
        # the timed steps below run the faster one from a fresh warm trainer state
        calib = {}
        for mode in ("eager", "graph"):
            t = warmed(mode == "graph")
            t0 = time.perf_counter()
            for i in range(5):
                t.step(*batches[n_warm + i], group=group)
            torch.cuda.synchronize()
            calib[mode] = (time.perf_counter() - t0) / 5 * 1e3
            del t
        launch = min(calib, key=calib.get)
    graph = launch == "graph"
    tr = warmed(graph)
    barrier()
    t0 = time.perf_counter()
    for i in range(n_steps):
        losses = tr.step(*batches[n_warm + i], group=group)
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    step_s = elapsed / n_steps
    flop = 3 * NerfPipeline.MLP_FLOP_PER_SAMPLE * nrays * (64 + 192)   # fwd + 2x bwd
    result = {
        "metric": "train step: Mrays/s (1024 rays/rank/step, 64c+128f) + ms/step",
        "value": nrays * world * n_steps / elapsed / 1e6, "unit": "Mrays/s",
        "n_gpus": world, "steps": n_steps, "warmup": n_warm,
        "ms_per_step": step_s * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None,
        "dtype": DTYPES["f16x3"] if args.train_mlp == "x3" else "fp32",
        "data": data + ", synthetic targets",
        "config": {"workload": "lego train step: 1024 random pixels of the test cameras per "
                               "rank, perturb 1, training-mode u, MSE coarse+fine, clip 40, Adam",
                   "baseline_config": "configs[2]", "N_rays": nrays, "N_samples": 64,
                   "N_importance": 128, "train_mlp": args.train_mlp,
                   "step_launch": ("one HIP graph replay per step (captured on the 3rd step)"
                                   if graph else "eager (op-by-op launches)") +
                                  (f"; chosen by a 5-step calibration (ms/step: eager "
                                   f"{calib['eager']:.2f}, graph {calib['graph']:.2f})"
                                   if calib else ""),
                   "parallelism": f"data parallel x{world} (RCCL all-reduce)"},
        "roofline": train_roofline(args.train_mlp, flop, step_s),
        "loss_last": float(losses["loss"].item()),
    }
    if not emit:
        return result
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return result


def train_roofline(mlp, flop, step_s):
    """C3: the whole step's algorithmic MLP FLOP/s (fwd + 2x bwd) against the MFMA
    peak of the arithmetic the MLP GEMMs run on (x3: 3 FP16 MFMA products per
    FP32 product; torch: FP32 hipBLASLt)."""
    algo = flop / step_s / 1e12
    if mlp == "x3":
        kernel, achieved, peak, unit = ("whole step (x3_layer_kernel + x3_wgrad_kernel dominate)",
                                        3 * algo, FP16_MFMA_PEAK_TFLOPS,
                                        "TFLOP/s (FP16 MFMA, 3 per FP32 product)")
    else:
        kernel, achieved, peak, unit = ("whole step (MLP GEMMs on hipBLASLt dominate)", algo,
                                        FP32_MFMA_PEAK_TFLOPS, "TFLOP/s")
    return {"bound": "mfma", "kernel": kernel, "achieved": achieved, "peak": peak, "unit": unit,
            "frac": achieved / peak, "algorithmic_tflops": algo,
            "frac_of_fp32_peak": algo / FP32_MFMA_PEAK_TFLOPS, "traffic": None,
            "flop_per_step": flop}


DTYPES = {"fp32": "fp32",
          "f16x3": "fp32 operands as 3-term fp16 splits on fp16 mfma, fp32 accumulate"}


def roofline(precision, timer, elapsed, world, H, W, pmc_workload=True):
    """Dominant kernel (the fused MLP: coarse + fine launches), timed by HIP events
    recorded on the stream it is launched on. pmc_workload: the launches are the
    whole-frame C2 launches the committed PMC summary measured (else traffic is
    null: band or ERT-compacted launches were not counted)."""
    from nerfhip.render import NerfPipeline
    mlp_ms = sum(a.elapsed_time(b) for a, b, _, _ in timer)
    # ERT-compacted launches record their device-side sample count (resolved here,
    # after the timed region) and no byte figure
    mlp_samples = sum(int(s) for _, _, s, _ in timer)
    n_launch = len(timer)
    mlp_bytes = sum(b if b is not None else int(s) * 16 + NerfPipeline.MLP_WEIGHT_BYTES
                    for _, _, s, b in timer)
    flops = mlp_samples * NerfPipeline.MLP_FLOP_PER_SAMPLE
    algo_tflops = flops / (mlp_ms * 1e-3) / 1e12 if mlp_ms > 0 else 0.0
    if precision == "fp32":
        kernel, achieved, peak, unit = ("mlp_fused_kernel", algo_tflops, FP32_MFMA_PEAK_TFLOPS,
                                        "TFLOP/s")
    else:   # FP16 MFMA FLOP executed (3 per FP32 product), against the dense FP16 peak
        exec_tflops = mlp_samples * X3_EXEC_FLOP_PER_SAMPLE / (mlp_ms * 1e-3) / 1e12 \
            if mlp_ms > 0 else 0.0
        kernel, achieved, peak, unit = ("mlp_x3_kernel", exec_tflops, FP16_MFMA_PEAK_TFLOPS,
                                        "TFLOP/s (FP16 MFMA executed, 3 per FP32 product)")
    # weight bytes the kernel stages L2 -> LDS: every 128-sample tile streams the
    # whole packed network (65 x 32 KiB x3 slices; 73 x 32 KiB FP32)
    slices = 65 if precision != "fp32" else 73
    staged = sum(-(-int(s) // 128) for _, _, s, _ in timer) * slices * 32768
    return {"bound": "mfma", "kernel": kernel,
            "achieved": achieved, "peak": peak, "unit": unit,
            "frac": achieved / peak,
            "algorithmic_tflops": algo_tflops,
            "frac_of_fp32_peak": algo_tflops / FP32_MFMA_PEAK_TFLOPS,
            "traffic": pmc_traffic(H, W, kernel) if pmc_workload else None,
            "traffic_unit": "HBM bytes per launch (rocprofv3 PMC, profiles/)",
            "algorithmic_bytes_per_launch": mlp_bytes / max(1, n_launch),
            "lds_staged_bytes_per_launch": staged / max(1, n_launch),
            "lds_staging_TBps": staged / (mlp_ms * 1e-3) / 1e12 if mlp_ms > 0 else 0.0,
            "launches": n_launch,
            "avg_launch_ms": mlp_ms / max(1, n_launch),
            "flop_per_sample": NerfPipeline.MLP_FLOP_PER_SAMPLE,
            "mlp_share_of_step": (mlp_ms / world) / (elapsed * 1e3) if world == 1 else None}


def byte_kernels(stages, steps):
    """The HBM-bound stages of the frame (compositing = the reference's
    integrate, fine sampling), timed live by HIP events on their launch stream
    over the timed frames: algorithmic bytes / time against the 8 TB/s roof."""
    out = {}
    for name, e0, e1, nb in stages:
        d = out.setdefault(name, {"launches": 0, "ms": 0.0, "bytes": 0})
        d["launches"] += 1
        d["ms"] += e0.elapsed_time(e1)
        d["bytes"] += nb
    for d in out.values():
        d["ms_per_frame"] = d["ms"] / max(1, steps)
        d["GBps"] = d["bytes"] / (d["ms"] * 1e-3) / 1e9 if d["ms"] > 0 else 0.0
        d["frac_hbm"] = d["GBps"] * 1e9 / HBM_PEAK_BPS
    return out


def pmc_traffic(H, W, kernel="mlp_fused_kernel"):
    """Measured HBM bytes per MLP launch from the newest committed PMC summary
    (tools/pmc.sh + tools/pmc_summary.py) taken on this same workload, else None."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "*_pmc_summary.json"))):
        with open(f) as fh:
            doc = json.load(fh)
        wl = doc.get("workload", {})
        e = doc.get("kernels", {}).get(kernel.replace("_kernel", ""), {})
        if wl.get("H") == H and wl.get("W") == W and "hbm_bytes_per_launch" in e:
            best = e["hbm_bytes_per_launch"]
    return best


def _strip(H, W, rows):
    r0 = max(0, H // 2 - rows // 2)
    return r0, slice(r0 * W, (r0 + rows) * W)


def oracle_parity(pipe, H, W, params, rows):
    """GPU vs the parity oracle (oracle/nerf_oracle.py, the numpy restatement
    pinned to the reference's golden renders) on a bounded strip of test view 0."""
    sys.path.insert(0, REPO)
    from oracle import nerf_oracle as O
    import torch
    pose, K = lego_camera(H, W, 0)
    r0, sl = _strip(H, W, rows)
    ro, rd = O.camera_rays(H, W, pose, K)
    cfg = O.RenderConfig(N_samples=64, N_importance=128)
    t0 = time.perf_counter()
    ref, _ = O.render(rows, W, pose, K, params, cfg, rays=(ro[sl], rd[sl]))
    t_cpu = time.perf_counter() - t0
    gpu = pipe.render_image(H, W, pose, K, p0=r0 * W, n=rows * W)
    torch.cuda.synchronize()
    g = {k: v.cpu().numpy() for k, v in gpu.items()}
    n = rows * W
    par = {"strip_rows": [r0, r0 + rows], "oracle_seconds": t_cpu, **_parity(g, ref, n)}
    par["_maps"] = (g["rgb_map"].reshape(rows, W, 3), ref["rgb_map"].reshape(rows, W, 3))
    return par


def torch_cpu_baseline(pipe, H, W, params, rows, parity):
    """The reference's CPU render path timed on this host's cores: the torch-CPU
    restatement of _render_pytorch (oracle/torch_render.py: torch's own CPU
    kernels, MKL GEMMs) on a bounded strip of test view 0, with its agreement
    with the GPU on the same strip."""
    sys.path.insert(0, REPO)
    from oracle import torch_render as TR
    import torch
    pose, K = lego_camera(H, W, 0)
    r0, sl = _strip(H, W, rows)
    ro, rd = TR.camera_rays(H, W, pose, K)
    t0 = time.perf_counter()
    ref = TR.render_rays(ro[sl].contiguous(), rd[sl].contiguous(), params)
    t_cpu = time.perf_counter() - t0
    gpu = pipe.render_image(H, W, pose, K, p0=r0 * W, n=rows * W)
    torch.cuda.synchronize()
    g = {k: v.cpu().numpy() for k, v in gpu.items()}
    n = rows * W
    return {"value": n / t_cpu / 1e6, "unit": "Mrays/s", "cores": int(torch.get_num_threads()),
            "kind": "port", "seconds": t_cpu, "host_cpus": os.cpu_count(),
            "cpu_model": _cpu_model(),
            "sample": f"rows {r0}-{r0 + rows - 1} of lego test view 0 at {H}x{W} ({n} rays, "
                      f"64c+128f) rendered by oracle/torch_render.py (torch-CPU restatement of "
                      f"_render_pytorch, {torch.get_num_threads()} threads)",
            "agreement_with_gpu": {k: v for k, v in _parity(g, ref, n).items()}}


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def psnr_vs_gt(pipe, H, W, parity):
    """North_star "PSNR within 0.01 dB on lego": the evaluator's PSNR / SSIM
    (evaluators/nerf.py:465-504; nerfhip.evaluate) of the HIP render of every
    packed lego test view (data/lego/test.npz: frames 0, 8, ..., 192) against its
    ground truth, and on the parity strip the same PSNR for the HIP render and
    for the oracle's render of those rays (|dPSNR| is the north_star figure)."""
    import torch
    from nerfhip.evaluate import load_packed, psnr, ssim
    gts, _, _, frames = load_packed(GT_PATH, H, W)
    vals, ssims = [], []
    for i, fr in enumerate(frames):
        pose, K = lego_camera(H, W, i)
        rgb = pipe.render_image(H, W, pose, K)["rgb_map"].view(H, W, 3).cpu().numpy()
        vals.append(psnr(rgb, gts[i]))
        ssims.append(ssim(rgb, gts[i]))
    torch.cuda.synchronize()
    out = {"frames": [int(f) for f in frames], "psnr": vals, "psnr_mean": float(np.mean(vals)),
           "ssim_mean": float(np.mean(ssims)),
           "metric": "evaluators/nerf.py PSNR (clip to [0,1], -10 log10 mse) and SSIM, "
                     "mean over the packed test views"}
    if parity and "_maps" in parity:
        g, o = parity.pop("_maps")
        r0, r1 = parity["strip_rows"]
        gt = gts[0][r0:r1]
        pg, po = psnr(g, gt), psnr(o, gt)
        out["strip"] = {"rows": [r0, r1], "frame": int(frames[0]), "psnr_hip": pg,
                        "psnr_oracle": po, "abs_delta_db": abs(pg - po)}
    return out


def cpu_baseline_c4(pipe, H, W, params, rows):
    """ESS + ERT: the oracle on the frame's first whole 2048-ray chunks (about
    `rows` rows), fresh grid and call counter on both sides."""
    sys.path.insert(0, REPO)
    from oracle import nerf_oracle as O
    from nerfhip.synthetic import make_occupancy_grid
    import torch
    threads = _threads()
    pose, K = lego_camera(H, W, 0)
    n = max(1, rows * W // 2048) * 2048
    ro, rd = O.camera_rays(H, W, pose, K)
    grid = make_occupancy_grid(0, 128, 1.2, 0.1)
    cfg = O.RenderConfig(N_samples=64, N_importance=128, enable_ess=True, enable_ert=True,
                         ert_threshold=0.01)
    t0 = time.perf_counter()
    ref, _ = O.render(1, n, pose, K, params, cfg, grid=grid.copy(), grid_counter=0,
                      rays=(ro[:n], rd[:n]))
    t_cpu = time.perf_counter() - t0
    pipe.grid_update_counter = 0
    gpu = pipe.render_image(H, W, pose, K, p0=0, n=n)
    torch.cuda.synchronize()
    g = {k: v.cpu().numpy() for k, v in gpu.items()}
    parity = _parity(g, ref, n)
    parity["rays"] = [0, n]
    base = {"value": n / t_cpu / 1e6, "unit": "Mrays/s", "cores": int(threads), "kind": "port",
            "seconds": t_cpu,
            "sample": f"rays 0-{n - 1} ({n // 2048} whole 2048-ray chunks) of lego test frame 0 "
                      f"at {H}x{W}, 64c+128f, ESS + ERT, rendered by oracle/nerf_oracle.py"}
    return base, parity


def _threads():
    try:
        from threadpoolctl import threadpool_info
        return max([t.get("num_threads", 1) for t in threadpool_info()] or [1])
    except Exception:
        return int(os.environ.get("OMP_NUM_THREADS", "1"))


def _parity(g, ref, n):
    def mx(a, b):
        m = ~np.isnan(b)
        return float(np.abs(a[m] - b[m]).max()) if m.any() else 0.0

    mse = float(np.mean((np.clip(g["rgb_map"], 0, 1) -
                         np.clip(ref["rgb_map"].reshape(n, 3), 0, 1)) ** 2))
    return {"max_abs_err_rgb_map_0": mx(g["rgb_map_0"], ref["rgb_map_0"].reshape(n, 3)),
            "max_abs_err_depth_map_0": mx(g["depth_map_0"], ref["depth_map_0"].reshape(n)),
            "max_abs_err_rgb_map": mx(g["rgb_map"], ref["rgb_map"].reshape(n, 3)),
            "psnr_fine_rgb": (float("inf") if mse == 0 else -10 * np.log10(mse))}


if __name__ == "__main__":
    main()
