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
TRAIN_PATH = os.path.join(REPO, "data", "lego", "train.npz")


COLL = ["RCCL"]             # the collective library named in "parallelism"
POSE_STRIDE = [GT_STRIDE]   # --all-poses: 1 (every one of the 200 test poses)


def lego_camera(H, W, idx):
    """Test view POSE_STRIDE * idx (mod 200): by default the frames 0, 8, ..., 192
    whose ground truth is packed; with --all-poses every test pose in turn."""
    cams = np.load(os.path.join(REPO, "tests", "golden", "lego_test_cameras.npz"))
    poses, angle = cams["poses"], float(cams["camera_angle_x"])
    focal = 0.5 * W / np.tan(0.5 * angle)            # blender.py:41-42
    K = np.array([[focal, 0, W / 2], [0, focal, H / 2], [0, 0, 1]], np.float32)
    return poses[(POSE_STRIDE[0] * idx) % len(poses)], K


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
    ap.add_argument("--config", default="c2", choices=["c2", "c3", "c4", "c5", "dist-check"],
                    help="c2: lego 800x800 64c+128f (BASELINE configs[1], the headline); "
                         "c3: train step, 1024 rays/rank (configs[2]); "
                         "c4: c2 with ESS + ERT (configs[3], lego.yaml:96-99); "
                         "c5: the lego test set (the 25 packed views cycled, one per step, or "
                         "with --all-poses all 200 test poses; PSNR/SSIM over the --gt-path "
                         "views from the sharded renders, configs[4]); dist-check: the "
                         "launcher and the timed region's collectives alone (no render: "
                         "tests/test_bench_launch.py runs it on the CPU over gloo)")
    ap.add_argument("--no-c4", action="store_true",
                    help="skip the C4 (ESS + ERT) sub-record of the default run")
    ap.add_argument("--checkpoint", default=None,
                    help="trained weights (a reference-format .pth or model dir); default: "
                         "checkpoints/lego (trained by tools/train_lego.py) when present")
    ap.add_argument("--synthetic", action="store_true",
                    help="synthetic generator weights even when the trained checkpoint exists")
    ap.add_argument("--no-gt", action="store_true",
                    help="skip the PSNR/SSIM-vs-ground-truth renders (profiling runs)")
    ap.add_argument("--no-perturb", action="store_true",
                    help="skip the perturb-1 eval timing reported under 'c2_perturb'")
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
    ap.add_argument("--all-poses", action="store_true",
                    help="time every one of the 200 lego test poses in turn (c5: --steps 200 "
                         "is the whole test split) instead of the 25 packed views")
    ap.add_argument("--gt-path", default=GT_PATH,
                    help="packed ground-truth views for psnr_vs_gt (tools/pack_lego.py; "
                         "data/lego/test_all.npz: all 200 test views)")
    args = ap.parse_args()
    if args.all_poses:
        POSE_STRIDE[0] = 1

    # `python bench.py --gpus N` with no torchrun environment starts its own N
    # ranks (one process per GPU) before this process touches the GPU
    rc = self_launch(args)
    if rc is not None:
        sys.exit(rc)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # NERF_DIST_BACKEND=gloo + more ranks than GPUs: a rehearsal of the N > 1 path
    # (every collective, barrier and max-over-ranks of the timed region) on a
    # one-GPU box, ranks sharing the device; the driver's runs use RCCL ("nccl"),
    # one rank per GPU.
    backend = os.environ.get("NERF_DIST_BACKEND", "nccl")
    COLL[0] = "RCCL" if backend == "nccl" else backend
    err = launch_mismatch(args.gpus, world, backend, args.config)
    if err:
        print(f"bench.py: {err}", file=sys.stderr)
        sys.exit(2)
    if args.config == "dist-check":
        return dist_check(args, world, rank, backend)

    from nerfhip import _lib
    from nerfhip.render import NerfPipeline
    from nerfhip.synthetic import make_occupancy_grid, make_params

    if backend != "nccl":
        local %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

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
    c5 = args.config == "c5"
    if args.config == "c3":
        return bench_train(args, world, rank, dev, params, data, barrier)

    def make_pipe(precision, ess_ert):
        pipe = NerfPipeline(dev, N_samples=64, N_importance=128, near=2.0, far=6.0,
                            mlp_precision=precision, enable_ess=ess_ert, enable_ert=ess_ert,
                            ert_threshold=0.01, ert_segment=args.ert_segment)
        pipe.set_weights(params)
        if ess_ert:
            pipe.set_grid(make_occupancy_grid(0, 128, 1.2, 0.1))
        return pipe

    def frame_fn(pipe, ess_ert, perturb=False):
        return make_frame_fn(pipe, H, W, rank, world, dev, ess_ert, perturb)

    shard_stats = {}

    def measure(precision, ess_ert, steps, warmup, perturb=False):
        """warmup + K timed frames (barrier + sync both sides, max over ranks)."""
        pipe = make_pipe(precision, ess_ert)
        frame = frame_fn(pipe, ess_ert, perturb)
        for i in range(warmup):
            frame(*lego_camera(H, W, i))
        torch.cuda.synchronize()
        barrier()
        pipe.replayed_chunks = 0
        pipe.timer = []
        pipe.stage_timer = []
        pipe.ert_stats = []
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            frame(*lego_camera(H, W, warmup + i))
        torch.cuda.synchronize()
        barrier()
        elapsed = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        timer, pipe.timer = pipe.timer, None
        stages, pipe.stage_timer = pipe.stage_timer, None
        shard_stats[(ess_ert, perturb)] = shard_report(pipe, timer, steps, H, W, rank, world,
                                                       ess_ert)
        roof = roofline(precision, timer, elapsed, world, H, W,
                        pmc_workload=world == 1 and not ess_ert and not perturb)
        roof["byte_kernels"] = byte_kernels(stages, steps)
        if precision == "f16x3" and not ess_ert and not perturb:
            roof.update(held_clock(pipe, H, W, roof["achieved"], roof["peak"]))
        return pipe, elapsed, roof

    pipe, elapsed, roof = measure(args.precision, c4, args.steps, args.warmup)
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
        "config": {"workload": (("lego 800x800 test set (all 200 test poses in turn), "
                                 if args.all_poses else
                                 "lego 800x800 test set (the 25 packed test views 0, 8, ..., "
                                 "192 cycled), ") if c5 else
                                "lego 800x800, ") + "64 coarse + 128 fine samples, 1 frame per step "
                               "(test poses cycled), " +
                               ("ESS + ERT on (threshold 0.01, synthetic occupancy grid, "
                                "2048-ray chunks)" if c4 else "ESS/ERT off") + ", perturb 0, eval",
                   "baseline_config": {"c2": "configs[1]", "c4": "configs[3]",
                                       "c5": "configs[4]"}[args.config],
                   "H": H, "W": W, "N_samples": 64, "N_importance": 128,
                   "mlp_precision": args.precision,
                   "parallelism": (f"2048-ray chunks dealt round-robin x{world} (chunk c -> rank "
                                   f"c mod {world}) + {COLL[0]} all-gather of pixels" if c4 else
                                   f"row-band tiles x{world} + {COLL[0]} all-gather of pixels")},
        "roofline": roof,
        "build_id": _lib.build_id(),
    }
    if c4:
        result["ert_compaction"] = ert_report(pipe, rays, world, args.ert_segment, dev)
    if world > 1 and rank == 0:
        result["shards"] = shard_stats[(c4, False)]
    cpu = host_cpus()
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        torch.set_num_threads(cpu["threads_used"])
        if c4:
            result["cpu_baseline"], result["parity"] = cpu_baseline_c4(
                make_pipe(args.precision, True), H, W, params, args.cpu_rows, cpu)
        else:
            result["parity"] = oracle_parity(pipe, H, W, params, args.cpu_rows)
            result["cpu_baseline"] = torch_cpu_baseline(pipe, H, W, params, cpu,
                                                        result["parity"])
            result["cpu_baseline_c1"] = torch_cpu_baseline_c1(params, cpu, dev)
        result["psnr_vs_ref"] = result["parity"]["psnr_fine_rgb"]
    if rank == 0 and world == 1 and not c5:
        # the whole frame against the reference's OWN render of it (make_ref_frames.py)
        if c4:
            pipe_c4 = make_pipe(args.precision, True)
            result["parity_vs_reference_frame"] = reference_frame_parity(
                pipe_c4, "r2_c4_frame16", H, W, ckpt)
            del pipe_c4
        else:
            result["parity_vs_reference_frame"] = reference_frame_parity(
                pipe, "r0_c2_frame0", H, W, ckpt)
    if (c5 or (world == 1 and not c4)) and not args.no_gt and os.path.exists(args.gt_path):
        ev = testset_eval(frame_fn(pipe, c4), H, W, rank, result.get("parity"), args.gt_path)
        if rank == 0:
            result["psnr_vs_gt"] = ev
    del pipe
    if args.precision != "fp32" and not args.no_fp32_run and not c5:
        _, el32, roof32 = measure("fp32", c4, args.steps, args.warmup)
        result["fp32_mfma"] = {"value": rays / el32 / 1e6, "ms_per_step": el32 / args.steps * 1e3,
                               "dtype": DTYPES["fp32"], "roofline": roof32}
    if args.config == "c2" and not args.no_c4:
        # BASELINE configs[3] timed in the same run: ESS + ERT, interleaved chunks
        torch.cuda.empty_cache()
        c4_steps = max(1, min(args.steps, 5))
        p4, el4, roof4 = measure(args.precision, True, c4_steps, 1)
        rays4 = H * W * c4_steps
        rec = {"metric": "Mrays/s + ms/frame, lego 800x800 (64c+128f) with ESS + ERT",
               "value": rays4 / el4 / 1e6, "unit": "Mrays/s", "steps": c4_steps, "warmup": 1,
               "ms_per_step": el4 / c4_steps * 1e3, "dtype": DTYPES[args.precision],
               "config": {"workload": "lego 800x800, 64c+128f, ESS + ERT (threshold 0.01, "
                                      "synthetic occupancy grid make_occupancy_grid(0, 128, 1.2, "
                                      "0.1) self-updated by the reference's rule), perturb 0, "
                                      "eval, 1 frame per step (test poses cycled)",
                          "baseline_config": "configs[3]",
                          "parallelism": f"2048-ray chunks round-robin x{world} + {COLL[0]} "
                                         f"all-gather"},
               "roofline": {k: roof4[k] for k in ("kernel", "achieved", "peak", "unit", "frac",
                                                  "avg_launch_ms", "launches")},
               "ert_compaction": ert_report(p4, rays4, world, args.ert_segment, dev)}
        del p4
        if rank == 0 and world == 1:
            p4 = make_pipe(args.precision, True)
            rec["parity_vs_reference_frame"] = reference_frame_parity(
                p4, "r2_c4_frame16", H, W, ckpt)
            del p4
        result["c4_ess_ert"] = rec
    if args.config == "c2" and not args.no_c4 and not args.no_perturb:
        # lego.yaml's own eval configuration (run.py --type evaluate): ESS + ERT
        # at 0.01 (lego.yaml:96-99) AND perturb 1 (:22): per-ray jittered depths
        # after the ESS fold (VR:1080-1085)
        torch.cuda.empty_cache()
        y_steps = max(1, min(args.steps, 5))
        py, ely, roofy = measure(args.precision, True, y_steps, 1, perturb=True)
        raysy = H * W * y_steps
        rec = {"metric": "Mrays/s + ms/frame, lego 800x800 (64c+128f), lego.yaml eval: ESS + "
                         "ERT + perturb 1",
               "value": raysy / ely / 1e6, "unit": "Mrays/s", "steps": y_steps, "warmup": 1,
               "ms_per_step": ely / y_steps * 1e3, "dtype": DTYPES[args.precision],
               "config": {"workload": "lego 800x800, 64c+128f, ESS + ERT (threshold 0.01, "
                                      "occupancy grid sphere 1.2 | 10 % noise as the Renderer "
                                      "draws it, self-updated by the reference's rule), perturb "
                                      "1 (one [H*W, 64] draw per frame), eval, 1 frame per step "
                                      "(test poses cycled)",
                          "baseline_config": "configs[3] as run.py --type evaluate renders it "
                                             "(lego.yaml)",
                          "parallelism": f"2048-ray chunks round-robin x{world} + {COLL[0]} "
                                         f"all-gather"},
               "roofline": {k: roofy[k] for k in ("kernel", "achieved", "peak", "unit", "frac",
                                                  "avg_launch_ms", "launches")},
               "ert_compaction": ert_report(py, raysy, world, args.ert_segment, dev)}
        del py
        if rank == 0 and world == 1:
            py = make_pipe(args.precision, True)
            rec["parity_vs_reference_frame"] = reference_frame_parity(
                py, "r3_c4_yaml_frame24", H, W, ckpt)
            del py
        result["lego_yaml_eval"] = rec
    if args.config == "c2" and not args.no_perturb:
        # what `run.py --type evaluate` with lego.yaml runs: perturb 1 at eval
        # (lego.yaml:22, VR:228-235), per-ray jittered coarse depths
        torch.cuda.empty_cache()
        pp_steps = max(1, min(args.steps, 5))
        _, elp, roofp = measure(args.precision, False, pp_steps, 1, perturb=True)
        raysp = H * W * pp_steps
        result["c2_perturb"] = {
            "metric": "Mrays/s + ms/frame, lego 800x800 (64c+128f), perturb 1 at eval",
            "value": raysp / elp / 1e6, "unit": "Mrays/s", "steps": pp_steps, "warmup": 1,
            "ms_per_step": elp / pp_steps * 1e3, "dtype": DTYPES[args.precision],
            "config": {"workload": "lego 800x800, 64c+128f, ESS/ERT off, perturb 1 (the "
                                   "stratified jitter drawn on the device per band inside the "
                                   "frame, one [n, 64] uniform draw), eval-mode fine u, 1 frame "
                                   "per step (test poses cycled)",
                       "baseline_config": "configs[1] as run.py --type evaluate renders it",
                       "parallelism": f"row-band tiles x{world} + {COLL[0]} all-gather of pixels"},
            "roofline": {k: roofp[k] for k in ("kernel", "achieved", "peak", "unit", "frac",
                                               "avg_launch_ms", "launches", "mlp_share_of_step")}}
    if world == 1 and args.config == "c2" and not args.no_c3:
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
        result["host"] = cpu
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


def visible_gpus():
    """ROCm devices this process may use, counted without initialising the GPU
    (torch.cuda.device_count() on this image reads the device list only)."""
    import torch
    return torch.cuda.device_count()


def launch_mismatch(gpus, world, backend, config):
    """Why this rank must not run, or None: --gpus has to equal the launch's
    world size, and with RCCL every rank needs a GPU of its own. A mismatch
    exits non-zero rather than timing fewer ranks than asked for."""
    if world != gpus:
        return (f"--gpus {gpus} but WORLD_SIZE {world}: launch N ranks with --gpus N "
                f"(torchrun --nproc-per-node N, or python bench.py --gpus N alone)")
    if backend == "nccl" and config != "dist-check":
        n = visible_gpus()
        if gpus > n:
            return (f"--gpus {gpus} but {n} visible GPU(s): RCCL needs one GPU per rank "
                    f"(NERF_DIST_BACKEND=gloo rehearses N ranks on fewer GPUs)")
    return None


def self_launch(args, argv=None):
    """`python bench.py --gpus N` (N > 1) outside torchrun: start N rank processes
    of this script with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 /
    MASTER_PORT set, one per visible GPU, and return the exit status for the
    parent (the first failing rank's, else 0); rank 0 prints the JSON line. The
    parent never touches the GPU: it counts devices, starts the ranks and waits.
    Returns None when this process is itself a rank (WORLD_SIZE set) or N is 1."""
    import signal
    import socket
    import subprocess
    if "WORLD_SIZE" in os.environ or args.gpus <= 1:
        return None
    backend = os.environ.get("NERF_DIST_BACKEND", "nccl")
    err = launch_mismatch(args.gpus, args.gpus, backend, args.config)
    if err:
        print(f"bench.py: {err}", file=sys.stderr)
        return 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    argv = sys.argv[1:] if argv is None else argv
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv,
                                      env=env, start_new_session=True))
    # a SIGTERM to the launcher (a driver's time limit) takes the ranks down too
    signal.signal(signal.SIGTERM, lambda *_: sys.exit(143))
    rc = 0
    try:
        pending = list(procs)
        while pending:
            for p in list(pending):
                code = p.poll()
                if code is None:
                    continue
                pending.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code
                    # one rank failed: the others would wait in a collective forever
                    for q in pending:
                        os.killpg(q.pid, signal.SIGTERM)
            time.sleep(0.2)
    finally:
        for p in procs:
            if p.poll() is None:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait()
    return rc


def dist_check(args, world, rank, backend):
    """--config dist-check: the multi-rank skeleton of every bench line without a
    render -- process group, W untimed and K timed steps of one small all-reduce
    bracketed by barriers, the elapsed time maxed over ranks, one JSON line on
    rank 0 with n_gpus = the world size. gloo runs it on the CPU
    (tests/test_bench_launch.py)."""
    import torch
    import torch.distributed as dist
    dev = torch.device("cpu")
    if backend == "nccl":
        dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
        torch.cuda.set_device(dev)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    x = torch.ones(1024, device=dev)

    def step():
        if world > 1:
            dist.all_reduce(x)
            x.div_(world)

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if rank == 0:
        print(json.dumps({"metric": "dist-check: all-reduce steps/s (launcher check, no render)",
                          "value": args.steps / max(elapsed, 1e-9), "unit": "steps/s",
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": elapsed / max(1, args.steps) * 1e3,
                          "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
                          "dtype": "fp32", "data": "synthetic",
                          "config": {"workload": "dist-check", "backend": backend,
                                     "ranks_pid": os.getpid()},
                          "allreduce_ok": bool(torch.all(x == 1.0).item())}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def make_frame_fn(pipe, H, W, rank, world, dev, ess_ert, perturb=False):
    """One sharded frame (frame(pose, K) -> the assembled maps on every rank):
    C2 row bands; C4 2048-ray chunks dealt round-robin (chunk c -> rank c mod P,
    SURVEY §8e), grid self-updates replayed. perturb: the reference's eval-mode
    stratified jitter (perturb 1, lego.yaml:22; VR:228-235), one [n, 64] uniform
    draw per band on the device (torch's Philox) inside the frame, so the coarse
    pass reads per-ray depth rows; with ESS + ERT (lego.yaml's own eval
    configuration) one [H * W, 64] draw per frame from a per-frame seed, the same
    on every rank, each chunk reading its rows. tests/test_gpu_dist.py drives
    this same function from two processes."""
    from nerfhip.dist import render_frame_interleaved, render_frame_sharded
    import torch

    def band(pose, K):
        def render(p0, n):
            if not perturb:
                return pipe.render_band(H, W, pose, K, p0, n)
            if n == 0:
                return {}
            tr = torch.rand((n, pipe.N_samples), device=dev)
            return pipe.render_image(H, W, pose, K, t_rand=tr, p0=p0, n=n)
        return render

    count = [0]

    def frame(pose, K):
        if ess_ert:
            tr = None
            if perturb:   # the frame's draws, the same on every rank (seeded per frame)
                g = torch.Generator(device=dev).manual_seed(7000 + count[0])
                tr = torch.rand((H * W, pipe.N_samples), device=dev, generator=g)
            count[0] += 1
            return render_frame_interleaved(
                lambda cs: pipe.render_chunks(H, W, pose, K, cs, t_rand=tr), H, W, rank, world,
                dev)
        return render_frame_sharded(band(pose, K), H, W, rank, world, dev)
    return frame


def bench_train(args, world, rank, dev, params, data, barrier, steps=None, warmup=None,
                emit=True):
    """C3: NerfTrainer.step on 1024 random pixels of one random lego train view
    per rank and step, their white-composited ground truth as the targets (the
    reference's training batch: blender.py:60-84 images, lego.yaml:14 N_rays
    1024, :19 no_batching; trainers/nerf.py:39-76 MSE coarse + fine), data
    parallel over ranks (weak scaling). The 100 train views are decoded from
    data/lego/train.npz (tools/pack_lego.py) and resident in HBM before timing;
    without that file the step falls back to test-camera rays with uniform
    random targets (same FLOPs; `data` says which). emit=False: return the
    record (the default bench run's "c3_train_step" sub-record) instead of
    printing it."""
    import torch
    import torch.distributed as dist
    from nerfhip.render import NerfPipeline
    from nerfhip.train import NerfTrainer, camera_rays_at
    H = W = 800
    images = None
    if os.path.exists(TRAIN_PATH):
        from nerfhip.evaluate import load_packed
        imgs, tposes, focal, _ = load_packed(TRAIN_PATH)
        assert imgs.shape[1:3] == (H, W), imgs.shape
        images = torch.from_numpy(imgs).to(dev)
        poses = torch.from_numpy(np.ascontiguousarray(tposes, dtype=np.float32)).to(dev)
        del imgs
        source = (f"{poses.shape[0]} lego train views (data/lego/train.npz, white-composited "
                  f"ground truth as targets, {images.numel() * 4 / 2 ** 30:.2f} GiB resident)")
    else:
        cams = np.load(os.path.join(REPO, "tests", "golden", "lego_test_cameras.npz"))
        focal = 0.5 * W / np.tan(0.5 * float(cams["camera_angle_x"]))
        poses = torch.from_numpy(cams["poses"].astype(np.float32)).to(dev)
        source = "lego test cameras with uniform random targets (data/lego/train.npz absent)"
    K = torch.tensor([[focal, 0, W / 2], [0, focal, H / 2], [0, 0, 1]], dtype=torch.float32,
                     device=dev)
    launch = "graph" if args.train_graph else args.train_launch
    if launch == "auto" and (world > 1 or args.train_mlp != "x3"):
        launch = "eager"   # the graph step is calibrated on one rank with the HIP ops only
    group = dist.group.WORLD if world > 1 else None
    gen = torch.Generator(device=dev).manual_seed(1000 + rank)
    nrays = 1024

    def batch():
        if images is None:
            pix = torch.randint(0, H * W, (nrays,), device=dev, generator=gen)
            view = torch.randint(0, poses.shape[0], (nrays,), device=dev, generator=gen)
            ro, rd = camera_rays_at(poses, K, pix, view, W)
            return ro, rd, torch.rand((nrays, 3), device=dev, generator=gen)
        # one train view per step (no_batching), 1024 of its pixels
        view = torch.randint(0, poses.shape[0], (1,), device=dev, generator=gen).expand(nrays)
        pix = torch.randint(0, H * W, (nrays,), device=dev, generator=gen)
        ro, rd = camera_rays_at(poses, K, pix, view, W)
        return ro, rd, images[view, pix // W, pix % W].contiguous()

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
        "data": data + "; rays and targets: " + source,
        "config": {"workload": "lego train step: 1024 random pixels of one random train view "
                               "per rank and step, their ground truth as targets, perturb 1, "
                               "training-mode u, MSE coarse+fine, clip 40, Adam"
                               if images is not None else
                               "lego train step: 1024 random pixels of the test cameras per "
                               "rank (train views absent), perturb 1, training-mode u, MSE "
                               "coarse+fine, clip 40, Adam",
                   "baseline_config": "configs[2]", "N_rays": nrays, "N_samples": 64,
                   "N_importance": 128, "train_mlp": args.train_mlp,
                   "step_launch": ("one HIP graph replay per step (captured on the 3rd step)"
                                   if graph else "eager (op-by-op launches)") +
                                  (f"; chosen by a 5-step calibration (ms/step: eager "
                                   f"{calib['eager']:.2f}, graph {calib['graph']:.2f})"
                                   if calib else ""),
                   "parallelism": f"data parallel x{world} ({COLL[0]} all-reduce)"},
        "roofline": train_roofline(args.train_mlp, flop, step_s),
        "loss_last": float(losses["loss"].item()),
        "build_id": __import__("nerfhip._lib", fromlist=["build_id"]).build_id(),
    }
    if not emit:
        return result
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return result


def held_clock(pipe, H, W, achieved, peak, reps=3):
    """The shader clock the chip holds while mlp_x3_kernel runs, measured right
    after the timed frames (chip warm, same weights, a frame's coarse pass:
    800 x 800 rays x 64 depths) by the kernel's diagnostic twin
    (nerf_mlp_forward_x3_clock: d s_memtime / d s_memrealtime x 100 MHz per
    workgroup, median; MI355X_MICROARCH.md DVFS give-back item 6), and the
    kernel's fraction of the dense FP16 MFMA peak at that clock (the nominal
    peak is quoted at 2.4 GHz)."""
    import torch
    from nerfhip._lib import call, ptr, stream_of
    dev = pipe.device
    ro, rd = pipe.camera_rays(H, W, *lego_camera(H, W, 0))
    n, S = ro.shape[0], 64
    z = torch.linspace(2.0, 6.0, S, device=dev)
    raw = torch.empty((n * S, 4), device=dev)
    clk = torch.zeros(4 * 4096, device=dev, dtype=torch.int64)
    trace = torch.zeros(512 * 4, device=dev, dtype=torch.int64)
    ghz = []
    for _ in range(reps):
        clk.zero_()
        trace.zero_()
        call("nerf_mlp_forward_x3_clock", ptr(pipe.coarse[0]), ptr(pipe.coarse[1]), ptr(ro),
             ptr(rd), ptr(z), 0, n, S, ptr(raw), ptr(clk), clk.numel(), ptr(trace),
             stream_of(dev))
        torch.cuda.synchronize()
        c = clk.view(-1, 4).cpu().numpy().astype(np.float64)
        c = c[c[:, 3] > c[:, 2]]
        ghz.append(float(np.median((c[:, 1] - c[:, 0]) / (c[:, 3] - c[:, 2]) * 0.1)))
    f = float(np.median(ghz))
    # the tile-start share: sample loads + encoding before the first MFMA, of the
    # tile's cycles (workgroups 0-3, their first 32 tiles, the last run)
    t = trace.view(-1, 4).cpu().numpy().astype(np.float64)
    t = t[(t[:, 2] > t[:, 0]) & (t[:, 1] >= t[:, 0])]
    start = float(np.median((t[:, 1] - t[:, 0]) / (t[:, 2] - t[:, 0]))) if len(t) else None
    return {"held_clock_ghz": f, "held_clock_runs_ghz": ghz,
            "peak_at_held_clock": peak * f / 2.4, "frac_at_held_clock": achieved / (peak * f / 2.4),
            "tile_start_share": start,
            "tile_cycles": float(np.median(t[:, 2] - t[:, 0])) if len(t) else None}


def train_roofline(mlp, flop, step_s):
    """C3: the whole step's algorithmic MLP FLOP/s (fwd + 2x bwd) against the MFMA
    peak of the arithmetic the MLP GEMMs run on (x3: 3 FP16 MFMA products per
    FP32 product; torch: FP32 hipBLASLt)."""
    algo = flop / step_s / 1e12
    if mlp == "x3":
        kernel, achieved, peak, unit = ("whole step (mlp_x3_train_kernel, mlp_x3_bwd_kernel and "
                                        "x3_wgrad_batch_kernel dominate)",
                                        3 * algo, FP16_MFMA_PEAK_TFLOPS,
                                        "TFLOP/s (FP16 MFMA, 3 per FP32 product)")
    else:
        kernel, achieved, peak, unit = ("whole step (MLP GEMMs on hipBLASLt dominate)", algo,
                                        FP32_MFMA_PEAK_TFLOPS, "TFLOP/s")
    out = {"bound": "mfma", "kernel": kernel, "achieved": achieved, "peak": peak, "unit": unit,
           "frac": achieved / peak, "algorithmic_tflops": algo,
           "frac_of_fp32_peak": algo / FP32_MFMA_PEAK_TFLOPS, "traffic": None,
           "flop_per_step": flop}
    c3 = c3_pmc_summary() if mlp == "x3" else None
    if c3:
        # measured HBM bytes per step (rocprofv3 PMC, profiles/*_c3_pmc_summary.json):
        # the step moves every activation and its gradient through HBM once each way
        out.update(traffic=c3["hbm_bytes_per_step"], traffic_unit="HBM bytes per step (PMC)",
                   hbm_TBps=c3["hbm_bytes_per_step"] / step_s / 1e12,
                   hbm_frac=c3["hbm_bytes_per_step"] / step_s / HBM_PEAK_BPS,
                   kernels_hbm_bytes_per_step={
                       k: round(v["hbm_bytes_per_step"]) for k, v in c3["kernels"].items()
                       if v["hbm_bytes_per_step"] > 1e8})
    return out


def c3_pmc_summary():
    """The newest committed C3 PMC summary (tools/pmc_step_summary.py), else None."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "*_c3_pmc_summary.json"))):
        with open(f) as fh:
            best = json.load(fh)
    return best


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
            # the share of the kernel's cycles its MFMA pipes were busy (PMC, committed
            # summary of the same workload): the clock-independent view of `frac`
            "mfma_busy_pmc": pmc_entry(H, W, kernel, "mfma_busy_frac") if pmc_workload else None,
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


def pmc_entry(H, W, kernel="mlp_fused_kernel", key="hbm_bytes_per_launch"):
    """A measured per-launch figure of the MLP kernel from the newest committed PMC
    summary (tools/pmc.sh + tools/pmc_summary.py) taken on this same workload,
    else None."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "*_pmc_summary.json"))):
        with open(f) as fh:
            doc = json.load(fh)
        wl = doc.get("workload", {})
        e = doc.get("kernels", {}).get(kernel.replace("_kernel", ""), {})
        if wl.get("H") == H and wl.get("W") == W:
            if key in e:
                best = e[key]
            elif key == "mfma_busy_frac" and e.get("GRBM_GUI_ACTIVE"):
                # SQ_VALU_MFMA_BUSY_CYCLES sums over the 1024 SIMDs, GRBM_GUI_ACTIVE
                # over the 8 XCDs (MI355X_MICROARCH.md)
                best = e["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024.0 / (e["GRBM_GUI_ACTIVE"] / 8.0)
    return best


def pmc_traffic(H, W, kernel="mlp_fused_kernel"):
    return pmc_entry(H, W, kernel)


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


def torch_cpu_baseline(pipe, H, W, params, cpu, parity):
    """The reference's CPU render path timed on this host's cores: the torch-CPU
    restatement of _render_pytorch (oracle/torch_render.py: torch's own CPU
    kernels, MKL GEMMs) on a bounded strip of test view 0 (sized to ~10-30 s on
    the threads used), with its agreement with the GPU on the same strip."""
    sys.path.insert(0, REPO)
    from oracle import torch_render as TR
    import torch
    rows = int(min(200, max(48, 3 * cpu["threads_used"])))
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
            "kind": "port", "seconds": t_cpu, "host": cpu,
            "sample": f"rows {r0}-{r0 + rows - 1} of lego test view 0 at {H}x{W} ({n} rays, "
                      f"64c+128f) rendered by oracle/torch_render.py (torch-CPU restatement of "
                      f"_render_pytorch) on {torch.get_num_threads()} threads",
            "agreement_with_gpu": {k: v for k, v in _parity(g, ref, n).items()}}


def torch_cpu_baseline_c1(params, cpu, dev):
    """BASELINE configs[0] / SURVEY §8d "C1 is timed fully": lego 400x400, 64
    coarse samples, no fine pass, ESS/ERT off -- the whole frame through the
    torch-CPU restatement on the host's cores (the reference's run.py:36-42
    times render(batch) the same way: wall clock around one frame), next to the
    HIP pipeline's time for the same frame."""
    sys.path.insert(0, REPO)
    from oracle import torch_render as TR
    import torch
    from nerfhip.render import NerfPipeline
    H = W = 400
    pose, K = lego_camera(H, W, 0)
    ro, rd = TR.camera_rays(H, W, pose, K)
    t0 = time.perf_counter()
    ref = TR.render_rays(ro, rd, params, N_importance=0)
    t_cpu = time.perf_counter() - t0
    pipe = NerfPipeline(dev, N_samples=64, N_importance=0)
    pipe.set_weights(params)
    pipe.render_image(H, W, pose, K)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        g = pipe.render_image(H, W, pose, K)
    torch.cuda.synchronize()
    t_gpu = (time.perf_counter() - t0) / 5
    e = float(np.abs(g["rgb_map_0"].cpu().numpy() - np.asarray(ref["rgb_map_0"]).reshape(-1, 3)).max())
    return {"value": H * W / t_cpu / 1e6, "unit": "Mrays/s", "seconds_per_frame": t_cpu,
            "cores": int(torch.get_num_threads()), "kind": "port",
            "sample": f"one whole lego test view 0 at {H}x{W}, 64 coarse samples, N_importance 0 "
                      f"(oracle/torch_render.py on {torch.get_num_threads()} threads)",
            "hip_ms_per_frame": t_gpu * 1e3, "hip_Mrays_s": H * W / t_gpu / 1e6,
            "max_abs_err_rgb_map_0_hip_vs_cpu": e}


def host_cpus():
    """This host's CPUs as the process sees them: logical CPUs, the affinity
    set, a cgroup CPU quota, physical cores and sockets (/proc/cpuinfo). The
    CPU baseline runs on threads_used = min(physical cores, affinity, quota)."""
    logical = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = logical
    quota = None
    for f in ("/sys/fs/cgroup/cpu.max",):
        try:
            with open(f) as fh:
                q, per = fh.read().split()[:2]
            if q != "max":
                quota = int(q) / int(per)
        except (OSError, ValueError):
            pass
    cores, sockets, phys = set(), set(), None
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("physical id"):
                    phys = line.split(":", 1)[1].strip()
                    sockets.add(phys)
                elif line.startswith("core id"):
                    cores.add((phys, line.split(":", 1)[1].strip()))
    except OSError:
        pass
    physical = len(cores) or logical
    use = min(physical, aff, max(1, int(quota)) if quota else aff)
    return {"cpu_model": _cpu_model(), "logical_cpus": logical, "sockets": len(sockets) or None,
            "physical_cores": physical, "affinity_cpus": aff, "cgroup_cpu_quota": quota,
            "threads_used": max(1, use)}


def shard_report(pipe, timer, steps, H, W, rank, world, ess_ert):
    """Per-rank work of the sharded frame (gathered to rank 0; None elsewhere):
    owned pixels / chunks, foreign grid-update chunks replayed (C4: every rank
    replays the reference's updating chunks it does not own, VR:1147-1157), and
    the MLP launches with their sample counts, per frame."""
    import torch.distributed as dist
    from nerfhip.dist import band, chunk_set
    if ess_ert:
        mine, n, _ = chunk_set(H, W, rank, world)
        owned = {"chunks": len(mine), "pixels": n}
    else:
        p0, n, _ = band(H, W, rank, world)
        owned = {"pixels": n}
    sizes = [int(t[2]) for t in (timer or [])]   # (ERT list launches: a device count)
    rec = {"rank": rank, **owned,
           "replayed_chunks_per_frame": pipe.replayed_chunks / max(1, steps),
           "mlp_launches_per_frame": len(sizes) / max(1, steps),
           "mlp_samples_per_launch_mean": float(np.mean(sizes)) if sizes else 0.0,
           "mlp_samples_per_launch_min": int(min(sizes)) if sizes else 0,
           "mlp_samples_per_launch_max": int(max(sizes)) if sizes else 0}
    if world == 1:
        return [rec]
    out = [None] * world
    dist.all_gather_object(out, rec)
    return out if rank == 0 else None


def ert_report(pipe, rays, world, segment, dev):
    """C4: MLP samples evaluated per ray with the ERT compaction, and how much of
    the frame the reference's termination rule touches (summed over ranks)."""
    import torch
    import torch.distributed as dist
    term = pipe.ert_termination()
    ev, full = pipe.evaluated_samples()
    v = [ev, full]
    for S in (64, 192):
        v += term.get(S, [0, 0, 0, 0])
    if world > 1:
        t = torch.tensor(v, device=dev, dtype=torch.float64)
        dist.all_reduce(t)
        v = [int(x) for x in t.tolist()]
    ev, full = v[0], v[1]
    out = {"evaluated_samples_per_ray": ev / rays, "full_samples_per_ray": full / rays,
           "evaluated_fraction": ev / max(1, full),
           "note": "MLP samples evaluated per ray (coarse 64 + fine 192 in full) with depth "
                   f"segments of {segment} and rays retired at T < 0.01 (their later weights are "
                   "zeroed by _raw2outputs_with_ert, VR:1115-1123)"}
    for i, (S, kind) in enumerate(((64, "coarse"), (192, "fine"))):
        n, ret, nch, chr_ = v[2 + 4 * i: 6 + 4 * i]
        out[kind] = {"rays_retired_frac": ret / max(1, n),
                     "chunks_with_retired_ray_frac": chr_ / max(1, nch), "chunks": nch}
    return out


def reference_frame_parity(pipe, name, H, W, ckpt):
    """The whole frame against the reference's OWN render of it
    (tests/golden/<name>.npz, tests/golden/make_ref_frames.py: the reference's
    Renderer on the CPU with the same checkpoint): map errors, fine-rgb pixels
    within 1e-5, PSNR of each against the frame's ground truth (evaluators/
    nerf.py:465-473) and their difference (north_star: within 0.01 dB); for C4
    also the final occupancy grid and call counter."""
    import hashlib
    import torch
    from nerfhip.evaluate import composite_white, decode_png, psnr
    from nerfhip.checkpoint import resolve
    path = os.path.join(REPO, "tests", "golden", name + ".npz")
    if not os.path.exists(path) or H != 800 or W != 800:
        return {"skipped": "no reference frame for this size"}
    z = np.load(path)
    if ckpt is None or "ckpt_sha256" not in z:
        return {"skipped": "synthetic weights: the reference frames use the lego checkpoint"}
    with open(resolve(ckpt), "rb") as f:
        if hashlib.sha256(f.read()).hexdigest() != str(z["ckpt_sha256"]):
            return {"skipped": "checkpoint differs from the one the reference frame used"}
    own = bool(z["grid_own"]) if "grid_own" in z else False
    gen = torch.Generator().manual_seed(int(z["seed"])) if int(z["perturb"]) else None
    if bool(z["ess"]):
        if own:   # the Renderer's own grid (VR:857-864), the generator's first draw
            torch.rand((128, 128, 128), generator=gen)
            bits = np.unpackbits(z["grid_init_bits"])[:128 ** 3].astype(bool)
            pipe.set_grid(bits.reshape(128, 128, 128))
        else:
            from nerfhip.synthetic import make_occupancy_grid
            gs = z["grid_spec"]
            pipe.set_grid(make_occupancy_grid(int(gs[0]), int(gs[1]), float(gs[2]),
                                              float(gs[3])))
        pipe.grid_update_counter = int(z["counter0"])
    t_rand = None
    if gen is not None:   # the reference's per-chunk perturb draws (VR:233, :1083)
        t_rand = torch.cat([torch.rand((min(2048, H * W - c), 64), generator=gen)
                            for c in range(0, H * W, 2048)]).to(pipe.device)
    pipe.ert_stats = []
    g = {k: v.cpu().numpy() for k, v in
         pipe.render_image(H, W, z["pose"], z["K"], t_rand=t_rand).items()}
    torch.cuda.synchronize()
    n = H * W
    gt = composite_white(decode_png(z["gt_png"]))
    ref_rgb = z["out_rgb_map"]
    e = np.abs(g["rgb_map"].reshape(n, 3).astype(np.float64) - ref_rgb.reshape(n, 3)).max(-1)
    mse = float(np.mean((g["rgb_map"].reshape(n, 3).astype(np.float64) - ref_rgb.reshape(n, 3)) ** 2))
    p_hip, p_ref = psnr(g["rgb_map"].reshape(H, W, 3), gt), psnr(ref_rgb, gt)
    out = {"frame": f"lego test view {int(z['frame'])}", "fixture": f"tests/golden/{name}.npz",
           "max_abs_err_rgb_map_0": float(np.abs(g["rgb_map_0"].reshape(n, 3)
                                                 - z["out_rgb_map_0"].reshape(n, 3)).max()),
           "max_abs_err_acc_map_0": float(np.abs(g["acc_map_0"].reshape(n)
                                                 - z["out_acc_map_0"].reshape(n)).max()),
           "max_abs_err_rgb_map": float(e.max()),
           "fine_rgb_pixels_within_1e-5": float(np.mean(e <= 1e-5)),
           "psnr_hip_vs_reference": float("inf") if mse == 0 else -10 * np.log10(mse),
           "psnr_vs_gt_hip": p_hip, "psnr_vs_gt_reference": p_ref, "dpsnr_db": p_hip - p_ref,
           "reference_cpu_seconds": float(z["cpu_seconds"]),
           "reference_torch_threads": int(z["torch_threads"])}
    if bool(z["ess"]):
        out["grid_final_equal"] = bool(np.array_equal(
            np.packbits(pipe.grid.cpu().numpy().astype(bool)), z["grid_final_bits"]))
        out["counter_final_equal"] = pipe.grid_update_counter == int(z["grid_counter_final"])
        pipe.evaluated_samples()
    return out


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def testset_eval(frame, H, W, rank, parity, gt_path=GT_PATH):
    """North_star "PSNR on lego" over the test set: the evaluator's PSNR / SSIM
    (evaluators/nerf.py:465-504; nerfhip.evaluate) of the HIP render of every
    packed lego test view (data/lego/test.npz: frames 0, 8, ..., 192, rendered at
    their packed poses, sharded over the ranks like the timed frames) against
    its ground truth, on rank 0; and on the parity strip the same PSNR for the
    HIP render and for the oracle's render of those rays."""
    import torch
    from nerfhip.evaluate import load_packed, psnr, ssim
    gts, poses, focal, frames = load_packed(gt_path, H, W)
    K = np.array([[focal, 0, W / 2], [0, focal, H / 2], [0, 0, 1]], np.float32)
    vals, ssims = [], []
    for i, fr in enumerate(frames):
        rgb = frame(poses[i], K)["rgb_map"]
        if rank == 0:
            rgb = rgb.reshape(H, W, 3).cpu().numpy()
            vals.append(psnr(rgb, gts[i]))
            ssims.append(ssim(rgb, gts[i]))
    torch.cuda.synchronize()
    if rank != 0:
        return None
    out = {"frames": [int(f) for f in frames], "views": len(vals), "psnr": vals,
           "psnr_mean": float(np.mean(vals)), "ssim_mean": float(np.mean(ssims)),
           "gt": os.path.relpath(gt_path, REPO),
           "metric": "evaluators/nerf.py PSNR (clip to [0,1], -10 log10 mse) and SSIM, "
                     "mean over the packed test views"}
    if parity and "_maps" in parity and int(frames[0]) == 0:
        g, o = parity.pop("_maps")
        r0, r1 = parity["strip_rows"]
        assert int(frames[0]) == 0
        gt = gts[0][r0:r1]
        pg, po = psnr(g, gt), psnr(o, gt)
        out["strip"] = {"rows": [r0, r1], "frame": int(frames[0]), "psnr_hip": pg,
                        "psnr_oracle": po, "abs_delta_db": abs(pg - po)}
    return out


def cpu_baseline_c4(pipe, H, W, params, rows, cpu):
    """ESS + ERT: the parity oracle (oracle/nerf_oracle.py) on whole 2048-ray
    chunks across the middle of test view 0 (through the object: ERT
    terminations and the chunk-wide argmax rule, VR:1115-1123), after replaying
    chunk 0 -- whose coarse ERT call updates the occupancy grid at counter 0
    (VR:1147-1155) -- on both sides, so the window sees the updated grid; each
    window chunk at its own call counter. Timed: the window on the CPU."""
    sys.path.insert(0, REPO)
    from oracle import nerf_oracle as O
    from nerfhip.synthetic import make_occupancy_grid
    import torch
    pose, K = lego_camera(H, W, 0)
    nch = max(1, rows * W // 2048)
    c0 = (H * W // 2) // 2048 - nch // 2
    a, b = c0 * 2048, (c0 + nch) * 2048
    ro, rd = O.camera_rays(H, W, pose, K)
    grid = make_occupancy_grid(0, 128, 1.2, 0.1)
    cfg = O.RenderConfig(N_samples=64, N_importance=128, enable_ess=True, enable_ert=True,
                         ert_threshold=0.01)
    O.render(1, 2048, pose, K, params, cfg, grid=grid, grid_counter=0,
             rays=(ro[:2048], rd[:2048]))                   # chunk 0: the grid update
    t0 = time.perf_counter()
    ref, _ = O.render(1, b - a, pose, K, params, cfg, grid=grid, grid_counter=2 * c0,
                      rays=(ro[a:b], rd[a:b]))
    t_cpu = time.perf_counter() - t0
    pipe.grid_update_counter = 0
    gpu = pipe.render_chunks(H, W, pose, K, list(range(c0, c0 + nch)))
    torch.cuda.synchronize()
    g = {k: v.cpu().numpy() for k, v in gpu.items()}
    n = b - a
    parity = _parity(g, ref, n)
    parity["rays"] = [a, b]
    parity["chunks"] = [c0, c0 + nch]
    parity["acc_map_mean_ref"] = float(np.nanmean(ref["acc_map"]))
    base = {"value": n / t_cpu / 1e6, "unit": "Mrays/s", "cores": int(_threads()),
            "kind": "port", "seconds": t_cpu, "host": cpu,
            "sample": f"rays {a}-{b - 1} ({nch} whole 2048-ray chunks through the object, after "
                      f"chunk 0's grid update) of lego test view 0 at {H}x{W}, 64c+128f, ESS + "
                      f"ERT, rendered by oracle/nerf_oracle.py (numpy)"}
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
