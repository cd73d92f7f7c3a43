#!/usr/bin/env python3
"""Train the lego NeRF on one MI355X with the HIP training step (GPU box).

The reference's training recipe (configs/nerf/lego.yaml, src/train/): coarse +
fine 8x256 MLPs with default ``nn.Linear`` initialisation, 64 stratified coarse
samples with perturb, 128 importance samples with training-mode u, loss =
MSE(coarse) + MSE(fine) (trainers/nerf.py:39-76), clip_grad_value_(40)
(trainer.py:59), Adam lr 5e-4 (lego.yaml:63) decayed exponentially by 0.1
(lr_scheduler.py:68-79, lego.yaml:67-70), precrop of the central 50 % for the
first 500 iterations (lego.yaml:26-27). Each step is ``NerfTrainer.step`` on
``--rays`` (N_rays 1024, lego.yaml:14) random pixels of one random train view
(no_batching: True, lego.yaml:19; ``--batching`` draws them across all views).
The reference's trainer renders one whole view per step, which does not fit
any GPU at 800x800 with autograd; ray batches are the recipe's own N_rays. The
0.1 decay is spread over this run's length instead of the reference's 250 000
iterations.

Images come from data/lego/train.npz (tools/pack_lego.py), white-composited as
blender.py:60-75 does. Checkpoints are the reference's format, written by
``nerfhip.checkpoint.save_model`` (net_utils.py:323-344) into ``<out>/model/``
(which holds nothing but ``latest.pth`` and ``<step>.pth``, as the reference's
``load_model`` listing expects, net_utils.py:295-297): {net, optim, scheduler,
recorder, epoch} with the optimizer state in the layout of the reference's
``make_optimizer`` (one param group per parameter, optimizer.py:8-28) and the
scheduler as its ExponentialLR state (gamma 0.1, decay_epochs = the steps this
run's schedule takes to decay 10x, last_epoch = step), so the reference's
``load_model`` resumes from it; ``<out>/net/latest.pth`` = {net, epoch} (the
weights only, what bench.py and the plugin read); logs and eval files go to
``<out>/``. At the end the test views of
data/lego/test.npz are rendered by the HIP inference pipeline and scored with
the reference evaluator's PSNR (evaluators/nerf.py:465-504).

    python tools/train_lego.py --out gpurun_out/lego --max-seconds 1000
    python tools/train_lego.py --out gpurun_out/lego --resume gpurun_out/lego/model/latest.pth
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "nerf-rep_for_test_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--data", default=os.path.join(REPO, "data", "lego"))
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "lego"))
    ap.add_argument("--steps", type=int, default=200000, help="total schedule length")
    ap.add_argument("--rays", type=int, default=1024)
    ap.add_argument("--batching", action="store_true",
                    help="rays from all views per step (default: one view, no_batching)")
    ap.add_argument("--lr", type=float, default=5e-4)
    ap.add_argument("--lr-final", type=float, default=5e-5)
    ap.add_argument("--precrop-iters", type=int, default=500)
    ap.add_argument("--precrop-frac", type=float, default=0.5)
    ap.add_argument("--max-seconds", type=float, default=1000.0)
    ap.add_argument("--resume", default=None)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--log-every", type=int, default=500)
    ap.add_argument("--ckpt-every", type=int, default=5000)
    ap.add_argument("--eval-frames", type=int, default=25)
    ap.add_argument("--mlp", default="x3", choices=["x3", "torch"])
    ap.add_argument("--detach-fine-samples", action="store_true",
                    help="stop the fine loss's gradient at the importance samples (original "
                         "NeRF); the reference lets it reach the coarse network")
    ap.add_argument("--graph", action="store_true", help="replay the step as a HIP graph")
    ap.add_argument("--check-finite", action="store_true",
                    help="stop at the first step whose loss or parameters are not finite")
    args = ap.parse_args()

    import torch
    from nerfhip.checkpoint import (exponential_lr_state, load_checkpoint, reference_optim_state,
                                    save_model, single_group_optim_state)
    from nerfhip.evaluate import load_packed, psnr
    from nerfhip.render import NerfPipeline
    from nerfhip.train import NerfTrainer, camera_rays_at
    from src.models.nerf.network import NeRF

    t_start = time.perf_counter()
    dev = torch.device("cuda:0")
    os.makedirs(os.path.join(args.out, "net"), exist_ok=True)
    model_dir = os.path.join(args.out, "model")
    imgs, poses, focal, _ = load_packed(os.path.join(args.data, "train.npz"))
    V, H, W, _ = imgs.shape
    images = torch.from_numpy(imgs).to(dev)
    poses_d = torch.from_numpy(np.ascontiguousarray(poses)).to(dev)
    K = torch.tensor([[focal, 0, W / 2], [0, focal, H / 2], [0, 0, 1]], dtype=torch.float32,
                     device=dev)
    print(f"train views {V} x {H}x{W} resident in HBM "
          f"({images.numel() * 4 / 2**30:.2f} GiB), focal {focal:.4f}", flush=True)

    torch.manual_seed(args.seed)
    init = {}
    for prefix in ("model", "model_fine"):          # nn.Linear default initialisation
        for k, v in NeRF().state_dict().items():
            init[f"{prefix}.{k}"] = v
    tr = NerfTrainer(dev, init, mlp=args.mlp, detach_fine_samples=args.detach_fine_samples,
                     graph=args.graph)
    names = [n for n, _ in tr.named_parameters()]
    from src.models.nerf.network import Network
    order = [n for n, p in Network().named_parameters() if p.requires_grad]
    assert sorted(order) == sorted(names), "trainer parameters differ from the Network's"
    step0 = 0
    if args.resume:
        ck = load_checkpoint(args.resume)
        tr.load(ck["net"])
        tr.opt.load_state_dict(single_group_optim_state(ck["optim"], names, order))
        step0 = int(ck["epoch"])
        print(f"resumed {args.resume} at step {step0}", flush=True)
    gamma = math.log(args.lr_final / args.lr) / args.steps
    gen = torch.Generator(device=dev).manual_seed(args.seed * 7919 + step0)

    def batch(step):
        n = args.rays
        view = torch.randint(0, V, (n if args.batching else 1,), device=dev, generator=gen)
        view = view.expand(n)
        if step < args.precrop_iters:
            dh, dw = int(H // 2 * args.precrop_frac), int(W // 2 * args.precrop_frac)
            y = torch.randint(H // 2 - dh, H // 2 + dh, (n,), device=dev, generator=gen)
            x = torch.randint(W // 2 - dw, W // 2 + dw, (n,), device=dev, generator=gen)
        else:
            y = torch.randint(0, H, (n,), device=dev, generator=gen)
            x = torch.randint(0, W, (n,), device=dev, generator=gen)
        ro, rd = camera_rays_at(poses_d, K, y * W + x, view, W)
        return ro, rd, images[view, y, x]

    class _State:       # what save_model calls state_dict() on
        def __init__(self, fn):
            self.state_dict = fn

    decay_epochs = math.log(0.1) / gamma        # steps per 10x decay of this run's schedule

    def save(step):
        state = {k: v.detach().cpu() for k, v in tr.state().items()}
        save_model(_State(lambda: state),
                   _State(lambda: reference_optim_state(tr.opt, names, order)),
                   _State(lambda: exponential_lr_state(args.lr, 0.1, decay_epochs, step,
                                                       len(order))),
                   _State(lambda: {"step": step}), model_dir, step, last=True)
        torch.save({"net": state, "epoch": step}, os.path.join(args.out, "net", "latest.pth"))

    step = step0
    t0 = time.perf_counter()
    last = (t0, step)
    log = []
    while step < args.steps and time.perf_counter() - t_start < args.max_seconds:
        tr.set_lr(args.lr * math.exp(gamma * step))
        losses = tr.step(*batch(step))
        step += 1
        if args.check_finite:
            bad = [k for k, p in tr.named_parameters() if not torch.isfinite(p).all()]
            if bad or not torch.isfinite(losses["loss"]):
                print(json.dumps({"non_finite_step": step, "params": bad[:8],
                                  "losses": {k: float(v) for k, v in losses.items()}}),
                      flush=True)
                break
        if step % args.log_every == 0:
            lc, lf = float(losses["loss_coarse"].detach()), float(losses["loss_fine"].detach())
            now = time.perf_counter()
            rec = {"step": step, "loss": lc + lf, "psnr_coarse": -10 * math.log10(lc),
                   "psnr_fine": -10 * math.log10(lf), "lr": args.lr * math.exp(gamma * step),
                   "ms_per_step": (now - last[0]) / (step - last[1]) * 1e3,
                   "elapsed_s": now - t_start}
            last = (now, step)
            log.append(rec)
            print(json.dumps(rec), flush=True)
        if step % args.ckpt_every == 0:
            save(step)
    torch.cuda.synchronize()
    save(step)
    with open(os.path.join(args.out, f"train_log_{step0}_{step}.json"), "w") as f:
        json.dump(log, f)
    print(f"trained steps {step0}..{step} in {time.perf_counter() - t0:.1f} s", flush=True)

    # PSNR of the HIP inference render on the packed test views
    del images
    test, tposes, tfocal, frames = load_packed(os.path.join(args.data, "test.npz"))
    pipe = NerfPipeline(dev, N_samples=64, N_importance=128)
    pipe.set_weights({k: v.detach() for k, v in tr.state().items()})
    Kt = np.array([[tfocal, 0, W / 2], [0, tfocal, H / 2], [0, 0, 1]], np.float32)
    vals = []
    for i in range(min(args.eval_frames, len(frames))):
        rgb = pipe.render_image(H, W, tposes[i], Kt)["rgb_map"].view(H, W, 3).cpu().numpy()
        vals.append(psnr(rgb, test[i]))
    res = {"step": step, "test_frames": [int(f) for f in frames[:len(vals)]], "psnr": vals,
           "psnr_mean": float(np.mean(vals))}
    with open(os.path.join(args.out, f"eval_{step}.json"), "w") as f:
        json.dump(res, f)
    print(json.dumps({"eval_step": step, "psnr_mean": res["psnr_mean"]}), flush=True)


if __name__ == "__main__":
    main()
