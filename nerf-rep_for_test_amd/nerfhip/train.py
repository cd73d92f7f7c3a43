"""NeRF training step on the GPU (BASELINE configs[2]).

One step = the reference's training-mode render of a ray batch
(src/models/nerf/renderer/volume_renderer.py:145-268 with perturb > 0 and the
fine-sampling u ~ U[0,1), no detach anywhere), loss = MSE(coarse rgb, target)
+ MSE(fine rgb, target) (src/train/trainers/nerf.py:39-76), backward,
clip_grad_value_(40) (trainers/trainer.py:59), Adam(lr 5e-4, eps 1e-8, no
weight decay) (src/train/optimizer.py, lego.yaml:63-66, config.py:98).

Division of labour: the stratified coarse depths come from the HIP kernel
(bit-exact, no gradient needed); the two 8x256 MLPs run forward and backward
on the hand-written x3 MFMA kernels (train_mlp.NerfMLPFn: FP32 operands as
3-term FP16 splits, layer GEMMs over feature-major activations, split-K weight
gradients); compositing, importance sampling and the loss stay in torch
autograd around them. mlp="torch" runs the MLPs as torch modules (FP32
hipBLASLt GEMMs) instead. Parity with the reference's own forward/backward is
pinned by tests/golden/t1_train_step.npz.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _lib
from ._lib import call, ptr
from .render import REF_CHUNK, coarse_depth_table, reference_draws_noise

XYZ_FREQS, DIR_FREQS = 10, 4


def freq_encode(x, n_freq):
    """freq.py:7-32: [x, sin(2^0 x), cos(2^0 x), ..., sin(2^(L-1) x), cos(...)]."""
    feats = [x]
    for f in range(n_freq):
        s = x * float(2 ** f)
        feats.append(torch.sin(s))
        feats.append(torch.cos(s))
    return torch.cat(feats, -1)


def query(model, pts, dirs):
    """VR:270-284: encode points and (per-sample) view directions, run the MLP."""
    n, s, _ = pts.shape
    x = freq_encode(pts.reshape(-1, 3), XYZ_FREQS)
    d = freq_encode(dirs[:, None, :].expand(n, s, 3).reshape(-1, 3), DIR_FREQS)
    return model(torch.cat([x, d], -1)).reshape(n, s, 4)


def composite(raw, z, rays_d, white_bkgd):
    """VR:286-357 (raw_noise_std = 0): weights and the four maps."""
    ones = torch.full_like(z[..., :1], 1e10)
    dists = torch.cat([z[..., 1:] - z[..., :-1], ones], -1)
    dists = dists * torch.norm(rays_d[..., None, :], dim=-1)
    rgb = torch.sigmoid(raw[..., :3])
    alpha = 1.0 - torch.exp(-F.relu(raw[..., 3]) * dists)
    trans = torch.cumprod(torch.cat([torch.ones_like(alpha[..., :1]), 1.0 - alpha + 1e-10], -1),
                          -1)[..., :-1]
    w = alpha * trans
    rgb_map = torch.sum(w[..., None] * rgb, -2)
    depth = torch.sum(w * z, -1)
    acc = torch.sum(w, -1)
    disp = 1.0 / torch.max(torch.full_like(depth, 1e-10), depth / acc)
    if white_bkgd:
        rgb_map = rgb_map + (1.0 - acc[..., None])
    return rgb_map, disp, acc, w, depth


def sample_pdf(mids, weights, u):
    """VR:239-268, differentiable in weights and mids (training-mode u given)."""
    weights = weights + 1e-5
    pdf = weights / torch.sum(weights, -1, keepdim=True)
    cdf = torch.cumsum(pdf, -1)
    cdf = torch.cat([torch.zeros_like(cdf[..., :1]), cdf], -1)
    inds = torch.searchsorted(cdf, u.contiguous(), right=True)
    below = torch.clamp(inds - 1, min=0)
    above = torch.clamp(inds, max=cdf.shape[-1] - 1)
    cdf_lo, cdf_hi = torch.gather(cdf, -1, below), torch.gather(cdf, -1, above)
    bin_lo, bin_hi = torch.gather(mids, -1, below), torch.gather(mids, -1, above)
    denom = cdf_hi - cdf_lo
    denom = torch.where(denom < 1e-5, torch.ones_like(denom), denom)
    t = (u - cdf_lo) / denom
    return bin_lo + t * (bin_hi - bin_lo)


def composite_ert(raw, z, rays_d, thr, white_bkgd, chunk=2048):
    """VR:1089-1133 (raw_noise_std = 0), differentiable: transmittance WITHOUT the
    +1e-10; where any ray of a 2048-ray chunk has T < thr, every ray of that
    chunk has its weights zeroed from its first such sample on (argmax of an
    all-False row is 0: a ray that never terminates loses all of its weights,
    quirk 1). Rows [0, n) start on a chunk boundary of the reference's loop."""
    n, S = z.shape
    ones = torch.full_like(z[..., :1], 1e10)
    dists = torch.cat([z[..., 1:] - z[..., :-1], ones], -1)
    dists = dists * torch.norm(rays_d[..., None, :], dim=-1)
    rgb = torch.sigmoid(raw[..., :3])
    alpha = 1.0 - torch.exp(-F.relu(raw[..., 3]) * dists)
    shifted = torch.cat([torch.zeros_like(alpha[:, :1]), alpha[:, :-1]], 1)
    trans = torch.cumprod(1.0 - shifted, 1)
    w = alpha * trans
    low = trans < thr
    nc = -(-n // chunk)
    ray_any = low.any(1)
    pad = torch.zeros(nc * chunk - n, dtype=torch.bool, device=z.device)
    chunk_any = torch.cat([ray_any, pad]).view(nc, chunk).any(1)
    cut = chunk_any.repeat_interleave(chunk)[:n]
    first = low.float().argmax(1)
    mask = (torch.arange(S, device=z.device)[None, :] >= first[:, None]) & cut[:, None]
    w = w * (~mask).float()
    rgb_map = torch.sum(w[..., None] * rgb, -2)
    depth = torch.sum(w * z, -1)
    acc = torch.sum(w, -1)
    disp = 1.0 / torch.max(torch.full_like(depth, 1e-10), depth / torch.sum(w, -1))
    if white_bkgd:
        rgb_map = rgb_map + (1.0 - acc[..., None])
    return rgb_map, disp, acc, w, depth


def render_train(coarse, fine, rays_o, rays_d, z, u, white_bkgd=True, query_fn=query,
                 detach_fine_samples=False, composite_fn=None, on_composite=None,
                 hip_ops=False, noise=None):
    """The differentiable part of a training step (VR:164-194): coarse depths z
    [n, S] (no gradient) -> coarse maps, importance samples from the coarse
    weights (u [n, N_importance]), fine maps. fine=None: coarse only.
    query_fn(model, pts, dirs) evaluates the MLP (torch module call, or the x3
    MFMA kernels of train_mlp.query_x3). The reference lets the fine loss's
    gradient flow through the importance samples into the coarse network (no
    detach, VR:181-184, 239-268); detach_fine_samples=True stops it there, as
    the original NeRF does (tf.stop_gradient on z_samples).
    composite_fn(raw, z, rays_d) -> (rgb, disp, acc, weights, depth) replaces
    _raw2outputs (e.g. composite_ert); on_composite(kind, z, raw, weights) is
    called after each composite (kind 0 coarse, 1 fine: the ESS grid hook).
    hip_ops: compositing (unless composite_fn is given) and importance sampling
    + merge on the HIP kernels of train_ops (no host syncs: graph-capturable).
    noise = (coarse [n, S], fine [n, S + NI]): density noise (raw_noise_std > 0,
    VR:310-314) added to raw before each composite; on_composite sees raw without
    it (the reference's grid update reads raw, VR:1150-1153)."""
    if composite_fn is None and hip_ops:
        from .train_ops import composite_hip

        def composite_fn(raw, zz, rd):
            return composite_hip(raw, zz, rd, white_bkgd)
    if composite_fn is None:
        def composite_fn(raw, zz, rd):
            return composite(raw, zz, rd, white_bkgd)
    # a query with a ray form (train_mlp.query_x3.rays) builds the points o + d z
    # itself (VR:165) and returns d z directly in the backward
    rays_q = getattr(query_fn, "rays", None)

    def q(model, zz):
        if rays_q is not None:
            return rays_q(model, rays_o, rays_d, zz)
        return query_fn(model, rays_o[:, None, :] + rays_d[:, None, :] * zz[..., None], rays_d)
    def noisy(raw, k):
        if noise is None:
            return raw
        from .train_ops import add_sigma_noise
        return add_sigma_noise(raw, noise[k])
    raw = q(coarse, z)
    rgb0, disp0, acc0, w, depth0 = composite_fn(noisy(raw, 0), z, rays_d)
    if on_composite is not None:
        on_composite(0, z, raw, w)
    out = {"rgb_map_0": rgb0, "disp_map_0": disp0, "acc_map_0": acc0, "depth_map_0": depth0}
    if fine is not None:
        if hip_ops:
            from .train_ops import sample_fine_hip
            z2 = sample_fine_hip(w.detach() if detach_fine_samples else w, z, u)
        else:
            mids = 0.5 * (z[..., 1:] + z[..., :-1])
            zf = sample_pdf(mids, w[..., 1:-1], u)
            if detach_fine_samples:
                zf = zf.detach()
            z2, _ = torch.sort(torch.cat([z, zf], -1), -1)
        raw2 = q(fine, z2)
        rgb, disp, acc, w2, depth = composite_fn(noisy(raw2, 1), z2, rays_d)
        if on_composite is not None:
            on_composite(1, z2, raw2, w2)
        out.update(rgb_map=rgb, disp_map=disp, acc_map=acc, depth_map=depth)
    return out


def render_rays_train(pipe, coarse, fine, rays_o, rays_d, perturb, query_fn,
                      detach_fine_samples=False, noise_std=0.0):
    """The reference's training-mode ``_render_pytorch`` over a ray block
    (VR:145-216 with ``self.net.training``): per 2048-ray chunk, in the
    reference's order, the perturb draw t_rand [m, S] (VR:228-235 / ESS
    :1080-1085) then the fine draw u [m, N_importance] (VR:247-249), both
    torch.rand on the device; coarse depths by the HIP kernels (stratified or
    ESS, no gradient); MLPs + compositing differentiable (render_train), ERT
    with its chunk rule (composite_ert), the ESS grid self-update and call
    counter of VR:1147-1157 on detached values, passes cut after a
    grid-updating chunk as in NerfPipeline.render_rays. ``pipe`` is the
    NerfPipeline holding the configuration, tables, grid and counter.
    noise_std > 0 (raw_noise_std): the composites' density noise drawn in the
    reference's chunk order (render.reference_draws_noise)."""
    n = rays_o.shape[0]
    S, NI = pipe.N_samples, pipe.N_importance
    dev = pipe.device
    st = _lib.stream_of(dev)
    outs = []
    p = 0
    while p < n:
        m = n - p
        if pipe.enable_ess and pipe.enable_ert:
            m = pipe._ess_phase_len(m)
        ro, rd = rays_o[p:p + m], rays_d[p:p + m]
        t_rand, u, nc, nf = reference_draws_noise(m, S, NI, perturb, True, dev, noise_std)
        z = torch.empty((m, S), device=dev, dtype=torch.float32)
        if pipe.enable_ess:
            if pipe.grid is None:
                raise _lib.NerfHipError("ESS enabled but no occupancy grid set")
            call("nerf_sample_coarse_ess", ptr(ro), ptr(rd), ptr(pipe.grid), pipe.grid_res,
                 ptr(pipe.z_base), ptr(t_rand), m, S, REF_CHUNK, pipe.ess_skip_threshold,
                 ptr(z), st)
        elif t_rand is not None:
            call("nerf_sample_coarse", ptr(pipe.z_base), ptr(t_rand), m, S, ptr(z), st)
        else:
            z.copy_(pipe.z_base.expand(m, S))
        counter0 = pipe.grid_update_counter
        comp, hook = None, None
        if pipe.enable_ert:
            def comp(raw, zz, rdd):
                return composite_ert(raw, zz, rdd, pipe.ert_threshold, pipe.white_bkgd)

            def hook(kind, zz, raw, w):
                ss = zz.shape[1]
                pipe._grid_updates(kind, counter0, rd, zz.detach().contiguous(), ss,
                                   raw.detach().reshape(-1, 4).contiguous(),
                                   w.detach().contiguous(), m, ss)
        else:
            def comp(raw, zz, rdd):
                return composite(raw, zz, rdd, pipe.white_bkgd)
        outs.append(render_train(coarse, fine if NI > 0 else None, ro, rd, z, u,
                                 pipe.white_bkgd, query_fn, detach_fine_samples,
                                 comp if pipe.enable_ert else None, hook, hip_ops=True,
                                 noise=(nc, nf) if noise_std > 0 else None))
        if pipe.enable_ert:
            pipe.grid_update_counter = counter0 + pipe._calls_per_chunk() * -(-m // REF_CHUNK)
        p += m
    return {k: torch.cat([o[k] for o in outs], 0) for k in outs[0]}


def mse_losses(out, target):
    """trainers/nerf.py:39-76: MSE coarse (+ MSE fine)."""
    loss_c = F.mse_loss(out["rgb_map_0"], target)
    res = {"loss_coarse": loss_c, "loss": loss_c}
    if "rgb_map" in out:
        loss_f = F.mse_loss(out["rgb_map"], target)
        res.update(loss_fine=loss_f, loss=loss_c + loss_f)
    return res


class NerfTrainer:
    """Coarse + fine networks, optimizer and one training step on a ROCm device."""

    def __init__(self, device, params, N_samples=64, N_importance=128, near=2.0, far=6.0,
                 white_bkgd=True, lr=5e-4, clip_value=40.0, mlp="x3",
                 detach_fine_samples=False, graph=False, ops="hip", adam=None):
        from src.models.nerf.network import NeRF
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise _lib.NerfHipError("NerfTrainer needs a ROCm GPU device (no CPU fallback)")
        _lib.lib()
        self.N_samples, self.N_importance = int(N_samples), int(N_importance)
        self.white_bkgd = bool(white_bkgd)
        self.clip_value = float(clip_value)
        if mlp not in ("x3", "torch"):
            raise ValueError("mlp must be 'x3' or 'torch'")
        self.mlp = mlp
        self.detach_fine_samples = bool(detach_fine_samples)
        self.coarse = NeRF().to(self.device)
        self.fine = NeRF().to(self.device)
        self.load(params)
        # graph=True: the whole step (both MLPs forward + backward, compositing,
        # sampling, loss, clip, Adam) is captured once per batch shape into a HIP
        # graph and replayed: one launch instead of several hundred. Adam then
        # keeps its step count and learning rate on the device (capturable,
        # lr tensor: set_lr updates it in place).
        if ops not in ("hip", "torch"):
            raise ValueError("ops must be 'hip' or 'torch'")
        if graph and ops != "hip":
            raise ValueError("graph=True needs ops='hip' (torch's cumprod backward syncs)")
        self.ops = ops
        self.graph = bool(graph)
        # adam: "hip" (the default: clip_grad_value_ + Adam in one nerf_adam_step
        # launch, lr and step count on the device, graph-capturable), or torch's
        # "fused" (eager only) / "capturable" multi-tensor Adam after a separate
        # clip_grad_value_
        adam = adam or "hip"
        if adam not in ("hip", "fused", "capturable") or (self.graph and adam == "fused"):
            raise ValueError("adam must be 'hip', 'fused' or 'capturable' (graph: not 'fused')")
        self.adam = adam
        if adam == "hip":
            from .adam import HipAdam
            self.opt = HipAdam(self.trained_parameters(), lr=lr, eps=1e-8, clip=self.clip_value)
        elif adam == "capturable":
            self.opt = torch.optim.Adam(self.trained_parameters(),
                                        lr=torch.tensor(lr, device=self.device), eps=1e-8,
                                        weight_decay=0.0, capturable=True, foreach=True)
        else:
            # one fused multi-tensor Adam kernel per step on the GPU
            self.opt = torch.optim.Adam(self.trained_parameters(), lr=lr, eps=1e-8,
                                        weight_decay=0.0, fused=self.device.type == "cuda")
        self._graphs = {}
        self._flat_draws = {}
        self._one = {}
        self._warm = {}
        self.z_base = coarse_depth_table(near, far, self.N_samples, False).to(self.device)

    def parameters(self):
        return list(self.coarse.parameters()) + list(self.fine.parameters())

    def trained_parameters(self):
        """The parameters a step updates: without a fine pass (N_importance 0,
        VR:181) the fine network takes no part and gets no gradient."""
        return list(self.coarse.parameters()) + (list(self.fine.parameters())
                                                 if self.N_importance > 0 else [])

    def named_parameters(self):
        for prefix, m in (("model", self.coarse), ("model_fine", self.fine)):
            for k, p in m.named_parameters():
                yield f"{prefix}.{k}", p

    def load(self, params):
        with torch.no_grad():
            for name, p in self.named_parameters():
                v = params[name]
                p.copy_(torch.as_tensor(v.detach().cpu() if hasattr(v, "detach") else v))

    def state(self):
        """model.* / model_fine.* tensors (for NerfPipeline.set_weights / checkpoints)."""
        return {k: p.detach() for k, p in self.named_parameters()}

    def forward(self, rays_o, rays_d, t_rand, u):
        n, S = rays_o.shape[0], self.N_samples
        z = torch.empty((n, S), device=self.device, dtype=torch.float32)
        t_rand = t_rand.contiguous()
        call("nerf_sample_coarse", ptr(self.z_base), ptr(t_rand), n, S, ptr(z),
             _lib.stream_of(self.device))
        from .train_mlp import query_x3
        return render_train(self.coarse, self.fine if self.N_importance > 0 else None,
                            rays_o, rays_d, z, u, self.white_bkgd,
                            query_x3 if self.mlp == "x3" else query, self.detach_fine_samples,
                            hip_ops=self.ops == "hip")

    def loss(self, out, target):
        if self.ops == "hip":   # one launch forward, one backward (train_ops.MSEPairFn)
            from .train_ops import mse_losses_hip
            return mse_losses_hip(out, target)
        return mse_losses(out, target)

    def set_lr(self, lr):
        for g in self.opt.param_groups:
            if torch.is_tensor(g["lr"]):
                g["lr"].fill_(lr)
            else:
                g["lr"] = lr

    def step(self, rays_o, rays_d, target, t_rand=None, u=None, group=None):
        """One optimisation step; returns the loss dict (device tensors). With a
        process group, each rank's gradients are averaged (data parallel: one
        flat bucket, one all-reduce over RCCL) before clipping and Adam.
        ``t_rand`` [n, N_samples] / ``u`` [n, N_importance] are the step's random
        draws (perturb jitter, training-mode fine u); None draws them on the
        device (t_rand, then u: torch.rand's stream, VR:233, :248).
        In graph mode the first two steps of a batch shape run eagerly (they
        create the packers' buffers, Adam's state and the BLAS handles), the
        third is captured and every step from then on replays the graph with
        the batch AND the draws copied into its static inputs (no RNG inside the
        graph: the draws come from the same stream, in the same order, as an
        eager step's); the returned losses are the graph's output tensors."""
        if self.graph:
            return self._step_graphed(rays_o, rays_d, target, t_rand, u, group)
        return self._step_eager(rays_o, rays_d, target, t_rand, u, group)

    def _draws(self, n, t_rand, u):
        """The step's draws: both from ONE torch.rand launch when neither is
        given (t_rand the first n * N_samples values, u the rest: the same
        numbers in the eager and the graph step, _step_graphed)."""
        if t_rand is None and u is None:
            S, NI = self.N_samples, self.N_importance
            flat = torch.rand((n * (S + NI),), device=self.device)
            return flat[:n * S].view(n, S), flat[n * S:].view(n, NI)
        if t_rand is None:
            t_rand = torch.rand((n, self.N_samples), device=self.device)
        if u is None:
            u = torch.rand((n, self.N_importance), device=self.device)
        return t_rand, u

    def _step_graphed(self, rays_o, rays_d, target, t_rand, u, group):
        key = (rays_o.shape[0], group is not None)
        g = self._graphs.get(key)
        if g is None:
            t_rand, u = self._draws(rays_o.shape[0], t_rand, u)
            if self._warm.get(key, 0) < 2:
                self._warm[key] = self._warm.get(key, 0) + 1
                return self._step_eager(rays_o, rays_d, target, t_rand, u, group)
            static = [x.detach().clone().contiguous() for x in (rays_o, rays_d, target)]
            # the draws: views of one flat buffer, so a replay draws them with one
            # torch.rand launch (the numbers _draws makes in an eager step)
            n, S = t_rand.shape
            flat = torch.empty((n * (S + u.shape[1]),), device=self.device, dtype=torch.float32)
            static += [flat[:n * S].view(n, S), flat[n * S:].view(n, u.shape[1])]
            static[3].copy_(t_rand)
            static[4].copy_(u)
            static = tuple(static)
            self._flat_draws[key] = flat
            graph = torch.cuda.CUDAGraph()
            torch.cuda.synchronize(self.device)
            with torch.cuda.graph(graph):
                out = self._step_eager(*static, group)
            g = self._graphs[key] = (graph, static, out)
            t_rand = u = None   # already in the static inputs
            given = (rays_o, rays_d, target, static[3], static[4])
        else:
            given = (rays_o, rays_d, target, t_rand, u)
        graph, static, out = g
        if given[3] is None and given[4] is None:   # both draws with one launch (_draws)
            flat = self._flat_draws[key]
            torch.rand(flat.shape, device=flat.device, out=flat)
        else:
            for dst, src in zip(static[3:], given[3:]):
                if src is None:   # the step's draw, straight into the graph's input
                    torch.rand(dst.shape, device=dst.device, out=dst)
        # the batch (and any given draw) into the static inputs: one multi-tensor copy
        pairs = [(dst, src) for dst, src in zip(static, given)
                 if src is not None and src is not dst]
        if pairs:
            torch._foreach_copy_([d for d, _ in pairs], [s for _, s in pairs])
        graph.replay()
        return out

    def _step_eager(self, rays_o, rays_d, target, t_rand=None, u=None, group=None):
        t_rand, u = self._draws(rays_o.shape[0], t_rand, u)
        self.opt.zero_grad(set_to_none=True)
        if self.mlp == "x3":   # both networks' weight streams in one packing launch set
            from .train_mlp import prepack
            prepack([self.coarse] + ([self.fine] if self.N_importance > 0 else []), side=True)
        losses = self.loss(self.forward(rays_o, rays_d, t_rand, u), target)
        loss = losses["loss"]
        one = self._one.get(loss.device)
        if one is None:   # d loss / d loss = 1, kept (no fill kernel per step)
            one = self._one[loss.device] = torch.ones((), device=loss.device, dtype=loss.dtype)
        if self.mlp == "x3" and self.N_importance > 0 and self.fine is not self.coarse:
            # one fused node per network: the fine network's weight gradients on a
            # side stream while the main one runs on through the coarse backward
            from .train_mlp import side_wgrad_scope
            with side_wgrad_scope([self.fine]):
                loss.backward(one)
        else:
            loss.backward(one)
        if group is not None:
            for p in self.trained_parameters():
                if p.grad is None:   # (a rank whose batch left a parameter untouched):
                    p.grad = torch.zeros_like(p)   # every rank sends the same bucket
            allreduce_mean([p.grad for p in self.trained_parameters()], group)
        if self.adam != "hip":   # (HipAdam clamps the gradients itself, in place)
            torch.nn.utils.clip_grad_value_(self.trained_parameters(), self.clip_value)
        self.opt.step()
        return losses


def allreduce_mean(grads, group):
    """Average gradients over the group in one flat bucket (2.4 MB per network).
    None entries are skipped (every rank has the same set: same configuration)."""
    import torch.distributed as dist
    grads = [g for g in grads if g is not None]
    if not grads:
        return
    flat = torch.cat([g.reshape(-1) for g in grads])
    dist.all_reduce(flat, group=group)
    flat /= dist.get_world_size(group)
    off = 0
    for g in grads:
        g.copy_(flat[off:off + g.numel()].view_as(g))
        off += g.numel()


def camera_rays_at(poses, K, pix_idx, view_idx, W):
    """Rays of arbitrary pixels (VR:115-143): pixel (x, y) = (i % W, i // W) of view
    view_idx[k]; unit directions. poses [V,4,4], K [3,3] (device)."""
    x = (pix_idx % W).float()
    y = (pix_idx // W).float()
    d = torch.stack([(x - K[0, 2]) / K[0, 0], -(y - K[1, 2]) / K[1, 1], -torch.ones_like(x)], -1)
    R = poses[view_idx, :3, :3]
    rd = torch.sum(d[:, None, :] * R, -1)
    rd = rd / torch.norm(rd, dim=-1, keepdim=True)
    ro = poses[view_idx, :3, 3]
    return ro.contiguous(), rd.contiguous()
