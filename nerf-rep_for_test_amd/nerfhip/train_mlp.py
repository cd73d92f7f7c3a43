"""The NeRF MLP of a training step on hand-written x3 MFMA kernels.

Forward and backward of ``NeRF.forward`` (src/models/nerf/network.py:49-74:
8 pts layers with the skip cat(input_pts, h) after layer 4, alpha head,
feature layer, views layer on cat(feature, input_views), rgb head) for P
samples, as a ``torch.autograd.Function`` so the rest of the training step
(compositing, importance sampling, loss; volume_renderer.py:145-357) stays in
torch autograd around it.

Activations live feature-major in HBM ([F][P]); every 256-wide layer is one
``nerf_x3_layer`` launch (FP32 operands as 3-term FP16 splits on FP16 MFMA,
DESIGN.md §3), in both directions:

  forward   h_L = relu(W_L h_{L-1} + b_L)
  dgrad     d_{L-1} = (W_L^T d_L) * (h_{L-1} > 0)
  wgrad     dW_L = d_L h_{L-1}^T  (``nerf_x3_wgrad``, split-K partials summed)

The frequency encoding and its derivative are HIP kernels that write / read
the feature-major rows directly (``nerf_freq_encode_fm`` / ``_backward``, the
encoding's max |.| fused); the rank-1 heads (alpha 256->1, rgb 128->3) and
the bias gradients (row sums) are small torch ops on the device.
Weights are repacked from the live parameters every call (device-side torch
ops, no host sync): packing order = ``pack_x3_matrix``.
"""
from __future__ import annotations

import functools

import ctypes
import os as _os

import torch

from . import _lib
from ._lib import call, ptr

XYZ_FREQS, DIR_FREQS = 10, 4


def wgrad_chunk(P):
    """Samples per weight-gradient workgroup: about 256 chunks (one workgroup per
    CU for a 256x256 output), a multiple of 32 in [256, 4096]."""
    return min(4096, max(256, -(-P // (256 * 32)) * 32))


def freq_encode(x, n_freq):
    """freq.py:7-32: [x, sin(2^0 x), cos(2^0 x), ..., sin(2^(L-1) x), cos(...)]."""
    feats = [x]
    for f in range(n_freq):
        s = x * float(2 ** f)
        feats.append(torch.sin(s))
        feats.append(torch.cos(s))
    return torch.cat(feats, -1)


def pack_x3_matrix(W):
    """W [M, K] float32 (device; M % 16 == 0, K % 32 == 0) -> (packed FP16 hi/lo
    fragments as a float32 tensor, int32 [1] scale exponent sw), both on W's
    device. max|W| * 2^sw lies in [2^11, 2^12). Fragment order: K step q, tile t,
    part (hi, lo), lane l = r + 16 g, element j = W[16t + r][32q + 8g + j]."""
    M, K = W.shape
    assert M % 16 == 0 and K % 32 == 0, (M, K)
    amax = W.abs().amax()
    _, ex = torch.frexp(amax)
    sw = torch.where(amax > 0, 12 - ex, torch.zeros_like(ex)).to(torch.int32).reshape(1)
    Ws = torch.ldexp(W, sw.to(W.dtype))
    hi = Ws.half()
    lo = (Ws - hi.float()).half()
    fr = torch.stack([hi, lo]).reshape(2, M // 16, 16, K // 32, 4, 8)
    fr = fr.permute(3, 1, 0, 4, 2, 5).contiguous()        # [q, t, part, g, r, j]
    return fr.view(torch.float32).reshape(-1), sw


_DESC_FIELDS = [("src", "<u8"), ("ldr", "<i8"), ("ldc", "<i8"), ("rowmap", "<u8"),
                ("colmap", "<u8"), ("M", "<i4"), ("K", "<i4"), ("out", "<u8"), ("sw", "<u8"),
                ("amax", "<u8")]
_HEAD_FIELDS = [("table", "<u8"), ("dst", "<u8"), ("n", "<i8")]


def _device_table(recs, fields, device):
    """Records (tuples) -> the packed C structs as a uint8 device tensor."""
    import numpy as np
    dt = np.dtype(fields)
    arr = np.array(recs, dtype=dt)
    return torch.from_numpy(arr.view(np.uint8).copy()).to(device)


class _PackSet:
    """Packing descriptors (X3PackDesc records: matrix -> fragments) and head
    gathers (X3HeadGather records) of one or more streams; run as ONE
    nerf_x3_pack launch set (amax, pack + gather, scale)."""

    def __init__(self, device):
        self.device = torch.device(device)
        self.key = None
        self.recs, self.heads = [], []
        self._keep = []

    def _matrix(self, W, rmap, cmap, transposed, out_ptr, sw_ptr, amax_ptr):
        dev = self.device
        rm = torch.tensor(rmap, dtype=torch.int32, device=dev)
        cm = torch.tensor(cmap, dtype=torch.int32, device=dev)
        self._keep += [rm, cm]
        ldr, ldc = (W.stride(1), W.stride(0)) if transposed else (W.stride(0), W.stride(1))
        self.recs.append((W.data_ptr(), ldr, ldc, rm.data_ptr(), cm.data_ptr(), len(rmap),
                          len(cmap), out_ptr, sw_ptr, amax_ptr))

    def _head(self, table, dst):
        """table: numpy uint64 [n] (addresses / scale slots | 1 / 0) -> gathered into dst."""
        t = torch.from_numpy(table.astype("<u8").view("<i8")).to(self.device)
        self._keep.append(t)
        self.heads.append((t.data_ptr(), dst.data_ptr(), int(table.shape[0])))

    def launch(self):
        if not hasattr(self, "_tables") or self._tables[0] is None:
            self._tables = (_device_table(self.recs, _DESC_FIELDS, self.device),
                            _device_table(self.heads, _HEAD_FIELDS, self.device)
                            if self.heads else None)
        descs, heads = self._tables
        call("nerf_x3_pack", ptr(descs), len(self.recs), ptr(heads), len(self.heads),
             _lib.stream_of(self.device))


class X3Packer(_PackSet):
    """All 21 weight matrices of one network's training step (forward W and
    backward W^T, padded as the layer kernels need them) packed by ONE
    nerf_x3_pack launch set from the live parameters; the output buffers, index
    maps and descriptor table are built once and reused while the parameters
    keep their storage (the optimizer updates them in place).

    Entries: name -> (param, transposed, rowmap, colmap); the padded matrix's
    element (i, k) is param[rowmap[i]][colmap[k]] (param^T when transposed)."""

    def __init__(self, device, forward=True, backward=True):
        super().__init__(device)
        self.forward = forward
        self.backward = backward

    def plan(self, p):
        ar = lambda n: list(range(n))   # noqa: E731
        enc64 = ar(63) + [-1]
        plan = {"fwd0": ("pts_linears.0.weight", False, ar(256), enc64),
                "fwd5": ("pts_linears.5.weight", False, ar(256), enc64 + list(range(63, 319))),
                "fwd_feat": ("feature_linear.weight", False, ar(256), ar(256)),
                "fwd_views": ("views_linears.0.weight", False, ar(128), ar(283) + [-1] * 5),
                "bwd_views": ("views_linears.0.weight", True, ar(256), ar(128)),
                "bwd_feat": ("feature_linear.weight", True, ar(256), ar(256)),
                "bwd5h": ("pts_linears.5.weight", True, list(range(63, 319)), ar(256)),
                "bwd5e": ("pts_linears.5.weight", True, enc64, ar(256)),
                "bwd0": ("pts_linears.0.weight", True, enc64, ar(256)),
                # d hv = W_rgb^T d_rgb: K = the 3 rgb rows of d_raw^T (+ 29 zero rows)
                "bwd_rgb": ("rgb_linear.weight", True, ar(128), ar(3) + [-1] * 29)}
        for i in (1, 2, 3, 4, 6, 7):
            plan[f"fwd{i}"] = (f"pts_linears.{i}.weight", False, ar(256), ar(256))
            plan[f"bwd{i}"] = (f"pts_linears.{i}.weight", True, ar(256), ar(256))
        if not self.forward:
            plan = {k: v for k, v in plan.items() if not k.startswith("fwd")}
        if not self.backward:
            plan = {k: v for k, v in plan.items() if not k.startswith("bwd")}
        return plan

    def _build(self, p):
        plan = self.plan(p)
        dev = self.device
        self.recs, self.heads, self._keep, self._tables = [], [], [], (None, None)
        self.names = list(plan)
        self.out = {}
        self.sw = torch.zeros(len(plan), device=dev, dtype=torch.int32)
        self.amax = torch.zeros(len(plan), device=dev, dtype=torch.int32)
        for n, (pname, tr, rmap, cmap) in enumerate(plan.values()):
            M, K = len(rmap), len(cmap)
            out = torch.empty(M * K, device=dev, dtype=torch.float32)   # M*K halfs x 2
            self.out[self.names[n]] = (out, M // 16, K // 32)
            self._matrix(p[pname], rmap, cmap, tr, out.data_ptr(), self.sw[n:n + 1].data_ptr(),
                         self.amax[n:n + 1].data_ptr())

    def pack(self, p):
        """p: parameter name -> tensor. Returns name -> (packed, sw [1], m_tiles, k_steps)."""
        key = tuple((k, v.data_ptr()) for k, v in sorted(p.items()) if k.endswith("weight"))
        if key != self.key:
            self._build(p)
            self.key = key
        self.launch()
        return {n: (o, self.sw[i:i + 1], mt, nk)
                for i, (n, (o, mt, nk)) in enumerate(self.out.items())}


def _src_pointers(p, names, idx, amax, nsrc):
    """Head gather table: index map over cat(names' parameters flattened, scales)
    -> element addresses (scales: their amax slot | 1; -1: 0)."""
    import numpy as np
    sizes = [p[k].numel() for k in names]
    starts = np.concatenate([[0], np.cumsum(sizes)])
    assert starts[-1] == nsrc and all(p[k].is_contiguous() for k in names)
    bases = np.array([p[k].data_ptr() for k in names], dtype=np.uint64)
    out = np.zeros(idx.shape[0], np.uint64)
    src = (idx >= 0) & (idx < nsrc)
    k = np.searchsorted(starts, idx[src], side="right") - 1
    out[src] = bases[k] + 4 * (idx[src] - starts[k]).astype(np.uint64)
    sc = idx >= nsrc
    out[sc] = np.uint64(amax.data_ptr()) + 4 * (idx[sc] - nsrc).astype(np.uint64) + np.uint64(1)
    return out


class NerfFoldDescC(ctypes.Structure):
    """NerfFoldDesc (include/nerfhip.h)."""
    _fields_ = [(k, ctypes.c_void_p) for k in ("Wv", "Wf", "bf", "bv", "Wc", "bc")]


def _fold(packers):
    """One nerf_fold_views launch for the forward streams of several networks."""
    arr = (NerfFoldDescC * len(packers))(*[NerfFoldDescC(*f.fold_ptrs) for f in packers])
    call("nerf_fold_views", ctypes.addressof(arr), len(packers), _lib.stream_of(packers[0].device))


class X3StreamPacker(_PackSet):
    """The training forward's weight stream, packed on the device from the live
    parameters: the 65 slices of nerf_mlp_train_forward_x3 -- the inference
    kernel's layout, the feature layer folded into the views layer each step
    by nerf_fold_views into (Wc, bc) (byte-identical to
    nerfhip.pack.pack_mlp_x3(params, folded=(Wc, bc))), each layer's matrix with
    the kernel's K permutation as its column map, written straight into its
    slices, and the head block (lane-packed biases, the alpha / rgb heads, the
    per-layer weight scales) gathered from the parameters (the views bias from
    bc) through an index map made once by nerfhip.pack.pack_mlp -- all in the
    nerf_x3_pack launch set, after the fold."""

    @staticmethod
    def plan():
        from .pack import _x3_layer_cols, layer_plan
        out, off = [], 0
        for li, (name, kind, tiles) in enumerate(layer_plan()):
            if name == "feature_linear":   # folded into the views layer
                continue
            cols = _x3_layer_cols(kind).reshape(-1)
            out.append((name + ".weight", list(range(16 * tiles)), [int(c) for c in cols], off, li))
            off += -(-16 * tiles * len(cols) // 8192)          # whole slices (views: 4.5 -> 5)
        return out, off

    def _build(self, p):
        import numpy as np
        from .pack import H_BIAS, HEAD_FLOATS, H_SCALES, SLICE_FLOATS, pack_mlp
        dev = self.device
        plan, nsl = self.plan()
        self.recs, self.heads, self._keep, self._tables = [], [], [], (None, None)
        self.stream = torch.zeros(nsl * SLICE_FLOATS, device=dev, dtype=torch.float32)
        self.sw = torch.zeros(len(plan), device=dev, dtype=torch.int32)
        self.amax = torch.zeros(len(plan), device=dev, dtype=torch.int32)
        self.Wc = torch.zeros((128, 283), device=dev, dtype=torch.float32)
        self.bc = torch.zeros((128,), device=dev, dtype=torch.float32)
        src = [p[k] for k in ("views_linears.0.weight", "feature_linear.weight",
                              "feature_linear.bias", "views_linears.0.bias")]
        assert all(t.is_contiguous() for t in src)
        self.fold_ptrs = tuple(t.data_ptr() for t in src) + (self.Wc.data_ptr(), self.bc.data_ptr())
        for n, (pname, rmap, cmap, off, _) in enumerate(plan):
            W = self.Wc if pname == "views_linears.0.weight" else p[pname]
            self._matrix(W, rmap, cmap, False,
                         self.stream.data_ptr() + 4 * off * SLICE_FLOATS,
                         self.sw[n:n + 1].data_ptr(), self.amax[n:n + 1].data_ptr())
        # head: which source element every head float is (pack_mlp on index-valued
        # parameters); sources = HEAD_SRC parameters flattened (the views bias: bc),
        # then the 9 scales
        src_n = [sum(int(np.prod(p[k].shape)) for k in HEAD_SRC[:i]) for i in range(len(HEAD_SRC))]
        fake = {}
        for k, v in PARAM_SHAPES.items():
            fake["model." + k] = np.zeros(v, np.float32)
        for k, o in zip(HEAD_SRC, src_n):
            shape = tuple(p[k].shape)
            fake["model." + k] = (o + 1 + np.arange(int(np.prod(shape)))).reshape(shape).astype(np.float32)
        _, head = pack_mlp(fake, "model")
        nsrc = src_n[-1] + int(np.prod(p[HEAD_SRC[-1]].shape))
        idx = np.rint(head).astype(np.int64) - 1              # -1: zero
        idx[H_BIAS + 8 * 256:H_BIAS + 9 * 256] = -1             # the feature bias: folded
        idx[H_SCALES:H_SCALES + 10] = -1                        # the feature layer's scale: 0
        for n, (_, _, _, _, li) in enumerate(plan):
            idx[H_SCALES + li] = nsrc + n
        assert idx.max() < nsrc + len(plan) and head.shape[0] == HEAD_FLOATS
        self.head = torch.zeros(HEAD_FLOATS, device=dev, dtype=torch.float32)
        pp = dict(p)
        pp["views_linears.0.bias"] = self.bc
        self._head(_src_pointers(pp, HEAD_SRC, idx, self.amax, nsrc), self.head)

    def pack(self, p):
        """p: parameter name (PARAM_NAMES) -> tensor. Returns (stream, head) on the device."""
        key = tuple((k, v.data_ptr()) for k, v in sorted(p.items()))
        if key != self.key:
            self._build(p)
            self.key = key
        _fold([self])
        self.launch()
        return self.stream, self.head


class X3BwdStreamPacker(_PackSet):
    """The backward chain's weight stream (nerf_mlp_train_backward_x3), packed on
    the device: the transposed matrices in consumption order, each with the
    register-resident K permutation (x3_cols_act) as its column map --
    Wc[:, :256]^T (4 slices; Wc = the fold of the feature layer into the views
    layer, nerf_fold_views, so d h7 comes out of one 128 -> 256 product),
    W_7^T, W_6^T (8 each), the encoding rows of W_5^T (2 slices of 4 tiles x 4
    K steps), the h4 rows of W_5^T, W_4^T .. W_1^T (8 each), W_0^T (2 slices):
    64 slices (the kernel without the encoding products skips slices 20, 21,
    62, 63) -- and its head: the lane-packed rgb and alpha weights at the
    forward head's offsets, the weight scales at 3100 + j (j: Wc 0, W_7 2,
    W_6 3, W_5,enc 4, W_5,h 5, W_4 .. W_1 6 .. 9, W_0 10; slot 1, the unfolded
    feature layer's, stays 0). Wc: the forward packer's fold of the same
    parameters (X3NetPacker), or None: this packer folds them itself."""

    @staticmethod
    def plan():
        from .pack import x3_cols_act
        ar = lambda n: list(range(n))   # noqa: E731
        act = [int(c) for c in x3_cols_act().reshape(-1)]
        act4 = [int(c) for c in x3_cols_act(4).reshape(-1)]
        enc = ar(63) + [-1]
        mats = [("fold", ar(256), act4, 0), ("pts_linears.7.weight", ar(256), act, 2),
                ("pts_linears.6.weight", ar(256), act, 3), ("pts_linears.5.weight", enc, act, 4),
                ("pts_linears.5.weight", [63 + i for i in range(256)], act, 5)]
        mats += [(f"pts_linears.{i}.weight", ar(256), act, 10 - i) for i in (4, 3, 2, 1)]
        mats += [("pts_linears.0.weight", enc, act, 10)]
        out, off = [], 0
        for name, rmap, cmap, j in mats:
            out.append((name, rmap, cmap, off, j))
            off += -(-len(rmap) * len(cmap) // 8192)
        return out, off

    def _build(self, p, Wc=None):
        import numpy as np
        from .pack import H_ALPHA_W, H_RGB_W, HEAD_FLOATS, SLICE_FLOATS, _group_pack
        dev = self.device
        plan, nsl = self.plan()
        self.recs, self.heads, self._keep, self._tables = [], [], [], (None, None)
        self.own_fold = Wc is None
        if Wc is None:   # standalone: its own fold of the parameters
            Wc = self.Wc = torch.zeros((128, 283), device=dev, dtype=torch.float32)
            self.bc = torch.zeros((128,), device=dev, dtype=torch.float32)
            self.fold_ptrs = tuple(p[k].data_ptr() for k in (
                "views_linears.0.weight", "feature_linear.weight", "feature_linear.bias",
                "views_linears.0.bias")) + (self.Wc.data_ptr(), self.bc.data_ptr())
        self.stream = torch.zeros(nsl * SLICE_FLOATS, device=dev, dtype=torch.float32)
        self.sw = torch.zeros(11, device=dev, dtype=torch.int32)
        self.amax = torch.zeros(11, device=dev, dtype=torch.int32)
        for name, rmap, cmap, off, j in plan:
            # transposed: element (i, k) = W[cmap[k]][rmap[i]]
            self._matrix(Wc if name == "fold" else p[name], rmap, cmap, True,
                         self.stream.data_ptr() + 4 * off * SLICE_FLOATS,
                         self.sw[j:j + 1].data_ptr(), self.amax[j:j + 1].data_ptr())
        # head: rgb W [3][4][32] and alpha W [4][64] lane-packed (pack_mlp's layout),
        # then the scales: sources = cat(rgb W (384), alpha W (256)), scales
        idx = np.full(HEAD_FLOATS, -1, np.int64)
        rgb_idx = np.arange(384).reshape(3, 128)
        for c in range(3):
            idx[H_RGB_W + c * 128:H_RGB_W + c * 128 + 128] = _group_pack(rgb_idx[c], 8).reshape(-1)
        idx[H_ALPHA_W:H_ALPHA_W + 256] = 384 + _group_pack(np.arange(256), 16).reshape(-1)
        idx[3100:3111] = 640 + np.arange(11)
        self.head = torch.zeros(HEAD_FLOATS, device=dev, dtype=torch.float32)
        self._head(_src_pointers(p, ["rgb_linear.weight", "alpha_linear.weight"], idx,
                                 self.amax, 640), self.head)

    def pack(self, p):
        key = tuple((k, v.data_ptr()) for k, v in sorted(p.items()))
        if key != self.key:
            self._build(p)
            self.key = key
        _fold([self])
        self.launch()
        return self.stream, self.head


class X3NetPacker:
    """Both fused kernels' streams of one network (X3StreamPacker for the
    forward, X3BwdStreamPacker for the backward), packed together by one
    nerf_x3_pack launch set at the network's forward (the backward of that
    forward reads the same parameters: autograd forbids changing them in
    between), so a training step packs each network once; prepack() packs
    several networks in one launch set for their next forwards."""

    def __init__(self, device):
        self.device = torch.device(device)
        self.fwd = X3StreamPacker(device)
        self.bwd = X3BwdStreamPacker(device)
        self.key = None         # storage key of the built tables
        self.gen = 0            # build generation: every build allocates new buffers
        self.pending = False    # packed by prepack() for the next streams() call
        self.pending_event = None   # prepack(side=True): the pack stream's completion
        # prepack(side=True) also zeroes the max |.| slots of the network's next
        # forward + backward (RayMLPFn) on the pack stream: handed out once
        self.stats = None
        self.stats_ready = False

    def _ensure_built(self, p):
        key = tuple((k, v.data_ptr()) for k, v in sorted(p.items()))
        if key != self.key:
            self.fwd._build(p)
            self.bwd._build(p, self.fwd.Wc)   # Wc^T: the forward's fold, made first
            self.fwd.key = self.bwd.key = self.key = key
            # the build's records point at its own new buffers (stream, scales,
            # maxima, Wc / bc, head): a device table made for an earlier build --
            # even one with the same parameter addresses -- points at freed
            # memory, so the table cache is keyed by the generation too
            self.gen += 1
            self.pending = False

    def records(self):
        return self.fwd.recs + self.bwd.recs, self.fwd.heads + self.bwd.heads

    def streams(self, p):
        """(fwd stream, fwd head, bwd stream, bwd head) of the live parameters:
        packed now, unless prepack() just did."""
        self._ensure_built(p)
        if not self.pending:
            _launch_packs([self])
        elif self.pending_event is not None:
            torch.cuda.current_stream(self.device).wait_event(self.pending_event)
        self.pending = False
        self.pending_event = None
        return self.fwd.stream, self.fwd.head, self.bwd.stream, self.bwd.head

    def take_stats(self):
        """The slots prepack zeroed for this network's next forward, or None."""
        if not (self.pending and self.stats_ready):
            return None
        self.stats_ready = False
        return self.stats

    def invalidate(self):
        self.stats_ready = False
        if self.pending_event is not None:   # a side-stream packing still writing the buffers
            torch.cuda.current_stream(self.device).wait_event(self.pending_event)
        self.pending = False
        self.pending_event = None


_PACK_TABLES = {}


def _launch_packs(nets):
    """One nerf_x3_pack launch set over several networks' records (the tables
    cached per set of built packers)."""
    key = tuple((id(n), n.gen) for n in nets)
    tabs = _PACK_TABLES.get(key)
    if tabs is None:
        recs, heads = [], []
        for n in nets:
            r, h = n.records()
            recs += r
            heads += h
        dev = nets[0].device
        if len(_PACK_TABLES) > 64:
            _PACK_TABLES.clear()
        tabs = _PACK_TABLES[key] = (_device_table(recs, _DESC_FIELDS, dev), len(recs),
                                    _device_table(heads, _HEAD_FIELDS, dev), len(heads))
    descs, n, htab, nh = tabs
    _fold([net.fwd for net in nets])   # the views matrices the packs read
    call("nerf_x3_pack", ptr(descs), n, ptr(htab), nh, _lib.stream_of(nets[0].device))


_NETS = {}
_STATS = {}   # prepack's zeroed amax / dmax slots, one buffer per set of networks


def _net_for(params, device):
    p = dict(zip(PARAM_NAMES, params))
    key = p["pts_linears.0.weight"].data_ptr()
    net = _NETS.get(key)
    if net is None:
        net = _NETS[key] = X3NetPacker(device)
    return net, p


def prepack(networks, side=False):
    """Pack the fused kernels' streams of several networks (each a list of its
    24 parameters in PARAM_NAMES order, or a NeRF module) in ONE launch set;
    each network's next forward uses them instead of packing (a training step
    calls it right before its forwards, after the previous optimizer step).
    side=True: the launch set runs on a side stream (after everything already
    on the current one), and each network's next forward makes its stream
    wait for it -- the launches between (draws, coarse depths) overlap it."""
    nets = []
    for params in networks:
        if isinstance(params, torch.nn.Module):
            params = mlp_params(params)
        net, p = _net_for(params, params[0].device)
        net._ensure_built(p)
        nets.append(net)
    if nets:
        ev = None
        if side:
            dev = nets[0].device
            ps = _side_stream(dev, "pack")
            ps.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(ps):
                _launch_packs(nets)
                # every network's amax / dmax slots in one buffer: one fill
                key = tuple(id(n) for n in nets)
                buf = _STATS.get(key)
                if buf is None or buf.device != dev:
                    buf = _STATS[key] = torch.empty(25 * len(nets), device=dev,
                                                    dtype=torch.float32)
                buf.zero_()
                for i, n in enumerate(nets):
                    n.stats = buf[25 * i:25 * (i + 1)]
                    n.stats_ready = True
            ev = torch.cuda.Event()
            ev.record(ps)
        else:
            _launch_packs(nets)
        for n in nets:
            n.pending = True
            n.pending_event = ev


def invalidate_packs():
    """Drop prepack()'s packing: every network's next forward packs again."""
    for net in _NETS.values():
        net.invalidate()


class _BwdIO(ctypes.Structure):
    """NerfX3BwdIO (include/nerfhip.h)."""
    _fields_ = [("d_raw", ctypes.c_void_p), ("bits", ctypes.c_void_p * 9),
                ("d", ctypes.c_void_p * 12), ("dmax", ctypes.c_void_p), ("ld", ctypes.c_int64),
                ("d_raw_t", ctypes.c_void_p), ("bs", ctypes.c_int64)]


class _TrainOut(ctypes.Structure):
    """NerfX3TrainOut (include/nerfhip.h)."""
    _fields_ = [("act", ctypes.c_void_p * 12), ("bits", ctypes.c_void_p * 9),
                ("amax", ctypes.c_void_p), ("ld", ctypes.c_int64), ("bs", ctypes.c_int64)]


_PACKERS = {}
_ZERO = {}


def _streams_for(params, device):
    """(fwd stream, fwd head, bwd stream, bwd head) of the network whose
    parameters these are, for its forward and that forward's backward."""
    net, p = _net_for(params, device)
    return net.streams(p)


def _packs_for(params, device, forward=True, backward=True):
    """Packed matrices of the network whose weight tensors these are (one packer
    per network and direction set, keyed by the first weight's storage);
    forward=False / backward=False: without that direction's matrices (the fused
    kernels stream their own)."""
    p = dict(zip(PARAM_NAMES, params))
    key = (p["pts_linears.0.weight"].data_ptr(), forward, backward)
    pk = _PACKERS.get(key)
    if pk is None:
        pk = _PACKERS[key] = X3Packer(device, forward=forward, backward=backward)
    return pk.pack(p)


def _layer(wp, sw, mt, nk, B, C, P, bias=None, relu=False, mask=None, ru=None, rw=None,
           amax=None, bits_out=None, mask_bits=None, head=None):
    """One nerf_x3_layer launch; amax (a device float, >= 0) is raised to max |C|.
    bits_out (int16 words, relu only) receives the ReLU mask of C as bits;
    mask_bits (such words, instead of mask) masks C; head = (W [n, 16 mt], b [n],
    out [P, 4], column): out[:, column:column + n] = C^T W^T + b
    (nerf_x3_layer_ex)."""
    if bits_out is None and mask_bits is None and head is None:
        call("nerf_x3_layer", ptr(wp), ptr(sw), mt, nk, ptr(bias), ptr(B), B.stride(0),
             ptr(mask), mask.stride(0) if mask is not None else 0, ptr(ru), ptr(rw), int(relu),
             ptr(C), C.stride(0), P, ptr(amax), _lib.stream_of(C.device))
        return
    hw, hb, hout, hcol = head if head is not None else (None, None, None, 0)
    call("nerf_x3_layer_ex", ptr(wp), ptr(sw), mt, nk, ptr(bias), ptr(B), B.stride(0),
         ptr(mask), mask.stride(0) if mask is not None else 0, ptr(ru), ptr(rw), int(relu),
         ptr(C), C.stride(0), P, ptr(amax), ptr(bits_out), ptr(mask_bits), ptr(hw), ptr(hb),
         hw.shape[0] if hw is not None else 0, ptr(hout), hcol, _lib.stream_of(C.device))


def relu_bits_words(P, m_tiles):
    """int16 words of one layer's ReLU mask (nerf_x3_layer_bits layout)."""
    return -(-P // 128) * 128 * m_tiles


def _encode(x, n_freq, out, amax):
    """out[j][p] = freq_encode(x)[p][j] (x [P, 3] contiguous, out a row-strided
    [3 + 6 n_freq, P] view); amax (a [1] device float) raised to max |out|."""
    call("nerf_freq_encode_fm", ptr(x), 3, x.shape[0], n_freq, ptr(out), out.stride(0),
         ptr(amax), _lib.stream_of(x.device))


def _absmax(x):
    """max |x| as a [1] device tensor (one reduction pass)."""
    return torch.linalg.vector_norm(x, float("inf")).reshape(1)


def _wgrad(A, B, amax_a=None, amax_b=None, with_bias=False):
    """sum over samples of A[m][p] B[n][p] -> [M, N] (A [M][P], B [N][P]); with_bias:
    also sum_p A[m][p] -> [M]. amax_a / amax_b: max |A|, max |B| when known."""
    M, P = A.shape
    N = B.shape[0]
    chunk = wgrad_chunk(P)
    chunks = max(1, -(-P // chunk))
    part = torch.empty((chunks, M, N), device=A.device, dtype=torch.float32)
    bpart = torch.empty((chunks, M), device=A.device, dtype=torch.float32) if with_bias else None
    amax_a = _absmax(A) if amax_a is None else amax_a
    amax_b = _absmax(B) if amax_b is None else amax_b
    st = _lib.stream_of(A.device)
    call("nerf_x3_wgrad", ptr(A), A.stride(0), M, ptr(B), B.stride(0), N, P, chunk,
         ptr(amax_a), ptr(amax_b), ptr(part), ptr(bpart), st)
    dw = torch.empty((M, N), device=A.device, dtype=torch.float32)
    call("nerf_sum_partials", ptr(part), chunks, M * N, ptr(dw), st)
    if not with_bias:
        return dw
    db = torch.empty((M,), device=A.device, dtype=torch.float32)
    call("nerf_sum_partials", ptr(bpart), chunks, M, ptr(db), st)
    return dw, db


class _WgradDesc(ctypes.Structure):
    """NerfWgradDesc (include/nerfhip.h)."""
    _fields_ = [("A", ctypes.c_void_p), ("lda", ctypes.c_int64), ("B", ctypes.c_void_p),
                ("ldb", ctypes.c_int64), ("P", ctypes.c_int64), ("amax_a", ctypes.c_void_p),
                ("amax_b", ctypes.c_void_p), ("part", ctypes.c_void_p),
                ("ldpart", ctypes.c_int64), ("bias_part", ctypes.c_void_p),
                ("ldbias", ctypes.c_int64), ("M", ctypes.c_int), ("N", ctypes.c_int),
                ("amax_a2", ctypes.c_void_p), ("amax_b2", ctypes.c_void_p),
                ("ldo", ctypes.c_int64), ("bsa", ctypes.c_int64), ("bsb", ctypes.c_int64),
                ("a2_row", ctypes.c_int)]


_NCU = {}


def _n_cu(device):
    d = torch.device(device)
    if d not in _NCU:
        _NCU[d] = torch.cuda.get_device_properties(d).multi_processor_count
    return _NCU[d]


def _dma_ok(t):
    if isinstance(t, BlockRows):
        return t.data_ptr() % 16 == 0
    return t.stride(1) == 1 and t.stride(0) % 4 == 0 and t.data_ptr() % 16 == 0


BLOCK = 16   # samples per block of the T16 layout


class BlockRows:
    """Rows r0 .. r0 + M of an [R, P] activation in the T16 layout of the fused
    training kernels (mlp_x3.hip Lay; NerfX3TrainOut.bs): buf is [nb, R, 16]
    (nb = ceil(P / 128) * 8 blocks of 16 samples: whole 128-sample tiles, R a
    multiple of 16); inside a block each 16-row group is one 1-KiB tile in
    which row 16 t + 4 g + q of sample s sits at t * 256 + q * 64 + g * 16 + s.
    So element q of every lane of a 16 x 16 MFMA accumulator tile (lane
    16 g + s holds rows 4 g .. 4 g + 3 of sample s) is 256 contiguous bytes: the
    training kernels write their outputs as whole lines, one store instruction
    per accumulator element, and a K step of the weight gradients (32 samples)
    reads two contiguous runs per operand (NerfWgradDesc bsa / bsb). Operands
    start on 16-row groups (r0 % 16 == 0)."""

    def __init__(self, buf, r0, M, P):
        assert buf.dim() == 3 and buf.shape[2] == BLOCK and buf.is_contiguous()
        assert buf.shape[1] % 16 == 0 and r0 % 16 == 0
        assert 0 <= r0 and r0 + M <= buf.shape[1] and buf.shape[0] * BLOCK >= P
        self.buf, self.r0, self.M, self.P = buf, int(r0), int(M), int(P)
        self.shape = (self.M, self.P)
        self.device = buf.device

    @staticmethod
    def alloc(R, P, dev):
        R = -(-R // 16) * 16
        nb = -(-P // 128) * (128 // BLOCK)
        return BlockRows(torch.empty((nb, R, BLOCK), device=dev, dtype=torch.float32), 0, R, P)

    def rows(self, a, b):
        """Rows a .. b of this operand (a view; a on a 16-row group)."""
        return BlockRows(self.buf, self.r0 + a, b - a, self.P)

    def data_ptr(self):
        return self.buf.data_ptr() + 4 * BLOCK * self.r0

    def numel(self):   # the whole buffer: the operand's extent lies inside it
        return self.buf.numel()

    def stride(self, dim):   # NerfWgradDesc lda (unused in T16) and bs
        return BLOCK if dim == 0 else 1

    @property
    def block_stride(self):
        return BLOCK * self.buf.shape[1]

    def _grid(self):
        nb, R, _ = self.buf.shape
        return self.buf.view(nb, R // 16, 4, 4, BLOCK)   # [b, t, q, g, s]

    def dense(self):
        """The same rows feature-major, [M, P] (tests, the fallback paths)."""
        nb, R, _ = self.buf.shape
        full = self._grid().permute(1, 3, 2, 0, 4).reshape(R, nb * BLOCK)   # row 16t + 4g + q
        return full[self.r0:self.r0 + self.M, :self.P]

    @staticmethod
    def from_dense(A, R=None):
        """A [M, P] copied into a new T16 buffer (tests, tools)."""
        M, P = A.shape
        out = BlockRows.alloc(R or M, P, A.device)
        nb, Rr, _ = out.buf.shape
        full = torch.zeros((Rr, nb * BLOCK), device=A.device, dtype=torch.float32)
        full[:M, :P] = A
        out._grid().copy_(full.view(Rr // 16, 4, 4, nb, BLOCK).permute(3, 0, 2, 1, 4))
        return out.rows(0, M)


def rows_of(t, a, b):
    """Rows a .. b of a feature-major tensor or a BlockRows operand."""
    return t.rows(a, b) if isinstance(t, BlockRows) else t[a:b]


WGRAD_COST_FLOOR = int(_os.environ.get("NERF_WGRAD_COST_FLOOR", "512"))


def wgrad_tile_chunks(shapes, P, n_cu=256, floor=None):
    """Memoised (the search repeats every backward with the same arguments)."""
    return list(_wgrad_tile_chunks(tuple(tuple(int(v) for v in s) for s in shapes), int(P),
                                   int(n_cu), floor))


@functools.lru_cache(maxsize=64)
def _wgrad_tile_chunks(shapes, P, n_cu, floor):
    """K split of every 256 x 256 output tile of a batched weight-gradient
    launch (order: descriptor, N tile, M tile): proportional to the operand
    rows the tile streams per K step (A rows + B rows, at least 128: a step
    has fixed costs), scaled so all tiles' workgroups fit one per CU -- a
    light tile (the heads, the 32- / 64-row remainders) finishes its share
    of the samples as late as a full one. shapes: (M, N) per descriptor."""
    costs = []
    for M, N in shapes:
        for j in range(-(-N // 256)):
            for i in range(-(-M // 256)):
                rows = min(256, M - 256 * i) + min(256, N - 256 * j)
                costs.append(max(rows, WGRAD_COST_FLOOR if floor is None else floor) / 512.0)
    cap = max(1, min(P // 32, 255))
    zs = [1] * len(costs)
    lam = 1.0
    while True:   # the largest scale whose workgroups fit the CUs
        nz = [max(1, min(cap, int(c * lam))) for c in costs]
        if sum(nz) > n_cu or nz == zs and lam > 4 * n_cu:
            break
        zs = nz
        lam *= 1.02
    return zs


class WgradBatch:
    """The weight gradients of one backward, deferred and computed together by
    ONE nerf_x3_wgrad_batch_z launch (each 256 x 256 output tile split over
    sample subsets, the split sized to the tile's rows: wgrad_tile_chunks), then
    ONE fixed-order partial sum for all weights and one for all biases.
    add() returns a slot; results()[slot] = (dW[, db]). Requests whose operands
    the batched kernel cannot take (P % 32, alignment) run through _wgrad."""

    def __init__(self, device):
        self.device = device
        self.req = []

    def add(self, A, B, amax_a=None, amax_b=None, with_bias=False, width=None, into=None,
            a_split=0):
        """width: the result has `width` columns, B's rows the first of them;
        into = (slot, c0): B's rows are columns c0 .. of slot's result (the
        same A; no result of its own). One contiguous gradient from operands in
        two buffers (the skip layer's [encoding | h4]).
        amax_a = (m1, m2) with a_split = r (a multiple of 16): A's rows < r take
        m1's FP16 split range, rows >= r m2's (two producers' rows in one
        operand, each at its own scale); a_split 0: one scale, max(m1, m2)."""
        if amax_a is None:
            amax_a = _absmax(A.dense() if isinstance(A, BlockRows) else A)
        if amax_b is None:
            amax_b = _absmax(B.dense() if isinstance(B, BlockRows) else B)
        assert not a_split or (isinstance(amax_a, tuple) and a_split % 16 == 0
                               and 0 < a_split < A.shape[0])
        self.req.append((A, B, amax_a, amax_b, with_bias, width, into, a_split))
        return len(self.req) - 1

    def results(self):
        req, self.req = self.req, []
        if not req:
            return []
        P = req[0][0].shape[1]
        blocked = any(isinstance(t, BlockRows) for r in req for t in r[:2])
        ok = (len(req) <= 16 and P % 32 == 0 and
              all(A.shape[1] == P and B.shape[1] == P and _dma_ok(A) and _dma_ok(B)
                  and A.numel() * 4 < (1 << 31) and B.numel() * 4 < (1 << 31)
                  for A, B, *_ in req))
        if not ok:
            one = lambda m: torch.maximum(*m) if isinstance(m, tuple) else m   # noqa: E731
            dn = lambda t: t.dense() if isinstance(t, BlockRows) else t   # noqa: E731
            assert not blocked or P % 32 != 0, "block-layout operands the batch cannot take"

            def wg(A, B, aa, ab, wb, r):
                if not r:
                    return _wgrad(dn(A), dn(B), one(aa), one(ab), wb)
                # two row blocks of A, each at its own scale (as the batched kernel)
                lo, hi = (_wgrad(dn(A)[rows], dn(B), m, one(ab), wb)
                          for rows, m in ((slice(0, r), aa[0]), (slice(r, None), aa[1])))
                if wb:
                    return torch.cat([lo[0], hi[0]]), torch.cat([lo[1], hi[1]])
                return torch.cat([lo, hi])
            res = [wg(A, B, aa, ab, wb, r) for A, B, aa, ab, wb, _, _, r in req]
            for k, (A, B, _, _, wb, width, into, _) in enumerate(req):
                if into is not None:   # the column blocks joined on the host
                    s, c0 = into
                    tgt = res[s][0] if isinstance(res[s], tuple) else res[s]
                    blk = res[k][0] if isinstance(res[k], tuple) else res[k]
                    tgt[:, c0:c0 + B.shape[0]] = blk
                    res[k] = None
                elif width is not None and width != B.shape[0]:
                    dw = res[k][0] if isinstance(res[k], tuple) else res[k]
                    full = torch.zeros((A.shape[0], width), device=dw.device, dtype=dw.dtype)
                    full[:, :B.shape[0]] = dw
                    res[k] = (full, res[k][1]) if isinstance(res[k], tuple) else full
            return res
        zs = wgrad_tile_chunks([(A.shape[0], B.shape[0]) for A, B, *_ in req], P, _n_cu(self.device))
        Z = max(zs)
        # output regions: [M][width] per request that owns one; joined requests
        # write their column block of the owner's region
        region, ld = {}, 0
        for k, (A, B, _, _, _, width, into, _) in enumerate(req):
            if into is None:
                region[k] = (ld, width or B.shape[0])
                ld += A.shape[0] * (width or B.shape[0])
        bsizes = [A.shape[0] if wb else 0 for A, _, _, _, wb, _, _, _ in req]
        ldb = sum(bsizes)
        # weight and bias partials side by side in one [Z][ld + ldb] array: one
        # fixed-order sum for both
        ldt = ld + ldb
        part = torch.empty((Z, ldt), device=self.device, dtype=torch.float32)
        descs = (_WgradDesc * len(req))()
        boff = 0
        def two(m):   # a scale given as (tensor, tensor): the kernel takes their max
            return (m[0].data_ptr(), m[1].data_ptr()) if isinstance(m, tuple) else (m.data_ptr(), None)
        for k, (A, B, aa, ab, wb, width, into, a_split) in enumerate(req):
            (a1, a2), (b1, b2) = two(aa), two(ab)
            off, wdt = region[into[0]] if into is not None else region[k]
            off += into[1] if into is not None else 0
            bs = lambda t: t.block_stride if isinstance(t, BlockRows) else 0   # noqa: E731
            descs[k] = _WgradDesc(A.data_ptr(), A.stride(0), B.data_ptr(), B.stride(0), P,
                                  a1, b1, part.data_ptr() + 4 * off, ldt,
                                  part.data_ptr() + 4 * (ld + boff) if wb else None, ldt,
                                  A.shape[0], B.shape[0], a2, b2, wdt, bs(A), bs(B), a_split)
            boff += bsizes[k]
        st = _lib.stream_of(self.device)
        zarr = (ctypes.c_int * len(zs))(*zs)
        call("nerf_x3_wgrad_batch_z", ctypes.addressof(descs), len(req), zarr, Z, st)
        total = torch.empty((ldt,), device=self.device, dtype=torch.float32)
        call("nerf_sum_partials", ptr(part), Z, ldt, ptr(total), st)
        flat, bflat = total[:ld], total[ld:]
        out, boff = [], 0
        for k, (A, B, _, _, wb, _, into, _) in enumerate(req):
            if into is not None:
                out.append(None)
                continue
            off, wdt = region[k]
            dw = flat[off:off + A.shape[0] * wdt].view(A.shape[0], wdt)
            if wb:
                out.append((dw, bflat[boff:boff + bsizes[k]]))
                boff += bsizes[k]
            else:
                out.append(dw)
        return out


PARAM_NAMES = ([f"pts_linears.{i}.{k}" for i in range(8) for k in ("weight", "bias")] +
               ["alpha_linear.weight", "alpha_linear.bias", "feature_linear.weight",
                "feature_linear.bias", "views_linears.0.weight", "views_linears.0.bias",
                "rgb_linear.weight", "rgb_linear.bias"])
# shapes of one NeRF's parameters (network.py:9-47) and the head's sources
PARAM_SHAPES = {**{f"pts_linears.{i}.weight": (256, 63 if i == 0 else 319 if i == 5 else 256)
                   for i in range(8)},
                **{f"pts_linears.{i}.bias": (256,) for i in range(8)},
                "alpha_linear.weight": (1, 256), "alpha_linear.bias": (1,),
                "feature_linear.weight": (256, 256), "feature_linear.bias": (256,),
                "views_linears.0.weight": (128, 283), "views_linears.0.bias": (128,),
                "rgb_linear.weight": (3, 128), "rgb_linear.bias": (3,)}
HEAD_SRC = ([f"pts_linears.{i}.bias" for i in range(8)] +
            ["feature_linear.bias", "views_linears.0.bias", "alpha_linear.weight",
             "alpha_linear.bias", "rgb_linear.weight", "rgb_linear.bias"])


# The forward as one fused launch (nerf_mlp_train_forward_x3) instead of ten
# layer launches, the backward's chain of products likewise
# (nerf_mlp_train_backward_x3); NERF_TRAIN_FUSED_FORWARD=0 /
# NERF_TRAIN_FUSED_BACKWARD=0 select the layer launches (the parity tests run
# both).
FUSED_FORWARD = _os.environ.get("NERF_TRAIN_FUSED_FORWARD", "1") != "0"
FUSED_BACKWARD = _os.environ.get("NERF_TRAIN_FUSED_BACKWARD", "1") != "0"

# Row padding of the feature-major activations: a row stride of P + 32 floats
# (not P, a multiple of 2^13 at the C3 sizes) spreads the rows' same-sample
# segments over HBM channels; measured on the weight-gradient kernel at P =
# 196 608: 138 -> 114 us (tools/train_kernels_bench.py).
ACT_PAD = 32


def _act(F, P, dev):
    """An uninitialised [F, P] activation tensor with row stride P + ACT_PAD."""
    return torch.empty((F, P + ACT_PAD), device=dev, dtype=torch.float32)[:, :P]


def _padded(W, cols, K):
    """[M, K] with W's columns at positions `cols` (the rest zero)."""
    out = torch.zeros((W.shape[0], K), device=W.device, dtype=torch.float32)
    out[:, cols] = W
    return out


# The fused forward + fused backward write their rows in the T16 layout
# (BlockRows: whole-line stores, contiguous weight-gradient K steps);
# NERF_TRAIN_T16=0 keeps them feature-major. The layer launches are
# feature-major only, so T16 needs both fused kernels.
T16 = _os.environ.get("NERF_TRAIN_T16", "1") != "0"
# the forward's rows in one T16 buffer (16-row groups): E = [enc 64 | h4 256],
# V = [h7 256 | view enc 32], HV 128, then h0..h3, h5, h6
_FWD_ROWS = {"E": (0, 320), "V": (320, 608), "HV": (608, 736)}
_FWD_H = {0: 736, 1: 992, 2: 1248, 3: 1504, 5: 1760, 6: 2016}
_FWD_R = 2272
# the fused backward's rows: hx = [d_hv 128 | d sigma, 15 spare | d rgb 3, 13 spare]
# (every wgrad operand starts a 16-row group), D0..D7, d_enc5, d_enc0
_BWD_HX, _BWD_D, _BWD_E5, _BWD_E0, _BWD_R = 0, 160, 2208, 2272, 2336


def _t16_ok(P):
    """T16 for a pass of P samples: the larger (backward) buffer within the 2 GiB
    of the kernels' 32-bit buffer offsets (P <= 229 760: a 1024-ray C3 step's
    fine pass is 196 608; larger passes stay feature-major)."""
    return T16 and 0 < P and -(-P // 128) * 128 * _BWD_R * 4 < (1 << 31)


def _fwd_rows_t16(buf, P):
    """E, H (h4 / h7 as rows of E / V), V, HV as BlockRows over one T16 buffer."""
    fb = BlockRows(buf, 0, _FWD_R, P)
    E = fb.rows(*_FWD_ROWS["E"])
    V = fb.rows(*_FWD_ROWS["V"])
    HV = fb.rows(*_FWD_ROWS["HV"])
    H = [fb.rows(r, r + 256) if i in _FWD_H else None for i, r in
         ((i, _FWD_H.get(i, 0)) for i in range(8))]
    H[4] = E.rows(64, 320)
    H[7] = V.rows(0, 256)
    return E, H, V, HV


class NerfMLPFn(torch.autograd.Function):
    """raw [P, 4] = NeRF(cat(freq_encode(pts), freq_encode(dirs))) on x3 kernels.
    Inputs: pts [P, 3] (gradient returned when it requires one), dirs [P, 3]
    (no gradient, as in the reference where view directions are constants),
    then the 24 parameters in PARAM_NAMES order."""

    @staticmethod
    def forward(ctx, pts, dirs, *params):
        p = dict(zip(PARAM_NAMES, params))
        dev = pts.device
        P = pts.shape[0]
        f32 = torch.float32
        E = _act(320, P, dev)           # cat(enc, pad, h4)
        # max |.| of every saved activation (the weight-gradient scales): slots
        # 0-7 = h0..h7 and 8 = feature from the layer kernels, 9 = xyz encoding,
        # 10 = view encoding (both from the encoding kernel), 11 = views layer
        stats = torch.zeros(25, device=dev, dtype=f32)   # amax + the backward's dmax: one fill
        amax, ctx.dmax_buf = stats[:12], stats[12:]
        pts_c = pts.detach().contiguous()
        # the fused backward reads the fused forward's rows (V = [h7; view enc]:
        # with the feature layer folded there is no d feature for the layer
        # launches' feature-row weight gradient): it follows the fused forward
        fused_f = FUSED_FORWARD and P > 0
        fused_b = FUSED_BACKWARD and fused_f
        if fused_f and fused_b and _t16_ok(P):
            ctx.fused_backward = True
            ctx.streams = _streams_for(params, dev)
            return NerfMLPFn._forward_fused(ctx, pts, pts_c, dirs, params, None, None, amax,
                                            None)
        if not fused_f:   # (the fused forward writes the encoding rows itself)
            _encode(pts_c, XYZ_FREQS, E, amax[9:10])               # E[:63] = enc^T
            E[63].zero_()
        H = [_act(256, P, dev) if i not in (4, 7) or (i == 7 and not fused_f) else None
             for i in range(8)]                      # h4 rows: E; fused: h7 rows in V
        H[4] = E[64:320]
        pk = None if fused_f and fused_b else \
            _packs_for(params, dev, forward=not fused_f, backward=not fused_b)
        ctx.fused_backward = fused_b
        # the fused kernels' weight streams (both directions, one packing)
        ctx.streams = _streams_for(params, dev) if fused_f or fused_b else None
        if fused_f:
            return NerfMLPFn._forward_fused(ctx, pts, pts_c, dirs, params, E, H, amax, pk)
        src = E[0:64]
        # the ReLU masks of h0..h7 as bits for the dgrad launches (32 B per sample
        # and layer instead of re-reading the 1 KiB of FP32 activations)
        bits = torch.empty((8, relu_bits_words(P, 16)), device=dev, dtype=torch.int16)
        raw = torch.empty((P, 4), device=dev, dtype=f32)   # heads write straight into it
        for i in range(8):
            wp, sw, mt, nk = pk[f"fwd{i}"]
            B = E if i == 5 else src
            _layer(wp, sw, mt, nk, B, H[i], P, bias=p[f"pts_linears.{i}.bias"], relu=True,
                   amax=amax[i:i + 1], bits_out=bits[i],
                   head=((p["alpha_linear.weight"], p["alpha_linear.bias"], raw, 3)
                         if i == 7 else None))                  # NET:61 alpha on h7
            src = H[i]
        h7 = H[7]
        V = _act(288, P, dev)           # cat(feature, views enc)
        V[283:].zero_()                                            # feature rows: its layer
        wf, swf, mt, nk = pk["fwd_feat"]
        _layer(wf, swf, mt, nk, h7, V[0:256], P, bias=p["feature_linear.bias"], relu=False,
               amax=amax[8:9])
        _encode(dirs.detach().contiguous(), DIR_FREQS, V[256:283], amax[10:11])
        wv, swv, mt, nk = pk["fwd_views"]
        HV = _act(128, P, dev)
        bits_v = torch.empty((relu_bits_words(P, 8),), device=dev, dtype=torch.int16)
        _layer(wv, swv, mt, nk, V, HV, P, bias=p["views_linears.0.bias"], relu=True,
               amax=amax[11:12], bits_out=bits_v,
               head=(p["rgb_linear.weight"], p["rgb_linear.bias"], raw, 0))   # NET:68-70
        ctx.save_for_backward(pts_c, E, *H[:4], *H[5:], V, HV, amax, bits, bits_v, *params)
        ctx.pts_grad = pts.requires_grad
        ctx.packs = pk
        return raw

    @staticmethod
    def _forward_fused(ctx, pts, pts_c, dirs, params, E, H, amax, pk, rays=None):
        """The forward as ONE nerf_mlp_train_forward_x3 launch (the inference
        kernel's per-tile body over the unfolded stream, writing every layer's
        output rows, ReLU bits and max |.|): what the ten layer launches of the
        unfused forward produce, and the backward reads. rays = (rays_o, rays_d,
        z) (RayMLPFn): the samples o + d z of the rays instead of pts / dirs."""
        dev = amax.device
        P = (pts_c.shape[0] if rays is None else rays[2].numel())
        stream, head = ctx.streams[:2]
        t16 = E is None    # the T16 layout: every row in one buffer (_fwd_rows_t16)
        if t16:
            fbuf = BlockRows.alloc(_FWD_R, P, dev).buf
            E, H, V, HV = _fwd_rows_t16(fbuf, P)
        else:
            V = _act(288, P, dev)   # cat(feature, views enc, 5 zero rows): all from the kernel
            HV = _act(128, P, dev)
        dirs_c = dirs.detach().contiguous() if rays is None else None
        bits = torch.empty((8, relu_bits_words(P, 16)), device=dev, dtype=torch.int16)
        bits_v = torch.empty((relu_bits_words(P, 8),), device=dev, dtype=torch.int16)
        raw = torch.empty((P, 4), device=dev, dtype=torch.float32)
        zero = _ZERO.get(str(dev))
        if zero is None:
            zero = _ZERO[str(dev)] = torch.zeros(1, device=dev, dtype=torch.float32)
        # h7 goes into V's first 256 rows and the feature rows are not stored: the
        # views layer's weight gradient is taken through h7 (G = d_hv [h7; enc]^T,
        # then G W_feat^T), which also gives the feature layer's (W_views,feat^T G),
        # so neither the feature rows nor their gradient DF ever reach HBM
        H[7] = rows_of(V, 0, 256)
        out = _TrainOut()
        for i in range(8):
            out.act[i] = H[i].data_ptr()
            out.bits[i] = bits[i].data_ptr()
        out.act[8] = None
        ctx.v_h7 = True
        out.act[9] = HV.data_ptr()
        out.act[10] = rows_of(E, 0, 64).data_ptr()
        out.act[11] = rows_of(V, 256, 288).data_ptr()
        out.bits[8] = bits_v.data_ptr()
        out.amax = amax.data_ptr()
        if t16:
            out.ld, out.bs = BLOCK, E.block_stride
            saved = (fbuf,)
        else:
            out.ld, out.bs = H[0].stride(0), 0
            assert all(t.stride(0) == out.ld for t in (E, V, HV)) and H[0].stride(1) == 1
            saved = (E, *H[:4], *H[5:], V, HV)
        ctx.t16 = t16
        if rays is None:
            call("nerf_mlp_train_forward_x3", ptr(stream), ptr(head), ptr(pts_c), ptr(dirs_c),
                 ptr(zero), P, ctypes.addressof(out), ptr(raw), _lib.stream_of(dev))
            ctx.save_for_backward(pts_c, *saved, amax, bits, bits_v, *params)
            ctx.pts_grad = pts.requires_grad
        else:
            ro, rd, z = rays
            n, S = z.shape
            call("nerf_mlp_train_forward_x3_rays", ptr(stream), ptr(head), ptr(ro), ptr(rd),
                 ptr(z), S, n, S, ctypes.addressof(out), ptr(raw), _lib.stream_of(dev))
            # the rays' directions stand where the points do: d z = sum_c d pts_c d_c
            ctx.save_for_backward(rd, *saved, amax, bits, bits_v, *params)
        ctx.packs = pk
        return raw

    @staticmethod
    def backward(ctx, d_raw):
        P = d_raw.shape[0]
        t16 = getattr(ctx, "t16", False)
        if t16:
            pts, fbuf, amax, bits, bits_v, *params = ctx.saved_tensors
            E, H, V, HV = _fwd_rows_t16(fbuf, P)
        else:
            pts, E, H0, H1, H2, H3, H5, H6, H7, V, HV, amax, bits, bits_v, *params = \
                ctx.saved_tensors
            H = [H0, H1, H2, H3, E[64:320], H5, H6, H7]
        p = dict(zip(PARAM_NAMES, params))
        pk = getattr(ctx, "packs", None)
        dev = d_raw.device
        f32 = torch.float32
        grads = {}
        v_h7 = getattr(ctx, "v_h7", False)   # V = [h7; view enc] (fused forward)
        # fused forward + backward: the alpha head's gradient rides on the views
        # layer's G tile (A = [d_hv; d sigma], both read against [h7; enc]), so the
        # fused backward writes d raw feature-major right behind d_hv (rows 128:
        # d sigma, 129..131: d rgb) and no separate alpha tile re-reads h7
        heads_merged = ctx.fused_backward and v_h7
        bbuf = BlockRows.alloc(_BWD_R, P, dev) if t16 else None   # the backward's rows
        if heads_merged:
            HX = bbuf.rows(_BWD_HX, _BWD_HX + 160) if t16 else _act(132, P, dev)
            d_sig = rows_of(HX, 128, 129)
            d_rgb = rows_of(HX, 144, 147) if t16 else HX[129:132]
        else:
            # d_raw^T (the rgb / alpha heads' wgrad operands; the layer launches'
            # d hv K step: 32 rows, 4 of them d_raw)
            DR = torch.empty((4, P), device=dev, dtype=f32) if ctx.fused_backward else \
                torch.zeros((32, P), device=dev, dtype=f32)
            DR[:4].copy_(d_raw.t())
            d_rgb, d_sig = DR[0:3], DR[3:4]
        wb = WgradBatch(dev)   # every weight gradient below: one batched launch at the end
        post = {}              # slot -> (weight name, bias name or None, column fix-up)
        # max |d| of each product (slots as NerfX3BwdIO.dmax); [11] / [12]: of
        # d rgb / d sigma
        # (zeroed with the forward's maxima; a second backward of the same graph
        # only raises them further: a larger scale, still a valid one)
        dmax = getattr(ctx, "dmax_buf", None)
        if dmax is None:
            dmax = torch.zeros(13, device=dev, dtype=f32)
        d_raw_c = d_raw.detach().to(f32).contiguous()
        if d_raw_c.data_ptr() % 16:
            d_raw_c = d_raw_c.clone()
        if not ctx.fused_backward:   # (the fused backward kernel raises [11] / [12] itself)
            call("nerf_raw_absmax", ptr(d_raw_c), P, ptr(dmax[11:]), _lib.stream_of(dev))
        # the heads' bias gradients come out of the batched launch too (its row
        # sums), not from separate reductions over P
        rays_S = getattr(ctx, "rays_S", 0)   # RayMLPFn: the gradient goes to z [n, S]
        need_enc = ctx.pts_grad and ctx.needs_input_grad[2 if rays_S else 0]
        if ctx.fused_backward:
            d_hv, DF, D, d_enc = NerfMLPFn._backward_fused(
                d_raw_c, ctx.streams[2:], bits, bits_v, dmax, need_enc,
                HX if heads_merged else None, bbuf)
        else:
            d_hv, DF, D, d_enc = NerfMLPFn._backward_layers(DR, p, pk, bits, bits_v, dmax,
                                                            need_enc)
        # T16: the view encoding rows and HV are adjacent forward rows (_FWD_ROWS),
        # d_hv / d sigma / d rgb adjacent backward rows (HX): the views layer's
        # encoding columns and the rgb head share ONE 147 x 160 tile,
        # [d_hv; d sigma; d rgb] [enc; HV]^T, of which they are two blocks (the
        # rest is discarded), instead of a 144 x 32 and a 16 x 128 tile: the
        # batched launch's cost goes by tiles (a K step of a light tile costs
        # about what a full one does, profiles/r5_wgrad_stream_studies/)
        enc_rgb = heads_merged and t16 and ENC_RGB_TILE
        if enc_rgb:
            post[wb.add(rows_of(HX, 0, 147), V.rows(256, 416), (dmax[10:11], dmax[11:12]),
                        (amax[10:11], amax[11:12]), with_bias=True, a_split=144)] = (
                "views_enc_rgb", "views_enc_rgb_bias", None)
        else:
            post[wb.add(d_rgb, HV, dmax[11:12], amax[11:12], with_bias=True)] = (
                "rgb_linear.weight", "rgb_linear.bias", None)
        if enc_rgb:   # [G; g_alpha] = [d_hv; d sigma] h7^T (the encoding columns: above)
            post[wb.add(rows_of(HX, 0, 129), V.rows(0, 256), (dmax[10:11], dmax[12:13]),
                        amax[7:8], with_bias=True, a_split=128)] = (
                "views_G", "views_GA_bias", None)
        elif heads_merged:   # [G; g_alpha] = [d_hv; d sigma] [h7; enc]^T
            # d sigma (row 128) keeps its own FP16 split range: rows 128.. at
            # max |d sigma|, not at max |d hv| (a much larger d hv would flush it)
            post[wb.add(rows_of(HX, 0, 129), V, (dmax[10:11], dmax[12:13]),
                        (amax[7:8], amax[10:11]), with_bias=True, a_split=128)] = (
                "views_G", "views_GA_bias", None)
        elif v_h7:   # G = d_hv [h7; enc]^T: both the views and the feature gradients (below)
            post[wb.add(d_hv, V, dmax[10:11], (amax[7:8], amax[10:11]),
                        with_bias=True)] = ("views_G", "views_linears.0.bias", None)
        else:
            post[wb.add(d_hv, V, dmax[10:11], (amax[8:9], amax[10:11]),
                        with_bias=True)] = (
                "views_linears.0.weight", "views_linears.0.bias", lambda g: g[:, :283])
            post[wb.add(DF, H[7], dmax[8:9], amax[7:8], with_bias=True)] = (
                "feature_linear.weight", "feature_linear.bias", None)
        if not heads_merged:
            post[wb.add(d_sig, H[7], dmax[12:13], amax[7:8], with_bias=True)] = (
                "alpha_linear.weight", "alpha_linear.bias", None)
        for i in range(7, -1, -1):
            # layer 0 reads the 63 encoding rows; the skip layer's [63 encoding
            # rows | h4] are two column blocks of one contiguous [256, 319] result
            # (each with its own scale), so no gradient needs a gather afterwards
            inp, in_max = ((rows_of(E, 0, 63), amax[9:10]) if i in (0, 5)
                           else (H[i - 1], amax[i - 1:i]))
            s = wb.add(D[i], inp, dmax[i:i + 1], in_max, with_bias=True,
                       width=319 if i == 5 else None)
            post[s] = (f"pts_linears.{i}.weight", f"pts_linears.{i}.bias", None)
            if i == 5:
                post[wb.add(D[5], H[4], dmax[5:6], amax[4:5], into=(s, 63))] = None
        # the weight gradients need nothing of the rest of the backward: with the
        # fused kernels they run on a side stream, so the launches after this
        # node (the fine network's d z -> sample_pdf / composite backward of the
        # coarse one) overlap them; the main stream joins at the end of the pass
        side = _side_stream(dev) if (ctx.fused_backward and SIDE_WGRAD and
                                     p["pts_linears.0.weight"].data_ptr() in _SIDE_SCOPE[0]) \
            else None
        if side is not None:
            side.wait_stream(torch.cuda.current_stream(dev))
        # with a side stream, this node's own input gradient is enqueued first: a
        # short launch that would otherwise queue behind the weight gradients'
        # workgroups (they fill every CU's LDS) and run only as they retire,
        # holding back the coarse network's backward that waits for it (round 6,
        # C3 graph step 2.757 / 2.735 ms vs 2.782 / 2.761 enqueued after:
        # profiles/r6_t16_sample_major/ab.log)
        d_pts = NerfMLPFn._input_grad(d_enc, E, pts, rays_S, P, dev) \
            if side is not None and DZ_FIRST else None
        with torch.cuda.stream(side) if side is not None else _nullctx():
            NerfMLPFn._weight_grads(wb, post, grads, heads_merged, v_h7, p, dev)
        if side is not None:
            _join_side(side, wb, grads, (amax, dmax), params, dev)
        if d_pts is None:
            d_pts = NerfMLPFn._input_grad(d_enc, E, pts, rays_S, P, dev)
        if rays_S:
            return (None, None, d_pts, *[grads[n] for n in PARAM_NAMES])
        return (d_pts, None, *[grads[n] for n in PARAM_NAMES])

    @staticmethod
    def _input_grad(d_enc, E, pts, rays_S, P, dev):
        """d z [P / S, S] (ray form) or d pts [P, 3] from the encoding rows' gradient
        (layer 5's and layer 0's, summed in the kernel); None without one."""
        if d_enc is None:
            return None
        f32 = torch.float32

        def lay(t):   # (row stride, T16 block stride) of an operand
            return (BLOCK, t.block_stride) if isinstance(t, BlockRows) else (t.stride(0), 0)
        assert lay(d_enc[0]) == lay(d_enc[1])
        (ldd, bsd), (lde, bse) = lay(d_enc[0]), lay(E)
        if rays_S:          # pts = the rays' o + d z: straight on to d z
            d_pts = torch.empty((P // rays_S, rays_S), device=dev, dtype=f32)
            call("nerf_freq_encode_fm_backward_dz", ptr(d_enc[0]), ptr(d_enc[1]), ldd, bsd,
                 ptr(E), lde, bse, ptr(pts), rays_S, P, XYZ_FREQS, ptr(d_pts),
                 _lib.stream_of(dev))
        else:
            d_pts = torch.empty((P, 3), device=dev, dtype=f32)
            call("nerf_freq_encode_fm_backward_sum", ptr(d_enc[0]), ptr(d_enc[1]), ldd, bsd,
                 ptr(E), lde, bse, ptr(pts), 3, P, XYZ_FREQS, ptr(d_pts),
                 _lib.stream_of(dev))
        return d_pts

    @staticmethod
    def _weight_grads(wb, post, grads, heads_merged, v_h7, p, dev):
        """The batched weight-gradient launch and its post-processing (the views /
        feature / alpha gradients through G) on the current stream."""
        f32 = torch.float32
        for slot, res in enumerate(wb.results()):
            if post[slot] is None:   # a column block joined into another slot's result
                continue
            wname, bname, fix = post[slot]
            gw, gb = (res if bname else (res, None))
            grads[wname] = fix(gw) if fix is not None else gw
            if bname:
                grads[bname] = gb
        ER = erb = None
        if "views_enc_rgb" in grads:   # the shared tile: vfg copies the rgb head out of it
            ER, erb = grads.pop("views_enc_rgb"), grads.pop("views_enc_rgb_bias")
            grads["rgb_linear.weight"] = torch.empty((3, 128), device=dev, dtype=f32)
            grads["rgb_linear.bias"] = torch.empty((3,), device=dev, dtype=f32)
        if heads_merged:   # the views / feature / alpha gradients in one launch (below)
            GA, ba = grads.pop("views_G"), grads.pop("views_GA_bias")
            for n, shape in (("views_linears.0.weight", (128, 283)),
                             ("feature_linear.weight", (256, 256)),
                             ("feature_linear.bias", (256,)), ("alpha_linear.weight", (1, 256)),
                             ("alpha_linear.bias", (1,)), ("views_linears.0.bias", (128,))):
                grads[n] = torch.empty(shape, device=dev, dtype=f32)
            Wf, bf, Wv = (p["feature_linear.weight"].detach().contiguous(),
                          p["feature_linear.bias"].detach().contiguous(),
                          p["views_linears.0.weight"].detach().contiguous())
            call("nerf_views_feature_grads", ptr(GA), GA.stride(0), ptr(ba), ptr(Wf), ptr(bf),
                 ptr(Wv), ptr(grads["views_linears.0.weight"]), ptr(grads["feature_linear.weight"]),
                 ptr(grads["feature_linear.bias"]), ptr(grads["alpha_linear.weight"]),
                 ptr(grads["alpha_linear.bias"]), ptr(grads["views_linears.0.bias"]),
                 *((None, 0, None, None, None) if ER is None else
                   (ptr(ER), ER.stride(0), ptr(erb), ptr(grads["rgb_linear.weight"]),
                    ptr(grads["rgb_linear.bias"]))),
                 _lib.stream_of(dev))
        elif v_h7:
            # feature = W_f h7 + b_f (NET:63) feeds the views layer (NET:64-65), so with
            # G = sum_p d_hv [h7; enc]^T and s = sum_p d_hv (the views bias gradient):
            #   dW_views = [G_h7 W_f^T + s b_f^T, G_enc],  dW_f = W_vf^T G_h7,  db_f = W_vf^T s
            G = grads.pop("views_G")
            sv = grads["views_linears.0.bias"]
            Gh = G[:, :256]
            Wvf = p["views_linears.0.weight"][:, :256]
            grads["views_linears.0.weight"] = torch.cat(
                [torch.addmm(sv[:, None] * p["feature_linear.bias"][None, :], Gh,
                             p["feature_linear.weight"].t()), G[:, 256:283]], 1)
            grads["feature_linear.weight"] = Wvf.t() @ Gh
            grads["feature_linear.bias"] = Wvf.t() @ sv


# NERF_TRAIN_ENC_RGB_TILE=0: the views layer's encoding columns and the rgb head
# in two tiles of their own (the A/B of the shared tile)
ENC_RGB_TILE = _os.environ.get("NERF_TRAIN_ENC_RGB_TILE", "1") != "0"
# NERF_TRAIN_SIDE_WGRAD=0: the weight gradients on the main stream, in line
SIDE_WGRAD = _os.environ.get("NERF_TRAIN_SIDE_WGRAD", "1") != "0"
# NERF_TRAIN_DZ_FIRST=0: with side-stream weight gradients, enqueue the node's
# input gradient after them (the A/B of the order)
DZ_FIRST = _os.environ.get("NERF_TRAIN_DZ_FIRST", "1") != "0"
_SIDE = {}
_SIDE_SCOPE = [frozenset()]   # a plain global: the autograd engine runs backward on its own thread


class side_wgrad_scope:
    """Backward passes inside this scope compute the weight gradients of the
    given networks' fused MLP nodes on a side stream (joined at the end of the
    pass), so the main stream runs on meanwhile -- worth it for a network whose
    backward has work after it (NerfTrainer: the fine network; the coarse one
    is last, and a side stream would only add two cross-queue waits). Only for
    passes in which each of those parameters receives ONE gradient, into a
    .grad that is None (NerfTrainer: one fused node per network,
    zero_grad(set_to_none)): a second gradient for the same parameter would be
    added on the main stream before the join. networks: modules or their first
    weight tensors."""

    def __init__(self, networks=()):
        keys = set()
        for n in networks:
            w = mlp_params(n)[0] if isinstance(n, torch.nn.Module) else n
            keys.add(w.data_ptr())
        self.on = frozenset(keys)

    def __enter__(self):
        self.prev = _SIDE_SCOPE[0]
        _SIDE_SCOPE[0] = self.on
        return self

    def __exit__(self, *a):
        _SIDE_SCOPE[0] = self.prev
        return False


def _side_stream(dev, role="wgrad"):
    s = _SIDE.get((str(dev), role))
    if s is None:
        s = _SIDE[(str(dev), role)] = torch.cuda.Stream(dev)
    return s


class _nullctx:
    def __enter__(self):
        return None

    def __exit__(self, *a):
        return False


def _join_side(side, wb, grads, stats, params, dev):
    """After the side-stream weight gradients: every buffer they read stays
    allocated until they are done (record_stream), the gradients are handed to
    the main stream, which waits for them at the end of the backward pass (an
    engine callback) -- or at once when anything reads them on the main stream
    sooner: a parameter that already holds a gradient (AccumulateGrad adds into
    it right away), grad mode (create_graph: AccumulateGrad copies), or a
    tensor / post-accumulate-grad hook on a parameter."""
    main = torch.cuda.current_stream(dev)

    def keep(t):
        if isinstance(t, tuple):
            for u in t:
                keep(u)
        elif isinstance(t, BlockRows):
            t.buf.record_stream(side)
        elif isinstance(t, torch.Tensor):
            t.record_stream(side)
    for r in wb.req:
        for t in r[:4]:
            keep(t)
    for t in stats:
        keep(t)
    for g in grads.values():
        g.record_stream(main)
    ev = torch.cuda.Event()
    ev.record(side)
    # the main stream must wait at once whenever something on it may read a
    # gradient before the pass ends: AccumulateGrad adding into an existing
    # .grad, or copying the gradient in grad mode (create_graph), and tensor /
    # post-accumulate hooks, which the engine runs on the main stream
    hooked = any(getattr(q, "_backward_hooks", None) or
                 getattr(q, "_post_accumulate_grad_hooks", None) for q in params)
    if torch.is_grad_enabled() or hooked or any(q.grad is not None for q in params):
        main.wait_event(ev)
    else:
        torch.autograd.Variable._execution_engine.queue_callback(lambda: main.wait_event(ev))


def _backward_layers_impl(DR, p, pk, bits, bits_v, dmax, need_enc):
    """The backward's chain of products as layer launches: d hv, DF, D0..D7 and
    (need_enc) the encoding gradient rows of layers 5 and 0, dmax raised as the
    fused kernel does."""
    dev = DR.device
    P = DR.shape[1]
    d_hv = _act(128, P, dev)   # d hv = (W_rgb^T d_rgb) * (hv > 0): the views layer's ReLU bits
    wrt, swrt, mt, nk = pk["bwd_rgb"]
    _layer(wrt, swrt, mt, nk, DR, d_hv, P, mask_bits=bits_v, amax=dmax[10:11])
    # d feature = W_v[:, :256]^T d_hv (K = 128 -> 4 steps), no mask (no ReLU)
    wvt, swvt, mt, nk = pk["bwd_views"]
    DF = _act(256, P, dev)
    _layer(wvt, swvt, mt, nk, d_hv, DF, P, amax=dmax[8:9])
    # d h7 = (W_feat^T DF + W_alpha^T d_sig) * (h7 > 0)
    wft, swft, _, _ = pk["bwd_feat"]
    D = [None] * 8
    D[7] = _act(256, P, dev)
    aw = p["alpha_linear.weight"].reshape(-1).contiguous()
    dsig = DR[3].contiguous()
    _layer(wft, swft, 16, 8, DF, D[7], P, mask_bits=bits[7], ru=aw, rw=dsig, amax=dmax[7:8])
    d_enc = None
    for i in range(7, 0, -1):
        D[i - 1] = _act(256, P, dev)
        if i == 5:
            wt, swt, mt, nk = pk["bwd5h"]
            _layer(wt, swt, mt, nk, D[5], D[4], P, mask_bits=bits[4], amax=dmax[4:5])
            if need_enc:
                we, swe, mt, nk = pk["bwd5e"]
                de5 = _act(64, P, dev)
                _layer(we, swe, mt, nk, D[5], de5, P)
        else:
            wt, swt, mt, nk = pk[f"bwd{i}"]
            _layer(wt, swt, mt, nk, D[i], D[i - 1], P, mask_bits=bits[i - 1],
                   amax=dmax[i - 1:i])
    if need_enc:
        wt, swt, mt, nk = pk["bwd0"]
        de0 = _act(64, P, dev)
        _layer(wt, swt, mt, nk, D[0], de0, P)
        d_enc = (de5[:63], de0[:63])
    return d_hv, DF, D, d_enc


def _backward_fused_impl(d_raw, streams, bits, bits_v, dmax, need_enc, hx=None, bbuf=None):
    """The same chain as ONE nerf_mlp_train_backward_x3 launch over the
    transposed weight stream (X3BwdStreamPacker, the feature layer folded into
    the views layer): every product's rows written feature-major and its max
    |.| raised, the ReLU masks from the forward's bits; d_enc = the layer-5 and
    layer-0 encoding rows. DF (d feature) does not exist: None (the views and
    feature weight gradients go through G, NerfMLPFn.backward). hx: a [132, P]
    row buffer: d_hv goes to rows 0..127 and d raw, feature-major, to rows
    128..131 (d sigma, d r, d g, d b)."""
    dev = d_raw.device
    P = d_raw.shape[0]
    stream, head = streams
    d_raw_c = d_raw.detach().to(torch.float32).contiguous()
    if d_raw_c.data_ptr() % 16:
        d_raw_c = d_raw_c.clone()
    if bbuf is not None:   # T16: every row in the one buffer (_BWD_*), hx its first rows
        assert hx is not None
        D = [bbuf.rows(_BWD_D + 256 * i, _BWD_D + 256 * (i + 1)) for i in range(8)]
        d_hv = hx.rows(0, 128)
        de5 = bbuf.rows(_BWD_E5, _BWD_E5 + 64) if need_enc else None
        de0 = bbuf.rows(_BWD_E0, _BWD_E0 + 64) if need_enc else None
    else:
        D = [_act(256, P, dev) for _ in range(8)]
        d_hv = _act(128, P, dev) if hx is None else hx[0:128]
        de5 = _act(64, P, dev) if need_enc else None
        de0 = _act(64, P, dev) if need_enc else None
    io = _BwdIO()
    io.d_raw = d_raw_c.data_ptr()
    for i in range(8):
        io.bits[i] = bits[i].data_ptr()
        io.d[i] = D[i].data_ptr()
    io.bits[8] = bits_v.data_ptr()
    io.d[8], io.d[9] = None, d_hv.data_ptr()
    io.d[10] = de5.data_ptr() if need_enc else None
    io.d[11] = de0.data_ptr() if need_enc else None
    io.dmax = dmax.data_ptr()
    if bbuf is not None:
        io.ld, io.bs = BLOCK, bbuf.block_stride
        io.d_raw_t = hx.rows(128, 132).data_ptr()
    else:
        io.ld, io.bs = D[0].stride(0), 0
        io.d_raw_t = hx[128].data_ptr() if hx is not None else None
        assert all(t.stride(0) == io.ld for t in [d_hv] + ([de5, de0] if need_enc else []))
    call("nerf_mlp_train_backward_x3", ptr(stream), ptr(head), P, int(bool(need_enc)),
         ctypes.addressof(io), _lib.stream_of(dev))
    d_enc = (rows_of(de5, 0, 63), rows_of(de0, 0, 63)) if need_enc else None
    return d_hv, None, D, d_enc


NerfMLPFn._backward_layers = staticmethod(_backward_layers_impl)
NerfMLPFn._backward_fused = staticmethod(_backward_fused_impl)


class RayMLPFn(torch.autograd.Function):
    """raw [n, S, 4] = NeRF(encodings of the samples rays_o + rays_d * z, VR:165,
    with view direction rays_d) on the fused x3 kernels, without the point
    tensor or the per-sample directions: the forward kernel builds each point
    from its ray (nerf_mlp_train_forward_x3_rays) and the backward returns the
    gradient w.r.t. z [n, S] (nerf_freq_encode_fm_backward_dz: sum_c d pts_c
    d_c, the autograd of o + d z with constant rays). Inputs: rays_o [n, 3],
    rays_d [n, 3] (no gradient), z [n, S], then the 24 parameters."""

    @staticmethod
    def forward(ctx, rays_o, rays_d, z, *params):
        n, S = z.shape
        P = n * S
        dev = z.device
        # amax + the backward's dmax: zeroed by prepack(side=True) for the trainer's
        # one forward per network and step, else one fill here
        net, _ = _net_for(params, dev)
        stats = net.take_stats()
        if stats is None:
            stats = torch.zeros(25, device=dev, dtype=torch.float32)
        amax, ctx.dmax_buf = stats[:12], stats[12:]
        ctx.fused_backward = FUSED_BACKWARD and P > 0
        if ctx.fused_backward and _t16_ok(P):   # every row in one T16 buffer (_forward_fused)
            E = H = None
        else:
            E = _act(320, P, dev)
            H = [_act(256, P, dev) if i not in (4, 7) else None for i in range(8)]
            H[4] = E[64:320]                             # h7: V's rows (_forward_fused)
        ctx.streams = _streams_for(params, dev)
        ctx.rays_S = S
        pk = None if ctx.fused_backward else _packs_for(params, dev, forward=False, backward=True)
        rays = (rays_o.detach().contiguous(), rays_d.detach().contiguous(),
                z.detach().contiguous())
        raw = NerfMLPFn._forward_fused(ctx, None, None, None, params, E, H, amax, pk, rays)
        ctx.pts_grad = z.requires_grad   # (_forward_fused saw the detached copy)
        return raw.view(n, S, 4)

    @staticmethod
    def backward(ctx, d_raw):
        return NerfMLPFn.backward(ctx, d_raw.reshape(-1, 4))


def query_x3_rays(model, rays_o, rays_d, z):
    """query_x3 of the samples rays_o + rays_d * z (VR:164-165, 270-284) with no
    point tensor: raw [n, S, 4], differentiable in z and the parameters."""
    _lib.require_gpu(z)
    return RayMLPFn.apply(rays_o, rays_d, z, *mlp_params(model))


def mlp_params(model):
    """The 24 parameters of a reference NeRF module in PARAM_NAMES order."""
    named = dict(model.named_parameters())
    return [named[n] for n in PARAM_NAMES]


def query_x3(model, pts, dirs):
    """Drop-in for train.query (VR:270-284): pts [n, s, 3], dirs [n, 3]
    (train.render_train takes query_x3.rays, the ray form, when the fused
    forward is on)."""
    n, s, _ = pts.shape
    _lib.require_gpu(pts)
    d = dirs[:, None, :].expand(n, s, 3).reshape(-1, 3)
    raw = NerfMLPFn.apply(pts.reshape(-1, 3), d, *mlp_params(model))
    return raw.reshape(n, s, 4)


if FUSED_FORWARD:
    query_x3.rays = query_x3_rays
