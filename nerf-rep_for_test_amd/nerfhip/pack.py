"""Pack the reference NeRF MLP parameters into the fused kernel's layout.

Input: the reference state_dict tensors of one ``NeRF`` (``network.py:9-74``),
names ``<prefix>.pts_linears.{0..7}``, ``views_linears.0``, ``feature_linear``,
``alpha_linear``, ``rgb_linear`` (torch ``nn.Linear`` layout [out, in]).

Output (see csrc/mlp_fused.hip):
  slices  float32 [73 * 8192]: 32 KiB slices of 1 KiB MFMA A-fragment blocks in
          consumption order. Block (q, m) of a layer holds, for lane l and
          t = 0..3, W[32m + (l & 31)][col(4q + t, l >> 5)] — rows = output
          features, K permuted by ``col``.
  head    float32 [3200]: lane-half packed biases and the VALU density/rgb heads.

K permutations (``col(s, h)`` = input feature used at k-step s by lane half h):
  act  : the previous layer's accumulator layout,
         32*(s>>4) + (r&3) + 8*(r>>2) + 4h with r = s & 15;
  enc L: k-step 0 -> (x | y), 1 -> (z | pad), 2+3f+c -> (sin 2^f p_c | cos 2^f p_c),
         mapped to the reference encoder's column order x,y,z, then per band
         sin(xyz), cos(xyz) (``freq.py:7-32``).
"""
from __future__ import annotations

import numpy as np

SLICES = 73
SLICE_FLOATS = 8192
BLOCKS_PER_SLICE = 32
HEAD_FLOATS = 3200
H_BIAS, H_BIAS_VIEWS, H_ALPHA_W, H_ALPHA_B, H_RGB_W, H_RGB_B = 0, 2304, 2432, 2688, 2692, 3076

IN_XYZ, IN_DIR, W = 63, 27, 256


def col_act(s, h):
    s = np.asarray(s)
    r = s & 15
    return 32 * (s >> 4) + (r & 3) + 8 * (r >> 2) + 4 * h


def col_enc(s, h, n_freq):
    """Reference encoder column for k-step s, half h (-1 = zero pad)."""
    if s == 0:
        return 1 if h else 0
    if s == 1:
        return -1 if h else 2
    j = s - 2
    f, c = divmod(j, 3)
    if f >= n_freq:
        return -1
    return 3 + 6 * f + (3 if h else 0) + c


def _layer_cols(kind):
    """[ksteps, 2] column map of a layer's input (-1 = zero)."""
    if kind == "l0":
        return np.array([[col_enc(s, h, 10) for h in (0, 1)] for s in range(32)])
    if kind == "act":
        return np.stack([col_act(np.arange(128), h) for h in (0, 1)], 1)
    if kind == "skip":
        enc = np.array([[col_enc(s, h, 10) for h in (0, 1)] for s in range(32)])
        act = np.stack([IN_XYZ + col_act(np.arange(128), h) for h in (0, 1)], 1)
        return np.concatenate([enc, act], 0)
    if kind == "views":
        act = np.stack([col_act(np.arange(128), h) for h in (0, 1)], 1)
        d = np.array([[col_enc(s, h, 4) for h in (0, 1)] for s in range(16)])
        d = np.where(d >= 0, W + d, -1)
        return np.concatenate([act, d], 0)
    raise ValueError(kind)


def layer_plan():
    """(param name suffix, kind, row tiles) in kernel consumption order."""
    plan = [("pts_linears.0", "l0", 8)]
    for i in range(1, 8):
        plan.append((f"pts_linears.{i}", "skip" if i == 5 else "act", 8))
    plan.append(("feature_linear", "act", 8))
    plan.append(("views_linears.0", "views", 4))
    return plan


def _blocks(Wt, cols, tiles):
    """Fragment blocks [Q*tiles, 64, 4] for weight [out, in] and column map."""
    ksteps = cols.shape[0]
    assert ksteps % 4 == 0
    Q = ksteps // 4
    lane = np.arange(64)
    row_in_tile = lane & 31
    half = lane >> 5
    out = np.zeros((Q, tiles, 64, 4), np.float32)
    Wp = np.concatenate([Wt, np.zeros((Wt.shape[0], 1), np.float32)], 1)  # col -1 -> 0
    for t in range(4):
        s = np.arange(Q) * 4 + t                        # [Q]
        c = cols[s][:, half]                            # [Q, 64]
        c = np.where(c < 0, Wt.shape[1], c)
        for m in range(tiles):
            rows = 32 * m + row_in_tile                 # [64]
            out[:, m, :, t] = Wp[rows[None, :], c]
    return out.reshape(Q * tiles, 64, 4)


def _half_pack(vec, tiles):
    """[2][16*tiles]: element [h][16m+r] = vec[32m + (r&3) + 8(r>>2) + 4h]."""
    m = np.arange(tiles)[:, None]
    r = np.arange(16)[None, :]
    out = np.empty((2, tiles * 16), np.float32)
    for h in (0, 1):
        out[h] = vec[(32 * m + (r & 3) + 8 * (r >> 2) + 4 * h).reshape(-1)]
    return out


def pack_mlp(params, prefix="model"):
    """params: mapping name -> array-like ([out,in] weights, [out] biases)."""
    def g(name):
        v = params[f"{prefix}.{name}"]
        v = v.detach().cpu().numpy() if hasattr(v, "detach") else np.asarray(v)
        return np.ascontiguousarray(v, np.float32)

    blocks = []
    head = np.zeros(HEAD_FLOATS, np.float32)
    for li, (name, kind, tiles) in enumerate(layer_plan()):
        Wt = g(name + ".weight")
        b = g(name + ".bias")
        cols = _layer_cols(kind)
        assert cols.max() < Wt.shape[1], (name, cols.max(), Wt.shape)
        blocks.append(_blocks(Wt, cols, tiles))
        if kind == "views":
            head[H_BIAS_VIEWS:H_BIAS_VIEWS + 128] = _half_pack(b, 4).reshape(-1)
        else:
            head[H_BIAS + li * 256:H_BIAS + li * 256 + 256] = _half_pack(b, 8).reshape(-1)
    allb = np.concatenate(blocks, 0)
    assert allb.shape[0] <= SLICES * BLOCKS_PER_SLICE
    slices = np.zeros((SLICES * BLOCKS_PER_SLICE, 64, 4), np.float32)
    slices[:allb.shape[0]] = allb
    head[H_ALPHA_W:H_ALPHA_W + 256] = _half_pack(g("alpha_linear.weight")[0], 8).reshape(-1)
    head[H_ALPHA_B] = g("alpha_linear.bias")[0]
    rw = g("rgb_linear.weight")
    for c in range(3):
        head[H_RGB_W + c * 128:H_RGB_W + c * 128 + 128] = _half_pack(rw[c], 4).reshape(-1)
    head[H_RGB_B:H_RGB_B + 3] = g("rgb_linear.bias")
    return slices.reshape(-1), head


# ----------------------------------------------------------------------------
# numpy emulation of the kernel's dataflow (CPU tests of the layout only)
# ----------------------------------------------------------------------------
def _enc_ksteps(p, n_freq, ksteps):
    """[ksteps, 2, P] B-operand values of the encoded input (float64)."""
    P = p.shape[0]
    out = np.zeros((ksteps, 2, P))
    for s in range(ksteps):
        for h in (0, 1):
            c = col_enc(s, h, n_freq)
            if c < 0:
                continue
            if c < 3:
                out[s, h] = p[:, c]
            else:
                f, rem = divmod(c - 3, 6)
                v = p[:, rem % 3] * (2.0 ** f)
                out[s, h] = np.sin(v) if rem < 3 else np.cos(v)
    return out


def _acc_to_ksteps(acc):
    """accumulators [tiles, 32 rows, P] -> B operands [tiles*16, 2, P]."""
    tiles = acc.shape[0]
    r = np.arange(16)
    out = np.empty((tiles * 16, 2, acc.shape[2]))
    for m in range(tiles):
        for h in (0, 1):
            out[m * 16 + r, h] = acc[m, (r & 3) + 8 * (r >> 2) + 4 * h]
    return out


def emulate(slices, head, pts, dirs):
    """Run the packed network the way the kernel does (float64). pts, dirs: [P,3]."""
    blocks = slices.reshape(-1, 64, 4).astype(np.float64)
    hd = head.astype(np.float64)
    enc = _enc_ksteps(pts.astype(np.float64), 10, 32)
    denc = _enc_ksteps(dirs.astype(np.float64), 4, 16)
    bi = 0

    def run_layer(Bk, tiles):
        nonlocal bi
        ks = Bk.shape[0]
        acc = np.zeros((tiles, 32, Bk.shape[2]))
        for q in range(ks // 4):
            for m in range(tiles):
                blk = blocks[bi]
                bi += 1
                for t in range(4):
                    A = blk[:, t].reshape(2, 32).T            # [row, slot]
                    acc[m] += A @ Bk[4 * q + t]                # [32, P]
        return acc

    def bias_act(acc, bvec, relu):
        tiles = acc.shape[0]
        out = acc.copy()
        for m in range(tiles):
            for h in (0, 1):
                for r in range(16):
                    row = (r & 3) + 8 * (r >> 2) + 4 * h
                    out[m, row] += bvec[h * tiles * 16 + 16 * m + r]
        return np.maximum(out, 0) if relu else out

    acc = run_layer(enc, 8)
    act = bias_act(acc, hd[H_BIAS:H_BIAS + 256], True)
    alpha = None
    for L in range(1, 9):
        Bk = _acc_to_ksteps(act)
        if L == 5:
            Bk = np.concatenate([enc, Bk], 0)
        acc = run_layer(Bk, 8)
        act = bias_act(acc, hd[H_BIAS + L * 256:H_BIAS + L * 256 + 256], L != 8)
        if L == 7:
            aw = _half_pack_inv(hd[H_ALPHA_W:H_ALPHA_W + 256], 8)
            alpha = np.einsum("f,fp->p", aw, act.reshape(256, -1)) + hd[H_ALPHA_B]
    Bk = np.concatenate([_acc_to_ksteps(act), denc], 0)
    # pad the 144 views k-steps to whole slices as the packer does
    acc = run_layer(Bk, 4)
    v = bias_act(acc, hd[H_BIAS_VIEWS:H_BIAS_VIEWS + 128], True).reshape(128, -1)
    rgb = np.stack([np.einsum("f,fp->p", _half_pack_inv(hd[H_RGB_W + c * 128:H_RGB_W + c * 128 + 128], 4), v)
                    + hd[H_RGB_B + c] for c in range(3)], -1)
    return np.concatenate([rgb, alpha[:, None]], -1)


def _half_pack_inv(packed, tiles):
    """Inverse of _half_pack: back to feature order [32*tiles]."""
    out = np.empty(32 * tiles)
    pk = packed.reshape(2, tiles * 16)
    for h in (0, 1):
        for m in range(tiles):
            for r in range(16):
                out[32 * m + (r & 3) + 8 * (r >> 2) + 4 * h] = pk[h, 16 * m + r]
    return out
