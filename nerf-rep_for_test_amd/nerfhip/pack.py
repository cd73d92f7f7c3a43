"""Pack the reference NeRF MLP parameters into the fused kernel's layout.

Input: the reference state_dict tensors of one ``NeRF`` (``network.py:9-74``),
names ``<prefix>.pts_linears.{0..7}``, ``views_linears.0``, ``feature_linear``,
``alpha_linear``, ``rgb_linear`` (torch ``nn.Linear`` layout [out, in]).

Output (see csrc/mlp_fused.hip, v_mfma_f32_16x16x4_f32 tiles):
  slices  float32 [73 * 8192]: 32 KiB slices of 1 KiB MFMA A-fragment blocks in
          consumption order. Block (q, m) of a layer holds, for lane l and
          t = 0..3, W[16m + (l & 15)][col(4q + t, l >> 4)] — rows = output
          features, K permuted by ``col``; blocks run quad-major (q, then m).
  head    float32 [3200]: lane-group packed biases and the VALU density/rgb heads.

K permutations (``col(s, g)`` = input feature used at k-step s by lane group g):
  act  : the previous layer's accumulator layout, 16*(s>>2) + 4g + (s&3);
  enc L: k-step 0 -> (x, y, z, pad); 1+t -> (sin a, cos a, sin b, cos b) for the
         (band f, coordinate c) pairs a = 2t, b = 2t+1 (pair p = 3f + c),
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
TILE = 16           # MFMA tile rows / samples per wave
GROUPS = 4          # lane groups = K slots per k-step


def col_act(s, g):
    s = np.asarray(s)
    return 16 * (s >> 2) + 4 * g + (s & 3)


def col_enc(s, g, n_freq):
    """Reference encoder column for k-step s, lane group g (-1 = zero pad)."""
    if s == 0:
        return g if g < 3 else -1
    pa = 2 * (s - 1) + (g >> 1)
    if pa >= 3 * n_freq:
        return -1
    f, c = divmod(pa, 3)
    return 3 + 6 * f + (3 if g & 1 else 0) + c


def _enc_cols(n_freq, ksteps):
    return np.array([[col_enc(s, g, n_freq) for g in range(GROUPS)] for s in range(ksteps)])


def _layer_cols(kind):
    """[ksteps, 4] column map of a layer's input (-1 = zero)."""
    act = np.stack([col_act(np.arange(64), g) for g in range(GROUPS)], 1)
    if kind == "l0":
        return _enc_cols(10, 16)
    if kind == "act":
        return act
    if kind == "skip":
        return np.concatenate([_enc_cols(10, 16), IN_XYZ + act], 0)
    if kind == "views":
        d = _enc_cols(4, 8)
        return np.concatenate([act, np.where(d >= 0, W + d, -1)], 0)
    raise ValueError(kind)


def layer_plan():
    """(param name suffix, kind, row tiles) in kernel consumption order."""
    plan = [("pts_linears.0", "l0", 16)]
    for i in range(1, 8):
        plan.append((f"pts_linears.{i}", "skip" if i == 5 else "act", 16))
    plan.append(("feature_linear", "act", 16))
    plan.append(("views_linears.0", "views", 8))
    return plan


def _blocks(Wt, cols, tiles):
    """Fragment blocks [Q*tiles, 64, 4] for weight [out, in] and column map."""
    ksteps = cols.shape[0]
    assert ksteps % 4 == 0
    Q = ksteps // 4
    lane = np.arange(64)
    row_in_tile = lane & 15
    grp = lane >> 4
    out = np.zeros((Q, tiles, 64, 4), np.float32)
    Wp = np.concatenate([Wt, np.zeros((Wt.shape[0], 1), np.float32)], 1)  # col -1 -> 0
    for t in range(4):
        s = np.arange(Q) * 4 + t                        # [Q]
        c = cols[s][:, grp]                             # [Q, 64]
        c = np.where(c < 0, Wt.shape[1], c)
        for m in range(tiles):
            rows = TILE * m + row_in_tile               # [64]
            out[:, m, :, t] = Wp[rows[None, :], c]
    return out.reshape(Q * tiles, 64, 4)


def _group_pack(vec, tiles):
    """[4][4*tiles]: element [g][4m+r] = vec[16m + 4g + r]."""
    m = np.arange(tiles)[:, None]
    r = np.arange(4)[None, :]
    out = np.empty((GROUPS, tiles * 4), np.float32)
    for g in range(GROUPS):
        out[g] = vec[(16 * m + 4 * g + r).reshape(-1)]
    return out


def pack_mlp(params, prefix="model"):
    """params: mapping name -> array-like ([out,in] weights, [out] biases)."""
    def get(name):
        v = params[f"{prefix}.{name}"]
        v = v.detach().cpu().numpy() if hasattr(v, "detach") else np.asarray(v)
        return np.ascontiguousarray(v, np.float32)

    blocks = []
    head = np.zeros(HEAD_FLOATS, np.float32)
    for li, (name, kind, tiles) in enumerate(layer_plan()):
        Wt = get(name + ".weight")
        b = get(name + ".bias")
        cols = _layer_cols(kind)
        assert cols.max() < Wt.shape[1], (name, cols.max(), Wt.shape)
        blocks.append(_blocks(Wt, cols, tiles))
        if kind == "views":
            head[H_BIAS_VIEWS:H_BIAS_VIEWS + 128] = _group_pack(b, 8).reshape(-1)
        else:
            head[H_BIAS + li * 256:H_BIAS + li * 256 + 256] = _group_pack(b, 16).reshape(-1)
    allb = np.concatenate(blocks, 0)
    assert allb.shape[0] <= SLICES * BLOCKS_PER_SLICE
    slices = np.zeros((SLICES * BLOCKS_PER_SLICE, 64, 4), np.float32)
    slices[:allb.shape[0]] = allb
    head[H_ALPHA_W:H_ALPHA_W + 256] = _group_pack(get("alpha_linear.weight")[0], 16).reshape(-1)
    head[H_ALPHA_B] = get("alpha_linear.bias")[0]
    rw = get("rgb_linear.weight")
    for c in range(3):
        head[H_RGB_W + c * 128:H_RGB_W + c * 128 + 128] = _group_pack(rw[c], 8).reshape(-1)
    head[H_RGB_B:H_RGB_B + 3] = get("rgb_linear.bias")
    return slices.reshape(-1), head


# ----------------------------------------------------------------------------
# numpy emulation of the kernel's dataflow (CPU tests of the layout only)
# ----------------------------------------------------------------------------
def _enc_ksteps(p, n_freq, ksteps):
    """[ksteps, 4, P] B-operand values of the encoded input (float64)."""
    P = p.shape[0]
    out = np.zeros((ksteps, GROUPS, P))
    for s in range(ksteps):
        for g in range(GROUPS):
            c = col_enc(s, g, n_freq)
            if c < 0:
                continue
            if c < 3:
                out[s, g] = p[:, c]
            else:
                f, rem = divmod(c - 3, 6)
                v = p[:, rem % 3] * (2.0 ** f)
                out[s, g] = np.sin(v) if rem < 3 else np.cos(v)
    return out


def _acc_to_ksteps(acc):
    """accumulators [tiles, 16 rows, P] -> B operands [tiles*4, 4, P]."""
    tiles = acc.shape[0]
    out = np.empty((tiles * 4, GROUPS, acc.shape[2]))
    for m in range(tiles):
        for g in range(GROUPS):
            for r in range(4):
                out[m * 4 + r, g] = acc[m, 4 * g + r]
    return out


def _group_pack_inv(packed, tiles):
    """Inverse of _group_pack: back to feature order [16*tiles]."""
    out = np.empty(TILE * tiles)
    pk = packed.reshape(GROUPS, tiles * 4)
    for g in range(GROUPS):
        for m in range(tiles):
            for r in range(4):
                out[16 * m + 4 * g + r] = pk[g, 4 * m + r]
    return out


def emulate(slices, head, pts, dirs):
    """Run the packed network the way the kernel does (float64). pts, dirs: [P,3]."""
    blocks = slices.reshape(-1, 64, 4).astype(np.float64)
    hd = head.astype(np.float64)
    enc = _enc_ksteps(pts.astype(np.float64), 10, 16)
    denc = _enc_ksteps(dirs.astype(np.float64), 4, 8)
    bi = 0

    def run_layer(Bk, tiles):
        nonlocal bi
        ks = Bk.shape[0]
        acc = np.zeros((tiles, TILE, Bk.shape[2]))
        for q in range(ks // 4):
            for m in range(tiles):
                blk = blocks[bi]
                bi += 1
                for t in range(4):
                    A = blk[:, t].reshape(GROUPS, TILE).T      # [row, slot]
                    acc[m] += A @ Bk[4 * q + t]                 # [16, P]
        if bi % 32:
            bi += 32 - bi % 32                                   # slices are padded
        return acc

    def bias_act(acc, bvec, relu):
        tiles = acc.shape[0]
        out = acc + _group_pack_inv(bvec, tiles).reshape(tiles, TILE)[:, :, None]
        return np.maximum(out, 0) if relu else out

    acc = run_layer(enc, 16)
    act = bias_act(acc, hd[H_BIAS:H_BIAS + 256], True)
    alpha = None
    for L in range(1, 9):
        Bk = _acc_to_ksteps(act)
        if L == 5:
            Bk = np.concatenate([enc, Bk], 0)
        acc = run_layer(Bk, 16)
        act = bias_act(acc, hd[H_BIAS + L * 256:H_BIAS + L * 256 + 256], L != 8)
        if L == 7:
            aw = _group_pack_inv(hd[H_ALPHA_W:H_ALPHA_W + 256], 16)
            alpha = np.einsum("f,fp->p", aw, act.reshape(256, -1)) + hd[H_ALPHA_B]
    Bk = np.concatenate([_acc_to_ksteps(act), denc], 0)
    acc = run_layer(Bk, 8)
    v = bias_act(acc, hd[H_BIAS_VIEWS:H_BIAS_VIEWS + 128], True).reshape(128, -1)
    rgb = np.stack([np.einsum("f,fp->p", _group_pack_inv(hd[H_RGB_W + c * 128:H_RGB_W + c * 128 + 128], 8), v)
                    + hd[H_RGB_B + c] for c in range(3)], -1)
    return np.concatenate([rgb, alpha[:, None]], -1)
