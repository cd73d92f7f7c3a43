"""numpy restatements of the reference's CUDA extension ops (test oracle only).

Reference: ``cuda/*.cu`` of the reference repository (module ``kilonerf_cuda``).
The CUDA sources cannot be built here (no nvcc, no MAGMA), so
these follow the source text. nvcc contracts ``a += b * c`` / ``a + b * c``
into fused multiply-adds by default; that is written out with ``fma32``.
The fast-math intrinsics of the sources (``__expf``, ``__sinf``, ``__cosf``) are
restated with accurate functions (the GPU port uses accurate ones too).
MAGMA's (version unpinned, not vendored) and thrust's algorithms are restated
by their mathematical definition: parity unpinned for their summation order.
"""
from __future__ import annotations

import numpy as np

from .nerf_oracle import fma32

F32 = np.float32


def get_rays_d(H, W, cx, cy, fx, fy, c2w):
    """generate_inputs.cu:11-35 (un-normalised; out[i] += in[j] * R[i][j])."""
    R = np.asarray(c2w, F32).reshape(3, 3)
    x = np.arange(W, dtype=F32)[None, :].repeat(H, 0)
    y = np.arange(H, dtype=F32)[:, None].repeat(W, 1)
    i0 = ((x - F32(cx)) / F32(fx)).astype(F32)
    i1 = (-(y - F32(cy)) / F32(fy)).astype(F32)
    i2 = np.full_like(i0, F32(-1.0))
    out = np.empty((H, W, 3), F32)
    for r in range(3):
        o = (i0 * R[r, 0]).astype(F32)
        o = fma32(i1, R[r, 1], o)
        out[..., r] = fma32(i2, R[r, 2], o)
    return out


def generate_query_indices_on_ray(origin, dirs, grid, active, depth_idx, vsize, gmin, gmax,
                                  strides, step, max_samples, max_depth, min_dist, initial):
    """generate_inputs.cu:60-126. Mutates active/depth_idx; returns (qidx, nets).
    qidx entries beyond each ray's emitted samples are unspecified (torch::empty)."""
    n = dirs.shape[0]
    qidx = np.full((n, max_samples), -7, np.int32)
    nets = np.full((n, max_samples), -1, np.int16)
    eps = F32(0.001)
    for r in range(n):
        if not initial and not active[r]:
            continue
        out = 0
        depth = 0 if initial else int(depth_idx[r])
        dist = fma32(F32(depth), F32(step), F32(min_dist))
        while depth < max_depth and out < max_samples:
            flat = 0
            inside = True
            for c in range(3):
                pc = fma32(dist, dirs[r, c], origin[c])
                vi = int(np.trunc(F32((pc - gmin[c]) / vsize[c])))
                flat += vi * int(strides[c])
                inside = inside and (F32(gmin[c] + eps) < pc) and (pc < F32(gmax[c] - eps))
            net = int(grid.reshape(-1)[flat]) if inside else -1
            if net != -1:
                nets[r, out] = net
                qidx[r, out] = r * max_depth + depth
                out += 1
            depth += 1
            dist = F32(dist + F32(step))
        if out < max_samples:
            active[r] = False
        else:
            active[r] = True
            depth_idx[r] = depth
    return qidx, nets


def compute_fourier_features(x, freqs):
    """fourier_features.cu:29-38: per scalar [x, cos(f x)..., sin(f x)...]."""
    x = np.asarray(x, F32).reshape(-1)
    f = np.asarray(freqs, F32)
    arg = (f[None, :] * x[:, None]).astype(F32)
    return np.concatenate([x[:, None], np.cos(arg).astype(F32), np.sin(arg).astype(F32)],
                          1).reshape(-1).astype(F32)


def integrate(rgb_sigma, dists, rgb_map, acc_map, T, mask, num_rays, spr, thr, initial):
    """integrate.cu:21-56 (in place on rgb_map [n,3], acc_map, T, mask)."""
    rs = np.asarray(rgb_sigma, F32).reshape(num_rays, spr, 4)
    for r in range(num_rays):
        t = F32(1.0) if initial else F32(T[r])
        act = t > F32(thr)
        out = np.zeros(3, F32)
        acc = F32(0.0)
        if act:
            if not initial:
                out = rgb_map[r].astype(F32).copy()
                acc = F32(acc_map[r])
            d = F32(dists[r])
            for s in range(spr):
                v = rs[r, s]
                alpha = F32(F32(1.0) - F32(np.exp(F32(-v[3] * d))))
                w = F32(alpha * t)
                t = F32(np.float64(t) * (np.float64(F32(F32(1.0) - alpha)) + 1e-10))
                out = np.array([fma32(v[c], w, out[c]) for c in range(3)], F32)
                acc = F32(acc + w)
            T[r] = t
            if t <= F32(thr):
                mask[r] = False
        if act or initial:
            rgb_map[r] = out
            acc_map[r] = acc


def replace_transparency_by_background_color(rgb_map, acc_map, bg):
    """integrate.cu:84-97: rgb += bg * (1 - acc) (in place)."""
    t = (F32(1.0) - acc_map.reshape(-1)).astype(F32)
    for c in range(3):
        rgb_map[:, c] = fma32(F32(bg[c]), t, rgb_map[:, c])


def gather_int32(m, x):
    return np.asarray(x)[np.asarray(m)]


def scatter_int32_float4(m, x, out):
    out[np.asarray(m)] = np.asarray(x)
    return out


def sort_by_key_int16(keys, values):
    """thrust::sort_by_key on primitive keys is a stable radix sort."""
    o = np.argsort(keys, kind="stable")
    return keys[o], values[o]


def global_to_local(points, mins, maxs, bspn):
    """global_to_local.cu:18-33 with the intended per-network min/max."""
    p = np.asarray(points, F32).reshape(-1, 3).copy()
    off = 0
    for k, b in enumerate(bspn):
        seg = p[off:off + b]
        p[off:off + b] = ((F32(2.0) * (seg - mins[k])) / (maxs[k] - mins[k]) - F32(1.0)).astype(F32)
        off += b
    return p.reshape(-1)


def grouped_gemm(mode, bias, X, W, out_f, in_f, bspn):
    """multimatmul.cu:244-361 (MAGMA col-major views resolved): fma chain in k order."""
    X = np.asarray(X, F32)
    out = np.empty((X.shape[0], out_f), F32)
    r = 0
    for k, b in enumerate(bspn):
        Wk = np.asarray(W, F32).reshape(-1)[k * out_f * in_f:(k + 1) * out_f * in_f]
        Wk = Wk.reshape(out_f, in_f).T if mode == 2 else Wk.reshape(in_f, out_f)   # [in, out]
        acc = np.zeros((b, out_f), F32)
        for kk in range(in_f):
            acc = fma32(X[r:r + b, kk][:, None], Wk[kk][None, :], acc)
        if mode == 0:
            acc = (acc + np.asarray(bias, F32).reshape(-1, out_f)[k]).astype(F32)
        out[r:r + b] = acc
        r += b
    return out


def multi_row_sum_reduction(M, bspn):
    M = np.asarray(M, F32)
    out = np.zeros((len(bspn), M.shape[1]), F32)
    r = 0
    for k, b in enumerate(bspn):
        acc = np.zeros(M.shape[1], F32)
        for i in range(b):
            acc = (acc + M[r + i]).astype(F32)
        out[k] = acc
        r += b
    return out


def multimatmul_A_transposed(A, B, bspn):
    A, B = np.asarray(A, F32), np.asarray(B, F32)
    out = np.zeros((len(bspn), A.shape[1], B.shape[1]), F32)
    r = 0
    for k, b in enumerate(bspn):
        acc = np.zeros((A.shape[1], B.shape[1]), F32)
        for i in range(b):
            acc = fma32(A[r + i][:, None], B[r + i][None, :], acc)
        out[k] = acc
        r += b
    return out


def kilonerf_param_size(hd=32):
    pe, de = 3 * 21, 3 * 9
    return (pe + 1) * hd + (hd + 1) * hd + (hd + 1) * (hd + 1) + (hd + de + 1) * hd + (hd + 1) * 3


def network_eval_query_index(qidx, params, mins, maxs, starts, ends, origin, c2w, W, cx, cy,
                             fx, fy, max_depth, min_dist, step, hd=32):
    """network_eval.cu:24-254 (hidden 32), one query at a time. out starts as ones."""
    psize = kilonerf_param_size(hd)
    R = np.asarray(c2w, F32).reshape(3, 3)
    out = np.ones((len(qidx), 4), F32)
    fb = [F32(2.0 ** i) for i in range(10)]
    for net in range(len(starts)):
        P = np.asarray(params, F32)[net * psize:(net + 1) * psize]
        for idx in range(int(starts[net]), int(ends[net])):
            y = int(qidx[idx])
            depth = y % max_depth
            y //= max_depth
            x = y % W
            y //= W
            inp = [F32((F32(x) - F32(cx)) / F32(fx)), F32(-(F32(y) - F32(cy)) / F32(fy)), F32(-1.0)]
            d = []
            for i in range(3):
                o = F32(inp[0] * R[i, 0])
                o = fma32(inp[1], R[i, 1], o)
                d.append(fma32(inp[2], R[i, 2], o))
            dist = fma32(F32(depth), F32(step), F32(min_dist))
            pos = [fma32(dist, d[i], origin[i]) for i in range(3)]
            nrm = F32(d[0] * d[0])
            nrm = fma32(d[1], d[1], nrm)
            nrm = fma32(d[2], d[2], nrm)
            nrm = F32(np.sqrt(nrm))
            d = [F32(v / nrm) for v in d]
            po = 0

            def layer(inputs, nout):
                nonlocal po
                h = P[po:po + nout].copy()
                po += nout
                for v in inputs:
                    h = fma32(F32(v), P[po:po + nout], h)
                    po += nout
                return h

            def emb(v, nf):
                return [v] + [F32(np.cos(F32(fb[e] * v))) for e in range(nf)] + \
                    [F32(np.sin(F32(fb[e] * v))) for e in range(nf)]

            e0 = []
            for j in range(3):
                v = F32((F32(2.0) * F32(pos[j] - mins[net][j])) / F32(maxs[net][j] - mins[net][j]) - F32(1.0))
                e0 += emb(v, 10)
            h0 = layer(e0, hd)
            h1 = layer(np.maximum(h0, F32(0)), hd)
            h2 = layer(np.maximum(h1, F32(0)), hd + 1)
            ed = []
            for j in range(3):
                ed += emb(d[j], 4)
            h3 = layer(list(h2[1:]) + ed, hd)
            rgb = layer(np.maximum(h3, F32(0)), 3)
            for i in range(3):
                out[idx, i] = F32(1.0 / (1.0 + np.float64(F32(np.exp(F32(-rgb[i]))))))
            out[idx, 3] = max(h2[0], F32(0.0))
    return out
