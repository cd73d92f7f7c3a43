import sys, numpy as np, torch
sys.path[:0] = ['nerf-rep_for_test_amd', '.', 'tests']
from goldlib import load, params_of
from oracle import nerf_oracle as O
from nerfhip.render import NerfPipeline
from nerfhip._lib import call, ptr, stream_of
F32 = np.float32
dev = torch.device('cuda:0')
def T(a): return torch.from_numpy(np.ascontiguousarray(a)).to(dev)
for name in ['f3b_ert_noterm', 'f1_c2_crop']:
    z = load(name); p = params_of(z)
    ert = bool(z['enable_ert'])
    pipe = NerfPipeline(dev, N_samples=64, N_importance=128, enable_ert=ert, ert_threshold=0.01)
    pipe.set_weights(p)
    H, W = int(z['H']), int(z['W']); n = H * W
    ro, rd = pipe.camera_rays(H, W, z['pose'], z['K'])
    oro, ord_ = O.camera_rays(H, W, z['pose'], z['K'])
    print(name, 'rays equal', np.array_equal(ro.cpu().numpy(), oro), np.array_equal(rd.cpu().numpy(), ord_))
    raw = pipe.mlp(pipe.coarse, ro, rd, pipe.z_base, 0, n, 64)
    zc = np.broadcast_to(O.coarse_depths(2., 6., 64, False), (n, 64))
    oraw = O.query_network((oro[:, None] + ord_[:, None] * zc[:, :, None]).astype(F32), ord_, p, 'model')
    g = raw.cpu().numpy().reshape(n, 64, 4)
    print('  coarse raw max abs diff', np.abs(g - oraw).max(), 'mag', np.abs(oraw).max(), 'nan', np.isnan(g).sum())
    out = pipe.alloc_outputs(n)
    w = pipe.composite(raw, pipe.z_base, 0, rd, n, 64, out['coarse'], 0)
    comp = (lambda r_, z_, d_: O.raw2outputs_ert(r_, z_, d_, 0.01)) if ert else (lambda r_, z_, d_: O.raw2outputs(r_, z_, d_))
    _, _, oacc, ow, _ = comp(g, np.ascontiguousarray(zc), ord_)   # oracle composite on OUR raw
    print('  coarse w maxdiff (same raw)', np.abs(w.cpu().numpy() - ow).max(), 'acc diff', np.abs(out['coarse'][2].cpu().numpy() - oacc).max())
    zall = torch.empty((n, 192), device=dev)
    zb = pipe.z_base
    call("nerf_sample_fine", ptr(zb), 0, ptr(w), ptr(pipe.u_eval), 0, n, 64, 128, ptr(zall), stream_of(dev))
    wn = w.cpu().numpy()
    mids = (F32(.5) * (zc[:, 1:] + zc[:, :-1])).astype(F32)
    oza = np.sort(np.concatenate([zc, O.sample_fine(mids, wn[:, 1:-1], O.linspace_f32(0, 1, 128))], -1), -1)
    gza = zall.cpu().numpy()
    print('  zall diff (same w)', np.abs(gza - oza).max(), 'rows differing', (gza != oza).any(1).sum(), 'sorted', (np.diff(gza, axis=1) >= 0).all())
    rawf = pipe.mlp(pipe.fine, ro, rd, zall, 192, n, 192)
    gf = rawf.cpu().numpy().reshape(n, 192, 4)
    orf = O.query_network((oro[:, None] + ord_[:, None] * gza[:, :, None]).astype(F32), ord_, p, 'model_fine')
    print('  fine raw maxdiff (same z)', np.abs(gf - orf).max(), 'mag', np.abs(orf).max(), 'nan', np.isnan(gf).sum())
    wf = pipe.composite(rawf, zall, 192, rd, n, 192, out['fine'], 0)
    rgbo, dispo, acco, wo, depo = comp(gf, gza, ord_)
    print('  fine acc diff (same raw)', np.abs(out['fine'][2].cpu().numpy() - acco).max(), 'ours acc zeros', (out['fine'][2].cpu().numpy() == 0).sum(), 'oracle acc zeros', (acco == 0).sum())
    d = O._dists(gza, ord_); a = 1 - np.exp(-(np.maximum(gf[..., 3], 0) * d))
    Tm = np.cumprod(1 - np.concatenate([np.zeros((n, 1)), a[:, :-1]], 1), 1).min()
    print('  fine min T (our raw/z)', Tm)
    zer = np.nonzero(out['fine'][2].cpu().numpy() == 0)[0]
    if len(zer):
        r = zer[0]; print('  zero-acc ray', r, 'sigma max', gf[r, :, 3].max(), 'zall head', gza[r, :6], 'w sum', wf.cpu().numpy()[r].sum(), 'coarse w sum', wn[r].sum())
