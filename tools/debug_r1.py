import sys, os, numpy as np, torch
sys.path[:0] = ['nerf-rep_for_test_amd', '.', 'tests']
from goldlib import load, params_of, grid_of
from oracle import nerf_oracle as O
from nerfhip.render import NerfPipeline
from nerfhip._lib import call, ptr, stream_of
dev = torch.device('cuda:0')
def t(a): return torch.from_numpy(np.ascontiguousarray(a)).to(dev)
# 1. sample_fine
z = load('f1_c2_crop'); zc, wc = z['int_zc'], z['int_wc']; n, S = zc.shape; NI = 128
pipe = NerfPipeline(dev, N_samples=64, N_importance=128)
zall = torch.empty((n, S+NI), device=dev)
zc_d, wc_d = t(zc), t(wc)
call("nerf_sample_fine", ptr(zc_d), S, ptr(wc_d), ptr(pipe.u_eval), 0, n, S, NI, ptr(zall), stream_of(dev))
got = zall.cpu().numpy()
mids = (np.float32(0.5)*(zc[:,1:]+zc[:,:-1])).astype(np.float32)
zf = O.sample_fine(mids, wc[:,1:-1], O.linspace_f32(0,1,NI))
ref = np.sort(np.concatenate([zc, zf], -1), -1)
bad = np.nonzero((got != ref).any(1))[0]
print('sample_fine rays differing', len(bad), 'of', n)
if len(bad):
    r = bad[0]; j = np.nonzero(got[r] != ref[r])[0]
    print(' ray', r, 'cols', j[:10], 'got', got[r, j[:5]], 'ref', ref[r, j[:5]], 'absdiff', np.abs(got[r]-ref[r]).max())
    print(' nan in got', np.isnan(got).sum(), 'inf', np.isinf(got).sum())
    print(' got row head', got[r,:8], '\n ref row head', ref[r,:8])
# 2. ESS f4b
z = load('f4b_ess_ert_update'); grid = grid_of(z); H, W = int(z['H']), int(z['W'])
oro, ord_ = O.camera_rays(H, W, z['pose'], z['K']); nn = oro.shape[0]; tr = z['t_rand']
pipe.set_grid(grid)
zz = torch.empty((nn, 64), device=dev)
call("nerf_sample_coarse_ess", ptr(t(oro)), ptr(t(ord_)), ptr(pipe.grid), 128, ptr(pipe.z_base), ptr(t(tr)), nn, 64, 2048, 0.5, ptr(zz), stream_of(dev))
g = zz.cpu().numpy()
for c0 in range(0, nn, 2048):
    sl = slice(c0, min(nn, c0+2048))
    rref = O.sample_coarse_ess(oro[sl], ord_[sl], grid, 2.0, 6.0, 64, False, 1.0, tr[sl])
    d = np.nonzero((g[sl] != rref).any(1))[0]
    print('ESS chunk', c0, 'rows differing', len(d), 'nan', np.isnan(g[sl]).sum(), 'inf', np.isinf(g[sl]).sum())
    if len(d):
        r = d[0]; print('  row', r, g[sl][r][:8], rref[r][:8], 'maxdiff', np.nanmax(np.abs(g[sl][r]-rref[r])))
    # no perturb version
    z2 = torch.empty((nn, 64), device=dev)
call("nerf_sample_coarse_ess", ptr(t(oro)), ptr(t(ord_)), ptr(pipe.grid), 128, ptr(pipe.z_base), None, nn, 64, 2048, 0.5, ptr(z2), stream_of(dev))
g2 = z2.cpu().numpy()
for c0 in range(0, nn, 2048):
    sl = slice(c0, min(nn, c0+2048))
    rref = O.sample_coarse_ess(oro[sl], ord_[sl], grid, 2.0, 6.0, 64, False, 0.0, None)
    print('ESS noperturb chunk', c0, 'rows differing', (g2[sl] != rref).any(1).sum(), 'row0 got', g2[sl][0][:6], 'ref', rref[0][:6])
# 3. ERT f3b decisions
for name in ['f3b_ert_noterm', 'f3_ert']:
    z = load(name)
    print(name, 'ref chunk_any', [bool(z[k]) for k in z if k.startswith('int_chunk_any')])
    ref_acc = z['out_acc_map'].reshape(-1); print('  ref fine acc zeros', (ref_acc == 0).sum(), 'nan disp', np.isnan(z['out_disp_map']).sum())
    p2 = NerfPipeline(dev, N_samples=64, N_importance=128, enable_ert=True, ert_threshold=0.01)
    p2.set_weights(params_of(z))
    res = {k: v.cpu().numpy() for k, v in p2.render_image(int(z['H']), int(z['W']), z['pose'], z['K']).items()}
    print('  ours fine acc zeros', (res['acc_map'] == 0).sum(), 'nan disp', np.isnan(res['disp_map']).sum(), 'coarse acc zeros', (res['acc_map_0']==0).sum(), 'ref coarse', (z['out_acc_map_0']==0).sum())
