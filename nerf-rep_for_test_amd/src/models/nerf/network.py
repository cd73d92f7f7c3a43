"""NeRF MLP module with the reference's parameter names and forward semantics
(reference ``src/models/nerf/network.py:9-74`` NeRF, ``:126-159`` Network).

The render path never calls ``forward``: the renderer packs these parameters
into the fused HIP kernel's layout (``nerfhip.pack``). ``forward`` is kept so
the module is a faithful torch model (checkpoints, CPU inspection).
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from src.config import cfg
from src.models.encoding import get_encoder


class NeRF(nn.Module):
    def __init__(self, D=8, W=256, input_ch=63, input_ch_views=27, skips=(4,), use_viewdirs=True):
        super().__init__()
        self.D, self.W = D, W
        self.input_ch, self.input_ch_views = input_ch, input_ch_views
        self.skips = list(skips)
        self.use_viewdirs = use_viewdirs
        widths_in = [input_ch] + [W + input_ch if (i - 1) in self.skips else W for i in range(1, D)]
        self.pts_linears = nn.ModuleList(nn.Linear(fi, W) for fi in widths_in)
        self.views_linears = nn.ModuleList([nn.Linear(input_ch_views + W, W // 2)])
        if use_viewdirs:
            self.feature_linear = nn.Linear(W, W)
            self.alpha_linear = nn.Linear(W, 1)
            self.rgb_linear = nn.Linear(W // 2, 3)
        else:
            self.output_linear = nn.Linear(W, 4)

    def forward(self, x):
        pts = x[..., :self.input_ch]
        views = x[..., self.input_ch:self.input_ch + self.input_ch_views]
        h = pts
        for i, layer in enumerate(self.pts_linears):
            h = F.relu(layer(h))
            if i in self.skips:
                h = torch.cat([pts, h], -1)
        if not self.use_viewdirs:
            return self.output_linear(h)
        sigma = self.alpha_linear(h)
        h = torch.cat([self.feature_linear(h), views], -1)
        for layer in self.views_linears:
            h = F.relu(layer(h))
        return torch.cat([self.rgb_linear(h), sigma], -1)


class Network(nn.Module):
    def __init__(self):
        super().__init__()
        ta, net = cfg.task_arg, cfg.network
        self.N_samples, self.N_importance = ta.N_samples, ta.N_importance
        self.chunk, self.batch_size = ta.chunk_size, ta.N_rays
        self.white_bkgd, self.use_viewdirs = ta.white_bkgd, ta.use_viewdirs
        self.device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
        self.embed_fn, self.input_ch = get_encoder(net.xyz_encoder)
        self.embeddirs_fn, self.input_ch_views = get_encoder(net.dir_encoder)

        def mk():
            return NeRF(D=net.nerf.D, W=net.nerf.W, input_ch=self.input_ch,
                        input_ch_views=self.input_ch_views, skips=net.nerf.skips,
                        use_viewdirs=self.use_viewdirs)
        self.model = mk()
        self.model_fine = mk()
