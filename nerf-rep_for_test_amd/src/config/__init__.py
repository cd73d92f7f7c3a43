"""Minimal stand-in for the reference's global ``cfg`` (``src/config/config.py``).

Only what the render path reads (``volume_renderer.py:31-59``,
``network.py:126-159``), with the values of ``configs/nerf/lego.yaml``. When this
package's ``volume_renderer.py`` is dropped into the reference tree, the
reference's own ``src.config`` is imported instead and nothing here is used.
``load_yaml`` merges a yaml file (safe loader) for standalone use.
"""
from __future__ import annotations

import copy


class Node(dict):
    """dict with attribute access, like yacs.CfgNode (new keys allowed)."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v

    @staticmethod
    def wrap(d):
        return Node({k: Node.wrap(v) if isinstance(v, dict) else v for k, v in d.items()})


LEGO_DEFAULTS = {
    "task": "nerf_replication",
    "scene": "lego",
    "renderer_module": "src.models.nerf.renderer.volume_renderer",
    "renderer_path": "src/models/nerf/renderer/volume_renderer.py",
    "task_arg": {"N_rays": 1024, "chunk_size": 4096, "white_bkgd": 1, "N_samples": 64,
                 "N_importance": 128, "use_viewdirs": True, "lindisp": False, "perturb": 1,
                 "raw_noise_std": 0},
    "network": {"nerf": {"W": 256, "D": 8, "V_D": 1, "skips": [4]},
                "xyz_encoder": {"type": "frequency", "input_dim": 3, "freq": 10},
                "dir_encoder": {"type": "frequency", "input_dim": 3, "freq": 4}},
    "enable_ess": True, "enable_ert": True, "ert_threshold": 0.01,
    "occupancy_grid_resolution": 128,
    "use_cuda_kernels": True, "cuda_blocks": 128, "cuda_threads": 256,
}

cfg = Node.wrap(copy.deepcopy(LEGO_DEFAULTS))


def _merge(dst, src):
    for k, v in src.items():
        if isinstance(v, dict) and isinstance(dst.get(k), dict):
            _merge(dst[k], v)
        else:
            dst[k] = Node.wrap(v) if isinstance(v, dict) else v


def load_yaml(path, into=None):
    import yaml
    with open(path) as f:
        data = yaml.safe_load(f) or {}
    target = cfg if into is None else into
    _merge(target, data)
    return target


def reset():
    cfg.clear()
    cfg.update(Node.wrap(copy.deepcopy(LEGO_DEFAULTS)))
