"""Novel-view camera paths (reference volume_renderer.py:359-419).

``spiral_poses`` restates ``Renderer.generate_spiral_poses``: a spiral of
``n_frames`` cameras around the mean camera position of a pose set, radius the
mean distance to it, ``n_rots`` turns in the (right, forward) plane with a
``zrate`` sine along up, every camera looking at the centre. Vectorised over
frames, float64 like the reference's numpy.
"""
from __future__ import annotations

import numpy as np


def _unit(v):
    return v / np.linalg.norm(v, axis=-1, keepdims=True)


def spiral_poses(poses, n_frames, n_rots=2, zrate=0.5):
    poses = np.asarray(poses)
    pos = poses[:, :3, 3]
    center = pos.mean(0)
    forward = _unit(poses[:, :3, 2].mean(0))
    up = _unit(poses[:, :3, 1].mean(0))
    right = _unit(np.cross(forward, up))
    up = np.cross(right, forward)
    radius = np.linalg.norm(pos - center, axis=1).mean()
    i = np.arange(n_frames)
    theta = 2 * np.pi * n_rots * i / n_frames
    phi = zrate * np.sin(2 * np.pi * i / n_frames)
    cam = (center + radius * (np.cos(theta)[:, None] * right + np.sin(theta)[:, None] * forward)
           + phi[:, None] * up)
    fwd = _unit(center - cam)
    rgt = _unit(np.cross(fwd, up))
    cup = np.cross(rgt, fwd)
    out = np.tile(np.eye(4), (n_frames, 1, 1))
    out[:, :3, 0], out[:, :3, 1], out[:, :3, 2], out[:, :3, 3] = rgt, cup, fwd, cam
    return out
