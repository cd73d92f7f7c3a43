"""Input encoders the render path uses (reference ``src/models/encoding``).

Only the frequency (positional) encoder is on the lego path
(``configs/nerf/lego.yaml`` xyz/dir_encoder.type = frequency); the hash-grid,
triplane and D-NeRF encoders are out of scope and raise.
The fused HIP MLP computes this encoding itself; ``embed_fn`` exists for the
``Network`` attribute contract and for torch-side callers.
"""
import torch


def frequency_encoder(n_freq: int, input_dim: int = 3):
    """x -> [x, sin(2^0 x), cos(2^0 x), ..., sin(2^(L-1) x), cos(2^(L-1) x)]
    (reference ``freq.py:7-32`` with include_input, log_sampling)."""
    bands = 2.0 ** torch.linspace(0.0, n_freq - 1, steps=n_freq)

    def embed(x):
        parts = [x]
        for f in bands:
            xf = x * f
            parts.append(torch.sin(xf))
            parts.append(torch.cos(xf))
        return torch.cat(parts, -1)

    return embed, input_dim * (1 + 2 * n_freq)


def get_encoder(cfg):
    """Reference ``encoding/__init__.py:6-18`` contract: returns (fn, out_dim)."""
    if cfg.type == "frequency":
        return frequency_encoder(int(cfg.freq), int(cfg.input_dim))
    raise NotImplementedError(f"encoder {cfg.type!r} is outside the render hot path")
