"""GPU: HIP-event timing of the training-MLP kernels at the C3 fine-pass size
(P = 1024 rays x 192 samples), interleaved variants in one process.

    python tools/train_kernels_bench.py
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "nerf-rep_for_test_amd"))


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    from nerfhip.train_mlp import _layer, _wgrad, pack_x3_matrix
    dev = torch.device("cuda:0")
    P = 1024 * 192
    g = torch.Generator(device=dev).manual_seed(0)
    W = torch.randn((256, 256), device=dev, generator=g) * 0.06
    B = torch.relu(torch.randn((256, P), device=dev, generator=g))
    M = torch.randn((256, P), device=dev, generator=g)
    bias = torch.randn(256, device=dev, generator=g)
    C = torch.empty((256, P), device=dev)
    wp, sw = pack_x3_matrix(W)
    amax = torch.zeros(1, device=dev)
    flop = 2 * 256 * 256 * P
    rows = []
    for name, fn in [
        ("layer bias+relu", lambda: _layer(wp, sw, 16, 8, B, C, P, bias=bias, relu=True)),
        ("layer bias+relu+amax", lambda: _layer(wp, sw, 16, 8, B, C, P, bias=bias, relu=True,
                                                amax=amax)),
        ("layer mask", lambda: _layer(wp, sw, 16, 8, B, C, P, mask=M)),
        ("layer mask+amax", lambda: _layer(wp, sw, 16, 8, B, C, P, mask=M, amax=amax)),
        ("wgrad 256x256", lambda: _wgrad(M, B, amax, amax)),
        ("wgrad 256x256+bias", lambda: _wgrad(M, B, amax, amax, with_bias=True)),
    ]:
        ms = timeit(fn)
        nbytes = 256 * P * 4 * (3 if "mask" in name else 2)
        rows.append(f"{name:24s} {ms * 1e3:8.1f} us  {flop / ms / 1e9:7.1f} TF(alg)  "
                    f"{nbytes / ms / 1e9:7.1f} GB/s(min bytes)")
    print("\n".join(rows), flush=True)

    # the weight-gradient kernel alone (no split-K sum), by row stride of A and B
    from nerfhip import _lib
    from nerfhip.train_mlp import wgrad_chunk
    chunk = wgrad_chunk(P)
    part = torch.empty((-(-P // chunk), 256, 256), device=dev)
    for pad in (0, 32, 64, 256, 1024):
        Ap = torch.randn((256, P + pad), device=dev, generator=g)[:, :P]
        Bp = torch.relu(torch.randn((256, P + pad), device=dev, generator=g))[:, :P]
        fn = lambda: _lib.call("nerf_x3_wgrad", Ap.data_ptr(), Ap.stride(0), 256, Bp.data_ptr(),
                               Bp.stride(0), 256, P, chunk, amax.data_ptr(), amax.data_ptr(),
                               part.data_ptr(), 0, _lib.stream_of(dev))
        ms = timeit(fn)
        print(f"wgrad kernel, row pad {pad:5d} floats {ms * 1e3:8.1f} us  "
              f"{2 * 256 * P * 4 / ms / 1e9:7.2f} TB/s (A+B once)", flush=True)


if __name__ == "__main__":
    main()
