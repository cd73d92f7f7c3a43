"""GPU: does a sample-chunked layer chain read its inputs from the Infinity
Cache (256 MiB)? 8 chained 256x256 x3 layer launches (forward: bias + ReLU +
amax + ReLU bits; backward: masked by those bits) at the C3 fine-pass size
(P = 1024 rays x 192 samples), layer-major over all samples (the shipped
order) against chunk-major (every layer of a sample chunk before the next
chunk), HIP-event medians; outputs compared bitwise.

    python tools/ab/ic_chunk_bench.py [chunk divisors ...]

Measured (round 2): chunking is SLOWER (8 layers fwd 1021 us at 1 chunk, 1038 /
1069 / 1277 us at 2 / 3 / 4): no Infinity Cache gain that pays for the shorter
persistent launches. NERF_X3_LAYER_NARROW=1 times the 4-byte load/store path.
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "nerf-rep_for_test_amd"))


def timeit(fn, reps=15):
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
    from nerfhip.train_mlp import _act, _layer, pack_x3_matrix, relu_bits_words
    dev = torch.device("cuda:0")
    P = 1024 * 192
    L = 8
    g = torch.Generator(device=dev).manual_seed(0)
    Ws = [torch.randn((256, 256), device=dev, generator=g) * 0.08 for _ in range(L)]
    bs = [torch.randn(256, device=dev, generator=g) * 0.1 for _ in range(L)]
    packs = [pack_x3_matrix(W) for W in Ws]
    packsT = [pack_x3_matrix(W.t().contiguous()) for W in Ws]
    X = _act(256, P, dev)
    X.copy_(torch.relu(torch.randn((256, P), device=dev, generator=g)))
    H = [_act(256, P, dev) for _ in range(L)]
    D = [_act(256, P, dev) for _ in range(L + 1)]
    D[L].copy_(torch.randn((256, P), device=dev, generator=g))
    words = relu_bits_words(P, 16)
    bits = torch.empty((L, words), device=dev, dtype=torch.int16)
    amax = torch.zeros(2 * L, device=dev)

    def fwd(chunk):
        for p0 in range(0, P, chunk):
            pc = min(chunk, P - p0)
            w0 = (p0 // 128) * 128 * 16
            src = X
            for i in range(L):
                wp, sw = packs[i]
                _layer(wp, sw, 16, 8, src[:, p0:p0 + pc], H[i][:, p0:p0 + pc], pc, bias=bs[i],
                       relu=True, amax=amax[i:i + 1], bits_out=bits[i, w0:])
                src = H[i]

    def bwd(chunk):
        for p0 in range(0, P, chunk):
            pc = min(chunk, P - p0)
            w0 = (p0 // 128) * 128 * 16
            for i in range(L - 1, -1, -1):
                wp, sw = packsT[i]
                _layer(wp, sw, 16, 8, D[i + 1][:, p0:p0 + pc], D[i][:, p0:p0 + pc], pc,
                       mask_bits=bits[i, w0:], amax=amax[L + i:L + i + 1])

    fwd(P)
    bwd(P)
    torch.cuda.synchronize()
    refH = [h.clone() for h in H]
    refD = [d.clone() for d in D[:L]]
    nbytes = L * 256 * P * 4 * 2
    divs = [int(a) for a in sys.argv[1:]] or [1, 2, 3, 4, 6, 8]
    for chunk in [P // d for d in divs]:
        chunk = -(-chunk // 128) * 128
        tf = timeit(lambda: fwd(chunk))
        tb = timeit(lambda: bwd(chunk))
        same = (all(torch.equal(a, b) for a, b in zip(H, refH)) and
                all(torch.equal(a, b) for a, b in zip(D[:L], refD)))
        print(f"chunk {chunk:7d} ({-(-P // chunk)} chunks): fwd chain {tf * 1e3:7.1f} us "
              f"({nbytes / tf / 1e6:6.0f} GB/s), bwd chain {tb * 1e3:7.1f} us "
              f"({nbytes / tb / 1e6:6.0f} GB/s), bitwise equal {same}", flush=True)


if __name__ == "__main__":
    main()
