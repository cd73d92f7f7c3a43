"""GPU: the batched weight-gradient launch (nerf_x3_wgrad_batch_z) of the C3
fine pass (P = 1024 rays x 192 samples) on feature-major operands ([rows][P + 32])
against the same operands in the 16-sample block layout ([P/16][rows][16],
train_mlp.BlockRows): results compared bit for bit, HIP-event times
interleaved.

    python tools/wgrad_layout_bench.py [P]
    WGRAD_DUMP=out.pt python tools/wgrad_layout_bench.py   # also save the results
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "nerf-rep_for_test_amd"))


def main():
    from nerfhip.train_mlp import BlockRows, WgradBatch
    dev = torch.device("cuda:0")
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 1024 * 192
    g = torch.Generator(device=dev).manual_seed(0)
    # the fine network's weight gradients (train_mlp backward): 8 layers + views tile
    shapes = [(256, 64, True), (256, 256, True), (256, 256, True), (256, 256, True),
              (256, 256, True), (256, 320, True), (256, 256, True), (256, 256, True),
              (256, 256, True), (132, 288, False)]
    ops = []
    for M, N, bias in shapes:
        A = torch.randn((M, P + 32), device=dev, generator=g)[:, :P]
        B = torch.relu(torch.randn((N, P + 32), device=dev, generator=g))[:, :P]
        ops.append((A, B, bias, BlockRows.from_dense(A), BlockRows.from_dense(B)))
    amax = [(A.abs().max().reshape(1), B.abs().max().reshape(1)) for A, B, *_ in ops]

    def run(blocked):
        wb = WgradBatch(dev)
        for (A, B, bias, Ab, Bb), (aa, ab) in zip(ops, amax):
            wb.add(Ab if blocked else A, Bb if blocked else B, aa, ab, with_bias=bias)
        return wb.results()

    r0, r1 = run(False), run(True)
    for a, b in zip(r0, r1) if not os.environ.get("NERFHIP_LIB") else ():   # (ablations)
        a = a if isinstance(a, tuple) else (a,)
        b = b if isinstance(b, tuple) else (b,)
        assert all(torch.equal(x, y) for x, y in zip(a, b)), "layouts differ"
    print("bitwise equal", flush=True)
    if os.environ.get("WGRAD_DUMP"):   # for bit-for-bit A/B of two library builds
        flat = [x.cpu() for r in r1 for x in (r if isinstance(r, tuple) else (r,))]
        torch.save(flat, os.environ["WGRAD_DUMP"])
    nbytes = sum((M + N) * P * 4 for M, N, _ in shapes)
    flop = sum(2 * M * N * P for M, N, _ in shapes)
    ts = {False: [], True: []}
    for rep in range(12):
        for blocked in (False, True):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run(blocked)
            e1.record()
            torch.cuda.synchronize()
            if rep >= 2:
                ts[blocked].append(e0.elapsed_time(e1))
    for blocked, t in ts.items():
        t.sort()
        ms = t[len(t) // 2]
        print(f"{'block layout ' if blocked else 'feature-major'}: {ms * 1e3:7.1f} us  "
              f"{nbytes / ms / 1e9:7.1f} TB/s (operand bytes)  "
              f"{3 * flop / ms / 1e9:7.1f} TF (x3 executed)", flush=True)


if __name__ == "__main__":
    main()
