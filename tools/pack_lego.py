#!/usr/bin/env python3
"""Pack the lego Blender views into compact, self-contained files (this container).

The GPU box has no /root/reference, so the images the training run and the
PSNR-vs-ground-truth evaluation need travel inside the repository tree (git-
ignored: data, not source). The PNG files are stored byte for byte (no
re-encoding, so decoding on the box yields exactly the reference dataset's
pixels) together with the camera poses of ``transforms_<split>.json``:

  data/lego/train.npz  100 train views (BASELINE configs[2] training data)
  data/lego/test.npz   every 8th test view (frames 0, 8, ..., 192): the PSNR set
  data/lego/test_all.npz  all 200 test views (--splits test --test-stride 1: the
                       whole test split for bench.py --config c5 --gt-path)

Keys: ``png_bytes`` uint8 (concatenated files), ``png_offsets`` int64 [N+1],
``frames`` int32 [N] (index into the split's json), ``poses`` float32 [N,4,4],
``camera_angle_x`` float64. Read with ``nerfhip.evaluate.load_packed``.

    python tools/pack_lego.py [--src /root/reference/data/nerf_synthetic/lego] [--out data/lego]
"""
import argparse
import json
import os

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = "/root/reference/data/nerf_synthetic/lego"


def pack(src, split, stride, out):
    meta = json.load(open(os.path.join(src, f"transforms_{split}.json")))
    frames = list(range(0, len(meta["frames"]), stride))
    blobs, poses = [], []
    for i in frames:
        f = meta["frames"][i]
        with open(os.path.join(src, f["file_path"] + ".png"), "rb") as fh:
            blobs.append(np.frombuffer(fh.read(), np.uint8))
        poses.append(np.array(f["transform_matrix"], np.float32))
    offs = np.zeros(len(blobs) + 1, np.int64)
    offs[1:] = np.cumsum([b.size for b in blobs])
    np.savez(out, png_bytes=np.concatenate(blobs), png_offsets=offs,
             frames=np.array(frames, np.int32), poses=np.stack(poses),
             camera_angle_x=np.float64(meta["camera_angle_x"]))
    print(f"{out}: {len(frames)} views, {os.path.getsize(out) / 2**20:.1f} MiB")


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", default=SRC)
    ap.add_argument("--out", default=os.path.join(REPO, "data", "lego"))
    ap.add_argument("--splits", default="train,test")
    ap.add_argument("--test-stride", type=int, default=8,
                    help="every n-th test view (8: the 25-view PSNR set test.npz; 1: all 200 "
                         "views, written as test_all.npz for bench.py --config c5 --gt-path)")
    args = ap.parse_args(argv)
    os.makedirs(args.out, exist_ok=True)
    for split in args.splits.split(","):
        stride = args.test_stride if split == "test" else 1
        name = "test_all" if split == "test" and stride == 1 else split
        pack(args.src, split, stride, os.path.join(args.out, f"{name}.npz"))


if __name__ == "__main__":
    main()
