#!/usr/bin/env python3
"""Instruction mix of the headline kernel, mlp_x3_kernel<false>, per 128-sample
tile and wave, from its ISA -- reconciled with the PMC per-wave counts
(profiles/r5_headline_pmc_breakdown.json).

    make -C nerf-rep_for_test_amd asm-mlp
    python tools/isa_mix.py [nerf-rep_for_test_amd/build/asm/mlp_x3.s] [--json out.json]

The kernel's tile loop (LLVM "Loop Header: Depth=1") holds the layer loop
L = 1..7 (Depth=2, mlp_x3.hip:697-729, not unrolled). Each basic block gets
its executions per tile and wave from the source structure:

* tile-loop blocks: 1, except the out-of-line blocks (sinf / cosf
  Payne-Hanek reductions for |x| beyond the fast path, and the 64-bit
  division path of n * S >= 2^32: never taken on these workloads) -> 0;
* layer-loop blocks: 7; the skip layer's extra slices and epilogue (L == 5)
  -> 1; the per-pair epilogue hooks and their joins (epi.on: L != 5) -> 6; the
  density-head dot (L == 7) -> 1; the encoding re-split (L == 4) -> 1; the
  part after the L == 7 break (next scale, split of X[0], the back edge) -> 6;
* blocks that issue the weight stream's LDS-DMA (buffer_load ... lds) run on
  the four loading waves only -> x 0.5 (the PMC counts average over waves).

Classes: mfma; valu_split (v_fma_mix: the FP32 -> FP16 hi/lo operand split);
valu_fp (fma / max / permlane / packed FP: epilogue bias, ReLU, running max,
density head); valu_other (moves, address and integer work, encoding,
selects); salu; s_nop; s_waitcnt; s_barrier; branch; lds; vmem.
"""
from __future__ import annotations

import argparse
import collections
import json
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASM = os.path.join(REPO, "nerf-rep_for_test_amd", "build", "asm", "mlp_x3.s")
PMC = os.path.join(REPO, "profiles", "r5_headline_pmc_breakdown.json")
SYMBOL = "_ZN7nerfhip13mlp_x3_kernelILb0EE"
TILE_SAMPLES, WAVE_SAMPLES = 128, 16


def kernel_lines(path, symbol=SYMBOL):
    out, on = [], False
    for line in open(path):
        if not on and line.startswith(symbol) and line.rstrip().endswith(":") is False:
            on = line.split(":")[0].startswith(symbol)
        if not on and re.match(re.escape(symbol) + r".*:", line):
            on = True
        if on:
            out.append(line.rstrip("\n"))
            if line.startswith(".Lfunc_end"):
                break
    return out


def cls(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_fma_mix"):
        return "valu_split"
    if op.startswith(("v_permlane", "v_max_f32", "v_max3_f32", "v_fma_f32", "v_fmac_f32",
                      "v_pk_", "v_add_f32", "v_mul_f32")):
        return "valu_fp"
    if op.startswith("v_"):
        return "valu_other"
    if op == "s_nop":
        return "s_nop"
    if op == "s_waitcnt":
        return "s_waitcnt"
    if op == "s_barrier":
        return "s_barrier"
    if op.startswith("s_cbranch") or op == "s_branch":
        return "branch"
    if op.startswith(("s_load", "s_buffer")):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("buffer_", "global_")):
        return "vmem"
    return "other"


def blocks_of(lines):
    blocks, cur = [], None
    for i, line in enumerate(lines):
        m = re.match(r"^(\.LBB\d+_(\d+)):|^; %bb\.(\d+):", line)
        if m:
            nxt = lines[i + 1] if i + 1 < len(lines) else ""
            dm = re.search(r"Depth=(\d+)", line + nxt)
            cur = {"name": m.group(1) or f"bb.{m.group(3)}",
                   "num": int(m.group(2) or m.group(3)), "depth": int(dm.group(1)) if dm else 0,
                   "c": collections.Counter(), "ops": collections.Counter(), "dma": False}
            blocks.append(cur)
            continue
        s = line.strip()
        if cur is None or not s or s.startswith((";", ".")) or s.endswith(":"):
            continue
        cur["c"][cls(s.split()[0])] += 1
        cur["ops"][s.split()[0]] += 1
        if "buffer_load" in s and " lds" in s:
            cur["dma"] = True
    return blocks


def weight(b, l5, l4, l7, after7):
    c, n, d = b["c"], b["num"], b["depth"]
    if d == 0:
        return 0.0
    if d == 1:
        w = 1.0
        if n >= 193 or (c["valu_other"] >= 80 and c["mfma"] == 0 and c["salu"] == 0):
            w = 0.0      # out-of-line: sinf / cosf large-argument reduction
        if b["name"] == "bb.7":
            w = 0.0      # the 64-bit division path
    else:
        w = 7.0
        if n in l5:
            w = 1.0
        elif c["valu_fp"] == 16 and c["mfma"] == 0:
            w = 6.0      # epilogue hook of a pair (epi.on: L != 5)
        elif c["valu_fp"] == 8 and c["lds"] == 2 and c["mfma"] == 0:
            w = 1.0      # the density head's dot (L == 7)
        elif sum(c.values()) == 1 and c["salu"] == 1 and n < min(l5):
            w = 6.0      # the join after a hook
        elif n in l4 or n in l7:
            w = 1.0
        elif n in after7:
            w = 6.0
    return w * (0.5 if b["dma"] else 1.0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm", nargs="?", default=ASM)
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    lines = kernel_lines(args.asm)
    blocks = blocks_of(lines)
    # the layer loop's L-specific regions, by block number (this build's layout:
    # the skip layer's slices are the only layer-loop blocks with both 48 MFMAs
    # and no operand split after the 8 slice bodies)
    d2 = [b for b in blocks if b["depth"] == 2]
    bodies = [b for b in d2 if b["c"]["mfma"] == 48]
    l5_start = [b for b in d2 if b["c"]["mfma"] == 48 and b["c"]["valu_split"] == 0][0]["num"] - 2
    l5_end = [b for b in d2 if b["c"]["mfma"] == 42][0]["num"]
    l5 = set(range(l5_start, l5_end + 1))
    tail = [b["num"] for b in d2 if b["num"] > l5_end]
    # after the skip-layer block: [movs, alpha quad sum (L7), join, L7 exit,
    # next-scale split (6), encoding split (L4), moves (6), back edge (6)]
    l7 = {tail[1], tail[3]} if len(tail) >= 8 else set()
    l4 = {tail[5]} if len(tail) >= 8 else set()
    after7 = {tail[4], tail[6], tail[7]} if len(tail) >= 8 else set()
    tot = collections.Counter()
    ops = collections.Counter()
    rows = []
    for b in blocks:
        w = weight(b, l5, l4, l7, after7)
        for k, v in b["c"].items():
            tot[k] += v * w
        for k, v in b["ops"].items():
            ops[k] += v * w
        if w and sum(b["c"].values()) >= 10:
            rows.append({"block": b["name"], "depth": b["depth"], "per_tile": w,
                         **{k: v for k, v in b["c"].items()}})
    valu = sum(tot[k] for k in ("mfma", "valu_split", "valu_fp", "valu_other"))
    out = {"kernel": "mlp_x3_kernel<false>", "asm": os.path.relpath(args.asm, REPO),
           "unit": "instructions per 128-sample tile and wave (16 samples)",
           "slice_bodies_in_layer_loop": len(bodies),
           "isa_per_tile_wave": {k: round(v, 1) for k, v in sorted(tot.items())},
           "isa_valu_incl_mfma": valu}
    if os.path.exists(PMC):
        doc = json.load(open(PMC))
        per_wave = doc["per_wave"]
        waves = doc["means_per_launch"]["SQ_WAVES"]
        # tiles per wave of the profiled launch: samples per launch / 128 / waves
        # per workgroup... the PMC pass ran the bench's coarse + fine launches:
        # MFMA per tile and wave is 3096 by construction (528 384 MAC x 16
        # samples x 3 / 8192), which fixes the tile count per wave
        tiles = per_wave["SQ_INSTS_MFMA"] / 3096.0
        pmc = {k: per_wave[k] / tiles for k in ("SQ_INSTS_MFMA", "SQ_INSTS_VALU", "SQ_INSTS_SALU",
                                                 "SQ_INSTS_LDS", "SQ_INSTS_VMEM",
                                                 "SQ_INSTS_BRANCH")}
        out["pmc_per_tile_wave"] = {k: round(v, 1) for k, v in pmc.items()}
        out["pmc_source"] = os.path.relpath(PMC, REPO)
        out["pmc_waves_per_launch"] = waves
        out["isa_over_pmc"] = {
            "mfma": tot["mfma"] / pmc["SQ_INSTS_MFMA"],
            "valu_incl_mfma": valu / pmc["SQ_INSTS_VALU"],
            "salu (s_nop, s_waitcnt, s_barrier not counted)": tot["salu"] / pmc["SQ_INSTS_SALU"],
            "lds": tot["lds"] / pmc["SQ_INSTS_LDS"], "vmem": tot["vmem"] / pmc["SQ_INSTS_VMEM"],
            "branch": tot["branch"] / pmc["SQ_INSTS_BRANCH"]}
    out["top_opcodes_per_tile_wave"] = {k: round(v, 1) for k, v in ops.most_common(40)}
    out["largest_blocks"] = sorted(rows, key=lambda r: -r["per_tile"] * sum(
        v for k, v in r.items() if k not in ("block", "depth", "per_tile")))[:24]
    txt = json.dumps(out, indent=1)
    print(txt)
    if args.json:
        with open(args.json, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    sys.exit(main())
