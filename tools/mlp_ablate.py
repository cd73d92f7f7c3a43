"""Timing-only A/B of MLP kernel variants, interleaved in one process.

    python tools/mlp_ablate.py build            # CPU: builds build/abl/lib_<v>.so
    python tools/mlp_ablate.py run [rounds]     # GPU: times each variant

Variants are compile-time switches in csrc/mlp_fused.hip (ABL_*). Outputs of
ablated variants are wrong by construction; only their time is meaningful.
"""
import ctypes
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "nerf-rep_for_test_amd")
OUT = os.path.join(PKG, "build", "abl")
VARIANTS = {"base": [], "nobar": ["-DABL_NOBAR"], "nodma": ["-DABL_NODMA"],
            "nobar_nodma": ["-DABL_NOBAR", "-DABL_NODMA"], "noenc": ["-DABL_NOENC"],
            "noepi": ["-DABL_NOEPI"],
            # placement of the weight-DMA pieces (MLP_DMA_POS / EVERY / FIRST)
            "pos1": ["-DMLP_DMA_POS=1"], "pos2": ["-DMLP_DMA_POS=2"], "pos3": ["-DMLP_DMA_POS=3"],
            "ev4": ["-DMLP_DMA_EVERY=4", "-DMLP_DMA_FIRST=1"],
            "ev4pos2": ["-DMLP_DMA_EVERY=4", "-DMLP_DMA_FIRST=1", "-DMLP_DMA_POS=2"],
            "ev3pos2": ["-DMLP_DMA_EVERY=3", "-DMLP_DMA_FIRST=2", "-DMLP_DMA_POS=2"],
            # the 3-term FP16 split kernel (mlp_x3.hip) and its ablations
            "x3": [], "x3_nodma": ["-DABL_NODMA"], "x3_nobar": ["-DABL_NOBAR"],
            "x3_nobar_nodma": ["-DABL_NOBAR", "-DABL_NODMA"],
            "x3_stagger": ["-DMLP_X3_SPREAD_DMA", "-DMLP_X3_STAGGER=1"], "x3_halflds": ["-DABL_HALFLDS"],
            "x3_halflds_nodma": ["-DABL_HALFLDS", "-DABL_NODMA"],
            "x3_noepi": ["-DABL_NOEPI"],
            "x3_spread": ["-DMLP_X3_SPREAD_DMA"],
            "x3_nodma_noepi": ["-DABL_NODMA", "-DABL_NOEPI"],
            "x3_floor": ["-DABL_NODMA", "-DABL_NOEPI", "-DABL_HALFLDS", "-DABL_NOBAR"],
            # cross-slice fragment prefetch off (the previous schedule)
            "x3_noxpf": ["-DMLP_X3_XPF=0"],
            # weight DMA as buffer_load ... lds (SGPR slice offset, constant lane offset)
            "x3_buf": ["-DMLP_DMA_BUF=1"],
            # operand split in hipcc's 7-instruction form
            "x3_nomix": ["-DMLP_X3_MIXASM=0"],
            # waves 4-7 half a slice behind (DMA two slices ahead)
            "x3_half": ["-DMLP_X3_HALF=1"],
            # weight DMA from waves 0-3 only (8 pieces each), back to back / split 4+4
            "x3_ld4": ["-DMLP_DMA_BUF=1", "-DMLP_X3_LOADERS=4"],
            "x3_ld4s": ["-DMLP_DMA_BUF=1", "-DMLP_X3_LOADERS=4", "-DMLP_X3_LOADER_SPLIT=2"],
            # the previous defaults: all 8 waves load (global form), hook VALU after the MFMAs
            "x3_prev": ["-DMLP_DMA_BUF=0", "-DMLP_X3_LOADERS=8", "-DMLP_X3_ILV=0"],
            "x3_noenc": ["-DABL_NOENC"],
            # hook VALU interleaved into the group's MFMAs, 2 / 4 per gap
            "x3_ilv2": ["-DMLP_X3_ILV=2"], "x3_ilv4": ["-DMLP_X3_ILV=4"],
            "x3_persist": ["-DMLP_X3_PERSIST=1"], "x3_pl": ["-DMLP_PERMLANE=1"],
            "x3_persist_pl": ["-DMLP_X3_PERSIST=1", "-DMLP_PERMLANE=1"],
            "x3_ld4_ilv2": ["-DMLP_DMA_BUF=1", "-DMLP_X3_LOADERS=4", "-DMLP_X3_ILV=2"],
            # static priority for the second-dispatched half / for the loading half
            "x3_prio_hi": ["-DMLP_X3_PRIO=1"], "x3_prio_lo": ["-DMLP_X3_PRIO=2"],
            # the loading half = waves 4-7, alone and with priority for waves 0-3
            "x3_ldhi": ["-DMLP_X3_LOADER_HI=1"],
            "x3_ldhi_prio_lo": ["-DMLP_X3_LOADER_HI=1", "-DMLP_X3_PRIO=2"],
            "x3_ilv1": ["-DMLP_X3_ILV=1"], "x3_ilv3": ["-DMLP_X3_ILV=3"],
            # workgroups of an XCD start staggered by k * N s_sleep(127) (k = 0..7)
            "x3_skew1": ["-DMLP_X3_SKEW=1"], "x3_skew2": ["-DMLP_X3_SKEW=2"],
            "x3_skew3": ["-DMLP_X3_SKEW=3"],
            # order of the 6 products per tile pair (x3_ops.h MLP_X3_ORD; shipped 4)
            "x3_ord0": ["-DMLP_X3_ORD=0"], "x3_ord1": ["-DMLP_X3_ORD=1"], "x3_ord2": ["-DMLP_X3_ORD=2"],
            "x3_ord3": ["-DMLP_X3_ORD=3"], "x3_ord4": ["-DMLP_X3_ORD=4"],
            "x3_ord5": ["-DMLP_X3_ORD=5"], "x3_ord7": ["-DMLP_X3_ORD=7"],
            "x3_ord8": ["-DMLP_X3_ORD=8"]}


def is_x3(v):
    return v.startswith("x3")
FLAGS = ["-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-ffp-contract=off", "-fno-slp-vectorize",
         "-fhip-fp32-correctly-rounded-divide-sqrt", "-shared"]


def build(names):
    """Build each variant's library; refuses a variant whose ISA reuses a register
    with an asm LDS read in flight (tools/check_async_lds.py)."""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import check_async_lds
    os.makedirs(OUT, exist_ok=True)
    for v in names:
        src = "mlp_x3.hip" if is_x3(v) else "mlp_fused.hip"
        asm = os.path.join(OUT, f"{v}.s")
        subprocess.check_call(["/opt/rocm/bin/hipcc", *[f for f in FLAGS if f != "-shared"],
                               *VARIANTS[v], "--offload-device-only", "-S",
                               os.path.join(PKG, "csrc", src), "-o", asm])
        if check_async_lds.main(asm) != 0:
            raise SystemExit(f"variant {v}: async LDS-read hazard in its ISA; not built")
        src = "mlp_x3.hip" if is_x3(v) else "mlp_fused.hip"
        cmd = ["/opt/rocm/bin/hipcc", *FLAGS, *VARIANTS[v], os.path.join(PKG, "csrc", "runtime.hip"),
               os.path.join(PKG, "csrc", src), "-o", os.path.join(OUT, f"lib_{v}.so")]
        subprocess.check_call(cmd)
        print("built", v)


def run(names, rounds, n_rays, S):
    sys.path.insert(0, PKG)
    import numpy as np
    import torch
    from nerfhip.pack import pack_mlp, pack_mlp_x3
    from nerfhip.synthetic import make_params
    dev = torch.device("cuda:0")
    params = make_params(0, 2.0, 0.0)
    packed = {}
    for x3, fn in ((False, pack_mlp), (True, pack_mlp_x3)):
        a, b = fn(params, "model")
        packed[x3] = (torch.from_numpy(a).to(dev), torch.from_numpy(b).to(dev))
    g = torch.Generator().manual_seed(0)
    ro = (torch.rand((n_rays, 3), generator=g) * 0.2 + torch.tensor([0.0, 2.7, 3.0])).to(dev)
    rd = torch.nn.functional.normalize(torch.randn((n_rays, 3), generator=g), dim=1).to(dev)
    z = torch.linspace(2.0, 6.0, S).to(dev)
    raw = torch.empty((n_rays * S, 4), device=dev)
    libs = {}
    for v in names:
        h = ctypes.CDLL(os.path.join(OUT, f"lib_{v}.so"))
        fn = h.nerf_mlp_forward_x3 if is_x3(v) else h.nerf_mlp_forward
        fn.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                                               ctypes.c_void_p, ctypes.c_void_p]
        libs[v] = fn
    stream = torch.cuda.current_stream().cuda_stream
    times = {v: [] for v in names}
    for r in range(rounds + 1):
        for v in names:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            sl, hd = packed[is_x3(v)]
            rc = libs[v](sl.data_ptr(), hd.data_ptr(), ro.data_ptr(), rd.data_ptr(),
                         z.data_ptr(), 0, n_rays, S, raw.data_ptr(), stream)
            e1.record()
            assert rc == 0, (v, rc)
            torch.cuda.synchronize()
            if r > 0:
                times[v].append(e0.elapsed_time(e1))
    flops = n_rays * S * 1186816
    ref = None
    for v in names:
        t = sorted(times[v])
        med = t[len(t) // 2]
        sl, hd = packed[is_x3(v)]
        raw.zero_()
        libs[v](sl.data_ptr(), hd.data_ptr(), ro.data_ptr(), rd.data_ptr(), z.data_ptr(), 0,
                n_rays, S, raw.data_ptr(), stream)
        torch.cuda.synchronize()
        out = raw.clone()
        if ref is None:
            ref = out
        diff = float((out - ref).abs().max())
        print(f"{v:14s} median {med:8.2f} ms  min {t[0]:8.2f}  TF {flops / med / 1e9:7.1f}  "
              f"frac {flops / med / 1e9 / 157.3:.3f}  maxdiff_vs_{names[0]} {diff:.3g}", flush=True)


if __name__ == "__main__":
    names = [v for v in VARIANTS if v in (sys.argv[3:] or VARIANTS)]
    if sys.argv[1] == "build":
        build(names)
    else:
        names = [v for v in names if os.path.exists(os.path.join(OUT, f"lib_{v}.so"))]
        run(names, int(sys.argv[2]) if len(sys.argv) > 2 else 5, 160000, 64)
