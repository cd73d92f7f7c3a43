"""ctypes binding of lib/libnerfhip.so (the C ABI declared in include/nerfhip.h).

There is no fallback: if the library is missing or no ROCm device is present,
``lib()`` raises, and so does every op built on it.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ABI_VERSION = 7   # include/nerfhip.h NERF_ABI_VERSION
LIB_PATH = os.environ.get("NERFHIP_LIB", os.path.join(PKG_ROOT, "lib", "libnerfhip.so"))

MLP_SLICES = 73
MLP_SLICE_FLOATS = 8192
MLP_HEAD_FLOATS = 3200

_P, _I, _I64, _F, _S, _SZ = C.c_void_p, C.c_int, C.c_int64, C.c_float, C.c_void_p, C.c_size_t

# name -> (restype, argtypes); mirrors include/nerfhip.h
SIGNATURES = {
    "nerf_last_error": (C.c_char_p, []),
    "nerf_version": (_I, []),
    "nerf_build_id": (C.c_char_p, []),
    "nerf_rays": (_I, [_P, _I, _I, _I64, _I64, _P, _P, _S]),
    "nerf_sample_coarse": (_I, [_P, _P, _I64, _I, _P, _S]),
    "nerf_mlp_forward": (_I, [_P, _P, _P, _P, _P, _I64, _I64, _I, _P, _S]),
    "nerf_mlp_forward_x3": (_I, [_P, _P, _P, _P, _P, _I64, _I64, _I, _P, _S]),
    "nerf_mlp_forward_x3_clock": (_I, [_P, _P, _P, _P, _P, _I64, _I64, _I, _P, _P, _I64, _P, _S]),
    "nerf_mlp_forward_x3_list": (_I, [_P, _P, _P, _P, _P, _I64, _I, _P, _P, _I64, _P, _S]),
    "nerf_mlp_train_forward_x3": (_I, [_P, _P, _P, _P, _P, _I64, _P, _P, _S]),
    "nerf_mlp_train_forward_x3_rays": (_I, [_P, _P, _P, _P, _P, _I64, _I64, _I, _P, _P, _S]),
    "nerf_mlp_train_backward_x3": (_I, [_P, _P, _I64, _I, _P, _S]),
    "nerf_ert_segment": (_I, [_P, _P, _I64, _P, _I64, _I, _I, _I, _I, _F, _P, _P, _P, _P, _S]),
    "nerf_x3_layer": (_I, [_P, _P, _I, _I, _P, _P, _I64, _P, _I64, _P, _P, _I, _P, _I64, _I64,
                           _P, _S]),
    "nerf_x3_layer_ex": (_I, [_P, _P, _I, _I, _P, _P, _I64, _P, _I64, _P, _P, _I, _P, _I64,
                              _I64, _P, _P, _P, _P, _P, _I, _P, _I, _S]),
    "nerf_adam_step": (_I, [_P, _I, _P, _P, _P, C.c_double, C.c_double, _F, _F, _S]),
    "nerf_sum_partials": (_I, [_P, _I64, _I64, _P, _S]),
    "nerf_x3_wgrad_batch": (_I, [_P, _I, _I, _S]),
    "nerf_x3_wgrad_batch_z": (_I, [_P, _I, _P, _I, _S]),
    "nerf_x3_wgrad": (_I, [_P, _I64, _I, _P, _I64, _I, _I64, _I64, _P, _P, _P, _P, _S]),
    "nerf_x3_pack": (_I, [_P, _I, _P, _I, _S]),
    "nerf_composite_train_fwd": (_I, [_P, _P, _P, _I64, _I, _I, _P, _P, _P, _P, _P, _P, _S]),
    "nerf_composite_train_bwd": (_I, [_P, _P, _P, _P, _P, _P, _P, _I64, _I, _I, _P, _P, _P, _P,
                                      _P, _P, _P, _S]),
    "nerf_views_feature_grads": (_I, [_P, _I64, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I64,
                                      _P, _P, _P, _S]),
    "nerf_mse_pair": (_I, [_P, _P, _P, _I64, _P, _S]),
    "nerf_mse_pair_backward": (_I, [_P, _P, _P, _I64, _P, _P, _P, _P, _P, _S]),
    "nerf_sample_pdf_bwd": (_I, [_P, _P, _P, _P, _P, _I64, _I, _I, _P, _S]),
    "nerf_freq_encode_fm": (_I, [_P, _I64, _I64, _I, _P, _I64, _P, _S]),
    "nerf_freq_encode_fm_backward": (_I, [_P, _I64, _P, _I64, _I64, _I, _P, _S]),
    "nerf_raw_absmax": (_I, [_P, _I64, _P, _S]),
    "nerf_freq_encode_fm_backward_sum": (_I, [_P, _P, _I64, _I64, _P, _I64, _I64, _P, _I64, _I64,
                                              _I, _P, _S]),
    "nerf_freq_encode_fm_backward_dz": (_I, [_P, _P, _I64, _I64, _P, _I64, _I64, _P, _I, _I64, _I,
                                             _P, _S]),
    "nerf_composite": (_I, [_P, _P, _I64, _P, _I64, _I, _I, _P, _P, _P, _P, _P, _S]),
    "nerf_add_sigma_noise": (_I, [_P, _P, _I64, _P, _S]),
    "nerf_grid_points": (_I, [_I64, _I64, _I, C.POINTER(_F), C.POINTER(_F), _P, _S]),
    "nerf_grid_decide": (_I, [_P, _I64, _I64, _I, _F, _P, _P, _S]),
    "nerf_fold_views": (_I, [_P, _I, _S]),
    "nerf_linear_fm": (_I, [_P, _I64, _P, _P, _I64, _I, _I64, _I, _I, _P, _I64, _I64, _S]),
    "nerf_composite_ert_workspace": (_SZ, [_I64, _I]),
    "nerf_composite_ert": (_I, [_P, _P, _I64, _P, _I64, _I, _I, _F, _I, _P, _P, _P, _P, _P, _P,
                                _S]),
    "nerf_sample_fine": (_I, [_P, _I64, _P, _P, _I64, _I64, _I, _I, _P, _S]),
    "nerf_sample_coarse_ess": (_I, [_P, _P, _P, _I, _P, _P, _I64, _I, _I, _F, _P, _S]),
    "nerf_grid_update": (_I, [_P, _P, _I64, _P, _P, _I64, _I, _P, _I, _S]),
    "kn_get_rays_d": (_I, [_I, _I, _F, _F, _F, _F, _P, _P, _S]),
    "kn_generate_query_indices_on_ray": (_I, [_P, _P, _I, _P, _P, _P, _P, _P, _P, _P, _F, _I, _I,
                                              _F, _I, _P, _P, _S]),
    "kn_compute_fourier_features": (_I, [_P, _I64, _P, _I, _P, _S]),
    "kn_integrate": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _F, _I, _S]),
    "kn_replace_transparency_by_background_color": (_I, [_P, _P, _I64, _P, _S]),
    "kn_gather_int32": (_I, [_P, _I64, _P, _P, _S]),
    "kn_scatter_int32_float4": (_I, [_P, _I64, _P, _P, _S]),
    "kn_sort_scratch_bytes": (_SZ, [_I64, _I]),
    "kn_sort_by_key_int16": (_I, [_P, _P, _I, _I64, _P, _S]),
    "kn_global_to_local": (_I, [_P, _P, _P, _P, _I, _S]),
    "kn_network_eval_query_index": (_I, [_P, _I64, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I,
                                         _F, _F, _F, _F, _I, _F, _F, _P, _S]),
    "kn_init_stream_pool": (_I, [_I64]),
    "kn_destroy_stream_pool": (_I, []),
    "kn_init_magma": (_I, []),
    "kn_init_multimatmul_grouped": (_I, [_I64, _I64, _I64, _P, _I, C.POINTER(C.c_int)]),
    "kn_deinit_multimatmul_grouped": (_I, [_I]),
    "kn_multimatmul_grouped": (_I, [_I, _I, _P, _P, _P, _I64, _I64, _P, _I, _P, _S]),
    "kn_multi_row_sum_reduction": (_I, [_P, _I64, _P, _I, _P, _S]),
    "kn_multimatmul_A_transposed": (_I, [_P, _I64, _P, _I64, _P, _I, _P, _S]),
    "kn_render_to_screen": (_I, []),
}

_lock = threading.Lock()
_lib = None


class NerfHipError(RuntimeError):
    pass


def tree_build_id():
    """sha256 (16 hex digits) of the csrc/ files in byte order, then
    include/nerfhip.h -- the digest the Makefile bakes into the library as
    nerf_build_id(); None when the sources are not beside the package."""
    import hashlib
    src = os.path.join(PKG_ROOT, "csrc")
    hdr = os.path.join(os.path.dirname(PKG_ROOT), "include", "nerfhip.h")
    if not (os.path.isdir(src) and os.path.exists(hdr)):
        return None
    h = hashlib.sha256()
    for f in sorted(os.listdir(src)):
        fp = os.path.join(src, f)
        if os.path.isfile(fp):
            with open(fp, "rb") as fh:
                h.update(fh.read())
    with open(hdr, "rb") as fh:
        h.update(fh.read())
    return h.hexdigest()[:16]


def build_id():
    """The source-tree digest compiled into the loaded library."""
    return lib().nerf_build_id().decode()


def lib():
    """Load the library once (raises NerfHipError if it is not built, or if it was
    built from sources other than the tree beside it: the measured binary is HEAD's)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise NerfHipError(
                    f"HIP library not found at {LIB_PATH}: build it with "
                    "`make -C nerf-rep_for_test_amd` (or __graft_entry__.build())")
            h = C.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(h, name)
                fn.restype = res
                fn.argtypes = args
            # the struct layouts and signatures of SIGNATURES are those of ABI_VERSION:
            # enforced for every library, NERFHIP_LIB variants included
            ver = h.nerf_version()
            if ver != ABI_VERSION:
                raise NerfHipError(f"{LIB_PATH} has ABI version {ver}, this module speaks "
                                   f"{ABI_VERSION} (include/nerfhip.h NERF_ABI_VERSION)")
            want = tree_build_id()
            got = h.nerf_build_id().decode()
            # NERFHIP_LIB points at a deliberately different build (timing-only
            # variants of tools/): its id is reported, not enforced
            if want is not None and got != want and "NERFHIP_LIB" not in os.environ:
                raise NerfHipError(
                    f"{LIB_PATH} was built from sources with id {got}, but the tree holds "
                    f"{want}: rebuild with `make -C nerf-rep_for_test_amd`")
            _lib = h
    return _lib


def check(rc: int, name: str) -> None:
    if rc != 0:
        msg = lib().nerf_last_error().decode(errors="replace")
        raise NerfHipError(f"{name} failed (code {rc}): {msg}")


def call(name: str, *args) -> None:
    check(getattr(lib(), name)(*args), name)


def ptr(t) -> int:
    """Device (or host) address of a torch tensor, or None for None.

    The caller must keep ``t`` referenced until the call using the address has
    been enqueued: the address of a temporary (``ptr(x.contiguous())``) can be
    handed to the next allocation by torch's caching allocator."""
    if t is None:
        return None
    return t.data_ptr()


def stream_of(device=None) -> int:
    import torch
    return torch.cuda.current_stream(device).cuda_stream


def require_gpu(t) -> None:
    if not t.is_cuda:
        raise NerfHipError("nerfhip ops need tensors on a ROCm GPU (got %s); there is no CPU "
                           "fallback" % t.device)
