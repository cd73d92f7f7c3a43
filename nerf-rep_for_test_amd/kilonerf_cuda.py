"""``kilonerf_cuda``: the reference extension's op contract on gfx950.

Same module name, op names and positional signatures as the reference's
pybind module (``cuda/pybind.cu:13-38``; headers ``cuda/*.cuh``), so
``import kilonerf_cuda`` in the reference renderer (``volume_renderer.py:10-16``)
resolves here. Each op calls the corresponding ``kn_*`` entry of
``lib/libnerfhip.so`` on torch's current stream. The CUDA launch-geometry
arguments (blocks/threads/version/implementation) are accepted and ignored:
launch shapes are chosen for MI355X. Errors raise ``RuntimeError``
(``NerfHipError``) instead of the reference's ``exit()``.
"""
import ctypes

import torch

from nerfhip import _lib
from nerfhip._lib import NerfHipError, call, ptr

__all__ = [
    "init_stream_pool", "destroy_stream_pool", "init_magma",
    "multimatmul_magma_grouped_static", "multimatmul_magma_grouped_static_without_bias",
    "multimatmul_magma_grouped_static_without_bias_transposed_weights",
    "init_multimatmul_magma_grouped", "deinit_multimatmul_magma_grouped",
    "multi_row_sum_reduction", "multimatmul_A_transposed",
    "gather_int32", "scatter_int32_float4", "sort_by_key_int16_int64", "sort_by_key_int16_int32",
    "get_rays_d", "generate_query_indices_on_ray", "global_to_local", "compute_fourier_features",
    "network_eval_query_index", "integrate", "replace_transparency_by_background_color",
    "render_to_screen",
]


def _st(t):
    return _lib.stream_of(t.device)


def _gpu(*ts):
    for t in ts:
        _lib.require_gpu(t)


def _host_i64(t):
    return t.detach().to("cpu", torch.int64).contiguous()


# ---------------------------------------------------------------- multimatmul.cuh
def init_stream_pool(num_streams):
    call("kn_init_stream_pool", int(num_streams))


def destroy_stream_pool():
    call("kn_destroy_stream_pool")


def init_magma():
    call("kn_init_magma")


def init_multimatmul_magma_grouped(num_networks, out_features, in_features, group_limits):
    gl = (ctypes.c_int32 * max(1, len(group_limits)))(*[int(x) for x in group_limits])
    h = ctypes.c_int(-1)
    call("kn_init_multimatmul_grouped", int(num_networks), int(out_features), int(in_features),
         ctypes.cast(gl, ctypes.c_void_p), len(group_limits), ctypes.byref(h))
    return h.value


def deinit_multimatmul_magma_grouped(aux_index):
    call("kn_deinit_multimatmul_grouped", int(aux_index))


def _grouped(mode, biases, input_vectors, weights, out_features, in_features,
             batch_size_per_network, aux_index):
    _gpu(input_vectors, weights)
    bspn = _host_i64(batch_size_per_network)
    out = torch.empty((input_vectors.shape[0], int(out_features)), device=input_vectors.device,
                      dtype=torch.float32)
    call("kn_multimatmul_grouped", int(aux_index), mode, ptr(biases) if mode == 0 else None,
         ptr(input_vectors), ptr(weights), int(out_features), int(in_features), ptr(bspn),
         bspn.numel(), ptr(out), _st(input_vectors))
    return out


def multimatmul_magma_grouped_static(biases, input_vectors, weights, out_features, in_features,
                                     batch_size_per_network, kernel_num_blocks, kernel_num_threads,
                                     group_limits, aux_index):
    return _grouped(0, biases, input_vectors, weights, out_features, in_features,
                    batch_size_per_network, aux_index)


def multimatmul_magma_grouped_static_without_bias(biases, input_vectors, weights, out_features,
                                                  in_features, batch_size_per_network,
                                                  kernel_num_blocks, kernel_num_threads,
                                                  group_limits, aux_index):
    return _grouped(1, biases, input_vectors, weights, out_features, in_features,
                    batch_size_per_network, aux_index)


def multimatmul_magma_grouped_static_without_bias_transposed_weights(
        biases, input_vectors, weights, out_features, in_features, batch_size_per_network,
        kernel_num_blocks, kernel_num_threads, group_limits, aux_index):
    return _grouped(2, biases, input_vectors, weights, out_features, in_features,
                    batch_size_per_network, aux_index)


def multi_row_sum_reduction(input_matrix, batch_size_per_network):
    _gpu(input_matrix)
    bspn = _host_i64(batch_size_per_network)
    cols = input_matrix.shape[1]
    out = torch.zeros((bspn.numel(), cols), device=input_matrix.device, dtype=torch.float32)
    call("kn_multi_row_sum_reduction", ptr(input_matrix), cols, ptr(bspn), bspn.numel(), ptr(out),
         _st(input_matrix))
    return out


def multimatmul_A_transposed(A, B, batch_size_per_network):
    _gpu(A, B)
    bspn = _host_i64(batch_size_per_network)
    out = torch.zeros((bspn.numel(), A.shape[1], B.shape[1]), device=A.device, dtype=torch.float32)
    call("kn_multimatmul_A_transposed", ptr(A), A.shape[1], ptr(B), B.shape[1], ptr(bspn),
         bspn.numel(), ptr(out), _st(A))
    return out


# ---------------------------------------------------------------- reorder.cuh
def gather_int32(map_tensor, input_tensor):
    _gpu(map_tensor, input_tensor)
    out = torch.empty((map_tensor.shape[0],), device=input_tensor.device, dtype=torch.int32)
    call("kn_gather_int32", ptr(map_tensor), map_tensor.shape[0], ptr(input_tensor), ptr(out),
         _st(input_tensor))
    return out


def scatter_int32_float4(map_tensor, input_tensor):
    _gpu(map_tensor, input_tensor)
    out = torch.empty((input_tensor.shape[0], 4), device=input_tensor.device, dtype=torch.float32)
    call("kn_scatter_int32_float4", ptr(map_tensor), input_tensor.shape[0], ptr(input_tensor),
         ptr(out), _st(input_tensor))
    return out


def _sort(keys, values, vbytes):
    _gpu(keys, values)
    n = keys.shape[0]
    scratch = torch.empty((_lib.lib().kn_sort_scratch_bytes(n, vbytes),), device=keys.device,
                          dtype=torch.uint8)
    call("kn_sort_by_key_int16", ptr(keys), ptr(values), vbytes, n, ptr(scratch), _st(keys))


def sort_by_key_int16_int64(keys_tensor, values_tensor):
    _sort(keys_tensor, values_tensor, 8)


def sort_by_key_int16_int32(keys_tensor, values_tensor):
    _sort(keys_tensor, values_tensor, 4)


# ---------------------------------------------------------------- generate_inputs.cuh
def get_rays_d(H, W, cx, cy, fx, fy, c2w_tensor, root_num_blocks, root_num_threads):
    _gpu(c2w_tensor)
    out = torch.empty((int(H), int(W), 3), device=c2w_tensor.device, dtype=torch.float32)
    c2w = c2w_tensor.contiguous()            # held until the launch is enqueued
    call("kn_get_rays_d", int(H), int(W), float(cx), float(cy), float(fx), float(fy),
         ptr(c2w), ptr(out), _st(c2w_tensor))
    return out


def generate_query_indices_on_ray(origin_tensor, directions_tensor, occupancy_grid_tensor,
                                  active_ray_mask_tensor, depth_indices_tensor, voxel_size_tensor,
                                  global_domain_min_tensor, global_domain_max_tensor, strides_tensor,
                                  distance_between_points, max_samples_per_ray, max_depth_index,
                                  min_distance, is_initial_query, kernel_max_num_blocks,
                                  kernel_max_num_threads, version):
    _gpu(directions_tensor, occupancy_grid_tensor, active_ray_mask_tensor)
    n = directions_tensor.shape[0]
    dev = directions_tensor.device
    qi = torch.empty((n, int(max_samples_per_ray)), device=dev, dtype=torch.int32)
    nets = torch.empty((n, int(max_samples_per_ray)), device=dev, dtype=torch.int16)
    call("kn_generate_query_indices_on_ray", ptr(origin_tensor), ptr(directions_tensor), n,
         ptr(occupancy_grid_tensor), ptr(active_ray_mask_tensor), ptr(depth_indices_tensor),
         ptr(voxel_size_tensor), ptr(global_domain_min_tensor), ptr(global_domain_max_tensor),
         ptr(strides_tensor), float(distance_between_points), int(max_samples_per_ray),
         int(max_depth_index), float(min_distance), int(bool(is_initial_query)), ptr(qi),
         ptr(nets), _st(directions_tensor))
    return qi, nets


# ---------------------------------------------------------------- global_to_local.cuh
def global_to_local(points_tensor, domain_mins_tensor, domain_maxs_tensor,
                    batch_size_per_network_tensor, kernel_num_blocks, kernel_num_threads):
    _gpu(points_tensor)
    bspn = _host_i64(batch_size_per_network_tensor)
    call("kn_global_to_local", ptr(points_tensor), ptr(domain_mins_tensor), ptr(domain_maxs_tensor),
         ptr(bspn), bspn.numel(), _st(points_tensor))


# ---------------------------------------------------------------- fourier_features.cuh
def compute_fourier_features(input_tensor, frequency_bands_tensor, kernel_max_num_blocks,
                             kernel_max_num_threads, implementation):
    _gpu(input_tensor, frequency_bands_tensor)
    n = input_tensor.numel()
    L = frequency_bands_tensor.numel()
    out = torch.empty((n * (2 * L + 1),), device=input_tensor.device, dtype=torch.float32)
    x, f = input_tensor.contiguous(), frequency_bands_tensor.contiguous()
    call("kn_compute_fourier_features", ptr(x), n, ptr(f), L, ptr(out), _st(input_tensor))
    return out


# ---------------------------------------------------------------- network_eval.cuh
def network_eval_query_index(query_indices_tensor, params_tensor, domain_mins_tensor,
                             domain_maxs_tensor, starts_tensor, ends_tensor, origin_tensor,
                             c2w_tensor, num_networks, hidden_dim, H, W, cx, cy, fx, fy,
                             max_depth_index, min_distance, distance_between_samples, num_blocks,
                             num_threads, version):
    _gpu(query_indices_tensor, params_tensor)
    b = query_indices_tensor.shape[0]
    out = torch.ones((b, 4), device=params_tensor.device, dtype=torch.float32)
    call("kn_network_eval_query_index", ptr(query_indices_tensor), b, ptr(params_tensor),
         ptr(domain_mins_tensor), ptr(domain_maxs_tensor), ptr(starts_tensor), ptr(ends_tensor),
         ptr(origin_tensor), ptr(c2w_tensor), int(num_networks), int(hidden_dim), int(H), int(W),
         float(cx), float(cy), float(fx), float(fy), int(max_depth_index), float(min_distance),
         float(distance_between_samples), ptr(out), _st(params_tensor))
    return out


# ---------------------------------------------------------------- integrate.cuh
def integrate(rgb_sigma_tensor, dists_tensor, rgb_map, acc_map_tensor, transmittance_tensor,
              active_ray_mask_tensor, num_rays, samples_per_ray, transmittance_threshold,
              is_initial_query, num_blocks, num_threads, version):
    """rgb_map is the int64 device address of a float32 [num_rays, 3] buffer (integrate.cuh:8)."""
    _gpu(rgb_sigma_tensor, dists_tensor, acc_map_tensor)
    call("kn_integrate", ptr(rgb_sigma_tensor), ptr(dists_tensor), int(rgb_map),
         ptr(acc_map_tensor), ptr(transmittance_tensor), ptr(active_ray_mask_tensor),
         int(num_rays), int(samples_per_ray), float(transmittance_threshold),
         int(bool(is_initial_query)), _st(rgb_sigma_tensor))


def replace_transparency_by_background_color(rgb_map_pointer, acc_map_tensor,
                                             background_color_tensor, num_blocks, num_threads):
    """acc_map must be [H, W] (the reference reads size(0)*size(1), integrate.cu:105)."""
    _gpu(acc_map_tensor, background_color_tensor)
    n = acc_map_tensor.size(0) * acc_map_tensor.size(1)
    bg = background_color_tensor.contiguous()
    call("kn_replace_transparency_by_background_color", int(rgb_map_pointer), ptr(acc_map_tensor),
         n, ptr(bg), _st(acc_map_tensor))


# ---------------------------------------------------------------- render_to_screen.h
def render_to_screen(renderer, cam, w, h):
    raise NerfHipError("render_to_screen: OpenGL viewer is not supported on this build")
