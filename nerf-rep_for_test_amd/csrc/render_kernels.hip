// Per-ray stages of the NeRF render path on gfx950 (everything except the MLP).
//
// These kernels are HBM/latency-bound bookkeeping around the MFMA-bound MLP;
// they are written to reproduce the reference's float32 results exactly where
// the reference is deterministic: one rounding per torch op (built with
// -ffp-contract=off, fmaf only where torch's CPU kernel fuses), torch's CPU
// summation orders (common.h), double-accumulated cumprod/cumsum like torch's
// CPU scans. Reference: src/models/nerf/renderer/volume_renderer.py (VR).
#include "common.h"

namespace nerfhip {

// ---------------------------------------------------------------------------
// rays (VR:115-143)
// ---------------------------------------------------------------------------
__global__ void rays_kernel(const float* __restrict__ cam, int W, int64_t p0, int64_t n,
                            float* __restrict__ rays_o, float* __restrict__ rays_d) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t p = p0 + i;
  const float x = (float)(p % W);   // torch.linspace(0, W-1, W) is exact integers
  const float y = (float)(p / W);
  const float* pose = cam;          // 4x4 row-major
  const float* K = cam + 16;        // 3x3 row-major
  const float dx = (x - K[2]) / K[0];
  const float dy = (-(y - K[5])) / K[4];
  const float dz = -1.0f;
  float d[3];
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    // torch.sum(dirs[..., None, :] * R, -1): products, then ((p0+p1)+p2)
    const float a = dx * pose[r * 4 + 0];
    const float b = dy * pose[r * 4 + 1];
    const float c = dz * pose[r * 4 + 2];
    d[r] = (a + b) + c;
  }
  const float nrm = torch_norm3(d[0], d[1], d[2]);
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    rays_d[i * 3 + r] = d[r] / nrm;
    rays_o[i * 3 + r] = pose[r * 4 + 3];
  }
}

// ---------------------------------------------------------------------------
// coarse depths (VR:218-237)
// ---------------------------------------------------------------------------
__device__ __forceinline__ float stratified(const float* zrow, int S, int s, float t) {
  // mids = .5*(z[1:]+z[:-1]); upper = [mids, z[-1]]; lower = [z[0], mids]
  const float up = (s < S - 1) ? 0.5f * (zrow[s + 1] + zrow[s]) : zrow[S - 1];
  const float lo = (s > 0) ? 0.5f * (zrow[s] + zrow[s - 1]) : zrow[0];
  return lo + (up - lo) * t;
}

__global__ void coarse_kernel(const float* __restrict__ z_base, const float* __restrict__ t_rand,
                              int64_t n, int S, float* __restrict__ z) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * S) return;
  const int s = (int)(i % S);
  z[i] = t_rand ? stratified(z_base, S, s, t_rand[i]) : z_base[s];
}

// ---------------------------------------------------------------------------
// compositing (VR:286-357) — one thread per ray
// ---------------------------------------------------------------------------
struct RaySpan {
  const float4* raw;   // [S] (rgb logits, sigma)
  const float* z;      // [S]
  float nd;            // torch.norm(rays_d) of the (already unit) direction
};

__device__ __forceinline__ float dist_at(const RaySpan& r, int S, int s) {
  const float d = (s < S - 1) ? (r.z[s + 1] - r.z[s]) : 1e10f;
  return d * r.nd;
}

__device__ __forceinline__ float alpha_at(const RaySpan& r, int S, int s) {
  const float sig = fmaxf(r.raw[s].w, 0.0f);                   // relu (raw + noise 0)
  return 1.0f - expf((-sig) * dist_at(r, S, s));               // VR:288
}

__device__ __forceinline__ float sigmoid_t(float x) { return 1.0f / (1.0f + expf(-x)); }

__device__ void write_maps(const RaySpan& r, int S, const float* w, int64_t ray, int white,
                           float* rgb, float* disp, float* acc, float* depth) {
  float c[3];
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) {
    c[ch] = tsum_dim2(S, [&](int s) {
      const float4 v = r.raw[s];
      const float x = ch == 0 ? v.x : (ch == 1 ? v.y : v.z);
      return w[s] * sigmoid_t(x);
    });
  }
  const float dep = tsum_last(S, [&](int s) { return w[s] * r.z[s]; });
  const float ac = tsum_last(S, [&](int s) { return w[s]; });
  const float ratio = dep / ac;
  disp[ray] = 1.0f / torch_max(1e-10f, ratio);
  acc[ray] = ac;
  depth[ray] = dep;
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) rgb[ray * 3 + ch] = white ? c[ch] + (1.0f - ac) : c[ch];
}

__global__ void composite_kernel(const float4* __restrict__ raw, const float* __restrict__ z,
                                 int64_t z_stride, const float* __restrict__ rays_d, int64_t n,
                                 int S, int white, float* __restrict__ rgb,
                                 float* __restrict__ disp, float* __restrict__ acc,
                                 float* __restrict__ depth, float* __restrict__ wout) {
  const int64_t ray = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (ray >= n) return;
  RaySpan r;
  r.raw = raw + ray * S;
  r.z = z + ray * z_stride;
  r.nd = torch_norm3(rays_d[ray * 3], rays_d[ray * 3 + 1], rays_d[ray * 3 + 2]);
  float* w = wout + ray * S;
  // w_s = alpha_s * cumprod([1, 1-alpha+1e-10])_s, scan accumulated in double (VR:329)
  double T = 1.0;
  for (int s = 0; s < S; ++s) {
    const float a = alpha_at(r, S, s);
    w[s] = a * (float)T;
    T = T * (double)((1.0f - a) + 1e-10f);
  }
  write_maps(r, S, w, ray, white, rgb, disp, acc, depth);
}

// ERT (VR:1089-1133): T = cumprod(1 - [0, alpha[:-1]]) without the 1e-10; if
// any ray of the 2048-ray chunk has T < thr, every ray's weights are cut from
// argmax(T < thr) on (0 for rays that never cross it). One block per chunk.
__global__ void composite_ert_kernel(const float4* __restrict__ raw, const float* __restrict__ z,
                                     int64_t z_stride, const float* __restrict__ rays_d,
                                     int64_t n, int S, int white, float thr, int chunk,
                                     float* __restrict__ rgb, float* __restrict__ disp,
                                     float* __restrict__ acc, float* __restrict__ depth,
                                     float* __restrict__ wout) {
  __shared__ int any_low;
  if (threadIdx.x == 0) any_low = 0;
  __syncthreads();
  const int64_t c0 = (int64_t)blockIdx.x * chunk;
  const int64_t c1 = c0 + chunk < n ? c0 + chunk : n;
  // pass 1: weights without the cut + first termination index per ray
  for (int64_t ray = c0 + threadIdx.x; ray < c1; ray += blockDim.x) {
    RaySpan r;
    r.raw = raw + ray * S;
    r.z = z + ray * z_stride;
    r.nd = torch_norm3(rays_d[ray * 3], rays_d[ray * 3 + 1], rays_d[ray * 3 + 2]);
    float* w = wout + ray * S;
    double T = 1.0;
    int first = -1;
    for (int s = 0; s < S; ++s) {
      const float a = alpha_at(r, S, s);
      const float Tf = (float)T;
      if (first < 0 && Tf < thr) first = s;
      w[s] = a * Tf;
      T = T * (double)(1.0f - a);
    }
    if (first >= 0) any_low = 1;   // benign race: every writer stores 1
    // stash the termination index in the (otherwise unused) depth slot
    depth[ray] = __int_as_float(first);
  }
  __syncthreads();
  const bool cut = any_low != 0;
  for (int64_t ray = c0 + threadIdx.x; ray < c1; ray += blockDim.x) {
    RaySpan r;
    r.raw = raw + ray * S;
    r.z = z + ray * z_stride;
    r.nd = 0.f;
    float* w = wout + ray * S;
    if (cut) {
      int first = __float_as_int(depth[ray]);
      if (first < 0) first = 0;        // argmax of an all-False row
      for (int s = first; s < S; ++s) w[s] = w[s] * 0.0f;
    }
    write_maps(r, S, w, ray, white, rgb, disp, acc, depth);
  }
}

// ---------------------------------------------------------------------------
// fine sampling (VR:239-268) + merge with the coarse depths (VR:181-183)
// one thread per ray; cdf and bins staged in LDS as [index][thread]
// ---------------------------------------------------------------------------
constexpr int FINE_BLOCK = 64;
constexpr int FINE_MAX_NB = 128;   // S <= 129 coarse samples

__global__ __launch_bounds__(FINE_BLOCK) void sample_fine_kernel(
    const float* __restrict__ z, int64_t z_stride, const float* __restrict__ weights,
    const float* __restrict__ u, int64_t u_stride, int64_t n, int S, int n_imp,
    float* __restrict__ z_all) {
  __shared__ float cdf_s[FINE_MAX_NB * FINE_BLOCK];
  __shared__ float bin_s[FINE_MAX_NB * FINE_BLOCK];
  const int t = threadIdx.x;
  const int64_t ray = (int64_t)blockIdx.x * FINE_BLOCK + t;
  if (ray >= n) return;
  const float* zr = z + ray * z_stride;
  const float* wr = weights + ray * S;
  const int nb = S - 1;       // bins = mids of z (63), cdf has nb entries
  const int nw = S - 2;       // weights[..., 1:-1]
  // pdf normaliser: torch.sum(weights + 1e-5, -1)
  const float tot = tsum_last(nw, [&](int s) { return wr[s + 1] + 1e-5f; });
  double run = 0.0;
  cdf_s[t] = 0.0f;
  for (int s = 0; s < nw; ++s) {
    const float pdf = (wr[s + 1] + 1e-5f) / tot;
    run += (double)pdf;
    cdf_s[(s + 1) * FINE_BLOCK + t] = (float)run;
  }
  for (int s = 0; s < nb; ++s) bin_s[s * FINE_BLOCK + t] = 0.5f * (zr[s + 1] + zr[s]);
  // fine samples are staged in the tail of this ray's output row
  float* out = z_all + ray * (int64_t)(S + n_imp);
  float* zf = out + S;
  const float* ur = u + ray * u_stride;
  for (int j = 0; j < n_imp; ++j) {
    const float uj = ur[j];
    // searchsorted(cdf, u, right=True): number of cdf entries <= u
    int lo = 0, hi = nb;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (cdf_s[mid * FINE_BLOCK + t] <= uj) lo = mid + 1; else hi = mid;
    }
    const int below = lo - 1 > 0 ? lo - 1 : 0;
    const int above = lo < nb - 1 ? lo : nb - 1;
    const float cg0 = cdf_s[below * FINE_BLOCK + t], cg1 = cdf_s[above * FINE_BLOCK + t];
    const float bg0 = bin_s[below * FINE_BLOCK + t], bg1 = bin_s[above * FINE_BLOCK + t];
    float denom = cg1 - cg0;
    denom = denom < 1e-5f ? 1.0f : denom;
    const float tt = (uj - cg0) / denom;
    zf[j] = bg0 + tt * (bg1 - bg0);
  }
  // torch.sort(cat(z, zf)) (values only): insertion-sort zf (already ascending
  // in eval mode), then merge it with the ascending coarse row front to back,
  // in place: while coarse values remain (a < S) the write index a+b stays
  // below the first unread fine sample at S+b; once they are exhausted the
  // remaining fine samples already sit at their final positions.
  for (int j = 1; j < n_imp; ++j) {
    const float v = zf[j];
    int k = j - 1;
    while (k >= 0 && zf[k] > v) { zf[k + 1] = zf[k]; --k; }
    zf[k + 1] = v;
  }
  int a = 0, b = 0;
  while (a < S && b < n_imp) {
    const float za = zr[a], zb = zf[b];
    if (zb < za) { out[a + b] = zb; ++b; } else { out[a + b] = za; ++a; }
  }
  while (a < S) { out[a + b] = zr[a]; ++a; }
}

// ---------------------------------------------------------------------------
// ESS (VR:1009-1087): one block of 64 lanes per chunk; lane = sample index
// ---------------------------------------------------------------------------
__device__ __forceinline__ int grid_coord(float p, int res) {
  // long(clamp((p - (-2)) / (2 - (-2)), 0, 1) * (res - 1)), clamped
  float v = (p - (-2.0f)) / (2.0f - (-2.0f));
  v = v < 0.0f ? 0.0f : (v > 1.0f ? 1.0f : v);
  int c = (int)(v * (float)(res - 1));
  return c < 0 ? 0 : (c > res - 1 ? res - 1 : c);
}

__device__ __forceinline__ float wave_min(float v) {
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

// ascending bitonic sort of one value per lane across the 64-lane wave
__device__ __forceinline__ float wave_sort64(float v, int lane) {
  for (int k = 2; k <= 64; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      const float o = __shfl_xor(v, j);
      const bool up = ((lane & k) == 0);
      const bool lower = ((lane & j) == 0);
      const float mn = fminf(v, o), mx = fmaxf(v, o);
      v = (lower == up) ? mn : mx;
    }
  }
  return v;
}

__global__ __launch_bounds__(64) void ess_kernel(
    const float* __restrict__ rays_o, const float* __restrict__ rays_d,
    const uint8_t* __restrict__ grid, int res, const float* __restrict__ z_base,
    const float* __restrict__ t_rand, int64_t n, int S, int chunk, float skip_thr,
    float* __restrict__ z) {
  const int lane = threadIdx.x;
  const int64_t c0 = (int64_t)blockIdx.x * chunk;
  const int64_t c1 = c0 + chunk < n ? c0 + chunk : n;
  const bool act = lane < S;
  const float PAD = __builtin_inff();
  float row = act ? z_base[lane] : PAD;   // the shared (expand-ed) row
  const float zorig = row;
  for (int64_t ray = c0; ray < c1; ++ray) {
    // emptiness of the ORIGINAL sample positions (VR:1027-1030)
    bool empty = false;
    if (act) {
      const float px = rays_o[ray * 3 + 0] + rays_d[ray * 3 + 0] * zorig;
      const float py = rays_o[ray * 3 + 1] + rays_d[ray * 3 + 1] * zorig;
      const float pz = rays_o[ray * 3 + 2] + rays_d[ray * 3 + 2] * zorig;
      const int gx = grid_coord(px, res), gy = grid_coord(py, res), gz = grid_coord(pz, res);
      empty = grid[((int64_t)gx * res + gy) * res + gz] == 0;
    }
    const uint64_t emask = __ballot(act && empty);
    const int n_empty = __popcll(emask);
    const float ratio = (float)n_empty / (float)S;     // exact (count / S)
    if (!(ratio > skip_thr)) continue;
    const int n_keep = S - n_empty;
    if (n_keep == 0) continue;
    const bool keep = act && !empty;
    const float kept = keep ? row : PAD;
    const float mn = wave_min(kept);
    const float mx = wave_max(keep ? row : -PAD);
    // stable compaction of kept values (in sample order) ...
    const uint64_t kmask = __ballot(keep);
    const int pos = __popcll(kmask & ((1ull << lane) - 1ull));
    // ... then torch.linspace(mn, mx, n_add) (CPU float32: one fma per element)
    const int n_add = S - n_keep;
    float v = PAD;
    const int ai = lane - n_keep;   // index into the added values for lane >= n_keep
    if (act && lane >= n_keep) {
      if (n_add == 1) {
        v = mn;
      } else {
        const float step = (mx - mn) / (float)(n_add - 1);
        const int half = n_add / 2;
        v = ai < half ? __builtin_fmaf(step, (float)ai, mn)
                      : __builtin_fmaf(-step, (float)(n_add - ai - 1), mx);
      }
    }
    // gather the compacted kept values into lanes [0, n_keep)
    const int src_lane = keep ? pos : -1;
    // lane L < n_keep receives the kept value whose pos == L: scatter via LDS
    __shared__ float tmp[64];
    if (keep) tmp[pos] = row;
    __syncthreads();
    if (lane < n_keep) v = tmp[lane];
    __syncthreads();
    (void)src_lane;
    row = wave_sort64(v, lane);
  }
  // per-ray rows (+ stratification, VR:1080-1085)
  __shared__ float srow[64];
  srow[lane] = row;
  __syncthreads();
  for (int64_t ray = c0; ray < c1; ++ray) {
    if (act) {
      const int64_t idx = ray * S + lane;
      z[idx] = t_rand ? stratified(srow, S, lane, t_rand[idx]) : srow[lane];
    }
  }
}

// occupancy-grid self-update (VR:1147-1155, VR:963-990)
__global__ void grid_update_kernel(const float* __restrict__ rays_d, const float* __restrict__ z,
                                   int64_t z_stride, const float4* __restrict__ raw,
                                   const float* __restrict__ w, int64_t n, int S,
                                   uint8_t* __restrict__ grid, int res) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * S) return;
  const int64_t ray = i / S;
  const int s = (int)(i % S);
  if (!(w[i] > 1e-4f)) return;
  if (!(fmaxf(raw[i].w, 0.0f) > 0.01f)) return;
  const float zz = z[ray * z_stride + s];
  const int gx = grid_coord(rays_d[ray * 3 + 0] * zz, res);
  const int gy = grid_coord(rays_d[ray * 3 + 1] * zz, res);
  const int gz = grid_coord(rays_d[ray * 3 + 2] * zz, res);
  grid[((int64_t)gx * res + gy) * res + gz] = 1;
}

}  // namespace nerfhip

using namespace nerfhip;

extern "C" {

int nerf_rays(const float* cam, int H, int W, int64_t p0, int64_t n, float* rays_o,
              float* rays_d, nerf_stream_t stream) {
  NERF_REQUIRE(cam && rays_o && rays_d, "nerf_rays: null pointer");
  NERF_REQUIRE(H > 0 && W > 0 && p0 >= 0 && n >= 0 && p0 + n <= (int64_t)H * W,
               "nerf_rays: pixel range outside the image");
  if (n == 0) return 0;
  hipLaunchKernelGGL(rays_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, as_stream(stream),
                     cam, W, p0, n, rays_o, rays_d);
  return check_launch("rays_kernel");
}

int nerf_sample_coarse(const float* z_base, const float* t_rand, int64_t n, int S, float* z,
                       nerf_stream_t stream) {
  NERF_REQUIRE(z_base && z, "nerf_sample_coarse: null pointer");
  NERF_REQUIRE(n >= 0 && S >= 1, "nerf_sample_coarse: bad size");
  if (n == 0) return 0;
  hipLaunchKernelGGL(coarse_kernel, dim3((unsigned)cdiv(n * S, 256)), dim3(256), 0,
                     as_stream(stream), z_base, t_rand, n, S, z);
  return check_launch("coarse_kernel");
}

int nerf_composite(const float* raw, const float* z, int64_t z_stride, const float* rays_d,
                   int64_t n, int S, int white_bkgd, float* rgb, float* disp, float* acc,
                   float* depth, float* weights, nerf_stream_t stream) {
  NERF_REQUIRE(raw && z && rays_d && rgb && disp && acc && depth && weights,
               "nerf_composite: null pointer (weights scratch is required)");
  NERF_REQUIRE(n >= 0 && S >= 2 && S < 1024, "nerf_composite: S must be in [2, 1024)");
  if (n == 0) return 0;
  hipLaunchKernelGGL(composite_kernel, dim3((unsigned)cdiv(n, 128)), dim3(128), 0,
                     as_stream(stream), (const float4*)raw, z, z_stride, rays_d, n, S,
                     white_bkgd, rgb, disp, acc, depth, weights);
  return check_launch("composite_kernel");
}

int nerf_composite_ert(const float* raw, const float* z, int64_t z_stride, const float* rays_d,
                       int64_t n, int S, int white_bkgd, float threshold, int chunk, float* rgb,
                       float* disp, float* acc, float* depth, float* weights,
                       nerf_stream_t stream) {
  NERF_REQUIRE(raw && z && rays_d && rgb && disp && acc && depth && weights,
               "nerf_composite_ert: null pointer (weights scratch is required)");
  NERF_REQUIRE(n >= 0 && S >= 2 && S < 1024 && chunk > 0, "nerf_composite_ert: bad size");
  if (n == 0) return 0;
  hipLaunchKernelGGL(composite_ert_kernel, dim3((unsigned)cdiv(n, chunk)), dim3(256), 0,
                     as_stream(stream), (const float4*)raw, z, z_stride, rays_d, n, S,
                     white_bkgd, threshold, chunk, rgb, disp, acc, depth, weights);
  return check_launch("composite_ert_kernel");
}

int nerf_sample_fine(const float* z, int64_t z_stride, const float* weights, const float* u,
                     int64_t u_stride, int64_t n, int S, int n_imp, float* z_all,
                     nerf_stream_t stream) {
  NERF_REQUIRE(z && weights && u && z_all, "nerf_sample_fine: null pointer");
  NERF_REQUIRE(n >= 0 && S >= 3 && S - 1 <= FINE_MAX_NB && n_imp >= 1,
               "nerf_sample_fine: need 3 <= S <= 129 coarse samples and n_imp >= 1");
  if (n == 0) return 0;
  hipLaunchKernelGGL(sample_fine_kernel, dim3((unsigned)cdiv(n, FINE_BLOCK)), dim3(FINE_BLOCK), 0,
                     as_stream(stream), z, z_stride, weights, u, u_stride, n, S, n_imp, z_all);
  return check_launch("sample_fine_kernel");
}

int nerf_sample_coarse_ess(const float* rays_o, const float* rays_d, const uint8_t* grid,
                           int res, const float* z_base, const float* t_rand, int64_t n, int S,
                           int chunk, float skip_threshold, float* z, nerf_stream_t stream) {
  NERF_REQUIRE(rays_o && rays_d && grid && z_base && z, "nerf_sample_coarse_ess: null pointer");
  NERF_REQUIRE(n >= 0 && S >= 2 && S <= 64 && chunk > 0 && res >= 2,
               "nerf_sample_coarse_ess: need 2 <= S <= 64");
  if (n == 0) return 0;
  hipLaunchKernelGGL(ess_kernel, dim3((unsigned)cdiv(n, chunk)), dim3(64), 0, as_stream(stream),
                     rays_o, rays_d, grid, res, z_base, t_rand, n, S, chunk, skip_threshold, z);
  return check_launch("ess_kernel");
}

int nerf_grid_update(const float* rays_d, const float* z, int64_t z_stride, const float* raw,
                     const float* weights, int64_t n, int S, uint8_t* grid, int res,
                     nerf_stream_t stream) {
  NERF_REQUIRE(rays_d && z && raw && weights && grid, "nerf_grid_update: null pointer");
  NERF_REQUIRE(n >= 0 && S >= 1 && res >= 2, "nerf_grid_update: bad size");
  if (n == 0) return 0;
  hipLaunchKernelGGL(grid_update_kernel, dim3((unsigned)cdiv(n * S, 256)), dim3(256), 0,
                     as_stream(stream), rays_d, z, z_stride, (const float4*)raw, weights, n, S,
                     grid, res);
  return check_launch("grid_update_kernel");
}

}  // extern "C"
