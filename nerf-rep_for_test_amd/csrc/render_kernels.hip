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
// compositing (VR:286-357) — one wave per ray, lanes over samples
//
// Per 64-sample block: one coalesced float4 raw load + z[s], z[s+1] per lane,
// alpha, an in-wave double-precision product scan for the transmittance
// (torch's CPU cumprod accumulates float in double, VR:329), w = alpha * T.
// The map sums are wave reductions (a different addition order than torch's
// CPU sum: differences are at the 1e-7 level, well inside the 1e-5 contract;
// the weights themselves, which feed _sample_fine, are elementwise).
// ---------------------------------------------------------------------------
__device__ __forceinline__ float sigmoid_t(float x) { return 1.0f / (1.0f + expf(-x)); }

__device__ __forceinline__ float wave_sum(float v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ double wave_prod_scan(double p, int lane) {   // inclusive
  for (int o = 1; o < 64; o <<= 1) {
    const double q = __shfl_up(p, o);
    if (lane >= o) p *= q;
  }
  return p;
}

struct Maps {
  float r, g, b, d, a;   // sum w*rgb, sum w*z, sum w
};

__device__ __forceinline__ void maps_add(Maps& m, float w, const float4& v, float z) {
  m.r += w * sigmoid_t(v.x);
  m.g += w * sigmoid_t(v.y);
  m.b += w * sigmoid_t(v.z);
  m.d += w * z;
  m.a += w;
}

// sigmoid on the hardware exp2 / reciprocal (each ~1 ulp): the colour maps move
// by < 4e-7, inside the 1e-6 the kernels are tested to; alpha and the weights,
// which feed _sample_fine's searchsorted, keep the accurate expf
__device__ __forceinline__ float sigmoid_fast(float x) {
  return __builtin_amdgcn_rcpf(1.0f + __expf(-x));
}
__device__ __forceinline__ void maps_add_fast(Maps& m, float w, const float4& v, float z) {
  m.r += w * sigmoid_fast(v.x);
  m.g += w * sigmoid_fast(v.y);
  m.b += w * sigmoid_fast(v.z);
  m.d += w * z;
  m.a += w;
}

__device__ __forceinline__ Maps maps_reduce(Maps m) {
  return Maps{wave_sum(m.r), wave_sum(m.g), wave_sum(m.b), wave_sum(m.d), wave_sum(m.a)};
}

// VR:331-334, 353-354: disp = 1/max(1e-10, depth/acc), white background.
__device__ __forceinline__ void maps_store(const Maps& m, int64_t ray, int white, float* rgb,
                                           float* disp, float* acc, float* depth) {
  disp[ray] = 1.0f / torch_max(1e-10f, m.d / m.a);
  acc[ray] = m.a;
  depth[ray] = m.d;
  const float bg = white ? 1.0f - m.a : 0.0f;
  rgb[ray * 3 + 0] = white ? m.r + bg : m.r;
  rgb[ray * 3 + 1] = white ? m.g + bg : m.g;
  rgb[ray * 3 + 2] = white ? m.b + bg : m.b;
}

// One ray by one wave. ERT: T without the +1e-10 (VR:1109-1111); `first` = the
// first s with T_s < thr or -1, and `cut` = the sums with w[first:] * 0
// (VR:1115-1123), valid when first >= 0.
template <bool ERT>
__device__ __forceinline__ void composite_ray(const float4* __restrict__ rr,
                                              const float* __restrict__ zr, float nd, int S,
                                              int lane, float thr, float* __restrict__ w_out,
                                              Maps& full, Maps& cut, int& first) {
  full = Maps{0, 0, 0, 0, 0};
  cut = Maps{0, 0, 0, 0, 0};
  first = -1;
  double carry = 1.0;
  for (int b = 0; b < S; b += 64) {
    const int s = b + lane;
    const bool act = s < S;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    float zs = 0.f, a = 0.f;
    if (act) {
      v = rr[s];
      zs = zr[s];
      const float dist = ((s < S - 1) ? (zr[s + 1] - zs) : 1e10f) * nd;   // VR:290-292
      a = 1.0f - expf((-fmaxf(v.w, 0.0f)) * dist);                       // VR:288
    }
    const double f = act ? (double)(ERT ? (1.0f - a) : ((1.0f - a) + 1e-10f)) : 1.0;
    const double inc = wave_prod_scan(f, lane);
    double ex = __shfl_up(inc, 1);
    if (lane == 0) ex = 1.0;
    const float T = (float)(carry * ex);
    carry = carry * __shfl(inc, 63);
    const float w = a * T;
    if (act) {
      if (w_out) w_out[s] = w;
      maps_add(full, w, v, zs);
    }
    if constexpr (ERT) {
      const uint64_t low = __ballot(act && T < thr);
      if (first < 0 && low) first = b + (int)__builtin_ctzll(low);
      if (act) maps_add(cut, (first < 0 || s < first) ? w : w * 0.0f, v, zs);
    }
  }
  full = maps_reduce(full);
  if constexpr (ERT) cut = maps_reduce(cut);
}

constexpr int COMP_WAVES = 4;

__global__ __launch_bounds__(64 * COMP_WAVES) void composite_kernel(
    const float4* __restrict__ raw, const float* __restrict__ z, int64_t z_stride,
    const float* __restrict__ rays_d, int64_t n, int S, int white, float* __restrict__ rgb,
    float* __restrict__ disp, float* __restrict__ acc, float* __restrict__ depth,
    float* __restrict__ wout) {
  const int lane = threadIdx.x & 63;
  const int64_t ray = (int64_t)blockIdx.x * COMP_WAVES + (threadIdx.x >> 6);
  if (ray >= n) return;   // wave-uniform
  const float nd = torch_norm3(rays_d[ray * 3], rays_d[ray * 3 + 1], rays_d[ray * 3 + 2]);
  Maps full, cut;
  int first;
  composite_ray<false>(raw + ray * S, z + ray * z_stride, nd, S, lane, 0.f,
                       wout ? wout + ray * S : nullptr, full, cut, first);
  if (lane == 0) maps_store(full, ray, white, rgb, disp, acc, depth);
}

// 16 lanes per ray, 4 rays per wave (S <= 256): lane t holds samples t + 16k,
// k < C, so every load instruction reads 16 consecutive float4 of each of 4
// rays. The transmittance is C interleaved 16-lane product scans in double
// (one per row of 16 consecutive samples, independent, so their shuffles are
// in flight together), each row then scaled by the product of the rows before
// it; the map sums are per-lane then a 16-lane butterfly. No LDS.
constexpr int COMP16_RPB = 16;   // rays per 256-thread block

// ERT (VR:1089-1133) in the same layout, pass 1 of 2: T is the exclusive
// product of (1 - alpha) WITHOUT the +1e-10 (VR:1109-1111); every ray writes
// its uncut maps to the outputs (and its weights), its cut maps -- weights
// zeroed from `first`, the first sample with T < thr, or from 0 when no sample
// crosses it (the argmax of an all-False row, VR:1115-1123) -- and `first` to
// the workspace, and marks its 2048-ray chunk when it crosses the threshold.
// Pass 2 (ert_fixup_kernel) applies the cut maps in the marked chunks.
struct ErtCut {
  Maps m;
  int first;
};

template <int C, bool ERT = false>
__global__ __launch_bounds__(256) void composite16_kernel(
    const float4* __restrict__ raw, const float* __restrict__ z, int64_t z_stride,
    const float* __restrict__ rays_d, int64_t n, int S, int white, float* __restrict__ rgb,
    float* __restrict__ disp, float* __restrict__ acc, float* __restrict__ depth,
    float* __restrict__ wout, float thr = 0.0f, int chunk = 1, ErtCut* __restrict__ cuts = nullptr,
    int* __restrict__ flags = nullptr) {
  const int lane = threadIdx.x & 63, t = lane & 15;
  const int64_t ray0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 4;
  if (ray0 >= n) return;   // wave-uniform
  const int64_t ray = ray0 + (lane >> 4);
  const bool live = ray < n;          // rays past n (last wave) recompute ray n-1, store nothing
  const int64_t rr = live ? ray : n - 1;
  const float nd = torch_norm3(rays_d[rr * 3], rays_d[rr * 3 + 1], rays_d[rr * 3 + 2]);
  const float4* rp = raw + rr * S;
  const float* zr = z + rr * z_stride;
  float4 v[C];
  float zs[C], zn[C];
#pragma unroll
  for (int k = 0; k < C; ++k) {
    const int s = t + 16 * k;
    v[k] = s < S ? rp[s] : make_float4(0.f, 0.f, 0.f, 0.f);
    zs[k] = s < S ? zr[s] : 0.0f;
    zn[k] = s + 1 < S ? zr[s + 1] : 0.0f;
  }
  float a[C];
  double p[C];
#pragma unroll
  for (int k = 0; k < C; ++k) {
    const int s = t + 16 * k;
    const float dist = ((s < S - 1) ? (zn[k] - zs[k]) : 1e10f) * nd;   // VR:290-292
    a[k] = s < S ? 1.0f - expf((-fmaxf(v[k].w, 0.0f)) * dist) : 0.0f;   // VR:288
    if constexpr (ERT) p[k] = s < S ? (double)(1.0f - a[k]) : 1.0;
    else p[k] = s < S ? (double)((1.0f - a[k]) + 1e-10f) : 1.0;
  }
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) {
    double q[C];
#pragma unroll
    for (int k = 0; k < C; ++k) q[k] = __shfl_up(p[k], o, 16);
#pragma unroll
    for (int k = 0; k < C; ++k)
      if (t >= o) p[k] *= q[k];
  }
  double ex[C], tot[C];
#pragma unroll
  for (int k = 0; k < C; ++k) {
    ex[k] = __shfl_up(p[k], 1, 16);
    tot[k] = __shfl(p[k], (lane & ~15) | 15);
  }
  Maps m{0, 0, 0, 0, 0};
  double carry = 1.0;
  if constexpr (!ERT) {
#pragma unroll
    for (int k = 0; k < C; ++k) {
      const int s = t + 16 * k;
      const float T = (float)(carry * (t == 0 ? 1.0 : ex[k]));
      carry = carry * tot[k];
      const float w = a[k] * T;
      if (s < S) {
        if (wout && live) wout[rr * S + s] = w;
        maps_add_fast(m, w, v[k], zs[k]);
      }
    }
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) {
      m.r += __shfl_xor(m.r, o, 16);
      m.g += __shfl_xor(m.g, o, 16);
      m.b += __shfl_xor(m.b, o, 16);
      m.d += __shfl_xor(m.d, o, 16);
      m.a += __shfl_xor(m.a, o, 16);
    }
    if (t == 0 && live) maps_store(m, ray, white, rgb, disp, acc, depth);
  } else {
    float w[C];
    int first = 1 << 30;   // this lane's first sample with T < thr
#pragma unroll
    for (int k = 0; k < C; ++k) {
      const int s = t + 16 * k;
      const float T = (float)(carry * (t == 0 ? 1.0 : ex[k]));
      carry = carry * tot[k];
      w[k] = a[k] * T;
      if (s < S && T < thr && first > s) first = s;
    }
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) first = min(first, __shfl_xor(first, o, 16));
    const bool low = first < S;
    const int f0 = low ? first : 0;   // argmax of an all-False row: 0 (quirk 1)
    Maps c{0, 0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < C; ++k) {
      const int s = t + 16 * k;
      if (s < S) {
        if (wout && live) wout[rr * S + s] = w[k];
        maps_add(m, w[k], v[k], zs[k]);
        maps_add(c, s < f0 ? w[k] : w[k] * 0.0f, v[k], zs[k]);
      }
    }
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) {
      m.r += __shfl_xor(m.r, o, 16);
      m.g += __shfl_xor(m.g, o, 16);
      m.b += __shfl_xor(m.b, o, 16);
      m.d += __shfl_xor(m.d, o, 16);
      m.a += __shfl_xor(m.a, o, 16);
      c.r += __shfl_xor(c.r, o, 16);
      c.g += __shfl_xor(c.g, o, 16);
      c.b += __shfl_xor(c.b, o, 16);
      c.d += __shfl_xor(c.d, o, 16);
      c.a += __shfl_xor(c.a, o, 16);
    }
    if (t == 0 && live) {
      maps_store(m, ray, white, rgb, disp, acc, depth);
      cuts[ray] = ErtCut{c, f0};
      if (low) flags[ray / chunk] = 1;   // benign race: every writer stores 1
    }
  }
}

// ERT pass 2: in every chunk where some ray crossed the threshold, each ray
// takes its cut maps and its weights from `first` on become w * 0 (VR:1115-1123).
// 16 lanes per ray.
__global__ __launch_bounds__(256) void ert_fixup_kernel(const ErtCut* __restrict__ cuts,
                                                        const int* __restrict__ flags, int64_t n,
                                                        int S, int chunk, int white,
                                                        float* __restrict__ rgb,
                                                        float* __restrict__ disp,
                                                        float* __restrict__ acc,
                                                        float* __restrict__ depth,
                                                        float* __restrict__ wout) {
  const int64_t ray = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 4;
  const int t = threadIdx.x & 15;
  if (ray >= n || !flags[ray / chunk]) return;
  const ErtCut c = cuts[ray];
  if (t == 0) maps_store(c.m, ray, white, rgb, disp, acc, depth);
  if (wout)
    for (int s = c.first + t; s < S; s += 16) wout[ray * S + s] = wout[ray * S + s] * 0.0f;
}

// ERT (VR:1089-1133): if any ray of the 2048-ray chunk has T < thr, every ray's
// weights are cut from argmax(T < thr) on (0 for rays that never cross it, so
// they composite to nothing). One block per chunk: the uncut maps go straight
// to the outputs, the cut ones wait in LDS for the chunk-wide decision.
constexpr int ERT_WAVES = 8;
constexpr int ERT_MAX_CHUNK = 2048;

__global__ __launch_bounds__(64 * ERT_WAVES) void composite_ert_kernel(
    const float4* __restrict__ raw, const float* __restrict__ z, int64_t z_stride,
    const float* __restrict__ rays_d, int64_t n, int S, int white, float thr, int chunk,
    float* __restrict__ rgb, float* __restrict__ disp, float* __restrict__ acc,
    float* __restrict__ depth, float* __restrict__ wout) {
  __shared__ Maps cut_s[ERT_MAX_CHUNK];
  __shared__ int first_s[ERT_MAX_CHUNK];
  __shared__ int any_low;
  if (threadIdx.x == 0) any_low = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int64_t c0 = (int64_t)blockIdx.x * chunk;
  const int nr = (int)((c0 + chunk < n ? c0 + chunk : n) - c0);
  for (int i = wave; i < nr; i += ERT_WAVES) {
    const int64_t ray = c0 + i;
    const float nd = torch_norm3(rays_d[ray * 3], rays_d[ray * 3 + 1], rays_d[ray * 3 + 2]);
    Maps full, cut;
    int first;
    composite_ray<true>(raw + ray * S, z + ray * z_stride, nd, S, lane, thr,
                        wout ? wout + ray * S : nullptr, full, cut, first);
    if (lane == 0) {
      maps_store(full, ray, white, rgb, disp, acc, depth);
      cut_s[i] = first >= 0 ? cut : Maps{0, 0, 0, 0, 0};
      first_s[i] = first >= 0 ? first : 0;          // argmax of an all-False row
      if (first >= 0) any_low = 1;                 // benign race: every writer stores 1
    }
  }
  __syncthreads();
  if (!any_low) return;
  for (int i = wave; i < nr; i += ERT_WAVES) {
    const int64_t ray = c0 + i;
    const int f0 = first_s[i];
    if (lane == 0) maps_store(cut_s[i], ray, white, rgb, disp, acc, depth);
    if (wout)
      for (int s = f0 + lane; s < S; s += 64) wout[ray * S + s] = wout[ray * S + s] * 0.0f;
  }
}

// ---------------------------------------------------------------------------
// ERT sample compaction (C4): the MLP of a pass with ERT runs over depth
// segments [s0, s1) of the sorted samples; after each, every ray still active
// carries its exclusive transmittance T over the segment (the composite's own
// alpha, VR:1091-1111) and is retired once T < thr (1 - 1e-6): every sample
// from there on is at or after the ray's first low-transmittance sample, whose
// weight the ERT composite zeroes in any chunk that cuts at all (and this ray
// makes its chunk cut), so its raw is never read. Active rays append the flat
// indices of their next segment [s1, s2) to the list the MLP reads next. The
// margin makes the retirement conservative against the composite's other
// product order (double accumulation both: ~1e-16 relative). One thread per
// ray; one atomic per wave for the list slots.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void ert_segment_kernel(
    const float4* __restrict__ raw, const float* __restrict__ z, int64_t z_stride,
    const float* __restrict__ rays_d, int64_t n, int S, int s0, int s1, int s2, float thr,
    double* __restrict__ T, unsigned char* __restrict__ active, int* __restrict__ list,
    int* __restrict__ count) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  int want = 0;
  if (r < n && active[r]) {
    double t = T[r];
    if (s1 > s0) {
      const float* zr = z + r * z_stride;
      const float nd = torch_norm3(rays_d[r * 3], rays_d[r * 3 + 1], rays_d[r * 3 + 2]);
      for (int s = s0; s < s1; ++s) {
        const float dist = ((s < S - 1) ? (zr[s + 1] - zr[s]) : 1e10f) * nd;
        const float a = 1.0f - expf((-fmaxf(raw[r * S + s].w, 0.0f)) * dist);
        t = t * (double)(1.0f - a);
      }
      T[r] = t;
    }
    if (t < (double)thr * (1.0 - 1e-6)) active[r] = 0;
    else want = s2 - s1;
  }
  // wave-aggregated slot allocation: exclusive prefix of `want`, one atomic
  int incl = want;
  for (int o = 1; o < 64; o <<= 1) {
    const int q = __shfl_up(incl, o);
    if (lane >= o) incl += q;
  }
  const int total = __shfl(incl, 63);
  int base = 0;
  if (lane == 63 && total > 0) base = atomicAdd(count, total);
  base = __shfl(base, 63);
  const int off = base + incl - want;
  for (int k = 0; k < want; ++k) list[off + k] = (int)(r * S + s1 + k);
}

// ---------------------------------------------------------------------------
// fine sampling (VR:239-268) + merge with the coarse depths (VR:181-183)
// 16 lanes per ray (4 rays per wave, 16 per block), so that four times the rays
// of a one-wave-per-ray layout are in flight: the kernel is a chain of short
// dependent LDS steps per ray, latency- not bandwidth-bound. Each lane carries
// its ray's searches together through a fixed-step (branch-free) binary
// search, so a search costs ~log2(S) LDS latencies for all of them.
// Per-ray LDS row (dynamic): zc[S] | cdf[S] | zf[max(p2, S - 2)] (+ padding),
// the weights (+1e-5) staged in the zf slot until the cdf is built.
// ---------------------------------------------------------------------------
constexpr int FINE_LANES = 16;                    // lanes per ray
constexpr int FINE_RPW = 64 / FINE_LANES;         // rays per wave
constexpr int FINE_WAVES = 4;
constexpr int FINE_RPB = FINE_RPW * FINE_WAVES;   // rays per block
constexpr int FINE_MAX_S = 130;                   // coarse samples per ray
constexpr int FINE_MAX_IMP = 256;                 // fine samples per ray

__host__ __device__ __forceinline__ int fine_p2(int n_imp) {
  int p2 = FINE_LANES;
  while (p2 < n_imp) p2 <<= 1;
  return p2;
}

// Q searches per lane over the ascending a[0..n) (n >= 1): pos[q] =
// #{a[i] <= x[q]} (UPPER, searchsorted right=True) or #{a[i] < x[q]}.
// Branch-free halving (the window [base, base + len) always holds the answer's
// boundary and never leaves a[0..n)): the step count depends on n only, and
// every step issues all the lane's LDS reads before any is consumed.
template <bool UPPER, int Q>
__device__ __forceinline__ void fine_search(const float* a, int n, const float (&x)[Q],
                                            int (&pos)[Q]) {
#pragma unroll
  for (int q = 0; q < Q; ++q) pos[q] = 0;
  int len = n;
  while (len > 1) {
    const int half = len >> 1;
    float v[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) v[q] = a[pos[q] + half - 1];
#pragma unroll
    for (int q = 0; q < Q; ++q)
      if (UPPER ? v[q] <= x[q] : v[q] < x[q]) pos[q] += half;
    len -= half;
  }
  float v[Q];
#pragma unroll
  for (int q = 0; q < Q; ++q) v[q] = a[pos[q] + len - 1];
#pragma unroll
  for (int q = 0; q < Q; ++q)
    if (UPPER ? v[q] <= x[q] : v[q] < x[q]) pos[q] += len;
}

// torch.sum(x, -1) in ATen's order (common.h tsum_last) by a 16-lane group:
// lane t < 8 folds vector lane t's four accumulators; the scalar tail and the
// in-order combination are evaluated redundantly by every lane of the group.
__device__ __forceinline__ float group_tsum_last(const float* v, int n, int lane) {
  if (n < 8) return tsum_last(n, [&](int i) { return v[i]; });
  const int nv = n >> 3, nilp = nv >> 2, l = lane & 7;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  for (int ii = 0; ii < nilp; ++ii) {
    const int b = ii * 32 + l;
    a0 = a0 + v[b];
    a1 = a1 + v[b + 8];
    a2 = a2 + v[b + 16];
    a3 = a3 + v[b + 24];
  }
  for (int q = nilp * 4; q < nv; ++q) a0 = a0 + v[q * 8 + l];
  const float part = ((a0 + a1) + a2) + a3;
  float fin = 0.f;
  for (int k = nv * 8; k < n; ++k) fin = fin + v[k];
  const int base = lane & ~(FINE_LANES - 1);
#pragma unroll
  for (int q = 0; q < 8; ++q) fin = fin + __shfl(part, base + q);
  return fin;
}

// QN / CN: fine / coarse samples per lane the instance is unrolled for
// (>= ceil(n_imp / 16), ceil(S / 16)); the launcher picks the smallest.
template <int QN, int CN>
__global__ __launch_bounds__(64 * FINE_WAVES) void sample_fine_kernel(
    const float* __restrict__ z, int64_t z_stride, const float* __restrict__ weights,
    const float* __restrict__ u, int64_t u_stride, int64_t n, int S, int n_imp, int row_len,
    float* __restrict__ z_all) {
  extern __shared__ float fine_sm[];
  const int lane = threadIdx.x & 63;
  const int t = lane & (FINE_LANES - 1);
  const int row = threadIdx.x / FINE_LANES;   // ray within the block
  const int64_t wave_ray0 = ((int64_t)blockIdx.x * FINE_WAVES + (threadIdx.x >> 6)) * FINE_RPW;
  if (wave_ray0 >= n) return;   // wave-uniform; no block barriers below
  const int64_t ray = wave_ray0 + (lane / FINE_LANES);
  const bool live = ray < n;    // rays past n (last wave only) run on dummy data
  const int nb = S - 1;         // bins = mids of z; the cdf has nb entries
  const int nw = S - 2;         // weights[..., 1:-1]
  const int p2 = fine_p2(n_imp);
  float* zc = fine_sm + (size_t)row * row_len;
  float* cdf = zc + S;
  float* zf = cdf + S;          // also the staged weights (wv) until the cdf is built
  const float* zr = z + (live ? ray : 0) * z_stride;
  const float* wr = weights + (live ? ray : 0) * S;
  for (int s = t; s < S; s += FINE_LANES) zc[s] = live ? zr[s] : (float)s;
  for (int s = t; s < nw; s += FINE_LANES) zf[s] = (live ? wr[s + 1] : 0.0f) + 1e-5f;
  __builtin_amdgcn_wave_barrier();
  // pdf = w / torch.sum(w, -1); cdf = [0, cumsum(pdf)] accumulated in double
  // (exact in any order: every pdf is a float in (2^-24, 1], the sums < 2)
  const float tot = group_tsum_last(zf, nw, lane);
  const int pc = (nw + FINE_LANES - 1) / FINE_LANES;   // weights per lane, contiguous
  const int s0 = t * pc;
  double pdf[CN];
  double own = 0.0;
#pragma unroll
  for (int k = 0; k < CN; ++k) {
    const int s = s0 + k;
    pdf[k] = (k < pc && s < nw) ? (double)(zf[s] / tot) : 0.0;
    own += pdf[k];
  }
  double incl = own;
#pragma unroll
  for (int o = 1; o < FINE_LANES; o <<= 1) {
    const double q = __shfl_up(incl, o, FINE_LANES);
    if (t >= o) incl += q;
  }
  double run = incl - own;   // exact (see above)
  __builtin_amdgcn_wave_barrier();
  if (t == 0) cdf[0] = 0.0f;
#pragma unroll
  for (int k = 0; k < CN; ++k) {
    const int s = s0 + k;
    run += pdf[k];
    if (k < pc && s < nw) cdf[s + 1] = (float)run;
  }
  __builtin_amdgcn_wave_barrier();
  // inverse CDF (searchsorted right=True, clamp, lerp; VR:254-266); fine sample
  // j = t + 16 q of this lane
  const float* ur = u + (live ? ray : 0) * u_stride;
  const int nq = t < n_imp ? (n_imp - 1 - t) / FINE_LANES + 1 : 0;
  float x[QN];
  int pos[QN];
#pragma unroll
  for (int q = 0; q < QN; ++q) x[q] = q < nq ? ur[t + FINE_LANES * q] : 0.0f;
  fine_search<true>(cdf, nb, x, pos);
  int lo_rank[QN];   // below + 1: a lower bound of #{z <= x} for the sample (see the merge)
#pragma unroll
  for (int q = 0; q < QN; ++q) {   // (queries q >= nq run on u = 0 and are never stored)
    const int inds = pos[q];
    const int below = inds - 1 > 0 ? inds - 1 : 0;
    lo_rank[q] = below + 1;
    const int above = inds < nb - 1 ? inds : nb - 1;
    const float cg0 = cdf[below], cg1 = cdf[above];
    const float bg0 = 0.5f * (zc[below + 1] + zc[below]);
    const float bg1 = 0.5f * (zc[above + 1] + zc[above]);
    float denom = cg1 - cg0;
    denom = denom < 1e-5f ? 1.0f : denom;
    const float tt = (x[q] - cg0) / denom;
    x[q] = bg0 + tt * (bg1 - bg0);
  }
  __builtin_amdgcn_wave_barrier();   // every read of the staged weights is done
#pragma unroll
  for (int q = 0; q < QN; ++q)
    if (q < nq) zf[t + FINE_LANES * q] = x[q];
  for (int j = n_imp + t; j < p2; j += FINE_LANES) zf[j] = __builtin_inff();
  __builtin_amdgcn_wave_barrier();
  // ascending bitonic sort of the (inf-padded) fine samples, per ray, skipped
  // when the inverse CDF of sorted u (eval: linspace) already produced them in
  // order
  bool unsorted = false;
  for (int j = t; j + 1 < n_imp; j += FINE_LANES) unsorted |= zf[j] > zf[j + 1];
  const unsigned long long bal = __ballot(unsorted);
  const bool sorted_in_place = ((bal >> (lane & ~(FINE_LANES - 1))) & 0xffffull) == 0;
  if (!sorted_in_place) {
    // bitonic sort in registers: element i = t + 16 q is x[q] of lane t (q <
    // p2 / 16 <= QN; inf past n_imp); partners 16 apart or more sit in the same
    // lane (a register pair), closer ones in the lane group (a shuffle). The
    // sorted values are unique, so any correct network gives the LDS sort's
    // result; this one keeps every step in registers (training: random u, no
    // sorted rows; the LDS version spent ~28 dependent LDS passes per ray here).
    const int nr = p2 / FINE_LANES;
#pragma unroll
    for (int q = 0; q < QN; ++q)
      if (q >= nq) x[q] = __builtin_inff();
    for (int k = 2; k <= p2; k <<= 1) {
      for (int jj = k >> 1; jj > 0; jj >>= 1) {
        if (jj >= FINE_LANES) {
#pragma unroll
          for (int bq = 1; bq < QN; bq <<= 1) {
            if (jj == bq * FINE_LANES) {
#pragma unroll
              for (int q = 0; q < QN; ++q) {
                if ((q & bq) == 0 && q < nr) {
                  const bool up = ((t + FINE_LANES * q) & k) == 0;
                  const float a = x[q], b = x[q | bq];
                  x[q] = up ? fminf(a, b) : fmaxf(a, b);
                  x[q | bq] = up ? fmaxf(a, b) : fminf(a, b);
                }
              }
            }
          }
        } else {
          const bool lower = (t & jj) == 0;
#pragma unroll
          for (int q = 0; q < QN; ++q) {
            const float o = __shfl_xor(x[q], jj);
            const bool up = ((t + FINE_LANES * q) & k) == 0;
            if (q < nr) x[q] = (lower == up) ? fminf(x[q], o) : fmaxf(x[q], o);
          }
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int q = 0; q < QN; ++q)
      if (q < nr) zf[t + FINE_LANES * q] = x[q];
    __builtin_amdgcn_wave_barrier();
  }
  // torch.sort(cat(z, z_fine)) values: merge by rank (ties: coarse first; equal
  // values are interchangeable)
  const int ncl = t < S ? (S - 1 - t) / FINE_LANES + 1 : 0;
  float xc[CN];
  int pcz[CN];
#pragma unroll
  for (int c = 0; c < CN; ++c) xc[c] = c < ncl ? zc[t + FINE_LANES * c] : 0.0f;
  fine_search<false>(zf, n_imp, xc, pcz);
  if (sorted_in_place) {
    // #{z <= x} of a fine sample from its own bin instead of a search: x is
    // bg0 + tt (bg1 - bg0) with tt >= 0 (cdf[below] <= u) and bg0 = the mid of
    // z[below], z[below + 1] >= z[below] (float rounding is monotone), so the
    // count is at least below + 1; a short forward walk (usually one or two
    // reads) finds it exactly. Only while x is still the value its bin produced,
    // i.e. when the ray's samples needed no sort (eval: sorted u).
#pragma unroll
    for (int q = 0; q < QN; ++q) {
      int r = lo_rank[q];
      while (r < S && zc[r] <= x[q]) ++r;
      pos[q] = r;
    }
  } else {
    fine_search<true>(zc, S, x, pos);
  }
  if (!live) return;
  float* out = z_all + ray * (int64_t)(S + n_imp);
#pragma unroll
  for (int c = 0; c < CN; ++c)
    if (c < ncl) out[t + FINE_LANES * c + pcz[c]] = xc[c];
#pragma unroll
  for (int q = 0; q < QN; ++q)
    if (q < nq) out[t + FINE_LANES * q + pos[q]] = x[q];
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

// ---------------------------------------------------------------------------
// Frequency encoding for the training MLP (freq.py:7-32), feature-major:
// out[j][p] with j = c (raw coordinate), 3 + 6f + c (sin 2^f x_c), 6 + 6f + c
// (cos 2^f x_c) -- the column order of torch.cat([x, sin, cos, ...], -1). A
// block is 64 samples x W waves, wave w taking the bands f = w, w + W, ...
// (wave 0 also the raw coordinates), so every output row is a coalesced 256-B
// store and the accurate sincosf calls of one sample (large arguments, up to
// 2^9 x) run on W waves instead of one thread's chain (C3 step: 122 -> 115 us
// for the 4 launches). The block's max |.| is raised into *amax once (float bits as
// uint: all values are >= 0). 2^f x is exact (power of two); sinf/cosf are the
// same device-library calls torch's sin/cos kernels make.
// ---------------------------------------------------------------------------
constexpr int kEncMaxWaves = 16;
__global__ __launch_bounds__(64 * kEncMaxWaves) void freq_encode_fm_kernel(
    const float* __restrict__ x, int64_t ldx, int64_t P, int L, float* __restrict__ out,
    int64_t ldo, unsigned* __restrict__ amax) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int64_t p = (int64_t)blockIdx.x * 64 + lane;
  float m = 0.0f;
  if (p < P) {
    float v[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      v[c] = x[p * ldx + c];
      if (wave == 0) {
        out[c * ldo + p] = v[c];
        m = fmaxf(m, fabsf(v[c]));
      }
    }
    for (int f = wave; f < L; f += nw) {
      const float k = (float)(1 << f);
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float a = v[c] * k;
        float sn, cs;
        sincosf(a, &sn, &cs);   // one range reduction for both (ocml: the same values)
        out[(3 + 6 * f + c) * ldo + p] = sn;
        out[(6 + 6 * f + c) * ldo + p] = cs;
        m = fmaxf(m, fmaxf(fabsf(sn), fabsf(cs)));
      }
    }
  }
  if (amax) {
    __shared__ float wmax[kEncMaxWaves];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if (lane == 0) wmax[wave] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int w = 1; w < nw; ++w) m = fmaxf(m, wmax[w]);
      atomicMax(amax, __float_as_uint(m));
    }
  }
}

// Element (row, p) of an [rows][P] operand, floats: feature-major rows
// (bs == 0: row * ld + p) or the training kernels' T16 layout (bs > 0: block
// stride bs, rows permuted inside their 16-row groups; mlp_x3.hip Lay).
__device__ __forceinline__ int64_t lay_idx(int row, int64_t p, int64_t ld, int64_t bs) {
  return bs ? (p >> 4) * bs + ((row >> 4) * 256 + (row & 3) * 64 + ((row >> 2) & 3) * 16) + (p & 15)
            : (int64_t)row * ld + p;
}

// d x_c = d_enc[c] + sum_f 2^f (cos(2^f x_c) d_sin - sin(2^f x_c) d_cos): the
// chain rule through the encoding (autograd of freq.py's cat of sin/cos).
// With d_enc2, d_enc = d_enc + d_enc2 elementwise first (the encoding feeds two
// layers: autograd's sum of their input gradients). With enc (the forward's
// encoding rows, layout (lde, bse)), sin / cos are read from it instead of
// recomputed (the same sincosf values: it is what the forward wrote). d_enc /
// d_enc2 in layout (ldd, bsd); lay_idx.
__global__ __launch_bounds__(256) void freq_encode_fm_backward_kernel(
    const float* __restrict__ d_enc, const float* __restrict__ d_enc2, int64_t ldd, int64_t bsd,
    const float* __restrict__ enc, int64_t lde, int64_t bse, const float* __restrict__ x,
    int64_t ldx, int64_t P, int L, float* __restrict__ dx) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  auto de = [&](int row) {
    const int64_t i = lay_idx(row, p, ldd, bsd);
    float v = d_enc[i];
    if (d_enc2) v = v + d_enc2[i];
    return v;
  };
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float v = x[p * ldx + c];
    float g = de(c);
    for (int f = 0; f < L; ++f) {
      const float k = (float)(1 << f);
      float sn, cs;
      if (enc) {
        sn = enc[lay_idx(3 + 6 * f + c, p, lde, bse)];
        cs = enc[lay_idx(6 + 6 * f + c, p, lde, bse)];
      } else {
        sincosf(v * k, &sn, &cs);
      }
      const float ds = de(3 + 6 * f + c) * cs - de(6 + 6 * f + c) * sn;
      g = g + ds * k;
    }
    dx[p * 3 + c] = g;
  }
}

// The same gradient taken on to the depths of the samples p = ray * S + step
// at o + d * z (VR:165; rays constant): dz[p] = sum_c dx_c * d_c, as torch's
// autograd of rays_o + rays_d * z sums it (mul, then the 3-term reduction).
// LC > 0: L == LC at compile time (every band's loads unrolled and in flight
// together; the runtime loop exposes one load latency per band)
template <int LC>
__global__ __launch_bounds__(256) void freq_encode_fm_backward_dz_kernel(
    const float* __restrict__ d_enc, const float* __restrict__ d_enc2, int64_t ldd, int64_t bsd,
    const float* __restrict__ enc, int64_t lde, int64_t bse, const float* __restrict__ rays_d,
    int S, int64_t P, int Lr, float* __restrict__ dz) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  const int L = LC > 0 ? LC : Lr;
  auto de = [&](int row) {
    const int64_t i = lay_idx(row, p, ldd, bsd);
    float v = d_enc[i];
    if (d_enc2) v = v + d_enc2[i];
    return v;
  };
  const int64_t ray = p / S;
  float acc = 0.0f;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    float g = de(c);
#pragma unroll
    for (int f = 0; f < L; ++f) {
      const float k = (float)(1 << f);
      const float sn = enc[lay_idx(3 + 6 * f + c, p, lde, bse)];
      const float cs = enc[lay_idx(6 + 6 * f + c, p, lde, bse)];
      const float ds = de(3 + 6 * f + c) * cs - de(6 + 6 * f + c) * sn;
      g = g + ds * k;
    }
    const float t = g * rays_d[ray * 3 + c];
    acc = c == 0 ? t : acc + t;
  }
  dz[p] = acc;
}

// L = 10, one wave per coordinate: a block of 3 waves takes 64 samples, wave c
// sums coordinate c's rows (a third of the loads per thread, so more waves in
// flight), and lane s of wave 0 adds the three products in c order through LDS
// (the same operations in the same order as the one-thread-per-sample kernel).
__global__ __launch_bounds__(192) void freq_encode_fm_backward_dz3_kernel(
    const float* __restrict__ d_enc, const float* __restrict__ d_enc2, int64_t ldd, int64_t bsd,
    const float* __restrict__ enc, int64_t lde, int64_t bse, const float* __restrict__ rays_d,
    int S, int64_t P, float* __restrict__ dz) {
  constexpr int L = 10;
  __shared__ float t3[3][64];
  const int c = threadIdx.x >> 6, s = threadIdx.x & 63;
  const int64_t p = (int64_t)blockIdx.x * 64 + s;
  const bool ok = p < P;
  const int64_t pp = ok ? p : 0;
  auto de = [&](int row) {
    const int64_t i = lay_idx(row, pp, ldd, bsd);
    float v = d_enc[i];
    if (d_enc2) v = v + d_enc2[i];
    return v;
  };
  float g = de(c);
#pragma unroll
  for (int f = 0; f < L; ++f) {
    const float k = (float)(1 << f);
    const float sn = enc[lay_idx(3 + 6 * f + c, pp, lde, bse)];
    const float cs = enc[lay_idx(6 + 6 * f + c, pp, lde, bse)];
    const float ds = de(3 + 6 * f + c) * cs - de(6 + 6 * f + c) * sn;
    g = g + ds * k;
  }
  t3[c][s] = g * rays_d[(pp / S) * 3 + c];
  __syncthreads();
  if (c == 0 && ok) {
    float acc = t3[0][s];
    acc = acc + t3[1][s];
    acc = acc + t3[2][s];
    dz[p] = acc;
  }
}

// max |rgb| / |sigma| of raw [P][4] (float bits: the values are >= 0)
__global__ __launch_bounds__(256) void raw_absmax_kernel(const float4* __restrict__ raw, int64_t P,
                                                         unsigned* __restrict__ amax) {
  float mr = 0.0f, ms = 0.0f;
  for (int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x; p < P; p += (int64_t)gridDim.x * 256) {
    const float4 v = raw[p];
    mr = fmaxf(mr, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fabsf(v.z)));
    ms = fmaxf(ms, fabsf(v.w));
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    mr = fmaxf(mr, __shfl_xor(mr, o));
    ms = fmaxf(ms, __shfl_xor(ms, o));
  }
  __shared__ float part[2][4];
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    part[0][wave] = mr;
    part[1][wave] = ms;
  }
  __syncthreads();
  if (threadIdx.x < 2) {   // one atomic per workgroup and value
    const float m = fmaxf(fmaxf(part[threadIdx.x][0], part[threadIdx.x][1]),
                          fmaxf(part[threadIdx.x][2], part[threadIdx.x][3]));
    atomicMax(amax + threadIdx.x, __float_as_uint(m));
  }
}

extern "C" {
int nerf_raw_absmax(const float* raw, int64_t P, float* amax, nerf_stream_t stream) {
  NERF_REQUIRE(raw && amax && P >= 0, "nerf_raw_absmax: bad arguments");
  NERF_REQUIRE(((uintptr_t)raw & 15) == 0, "nerf_raw_absmax: raw must be 16-byte aligned");
  if (P == 0) return 0;
  // 4 float4 per thread at least: a few hundred atomics per launch, not thousands
  const int64_t blocks = cdiv(P, 1024) < 256 ? cdiv(P, 1024) : 256;
  hipLaunchKernelGGL(raw_absmax_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream),
                     (const float4*)raw, P, (unsigned*)amax);
  return check_launch("raw_absmax_kernel");
}

int nerf_ert_segment(const float* raw, const float* z, int64_t z_stride, const float* rays_d,
                     int64_t n, int S, int s0, int s1, int s2, float thr, double* T,
                     unsigned char* active, int* list, int* count, nerf_stream_t stream) {
  NERF_REQUIRE(raw && z && rays_d && T && active && list && count,
               "nerf_ert_segment: null pointer");
  NERF_REQUIRE(n >= 0 && S >= 1 && 0 <= s0 && s0 <= s1 && s1 <= s2 && s2 <= S &&
                   n * (int64_t)S < (1ll << 31),
               "nerf_ert_segment: bad segment");
  if (n == 0) return 0;
  hipLaunchKernelGGL(ert_segment_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0,
                     as_stream(stream), (const float4*)raw, z, z_stride, rays_d, n, S, s0, s1, s2,
                     thr, T, active, list, count);
  return check_launch("ert_segment_kernel");
}


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

// One nn.Linear (+ ReLU) of a NeRF of any topology (NET:9-74), FP32, over
// feature-major activations: Y[m * sym + p * syp] = act(b[m] + sum_k W[m][k] X[k][p])
// for m < M, p < P (W row-major [M][ldw >= K], torch's Linear layout; X [K][ldx]; the
// output strides write feature-major rows (sym = ldy, syp = 1) or the [P][4]
// raw record (sym = 1, syp = 4)). The k sum runs in ascending order as one FMA
// chain per output. The lego topology never comes here (its fused kernels);
// this is the layer-by-layer path for other D / W / skips / encoding widths.
// Tile 64 (m) x 64 (p), K steps of 16 through LDS, 4 x 4 outputs per thread.
__global__ __launch_bounds__(256) void linear_fm_kernel(const float* __restrict__ W, int64_t ldw,
                                                        const float* __restrict__ b,
                                                        const float* __restrict__ X, int64_t ldx,
                                                        int K, int64_t P, int M, int relu,
                                                        float* __restrict__ Y, int64_t sym,
                                                        int64_t syp) {
  __shared__ float ws[16][64 + 1];   // [k][m]
  __shared__ float xs[16][64];       // [k][p]
  const int tid = threadIdx.x, tm = tid >> 4, tp = tid & 15;
  const int m0 = blockIdx.y * 64;
  const int64_t p0 = (int64_t)blockIdx.x * 64;
  float acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = 0.0f;
  for (int k0 = 0; k0 < K; k0 += 16) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int e = tid + 256 * r;          // 1024 elements of each tile
      const int wk = e & 15, wm = e >> 4;   // W tile: k fastest (rows of W contiguous)
      const int gm = m0 + wm, gk = k0 + wk;
      ws[wk][wm] = (gm < M && gk < K) ? W[(int64_t)gm * ldw + gk] : 0.0f;
      const int xk = e >> 6, xp = e & 63;   // X tile: p fastest
      const int64_t gp = p0 + xp;
      xs[xk][xp] = (k0 + xk < K && gp < P) ? X[(int64_t)(k0 + xk) * ldx + gp] : 0.0f;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      float a[4], x[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = ws[k][tm + 16 * i];
#pragma unroll
      for (int j = 0; j < 4; ++j) x[j] = xs[k][tp + 16 * j];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_fmaf(a[i], x[j], acc[i][j]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + tm + 16 * i;
    if (m >= M) continue;
    const float bias = b ? b[m] : 0.0f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t p = p0 + tp + 16 * j;
      if (p >= P) continue;
      float v = acc[i][j] + bias;
      if (relu) v = fmaxf(v, 0.0f);
      Y[(int64_t)m * sym + p * syp] = v;
    }
  }
}

int nerf_linear_fm(const float* W, int64_t ldw, const float* b, const float* X, int64_t ldx, int K,
                   int64_t P, int M, int relu, float* Y, int64_t sym, int64_t syp,
                   nerf_stream_t stream) {
  NERF_REQUIRE(W && X && Y, "nerf_linear_fm: null pointer");
  NERF_REQUIRE(K >= 1 && M >= 1 && P >= 0 && ldx >= P && ldw >= K, "nerf_linear_fm: bad size");
  NERF_REQUIRE(cdiv(P, 64) < (1ll << 31) && cdiv(M, 64) < 65536, "nerf_linear_fm: too large");
  if (P == 0) return 0;
  hipLaunchKernelGGL(linear_fm_kernel, dim3((unsigned)cdiv(P, 64), (unsigned)cdiv(M, 64)),
                     dim3(256), 0, as_stream(stream), W, ldw, b, X, ldx, K, P, M, relu, Y, sym,
                     syp);
  return check_launch("linear_fm_kernel");
}

// VR:310-314 / :1098-1103 (raw_noise_std > 0): the density logit of every
// sample plus its noise (torch.randn * raw_noise_std, drawn by the caller in
// the reference's order), one FP32 add as `raw[..., 3] + noise`; rgb logits
// copied. The composite kernels then read the noisy raw.
__global__ __launch_bounds__(256) void add_sigma_noise_kernel(const float4* __restrict__ raw,
                                                              const float* __restrict__ noise,
                                                              int64_t count,
                                                              float4* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count;
       i += (int64_t)gridDim.x * blockDim.x) {
    float4 v = raw[i];
    v.w = v.w + noise[i];
    out[i] = v;
  }
}

int nerf_add_sigma_noise(const float* raw, const float* noise, int64_t count, float* out,
                         nerf_stream_t stream) {
  NERF_REQUIRE(raw && noise && out, "nerf_add_sigma_noise: null pointer");
  NERF_REQUIRE(count >= 0, "nerf_add_sigma_noise: bad size");
  if (count == 0) return 0;
  const int64_t blocks = std::min<int64_t>(cdiv(count, 256), 256 * 64);
  hipLaunchKernelGGL(add_sigma_noise_kernel, dim3((unsigned)blocks), dim3(256), 0,
                     as_stream(stream), (const float4*)raw, noise, count, (float4*)out);
  return check_launch("add_sigma_noise_kernel");
}

// ---------------------------------------------------------------------------
// VR:875-961 _populate_occupancy_grid_kilonerf_method: the 27 sub-points of
// cells [cell0, cell0 + ncells) in the method's flat order (cell f: z = f / res^2,
// y = (f % res^2) / res, x = f % res, :903-906), sub-point s = 9 dz + 3 dy + dx
// (:913-920), point = (bbox_min + (x, y, z) * cell) + (d / 2) * cell, every
// product and sum rounded as torch's separate float32 ops (:908-918).
__global__ __launch_bounds__(256) void grid_points_kernel(int64_t cell0, int64_t count, int res,
                                                          float bx, float by, float bz, float cx,
                                                          float cy, float cz,
                                                          float* __restrict__ pts) {
  const int64_t rr = (int64_t)res * res;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t f = cell0 + i / 27;
    const int s = (int)(i % 27);
    const float x = (float)(f % res), y = (float)((f % rr) / res), z = (float)(f / rr);
    const float ox = (float)(s % 3) / 2.0f, oy = (float)((s / 3) % 3) / 2.0f,
                oz = (float)(s / 9) / 2.0f;
    const float mx = __fadd_rn(bx, __fmul_rn(x, cx)), my = __fadd_rn(by, __fmul_rn(y, cy)),
                mz = __fadd_rn(bz, __fmul_rn(z, cz));
    pts[3 * i + 0] = __fadd_rn(mx, __fmul_rn(ox, cx));
    pts[3 * i + 1] = __fadd_rn(my, __fmul_rn(oy, cy));
    pts[3 * i + 2] = __fadd_rn(mz, __fmul_rn(oz, cz));
  }
}

// VR:937-953: per cell the largest relu(sigma) of its 27 points (torch's max
// propagates NaN, and NaN > thr is false), > thr marks the cell -- at grid
// index cell_of[f] (the reference's list(set(...)) order, built on the host)
// or, with cell_of NULL, at the cell's own [x][y][z] index.
__global__ __launch_bounds__(256) void grid_decide_kernel(const float4* __restrict__ raw,
                                                          int64_t cell0, int64_t ncells, int res,
                                                          float thr,
                                                          const int32_t* __restrict__ cell_of,
                                                          uint8_t* __restrict__ grid) {
  const int64_t rr = (int64_t)res * res;
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < ncells;
       c += (int64_t)gridDim.x * blockDim.x) {
    float m = 0.0f;
    bool nan = false;
#pragma unroll
    for (int k = 0; k < 27; ++k) {
      const float v = raw[c * 27 + k].w;
      nan |= v != v;
      m = fmaxf(m, v);   // relu then max: max(0, v_0, ..., v_26)
    }
    if (!nan && m > thr) {
      const int64_t f = cell0 + c;
      const int64_t own = ((f % res) * res + (f % rr) / res) * res + f / rr;
      grid[cell_of ? (int64_t)cell_of[f] : own] = 1;
    }
  }
}

int nerf_grid_points(int64_t cell0, int64_t ncells, int res, const float bbox_min[3],
                     const float cell_size[3], float* pts, nerf_stream_t stream) {
  NERF_REQUIRE(pts && bbox_min && cell_size, "nerf_grid_points: null pointer");
  NERF_REQUIRE(res >= 1 && res <= 1024 && cell0 >= 0 && ncells >= 0 &&
                   cell0 + ncells <= (int64_t)res * res * res,
               "nerf_grid_points: bad cell range");
  if (ncells == 0) return 0;
  const int64_t count = ncells * 27;
  const int64_t blocks = std::min<int64_t>(cdiv(count, 256), 256 * 64);
  hipLaunchKernelGGL(grid_points_kernel, dim3((unsigned)blocks), dim3(256), 0,
                     as_stream(stream), cell0, count, res, bbox_min[0], bbox_min[1], bbox_min[2],
                     cell_size[0], cell_size[1], cell_size[2], pts);
  return check_launch("grid_points_kernel");
}

int nerf_grid_decide(const float* raw, int64_t cell0, int64_t ncells, int res, float threshold,
                     const int32_t* cell_of, uint8_t* grid, nerf_stream_t stream) {
  NERF_REQUIRE(raw && grid, "nerf_grid_decide: null pointer");
  NERF_REQUIRE(res >= 1 && res <= 1024 && cell0 >= 0 && ncells >= 0 &&
                   cell0 + ncells <= (int64_t)res * res * res,
               "nerf_grid_decide: bad cell range");
  if (ncells == 0) return 0;
  const int64_t blocks = std::min<int64_t>(cdiv(ncells, 256), 256 * 64);
  hipLaunchKernelGGL(grid_decide_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream),
                     (const float4*)raw, cell0, ncells, res, threshold, cell_of, grid);
  return check_launch("grid_decide_kernel");
}

int nerf_composite(const float* raw, const float* z, int64_t z_stride, const float* rays_d,
                   int64_t n, int S, int white_bkgd, float* rgb, float* disp, float* acc,
                   float* depth, float* weights, nerf_stream_t stream) {
  NERF_REQUIRE(raw && z && rays_d && rgb && disp && acc && depth,
               "nerf_composite: null pointer");
  NERF_REQUIRE(n >= 0 && S >= 2 && S < 1024, "nerf_composite: S must be in [2, 1024)");
  if (n == 0) return 0;
  if (S <= 256) {
    const int c = (S + 15) / 16;
    const dim3 grid((unsigned)cdiv(n, COMP16_RPB)), block(256);
#define NERF_COMP16(CC)                                                                        \
  hipLaunchKernelGGL((composite16_kernel<CC>), grid, block, 0, as_stream(stream),              \
                     (const float4*)raw, z, z_stride, rays_d, n, S, white_bkgd, rgb, disp, acc, \
                     depth, weights)
    if (c <= 4) NERF_COMP16(4);
    else if (c <= 8) NERF_COMP16(8);
    else if (c <= 12) NERF_COMP16(12);
    else NERF_COMP16(16);
#undef NERF_COMP16
    return check_launch("composite16_kernel");
  }
  hipLaunchKernelGGL(composite_kernel, dim3((unsigned)cdiv(n, COMP_WAVES)), dim3(64 * COMP_WAVES), 0,
                     as_stream(stream), (const float4*)raw, z, z_stride, rays_d, n, S,
                     white_bkgd, rgb, disp, acc, depth, weights);
  return check_launch("composite_kernel");
}

size_t nerf_composite_ert_workspace(int64_t n, int chunk) {
  if (n <= 0 || chunk <= 0) return 16;
  const size_t flags = ((size_t)cdiv(n, chunk) * sizeof(int) + 15) / 16 * 16;
  return flags + (size_t)n * sizeof(ErtCut);
}

int nerf_composite_ert(const float* raw, const float* z, int64_t z_stride, const float* rays_d,
                       int64_t n, int S, int white_bkgd, float threshold, int chunk, float* rgb,
                       float* disp, float* acc, float* depth, float* weights, void* workspace,
                       nerf_stream_t stream) {
  NERF_REQUIRE(raw && z && rays_d && rgb && disp && acc && depth,
               "nerf_composite_ert: null pointer");
  NERF_REQUIRE(n >= 0 && S >= 2 && S < 1024 && chunk > 0 && chunk <= ERT_MAX_CHUNK,
               "nerf_composite_ert: need 2 <= S < 1024 and 0 < chunk <= 2048");
  if (n == 0) return 0;
  if (S > 256) {   // one block per chunk, the cut maps in LDS
    hipLaunchKernelGGL(composite_ert_kernel, dim3((unsigned)cdiv(n, chunk)), dim3(64 * ERT_WAVES),
                       0, as_stream(stream), (const float4*)raw, z, z_stride, rays_d, n, S,
                       white_bkgd, threshold, chunk, rgb, disp, acc, depth, weights);
    return check_launch("composite_ert_kernel");
  }
  NERF_REQUIRE(workspace && ((uintptr_t)workspace & 15) == 0,
               "nerf_composite_ert: workspace (nerf_composite_ert_workspace bytes, 16-B aligned)");
  const int64_t nch = cdiv(n, chunk);
  int* flags = (int*)workspace;
  ErtCut* cuts = (ErtCut*)((char*)workspace + ((size_t)nch * sizeof(int) + 15) / 16 * 16);
  hipError_t e = hipMemsetAsync(flags, 0, (size_t)nch * sizeof(int), as_stream(stream));
  if (e != hipSuccess) return fail((int)e, "nerf_composite_ert: flag reset failed");
  const int c = (S + 15) / 16;
  const dim3 grid((unsigned)cdiv(n, COMP16_RPB)), block(256);
#define NERF_COMP16E(CC)                                                                       \
  hipLaunchKernelGGL((composite16_kernel<CC, true>), grid, block, 0, as_stream(stream),        \
                     (const float4*)raw, z, z_stride, rays_d, n, S, white_bkgd, rgb, disp, acc, \
                     depth, weights, threshold, chunk, cuts, flags)
  if (c <= 4) NERF_COMP16E(4);
  else if (c <= 8) NERF_COMP16E(8);
  else if (c <= 12) NERF_COMP16E(12);
  else NERF_COMP16E(16);
#undef NERF_COMP16E
  const int rc = check_launch("composite16_kernel<ERT>");
  if (rc) return rc;
  hipLaunchKernelGGL(ert_fixup_kernel, dim3((unsigned)cdiv(n * 16, 256)), dim3(256), 0,
                     as_stream(stream), (const ErtCut*)cuts, (const int*)flags, n, S, chunk,
                     white_bkgd, rgb, disp, acc, depth, weights);
  return check_launch("ert_fixup_kernel");
}

int nerf_sample_fine(const float* z, int64_t z_stride, const float* weights, const float* u,
                     int64_t u_stride, int64_t n, int S, int n_imp, float* z_all,
                     nerf_stream_t stream) {
  NERF_REQUIRE(z && weights && u && z_all, "nerf_sample_fine: null pointer");
  NERF_REQUIRE(n >= 0 && S >= 3 && S <= FINE_MAX_S && n_imp >= 1 && n_imp <= FINE_MAX_IMP,
               "nerf_sample_fine: need 3 <= S <= 130 coarse and 1 <= n_imp <= 256 fine samples");
  if (n == 0) return 0;
  // row: zc[S] | cdf[S] | zf, padded so rays sit 16 floats apart mod 32 banks:
  // the two rays of a ds_read_b32 lane group hit disjoint banks on aligned runs
  const int p2 = fine_p2(n_imp);
  int row = 2 * S + (p2 > S - 2 ? p2 : S - 2);
  row += (48 - row % 32) % 32;
  const int q = (int)cdiv(n_imp, FINE_LANES), c = (int)cdiv(S, FINE_LANES);
  const dim3 grid((unsigned)cdiv(n, FINE_RPB)), block(64 * FINE_WAVES);
  const size_t lds = FINE_RPB * (size_t)row * sizeof(float);
#define NERF_FINE_LAUNCH(QN, CN)                                                          \
  hipLaunchKernelGGL((sample_fine_kernel<QN, CN>), grid, block, lds, as_stream(stream), z, \
                     z_stride, weights, u, u_stride, n, S, n_imp, row, z_all)
#define NERF_FINE_C(QN)                          \
  if (c <= 2) NERF_FINE_LAUNCH(QN, 2);           \
  else if (c <= 4) NERF_FINE_LAUNCH(QN, 4);      \
  else NERF_FINE_LAUNCH(QN, 9);
  if (q <= 2) { NERF_FINE_C(2) }
  else if (q <= 4) { NERF_FINE_C(4) }
  else if (q <= 8) { NERF_FINE_C(8) }
  else { NERF_FINE_C(16) }
#undef NERF_FINE_C
#undef NERF_FINE_LAUNCH
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

int nerf_freq_encode_fm(const float* x, int64_t ldx, int64_t P, int n_freq, float* out,
                        int64_t ldo, float* amax, nerf_stream_t stream) {
  NERF_REQUIRE(x && out, "nerf_freq_encode_fm: null pointer");
  NERF_REQUIRE(P >= 0 && ldx >= 3 && ldo >= P && n_freq >= 0 && n_freq <= 24,
               "nerf_freq_encode_fm: bad size");
  if (P == 0) return 0;
  const int waves = n_freq < 1 ? 1 : (n_freq < kEncMaxWaves ? n_freq : kEncMaxWaves);
  hipLaunchKernelGGL(freq_encode_fm_kernel, dim3((unsigned)cdiv(P, 64)), dim3(64 * waves), 0,
                     as_stream(stream), x, ldx, P, n_freq, out, ldo, (unsigned*)amax);
  return check_launch("freq_encode_fm_kernel");
}

int nerf_freq_encode_fm_backward(const float* d_enc, int64_t ldd, const float* x, int64_t ldx,
                                 int64_t P, int n_freq, float* dx, nerf_stream_t stream) {
  return nerf_freq_encode_fm_backward_sum(d_enc, nullptr, ldd, 0, nullptr, ldd, 0, x, ldx, P,
                                          n_freq, dx, stream);
}

// an operand layout (ld, bs) as lay_idx reads it: feature-major rows need ld >= P
static bool enc_lay_ok(int64_t ld, int64_t bs, int64_t P) {
  return bs == 0 ? ld >= P : bs > 0 && bs % 256 == 0;
}

int nerf_freq_encode_fm_backward_dz(const float* d_enc, const float* d_enc2, int64_t ldd,
                                    int64_t bsd, const float* enc, int64_t lde, int64_t bse,
                                    const float* rays_d, int S, int64_t P, int n_freq, float* dz,
                                    nerf_stream_t stream) {
  NERF_REQUIRE(d_enc && enc && rays_d && dz, "nerf_freq_encode_fm_backward_dz: null pointer");
  NERF_REQUIRE(P >= 0 && S >= 1 && P % S == 0 && enc_lay_ok(ldd, bsd, P) &&
                   enc_lay_ok(lde, bse, P) && n_freq >= 0 && n_freq <= 24,
               "nerf_freq_encode_fm_backward_dz: bad size");
  if (P == 0) return 0;
  if (n_freq == 10)   // the xyz encoding (L = 10)
    hipLaunchKernelGGL(freq_encode_fm_backward_dz3_kernel, dim3((unsigned)cdiv(P, 64)),
                       dim3(192), 0, as_stream(stream), d_enc, d_enc2, ldd, bsd, enc, lde, bse,
                       rays_d, S, P, dz);
  else
    hipLaunchKernelGGL(freq_encode_fm_backward_dz_kernel<0>, dim3((unsigned)cdiv(P, 256)),
                       dim3(256), 0, as_stream(stream), d_enc, d_enc2, ldd, bsd, enc, lde, bse,
                       rays_d, S, P, n_freq, dz);
  return check_launch("freq_encode_fm_backward_dz_kernel");
}

int nerf_freq_encode_fm_backward_sum(const float* d_enc, const float* d_enc2, int64_t ldd,
                                     int64_t bsd, const float* enc, int64_t lde, int64_t bse,
                                     const float* x, int64_t ldx, int64_t P, int n_freq,
                                     float* dx, nerf_stream_t stream) {
  NERF_REQUIRE(d_enc && x && dx, "nerf_freq_encode_fm_backward: null pointer");
  NERF_REQUIRE(P >= 0 && ldx >= 3 && enc_lay_ok(ldd, bsd, P) &&
                   (!enc || enc_lay_ok(lde, bse, P)) && n_freq >= 0 && n_freq <= 24,
               "nerf_freq_encode_fm_backward: bad size");
  if (P == 0) return 0;
  hipLaunchKernelGGL(freq_encode_fm_backward_kernel, dim3((unsigned)cdiv(P, 256)), dim3(256), 0,
                     as_stream(stream), d_enc, d_enc2, ldd, bsd, enc, lde, bse, x, ldx, P, n_freq,
                     dx);
  return check_launch("freq_encode_fm_backward_kernel");
}

}  // extern "C"
