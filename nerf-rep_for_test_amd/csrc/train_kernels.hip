// Training-step kernels around the MLPs (BASELINE configs[2]):
// the differentiable compositing of _raw2outputs (VR:286-357) and importance
// sampling of _sample_fine (VR:239-268, training-mode u) + the sorted merge of
// VR:181-184, forward and backward, so the whole step runs on hand-written
// kernels without data-dependent host syncs (torch's cumprod backward tests its
// input for zeros on the host, which a HIP graph cannot capture).
//
// Compositing: one wave per ray, lanes over samples; the transmittance is the
// reference's exclusive cumprod of
// (1 - a + 1e-10) accumulated in double like torch's CPU kernel, the map sums
// in torch's CPU summation orders (common.h tsum_last / tsum_dim2).
// The forward also stores T (the backward reads it instead of dividing w by a).
// Backward, with G_i = dL/dw_i + g_rgb . c_i + g_acc' + g_depth' z_i the total
// gradient reaching weight i (white background folds -sum(g_rgb) into g_acc'):
//   dL/da_i = T_i (G_i - B_i),  B_i = sum_{j>i} G_j a_j prod_{i<k<j} x_k,
//   x_k = 1 - a_k + 1e-10, B by the reverse recurrence B_i = G_{i+1} a_{i+1} +
//   x_{i+1} B_{i+1} (no division: zero-safe), then a = 1 - exp(-relu(r) d).
//
// Importance sampling: one wave per ray (LDS rows as the inference
// sample_fine kernel), forward = nerf_sample_fine; the backward recomputes the
// cdf and each fine sample's bin, locates the sample in the merged row, and
// takes dL/dz_all there back to dL/dweights through t = (u - c0)/(c1 - c0),
// the cdf (reverse cumsum) and the normalisation pdf = w'/sum(w').
#include "common.h"

namespace nerfhip {

// ---------------------------------------------------------------------------
// compositing
// ---------------------------------------------------------------------------
__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

// One wave per ray (a 1024-ray batch is 1024 waves), lanes over the samples.
constexpr int CT_WAVES = 4;
constexpr int CT_MAX_S = 256;
struct CtLds {
  float w[CT_MAX_S], z[CT_MAX_S], c[3][CT_MAX_S], gd[CT_MAX_S];
};

__device__ __forceinline__ double ct_prod_scan(double p, int lane) {   // inclusive
  for (int o = 1; o < 64; o <<= 1) {
    const double q = __shfl_up(p, o);
    if (lane >= o) p *= q;
  }
  return p;
}

__global__ __launch_bounds__(64 * CT_WAVES) void composite_train_fwd_kernel(
    const float4* __restrict__ raw, const float* __restrict__ z, const float* __restrict__ rays_d,
    int64_t n, int S, int white, float* __restrict__ rgb, float* __restrict__ disp,
    float* __restrict__ acc, float* __restrict__ depth, float* __restrict__ w,
    float* __restrict__ trans) {
  __shared__ CtLds sm[CT_WAVES];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int64_t r = (int64_t)blockIdx.x * CT_WAVES + wave;
  if (r >= n) return;   // wave-uniform; no block barriers below
  CtLds& L = sm[wave];
  const float4* rr = raw + r * S;
  const float* zr = z + r * S;
  const float nd = torch_norm3(rays_d[r * 3], rays_d[r * 3 + 1], rays_d[r * 3 + 2]);
  double carry = 1.0;
  for (int b = 0; b < S; b += 64) {
    const int s = b + lane;
    const bool act = s < S;
    float a = 0.0f, zs = 0.0f;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (act) {
      v = rr[s];
      zs = zr[s];
      const float dist = ((s < S - 1) ? (zr[s + 1] - zs) : 1e10f) * nd;   // VR:290-292
      a = 1.0f - expf((-fmaxf(v.w, 0.0f)) * dist);                       // VR:288
    }
    // exclusive cumprod of (1 - a + 1e-10), accumulated in double (VR:329)
    const double inc = ct_prod_scan(act ? (double)((1.0f - a) + 1e-10f) : 1.0, lane);
    double ex = __shfl_up(inc, 1);
    if (lane == 0) ex = 1.0;
    const float T = (float)(carry * ex);
    carry = carry * __shfl(inc, 63);
    if (act) {
      const float ws = a * T;
      w[r * S + s] = ws;
      trans[r * S + s] = T;
      L.w[s] = ws;
      L.z[s] = zs;
      L.c[0][s] = ws * sigm(v.x);
      L.c[1][s] = ws * sigm(v.y);
      L.c[2][s] = ws * sigm(v.z);
    }
  }
  __builtin_amdgcn_wave_barrier();
  // the map sums in torch's CPU orders, one lane per sum (VR:331-334)
  float m = 0.0f;
  if (lane < 3) {
    const float* cr = L.c[lane];
    m = tsum_dim2(S, [&](int i) { return cr[i]; });
  } else if (lane == 3) {
    m = tsum_last(S, [&](int i) { return L.w[i] * L.z[i]; });
  } else if (lane == 4) {
    m = tsum_last(S, [&](int i) { return L.w[i]; });
  }
  const float m0 = __shfl(m, 0), m1 = __shfl(m, 1), m2 = __shfl(m, 2);
  const float dp = __shfl(m, 3), ac = __shfl(m, 4);
  if (lane == 0) {
    disp[r] = 1.0f / torch_max(1e-10f, dp / ac);
    acc[r] = ac;
    depth[r] = dp;
    rgb[r * 3 + 0] = white ? m0 + (1.0f - ac) : m0;
    rgb[r * 3 + 1] = white ? m1 + (1.0f - ac) : m1;
    rgb[r * 3 + 2] = white ? m2 + (1.0f - ac) : m2;
  }
}

// Gradients: g_rgb [n,3], g_disp / g_acc / g_depth [n], g_w [n,S] (any may be
// null = zero). Outputs d_raw [n,S,4] and d_z [n,S] (null: not needed).
// B_{s-1} = h_s(B_s) with h_s(x) = G_s a_s + x_s x and B_{S-1} = 0: per 64-sample
// block (from the last), a reverse inclusive scan composes the affine maps
// (double), lane i applies the composition from i+1 up to the carried B.
__global__ __launch_bounds__(64 * CT_WAVES) void composite_train_bwd_kernel(
    const float4* __restrict__ raw, const float* __restrict__ z, const float* __restrict__ rays_d,
    const float* __restrict__ w, const float* __restrict__ trans, const float* __restrict__ acc,
    const float* __restrict__ depth, int64_t n, int S, int white,
    const float* __restrict__ g_rgb, const float* __restrict__ g_disp,
    const float* __restrict__ g_acc, const float* __restrict__ g_depth,
    const float* __restrict__ g_w, float4* __restrict__ d_raw, float* __restrict__ d_z) {
  __shared__ CtLds sm[CT_WAVES];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int64_t r = (int64_t)blockIdx.x * CT_WAVES + wave;
  if (r >= n) return;
  CtLds& L = sm[wave];
  const float4* rr = raw + r * S;
  const float* zr = z + r * S;
  const float nd = torch_norm3(rays_d[r * 3], rays_d[r * 3 + 1], rays_d[r * 3 + 2]);
  float gr[3] = {0.f, 0.f, 0.f};
  if (g_rgb) for (int c = 0; c < 3; ++c) gr[c] = g_rgb[r * 3 + c];
  float ga = g_acc ? g_acc[r] : 0.0f;
  float gd = g_depth ? g_depth[r] : 0.0f;
  if (white) ga -= (gr[0] + gr[1]) + gr[2];          // rgb_map += 1 - acc (VR:353-354)
  if (g_disp) {   // disp = 1 / max(1e-10, depth / acc): through depth / acc where > 1e-10
    const float ac = acc[r], dp = depth[r], q = dp / ac;
    if (q > 1e-10f) {
      const float gq = -g_disp[r] / (q * q);
      gd += gq / ac;
      ga -= gq * dp / (ac * ac);
    }
  }
  double carry = 0.0;   // B at the top index of the block being processed
  for (int b = ((S - 1) / 64) * 64; b >= 0; b -= 64) {
    const int s = b + lane;
    const bool act = s < S;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    float zs = 0.f, dist = 0.f, sig = 0.f, e = 1.f, a = 0.f, ws = 0.f, T = 0.f, G = 0.f;
    float c0 = 0.f, c1 = 0.f, c2 = 0.f;
    if (act) {
      v = rr[s];
      zs = zr[s];
      dist = ((s < S - 1) ? (zr[s + 1] - zs) : 1e10f) * nd;
      sig = fmaxf(v.w, 0.0f);
      e = expf(-sig * dist);
      a = 1.0f - e;
      ws = w[r * S + s];
      T = trans[r * S + s];
      c0 = sigm(v.x);
      c1 = sigm(v.y);
      c2 = sigm(v.z);
      G = (g_w ? g_w[r * S + s] : 0.0f) + gr[0] * c0 + gr[1] * c1 + gr[2] * c2 + ga + gd * zs;
    }
    // h_s = (m, c) = (x_s, G_s a_s); identity past the last sample
    double hm = act ? (double)((1.0f - a) + 1e-10f) : 1.0;
    double hc = act ? (double)G * (double)a : 0.0;
    // reverse inclusive scan: H_s = h_s o h_{s+1} o ... (lane' = 63 - lane)
    double M = __shfl(hm, 63 - lane), C = __shfl(hc, 63 - lane);
    for (int o = 1; o < 64; o <<= 1) {
      const double Mo = __shfl_up(M, o), Co = __shfl_up(C, o);
      if (lane >= o) {   // (this) o (earlier lanes' = higher indices)
        C = C + M * Co;
        M = M * Mo;
      }
    }
    // back to index order: H at lane i; B_i = H_{i+1}(carry), B_top = carry
    const double Mi = __shfl(M, 63 - lane), Ci = __shfl(C, 63 - lane);
    double Mn = __shfl_down(Mi, 1), Cn = __shfl_down(Ci, 1);
    if (lane == 63) { Mn = 1.0; Cn = 0.0; }
    const float B = (float)(Cn + Mn * carry);
    carry = __shfl(Ci, 0) + __shfl(Mi, 0) * carry;   // B_{b-1}
    if (act) {
      const float ga_s = T * (G - B);                    // dL/da_s
      float4 dr;
      dr.x = ws * gr[0] * c0 * (1.0f - c0);
      dr.y = ws * gr[1] * c1 * (1.0f - c1);
      dr.z = ws * gr[2] * c2 * (1.0f - c2);
      dr.w = v.w > 0.0f ? ga_s * dist * e : 0.0f;       // da/dr3 = d e where r3 > 0
      d_raw[r * S + s] = dr;
      L.gd[s] = (s < S - 1) ? ga_s * sig * e * nd : 0.0f;   // dL/d(z[s+1] - z[s])
      L.w[s] = ws;
    }
  }
  if (d_z) {
    __builtin_amdgcn_wave_barrier();
    for (int s = lane; s < S; s += 64)
      d_z[r * S + s] = L.w[s] * gd - L.gd[s] + (s > 0 ? L.gd[s - 1] : 0.0f);
  }
}

// ---------------------------------------------------------------------------
// importance sampling backward (forward: nerf_sample_fine)
// ---------------------------------------------------------------------------
constexpr int PDF_WAVES = 4;
constexpr int PDF_MAX_S = 130;
constexpr int PDF_MAX_IMP = 256;
constexpr int PDF_ROW = PDF_MAX_S + 2;
constexpr int PDF_MAX_ALL = PDF_MAX_S + PDF_MAX_IMP;

struct PdfLds {
  float zc[PDF_ROW];
  float wv[PDF_ROW];
  float cdf[PDF_ROW];
  float bins[PDF_ROW];
  float zf[PDF_MAX_IMP];      // fine samples (u order)
  float4 c01[PDF_MAX_IMP];    // per fine sample: dL/dcdf[below], dL/dcdf[above], below | above << 16
  float gz[PDF_MAX_ALL];      // the ray's row of dL/dz_all
  float za[PDF_MAX_ALL];      // the ray's merged depths (z_all), when given
  float gcdf[PDF_ROW];
  float gpdf[PDF_ROW];
};

__device__ __forceinline__ float wave_tsum_last_pdf(const float* v, int n, int lane) {
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
#pragma unroll
  for (int q = 0; q < 8; ++q) fin = fin + __shfl(part, q);
  return fin;
}

__device__ __forceinline__ double wave_sum_scan_d(double p, int lane) {
  for (int o = 1; o < 64; o <<= 1) {
    const double q = __shfl_up(p, o);
    if (lane >= o) p += q;
  }
  return p;
}

__device__ __forceinline__ int ub(const float* a, int n, float x) {   // # a[i] <= x
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a[mid] <= x) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// d_w [n, S] = dL/dweights of the coarse pass given g_zall [n, S + n_imp]
// (dL/d z_all). z [n, S] coarse depths (per-ray rows), weights [n, S], u [n, n_imp],
// z_all [n, S + n_imp] the forward's merged rows (nullable).
// A fine sample's place in the merged row is its rank among the fine samples
// (ties in u order) + the coarse depths <= it (torch.sort of cat(z, z_f), coarse
// first on ties); with z_all given it is found by one search of the row, the
// rank count over all fine samples only for a sample whose value occurs twice.
// Every row of the ray (depths, its dL/dz_all row, z_all) is staged into LDS at
// the start, so no global load waits inside the per-sample steps.
__global__ __launch_bounds__(64 * PDF_WAVES) void sample_pdf_bwd_kernel(
    const float* __restrict__ z, const float* __restrict__ weights, const float* __restrict__ u,
    const float* __restrict__ g_zall, const float* __restrict__ z_all, int64_t n, int S,
    int n_imp, float* __restrict__ d_w) {
  __shared__ PdfLds sm[PDF_WAVES];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int64_t ray = (int64_t)blockIdx.x * PDF_WAVES + wave;
  if (ray >= n) return;   // wave-uniform; no block barriers below
  PdfLds& L = sm[wave];
  const int nall = S + n_imp;
  const float* zr = z + ray * S;
  const float* wr = weights + ray * S;
  const float* ur = u + ray * n_imp;
  const float* gz = g_zall + ray * (int64_t)nall;
  const int nb = S - 1, nw = S - 2;
  for (int s = lane; s < S; s += 64) L.zc[s] = zr[s];
  for (int s = lane; s < nw; s += 64) L.wv[s] = wr[s + 1] + 1e-5f;
  for (int s = lane; s < nall; s += 64) L.gz[s] = gz[s];
  if (z_all)
    for (int s = lane; s < nall; s += 64) L.za[s] = z_all[ray * (int64_t)nall + s];
  float uj[PDF_MAX_IMP / 64];
#pragma unroll
  for (int q = 0; q < PDF_MAX_IMP / 64; ++q) {
    const int j = lane + 64 * q;
    uj[q] = j < n_imp ? ur[j] : 0.0f;
  }
  __builtin_amdgcn_wave_barrier();
  for (int s = lane; s < nb; s += 64) L.bins[s] = 0.5f * (L.zc[s + 1] + L.zc[s]);
  const float tot = wave_tsum_last_pdf(L.wv, nw, lane);
  double carry = 0.0;
  if (lane == 0) L.cdf[0] = 0.0f;
  for (int b = 0; b < nw; b += 64) {
    const int s = b + lane;
    const double pdf = s < nw ? (double)(L.wv[s] / tot) : 0.0;
    const double inc = carry + wave_sum_scan_d(pdf, lane);
    if (s < nw) L.cdf[s + 1] = (float)inc;
    carry = __shfl(inc, 63);
  }
  __builtin_amdgcn_wave_barrier();
  // recompute each fine sample and the derivatives of its t
  float dc0[PDF_MAX_IMP / 64], dc1[PDF_MAX_IMP / 64], tf[PDF_MAX_IMP / 64];
  int lohi[PDF_MAX_IMP / 64];
#pragma unroll
  for (int q = 0; q < PDF_MAX_IMP / 64; ++q) {
    const int j = lane + 64 * q;
    if (j < n_imp) {
      const int inds = ub(L.cdf, nb, uj[q]);
      const int below = inds - 1 > 0 ? inds - 1 : 0;
      const int above = inds < nb - 1 ? inds : nb - 1;
      const float c0 = L.cdf[below], c1 = L.cdf[above];
      const float b0 = L.bins[below], b1 = L.bins[above];
      const float D = c1 - c0;
      const bool clamped = D < 1e-5f;
      const float den = clamped ? 1.0f : D;
      const float t = (uj[q] - c0) / den;
      L.zf[j] = b0 + t * (b1 - b0);
      lohi[q] = below | (above << 16);
      dc0[q] = clamped ? -1.0f : (t - 1.0f) / den;
      dc1[q] = clamped ? 0.0f : -t / den;
      tf[q] = b1 - b0;   // times dL/dz_f, below
    }
  }
  __builtin_amdgcn_wave_barrier();
  // position of fine sample j in the merged row, its dL/dt, and its two cdf terms
#pragma unroll
  for (int q = 0; q < PDF_MAX_IMP / 64; ++q) {
    const int j = lane + 64 * q;
    if (j < n_imp) {
      const float x = L.zf[j];
      int pos = -1;
      if (z_all) {   // unique value: the last entry <= x is this sample
        const int up = ub(L.za, nall, x);
        if (up >= 1 && L.za[up - 1] == x && (up < 2 || L.za[up - 2] != x)) pos = up - 1;
      }
      if (pos < 0) {
        int rank = 0;
#pragma unroll 8
        for (int k = 0; k < n_imp; ++k) {
          const float y = L.zf[k];
          rank += (y < x) || (y == x && k < j);
        }
        pos = rank + ub(L.zc, S, x);
      }
      const float gt = tf[q] * L.gz[pos];
      L.c01[j] = make_float4(gt * dc0[q], gt * dc1[q], __int_as_float(lohi[q]), 0.0f);
    }
  }
  __builtin_amdgcn_wave_barrier();
  // dL/dcdf[k], summed in sample order (deterministic): one 16-B broadcast read per sample
  for (int k = lane; k < nb; k += 64) {
    float acc = 0.0f;
#pragma unroll 8
    for (int j = 0; j < n_imp; ++j) {
      const float4 c = L.c01[j];
      const int lh = __float_as_int(c.z);
      if ((lh & 0xffff) == k) acc += c.x;
      if ((lh >> 16) == k) acc += c.y;
    }
    L.gcdf[k] = acc;
  }
  __builtin_amdgcn_wave_barrier();
  // cdf[k] = sum_{i<k} pdf[i]: dL/dpdf[i] = sum_{k>i} dL/dcdf[k] (reverse cumsum)
  double rc = 0.0;
  for (int b = ((nw - 1) / 64) * 64; b >= 0; b -= 64) {
    const int i = b + lane;
    const double v = (i < nw) ? (double)L.gcdf[i + 1] : 0.0;
    // suffix sum within the block: reverse the lane order for an inclusive scan
    const double rv = __shfl(v, 63 - lane);
    const double sc = wave_sum_scan_d(rv, lane);
    const double suf = __shfl(sc, 63 - lane) + rc;
    if (i < nw) L.gpdf[i] = (float)suf;
    rc = rc + __shfl(sc, 63);
  }
  __builtin_amdgcn_wave_barrier();
  // pdf = w' / tot: dL/dw'_i = (gpdf_i - sum_m gpdf_m w'_m / tot) / tot
  float part = 0.0f;
  for (int i = lane; i < nw; i += 64) part += L.gpdf[i] * L.wv[i];
  for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o);
  const float mean = part / tot;
  float* dw = d_w + ray * S;
  for (int s = lane; s < S; s += 64) {
    const int i = s - 1;
    dw[s] = (i >= 0 && i < nw) ? (L.gpdf[i] - mean) / tot : 0.0f;
  }
}

// The training loss (trainers/nerf.py:39-76): mean squared error of the
// coarse and the fine rgb against the target, and their sum, in ONE workgroup
// (n * 3 elements; float32 per-thread sums, then a fixed tree over the block);
// its backward: d a = (2 / N) * (a - t) * g for both maps in one launch
// (torch's mse_loss_backward: norm * (input - target) * grad_output).
constexpr int kMseThreads = 1024;
__global__ __launch_bounds__(kMseThreads) void mse_pair_kernel(const float* __restrict__ a,
                                                              const float* __restrict__ b,
                                                              const float* __restrict__ t,
                                                              int64_t N, float* __restrict__ out) {
  __shared__ float sa[kMseThreads], sb[kMseThreads];
  float ua = 0.0f, ub = 0.0f;
  for (int64_t i = threadIdx.x; i < N; i += kMseThreads) {
    const float da = a[i] - t[i];
    ua += da * da;
    if (b) {
      const float db = b[i] - t[i];
      ub += db * db;
    }
  }
  sa[threadIdx.x] = ua;
  sb[threadIdx.x] = ub;
  __syncthreads();
  for (int o = kMseThreads / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      sa[threadIdx.x] += sa[threadIdx.x + o];
      sb[threadIdx.x] += sb[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float lc = sa[0] / (float)N, lf = sb[0] / (float)N;
    out[0] = lc;
    out[1] = lf;
    out[2] = b ? lc + lf : lc;
  }
}

__global__ __launch_bounds__(256) void mse_pair_bwd_kernel(const float* __restrict__ a,
                                                           const float* __restrict__ b,
                                                           const float* __restrict__ t, int64_t N,
                                                           const float* __restrict__ g0,
                                                           const float* __restrict__ g1,
                                                           const float* __restrict__ g2,
                                                           float* __restrict__ da,
                                                           float* __restrict__ db) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const float norm = 2.0f / (float)N;
  // d loss_c, d loss_f, d (loss_c + loss_f); a null gradient is 0
  const float l = g2 ? *g2 : 0.0f;
  const float gc = g0 ? *g0 + l : l, gf = g1 ? *g1 + l : l;
  da[i] = norm * (a[i] - t[i]) * gc;
  if (b) db[i] = norm * (b[i] - t[i]) * gf;
}

extern "C" {

int nerf_mse_pair(const float* a, const float* b, const float* target, int64_t N, float* out,
                  nerf_stream_t stream) {
  NERF_REQUIRE(a && target && out && N > 0, "nerf_mse_pair: bad arguments");
  hipLaunchKernelGGL(mse_pair_kernel, dim3(1), dim3(kMseThreads), 0, as_stream(stream), a, b,
                     target, N, out);
  return check_launch("mse_pair_kernel");
}

int nerf_mse_pair_backward(const float* a, const float* b, const float* target, int64_t N,
                           const float* g0, const float* g1, const float* g2, float* da,
                           float* db, nerf_stream_t stream) {
  NERF_REQUIRE(a && target && da && (!b || db) && N > 0, "nerf_mse_pair_backward: bad arguments");
  hipLaunchKernelGGL(mse_pair_bwd_kernel, dim3((unsigned)cdiv(N, 256)), dim3(256), 0,
                     as_stream(stream), a, b, target, N, g0, g1, g2, da, db);
  return check_launch("mse_pair_bwd_kernel");
}

int nerf_composite_train_fwd(const float* raw, const float* z, const float* rays_d, int64_t n,
                             int S, int white, float* rgb, float* disp, float* acc, float* depth,
                             float* weights, float* trans, nerf_stream_t stream) {
  NERF_REQUIRE(raw && z && rays_d && rgb && disp && acc && depth && weights && trans,
               "nerf_composite_train_fwd: null pointer");
  NERF_REQUIRE(n >= 0 && S >= 1 && S <= CT_MAX_S, "nerf_composite_train_fwd: bad size");
  if (n == 0) return 0;
  hipLaunchKernelGGL(composite_train_fwd_kernel, dim3((unsigned)cdiv(n, CT_WAVES)),
                     dim3(64 * CT_WAVES), 0,
                     as_stream(stream), (const float4*)raw, z, rays_d, n, S, white, rgb, disp,
                     acc, depth, weights, trans);
  return check_launch("composite_train_fwd_kernel");
}

int nerf_composite_train_bwd(const float* raw, const float* z, const float* rays_d,
                             const float* weights, const float* trans, const float* acc,
                             const float* depth,
                             int64_t n, int S, int white, const float* g_rgb, const float* g_disp,
                             const float* g_acc, const float* g_depth, const float* g_weights,
                             float* d_raw, float* d_z, nerf_stream_t stream) {
  NERF_REQUIRE(raw && z && rays_d && weights && trans && acc && depth && d_raw,
               "nerf_composite_train_bwd: null pointer");
  NERF_REQUIRE(n >= 0 && S >= 1 && S <= CT_MAX_S, "nerf_composite_train_bwd: bad size");
  if (n == 0) return 0;
  hipLaunchKernelGGL(composite_train_bwd_kernel, dim3((unsigned)cdiv(n, CT_WAVES)),
                     dim3(64 * CT_WAVES), 0,
                     as_stream(stream), (const float4*)raw, z, rays_d, weights, trans, acc, depth,
                     n, S,
                     white, g_rgb, g_disp, g_acc, g_depth, g_weights, (float4*)d_raw, d_z);
  return check_launch("composite_train_bwd_kernel");
}

int nerf_sample_pdf_bwd(const float* z, const float* weights, const float* u,
                        const float* g_zall, const float* z_all, int64_t n, int S, int n_imp,
                        float* d_weights, nerf_stream_t stream) {
  NERF_REQUIRE(z && weights && u && g_zall && d_weights, "nerf_sample_pdf_bwd: null pointer");
  NERF_REQUIRE(n >= 0 && S >= 3 && S <= PDF_MAX_S && n_imp >= 1 && n_imp <= PDF_MAX_IMP,
               "nerf_sample_pdf_bwd: bad size");
  if (n == 0) return 0;
  hipLaunchKernelGGL(sample_pdf_bwd_kernel, dim3((unsigned)cdiv(n, PDF_WAVES)),
                     dim3(64 * PDF_WAVES), 0, as_stream(stream), z, weights, u, g_zall, z_all, n,
                     S, n_imp, d_weights);
  return check_launch("sample_pdf_bwd_kernel");
}

// out[i] = sum over c = 0..C-1 (in that order) of part[c * n + i]: the split-K
// partials of the weight-gradient kernel summed in a fixed order. One output
// per lane, 8 partials in flight per lane (the partials are re-read right
// after they were written, mostly from the Infinity Cache).
__global__ __launch_bounds__(256) void sum_partials_kernel(const float* __restrict__ part,
                                                           int64_t C, int64_t n,
                                                           float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float* p = part + i;
  float s = 0.0f;
  int64_t c = 0;
  for (; c + 8 <= C; c += 8) {
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = p[(c + k) * n];
#pragma unroll
    for (int k = 0; k < 8; ++k) s += v[k];
  }
  for (; c < C; ++c) s += p[c * n];
  out[i] = s;
}

// The views / feature / alpha weight gradients from the merged G tile of the
// batched weight-gradient launch (nerfhip.train_mlp, NET:61-65): GA = [d_hv;
// d sigma] [h7; view enc]^T ([129][288], row stride ldga), ba = its row sums
// ([129]); feature = W_f h7 + b_f feeds the views layer, so with Gh = GA[0:128,
// 0:256] and s = ba[0:128]:
//   dW_views = [Gh W_f^T + s b_f^T, GA[0:128, 256:283]],  db_views = s,
//   dW_f = W_views[:, :256]^T Gh,  db_f = W_views[:, :256]^T s,
//   dW_alpha = GA[128, 0:256],  db_alpha = ba[128].
// One launch in place of two small hipBLASLt GEMMs, a GEMV and the copies
// around them. The two products run as 32 x 32 output tiles (dW_views,feat:
// 4 x 8 tiles over K = 256; dW_f: 8 x 8 over K = 128), both operands' whole K
// extent staged through LDS at once (every load of a thread in flight
// together: a chunked K loop exposed one load latency per chunk), each thread
// 2 x 2 outputs, every output one FP32 FMA chain in ascending k (the order of
// a one-thread-per-output loop); one more workgroup takes db_f (a GEMV,
// ascending i) and the copies.
constexpr int kVfTilesV = 4 * 8, kVfTilesF = 8 * 8;
__global__ __launch_bounds__(256) void views_feature_grads_kernel(
    const float* __restrict__ GA, int64_t ldga, const float* __restrict__ ba,
    const float* __restrict__ Wf, const float* __restrict__ bf, const float* __restrict__ Wv,
    float* __restrict__ dWv, float* __restrict__ dWf, float* __restrict__ dbf,
    float* __restrict__ dWa, float* __restrict__ dba, float* __restrict__ dbv,
    const float* __restrict__ GE, int64_t ldge, const float* __restrict__ be,
    float* __restrict__ dWr, float* __restrict__ dbr) {
  const int t = threadIdx.x;
  const int blk = blockIdx.x;
  if (blk == kVfTilesV + kVfTilesF) {   // db_f, the copies
    float acc = 0.0f;
#pragma unroll 32
    for (int i = 0; i < 128; ++i) acc = __builtin_fmaf(Wv[(int64_t)i * 283 + t], ba[i], acc);
    dbf[t] = acc;
    dWa[t] = GA[128 * ldga + t];
    if (t < 128) dbv[t] = ba[t];
    if (t == 0) dba[0] = ba[128];
    for (int e = t; e < 128 * 27; e += 256) {
      const int i = e / 27, j = e % 27;
      dWv[i * 283 + 256 + j] = GE ? GE[(int64_t)i * ldge + j] : GA[(int64_t)i * ldga + 256 + j];
    }
    if (GE) {   // the rgb head from the shared tile: rows 144..146 x columns 32..159
      for (int e = t; e < 3 * 128; e += 256)
        dWr[e] = GE[(int64_t)(144 + e / 128) * ldge + 32 + e % 128];
      if (t < 3) dbr[t] = be[144 + t];
    }
    return;
  }
  // C[m][n] = sum_k A(m, k) B(k, n) over a 32 x 32 tile
  const bool views = blk < kVfTilesV;
  const int tile = views ? blk : blk - kVfTilesV;
  const int m0 = 32 * (tile >> 3), n0 = 32 * (tile & 7);
  const int K = views ? 256 : 128;
  // 67.6 KB: gfx950's 160 KiB per workgroup (the Makefile builds for gfx950 only)
  __shared__ float As[256][33], Bs[256][33];   // As[k][m], Bs[k][n]
  static_assert(sizeof(As) + sizeof(Bs) <= 160 * 1024, "gfx950 LDS per workgroup");
  const int tm = t >> 4, tn = t & 15;          // outputs (m0 + 2 tm + a, n0 + 2 tn + b)
  if (views) {
    // A(m, k) = GA[m][k], B(k, n) = W_f[n][k] (k contiguous): 32 rows x 256 k each
#pragma unroll 8
    for (int q = 0; q < 32; ++q) {
      const int e = t + 256 * q, r = e >> 8, c = e & 255;
      As[c][r] = GA[(int64_t)(m0 + r) * ldga + c];
      Bs[c][r] = Wf[(int64_t)(n0 + r) * 256 + c];
    }
  } else {
    // A(m, k) = W_views[k][m], B(k, n) = GA[k][n] (m / n contiguous): 128 k x 32
#pragma unroll 8
    for (int q = 0; q < 16; ++q) {
      const int e = t + 256 * q, r = e >> 5, c = e & 31;
      As[r][c] = Wv[(int64_t)r * 283 + m0 + c];
      Bs[r][c] = GA[(int64_t)r * ldga + n0 + c];
    }
  }
  __syncthreads();
  float acc[2][2] = {{0.0f, 0.0f}, {0.0f, 0.0f}};
#pragma unroll 8
  for (int k = 0; k < K; ++k) {
    const float a0 = As[k][2 * tm], a1 = As[k][2 * tm + 1];
    const float b0 = Bs[k][2 * tn], b1 = Bs[k][2 * tn + 1];
    acc[0][0] = __builtin_fmaf(a0, b0, acc[0][0]);
    acc[0][1] = __builtin_fmaf(a0, b1, acc[0][1]);
    acc[1][0] = __builtin_fmaf(a1, b0, acc[1][0]);
    acc[1][1] = __builtin_fmaf(a1, b1, acc[1][1]);
  }
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int m = m0 + 2 * tm + a, n = n0 + 2 * tn + b;
      if (views) dWv[m * 283 + n] = __builtin_fmaf(ba[m], bf[n], acc[a][b]);
      else dWf[m * 256 + n] = acc[a][b];
    }
}

int nerf_views_feature_grads(const float* GA, int64_t ldga, const float* ba, const float* Wf,
                             const float* bf, const float* Wv, float* dWv, float* dWf, float* dbf,
                             float* dWa, float* dba, float* dbv, const float* GE, int64_t ldge,
                             const float* be, float* dWr, float* dbr, nerf_stream_t stream) {
  NERF_REQUIRE(GA && ba && Wf && bf && Wv && dWv && dWf && dbf && dWa && dba && dbv &&
                   ldga >= (GE ? 256 : 283) && (!GE || (ldge >= 160 && be && dWr && dbr)),
               "nerf_views_feature_grads: bad arguments");
  hipLaunchKernelGGL(views_feature_grads_kernel, dim3(kVfTilesV + kVfTilesF + 1), dim3(256), 0,
                     as_stream(stream), GA, ldga, ba, Wf, bf, Wv, dWv, dWf, dbf, dWa, dba, dbv,
                     GE, ldge, be, dWr, dbr);
  return check_launch("views_feature_grads_kernel");
}

int nerf_sum_partials(const float* part, int64_t C, int64_t n, float* out, nerf_stream_t stream) {
  NERF_REQUIRE(part && out, "nerf_sum_partials: null pointer");
  NERF_REQUIRE(C >= 1 && n >= 0, "nerf_sum_partials: bad size");
  if (n == 0) return 0;
  hipLaunchKernelGGL(sum_partials_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0,
                     as_stream(stream), part, C, n, out);
  return check_launch("sum_partials_kernel");
}

int nerf_adam_step(const NerfAdamTensor* tensors, int n, const float* lr, float* step,
                   unsigned* done, double beta1, double beta2, float eps, float clip,
                   nerf_stream_t stream);

}  // extern "C"

// One Adam step (trainers' torch.optim.Adam, weight decay 0, no amsgrad) over
// every parameter of the step in ONE launch, the gradient first clamped to
// [-clip, clip] in place (clip_grad_value_, trainer.py:59; clip < 0: none,
// clip 0 zeroes every gradient as clip_grad_value_(0) does),
// in torch's single-tensor Adam's float32 operation order (lerp, mul +
// addcmul, addcdiv; the bias corrections in double, as its Python scalars):
//   m = m + (1 - b1) (g - m),  v = v b2 + (1 - b2) g g,
//   p = p - lr / (1 - b1^t) * (m / (sqrt(v) / sqrt(1 - b2^t) + eps)),  t = step + 1.
// lr and the step count live on the device (a HIP graph replays the launch);
// adam_advance_kernel then writes step = t (an arrival counter letting the
// last workgroup write it measured slower: ~1 200 workgroups' atomics on one
// word, 21 vs 13 + 5 µs).
constexpr int kAdamMax = 64;
constexpr int kAdamPer = 4;                 // elements per thread, loaded together
constexpr int kAdamBlock = 256 * kAdamPer;  // elements per workgroup (~1 200 workgroups for
                                            // both networks)
struct AdamBatch {
  NerfAdamTensor t[kAdamMax];
  int blk_end[kAdamMax];           // prefix sums of the tensors' workgroups
  int nt;
};

// Every load of a thread is issued before any of its stores (the tensors are
// distinct arrays, declared so): one HBM latency per thread instead of one per
// element, which a loop with a store between dependent loads would expose.
__global__ __launch_bounds__(256) void adam_kernel(const AdamBatch b, const float* __restrict__ lr,
                                                   const float* __restrict__ step, double beta1,
                                                   double beta2, float eps, float clip) {
  const int blk = (int)blockIdx.x;
  int k = 0;
  while (k + 1 < b.nt && blk >= b.blk_end[k]) ++k;
  const NerfAdamTensor& T = b.t[k];
  const int64_t base = (int64_t)(blk - (k ? b.blk_end[k - 1] : 0)) * kAdamBlock;
  float* __restrict__ P = T.p;
  float* __restrict__ G = T.g;
  float* __restrict__ M = T.m;
  float* __restrict__ V = T.v;
  // the bias corrections in double, as torch's Python scalars (every thread: no
  // LDS round trip and barrier in front of the loads)
  const float t = *step + 1.0f;
  const float step_size = (float)((double)*lr / (1.0 - pow(beta1, (double)t)));
  const float bc2s = (float)sqrt(1.0 - pow(beta2, (double)t));
  const float w1 = (float)(1.0 - beta1), w2 = (float)(1.0 - beta2), b2 = (float)beta2;

  float g[kAdamPer], m0[kAdamPer], v0[kAdamPer], p0[kAdamPer];
#pragma unroll
  for (int r = 0; r < kAdamPer; ++r) {
    const int64_t i = base + r * 256 + threadIdx.x;
    const bool in = i < T.n;
    g[r] = in ? G[i] : 0.0f;
    m0[r] = in ? M[i] : 0.0f;
    v0[r] = in ? V[i] : 0.0f;
    p0[r] = in ? P[i] : 0.0f;
  }
#pragma unroll
  for (int r = 0; r < kAdamPer; ++r) {
    const int64_t i = base + r * 256 + threadIdx.x;
    if (i < T.n) {
      float gr = g[r];
      if (clip >= 0.0f) {   // torch.clamp keeps a NaN (fminf/fmaxf would drop it)
        gr = (gr != gr) ? gr : fminf(fmaxf(gr, -clip), clip);
        G[i] = gr;
      }
      const float m = m0[r] + w1 * (gr - m0[r]);          // lerp (weight < 0.5)
      const float v = v0[r] * b2 + (w2 * gr) * gr;        // mul_, addcmul_
      M[i] = m;
      V[i] = v;
      const float denom = sqrtf(v) / bc2s + eps;
      P[i] = p0[r] + (-step_size) * (m / denom);          // addcdiv_
    }
  }
}

// step = t after every workgroup of the step has read the old count: the next
// launch on the stream (a device-wide fence + finish counter per workgroup, as
// round 3 had it, cost ~30 us: on gfx950 the release writes the XCD's L2 back)
__global__ void adam_advance_kernel(float* __restrict__ step) { *step = *step + 1.0f; }

extern "C" int nerf_adam_step(const NerfAdamTensor* tensors, int n, const float* lr, float* step,
                              unsigned* done, double beta1, double beta2, float eps, float clip,
                              nerf_stream_t stream) {
  NERF_REQUIRE(tensors && lr && step && n >= 1 && n <= kAdamMax,
               "nerf_adam_step: bad arguments");
  AdamBatch b;
  int blocks = 0;
  for (int k = 0; k < n; ++k) {
    const NerfAdamTensor& T = tensors[k];
    NERF_REQUIRE(T.p && T.g && T.m && T.v && T.n >= 0 && T.n < (1ll << 31),
                 "nerf_adam_step: bad tensor");
    b.t[k] = T;
    blocks += (int)cdiv(T.n, kAdamBlock);
    b.blk_end[k] = blocks;
  }
  b.nt = n;
  if (blocks == 0) return 0;
  (void)done;
  hipLaunchKernelGGL(adam_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), b, lr,
                     step, beta1, beta2, eps, clip);
  hipLaunchKernelGGL(adam_advance_kernel, dim3(1), dim3(1), 0, as_stream(stream), step);
  return check_launch("adam_kernel");
}

// The training forward's per-step fold of the feature layer into the views
// layer (network.py:63-67: feature = W_f h7 + b_f has no activation, so
// W_v [feat | dir] . cat(feature, d) + b_v = (W_v,feat W_f) h7 + W_v,dir d +
// (W_v,feat b_f + b_v)): Wc [128][283] = [W_v,feat W_f | W_v,dir] and
// bc = W_v,feat b_f + b_v from the live parameters, FP32
// (nerfhip.pack.fold_feature_into_views does the same map in float64 for
// inference). Block (4 rows, 64 columns, network): wave w sums k in
// [64 w, 64 w + 64) for column j = its lane (W_f read by row segments,
// coalesced, all 64 loads in flight), the 4 partial sums added in wave order
// through LDS; the column-group-0 blocks also take the bias (wave w: row w, a
// 64-lane split of the sum, then a butterfly) and copy the direction columns.
constexpr int kFoldMax = 4;
constexpr int kFoldRows = 4;
struct FoldBatch {
  NerfFoldDesc d[kFoldMax];
};

__global__ __launch_bounds__(256) void fold_views_kernel(const FoldBatch fb) {
  const NerfFoldDesc& d = fb.d[blockIdx.z];
  const int m0 = blockIdx.x * kFoldRows, j0 = blockIdx.y * 64, t = threadIdx.x;
  const int w = t >> 6, lane = t & 63;
  __shared__ float wrow[kFoldRows][256];
  __shared__ float part[4][kFoldRows][64];
#pragma unroll
  for (int r = 0; r < kFoldRows; ++r) wrow[r][t] = d.Wv[(m0 + r) * 283 + t];
  float wf[64];
#pragma unroll
  for (int k = 0; k < 64; ++k) wf[k] = d.Wf[(64 * w + k) * 256 + j0 + lane];
  __syncthreads();
  float acc[kFoldRows] = {};
#pragma unroll
  for (int k = 0; k < 64; ++k)
#pragma unroll
    for (int r = 0; r < kFoldRows; ++r) acc[r] = __builtin_fmaf(wrow[r][64 * w + k], wf[k], acc[r]);
#pragma unroll
  for (int r = 0; r < kFoldRows; ++r) part[w][r][lane] = acc[r];
  __syncthreads();
  {
    const int r = w;   // wave w writes row m0 + w
    const float v = ((part[0][r][lane] + part[1][r][lane]) + part[2][r][lane]) + part[3][r][lane];
    d.Wc[(m0 + r) * 283 + j0 + lane] = v;
  }
  if (blockIdx.y != 0) return;
  if (t < 27) {
#pragma unroll
    for (int r = 0; r < kFoldRows; ++r)
      d.Wc[(m0 + r) * 283 + 256 + t] = d.Wv[(m0 + r) * 283 + 256 + t];
  }
  float b = 0.0f;
#pragma unroll
  for (int q = 0; q < 4; ++q) b = __builtin_fmaf(wrow[w][lane * 4 + q], d.bf[lane * 4 + q], b);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) b += __shfl_xor(b, o);
  if (lane == 0) d.bc[m0 + w] = b + d.bv[m0 + w];
}

extern "C" int nerf_fold_views(const NerfFoldDesc* nets, int n, nerf_stream_t stream) {
  NERF_REQUIRE(nets && n >= 1 && n <= kFoldMax, "nerf_fold_views: bad arguments");
  FoldBatch fb;
  for (int k = 0; k < n; ++k) {
    const NerfFoldDesc& d = nets[k];
    NERF_REQUIRE(d.Wv && d.Wf && d.bf && d.bv && d.Wc && d.bc, "nerf_fold_views: null pointer");
    fb.d[k] = d;
  }
  hipLaunchKernelGGL(fold_views_kernel, dim3(128 / kFoldRows, 4, (unsigned)n), dim3(256), 0, as_stream(stream),
                     fb);
  return check_launch("fold_views_kernel");
}

}  // namespace nerfhip
