// The reference extension's op contract (`kilonerf_cuda`, cuda/pybind.cu:13-38)
// as native gfx950 kernels behind the C ABI.
//
// Semantics follow the CUDA sources with nvcc's default contraction made
// explicit (a += b*c -> fmaf) since this library builds with -ffp-contract=off.
// Deliberate differences, documented in DESIGN.md: accurate sinf/cosf/expf
// instead of the __sinf/__cosf/__expf fast paths (network_eval.cu:136-139,
// integrate.cu:37); per-call parameters are kernel arguments instead of
// __constant__ uploads; the aliased `extern __shared__` min/max arrays
// (global_to_local.cu:14-15, network_eval.cu:54-55) are replaced by their
// intended per-network values; the MAGMA grouped GEMM / GEMV and the thrust
// reorder primitives are native kernels.
#include <hip/hip_runtime.h>

#include <map>
#include <mutex>
#include <vector>

#include "common.h"

namespace nerfhip {

// ---------------------------------------------------------------------------
// get_rays_d (generate_inputs.cu:11-52)
// ---------------------------------------------------------------------------
__global__ void kn_rays_d_kernel(int H, int W, float cx, float cy, float fx, float fy,
                                 const float* __restrict__ c2w, float* __restrict__ out) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= (int64_t)H * W) return;
  const int x = (int)(p % W), y = (int)(p / W);
  const float in0 = ((float)x - cx) / fx;
  const float in1 = -((float)y - cy) / fy;
  const float in2 = -1.0f;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    float o = in0 * c2w[i * 3 + 0];
    o = __builtin_fmaf(in1, c2w[i * 3 + 1], o);
    o = __builtin_fmaf(in2, c2w[i * 3 + 2], o);
    out[p * 3 + i] = o;
  }
}

// ---------------------------------------------------------------------------
// generate_query_indices_on_ray (generate_inputs.cu:60-126)
// ---------------------------------------------------------------------------
__global__ void kn_query_indices_kernel(const float* __restrict__ origin,
                                        const float* __restrict__ dirs,
                                        const int16_t* __restrict__ grid,
                                        uint8_t* __restrict__ active, int16_t* __restrict__ depth_idx,
                                        const float* __restrict__ vsize,
                                        const float* __restrict__ gmin,
                                        const float* __restrict__ gmax,
                                        const int32_t* __restrict__ strides, int num_rays,
                                        float step, int max_samples, int max_depth,
                                        float min_dist, int initial, int32_t* __restrict__ qidx,
                                        int16_t* __restrict__ nets) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= num_rays) return;
  int out = idx * max_samples;
  const int out_end = out + max_samples;
  const bool act = initial ? true : (active[idx] != 0);
  if (act) {
    const float d0 = dirs[3 * idx], d1 = dirs[3 * idx + 1], d2 = dirs[3 * idx + 2];
    int depth = initial ? 0 : depth_idx[idx];
    float dist = __builtin_fmaf((float)depth, step, min_dist);
    while (depth < max_depth && out < out_end) {
      int flat = 0;
      bool inside = true;
      const float dv[3] = {d0, d1, d2};
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float pc = __builtin_fmaf(dist, dv[c], origin[c]);
        const int vi = (int)((pc - gmin[c]) / vsize[c]);
        flat += vi * strides[c];
        const float eps = 0.001f;
        inside = inside && (gmin[c] + eps < pc) && (pc < gmax[c] - eps);
      }
      const int16_t net = inside ? grid[flat] : (int16_t)-1;
      if (net != -1) {
        nets[out] = net;
        qidx[out] = idx * max_depth + depth;
        ++out;
      }
      ++depth;
      dist = dist + step;
    }
    if (out < out_end) {
      active[idx] = 0;
    } else {
      active[idx] = 1;
      depth_idx[idx] = (int16_t)depth;
    }
  }
  while (out < out_end) nets[out++] = -1;
}

// ---------------------------------------------------------------------------
// compute_fourier_features (fourier_features.cu:8-100): LDS-staged so the
// (2L+1)-float rows leave as coalesced 16-byte stores
// ---------------------------------------------------------------------------
constexpr int FF_BLOCK = 256;

__global__ __launch_bounds__(FF_BLOCK) void kn_fourier_kernel(const float* __restrict__ in,
                                                              int64_t n,
                                                              const float* __restrict__ freqs,
                                                              int L, float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float ff_smem[];
  const int per = 2 * L + 1;
  const int64_t i0 = (int64_t)blockIdx.x * FF_BLOCK;
  const int cnt = (int)((n - i0) < FF_BLOCK ? (n - i0) : FF_BLOCK);
  const int t = threadIdx.x;
  if (t < cnt) {
    const float x = in[i0 + t];
    float* row = ff_smem + t * per;
    row[0] = x;
    for (int r = 0; r < L; ++r) {
      float s, c;
      sincosf(freqs[r] * x, &s, &c);
      row[1 + r] = c;
      row[1 + L + r] = s;
    }
  }
  __syncthreads();
  const int64_t base = i0 * per;
  const int total = cnt * per;
  float* dst = out + base;
  // scalar head up to 16-byte alignment, float4 body, scalar tail
  const int head = (int)((4 - (base & 3)) & 3) < total ? (int)((4 - (base & 3)) & 3) : total;
  for (int k = t; k < head; k += FF_BLOCK) dst[k] = ff_smem[k];
  const int nvec = (total - head) >> 2;
  for (int k = t; k < nvec; k += FF_BLOCK) {
    const int o = head + 4 * k;
    reinterpret_cast<float4*>(dst + head)[k] =
        make_float4(ff_smem[o], ff_smem[o + 1], ff_smem[o + 2], ff_smem[o + 3]);
  }
  for (int k = head + 4 * nvec + t; k < total; k += FF_BLOCK) dst[k] = ff_smem[k];
}

// ---------------------------------------------------------------------------
// integrate + replace_transparency_by_background_color (integrate.cu:9-112)
// ---------------------------------------------------------------------------
// One thread per ray, as the reference (its per-sample float recurrence for T
// is kept bit-for-bit), but each wave stages its 64 rays' samples through LDS
// in 8-sample chunks: the global loads are whole 128-B lines (8 lanes per ray
// chunk) instead of 64 rays' scattered 16-B pieces per instruction.
constexpr int KI_CHUNK = 8;
constexpr int KI_WAVES = 4;

__global__ __launch_bounds__(64 * KI_WAVES) void kn_integrate_kernel(
    const float4* __restrict__ rgb_sigma, const float* __restrict__ dists,
    float* __restrict__ rgb_map, float* __restrict__ acc_map, float* __restrict__ trans,
    uint8_t* __restrict__ mask, int num_rays, int spr, float thr, int initial) {
  __shared__ float4 stage[KI_WAVES][64][KI_CHUNK + 1];   // +1: spread the rows over banks
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int ray0 = (blockIdx.x * KI_WAVES + wave) * 64;
  if (ray0 >= num_rays) return;   // wave-uniform
  const int ray = ray0 + lane;
  const bool in = ray < num_rays;
  float T = in ? (initial ? 1.0f : trans[ray]) : 0.0f;
  const bool act = in && T > thr;
  float r = 0.f, g = 0.f, b = 0.f, acc = 0.f;
  if (act && !initial) {
    r = rgb_map[ray * 3];
    g = rgb_map[ray * 3 + 1];
    b = rgb_map[ray * 3 + 2];
    acc = acc_map[ray];
  }
  const float dist = in ? dists[ray] : 0.f;
  const uint64_t need = __ballot(act);
  for (int c0 = 0; c0 < spr && need; c0 += KI_CHUNK) {
    const int cn = spr - c0 < KI_CHUNK ? spr - c0 : KI_CHUNK;
    // cooperative load: element e = (ray_local, s) with s fastest
    for (int e = lane; e < 64 * KI_CHUNK; e += 64) {
      const int rl = e / KI_CHUNK, sl = e % KI_CHUNK;
      if (sl < cn && ray0 + rl < num_rays && ((need >> rl) & 1))
        stage[wave][rl][sl] = rgb_sigma[(int64_t)(ray0 + rl) * spr + c0 + sl];
    }
    __builtin_amdgcn_wave_barrier();
    if (act) {
      for (int sl = 0; sl < cn; ++sl) {
        const float4 v = stage[wave][lane][sl];
        const float alpha = 1.0f - expf(-v.w * dist);
        const float w = alpha * T;
        // `T *= 1.0f - alpha + 1e-10` is evaluated in double (1e-10 is a double literal)
        T = (float)((double)T * ((double)(1.0f - alpha) + 1e-10));
        r = __builtin_fmaf(v.x, w, r);
        g = __builtin_fmaf(v.y, w, g);
        b = __builtin_fmaf(v.z, w, b);
        acc = acc + w;
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
  if (act) {
    trans[ray] = T;
    if (T <= thr) mask[ray] = 0;
  }
  if (act || (in && initial)) {
    rgb_map[ray * 3] = r;
    rgb_map[ray * 3 + 1] = g;
    rgb_map[ray * 3 + 2] = b;
    acc_map[ray] = acc;
  }
}

__global__ void kn_background_kernel(float* __restrict__ rgb, const float* __restrict__ acc,
                                     int64_t n, const float* __restrict__ bg) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float t = 1.0f - acc[i];
#pragma unroll
  for (int c = 0; c < 3; ++c) rgb[i * 3 + c] = __builtin_fmaf(bg[c], t, rgb[i * 3 + c]);
}

// ---------------------------------------------------------------------------
// reorder (reorder.cu:13-49)
// ---------------------------------------------------------------------------
__global__ void kn_gather_kernel(const int32_t* __restrict__ map, int64_t n,
                                 const int32_t* __restrict__ in, int32_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = in[map[i]];
}

__global__ void kn_scatter_kernel(const int32_t* __restrict__ map, int64_t n,
                                  const float4* __restrict__ in, float4* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[map[i]] = in[i];
}

// Stable LSD radix sort on 16-bit keys: 4 passes of 4-bit digits.
// pass: per-tile digit histograms -> one exclusive scan in digit-major order ->
// stable scatter (in-tile ranks from 64-lane ballots, wave/sub-tile order kept).
constexpr int RS_TILE = 1024;
constexpr int RS_BLOCK = 256;
constexpr int RS_DIGITS = 16;

__device__ __forceinline__ int rs_digit(int16_t k, int shift) {
  return (int)((((uint16_t)k) ^ 0x8000u) >> shift) & 15;
}

__global__ __launch_bounds__(RS_BLOCK) void rs_hist_kernel(const int16_t* __restrict__ keys,
                                                           int64_t n, int shift,
                                                           uint32_t* __restrict__ hist,
                                                           int ntiles) {
  __shared__ uint32_t h[RS_DIGITS];
  if (threadIdx.x < RS_DIGITS) h[threadIdx.x] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * RS_TILE;
  for (int k = threadIdx.x; k < RS_TILE; k += RS_BLOCK) {
    const int64_t i = base + k;
    if (i < n) atomicAdd(&h[rs_digit(keys[i], shift)], 1u);
  }
  __syncthreads();
  if (threadIdx.x < RS_DIGITS) hist[(int64_t)threadIdx.x * ntiles + blockIdx.x] = h[threadIdx.x];
}

__global__ __launch_bounds__(1024) void rs_scan_kernel(uint32_t* __restrict__ hist, int64_t len) {
  // single-block exclusive scan (hist has 16 * ntiles entries)
  __shared__ uint32_t part[1024];
  const int t = threadIdx.x;
  const int64_t per = (len + 1023) / 1024;
  const int64_t b = t * per, e = (b + per < len) ? b + per : len;
  uint32_t s = 0;
  for (int64_t i = b; i < e; ++i) s += hist[i];
  part[t] = s;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    const uint32_t v = t >= off ? part[t - off] : 0u;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint32_t run = part[t] - s;
  for (int64_t i = b; i < e; ++i) {
    const uint32_t v = hist[i];
    hist[i] = run;
    run += v;
  }
}

template <typename V>
__global__ __launch_bounds__(RS_BLOCK) void rs_scatter_kernel(
    const int16_t* __restrict__ kin, const V* __restrict__ vin, int16_t* __restrict__ kout,
    V* __restrict__ vout, int64_t n, int shift, const uint32_t* __restrict__ offs, int ntiles) {
  __shared__ uint32_t base[RS_DIGITS];
  __shared__ uint32_t wcnt[RS_BLOCK / 64][RS_DIGITS];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  if (t < RS_DIGITS) base[t] = offs[(int64_t)t * ntiles + blockIdx.x];
  const int64_t tile = (int64_t)blockIdx.x * RS_TILE;
  for (int sub = 0; sub < RS_TILE; sub += RS_BLOCK) {
    const int64_t i = tile + sub + t;
    const bool ok = i < n;
    const int16_t k = ok ? kin[i] : (int16_t)0;
    const int d = ok ? rs_digit(k, shift) : -1;
    // rank among earlier lanes of this wave with the same digit
    int rank = 0, mycount_d = 0;
    for (int dd = 0; dd < RS_DIGITS; ++dd) {
      const uint64_t m = __ballot(d == dd);
      if (d == dd) rank = __popcll(m & ((1ull << lane) - 1ull));
      if (lane == dd) mycount_d = __popcll(m);
    }
    __syncthreads();                       // base[] ready / previous sub-tile done
    if (lane < RS_DIGITS) wcnt[w][lane] = (uint32_t)mycount_d;
    __syncthreads();
    if (ok) {
      uint32_t pos = base[d] + (uint32_t)rank;
      for (int ww = 0; ww < w; ++ww) pos += wcnt[ww][d];
      kout[pos] = k;
      vout[pos] = vin[i];
    }
    __syncthreads();
    if (t < RS_DIGITS) {
      uint32_t add = 0;
      for (int ww = 0; ww < RS_BLOCK / 64; ++ww) add += wcnt[ww][t];
      base[t] += add;
    }
  }
}

// ---------------------------------------------------------------------------
// per-network segments: offsets passed by value, 128 networks per launch
// ---------------------------------------------------------------------------
constexpr int SEG_BATCH = 448;   // networks per launch: the offsets travel as a
                                  // kernel argument (3.6 KB, under the 4 KB kernarg budget)
struct SegBatch {
  int count;
  int64_t off[SEG_BATCH + 1];   // row offsets (relative to the whole batch input)
};

template <typename F>
static int for_each_segment_batch(const int64_t* bspn, int num_networks, F&& fn) {
  int64_t row = 0;
  for (int b0 = 0; b0 < num_networks; b0 += SEG_BATCH) {
    SegBatch sb;
    sb.count = num_networks - b0 < SEG_BATCH ? num_networks - b0 : SEG_BATCH;
    int64_t maxrows = 0;
    for (int k = 0; k < sb.count; ++k) {
      sb.off[k] = row;
      if (bspn[b0 + k] < 0) return fail(NERF_E_ARG, "negative batch_size_per_network entry");
      row += bspn[b0 + k];
      maxrows = bspn[b0 + k] > maxrows ? bspn[b0 + k] : maxrows;
    }
    sb.off[sb.count] = row;
    const int rc = fn(sb, b0, maxrows);
    if (rc) return rc;
  }
  return 0;
}

__global__ void kn_g2l_kernel(float* __restrict__ pts, const float* __restrict__ mins,
                              const float* __restrict__ maxs, SegBatch sb, int net0) {
  const int k = blockIdx.y;
  const int64_t r0 = sb.off[k], r1 = sb.off[k + 1];
  const int net = net0 + k;
  for (int64_t i = r0 * 3 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < r1 * 3;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % 3);
    const float mn = mins[net * 3 + c], mx = maxs[net * 3 + c];
    pts[i] = (2.0f * (pts[i] - mn)) / (mx - mn) - 1.0f;
  }
}

// grouped GEMM fallback for shapes beyond the MFMA kernels' LDS budget: one
// thread per output element, fma chain over k
__global__ void kn_grouped_gemm_kernel(int mode, const float* __restrict__ bias,
                                       const float* __restrict__ X, const float* __restrict__ W,
                                       int out_f, int in_f, float* __restrict__ out, SegBatch sb,
                                       int net0) {
  const int k = blockIdx.y;
  const int64_t r0 = sb.off[k], rows = sb.off[k + 1] - r0;
  const int net = net0 + k;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= rows * out_f) return;
  const int64_t row = r0 + e / out_f;
  const int col = (int)(e % out_f);
  const float* x = X + row * in_f;
  const float* w = W + (int64_t)net * out_f * in_f;
  float acc = 0.0f;
  if (mode == 2) {
    for (int kk = 0; kk < in_f; ++kk) acc = __builtin_fmaf(x[kk], w[(int64_t)col * in_f + kk], acc);
  } else {
    for (int kk = 0; kk < in_f; ++kk) acc = __builtin_fmaf(x[kk], w[(int64_t)kk * out_f + col], acc);
  }
  if (mode == 0) acc = acc + bias[(int64_t)net * out_f + col];
  out[row * out_f + col] = acc;
}

__global__ void kn_at_b_kernel(const float* __restrict__ A, int64_t ac, const float* __restrict__ B,
                               int64_t bc, float* __restrict__ out, SegBatch sb, int net0) {
  const int k = blockIdx.y;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= ac * bc) return;
  const int64_t a = e / bc, b = e % bc;
  float s = 0.0f;
  for (int64_t r = sb.off[k]; r < sb.off[k + 1]; ++r) s = __builtin_fmaf(A[r * ac + a], B[r * bc + b], s);
  out[(int64_t)(net0 + k) * ac * bc + e] = s;
}

// ---------------------------------------------------------------------------
// grouped GEMM family on FP32 MFMA (v_mfma_f32_16x16x4_f32). MAGMA's
// accumulation order (multimatmul.cu) is unknown and differs from any fixed
// chain; results are compared with the sequential restatement within the
// summation-order bound 2 n u sum|terms| (tests/test_gpu_kilonerf.py).
// ---------------------------------------------------------------------------
typedef float kn_f32x4 __attribute__((ext_vector_type(4)));
constexpr int GG_ROWS = 128;               // rows per workgroup: 4 waves x 32 (two 16-row tiles)
constexpr int GG_MAX_IN = 120;             // K (padded to 4) held in LDS
constexpr int GG_MAX_OUT = 64;             // N (padded to 16): 4 accumulator tiles per row tile
// LDS row strides, bank-conflict-free for the MFMA operand reads (ds_read_b32:
// bank (a/4) mod 32 over each 32-lane half = 2 K rows x 16 lanes): W rows
// (k0 + kq) * ws + l16 need ws = 16 mod 32; X rows (r0 + l16) * xs + kq need
// xs = 2 mod 32.
// LDS image (floats): W_net as stored (mode 0/1: [in_f][out_f], mode 2:
// [out_f][in_f]) rounded up to whole 64-float LDS-DMA pieces, then the X tile
// as stored ([128][in_f] dense), whose region the output tile ([nrow][out_f]
// dense) reuses.
__host__ __device__ __forceinline__ int gg_wfloats(int in_f, int out_f) {
  return (in_f * out_f + 63) & ~63;
}
__host__ __device__ __forceinline__ size_t gg_lds_bytes(int in_f, int out_f) {
  return (size_t)(gg_wfloats(in_f, out_f) + GG_ROWS * (in_f > out_f ? in_f : out_f)) * sizeof(float);
}

// out[r] = X[r] . W_net (+ bias_net), rows of network net0 + blockIdx.y, 128 per
// workgroup (blockIdx.x). W_net and the X tile (one contiguous run of nrow *
// in_f floats) land in LDS by buffer-form LDS-DMA (4 B per lane, 64-float
// pieces, reads past either run return 0): every load of the workgroup is in
// flight at once and no register holds staged data (register staging with one
// load -> store trip per row batch measured 0.45 ms at 4096 networks, a
// chain of HBM latencies per workgroup). Wave w owns tile rows 32w .. 32w+31:
// A = X (16 rows x 4 k), B = W (4 k x 16 columns), one accumulator per (row
// tile, 16-column tile); K and column padding are zeroed in registers. The
// output tile is staged back through LDS (the X region) and written as one
// contiguous run of nrow * out_f floats.
// Row offsets of the networks: a kernel-argument batch (SegBatch, at most
// SEG_BATCH networks per launch) or a device array (a grouped-GEMM handle's
// buffer: every network in one launch).
__device__ __forceinline__ int64_t off_at(const SegBatch& sb, int k) { return sb.off[k]; }
__device__ __forceinline__ int64_t off_at(const int64_t* off, int k) { return off[k]; }

template <typename Off>
__global__ __launch_bounds__(256) void kn_grouped_gemm_mfma_kernel(
    int mode, const float* __restrict__ bias, const float* __restrict__ X,
    const float* __restrict__ W, int out_f, int in_f, float* __restrict__ out, Off sb,
    int net0) {
  extern __shared__ float gg_sm[];
  const int k = blockIdx.y;
  const int64_t r0 = off_at(sb, k), rows = off_at(sb, k + 1) - r0;
  const int64_t t0 = (int64_t)blockIdx.x * GG_ROWS;
  if (t0 >= rows) return;   // block-uniform
  const int net = net0 + k;
  const int kp = (in_f + 3) & ~3, np = (out_f + 15) & ~15;
  float* Ws = gg_sm;                               // W_net as stored
  float* Xs = gg_sm + gg_wfloats(in_f, out_f);     // [128][in_f]; then the output tile
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nrow = (int)(rows - t0 < GG_ROWS ? rows - t0 : GG_ROWS);
  {
    const int nx = nrow * in_f, nw = in_f * out_f;
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(X + (r0 + t0) * in_f), 0, nx * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(W + (int64_t)net * nw), 0, nw * 4, 0x00020000);
    for (int p = wave; p < (nx + 63) / 64; p += 4)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (__attribute__((address_space(3))) void*)(Xs + 64 * p),
                                               4, (p * 64 + lane) * 4, 0, 0, 0);
    for (int p = wave; p < (nw + 63) / 64; p += 4)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (__attribute__((address_space(3))) void*)(Ws + 64 * p),
                                               4, (p * 64 + lane) * 4, 0, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  const int kq = lane >> 4, l16 = lane & 15;
  const int nt = np / 16;
  kn_f32x4 acc[2][GG_MAX_OUT / 16];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int c = 0; c < GG_MAX_OUT / 16; ++c) acc[t][c] = kn_f32x4{0.f, 0.f, 0.f, 0.f};
  const bool busy = wave * 32 < nrow;   // wave-uniform
  if (busy) {
    // rows >= nrow read whatever the LDS holds: they only reach output rows that
    // are never stored
    const float* xa = Xs + (wave * 32 + l16) * in_f + kq;
    const int cstride = mode == 2 ? in_f : 1, kstride = mode == 2 ? 1 : out_f;
    const float* wb = Ws + kq * kstride + l16 * cstride;
    for (int k0 = 0; k0 < kp; k0 += 4) {
      const bool kok = k0 + kq < in_f;
      const float a0 = kok ? xa[k0] : 0.0f, a1 = kok ? xa[16 * in_f + k0] : 0.0f;
#pragma unroll
      for (int c = 0; c < GG_MAX_OUT / 16; ++c)
        if (c < nt) {
          const float b = (kok && 16 * c + l16 < out_f) ? wb[k0 * kstride + 16 * c * cstride] : 0.0f;
          acc[0][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b, acc[0][c], 0, 0, 0);
          acc[1][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b, acc[1][c], 0, 0, 0);
        }
    }
  }
  __syncthreads();   // every wave is done with Xs: it now holds the output tile
  float* Os = Xs;    // [nrow][out_f], dense
  if (busy) {
    // lane holds rows 4 kq + i of each row tile, column l16 of each 16-column tile
#pragma unroll
    for (int c = 0; c < GG_MAX_OUT / 16; ++c) {
      const int col = 16 * c + l16;
      if (c < nt && col < out_f) {
        const float bb = mode == 0 ? bias[(int64_t)net * out_f + col] : 0.0f;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int rr = wave * 32 + 16 * t + 4 * kq + i;
            if (rr < nrow) Os[rr * out_f + col] = mode == 0 ? acc[t][c][i] + bb : acc[t][c][i];
          }
      }
    }
  }
  __syncthreads();
  float* o = out + (r0 + t0) * out_f;
  const int n = nrow * out_f;
  for (int i = threadIdx.x; i < n; i += 256) o[i] = Os[i];
}

constexpr int AB_MAX_T = 4;     // 16-wide tiles per side (a_cols, b_cols <= 64)
constexpr int AB_WAVES = 8;     // waves per network
constexpr int AB_UNROLL = 4;    // row quads per wave whose loads are in flight together
                                // (8: 0.252 vs 0.214 ms at 4096 networks)

// out_net = A_net^T B_net ([ac][bc]) over the network's rows, one workgroup
// per network: wave w takes row quads w, w + 8, ...; A operand = A^T (16 a x
// 4 rows), B operand = B (4 rows x 16 b). The loads of AB_UNROLL row quads are
// issued before their MFMAs (a network's ~256 rows are a few such batches, so
// the kernel is bound by how many loads are in flight, not by the MFMAs); the
// 8 waves' partial tiles are summed in LDS in wave order.
__global__ __launch_bounds__(64 * AB_WAVES) void kn_at_b_mfma_kernel(
    const float* __restrict__ A, int ac, const float* __restrict__ B, int bc,
    float* __restrict__ out, SegBatch sb, int net0) {
  extern __shared__ float ab_sm[];
  const int k = blockIdx.x;
  const int64_t r0 = sb.off[k], r1 = sb.off[k + 1];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int kq = lane >> 4, l16 = lane & 15;
  const int ta = (ac + 15) / 16, tb = (bc + 15) / 16;
  kn_f32x4 acc[AB_MAX_T][AB_MAX_T];
#pragma unroll
  for (int i = 0; i < AB_MAX_T; ++i)
#pragma unroll
    for (int j = 0; j < AB_MAX_T; ++j) acc[i][j] = kn_f32x4{0.f, 0.f, 0.f, 0.f};
  constexpr int kStep = 4 * AB_WAVES;
  for (int64_t rb = r0 + 4 * wave; rb < r1; rb += (int64_t)kStep * AB_UNROLL) {
    float a[AB_UNROLL][AB_MAX_T], b[AB_UNROLL][AB_MAX_T];
#pragma unroll
    for (int u = 0; u < AB_UNROLL; ++u) {
      const int64_t r = rb + (int64_t)kStep * u + kq;
      const bool ok = r < r1;
#pragma unroll
      for (int i = 0; i < AB_MAX_T; ++i) {
        const int c = 16 * i + l16;
        a[u][i] = (i < ta && ok && c < ac) ? A[r * ac + c] : 0.0f;
        b[u][i] = (i < tb && ok && c < bc) ? B[r * bc + c] : 0.0f;
      }
    }
#pragma unroll
    for (int u = 0; u < AB_UNROLL; ++u)
#pragma unroll
      for (int i = 0; i < AB_MAX_T; ++i)
#pragma unroll
        for (int j = 0; j < AB_MAX_T; ++j)
          if (i < ta && j < tb)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][i], b[u][j], acc[i][j], 0, 0, 0);
  }
  // partial tile (i, j) of wave w at ab_sm[((w * ta + i) * tb + j) * 256 + 64 * e + lane]
#pragma unroll
  for (int i = 0; i < AB_MAX_T; ++i)
#pragma unroll
    for (int j = 0; j < AB_MAX_T; ++j)
      if (i < ta && j < tb)
#pragma unroll
        for (int e = 0; e < 4; ++e) ab_sm[((wave * ta + i) * tb + j) * 256 + 64 * e + lane] = acc[i][j][e];
  __syncthreads();
  const int per = ta * tb * 256;
  float* o = out + (int64_t)(net0 + k) * ac * bc;
  for (int idx = threadIdx.x; idx < per; idx += 64 * AB_WAVES) {
    const int tile = idx >> 8, e = (idx >> 6) & 3, ln = idx & 63;
    const int i = tile / tb, j = tile - i * tb;
    const int ra = 16 * i + 4 * (ln >> 4) + e, cbx = 16 * j + (ln & 15);
    if (ra < ac && cbx < bc) {
      float s = ab_sm[idx];
      for (int w = 1; w < AB_WAVES; ++w) s = s + ab_sm[w * per + idx];
      o[(int64_t)ra * bc + cbx] = s;
    }
  }
}

// out_net[c] = sum over the network's rows of M[r][c]: one workgroup per
// (network, 32 columns); 8 row phases per column (loads of a phase unrolled so
// several are in flight) summed in LDS in phase order.
constexpr int RSB_COLS = 32, RSB_PH = 8;
__global__ __launch_bounds__(256) void kn_row_sum_blk_kernel(const float* __restrict__ M,
                                                             int64_t cols, float* __restrict__ out,
                                                             SegBatch sb, int net0) {
  __shared__ float part[RSB_PH][RSB_COLS];
  const int k = blockIdx.y;
  const int64_t r0 = sb.off[k], r1 = sb.off[k + 1];
  const int cl = threadIdx.x % RSB_COLS, ph = threadIdx.x / RSB_COLS;
  const int64_t c = (int64_t)blockIdx.x * RSB_COLS + cl;
  float s = 0.0f;
  if (c < cols) {
#pragma unroll 8
    for (int64_t r = r0 + ph; r < r1; r += RSB_PH) s = s + M[r * cols + c];
  }
  part[ph][cl] = s;
  __syncthreads();
  if (ph == 0 && c < cols) {
    float t = part[0][cl];
#pragma unroll
    for (int p = 1; p < RSB_PH; ++p) t = t + part[p][cl];
    out[(int64_t)(net0 + k) * cols + c] = t;
  }
}

// ---------------------------------------------------------------------------
// network_eval_query_index (network_eval.cu:24-254), hidden_dim = 32
// ---------------------------------------------------------------------------
template <int HD>
__global__ __launch_bounds__(256) void kn_network_eval_kernel(
    const int32_t* __restrict__ qidx, const float* __restrict__ params,
    const float* __restrict__ mins, const float* __restrict__ maxs,
    const int32_t* __restrict__ starts, const int32_t* __restrict__ ends,
    const float* __restrict__ origin, const float* __restrict__ c2w, int W, float cx, float cy,
    float fx, float fy, int max_depth, float min_dist, float step, float* __restrict__ out) {
  constexpr int NP = 10, ND = 4, PE = 3 * (2 * NP + 1), DE = 3 * (2 * ND + 1);
  constexpr int PSIZE = (PE + 1) * HD + (HD + 1) * HD + (HD + 1) * (HD + 1) +
                        (HD + DE + 1) * HD + (HD + 1) * 3;
  __shared__ float cache[PSIZE];
  const int net = blockIdx.x;
  const int s0 = starts[net], s1 = ends[net];
  if (s0 == s1) return;
  for (int i = threadIdx.x; i < PSIZE; i += blockDim.x) cache[i] = params[(int64_t)net * PSIZE + i];
  __syncthreads();
  float mn[3], mx[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) { mn[c] = mins[net * 3 + c]; mx[c] = maxs[net * 3 + c]; }
  const float fb[10] = {1.f, 2.f, 4.f, 8.f, 16.f, 32.f, 64.f, 128.f, 256.f, 512.f};
  for (int idx = s0 + threadIdx.x; idx < s1; idx += blockDim.x) {
    int y = qidx[idx];
    const int depth = y % max_depth;
    y /= max_depth;
    const int x = y % W;
    y /= W;
    const float in[3] = {((float)x - cx) / fx, -((float)y - cy) / fy, -1.0f};
    float dir[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      float o = in[0] * c2w[i * 3 + 0];
      o = __builtin_fmaf(in[1], c2w[i * 3 + 1], o);
      o = __builtin_fmaf(in[2], c2w[i * 3 + 2], o);
      dir[i] = o;
    }
    const float dist = __builtin_fmaf((float)depth, step, min_dist);
    float pos[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) pos[i] = __builtin_fmaf(dist, dir[i], origin[i]);
    float nrm = dir[0] * dir[0];
    nrm = __builtin_fmaf(dir[1], dir[1], nrm);
    nrm = __builtin_fmaf(dir[2], dir[2], nrm);
    nrm = sqrtf(nrm);
#pragma unroll
    for (int i = 0; i < 3; ++i) dir[i] = dir[i] / nrm;

    int po = 0;
    float h0[HD];
#pragma unroll
    for (int i = 0; i < HD; ++i) h0[i] = cache[po++];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const float e0 = (2.0f * (pos[j] - mn[j])) / (mx[j] - mn[j]) - 1.0f;
#pragma unroll
      for (int e = 0; e < 2 * NP + 1; ++e) {
        const float v = e == 0 ? e0 : (e <= NP ? cosf(fb[e - 1] * e0) : sinf(fb[e - 1 - NP] * e0));
#pragma unroll
        for (int i = 0; i < HD; ++i) h0[i] = __builtin_fmaf(v, cache[po++], h0[i]);
      }
    }
    float h1[HD];
#pragma unroll
    for (int i = 0; i < HD; ++i) h1[i] = cache[po++];
#pragma unroll
    for (int j = 0; j < HD; ++j) {
      const float v = fmaxf(h0[j], 0.0f);
#pragma unroll
      for (int i = 0; i < HD; ++i) h1[i] = __builtin_fmaf(v, cache[po++], h1[i]);
    }
    float h2[HD + 1];
#pragma unroll
    for (int i = 0; i < HD + 1; ++i) h2[i] = cache[po++];
#pragma unroll
    for (int j = 0; j < HD; ++j) {
      const float v = fmaxf(h1[j], 0.0f);
#pragma unroll
      for (int i = 0; i < HD + 1; ++i) h2[i] = __builtin_fmaf(v, cache[po++], h2[i]);
    }
    float h3[HD];
#pragma unroll
    for (int i = 0; i < HD; ++i) h3[i] = cache[po++];
#pragma unroll
    for (int j = 0; j < HD; ++j) {
      const float v = h2[j + 1];
#pragma unroll
      for (int i = 0; i < HD; ++i) h3[i] = __builtin_fmaf(v, cache[po++], h3[i]);
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) {
#pragma unroll
      for (int e = 0; e < 2 * ND + 1; ++e) {
        const float v = e == 0 ? dir[j] : (e <= ND ? cosf(fb[e - 1] * dir[j]) : sinf(fb[e - 1 - ND] * dir[j]));
#pragma unroll
        for (int i = 0; i < HD; ++i) h3[i] = __builtin_fmaf(v, cache[po++], h3[i]);
      }
    }
    float rgb[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) rgb[i] = cache[po++];
#pragma unroll
    for (int j = 0; j < HD; ++j) {
      const float v = fmaxf(h3[j], 0.0f);
#pragma unroll
      for (int i = 0; i < 3; ++i) rgb[i] = __builtin_fmaf(v, cache[po++], rgb[i]);
    }
#pragma unroll
    for (int i = 0; i < 3; ++i)   // sigmoid: 1.0 / (1.0 + exp(-x)) in double (network_eval.cu:15)
      out[(int64_t)idx * 4 + i] = (float)(1.0 / (1.0 + (double)expf(-rgb[i])));
    out[(int64_t)idx * 4 + 3] = fmaxf(h2[0], 0.0f);
  }
}

// ---------------------------------------------------------------------------
// host state: stream pool and grouped-GEMM handles
// ---------------------------------------------------------------------------
struct GemmHandle {
  int64_t num_networks, out_f, in_f;
  std::vector<int> group_limits;
  int64_t* d_off = nullptr;   // device row offsets [num_networks + 1], rewritten per call
  int64_t* h_off = nullptr;   // pinned staging of the offsets (the copy reads it async)
  hipEvent_t staged = nullptr;  // the last upload from h_off: h_off is reused after it
};

static std::mutex g_mu;
static std::vector<hipStream_t> g_streams;
static std::map<int, GemmHandle> g_gemm;
static int g_gemm_next = 0;

}  // namespace nerfhip

using namespace nerfhip;

extern "C" {

int kn_get_rays_d(int H, int W, float cx, float cy, float fx, float fy, const float* c2w,
                  float* out, nerf_stream_t stream) {
  NERF_REQUIRE(c2w && out && H >= 0 && W >= 0, "kn_get_rays_d: bad argument");
  const int64_t n = (int64_t)H * W;
  if (n == 0) return 0;
  hipLaunchKernelGGL(kn_rays_d_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0,
                     as_stream(stream), H, W, cx, cy, fx, fy, c2w, out);
  return check_launch("kn_rays_d_kernel");
}

int kn_generate_query_indices_on_ray(const float* origin, const float* directions, int num_rays,
                                     const int16_t* grid, uint8_t* active, int16_t* depth_idx,
                                     const float* vsize, const float* gmin, const float* gmax,
                                     const int32_t* strides, float step, int max_samples,
                                     int max_depth, float min_dist, int initial, int32_t* qidx,
                                     int16_t* nets, nerf_stream_t stream) {
  NERF_REQUIRE(origin && directions && grid && active && depth_idx && vsize && gmin && gmax &&
                   strides && qidx && nets,
               "kn_generate_query_indices_on_ray: null pointer");
  NERF_REQUIRE(num_rays >= 0 && max_samples >= 0 && max_depth >= 0,
               "kn_generate_query_indices_on_ray: bad size");
  if (num_rays == 0) return 0;
  hipLaunchKernelGGL(kn_query_indices_kernel, dim3((unsigned)cdiv(num_rays, 256)), dim3(256), 0,
                     as_stream(stream), origin, directions, grid, active, depth_idx, vsize, gmin,
                     gmax, strides, num_rays, step, max_samples, max_depth, min_dist, initial,
                     qidx, nets);
  return check_launch("kn_query_indices_kernel");
}

int kn_compute_fourier_features(const float* input, int64_t n, const float* freqs, int L,
                                float* out, nerf_stream_t stream) {
  NERF_REQUIRE(input && freqs && out && n >= 0 && L >= 0 && L <= 32,
               "kn_compute_fourier_features: bad argument");
  if (n == 0) return 0;
  const size_t smem = (size_t)FF_BLOCK * (2 * L + 1) * sizeof(float);
  hipLaunchKernelGGL(kn_fourier_kernel, dim3((unsigned)cdiv(n, FF_BLOCK)), dim3(FF_BLOCK), smem,
                     as_stream(stream), input, n, freqs, L, out);
  return check_launch("kn_fourier_kernel");
}

int kn_integrate(const float* rgb_sigma, const float* dists, float* rgb_map, float* acc_map,
                 float* transmittance, uint8_t* mask, int num_rays, int spr, float thr,
                 int initial, nerf_stream_t stream) {
  NERF_REQUIRE(rgb_sigma && dists && rgb_map && acc_map && transmittance && mask,
               "kn_integrate: null pointer");
  NERF_REQUIRE(num_rays >= 0 && spr >= 0, "kn_integrate: bad size");
  if (num_rays == 0) return 0;
  hipLaunchKernelGGL(kn_integrate_kernel, dim3((unsigned)cdiv(num_rays, 64 * KI_WAVES)),
                     dim3(64 * KI_WAVES), 0,
                     as_stream(stream), (const float4*)rgb_sigma, dists, rgb_map, acc_map,
                     transmittance, mask, num_rays, spr, thr, initial);
  return check_launch("kn_integrate_kernel");
}

int kn_replace_transparency_by_background_color(float* rgb_map, const float* acc_map, int64_t n,
                                                const float* bg, nerf_stream_t stream) {
  NERF_REQUIRE(rgb_map && acc_map && bg && n >= 0, "kn_replace_transparency: bad argument");
  if (n == 0) return 0;
  hipLaunchKernelGGL(kn_background_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0,
                     as_stream(stream), rgb_map, acc_map, n, bg);
  return check_launch("kn_background_kernel");
}

int kn_gather_int32(const int32_t* map, int64_t n_out, const int32_t* input, int32_t* out,
                    nerf_stream_t stream) {
  NERF_REQUIRE(map && input && out && n_out >= 0, "kn_gather_int32: bad argument");
  if (n_out == 0) return 0;
  hipLaunchKernelGGL(kn_gather_kernel, dim3((unsigned)cdiv(n_out, 256)), dim3(256), 0,
                     as_stream(stream), map, n_out, input, out);
  return check_launch("kn_gather_kernel");
}

int kn_scatter_int32_float4(const int32_t* map, int64_t n, const float* input, float* out,
                            nerf_stream_t stream) {
  NERF_REQUIRE(map && input && out && n >= 0, "kn_scatter_int32_float4: bad argument");
  if (n == 0) return 0;
  hipLaunchKernelGGL(kn_scatter_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0,
                     as_stream(stream), map, n, (const float4*)input, (float4*)out);
  return check_launch("kn_scatter_kernel");
}

size_t kn_sort_scratch_bytes(int64_t n, int value_bytes) {
  const int64_t ntiles = cdiv(n > 0 ? n : 1, RS_TILE);
  const size_t a = (size_t)n * 2, b = (size_t)n * (size_t)value_bytes;
  return ((a + 255) / 256) * 256 + ((b + 255) / 256) * 256 + (size_t)RS_DIGITS * ntiles * 4 + 256;
}

int kn_sort_by_key_int16(int16_t* keys, void* values, int value_bytes, int64_t n, void* scratch,
                         nerf_stream_t stream) {
  NERF_REQUIRE(keys && values && scratch && n >= 0 && (value_bytes == 4 || value_bytes == 8),
               "kn_sort_by_key_int16: bad argument");
  if (n <= 1) return 0;
  NERF_REQUIRE(n < (1ll << 31), "kn_sort_by_key_int16: too many elements");
  const int ntiles = (int)cdiv(n, RS_TILE);
  char* sp = (char*)scratch;
  int16_t* k2 = (int16_t*)sp;
  sp += (((size_t)n * 2 + 255) / 256) * 256;
  void* v2 = sp;
  sp += (((size_t)n * value_bytes + 255) / 256) * 256;
  uint32_t* hist = (uint32_t*)sp;
  hipStream_t s = as_stream(stream);
  int16_t* kin = keys;
  int16_t* kout = k2;
  void* vin = values;
  void* vout = v2;
  for (int shift = 0; shift < 16; shift += 4) {
    hipLaunchKernelGGL(rs_hist_kernel, dim3(ntiles), dim3(RS_BLOCK), 0, s, kin, n, shift, hist,
                       ntiles);
    hipLaunchKernelGGL(rs_scan_kernel, dim3(1), dim3(1024), 0, s, hist, (int64_t)RS_DIGITS * ntiles);
    if (value_bytes == 4)
      hipLaunchKernelGGL(rs_scatter_kernel<int32_t>, dim3(ntiles), dim3(RS_BLOCK), 0, s, kin,
                         (const int32_t*)vin, kout, (int32_t*)vout, n, shift, hist, ntiles);
    else
      hipLaunchKernelGGL(rs_scatter_kernel<int64_t>, dim3(ntiles), dim3(RS_BLOCK), 0, s, kin,
                         (const int64_t*)vin, kout, (int64_t*)vout, n, shift, hist, ntiles);
    const int rc = check_launch("radix sort pass");
    if (rc) return rc;
    int16_t* tk = kin; kin = kout; kout = tk;
    void* tv = vin; vin = vout; vout = tv;
  }
  return 0;   // 4 passes: the sorted data is back in keys/values
}

int kn_global_to_local(float* points, const float* mins, const float* maxs,
                       const int64_t* bspn, int num_networks, nerf_stream_t stream) {
  NERF_REQUIRE(points && mins && maxs && bspn && num_networks >= 0,
               "kn_global_to_local: bad argument");
  return for_each_segment_batch(bspn, num_networks, [&](const SegBatch& sb, int net0, int64_t mr) {
    if (mr == 0) return 0;
    const unsigned gx = (unsigned)(cdiv(mr * 3, 256) < 64 ? cdiv(mr * 3, 256) : 64);
    hipLaunchKernelGGL(kn_g2l_kernel, dim3(gx, sb.count), dim3(256), 0, as_stream(stream), points,
                       mins, maxs, sb, net0);
    return check_launch("kn_g2l_kernel");
  });
}

int kn_network_eval_query_index(const int32_t* qidx, int64_t batch, const float* params,
                                const float* mins, const float* maxs, const int32_t* starts,
                                const int32_t* ends, const float* origin, const float* c2w,
                                int num_networks, int hidden_dim, int H, int W, float cx, float cy,
                                float fx, float fy, int max_depth, float min_dist, float step,
                                float* out, nerf_stream_t stream) {
  (void)H;
  NERF_REQUIRE(qidx && params && mins && maxs && starts && ends && origin && c2w && out,
               "kn_network_eval_query_index: null pointer");
  NERF_REQUIRE(batch >= 0 && num_networks >= 0 && W > 0 && max_depth > 0,
               "kn_network_eval_query_index: bad size");
  if (hidden_dim != 32)
    return fail(NERF_E_UNSUPPORTED, "kn_network_eval_query_index: unsupported hidden_dim (only 32, "
                                    "as network_eval.cu:281-288)");
  if (num_networks == 0) return 0;
  hipLaunchKernelGGL(kn_network_eval_kernel<32>, dim3(num_networks), dim3(256), 0,
                     as_stream(stream), qidx, params, mins, maxs, starts, ends, origin, c2w, W, cx,
                     cy, fx, fy, max_depth, min_dist, step, out);
  return check_launch("kn_network_eval_kernel");
}

int kn_init_stream_pool(int64_t num_streams) {
  NERF_REQUIRE(num_streams >= 0 && num_streams <= 64, "kn_init_stream_pool: 0..64 streams");
  std::lock_guard<std::mutex> lk(g_mu);
  for (auto s : g_streams) (void)hipStreamDestroy(s);
  g_streams.clear();
  for (int64_t i = 0; i < num_streams; ++i) {
    hipStream_t s;
    const hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    if (e != hipSuccess) return fail((int)e, "kn_init_stream_pool: hipStreamCreate failed");
    g_streams.push_back(s);
  }
  return 0;
}

int kn_destroy_stream_pool(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  for (auto s : g_streams) (void)hipStreamDestroy(s);
  g_streams.clear();
  return 0;
}

int kn_init_magma(void) { return 0; }

int kn_init_multimatmul_grouped(int64_t num_networks, int64_t out_f, int64_t in_f,
                                const int32_t* group_limits, int n_group_limits, int* handle) {
  NERF_REQUIRE(handle && num_networks >= 0 && out_f > 0 && in_f > 0 && n_group_limits >= 0,
               "kn_init_multimatmul_grouped: bad argument");
  std::lock_guard<std::mutex> lk(g_mu);
  GemmHandle hd{num_networks, out_f, in_f, {}};
  for (int i = 0; i < n_group_limits; ++i) hd.group_limits.push_back(group_limits[i]);
  int dev = 0, max_y = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&max_y, hipDeviceAttributeMaxGridDimY, dev) != hipSuccess) {
    (void)hipGetLastError();
    max_y = 0;
  }
  if (num_networks > 0 && num_networks <= max_y) {   // grid.y bound of the one-launch path
    // without the buffers (no device, out of memory) calls take the batched launches
    const size_t nb = (size_t)(num_networks + 1) * sizeof(int64_t);
    if (hipMalloc(&hd.d_off, nb) != hipSuccess ||
        hipHostMalloc((void**)&hd.h_off, nb, hipHostMallocDefault) != hipSuccess ||
        hipEventCreateWithFlags(&hd.staged, hipEventDisableTiming) != hipSuccess) {
      (void)hipGetLastError();
      if (hd.d_off) (void)hipFree(hd.d_off);
      if (hd.h_off) (void)hipHostFree(hd.h_off);
      hd.d_off = nullptr;
      hd.h_off = nullptr;
      hd.staged = nullptr;
    }
  }
  *handle = g_gemm_next++;
  g_gemm[*handle] = hd;
  return 0;
}

int kn_deinit_multimatmul_grouped(int handle) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_gemm.find(handle);
  if (it == g_gemm.end()) return fail(NERF_E_HANDLE, "kn_deinit_multimatmul_grouped: unknown handle");
  // a launch may still read the offsets: free them once the device is done
  if (it->second.d_off) {
    (void)hipDeviceSynchronize();
    (void)hipFree(it->second.d_off);
    (void)hipHostFree(it->second.h_off);
    (void)hipEventDestroy(it->second.staged);
  }
  g_gemm.erase(it);
  return 0;
}

int kn_multimatmul_grouped(int handle, int mode, const float* biases, const float* X,
                           const float* W, int64_t out_f, int64_t in_f, const int64_t* bspn,
                           int num_networks, float* out, nerf_stream_t stream) {
  int64_t* d_off = nullptr;
  int64_t* h_off = nullptr;
  hipEvent_t staged = nullptr;
  int64_t hnets = 0;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_gemm.find(handle);
    if (it == g_gemm.end()) return fail(NERF_E_HANDLE, "kn_multimatmul_grouped: unknown handle");
    d_off = it->second.d_off;
    h_off = it->second.h_off;
    staged = it->second.staged;
    hnets = it->second.num_networks;
  }
  // a captured graph would replay the upload of one call's offsets: take the
  // batched launches (offsets as kernel arguments) while the stream captures
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(as_stream(stream), &cap) != hipSuccess) {
    (void)hipGetLastError();
    cap = hipStreamCaptureStatusActive;
  }
  if (cap != hipStreamCaptureStatusNone) d_off = nullptr;
  NERF_REQUIRE(X && W && out && bspn && (mode != 0 || biases) && mode >= 0 && mode <= 2,
               "kn_multimatmul_grouped: bad argument");
  NERF_REQUIRE(out_f > 0 && in_f > 0 && out_f < (1 << 20) && in_f < (1 << 20),
               "kn_multimatmul_grouped: bad feature sizes");
  if (d_off && num_networks >= 1 && num_networks <= hnets && in_f <= GG_MAX_IN &&
      out_f <= GG_MAX_OUT) {
    // every network in ONE launch: the row offsets go to the handle's device
    // buffer by a stream-ordered copy from its pinned staging array, which is
    // rewritten only once the previous call's copy has read it (a handle serves
    // one stream at a time, as the reference's MAGMA queues do)
    int64_t row = 0, maxrows = 0;
    for (int k = 0; k < num_networks; ++k) {
      if (bspn[k] < 0) return fail(NERF_E_ARG, "negative batch_size_per_network entry");
      row += bspn[k];
      maxrows = bspn[k] > maxrows ? bspn[k] : maxrows;
    }
    if (maxrows == 0) return 0;
    hipError_t e = hipEventSynchronize(staged);
    if (e != hipSuccess) return fail((int)e, "kn_multimatmul_grouped: staging wait failed");
    row = 0;
    for (int k = 0; k < num_networks; ++k) {
      h_off[k] = row;
      row += bspn[k];
    }
    h_off[num_networks] = row;
    e = hipMemcpyAsync(d_off, h_off, (size_t)(num_networks + 1) * sizeof(int64_t),
                       hipMemcpyHostToDevice, as_stream(stream));
    if (e == hipSuccess) e = hipEventRecord(staged, as_stream(stream));
    if (e != hipSuccess) return fail((int)e, "kn_multimatmul_grouped: offset upload failed");
    hipLaunchKernelGGL(kn_grouped_gemm_mfma_kernel<const int64_t*>,
                       dim3((unsigned)cdiv(maxrows, GG_ROWS), (unsigned)num_networks), dim3(256),
                       gg_lds_bytes((int)in_f, (int)out_f), as_stream(stream), mode, biases, X, W,
                       (int)out_f, (int)in_f, out, (const int64_t*)d_off, 0);
    return check_launch("kn_grouped_gemm_mfma_kernel");
  }
  return for_each_segment_batch(bspn, num_networks, [&](const SegBatch& sb, int net0, int64_t mr) {
    if (mr == 0) return 0;
    if (in_f <= GG_MAX_IN && out_f <= GG_MAX_OUT) {
      const size_t lds = gg_lds_bytes((int)in_f, (int)out_f);
      hipLaunchKernelGGL(kn_grouped_gemm_mfma_kernel<SegBatch>, dim3((unsigned)cdiv(mr, GG_ROWS), sb.count),
                         dim3(256), lds, as_stream(stream), mode, biases, X, W, (int)out_f,
                         (int)in_f, out, sb, net0);
      return check_launch("kn_grouped_gemm_mfma_kernel");
    }
    hipLaunchKernelGGL(kn_grouped_gemm_kernel, dim3((unsigned)cdiv(mr * out_f, 256), sb.count),
                       dim3(256), 0, as_stream(stream), mode, biases, X, W, (int)out_f, (int)in_f,
                       out, sb, net0);
    return check_launch("kn_grouped_gemm_kernel");
  });
}

int kn_multi_row_sum_reduction(const float* M, int64_t cols, const int64_t* bspn, int num_networks,
                               float* out, nerf_stream_t stream) {
  NERF_REQUIRE(M && bspn && out && cols > 0 && num_networks >= 0,
               "kn_multi_row_sum_reduction: bad argument");
  return for_each_segment_batch(bspn, num_networks, [&](const SegBatch& sb, int net0, int64_t) {
    hipLaunchKernelGGL(kn_row_sum_blk_kernel, dim3((unsigned)cdiv(cols, RSB_COLS), sb.count), dim3(256),
                       0, as_stream(stream), M, cols, out, sb, net0);
    return check_launch("kn_row_sum_blk_kernel");
  });
}

int kn_multimatmul_A_transposed(const float* A, int64_t a_cols, const float* B, int64_t b_cols,
                                const int64_t* bspn, int num_networks, float* out,
                                nerf_stream_t stream) {
  NERF_REQUIRE(A && B && bspn && out && a_cols > 0 && b_cols > 0 && num_networks >= 0,
               "kn_multimatmul_A_transposed: bad argument");
  return for_each_segment_batch(bspn, num_networks, [&](const SegBatch& sb, int net0, int64_t) {
    if (a_cols <= 16 * AB_MAX_T && b_cols <= 16 * AB_MAX_T) {
      const size_t lds = AB_WAVES * cdiv(a_cols, 16) * cdiv(b_cols, 16) * 256 * sizeof(float);
      hipLaunchKernelGGL(kn_at_b_mfma_kernel, dim3((unsigned)sb.count), dim3(64 * AB_WAVES), lds,
                         as_stream(stream), A, (int)a_cols, B, (int)b_cols, out, sb, net0);
      return check_launch("kn_at_b_mfma_kernel");
    }
    hipLaunchKernelGGL(kn_at_b_kernel, dim3((unsigned)cdiv(a_cols * b_cols, 256), sb.count),
                       dim3(256), 0, as_stream(stream), A, a_cols, B, b_cols, out, sb, net0);
    return check_launch("kn_at_b_kernel");
  });
}

int kn_render_to_screen(void) {
  return fail(NERF_E_UNSUPPORTED,
              "render_to_screen: the OpenGL/GLUT viewer (cuda/render_to_screen.cpp) is not part of "
              "this library");
}

}  // extern "C"
