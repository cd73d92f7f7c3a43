// Fused NeRF MLP forward on gfx950 with a 3-term FP16 split of FP32 operands
// (reference src/models/nerf/network.py:49-74, NET): every FP32 product w*x is
// computed as wh*xh + wh*xl + wl*xh on v_mfma_f32_16x16x32_f16 (exact 22-bit
// products, FP32 accumulation), where x = xh + xl, w = wh + wl are the FP16
// round-to-nearest splits of power-of-two-scaled values. 3 MFMAs of 16 cycles
// replace 8 of 32 (FP32 16x16x4) per 16x16x32 tile step: 5.3x the arithmetic
// rate. The dropped wl*xl term and the split residuals are ~2^-22 relative per
// product; scales keep every split in FP16's normal range:
//   * weights: per layer 2^sw (pack time), max |w| * 2^sw in [2^11, 2^12);
//   * activations: per sample and layer 2^e from the sample's max |x| (which
//     includes its encoded input for the skip layer and its view encoding for
//     the views layer), max |x| * 2^e in [2^13, 2^14). A lane holds one sample
//     column of every B operand and accumulator, so the scale is per lane (max
//     over the sample's 4 lane groups: a 2-step butterfly);
//   both undone exactly (power-of-two multiply) before the bias.
//
// Same decomposition and weight streaming as mlp_fused.hip (mlp_stream.h):
// 8 waves x 16 samples, 73 slices of 32 KiB; a slice of a 256-row layer holds
// one 32-deep K step as 16 tiles x (hi, lo) fragment blocks (block 2m + part);
// the views layer packs two K steps per slice (block 16q + 2m + part) and the
// direction step alone in the last slice.
//
// Register dataflow: the accumulator of tile m holds, on lane l, sample l&15
// and rows 16m + 4(l>>4) + r. K step q of the next layer takes, on lane group
// g = l>>4, slots j = 0..7 = rows 16(2q + (j>>2)) + 4g + (j&3), i.e. registers
// r of tiles 2q and 2q+1 (nerfhip/pack.py packs W with that K permutation).
#include "mlp_stream.h"

namespace nerfhip {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

struct Split {   // B operand of one K step: FP16 hi and lo parts
  half8 h, l;
};

constexpr int kX3Threads = 64 * kStreamWaves;
constexpr int kX3Tile = 16 * kStreamWaves;

#define MFMA16(a, b, c) __builtin_amdgcn_mfma_f32_16x16x32_f16((a), (b), (c), 0, 0, 0)

template <int BLOCK>
__device__ __forceinline__ half8 frag16(unsigned base) {
  u32x4 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(base), "i"(BLOCK * 1024) : "memory");
  return __builtin_bit_cast(half8, v);
}

struct Frags {   // one group's A fragments: tiles m, m+1 x (hi, lo)
  half8 h0, l0, h1, l1;
};

template <int G>
__device__ __forceinline__ void load_frags(Frags& f, unsigned base) {
  f.h0 = frag16<4 * G + 0>(base);
  f.l0 = frag16<4 * G + 1>(base);
  f.h1 = frag16<4 * G + 2>(base);
  f.l1 = frag16<4 * G + 3>(base);
}

__device__ __forceinline__ void mfma3x2(f32x4& c0, f32x4& c1, const Frags& a, const Split& b) {
  c0 = MFMA16(a.h0, b.h, c0);
  c1 = MFMA16(a.h1, b.h, c1);
  c0 = MFMA16(a.h0, b.l, c0);
  c1 = MFMA16(a.h1, b.l, c1);
  c0 = MFMA16(a.l0, b.h, c0);
  c1 = MFMA16(a.l1, b.h, c1);
}

// Group G of NG: drain its fragment reads (issued one group earlier), issue
// group G+1's into the other register set, 6 MFMAs, then (every other group)
// one LDS-DMA piece of the slice three ahead.
template <int G, int NG, typename Cfg, typename Acc, typename BV>
__device__ __forceinline__ void run_group3(Acc& acc, unsigned base, const BV& bv, Frags& x,
                                           Frags& y, const Dma& dma) {
  if constexpr (G < NG) {
    lds_drain();
    if constexpr (G + 1 < NG) {
      if constexpr ((G & 1) == 0) load_frags<G + 1>(y, base);
      else load_frags<G + 1>(x, base);
    }
    __builtin_amdgcn_sched_barrier(0);
    constexpr int m = Cfg::tile(G);
    if constexpr ((G & 1) == 0) mfma3x2(acc[m], acc[m + 1], x, bv[Cfg::bsel(G)]);
    else mfma3x2(acc[m], acc[m + 1], y, bv[Cfg::bsel(G)]);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr ((G & 1) == 0 && G / 2 < kBlocksPerWave) {
      if (dma.src) stage_piece(dma.src, dma.dst, dma.wave, dma.lane, G / 2);
    }
    __builtin_amdgcn_sched_barrier(0);
    run_group3<G + 1, NG, Cfg>(acc, base, bv, x, y, dma);
  }
}

template <int NG, typename Cfg, typename Acc, typename BV>
__device__ __forceinline__ void run_slice3(Acc& acc, const float* buf, int lane, const BV& bv,
                                           const Dma& dma) {
  const unsigned base = lds_base(buf, lane);
  Frags x, y;
  load_frags<0>(x, base);
  y = x;
  run_group3<0, NG, Cfg>(acc, base, bv, x, y, dma);
}

// 256-row layer slice = one K step (operand Q): groups G -> tiles 2G, 2G+1.
template <int Q>
struct Step256 {
  static constexpr int tile(int g) { return 2 * g; }
  static constexpr int bsel(int) { return Q; }
};
// views slices = two K steps (operands Q0, Q0+1) x 8 tiles.
template <int Q0>
struct StepViews {
  static constexpr int tile(int g) { return 2 * (g & 3); }
  static constexpr int bsel(int g) { return Q0 + (g >> 2); }
};

template <int Q, typename BV>
__device__ __forceinline__ void step256(f32x4 (&acc)[16], const float* buf, const BV& b, int lane,
                                        const Dma& dma) {
  run_slice3<8, Step256<Q>>(acc, buf, lane, b, dma);
}

// ---------------------------------------------------------------------------
// activations: scale, FP16 split, B operands
// ---------------------------------------------------------------------------
// max over the 4 lane groups holding one sample (lanes l, l^16, l^32, l^48)
__device__ __forceinline__ float sample_max(float v) {
  v = fmaxf(v, __shfl_xor(v, 16));
  return fmaxf(v, __shfl_xor(v, 32));
}

// exponent e with max * 2^e in [2^13, 2^14) (0 for an all-zero sample)
__device__ __forceinline__ int act_exponent(float mx) {
  if (!(mx > 0.0f)) return 0;
  int E;
  (void)frexpf(mx, &E);   // mx in [2^(E-1), 2^E)
  return 14 - E;
}

__device__ __forceinline__ void split8(const float (&v)[8], float s, Split& out) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float x = v[j] * s;
    const _Float16 h = (_Float16)x;
    out.h[j] = h;
    out.l[j] = (_Float16)(x - (float)h);
  }
}

// B operands of the 8 K steps of a 256-wide activation held in tiles
template <int Q>
__device__ __forceinline__ void act_operands(const f32x4 (&a)[16], float s, Split (&X)[Q]) {
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[j] = a[2 * q][j];
      v[4 + j] = a[2 * q + 1][j];
    }
    split8(v, s, X[q]);
  }
}

template <int T>
__device__ __forceinline__ float tiles_absmax(const f32x4 (&a)[T]) {
  float m = 0.0f;
#pragma unroll
  for (int t = 0; t < T; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) m = fmaxf(m, fabsf(a[t][r]));
  return m;
}

// acc * 2^-(sw + e) + bias (+ ReLU), in place: the layer's FP32 activations.
// The power-of-two product is exact, so one fma rounds exactly like the
// reference's separate add; ReLU is a max against a uniform floor (0, or
// -inf for the feature layer) instead of a per-value select.
template <int T>
__device__ __forceinline__ void epilogue(f32x4 (&acc)[T], int shift, const float* bias, bool relu) {
  const float inv = ldexpf(1.0f, -shift);
  const float floor = relu ? 0.0f : -__builtin_inff();
#pragma unroll
  for (int m = 0; m < T; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      acc[m][r] = fmaxf(__builtin_fmaf(acc[m][r], inv, bias[4 * m + r]), floor);
}

// Frequency encoding of xyz (L=10) in this kernel's K order, lane group g:
// slot i = 8q + j (q = 0, 1) holds sin (i even) / cos (i odd) of pair
// 8g + i/2 = (band f, coordinate c) = divmod(pair, 3), for pairs < 30; lane
// group 3 ends with x, y, z, 0 in slots 12..15.
__device__ __forceinline__ void encode_xyz(const float (&p)[3], int g, float (&e)[16]) {
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const int pr = 8 * g + t;
    if (pr < 30) {
      const int f = pr / 3, c = pr - 3 * f;
      const float x = c == 0 ? p[0] : (c == 1 ? p[1] : p[2]);
      const float arg = x * (float)(1 << f);   // exact power of two (freq.py:19)
      float sv, cv;
      sincosf(arg, &sv, &cv);
      e[2 * t] = sv;
      e[2 * t + 1] = cv;
    } else {
      e[2 * t] = t == 6 ? p[0] : (t == 7 ? p[2] : 0.0f);
      e[2 * t + 1] = t == 6 ? p[1] : 0.0f;
    }
  }
}

// view-direction encoding (L=4): slots j = 2t, 2t+1 = sin, cos of (band g,
// coordinate t), t < 3; slot 6 = raw coordinate g (g < 3); slot 7 = 0.
__device__ __forceinline__ void encode_dir(const float (&d)[3], int g, float (&e)[8]) {
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    const float arg = d[t] * (float)(1 << g);
    float sv, cv;
    sincosf(arg, &sv, &cv);
    e[2 * t] = sv;
    e[2 * t + 1] = cv;
  }
  e[6] = g == 0 ? d[0] : (g == 1 ? d[1] : (g == 2 ? d[2] : 0.0f));
  e[7] = 0.0f;
}

__device__ __forceinline__ float absmax8(const float* v, int n) {
  float m = 0.0f;
  for (int i = 0; i < n; ++i) m = fmaxf(m, fabsf(v[i]));
  return m;
}

__device__ __forceinline__ void zero(f32x4* a, int n) {
  for (int m = 0; m < n; ++m) a[m] = f32x4(0.0f);
}

__global__ __launch_bounds__(kX3Threads, 2) void mlp_x3_kernel(
    const float4* __restrict__ slices, const float* __restrict__ head,
    const float* __restrict__ rays_o, const float* __restrict__ rays_d,
    const float* __restrict__ z, int64_t z_stride, int64_t total, int S,
    float4* __restrict__ raw) {
  __shared__ __attribute__((aligned(16))) float ring[4 * kSliceFloats];
  __shared__ __attribute__((aligned(16))) float hd[kHeadFloats];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int g4 = lane >> 4;
  const Ring R{ring, slices, wave, lane};

  for (int t = 0; t < 3; ++t)
    for (int j = 0; j < kBlocksPerWave; ++j)
      stage_piece(slices + (size_t)t * (kSliceFloats / 4), R.buf(t), wave, lane, j);
  for (int i = tid; i < kHeadFloats / 4; i += kX3Threads)
    reinterpret_cast<float4*>(hd)[i] = reinterpret_cast<const float4*>(head)[i];

  const int64_t gs = (int64_t)blockIdx.x * kX3Tile + wave * 16 + (lane & 15);
  const bool valid = gs < total;
  const int64_t gc = valid ? gs : total - 1;
  const int64_t ray = gc / S;
  const int step = (int)(gc - ray * S);
  const float zv = z[ray * z_stride + step];
  float p[3], dv[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    dv[c] = rays_d[ray * 3 + c];
    p[c] = rays_o[ray * 3 + c] + dv[c] * zv;      // VR:165: o + d*z, two roundings
  }
  float encf[16];
  encode_xyz(p, g4, encf);
  const float enc_max = sample_max(absmax8(encf, 16));

  f32x4 acc[16];
  Split X[8];
  Split E[2];
  __syncthreads();   // head, z/rays loads and the three prologue slices resident

  // ---- layer 0: 63 -> 256 (slices 0, 1) ------------------------------------
  int e = act_exponent(enc_max);
  {
    const float s = ldexpf(1.0f, e);
    split8(*reinterpret_cast<const float(*)[8]>(&encf[0]), s, E[0]);
    split8(*reinterpret_cast<const float(*)[8]>(&encf[8]), s, E[1]);
  }
  zero(acc, 16);
  step256<0>(acc, R.buf(0), E, lane, R.dma_for(0)); slice_end<2>();
  step256<1>(acc, R.buf(1), E, lane, R.dma_for(1)); slice_end<2>();
  epilogue(acc, (int)hd[kHeadScales + 0] + e, hd + kHeadBias + g4 * 64, true);
  int g = 2;

  float alpha = 0.0f;
  for (int L = 1; L <= 8; ++L) {
    // scale of this layer's input (the skip layer shares it with the encoding)
    float mx = tiles_absmax(acc);
    if (L == 5) mx = fmaxf(mx, enc_max);
    e = act_exponent(sample_max(mx));
    const float s = ldexpf(1.0f, e);
    act_operands(acc, s, X);
    zero(acc, 16);
    if (L == 5) {   // cat(input_pts, h): the encoded input first (NET:57-58)
      split8(*reinterpret_cast<const float(*)[8]>(&encf[0]), s, E[0]);
      split8(*reinterpret_cast<const float(*)[8]>(&encf[8]), s, E[1]);
      step256<0>(acc, R.buf(g), E, lane, R.dma_for(g)); slice_end<2>();
      step256<1>(acc, R.buf(g + 1), E, lane, R.dma_for(g + 1)); slice_end<2>();
      g += 2;
    }
    step256<0>(acc, R.buf(g + 0), X, lane, R.dma_for(g + 0)); slice_end<2>();
    step256<1>(acc, R.buf(g + 1), X, lane, R.dma_for(g + 1)); slice_end<2>();
    step256<2>(acc, R.buf(g + 2), X, lane, R.dma_for(g + 2)); slice_end<2>();
    step256<3>(acc, R.buf(g + 3), X, lane, R.dma_for(g + 3)); slice_end<2>();
    step256<4>(acc, R.buf(g + 4), X, lane, R.dma_for(g + 4)); slice_end<2>();
    step256<5>(acc, R.buf(g + 5), X, lane, R.dma_for(g + 5)); slice_end<2>();
    step256<6>(acc, R.buf(g + 6), X, lane, R.dma_for(g + 6)); slice_end<2>();
    step256<7>(acc, R.buf(g + 7), X, lane, R.dma_for(g + 7)); slice_end<2>();
    g += 8;
    epilogue(acc, (int)hd[kHeadScales + L] + e, hd + kHeadBias + L * 256 + g4 * 64, L != 8);
    if (L == 7) {   // density head on h (NET:61), FP32 on the VALU
      const float* aw = hd + kHeadAlphaW + g4 * 64;
      float part = 0.0f;
#pragma unroll
      for (int m = 0; m < 16; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r) part = __builtin_fmaf(acc[m][r], aw[4 * m + r], part);
      alpha = quad_sum(part) + hd[kHeadAlphaB];
    }
  }

  // ---- views layer: cat(feature, input_views) 283 -> 128, ReLU (NET:62-67) -
  float dirf[8];
  encode_dir(dv, g4, dirf);
  e = act_exponent(sample_max(fmaxf(tiles_absmax(acc), absmax8(dirf, 8))));
  {
    const float s = ldexpf(1.0f, e);
    act_operands(acc, s, X);
    split8(dirf, s, E[0]);
  }
  f32x4 acc8[8];
  zero(acc8, 8);
  run_slice3<8, StepViews<0>>(acc8, R.buf(g), lane, X, R.dma_for(g)); slice_end<2>();           // 68
  run_slice3<8, StepViews<2>>(acc8, R.buf(g + 1), lane, X, R.dma_for(g + 1)); slice_end<2>();   // 69
  run_slice3<8, StepViews<4>>(acc8, R.buf(g + 2), lane, X, R.dma_for(g + 2)); slice_end<1>();   // 70
  run_slice3<8, StepViews<6>>(acc8, R.buf(g + 3), lane, X, R.dma_for(g + 3)); slice_end<0>();   // 71
  run_slice3<4, Step256<0>>(acc8, R.buf(g + 4), lane, E, R.dma_for(g + 4));                     // 72
  epilogue(acc8, (int)hd[kHeadScales + 9] + e, hd + kHeadBiasViews + g4 * 32, true);

  // ---- rgb head (NET:68-70), FP32 on the VALU --------------------------------
  float part[3] = {0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c)
        part[c] = __builtin_fmaf(acc8[m][r], hd[kHeadRgbW + c * 128 + g4 * 32 + 4 * m + r], part[c]);
  float rgb[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) rgb[c] = quad_sum(part[c]) + hd[kHeadRgbB + c];
  if (valid && g4 == 0) raw[gs] = make_float4(rgb[0], rgb[1], rgb[2], alpha);
}

}  // namespace nerfhip

using namespace nerfhip;

extern "C" int nerf_mlp_forward_x3(const float* w_slices, const float* w_head, const float* rays_o,
                                   const float* rays_d, const float* z, int64_t z_stride,
                                   int64_t n, int S, float* raw, nerf_stream_t stream) {
  NERF_REQUIRE(w_slices && w_head && rays_o && rays_d && z && raw,
               "nerf_mlp_forward_x3: null pointer");
  NERF_REQUIRE(n >= 0 && S >= 1 && z_stride >= 0, "nerf_mlp_forward_x3: bad size");
  NERF_REQUIRE(((uintptr_t)w_slices & 15) == 0 && ((uintptr_t)w_head & 15) == 0 &&
                   ((uintptr_t)raw & 15) == 0,
               "nerf_mlp_forward_x3: weights/raw must be 16-byte aligned");
  const int64_t total = n * S;
  if (total == 0) return 0;
  const int64_t blocks = cdiv(total, kX3Tile);
  NERF_REQUIRE(blocks < (1ll << 31), "nerf_mlp_forward_x3: too many samples for one launch");
  hipLaunchKernelGGL(mlp_x3_kernel, dim3((unsigned)blocks), dim3(kX3Threads), 0,
                     as_stream(stream), (const float4*)w_slices, w_head, rays_o, rays_d, z,
                     z_stride, total, S, (float4*)raw);
  return check_launch("mlp_x3_kernel");
}
