// Fused NeRF MLP forward on gfx950: frequency encoding + the 8x256 network of
// reference src/models/nerf/network.py:49-74 (NET), FP32 MFMA.
//
// Work decomposition
//   workgroup = 8 waves (2 per SIMD) = 128 consecutive samples
//   (sample = ray * S + step); wave = 16 samples = the N dimension of
//   v_mfma_f32_16x16x4_f32. Every layer is out^T[F x 16] = W[F x K] . in^T[K x 16]:
//   weights are the A operand (rows = output features), activations the B operand.
//
// Register dataflow (no LDS round trip for activations)
//   The 16x16 accumulator of output tile m holds, on lane l, sample l&15 and
//   output features 16m + 4(l>>4) + r in register r (0..3). The next layer
//   consumes register r of tile m as its B operand at k-step s = 4m + r: lane
//   group g4 = l>>4 supplies K slot g4 of that step. The host packs each weight
//   matrix with exactly that K permutation (nerfhip/pack.py), so accumulators
//   feed the next MFMA chain in place. Encoded inputs use their own K order:
//   k-step 0 = (x, y, z, 0), 1+t = (sin a, cos a, sin b, cos b) for the
//   (band, coordinate) pairs a = 2t, b = 2t+1.
//   Per wave: 64 activation VGPRs + 64 accumulator AGPRs, so two waves fit per
//   SIMD and fragment reads are prefetched one MFMA group ahead.
//
// Weight streaming (mlp_stream.h)
//   The packed network is 73 slices of 32 KiB (32 "blocks" of 64 lanes x 16 B:
//   one ds_read_b128 per lane = 4 consecutive k-steps of one 16-row tile).
//   Slices stream L2 -> LDS with global_load_lds_dwordx4 into a 4-deep ring,
//   issued three slices ahead; one counted vmcnt + s_barrier per slice.
//   Density (1x256) and rgb (3x128) heads run on the VALU (fma chains + a
//   4-lane butterfly) instead of padding 15/13 of 16 MFMA rows.
#include "common.h"
#include "mlp_stream.h"

namespace nerfhip {

constexpr int kWaves = kStreamWaves;
constexpr int kThreads = 64 * kWaves;
constexpr int kTile = 16 * kWaves;            // samples per workgroup

#define MFMA(a, b, c) __builtin_amdgcn_mfma_f32_16x16x4f32((a), (b), (c), 0, 0, 0)

// One group = 8 MFMAs: two 16-row tiles x the 4 k-steps of one quad; `mid`
// runs between the 4th and 5th MFMA (pinned there by sched barriers).
template <typename Mid>
__device__ __forceinline__ void mfma_group(f32x4& c0, f32x4& c1, const float4& a0,
                                           const float4& a1, const f32x4& bv, Mid mid) {
  c0 = MFMA(a0.x, bv[0], c0);
  c1 = MFMA(a1.x, bv[0], c1);
  c0 = MFMA(a0.y, bv[1], c0);
  c1 = MFMA(a1.y, bv[1], c1);
  __builtin_amdgcn_sched_barrier(0);
  mid();
  __builtin_amdgcn_sched_barrier(0);
  c0 = MFMA(a0.z, bv[2], c0);
  c1 = MFMA(a1.z, bv[2], c1);
  c0 = MFMA(a0.w, bv[3], c0);
  c1 = MFMA(a1.w, bv[3], c1);
}

// Where each wave issues its 4 weight-DMA pieces per slice (timing knobs, see
// tools/mlp_ablate.py): MLP_DMA_POS 0 = after the group's LDS drain, 1 = after
// its fragment reads, 2 = between its MFMAs, 3 = after its MFMAs;
// MLP_DMA_EVERY = group spacing of the pieces (from group MLP_DMA_FIRST).
#ifndef MLP_DMA_POS
#define MLP_DMA_POS 0
#endif
#ifndef MLP_DMA_EVERY
#define MLP_DMA_EVERY 2
#endif
#ifndef MLP_DMA_FIRST
#define MLP_DMA_FIRST 0
#endif

// Group G of NG over blocks 2G, 2G+1: drain group G's reads (issued one group
// earlier), issue group G+1's into the other named register pair, then group
// G's 8 MFMAs into tiles TILE(G), TILE(G)+1 with B operands BSEL(G).
template <int G, int NG, typename Cfg, typename Acc, typename BV>
__device__ __forceinline__ void run_group(Acc& acc, unsigned base, const BV& bv, float4& x0,
                                          float4& x1, float4& y0, float4& y1, const Dma& dma) {
  if constexpr (G < NG) {
    constexpr bool kDma = G >= MLP_DMA_FIRST && (G - MLP_DMA_FIRST) % MLP_DMA_EVERY == 0 &&
                          (G - MLP_DMA_FIRST) / MLP_DMA_EVERY < kBlocksPerWave;
    constexpr int kPiece = (G - MLP_DMA_FIRST) / MLP_DMA_EVERY;
    auto piece = [&]() {
      if constexpr (kDma) {
        if (dma.live) stage_piece<kPiece>(dma);
      }
    };
    lds_drain();
    if constexpr (MLP_DMA_POS == 0) piece();
    if constexpr (G + 1 < NG) {
      if constexpr ((G & 1) == 0) {
        y0 = frag_async<2 * G + 2>(base);
        y1 = frag_async<2 * G + 3>(base);
      } else {
        x0 = frag_async<2 * G + 2>(base);
        x1 = frag_async<2 * G + 3>(base);
      }
    }
    if constexpr (MLP_DMA_POS == 1) piece();
    __builtin_amdgcn_sched_barrier(0);
    constexpr int m = Cfg::tile(G);
    auto mid = [&]() {
      if constexpr (MLP_DMA_POS == 2) piece();
    };
    if constexpr ((G & 1) == 0)
      mfma_group(acc[m], acc[m + 1], x0, x1, bv[Cfg::bsel(G)], mid);
    else
      mfma_group(acc[m], acc[m + 1], y0, y1, bv[Cfg::bsel(G)], mid);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (MLP_DMA_POS == 3) piece();
    __builtin_amdgcn_sched_barrier(0);
    run_group<G + 1, NG, Cfg>(acc, base, bv, x0, x1, y0, y1, dma);
  }
}

template <int NG, typename Cfg, typename Acc, typename BV>
__device__ __forceinline__ void run_groups(Acc& acc, const float* buf, int lane, const BV& bv,
                                           const Dma& dma) {
  const unsigned base = lds_base(buf, lane);
  float4 x0 = frag_async<0>(base), x1 = frag_async<1>(base);
  float4 y0 = x0, y1 = x1;
  run_group<0, NG, Cfg>(acc, base, bv, x0, x1, y0, y1, dma);
}

// Slice shapes: which accumulator tiles and B-operand vectors group g uses.
// 256-row layers: 2 quads x 16 tiles (quad g>>3, tiles 2(g&7), +1);
// 128-row layers: 4 quads x 8 tiles (quad g>>2, tiles 2(g&3), +1).
template <int QBASE>
struct Slice256 {
  static constexpr int tile(int g) { return 2 * (g & 7); }
  static constexpr int bsel(int g) { return QBASE + (g >> 3); }
};
template <int QBASE>
struct Slice128 {
  static constexpr int tile(int g) { return 2 * (g & 3); }
  static constexpr int bsel(int g) { return QBASE + (g >> 2); }
};

// 256-row layer slice SL of a layer (B operand vectors b[2*SL], b[2*SL+1]).
template <int SL, typename BV>
__device__ __forceinline__ void slice256(f32x4 (&acc)[16], const float* buf, const BV& b,
                                         int lane, const Dma& dma) {
  run_groups<16, Slice256<2 * SL>>(acc, buf, lane, b, dma);
}

// 128-row layer slice of NQ quads starting at B operand vector Q0.
template <int NQ, int Q0, typename BV>
__device__ __forceinline__ void slice128(f32x4 (&acc)[8], const float* buf, const BV& b,
                                         int lane, const Dma& dma) {
  run_groups<4 * NQ, Slice128<Q0>>(acc, buf, lane, b, dma);
}

// Frequency encoding in the kernel's K order (see header) for lane group g4.
// NF bands -> 1 + ceil(3*NF/2) k-steps, zero padded to 4*NV.
template <int NF, int NV>
__device__ __forceinline__ void encode(const float (&p)[3], int g4, f32x4 (&out)[NV]) {
#pragma unroll
  for (int v = 0; v < NV; ++v) out[v] = f32x4(0.0f);
  out[0][0] = g4 == 0 ? p[0] : (g4 == 1 ? p[1] : (g4 == 2 ? p[2] : 0.0f));
  constexpr int NPAIR = 3 * NF;
#pragma unroll
  for (int t = 0; 2 * t < NPAIR; ++t) {
    const int pa = 2 * t + (g4 >> 1);        // (band, coordinate) pair of this lane group
    float v = 0.0f;
    if (pa < NPAIR) {
      const int f = pa / 3, c = pa - 3 * (pa / 3);
      const float x = c == 0 ? p[0] : (c == 1 ? p[1] : p[2]);
      const float arg = x * (float)(1 << f);    // 2^f exact: x * 2^f is exact
      float sv, cv;
      sincosf(arg, &sv, &cv);
      v = (g4 & 1) ? cv : sv;
    }
    out[(1 + t) >> 2][(1 + t) & 3] = v;
  }
}

template <int T>
__device__ __forceinline__ void bias_act(f32x4 (&act)[T], const f32x4 (&acc)[T],
                                         const float* bias, bool relu) {
#pragma unroll
  for (int m = 0; m < T; ++m) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float v = acc[m][r] + bias[4 * m + r];
      act[m][r] = relu ? fmaxf(v, 0.0f) : v;
    }
  }
}

// The 8 slices g .. g+7 of a 256-wide input layer (B = previous activations).
__device__ __forceinline__ void layer_body(f32x4 (&acc)[16], const f32x4 (&act)[16],
                                           const Ring& R, int g) {
  slice256<0>(acc, R.buf(g + 0), act, R.lane, R.dma_for(g + 0)); slice_end<2>();
  slice256<1>(acc, R.buf(g + 1), act, R.lane, R.dma_for(g + 1)); slice_end<2>();
  slice256<2>(acc, R.buf(g + 2), act, R.lane, R.dma_for(g + 2)); slice_end<2>();
  slice256<3>(acc, R.buf(g + 3), act, R.lane, R.dma_for(g + 3)); slice_end<2>();
  slice256<4>(acc, R.buf(g + 4), act, R.lane, R.dma_for(g + 4)); slice_end<2>();
  slice256<5>(acc, R.buf(g + 5), act, R.lane, R.dma_for(g + 5)); slice_end<2>();
  slice256<6>(acc, R.buf(g + 6), act, R.lane, R.dma_for(g + 6)); slice_end<2>();
  slice256<7>(acc, R.buf(g + 7), act, R.lane, R.dma_for(g + 7)); slice_end<2>();
}

__global__ __launch_bounds__(kThreads, 2) void mlp_fused_kernel(
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

  // prologue: slices 0, 1, 2 in flight; slice 3 is staged while slice 0 runs
  for (int t = 0; t < 3; ++t)
    stage_slice(make_dma(slices, t, R.buf(t), wave, lane));
  for (int i = tid; i < kHeadFloats / 4; i += kThreads)
    reinterpret_cast<float4*>(hd)[i] = reinterpret_cast<const float4*>(head)[i];

  // this lane's sample (the 4 lanes l, l+16, l+32, l+48 share sample l&15)
  const int64_t gs = (int64_t)blockIdx.x * kTile + wave * 16 + (lane & 15);
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
  f32x4 enc[4];
  encode<10, 4>(p, g4, enc);

  f32x4 acc[16], act[16];
  __syncthreads();   // head, z/rays loads and all three prologue slices resident

  // ---- layer 0: 63 -> 256 (slices 0, 1) ------------------------------------
#pragma unroll
  for (int m = 0; m < 16; ++m) acc[m] = f32x4(0.0f);
  slice256<0>(acc, R.buf(0), enc, lane, R.dma_for(0)); slice_end<2>();
  slice256<1>(acc, R.buf(1), enc, lane, R.dma_for(1)); slice_end<2>();
  bias_act(act, acc, hd + kHeadBias + 0 * 256 + g4 * 64, true);
  int g = 2;   // next slice to compute

  float alpha = 0.0f;
  // ---- layers 1..7 (skip input at 5) + feature (8, no ReLU) ----------------
  for (int L = 1; L <= 8; ++L) {
#pragma unroll
    for (int m = 0; m < 16; ++m) acc[m] = f32x4(0.0f);
    if (L == 5) {   // cat(input_pts, h): the encoded input first (NET:57-58)
      slice256<0>(acc, R.buf(g), enc, lane, R.dma_for(g)); slice_end<2>();
      slice256<1>(acc, R.buf(g + 1), enc, lane, R.dma_for(g + 1)); slice_end<2>();
      g += 2;
    }
    layer_body(acc, act, R, g);
    g += 8;
    bias_act(act, acc, hd + kHeadBias + L * 256 + g4 * 64, L != 8);
    if (L == 7) {   // density head on h (NET:61): VALU dot + lane-group butterfly
      const float* aw = hd + kHeadAlphaW + g4 * 64;
      float part = 0.0f;
#pragma unroll
      for (int m = 0; m < 16; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r) part = __builtin_fmaf(act[m][r], aw[4 * m + r], part);
      alpha = quad_sum(part) + hd[kHeadAlphaB];
    }
  }

  // ---- views layer: cat(feature, input_views) 283 -> 128, ReLU (NET:62-67) -
  // slices 68..72; the counted waits shrink as the ring runs dry
  f32x4 acc8[8];
#pragma unroll
  for (int m = 0; m < 8; ++m) acc8[m] = f32x4(0.0f);
  slice128<4, 0>(acc8, R.buf(g), act, lane, R.dma_for(g)); slice_end<2>();           // 68
  slice128<4, 4>(acc8, R.buf(g + 1), act, lane, R.dma_for(g + 1)); slice_end<2>();   // 69
  slice128<4, 8>(acc8, R.buf(g + 2), act, lane, R.dma_for(g + 2)); slice_end<1>();   // 70
  slice128<4, 12>(acc8, R.buf(g + 3), act, lane, R.dma_for(g + 3)); slice_end<0>();  // 71
  f32x4 dir[2];
  encode<4, 2>(dv, g4, dir);
  slice128<2, 0>(acc8, R.buf(g + 4), dir, lane, R.dma_for(g + 4));                   // 72

  // ---- rgb head (NET:68-70) on the VALU ------------------------------------
  const float* bvw = hd + kHeadBiasViews + g4 * 32;
  float part[3] = {0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int m = 0; m < 8; ++m) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float v = fmaxf(acc8[m][r] + bvw[4 * m + r], 0.0f);
#pragma unroll
      for (int c = 0; c < 3; ++c)
        part[c] = __builtin_fmaf(v, hd[kHeadRgbW + c * 128 + g4 * 32 + 4 * m + r], part[c]);
    }
  }
  float rgb[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) rgb[c] = quad_sum(part[c]) + hd[kHeadRgbB + c];
  if (valid && g4 == 0) raw[gs] = make_float4(rgb[0], rgb[1], rgb[2], alpha);
}

}  // namespace nerfhip

using namespace nerfhip;

extern "C" int nerf_mlp_forward(const float* w_slices, const float* w_head, const float* rays_o,
                                const float* rays_d, const float* z, int64_t z_stride, int64_t n,
                                int S, float* raw, nerf_stream_t stream) {
  NERF_REQUIRE(w_slices && w_head && rays_o && rays_d && z && raw,
               "nerf_mlp_forward: null pointer");
  NERF_REQUIRE(n >= 0 && S >= 1 && z_stride >= 0, "nerf_mlp_forward: bad size");
  NERF_REQUIRE(((uintptr_t)w_slices & 15) == 0 && ((uintptr_t)w_head & 15) == 0 &&
                   ((uintptr_t)raw & 15) == 0,
               "nerf_mlp_forward: weights/raw must be 16-byte aligned");
  const int64_t total = n * S;
  if (total == 0) return 0;
  const int64_t blocks = cdiv(total, kTile);
  NERF_REQUIRE(blocks < (1ll << 31), "nerf_mlp_forward: too many samples for one launch");
  hipLaunchKernelGGL(mlp_fused_kernel, dim3((unsigned)blocks), dim3(kThreads), 0,
                     as_stream(stream), (const float4*)w_slices, w_head, rays_o, rays_d, z,
                     z_stride, total, S, (float4*)raw);
  return check_launch("mlp_fused_kernel");
}
