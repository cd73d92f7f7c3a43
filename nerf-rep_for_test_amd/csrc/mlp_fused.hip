// Fused NeRF MLP forward on gfx950: frequency encoding + the 8x256 network of
// reference src/models/nerf/network.py:49-74 (NET), FP32 MFMA.
//
// Work decomposition
//   workgroup = 4 waves = 128 consecutive samples (sample = ray * S + step);
//   wave = 32 samples = the N dimension of v_mfma_f32_32x32x2_f32.
//   Every layer is out^T[F x 32] = W[F x K] . in^T[K x 32]: weights are the
//   A operand (rows = output features), activations the B operand.
//
// Register dataflow (no LDS round trip for activations)
//   The 32x32 accumulator of output tile m holds, on lane l, sample l&31 and
//   output features 32m + (r&3) + 8(r>>2) + 4(l>>5) in register r (0..15).
//   The next layer consumes register r of tile m as its B operand at k-step
//   s = 16m + r: lane half h = l>>5 supplies K index "slot h" of that step. The
//   host packs each weight matrix with exactly that K permutation
//   (nerfhip/pack.py), so accumulators feed the next MFMA chain in place.
//   Encoded inputs use their own K order: k-step 0 = (x | y), 1 = (z | 0),
//   2+3f+c = (sin(2^f p_c) | cos(2^f p_c)).
//
// Weight streaming
//   The packed network is 73 slices of 32 KiB (32 "blocks" of 64 lanes x 16 B:
//   one ds_read_b128 per lane = 4 consecutive k-steps of one 32-row tile).
//   Slices stream HBM/L2 -> LDS with global_load_lds_dwordx4 into a 2-deep
//   ring (two LDS arrays, statically selected), one barrier per slice; 128
//   MFMAs (8192 cycles per SIMD) per slice hide the next slice's load.
//   Density (1x256) and rgb (3x128) heads run on the VALU (fma chains + one
//   cross-half add) instead of padding 31/29 of 32 MFMA rows.
#include "common.h"

namespace nerfhip {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kThreads = 256;
constexpr int kTile = 128;
constexpr int kSliceFloats = NERF_MLP_SLICE_FLOATS;
constexpr int kSlices = NERF_MLP_SLICES;
constexpr int kHeadFloats = NERF_MLP_HEAD_FLOATS;

// head block layout (floats); bias/weight vectors are lane-half packed:
// element [h][16m + r] belongs to output feature 32m + (r&3) + 8(r>>2) + 4h.
constexpr int kHeadBias = 0;          // layers 0..8 (pts 0..7, feature): [9][2][128]
constexpr int kHeadBiasViews = 2304;  // [2][64]
constexpr int kHeadAlphaW = 2432;     // [2][128]
constexpr int kHeadAlphaB = 2688;     // [1]
constexpr int kHeadRgbW = 2692;       // [3][2][64]
constexpr int kHeadRgbB = 3076;       // [3]

typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ void stage_slice(const float4* __restrict__ slices, int g,
                                            float* dst, int wave, int lane) {
  if (g >= kSlices) return;
  const float4* src = slices + (size_t)g * (kSliceFloats / 4);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int b = wave * 8 + j;
    __builtin_amdgcn_global_load_lds((const void*)(src + b * 64 + lane),
                                     (lds_ptr_t)(dst + b * 256), 16, 0, 0);
  }
  // keep the DMA issue ahead of this slice's MFMAs (the scheduler would
  // otherwise sink it to the barrier and expose its latency)
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ float4 frag(const float* buf, int block, int lane) {
  return *reinterpret_cast<const float4*>(buf + (block * 64 + lane) * 4);
}

#define MFMA(a, b, c) __builtin_amdgcn_mfma_f32_32x32x2f32((a), (b), (c), 0, 0, 0)

// 256-row layer slice: 4 quads x 8 tiles, B operand = 16 k-steps in bv.
__device__ __forceinline__ void slice256(f32x16 (&acc)[8], const float* buf, const f32x16& bv,
                                         int lane) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const float4 a = frag(buf, q * 8 + m, lane);
      acc[m] = MFMA(a.x, bv[4 * q + 0], acc[m]);
      acc[m] = MFMA(a.y, bv[4 * q + 1], acc[m]);
      acc[m] = MFMA(a.z, bv[4 * q + 2], acc[m]);
      acc[m] = MFMA(a.w, bv[4 * q + 3], acc[m]);
    }
  }
}

// 128-row layer slice: NQ quads x 4 tiles; k-steps from b0 (quads 0..3), b1 (4..7).
template <int NQ>
__device__ __forceinline__ void slice128(f32x16 (&acc)[4], const float* buf, const f32x16& b0,
                                         const f32x16& b1, int lane) {
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const f32x16& bv = q < 4 ? b0 : b1;
    const int qq = q & 3;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const float4 a = frag(buf, q * 4 + m, lane);
      acc[m] = MFMA(a.x, bv[4 * qq + 0], acc[m]);
      acc[m] = MFMA(a.y, bv[4 * qq + 1], acc[m]);
      acc[m] = MFMA(a.z, bv[4 * qq + 2], acc[m]);
      acc[m] = MFMA(a.w, bv[4 * qq + 3], acc[m]);
    }
  }
}

// Frequency encoding in the kernel's K order (see header). p: input 3-vector;
// nf bands; out: 2 + 3*nf k-steps (rest zero). Lane half h picks sin|cos.
template <int NF, int NV>
__device__ __forceinline__ void encode(const float (&p)[3], int h, f32x16 (&out)[NV]) {
#pragma unroll
  for (int v = 0; v < NV; ++v) out[v] = f32x16(0.0f);
  out[0][0] = h ? p[1] : p[0];
  out[0][1] = h ? 0.0f : p[2];
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    const float scale = (float)(1 << f);      // 2^f exact: x * 2^f is exact
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const int s = 2 + 3 * f + c;
      const float arg = p[c] * scale;
      float sv, cv;
      sincosf(arg, &sv, &cv);
      out[s >> 4][s & 15] = h ? cv : sv;
    }
  }
}

__device__ __forceinline__ void bias_act(f32x16 (&act)[8], const f32x16 (&acc)[8],
                                         const float* bias, bool relu) {
#pragma unroll
  for (int m = 0; m < 8; ++m) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float v = acc[m][r] + bias[16 * m + r];
      act[m][r] = relu ? fmaxf(v, 0.0f) : v;
    }
  }
}

__global__ __launch_bounds__(kThreads, 1) void mlp_fused_kernel(
    const float4* __restrict__ slices, const float* __restrict__ head,
    const float* __restrict__ rays_o, const float* __restrict__ rays_d,
    const float* __restrict__ z, int64_t z_stride, int64_t total, int S,
    float4* __restrict__ raw) {
  __shared__ __attribute__((aligned(16))) float ring0[kSliceFloats];
  __shared__ __attribute__((aligned(16))) float ring1[kSliceFloats];
  __shared__ __attribute__((aligned(16))) float hd[kHeadFloats];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int h = lane >> 5;

  stage_slice(slices, 0, ring0, wave, lane);
  for (int i = tid; i < kHeadFloats / 4; i += kThreads)
    reinterpret_cast<float4*>(hd)[i] = reinterpret_cast<const float4*>(head)[i];

  // this lane's sample (lanes l and l+32 share sample l&31)
  const int64_t gs = (int64_t)blockIdx.x * kTile + wave * 32 + (lane & 31);
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
  f32x16 enc[2];
  encode<10, 2>(p, h, enc);

  f32x16 acc[8], act[8];
  __syncthreads();   // slice 0 + head resident

  // ---- layer 0: 63 -> 256 (2 slices) --------------------------------------
#pragma unroll
  for (int m = 0; m < 8; ++m) acc[m] = f32x16(0.0f);
  stage_slice(slices, 1, ring1, wave, lane);
  slice256(acc, ring0, enc[0], lane);
  __syncthreads();
  stage_slice(slices, 2, ring0, wave, lane);
  slice256(acc, ring1, enc[1], lane);
  __syncthreads();
  bias_act(act, acc, hd + kHeadBias + 0 * 256 + h * 128, true);
  int g = 2;   // next slice to compute (always even at a layer start)

  float alpha = 0.0f;
  // ---- layers 1..7 (skip input at 5) + feature (8, no ReLU) ----------------
  for (int L = 1; L <= 8; ++L) {
#pragma unroll
    for (int m = 0; m < 8; ++m) acc[m] = f32x16(0.0f);
    if (L == 5) {   // cat(input_pts, h): the encoded input first (NET:57-58)
      stage_slice(slices, g + 1, ring1, wave, lane);
      slice256(acc, ring0, enc[0], lane);
      __syncthreads();
      stage_slice(slices, g + 2, ring0, wave, lane);
      slice256(acc, ring1, enc[1], lane);
      __syncthreads();
      g += 2;
    }
#pragma unroll
    for (int i = 0; i < 8; i += 2) {
      stage_slice(slices, g + 1, ring1, wave, lane);
      slice256(acc, ring0, act[i], lane);
      __syncthreads();
      stage_slice(slices, g + 2, ring0, wave, lane);
      slice256(acc, ring1, act[i + 1], lane);
      __syncthreads();
      g += 2;
    }
    bias_act(act, acc, hd + kHeadBias + L * 256 + h * 128, L != 8);
    if (L == 7) {   // density head on h (NET:61): VALU dot + cross-half add
      const float* aw = hd + kHeadAlphaW + h * 128;
      float part = 0.0f;
#pragma unroll
      for (int m = 0; m < 8; ++m)
#pragma unroll
        for (int r = 0; r < 16; ++r) part = __builtin_fmaf(act[m][r], aw[16 * m + r], part);
      alpha = (part + __shfl_xor(part, 32)) + hd[kHeadAlphaB];
    }
  }

  // ---- views layer: cat(feature, input_views) 283 -> 128, ReLU (NET:62-67) -
  f32x16 acc4[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) acc4[m] = f32x16(0.0f);
#pragma unroll
  for (int i = 0; i < 4; i += 2) {
    stage_slice(slices, g + 1, ring1, wave, lane);
    slice128<8>(acc4, ring0, act[2 * i], act[2 * i + 1], lane);
    __syncthreads();
    stage_slice(slices, g + 2, ring0, wave, lane);
    slice128<8>(acc4, ring1, act[2 * i + 2], act[2 * i + 3], lane);
    __syncthreads();
    g += 2;
  }
  f32x16 dir[1];
  encode<4, 1>(dv, h, dir);
  slice128<4>(acc4, ring0, dir[0], dir[0], lane);

  // ---- rgb head (NET:68-70) on the VALU ------------------------------------
  const float* bvw = hd + kHeadBiasViews + h * 64;
  float part[3] = {0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int m = 0; m < 4; ++m) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float v = fmaxf(acc4[m][r] + bvw[16 * m + r], 0.0f);
#pragma unroll
      for (int c = 0; c < 3; ++c)
        part[c] = __builtin_fmaf(v, hd[kHeadRgbW + c * 128 + h * 64 + 16 * m + r], part[c]);
    }
  }
  float rgb[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) rgb[c] = (part[c] + __shfl_xor(part[c], 32)) + hd[kHeadRgbB + c];
  if (valid && h == 0) raw[gs] = make_float4(rgb[0], rgb[1], rgb[2], alpha);
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
