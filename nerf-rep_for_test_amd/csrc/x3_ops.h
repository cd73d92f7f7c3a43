// Device helpers of the x3 MLP kernels (mlp_x3.hip: the inference kernel
// and the training kernels): FP16 hi/lo operand splits, per-sample
// power-of-two scales, the 16x16x32 f16 MFMA triple, LDS fragment reads,
// encodings.
#pragma once

#include "mlp_stream.h"

namespace nerfhip {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half2_t __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x8 __attribute__((ext_vector_type(8)));

// B operand of one K step in 8 VGPRs: the 8 FP32 activations before the split,
// the FP16 hi halves (VGPRs 0-3) and lo halves (VGPRs 4-7) after it.
typedef f32x8 Op;

#define MFMA16(a, b, c) __builtin_amdgcn_mfma_f32_16x16x32_f16((a), (b), (c), 0, 0, 0)

__device__ __forceinline__ unsigned lds_addr(const float* p) {
  return (unsigned)(uintptr_t)(__attribute__((address_space(3))) const float*)(p);
}

__device__ __forceinline__ half8 op_hi(const Op& v) {
  return __builtin_bit_cast(half8, __builtin_shufflevector(v, v, 0, 1, 2, 3));
}
__device__ __forceinline__ half8 op_lo(const Op& v) {
  return __builtin_bit_cast(half8, __builtin_shufflevector(v, v, 4, 5, 6, 7));
}

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

// FIRST: the layer's first K step starts the accumulators from zero (no
// clearing pass over them between layers).
// The order of a tile pair's 6 products: each tile's three back to back (one
// dependent accumulator chain, the A fragment held for two MFMAs). Measured
// 2.7 % faster on the inference kernel than the two tiles interleaved (same
// per-tile summation order, bitwise-equal results; round 2, timing-only A/B:
// 23.35 vs 23.99 ms over 160 000 x 64 samples, profiles/r2_x3_order.log) --
// the chip holds a higher clock under the chained order.
template <bool FIRST>
__device__ __forceinline__ void mfma3x2(f32x4& c0, f32x4& c1, const Frags& a, const Op& b) {
  const half8 bh = op_hi(b), bl = op_lo(b);
  c0 = MFMA16(a.h0, bh, FIRST ? f32x4(0.0f) : c0);
  c0 = MFMA16(a.h0, bl, c0);
  c0 = MFMA16(a.l0, bh, c0);
  c1 = MFMA16(a.h1, bh, FIRST ? f32x4(0.0f) : c1);
  c1 = MFMA16(a.h1, bl, c1);
  c1 = MFMA16(a.l1, bh, c1);
}

// Slice shapes: the tiles, the B operand and whether the group starts its
// tiles from zero (F: the layer's first slice; each tile only once).
// 256-row layer slice = one K step (operand Q): groups G -> tiles 2G, 2G+1.
template <int Q, bool F = false>
struct Step256 {
  static constexpr bool first(int) { return F; }
  static constexpr int tile(int g) { return 2 * g; }
  static constexpr int bsel(int) { return Q; }
};
// views slices = two K steps (operands Q0, Q0+1) x 8 tiles: groups 4-7
// revisit the tiles of groups 0-3 with the second K step.
template <int Q0, bool F = false>
struct StepViews {
  static constexpr bool first(int g) { return F && g < 4; }
  static constexpr int tile(int g) { return 2 * (g & 3); }
  static constexpr int bsel(int g) { return Q0 + (g >> 2); }
};

// 64-row slices (the encoding rows of the backward: 4 tiles) = four K steps
// (operands Q0 .. Q0+3) x 2 tile pairs: groups 2k, 2k+1 = K step Q0+k.
template <int Q0, bool F = false>
struct StepEnc4 {
  static constexpr bool first(int g) { return F && g < 2; }
  static constexpr int tile(int g) { return 2 * (g & 1); }
  static constexpr int bsel(int g) { return Q0 + (g >> 1); }
};

// ---------------------------------------------------------------------------
// activations: scale, FP16 split, B operands
// ---------------------------------------------------------------------------
// max over the 4 lane groups holding one sample (lanes l, l^16, l^32, l^48)
__device__ __forceinline__ float sample_max(float v) {
  float a, b;
  pair16(v, a, b);
  v = fmaxf(a, b);
  pair32(v, a, b);
  return fmaxf(a, b);
}

// exponent e with max * 2^e in [2^13, 2^14) (0 for an all-zero sample), at
// most kMaxActExp: a sample whose values are all below 2^-50 (training: the
// gradient of a sample far behind an opaque surface underflows towards the
// FP32 denormals) would otherwise get 2^e = inf and 0 * inf = NaN; capped, its
// splits flush to 0, below the FP32 rounding of any sum it enters.
constexpr int kMaxActExp = 64;
__device__ __forceinline__ int act_exponent(float mx) {
  if (!(mx > 0.0f)) return 0;
  int E;
  (void)frexpf(mx, &E);   // mx in [2^(E-1), 2^E)
  return min(14 - E, kMaxActExp);
}

// FP16 hi/lo of two scaled values, packed: (hi pair, lo pair) as two dwords
__device__ __forceinline__ void split2(float a, float b, float s, float& hp, float& lp) {
  // hi = f16(a*s), lo = f16(a*s - hi): one mixed-precision fma each (a*s is
  // exact: s is a power of two), written straight into the halves of the packed
  // registers; the residual reads hi's f16 half in place (op_sel). 4 VALU per
  // pair (hipcc's form: 7, with a second, FP32 route to the packed hi pair).
  float h, l;
  asm("v_fma_mixlo_f16 %0, %1, %2, 0" : "=v"(h) : "v"(a), "v"(s));
  asm("v_fma_mixhi_f16 %0, %1, %2, 0" : "+v"(h) : "v"(b), "v"(s));
  asm("v_fma_mixlo_f16 %0, %1, %2, -%3 op_sel_hi:[0,0,1]" : "=v"(l) : "v"(a), "v"(s), "v"(h));
  asm("v_fma_mixhi_f16 %0, %1, %2, -%3 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "+v"(l) : "v"(b), "v"(s), "v"(h));
  hp = h;
  lp = l;
}

__device__ __forceinline__ void split_op(Op& v, float s) {
  Op o;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float hp, lp;
    split2(v[2 * k], v[2 * k + 1], s, hp, lp);
    o[k] = hp;
    o[4 + k] = lp;
  }
  v = o;
}

// Frequency encoding of xyz (L=10) in this kernel's K order, lane group g:
// slot i = 8q + j (q = 0, 1) holds sin (i even) / cos (i odd) of pair
// 8g + i/2 = (band f, coordinate c) = divmod(pair, 3), for pairs < 30; lane
// group 3 ends with x, y, z, 0 in slots 12..15.
__device__ __forceinline__ void encode_xyz(const float (&p)[3], int g, Op (&e)[2]) {
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const int pr = 8 * g + t;
    float a, b;
    if (pr < 30) {
      const int f = pr / 3, c = pr - 3 * f;
      const float x = c == 0 ? p[0] : (c == 1 ? p[1] : p[2]);
      const float arg = x * (float)(1 << f);   // exact power of two (freq.py:19)
      sincosf(arg, &a, &b);
    } else {
      a = t == 6 ? p[0] : (t == 7 ? p[2] : 0.0f);
      b = t == 6 ? p[1] : 0.0f;
    }
    e[t >> 2][(2 * t) & 7] = a;
    e[t >> 2][(2 * t + 1) & 7] = b;
  }
}

// view-direction encoding (L=4): slots j = 2t, 2t+1 = sin, cos of (band g,
// coordinate t), t < 3; slot 6 = raw coordinate g (g < 3); slot 7 = 0.
__device__ __forceinline__ void encode_dir(const float (&d)[3], int g, Op& e) {
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

__device__ __forceinline__ float op_absmax(const Op& v) {
  float m = 0.0f;
#pragma unroll
  for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(v[j]));
  return m;
}

}  // namespace nerfhip
