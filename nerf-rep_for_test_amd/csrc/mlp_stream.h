// Weight streaming shared by the fused MLP kernels (mlp_fused.hip: FP32 MFMA,
// mlp_x3.hip: 3-term FP16 split MFMA): a packed network of 73 slices of
// 32 KiB (32 blocks of 64 lanes x 16 B) streams L2 -> LDS by LDS-DMA through a
// 4-deep ring while 8 waves multiply the resident slice; fragments are read
// with inline-asm ds_read_b128 at immediate block offsets.
#pragma once

#include "common.h"

namespace nerfhip {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;

constexpr int kSliceFloats = NERF_MLP_SLICE_FLOATS;
constexpr int kSlices = NERF_MLP_SLICES;
constexpr int kHeadFloats = NERF_MLP_HEAD_FLOATS;
constexpr int kStreamWaves = 8;                     // waves per workgroup
constexpr int kBlocksPerWave = 32 / kStreamWaves;   // glds pieces each wave stages per slice

// head block layout (floats); bias/weight vectors are lane-group packed:
// element [g4][4m + r] belongs to output feature 16m + 4*g4 + r.
constexpr int kHeadBias = 0;          // layers 0..8 (pts 0..7, feature): [9][4][64]
constexpr int kHeadBiasViews = 2304;  // [4][32]
constexpr int kHeadAlphaW = 2432;     // [4][64]
constexpr int kHeadAlphaB = 2688;     // [1]
constexpr int kHeadRgbW = 2692;       // [3][4][32]
constexpr int kHeadRgbB = 3076;       // [3]
constexpr int kHeadScales = 3080;     // mlp_x3: per-layer weight scale exponents [10]

// One 1-KiB LDS-DMA piece (of the 4 each wave stages per slice): block
// wave*4 + j of slice `src` into the same block of LDS buffer `dst`.
// The piece index J is the instruction's immediate offset, which applies to the
// global and the LDS address alike: a wave's 4 pieces of a slice share one
// address VGPR pair and one M0 value.
// DMA of one future slice by one wave, spread over the MFMA groups of the
// current one: this lane's source (block wave*4 of the slice) and the wave's
// LDS destination; live is false when there is no slice left to stage.
// MLP_DMA_BUF (set by the including kernel file, not a tuning switch: the x3
// kernel defines 1, the FP32 kernel leaves 0): the pieces as `buffer_load_dwordx4
// ... lds` against one buffer descriptor of the packed network -- the slice's
// byte offset rides in an SGPR (soffset) and each lane's 32-bit offset in the
// wave's 4 blocks is constant for the whole kernel -- instead of
// global_load_lds with a 64-bit per-lane address per slice.
#ifndef MLP_DMA_BUF
#define MLP_DMA_BUF 0
#endif

#if MLP_DMA_BUF
struct Dma {
  __amdgpu_buffer_rsrc_t rsrc;
  unsigned soff;   // slice byte offset (wave-uniform)
  unsigned voff;   // this lane's byte offset in the slice: block wave*4, lane
  float* dst;
  int wave;
  int live;
};

// blocks b0.. of slice t of a packed network of nslices slices at `slices`
// (t >= nslices or !live: nothing to stage)
__device__ __forceinline__ Dma make_dma_blocks(const float4* slices, int t, float* buf, int b0,
                                               int wave, int lane, bool live,
                                               int nslices = kSlices) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
      (void*)slices, 0, nslices * kSliceFloats * 4, 0x00020000);
  return Dma{r, (unsigned)__builtin_amdgcn_readfirstlane(t * kSliceFloats * 4),
             (unsigned)((b0 * 64 + lane) * 16), buf + b0 * 256, wave,
             __builtin_amdgcn_readfirstlane(live && t < nslices ? 1 : 0)};
}

// slice t of the packed network at `slices` (t >= kSlices: nothing to stage)
__device__ __forceinline__ Dma make_dma(const float4* slices, int t, float* buf, int wave,
                                        int lane) {
  return make_dma_blocks(slices, t, buf, wave * kBlocksPerWave, wave, lane, true);
}

// piece J (0..7) of the wave's blocks: the 12-bit instruction offset reaches
// pieces 0-3; pieces 4-7 move the LDS base and soffset by 4 KiB
template <int J>
__device__ __forceinline__ void stage_piece(const Dma& d) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(d.rsrc, (lds_ptr_t)(d.dst + (J / 4) * 1024), 16,
                                           d.voff, d.soff + (J / 4) * 4096, (J % 4) * 1024, 0);
}
#else
struct Dma {
  const float4* src;
  float* dst;
  int wave;
  int live;    // wave-uniform: a slice is left to stage
};

// slice t of the packed network at `slices` (t >= kSlices: nothing to stage)
__device__ __forceinline__ Dma make_dma(const float4* slices, int t, float* buf, int wave,
                                        int lane) {
  const int b = wave * kBlocksPerWave;
  const float4* slice = t < kSlices ? slices + (size_t)t * (kSliceFloats / 4) : nullptr;
  return Dma{slice + b * 64 + lane, buf + b * 256, wave,
             __builtin_amdgcn_readfirstlane(slice != nullptr ? 1 : 0)};
}

template <int J>
__device__ __forceinline__ void stage_piece(const Dma& d) {
  __builtin_amdgcn_global_load_lds((const void*)d.src, (lds_ptr_t)d.dst, 16, J * 1024, 0);
}
#endif

// all 4 pieces of a slice (prologue)
__device__ __forceinline__ void stage_slice(const Dma& d) {
  stage_piece<0>(d);
  stage_piece<1>(d);
  stage_piece<2>(d);
  stage_piece<3>(d);
}

// LDS fragment reads are issued as inline asm: hipcc neither tracks nor waits
// for them, so the schedule below owns every lgkmcnt wait of the slice loop
// (hipcc's own waits there are lgkmcnt(0) placed after the next group's reads,
// which serialises the LDS latency with the MFMAs). One per-lane base address
// per buffer; the block offset is an instruction immediate.
__device__ __forceinline__ unsigned lds_base(const float* buf, int lane) {
  return (unsigned)(uintptr_t)(__attribute__((address_space(3))) const float*)(buf) +
         (unsigned)(lane * 16);
}

template <int BLOCK>
__device__ __forceinline__ float4 frag_async(unsigned base) {
  f32x4 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(base), "i"(BLOCK * 1024) : "memory");
  return make_float4(v[0], v[1], v[2], v[3]);
}

__device__ __forceinline__ void lds_drain() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);   // keep MFMAs behind the wait (guide rule 18)
}

// 4-deep slice ring: while slice g is computed, slices g+1 and g+2 are landed
// or landing and slice g+3 is being staged into buffer (g+3)%4 (freed by the
// barrier that ended slice g-1). At the end of slice g each wave waits only for
// its own DMA of slice g+1 (counted vmcnt: the pieces of g+2 and g+3 may stay
// in flight), then one raw s_barrier makes slice g+1 visible to all waves.
struct Ring {
  float* base;                     // 4 x kSliceFloats
  const float4* slices;            // packed network in HBM
  int wave, lane;
  int rot = 0;                     // ring rotation of a persistent stream (tiles x slices)
  __device__ float* buf(int g) const { return base + ((g + rot) & 3) * kSliceFloats; }
  __device__ Dma dma_for(int g) const {   // the DMA issued while computing slice g
    const int t = g + 3;
    return make_dma(slices, t, buf(t), wave, lane);
  }
};

// PENDING slices (of PIECES pieces each per wave) allowed to stay in flight
template <int PENDING, int PIECES = 4>
__device__ __forceinline__ void slice_end() {
  constexpr int n = (PENDING >= 2 ? 2 : PENDING) * PIECES;
  static_assert(n < 64, "vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(n) : "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// Cross-lane exchange of the 4 lane groups (rows of 16 lanes) that hold one
// sample: gfx950's v_permlane16_swap / v_permlane32_swap (VALU, no LDS traffic
// or lgkmcnt wait, unlike ds_bpermute): swapping a value with itself leaves the
// row pair (r0, r1) as (r0, r0) | (r1, r1), so a lane sees its xor-16 (xor-32)
// partner in the other result.
// (v[l], v[l ^ 16]) in some order: both results of the swap
__device__ __forceinline__ void pair16(float v, float& a, float& b) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  a = __uint_as_float(r[0]);
  b = __uint_as_float(r[1]);
}
__device__ __forceinline__ void pair32(float v, float& a, float& b) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  a = __uint_as_float(r[0]);
  b = __uint_as_float(r[1]);
}

// sum over the 4 lane groups holding one sample (lanes l, l^16, l^32, l^48);
// every lane of the quad ends with the bitwise-same value
// ((v_l + v_l^16) + (v_l^32 + v_l^48): addition commutes)
__device__ __forceinline__ float quad_sum(float v) {
  float a, b;
  pair16(v, a, b);
  v = a + b;
  pair32(v, a, b);
  return a + b;
}

}  // namespace nerfhip
