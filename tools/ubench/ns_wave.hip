// Timing skeleton (no correctness) of the x3 MLP's slice loop with WPS waves
// per SIMD and NS 16-sample groups per wave: does one wave per SIMD holding
// 32 or 48 samples (each A fragment feeding NS B tiles: 1/NS of the LDS
// fragment reads per MFMA, and NS/2 x the samples per staged weight byte)
// beat the shipped two waves of 16 samples?
//
// Per slice (one 32-deep K step of a 256-row layer), as mlp_x3.hip: 8 groups,
// each draining its fragment reads (issued one group earlier), issuing the next
// group's, and running 6 MFMAs per sample group (2 tiles x 3 FP16 products);
// waves 0-3 stage the slice three ahead (8 buffer-form LDS-DMA pieces each,
// after group 0, or one per group with SPREAD); the operand split of the next
// K step in the MFMA shadows; a counted vmcnt + s_barrier per slice; the last
// slice of each layer runs the epilogue (scale-undo + bias + ReLU + running
// max) pair by pair; per layer the sample max / exponent and the first split.
// Random FP16 weights and activations (the clock the chip holds depends on the
// data: MI355X_MICROARCH.md 'DVFS give-back').
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -fno-slp-vectorize -ffp-contract=off \
//         -I nerf-rep_for_test_amd/csrc -o ns_wave tools/ubench/ns_wave.hip
#define MLP_DMA_BUF 1
#include "x3_ops.h"

#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace nerfhip;

#ifndef SPREAD
#define SPREAD 0
#endif
#ifndef SPLITW
#define SPLITW 0   // 1: counted lgkmcnt waits at each fragment's first MFMA (NS = 1 only)
#endif
#ifndef LOADHI
#define LOADHI 0   // 1: waves 4-7 stage the weights (the shipped kernel: waves 0-3)
#endif
#ifndef PRIO
#define PRIO 0     // 1: s_setprio 1 on the waves that do not stage weights
#endif

constexpr int kSl = 64;   // slices per tile (8 layers x 8 K steps)

template <int NS>
struct St {
  f32x4 acc[NS][16];
  Op X[NS][8];
  Op T[NS];
  float s[NS];
  float amax[NS];
};

template <int G, int NS, int Q>
__device__ __forceinline__ void grp(St<NS>& st, unsigned base, unsigned nbase, Frags& x, Frags& y,
                                    const Dma& dma) {
  if constexpr (G < 8) {
#if SPLITW
    // wait for each fragment right before its first MFMA (LDS reads return in
    // order): h0, then l0, h1, l1 with the next group's 4 reads behind them
    asm volatile("s_waitcnt lgkmcnt(3)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
#else
    lds_drain();
#endif
    if constexpr (G + 1 < 8) {
      if constexpr ((G & 1) == 0) load_frags<G + 1>(y, base);
      else load_frags<G + 1>(x, base);
    } else {
      load_frags<0>(x, nbase);
    }
    __builtin_amdgcn_sched_barrier(0);
#if SPLITW
    static_assert(NS == 1, "SPLITW: one sample group");
    {
      const Frags& f = (G & 1) ? y : x;
      f32x4& c0 = st.acc[0][2 * G];
      f32x4& c1 = st.acc[0][2 * G + 1];
      const half8 bh = op_hi(st.X[0][Q]), bl = op_lo(st.X[0][Q]);
      c0 = MFMA16(f.h0, bh, Q == 0 ? f32x4(0.0f) : c0);
      c0 = MFMA16(f.h0, bl, c0);
      asm volatile("s_waitcnt lgkmcnt(6)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      c0 = MFMA16(f.l0, bh, c0);
      asm volatile("s_waitcnt lgkmcnt(5)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      c1 = MFMA16(f.h1, bh, Q == 0 ? f32x4(0.0f) : c1);
      c1 = MFMA16(f.h1, bl, c1);
      asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      c1 = MFMA16(f.l1, bh, c1);
    }
#else
#pragma unroll
    for (int n = 0; n < NS; ++n) {
      if constexpr ((G & 1) == 0) mfma3x2<Q == 0>(st.acc[n][2 * G], st.acc[n][2 * G + 1], x, st.X[n][Q]);
      else mfma3x2<Q == 0>(st.acc[n][2 * G], st.acc[n][2 * G + 1], y, st.X[n][Q]);
    }
#endif
    if constexpr (Q < 7) {   // split of operand Q+1, values G, G+1 (even G)
      if constexpr ((G & 1) == 0) {
#pragma unroll
        for (int n = 0; n < NS; ++n) {
          float hp, lp;
          split2(st.X[n][Q + 1][G], st.X[n][Q + 1][G + 1], st.s[n], hp, lp);
          asm volatile("" : "+v"(hp), "+v"(lp));
          st.T[n][G / 2] = hp;
          st.T[n][4 + G / 2] = lp;
        }
      }
      if constexpr (G == 7) {
#pragma unroll
        for (int n = 0; n < NS; ++n) st.X[n][Q + 1] = st.T[n];
      }
    } else if constexpr (G >= 1) {   // epilogue of pair G-1
      constexpr int p = G - 1;
#pragma unroll
      for (int n = 0; n < NS; ++n) {
        Op v;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = fmaxf(__builtin_fmaf(st.acc[n][2 * p][r], 0.00048828125f, 0.001f * r), 0.0f);
          v[4 + r] = fmaxf(__builtin_fmaf(st.acc[n][2 * p + 1][r], 0.00048828125f, -0.001f * r), 0.0f);
        }
#pragma unroll
        for (int j = 0; j < 8; j += 2)
          asm("v_max3_f32 %0, %0, |%1|, |%2|" : "+v"(st.amax[n]) : "v"(v[j]), "v"(v[j + 1]));
        asm volatile("" : "+v"(v));
        st.X[n][p] = v;
      }
    }
#pragma unroll
    for (int k = 0; k < 6 * NS; ++k) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (dma.live) {
#if SPREAD
      stage_piece<G>(dma);
#else
      if constexpr (G == 0) {
        stage_piece<0>(dma); stage_piece<1>(dma); stage_piece<2>(dma); stage_piece<3>(dma);
        stage_piece<4>(dma); stage_piece<5>(dma); stage_piece<6>(dma); stage_piece<7>(dma);
      }
#endif
    }
    __builtin_amdgcn_sched_barrier(0);
    grp<G + 1, NS, Q>(st, base, nbase, x, y, dma);
  }
}

template <int NS>
__device__ __forceinline__ void epi_last(St<NS>& st) {
  lds_drain();
#pragma unroll
  for (int n = 0; n < NS; ++n) {
    Op v;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      v[r] = fmaxf(__builtin_fmaf(st.acc[n][14][r], 0.00048828125f, 0.001f * r), 0.0f);
      v[4 + r] = fmaxf(__builtin_fmaf(st.acc[n][15][r], 0.00048828125f, -0.001f * r), 0.0f);
    }
#pragma unroll
    for (int j = 0; j < 8; j += 2)
      asm("v_max3_f32 %0, %0, |%1|, |%2|" : "+v"(st.amax[n]) : "v"(v[j]), "v"(v[j + 1]));
    st.X[n][7] = v;
    const int e = act_exponent(sample_max(st.amax[n]));
    st.s[n] = ldexpf(1.0f, e);
    st.amax[n] = 0.0f;
    split_op(st.X[n][0], st.s[n]);
  }
}

template <int Q, int NS>
__device__ __forceinline__ void slice(St<NS>& st, float* ring, const float4* w, int& g, int wave,
                                      int lane, Frags& x, Frags& y) {
  float* buf = ring + (g & 3) * kSliceFloats;
  float* nbuf = ring + ((g + 1) & 3) * kSliceFloats;
  const int t = g + 3;
  const Dma d = make_dma_blocks(w, t % kSl, ring + (t & 3) * kSliceFloats, (wave & 3) * 8, wave,
                                lane, LOADHI ? wave >= 4 : wave < 4, kSl);
  grp<0, NS, Q>(st, lds_base(buf, lane), lds_base(nbuf, lane), x, y, d);
  if constexpr (Q == 7) epi_last(st);
  slice_end<1, 8>();
  ++g;
}

template <int WPS, int NS>
__global__ __launch_bounds__(256 * WPS, 1) void ns_kernel(const float4* __restrict__ w, int tiles,
                                                          float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) float ring[4 * kSliceFloats];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int t = 0; t < 3; ++t) {
    const Dma d = make_dma_blocks(w, t, ring + t * kSliceFloats, (wave & 3) * 8, wave, lane,
                                  LOADHI ? wave >= 4 : wave < 4, kSl);
    if (d.live) {
      stage_piece<0>(d); stage_piece<1>(d); stage_piece<2>(d); stage_piece<3>(d);
      stage_piece<4>(d); stage_piece<5>(d); stage_piece<6>(d); stage_piece<7>(d);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
#if PRIO
  if (LOADHI ? wave < 4 : wave >= 4) __builtin_amdgcn_s_setprio(1);
#endif
  St<NS> st;
  float osum = 0.0f;
  int g = 0;
  for (int tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
    unsigned hsh = (unsigned)(tile * 7919 + threadIdx.x * 104729);
#pragma unroll
    for (int n = 0; n < NS; ++n) {
#pragma unroll
      for (int q = 0; q < 8; ++q)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          hsh = hsh * 1664525u + 1013904223u;
          st.X[n][q][j] = (float)(hsh >> 8) * 5.9604645e-08f;
        }
      st.s[n] = 8192.0f;
      st.amax[n] = 0.0f;
      split_op(st.X[n][0], st.s[n]);
    }
    Frags x, y;
    load_frags<0>(x, lds_base(ring + (g & 3) * kSliceFloats, lane));
#pragma unroll 1
    for (int L = 0; L < 8; ++L) {
      slice<0>(st, ring, w, g, wave, lane, x, y);
      slice<1>(st, ring, w, g, wave, lane, x, y);
      slice<2>(st, ring, w, g, wave, lane, x, y);
      slice<3>(st, ring, w, g, wave, lane, x, y);
      slice<4>(st, ring, w, g, wave, lane, x, y);
      slice<5>(st, ring, w, g, wave, lane, x, y);
      slice<6>(st, ring, w, g, wave, lane, x, y);
      slice<7>(st, ring, w, g, wave, lane, x, y);
    }
    lds_drain();
#pragma unroll
    for (int n = 0; n < NS; ++n) osum += st.X[n][3][1] + st.acc[n][0][0];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  out[blockIdx.x * 256 * WPS + threadIdx.x] = osum;
}

template <int WPS, int NS>
double run(const float4* dw, float* dout, int grid, int samples, hipEvent_t e0, hipEvent_t e1) {
  const int per = 64 * WPS * NS;   // samples per workgroup tile
  const int tiles = samples / per;
  hipLaunchKernelGGL((ns_kernel<WPS, NS>), dim3(grid), dim3(256 * WPS), 0, 0, dw, tiles, dout);
  hipEventRecord(e0);
  hipLaunchKernelGGL((ns_kernel<WPS, NS>), dim3(grid), dim3(256 * WPS), 0, 0, dw, tiles, dout);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double flop = (double)tiles * per * kSl * 256.0 * 32 * 2 * 3;
  printf("LOADHI=%d PRIO=%d SPLITW=%d WPS=%d NS=%d SPREAD=%d samples=%d: %.3f ms  %.1f TF/s  frac %.4f\n", LOADHI, PRIO, SPLITW, WPS, NS, SPREAD,
         tiles * per, ms, flop / ms / 1e9, flop / ms / 1e9 / 2516.8);
  return ms;
}

int main(int argc, char** argv) {
  const int samples = argc > 1 ? atoi(argv[1]) : 256 * 192 * 120;
  std::vector<unsigned short> hw(kSl * kSliceFloats * 2);
  srand(1);
  for (auto& v : hw) v = (unsigned short)(0x2000 + (rand() & 0x0fff) + ((rand() & 1) << 15));
  float4* dw;
  float* dout;
  hipMalloc(&dw, kSl * kSliceFloats * 4);
  hipMalloc(&dout, 256 * 512 * 4);
  hipMemcpy(dw, hw.data(), kSl * kSliceFloats * 4, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  int dev;
  hipGetDevice(&dev);
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, dev);
  const int grid = prop.multiProcessorCount;
  for (int rep = 0; rep < 3; ++rep) {
    run<2, 1>(dw, dout, grid, samples, e0, e1);
#if !SPLITW && !LOADHI && !PRIO
    run<1, 2>(dw, dout, grid, samples, e0, e1);
    run<1, 3>(dw, dout, grid, samples, e0, e1);
#endif
  }
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) { printf("error %s\n", hipGetErrorString(err)); return 1; }
  return 0;
}
