// Timing microbenchmark (no correctness): the core loop of an "activations in
// LDS, weights streamed L2 -> VGPR" layout for the x3 MLP. A workgroup holds
// 128 samples; wave w owns output rows 32w..32w+31 of every 256-row layer for
// all 128 samples (2 m-tiles x 8 n-tiles of 16x16x32 f16 MFMA, 3 products per
// FP32 product as in mlp_x3.hip). Per slice (one 32-deep K step): 4 x 1 KiB
// weight blocks per wave by buffer_load_dwordx4 (D slices ahead), 16
// ds_read_b128 of B fragments, 48 MFMAs. Per layer (8 slices): the epilogue
// (scale-undo + bias + ReLU, per-sample max exchanged through LDS, FP16
// split, 16 ds_write_b128 of the next layer's B fragments), 3 barriers.
//   hipcc -O3 --offload-arch=gfx950 -o act_lds act_lds.hip && ./act_lds
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

#ifndef DEPTH
#define DEPTH 3   // weight slices in flight ahead of the one being multiplied
#endif
#ifndef NOEPI
#define NOEPI 0
#endif
#ifndef NOW
#define NOW 0     // 1: no weight loads (registers reused)
#endif
#ifndef ROT
#define ROT 0     // >0: workgroup b reads slice (g + ROT*b) mod 64 (desynchronised streams)
#endif
#ifndef NOLDS
#define NOLDS 0   // 1: no B-fragment LDS reads
#endif

#define MFMA(a, b, c) __builtin_amdgcn_mfma_f32_16x16x32_f16((a), (b), (c), 0, 0, 0)

template <int OFF>
__device__ __forceinline__ half8 rd(unsigned addr) {
  u32x4 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF) : "memory");
  return __builtin_bit_cast(half8, v);
}
__device__ __forceinline__ void drain() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

struct WSet { half8 h0, l0, h1, l1; };   // m-tiles 2w, 2w+1 x (hi, lo)
struct BGrp { half8 h0, l0, h1, l1; };   // n-tiles 2i, 2i+1 x (hi, lo)

__device__ __forceinline__ WSet wload(__amdgpu_buffer_rsrc_t r, unsigned vo, int slice) {
  WSet s;
#if NOW
  s.h0 = s.l0 = s.h1 = s.l1 = half8((_Float16)0.01f);
  (void)r; (void)vo; (void)slice;
#else
  int sl = ROT ? ((slice + ROT * (int)blockIdx.x) & 63) : slice;
#ifdef SMALL
  sl &= SMALL - 1;   // only SMALL distinct slices (L2 footprint SMALL x 32 KiB)
#endif
  const int so = __builtin_amdgcn_readfirstlane(sl * 32768);
  s.h0 = __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(r, vo, so, 0));
  s.l0 = __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(r, vo + 1024, so, 0));
  s.h1 = __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(r, vo + 2048, so, 0));
  s.l1 = __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(r, vo + 3072, so, 0));
#endif
  return s;
}

template <int G>
__device__ __forceinline__ void bload(BGrp& b, unsigned base) {
#if NOLDS
  (void)base;
  b.h0 = b.l0 = b.h1 = b.l1 = half8((_Float16)0.01f);
#else
  b.h0 = rd<(4 * G + 0) * 1024>(base);
  b.l0 = rd<(4 * G + 1) * 1024>(base);
  b.h1 = rd<(4 * G + 2) * 1024>(base);
  b.l1 = rd<(4 * G + 3) * 1024>(base);
#endif
}

template <bool FIRST>
__device__ __forceinline__ void mf12(f32x4 (&acc)[2][8], const WSet& w, const BGrp& b, int n) {
  // n-tiles n, n+1; m-tiles 0, 1; hh, hl, lh
  acc[0][n] = MFMA(w.h0, b.h0, FIRST ? f32x4(0.0f) : acc[0][n]);
  acc[1][n] = MFMA(w.h1, b.h0, FIRST ? f32x4(0.0f) : acc[1][n]);
  acc[0][n + 1] = MFMA(w.h0, b.h1, FIRST ? f32x4(0.0f) : acc[0][n + 1]);
  acc[1][n + 1] = MFMA(w.h1, b.h1, FIRST ? f32x4(0.0f) : acc[1][n + 1]);
  acc[0][n] = MFMA(w.h0, b.l0, acc[0][n]);
  acc[1][n] = MFMA(w.h1, b.l0, acc[1][n]);
  acc[0][n + 1] = MFMA(w.h0, b.l1, acc[0][n + 1]);
  acc[1][n + 1] = MFMA(w.h1, b.l1, acc[1][n + 1]);
  acc[0][n] = MFMA(w.l0, b.h0, acc[0][n]);
  acc[1][n] = MFMA(w.l1, b.h0, acc[1][n]);
  acc[0][n + 1] = MFMA(w.l0, b.h1, acc[0][n + 1]);
  acc[1][n + 1] = MFMA(w.l1, b.h1, acc[1][n + 1]);
}

// one slice: B groups 0..3 (group 0 prefetched by the caller into x)
template <bool FIRST>
__device__ __forceinline__ void slice(f32x4 (&acc)[2][8], const WSet& w, unsigned base,
                                      unsigned nbase, BGrp& x, BGrp& y, bool next) {
  drain();
  bload<1>(y, base);
  __builtin_amdgcn_sched_barrier(0);
  mf12<FIRST>(acc, w, x, 0);
  __builtin_amdgcn_sched_barrier(0);
  drain();
  bload<2>(x, base);
  __builtin_amdgcn_sched_barrier(0);
  mf12<FIRST>(acc, w, y, 2);
  __builtin_amdgcn_sched_barrier(0);
  drain();
  bload<3>(y, base);
  __builtin_amdgcn_sched_barrier(0);
  mf12<FIRST>(acc, w, x, 4);
  __builtin_amdgcn_sched_barrier(0);
  drain();
  if (next) bload<0>(x, nbase);
  __builtin_amdgcn_sched_barrier(0);
  mf12<FIRST>(acc, w, y, 6);
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ float smax(float v) {
  v = fmaxf(v, __shfl_xor(v, 16));
  return fmaxf(v, __shfl_xor(v, 32));
}

__global__ __launch_bounds__(512, 2) void ub_kernel(const u32x4* __restrict__ wts, int tiles,
                                                    float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) u32x4 act[8 * 8 * 2 * 64];   // 128 KiB
  __shared__ float xch[8 * 128];
  __shared__ float scl[128];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g4 = lane >> 4;
  for (int i = threadIdx.x; i < 8 * 8 * 2 * 64; i += 512) {
    const unsigned h = 0x2c002c00u + (unsigned)(i & 255) * 0x00010001u;
    act[i] = u32x4{h, h ^ 0x10001u, h, h};
  }
  __syncthreads();
#ifdef SKEW
  for (int i = 0; i < (int)((blockIdx.x >> 3) & 7) * SKEW; ++i) __builtin_amdgcn_s_sleep(127);
#endif
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)wts, 0, 64 * 32768, 0x00020000);
  const unsigned vo = (unsigned)((4 * wave * 64 + lane) * 16);
  const unsigned abase = (unsigned)(uintptr_t)(__attribute__((address_space(3))) u32x4*)act + lane * 16;
  f32x4 acc[2][8];
  float osum = 0.0f;
  for (int tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
    WSet W[4];
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) W[d] = wload(rw, vo, d);
    BGrp x, y;
    bload<0>(x, abase);
#pragma unroll 1
    for (int L = 0; L < 8; ++L) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int g = 8 * L + q;
#ifndef NOW2   // NOW2: the first DEPTH slices' random weights reused (no loads in the loop)
        if (g + DEPTH < 64) W[(q + DEPTH) & 3] = wload(rw, vo, g + DEPTH);
#else
        if (g + DEPTH < 64 && L == 0 && q == 0) W[(q + DEPTH) & 3] = wload(rw, vo, g + DEPTH);
#endif
        const unsigned base = abase + q * 16384, nbase = abase + ((q + 1) & 7) * 16384;
        if (q == 0) slice<true>(acc, W[q & 3], base, nbase, x, y, true);
        else slice<false>(acc, W[q & 3], base, nbase, x, y, q < 7);
      }
#if !NOEPI
      // epilogue: v = max(acc * inv + bias, 0); per-sample max over the wave's 32 rows
      const float inv = 0.0009765625f;
      float mx[8];
      f32x4 v[2][8];
#pragma unroll
      for (int n = 0; n < 8; ++n) {
        mx[n] = 0.0f;
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            v[m][n][r] = fmaxf(__builtin_fmaf(acc[m][n][r], inv, 0.001f * (r + 4 * m)), 0.0f);
            mx[n] = fmaxf(mx[n], v[m][n][r]);
          }
        mx[n] = smax(mx[n]);
      }
      if (g4 == 0) {
#pragma unroll
        for (int n = 0; n < 8; ++n) xch[wave * 128 + 16 * n + lane] = mx[n];
      }
      __syncthreads();
      if (lane < 16) {
        float m = 0.0f;
#pragma unroll
        for (int k = 0; k < 8; ++k) m = fmaxf(m, xch[k * 128 + 16 * wave + lane]);
        int e;
        (void)frexpf(m, &e);
        scl[16 * wave + lane] = ldexpf(1.0f, 14 - e);
      }
      __syncthreads();
#pragma unroll
      for (int n = 0; n < 8; ++n) {
        const float s = scl[16 * n + (lane & 15)];
        half8 h, l;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float a = v[j >> 2][n][j & 3] * s;
          h[j] = (_Float16)a;
          l[j] = (_Float16)(a - (float)h[j]);
        }
        act[((wave * 8 + n) * 2 + 0) * 64 + lane] = __builtin_bit_cast(u32x4, h);
        act[((wave * 8 + n) * 2 + 1) * 64 + lane] = __builtin_bit_cast(u32x4, l);
      }
      __syncthreads();
      bload<0>(x, abase);
#else
      bload<0>(x, abase);
#endif
    }
#pragma unroll
    for (int n = 0; n < 8; ++n) osum += acc[0][n][0] + acc[1][n][3];
  }
  out[blockIdx.x * 512 + threadIdx.x] = osum;
}

int main(int argc, char** argv) {
  const int tiles = argc > 1 ? atoi(argv[1]) : 256 * 200;
  std::vector<unsigned short> hw(64 * 32768 / 2);
  srand(1);
  for (auto& v : hw) v = (unsigned short)(0x2000 + (rand() & 0x0fff) + ((rand() & 1) << 15));
  u32x4* dw;
  float* dout;
  hipMalloc(&dw, 64 * 32768);
  hipMalloc(&dout, 256 * 512 * 4);
  hipMemcpy(dw, hw.data(), 64 * 32768, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  int dev;
  hipGetDevice(&dev);
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, dev);
  const int grid = prop.multiProcessorCount;
  for (int rep = 0; rep < 4; ++rep) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(ub_kernel, dim3(grid), dim3(512), 0, 0, dw, tiles, dout);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double flop = (double)tiles * 64 * 8 * 48 * 16384.0;
    printf("ROT=%d DEPTH=%d NOEPI=%d NOW=%d NOLDS=%d tiles=%d: %.3f ms  %.1f TF/s  frac %.3f  (%.2f us/tile/CU)\n",
           ROT, DEPTH, NOEPI, NOW, NOLDS, tiles, ms, flop / ms / 1e9, flop / ms / 1e9 / 2516.8,
           ms * 1e3 / ((double)tiles / grid));
  }
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) { printf("error %s\n", hipGetErrorString(err)); return 1; }
  return 0;
}
