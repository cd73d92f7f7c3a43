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
struct BFr { half8 h, l; };              // one n-tile's B fragment (hi, lo)

#ifndef NT
#define NT 8      // n-tiles (16 samples each) per workgroup
#endif
#ifndef WPS
#define WPS 2     // workgroups per CU (launch bound)
#endif
#ifndef AHEAD
#define AHEAD 2   // B-fragment groups (n-tiles) read ahead of the one multiplied
#endif

__device__ __forceinline__ WSet wload(__amdgpu_buffer_rsrc_t r, unsigned vo, int slice) {
  WSet s;
  int sl = slice;
  const int so = __builtin_amdgcn_readfirstlane(sl * 32768);
  s.h0 = __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(r, vo, so, 0));
  s.l0 = __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(r, vo + 1024, so, 0));
  s.h1 = __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(r, vo + 2048, so, 0));
  s.l1 = __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(r, vo + 3072, so, 0));
  return s;
}

// group k of a layer: K step q = k >> 3, n-tile n = k & 7; LDS offset of its
// fragment pair: q * 16 KiB + n * 2 KiB (+ 1 KiB for lo)
template <int K>
__device__ __forceinline__ void bread(BFr& b, unsigned abase) {
  b.h = rd<(K % NT) * 2048>(abase + (K / NT) * (NT * 2048));
  b.l = rd<(K % NT) * 2048 + 1024>(abase + (K / NT) * (NT * 2048));
}

template <int N>
__device__ __forceinline__ void lgkm() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(N) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}

constexpr int NS = DEPTH + 1;   // weight slots
template <int K, int G0>
__device__ __forceinline__ void groups(f32x4 (&acc)[2][NT], WSet (&W)[NS], BFr (&B)[4],
                                       unsigned abase, __amdgpu_buffer_rsrc_t rw, unsigned vo,
                                       int g0, bool more) {
  if constexpr (K < 8 * NT) {
    constexpr int q = K / NT, n = K % NT;
    if constexpr (n == 0) {
#ifndef NOW2
      if (more || q + DEPTH < 8) W[(G0 + q + DEPTH) % NS] = wload(rw, vo, g0 + q + DEPTH);
#endif
    }
    // group K's reads done: the younger in flight are groups K+1 .. K+AHEAD-1
    constexpr int younger = (K + AHEAD - 1 < 8 * NT ? AHEAD - 1 : 8 * NT - 1 - K);
    lgkm<2 * younger>();
    if constexpr (K + AHEAD < 8 * NT) bread<K + AHEAD>(B[(K + AHEAD) & 3], abase);
    __builtin_amdgcn_sched_barrier(0);
    const WSet& w = W[(G0 + q) % NS];
    const BFr& b = B[K & 3];
    constexpr bool F = q == 0;
    acc[0][n] = MFMA(w.h0, b.h, F ? f32x4(0.0f) : acc[0][n]);
    acc[1][n] = MFMA(w.h1, b.h, F ? f32x4(0.0f) : acc[1][n]);
    acc[0][n] = MFMA(w.h0, b.l, acc[0][n]);
    acc[1][n] = MFMA(w.h1, b.l, acc[1][n]);
    acc[0][n] = MFMA(w.l0, b.h, acc[0][n]);
    acc[1][n] = MFMA(w.l1, b.h, acc[1][n]);
    __builtin_amdgcn_sched_barrier(0);
    groups<K + 1, G0>(acc, W, B, abase, rw, vo, g0, more);
  }
}

__device__ __forceinline__ float smax(float v) {
  v = fmaxf(v, __shfl_xor(v, 16));
  return fmaxf(v, __shfl_xor(v, 32));
}

__global__ __launch_bounds__(512, 2 * WPS) void ub_kernel(const u32x4* __restrict__ wts, int tiles,
                                                    float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) u32x4 act[8 * NT * 2 * 64];
  __shared__ float xch[8 * 16 * NT];
  __shared__ float scl[16 * NT];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g4 = lane >> 4;
  for (int i = threadIdx.x; i < 8 * NT * 2 * 64; i += 512) {
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
  f32x4 acc[2][NT];
  float osum = 0.0f;
  for (int tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
    WSet W[NS];
#pragma unroll
#ifdef NOW2
    for (int d = 0; d < NS; ++d) W[d] = wload(rw, vo, d);
#else
    for (int d = 0; d < DEPTH; ++d) W[d] = wload(rw, vo, d);
#endif
#pragma unroll
    for (int L = 0; L < 8; ++L) {
      BFr B[4];
#pragma unroll
      for (int k = 0; k < AHEAD; ++k) {
        B[k].h = rd<0>(abase + (k / NT) * (NT * 2048) + (k % NT) * 2048);
        B[k].l = rd<1024>(abase + (k / NT) * (NT * 2048) + (k % NT) * 2048);
      }
      switch (L) {
        case 0: groups<0, 0>(acc, W, B, abase, rw, vo, 0, true); break;
        case 1: groups<0, 8 % NS>(acc, W, B, abase, rw, vo, 8, true); break;
        case 2: groups<0, 16 % NS>(acc, W, B, abase, rw, vo, 16, true); break;
        case 3: groups<0, 24 % NS>(acc, W, B, abase, rw, vo, 24, true); break;
        case 4: groups<0, 32 % NS>(acc, W, B, abase, rw, vo, 32, true); break;
        case 5: groups<0, 40 % NS>(acc, W, B, abase, rw, vo, 40, true); break;
        case 6: groups<0, 48 % NS>(acc, W, B, abase, rw, vo, 48, true); break;
        default: groups<0, 56 % NS>(acc, W, B, abase, rw, vo, 56, false); break;
      }
#if !NOEPI
      // epilogue: v = max(acc * inv + bias, 0); per-sample max over the wave's 32 rows
      const float inv = 0.0009765625f;
      float mx[NT];
      f32x4 v[2][NT];
#pragma unroll
      for (int n = 0; n < NT; ++n) {
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
        for (int n = 0; n < NT; ++n) xch[wave * 16 * NT + 16 * n + lane] = mx[n];
      }
      __syncthreads();
      if (lane < 16 && wave < NT) {
        float m = 0.0f;
#pragma unroll
        for (int k = 0; k < 8; ++k) m = fmaxf(m, xch[k * 16 * NT + 16 * wave + lane]);
        int e;
        (void)frexpf(m, &e);
        scl[16 * wave + lane] = ldexpf(1.0f, 14 - e);
      }
      __syncthreads();
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        const float s = scl[16 * n + (lane & 15)];
        half8 h, l;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float a = v[j >> 2][n][j & 3] * s;
          h[j] = (_Float16)a;
          l[j] = (_Float16)(a - (float)h[j]);
        }
        act[((wave * NT + n) * 2 + 0) * 64 + lane] = __builtin_bit_cast(u32x4, h);
        act[((wave * NT + n) * 2 + 1) * 64 + lane] = __builtin_bit_cast(u32x4, l);
      }
      __syncthreads();
#endif
    }
#pragma unroll
    for (int n = 0; n < NT; ++n) osum += acc[0][n][0] + acc[1][n][3];
  }
  out[blockIdx.x * 512 + threadIdx.x] = osum;
}

#ifdef NOW2
#define NOW2X 1
#else
#define NOW2X 0
#endif
int main(int argc, char** argv) {
  const int tiles = argc > 1 ? atoi(argv[1]) : 256 * 200 * 8 / NT;
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
  const int grid = prop.multiProcessorCount * WPS;
  for (int rep = 0; rep < 4; ++rep) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(ub_kernel, dim3(grid), dim3(512), 0, 0, dw, tiles, dout);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double flop = (double)tiles * 64 * 8 * (6 * NT) * 16384.0;
    printf("NT=%d WPS=%d AHEAD=%d DEPTH=%d NOEPI=%d NOW2=%d tiles=%d: %.3f ms  %.1f TF/s  frac %.3f  (%.2f us/tile/CU)\n",
           NT, WPS, AHEAD, DEPTH, NOEPI, NOW2X, tiles, ms, flop / ms / 1e9, flop / ms / 1e9 / 2516.8,
           ms * 1e3 / ((double)tiles / grid));
  }
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) { printf("error %s\n", hipGetErrorString(err)); return 1; }
  return 0;
}
