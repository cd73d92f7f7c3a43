// Write-pattern microbenchmark for the training kernels' activation stores
// (mlp_x3.hip ActStore): 256 FP32 rows x P samples written by 8-wave
// workgroups that own 128-sample tiles, 16 samples per wave.
//   mode 0: feature-major [F][P + 32] rows, one buffer_store_b32 per (pair, r):
//           lane l -> sample l & 15, rows 4 (l >> 4) + r (the shipped pattern:
//           each instruction writes four 64-B half lines; the other half of
//           every 128-B line comes from the neighbouring wave)
//   mode 1: the same rows, 32 samples per wave-instruction pair (lanes 0-31 one
//           row, 32-63 the next): every instruction writes two full 128-B lines
//   mode 2: 16-sample tile layout [P / 16][F][16]: mode 0's lanes, rows of a
//           tile contiguous (rows 2k, 2k+1 = one 128-B line, both from one wave)
// aux: buffer cache policy bits (0 default, 2 nt).
// hipcc --offload-arch=gfx950 -O3 store_pattern.hip -o store_pattern
// ./store_pattern <mode> <aux> [iters]; rocprofv3 --pmc TCC_EA0_WRREQ_sum
// TCC_EA0_WRREQ_64B_sum -- ./store_pattern ...
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

constexpr int F = 256;
constexpr int P = 196608;
constexpr int LD = P + 32;

template <int MODE, int AUX>
__global__ __launch_bounds__(512) void store_kernel(float* out, int ntiles) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(out, 0, (int)((long)F * LD * 4), 0x00020000);
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const float v = (float)(t + lane);
#pragma unroll
    for (int G = 0; G < 8; ++G) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int row_base = 32 * G + 16 * h + r;
          unsigned vo;
          if (MODE == 0) {
            const int s = t * 128 + 16 * wave + (lane & 15);
            vo = (unsigned)(((row_base + 4 * (lane >> 4)) * (long)LD + s) * 4);
          } else if (MODE == 1) {
            // same bytes per instruction: 64 lanes = 32 samples x 2 rows
            const int s = t * 128 + 32 * (wave & 3) + (lane & 31);
            const int row = row_base + 4 * (2 * (wave >> 2) + (lane >> 5));
            vo = (unsigned)((row * (long)LD + s) * 4);
          } else {
            const int s = t * 128 + 16 * wave + (lane & 15);
            const int row = row_base + 4 * (lane >> 4);
            vo = (unsigned)((((long)(s >> 4) * F + row) * 16 + (s & 15)) * 4);
          }
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rs, (int)vo, 0, AUX);
        }
      }
    }
  }
}

int main(int argc, char** argv) {
  const int mode = argc > 1 ? atoi(argv[1]) : 0;
  const int aux = argc > 2 ? atoi(argv[2]) : 0;
  const int iters = argc > 3 ? atoi(argv[3]) : 20;
  float* d;
  hipMalloc(&d, (size_t)F * LD * 4);
  const int ntiles = P / 128;
  auto launch = [&]() {
#define L(M, A) hipLaunchKernelGGL((store_kernel<M, A>), dim3(256), dim3(512), 0, 0, d, ntiles)
    if (mode == 0) { if (aux) L(0, 2); else L(0, 0); }
    else if (mode == 1) { if (aux) L(1, 2); else L(1, 0); }
    else { if (aux) L(2, 2); else L(2, 0); }
#undef L
  };
  for (int i = 0; i < 3; ++i) launch();
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a);
  for (int i = 0; i < iters; ++i) launch();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  const double bytes = (double)F * P * 4;
  printf("mode %d aux %d: %.1f us per launch, %.2f TB/s\n", mode, aux, 1e3 * ms / iters,
         bytes / (1e-3 * ms / iters) / 1e12);
  hipFree(d);
  return 0;
}
