// Shared helpers for the gfx950 NeRF kernels: error state, launch checks and
// the torch-CPU float32 summation orders the compositing kernels reproduce.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <string>

#include "../../include/nerfhip.h"

namespace nerfhip {

void set_error(const std::string& msg);
int fail(int code, const std::string& msg);

inline hipStream_t as_stream(nerf_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

// Check the last launch; returns 0 or the hip error (message recorded).
int check_launch(const char* what);

#define NERF_REQUIRE(cond, msg)                                  \
  do {                                                           \
    if (!(cond)) return ::nerfhip::fail(NERF_E_ARG, (msg));      \
  } while (0)

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// CU count of the device a stream launches on (persistent grids: one workgroup
// per CU), cached per device ordinal; races only write the same value. The
// null/legacy stream resolves to the calling thread's current device.
inline int stream_cu_count(nerf_stream_t s) {
  static std::atomic<int> cache[64];
  hipDevice_t dev = 0;
  if (hipStreamGetDevice(as_stream(s), &dev) != hipSuccess) {
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess) return 256;
    dev = cur;
  }
  if (dev < 0 || dev >= 64) return 256;
  int n = cache[dev].load(std::memory_order_relaxed);
  if (n > 0) return n;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      n <= 0)
    return 256;
  cache[dev].store(n, std::memory_order_relaxed);
  return n;
}

// ---------------------------------------------------------------------------
// torch CPU float32 reductions (ATen SumKernel, x86 build): bit-exact orders.
// Documented and pinned in oracle/nerf_oracle.py (tsum_last / tsum_dim2).
// ---------------------------------------------------------------------------

// torch.sum(x, -1) over n contiguous values given by get(i), n < 512.
//   n >= 8: 8-lane vectors, 4 vector accumulators (vector v -> acc v%4 for the
//   first 4*floor(nv/4) vectors, then acc 0), combined ((a0+a1)+a2)+a3; then a
//   scalar tail sum; then the 8 lanes added to it in order.
//   n < 8: the same 4-accumulator scheme on scalars.
template <typename G>
__device__ __forceinline__ float tsum_last(int n, G get) {
  if (n < 8) {
    float p[4] = {0.f, 0.f, 0.f, 0.f};
    const int nilp = n >> 2;
    if (nilp) {
#pragma unroll
      for (int k = 0; k < 4; ++k) p[k] = p[k] + get(k);
    }
    for (int i = nilp * 4; i < n; ++i) p[0] = p[0] + get(i);
    return ((p[0] + p[1]) + p[2]) + p[3];
  }
  const int nv = n >> 3;
  const int nilp = nv >> 2;
  float a0[8], a1[8], a2[8], a3[8];
#pragma unroll
  for (int l = 0; l < 8; ++l) a0[l] = a1[l] = a2[l] = a3[l] = 0.f;
  for (int ii = 0; ii < nilp; ++ii) {
    const int b = ii * 32;
#pragma unroll
    for (int l = 0; l < 8; ++l) {
      a0[l] = a0[l] + get(b + l);
      a1[l] = a1[l] + get(b + 8 + l);
      a2[l] = a2[l] + get(b + 16 + l);
      a3[l] = a3[l] + get(b + 24 + l);
    }
  }
  for (int v = nilp * 4; v < nv; ++v) {
#pragma unroll
    for (int l = 0; l < 8; ++l) a0[l] = a0[l] + get(v * 8 + l);
  }
  float fin = 0.f;
  for (int k = nv * 8; k < n; ++k) fin = fin + get(k);
#pragma unroll
  for (int l = 0; l < 8; ++l) fin = fin + (((a0[l] + a1[l]) + a2[l]) + a3[l]);
  return fin;
}

// torch.sum(x, -2) of [.., n, C] for one channel (strided reduction), n < 1024:
// 4 scalar accumulators (i -> i%4) over 16-row (64-value) blocks; a block's sum
// is started fresh and then added into the level-1 running sum; values past the
// last whole block go into a fresh level-0 sum that is added BEFORE the level-1
// sum; scalar tail (n%4) into accumulator 0; then ((p0+p1)+p2)+p3.
template <typename G>
__device__ __forceinline__ float tsum_dim2(int n, G get) {
  const int nilp = n >> 2;
  float lv0[4] = {0.f, 0.f, 0.f, 0.f};
  float lv1[4] = {0.f, 0.f, 0.f, 0.f};
  int i = 0;
  for (; i + 16 <= nilp; i += 16) {
#pragma unroll
    for (int k = 0; k < 4; ++k) lv0[k] = 0.f;
    for (int j = 0; j < 16; ++j) {
#pragma unroll
      for (int k = 0; k < 4; ++k) lv0[k] = lv0[k] + get((i + j) * 4 + k);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) lv1[k] = lv1[k] + lv0[k];
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) lv0[k] = 0.f;
  for (; i < nilp; ++i) {
#pragma unroll
    for (int k = 0; k < 4; ++k) lv0[k] = lv0[k] + get(i * 4 + k);
  }
  float p[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) p[k] = lv0[k] + lv1[k];
  for (int t = nilp * 4; t < n; ++t) p[0] = p[0] + get(t);
  return ((p[0] + p[1]) + p[2]) + p[3];
}

// torch.norm(v, dim=-1) of a 3-vector on the CPU: sqrt(fma(z,z,fma(y,y,x*x))).
__device__ __forceinline__ float torch_norm3(float x, float y, float z) {
  return __builtin_sqrtf(__builtin_fmaf(z, z, __builtin_fmaf(y, y, x * x)));
}

// torch.max(a, b) propagates NaN (fmaxf would drop it).
__device__ __forceinline__ float torch_max(float a, float b) {
  return (a != a || b != b) ? __builtin_nanf("") : (a > b ? a : b);
}

}  // namespace nerfhip
