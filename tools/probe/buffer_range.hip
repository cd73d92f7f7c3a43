// Which offsets the buffer range check of a raw (stride 0) buffer store sees on
// gfx950: voffset alone, or voffset + soffset (+ the instruction offset).
// Every address this probe can reach lies inside its own 64-KiB allocation, so a
// store that the range check does not drop lands in memory we own and is seen.
// Used by DESIGN.md §3 (the training kernels drop the stores of samples past P
// with voffset 0x7fffffff, and put the row offset in soffset).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  std::printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int kBytes = 65536;
constexpr int kRecords = 4096;

__global__ void store_probe(unsigned* buf, int case_id) {
  if (threadIdx.x != 0) return;
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)buf, 0, kRecords, 0x00020000);
  const unsigned v = 0xA5A50000u | (unsigned)case_id;
  switch (case_id) {
    case 0: __builtin_amdgcn_raw_buffer_store_b32(v, rs, 0, 8192, 0); break;          // soffset past
    case 1: __builtin_amdgcn_raw_buffer_store_b32(v, rs, 8192, 0, 0); break;          // voffset past
    case 2: __builtin_amdgcn_raw_buffer_store_b32(v, rs, 4000, 200, 0); break;        // sum past, v in
    case 3: __builtin_amdgcn_raw_buffer_store_b32(v, rs, 0x7fffffff, 8, 0); break;    // the drop idiom
    case 4: __builtin_amdgcn_raw_buffer_store_b32(v, rs, 4092, 0, 0); break;          // last record
    case 5: __builtin_amdgcn_raw_buffer_store_b32(v, rs, 4094, 0, 0); break;          // straddles the end
    default: break;
  }
}

int main() {
  unsigned* d = nullptr;
  CHECK(hipMalloc(&d, kBytes));
  unsigned h[kBytes / 4];
  const char* what[] = {"voffset 0, soffset 8192", "voffset 8192, soffset 0",
                        "voffset 4000, soffset 200", "voffset 0x7fffffff, soffset 8",
                        "voffset 4092 (last dword)", "voffset 4094 (straddles num_records)"};
  std::printf("num_records %d\n", kRecords);
  for (int c = 0; c < 6; ++c) {
    CHECK(hipMemset(d, 0, kBytes));
    hipLaunchKernelGGL(store_probe, dim3(1), dim3(64), 0, 0, d, c);
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemcpy(h, d, kBytes, hipMemcpyDeviceToHost));
    int hits = 0;
    for (int i = 0; i < kBytes / 4; ++i)
      if (h[i]) { ++hits; std::printf("case %d (%s): written at byte %d\n", c, what[c], 4 * i); }
    if (!hits) std::printf("case %d (%s): dropped\n", c, what[c]);
  }
  CHECK(hipFree(d));
  return 0;
}
