// Error state of the C ABI (per calling thread) and launch checks.
#include "common.h"

namespace nerfhip {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

int check_launch(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    g_last_error = std::string(what) + ": " + hipGetErrorString(e);
    return (int)e;
  }
  return 0;
}

}  // namespace nerfhip

extern "C" {

const char* nerf_last_error(void) { return nerfhip::g_last_error.c_str(); }

int nerf_version(void) { return NERF_ABI_VERSION; }

#ifndef NERF_BUILD_ID
#define NERF_BUILD_ID "unknown"
#endif
const char* nerf_build_id(void) { return NERF_BUILD_ID; }

}  // extern "C"
