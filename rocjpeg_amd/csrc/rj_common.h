// rj_common.h -- status codes, logging and HIP error plumbing (the role of the reference's
// src/rocjpeg_commons.h:33-111: ERR always to stderr, INFO only with ROCJPEG_AMD_DEBUG=1).
#pragma once
#include <cstdio>
#include <cstdlib>

namespace rj {

enum Status : int {
  kOk = 0,
  kNotInitialized = -1,
  kInvalidParameter = -2,
  kBadJpeg = -3,
  kNotSupported = -4,
  kOutOfMemory = -5,
  kExecutionFailed = -6,
  kRuntimeError = -11,
};

inline bool DebugEnabled() {
  static const bool on = [] {
    const char *v = std::getenv("ROCJPEG_AMD_DEBUG");
    return v != nullptr && v[0] == '1';
  }();
  return on;
}

}  // namespace rj

#define RJ_ERR(...)                                           \
  do {                                                        \
    std::fprintf(stderr, "[rocjpeg_amd][ERR] " __VA_ARGS__);  \
    std::fputc('\n', stderr);                                 \
  } while (0)

#define RJ_INFO(...)                                            \
  do {                                                          \
    if (::rj::DebugEnabled()) {                                 \
      std::fprintf(stderr, "[rocjpeg_amd][INF] " __VA_ARGS__);  \
      std::fputc('\n', stderr);                                 \
    }                                                           \
  } while (0)

// HIP failure -> ROCJPEG_STATUS_EXECUTION_FAILED (rocjpeg_commons.h:51-57)
#define RJ_HIP(call)                                                                   \
  do {                                                                                 \
    hipError_t e_ = (call);                                                            \
    if (e_ != hipSuccess) {                                                            \
      RJ_ERR("HIP failure %s at %s:%d: %s", hipGetErrorName(e_), __FILE__, __LINE__, #call); \
      return ::rj::kExecutionFailed;                                                   \
    }                                                                                  \
  } while (0)

#define RJ_CHECK(call)            \
  do {                            \
    int s_ = (call);              \
    if (s_ != ::rj::kOk) return s_; \
  } while (0)
