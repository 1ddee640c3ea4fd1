// Test stub of rj::Decoder for the coalescing logic (tests/test_coalesce_cpu.py builds
// rocjpeg_amd/csrc/rj_coalesce.cpp against it, on the CPU, under AddressSanitizer).  Decode checks
// the invariants the library relies on: a handle is never used by two threads at once, and a
// call's streams and destinations are the caller's own; a stream marked bad fails its batch.
#pragma once
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>

#include "rocjpeg.h"

namespace rj {
class Stream {
 public:
  bool bad = false;
  int owner = -1;  // the thread whose call holds this stream
};
class Decoder {
 public:
  std::atomic<int> active{0};
  std::atomic<long> images{0}, attempts{0};  // images decoded successfully / handed to Decode
  bool Coalescable() const { return true; }
  // host validation without decoding (rj_decoder.h Decoder::Check): a bad stream fails its call
  int Check(Stream *const *s, int n, const RocJpegDecodeParams *p, const RocJpegImage *d) {
    if (s == nullptr || p == nullptr || d == nullptr) std::abort();
    for (int i = 0; i < n; i++)
      if (s[i]->bad) return ROCJPEG_STATUS_BAD_JPEG;
    return 0;
  }
  int Decode(Stream *const *s, int n, const RocJpegDecodeParams *p, RocJpegImage *d) {
    if (active.fetch_add(1) != 0) {
      std::fprintf(stderr, "handle used by two threads at once\n");
      std::abort();
    }
    int st = 0;
    for (int i = 0; i < n; i++) {
      if (s[i] == nullptr || d == nullptr || p == nullptr) std::abort();
      // the destination's first pitch carries the owner thread of its stream: a stream and its
      // destination travel together through a combined call
      if (int(d[i].pitch[0]) != s[i]->owner) {
        std::fprintf(stderr, "stream / destination mismatch\n");
        std::abort();
      }
      if (s[i]->bad) st = ROCJPEG_STATUS_BAD_JPEG;
    }
    std::this_thread::sleep_for(std::chrono::microseconds(200 + 20 * n));
    attempts += n;
    if (st == 0) images += n;
    active.fetch_sub(1);
    return st;
  }
};
}  // namespace rj
