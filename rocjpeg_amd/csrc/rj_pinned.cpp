// rj_pinned.cpp -- the pinned host arena of parsed bitstreams (rj_pinned.h).
#include "rj_pinned.h"

#include <emmintrin.h>
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <mutex>
#include <utility>
#include <vector>

namespace rj {

struct PinnedChunk {
  uint8_t *base = nullptr;
  size_t size = 0;
};

namespace {

constexpr size_t kChunkBytes = 64ull << 20;
constexpr size_t kMaxFreeChunks = 8;  // released chunks kept for reuse (512 MB)

struct Arena {
  std::mutex mu;
  std::vector<uint8_t *> free_chunks;  // buffers of released kChunkBytes chunks
  int state = 0;                        // 0 unprobed, 1 usable, -1 disabled
  size_t pinned = 0;                    // bytes held from hipHostMalloc (live chunks + free_chunks)
  size_t cap = 0;                       // at most this many (ROCJPEG_AMD_PARSE_PIN_MAX_MB, default 4 GB)
};

Arena &TheArena() {
  static Arena *a = new Arena;  // never destroyed: slots may outlive static destructors
  return *a;
}

// The chunk a thread carves its slots from.  Per thread, so that the streams one thread parses
// one after another stay adjacent when several threads parse at once (jpegdecodeperf: a thread per
// handle, each parsing its own files): a decode call then uploads a thread's streams in a few
// large DMAs.  With one shared chunk, concurrent parses interleave their slots and a 512-image
// call became ~500 DMAs of one stream each (profiles/r6_experiments/host_input_threads.txt).
struct ThreadChunk {
  std::shared_ptr<PinnedChunk> cur;
  size_t used = 0;
};
ThreadChunk &MyChunk() {
  static thread_local ThreadChunk t;
  return t;
}

void ReturnBuffer(uint8_t *p, size_t size) {
  Arena &a = TheArena();
  {
    std::lock_guard<std::mutex> l(a.mu);
    if (size == kChunkBytes && a.free_chunks.size() < kMaxFreeChunks) {
      a.free_chunks.push_back(p);
      return;
    }
    a.pinned -= size;
  }
  (void)hipHostFree(p);
}

// caller holds a.mu
std::shared_ptr<PinnedChunk> NewChunk(Arena &a, size_t size) {
  uint8_t *p = nullptr;
  if (size == kChunkBytes && !a.free_chunks.empty()) {
    p = a.free_chunks.back();
    a.free_chunks.pop_back();
  } else if (a.pinned + size > a.cap) {
    return nullptr;  // over the cap: the stream borrows the caller's bytes (staged by the decode call)
  } else if (hipHostMalloc(reinterpret_cast<void **>(&p), size, hipHostMallocNonCoherent) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  } else {
    a.pinned += size;
  }
  return std::shared_ptr<PinnedChunk>(new PinnedChunk{p, size}, [](PinnedChunk *c) {
    ReturnBuffer(c->base, c->size);
    delete c;
  });
}

}  // namespace

PinnedSlot PinnedAlloc(size_t bytes) {
  PinnedSlot s;
  Arena &a = TheArena();
  const size_t need = (bytes + 255) & ~size_t(255);
  std::shared_ptr<PinnedChunk> retired;  // released after the lock (its deleter takes the lock)
  std::lock_guard<std::mutex> l(a.mu);
  if (a.state == 0) {
    const char *v = std::getenv("ROCJPEG_AMD_PARSE_PIN");
    int ndev = 0;
    const bool off = v != nullptr && v[0] == '0';
    a.state = (!off && hipGetDeviceCount(&ndev) == hipSuccess && ndev > 0) ? 1 : -1;
    (void)hipGetLastError();
    const char *m = std::getenv("ROCJPEG_AMD_PARSE_PIN_MAX_MB");
    a.cap = (m != nullptr ? size_t(std::strtoull(m, nullptr, 10)) : size_t(4096)) << 20;
  }
  if (a.state < 0 || bytes == 0) return s;
  std::shared_ptr<PinnedChunk> c;
  uint8_t *p = nullptr;
  if (need > kChunkBytes / 4) {  // a large stream gets a chunk of its own
    c = NewChunk(a, need);
    if (c) p = c->base;
  } else {
    ThreadChunk &t = MyChunk();
    if (!t.cur || t.used + need > t.cur->size) {
      retired = std::move(t.cur);
      t.cur = NewChunk(a, kChunkBytes);
      t.used = 0;
    }
    if (t.cur) {
      c = t.cur;
      p = c->base + t.used;
      t.used += need;
    }
  }
  if (p != nullptr) {
    s.ptr = p;
    s.bytes = bytes;
    s.chunk = std::move(c);
  }
  return s;
}

void CopyToStaging(void *dst, const void *src, size_t n) {
  uint8_t *d = static_cast<uint8_t *>(dst);
  const uint8_t *s = static_cast<const uint8_t *>(src);
  if (n < 4096) {
    std::memcpy(d, s, n);
    return;
  }
  const size_t head = (16 - (reinterpret_cast<uintptr_t>(d) & 15)) & 15;
  std::memcpy(d, s, head);
  d += head;
  s += head;
  n -= head;
  size_t i = 0;
  for (; i + 64 <= n; i += 64) {
    const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i *>(s + i));
    const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i *>(s + i + 16));
    const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i *>(s + i + 32));
    const __m128i e = _mm_loadu_si128(reinterpret_cast<const __m128i *>(s + i + 48));
    _mm_stream_si128(reinterpret_cast<__m128i *>(d + i), a);
    _mm_stream_si128(reinterpret_cast<__m128i *>(d + i + 16), b);
    _mm_stream_si128(reinterpret_cast<__m128i *>(d + i + 32), c);
    _mm_stream_si128(reinterpret_cast<__m128i *>(d + i + 48), e);
  }
  std::memcpy(d + i, s + i, n - i);
  _mm_sfence();
}

}  // namespace rj
