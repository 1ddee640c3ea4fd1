// rj_coalesce.cpp -- see rj_coalesce.h.
#include "rj_coalesce.h"

#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <vector>

#include "rj_decoder.h"

namespace rj {
namespace {

constexpr int kSmallCall = 16;   // calls of at most this many images take part
constexpr int kMaxImages = 64;   // images per combined call
std::atomic<uint64_t> g_calls{0}, g_combined{0}, g_members{0};

struct Request {
  Decoder *dec;
  Stream *const *streams;
  int n;
  const RocJpegDecodeParams *params;
  RocJpegImage *dst;
  int status = 0;
  bool done = false;
};

bool SameParams(const RocJpegDecodeParams &a, const RocJpegDecodeParams &b) {
  return a.output_format == b.output_format && a.crop_rectangle.left == b.crop_rectangle.left &&
         a.crop_rectangle.top == b.crop_rectangle.top && a.crop_rectangle.right == b.crop_rectangle.right &&
         a.crop_rectangle.bottom == b.crop_rectangle.bottom;
}

// One device's queue of waiting calls and whether a leader is decoding.
struct DeviceQueue {
  std::mutex mu;
  std::condition_variable cv;
  std::deque<Request *> pending;
  bool busy = false;
};

DeviceQueue &QueueFor(int device) {
  static std::mutex mu;
  static std::vector<std::unique_ptr<DeviceQueue>> qs;
  std::lock_guard<std::mutex> lk(mu);
  if (device >= int(qs.size())) qs.resize(size_t(device) + 1);
  if (!qs[size_t(device)]) qs[size_t(device)].reset(new DeviceQueue);
  return *qs[size_t(device)];
}

bool Enabled() {
  static const bool on = [] {
    const char *e = std::getenv("RJ_COALESCE");
    return !(e && e[0] == '0');
  }();
  return on;
}

// The group's calls as one call on `dec`; on failure each call alone (its own status).
void RunGroup(Decoder *dec, std::vector<Request *> &group) {
  if (group.size() == 1) {
    Request *r = group[0];
    r->status = dec->Decode(r->streams, r->n, r->params, r->dst);
    return;
  }
  g_combined.fetch_add(1, std::memory_order_relaxed);
  g_members.fetch_add(group.size(), std::memory_order_relaxed);
  std::vector<Stream *> streams;
  std::vector<RocJpegImage> dst;
  for (Request *r : group) {
    streams.insert(streams.end(), r->streams, r->streams + r->n);
    dst.insert(dst.end(), r->dst, r->dst + r->n);
  }
  const int st = dec->Decode(streams.data(), int(streams.size()), group[0]->params, dst.data());
  if (st == 0) {
    for (Request *r : group) r->status = 0;
    return;
  }
  for (Request *r : group) r->status = dec->Decode(r->streams, r->n, r->params, r->dst);
}

}  // namespace

int CoalescedDecode(Decoder *dec, int device, Stream *const *streams, int n, const RocJpegDecodeParams *params,
                    RocJpegImage *dst) {
  if (!Enabled() || n > kSmallCall || n <= 0 || device < 0 || streams == nullptr || params == nullptr ||
      dst == nullptr)
    return dec->Decode(streams, n, params, dst);
  g_calls.fetch_add(1, std::memory_order_relaxed);
  DeviceQueue &q = QueueFor(device);
  Request me{dec, streams, n, params, dst};
  std::unique_lock<std::mutex> lk(q.mu);
  q.pending.push_back(&me);
  while (!me.done) {
    if (q.busy) {
      q.cv.wait(lk);
      continue;
    }
    // leader: the oldest waiting call and every other with the same parameters, up to kMaxImages
    q.busy = true;
    std::vector<Request *> group;
    int images = 0;
    const RocJpegDecodeParams p0 = *q.pending.front()->params;
    for (auto it = q.pending.begin(); it != q.pending.end();) {
      Request *r = *it;
      if (SameParams(*r->params, p0) && (group.empty() || images + r->n <= kMaxImages)) {
        group.push_back(r);
        images += r->n;
        it = q.pending.erase(it);
      } else {
        ++it;
      }
    }
    lk.unlock();
    try {
      RunGroup(dec, group);
    } catch (...) {
      for (Request *r : group) r->status = ROCJPEG_STATUS_RUNTIME_ERROR;
    }
    lk.lock();
    for (Request *r : group) r->done = true;
    q.busy = false;
    q.cv.notify_all();
  }
  return me.status;
}

void CoalesceStats(uint64_t *calls, uint64_t *combined, uint64_t *members) {
  if (calls) *calls = g_calls.load();
  if (combined) *combined = g_combined.load();
  if (members) *members = g_members.load();
}

}  // namespace rj
