// rj_coalesce.cpp -- see rj_coalesce.h.
#include "rj_coalesce.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>
#include <unordered_map>
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
  bool taken = false;  // in a leader's group (decoding)
  bool done = false;
};

bool SameParams(const RocJpegDecodeParams &a, const RocJpegDecodeParams &b) {
  return a.output_format == b.output_format && a.crop_rectangle.left == b.crop_rectangle.left &&
         a.crop_rectangle.top == b.crop_rectangle.top && a.crop_rectangle.right == b.crop_rectangle.right &&
         a.crop_rectangle.bottom == b.crop_rectangle.bottom;
}

using Clock = std::chrono::steady_clock;

// One device's queue of waiting calls and how many leaders are decoding.
struct DeviceQueue {
  std::mutex mu;
  std::condition_variable cv;      // a group finished
  std::condition_variable arrive;  // a call was queued (a gathering leader waits on it)
  std::deque<Request *> pending;
  int busy = 0;
  // threads that called on this device recently, and the last group's decode time: a leader
  // waits briefly for the recent callers that are not queued yet (they return from the previous
  // group together and call again within microseconds), so that they form one group instead of
  // two alternating half groups
  std::unordered_map<std::thread::id, Clock::time_point> seen;
  double group_us = 0;
};

int EnvInt(const char *name, int dflt) {
  const char *e = std::getenv(name);
  return e ? std::atoi(e) : dflt;
}
// at most this many combined calls decode at once per device (each on its leader's handle)
int Inflight() {
  static const int v = std::max(1, EnvInt("RJ_COALESCE_INFLIGHT", 1));
  return v;
}
// the longest a leader waits for recent callers to arrive (microseconds; 0: no wait)
int GatherUs() {
  static const int v = std::max(0, EnvInt("RJ_COALESCE_WAIT_US", 300));
  return v;
}
constexpr auto kRecent = std::chrono::milliseconds(10);  // a caller counts as active this long

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

// The group's calls as one call on `dec`.  Each member is first checked as its own call would
// be (Decoder::Check: the host validation a decode runs before any device work); a member that
// fails there gets that status at once and stays out of the combined call, so one caller's bad
// stream or destination costs the others nothing.  Should the combined call still fail (a device
// error), each remaining call is decoded alone and gets its own status.
void RunGroup(Decoder *dec, std::vector<Request *> &group) {
  if (group.size() == 1) {
    Request *r = group[0];
    r->status = dec->Decode(r->streams, r->n, r->params, r->dst);
    return;
  }
  std::vector<Request *> ok;
  ok.reserve(group.size());
  for (Request *r : group) {
    r->status = dec->Check(r->streams, r->n, r->params, r->dst);
    if (r->status == 0) ok.push_back(r);
  }
  if (ok.empty()) return;
  if (ok.size() == 1) {
    ok[0]->status = dec->Decode(ok[0]->streams, ok[0]->n, ok[0]->params, ok[0]->dst);
    return;
  }
  g_combined.fetch_add(1, std::memory_order_relaxed);
  g_members.fetch_add(ok.size(), std::memory_order_relaxed);
  std::vector<Stream *> streams;
  std::vector<RocJpegImage> dst;
  for (Request *r : ok) {
    streams.insert(streams.end(), r->streams, r->streams + r->n);
    dst.insert(dst.end(), r->dst, r->dst + r->n);
  }
  const int st = dec->Decode(streams.data(), int(streams.size()), ok[0]->params, dst.data());
  if (st == 0) return;
  for (Request *r : ok) r->status = dec->Decode(r->streams, r->n, r->params, r->dst);
}

}  // namespace

int CoalescedDecode(Decoder *dec, int device, Stream *const *streams, int n, const RocJpegDecodeParams *params,
                    RocJpegImage *dst) {
  if (!Enabled() || n > kSmallCall || n <= 0 || device < 0 || streams == nullptr || params == nullptr ||
      dst == nullptr || !dec->Coalescable())
    return dec->Decode(streams, n, params, dst);
  g_calls.fetch_add(1, std::memory_order_relaxed);
  DeviceQueue &q = QueueFor(device);
  Request me{dec, streams, n, params, dst};
  std::unique_lock<std::mutex> lk(q.mu);
  const Clock::time_point now = Clock::now();
  q.seen[std::this_thread::get_id()] = now;  // (may throw: nothing is queued yet)
  if (q.seen.size() > 256)
    for (auto it = q.seen.begin(); it != q.seen.end();) it = now - it->second > kRecent ? q.seen.erase(it) : ++it;
  q.pending.push_back(&me);
  // `me` lives on this stack: should anything below throw while it is still queued (not yet in a
  // group), it leaves the queue before the unwind (the lock is held wherever that can happen)
  struct Unqueue {
    DeviceQueue &q;
    Request &me;
    ~Unqueue() {
      if (me.taken) return;
      auto it = std::find(q.pending.begin(), q.pending.end(), &me);
      if (it != q.pending.end()) q.pending.erase(it);
    }
  } unqueue{q, me};
  q.arrive.notify_all();
  while (!me.done) {
    // a call already in another leader's group only waits for it; a queued call leads when a
    // decode slot is free
    if (me.taken || q.busy >= Inflight()) {
      q.cv.wait(lk);
      continue;
    }
    // leader.  First the gathering window: while fewer calls are queued than threads called
    // recently, wait for them up to min(GatherUs, a quarter of the last group's time)
    q.busy++;
    if (GatherUs() > 0) {
      const Clock::time_point t0 = Clock::now();
      size_t recent = 0;
      for (const auto &kv : q.seen) recent += t0 - kv.second <= kRecent ? 1 : 0;
      // with k groups in flight the recent callers form k cohorts, each led by one leader
      recent = (recent + size_t(Inflight()) - 1) / size_t(Inflight());
      const double wait_us = std::min(double(GatherUs()), std::max(30.0, 0.25 * q.group_us));
      const Clock::time_point deadline = t0 + std::chrono::microseconds(int64_t(wait_us));
      while (!me.taken && q.pending.size() < recent && Clock::now() < deadline) q.arrive.wait_until(lk, deadline);
      if (me.taken) {  // another leader took this call while the lock was released: it only waits now
        q.busy--;
        q.cv.notify_all();
        continue;
      }
    }
    // the oldest waiting call and every other with the same parameters, up to kMaxImages (the
    // group's storage first: no allocation may fail once a member is marked taken)
    std::vector<Request *> group;
    group.reserve(q.pending.size());
    int images = 0;
    const RocJpegDecodeParams p0 = *q.pending.front()->params;
    for (auto it = q.pending.begin(); it != q.pending.end();) {
      Request *r = *it;
      if (SameParams(*r->params, p0) && (group.empty() || images + r->n <= kMaxImages)) {
        r->taken = true;
        group.push_back(r);
        images += r->n;
        it = q.pending.erase(it);
      } else {
        ++it;
      }
    }
    lk.unlock();
    const Clock::time_point g0 = Clock::now();
    try {
      RunGroup(dec, group);
    } catch (...) {
      for (Request *r : group) r->status = ROCJPEG_STATUS_RUNTIME_ERROR;
    }
    const double us = std::chrono::duration<double, std::micro>(Clock::now() - g0).count();
    lk.lock();
    q.group_us = us;
    for (Request *r : group) r->done = true;
    q.busy--;
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
