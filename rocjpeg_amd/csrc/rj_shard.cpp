// rj_shard.cpp -- the work table of a multi-GPU batched decode (SURVEY.md 8e,
// include/rocjpeg_amd.h rocJpegAmdBuildWorkTable / rocJpegAmdAssignShards).
//
// The reference decodes on one device per handle (src/rocjpeg_api.cpp:107-120) and scales
// only by one handle per thread (samples/jpegDecodePerf/jpegdecodeperf.cpp:228-257).  Here a
// batch is split across GPUs by whole images: one process per GPU, rank 0 reads the headers
// and balances the shards, the table travels by one RCCL broadcast (rocjpeg_amd/shard.py), and
// each rank calls rocJpegDecodeBatched (src/rocjpeg_decoder.cpp:196-292 semantics) on its own
// images.  Nothing here touches a GPU.
#include <algorithm>
#include <atomic>
#include <cstring>
#include <queue>
#include <thread>
#include <vector>

#include "../../include/rocjpeg.h"
#include "../../include/rocjpeg_amd.h"
#include "rj_common.h"
#include "rj_stream.h"

#define RJ_EXPORT extern "C" __attribute__((visibility("default")))

static_assert(sizeof(RocJpegAmdWorkItem) == 64, "work-table record: 64 B (SURVEY.md 8e)");

namespace {

// One record from the image's headers.  Baseline: the header walk only (the O(bytes) FF D9
// scan is left to the rank that decodes the image); progressive: the full scan walk.
void FillItem(const unsigned char *data, uint32_t size, uint32_t index, uint64_t offset, RocJpegAmdWorkItem *it) {
  std::memset(it, 0, sizeof(*it));
  it->stream_offset = offset;
  it->stream_bytes = size;
  it->index = index;
  it->shard = -1;
  it->dest_device = -1;
  it->subsampling = -1;
  rj::Stream s;
  if (data == nullptr || !s.Parse(data, size, /*defer_scan=*/true)) {
    it->flags = ROCJPEG_AMD_WORK_BAD;
    return;
  }
  const rj::StreamInfo &in = s.info();
  const rj::DecodePlan &p = s.plan();
  it->width = in.width;
  it->height = in.height;
  it->subsampling = in.css;
  it->ecs_bytes = in.ecs_size;
  if (p.status != 0) it->flags |= ROCJPEG_AMD_WORK_UNSUPPORTED;
  uint64_t per_byte = ROCJPEG_AMD_COST_BYTE;
  if (p.progressive) {
    it->flags |= ROCJPEG_AMD_WORK_PROGRESSIVE;
    per_byte = ROCJPEG_AMD_COST_BYTE_PROG;
  } else {
    const uint32_t total = p.mcux * p.mcuy, ri = in.restart_interval;
    it->restart_intervals = (ri && total) ? (total + ri - 1) / ri : 1u;
  }
  // K1's time on a shard is set by its longest serial chain as well as by its total bytes: the
  // mean restart-interval length (capped where the chunk lanes take over, RJ_SPLIT_BYTES) weighs
  // in, so LPT deals images with long intervals (e.g. the 3840-wide rows of C4) across the shards
  // before the rest
  const uint64_t ival = p.progressive ? 0u : std::min<uint64_t>(it->ecs_bytes / std::max(1u, it->restart_intervals),
                                                                ROCJPEG_AMD_COST_INTERVAL_CAP);
  it->cost = (it->flags & ROCJPEG_AMD_WORK_UNSUPPORTED)
                 ? 0
                 : per_byte * it->ecs_bytes + uint64_t(in.width) * in.height + ROCJPEG_AMD_COST_INTERVAL * ival;
}

}  // namespace

RJ_EXPORT RocJpegStatus rocJpegAmdBuildWorkTable(const unsigned char *blob, uint64_t blob_bytes,
                                                 const uint64_t *offsets, const uint32_t *sizes, int count,
                                                 RocJpegAmdWorkItem *items) {
  if (count < 0 || (count > 0 && (blob == nullptr || offsets == nullptr || sizes == nullptr || items == nullptr)))
    return ROCJPEG_STATUS_INVALID_PARAMETER;
  // every stream must lie inside the blob (checked before any worker reads a byte)
  for (int i = 0; i < count; i++)
    if (offsets[i] > blob_bytes || sizes[i] > blob_bytes - offsets[i]) return ROCJPEG_STATUS_INVALID_PARAMETER;
  // a worker never lets an exception escape its thread (that would std::terminate the caller):
  // the first failure is recorded and the call returns RUNTIME_ERROR
  std::atomic<bool> failed{false};
  auto run = [&](int a, int b) {
    try {
      for (int i = a; i < b; i++) FillItem(blob + offsets[i], sizes[i], uint32_t(i), offsets[i], items + i);
    } catch (...) {
      failed.store(true);
    }
  };
  const int nt = count >= 512 ? int(std::min<unsigned>(8, std::max(1u, std::thread::hardware_concurrency()))) : 1;
  std::vector<std::thread> th;
  th.reserve(size_t(nt));
  for (int t = 1; t < nt; t++) {
    try {
      th.emplace_back(run, int(int64_t(count) * t / nt), int(int64_t(count) * (t + 1) / nt));
    } catch (...) {  // no thread: this range (and the ones after it) run on the calling thread
      run(int(int64_t(count) * t / nt), count);
      break;
    }
  }
  run(0, count / nt);
  for (auto &x : th) x.join();
  return failed.load() ? ROCJPEG_STATUS_RUNTIME_ERROR : ROCJPEG_STATUS_SUCCESS;
}

RJ_EXPORT RocJpegStatus rocJpegAmdAssignShards(RocJpegAmdWorkItem *items, int count, int num_shards,
                                               const int *shard_devices, uint64_t *shard_cost) {
  if (count < 0 || num_shards < 1 || (count > 0 && items == nullptr)) return ROCJPEG_STATUS_INVALID_PARAMETER;
  try {
    std::vector<uint32_t> order(static_cast<size_t>(count));
    for (int i = 0; i < count; i++) order[i] = uint32_t(i);
    std::stable_sort(order.begin(), order.end(),
                     [&](uint32_t a, uint32_t b) { return items[a].cost > items[b].cost; });
    // min-heap of (assigned cost, shard): the lightest shard takes the next-heaviest image
    using Load = std::pair<uint64_t, int>;
    std::priority_queue<Load, std::vector<Load>, std::greater<Load>> heap;
    for (int s = 0; s < num_shards; s++) heap.push({0, s});
    std::vector<uint64_t> load(static_cast<size_t>(num_shards), 0);
    for (uint32_t i : order) {
      const Load l = heap.top();
      heap.pop();
      items[i].shard = l.second;
      items[i].dest_device = shard_devices ? shard_devices[l.second] : l.second;
      load[l.second] = l.first + items[i].cost;
      heap.push({load[l.second], l.second});
    }
    if (shard_cost)
      for (int s = 0; s < num_shards; s++) shard_cost[s] = load[s];
  } catch (...) {
    return ROCJPEG_STATUS_RUNTIME_ERROR;
  }
  return ROCJPEG_STATUS_SUCCESS;
}
