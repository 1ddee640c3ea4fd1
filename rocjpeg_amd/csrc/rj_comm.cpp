// rj_comm.cpp -- multi-GPU batched decode behind the C ABI (include/rocjpeg_amd.h
// "Multi-GPU batched decode through the C ABI").
//
// The reference has one device per handle (src/rocjpeg_api.cpp:107-120) and scales only by one
// handle per thread (samples/jpegDecodePerf/jpegdecodeperf.cpp:228-257); its batched call is
// src/rocjpeg_decoder.cpp:196-292.  Here a C caller with one process (or thread) per GPU:
//   rocJpegAmdCommGetUniqueId (one rank) -> shares the id -> rocJpegAmdCommInitRank (every rank)
//   rocJpegAmdDecodeBatchedSharded: rank 0 walks the headers into the 64-byte work table and
//     assigns images by LPT (rj_shard.cpp), ONE RCCL broadcast of the table over xGMI (the path's
//     only collective), then every rank parses and decodes its own images with
//     rocJpegDecodeBatched into the caller's destinations.
// RCCL is loaded at run time (dlopen librccl.so.1): the library needs it only when a
// communicator is created, and a process that already holds RCCL (e.g. PyTorch's copy) shares it.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/rocjpeg.h"
#include "../../include/rocjpeg_amd.h"
#include "rj_common.h"

#define RJ_EXPORT extern "C" __attribute__((visibility("default")))

static_assert(sizeof(RocJpegAmdCommId) == sizeof(ncclUniqueId), "RocJpegAmdCommId mirrors ncclUniqueId");

namespace {

struct Rccl {
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) init_rank = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclCommCount) count = nullptr;
  decltype(&ncclCommUserRank) user_rank = nullptr;
  decltype(&ncclBroadcast) broadcast = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  bool ok = false;
};

const Rccl &LoadRccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void *h = nullptr;
    for (const char *name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
      if ((h = dlopen(name, RTLD_NOW | RTLD_LOCAL)) != nullptr) break;
    if (h == nullptr) {
      RJ_ERR("librccl.so.1 not found: %s", dlerror());
      return;
    }
    r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(dlsym(h, "ncclGetUniqueId"));
    r.init_rank = reinterpret_cast<decltype(r.init_rank)>(dlsym(h, "ncclCommInitRank"));
    r.destroy = reinterpret_cast<decltype(r.destroy)>(dlsym(h, "ncclCommDestroy"));
    r.count = reinterpret_cast<decltype(r.count)>(dlsym(h, "ncclCommCount"));
    r.user_rank = reinterpret_cast<decltype(r.user_rank)>(dlsym(h, "ncclCommUserRank"));
    r.broadcast = reinterpret_cast<decltype(r.broadcast)>(dlsym(h, "ncclBroadcast"));
    r.error_string = reinterpret_cast<decltype(r.error_string)>(dlsym(h, "ncclGetErrorString"));
    r.ok = r.get_unique_id && r.init_rank && r.destroy && r.count && r.user_rank && r.broadcast && r.error_string;
    if (!r.ok) RJ_ERR("librccl.so.1 lacks an entry point this library needs");
  });
  return r;
}

RocJpegStatus Fail(const Rccl &r, ncclResult_t e, const char *what) {
  RJ_ERR("%s: %s", what, r.error_string ? r.error_string(e) : "RCCL error");
  return ROCJPEG_STATUS_EXECUTION_FAILED;
}

}  // namespace

// One rank's communicator: the RCCL comm, its device, a stream for the collective and a
// grow-only device buffer for the table.
struct RocJpegAmdCommImpl {
  ncclComm_t comm = nullptr;
  int device = 0, rank = 0, nranks = 1;
  hipStream_t stream = nullptr;
  void *dbuf = nullptr;
  size_t dbuf_bytes = 0;
};

RJ_EXPORT RocJpegStatus rocJpegAmdCommGetUniqueId(RocJpegAmdCommId *id) {
  if (id == nullptr) return ROCJPEG_STATUS_INVALID_PARAMETER;
  const Rccl &r = LoadRccl();
  if (!r.ok) return ROCJPEG_STATUS_NOT_INITIALIZED;
  ncclUniqueId u;
  const ncclResult_t e = r.get_unique_id(&u);
  if (e != ncclSuccess) return Fail(r, e, "ncclGetUniqueId");
  std::memcpy(id, &u, sizeof(u));
  return ROCJPEG_STATUS_SUCCESS;
}

RJ_EXPORT RocJpegStatus rocJpegAmdCommInitRank(int device_id, int nranks, const RocJpegAmdCommId *id, int rank,
                                               RocJpegAmdComm *comm) {
  if (id == nullptr || comm == nullptr || nranks < 1 || rank < 0 || rank >= nranks)
    return ROCJPEG_STATUS_INVALID_PARAMETER;
  *comm = nullptr;
  const Rccl &r = LoadRccl();
  if (!r.ok) return ROCJPEG_STATUS_NOT_INITIALIZED;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device_id < 0 || device_id >= ndev) return ROCJPEG_STATUS_INVALID_PARAMETER;
  int prev = 0;
  (void)hipGetDevice(&prev);
  RocJpegAmdCommImpl *c = new (std::nothrow) RocJpegAmdCommImpl;
  if (c == nullptr) return ROCJPEG_STATUS_OUTOF_MEMORY;
  c->device = device_id;
  c->rank = rank;
  c->nranks = nranks;
  RocJpegStatus st = ROCJPEG_STATUS_SUCCESS;
  if (hipSetDevice(device_id) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    st = ROCJPEG_STATUS_NOT_INITIALIZED;
  } else {
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    const ncclResult_t e = r.init_rank(&c->comm, nranks, u, rank);
    if (e != ncclSuccess) st = Fail(r, e, "ncclCommInitRank");
  }
  (void)hipSetDevice(prev);
  if (st != ROCJPEG_STATUS_SUCCESS) {
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return st;
  }
  *comm = c;
  return ROCJPEG_STATUS_SUCCESS;
}

RJ_EXPORT RocJpegStatus rocJpegAmdCommDestroy(RocJpegAmdComm c) {
  if (c == nullptr) return ROCJPEG_STATUS_INVALID_PARAMETER;
  const Rccl &r = LoadRccl();
  int prev = 0;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(c->device);
  if (c->comm && r.ok) (void)r.destroy(c->comm);
  if (c->dbuf) (void)hipFree(c->dbuf);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  (void)hipSetDevice(prev);
  delete c;
  return ROCJPEG_STATUS_SUCCESS;
}

RJ_EXPORT RocJpegStatus rocJpegAmdCommInfo(RocJpegAmdComm c, int *rank, int *nranks, int *device_id) {
  if (c == nullptr) return ROCJPEG_STATUS_INVALID_PARAMETER;
  if (rank) *rank = c->rank;
  if (nranks) *nranks = c->nranks;
  if (device_id) *device_id = c->device;
  return ROCJPEG_STATUS_SUCCESS;
}

// The one collective: rank 0's `count` records travel to every rank (device buffers on each
// rank's GPU, RCCL broadcast over xGMI).  Every rank passes the same count.
RJ_EXPORT RocJpegStatus rocJpegAmdBroadcastWorkTable(RocJpegAmdComm c, RocJpegAmdWorkItem *items, int count) {
  if (c == nullptr || count < 0 || (count > 0 && items == nullptr)) return ROCJPEG_STATUS_INVALID_PARAMETER;
  if (count == 0 || c->nranks == 1) return ROCJPEG_STATUS_SUCCESS;
  const Rccl &r = LoadRccl();
  if (!r.ok) return ROCJPEG_STATUS_NOT_INITIALIZED;
  const size_t bytes = size_t(count) * sizeof(RocJpegAmdWorkItem);
  int prev = 0;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(c->device);
  RocJpegStatus st = ROCJPEG_STATUS_SUCCESS;
  if (c->dbuf_bytes < bytes) {
    if (c->dbuf) (void)hipFree(c->dbuf);
    c->dbuf = nullptr;
    c->dbuf_bytes = 0;
    if (hipMalloc(&c->dbuf, bytes) != hipSuccess) st = ROCJPEG_STATUS_OUTOF_MEMORY;
    else c->dbuf_bytes = bytes;
  }
  if (st == ROCJPEG_STATUS_SUCCESS && c->rank == 0 &&
      hipMemcpyAsync(c->dbuf, items, bytes, hipMemcpyHostToDevice, c->stream) != hipSuccess)
    st = ROCJPEG_STATUS_EXECUTION_FAILED;
  if (st == ROCJPEG_STATUS_SUCCESS) {
    const ncclResult_t e = r.broadcast(c->dbuf, c->dbuf, bytes, ncclUint8, 0, c->comm, c->stream);
    if (e != ncclSuccess) st = Fail(r, e, "ncclBroadcast");
  }
  if (st == ROCJPEG_STATUS_SUCCESS && c->rank != 0 &&
      hipMemcpyAsync(items, c->dbuf, bytes, hipMemcpyDeviceToHost, c->stream) != hipSuccess)
    st = ROCJPEG_STATUS_EXECUTION_FAILED;
  if (hipStreamSynchronize(c->stream) != hipSuccess && st == ROCJPEG_STATUS_SUCCESS) st = ROCJPEG_STATUS_EXECUTION_FAILED;
  (void)hipSetDevice(prev);
  return st;
}

// Rank 0: the table from the headers + LPT over the communicator's ranks (shard = rank); then
// the broadcast.  Every rank passes the same blob description.
RJ_EXPORT RocJpegStatus rocJpegAmdShardPlan(RocJpegAmdComm c, const unsigned char *blob, uint64_t blob_bytes,
                                            const uint64_t *offsets, const uint32_t *sizes, int count,
                                            RocJpegAmdWorkItem *items) {
  if (c == nullptr || count < 0 || (count > 0 && items == nullptr)) return ROCJPEG_STATUS_INVALID_PARAMETER;
  if (c->rank == 0) {
    RocJpegStatus st = rocJpegAmdBuildWorkTable(blob, blob_bytes, offsets, sizes, count, items);
    if (st == ROCJPEG_STATUS_SUCCESS) st = rocJpegAmdAssignShards(items, count, c->nranks, nullptr, nullptr);
    // a failed plan on rank 0 still takes part in the broadcast (the other ranks wait in it): it
    // sends a table that assigns nothing, then reports its error
    if (st != ROCJPEG_STATUS_SUCCESS) {
      for (int i = 0; i < count; i++) {
        std::memset(items + i, 0, sizeof(RocJpegAmdWorkItem));
        items[i].shard = -1;
        items[i].index = uint32_t(i);
      }
      (void)rocJpegAmdBroadcastWorkTable(c, items, count);
      return st;
    }
  }
  return rocJpegAmdBroadcastWorkTable(c, items, count);
}

// Plan + this rank's share of rocJpegDecodeBatched (src/rocjpeg_decoder.cpp:196-292 semantics
// per rank).  destinations: `count` entries in batch order; only this rank's images are
// written.  items (optional, `count` records): the broadcast table, so the caller knows where
// each image was decoded.  Parse failures of this rank's images return BAD_JPEG before any
// decode, as the reference's rocJpegStreamParse would have.
RJ_EXPORT RocJpegStatus rocJpegAmdDecodeBatchedSharded(RocJpegHandle handle, RocJpegAmdComm c,
                                                       const unsigned char *blob, uint64_t blob_bytes,
                                                       const uint64_t *offsets, const uint32_t *sizes, int count,
                                                       const RocJpegDecodeParams *params,
                                                       RocJpegImage *destinations, RocJpegAmdWorkItem *items) {
  if (handle == nullptr || c == nullptr || params == nullptr || count < 0 ||
      (count > 0 && (destinations == nullptr || offsets == nullptr || sizes == nullptr || blob == nullptr)))
    return ROCJPEG_STATUS_INVALID_PARAMETER;
  try {
    std::vector<RocJpegAmdWorkItem> own;
    RocJpegAmdWorkItem *tab = items;
    if (tab == nullptr) {
      own.resize(size_t(count));
      tab = own.data();
    }
    RocJpegStatus st = rocJpegAmdShardPlan(c, blob, blob_bytes, offsets, sizes, count, tab);
    if (st != ROCJPEG_STATUS_SUCCESS) return st;
    std::vector<int> mine;
    for (int i = 0; i < count; i++)
      if (tab[i].shard == c->rank) mine.push_back(int(tab[i].index));
    for (int i : mine)  // the table comes from rank 0: check its indices against this rank's view
      if (i < 0 || i >= count || offsets[i] > blob_bytes || sizes[i] > blob_bytes - offsets[i])
        return ROCJPEG_STATUS_RUNTIME_ERROR;
    std::vector<RocJpegStreamHandle> streams(mine.size(), nullptr);
    std::vector<RocJpegImage> dst(mine.size());
    for (size_t k = 0; k < mine.size() && st == ROCJPEG_STATUS_SUCCESS; k++) {
      st = rocJpegStreamCreate(&streams[k]);
      if (st == ROCJPEG_STATUS_SUCCESS) st = rocJpegStreamParse(blob + offsets[mine[k]], sizes[mine[k]], streams[k]);
      dst[k] = destinations[mine[k]];
    }
    if (st == ROCJPEG_STATUS_SUCCESS && !mine.empty())
      st = rocJpegDecodeBatched(handle, streams.data(), int(mine.size()), params, dst.data());
    for (RocJpegStreamHandle s : streams)
      if (s) (void)rocJpegStreamDestroy(s);
    return st;
  } catch (const std::bad_alloc &) {
    return ROCJPEG_STATUS_OUTOF_MEMORY;
  } catch (...) {
    return ROCJPEG_STATUS_RUNTIME_ERROR;
  }
}
