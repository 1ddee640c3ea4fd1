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
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstddef>
#include <cstdlib>
#include <cstring>
#include <thread>
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

// The work table travels in fixed-size chunks of 64-B records; chunk 0 starts with a header
// record from rank 0 (its status and count), so every rank runs the same number of broadcasts
// -- rank 0's -- whatever its own arguments were.
constexpr uint32_t kChunkRecords = 4096;
constexpr size_t kChunkBytes = size_t(kChunkRecords) * sizeof(RocJpegAmdWorkItem);
constexpr uint32_t kTableMagic = 0x524A5442u;  // "RJTB"
struct TableHeader {
  uint32_t magic;
  int32_t status;   // rank 0's plan status: every rank returns it
  uint32_t count;   // records that follow
  uint32_t chunks;  // broadcasts of this table (chunk 0 included)
  uint32_t seq;     // the communicator's exchange number (equal on every rank)
  uint32_t pad0;
  uint64_t check;   // FNV-1a over the header fields before it and every record
  uint8_t pad[32];
};
static_assert(sizeof(TableHeader) == sizeof(RocJpegAmdWorkItem), "header record: 64 B");

uint64_t Fnv(const void *p, size_t n, uint64_t h = 1469598103934665603ull) {
  const uint8_t *b = static_cast<const uint8_t *>(p);
  for (size_t i = 0; i < n; i++) h = (h ^ b[i]) * 1099511628211ull;
  return h;
}
uint32_t ChunksFor(uint32_t count) { return count < kChunkRecords ? 1u : 1u + (count - (kChunkRecords - 1) + kChunkRecords - 1) / kChunkRecords; }

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
  void *dbuf = nullptr;  // one broadcast chunk (kChunkBytes), allocated at init
  std::vector<RocJpegAmdWorkItem> scratch;  // a chunk on the host
  uint32_t seq = 0;                          // exchanges so far (every rank counts them alike)
  struct ShmBus *shm = nullptr;              // test transport (RJ_COMM_TEST_SHM), else RCCL
  uint32_t shm_gen = 0;
};

// Test transport: RJ_COMM_TEST_SHM=<file> at rocJpegAmdCommInitRank makes the communicator move
// each chunk through a shared host mapping of <file> instead of RCCL, so that several ranks can
// share ONE GPU (RCCL refuses two ranks on one device) and the multi-rank protocol above -- the
// chunking, the status header, the checks, the error paths -- runs with real device buffers and
// copies on a one-GPU box (tests/test_comm_gpu.py).  Same chunks, same order, same buffers as
// the RCCL broadcast; only the wire differs.  Compiled only into the test build of the library
// (-DRJ_COMM_TEST_TRANSPORT: rocjpeg_amd/librocjpeg_amd_testcomm.so); the product library has
// no such switch.
struct ShmBus {
  std::atomic<uint32_t> gen;   // chunks rank 0 has published
  std::atomic<uint32_t> acks;  // chunks taken by receivers, summed
  uint32_t pad[14];
  uint8_t data[kChunkBytes];
};

namespace {
bool ShmWait(const std::atomic<uint32_t> &v, uint32_t target) {
  const auto t0 = std::chrono::steady_clock::now();
  while (v.load(std::memory_order_acquire) < target) {
    if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60)) return false;
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
  return true;
}

// one chunk: rank 0's device buffer -> every rank's device buffer (through the mapping)
ncclResult_t ShmBroadcast(RocJpegAmdCommImpl *c) {
  ShmBus *b = c->shm;
  const uint32_t g = ++c->shm_gen;
  if (c->rank == 0) {
    if (!ShmWait(b->acks, (g - 1) * uint32_t(c->nranks - 1))) return ncclSystemError;  // previous chunk taken
    if (hipMemcpyAsync(b->data, c->dbuf, kChunkBytes, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess)
      return ncclUnhandledCudaError;
    b->gen.store(g, std::memory_order_release);
  } else {
    if (!ShmWait(b->gen, g)) return ncclSystemError;
    if (hipMemcpyAsync(c->dbuf, b->data, kChunkBytes, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess)
      return ncclUnhandledCudaError;
    b->acks.fetch_add(1, std::memory_order_acq_rel);
  }
  return ncclSuccess;
}

ncclResult_t BroadcastChunk(const Rccl &r, RocJpegAmdCommImpl *c) {
  if (c->shm) return ShmBroadcast(c);
  return r.broadcast(c->dbuf, c->dbuf, kChunkBytes, ncclUint8, 0, c->comm, c->stream);
}

ShmBus *MapShm(const char *path) {
  const int fd = open(path, O_RDWR | O_CREAT, 0600);
  if (fd < 0) return nullptr;
  struct stat st;
  if (fstat(fd, &st) != 0 || (size_t(st.st_size) < sizeof(ShmBus) && ftruncate(fd, sizeof(ShmBus)) != 0)) {
    close(fd);
    return nullptr;
  }
  void *p = mmap(nullptr, sizeof(ShmBus), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  return p == MAP_FAILED ? nullptr : static_cast<ShmBus *>(p);
}
}  // namespace

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
  // the broadcast's device buffer is allocated here, before the communicator exists: a local
  // allocation failure then fails this rank's init, never a later collective (which the other
  // ranks would enter alone)
  if (hipSetDevice(device_id) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    st = ROCJPEG_STATUS_NOT_INITIALIZED;
  } else if (hipMalloc(&c->dbuf, kChunkBytes) != hipSuccess) {
    c->dbuf = nullptr;
    st = ROCJPEG_STATUS_OUTOF_MEMORY;
#ifdef RJ_COMM_TEST_TRANSPORT
  } else if (const char *shm = std::getenv("RJ_COMM_TEST_SHM")) {
    if ((c->shm = MapShm(shm)) == nullptr) st = ROCJPEG_STATUS_NOT_INITIALIZED;
#endif
  } else {
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    const ncclResult_t e = r.init_rank(&c->comm, nranks, u, rank);
    if (e != ncclSuccess) st = Fail(r, e, "ncclCommInitRank");
  }
  (void)hipSetDevice(prev);
  if (st != ROCJPEG_STATUS_SUCCESS) {
    if (c->dbuf) (void)hipFree(c->dbuf);
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
  if (c->shm) (void)munmap(c->shm, sizeof(ShmBus));
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

// The one collective, with its status.  Rank 0 sends `status` and its `count` records; every
// rank takes part in exactly ChunksFor(rank 0's count) broadcasts, whatever it passed itself,
// so a rank with bad local arguments (or a failed plan on rank 0) never leaves the others
// waiting in a collective.  Receivers get rank 0's status in *status0 and its records in `items`
// (up to their own `count`); a count that differs from rank 0's is INVALID_PARAMETER on that
// rank after the collective.  The header carries a per-communicator sequence number and a hash
// of every record: a stale device buffer (rank 0's upload of chunk 0 failed: then it sends only
// that chunk) or a damaged later chunk is EXECUTION_FAILED on the receivers, never a wrong table.
// A receiver whose own device copy fails cannot follow the exchange any further (the device is
// unusable); that is the one case in which other ranks can be left waiting.
namespace {
RocJpegStatus BroadcastWithStatus(RocJpegAmdCommImpl *c, RocJpegAmdWorkItem *items, int count, RocJpegStatus status,
                                  RocJpegStatus *status0) {
  *status0 = status;
  const bool own_ok = count >= 0 && (count == 0 || items != nullptr);
  if (c->nranks == 1) return own_ok ? ROCJPEG_STATUS_SUCCESS : ROCJPEG_STATUS_INVALID_PARAMETER;
  const Rccl &r = LoadRccl();
  if (!r.ok) return ROCJPEG_STATUS_NOT_INITIALIZED;  // then no communicator exists on any rank
  std::vector<RocJpegAmdWorkItem> &buf = c->scratch;
  buf.resize(kChunkRecords);  // may throw: before any collective
  int prev = 0;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(c->device);
  const uint32_t seq = ++c->seq;
  RocJpegStatus st = ROCJPEG_STATUS_SUCCESS;
  uint32_t chunks = 1, total = 0;
  uint64_t want = 0, hash = 0;
  if (c->rank == 0) {
    if (!own_ok && status == ROCJPEG_STATUS_SUCCESS) *status0 = status = ROCJPEG_STATUS_INVALID_PARAMETER;
    total = own_ok ? uint32_t(count) : 0u;  // rank 0 with bad arguments sends its status and no records
    chunks = ChunksFor(total);
  }
  for (uint32_t k = 0; k < chunks; k++) {
    // chunk 0 holds the header + (kChunkRecords - 1) records, the others kChunkRecords
    const uint32_t first = k == 0 ? 0u : (kChunkRecords - 1) + (k - 1) * kChunkRecords;
    const uint32_t slot0 = k == 0 ? 1u : 0u;
    if (c->rank == 0) {
      const uint32_t n = std::min<uint32_t>(total - std::min(total, first), kChunkRecords - slot0);
      if (n) std::memcpy(buf.data() + slot0, items + first, n * sizeof(RocJpegAmdWorkItem));
      if (k == 0) {
        TableHeader h{};
        h.magic = kTableMagic;
        h.status = int32_t(status);
        h.count = total;
        h.chunks = chunks;
        h.seq = seq;
        h.check = Fnv(items, size_t(total) * sizeof(RocJpegAmdWorkItem), Fnv(&h, offsetof(TableHeader, check)));
        std::memcpy(buf.data(), &h, sizeof(h));
      }
      // synchronised before the next chunk rewrites the pageable host buffer (an
      // asynchronous copy from pageable memory may still be reading it)
      if (hipMemcpyAsync(c->dbuf, buf.data(), kChunkBytes, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
          hipStreamSynchronize(c->stream) != hipSuccess) {
        st = ROCJPEG_STATUS_EXECUTION_FAILED;
        if (k == 0) chunks = 1;  // the receivers find a stale header in chunk 0 and stop after it
      }
    }
    // every rank: the same number of same-sized broadcasts
    const ncclResult_t e = BroadcastChunk(r, c);
    if (e != ncclSuccess) {
      st = Fail(r, e, "ncclBroadcast");
      break;  // the communicator is broken: nothing more can be exchanged
    }
    if (c->rank == 0) continue;
    if (hipMemcpyAsync(buf.data(), c->dbuf, kChunkBytes, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess) {
      st = ROCJPEG_STATUS_EXECUTION_FAILED;
      break;
    }
    if (k == 0) {
      TableHeader h;
      std::memcpy(&h, buf.data(), sizeof(h));
      if (h.magic != kTableMagic || h.seq != seq || h.chunks != ChunksFor(h.count)) {
        st = ROCJPEG_STATUS_EXECUTION_FAILED;  // rank 0 sent only this chunk
        break;
      }
      total = h.count;
      chunks = h.chunks;
      want = h.check;
      hash = Fnv(&h, offsetof(TableHeader, check));
      *status0 = RocJpegStatus(h.status);
    }
    const uint32_t n = std::min<uint32_t>(total - std::min(total, first), kChunkRecords - slot0);
    hash = Fnv(buf.data() + slot0, n * sizeof(RocJpegAmdWorkItem), hash);
    if (own_ok) {
      const uint32_t lim = std::min<uint32_t>(total, uint32_t(count));
      const uint32_t m = std::min<uint32_t>(lim - std::min(lim, first), kChunkRecords - slot0);
      if (m) std::memcpy(items + first, buf.data() + slot0, m * sizeof(RocJpegAmdWorkItem));
    }
  }
  if (hipStreamSynchronize(c->stream) != hipSuccess && st == ROCJPEG_STATUS_SUCCESS) st = ROCJPEG_STATUS_EXECUTION_FAILED;
  (void)hipSetDevice(prev);
  if (st != ROCJPEG_STATUS_SUCCESS) return st;
  if (c->rank != 0 && hash != want) return ROCJPEG_STATUS_EXECUTION_FAILED;
  if (!own_ok || (c->rank != 0 && total != uint32_t(count))) return ROCJPEG_STATUS_INVALID_PARAMETER;
  return ROCJPEG_STATUS_SUCCESS;
}
}  // namespace

// rank 0's `count` records -> every rank (each passes the same count)
RJ_EXPORT RocJpegStatus rocJpegAmdBroadcastWorkTable(RocJpegAmdComm c, RocJpegAmdWorkItem *items, int count) {
  if (c == nullptr) return ROCJPEG_STATUS_INVALID_PARAMETER;
  try {
    RocJpegStatus st0 = ROCJPEG_STATUS_SUCCESS;
    const RocJpegStatus st = BroadcastWithStatus(c, items, count, ROCJPEG_STATUS_SUCCESS, &st0);
    return st != ROCJPEG_STATUS_SUCCESS ? st : st0;
  } catch (const std::bad_alloc &) {
    return ROCJPEG_STATUS_OUTOF_MEMORY;  // only the host scratch can throw, before any collective
  } catch (...) {
    return ROCJPEG_STATUS_RUNTIME_ERROR;
  }
}

namespace {
// rank 0: table + LPT over the ranks (shard = rank); then the broadcast with rank 0's status.
// Every rank returns rank 0's plan status when that failed.
RocJpegStatus PlanAndBroadcast(RocJpegAmdCommImpl *c, const unsigned char *blob, uint64_t blob_bytes,
                               const uint64_t *offsets, const uint32_t *sizes, int count, RocJpegAmdWorkItem *items,
                               bool local_ok) {
  RocJpegStatus plan = local_ok ? ROCJPEG_STATUS_SUCCESS : ROCJPEG_STATUS_INVALID_PARAMETER;
  if (c->rank == 0 && plan == ROCJPEG_STATUS_SUCCESS) {
    plan = rocJpegAmdBuildWorkTable(blob, blob_bytes, offsets, sizes, count, items);
    if (plan == ROCJPEG_STATUS_SUCCESS) plan = rocJpegAmdAssignShards(items, count, c->nranks, nullptr, nullptr);
    if (plan != ROCJPEG_STATUS_SUCCESS) {  // a table that assigns nothing goes out with the status
      for (int i = 0; i < count; i++) {
        std::memset(items + i, 0, sizeof(RocJpegAmdWorkItem));
        items[i].shard = -1;
        items[i].index = uint32_t(i);
      }
    }
  }
  RocJpegStatus st0 = plan;
  const RocJpegStatus st = BroadcastWithStatus(c, local_ok ? items : nullptr, local_ok ? count : 0, plan, &st0);
  if (st != ROCJPEG_STATUS_SUCCESS && st != ROCJPEG_STATUS_INVALID_PARAMETER) return st;  // the exchange failed
  if (st0 != ROCJPEG_STATUS_SUCCESS) return st0;  // rank 0's plan failed: every rank reports it
  return local_ok ? st : ROCJPEG_STATUS_INVALID_PARAMETER;
}

bool BlobArgsOk(const unsigned char *blob, const uint64_t *offsets, const uint32_t *sizes, int count,
                const RocJpegAmdWorkItem *items) {
  return count >= 0 && (count == 0 || (blob != nullptr && offsets != nullptr && sizes != nullptr && items != nullptr));
}
}  // namespace

RJ_EXPORT RocJpegStatus rocJpegAmdShardPlan(RocJpegAmdComm c, const unsigned char *blob, uint64_t blob_bytes,
                                            const uint64_t *offsets, const uint32_t *sizes, int count,
                                            RocJpegAmdWorkItem *items) {
  if (c == nullptr) return ROCJPEG_STATUS_INVALID_PARAMETER;
  try {
    // only rank 0 reads the blob; the other ranks receive into items
    const bool ok = c->rank == 0 ? BlobArgsOk(blob, offsets, sizes, count, items)
                                 : (count >= 0 && (count == 0 || items != nullptr));
    return PlanAndBroadcast(c, blob, blob_bytes, offsets, sizes, count, items, ok);
  } catch (const std::bad_alloc &) {
    return ROCJPEG_STATUS_OUTOF_MEMORY;
  } catch (...) {
    return ROCJPEG_STATUS_RUNTIME_ERROR;
  }
}

// A rank's share of a sharded batch, kept resident: its images' stream handles (parsed by the
// GPU marker scan, bitstreams and interval tables in the handle's HBM) and their batch indices.
struct RocJpegAmdShardImpl {
  RocJpegHandle handle = nullptr;
  int count = 0;                              // images of the whole batch
  std::vector<int> index;                     // this rank's images, batch order
  std::vector<RocJpegStreamHandle> streams;   // one per entry of index
  std::vector<RocJpegImage> dst;              // per-call destination scratch
  ~RocJpegAmdShardImpl() {
    for (RocJpegStreamHandle s : streams)
      if (s) (void)rocJpegStreamDestroy(s);
  }
};

namespace {
// this rank's images of the broadcast table, parsed (GPU marker scan) and resident
RocJpegStatus MakeShard(RocJpegHandle handle, RocJpegAmdCommImpl *c, const unsigned char *blob, uint64_t blob_bytes,
                        const uint64_t *offsets, const uint32_t *sizes, int count, const RocJpegAmdWorkItem *tab,
                        RocJpegAmdShardImpl *sh) {
  sh->handle = handle;
  sh->count = count;
  for (int i = 0; i < count; i++)
    if (tab[i].shard == c->rank) sh->index.push_back(int(tab[i].index));
  for (int i : sh->index)  // the table comes from rank 0: check its indices against this rank's view
    if (i < 0 || i >= count || offsets[i] > blob_bytes || sizes[i] > blob_bytes - offsets[i])
      return ROCJPEG_STATUS_RUNTIME_ERROR;
  const size_t n = sh->index.size();
  sh->streams.assign(n, nullptr);
  sh->dst.resize(n);
  std::vector<const unsigned char *> data(n);
  std::vector<size_t> len(n);
  for (size_t k = 0; k < n; k++) {
    const RocJpegStatus st = rocJpegStreamCreate(&sh->streams[k]);
    if (st != ROCJPEG_STATUS_SUCCESS) return st;
    data[k] = blob + offsets[sh->index[k]];
    len[k] = sizes[sh->index[k]];
  }
  if (n == 0) return ROCJPEG_STATUS_SUCCESS;
  // the O(bytes) part of the parse on the GPU; bitstreams stay resident in this handle's HBM
  RocJpegStatus st = rocJpegAmdStreamParseDevice(handle, data.data(), len.data(), int(n), sh->streams.data());
  // progressive streams are parsed on the host by that call: make them resident as well
  if (st == ROCJPEG_STATUS_SUCCESS) st = rocJpegAmdStreamsToDevice(handle, sh->streams.data(), int(n));
  return st;
}

RocJpegStatus DecodeShard(RocJpegAmdShardImpl *sh, const RocJpegDecodeParams *params, RocJpegImage *destinations) {
  const size_t n = sh->index.size();
  if (n == 0) return ROCJPEG_STATUS_SUCCESS;
  for (size_t k = 0; k < n; k++) sh->dst[k] = destinations[sh->index[k]];
  return rocJpegDecodeBatched(sh->handle, sh->streams.data(), int(n), params, sh->dst.data());
}
}  // namespace

RJ_EXPORT RocJpegStatus rocJpegAmdShardCreate(RocJpegHandle handle, RocJpegAmdComm c, const unsigned char *blob,
                                              uint64_t blob_bytes, const uint64_t *offsets, const uint32_t *sizes,
                                              int count, RocJpegAmdWorkItem *items, RocJpegAmdShard *shard) {
  if (c == nullptr) return ROCJPEG_STATUS_INVALID_PARAMETER;
  if (shard) *shard = nullptr;
  try {
    std::vector<RocJpegAmdWorkItem> own;
    RocJpegAmdWorkItem *tab = items;
    if (tab == nullptr && count > 0) {
      own.resize(size_t(count));
      tab = own.data();
    }
    // every rank reads its own images from the blob: each checks its arguments, and a rank with
    // bad ones still takes part in the broadcast before it returns INVALID_PARAMETER
    const bool ok = handle != nullptr && shard != nullptr && BlobArgsOk(blob, offsets, sizes, count, count ? tab : nullptr);
    RocJpegStatus st = PlanAndBroadcast(c, blob, blob_bytes, offsets, sizes, count, tab, ok);
    if (st != ROCJPEG_STATUS_SUCCESS) return st;
    auto *sh = new RocJpegAmdShardImpl;
    st = MakeShard(handle, c, blob, blob_bytes, offsets, sizes, count, tab, sh);
    if (st != ROCJPEG_STATUS_SUCCESS) {
      delete sh;
      return st;
    }
    *shard = sh;
    return ROCJPEG_STATUS_SUCCESS;
  } catch (const std::bad_alloc &) {
    return ROCJPEG_STATUS_OUTOF_MEMORY;
  } catch (...) {
    return ROCJPEG_STATUS_RUNTIME_ERROR;
  }
}

RJ_EXPORT RocJpegStatus rocJpegAmdShardDecode(RocJpegAmdShard shard, const RocJpegDecodeParams *params,
                                              RocJpegImage *destinations) {
  if (shard == nullptr || params == nullptr || (shard->count > 0 && destinations == nullptr))
    return ROCJPEG_STATUS_INVALID_PARAMETER;
  try {
    return DecodeShard(shard, params, destinations);
  } catch (const std::bad_alloc &) {
    return ROCJPEG_STATUS_OUTOF_MEMORY;
  } catch (...) {
    return ROCJPEG_STATUS_RUNTIME_ERROR;
  }
}

RJ_EXPORT RocJpegStatus rocJpegAmdShardGetImages(RocJpegAmdShard shard, int *num_images, int *indices, int capacity) {
  if (shard == nullptr || num_images == nullptr || capacity < 0) return ROCJPEG_STATUS_INVALID_PARAMETER;
  *num_images = int(shard->index.size());
  for (int k = 0; indices != nullptr && k < capacity && k < int(shard->index.size()); k++) indices[k] = shard->index[k];
  return ROCJPEG_STATUS_SUCCESS;
}

RJ_EXPORT RocJpegStatus rocJpegAmdShardDestroy(RocJpegAmdShard shard) {
  if (shard == nullptr) return ROCJPEG_STATUS_INVALID_PARAMETER;
  delete shard;
  return ROCJPEG_STATUS_SUCCESS;
}

// One call: rocJpegAmdShardCreate + rocJpegAmdShardDecode + rocJpegAmdShardDestroy
// (src/rocjpeg_decoder.cpp:196-292 semantics per rank).  destinations: `count` entries in batch
// order; only this rank's images are written.  items (optional, `count` records): the broadcast
// table, so the caller knows where each image was decoded.  Parse failures of this rank's images
// return BAD_JPEG before any decode, as the reference's rocJpegStreamParse would have.
RJ_EXPORT RocJpegStatus rocJpegAmdDecodeBatchedSharded(RocJpegHandle handle, RocJpegAmdComm c,
                                                       const unsigned char *blob, uint64_t blob_bytes,
                                                       const uint64_t *offsets, const uint32_t *sizes, int count,
                                                       const RocJpegDecodeParams *params,
                                                       RocJpegImage *destinations, RocJpegAmdWorkItem *items) {
  if (c == nullptr) return ROCJPEG_STATUS_INVALID_PARAMETER;
  // arguments only this rank uses are checked after the collective (rocJpegAmdShardCreate joins
  // it on every path)
  const bool local_ok = params != nullptr && (count <= 0 || destinations != nullptr);
  RocJpegAmdShard sh = nullptr;
  RocJpegStatus st = rocJpegAmdShardCreate(local_ok ? handle : nullptr, c, blob, blob_bytes, offsets, sizes, count,
                                           items, &sh);
  if (st != ROCJPEG_STATUS_SUCCESS) return st;
  st = rocJpegAmdShardDecode(sh, params, destinations);
  (void)rocJpegAmdShardDestroy(sh);
  return st;
}

RJ_EXPORT RocJpegStatus rocJpegAmdGetAbiVersion(int *version) {
  if (version == nullptr) return ROCJPEG_STATUS_INVALID_PARAMETER;
  *version = ROCJPEG_AMD_ABI_VERSION;
  return ROCJPEG_STATUS_SUCCESS;
}
