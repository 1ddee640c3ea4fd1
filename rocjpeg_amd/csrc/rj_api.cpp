// rj_api.cpp -- the C ABI (include/rocjpeg.h, include/rocjpeg_amd.h).
//
// Mirrors the reference shim src/rocjpeg_api.cpp:38-277: NULL arguments ->
// ROCJPEG_STATUS_INVALID_PARAMETER, parse failure -> ROCJPEG_STATUS_BAD_JPEG, allocation
// failure at create -> ROCJPEG_STATUS_NOT_INITIALIZED, any C++ exception ->
// ROCJPEG_STATUS_RUNTIME_ERROR.  No exception crosses the ABI.
#include <cstring>
#include <exception>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/rocjpeg.h"
#include "../../include/rocjpeg_amd.h"
#include "rj_coalesce.h"
#include "rj_common.h"
#include "rj_decoder.h"
#include "rj_stream.h"

#define RJ_EXPORT extern "C" __attribute__((visibility("default")))

namespace {

struct DecoderHandle {
  explicit DecoderHandle(RocJpegBackend b, int dev) : decoder(b, dev) {}
  rj::Decoder decoder;
};

template <typename F>
RocJpegStatus Guard(F &&f) {
  try {
    return RocJpegStatus(f());
  } catch (const std::bad_alloc &e) {
    RJ_ERR("out of memory: %s", e.what());
    return ROCJPEG_STATUS_OUTOF_MEMORY;
  } catch (const std::exception &e) {
    RJ_ERR("%s", e.what());
    return ROCJPEG_STATUS_RUNTIME_ERROR;
  } catch (...) {
    return ROCJPEG_STATUS_RUNTIME_ERROR;
  }
}

inline rj::Stream *AsStream(RocJpegStreamHandle h) { return static_cast<rj::Stream *>(h); }
inline rj::Decoder *AsDecoder(RocJpegHandle h) { return &static_cast<DecoderHandle *>(h)->decoder; }

}  // namespace

// rocjpeg_api.cpp:38-52
RJ_EXPORT RocJpegStatus rocJpegStreamCreate(RocJpegStreamHandle *jpeg_stream_handle) {
  if (jpeg_stream_handle == nullptr) return ROCJPEG_STATUS_INVALID_PARAMETER;
  rj::Stream *s = new (std::nothrow) rj::Stream();
  if (s == nullptr) return ROCJPEG_STATUS_NOT_INITIALIZED;
  *jpeg_stream_handle = s;
  return ROCJPEG_STATUS_SUCCESS;
}

// rocjpeg_api.cpp:68-77
RJ_EXPORT RocJpegStatus rocJpegStreamParse(const unsigned char *data, size_t length, RocJpegStreamHandle h) {
  if (data == nullptr || h == nullptr) return ROCJPEG_STATUS_INVALID_PARAMETER;
  return Guard([&] {
    if (length > 0xFFFFFFFFull) return int(ROCJPEG_STATUS_BAD_JPEG);
    return AsStream(h)->Parse(data, uint32_t(length)) ? int(ROCJPEG_STATUS_SUCCESS) : int(ROCJPEG_STATUS_BAD_JPEG);
  });
}

// rocjpeg_api.cpp:86-93
RJ_EXPORT RocJpegStatus rocJpegStreamDestroy(RocJpegStreamHandle h) {
  if (h == nullptr) return ROCJPEG_STATUS_INVALID_PARAMETER;
  delete AsStream(h);
  return ROCJPEG_STATUS_SUCCESS;
}

// rocjpeg_api.cpp:107-120
RJ_EXPORT RocJpegStatus rocJpegCreate(RocJpegBackend backend, int device_id, RocJpegHandle *handle) {
  if (handle == nullptr) return ROCJPEG_STATUS_INVALID_PARAMETER;
  DecoderHandle *d = new (std::nothrow) DecoderHandle(backend, device_id);
  if (d == nullptr) return ROCJPEG_STATUS_NOT_INITIALIZED;
  *handle = d;
  return Guard([&] { return d->decoder.Initialize(); });
}

// rocjpeg_api.cpp:132-139
RJ_EXPORT RocJpegStatus rocJpegDestroy(RocJpegHandle handle) {
  if (handle == nullptr) return ROCJPEG_STATUS_INVALID_PARAMETER;
  delete static_cast<DecoderHandle *>(handle);
  return ROCJPEG_STATUS_SUCCESS;
}

// rocjpeg_api.cpp:160-177
RJ_EXPORT RocJpegStatus rocJpegGetImageInfo(RocJpegHandle handle, RocJpegStreamHandle s, uint8_t *num_components,
                                            RocJpegChromaSubsampling *subsampling, uint32_t *widths,
                                            uint32_t *heights) {
  if (handle == nullptr || num_components == nullptr || subsampling == nullptr || widths == nullptr ||
      heights == nullptr)
    return ROCJPEG_STATUS_INVALID_PARAMETER;
  return Guard([&] { return AsDecoder(handle)->GetImageInfo(AsStream(s), num_components, subsampling, widths, heights); });
}

// rocjpeg_api.cpp:192-209
RJ_EXPORT RocJpegStatus rocJpegDecode(RocJpegHandle handle, RocJpegStreamHandle s, const RocJpegDecodeParams *params,
                                      RocJpegImage *destination) {
  if (handle == nullptr || params == nullptr || destination == nullptr) return ROCJPEG_STATUS_INVALID_PARAMETER;
  if (s == nullptr) return ROCJPEG_STATUS_INVALID_PARAMETER;  // rocjpeg_decoder.cpp:107-109
  return Guard([&] {
    rj::Stream *st = AsStream(s);
    rj::Decoder *d = AsDecoder(handle);
    return rj::CoalescedDecode(d, d->device(), &st, 1, params, destination);
  });
}

// rocjpeg_api.cpp:222-237
RJ_EXPORT RocJpegStatus rocJpegDecodeBatched(RocJpegHandle handle, RocJpegStreamHandle *streams, int batch_size,
                                             const RocJpegDecodeParams *params, RocJpegImage *destinations) {
  if (handle == nullptr || streams == nullptr || params == nullptr || destinations == nullptr)
    return ROCJPEG_STATUS_INVALID_PARAMETER;
  if (batch_size < 0) return ROCJPEG_STATUS_INVALID_PARAMETER;
  return Guard([&] {
    std::vector<rj::Stream *> v(static_cast<size_t>(batch_size));
    for (int i = 0; i < batch_size; i++) v[i] = AsStream(streams[i]);
    rj::Decoder *d = AsDecoder(handle);
    return rj::CoalescedDecode(d, d->device(), v.data(), batch_size, params, destinations);
  });
}

// rocjpeg_api.cpp:246-277
RJ_EXPORT const char *rocJpegGetErrorName(RocJpegStatus status) {
  switch (status) {
    case ROCJPEG_STATUS_SUCCESS: return "ROCJPEG_STATUS_SUCCESS";
    case ROCJPEG_STATUS_NOT_INITIALIZED: return "ROCJPEG_STATUS_NOT_INITIALIZED";
    case ROCJPEG_STATUS_INVALID_PARAMETER: return "ROCJPEG_STATUS_INVALID_PARAMETER";
    case ROCJPEG_STATUS_BAD_JPEG: return "ROCJPEG_STATUS_BAD_JPEG";
    case ROCJPEG_STATUS_JPEG_NOT_SUPPORTED: return "ROCJPEG_STATUS_JPEG_NOT_SUPPORTED";
    case ROCJPEG_STATUS_EXECUTION_FAILED: return "ROCJPEG_STATUS_EXECUTION_FAILED";
    case ROCJPEG_STATUS_ARCH_MISMATCH: return "ROCJPEG_STATUS_ARCH_MISMATCH";
    case ROCJPEG_STATUS_INTERNAL_ERROR: return "ROCJPEG_STATUS_INTERNAL_ERROR";
    case ROCJPEG_STATUS_IMPLEMENTATION_NOT_SUPPORTED: return "ROCJPEG_STATUS_IMPLEMENTATION_NOT_SUPPORTED";
    case ROCJPEG_STATUS_HW_JPEG_DECODER_NOT_SUPPORTED: return "ROCJPEG_STATUS_HW_JPEG_DECODER_NOT_SUPPORTED";
    case ROCJPEG_STATUS_RUNTIME_ERROR: return "ROCJPEG_STATUS_RUNTIME_ERROR";
    case ROCJPEG_STATUS_OUTOF_MEMORY: return "ROCJPEG_STATUS_OUTOF_MEMORY";
    case ROCJPEG_STATUS_NOT_IMPLEMENTED: return "ROCJPEG_STATUS_NOT_IMPLEMENTED";
    default: return "UNKNOWN_ERROR";
  }
}

// ---------------------------------------------------------------- extensions (rocjpeg_amd.h)
RJ_EXPORT RocJpegStatus rocJpegAmdStreamGetInfo(RocJpegStreamHandle s, uint8_t *nc, RocJpegChromaSubsampling *css,
                                                uint32_t *widths, uint32_t *heights, uint32_t *nintervals) {
  if (s == nullptr || nc == nullptr || css == nullptr || widths == nullptr || heights == nullptr)
    return ROCJPEG_STATUS_INVALID_PARAMETER;
  return Guard([&] {
    rj::Stream *st = AsStream(s);
    std::lock_guard<std::mutex> lock(st->mutex());
    int c = -1;
    const int r = rj::ImageInfo(st->info(), nc, &c, widths, heights);
    *css = RocJpegChromaSubsampling(c);
    if (nintervals) *nintervals = uint32_t(st->plan().progressive ? st->plan().pivals.size() : st->plan().segs.size());
    return r;
  });
}

RJ_EXPORT RocJpegStatus rocJpegAmdStreamsToDevice(RocJpegHandle handle, RocJpegStreamHandle *streams, int count) {
  if (handle == nullptr || streams == nullptr || count < 0) return ROCJPEG_STATUS_INVALID_PARAMETER;
  return Guard([&] {
    std::vector<rj::Stream *> v(static_cast<size_t>(count));
    for (int i = 0; i < count; i++) v[i] = AsStream(streams[i]);
    return AsDecoder(handle)->StreamsToDevice(v.data(), count);
  });
}

RJ_EXPORT RocJpegStatus rocJpegAmdStreamParseDevice(RocJpegHandle handle, const unsigned char *const *data,
                                                    const size_t *lengths, int count, RocJpegStreamHandle *streams) {
  if (handle == nullptr || data == nullptr || lengths == nullptr || streams == nullptr || count < 0)
    return ROCJPEG_STATUS_INVALID_PARAMETER;
  return Guard([&] {
    std::vector<rj::Stream *> v(static_cast<size_t>(count));
    for (int i = 0; i < count; i++) {
      if (streams[i] == nullptr) return int(ROCJPEG_STATUS_INVALID_PARAMETER);
      v[i] = AsStream(streams[i]);
    }
    return AsDecoder(handle)->ParseOnDevice(v.data(), data, lengths, count);
  });
}

RJ_EXPORT RocJpegStatus rocJpegAmdStreamGetIntervals(RocJpegStreamHandle s, RocJpegAmdInterval *out, uint32_t capacity,
                                                     uint32_t *count) {
  if (s == nullptr || count == nullptr) return ROCJPEG_STATUS_INVALID_PARAMETER;
  return Guard([&] {
    rj::Stream *st = AsStream(s);
    std::lock_guard<std::mutex> lock(st->mutex());
    const rj::DecodePlan &p = st->plan();
    *count = uint32_t(p.segs.size());
    for (uint32_t i = 0; out != nullptr && i < capacity && i < p.segs.size(); i++) {
      const RjSegDev &g = p.segs[i];
      out[i] = RocJpegAmdInterval{g.src_off, g.src_len, g.dst_off, g.dst_len, g.mcu_first, g.mcu_count, g.flags,
                                  g.ent_off, g.chunk0, 0u};
    }
    return int(ROCJPEG_STATUS_SUCCESS);
  });
}

RJ_EXPORT RocJpegStatus rocJpegAmdStreamGetDestuffBlocks(RocJpegStreamHandle s, uint32_t *out4, uint32_t capacity,
                                                         uint32_t *count, uint32_t *ecs_size) {
  if (s == nullptr || count == nullptr) return ROCJPEG_STATUS_INVALID_PARAMETER;
  return Guard([&] {
    rj::Stream *st = AsStream(s);
    std::lock_guard<std::mutex> lock(st->mutex());
    const rj::DecodePlan &p = st->plan();
    *count = uint32_t(p.ds.size());
    if (ecs_size) *ecs_size = st->info().ecs_size;
    for (uint32_t i = 0; out4 != nullptr && i < capacity && i < p.ds.size(); i++) {
      out4[4 * i] = p.ds[i].src_off;
      out4[4 * i + 1] = p.ds[i].len;
      out4[4 * i + 2] = p.ds[i].dst_off;
      out4[4 * i + 3] = p.ds[i].zero_end;
    }
    return int(ROCJPEG_STATUS_SUCCESS);
  });
}

RJ_EXPORT RocJpegStatus rocJpegAmdSetProfiling(RocJpegHandle handle, int enable) {
  if (handle == nullptr) return ROCJPEG_STATUS_INVALID_PARAMETER;
  AsDecoder(handle)->SetProfiling(enable != 0);
  return ROCJPEG_STATUS_SUCCESS;
}

RJ_EXPORT RocJpegStatus rocJpegAmdGetLastTimings(RocJpegHandle handle, RocJpegAmdTimings *t) {
  if (handle == nullptr || t == nullptr) return ROCJPEG_STATUS_INVALID_PARAMETER;
  *t = AsDecoder(handle)->last_timings();
  return ROCJPEG_STATUS_SUCCESS;
}

RJ_EXPORT RocJpegStatus rocJpegAmdSetPathPolicy(RocJpegHandle handle, int policy) {
  if (handle == nullptr || policy < 0 || policy > 1) return ROCJPEG_STATUS_INVALID_PARAMETER;
  AsDecoder(handle)->SetPathPolicy(policy);
  return ROCJPEG_STATUS_SUCCESS;
}

RJ_EXPORT RocJpegStatus rocJpegAmdGetStream(RocJpegHandle handle, void **hip_stream) {
  if (handle == nullptr || hip_stream == nullptr) return ROCJPEG_STATUS_INVALID_PARAMETER;
  *hip_stream = AsDecoder(handle)->stream();
  return ROCJPEG_STATUS_SUCCESS;
}

RJ_EXPORT RocJpegStatus rocJpegAmdStreamGetLeanTables(RocJpegStreamHandle s, void *out, size_t bytes, size_t *needed) {
  if (s == nullptr || needed == nullptr) return ROCJPEG_STATUS_INVALID_PARAMETER;
  return Guard([&] {
    rj::Stream *st = AsStream(s);
    std::lock_guard<std::mutex> lock(st->mutex());
    *needed = sizeof(RjLeanTables);
    if (st->plan().progressive || st->plan().status != 0) return int(ROCJPEG_STATUS_JPEG_NOT_SUPPORTED);
    if (out != nullptr && bytes >= sizeof(RjLeanTables)) std::memcpy(out, st->LeanTables(), sizeof(RjLeanTables));
    return int(ROCJPEG_STATUS_SUCCESS);
  });
}

RJ_EXPORT RocJpegStatus rocJpegAmdGetCoalesceStats(uint64_t *calls, uint64_t *combined, uint64_t *combined_members) {
  rj::CoalesceStats(calls, combined, combined_members);
  return ROCJPEG_STATUS_SUCCESS;
}

RJ_EXPORT RocJpegStatus rocJpegAmdGetLastParseTimings(RocJpegHandle handle, double *ms, int count) {
  if (handle == nullptr || ms == nullptr || count < 0) return ROCJPEG_STATUS_INVALID_PARAMETER;
  double t[6];
  AsDecoder(handle)->last_scan_ms(t);
  for (int i = 0; i < count && i < 6; i++) ms[i] = t[i];
  return ROCJPEG_STATUS_SUCCESS;
}
