// rj_decoder.cpp -- batch planner + launch sequence (see rj_decoder.h).
#include "rj_decoder.h"

#include <sched.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <thread>

#include "rj_common.h"
#include "rj_kernels.h"

namespace rj {

namespace {

inline uint64_t AlignUp(uint64_t v, uint64_t a) { return (v + a - 1) / a * a; }

// Can the fused kernel (rj_fused.hip) produce exactly what the reference semantics ask for?
// It handles the whole-image output window of RGB / RGB_PLANAR / Y / YUV_PLANAR for the
// canonical sampling geometry of each subsampling class.  ROI crops (with the reference's
// offset quirks), NATIVE layouts and "pitch > width" copies go to the general path.
bool FusedEligible(const StreamInfo &in, const DecodePlan &p, int fmt, bool roi, const RocJpegImage &o) {
  if (roi) return false;
  if (!(fmt == ROCJPEG_OUTPUT_RGB || fmt == ROCJPEG_OUTPUT_RGB_PLANAR || fmt == ROCJPEG_OUTPUT_Y ||
        fmt == ROCJPEG_OUTPUT_YUV_PLANAR))
    return false;
  const int css = in.css;
  if (in.ncomp == 1) {
    if (css != kCss400) return false;
  } else {
    if (in.ncomp != 3) return false;
    if (in.comp[0].h != p.hmax || in.comp[0].v != p.vmax) return false;
    if (in.comp[1].h != in.comp[2].h || in.comp[1].v != in.comp[2].v) return false;
    const int rh = p.hmax / in.comp[1].h, rv = p.vmax / in.comp[1].v;
    if (p.hmax % in.comp[1].h || p.vmax % in.comp[1].v || rh > 2 || rv > 2) return false;
    const bool ok = (css == kCss444 && rh == 1 && rv == 1) || (css == kCss440 && rh == 1 && rv == 2) ||
                    (css == kCss422 && rh == 2 && rv == 1) || (css == kCss420 && rh == 2 && rv == 2);
    if (!ok) return false;
  }
  const uint32_t W = in.width;
  for (int c = 0; c < 4; c++)  // k_fused addresses the destination with 32-bit offsets
    if (o.pitch[c] >= (1u << 24) || uint64_t(o.pitch[c]) * (p.mcuy * 8u * p.vmax) >= (1ull << 31)) return false;
  if (p.nblk_mcu == 0 || rj_fused_strip_mcus(p.hmax, p.nblk_mcu) == 0) return false;  // strip limits of k_fused
  // copy-type channels write `pitch` bytes per row in the reference: only pitch == width is fused
  if ((fmt == ROCJPEG_OUTPUT_Y || fmt == ROCJPEG_OUTPUT_YUV_PLANAR) && css != kCss422 && o.pitch[0] != W) return false;
  if (fmt == ROCJPEG_OUTPUT_YUV_PLANAR && in.ncomp == 3) {
    if (css == kCss444 || css == kCss440) {
      if (o.pitch[1] != W || o.pitch[2] != W) return false;
    }
  }
  return true;
}

}  // namespace

int Decoder::HostThreads() {
  if (const char *v = getenv("RJ_HOST_THREADS"))
    if (atoi(v) > 0) return std::min(64, atoi(v));
  // 8: on the GPU box (a 16-CPU share) 4-8 staging threads beat 16-32 (the copies then compete
  // with the caller's own threads for the share; tools/host_input.py)
  return int(std::min(8u, std::max(1u, std::thread::hardware_concurrency())));
}

int DeviceBuffer::Ensure(size_t bytes) {
  if (bytes <= cap_) return kOk;
  Release();
  const size_t want = std::max<size_t>(AlignUp(bytes + bytes / 4, 1 << 20), 1 << 20);
  if (hipMalloc(&ptr_, want) != hipSuccess) {
    ptr_ = nullptr;
    (void)hipGetLastError();
    return kOutOfMemory;
  }
  cap_ = want;
  return kOk;
}

void DeviceBuffer::Release() {
  if (ptr_) (void)hipFree(ptr_);
  ptr_ = nullptr;
  cap_ = 0;
}

int PinnedBuffer::Ensure(size_t bytes) {
  if (bytes <= cap_) return kOk;
  Release();
  const size_t want = std::max<size_t>(AlignUp(bytes + bytes / 4, 1 << 20), 1 << 20);
  if (hipHostMalloc(&ptr_, want, hipHostMallocNonCoherent) != hipSuccess) {
    ptr_ = nullptr;
    (void)hipGetLastError();
    return kOutOfMemory;
  }
  cap_ = want;
  return kOk;
}

void PinnedBuffer::Release() {
  if (ptr_) (void)hipHostFree(ptr_);
  ptr_ = nullptr;
  cap_ = 0;
}

Decoder::~Decoder() {
  if (stream_) {
    (void)hipSetDevice(device_);
    (void)hipStreamSynchronize(stream_);
    for (auto &e : ev_)
      if (e) (void)hipEventDestroy(e);
    for (auto &e : pev_)
      if (e) (void)hipEventDestroy(e);
    for (auto &e : pk1_)
      if (e) (void)hipEventDestroy(e);
    for (auto &e : kev_)
      if (e) (void)hipEventDestroy(e);
    for (auto &e : prog_ev_)
      if (e) (void)hipEventDestroy(e);
    for (auto &e : prog_join_)
      if (e) (void)hipEventDestroy(e);
    for (auto &e : prog_lev_ev_) (void)hipEventDestroy(e);
    for (auto &e : pk_ev_) (void)hipEventDestroy(e);
    for (auto *arr : {k1s_, k2s_, k2e_})
      for (int q = 0; q < kMaxPipe; q++)
        if (arr[q]) (void)hipEventDestroy(arr[q]);
    for (auto &q : pstream_)
      if (q) (void)hipStreamDestroy(q);
    for (auto &e : live_ev_)
      if (e) (void)hipEventDestroy(e);
    for (auto &e : live_t_)
      if (e) (void)hipEventDestroy(e);
    if (split_ev_) (void)hipEventDestroy(split_ev_);
    if (bev_) (void)hipEventDestroy(bev_);
    if (kfork_ev_) (void)hipEventDestroy(kfork_ev_);
    if (kjoin_ev_) (void)hipEventDestroy(kjoin_ev_);
    for (auto &e : place_ev_)
      if (e) (void)hipEventDestroy(e);
    if (bstream_) (void)hipStreamDestroy(bstream_);
    if (lstream_) (void)hipStreamDestroy(lstream_);
    (void)hipStreamDestroy(stream_);
  }
  if (h_wide_flag_) (void)hipHostFree(h_wide_flag_);
}

int Decoder::Initialize() {
  // InitHIP (rocjpeg_decoder.cpp:46-61)
  int count = 0;
  RJ_HIP(hipGetDeviceCount(&count));
  if (count < 1) {
    RJ_ERR("no GPU found");
    return kNotInitialized;
  }
  if (device_ >= count) {
    RJ_ERR("device %d not found (%d devices)", device_, count);
    return kInvalidParameter;
  }
  RJ_HIP(hipSetDevice(device_));
  hipDeviceProp_t prop;
  RJ_HIP(hipGetDeviceProperties(&prop, device_));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    RJ_ERR("device %d is %s; this build carries gfx950 (MI355X) kernels only", device_, prop.gcnArchName);
    return -7;  // ROCJPEG_STATUS_ARCH_MISMATCH
  }
  RJ_HIP(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
  for (auto &e : ev_) RJ_HIP(hipEventCreate(&e));
  if (const char *g = getenv("RJ_PIPE_GROUPS")) {
    pipe_groups_ = std::max(1, std::min(kMaxPipe, atoi(g)));
    pipe_groups_set_ = true;
  }
  if (const char *m = getenv("RJ_PIPE_MIN")) pipe_min_ = uint32_t(std::max(1, atoi(m)));
  if (const char *o = getenv("RJ_SORT_LANES")) sort_lanes_ = atoi(o) != 0;
  if (const char *l = getenv("RJ_LPT")) lpt_ = atoi(l) != 0;
  if (const char *l = getenv("RJ_K1_SOLO")) k1_solo_lds_ = uint32_t(std::max(0, atoi(l)));
  if (const char *so = getenv("RJ_SPLIT_OUTLIERS")) outlier_split_ = atoi(so) != 0;
  if (const char *f5 = getenv("RJ_K1_FIVE")) five_waves_ = atoi(f5);
  if (const char *t5 = getenv("RJ_K1_SPLIT5_T")) split5_t_ = atof(t5);
  if (const char *kc = getenv("RJ_K1_CHUNK")) k1_chunk_ = atoi(kc) != 0;
  if (const char *cm = getenv("RJ_CHUNK_MIN")) chunk_min_ = uint32_t(std::max(16, atoi(cm)));
  if (const char *hy = getenv("RJ_K1_HYP")) hyp_max_ = uint32_t(std::max(1, atoi(hy)));
  if (const char *hw = getenv("RJ_K1_HYP_WARM")) hyp_warm_ = atoi(hw) != 0;
  if (const char *hc = getenv("RJ_K1_HYP_CHUNK_MIN")) hyp_chunk_min_ = uint32_t(std::max(16, atoi(hc))) & ~15u;
  if (const char *sf = getenv("RJ_SPLIT_OUTLIER_FRAC")) outlier_frac_ = atof(sf);
  if (const char *st = getenv("RJ_SPLIT_OUTLIER_T")) outlier_t_ = std::max(0.5, std::min(1.0, atof(st)));
  cu_count_ = std::max(1, prop.multiProcessorCount);
  RJ_HIP(hipHostMalloc(reinterpret_cast<void **>(&h_wide_flag_), 64, hipHostMallocMapped | hipHostMallocCoherent));
  RJ_HIP(hipHostGetDevicePointer(reinterpret_cast<void **>(&d_wide_flag_), h_wide_flag_, 0));
  *reinterpret_cast<volatile uint32_t *>(h_wide_flag_) = 0;
  // (the side streams -- pstream_, lstream_, bstream_ -- are created on first use: streams take
  // the process's hardware queues round-robin at creation, and DecodeSplit's part handles each
  // need a queue of their own for their stream_; unused side streams would push them onto shared ones)
  for (auto &e : live_ev_) RJ_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  for (auto &e : live_t_) RJ_HIP(hipEventCreate(&e));
  RJ_HIP(hipEventCreateWithFlags(&split_ev_, hipEventDisableTiming));
  RJ_HIP(hipEventCreateWithFlags(&bev_, hipEventDisableTiming));
  if (const char *sp = getenv("RJ_SYNC_SPIN")) spin_sync_ = atoi(sp) != 0;
  if (const char *kl = getenv("RJ_K0_LDS")) k0_lds_ = atoi(kl) != 0;
  if (const char *kl2 = getenv("RJ_K2_LPT")) k2_lpt_ = atoi(kl2) != 0;
  if (const char *sp2 = getenv("RJ_SORT_PAR")) sort_par_ = atoi(sp2) != 0;
  if (const char *ks = getenv("RJ_K2_SPLIT_SIDE")) k2_split_side_ = atoi(ks) != 0;
  RJ_HIP(hipEventCreateWithFlags(&kfork_ev_, hipEventDisableTiming));
  RJ_HIP(hipEventCreateWithFlags(&kjoin_ev_, hipEventDisableTiming));
  for (auto &e : place_ev_) RJ_HIP(hipEventCreate(&e));
  if (const char *pt = getenv("RJ_PLACE_TUNE")) place_tune_ = atoi(pt) != 0;
  if (const char *pk = getenv("RJ_PLACE_KEEP")) place_keep_ = atoi(pk) != 0;
  if (const char *pc = getenv("RJ_PLACE_CANDS")) place_cands_ = std::max(1, std::min(kPlaceCands, atoi(pc)));
  if (const char *es = getenv("RJ_ENT_SHIFT_KB")) ent_shift_ = uint64_t(std::max(0, atoi(es))) << 10;
  if (const char *ub = getenv("RJ_UPLOAD_B_SIDE")) side_b_ = atoi(ub) != 0;
  if (const char *lk = getenv("RJ_K2_LIVE")) {  // 0 off; 2 (test): the live launch always gives up
    live_k2_ = atoi(lk) != 0;  // 1: on
    live_test_giveup_ = atoi(lk) == 2;
  }
  if (const char *ll = getenv("RJ_K2_LIVE_LDS")) live_lds_ = uint32_t(std::max(0, atoi(ll)));
  if (const char *sh = getenv("RJ_SPLIT_HOST")) split_host_ = atoi(sh) != 0;
  if (const char *sp = getenv("RJ_SPLIT_PARTS")) split_parts_ = std::max(2, std::min(4, atoi(sp)));
  for (auto &e : pev_) RJ_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  for (auto &e : pk1_) RJ_HIP(hipEventCreate(&e));
  for (auto &e : kev_) RJ_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  for (auto &e : prog_ev_) RJ_HIP(hipEventCreate(&e));
  for (auto &e : prog_join_) RJ_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  // development diagnostics, read once (never per call)
  const char *dbg_names[] = {"RJ_DEBUG_SCAN", "RJ_DEBUG_PROG", "RJ_DEBUG_WAVES", "RJ_DEBUG_HOST",
                             "RJ_DEBUG_STAMPS", "RJ_DEBUG_K1", "RJ_DEBUG_K1_PIECES", "RJ_TEST_PROG_GIVEUP"};
  for (int k = 0; k < 8; k++)
    if (getenv(dbg_names[k])) dbg_ |= 1u << k;
  if (const char *pp = getenv("RJ_PROG_PIPE")) prog_pipe_enabled_ = atoi(pp) != 0;
  if (const char *pw = getenv("RJ_PROG_WAVE_ALL")) prog_wave_all_ = atoi(pw) != 0;
  if (const char *pd = getenv("RJ_PROG_DC_LANES")) prog_dc_lanes_ = atoi(pd) != 0;
  for (auto *arr : {k1s_, k2s_, k2e_})
    for (int q = 0; q < kMaxPipe; q++) RJ_HIP(hipEventCreate(&arr[q]));
  (void)backend_;  // HARDWARE and HYBRID both run the HIP decoder
  return kOk;
}

int Decoder::GetImageInfo(Stream *s, uint8_t *nc, RocJpegChromaSubsampling *css, uint32_t *w, uint32_t *h) {
  std::lock_guard<std::mutex> lock(mu_);
  if (s == nullptr || nc == nullptr || css == nullptr || w == nullptr || h == nullptr) return kInvalidParameter;
  std::lock_guard<std::mutex> sl(s->mutex());  // a concurrent re-parse must not tear the info
  int c = -1;
  const int st = ImageInfo(s->info(), nc, &c, w, h);
  *css = RocJpegChromaSubsampling(c);
  return st;
}

int Decoder::StreamsToDevice(Stream *const *streams, int n) {
  std::lock_guard<std::mutex> lock(mu_);
  if (streams == nullptr || n < 0) return kInvalidParameter;
  RJ_HIP(hipSetDevice(device_));
  for (int i = 0; i < n; i++) {
    Stream *s = streams[i];
    if (s == nullptr) return kInvalidParameter;
    std::lock_guard<std::mutex> sl(s->mutex());
    if (s->resident.device == device_ && s->resident.generation == s->generation()) continue;
    s->ReleaseResident();
    const StreamInfo &in = s->info();
    const DecodePlan &p = s->plan();
    if (p.status != 0) continue;
    if (s->scan_pending()) return kBadJpeg;  // header-only parse never completed
    // every allocation lands in s->resident at once: an error part-way is freed by
    // ReleaseResident (the stream's destructor or its next parse)
    Stream::Resident &r = s->resident;
    r.device = device_;
    r.generation = s->generation() - 1;  // not valid until every copy below succeeded
    RJ_HIP(hipMalloc(reinterpret_cast<void **>(&r.ecs), in.ecs_size + 16));  // K0 reads <= 8 B past the end
    RJ_HIP(hipMalloc(reinterpret_cast<void **>(&r.segs), std::max<size_t>(p.segs.size() * sizeof(RjSegDev), 16)));
    RJ_HIP(hipMalloc(reinterpret_cast<void **>(&r.ds), std::max<size_t>(p.ds.size() * sizeof(RjDsBlock), 16)));
    RJ_HIP(hipMemcpy(r.ecs, in.ecs, in.ecs_size, hipMemcpyHostToDevice));
    RJ_HIP(hipMemcpy(r.segs, p.segs.data(), p.segs.size() * sizeof(RjSegDev), hipMemcpyHostToDevice));
    if (!p.ds.empty()) RJ_HIP(hipMemcpy(r.ds, p.ds.data(), p.ds.size() * sizeof(RjDsBlock), hipMemcpyHostToDevice));
    if (p.progressive) {  // scans, intervals and Huffman tables travel with the bitstream
      RJ_HIP(hipMalloc(reinterpret_cast<void **>(&r.pscans), std::max<size_t>(p.pscans.size() * sizeof(RjProgScanDev), 16)));
      RJ_HIP(hipMalloc(reinterpret_cast<void **>(&r.pivals), std::max<size_t>(p.pivals.size() * sizeof(RjProgIvalDev), 16)));
      RJ_HIP(hipMalloc(reinterpret_cast<void **>(&r.ptabs), std::max<size_t>(p.ptabs.size() * sizeof(RjHuffDev), 16)));
      RJ_HIP(hipMemcpy(r.pscans, p.pscans.data(), p.pscans.size() * sizeof(RjProgScanDev), hipMemcpyHostToDevice));
      RJ_HIP(hipMemcpy(r.pivals, p.pivals.data(), p.pivals.size() * sizeof(RjProgIvalDev), hipMemcpyHostToDevice));
      if (!p.ptabs.empty())
        RJ_HIP(hipMemcpy(r.ptabs, p.ptabs.data(), p.ptabs.size() * sizeof(RjHuffDev), hipMemcpyHostToDevice));
    }
    r.generation = s->generation();
  }
  return kOk;
}

int Decoder::ParseOnDevice(Stream *const *streams, const uint8_t *const *data, const size_t *len, int n) {
  std::lock_guard<std::mutex> lock(mu_);
  if (streams == nullptr || data == nullptr || len == nullptr || n < 0) return kInvalidParameter;
  // Whatever ended the call (a header that failed to parse, a HIP error, an exception from a
  // host worker), no stream is left half-parsed: a stream whose header walk deferred its marker
  // scan gets the host scan.
  auto settle = [&] {
    for (int i = 0; i < n; i++) {
      Stream *s = streams[i];
      if (s != nullptr && s->scan_pending() && data[i] != nullptr) s->Parse(data[i], uint32_t(len[i]));
    }
  };
  int st;
  try {
    st = ParseOnDeviceImpl(streams, data, len, n);
  } catch (...) {
    settle();
    throw;
  }
  settle();
  return st;
}

int Decoder::ParseOnDeviceImpl(Stream *const *streams, const uint8_t *const *data, const size_t *len, int n) {
  RJ_HIP(hipSetDevice(device_));
  const auto t0 = std::chrono::steady_clock::now();
  for (double &x : scan_ms_) x = 0;  // a call that fails early reports no stages of an earlier one
  timings_.scan_device_streams = timings_.scan_host_fallbacks = 0;
  for (int i = 0; i < n; i++)
    if (streams[i] == nullptr || data[i] == nullptr) return kInvalidParameter;
  // ---- host: headers only (O(header) per stream), over the handle's host threads ----
  std::vector<uint8_t> hdr(size_t(n), 0);  // 1: device scan pending, 2: parsed otherwise, 0: bad
  {
    const int nt = n >= 64 ? pool_.threads() : 1;  // small batches stay on the calling thread
    const int per = (n + nt * 4 - 1) / (nt * 4);
    pool_.Run((n + per - 1) / per,
              [&](int t) {
                for (int i = t * per; i < std::min(n, (t + 1) * per); i++) {
                  Stream *s = streams[i];
                  if (len[i] > 0xFFFFFFFFull || !s->Parse(data[i], uint32_t(len[i]), true)) continue;
                  if (!s->scan_pending() && !s->plan().progressive)
                    s->Parse(data[i], uint32_t(len[i]));  // not decodable: host parse, same info
                  hdr[size_t(i)] = s->scan_pending() ? 1 : 2;
                }
              },
              nullptr, nt == 1);
  }
  std::vector<int> pend;
  for (int i = 0; i < n; i++) {
    if (hdr[size_t(i)] == 0) return kBadJpeg;
    if (hdr[size_t(i)] == 1) pend.push_back(i);
  }
  timings_.scan_device_streams = timings_.scan_host_fallbacks = 0;
  for (double &x : scan_ms_) x = 0;
  const auto t_hdr = std::chrono::steady_clock::now();
  scan_ms_[0] = std::chrono::duration<double, std::milli>(t_hdr - t0).count();
  if (pend.empty()) return kOk;
  // ---- layout: one upload (bytes + jobs), one kernel, one read-back (tables + results) ----
  struct Lay {
    uint64_t src, segs, ds, rst, oth, drop;
    uint32_t expected, ds_cap, drop_cap;
  };
  std::vector<Lay> lay(pend.size());
  uint64_t bytes = 0, nsegs = 0, nds = 0, nrst = 0, noth = 0, ndrop = 0;
  constexpr uint32_t kOthCap = 4096;
  for (size_t k = 0; k < pend.size(); k++) {
    const Stream *s = streams[pend[k]];
    const DecodePlan &p = s->plan();
    const uint32_t avail = s->info().ecs_size, ri = s->info().restart_interval;
    const uint32_t total = p.mcux * p.mcuy;
    Lay &L = lay[k];
    L.expected = ri ? (total + ri - 1) / ri : 1;
    L.ds_cap = avail / RJ_DS_BLOCK + L.expected + 1;
    L.drop_cap = avail / 2 + 64;
    L.src = bytes;
    bytes += AlignUp(uint64_t(avail) + 16, 256);
    L.segs = nsegs;
    nsegs += L.expected;
    L.ds = nds;
    nds += L.ds_cap;
    L.rst = nrst;
    nrst += L.expected + 1;
    L.oth = noth;
    noth += kOthCap;
    L.drop = ndrop;
    ndrop += L.drop_cap;
  }
  const uint64_t np = pend.size();
  const uint64_t off_jobs = AlignUp(bytes, 256);
  const uint64_t up_bytes = AlignUp(off_jobs + np * sizeof(RjScanJob), 256);
  const uint64_t off_out = up_bytes;  // read-back region: results, table copies
  const uint64_t off_segs = AlignUp(off_out + np * sizeof(RjScanOut), 256);
  const uint64_t off_ds = AlignUp(off_segs + nsegs * sizeof(RjSegDev), 256);
  const uint64_t down_end = AlignUp(off_ds + nds * sizeof(RjDsBlock), 256);
  const uint64_t off_rst = down_end;
  const uint64_t off_oth = AlignUp(off_rst + nrst * 4, 256);
  const uint64_t off_drop = AlignUp(off_oth + noth * 4, 256);
  const uint64_t total_bytes = AlignUp(off_drop + ndrop * 4, 256);
  RJ_CHECK(d_scan_.Ensure(total_bytes));
  RJ_CHECK(h_scan_.Ensure(down_end));
  uint8_t *h = h_scan_.data();
  uint8_t *d = d_scan_.as<uint8_t>();
  std::vector<Stream::Resident> res(np);
  // one HBM block for every stream's resident buffers (ECS + 32 B, interval table, K0 table),
  // shared by the streams and freed with the last of them (no per-stream hipMalloc)
  uint64_t rbytes = 0;
  std::vector<uint64_t> roff(np);
  for (size_t k = 0; k < np; k++) {
    roff[k] = rbytes;
    rbytes += AlignUp(uint64_t(streams[pend[k]]->info().ecs_size) + 32, 256) +
              AlignUp(lay[k].expected * sizeof(RjSegDev), 256) + AlignUp(lay[k].ds_cap * sizeof(RjDsBlock), 256);
  }
  uint8_t *rblock = nullptr;
  const auto t_lay = std::chrono::steady_clock::now();
  RJ_HIP(hipMalloc(reinterpret_cast<void **>(&rblock), std::max<uint64_t>(rbytes, 256)));
  const auto t_alloc = std::chrono::steady_clock::now();
  scan_ms_[1] = std::chrono::duration<double, std::milli>(t_alloc - t_lay).count();
  const int dev = device_;
  std::shared_ptr<uint8_t> block(rblock, [dev](uint8_t *p) {
    int cur = 0;
    if (hipGetDevice(&cur) == hipSuccess) {
      (void)hipSetDevice(dev);
      (void)hipFree(p);
      (void)hipSetDevice(cur);
    }
  });
  RjScanJob *jobs = reinterpret_cast<RjScanJob *>(h + off_jobs);
  for (size_t k = 0; k < np; k++) {  // the jobs (they need only the layout), uploaded first
    const Stream *s = streams[pend[k]];
    const DecodePlan &p = s->plan();
    const Lay &L = lay[k];
    const uint32_t avail = s->info().ecs_size;
    Stream::Resident &r = res[k];
    r.device = device_;
    r.generation = s->generation();
    r.block = block;
    r.ecs = rblock + roff[k];
    r.segs = reinterpret_cast<RjSegDev *>(r.ecs + AlignUp(uint64_t(avail) + 32, 256));
    r.ds = reinterpret_cast<RjDsBlock *>(reinterpret_cast<uint8_t *>(r.segs) + AlignUp(L.expected * sizeof(RjSegDev), 256));
    RjScanJob &J = jobs[k];
    std::memset(&J, 0, sizeof(J));
    J.src_off = L.src;
    J.avail = avail;
    J.ri = s->info().restart_interval;
    J.total_mcus = p.mcux * p.mcuy;
    J.nblk_mcu = p.nblk_mcu;
    J.expected = L.expected;
    J.rst_cap = L.expected + 1;
    J.oth_cap = kOthCap;
    J.drop_cap = L.drop_cap;
    J.ds_cap = L.ds_cap;
    J.ecs = r.ecs;
    J.segs = r.segs;
    J.segs_copy = reinterpret_cast<RjSegDev *>(d + off_segs) + L.segs;
    J.ds = r.ds;
    J.ds_copy = reinterpret_cast<RjDsBlock *>(d + off_ds) + L.ds;
    J.rst = reinterpret_cast<uint32_t *>(d + off_rst) + L.rst;
    J.oth = reinterpret_cast<uint32_t *>(d + off_oth) + L.oth;
    J.drop = reinterpret_cast<uint32_t *>(d + off_drop) + L.drop;
    J.out = reinterpret_cast<RjScanOut *>(d + off_out) + k;
  }
  RJ_HIP(hipMemcpyAsync(d + off_jobs, h + off_jobs, up_bytes - off_jobs, hipMemcpyHostToDevice, stream_));
  RJ_HIP(hipMemsetAsync(d + off_out, 0, np * sizeof(RjScanOut), stream_));
  {  // the bytes into the pinned staging blob over the handle's host threads, in pieces of
     // streams; the calling thread uploads each finished prefix of pieces while the threads copy
     // the next (HostPool::Run's in-order done callback), so the copy and the DMA overlap.  (Per
     // piece scan launches were measured: k_scan runs one wave per stream, so a piece's launch
     // occupies only its streams' CUs and the serialised launches took 10x the one launch.)
    constexpr uint64_t kPiece = 8ull << 20;
    std::vector<size_t> piece0{0};
    for (size_t k = 0; k < np; k++)
      if (lay[k].src - lay[piece0.back()].src >= kPiece) piece0.push_back(k);
    piece0.push_back(np);
    const int npieces = int(piece0.size()) - 1;
    uint64_t uploaded = 0;
    int up_err = 0;
    pool_.Run(npieces,
              [&](int t) {
                for (size_t k = piece0[size_t(t)]; k < piece0[size_t(t) + 1]; k++) {
                  const Stream *s = streams[pend[k]];
                  CopyToStaging(h + lay[k].src, s->info().ecs, s->info().ecs_size);
                  std::memset(h + lay[k].src + s->info().ecs_size, 0, 16);
                }
              },
              [&](int t) {
                const uint64_t end = piece0[size_t(t) + 1] < np ? lay[piece0[size_t(t) + 1]].src : bytes;
                if (!up_err && hipMemcpyAsync(d + uploaded, h + uploaded, end - uploaded, hipMemcpyHostToDevice,
                                              stream_) != hipSuccess)
                  up_err = 1;
                uploaded = end;
              });
    if (up_err) return kExecutionFailed;
    RJ_HIP(LaunchScan(stream_, reinterpret_cast<const RjScanJob *>(d + off_jobs), uint32_t(np), d));
  }
  const auto t_copy = std::chrono::steady_clock::now();
  scan_ms_[2] = std::chrono::duration<double, std::milli>(t_copy - t_alloc).count();
  const auto t1 = std::chrono::steady_clock::now();
  RJ_HIP(hipMemcpyAsync(h + off_out, d + off_out, down_end - off_out, hipMemcpyDeviceToHost, stream_));
  RJ_HIP(hipStreamSynchronize(stream_));
  const auto t2 = std::chrono::steady_clock::now();
  scan_ms_[3] = std::chrono::duration<double, std::milli>(t2 - t1).count();
  // ---- host: adopt the device tables (or scan on the host where a list overflowed), over the
  // handle's host threads (each stream under its own lock) ----
  std::atomic<uint32_t> ndev{0}, nfall{0};
  {
    const int nt = np >= 64 ? pool_.threads() : 1;
    const size_t per = (np + size_t(nt) * 4 - 1) / (size_t(nt) * 4);
    pool_.Run(int((np + per - 1) / per),
              [&](int t) {
                for (size_t k = size_t(t) * per; k < std::min(np, size_t(t + 1) * per); k++) {
                  Stream *s = streams[pend[k]];
                  const RjScanOut &o = reinterpret_cast<const RjScanOut *>(h + off_out)[k];
                  const Lay &L = lay[k];
                  Stream::Resident &r = res[k];
                  if (o.flags) {
                    r = Stream::Resident();  // this stream keeps no share of the block
                    s->Parse(data[pend[k]], uint32_t(len[pend[k]]));
                    nfall++;
                    continue;
                  }
                  ndev++;
                  std::lock_guard<std::mutex> sl(s->mutex());
                  s->CompleteFromDevice(o.ecs_end, reinterpret_cast<const RjSegDev *>(h + off_segs) + L.segs,
                                        L.expected, reinterpret_cast<const RjDsBlock *>(h + off_ds) + L.ds, o.nds);
                  s->resident = r;
                }
              },
              nullptr, nt == 1);
  }
  timings_.scan_device_streams = ndev.load();
  timings_.scan_host_fallbacks = nfall.load();
  if (timings_.scan_host_fallbacks) RJ_INFO("marker scan list overflow on %u streams: host scan", timings_.scan_host_fallbacks);
  const auto t3 = std::chrono::steady_clock::now();
  scan_ms_[4] = std::chrono::duration<double, std::milli>(t3 - t2).count();
  scan_ms_[5] = std::chrono::duration<double, std::milli>(t3 - t0).count();
  if (Dbg(kDebugScan))
    fprintf(stderr, "[rj scan] %zu streams: headers %.3f alloc %.3f copy+upload %.3f kernel+readback %.3f adopt %.3f total %.3f ms\n",
            size_t(np), scan_ms_[0], scan_ms_[1], scan_ms_[2], scan_ms_[3], scan_ms_[4], scan_ms_[5]);
  return kOk;
}

int Decoder::PtrDevice(const void *p) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  for (const PtrRange &r : ptr_cache_)
    if (a >= r.lo && a < r.hi) return r.device;
  int dev = -1;  // host memory unless HIP says device / managed
  uintptr_t lo = a, hi = a + 1;
  hipPointerAttribute_t at;
  if (hipPointerGetAttributes(&at, p) == hipSuccess) {
    if (at.type == hipMemoryTypeDevice) dev = at.device;
    else if (at.type == hipMemoryTypeManaged || at.isManaged) dev = device_;  // kernels write it in place
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    if (hipMemGetAddressRange(&base, &size, const_cast<void *>(p)) == hipSuccess && size) {
      lo = reinterpret_cast<uintptr_t>(base);
      hi = lo + size;
    } else {
      (void)hipGetLastError();
    }
  } else {
    (void)hipGetLastError();  // pageable host memory
  }
  if (dev >= 0 && dev != device_) {  // another GPU: copies go peer to peer (xGMI) where allowed
    if (peer_enabled_.size() <= size_t(dev)) peer_enabled_.resize(size_t(dev) + 1, 0);
    if (!peer_enabled_[dev]) {
      int can = 0;
      if (hipDeviceCanAccessPeer(&can, device_, dev) == hipSuccess && can) (void)hipDeviceEnablePeerAccess(dev, 0);
      (void)hipGetLastError();  // already enabled, or no peer path: hipMemcpy2DAsync stages it
      peer_enabled_[dev] = 1;
    }
  }
  ptr_cache_.push_back({lo, hi, dev});
  return dev;
}

int Decoder::Decode(Stream *const *streams, int n, const RocJpegDecodeParams *params, RocJpegImage *dst) {
  if (streams == nullptr || params == nullptr || dst == nullptr || n < 0) return kInvalidParameter;
  for (int i = 0; i < n; i++)
    if (streams[i] == nullptr) return kInvalidParameter;
  // (DecodeOne counts the staged streams under the stream locks it takes anyway, and hands a
  // large staged call back for DecodeSplit before any work)
  const bool may_split = split_host_ && n >= kSplitHostMin && !profiling_ && path_policy_ == 0;
  const int r = DecodeOne(streams, n, params, dst, may_split);
  return r == kWantSplit ? DecodeSplit(streams, n, params, dst) : r;
}

int Decoder::DecodeSplit(Stream *const *streams, int n, const RocJpegDecodeParams *params, RocJpegImage *dst) {
  // the whole call's host validation first: a call that would fail it writes nothing, as unsplit
  const int cst = Check(streams, n, params, dst);
  if (cst != kOk) return cst;
  {
    std::lock_guard<std::mutex> lock(mu_);
    while (int(helpers_.size()) < split_parts_ - 1) {
      std::unique_ptr<Decoder> h(new Decoder(backend_, device_));
      if (h->Initialize() != kOk) break;  // (fewer parts: as many handles as this device gives)
      h->split_host_ = false;
      helpers_.push_back(std::move(h));
    }
  }
  const int P = std::min(split_parts_, int(helpers_.size()) + 1);
  if (P < 2) {
    split_host_ = false;  // no second handle on this device: every call decodes whole
    return DecodeOne(streams, n, params, dst);
  }
  // Part k decodes on its own handle and thread; the parts' uploads run in order on the copy
  // engine (part k's waits for part k - 1's, an event), so each part's kernels run while the
  // later parts' bytes cross PCIe.  The shares shrink: what is left exposed after the last
  // upload is the last part's decode (profiles/r6_experiments/host_input_parts_ab.txt).
  static const double kShare[5][4] = {{1, 0, 0, 0}, {1, 0, 0, 0}, {0.5, 0.5, 0, 0}, {0.4, 0.35, 0.25, 0},
                                      {0.3, 0.28, 0.24, 0.18}};
  int cut[5] = {0, 0, 0, 0, 0};
  double acc = 0;
  for (int k = 0; k < P; k++) {
    acc += kShare[P][k];
    cut[k + 1] = k + 1 == P ? n : std::max(cut[k] + 1, std::min(n - (P - 1 - k), int(acc * n + 0.5)));
  }
  Decoder *owner[4] = {this, nullptr, nullptr, nullptr};
  for (int k = 1; k < P; k++) owner[k] = helpers_[size_t(k - 1)].get();
  std::mutex m;
  std::condition_variable cv;
  bool go[5] = {true, false, false, false, false};
  auto signal = [&](int k) {  // part k may start: part k - 1's uploads are enqueued (or it failed)
    std::lock_guard<std::mutex> l(m);
    if (!go[k]) {
      go[k] = true;
      cv.notify_all();
    }
  };
  for (int k = 0; k + 1 < P; k++) {
    Decoder *next = owner[k + 1];
    Decoder *self = owner[k];
    next->upload_after_ = self->split_ev_;
    self->uploaded_ = [&, k, self, next] {
      if (hipEventRecord(self->split_ev_, self->stream_) != hipSuccess) next->upload_after_ = nullptr;
      signal(k + 1);
    };
  }
  int st[4] = {kOk, kOk, kOk, kOk};
  std::exception_ptr err;
  auto run = [&](int k) {
    {
      std::unique_lock<std::mutex> l(m);
      cv.wait(l, [&] { return go[k]; });
    }
    try {
      st[k] = owner[k]->DecodeOne(streams + cut[k], cut[k + 1] - cut[k], params, dst + cut[k]);
    } catch (...) {
      st[k] = kRuntimeError;
      if (k == 0) err = std::current_exception();
    }
    if (k + 1 < P) {  // a part that never uploaded leaves nothing to wait for
      bool up;
      {
        std::lock_guard<std::mutex> l(m);
        up = go[k + 1];
      }
      if (!up) owner[k + 1]->upload_after_ = nullptr;
      signal(k + 1);
    }
  };
  for (int k = 0; k < P; k++) owner[k]->split_part_ = true;
  std::vector<std::thread> threads;
  for (int k = 1; k < P; k++) threads.emplace_back(run, k);
  run(0);
  for (std::thread &t : threads) t.join();
  for (int k = 0; k < P; k++) {
    owner[k]->uploaded_ = nullptr;
    owner[k]->upload_after_ = nullptr;
    owner[k]->split_part_ = false;
  }
  if (err) std::rethrow_exception(err);
  for (int k = 0; k < P; k++)
    if (st[k] != kOk) return st[k];
  return kOk;
}

void Decoder::PlaceStep(float ms) {
  const int k = place_state_ - 1;  // the candidate this call ran with (in d_entries_)
  place_ms_[k] = ms;
  if (place_best_ < 0 || ms < place_ms_[place_best_] * 0.995f) place_best_ = k;  // (0.5 %: the calls' noise)
  const size_t cap = d_entries_.capacity();
  place_bufs_[k].Swap(d_entries_);  // stays allocated, so that the next candidate is other memory
  if (k + 1 < place_cands_ && d_entries_.Ensure(cap) == kOk) {
    place_state_ = k + 2;
    return;
  }
  d_entries_.Release();  // done (or out of memory for another candidate): keep the fastest
  d_entries_.Swap(place_bufs_[place_best_]);
  if (!place_keep_)
    for (DeviceBuffer &b : place_bufs_) b.Release();
  place_state_ = -1;
}

// The end of a call: the calling thread polls the stream (yielding between polls) instead of
// sleeping in hipStreamSynchronize when spin_sync_ is set (env RJ_SYNC_SPIN=1).
hipError_t Decoder::SideStream(hipStream_t &s, bool lowest_priority) {
  if (s != nullptr) return hipSuccess;
  if (!lowest_priority) return hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  int lo = 0, hi = 0;  // "least" is the numerically greatest
  const hipError_t e = hipDeviceGetStreamPriorityRange(&lo, &hi);
  return e != hipSuccess ? e : hipStreamCreateWithPriority(&s, hipStreamNonBlocking, lo);
}

hipError_t Decoder::WaitCall() {
  if (spin_sync_) {
    hipError_t e;
    while ((e = hipStreamQuery(stream_)) == hipErrorNotReady) sched_yield();
    if (e != hipSuccess) return e;
  }
  return hipStreamSynchronize(stream_);
}

int Decoder::DecodeOne(Stream *const *streams, int n, const RocJpegDecodeParams *params, RocJpegImage *dst,
                       bool may_split) {
  const auto t_call = std::chrono::steady_clock::now();
  std::lock_guard<std::mutex> lock(mu_);
  // Hold every stream's lock for the call: a concurrent re-parse must not move its bytes.  Locks
  // are taken in address order (no deadlock between calls sharing streams); a batch already in
  // increasing order -- the usual one, streams created in sequence -- is not sorted again.
  std::vector<std::unique_lock<std::mutex>> locks;
  std::vector<Stream *> &uniq = lock_order_;
  uniq.assign(streams, streams + n);
  const std::less<Stream *> before;
  bool increasing = true;
  for (int i = 1; i < n && increasing; i++) increasing = before(uniq[i - 1], uniq[i]);
  if (!increasing) {
    std::sort(uniq.begin(), uniq.end(), before);
    uniq.erase(std::unique(uniq.begin(), uniq.end()), uniq.end());
  }
  locks.reserve(uniq.size());
  for (Stream *s : uniq) locks.emplace_back(s->mutex());
  if (may_split) {
    int staged = 0;
    for (int i = 0; i < n; i++) {
      const Stream *s = streams[i];
      staged += (s->resident.device == device_ && s->resident.generation == s->generation()) ? 0 : 1;
    }
    if (staged >= kSplitHostMin) return kWantSplit;  // (nothing done yet; the locks are released)
  }
  const auto t_locked = std::chrono::steady_clock::now();
  const int r = DecodeLocked(streams, n, params, dst);
  // an error return may leave copies in flight on the stream (from the parse-time pinned arena
  // or the staging buffers): they finish before the streams' locks are released, so a
  // re-parse or destroy cannot recycle memory a DMA is still reading
  if (r != kOk) {
    (void)hipStreamSynchronize(stream_);
    if (bstream_) (void)hipStreamSynchronize(bstream_);
  }
  if (Dbg(kDebugHost)) {  // development: the call's host time outside DecodeLocked's planning
    const auto t_ret = std::chrono::steady_clock::now();
    locks.clear();
    const auto t_unlocked = std::chrono::steady_clock::now();
    auto ms = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
      return std::chrono::duration<double, std::milli>(b - a).count();
    };
    fprintf(stderr, "[rj call] caller since the last return %.3f | locks %.3f | after the sync %.3f | unlock %.3f ms\n",
            dbg_returned_.time_since_epoch().count() ? ms(dbg_returned_, t_call) : 0.0, ms(t_call, t_locked),
            ms(dbg_synced_, t_ret), ms(t_ret, t_unlocked));
    dbg_returned_ = std::chrono::steady_clock::now();
  }
  return r;
}

// The destination channels an output format needs (rocjpeg_decoder.cpp:143-180; DecodeLocked's
// job builder makes the same checks as it lays out the jobs).
static int CheckDestination(int fmt, int css, const RocJpegImage &o) {
  auto need = [&](int c) { return o.channel[c] != nullptr; };
  switch (fmt) {
    case ROCJPEG_OUTPUT_YUV_PLANAR:
      if (!need(0)) return kInvalidParameter;
      if ((css == kCss422 || css == kCss420 || css == kCss444 || css == kCss440) && (!need(1) || !need(2)))
        return kInvalidParameter;
      return kOk;
    case ROCJPEG_OUTPUT_Y:
    case ROCJPEG_OUTPUT_RGB:
      return need(0) ? kOk : kInvalidParameter;
    case ROCJPEG_OUTPUT_RGB_PLANAR:
      return (need(0) && need(1) && need(2)) ? kOk : kInvalidParameter;
    default:
      return kOk;  // NATIVE writes what it has channels for; unknown formats write nothing
  }
}

int Decoder::Check(Stream *const *streams, int n, const RocJpegDecodeParams *params, const RocJpegImage *dst) {
  if (streams == nullptr || params == nullptr || dst == nullptr || n < 0) return kInvalidParameter;
  for (int i = 0; i < n; i++) {
    if (streams[i] == nullptr) return kInvalidParameter;
    std::lock_guard<std::mutex> sl(streams[i]->mutex());
    const DecodePlan &p = streams[i]->plan();
    if (p.status != 0) return p.status;
    if (streams[i]->scan_pending()) return kBadJpeg;
  }
  for (int i = 0; i < n; i++) {
    std::lock_guard<std::mutex> sl(streams[i]->mutex());
    const int st = CheckDestination(int(params->output_format), streams[i]->info().css, dst[i]);
    if (st != kOk) return st;
  }
  return kOk;
}

// progressive images per call up to which every scan goes to the wave grid (see prog_wave_all)
static constexpr int kProgWaveAllImages = 1280;  // measured crossover (C5 1080p: 1024 -> one grid, 2048 -> two)

int Decoder::DecodeLocked(Stream *const *streams, int n, const RocJpegDecodeParams *params, RocJpegImage *dst) {
  const auto t_host0 = std::chrono::steady_clock::now();
  RJ_HIP(hipSetDevice(device_));
  timings_ = RocJpegAmdTimings();
  if (n == 0) return kOk;
  const int fmt = int(params->output_format);

  // ---- per-image validation (SubmitDecode checks, destination checks) ----
  for (int i = 0; i < n; i++) {
    const DecodePlan &p = streams[i]->plan();
    if (p.status != 0) return p.status;
    if (streams[i]->scan_pending()) return kBadJpeg;  // header-only parse never completed
  }
  // ---- destinations on another device or in host memory: decoded into staging, then copied
  // (the allocation lookup is cached per call by address range) ----
  ptr_cache_.clear();
  routes_.clear();
  std::vector<uint8_t> &routed = sc_.routed;
  routed.assign(n, 0);
  for (int i = 0; i < n; i++)
    for (int c = 0; c < 4; c++)
      if (dst[i].channel[c] != nullptr && PtrDevice(dst[i].channel[c]) != device_) routed[i] = 1;
  uint64_t route_bytes = 0;

  const auto t_dedupe = std::chrono::steady_clock::now();
  // ---- table de-duplication ----
  std::vector<uint32_t> &tab_of = sc_.tab_of;
  tab_of.resize(n);
  std::vector<const RjTableSet *> tabs;
  std::vector<Stream *> &owner_stream = sc_.owner_stream;  // stream whose tables tabs[idx] are
  {
    std::vector<const DecodePlan *> owner;  // plan whose derived tables tabs[idx] points at
    owner_stream.clear();
    std::unordered_map<uint64_t, std::vector<uint32_t>> seen;
    uint32_t last = UINT32_MAX;  // batches are usually one encoder's output: try the last hit first
    for (int i = 0; i < n; i++) {
      const DecodePlan &p = streams[i]->plan();
      auto same = [&](uint32_t c) {
        return owner[c] == &p || (owner[c]->table_hash == p.table_hash &&
                                  std::memcmp(owner[c]->table_key, p.table_key, sizeof(p.table_key)) == 0);
      };
      uint32_t idx = UINT32_MAX;
      if (last != UINT32_MAX && same(last)) {
        idx = last;
      } else {
        auto &cands = seen[p.table_hash];
        for (uint32_t c : cands)
          if (same(c)) { idx = c; break; }
        if (idx == UINT32_MAX) {
          idx = uint32_t(tabs.size());
          tabs.push_back(&p.tables);
          owner.push_back(&p);
          owner_stream.push_back(streams[i]);
          cands.push_back(idx);
        }
      }
      tab_of[i] = last = idx;
    }
  }

  const auto t_layout = std::chrono::steady_clock::now();
  // ---- layout ----
  std::vector<RjImageDev> &imgs = sc_.imgs;
  imgs.resize(n);
  std::vector<RjJobDev> &jobs = sc_.jobs;
  jobs.clear();
  uint64_t destuff_total = 0, coef_blocks = 0, ent_total = 0, plane_bytes = 0, stage_bytes = 0;
  uint32_t seg_total = 0, rows_total = 0, chunk_total = 0, ds_total = 0;
  uint64_t ecs_bytes = 0, out_bytes = 0, ecs_stage_bytes = 0, ecs_copy_bytes = 0;
  std::vector<uint64_t> &stage_off = sc_.stage_off, &ecs_off = sc_.ecs_off;
  stage_off.assign(n, UINT64_MAX);
  ecs_off.assign(n, UINT64_MAX);
  std::vector<uint32_t> &row_prefix = sc_.row_prefix, &grow_prefix = sc_.grow_prefix;  // K2 rows: fused / general
  row_prefix.resize(n);
  grow_prefix.resize(n);
  uint32_t fused_rows = 0, general_rows = 0, fused_images = 0;
  std::vector<uint8_t> &is_fused = sc_.is_fused;
  is_fused.assign(n, 0);
  // progressive images: their own K2 row spaces (dense coefficients), K1p intervals, buffers
  std::vector<uint32_t> &prow_prefix = sc_.prow_prefix, &pgrow_prefix = sc_.pgrow_prefix;
  prow_prefix.resize(n);
  pgrow_prefix.resize(n);
  uint32_t pfused_rows = 0, pgeneral_rows = 0, prog_images = 0, prog_levels = 0, pival_total = 0;
  uint64_t coef_dw_total = 0, nz_total = 0, prec_total = 0;
  for (int i = 0; i < n; i++) {
    Stream *s = streams[i];
    const StreamInfo &in = s->info();
    const DecodePlan &p = s->plan();
    RjImageDev &d = imgs[i];
    std::memset(&d, 0, sizeof(d));
    d.width = in.width;
    d.height = in.height;
    d.mcux = p.mcux;
    d.mcuy = p.mcuy;
    d.ncomp = in.ncomp;
    d.nblk_mcu = p.nblk_mcu;
    d.interleaved = p.interleaved;
    d.css = uint8_t(in.css);
    d.hmax = p.hmax;
    d.vmax = p.vmax;
    d.fmt = uint8_t(fmt);
    for (int c = 0; c < 4; c++) {
      d.comp_h[c] = in.comp[c].h;
      d.comp_v[c] = in.comp[c].v;
      d.comp_td[c] = in.scomp[c].td;
      d.comp_ta[c] = in.scomp[c].ta;
      d.comp_tq[c] = p.progressive ? uint8_t(c) : in.comp[c].tq;  // progressive: latched per component
      d.comp_blk0[c] = p.comp_blk0[c];
    }
    std::memcpy(d.blk_comp, p.blk_comp, RJ_MAX_BLK_MCU);
    std::memcpy(d.blk_dx, p.blk_dx, RJ_MAX_BLK_MCU);
    std::memcpy(d.blk_dy, p.blk_dy, RJ_MAX_BLK_MCU);
    d.tabset = tab_of[i];
    {  // the int32 IDCT is exact while |coefficient x quantiser| < 2^14 (rj_math.h)
      uint32_t qmax = 1;
      for (int c = 0; c < in.ncomp; c++) qmax = std::max<uint32_t>(qmax, p.qmax[d.comp_tq[c] & 3]);
      d.idct_thr = 16383u / qmax;
    }
    d.nseg = uint32_t(p.segs.size());
    d.seg_prefix = seg_total;
    seg_total += d.nseg;
    d.ds_prefix = ds_total;
    ds_total += uint32_t(p.ds.size());
    d.destuff_off = destuff_total;
    destuff_total += AlignUp(p.destuff_bytes, 256);
    coef_blocks += uint64_t(p.mcux) * p.mcuy * p.nblk_mcu;
    d.ent_off = ent_total;
    ent_total += AlignUp(p.entries, RJ_ENT_GROUP);
    d.ri_mcus = in.restart_interval;
    d.chunk_prefix = chunk_total;
    chunk_total += p.nchunks;
    for (int c = 0; c < in.ncomp; c++) {
      d.plane_pitch[c] = p.wblk[c] * 8;
      d.plane_rows[c] = p.hblk[c] * 8;
    }
    d.pival_prefix = pival_total;
    if (p.progressive) {
      d.progressive = 1;
      d.coef_off = coef_dw_total;
      coef_dw_total += AlignUp(p.coef_blocks * 32, 64);
      d.nz_off = nz_total;
      nz_total += AlignUp(p.nz_blocks, 8);
      d.prec_off = prec_total;
      prec_total += AlignUp(p.prec_words, 8);
      d.npscans = uint32_t(p.pscans.size());
      for (int c = 0; c < 3; c++) {
        d.cblk0[c] = p.cblk0[c];
        d.wblk[c] = p.wblk[c];
        d.nzblk0[c] = p.nzblk0[c];
        d.cwblk[c] = p.cwblk[c];
        d.chblk[c] = p.chblk[c];
      }
      pival_total += uint32_t(p.pivals.size());
      prog_images++;
      prog_levels = std::max(prog_levels, p.plevels);
    }
    ecs_bytes += in.ecs_size;
    if (!(s->resident.device == device_ && s->resident.generation == s->generation())) {
      // non-resident: its tables go with the descriptors (blob A), its bitstream into the ECS
      // staging, which is uploaded in chunks as the host threads fill it
      stage_off[i] = stage_bytes;
      stage_bytes += AlignUp(p.segs.size() * sizeof(RjSegDev), 256) + AlignUp(p.ds.size() * sizeof(RjDsBlock), 256);
      if (s->pinned_ecs() == nullptr) {  // copied by the host threads (offsets in the copy space)
        ecs_off[i] = ecs_copy_bytes;
        ecs_copy_bytes += AlignUp(in.ecs_size + 16, 256);  // K0 reads <= 8 B past the end
      }
      if (p.progressive)
        stage_bytes += AlignUp(p.pscans.size() * sizeof(RjProgScanDev), 256) +
                       AlignUp(p.pivals.size() * sizeof(RjProgIvalDev), 256) +
                       AlignUp(p.ptabs.size() * sizeof(RjHuffDev), 256);
    }

    // output window: ROI semantics of rocjpeg_decoder.cpp:124-141 (no ROI decode on gfx950)
    const uint32_t roi_w = uint32_t(int(params->crop_rectangle.right) - int(params->crop_rectangle.left));
    const uint32_t roi_h = uint32_t(int(params->crop_rectangle.bottom) - int(params->crop_rectangle.top));
    const bool roi = roi_w > 0 && roi_h > 0 && roi_w <= in.width && roi_h <= in.height;
    d.roi = roi;
    d.out_w = roi ? int32_t(roi_w) : in.width;
    d.out_h = roi ? int32_t(roi_h) : in.height;
    d.top = roi ? params->crop_rectangle.top : 0;
    d.left = roi ? params->crop_rectangle.left : 0;
    const RocJpegImage &o = dst[i];
    for (int c = 0; c < 4; c++) {
      d.dst[c] = o.channel[c];
      d.dst_pitch[c] = o.pitch[c];
    }
    row_prefix[i] = fused_rows;
    grow_prefix[i] = general_rows;
    prow_prefix[i] = pfused_rows;
    pgrow_prefix[i] = pgeneral_rows;

    // ---- output jobs (general path): rocjpeg_decoder.cpp:143-180 ----
    const size_t jobs_before = jobs.size();
    const uint32_t jobs_rows_before = rows_total;
    const int css = in.css;
    const int32_t pw = d.out_w, ph = d.out_h, top = d.top, left = d.left;
    auto need = [&](int c) { return o.channel[c] != nullptr; };
    uint32_t ext_rows[4] = {}, ext_bytes[4] = {};  // what the call writes per channel (routing)
    auto job = [&](uint32_t kind, uint32_t sel, int dc, int32_t rows, uint32_t bytes, uint32_t pitch, int32_t r0,
                   int32_t b0) {
      if (rows <= 0 || bytes == 0) return;
      ext_rows[dc] = std::max(ext_rows[dc], uint32_t(rows));
      ext_bytes[dc] = std::max(ext_bytes[dc], bytes);
      RjJobDev j;
      std::memset(&j, 0, sizeof(j));
      j.image = uint32_t(i);
      j.kind = kind;
      j.chan_sel = sel;
      j.rows = uint32_t(rows);
      j.row_bytes = bytes;
      j.dst_pitch = pitch;
      j.dst = o.channel[dc];
      j.src_row0 = r0;
      j.src_byte0 = b0;
      j.row_prefix = rows_total;
      rows_total += j.rows;
      out_bytes += uint64_t(rows) * bytes;
      jobs.push_back(j);
    };
    auto copy = [&](int sp, int chan, int dc, int32_t rows, int32_t r0, int32_t b0) {  // CopyChannel
      if (o.channel[dc] != nullptr && o.pitch[dc] != 0)
        job(RJ_JOB_COPY, uint32_t(sp | (chan << 4)), dc, rows, o.pitch[dc], o.pitch[dc], r0, b0);
    };
    const auto sel = [](int sp, int chan, int stride) { return uint32_t(sp | (chan << 4) | (stride << 8)); };
    switch (fmt) {
      case ROCJPEG_OUTPUT_NATIVE:
        if (css == kCss422) {
          copy(0, 0, 0, ph, top, 2 * left);
        } else {
          copy(0, 0, 0, ph, top, left);
          if (css == kCss420) copy(1, 1, 1, ph >> 1, top >> 1, left);
          if (css == kCss444) { copy(1, 1, 1, ph, top, left); copy(1, 2, 2, ph, top, left); }
          if (css == kCss440) { copy(1, 1, 1, ph >> 1, top >> 1, left); copy(1, 2, 2, ph >> 1, top >> 1, left); }
        }
        break;
      case ROCJPEG_OUTPUT_YUV_PLANAR:
        if (css == kCss422) {
          if (!need(0) || !need(1) || !need(2)) return kInvalidParameter;
          job(RJ_JOB_Y, 0, 0, ph, uint32_t(pw), o.pitch[0], top, left);
          job(RJ_JOB_CHROMA, sel(0, 0, 4), 1, ph, uint32_t(pw >> 1), o.pitch[1], top, 2 * left + 1);
          job(RJ_JOB_CHROMA, sel(0, 0, 4), 2, ph, uint32_t(pw >> 1), o.pitch[1], top, 2 * left + 3);
        } else {
          if (!need(0)) return kInvalidParameter;
          copy(0, 0, 0, ph, top, left);
          if (css == kCss420) {
            if (!need(1) || !need(2)) return kInvalidParameter;
            job(RJ_JOB_CHROMA, sel(1, 1, 2), 1, ph >> 1, uint32_t(pw >> 1), o.pitch[1], top >> 1, left);
            job(RJ_JOB_CHROMA, sel(1, 1, 2), 2, ph >> 1, uint32_t(pw >> 1), o.pitch[1], top >> 1, left + 1);
          } else if (css == kCss444) {
            if (!need(1) || !need(2)) return kInvalidParameter;
            copy(1, 1, 1, ph, top, left);
            copy(1, 2, 2, ph, top, left);
          } else if (css == kCss440) {
            if (!need(1) || !need(2)) return kInvalidParameter;
            copy(1, 1, 1, ph >> 1, top >> 1, left);
            copy(1, 2, 2, ph >> 1, top >> 1, left);
          }
        }
        break;
      case ROCJPEG_OUTPUT_Y:
        if (!need(0)) return kInvalidParameter;
        if (css == kCss422) job(RJ_JOB_Y, 0, 0, ph, uint32_t(pw), o.pitch[0], top, left);
        else copy(0, 0, 0, ph, top, left);
        break;
      case ROCJPEG_OUTPUT_RGB:
        if (!need(0)) return kInvalidParameter;
        job(RJ_JOB_RGB, 0, 0, ph, uint32_t(3 * pw), o.pitch[0], 0, 0);
        break;
      case ROCJPEG_OUTPUT_RGB_PLANAR:
        if (!need(0) || !need(1) || !need(2)) return kInvalidParameter;
        for (int k = 0; k < 3; k++) job(RJ_JOB_RGB_PLANE, uint32_t(k << 4), k, ph, uint32_t(pw), o.pitch[0], 0, 0);
        break;
      default:
        break;  // reference: unknown format writes nothing and succeeds
    }
    if (routed[i]) {
      for (int c = 0; c < 4; c++) {
        if (ext_rows[c] == 0 || o.channel[c] == nullptr) continue;
        routes_.push_back(RouteCopy{uint32_t(i), uint32_t(c), ext_rows[c], ext_bytes[c], o.pitch[c], route_bytes,
                                    o.channel[c]});
        route_bytes += AlignUp(uint64_t(ext_rows[c] - 1) * o.pitch[c] + ext_bytes[c], 256);
      }
    }
    // fast path: drop the general jobs again and count fused strips instead
    if (path_policy_ == 0 && FusedEligible(in, p, fmt, roi, o)) {
      rows_total = jobs_rows_before;
      jobs.resize(jobs_before);
      if (p.progressive) {
        pfused_rows += p.mcuy;
      } else {
        fused_rows += p.mcuy;  // k_fused: one workgroup per MCU row
        fused_images++;
      }
      is_fused[i] = 1;
    } else {
      for (int c = 0; c < in.ncomp; c++) {
        d.plane_off[c] = plane_bytes;
        plane_bytes += AlignUp(uint64_t(d.plane_pitch[c]) * d.plane_rows[c], 256);
      }
      (p.progressive ? pgeneral_rows : general_rows) += p.mcuy;
    }
  }

  // ---- K1p lanes (progressive images): per dependency level, the intervals grouped by scan
  // kind (each group padded to whole waves: the kind is wave-uniform), longest first within a
  // group (a wave lasts as long as its longest lane) ----
  std::vector<uint32_t> &prog_lanes = sc_.prog_lanes;
  prog_lanes.clear();
  uint32_t prog_level_off[257] = {}, fold_off[257] = {}, fold_chunks[257] = {}, wave_off[257] = {};
  bool prog_pipe = false, prog_wave_all = false;
  uint32_t wave_first_end = 0;  // pipelined, large batch: wave list [wave_off[0], here) = first scans
  std::vector<RjFoldJob> &fold_jobs = sc_.fold_jobs;
  const uint32_t nlev = std::min<uint32_t>(prog_levels, 256);
  if (prog_images) {
    // pipelined launch: every interval of the call in one k_prog_wave grid, a refinement scan
    // following its producer scans block by block (progress counters) -- possible when every
    // refinement scan has at most 3 producers (rj_prog_stream.cpp); otherwise level by level
    // (DC and AC-first scans in lanes, refinement waves, a fold per level)
    prog_pipe = prog_pipe_enabled_;
    for (int i = 0; i < n && prog_pipe; i++)
      for (const RjProgScanDev &sc : streams[i]->plan().pscans)
        if (sc.kind == RJ_PK_AC_REFINE && sc.nprod == 0xFF) prog_pipe = false;
    // pipelined layouts: up to ~1280 images every scan goes in one wave grid (each image's scans
    // run side by side); beyond, the AC first scans get a grid of their own ahead of the
    // refinement grid -- with ten waves per image one grid outgrows the chip's wave slots several
    // times over (C5 1080p: 1024 images 111 ms one grid vs 117 ms two; 2048 images 243 vs 200)
    prog_wave_all = prog_pipe && (prog_wave_all_ >= 0 ? prog_wave_all_ != 0 : prog_images <= kProgWaveAllImages);
    // DC scans in lanes (one lane per interval, 64 images per wave) on the side stream in the
    // pipelined layouts too: nothing in the wave grid waits for them, and the wave decoder's
    // scalar chains are what a batch runs out of
    auto in_lanes = [&](uint32_t kind) {
      return prog_pipe ? (prog_dc_lanes_ && (kind == RJ_PK_DC_FIRST || kind == RJ_PK_DC_REFINE))
                       : kind != RJ_PK_AC_REFINE;
    };
    // algorithmic bytes of an interval: destuffed bytes read + what its decode writes (DC first:
    // one halfword per block; DC refinement: one bit per block; AC first: the band's halfwords +
    // the nonzero mask; AC refinement: mask read + one 32-B record per block)
    auto ival_bytes = [](const RjProgScanDev &sc, const RjProgIvalDev &iv) -> uint64_t {
      const uint64_t blocks = uint64_t(iv.nunits) * sc.nblk;
      return iv.dst_len + (sc.kind == RJ_PK_DC_FIRST    ? blocks * 2
                           : sc.kind == RJ_PK_DC_REFINE ? (blocks + 7) / 8
                           : sc.kind == RJ_PK_AC_FIRST  ? blocks * ((sc.se - sc.ss + 1u) * 2u + 8u)
                                                        : blocks * 40u);
    };
    constexpr uint32_t kPB = 2048;  // 64-B length buckets
    std::vector<uint32_t> &bk = sc_.prog_bucket;
    for (uint32_t L = 0; L < nlev; L++) {
      prog_level_off[L] = uint32_t(prog_lanes.size());
      for (uint32_t K = 0; K < 3; K++) {  // AC refinement: waves, below
        if (!in_lanes(K)) continue;
        bk.assign(kPB + 1, 0);
        uint32_t cnt = 0;
        for (int i = 0; i < n; i++) {
          const DecodePlan &p = streams[i]->plan();
          if (!p.progressive) continue;
          for (const RjProgIvalDev &iv : p.pivals) {
            const RjProgScanDev &sc = p.pscans[iv.scan];
            if (sc.level != L || sc.kind != K || (iv.flags & RJ_SEG_MISSING)) continue;
            bk[kPB - 1 - std::min<uint32_t>(iv.dst_len >> 6, kPB - 1)]++;
            cnt++;
          }
        }
        if (cnt == 0) continue;
        for (uint32_t b = 0, cum = 0; b <= kPB; b++) {
          const uint32_t c = bk[b];
          bk[b] = cum;
          cum += c;
        }
        const size_t base = prog_lanes.size();
        prog_lanes.resize(base + AlignUp(cnt, 64), 0xFFFFFFFFu);
        for (int i = 0; i < n; i++) {
          const DecodePlan &p = streams[i]->plan();
          if (!p.progressive) continue;
          const uint32_t g0 = imgs[i].pival_prefix;
          for (uint32_t q = 0; q < p.pivals.size(); q++) {
            const RjProgIvalDev &iv = p.pivals[q];
            const RjProgScanDev &sc = p.pscans[iv.scan];
            if (sc.level != L || sc.kind != K || (iv.flags & RJ_SEG_MISSING)) continue;
            prog_lanes[base + bk[kPB - 1 - std::min<uint32_t>(iv.dst_len >> 6, kPB - 1)]++] = g0 + q;
            timings_.prog_kernel_bytes[0] += ival_bytes(sc, iv);
          }
        }
      }
    }
    prog_level_off[nlev] = uint32_t(prog_lanes.size());
    if (prog_pipe) {
      // the grid's order: any order that lists a scan's producers before it is deadlock-free
      // (workgroups dispatch in order; a waiting wave's producers are resident or done).  When
      // the batch has more intervals than the chip has wave slots, the late ones should be those
      // with slack: the largest component's AC scans first (its refinement chain is the critical
      // path), then the other components' AC scans, then the DC scans; level order within each.
      wave_off[0] = uint32_t(prog_lanes.size());
      // large batches: the first scans in a grid of their own ahead of the refinement grid
      // (phase 0), the rest after (phase 1); small batches: everything in one grid.  Order key
      // (phase, rank, level), counting sort (two passes over the intervals)
      const uint32_t nkeys = 2 * 4 * nlev;
      std::vector<uint32_t> &bucket = sc_.prog_bucket;
      bucket.assign(nkeys + 1, 0);
      std::vector<uint16_t> scan_key;
      auto keys_of = [&](const DecodePlan &p, uint32_t nc) {
        scan_key.resize(p.pscans.size());
        for (size_t q = 0; q < p.pscans.size(); q++) {
          const RjProgScanDev &sc = p.pscans[q];
          uint32_t r = 3;
          if (sc.kind == RJ_PK_AC_FIRST || sc.kind == RJ_PK_AC_REFINE) {
            const uint32_t c = sc.comp[0];
            const uint64_t bc = uint64_t(p.cwblk[c]) * p.chblk[c];
            r = 0;
            for (uint32_t o = 0; o < nc && o < 3; o++) {
              const uint64_t bo = uint64_t(p.cwblk[o]) * p.chblk[o];
              if (bo > bc || (bo == bc && o < c)) r++;
            }
            r = std::min<uint32_t>(r, 2);
          }
          const uint32_t phase = (!prog_wave_all && sc.kind != RJ_PK_AC_FIRST) ? 1u : 0u;
          scan_key[q] = uint16_t((phase * 4 + r) * nlev + std::min<uint32_t>(sc.level, nlev - 1));
        }
      };
      for (int i = 0; i < n; i++) {
        const DecodePlan &p = streams[i]->plan();
        if (!p.progressive) continue;
        keys_of(p, streams[i]->info().ncomp);
        for (const RjProgIvalDev &iv : p.pivals)
          if (!in_lanes(p.pscans[iv.scan].kind)) bucket[scan_key[iv.scan] + 1]++;
      }
      for (uint32_t b = 0; b < nkeys; b++) bucket[b + 1] += bucket[b];
      const uint32_t base = uint32_t(prog_lanes.size());
      wave_first_end = base + bucket[4 * nlev];  // phase 1 starts here
      prog_lanes.resize(base + bucket[nkeys]);
      for (int i = 0; i < n; i++) {
        const DecodePlan &p = streams[i]->plan();
        if (!p.progressive) continue;
        keys_of(p, streams[i]->info().ncomp);
        for (uint32_t q = 0; q < p.pivals.size(); q++) {
          const RjProgIvalDev &iv = p.pivals[q];
          if (in_lanes(p.pscans[iv.scan].kind)) continue;
          // missing intervals too: they report DONE
          prog_lanes[base + bucket[scan_key[iv.scan]]++] = imgs[i].pival_prefix + q;
          if (!(iv.flags & RJ_SEG_MISSING)) timings_.prog_kernel_bytes[1] += ival_bytes(p.pscans[iv.scan], iv);
        }
      }
      if (prog_wave_all) wave_first_end = wave_off[0];
      for (uint32_t L = 1; L < nlev; L++) wave_off[L] = wave_off[0];
    } else {
      // AC refinement intervals (one wave each), per level, after the lane lists
      for (uint32_t L = 0; L < nlev; L++) {
        wave_off[L] = uint32_t(prog_lanes.size());
        for (int i = 0; i < n; i++) {
          const DecodePlan &p = streams[i]->plan();
          if (!p.progressive) continue;
          for (uint32_t q = 0; q < p.pivals.size(); q++) {
            const RjProgIvalDev &iv = p.pivals[q];
            const RjProgScanDev &sc = p.pscans[iv.scan];
            if (sc.level == L && sc.kind == RJ_PK_AC_REFINE && !(iv.flags & RJ_SEG_MISSING)) {
              prog_lanes.push_back(imgs[i].pival_prefix + q);
              timings_.prog_kernel_bytes[1] += ival_bytes(sc, iv);
            }
          }
        }
      }
    }
    wave_off[nlev] = uint32_t(prog_lanes.size());
    // k_prog_fold jobs of every level >= 1: (image, component) pairs some refinement scan of
    // that level covers, every block of the component's dense raster
    fold_jobs.clear();
    // pipelined: one fold over every level after the refinement grid (slot 0)
    for (uint32_t L = prog_pipe ? 0u : 1u; L < (prog_pipe ? 1u : nlev); L++) {
      fold_off[L] = uint32_t(fold_jobs.size());
      uint32_t chunks = 0;
      for (int i = 0; i < n; i++) {
        const DecodePlan &p = streams[i]->plan();
        if (!p.progressive) continue;
        for (uint32_t c = 0; c < streams[i]->info().ncomp; c++) {
          bool hit = false;
          for (const RjProgScanDev &sc : p.pscans) {
            if (!prog_pipe && sc.level != L) continue;
            if (sc.kind == RJ_PK_AC_REFINE && sc.comp[0] == c) hit = true;
            if (sc.kind == RJ_PK_DC_REFINE)
              for (uint32_t q = 0; q < sc.ns; q++) hit = hit || sc.comp[q] == c;
          }
          if (!hit) continue;
          RjFoldJob fj;
          fj.image = uint32_t(i);
          fj.comp = c;
          fj.nblocks = p.wblk[c] * p.hblk[c];
          fj.chunk0 = chunks;
          timings_.prog_kernel_bytes[2] += uint64_t(fj.nblocks) * 256;  // dense block read + written
          chunks += (fj.nblocks + 63) / 64;
          fold_jobs.push_back(fj);
        }
      }
      fold_chunks[L] = chunks;
    }
    fold_off[prog_pipe ? 1u : nlev] = uint32_t(fold_jobs.size());
    timings_.prog_kernel_bytes[2] += prec_total * 8;  // the refinement records
  }

  const auto t_lanes = std::chrono::steady_clock::now();
  // ---- the call's chunk length (rj_device.h rj_chunks_cb): the baseline bytes over one round of
  // the chip's K1 decoder lanes, at least chunk_min_ -- a large batch of short intervals keeps
  // one lane per interval (the lean K1), a restart-less or small call is cut to fill the chip ----
  uint64_t src_total = 0;
  uint32_t src_max = 0;
  for (int i = 0; i < n; i++) {
    const DecodePlan &p = streams[i]->plan();
    src_total += p.src_total;
    src_max = std::max(src_max, p.src_max);
  }
  // (a call whose intervals alone fill half a round keeps them whole below RJ_SPLIT_BYTES: lean
  // K1 with its outlier split)
  const uint64_t round_lanes = uint64_t(cu_count_) * RJ_K1_WG;
  uint64_t cb_fill = std::max<uint64_t>(chunk_min_, (src_total + round_lanes - 1) / round_lanes);
  if (2ull * seg_total >= round_lanes || split_part_) {
    // (a DecodeSplit part keeps its intervals whole too: the other parts' kernels share the chip)
    cb_fill = std::max<uint64_t>(cb_fill, RJ_SPLIT_BYTES / 2);
  } else {
    // the lanes pack into workgroups with padding (an interval's chunks never straddle one):
    // lengthen the chunks until the layout is one workgroup per CU (a second round doubles K1)
    for (int it = 0; it < 8 && cb_fill < (1u << 30); it++) {
      uint64_t lanes = 0, dev = 0;
      for (int i = 0; i < n; i++)
        for (const RjSegDev &sg : streams[i]->plan().segs) {
          const uint32_t nch = rj_chunks_cb(sg.src_len, uint32_t(cb_fill));
          if (nch > RJ_K1_WG) {
            dev += nch;
          } else {
            if (lanes % RJ_K1_WG + nch > RJ_K1_WG) lanes = AlignUp(lanes, RJ_K1_WG);
            lanes += nch;
          }
        }
      const uint64_t wgs = (lanes + RJ_K1_WG - 1) / RJ_K1_WG + (dev + RJ_K1_WG - 1) / RJ_K1_WG;
      if (wgs <= uint64_t(cu_count_)) break;
      cb_fill = cb_fill * wgs / uint64_t(cu_count_) + 16;
    }
  }
  uint32_t chunk_bytes = uint32_t(std::min<uint64_t>(1u << 30, cb_fill));
  // ---- K1 lane layout (rj_device.h RjCoefBuf): one lane per chunk; an interval of at most
  // RJ_K1_WG chunks never straddles a workgroup (padding lanes), longer ones go after them.
  // Common case -- no interval split -- is the identity (lane = interval), nothing uploaded. ----
  // MCU-phase hypotheses per speculative chunk (rj_device.h rj_chunk_lanes) and the chunk length
  // they go with: the most hypotheses (up to the call's largest MCU's block count, RJ_MAX_HYP)
  // for which some chunk length from hyp_chunk_min_ (192 B) up to the call's length above fits
  // one round of the chip's decoder lanes with the workgroup padding, at the shortest such
  // length; 1 otherwise (the length above), and always on the round-3 chunk path (k_entropy,
  // RJ_K1_CHUNK=0).  Measured (profiles/r5_experiments/k1_hyp_chunk_floor_sweep.txt): with six
  // hypotheses one image is fastest at 192 B (the lane's chain is its warm-up, its chunk and a
  // short overlap), sixteen at 384 B (shorter chunks would cost hypotheses)
  uint32_t hyp = 1;
  if (rj_chunks_cb(src_max, chunk_bytes) > 1 && k1_chunk_ && hyp_max_ > 1) {
    uint32_t nblk_max = 1;
    for (int i = 0; i < n; i++) nblk_max = std::max(nblk_max, uint32_t(streams[i]->plan().nblk_mcu));
    auto fits = [&](uint32_t cb, uint32_t H) {
      uint64_t lanes = 0, dev = 0;
      for (int i = 0; i < n; i++)
        for (const RjSegDev &sg : streams[i]->plan().segs) {
          const uint32_t nl = rj_chunk_lanes(rj_chunks_cb(sg.src_len, cb), H);
          if (nl > RJ_K1_WG) {
            dev += nl;
          } else {
            if (lanes % RJ_K1_WG + nl > RJ_K1_WG) lanes = AlignUp(lanes, RJ_K1_WG);
            lanes += nl;
          }
        }
      return (lanes + RJ_K1_WG - 1) / RJ_K1_WG + (dev + RJ_K1_WG - 1) / RJ_K1_WG <= uint64_t(cu_count_);
    };
    // lanes only grow with H and shrink with the chunk length: a call that fills the chip with one
    // hypothesis at its own length (every large call) is rejected by the first test
    // (chunks longer than the length above, for more hypotheses, measured slower from 16 images up:
    // profiles/r5_experiments/k1_hyp_longer_chunks.txt)
    const uint32_t cb_hi = chunk_bytes;
    if (fits(cb_hi, 2))
      for (uint32_t H = std::min<uint32_t>({uint32_t(RJ_MAX_HYP), nblk_max, hyp_max_}); H > 1; H--) {
        if (!fits(cb_hi, H)) continue;
        hyp = H;
        uint32_t cb = std::min(hyp_chunk_min_, chunk_bytes);
        while (cb < cb_hi && !fits(cb, H)) cb += 64;
        chunk_bytes = std::min(cb, cb_hi);
        break;
      }
  }
  timings_.chunk_bytes = chunk_bytes;
  const bool any_split = rj_chunks_cb(src_max, chunk_bytes) > 1;
  timings_.chunk_hyp = hyp;
  std::vector<uint32_t> &seg_lane0 = sc_.seg_lane0, &lane_seg = sc_.lane_seg;
  seg_lane0.clear();
  lane_seg.clear();
  uint32_t lanes_wg = seg_total, split_intervals = 0;
  if (any_split) {
    seg_lane0.resize(seg_total);
    lanes_wg = 0;
    uint32_t gs = 0;
    for (int i = 0; i < n; i++)
      for (const RjSegDev &sg : streams[i]->plan().segs) {
        const uint32_t nch = rj_chunks_cb(sg.src_len, chunk_bytes), nl = rj_chunk_lanes(nch, hyp);
        split_intervals += nch > 1 ? 1u : 0u;
        if (nl <= RJ_K1_WG) {
          if (lanes_wg % RJ_K1_WG + nl > RJ_K1_WG) lanes_wg = uint32_t(AlignUp(lanes_wg, RJ_K1_WG));
          seg_lane0[gs] = lanes_wg;
          lanes_wg += nl;
        } else {
          seg_lane0[gs] = UINT32_MAX;
        }
        gs++;
      }
    lanes_wg = uint32_t(AlignUp(lanes_wg, RJ_K1_WG));
  }
  uint32_t lanes_all = lanes_wg;
  if (any_split) {
    uint32_t gs = 0;
    for (int i = 0; i < n; i++)
      for (const RjSegDev &sg : streams[i]->plan().segs) {
        if (seg_lane0[gs] == UINT32_MAX) {
          seg_lane0[gs] = lanes_all;
          lanes_all += rj_chunk_lanes(rj_chunks_cb(sg.src_len, chunk_bytes), hyp);
        }
        gs++;
      }
    lane_seg.assign(lanes_all, UINT32_MAX);
    gs = 0;
    for (int i = 0; i < n; i++)
      for (const RjSegDev &sg : streams[i]->plan().segs) {
        const uint32_t nl = rj_chunk_lanes(rj_chunks_cb(sg.src_len, chunk_bytes), hyp);
        for (uint32_t q = 0; q < nl; q++) lane_seg[seg_lane0[gs] + q] = gs;
        gs++;
      }
  }
  const uint32_t lanes_dev = lanes_all - lanes_wg;
  // the split intervals' chunk regions, after the images' serial regions (rj_chunk_regions)
  std::vector<unsigned long long> &seg_ent = sc_.seg_ent;
  seg_ent.clear();
  if (any_split) {
    seg_ent.assign(seg_total, 0ull);
    uint64_t at = AlignUp(ent_total, RJ_ENT_GROUP);
    uint32_t gs = 0;
    for (int i = 0; i < n; i++)
      for (const RjSegDev &sg : streams[i]->plan().segs) {
        const uint32_t nch = rj_chunks_cb(sg.src_len, chunk_bytes);
        if (nch > 1) {
          seg_ent[gs] = at;
          at += rj_chunk_regions(sg.src_len, nch, hyp);
        }
        gs++;
      }
    ent_total = at;
  }

  // ---- lean K1 (rj_huff.hip): when every baseline image of the call is a "row" image (each
  // restart interval inside one MCU row) and no interval is split, K1 writes raw entries and K2
  // restores the DC predictions ----
  bool lean = !any_split && seg_total > 0;
  for (int i = 0; i < n && lean; i++) {
    const DecodePlan &p = streams[i]->plan();
    if (p.progressive) continue;
    const uint32_t ri = streams[i]->info().restart_interval;
    lean = ri > 0 && p.mcux % ri == 0 && p.nblk_mcu <= RJ_MAX_BLK_MCU;
  }
  if (lean)
    for (int i = 0; i < n; i++) imgs[i].dc_diff = streams[i]->plan().progressive ? 0u : 1u;
  timings_.lean_k1 = lean ? 1u : 0u;
  // ---- otherwise K1 is the chunk-lane kernel on the lean machinery (rj_huff.hip k_huff_chunk:
  // absolute DC entries, rj_entropy.hip's records / resolution / serial fallback) ----
  bool hc = !lean && k1_chunk_ && seg_total > 0;
  for (int i = 0; i < n && hc; i++) hc = streams[i]->plan().progressive || streams[i]->plan().nblk_mcu <= RJ_MAX_BLK_MCU;
  timings_.chunk_k1 = hc ? 1u : 0u;

  // ---- non-resident bitstreams: runs of streams whose ECS sit next to each other in the
  // parse-time pinned arena (rj_pinned.h) go up with one DMA per run, straight from the arena;
  // the device staging mirrors each run (gaps included).  Streams without a pinned copy follow
  // in the copy space, filled by the host threads below. ----
  std::vector<PinRun> &pin_runs = sc_.pin_runs;
  pin_runs.clear();
  uint64_t pin_bytes = 0;
  {
    constexpr uint64_t kMaxGap = 64u << 10;  // bytes between two slots a run may carry along
    for (int i = 0; i < n; i++) {
      if (stage_off[i] == UINT64_MAX) continue;
      const uint8_t *hp = streams[i]->pinned_ecs();
      if (hp == nullptr) continue;
      const uint64_t len = uint64_t(streams[i]->info().ecs_size) + 16;
      const PinnedChunk *ch = streams[i]->pinned_chunk();
      if (!pin_runs.empty() && pin_runs.back().chunk == ch && hp >= pin_runs.back().host &&
          uint64_t(hp - pin_runs.back().host) <= pin_runs.back().len + kMaxGap) {
        PinRun &r = pin_runs.back();
        r.len = std::max<uint64_t>(r.len, uint64_t(hp - r.host) + len);
      } else {
        pin_runs.push_back(PinRun{hp, len, 0, ch});
      }
      ecs_off[i] = uint64_t(hp - pin_runs.back().host) | (uint64_t(pin_runs.size() - 1) << 40);  // run-relative for now
    }
    for (PinRun &r : pin_runs) {
      r.dev = pin_bytes;
      pin_bytes += AlignUp(r.len, 256);
    }
    for (int i = 0; i < n; i++) {
      if (stage_off[i] == UINT64_MAX) continue;
      if (streams[i]->pinned_ecs() != nullptr)
        ecs_off[i] = pin_runs[ecs_off[i] >> 40].dev + (ecs_off[i] & ((1ull << 40) - 1));
      else
        ecs_off[i] += pin_bytes;
    }
    ecs_stage_bytes = pin_bytes + ecs_copy_bytes;
  }

  // ---- one pinned staging blob, uploaded in two parts: A (descriptors, tables, non-resident
  // bitstreams) before K0; B (K1 lane order, K2 row lists) after K0 is launched -- the lane
  // sort and row classes below are host work that then runs while K0 executes. ----
  const bool sorted = !any_split && sort_lanes_ && (seg_total >= 256 || seg_total >= pipe_min_ || lean);
  int ngroups = 1;
  // the lean K1 runs as one launch, longest intervals first (K2 after it): its workgroups then
  // end close together, and the pipelined split did not overlap K1 with K2 in measurements
  const int groups_wanted = (lean && !pipe_groups_set_) ? 1 : pipe_groups_;
  if (sorted && groups_wanted > 1 && seg_total >= pipe_min_) ngroups = groups_wanted;
  const uint64_t off_imgs = 0;
  const uint64_t off_tabs = AlignUp(off_imgs + n * sizeof(RjImageDev), 256);
  const uint64_t off_jobs = AlignUp(off_tabs + tabs.size() * sizeof(RjTableSet), 256);
  const uint64_t off_rows = AlignUp(off_jobs + std::max<size_t>(jobs.size(), 1) * sizeof(RjJobDev), 256);
  const uint64_t off_grows = AlignUp(off_rows + n * sizeof(uint32_t), 256);
  const uint64_t off_prows = AlignUp(off_grows + n * sizeof(uint32_t), 256);
  const uint64_t off_pgrows = AlignUp(off_prows + n * sizeof(uint32_t), 256);
  const uint64_t off_plane = AlignUp(off_pgrows + n * sizeof(uint32_t), 256);
  const uint64_t off_fold = AlignUp(off_plane + prog_lanes.size() * sizeof(uint32_t), 256);
  const uint64_t off_lean = AlignUp(off_fold + fold_jobs.size() * sizeof(RjFoldJob), 256);
  const uint64_t off_wide = AlignUp(off_lean + ((lean || hc) ? tabs.size() * sizeof(RjLeanTables) : 0), 256);
  // K0's block -> image map: the image holding block 64 k, for k <= ds_total / 64 (+ a sentinel)
  const uint32_t n_dsmap = ds_total / 64u + 2u;
  const uint64_t off_live = AlignUp(off_wide + kWideSites * sizeof(uint32_t), 64);
  const uint64_t off_live_cu = AlignUp(off_live + RJ_LIVE_CTRS * sizeof(uint32_t), 256);
  const uint64_t off_dsmap = AlignUp(off_live_cu + RJ_LIVE_CU_KEYS * sizeof(uint32_t), 256);
  const uint64_t off_stage = AlignUp(off_dsmap + n_dsmap * sizeof(uint32_t), 256);
  const uint64_t blob_a = AlignUp(off_stage + stage_bytes, 256);
  // (a lean launch may split intervals: head + tail lanes, up to 2 per interval + one wave of padding)
  const uint64_t n_lane_seg = any_split ? lane_seg.size() : (sorted ? (lean ? 2ull * seg_total + 64 : seg_total) : 0);
  const uint64_t off_lane_seg = blob_a;
  const uint64_t off_seg_lane0 = AlignUp(off_lane_seg + n_lane_seg * 4, 256);
  const uint64_t off_seg_ent = AlignUp(off_seg_lane0 + uint64_t(seg_lane0.size()) * 4, 256);
  const uint64_t off_row_list = AlignUp(off_seg_ent + uint64_t(seg_ent.size()) * 8, 256);
  // K2's plain launch over the rows in lane order -- longest interval first, the order K1 ran
  // them -- from an explicit (image, row) list (env RJ_K2_LPT=1): every interval one MCU row
  bool k2_lpt = k2_lpt_ && lean && sorted && lpt_ && ngroups == 1 && prog_images == 0 && general_rows == 0 &&
                fused_images == uint32_t(n);
  for (int i = 0; i < n && k2_lpt; i++) k2_lpt = streams[i]->plan().rows_aligned;
  const uint64_t n_row_list = ngroups > 1 ? uint64_t(fused_rows) + general_rows : (k2_lpt ? seg_total : 0);  // upper bound
  const uint64_t blob = AlignUp(off_row_list + n_row_list * sizeof(uint2), 256);
  RJ_CHECK(h_stage_.Ensure(blob));
  RJ_CHECK(d_desc_.Ensure(blob));
  RJ_CHECK(d_destuff_.Ensure(std::max<uint64_t>(destuff_total, 256)));
  RJ_CHECK(d_piece_.Ensure(std::max<uint64_t>(uint64_t(lanes_all) * sizeof(RjPiece), 256)));
  RJ_CHECK(d_rec_.Ensure(std::max<uint64_t>(uint64_t(lanes_all) * RJ_MAX_RECORDS * sizeof(RjRecord), 256)));
  RJ_CHECK(d_chunkres_.Ensure(std::max<uint64_t>(uint64_t(lanes_all) * sizeof(RjChunkRes), 256)));
  RJ_CHECK(d_fallback_.Ensure(std::max<uint64_t>(uint64_t(seg_total) * 4, 256)));
  RJ_CHECK(d_entries_.Ensure((ent_total + RJ_ENT_SLACK) * 4 + ent_shift_));
  if (prog_images) {
    RJ_CHECK(d_coef_.Ensure(coef_dw_total * 4));
    RJ_CHECK(d_nz_.Ensure(nz_total * 8));
    RJ_CHECK(d_prec_.Ensure(std::max<uint64_t>(prec_total * 8, 256)));
    RJ_CHECK(d_pprog_.Ensure(std::max<uint64_t>(uint64_t(pival_total + 1) * 4, 256)));  // + error flag
  }
  RjCoefBuf cbuf;
  cbuf.ent = d_entries_.as<uint32_t>() + ent_shift_ / 4;
  cbuf.piece = d_piece_.as<RjPiece>();
  cbuf.rec = d_rec_.as<RjRecord>();
  cbuf.res = d_chunkres_.as<RjChunkRes>();
  cbuf.fallback = d_fallback_.as<uint32_t>();
  cbuf.count = nullptr;
  cbuf.dense = d_coef_.as<uint32_t>();
  cbuf.wide_flag = d_wide_flag_;
  cbuf.piece_shift = 0;
  cbuf.chunk_bytes = chunk_bytes;
  cbuf.hyp = hyp;
  // chunk warm-up (k_huff_chunk): up to half a chunk while the call's lanes leave the chip half
  // idle, an eighth once they fill it (profiles/r4_experiments/k1_chunk_warmup_ab.txt)
  cbuf.warm_shift = 2ull * lanes_all <= uint64_t(cu_count_) * RJ_K1_WG ? 1u : 3u;
  // (RJ_K1_HYP_WARM=0: no warm-up under phase hypotheses -- measured slower: the in-phase
  // hypothesis still needs the warm-up to align its symbols before its records begin,
  // profiles/r5_experiments/k1_hyp_small_calls_warm.txt)
  if (hyp > 1 && !hyp_warm_) cbuf.warm_shift = 31u;
  cbuf.seg_ent = nullptr;  // set with the split layout below
  cbuf.wide_cap = 0;       // set per fix-up site (wide() below)
  if (profiling_) {
    RJ_CHECK(d_count_.Ensure(256));
    cbuf.count = d_count_.as<unsigned long long>();
  }
  // records persist across calls: a per-call epoch (28 bits, never 0) tells this call's apart
  epoch_ = (epoch_ + 1) & 0x0FFFFFFFu;
  if (epoch_ == 0) epoch_ = 1;
  RJ_CHECK(d_planes_.Ensure(std::max<uint64_t>(plane_bytes, 256)));
  // K2 fix-up lists (rows outside the int32 IDCT's exact domain): one slice per K2 launch, the
  // counters zeroed in upload A; capacity = every K2 launch's rows together
  RJ_CHECK(d_wide_.Ensure((uint64_t(fused_rows) + general_rows + pfused_rows + pgeneral_rows + seg_total + 1) *
                          sizeof(uint2)));
  if (!routes_.empty()) {  // routed images write device-local staging at the caller's pitch
    RJ_CHECK(d_route_.Ensure(route_bytes));
    uint8_t *rb = d_route_.as<uint8_t>();
    for (const RouteCopy &rc : routes_) imgs[rc.image].dst[rc.chan] = rb + rc.off;
    for (RjJobDev &j : jobs) {
      if (!routed[j.image]) continue;
      for (const RouteCopy &rc : routes_)
        if (rc.image == j.image && rc.user == j.dst) {
          j.dst = rb + rc.off;
          break;
        }
    }
  }
  uint8_t *h = h_stage_.data();
  uint8_t *dbase = d_desc_.as<uint8_t>();
  if (ecs_stage_bytes) {
    if (ecs_copy_bytes) RJ_CHECK(h_ecs_.Ensure(ecs_copy_bytes));
    RJ_CHECK(d_ecs_.Ensure(ecs_stage_bytes));
  }
  uint8_t *hecs = h_ecs_.data();
  uint8_t *decs = d_ecs_.as<uint8_t>();
  // descriptor pointers (staged tables in blob A, staged bitstreams in the ECS staging)
  auto staged = [&](const DecodePlan &p, uint64_t so, uint64_t &bo, uint64_t &po, uint64_t &vo, uint64_t &to) {
    bo = so + AlignUp(p.segs.size() * sizeof(RjSegDev), 256);
    po = bo + AlignUp(p.ds.size() * sizeof(RjDsBlock), 256);
    vo = po + AlignUp(p.pscans.size() * sizeof(RjProgScanDev), 256);
    to = vo + AlignUp(p.pivals.size() * sizeof(RjProgIvalDev), 256);
  };
  for (int i = 0; i < n; i++) {
    Stream *s = streams[i];
    RjImageDev &d = imgs[i];
    if (stage_off[i] == UINT64_MAX) {
      d.ecs = s->resident.ecs;
      d.segs = s->resident.segs;
      d.ds = s->resident.ds;
      if (s->plan().progressive) {
        d.pscans = s->resident.pscans;
        d.pivals = s->resident.pivals;
        d.ptabs = s->resident.ptabs;
      }
    } else {
      const DecodePlan &p = s->plan();
      const uint64_t so = off_stage + stage_off[i];
      uint64_t bo, po, vo, to;
      staged(p, so, bo, po, vo, to);
      d.segs = reinterpret_cast<const RjSegDev *>(dbase + so);
      d.ds = reinterpret_cast<const RjDsBlock *>(dbase + bo);
      d.ecs = decs + ecs_off[i];
      if (p.progressive) {
        d.pscans = reinterpret_cast<const RjProgScanDev *>(dbase + po);
        d.pivals = reinterpret_cast<const RjProgIvalDev *>(dbase + vo);
        d.ptabs = reinterpret_cast<const RjHuffDev *>(dbase + to);
      }
    }
  }
  if (profiling_) RJ_HIP(hipEventRecord(ev_[0], stream_));
  if (upload_after_ != nullptr) RJ_HIP(hipStreamWaitEvent(stream_, upload_after_, 0));  // DecodeSplit: after the previous part's uploads
  for (const PinRun &r : pin_runs)  // parse-time pinned bitstreams: straight to the device
    RJ_HIP(hipMemcpyAsync(decs + r.dev, r.host, r.len, hipMemcpyHostToDevice, stream_));
  if (stage_bytes || ecs_copy_bytes) {
    // host threads copy the non-resident streams' tables and bitstreams into pinned memory, in
    // chunks of consecutive images (~2 MB of bitstream each); this thread uploads the finished
    // prefix of the staging area in DMA transfers of >= 32 MB (a 285-MB batch in 4-MB transfers
    // ran at ~40 GB/s, in one transfer at 57), so the copies, the DMA and the next chunks'
    // copies overlap
    std::vector<uint32_t> &chunk_img = sc_.chunk_img;  // chunk k: images [chunk_img[k], chunk_img[k + 1])
    chunk_img.clear();
    constexpr uint64_t kChunkBytes = 2ull << 20, kDmaBytes = 32ull << 20;
    uint64_t acc = 0;
    for (int i = 0; i < n; i++) {
      if (stage_off[i] == UINT64_MAX) continue;
      if (chunk_img.empty() || acc >= kChunkBytes) {
        chunk_img.push_back(uint32_t(i));
        acc = 0;
      }
      acc += streams[i]->pinned_ecs() ? 4096u : streams[i]->info().ecs_size;  // pinned: tables only
    }
    chunk_img.push_back(uint32_t(n));
    const int nchunk = int(chunk_img.size()) - 1;
    hipError_t up_err = hipSuccess;
    uint64_t dma_lo = UINT64_MAX, dma_hi = 0;  // staged but not yet uploaded
    pool_.Run(
        nchunk,
        [&](int k) {
          for (uint32_t i = chunk_img[k]; i < chunk_img[k + 1]; i++) {
            if (stage_off[i] == UINT64_MAX) continue;
            const Stream *s = streams[i];
            const DecodePlan &p = s->plan();
            const uint64_t so = off_stage + stage_off[i];
            uint64_t bo, po, vo, to;
            staged(p, so, bo, po, vo, to);
            std::memcpy(h + so, p.segs.data(), p.segs.size() * sizeof(RjSegDev));
            if (!p.ds.empty()) std::memcpy(h + bo, p.ds.data(), p.ds.size() * sizeof(RjDsBlock));
            if (p.progressive) {
              std::memcpy(h + po, p.pscans.data(), p.pscans.size() * sizeof(RjProgScanDev));
              std::memcpy(h + vo, p.pivals.data(), p.pivals.size() * sizeof(RjProgIvalDev));
              if (!p.ptabs.empty()) std::memcpy(h + to, p.ptabs.data(), p.ptabs.size() * sizeof(RjHuffDev));
            }
            if (s->pinned_ecs() == nullptr)
              CopyToStaging(hecs + (ecs_off[i] - pin_bytes), s->info().ecs, s->info().ecs_size);
          }
        },
        [&](int k) {
          uint32_t i0 = chunk_img[k], i1 = chunk_img[k + 1];
          while (i0 < i1 && stage_off[i0] == UINT64_MAX) i0++;
          uint64_t lo = UINT64_MAX, hi = 0;
          for (uint32_t i = i0; i < i1; i++)
            if (stage_off[i] != UINT64_MAX && streams[i]->pinned_ecs() == nullptr) {  // copy space
              lo = std::min(lo, ecs_off[i] - pin_bytes);
              hi = std::max(hi, ecs_off[i] - pin_bytes + streams[i]->info().ecs_size);
            }
          if (hi > lo) {
            dma_lo = std::min(dma_lo, lo);
            dma_hi = std::max(dma_hi, hi);
          }
          if (dma_hi > dma_lo && (dma_hi - dma_lo >= kDmaBytes || k == nchunk - 1) && up_err == hipSuccess) {
            up_err = hipMemcpyAsync(decs + pin_bytes + dma_lo, hecs + dma_lo, dma_hi - dma_lo, hipMemcpyHostToDevice,
                                    stream_);
            dma_lo = UINT64_MAX;
            dma_hi = 0;
          }
        });
    RJ_HIP(up_err);
  }
  std::memcpy(h + off_imgs, imgs.data(), n * sizeof(RjImageDev));
  for (size_t t = 0; t < tabs.size(); t++) std::memcpy(h + off_tabs + t * sizeof(RjTableSet), tabs[t], sizeof(RjTableSet));
  if (lean || hc)
    for (size_t t = 0; t < tabs.size(); t++)
      std::memcpy(h + off_lean + t * sizeof(RjLeanTables), owner_stream[t]->LeanTables(), sizeof(RjLeanTables));
  const RjLeanTables *d_lean = reinterpret_cast<const RjLeanTables *>(dbase + off_lean);
  if (!jobs.empty()) std::memcpy(h + off_jobs, jobs.data(), jobs.size() * sizeof(RjJobDev));
  std::memcpy(h + off_rows, row_prefix.data(), n * sizeof(uint32_t));
  std::memcpy(h + off_grows, grow_prefix.data(), n * sizeof(uint32_t));
  std::memcpy(h + off_prows, prow_prefix.data(), n * sizeof(uint32_t));
  std::memcpy(h + off_pgrows, pgrow_prefix.data(), n * sizeof(uint32_t));
  if (!prog_lanes.empty()) std::memcpy(h + off_plane, prog_lanes.data(), prog_lanes.size() * sizeof(uint32_t));
  if (!fold_jobs.empty()) std::memcpy(h + off_fold, fold_jobs.data(), fold_jobs.size() * sizeof(RjFoldJob));
  const uint32_t *d_rows = reinterpret_cast<const uint32_t *>(dbase + off_rows);
  const uint32_t *d_grows = reinterpret_cast<const uint32_t *>(dbase + off_grows);
  const RjImageDev *d_imgs = reinterpret_cast<const RjImageDev *>(dbase + off_imgs);
  const RjTableSet *d_tabs = reinterpret_cast<const RjTableSet *>(dbase + off_tabs);
  const RjJobDev *d_jobs = reinterpret_cast<const RjJobDev *>(dbase + off_jobs);
  const uint2 *d_row_list = reinterpret_cast<const uint2 *>(dbase + off_row_list);
  const uint32_t *d_lane_seg = reinterpret_cast<const uint32_t *>(dbase + off_lane_seg);
  std::memset(h + off_wide, 0, kWideSites * sizeof(uint32_t));
  std::memset(h + off_live, 0, RJ_LIVE_CTRS * sizeof(uint32_t));
  std::memset(h + off_live_cu, 0, RJ_LIVE_CU_KEYS * sizeof(uint32_t));
  {
    uint32_t *map = reinterpret_cast<uint32_t *>(h + off_dsmap);
    for (uint32_t k = 0; k < n_dsmap; k++) map[k] = uint32_t(n - 1);
    for (int i = 0; i < n; i++) {  // images in block order: image i holds [ds_prefix, next ds_prefix)
      const uint32_t b0 = imgs[i].ds_prefix, b1 = i + 1 < n ? imgs[i + 1].ds_prefix : ds_total;
      for (uint32_t k = (b0 + 63u) / 64u; k * 64u < b1; k++) map[k] = uint32_t(i);
    }
  }
  uint32_t *const d_wide_cnt = reinterpret_cast<uint32_t *>(dbase + off_wide);
  uint64_t wide_used = 0;
  wide_sites_.clear();
  // the next K2 launch's fix-up list: its counter and `rows` slots
  auto wide = [&](uint32_t rows, uint32_t *&cnt, uint2 *&list, bool planes, bool dense) {
    cnt = d_wide_cnt + std::min<int>(int(wide_sites_.size()), kWideSites - 1);
    cbuf.wide_cap = rows;  // the launches that follow (until the next site) append at most this many
    list = d_wide_.as<uint2>() + wide_used;
    wide_used += rows;
    if (rows) wide_sites_.push_back({planes, dense, rows, cnt, list});
  };
  uint32_t *wcnt = nullptr;
  uint2 *wlist = nullptr;

  const auto t_k0 = std::chrono::steady_clock::now();
  RJ_HIP(hipMemcpyAsync(dbase, h, blob_a, hipMemcpyHostToDevice, stream_));
  if (uploaded_) uploaded_();  // DecodeSplit: this part's uploads are enqueued
  if (cbuf.count) RJ_HIP(hipMemsetAsync(cbuf.count, 0, sizeof(unsigned long long), stream_));
  if (profiling_) RJ_HIP(hipEventRecord(ev_[1], stream_));
  RJ_HIP(LaunchDestuff(stream_, d_imgs, n, ds_total, d_destuff_.as<uint8_t>(),
                      reinterpret_cast<const uint32_t *>(dbase + off_dsmap), k0_lds_));
  const uint8_t *k1_src = d_destuff_.as<uint8_t>();
  if (prog_images) {  // progressive images: K1p level by level, then their K2 rows (dense)
    const uint32_t *d_plane = reinterpret_cast<const uint32_t *>(dbase + off_plane);
    if (profiling_) RJ_HIP(hipEventRecord(prog_ev_[0], stream_));
    RJ_HIP(hipMemsetAsync(d_coef_.as<uint32_t>(), 0, coef_dw_total * 4, stream_));
    RJ_HIP(hipMemsetAsync(d_nz_.as<unsigned long long>(), 0, nz_total * 8, stream_));
    if (prec_total) RJ_HIP(hipMemsetAsync(d_prec_.as<unsigned long long>(), 0, prec_total * 8, stream_));
    const RjFoldJob *d_fold = reinterpret_cast<const RjFoldJob *>(dbase + off_fold);
    const bool dbg_lev = profiling_ && Dbg(kDebugProg);
    if (dbg_lev && prog_lev_ev_.size() < nlev + 1) {
      for (size_t q = prog_lev_ev_.size(); q < nlev + 1; q++) {
        hipEvent_t e;
        RJ_HIP(hipEventCreate(&e));
        prog_lev_ev_.push_back(e);
      }
    }
    if (dbg_lev) RJ_HIP(hipEventRecord(prog_lev_ev_[0], stream_));
    // profiling: an event pair around every progressive launch (on the launch's own stream)
    pk_span_.clear();
    uint32_t pk_used = 0;
    if (profiling_) {
      const size_t need = 2 * (3 * size_t(nlev) + 2);
      while (pk_ev_.size() < need) {
        hipEvent_t e;
        RJ_HIP(hipEventCreate(&e));
        pk_ev_.push_back(e);
      }
    }
    auto pk_begin = [&](hipStream_t s) { return profiling_ ? hipEventRecord(pk_ev_[pk_used], s) : hipSuccess; };
    auto pk_end = [&](hipStream_t s, uint32_t kind, uint32_t count) {
      if (!profiling_) return hipSuccess;
      const hipError_t e = hipEventRecord(pk_ev_[pk_used + 1], s);
      if (count) pk_span_.push_back({kind, pk_used, pk_used + 1});
      pk_used += 2;
      return e;
    };
    if (prog_pipe) {
      // side by side: the DC lanes of every level (DC first, then DC refinements) on a second
      // stream, and every AC interval in one k_prog_wave grid (level order, a scan following its
      // producers); one fold over all levels once both are done
      RJ_HIP(hipMemsetAsync(d_pprog_.as<uint32_t>(), 0, uint64_t(pival_total + 1) * 4, stream_));
      // large batch: the first scans' grid (nothing in it waits) before the refinement grid
      if (wave_first_end > wave_off[0]) {
        RJ_HIP(pk_begin(stream_));
        RJ_HIP(LaunchProgressiveWave(stream_, d_imgs, n, d_plane + wave_off[0], wave_first_end - wave_off[0],
                                     d_destuff_.as<uint8_t>(), d_coef_.as<uint32_t>(), d_nz_.as<unsigned long long>(),
                                     d_prec_.as<unsigned long long>(), nullptr, 0u));
        RJ_HIP(pk_end(stream_, 1, wave_first_end - wave_off[0]));
      }
      // (lanes only in the level-by-level layout; the side stream stays for scripts whose
      // DC scans would need lanes)
      const bool side = prog_level_off[nlev] > prog_level_off[0];
      if (side) {
        RJ_HIP(hipEventRecord(prog_join_[0], stream_));
        RJ_HIP(SideStream(pstream_[0]));
        RJ_HIP(hipStreamWaitEvent(pstream_[0], prog_join_[0], 0));
        for (uint32_t L = 0; L < nlev; L++) {
          RJ_HIP(pk_begin(pstream_[0]));
          RJ_HIP(LaunchProgressive(pstream_[0], d_imgs, n, d_plane + prog_level_off[L],
                                   prog_level_off[L + 1] - prog_level_off[L], d_destuff_.as<uint8_t>(),
                                   d_coef_.as<uint32_t>(), d_nz_.as<unsigned long long>(),
                                   d_prec_.as<unsigned long long>()));
          RJ_HIP(pk_end(pstream_[0], 0, prog_level_off[L + 1] - prog_level_off[L]));
        }
        RJ_HIP(hipEventRecord(prog_join_[1], pstream_[0]));
      }
      unsigned long long *wstamps = nullptr;
      if (Dbg(kDebugWaves)) {
        RJ_CHECK(d_wstamp_.Ensure(std::max<uint64_t>(uint64_t(wave_off[nlev] - wave_first_end) * 32, 256)));
        wstamps = d_wstamp_.as<unsigned long long>();
      }
      RJ_HIP(pk_begin(stream_));
      RJ_HIP(LaunchProgressiveWave(stream_, d_imgs, n, d_plane + wave_first_end, wave_off[nlev] - wave_first_end,
                                   d_destuff_.as<uint8_t>(), d_coef_.as<uint32_t>(), d_nz_.as<unsigned long long>(),
                                   d_prec_.as<unsigned long long>(), d_pprog_.as<uint32_t>(), pival_total, wstamps,
                                   (prog_wave_all ? 0u : RJ_WAVE_FIRST_DONE) |
                                       (Dbg(kTestProgGiveUp) ? RJ_WAVE_TEST_GIVEUP : 0u)));
      RJ_HIP(pk_end(stream_, 1, wave_off[nlev] - wave_first_end));
      if (side) RJ_HIP(hipStreamWaitEvent(stream_, prog_join_[1], 0));
      RJ_HIP(pk_begin(stream_));
      RJ_HIP(LaunchProgressiveFold(stream_, d_imgs, d_fold + fold_off[0], fold_off[1] - fold_off[0], fold_chunks[0],
                                   RJ_FOLD_ALL, d_coef_.as<uint32_t>(), d_nz_.as<unsigned long long>(),
                                   d_prec_.as<unsigned long long>()));
      RJ_HIP(pk_end(stream_, 2, fold_chunks[0]));
      if (dbg_lev)
        for (uint32_t L = 1; L <= nlev; L++) RJ_HIP(hipEventRecord(prog_lev_ev_[L], stream_));
    }
    for (uint32_t L = 0; L < nlev && !prog_pipe; L++) {
      RJ_HIP(pk_begin(stream_));
      RJ_HIP(LaunchProgressive(stream_, d_imgs, n, d_plane + prog_level_off[L], prog_level_off[L + 1] - prog_level_off[L],
                               d_destuff_.as<uint8_t>(), d_coef_.as<uint32_t>(), d_nz_.as<unsigned long long>(),
                               d_prec_.as<unsigned long long>()));
      RJ_HIP(pk_end(stream_, 0, prog_level_off[L + 1] - prog_level_off[L]));
      RJ_HIP(pk_begin(stream_));
      RJ_HIP(LaunchProgressiveWave(stream_, d_imgs, n, d_plane + wave_off[L], wave_off[L + 1] - wave_off[L],
                                   d_destuff_.as<uint8_t>(), d_coef_.as<uint32_t>(), d_nz_.as<unsigned long long>(),
                                   d_prec_.as<unsigned long long>(), nullptr, 0u));
      RJ_HIP(pk_end(stream_, 1, wave_off[L + 1] - wave_off[L]));
      if (L >= 1) {
        RJ_HIP(pk_begin(stream_));
        RJ_HIP(LaunchProgressiveFold(stream_, d_imgs, d_fold + fold_off[L], fold_off[L + 1] - fold_off[L], fold_chunks[L],
                                     L, d_coef_.as<uint32_t>(), d_nz_.as<unsigned long long>(),
                                     d_prec_.as<unsigned long long>()));
        RJ_HIP(pk_end(stream_, 2, fold_chunks[L]));
      }
      if (dbg_lev) RJ_HIP(hipEventRecord(prog_lev_ev_[L + 1], stream_));
    }
    if (profiling_) RJ_HIP(hipEventRecord(prog_ev_[1], stream_));
    wide(pfused_rows, wcnt, wlist, false, true);
    RJ_HIP(LaunchRowsDense(stream_, false, d_imgs, n, reinterpret_cast<const uint32_t *>(dbase + off_prows), pfused_rows,
                           cbuf, d_tabs, nullptr, wcnt, wlist));
    wide(pgeneral_rows, wcnt, wlist, true, true);
    RJ_HIP(LaunchRowsDense(stream_, true, d_imgs, n, reinterpret_cast<const uint32_t *>(dbase + off_pgrows),
                           pgeneral_rows, cbuf, d_tabs, d_planes_.as<uint8_t>(), wcnt, wlist));
    if (profiling_) RJ_HIP(hipEventRecord(prog_ev_[2], stream_));
  }
  if (profiling_) RJ_HIP(hipEventRecord(ev_[2], stream_));

  // ---- (host, while K0 runs) lane order: with no interval split K1 is issue-bound and a wave
  // lasts as long as its longest lane, so lanes are sorted by interval length (shortest first;
  // 32-B buckets) -- the lanes of a wave then do about equal work.
  // Pipelined launch: the sorted lanes are cut into `ngroups` classes of equal count; class g's
  // K1 lanes run on stream g, then the K2 rows of class g once K1 of classes 0..g is done, so
  // K2 work overlaps the K1 tail.  A row's class = the latest class among the intervals it
  // touches (a row can span intervals of several classes).  When every interval of every image
  // is exactly one MCU row and all rows take the same K2 path, class g's rows are its lanes'
  // intervals (K2 reads lane_seg); otherwise explicit (image, row) lists are uploaded. ----
  uint32_t lane_off[kMaxPipe + 1] = {}, frow_off[kMaxPipe + 1] = {}, grow_off[kMaxPipe + 1] = {};
  uint32_t class_max[kMaxPipe] = {};  // longest interval (bytes) of each class
  bool rows_from_lanes = false;
  uint32_t len_lanes = 0;  // lanes [0, len_lanes) have their exact length in sc_.lane_len
  bool lanes_desc = false;  // lane order: longest interval first
  if (sorted) {
    constexpr uint32_t kBuckets = 4096;  // 32-B length buckets up to 128 KB
    const bool desc = lpt_ && ngroups == 1;  // one launch: longest intervals first
    lanes_desc = desc;
    static_assert(kBuckets == 4096, "DecodePlan::seg_bucket (FinishSegs)");
    auto bucket = [desc](uint32_t b) { return desc ? kBuckets - 1 - b : b; };
    std::vector<uint32_t> &pos = sc_.bucket_pos;
    pos.assign(kBuckets, 0);
    bool aligned = fused_images == uint32_t(n - int(prog_images)) || fused_images == 0;
    for (int i = 0; i < n && aligned; i++) aligned = streams[i]->plan().progressive || streams[i]->plan().rows_aligned;
    const bool want_pos = ngroups > 1;
    rows_from_lanes = ngroups > 1 && aligned;
    // the lean splits below (longest lanes first) read the intervals' exact lengths in lane order
    const bool want_len = lean && desc && ngroups == 1 && (outlier_split_ || (five_waves_ && split5_t_ > 0.0));
    // a large lean call sorts on the pool: each part of the images counts its buckets, then places
    // its intervals after the earlier parts' (the order is the sequential one)
    // (env RJ_SORT_PAR=1; off by default: the workers' wake-ups made some calls' sort 0.27-0.55 ms
    // against 0.09-0.12 ms, profiles/r6_experiments/sort_par.txt)
    const bool par = sort_par_ && want_len && !want_pos && !rows_from_lanes && !k2_lpt && pool_.threads() > 1 &&
                     seg_total >= 16384;
    const int nparts = par ? std::min(4, pool_.threads()) : 1;
    std::vector<uint32_t> &phist = sc_.part_hist;
    if (par) {
      phist.assign(size_t(nparts) * kBuckets, 0);
      pool_.Run(nparts, [&](int t) {
        uint32_t *H = phist.data() + size_t(t) * kBuckets;
        for (int i = n * t / nparts; i < n * (t + 1) / nparts; i++) {
          const DecodePlan &p = streams[i]->plan();
          if (p.progressive) continue;
          for (const uint16_t b : p.seg_bucket) H[bucket(b)]++;
        }
      }, nullptr);
      for (int t = 0; t < nparts; t++)
        for (uint32_t b = 0; b < kBuckets; b++) pos[b] += phist[size_t(t) * kBuckets + b];
    } else {
      for (int i = 0; i < n; i++) {
        const DecodePlan &p = streams[i]->plan();
        if (p.progressive) continue;  // no K1 intervals, no rows in these launches
        for (const uint16_t b : p.seg_bucket) pos[bucket(b)]++;
      }
    }
    sc_.bucket_cnt.assign(pos.begin(), pos.end());  // (the outlier split counts on it)
    for (uint32_t b = 0, cum = 0; b < kBuckets; b++) {
      const uint32_t c = pos[b];
      pos[b] = cum;
      cum += c;
    }
    lane_seg.resize(seg_total);  // built in cached memory, copied into the pinned blob below
    uint32_t *ls = lane_seg.data();
    std::vector<uint32_t> &seg_pos = sc_.seg_pos;  // pipelined launch: each interval's lane
    if (ngroups > 1) seg_pos.resize(seg_total);
    // rows from lanes: K2 row w of class g is lane lane_off[g] + w's interval, listed as
    // (image, row) in lane order -- K2 then starts each row from its record and the interval's
    // own piece, with no search over the images (rj_fused.hip row_body)
    std::vector<uint2> &row_list = sc_.row_list;
    if (rows_from_lanes || k2_lpt) row_list.resize(seg_total);
    uint2 *rl = (rows_from_lanes || k2_lpt) ? row_list.data() : nullptr;
    uint32_t gs = 0;
    std::vector<uint64_t> &lane_len = sc_.lane_len;
    if (want_len) lane_len.resize(seg_total);
    // only the lanes a split may take (the longest; the splits' own lane budgets below) need theirs
    const int64_t cu = cu_count_;
    len_lanes = uint32_t(std::min<int64_t>(
        seg_total, std::max<int64_t>({int64_t(0), 64 * cu * 2 * (RJ_HL_SPLIT_DEC / 64) - int64_t(seg_total),
                                      64 * 5 * cu - int64_t(seg_total)}) + 128));
    if (par) {
      // part t's intervals of bucket b start after the earlier parts' ones of that bucket
      for (uint32_t b = 0; b < kBuckets; b++) {
        uint32_t at = pos[b];
        for (int t = 0; t < nparts; t++) {
          uint32_t &c = phist[size_t(t) * kBuckets + b];
          const uint32_t cnt = c;
          c = at;
          at += cnt;
        }
      }
      pool_.Run(nparts, [&](int t) {
        uint32_t *P = phist.data() + size_t(t) * kBuckets;
        for (int i = n * t / nparts; i < n * (t + 1) / nparts; i++) {
          const DecodePlan &p = streams[i]->plan();
          uint32_t g = imgs[i].seg_prefix;
          for (size_t q = 0; q < p.segs.size(); q++) {
            const uint32_t l = P[bucket(p.seg_bucket[q])]++;
            ls[l] = g++;
            if (l < len_lanes) lane_len[l] = p.seg_lenblk[q];
          }
        }
      }, nullptr);
    }
    for (int i = 0; i < n && !par; i++) {
      const DecodePlan &p = streams[i]->plan();
      if (want_len) {
        for (size_t q = 0; q < p.segs.size(); q++) {
          const uint32_t l = pos[bucket(p.seg_bucket[q])]++;
          ls[l] = gs++;
          if (l < len_lanes) lane_len[l] = p.seg_lenblk[q];
          if (rl) rl[l] = uint2{uint32_t(i), uint32_t(q)};
        }
      } else if (rl != nullptr || want_pos) {
        uint32_t r = 0;
        for (size_t q = 0; q < p.segs.size(); q++) {
          const uint32_t l = pos[bucket(p.seg_bucket[q])]++;
          ls[l] = gs;
          if (rl) rl[l] = uint2{uint32_t(i), r++};
          if (want_pos) seg_pos[gs] = l;
          gs++;
        }
      } else {  // one launch, no split planning: the lane order only
        for (const uint16_t b : p.seg_bucket) ls[pos[bucket(b)]++] = gs++;
      }
    }
    if (rl) std::memcpy(h + off_row_list, rl, uint64_t(seg_total) * sizeof(uint2));
    for (int g = 0; g <= ngroups; g++) lane_off[g] = uint32_t(uint64_t(seg_total) * g / ngroups);
    if (ngroups > 1) {
      auto class_of = [&](uint32_t l) {  // no division in the per-interval loop
        uint8_t g = 0;
        while (g + 1 < ngroups && l >= lane_off[g + 1]) g++;
        return g;
      };
      if (rows_from_lanes) {
        for (int g = 0; g < ngroups; g++) {  // class g's rows = its lanes
          frow_off[g + 1] = fused_images ? lane_off[g + 1] : 0;
          grow_off[g + 1] = fused_images ? 0 : lane_off[g + 1];
        }
      } else {
        std::vector<uint8_t> &row_group = sc_.row_group;
        row_group.assign(uint64_t(fused_rows) + general_rows, 0);
        uint32_t frow_cnt[kMaxPipe] = {}, grow_cnt[kMaxPipe] = {};
        gs = 0;
        for (int i = 0; i < n; i++) {
          const DecodePlan &p = streams[i]->plan();
          if (p.progressive) continue;
          uint8_t *rg = row_group.data() + (is_fused[i] ? row_prefix[i] : fused_rows + grow_prefix[i]);
          for (const RjSegDev &sg : p.segs) {
            const uint8_t g = class_of(seg_pos[gs++]);
            class_max[g] = std::max(class_max[g], sg.src_len);
            if (sg.mcu_count == 0 || p.mcux == 0) continue;
            const uint32_t r0 = sg.mcu_first / p.mcux;
            const uint32_t r1 = std::min<uint32_t>((sg.mcu_first + sg.mcu_count - 1) / p.mcux, p.mcuy - 1);
            for (uint32_t r = r0; r <= r1; r++) rg[r] = std::max(rg[r], g);
          }
          for (uint32_t r = 0; r < p.mcuy; r++) (is_fused[i] ? frow_cnt : grow_cnt)[rg[r]]++;
        }
        for (int g = 0; g < ngroups; g++) {
          frow_off[g + 1] = frow_off[g] + frow_cnt[g];
          grow_off[g + 1] = grow_off[g] + grow_cnt[g];
        }
        uint32_t fpos[kMaxPipe], gpos[kMaxPipe];
        for (int g = 0; g < ngroups; g++) {
          fpos[g] = frow_off[g];
          gpos[g] = fused_rows + grow_off[g];
        }
        row_list.resize(uint64_t(fused_rows) + general_rows);
        rl = row_list.data();
        for (int i = 0; i < n; i++) {
          const DecodePlan &p = streams[i]->plan();
          if (p.progressive) continue;
          const uint8_t *rg = row_group.data() + (is_fused[i] ? row_prefix[i] : fused_rows + grow_prefix[i]);
          uint32_t *wp = is_fused[i] ? fpos : gpos;
          for (uint32_t r = 0; r < p.mcuy; r++) rl[wp[rg[r]]++] = uint2{uint32_t(i), r};
        }
        std::memcpy(h + off_row_list, rl, row_list.size() * sizeof(uint2));
      }
    }
  }
  // ---- lean outlier split (rj_huff.hip; the default, RJ_SPLIT_OUTLIERS=0 turns it off): the
  // intervals longer than 9/16 of the longest one get a head lane and a tail lane (which starts
  // at rj_split_byte and is joined where the two decoders' MCU starts meet) -- the longest chain
  // then drops to ~9/16 of it -- in a launch that keeps one decoder wave per SIMD; skipped when
  // more than outlier_frac_ of the intervals would split (near-uniform lengths, e.g. C2:
  // splitting nearly everything is slower).  C4's mixed resolutions: 42,376 of
  // 75,350 split, +12 %. ----
  const auto t_sorted = std::chrono::steady_clock::now();
  uint32_t nsplit = 0, nl_split = 0;
  RjHuffSplit hsplit{0, 0};
  // lane j's interval: (destuffed bytes, blocks), gathered by the lane sort
  auto lane_len = [&](uint32_t j) {
    const uint64_t v = sc_.lane_len[j];
    return uint2{uint32_t(v), uint32_t(v >> 32)};
  };
  if (lean && sorted && lanes_desc && ngroups == 1 && !any_split && outlier_split_ && seg_total > 0) {
    // one round of the split grid: two workgroups per CU of RJ_HL_SPLIT_DEC decoder lanes
    const int64_t waves = int64_t(cu_count_) * 2 * (RJ_HL_SPLIT_DEC / 64);
    const int64_t kmax = 64 * waves - int64_t(seg_total);
    uint64_t lim = 0;
    {
      // count the outliers on the lane sort's 32-B length histogram first (longest bucket
      // first); exact lengths only for the lanes the call does split
      const std::vector<uint32_t> &hist = sc_.bucket_cnt;
      const uint32_t nb = uint32_t(hist.size());
      uint32_t k0 = 0;
      while (k0 < nb && hist[k0] == 0) k0++;
      const uint32_t blim = uint32_t(double(nb - 1 - k0) * outlier_t_);
      uint32_t cnt = 0;
      for (uint32_t k = k0; k < nb && nb - 1 - k > blim; k++) cnt += hist[k];
      if (cnt == 0 || double(cnt) > outlier_frac_ * double(seg_total)) lim = UINT64_MAX;  // nothing to split
      else lim = uint64_t(double(lane_len(0).x) * outlier_t_);
    }
    uint64_t cap = 0;
    while (int64_t(nsplit) < kmax && nsplit < seg_total && lim != UINT64_MAX) {
      const uint2 sl = lane_len(nsplit);
      if (sl.x < RJ_SPLIT_MIN_BYTES) break;  // lanes are sorted longest first
      if (sl.x <= lim) break;
      cap = std::max<uint64_t>(cap, rj_group(8ull * (sl.x - rj_split_byte(sl.x)) + sl.y +
                                             uint64_t(RJ_MAX_BLK_MCU) * RJ_ENT_PER_BLOCK + 1));
      nsplit++;
    }
    if (double(nsplit) > outlier_frac_ * double(seg_total)) nsplit = 0;
    if (nsplit > 0) {
      const uint32_t wsplit = (nsplit + 31) / 32;
      nl_split = wsplit * 64 + (seg_total - nsplit);
      std::vector<uint32_t> &l2 = sc_.lane_split;
      l2.assign(nl_split, UINT32_MAX);
      for (uint32_t j = 0; j < nsplit; j++) {
        l2[(j / 32) * 64 + (j % 32)] = lane_seg[j] | RJ_LANE_HEAD;
        l2[(j / 32) * 64 + 32 + (j % 32)] = lane_seg[j] | RJ_LANE_TAIL;
      }
      std::memcpy(l2.data() + uint64_t(wsplit) * 64, lane_seg.data() + nsplit, uint64_t(seg_total - nsplit) * 4);
      hsplit.ent = AlignUp(ent_total, RJ_ENT_GROUP);
      hsplit.cap = cap;
      RJ_CHECK(d_entries_.Ensure((hsplit.ent + uint64_t(wsplit) * 32 * cap + RJ_ENT_SLACK) * 4 + ent_shift_));
      RJ_CHECK(d_piece_.Ensure(2ull * seg_total * sizeof(RjPiece)));
      cbuf.ent = d_entries_.as<uint32_t>() + ent_shift_ / 4;
      cbuf.piece = d_piece_.as<RjPiece>();
      cbuf.piece_shift = 1;  // interval s: pieces 2s (head) and 2s + 1 (tail)
    }
  }
  timings_.lean_split = nsplit;
  // ---- five decoder waves per CU (rj_huff.hip k_huff<RJ_HL_DEC5>): a lean call whose intervals
  // overflow one round of four decoder waves per CU by at most one wave per CU (C2: 69,632
  // intervals on 65,536 lanes) gives the last workgroups -- the shortest intervals of the round --
  // a fifth decoder wave with the overflow (the longest overflow wave beside the shortest round)
  // instead of a second round that starts only when the first workgroups finish.  The longest
  // intervals (above split5_t_ of the longest, while the waves still fit) are decoded by a head and
  // a tail lane in the same launch (32 pairs per wave, first): the chain that sets K1's time is
  // then the longest interval left whole ----
  static_assert(RJ_HL_DEC5 == 256 + 64, "five-wave layout: one overflow wave per workgroup");
  uint32_t nl_five = 0, nsplit5 = 0, nsplit_rows = 0;
  if (lean && sorted && lanes_desc && ngroups == 1 && !any_split && nsplit == 0 && five_waves_) {
    const uint32_t cu = uint32_t(cu_count_);
    const uint64_t round = uint64_t(cu) * 256;
    if (seg_total > round && seg_total <= uint64_t(cu) * RJ_HL_DEC5) {
      uint32_t ns = 0;
      uint64_t cap = 0;
      if (split5_t_ > 0.0) {
        const double lim = double(lane_len(0).x) * split5_t_;
        while (ns < len_lanes) {
          const uint32_t len = lane_len(ns).x;
          if (len < RJ_SPLIT_MIN_BYTES || double(len) <= lim) break;
          ns++;
        }
        while (ns > 0 && (ns + 31) / 32 + (seg_total - ns + 63) / 64 > 5ull * cu) ns = ns > 32 ? ns - 32 : 0;
        for (uint32_t j = 0; j < ns; j++) {
          const uint2 v = lane_len(j);
          cap = std::max<uint64_t>(cap, rj_group(8ull * (v.x - rj_split_byte(v.x)) + v.y +
                                                 uint64_t(RJ_MAX_BLK_MCU) * RJ_ENT_PER_BLOCK + 1));
        }
      }
      const uint32_t wsp = (ns + 31) / 32, wav = wsp + uint32_t((seg_total - ns + 63) / 64);
      const uint32_t host = wav > 4 * cu ? wav - 4 * cu : 0u;  // workgroups that take a fifth wave
      nl_five = cu * RJ_HL_DEC5;
      // written in place into blob B (its lane list holds 2 x seg_total + 64 >= nl_five words)
      uint32_t *const l5 = reinterpret_cast<uint32_t *>(h + off_lane_seg);
      std::fill(l5, l5 + nl_five, UINT32_MAX);
      uint32_t top = 0;  // global waves holding split pairs: [0, top)
      for (uint32_t k = 0; k < wav; k++) {
        // a workgroup that takes a fifth wave lists its four in reverse (shortest first): the
        // fifth decoder wave shares a SIMD with the first (waves go to the SIMDs in order)
        uint32_t w, q;
        if (k < 4 * cu) {
          w = k / 4;
          q = k % 4;
          if (five_waves_ == 2 && w >= cu - host) q = 3 - q;
        } else {
          w = cu - 1 - (k - 4 * cu);
          q = 4;
        }
        uint32_t *dst = &l5[uint64_t(w) * RJ_HL_DEC5 + q * 64];
        if (k < wsp) {  // 32 heads, then their 32 tails
          for (uint32_t i = 0; i < 32 && k * 32 + i < ns; i++) {
            dst[i] = lane_seg[k * 32 + i] | RJ_LANE_HEAD;
            dst[32 + i] = lane_seg[k * 32 + i] | RJ_LANE_TAIL;
          }
          top = std::max(top, w * 5 + q + 1);
        } else {
          const uint64_t j0 = ns + uint64_t(k - wsp) * 64;
          std::memcpy(dst, &lane_seg[j0], std::min<uint64_t>(64, seg_total - j0) * 4);
        }
      }
      if (ns > 0) {  // tail regions by global wave (rj_huff.hip: pair slot (g >> 6) * 32 + (g & 31))
        nsplit5 = ns;
        // every interval one MCU row: the split intervals' rows go to the split-aware K2 instance
        // as an explicit (image, row) list after the lane list, the rest to the plain instance
        bool row_ivals = true;
        for (int i = 0; i < n && row_ivals; i++) row_ivals = imgs[i].ri_mcus == imgs[i].mcux;
        if (row_ivals && nl_five + 2ull * ns <= n_lane_seg) {
          // the split intervals as a bit set, read back in interval (= image, row) order
          std::vector<uint64_t> &mark = sc_.split_bits;
          mark.assign((uint64_t(seg_total) + 63) / 64, 0ull);
          for (uint32_t j = 0; j < ns; j++) mark[lane_seg[j] >> 6] |= 1ull << (lane_seg[j] & 63);
          uint2 *sr = reinterpret_cast<uint2 *>(l5 + nl_five);
          uint32_t k = 0;
          int i = 0;
          for (size_t w = 0; w < mark.size(); w++)
            for (uint64_t bits = mark[w]; bits != 0; bits &= bits - 1) {
              const uint32_t gs = uint32_t(w * 64 + uint32_t(__builtin_ctzll(bits)));
              while (imgs[i].seg_prefix + imgs[i].nseg <= gs) i++;
              sr[k++] = uint2{uint32_t(i), gs - imgs[i].seg_prefix};
            }
          nsplit_rows = k;
        }
        hsplit.ent = AlignUp(ent_total, RJ_ENT_GROUP);
        hsplit.cap = cap;
        RJ_CHECK(d_entries_.Ensure((hsplit.ent + uint64_t(top) * 32 * cap + RJ_ENT_SLACK) * 4 + ent_shift_));
        RJ_CHECK(d_piece_.Ensure(2ull * seg_total * sizeof(RjPiece)));
        cbuf.ent = d_entries_.as<uint32_t>() + ent_shift_ / 4;
        cbuf.piece = d_piece_.as<RjPiece>();
        cbuf.piece_shift = 1;  // interval s: pieces 2s (head) and 2s + 1 (tail)
        timings_.lean_split = ns;
      }
    }
  }
  timings_.lean_five = nl_five ? 1u : 0u;
  const auto t_five = std::chrono::steady_clock::now();
  if (any_split) {
    std::memcpy(h + off_lane_seg, lane_seg.data(), uint64_t(lane_seg.size()) * 4);
    std::memcpy(h + off_seg_lane0, seg_lane0.data(), uint64_t(seg_lane0.size()) * 4);
    std::memcpy(h + off_seg_ent, seg_ent.data(), uint64_t(seg_ent.size()) * 8);
    cbuf.lane_seg = d_lane_seg;
    cbuf.seg_lane0 = reinterpret_cast<const uint32_t *>(dbase + off_seg_lane0);
    cbuf.seg_ent = reinterpret_cast<const unsigned long long *>(dbase + off_seg_ent);
  } else if (sorted) {  // lanes in length order; pieces stay at the interval's own slot
    if (nsplit) std::memcpy(h + off_lane_seg, sc_.lane_split.data(), uint64_t(nl_split) * 4);
    else if (nl_five) {}  // written in place
    else std::memcpy(h + off_lane_seg, lane_seg.data(), uint64_t(seg_total) * 4);
    cbuf.lane_seg = d_lane_seg;
    cbuf.seg_lane0 = nullptr;
  } else {  // identity layout
    cbuf.lane_seg = nullptr;
    cbuf.seg_lane0 = nullptr;
  }
  // part B: everything up to the row lists, or only the lane list actually used
  const uint64_t blob_b = (!any_split && sorted && ngroups == 1 && !k2_lpt)
                              ? std::min<uint64_t>(blob, AlignUp(off_lane_seg + uint64_t(nsplit ? nl_split : (nl_five ? nl_five + 2 * nsplit_rows : seg_total)) * 4, 256))
                              : blob;
  if (blob_b > blob_a) {
    if (side_b_ && stage_bytes == 0 && ecs_stage_bytes == 0) {
      // on its own stream: the lane lists cross PCIe while K0 runs, and K1 waits for them by an
      // event (behind K0 in the call's stream the copy ran only once K0 was done: ~25 us before K1).
      // Only calls with nothing staged: beside staged bitstreams (DecodeSplit's two halves) the
      // small copy queued behind the other half's upload (host input 126k -> 98-108k images/s)
      RJ_HIP(SideStream(bstream_));
      RJ_HIP(hipMemcpyAsync(dbase + blob_a, h + blob_a, blob_b - blob_a, hipMemcpyHostToDevice, bstream_));
      RJ_HIP(hipEventRecord(bev_, bstream_));
      RJ_HIP(hipStreamWaitEvent(stream_, bev_, 0));
    } else {
      RJ_HIP(hipMemcpyAsync(dbase + blob_a, h + blob_a, blob_b - blob_a, hipMemcpyHostToDevice, stream_));
    }
  }

  const auto t_end = std::chrono::steady_clock::now();
  timings_.host_ms = std::chrono::duration<float, std::milli>(t_end - t_host0).count();
  if (Dbg(kDebugHost))
    fprintf(stderr, "[rj place] entries %p output %p\n", static_cast<void *>(cbuf.ent),
            n ? static_cast<void *>(dst[0].channel[0]) : nullptr);
  if (Dbg(kDebugHost)) {  // development: where the host planning time goes
    auto ms = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
      return std::chrono::duration<double, std::milli>(b - a).count();
    };
    fprintf(stderr,
            "[rj host] validate %.3f dedupe %.3f layout %.3f lanes+blob-A %.3f | after K0: sort %.3f split %.3f "
            "blob-B %.3f ms\n",
            ms(t_host0, t_dedupe), ms(t_dedupe, t_layout), ms(t_layout, t_lanes), ms(t_lanes, t_k0),
            ms(t_k0, t_sorted), ms(t_sorted, t_five), ms(t_five, t_end));
  }
  bool live = false;
  bool place_warm = false, place_timed = false;
  RjLive lv{};
  *reinterpret_cast<volatile uint32_t *>(h_wide_flag_ + 1) = 0;  // a lost live row (never expected)
  if (ngroups > 1) {
    RJ_HIP(hipEventRecord(pev_[kMaxPipe - 1], stream_));  // K0 and upload B done
    for (int g = 0; g < ngroups; g++) {
      if (g < ngroups - 1) RJ_HIP(SideStream(pstream_[g]));
      hipStream_t st = g == ngroups - 1 ? stream_ : pstream_[g];
      if (st != stream_) RJ_HIP(hipStreamWaitEvent(st, pev_[kMaxPipe - 1], 0));
      if (profiling_) RJ_HIP(hipEventRecord(k1s_[g], st));
      if (lean)
        RJ_HIP(LaunchHuffLanes(st, d_imgs, n, lane_off[g], lane_off[g + 1] - lane_off[g], k1_src,
                               d_tabs, d_lean, cbuf));
      else if (hc)
        RJ_HIP(LaunchHuffChunks(st, d_imgs, n, lane_off[g], lane_off[g + 1] - lane_off[g], 0u,
                                d_destuff_.as<uint8_t>(), d_tabs, d_lean, cbuf, epoch_));
      else
        RJ_HIP(LaunchEntropyLanes(st, d_imgs, n, lane_off[g], lane_off[g + 1] - lane_off[g], d_destuff_.as<uint8_t>(),
                                  d_tabs, cbuf, epoch_));
      if (profiling_) RJ_HIP(hipEventRecord(pk1_[g], st));
      RJ_HIP(hipEventRecord(kev_[g], st));
      for (int q = 0; q < g; q++) RJ_HIP(hipStreamWaitEvent(st, kev_[q], 0));  // rows spanning classes
      if (profiling_) RJ_HIP(hipEventRecord(k2s_[g], st));
      if (rows_from_lanes) {
        wide(lane_off[g + 1] - lane_off[g], wcnt, wlist, fused_images == 0, false);
        RJ_HIP(LaunchRows(st, fused_images == 0, d_imgs, n, nullptr, d_row_list + lane_off[g],
                          lane_off[g + 1] - lane_off[g], cbuf, d_tabs, d_planes_.as<uint8_t>(), wcnt, wlist));
      } else {
        wide(frow_off[g + 1] - frow_off[g], wcnt, wlist, false, false);
        RJ_HIP(LaunchRows(st, false, d_imgs, n, d_rows, d_row_list + frow_off[g], frow_off[g + 1] - frow_off[g],
                          cbuf, d_tabs, nullptr, wcnt, wlist));
        wide(grow_off[g + 1] - grow_off[g], wcnt, wlist, true, false);
        RJ_HIP(LaunchRows(st, true, d_imgs, n, d_grows, d_row_list + fused_rows + grow_off[g],
                          grow_off[g + 1] - grow_off[g], cbuf, d_tabs, d_planes_.as<uint8_t>(), wcnt, wlist));
      }
      if (profiling_) RJ_HIP(hipEventRecord(k2e_[g], st));
      if (st != stream_) RJ_HIP(hipEventRecord(pev_[g], st));
    }
    for (int g = 0; g + 1 < ngroups; g++) RJ_HIP(hipStreamWaitEvent(stream_, pev_[g], 0));
  } else {
    if (lean) {  // no split interval: one pass, no resolution / serial stages
      const uint32_t k1_lanes = nsplit ? nl_split : (nl_five ? nl_five : seg_total);
      // live rows (rj_device.h RjLive): K2 beside K1 when every row is one interval of a fused
      // baseline image and the whole K1 grid is resident at once (one workgroup per CU)
      const uint32_t k1_dec = nl_five ? uint32_t(RJ_HL_DEC5) : 256u;
      const uint32_t k1_groups = (k1_lanes + k1_dec - 1) / k1_dec;
      bool rows_one_ival = true;
      for (int i = 0; i < n && rows_one_ival; i++) rows_one_ival = imgs[i].ri_mcus == imgs[i].mcux && imgs[i].mcuy < (1u << RJ_LIVE_ROW_BITS);
      live = live_k2_ && rows_one_ival && nsplit == 0 && (nsplit5 == 0 || nsplit_rows > 0) && prog_images == 0 &&
             general_rows == 0 && fused_rows > 0 && fused_images == uint32_t(n) && k1_groups <= uint32_t(cu_count_) &&
             n < (1 << (32 - RJ_LIVE_ROW_BITS));
      if (live) {
        const size_t had = d_live_.capacity();
        RJ_CHECK(d_live_.Ensure(uint64_t(fused_rows) * sizeof(unsigned long long)));
        if (d_live_.capacity() != had)  // fresh slots: no tag may match an epoch by chance
          RJ_HIP(hipMemsetAsync(d_live_.as<void>(), 0, d_live_.capacity(), stream_));
        lv.slot = d_live_.as<unsigned long long>();
        lv.ctr = reinterpret_cast<uint32_t *>(dbase + off_live);
        lv.cu_busy = reinterpret_cast<uint32_t *>(dbase + off_live_cu);
        lv.epoch = epoch_;
        lv.k1_groups = live_test_giveup_ ? 0xFFFFFFFFu : k1_groups;
        lv.k1_waves = k1_groups * (k1_dec / 64u);
        lv.rows = fused_rows;
        RJ_HIP(hipEventRecord(live_ev_[0], stream_));  // descriptors and lane lists uploaded, K0 done
        RJ_HIP(SideStream(lstream_, true));
        RJ_HIP(hipStreamWaitEvent(lstream_, live_ev_[0], 0));
      }
      // entry-buffer placement search (rj_decoder.h): a large call times K1 + K2 while it runs.
      // Resident bitstreams only: a staged call's time is its upload's, and its allocations and
      // frees (which wait for the device) would stall DecodeSplit's other half
      const bool place_call = place_tune_ && !live && fused_rows >= kPlaceMinRows && stage_bytes == 0 &&
                              ecs_stage_bytes == 0;
      place_warm = place_call && place_state_ == 0;
      place_timed = place_call && place_state_ >= 1;
      if (place_timed) RJ_HIP(hipEventRecord(place_ev_[0], stream_));
      RJ_HIP(LaunchHuffLanes(stream_, d_imgs, n, 0u, k1_lanes, k1_src, d_tabs, d_lean, cbuf, k1_solo_lds_,
                             (nsplit || nsplit5) ? &hsplit : nullptr, nl_five != 0, live ? &lv : nullptr));
      if (live) {
        wide(fused_rows, wcnt, wlist, false, false);  // one list: the live, rest and split launches decode disjoint rows
        if (profiling_) RJ_HIP(hipEventRecord(live_t_[0], lstream_));
        RJ_HIP(LaunchRowsLive(lstream_, d_imgs, n, lv, cbuf, d_tabs, wcnt, wlist, live_lds_));
        if (profiling_) RJ_HIP(hipEventRecord(live_t_[1], lstream_));
        RJ_HIP(hipEventRecord(live_ev_[1], lstream_));
      }
      if (profiling_) RJ_HIP(hipEventRecord(ev_[6], stream_));
      if (profiling_) RJ_HIP(hipEventRecord(ev_[7], stream_));
    } else {
      for (int stage = 0; stage < 3; stage++) {
        if (stage == 0 && hc)
          RJ_HIP(LaunchHuffChunks(stream_, d_imgs, n, 0u, lanes_wg, lanes_dev, d_destuff_.as<uint8_t>(), d_tabs,
                                  d_lean, cbuf, epoch_));
        else
          RJ_HIP(LaunchEntropy(stream_, stage, d_imgs, n, lanes_wg, lanes_dev, seg_total, d_destuff_.as<uint8_t>(),
                               d_tabs, cbuf, epoch_));
        if (profiling_ && stage < 2) RJ_HIP(hipEventRecord(ev_[6 + stage], stream_));
      }
    }
    if (profiling_) RJ_HIP(hipEventRecord(ev_[3], stream_));
    const uint2 *split_rows = nsplit_rows ? reinterpret_cast<const uint2 *>(dbase + off_lane_seg + uint64_t(nl_five) * 4) : nullptr;
    if (live) {  // the published rows no live ticket took, the synced split rows, then join the live K2
      if (profiling_) RJ_HIP(hipEventRecord(live_t_[2], stream_));
      RJ_HIP(LaunchRowsRest(stream_, d_imgs, n, lv, cbuf, d_tabs, wcnt, wlist));
      RJ_HIP(LaunchRowsSplit(stream_, d_imgs, n, split_rows, nsplit_rows, cbuf, d_tabs, wcnt, wlist));
      if (profiling_) RJ_HIP(hipEventRecord(live_t_[3], stream_));
      RJ_HIP(hipStreamWaitEvent(stream_, live_ev_[1], 0));
    } else {
      wide(fused_rows, wcnt, wlist, false, false);
      // the split rows' launch beside the plain one, on the side stream (both after K1; one fix-up
      // list, appended atomically): each fills the other's tail (env RJ_K2_SPLIT_SIDE=1; off by default,
      // profiles/r6_experiments/k2_split_side_ab.txt)
      const bool split_side = k2_split_side_ && nsplit_rows > 0 && cbuf.piece_shift != 0;
      if (split_side) {
        RJ_HIP(SideStream(bstream_));
        RJ_HIP(hipEventRecord(kfork_ev_, stream_));
        RJ_HIP(hipStreamWaitEvent(bstream_, kfork_ev_, 0));
      }
#ifndef RJ_EXP_SKIP_K2  // timing build: K0 + K1 only (the output is not written)
      RJ_HIP(LaunchRows(stream_, false, d_imgs, n, k2_lpt ? nullptr : d_rows, k2_lpt ? d_row_list : nullptr, fused_rows,
                        cbuf, d_tabs, nullptr, wcnt, wlist, split_rows, nsplit_rows, split_side ? bstream_ : nullptr));
#endif
      if (split_side) {
        RJ_HIP(hipEventRecord(kjoin_ev_, bstream_));
        RJ_HIP(hipStreamWaitEvent(stream_, kjoin_ev_, 0));
      }
      if (place_timed) RJ_HIP(hipEventRecord(place_ev_[1], stream_));
    }
    wide(general_rows, wcnt, wlist, true, false);
    RJ_HIP(LaunchRows(stream_, true, d_imgs, n, d_grows, nullptr, general_rows, cbuf, d_tabs,
                      d_planes_.as<uint8_t>(), wcnt, wlist));
  }
  if (profiling_) RJ_HIP(hipEventRecord(ev_[4], stream_));
  RJ_HIP(LaunchOutputJobs(stream_, d_imgs, d_jobs, int(jobs.size()), rows_total, d_planes_.as<uint8_t>()));
  if (profiling_) RJ_HIP(hipEventRecord(ev_[5], stream_));
  for (const RouteCopy &rc : routes_)  // to the caller's device / host memory
    RJ_HIP(hipMemcpy2DAsync(rc.user, rc.pitch, d_route_.as<uint8_t>() + rc.off, rc.pitch, rc.row_bytes, rc.rows,
                            hipMemcpyDefault, stream_));
  RJ_HIP(WaitCall());
  dbg_synced_ = std::chrono::steady_clock::now();
  if (live && *reinterpret_cast<volatile uint32_t *>(h_wide_flag_ + 1)) {
    // a live K2 workgroup gave up on its row (never expected; rj_fused.hip live_claim): decode
    // every row again in stream order, then redo the output stage -- all idempotent
    *reinterpret_cast<volatile uint32_t *>(h_wide_flag_ + 1) = 0;
    RJ_ERR("live rows: a row was not published in time; the call's rows are decoded again");
    wide(fused_rows, wcnt, wlist, false, false);
    RJ_HIP(LaunchRows(stream_, false, d_imgs, n, d_rows, nullptr, fused_rows, cbuf, d_tabs, nullptr, wcnt, wlist,
                      nsplit_rows ? reinterpret_cast<const uint2 *>(dbase + off_lane_seg + uint64_t(nl_five) * 4) : nullptr,
                      nsplit_rows));
    for (const RouteCopy &rc : routes_)
      RJ_HIP(hipMemcpy2DAsync(rc.user, rc.pitch, d_route_.as<uint8_t>() + rc.off, rc.pitch, rc.row_bytes, rc.rows,
                              hipMemcpyDefault, stream_));
    RJ_HIP(hipStreamSynchronize(stream_));
  }
  timings_.wide_rows = 0;
  if (*reinterpret_cast<volatile uint32_t *>(h_wide_flag_)) {
    // rows outside the int32 IDCT's exact domain (corrupt data, large quantisers): decode them
    // again in 64-bit, then redo the output jobs (general rows) and routed copies, all idempotent
    *reinterpret_cast<volatile uint32_t *>(h_wide_flag_) = 0;
    uint32_t wc[kWideSites];
    RJ_HIP(hipMemcpy(wc, d_wide_cnt, sizeof(wc), hipMemcpyDeviceToHost));
    for (int k = 0; k < kWideSites; k++) timings_.wide_rows += wc[k];
    for (const WideSite &ws : wide_sites_)
      RJ_HIP(LaunchRowsFix(stream_, ws.planes, ws.dense, d_imgs, n, cbuf, d_tabs,
                           ws.planes ? d_planes_.as<uint8_t>() : nullptr, ws.cnt, ws.list, ws.cap));
    RJ_HIP(LaunchOutputJobs(stream_, d_imgs, d_jobs, int(jobs.size()), rows_total, d_planes_.as<uint8_t>()));
    for (const RouteCopy &rc : routes_)
      RJ_HIP(hipMemcpy2DAsync(rc.user, rc.pitch, d_route_.as<uint8_t>() + rc.off, rc.pitch, rc.row_bytes, rc.rows,
                              hipMemcpyDefault, stream_));
    RJ_HIP(hipStreamSynchronize(stream_));
  }
  // (after every launch that reads this call's entries: the search may free an entry buffer)
  if (place_warm && ++place_warm_ >= 2) place_state_ = 1;
  if (place_timed) {
    float ms = 0.f;
    RJ_HIP(hipEventElapsedTime(&ms, place_ev_[0], place_ev_[1]));
    PlaceStep(ms);
  }
  for (int k = 0; k < 4; k++) timings_.place_ms[k] = k < kPlaceCands ? place_ms_[k] : 0.f;
  timings_.place_tried = place_state_ < 0 ? uint32_t(place_cands_) : uint32_t(std::max(0, place_state_ - 1));
  timings_.place_pick = place_state_ < 0 ? place_best_ : -1;
  if (prog_images && prog_pipe) {  // a refinement wave that gave up waiting (never expected)
    uint32_t err = 0;
    RJ_HIP(hipMemcpy(&err, d_pprog_.as<uint32_t>() + pival_total, 4, hipMemcpyDeviceToHost));
    if (err) {
      RJ_ERR("progressive refinement: a producer did not report progress");
      return kExecutionFailed;
    }
    if (Dbg(kDebugWaves)) {  // per scan of the batch's first image layout: wave timing
      const uint32_t nw = wave_off[nlev] - wave_first_end;
      std::vector<unsigned long long> st(size_t(nw) * 4);
      RJ_HIP(hipMemcpy(st.data(), d_wstamp_.as<unsigned long long>(), st.size() * 8, hipMemcpyDeviceToHost));
      unsigned long long t0 = ~0ull;
      for (uint32_t w = 0; w < nw; w++) t0 = std::min(t0, st[4 * w]);
      struct Acc {
        double start = 0, ready = 0, end = 0, maxend = 0, nwin = 0, nstep = 0;
        uint32_t cnt = 0;
      };
      std::vector<Acc> acc(256);
      for (uint32_t w = 0; w < nw; w++) {
        const uint32_t gi = prog_lanes[wave_first_end + w];
        int i = 0;
        while (i + 1 < n && imgs[i + 1].pival_prefix <= gi) i++;
        const uint32_t scan = streams[i]->plan().pivals[gi - imgs[i].pival_prefix].scan & 255u;
        Acc &a = acc[scan];
        const double us = 0.01;  // wall_clock64: 100 MHz
        a.start += (st[4 * w] - t0) * us;
        a.ready += (st[4 * w + 1] - t0) * us;
        a.end += (st[4 * w + 2] - t0) * us;
        a.maxend = std::max(a.maxend, (st[4 * w + 2] - t0) * us);
        a.nwin += double(st[4 * w + 3] >> 32);
        a.nstep += double(st[4 * w + 3] & 0xFFFFFFFFu);
        a.cnt++;
      }
      for (uint32_t q = 0; q < 256; q++)
        if (acc[q].cnt)
          fprintf(stderr,
                  "[rj waves] scan %2u: %5u waves, mean start %8.0f us, ready %8.0f, end %8.0f, max end %8.0f, "
                  "windows %9.0f, steps %9.0f\n",
                  q, acc[q].cnt, acc[q].start / acc[q].cnt, acc[q].ready / acc[q].cnt, acc[q].end / acc[q].cnt,
                  acc[q].maxend, acc[q].nwin / acc[q].cnt, acc[q].nstep / acc[q].cnt);
    }
  }
#ifdef RJ_EXP_STAMPS
  if (Dbg(kDebugStamps)) DumpRowStamps();
#endif
#ifdef RJ_HL_STAMPS
  if (Dbg(kDebugStamps)) DumpHuffStamps();
#endif

  if (nsplit && n == 1 && Dbg(kDebugK1Pieces)) {  // development: every interval's pieces (split launch)
    std::vector<RjPiece> pc(2ull * seg_total);
    RJ_HIP(hipMemcpy(pc.data(), d_piece_.as<RjPiece>(), pc.size() * sizeof(RjPiece), hipMemcpyDeviceToHost));
    for (uint32_t q = 0; q < seg_total; q++) {
      const RjPiece &a = pc[2 * q], &t = pc[2 * q + 1];
      const RjSegDev &sg = streams[0]->plan().segs[q];
      fprintf(stderr, "[K1 split] seg %u dst_len %u flags %u: npieces %u head n %u", q, sg.dst_len, sg.flags, a.npieces,
              a.nblk);
      if (a.npieces == 2) fprintf(stderr, " | tail first %u n %u skip %u ent+%llu", t.first_blk, t.nblk, t.npieces,
                                  (unsigned long long)(t.ent - hsplit.ent));
      fprintf(stderr, "\n");
    }
  }
  timings_.images = uint32_t(n);
  timings_.intervals = seg_total;
  timings_.chunks = lanes_all;
  timings_.split_intervals = split_intervals;
  timings_.pipe_groups = uint32_t(ngroups);
  timings_.pipe_lane_rows = rows_from_lanes ? 1u : 0u;
  timings_.ecs_bytes = ecs_bytes;
  timings_.coef_bytes = coef_blocks * 128;  // dense-equivalent; the sparse bytes are data-dependent
  timings_.output_bytes = out_bytes;
  timings_.fused_images = fused_images;
  timings_.routed_images = 0;
  for (int i = 0; i < n; i++) timings_.routed_images += routed[i];
  timings_.prog_images = prog_images;
  timings_.prog_intervals = pival_total;
  timings_.prog_levels = prog_levels;
  timings_.prog_coef_bytes = coef_dw_total * 4;
  if (profiling_) {
    float ms[5];
    RJ_HIP(hipEventElapsedTime(&ms[0], ev_[0], ev_[1]));
    RJ_HIP(hipEventElapsedTime(&ms[1], ev_[1], ev_[2]));
    RJ_HIP(hipEventElapsedTime(&ms[4], ev_[4], ev_[5]));
    RJ_HIP(hipEventElapsedTime(&timings_.total_ms, ev_[0], ev_[5]));
    if (ngroups > 1) {  // K1 ends with the last class; K2 of the earlier classes overlaps it
      float k1 = 0, k12 = 0;
      for (int g = 0; g < ngroups; g++) {
        float t = 0;
        RJ_HIP(hipEventElapsedTime(&t, ev_[2], pk1_[g]));
        k1 = std::max(k1, t);
      }
      RJ_HIP(hipEventElapsedTime(&k12, ev_[2], ev_[4]));
      if (Dbg(kDebugK1)) {
        float prev = 0;
        for (int g = 0; g < ngroups; g++) {
          float t = 0, t1s = 0, t2s = 0, t2e = 0;
          RJ_HIP(hipEventElapsedTime(&t, ev_[2], pk1_[g]));
          RJ_HIP(hipEventElapsedTime(&t1s, ev_[2], k1s_[g]));
          RJ_HIP(hipEventElapsedTime(&t2s, ev_[2], k2s_[g]));
          RJ_HIP(hipEventElapsedTime(&t2e, ev_[2], k2e_[g]));
          fprintf(stderr, "[rj] class %d: %u lanes, max %u B, K1 %.3f..%.3f ms (+%.3f), K2 %.3f..%.3f ms\n", g,
                  lane_off[g + 1] - lane_off[g], class_max[g], t1s, t, t - prev, t2s, t2e);
          prev = t;
        }
      }
      ms[2] = k1;
      ms[3] = k12 - k1;
      timings_.entropy_chunks_ms = k1;
      for (int g = 0; g < ngroups; g++) {
        float a = 0, b = 0;
        RJ_HIP(hipEventElapsedTime(&a, k1s_[g], pk1_[g]));
        RJ_HIP(hipEventElapsedTime(&b, k2s_[g], k2e_[g]));
        timings_.k1_launch_ms_sum += a;
        timings_.k2_launch_ms_sum += b;
        timings_.k1_launches += lane_off[g + 1] > lane_off[g] ? 1u : 0u;
        timings_.k2_launches += (frow_off[g + 1] > frow_off[g] ? 1u : 0u) + (grow_off[g + 1] > grow_off[g] ? 1u : 0u);
      }
    } else {
      RJ_HIP(hipEventElapsedTime(&ms[2], ev_[2], ev_[3]));
      RJ_HIP(hipEventElapsedTime(&ms[3], ev_[3], ev_[4]));
      RJ_HIP(hipEventElapsedTime(&timings_.entropy_chunks_ms, ev_[2], ev_[6]));
      RJ_HIP(hipEventElapsedTime(&timings_.entropy_resolve_ms, ev_[6], ev_[7]));
      RJ_HIP(hipEventElapsedTime(&timings_.entropy_serial_ms, ev_[7], ev_[3]));
      timings_.k1_launch_ms_sum = timings_.entropy_chunks_ms;
      timings_.k1_launches = (lanes_wg ? 1u : 0u) + (lanes_dev ? 1u : 0u);
      timings_.k2_launch_ms_sum = ms[3];
      // (a split call's fused rows run as two launches, plain then split-aware, counted as one:
      // together they are the K2 of the batch, and their rocprofv3 averages add up to it)
      timings_.k2_launches = (fused_rows ? 1u : 0u) + (general_rows ? 1u : 0u);
      if (!lean) {  // (the lean launch has no resolution: the flags are another call's)
        std::vector<uint32_t> fb(seg_total);
        RJ_HIP(hipMemcpy(fb.data(), d_fallback_.as<uint32_t>(), fb.size() * 4, hipMemcpyDeviceToHost));
        for (uint32_t f : fb) timings_.serial_fallbacks += f ? 1u : 0u;
      }
    }
    if (prog_images) {
      RJ_HIP(hipEventElapsedTime(&timings_.prog_entropy_ms, prog_ev_[0], prog_ev_[1]));
      RJ_HIP(hipEventElapsedTime(&timings_.prog_rows_ms, prog_ev_[1], prog_ev_[2]));
      RJ_HIP(hipEventElapsedTime(&timings_.destuff_ms, ev_[1], prog_ev_[0]));  // K0 alone
      for (const ProgSpan &sp : pk_span_) {
        float t = 0;
        RJ_HIP(hipEventElapsedTime(&t, pk_ev_[sp.e0], pk_ev_[sp.e1]));
        timings_.prog_kernel_ms[sp.kind] += t;
        timings_.prog_kernel_launches[sp.kind]++;
      }
      if (Dbg(kDebugProg) && prog_lev_ev_.size() >= nlev + 1) {
        for (uint32_t L = 0; L < nlev; L++) {
          float t = 0;
          RJ_HIP(hipEventElapsedTime(&t, prog_lev_ev_[L], prog_lev_ev_[L + 1]));
          fprintf(stderr, "[rj prog] level %u: %u lanes, %.3f ms\n", L, prog_level_off[L + 1] - prog_level_off[L], t);
        }
      }
    }
    timings_.live = live ? 1u : 0u;
    timings_.live_rows = timings_.rest_rows = 0;
    timings_.live_ms = timings_.rest_ms = 0.0f;
    if (live) {
      uint32_t c[RJ_LIVE_CTRS];
      RJ_HIP(hipMemcpy(c, lv.ctr, sizeof(c), hipMemcpyDeviceToHost));
      const uint32_t pub = std::min(c[RJ_LIVE_RESERVED], lv.rows);
      timings_.live_rows = std::min(c[RJ_LIVE_FINAL], pub);
      timings_.rest_rows = pub - timings_.live_rows;
      timings_.live_pad = c[RJ_LIVE_GIVEUP];
      RJ_HIP(hipEventElapsedTime(&timings_.live_ms, live_t_[0], live_t_[1]));
      RJ_HIP(hipEventElapsedTime(&timings_.rest_ms, live_t_[2], live_t_[3]));
    }
    unsigned long long cnt = 0;
    RJ_HIP(hipMemcpy(&cnt, cbuf.count, sizeof(cnt), hipMemcpyDeviceToHost));
    timings_.entry_bytes = cnt * 4;
    timings_.h2d_ms = ms[0];
    if (!prog_images) timings_.destuff_ms = ms[1];
    timings_.huffman_ms = ms[2];
    timings_.idct_ms = ms[3];
    timings_.output_ms = ms[4];
    if (Dbg(kDebugK1)) {  // development diagnostics of the chunked decode
      std::vector<RjChunkRes> cr(lanes_all);
      RJ_HIP(hipMemcpy(cr.data(), d_chunkres_.as<RjChunkRes>(), cr.size() * sizeof(RjChunkRes), hipMemcpyDeviceToHost));
      double sum_ov = 0, sum_it = 0;
      uint32_t nsync = 0, ndone = 0, nfail = 0, max_ov = 0, max_it = 0;
      uint32_t hist[8] = {};
      for (const RjChunkRes &r : cr) {
        if (r.status == RJ_CHUNK_SYNC) {
          nsync++;
          const uint32_t ov = r.pad[0] - r.pad[1];
          sum_ov += ov;
          max_ov = std::max(max_ov, ov);
          int h = 0;
          while (h < 7 && (256u << h) <= ov) h++;
          hist[h]++;
        } else if (r.status == RJ_CHUNK_DONE) {
          ndone++;
        } else if (r.status == RJ_CHUNK_FAIL) {
          nfail++;
        }
        if (r.status) { sum_it += r.pad[2]; max_it = std::max(max_it, r.pad[2]); }
      }
      fprintf(stderr, "[K1] sync %u done %u fail %u | overlap bits mean %.0f max %u | hist(<256<<h):", nsync, ndone,
              nfail, nsync ? sum_ov / nsync : 0.0, max_ov);
      for (int h = 0; h < 8; h++) fprintf(stderr, " %u", hist[h]);
      fprintf(stderr, " | iters mean %.0f max %u\n", (nsync + ndone) ? sum_it / (nsync + ndone) : 0.0, max_it);
      if (n == 1 && Dbg(kDebugK1Pieces)) {  // one image: its first interval's pieces and chunks
        const uint32_t l0 = seg_lane0[0], nch = rj_chunks_cb(streams[0]->plan().segs[0].src_len, timings_.chunk_bytes),
                       H = timings_.chunk_hyp;
        std::vector<RjPiece> pc(nch);
        RJ_HIP(hipMemcpy(pc.data(), d_piece_.as<RjPiece>() + l0, nch * sizeof(RjPiece), hipMemcpyDeviceToHost));
        fprintf(stderr, "[K1] seg0 lanes %u.. nch %u npieces %u\n", l0, nch, pc[0].npieces);
        for (uint32_t q = 0; q < std::min<uint32_t>(pc[0].npieces, nch); q++)
          fprintf(stderr, "  piece %u: ent %llu first %u n %u dcd %d %d %d\n", q, (unsigned long long)pc[q].ent,
                  pc[q].first_blk, pc[q].nblk, pc[q].dcd[0], pc[q].dcd[1], pc[q].dcd[2]);
        for (uint32_t c = 0; c < nch; c++) {
          const RjChunkRes &r = cr[l0 + rj_chunk_lane(nch, H, c, 0)];
          fprintf(stderr, "  chunk %u: st %u tgt %u rec %u rb %u ne %u stop %u end %u\n", c, r.status, r.tgt, r.rec,
                  r.rb, r.ne, r.pad[0], r.pad[1]);
        }
      }
    }
  }
  return kOk;
}

}  // namespace rj
