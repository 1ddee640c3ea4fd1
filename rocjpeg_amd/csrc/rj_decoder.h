// rj_decoder.h -- decode orchestration behind rocJpegDecode / rocJpegDecodeBatched.
//
// Role of the reference's RocJpegDecoder (src/rocjpeg_decoder.{h,cpp}): one HIP device and
// one private stream per handle (rocjpeg_decoder.cpp:46-61), calls serialised by a
// per-handle mutex (rocjpeg_decoder.h:174), synchronous return (:183, :290).  Instead of a
// VA submit per image it plans the whole batch at once: one descriptor upload, then
// K0 destuff -> K1 Huffman -> K2 (fused) or K2a+K2b (general) over every image together.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <functional>
#include <memory>
#include <mutex>
#include <unordered_map>
#include <utility>
#include <vector>

#include "../../include/rocjpeg.h"
#include "../../include/rocjpeg_amd.h"
#include "rj_device.h"
#include "rj_pool.h"
#include "rj_stream.h"

namespace rj {

class DeviceBuffer {
 public:
  ~DeviceBuffer() { Release(); }
  int Ensure(size_t bytes);  // grow-only
  void Release();
  template <typename T> T *as() const { return static_cast<T *>(ptr_); }
  size_t capacity() const { return cap_; }
  void Swap(DeviceBuffer &o) {
    std::swap(ptr_, o.ptr_);
    std::swap(cap_, o.cap_);
  }

 private:
  void *ptr_ = nullptr;
  size_t cap_ = 0;
};

class PinnedBuffer {
 public:
  ~PinnedBuffer() { Release(); }
  int Ensure(size_t bytes);
  void Release();
  uint8_t *data() const { return static_cast<uint8_t *>(ptr_); }

 private:
  void *ptr_ = nullptr;
  size_t cap_ = 0;
};

class Decoder {
 public:
  Decoder(RocJpegBackend backend, int device_id) : backend_(backend), device_(device_id) {}
  ~Decoder();
  int Initialize();
  int GetImageInfo(Stream *s, uint8_t *nc, RocJpegChromaSubsampling *css, uint32_t *w, uint32_t *h);
  int Decode(Stream *const *streams, int n, const RocJpegDecodeParams *params, RocJpegImage *dst);
  // The host-side validation Decode runs before any device work (stream status, destination
  // channels the format needs), without decoding: the status Decode would return for these images
  // if it fails there, else kOk (rj_coalesce.cpp pre-validates a combined call's members).
  int Check(Stream *const *streams, int n, const RocJpegDecodeParams *params, const RocJpegImage *dst);
  int StreamsToDevice(Stream *const *streams, int n);
  // rocJpegStreamParse + rocJpegAmdStreamsToDevice for a batch, with the O(bytes) marker scan
  // (FF D9 end, restart intervals, destuffing tables) on this handle's GPU (rj_scan.hip)
  int ParseOnDevice(Stream *const *streams, const uint8_t *const *data, const size_t *len, int n);
  void SetProfiling(bool on) { profiling_ = on; }
  void SetPathPolicy(int p) { path_policy_ = p; }
  // (copies under the handle's lock: a concurrent call on the handle writes them)
  RocJpegAmdTimings last_timings() {
    std::lock_guard<std::mutex> lock(mu_);
    return timings_;
  }
  // the last ParseOnDevice call's stages, ms: headers, resident allocation, staging copy + upload,
  // jobs upload + kernel + read-back, adoption, total
  void last_scan_ms(double out[6]) {
    std::lock_guard<std::mutex> lock(mu_);
    for (int k = 0; k < 6; k++) out[k] = scan_ms_[k];
  }
  hipStream_t stream() const { return stream_; }
  int device() const { return device_; }
  // a call on this handle may be decoded inside another handle's combined call (rj_coalesce.h):
  // not while the caller profiles (its timings are per handle) or forces the general output path
  bool Coalescable() const { return !profiling_ && path_policy_ == 0; }

 private:
  int DecodeLocked(Stream *const *streams, int n, const RocJpegDecodeParams *params, RocJpegImage *dst);
  int DecodeOne(Stream *const *streams, int n, const RocJpegDecodeParams *params, RocJpegImage *dst,
                bool may_split = false);
  static constexpr int kWantSplit = -1000;  // DecodeOne(may_split): a staged call for DecodeSplit
  // A large call whose bitstreams are in host memory (every call stages them over PCIe): its
  // images are cut into parts, each decoded by its own handle (helpers: same device, their own
  // streams and buffers) on its own host thread, so one part's upload overlaps the earlier
  // parts' kernels -- what caller threads with a handle each get (tools/host_input_threads.py).
  // env RJ_SPLIT_HOST=0 turns it off; never while profiling (the timings are per handle).
  int DecodeSplit(Stream *const *streams, int n, const RocJpegDecodeParams *params, RocJpegImage *dst);
  std::atomic<bool> split_host_{true};
  std::vector<Stream *> lock_order_;  // DecodeOne's stream lock order (under mu_)
  std::vector<std::unique_ptr<Decoder>> helpers_;  // parts 1 .. split_parts_ - 1
  int split_parts_ = 2;                             // env RJ_SPLIT_PARTS (2..4; 3 measured slower inside bench.py: host_input_parts_ab.txt)
  bool split_part_ = false;                         // this handle decodes a DecodeSplit part
  static constexpr int kSplitHostMin = 1024;  // staged (non-resident) images a call needs to split
  hipEvent_t split_ev_ = nullptr;                // DecodeSplit: this part's uploads are done (recorded on stream_)
  hipEvent_t upload_after_ = nullptr;            // DecodeSplit part > 0: wait for this before uploading
  std::function<void()> uploaded_;               // DecodeSplit part < last: called once its uploads are enqueued
  int ParseOnDeviceImpl(Stream *const *streams, const uint8_t *const *data, const size_t *len, int n);
  // Device of the allocation holding p (hipPointerGetAttributes, cached per call by address
  // range); -1: host memory (pinned or pageable).
  int PtrDevice(const void *p);

  // Destinations that do not live on this handle's device (another GPU, host memory): the
  // image is decoded into device-local staging at the caller's pitch, then copied to where
  // the caller's pointer lives (hipMemcpy2DAsync; peer copies go over xGMI) -- SURVEY.md 8e.
  struct PtrRange {
    uintptr_t lo, hi;
    int device;
  };
  std::vector<PtrRange> ptr_cache_;
  struct RouteCopy {
    uint32_t image, chan, rows, row_bytes, pitch;
    uint64_t off;  // staging offset
    void *user;
  };
  std::vector<RouteCopy> routes_;
  std::vector<int> peer_enabled_;
  DeviceBuffer d_route_;

  RocJpegBackend backend_;
  int device_;
  hipStream_t stream_ = nullptr;
  std::mutex mu_;
  bool profiling_ = false;
  int path_policy_ = 0;
  RocJpegAmdTimings timings_ = {};
  double scan_ms_[6] = {};
  hipEvent_t ev_[8] = {};  // 0..5 stage boundaries, 6..7 inside K1
  // pipelined launch (rj_decoder.cpp): interval length classes 0..pipe_groups_-2 on pstream_,
  // the last class on stream_; pev_ joins them (no timing), pk1_ times each class's K1
  enum DebugFlag : uint32_t {  // env RJ_DEBUG_* (development diagnostics), bit k = dbg_names[k]
    kDebugScan = 1u << 0, kDebugProg = 1u << 1, kDebugWaves = 1u << 2, kDebugHost = 1u << 3,
    kDebugStamps = 1u << 4, kDebugK1 = 1u << 5, kDebugK1Pieces = 1u << 6, kTestProgGiveUp = 1u << 7
  };
  uint32_t dbg_ = 0;
  std::chrono::steady_clock::time_point dbg_synced_;  // RJ_DEBUG_HOST: the call's stream sync returned
  std::chrono::steady_clock::time_point dbg_returned_;  // RJ_DEBUG_HOST: the last call returned
  bool Dbg(uint32_t f) const { return (dbg_ & f) != 0; }
  static constexpr int kMaxPipe = 4;  // = HIP's default hardware queues per process
  static constexpr int kWideSites = 4 + 2 * kMaxPipe;  // K2 launches per call, bound (fix-up counters)
  // 2 by default: the caller's own stream (e.g. torch's) takes a hardware queue too, and two
  // streams sharing one queue serialise (measured: 4 classes sometimes double the K1 span)
  int pipe_groups_ = 2;            // env RJ_PIPE_GROUPS (1 = sequential); the lean K1 defaults to 1
  bool pipe_groups_set_ = false;
  uint32_t pipe_min_ = 2048;       // env RJ_PIPE_MIN: fewest intervals worth pipelining
  bool sort_lanes_ = true;         // env RJ_SORT_LANES=0: K1 lanes in interval order
  bool lpt_ = true;                 // env RJ_LPT=0: one K1 launch takes the shortest intervals first
  // env RJ_K1_SOLO=<bytes>: extra dynamic LDS per lean K1 workgroup, so that one fits per CU: the
  // workgroups past the first round (LPT order: the shortest) then wait for the CUs that finish
  // first instead of doubling up on a CU beside a long-interval workgroup
  uint32_t k1_solo_lds_ = 16384;
  uint32_t chunk_min_ = RJ_CHUNK_MIN_BYTES;  // env RJ_CHUNK_MIN: floor of the call's chunk length (bytes)
  bool k1_chunk_ = true;           // env RJ_K1_CHUNK=0: chunk-layout calls take k_entropy's K1 (A/B)
  int five_waves_ = 2;             // env RJ_K1_FIVE: 0 a lean call's overflow past one round of lanes runs as a second round;
                                   // 1 fifth waves; 2 fifth waves beside their workgroup's shortest wave
  double split5_t_ = 0.8;          // env RJ_K1_SPLIT5_T (0: off): five-wave lean calls split the intervals above this share of
                                   // the longest, as many as the five waves per CU hold
  bool outlier_split_ = true;      // env RJ_SPLIT_OUTLIERS=0: never split the outlier intervals (one decoder wave per SIMD)
  double outlier_t_ = 9.0 / 16;    // env RJ_SPLIT_OUTLIER_T: outliers are longer than this share of the longest interval
  double outlier_frac_ = 0.7;      // env RJ_SPLIT_OUTLIER_FRAC: at most this share of the intervals split in that mode
                                   // (C4's mix: 56 % above 9/16 of the longest; C2's near-uniform rows: 84 %)
  int cu_count_ = 256;
  DeviceBuffer d_wide_;            // K2 fix-up lists (rows outside the int32 IDCT's domain)
  uint32_t *h_wide_flag_ = nullptr;  // host-mapped, coherent: K2 recorded a row for the fix-up
  uint32_t *d_wide_flag_ = nullptr;
  struct WideSite {                // one K2 launch of the current call
    bool planes, dense;
    uint32_t cap;
    uint32_t *cnt;
    uint2 *list;
  };
  std::vector<WideSite> wide_sites_;
  hipStream_t pstream_[kMaxPipe - 1] = {};
  hipEvent_t pev_[kMaxPipe] = {};
  hipEvent_t pk1_[kMaxPipe] = {};
  hipEvent_t kev_[kMaxPipe] = {};  // K1 of class g done (K2 of later classes waits on it)
  hipEvent_t k1s_[kMaxPipe] = {}, k2s_[kMaxPipe] = {}, k2e_[kMaxPipe] = {};  // profiling: launch spans
  DeviceBuffer d_count_;  // profiling: entries written by K1
  // live rows (rj_device.h RjLive): K2 beside the lean five-wave K1 on lstream_ (lowest priority,
  // so the stream-ordered kernels win dispatch arbitration); env RJ_K2_LIVE=1 turns it on (off by
  // default: beside K1 it slowed K1 by more than it saved)
  bool live_k2_ = false;
  bool live_test_giveup_ = false;
  uint32_t live_lds_ = 0;  // env RJ_K2_LIVE_LDS: extra LDS per live K2 workgroup (fewer of them per CU)
  hipStream_t lstream_ = nullptr;
  hipEvent_t live_ev_[2] = {};  // fork (descriptors uploaded), join (the live K2 done)
  hipEvent_t live_t_[4] = {};   // profiling: live K2 span (its stream), rest + split span (after K1)
  DeviceBuffer d_live_;          // published-row slots
  // upload B (K1 lane order, K2 row lists) on its own stream while K0 runs; K1 waits for it by an
  // event instead of behind K0 in the call's stream (env RJ_UPLOAD_B_SIDE=0: in stream order)
  bool side_b_ = true;
  bool sort_par_ = false;       // env RJ_SORT_PAR=1: a large lean call's lane sort on the host pool
  bool k2_lpt_ = false;         // env RJ_K2_LPT=1: a lean call's K2 rows in K1's lane order (longest first)
  bool k2_split_side_ = false;  // env RJ_K2_SPLIT_SIDE=1: the split rows' K2 launch beside the plain one (one process in two ran 11 % slower: off)
  hipEvent_t kfork_ev_ = nullptr, kjoin_ev_ = nullptr;  // K2's plain / split launches: fork, join
  bool k0_lds_ = true;      // env RJ_K0_LDS=0: K0 stores a compacted chunk's bytes one by one (A/B)
  uint64_t ent_shift_ = 0;  // env RJ_ENT_SHIFT_KB (placement probe): the entry streams start this far into their buffer
  // Entry-buffer placement search: K2's time depends on where its entry buffer lies in HBM
  // relative to the output (one process, fixed buffers: 2.32-2.34 or 2.44-2.47 ms per C2 call,
  // stable for a given pair, not predictable from virtual addresses -- DESIGN.md 4 K2).  The
  // first large lean calls of a handle time K1 + K2 (two events) with the entry buffer they
  // have, then with up to kPlaceCands - 1 freshly allocated ones (the earlier ones stay
  // allocated meanwhile, so each is new memory), and keep the fastest.  env RJ_PLACE_TUNE=0: off.
  static constexpr int kPlaceCands = 4;  // (the most RJ_PLACE_CANDS allows; 3 by default)
  static constexpr uint32_t kPlaceMinRows = 16384;  // MCU rows of a call worth timing (C2: 69,632)
  bool place_tune_ = true;
  int place_cands_ = 3;            // env RJ_PLACE_CANDS (1..kPlaceCands): candidates tried
  // the other candidates stay allocated until the handle is destroyed: freeing ~5 GB of VRAM made
  // the host-input path's uploads run at half speed for a while afterwards (126k -> 98k images/s;
  // profiles/r6_experiments/k2_placement_probe.txt); env RJ_PLACE_KEEP=0 frees them
  bool place_keep_ = true;
  int place_state_ = 0;  // 0: warming up; 1..kPlaceCands: measuring candidate state-1; -1 done
  int place_warm_ = 0;   // large calls before the first measurement (2: the second call still ran slower)
  int place_best_ = -1;
  float place_ms_[4] = {};
  DeviceBuffer place_bufs_[kPlaceCands];
  hipEvent_t place_ev_[2] = {};
  void PlaceStep(float ms);
  bool spin_sync_ = false;  // env RJ_SYNC_SPIN=1: WaitCall polls the stream instead of sleeping
  hipError_t WaitCall();
  hipError_t SideStream(hipStream_t &s, bool lowest_priority = false);  // created on first use
  hipStream_t bstream_ = nullptr;
  hipEvent_t bev_ = nullptr;

  // a run of non-resident streams whose parse-time pinned copies are adjacent (one DMA)
  struct PinRun {
    const uint8_t *host;
    uint64_t len, dev;  // bytes; offset in the device ECS staging
    const PinnedChunk *chunk;
  };
  // host planning scratch, reused across calls (no per-call allocation / page faults)
  struct Scratch {
    std::vector<PinRun> pin_runs;
    std::vector<unsigned long long> seg_ent;  // per interval: its chunk regions (split intervals)
    std::vector<RjImageDev> imgs;
    std::vector<RjJobDev> jobs;
    std::vector<uint64_t> stage_off, ecs_off;
    std::vector<uint32_t> chunk_img;
    std::vector<uint32_t> tab_of, row_prefix, grow_prefix, seg_lane0, lane_seg, bucket_pos, seg_pos, lane_split;
    std::vector<uint32_t> bucket_cnt;  // the lane sort's 32-B length histogram (its bucket order)
    std::vector<uint64_t> lane_len;    // per lane (sorted order): the interval's seg_lenblk
    std::vector<uint32_t> part_hist;   // the lane sort on the pool: per part, bucket counts / next slots
    std::vector<uint64_t> split_bits;  // per interval: split by the five-wave layout
    std::vector<uint8_t> is_fused, row_group, routed;
    std::vector<uint2> row_list;
    std::vector<uint32_t> prow_prefix, pgrow_prefix, prog_lanes, prog_bucket;  // progressive images
    std::vector<RjFoldJob> fold_jobs;
    std::vector<Stream *> owner_stream;
  } sc_;
  hipEvent_t prog_ev_[3] = {};  // profiling: K1p start, K1p end (dense K2 start), dense K2 end
  std::vector<hipEvent_t> prog_lev_ev_;  // development (RJ_DEBUG_PROG): per-level K1p spans
  hipEvent_t prog_join_[2] = {};         // pipelined refinement: side stream fork / join
  bool prog_pipe_enabled_ = true;        // env RJ_PROG_PIPE=0: level-by-level refinement
  bool prog_dc_lanes_ = true;            // env RJ_PROG_DC_LANES=0: pipelined layouts decode DC scans in waves
  int prog_wave_all_ = -1;               // env RJ_PROG_WAVE_ALL=0/1: force the pipelined layout (-1: by batch)
  // profiling: one event pair per progressive launch, on the stream it runs on; kind 0 k_prog,
  // 1 k_prog_wave, 2 k_prog_fold
  struct ProgSpan {
    uint32_t kind, e0, e1;
  };
  std::vector<hipEvent_t> pk_ev_;
  std::vector<ProgSpan> pk_span_;

  DeviceBuffer d_desc_, d_stage_, d_destuff_, d_entries_, d_planes_;
  DeviceBuffer d_piece_, d_rec_, d_chunkres_, d_fallback_;  // K1 chunk bookkeeping
  DeviceBuffer d_coef_, d_nz_, d_prec_, d_pprog_, d_wstamp_;  // d_wstamp_: RJ_DEBUG_WAVES
  DeviceBuffer d_scan_;  // marker scan: uploaded bytes, jobs, scratch lists, read-back tables
  PinnedBuffer h_scan_;  // progressive: dense coefficients, nonzero masks, refinement records
  uint32_t epoch_ = 0;
  PinnedBuffer h_stage_;
  PinnedBuffer h_ecs_;    // staged bitstreams of non-resident streams (uploaded in chunks)
  DeviceBuffer d_ecs_;
  // host threads of the per-call staging copies: RJ_HOST_THREADS, else up to 8 (the caller's
  // thread counts as one)
  HostPool pool_{HostThreads()};
  uint32_t hyp_max_ = RJ_MAX_HYP;  // env RJ_K1_HYP: most MCU-phase hypotheses per speculative chunk (1: off)
  bool hyp_warm_ = true;           // env RJ_K1_HYP_WARM=0: no speculative warm-up under hypotheses
  uint32_t hyp_chunk_min_ = 192;   // env RJ_K1_HYP_CHUNK_MIN: shortest chunk under phase hypotheses
  static int HostThreads();
};

}  // namespace rj
