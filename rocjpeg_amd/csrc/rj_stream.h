// rj_stream.h -- host JPEG bitstream parser behind rocJpegStreamParse.
//
// Replaces RocJpegStreamParser (reference src/rocjpeg_parser.{h,cpp}): same acceptance
// rules and the same fields (so GetImageInfo and every error path behave identically),
// plus what the GPU decoder needs and the VCN path never built on the host:
//   * the restart-interval table (RST scan folded into the FFD9 scan the reference already
//     does in ParseEOI, rocjpeg_parser.cpp:400-416),
//   * MCU geometry, canonical Huffman LUTs and natural-order quant tables (RjTableSet).
#pragma once
#include <stdint.h>

#include <memory>
#include <mutex>
#include <vector>

#include "rj_device.h"
#include "rj_pinned.h"

namespace rj {

// ChromaSubsampling of the reference parser (src/rocjpeg_parser.h:148-156).
enum Css { kCss444 = 0, kCss440 = 1, kCss422 = 2, kCss420 = 3, kCss411 = 4, kCss400 = 5, kCssUnknown = -1 };

struct StreamInfo {
  // --- fields the reference parser fills (src/rocjpeg_parser.h:62-172) ---
  uint16_t width = 0, height = 0;
  uint8_t precision = 0, ncomp = 0;
  struct { uint8_t id, h, v, tq; } comp[4] = {};
  uint8_t qt_loaded[4] = {};
  uint8_t qt_zz[4][64] = {};
  uint8_t ht_loaded[2] = {};
  struct { uint8_t dc_bits[16], dc_vals[12], ac_bits[16], ac_vals[162]; } ht[2] = {};
  uint8_t scan_ncomp = 0;
  struct { uint8_t cs, td, ta; } scomp[4] = {};
  uint16_t restart_interval = 0;
  uint32_t num_mcus = 0;
  const uint8_t *ecs = nullptr;   // borrowed from the caller (rocjpeg_parser.cpp:413)
  uint32_t ecs_size = 0;
  int css = kCssUnknown;
  bool sof_seen = false;
};

// Everything the batch planner needs to decode this stream on the GPU.
struct DecodePlan {
  int status = 0;  // RocJpegStatus the decode call returns for this stream (0 = decodable)
  uint32_t mcux = 0, mcuy = 0;
  uint8_t hmax = 1, vmax = 1, nblk_mcu = 0, interleaved = 0;
  uint8_t blk_comp[RJ_MAX_BLK_MCU] = {}, blk_dx[RJ_MAX_BLK_MCU] = {}, blk_dy[RJ_MAX_BLK_MCU] = {};
  uint8_t comp_blk0[4] = {};
  uint32_t wblk[4] = {}, hblk[4] = {};
  std::vector<RjSegDev> segs;      // one per restart interval
  // batch planner caches (FinishSegs): per interval its 32-B length bucket (the K1 lane sort
  // reads 2 B per interval instead of the 48-B descriptor), and whether every interval is
  // exactly one MCU row
  std::vector<uint16_t> seg_bucket;
  std::vector<uint64_t> seg_lenblk;  // per interval: destuffed bytes (0: missing) | blocks << 32 (split planning)
  bool rows_aligned = false;
  uint64_t src_total = 0;          // entropy-coded bytes of the intervals (call-time chunk length)
  uint32_t src_max = 0;            // the longest interval's
  std::vector<RjDsBlock> ds;       // K0 blocks over all intervals
  uint64_t destuff_bytes = 0;      // destuffed buffer size incl. per-interval alignment
  uint64_t entries = 0;            // sparse-coefficient entries reserved (worst case)
  uint32_t nchunks = 0;            // K1 lanes (chunks) over all intervals
  RjTableSet tables;               // derived tables
  uint8_t ht_valid[2] = {};        // DHT slot loaded and both its tables valid (BuildHuffman)
  uint16_t qmax[4] = {1, 1, 1, 1}; // largest entry of each quant table slot (the IDCT's exact domain)
  // De-duplication key: the raw DHT/DQT content the derived tables are a function of (the
  // batch planner compares these ~670 B instead of the 14.5 KB RjTableSet) and its hash.  The
  // last two bytes are the AC table each DC table's two-symbol entries pair with (Stream::
  // LeanTables; 0xFF: none), so streams with equal tables but another component-to-table map
  // get table sets of their own.
  static constexpr size_t kTableKeyBytes = 2 + 2 * (16 + 12 + 16 + 162) + 4 * 64 + 2;
  uint8_t table_key[kTableKeyBytes] = {};
  uint64_t table_hash = 0;

  // progressive (SOF2) streams: every scan's restart intervals (K0 destuffs them like baseline
  // intervals; `segs` stays empty), the per-scan Huffman tables, the dense coefficient layout
  // and the scans' dependency levels (rj_prog.hip)
  bool progressive = false;
  std::vector<RjProgScanDev> pscans;
  std::vector<RjProgIvalDev> pivals;
  std::vector<RjHuffDev> ptabs;
  uint32_t plevels = 0;            // dependency levels (max scan level + 1)
  uint32_t cblk0[3] = {}, nzblk0[3] = {}, cwblk[3] = {}, chblk[3] = {};
  uint64_t coef_blocks = 0;        // dense blocks (MCU-padded)
  uint64_t nz_blocks = 0;          // nonzero masks
  uint64_t prec_words = 0;         // refinement records (u64 words)
  uint8_t pqlat[3][64] = {};       // each component's latched quant table (zigzag order)
  std::vector<uint32_t> pscan_src; // per scan: absolute stream offsets of its data [begin, end)
};

void FinishSegs(DecodePlan &p);

class Stream {
 public:
  // RocJpegStreamParser::ParseJpegStream semantics; true = parsed (else BAD_JPEG).
  bool Parse(const uint8_t *data, uint32_t size, bool defer_scan = false);
  // defer_scan: header only; the O(bytes) marker scan runs on the GPU (Decoder::ParseOnDevice),
  // which then hands the interval tables back through CompleteFromDevice
  bool scan_pending() const { return scan_pending_; }
  void CompleteFromDevice(uint32_t ecs_size, const RjSegDev *segs, uint32_t nsegs, const RjDsBlock *ds, uint32_t nds);
  const StreamInfo &info() const { return info_; }
  const DecodePlan &plan() const { return plan_; }
  uint64_t generation() const { return generation_; }
  std::mutex &mutex() { return mu_; }

  // Device-resident copy of the ECS bytes + interval table (rocJpegAmdStreamsToDevice).
  struct Resident {
    int device = -1;
    uint64_t generation = 0;
    uint8_t *ecs = nullptr;
    RjSegDev *segs = nullptr;
    RjDsBlock *ds = nullptr;
    RjProgScanDev *pscans = nullptr;  // progressive only
    RjProgIvalDev *pivals = nullptr;
    RjHuffDev *ptabs = nullptr;
    // set: the buffers above are carved from a block shared by the streams of one
    // rocJpegAmdStreamParseDevice call; the block is freed with its last stream
    std::shared_ptr<uint8_t> block;
  } resident;
  void ReleaseResident();
  ~Stream() { ReleaseResident(); }
  // the entropy-coded bytes (+ 16 zero bytes) copied at parse time into the pinned arena
  // (rj_pinned.h); nullptr when the stream borrows the caller's bytes only
  const uint8_t *pinned_ecs() const { return pin_.ptr; }
  const PinnedChunk *pinned_chunk() const { return pin_.id(); }
  // lean K1 tables (rj_huff.hip) of this stream's DHTs, built on first use (callers hold mutex())
  const RjLeanTables *LeanTables();

 private:
  void BuildPlan();
  bool BuildPlanHeader();   // geometry, tables, status; false: not decodable
  void BuildIntervals();    // host marker scan: restart intervals, K0 blocks
  bool scan_pending_ = false;
  bool ParseProgressive(const uint8_t *data, uint32_t size);  // SOF2 (beyond the reference)
  void BuildProgressivePlan(const uint8_t *data);
  void PinEcs();             // copy the ECS into the pinned arena (decodable streams)
  StreamInfo info_;
  DecodePlan plan_;
  PinnedSlot pin_;
  std::unique_ptr<RjLeanTables> lean_;
  uint64_t generation_ = 0;
  std::mutex mu_;
};

// GetImageInfo restatement (rocjpeg_decoder.cpp:307-358); returns RocJpegStatus.
int ImageInfo(const StreamInfo &s, uint8_t *num_components, int *subsampling, uint32_t *widths, uint32_t *heights);

// True when the frame header ahead of the first SOS is SOF2 (progressive Huffman).
bool IsProgressiveStream(const uint8_t *data, uint32_t size);

// Canonical Huffman table -> lean K1 first level (2^RJ_HL_DC_BITS or 2^RJ_HL_AC_BITS entries)
// and, for AC, RJ_HL_SUBS second-level subtables (subs).  An over-subscribed table is refused
// before any entry is written (false; first/subs then hold only 'bad' entries).
bool BuildLeanTable(const uint8_t bits[16], const uint8_t *vals, bool is_dc, uint32_t *first, uint32_t *subs);

// Canonical Huffman table -> RjHuffDev; false for an invalid table.
bool BuildHuffman(const uint8_t bits[16], const uint8_t *vals, bool is_dc, RjHuffDev *out);

}  // namespace rj
