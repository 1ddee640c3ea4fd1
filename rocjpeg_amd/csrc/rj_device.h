// rj_device.h -- descriptors shared by the host planner (rj_decoder.cpp) and the HIP kernels
// (rj_kernels.hip).  Plain PODs; every pointer is a device pointer on the handle's GPU.
//
// HBM layout of one batch (all regions carved from the handle's arena, rj_decoder.cpp):
//   images[]   RjImageDev          one per image in the batch
//   tabsets[]  RjTableSet          de-duplicated Huffman LUTs + natural-order quant tables
//   segs       RjSegDev per image  restart intervals (resident with the stream's ECS bytes)
//   destuffed  u8                  byte-unstuffed entropy data, each interval 16-B aligned
//   entries    uint32              sparse coefficients (K1 -> K2): per restart interval one
//                                  stream, per block its DC entry (zigzag pos 0, absolute value)
//                                  then its nonzero AC entries; a terminator (pos 127) after the
//                                  interval's last block.  Region per interval sized for the
//                                  worst case (64 entries per block), 64-B aligned.
//   row index  uint32 per MCU row  entry index (image-relative) of the row's first block
//   planes     u8                  per component, padded to the MCU grid (general path only)
#pragma once
#include <hip/hip_runtime.h>  // uint2/uint4 vector types (all users are built with hipcc)
#include <stdint.h>

#define RJ_MAX_BLK_MCU 10

// k_fused strips: one 64-lane workgroup per strip of S MCUs of one MCU row, at most one block
// per lane and at most RJ_FUSED_MAX_PX pixels wide (4:2:0 -> 10 MCUs = 160 px, 60 blocks).
#define RJ_FUSED_MAX_BLK 64
#define RJ_FUSED_MAX_PX 512
__host__ __device__ inline uint32_t rj_fused_strip_mcus(uint32_t hmax, uint32_t nblk_mcu) {
  const uint32_t a = RJ_FUSED_MAX_PX / (8u * hmax), b = RJ_FUSED_MAX_BLK / nblk_mcu;
  return a < b ? a : b;
}

// Sparse coefficient storage written by K1 and read by K2 (rj_fused.hip).
//   entry = uint16 value | zigzag position << 16 (positions 0..63; RJ_ENT_TERM ends an interval)
struct RjCoefBuf {
  uint32_t *ent;  // entry streams, one region per interval (image.ent_off + seg.ent_off)
  uint32_t *row;  // per MCU row (image.row_off + my): first entry of the row, image-relative
};
#define RJ_ENT_PER_BLOCK 64       // worst case: DC + 63 AC (each position written at most once)
#define RJ_ENT_GROUP 16           // K1 writes entries in 64-B groups; regions are group-aligned
#define RJ_ENT_TERM (127u << 16)  // end-of-interval marker
#define RJ_ENT_SLACK 1024         // entries of read slack after the last region (K2 reads 512-entry windows)
// entries reserved for an interval of `blocks` blocks: worst case + terminator, group-aligned
__host__ __device__ inline uint64_t rj_interval_entries(uint64_t blocks) {
  return (blocks * RJ_ENT_PER_BLOCK + 1 + RJ_ENT_GROUP - 1) / RJ_ENT_GROUP * RJ_ENT_GROUP;
}

// One restart interval of one image (host parser rj_stream.cpp builds these).
struct RjSegDev {
  uint32_t src_off;    // raw ECS byte offset of the interval's first data byte
  uint32_t src_len;    // raw bytes (RST markers and trailing fill FFs excluded)
  uint32_t dst_off;    // destuffed byte offset (16-B aligned), relative to image.destuff_off
  uint32_t mcu_first;  // first MCU of the interval
  uint32_t mcu_count;  // MCUs in the interval
  uint32_t flags;      // RJ_SEG_MISSING: marker not found -> interval decodes to zero blocks
  uint32_t ent_off;    // first sparse-coefficient entry of the interval, relative to image.ent_off
  uint32_t pad;
};
#define RJ_SEG_MISSING 1u

// Canonical Huffman decoder for one table (T.81 Annex C), laid out for the GPU.
//   lut[0..511]      first level, indexed by the next 9 bits:
//                      (code_len << 8) | symbol      for codes of <= 9 bits
//                      0x8000 | sub                  longer codes: second level `sub`
//                      0xFFFF                        second-level pool exhausted: canonical search
//                      0x1100 (len 17, symbol 0)     no code: libjpeg's "bad code" result
//   lut[512 + sub*128 + next 7 bits]  second level for codes of 10..16 bits (same encoding)
#define RJ_LUT_L1 512
#define RJ_L2_SUBTABLES 8
#define RJ_LUT_ENTRIES (RJ_LUT_L1 + RJ_L2_SUBTABLES * 128)
#define RJ_LUT_BAD 0x1100u
struct RjHuffDev {
  uint16_t lut[RJ_LUT_ENTRIES];
  uint32_t maxcode16[18];  // exclusive upper bound of length-l codes, left-justified to 16 bits
  int32_t valoff[18];      // symbol index = (code >> (16 - l)) + valoff[l]
  uint8_t vals[256];
};

struct RjTableSet {
  RjHuffDev dc[2];
  RjHuffDev ac[2];
  uint16_t qz[4][64];  // zigzag (DQT) order, as stored by the parser (rocjpeg_parser.cpp:239)
};

// Output jobs of the general (two-stage) path: one per written channel.
enum RjJobKind : uint32_t {
  RJ_JOB_COPY = 0,      // CopyChannel: surface plane bytes, dst pitch bytes per row
  RJ_JOB_RGB = 1,       // interleaved RGB
  RJ_JOB_RGB_PLANE = 2, // one of R/G/B planes (chan_sel)
  RJ_JOB_Y = 3,         // luma samples (also YUYV luma extraction)
  RJ_JOB_CHROMA = 4,    // planar U or V extracted from the surface model
};

struct RjJobDev {
  uint32_t image;
  uint32_t kind;
  uint32_t chan_sel;     // which surface plane / which RGB component / U(1) or V(2)
  uint32_t rows;         // rows written
  uint32_t row_bytes;    // bytes written per row
  uint32_t dst_pitch;
  uint8_t *dst;
  int32_t src_row0;      // surface row of output row 0
  int32_t src_byte0;     // surface byte (or pixel) column of output byte 0
  uint32_t row_prefix;   // exclusive prefix of rows over jobs (grid mapping)
  uint32_t pad;
};

struct RjImageDev {
  uint32_t width, height;
  uint32_t mcux, mcuy;
  uint8_t ncomp, nblk_mcu, interleaved, css;
  uint8_t hmax, vmax, fmt, roi;
  uint8_t comp_h[4], comp_v[4];
  uint8_t comp_td[4], comp_ta[4], comp_tq[4];
  uint8_t blk_comp[RJ_MAX_BLK_MCU], blk_dx[RJ_MAX_BLK_MCU], blk_dy[RJ_MAX_BLK_MCU];
  uint8_t comp_blk0[4];  // first block of each component inside an MCU
  uint32_t tabset;
  // inputs
  const uint8_t *ecs;
  const RjSegDev *segs;
  uint32_t nseg;
  uint32_t seg_prefix;   // exclusive prefix of segments over the batch
  uint64_t destuff_off;  // into the destuffed buffer
  uint64_t ent_off;      // in entries (sparse coefficients), group-aligned
  uint32_t ri_mcus;      // MCUs per restart interval (0: one interval)
  uint32_t row_off;      // first MCU row of this image in the batch's row index
  // component planes (general path)
  uint64_t plane_off[4];
  uint32_t plane_pitch[4], plane_rows[4];
  // output window (ROI semantics of rocjpeg_decoder.cpp:124-141)
  int32_t out_w, out_h, top, left;
  uint8_t *dst[4];
  uint32_t dst_pitch[4];
};
