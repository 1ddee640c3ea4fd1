/*
 * jpeg_oracle.h -- CPU ORACLE.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker / CPU baseline.  The product (librocjpeg_amd.so)
 * never links or calls it: the product path fails loudly without its HIP kernels.
 *
 * What it restates (file:line into the reference, fgladwin/rocJPEG @ 2025-03-03):
 *   - oj_parse          : RocJpegStreamParser::ParseJpegStream and sub-parsers
 *                         (src/rocjpeg_parser.cpp:43-470), incl. its error behaviour.
 *   - oj_image_info     : RocJpegDecoder::GetImageInfo (src/rocjpeg_decoder.cpp:307-358).
 *   - oj_decode_coefs / oj_decode_planes : the decode core the reference hands to VCN
 *                         (src/rocjpeg_vaapi_decoder.cpp:574-692).  No reference source
 *                         exists for it; restated from ITU-T T.81 (Annex C/F, baseline
 *                         Huffman) and libjpeg's ISLOW IDCT (jidctint.c), and PINNED
 *                         against IJG libjpeg 9.4 dumps (oracle/libjpeg_golden.c).
 *   - oj_decode         : RocJpegDecoder::Decode output stage (src/rocjpeg_decoder.cpp:
 *                         104-185, 372-636) over a model of the VCN surface, with the
 *                         colour conversion of src/rocjpeg_hip_kernels.cpp (e.g. NV12->RGB
 *                         :1377-1576: fmaf with 1.5748/-0.1873/-0.4681/1.8556, nearest
 *                         chroma, v_cvt_pk_u8_f32 = round-to-nearest-even + saturate).
 *                         The CSC restatement is pinned against the reference's own HIP
 *                         kernels compiled into oracle/_ref (run on the GPU box).
 */
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  uint16_t width, height;
  uint8_t precision;
  uint8_t ncomp;
  struct { uint8_t id, h, v, tq; } comp[4];
  uint8_t qt_loaded[4];
  uint8_t qt_zz[4][64];            /* DQT order (zigzag), as rocjpeg_parser.cpp:239 */
  uint8_t ht_loaded[2];
  struct { uint8_t dc_bits[16], dc_vals[12], ac_bits[16], ac_vals[162]; } ht[2];
  uint8_t scan_ncomp;
  struct { uint8_t cs, td, ta; } scomp[4];
  uint16_t restart_interval;
  uint32_t num_mcus;               /* comp-0 factors, rocjpeg_parser.cpp:194-198 */
  uint32_t ecs_offset, ecs_size;   /* slice data: SOS end .. FFD9 (rocjpeg_parser.cpp:400-416) */
  int css;                         /* ChromaSubsampling (rocjpeg_parser.cpp:432-470) */
  uint8_t sof_seen;
} oj_params;

/* 1 = parsed, 0 = reference would return false (-> ROCJPEG_STATUS_BAD_JPEG). */
int oj_parse(const uint8_t *data, size_t len, oj_params *p);

/* GetImageInfo restatement; returns RocJpegStatus. */
int oj_image_info(const oj_params *p, uint8_t *nc, int *css, uint32_t widths[4], uint32_t heights[4]);

/* Coefficient grids (natural order, int16) per component, padded to the MCU grid
 * exactly like libjpeg's coefficient arrays.  dims[c] = {wblk, hblk}.  Returns 0 on
 * success.  out may be NULL to query dims; total size = sum(wblk*hblk*64). */
int oj_coef_dims(const uint8_t *data, size_t len, int32_t dims[4][2]);
int oj_decode_coefs(const uint8_t *data, size_t len, int16_t *out);

/* ISLOW planes per component at native resolution, padded to the MCU grid
 * (width = wblk*8, height = hblk*8), concatenated. */
int oj_decode_planes(const uint8_t *data, size_t len, uint8_t *out);

/* Full rocJpegDecode semantics: parse + decode + output stage.  Writes only the bytes
 * the reference writes inside the logical W x H (or ROI) region.  Returns RocJpegStatus. */
int oj_decode(const uint8_t *data, size_t len, int output_format,
              int16_t crop_left, int16_t crop_top, int16_t crop_right, int16_t crop_bottom,
              uint8_t *channel[4], const uint32_t pitch[4]);

/* The output stage alone (src/rocjpeg_decoder.cpp:124-180, 372-636 over the VCN surface model)
 * on given component planes: planes[c] is plane_w[c] x plane_h[c] bytes (the decoded, MCU-padded
 * planes; reads past them clamp to the edge); css is the parser's ChromaSubsampling, W x H the
 * picture size.  oj_decode = decode + this.  Lets the tests pin the output stage against the
 * reference's own kernels on arbitrary planes. */
int oj_output_stage(const uint8_t *const planes[3], const int32_t plane_w[3], const int32_t plane_h[3], int css,
                    int W, int H, int output_format, int16_t crop_left, int16_t crop_top, int16_t crop_right,
                    int16_t crop_bottom, uint8_t *channel[4], const uint32_t pitch[4]);

/* One pixel of the reference colour conversion (rocjpeg_hip_kernels.cpp:1431-1443). */
void oj_csc_pixel(uint8_t y, uint8_t u, uint8_t v, uint8_t rgb[3]);
void oj_csc_bulk(const uint8_t *y, const uint8_t *u, const uint8_t *v, size_t n, uint8_t *rgb);
/* v_cvt_pk_u8_f32 semantics restated: RNE, saturate to [0,255] (NaN -> 0). */
uint8_t oj_cvt_u8(float f);

#ifdef __cplusplus
}
#endif
