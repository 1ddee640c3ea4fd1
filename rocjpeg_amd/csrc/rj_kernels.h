// rj_kernels.h -- host-side launchers of the gfx950 decode kernels (rj_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rj_device.h"

namespace rj {

// K0: byte-unstuffing of the entropy-coded data (one wavefront per RjDsBlock).
// ds_map (may be null): the image holding K0 block 64 k, for k <= nblocks / 64, + a sentinel
// lds: the block's output assembled in LDS, aligned dword stores (false: the byte-store form)
hipError_t LaunchDestuff(hipStream_t st, const RjImageDev *imgs, int nimg, uint32_t nblocks, uint8_t *destuffed,
                         const uint32_t *ds_map = nullptr, bool lds = true);

// K1 (rj_entropy.hip): Huffman entropy decode -> sparse entry streams + pieces.  stage 0: one
// lane per interval chunk; 1: sync resolution; 2: serial re-decode of the flagged intervals.
// lanes_wg: lanes of intervals that fit one workgroup (laid out first); lanes_dev: the others.
hipError_t LaunchEntropy(hipStream_t st, int stage, const RjImageDev *imgs, int nimg, uint32_t lanes_wg,
                         uint32_t lanes_dev, uint32_t nseg, const uint8_t *destuffed, const RjTableSet *tabsets,
                         RjCoefBuf coefs, uint32_t epoch);

// K1 exact lanes [lane0, lane0 + nlanes) only (pipelined launch: no interval is split, so the
// chunk pass alone is the whole entropy decode of those lanes' intervals).
hipError_t LaunchEntropyLanes(hipStream_t st, const RjImageDev *imgs, int nimg, uint32_t lane0, uint32_t nlanes,
                              const uint8_t *destuffed, const RjTableSet *tabsets, RjCoefBuf coefs, uint32_t epoch);

// Lean K1 (rj_huff.hip): lanes [lane0, lane0 + nlanes), one whole interval each, raw entries;
// only for calls whose every baseline image is a row image and no interval is split.
// split != null: the outlier split launch -- lane_seg lists per wave 32 head lanes then their 32
// tail lanes (RJ_LANE_HEAD / RJ_LANE_TAIL), split waves first, then whole intervals 64 per wave;
// pieces at interval << 1 (coefs.piece_shift = 1); 512-thread workgroups, two per CU (one
// decoder wave per SIMD, as in the unsplit launch).
// five_waves: RJ_HL_DEC5 lanes per workgroup (five decoder waves, one workgroup per CU): a call
// whose intervals overflow one round of four waves per CU by at most one wave per CU lists the
// overflow as fifth waves (lane_seg laid out per workgroup, empty lanes 0xFFFFFFFF).
hipError_t LaunchHuffLanes(hipStream_t st, const RjImageDev *imgs, int nimg, uint32_t lane0, uint32_t nlanes,
                           const uint8_t *destuffed, const RjTableSet *tabsets, const RjLeanTables *lean,
                           RjCoefBuf coefs, uint32_t extra_lds = 0, const RjHuffSplit *split = nullptr,
                           bool five_waves = false, const RjLive *live = nullptr);
// K1 chunk lanes on the lean machinery (rj_huff.hip k_huff_chunk): stage 0 of LaunchEntropy's
// layout (from lane0: lanes_wg lanes with workgroup-scope records, then lanes_dev), absolute DC entries.
hipError_t LaunchHuffChunks(hipStream_t st, const RjImageDev *imgs, int nimg, uint32_t lane0, uint32_t lanes_wg,
                            uint32_t lanes_dev,
                            const uint8_t *destuffed, const RjTableSet *tabsets, const RjLeanTables *lean,
                            RjCoefBuf coefs, uint32_t epoch);
// K2b (general path): every output format / ROI of rocjpeg_decoder.cpp:143-180 from the planes.
hipError_t LaunchOutputJobs(hipStream_t st, const RjImageDev *imgs, const RjJobDev *jobs, int njobs, uint32_t total_rows,
                            const uint8_t *planes);

// K2: one wavefront per MCU row (row_prefix[i] = first row of image i in this launch; images
// with no rows in it have equal consecutive prefixes; or, when row_list is given, wave w takes
// the (image, MCU row) pair row_list[w]).  Sparse entries -> dequant + ISLOW IDCT
// -> either the fused output (upsample + CSC / layout straight into the caller's buffers, only
// for rj_decoder.cpp::FusedEligible images) or the MCU-padded component planes (to_planes).
// wide_cnt (zero on entry) / wide_list (nrows slots): this launch's fix-up list; rows with
// coefficients outside the int32 IDCT's exact domain are recorded there (and coefs.wide_flag
// raised) for the host to issue LaunchRowsFix after the call's kernels.
// split_rows (a lean split call whose every interval is one MCU row): the rows of the split
// intervals, decoded by the split-aware instance; every other row by the plain instance, whose
// waves leave at once on a split interval's row (two launches).
hipError_t LaunchRows(hipStream_t st, bool to_planes, const RjImageDev *imgs, int nimg, const uint32_t *row_prefix,
                      const uint2 *row_list, uint32_t nrows, RjCoefBuf coefs, const RjTableSet *tabsets,
                      uint8_t *planes, uint32_t *wide_cnt, uint2 *wide_list, const uint2 *split_rows = nullptr,
                      uint32_t nsplit_rows = 0, hipStream_t split_st = nullptr);
// (split_st: the split rows' launch goes there, beside the plain launch; the caller forks and joins)
// Live rows (rj_device.h RjLive): K2 beside K1 (second stream; grid = lv.rows, one workgroup per
// ticket), and the stream-ordered K2 after K1 over the published rows no ticket took.
hipError_t LaunchRowsLive(hipStream_t st, const RjImageDev *imgs, int nimg, const RjLive &lv, RjCoefBuf coefs,
                          const RjTableSet *tabsets, uint32_t *wide_cnt, uint2 *wide_list, uint32_t extra_lds = 0);
hipError_t LaunchRowsRest(hipStream_t st, const RjImageDev *imgs, int nimg, const RjLive &lv, RjCoefBuf coefs,
                          const RjTableSet *tabsets, uint32_t *wide_cnt, uint2 *wide_list);
// The split-aware instance alone over an (image, row) list, decoding only the rows whose head met
// its tail (the other split rows were published whole).
hipError_t LaunchRowsSplit(hipStream_t st, const RjImageDev *imgs, int nimg, const uint2 *split_rows,
                           uint32_t nsplit_rows, RjCoefBuf coefs, const RjTableSet *tabsets, uint32_t *wide_cnt,
                           uint2 *wide_list);
// The fix-up launch of one K2 launch's list (same variant; cap = that launch's rows).
hipError_t LaunchRowsFix(hipStream_t st, bool to_planes, bool dense, const RjImageDev *imgs, int nimg, RjCoefBuf coefs,
                         const RjTableSet *tabsets, uint8_t *planes, const uint32_t *wide_cnt, const uint2 *wide_list,
                         uint32_t cap);

// K1p (rj_prog.hip): progressive scans, one lane per restart interval of one scan; `lanes`
// lists batch-global interval indices (RjImageDev.pival_prefix), grouped so every wave holds
// one scan kind (0xFFFFFFFF: padding).  One launch per dependency level.
hipError_t LaunchProgressive(hipStream_t st, const RjImageDev *imgs, int nimg, const uint32_t *lanes, uint32_t nlanes,
                             const uint8_t *destuffed, uint32_t *coef, unsigned long long *nz,
                             unsigned long long *recs);
// K1p AC scans, one wave per interval (n intervals listed in ivals, batch-global indices): AC
// refinement, and AC first scans (pipelined launch: progress != null, scans in level order).
hipError_t LaunchProgressiveWave(hipStream_t st, const RjImageDev *imgs, int nimg, const uint32_t *ivals, uint32_t n,
                                 const uint8_t *destuffed, uint32_t *coef, unsigned long long *nz,
                                 unsigned long long *recs, uint32_t *progress, uint32_t progress_n,
                                 unsigned long long *stamps = nullptr, uint32_t flags = 0);
// k_prog_fold: level `level`'s refinement records into the dense coefficients / nonzero masks.
hipError_t LaunchProgressiveFold(hipStream_t st, const RjImageDev *imgs, const RjFoldJob *jobs, uint32_t njobs,
                                 uint32_t nchunks, uint32_t level, uint32_t *coef, unsigned long long *nz,
                                 const unsigned long long *recs);

// K2 over progressive images' MCU rows: dense coefficients (RjCoefBuf.dense) instead of entries.
hipError_t LaunchRowsDense(hipStream_t st, bool to_planes, const RjImageDev *imgs, int nimg, const uint32_t *row_prefix,
                           uint32_t nrows, RjCoefBuf coefs, const RjTableSet *tabsets, uint8_t *planes,
                           uint32_t *wide_cnt, uint2 *wide_list);

// GPU marker scan (rj_scan.hip): one wave per stream.
hipError_t LaunchScan(hipStream_t st, const RjScanJob *jobs, uint32_t njobs, const uint8_t *arena);

#ifdef RJ_EXP_STAMPS
void DumpRowStamps();
#endif
#ifdef RJ_HL_STAMPS
void DumpHuffStamps();
#endif

}  // namespace rj
