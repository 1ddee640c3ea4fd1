// rj_kernels.h -- host-side launchers of the gfx950 decode kernels (rj_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rj_device.h"

namespace rj {

// K0: byte-unstuffing of every restart interval (one wavefront per interval).
hipError_t LaunchDestuff(hipStream_t st, const RjImageDev *imgs, int nimg, uint32_t nseg, uint8_t *destuffed,
                         uint32_t *seg_len);

// K1: Huffman entropy decode, one lane per restart interval -> sparse coefficients.
hipError_t LaunchHuffman(hipStream_t st, const RjImageDev *imgs, int nimg, uint32_t nseg, const uint8_t *destuffed,
                         const uint32_t *seg_len, const RjTableSet *tabsets, RjCoefBuf coefs);

// K2a (general path): dequantise + ISLOW IDCT of every block into MCU-padded component planes.
hipError_t LaunchIdctPlanes(hipStream_t st, const RjImageDev *imgs, int nimg, uint64_t nblocks, RjCoefBuf coefs,
                            const RjTableSet *tabsets, uint8_t *planes);

// K2b (general path): every output format / ROI of rocjpeg_decoder.cpp:143-180 from the planes.
hipError_t LaunchOutputJobs(hipStream_t st, const RjImageDev *imgs, const RjJobDev *jobs, int njobs, uint32_t total_rows,
                            const uint8_t *planes);

// K2 (fused fast path): dequant + IDCT + nearest upsample + YUV->RGB / layout straight from the
// coefficients to the caller's buffers, one single-wave workgroup per MCU row (looping over the
// row's strips); row_prefix[i] = first row of image i (fused images only).  Only for images whose
// output window is tile-local (no ROI quirks); see rj_decoder.cpp::FusedEligible.
hipError_t LaunchFusedOutput(hipStream_t st, const RjImageDev *imgs, int nimg, const uint32_t *row_prefix,
                             uint32_t nrows, RjCoefBuf coefs, const RjTableSet *tabsets);

}  // namespace rj
