/*
 * rocjpeg.h -- public C ABI of the MI355X-native rocJPEG drop-in (librocjpeg_amd.so).
 *
 * Every type, enumerator value, struct layout and function signature here is the one
 * declared by the reference's api/rocjpeg.h (fgladwin/rocJPEG @ 2025-03-03), so code
 * written against rocJPEG compiles and links unchanged.  Per-item citations are
 * api/rocjpeg.h line numbers in the reference.
 *
 * Behavioural contract (matches the reference, src/rocjpeg_api.cpp / rocjpeg_decoder.cpp):
 *   - handles are opaque heap objects; *Create allocates, *Destroy frees;
 *   - a parsed stream BORROWS the caller's bitstream until the next parse/destroy;
 *   - destinations are caller-allocated device memory on the handle's device;
 *   - decode calls are synchronous (they return after the work has completed);
 *   - a handle serialises its own calls; use one handle per host thread to scale.
 * Difference by design: the decode core is a set of HIP kernels (Huffman per restart
 * interval, ISLOW IDCT, chroma upsample, colour conversion) instead of the VCN engine;
 * both ROCJPEG_BACKEND_HARDWARE and ROCJPEG_BACKEND_HYBRID select it.
 */
#ifndef ROC_JPEG_H
#define ROC_JPEG_H

#define ROCJPEGAPI

#include <stddef.h>
#include <stdint.h>
#include "rocjpeg_version.h"
/* The reference header pulls in the HIP runtime (api/rocjpeg.h:28) and its callers rely on
 * that for hipMalloc & co.; keep that source compatibility when HIP is installed.  Nothing
 * in this ABI uses a HIP type. */
#if !defined(ROCJPEG_NO_HIP_INCLUDE) && defined(__has_include)
#if __has_include(<hip/hip_runtime.h>)
#include <hip/hip_runtime.h>
#endif
#endif

#if defined(__cplusplus)
extern "C" {
#endif

/* api/rocjpeg.h:46 */
#define ROCJPEG_MAX_COMPONENT 4

/* api/rocjpeg.h:53-67 */
typedef enum {
  ROCJPEG_STATUS_SUCCESS = 0,
  ROCJPEG_STATUS_NOT_INITIALIZED = -1,
  ROCJPEG_STATUS_INVALID_PARAMETER = -2,
  ROCJPEG_STATUS_BAD_JPEG = -3,
  ROCJPEG_STATUS_JPEG_NOT_SUPPORTED = -4,
  ROCJPEG_STATUS_OUTOF_MEMORY = -5,
  ROCJPEG_STATUS_EXECUTION_FAILED = -6,
  ROCJPEG_STATUS_ARCH_MISMATCH = -7,
  ROCJPEG_STATUS_INTERNAL_ERROR = -8,
  ROCJPEG_STATUS_IMPLEMENTATION_NOT_SUPPORTED = -9,
  ROCJPEG_STATUS_HW_JPEG_DECODER_NOT_SUPPORTED = -10,
  ROCJPEG_STATUS_RUNTIME_ERROR = -11,
  ROCJPEG_STATUS_NOT_IMPLEMENTED = -12,
} RocJpegStatus;

/* api/rocjpeg.h:86-94 */
typedef enum {
  ROCJPEG_CSS_444 = 0,
  ROCJPEG_CSS_440 = 1,
  ROCJPEG_CSS_422 = 2,
  ROCJPEG_CSS_420 = 3,
  ROCJPEG_CSS_411 = 4,
  ROCJPEG_CSS_400 = 5,
  ROCJPEG_CSS_UNKNOWN = -1
} RocJpegChromaSubsampling;

/* api/rocjpeg.h:104-107: per-channel device pointer and pitch in bytes */
typedef struct {
  uint8_t *channel[ROCJPEG_MAX_COMPONENT];
  uint32_t pitch[ROCJPEG_MAX_COMPONENT];
} RocJpegImage;

/* api/rocjpeg.h:124-141
 *   NATIVE     : 4:4:4 / 4:4:0 -> Y,U,V planes; 4:2:2 -> packed YUYV in channel 0;
 *                4:2:0 -> Y + interleaved UV (NV12); 4:0:0 -> Y
 *   YUV_PLANAR : Y, U, V planes (4:0:0 -> Y only)
 *   Y          : luma only
 *   RGB        : interleaved RGB in channel 0
 *   RGB_PLANAR : R, G, B planes (all three use pitch[0], as the reference does) */
typedef enum {
  ROCJPEG_OUTPUT_NATIVE = 0,
  ROCJPEG_OUTPUT_YUV_PLANAR = 1,
  ROCJPEG_OUTPUT_Y = 2,
  ROCJPEG_OUTPUT_RGB = 3,
  ROCJPEG_OUTPUT_RGB_PLANAR = 4,
  ROCJPEG_OUTPUT_FORMAT_MAX = 5
} RocJpegOutputFormat;

/* api/rocjpeg.h:153-166 (target_dimension is reserved/unused, as in the reference) */
typedef struct {
  RocJpegOutputFormat output_format;
  struct {
    int16_t left;
    int16_t top;
    int16_t right;
    int16_t bottom;
  } crop_rectangle;
  struct {
    uint32_t width;
    uint32_t height;
  } target_dimension;
} RocJpegDecodeParams;

/* api/rocjpeg.h:176-179 */
typedef enum {
  ROCJPEG_BACKEND_HARDWARE = 0,
  ROCJPEG_BACKEND_HYBRID = 1
} RocJpegBackend;

/* api/rocjpeg.h:187, 241 */
typedef void *RocJpegStreamHandle;
typedef void *RocJpegHandle;

/* api/rocjpeg.h:204 -- allocate a stream handle */
RocJpegStatus ROCJPEGAPI rocJpegStreamCreate(RocJpegStreamHandle *jpeg_stream_handle);

/* api/rocjpeg.h:219 -- parse headers; builds the restart-interval table.  The stream keeps
 * pointing into `data` (no copy) until the next parse or destroy. */
RocJpegStatus ROCJPEGAPI rocJpegStreamParse(const unsigned char *data, size_t length,
                                            RocJpegStreamHandle jpeg_stream_handle);

/* api/rocjpeg.h:234 */
RocJpegStatus ROCJPEGAPI rocJpegStreamDestroy(RocJpegStreamHandle jpeg_stream_handle);

/* api/rocjpeg.h:258 -- bind a decoder to HIP device `device_id` (own stream, own arena) */
RocJpegStatus ROCJPEGAPI rocJpegCreate(RocJpegBackend backend, int device_id, RocJpegHandle *handle);

/* api/rocjpeg.h:273 */
RocJpegStatus ROCJPEGAPI rocJpegDestroy(RocJpegHandle handle);

/* api/rocjpeg.h:296 -- widths/heights are uint32_t[4]; chroma sizes use floor division */
RocJpegStatus ROCJPEGAPI rocJpegGetImageInfo(RocJpegHandle handle, RocJpegStreamHandle jpeg_stream_handle,
                                             uint8_t *num_components, RocJpegChromaSubsampling *subsampling,
                                             uint32_t *widths, uint32_t *heights);

/* api/rocjpeg.h:314 */
RocJpegStatus ROCJPEGAPI rocJpegDecode(RocJpegHandle handle, RocJpegStreamHandle jpeg_stream_handle,
                                       const RocJpegDecodeParams *decode_params, RocJpegImage *destination);

/* api/rocjpeg.h:331 -- decode_params shared by the whole batch */
RocJpegStatus ROCJPEGAPI rocJpegDecodeBatched(RocJpegHandle handle, RocJpegStreamHandle *jpeg_stream_handles,
                                              int batch_size, const RocJpegDecodeParams *decode_params,
                                              RocJpegImage *destinations);

/* api/rocjpeg.h:343 */
extern const char *ROCJPEGAPI rocJpegGetErrorName(RocJpegStatus rocjpeg_status);

#if defined(__cplusplus)
}
#endif

#endif /* ROC_JPEG_H */
