/* abi_probe.c -- prints the binary layout of the rocJPEG API types as JSON, and fails to compile
 * unless every entry point has the reference signature (api/rocjpeg.h:204-343).  Built twice by
 * tests/test_abi_cpu.py: against include/rocjpeg.h and against the reference header where it lies
 * (/root/reference/api); the two outputs must be identical for a relink drop-in. */
#include <stddef.h>
#include <stdio.h>

#include "rocjpeg.h"

typedef RocJpegStatus (*p_stream_create)(RocJpegStreamHandle *);
typedef RocJpegStatus (*p_stream_parse)(const unsigned char *, size_t, RocJpegStreamHandle);
typedef RocJpegStatus (*p_stream_destroy)(RocJpegStreamHandle);
typedef RocJpegStatus (*p_create)(RocJpegBackend, int, RocJpegHandle *);
typedef RocJpegStatus (*p_destroy)(RocJpegHandle);
typedef RocJpegStatus (*p_info)(RocJpegHandle, RocJpegStreamHandle, uint8_t *, RocJpegChromaSubsampling *, uint32_t *,
                                uint32_t *);
typedef RocJpegStatus (*p_decode)(RocJpegHandle, RocJpegStreamHandle, const RocJpegDecodeParams *, RocJpegImage *);
typedef RocJpegStatus (*p_batched)(RocJpegHandle, RocJpegStreamHandle *, int, const RocJpegDecodeParams *,
                                   RocJpegImage *);
typedef const char *(*p_errname)(RocJpegStatus);

#ifdef ABI_SIGNATURES
/* compiled (-c, never linked or called) with -DABI_SIGNATURES: each assignment type-checks a
 * declaration against the reference signature */
void abi_probe_signatures(void **out) {
  p_stream_create a = rocJpegStreamCreate;
  p_stream_parse b = rocJpegStreamParse;
  p_stream_destroy c = rocJpegStreamDestroy;
  p_create d = rocJpegCreate;
  p_destroy e = rocJpegDestroy;
  p_info f = rocJpegGetImageInfo;
  p_decode g = rocJpegDecode;
  p_batched h = rocJpegDecodeBatched;
  p_errname i = rocJpegGetErrorName;
  out[0] = (void *)a; out[1] = (void *)b; out[2] = (void *)c; out[3] = (void *)d; out[4] = (void *)e;
  out[5] = (void *)f; out[6] = (void *)g; out[7] = (void *)h; out[8] = (void *)i;
}
#endif

#define F(t, m) printf("\"%s.%s\": [%zu, %zu],\n", #t, #m, offsetof(t, m), sizeof(((t *)0)->m))
#define E(v) printf("\"%s\": %d,\n", #v, (int)(v))
int main(void) {
  printf("{\n");
  printf("\"sizeof.RocJpegImage\": %zu,\n\"sizeof.RocJpegDecodeParams\": %zu,\n", sizeof(RocJpegImage),
         sizeof(RocJpegDecodeParams));
  printf("\"sizeof.RocJpegStatus\": %zu,\n\"sizeof.RocJpegChromaSubsampling\": %zu,\n", sizeof(RocJpegStatus),
         sizeof(RocJpegChromaSubsampling));
  printf("\"sizeof.RocJpegOutputFormat\": %zu,\n\"sizeof.RocJpegBackend\": %zu,\n", sizeof(RocJpegOutputFormat),
         sizeof(RocJpegBackend));
  printf("\"sizeof.handles\": [%zu, %zu],\n", sizeof(RocJpegHandle), sizeof(RocJpegStreamHandle));
  F(RocJpegImage, channel); F(RocJpegImage, pitch);
  F(RocJpegDecodeParams, output_format); F(RocJpegDecodeParams, crop_rectangle);
  F(RocJpegDecodeParams, crop_rectangle.left); F(RocJpegDecodeParams, crop_rectangle.top);
  F(RocJpegDecodeParams, crop_rectangle.right); F(RocJpegDecodeParams, crop_rectangle.bottom);
  F(RocJpegDecodeParams, target_dimension); F(RocJpegDecodeParams, target_dimension.width);
  F(RocJpegDecodeParams, target_dimension.height);
  E(ROCJPEG_MAX_COMPONENT);
  E(ROCJPEG_STATUS_SUCCESS); E(ROCJPEG_STATUS_NOT_INITIALIZED); E(ROCJPEG_STATUS_INVALID_PARAMETER);
  E(ROCJPEG_STATUS_BAD_JPEG); E(ROCJPEG_STATUS_JPEG_NOT_SUPPORTED); E(ROCJPEG_STATUS_OUTOF_MEMORY);
  E(ROCJPEG_STATUS_EXECUTION_FAILED); E(ROCJPEG_STATUS_ARCH_MISMATCH); E(ROCJPEG_STATUS_INTERNAL_ERROR);
  E(ROCJPEG_STATUS_IMPLEMENTATION_NOT_SUPPORTED); E(ROCJPEG_STATUS_HW_JPEG_DECODER_NOT_SUPPORTED);
  E(ROCJPEG_STATUS_RUNTIME_ERROR); E(ROCJPEG_STATUS_NOT_IMPLEMENTED);
  E(ROCJPEG_CSS_444); E(ROCJPEG_CSS_440); E(ROCJPEG_CSS_422); E(ROCJPEG_CSS_420); E(ROCJPEG_CSS_411);
  E(ROCJPEG_CSS_400); E(ROCJPEG_CSS_UNKNOWN);
  E(ROCJPEG_OUTPUT_NATIVE); E(ROCJPEG_OUTPUT_YUV_PLANAR); E(ROCJPEG_OUTPUT_Y); E(ROCJPEG_OUTPUT_RGB);
  E(ROCJPEG_OUTPUT_RGB_PLANAR); E(ROCJPEG_OUTPUT_FORMAT_MAX);
  E(ROCJPEG_BACKEND_HARDWARE); E(ROCJPEG_BACKEND_HYBRID);
  printf("\"end\": 0\n}\n");
  return 0;
}
