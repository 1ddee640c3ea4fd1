/*
 * jpegdecode_c.c -- a plain C caller of the drop-in C ABI (include/rocjpeg.h), written for this
 * repository's tests.  It follows the call sequence of the reference sample
 * samples/jpegDecode/jpegdecode.cpp:72-163 (stream create/parse, decoder create, image info,
 * caller-allocated device planes sized as samples/rocjpeg_samples_utils.h:318-399 sizes them,
 * rocJpegDecode, copy back) and, with several files, the batched one of
 * samples/jpegDecodeBatched/jpegdecodebatched.cpp:82-194.  Only the nine reference entry points
 * and the HIP runtime are used.
 *
 *   jpegdecode_c <fmt> <out.raw> <in1.jpg> [in2.jpg ...]
 *
 * fmt: the RocJpegOutputFormat value.  Writes, per input, every channel's pitch x rows bytes
 * back to back into out.raw.  Exit code 0 = all decoded.
 */
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rocjpeg.h"

#define CHECK(call)                                                                         \
  do {                                                                                      \
    RocJpegStatus st_ = (call);                                                             \
    if (st_ != ROCJPEG_STATUS_SUCCESS) {                                                    \
      fprintf(stderr, "%s failed: %s\n", #call, rocJpegGetErrorName(st_));                  \
      return 2;                                                                             \
    }                                                                                       \
  } while (0)

static unsigned char *read_file(const char *path, size_t *n) {
  FILE *f = fopen(path, "rb");
  if (!f) return NULL;
  fseek(f, 0, SEEK_END);
  long len = ftell(f);
  fseek(f, 0, SEEK_SET);
  unsigned char *b = (unsigned char *)malloc((size_t)len);
  if (b && fread(b, 1, (size_t)len, f) != (size_t)len) {
    free(b);
    b = NULL;
  }
  fclose(f);
  *n = (size_t)len;
  return b;
}

/* channel sizes as the reference samples compute them (rocjpeg_samples_utils.h:318-399) */
static int channel_sizes(RocJpegOutputFormat fmt, RocJpegChromaSubsampling css, const uint32_t *w, const uint32_t *h,
                         uint32_t rows[4], uint32_t pitch[4]) {
  memset(rows, 0, 4 * sizeof(uint32_t));
  memset(pitch, 0, 4 * sizeof(uint32_t));
  const uint32_t W = w[0], H = h[0];
  switch (fmt) {
    case ROCJPEG_OUTPUT_NATIVE:
      if (css == ROCJPEG_CSS_444) { for (int c = 0; c < 3; c++) { rows[c] = H; pitch[c] = W; } return 3; }
      if (css == ROCJPEG_CSS_440) { rows[0] = H; pitch[0] = W; rows[1] = rows[2] = H >> 1; pitch[1] = pitch[2] = W; return 3; }
      if (css == ROCJPEG_CSS_422) { rows[0] = H; pitch[0] = 2 * W; return 1; }
      if (css == ROCJPEG_CSS_420) { rows[0] = H; pitch[0] = W; rows[1] = H >> 1; pitch[1] = W; return 2; }
      rows[0] = H; pitch[0] = W; return 1;
    case ROCJPEG_OUTPUT_YUV_PLANAR:
      if (css == ROCJPEG_CSS_400) { rows[0] = H; pitch[0] = W; return 1; }
      rows[0] = H; pitch[0] = W;
      for (int c = 1; c < 3; c++) { rows[c] = h[c]; pitch[c] = w[c]; }
      return 3;
    case ROCJPEG_OUTPUT_Y:
      rows[0] = H; pitch[0] = W; return 1;
    case ROCJPEG_OUTPUT_RGB:
      rows[0] = H; pitch[0] = 3 * W; return 1;
    case ROCJPEG_OUTPUT_RGB_PLANAR:
      for (int c = 0; c < 3; c++) { rows[c] = H; pitch[c] = W; }
      return 3;
    default:
      return 0;
  }
}

int main(int argc, char **argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: %s <fmt> <out.raw> <in.jpg>...\n", argv[0]);
    return 1;
  }
  const RocJpegOutputFormat fmt = (RocJpegOutputFormat)atoi(argv[1]);
  const int n = argc - 3;
  FILE *out = fopen(argv[2], "wb");
  if (!out) return 1;

  RocJpegHandle handle;
  CHECK(rocJpegCreate(ROCJPEG_BACKEND_HARDWARE, 0, &handle));
  RocJpegStreamHandle *streams = (RocJpegStreamHandle *)calloc((size_t)n, sizeof(RocJpegStreamHandle));
  RocJpegImage *images = (RocJpegImage *)calloc((size_t)n, sizeof(RocJpegImage));
  unsigned char **bytes = (unsigned char **)calloc((size_t)n, sizeof(unsigned char *));
  uint32_t (*rows)[4] = calloc((size_t)n, sizeof(*rows));
  int *nch = (int *)calloc((size_t)n, sizeof(int));
  for (int i = 0; i < n; i++) {
    size_t len = 0;
    bytes[i] = read_file(argv[3 + i], &len);
    if (!bytes[i]) return 1;
    CHECK(rocJpegStreamCreate(&streams[i]));
    CHECK(rocJpegStreamParse(bytes[i], len, streams[i]));
    uint8_t num_components;
    RocJpegChromaSubsampling css;
    uint32_t w[ROCJPEG_MAX_COMPONENT], h[ROCJPEG_MAX_COMPONENT];
    CHECK(rocJpegGetImageInfo(handle, streams[i], &num_components, &css, w, h));
    uint32_t pitch[4];
    nch[i] = channel_sizes(fmt, css, w, h, rows[i], pitch);
    for (int c = 0; c < nch[i]; c++) {
      if (hipMalloc((void **)&images[i].channel[c], (size_t)pitch[c] * rows[i][c]) != hipSuccess) return 3;
      /* a known fill, so that bytes the decoder does not write compare equal to the oracle's */
      if (hipMemset(images[i].channel[c], 0xA5, (size_t)pitch[c] * rows[i][c]) != hipSuccess) return 3;
      images[i].pitch[c] = pitch[c];
    }
  }
  RocJpegDecodeParams params;
  memset(&params, 0, sizeof(params));
  params.output_format = fmt;
  if (n == 1) CHECK(rocJpegDecode(handle, streams[0], &params, &images[0]));
  else CHECK(rocJpegDecodeBatched(handle, streams, n, &params, images));
  for (int i = 0; i < n; i++) {
    for (int c = 0; c < nch[i]; c++) {
      const size_t sz = (size_t)images[i].pitch[c] * rows[i][c];
      unsigned char *hbuf = (unsigned char *)malloc(sz);
      if (hipMemcpy(hbuf, images[i].channel[c], sz, hipMemcpyDeviceToHost) != hipSuccess) return 3;
      fwrite(hbuf, 1, sz, out);
      free(hbuf);
      (void)hipFree(images[i].channel[c]);
    }
    CHECK(rocJpegStreamDestroy(streams[i]));
    free(bytes[i]);
  }
  CHECK(rocJpegDestroy(handle));
  fclose(out);
  printf("decoded %d image(s)\n", n);
  return 0;
}
