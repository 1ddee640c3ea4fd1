/*
 * jpegdecode_sharded_c.c -- a plain C caller of the multi-GPU batched decode behind the C ABI
 * (include/rocjpeg_amd.h rocJpegAmdDecodeBatchedSharded), written for this repository's tests.
 * One process per rank, forked before any HIP call (the jpegdecodeperf sample's one-handle-per-
 * thread scaling, samples/jpegDecodePerf/jpegdecodeperf.cpp:228-257, as processes): rank 0 makes
 * the communicator id and sends it to the other ranks through pipes; every rank opens its GPU
 * (rank modulo the visible devices), joins the communicator, and decodes its shard of the files
 * with one rocJpegAmdDecodeBatchedSharded call.
 *
 *   jpegdecode_sharded_c <nranks> <fmt> <out_prefix> <in1.jpg> [in2.jpg ...]
 *
 * Rank r writes <out_prefix>.<r>: per image it decoded, a uint32 batch index, a uint32 byte
 * count, then every channel's pitch x rows bytes.  Exit code 0 = every rank succeeded.
 */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/wait.h>
#include <unistd.h>

#include "rocjpeg.h"
#include "rocjpeg_amd.h"

#define CHECK(call)                                                                         \
  do {                                                                                      \
    RocJpegStatus st_ = (call);                                                             \
    if (st_ != ROCJPEG_STATUS_SUCCESS) {                                                    \
      fprintf(stderr, "rank %d: %s failed: %s\n", rank, #call, rocJpegGetErrorName(st_));   \
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

/* RGB-family and planar sizes (rocjpeg_samples_utils.h:318-399), enough for this test's formats */
static int channel_sizes(RocJpegOutputFormat fmt, RocJpegChromaSubsampling css, const uint32_t *w, const uint32_t *h,
                         uint32_t rows[4], uint32_t pitch[4]) {
  memset(rows, 0, 4 * sizeof(uint32_t));
  memset(pitch, 0, 4 * sizeof(uint32_t));
  switch (fmt) {
    case ROCJPEG_OUTPUT_RGB: rows[0] = h[0]; pitch[0] = 3 * w[0]; return 1;
    case ROCJPEG_OUTPUT_RGB_PLANAR: for (int c = 0; c < 3; c++) { rows[c] = h[0]; pitch[c] = w[0]; } return 3;
    case ROCJPEG_OUTPUT_Y: rows[0] = h[0]; pitch[0] = w[0]; return 1;
    case ROCJPEG_OUTPUT_YUV_PLANAR:
      rows[0] = h[0]; pitch[0] = w[0];
      if (css == ROCJPEG_CSS_400) return 1;
      for (int c = 1; c < 3; c++) { rows[c] = h[c]; pitch[c] = w[c]; }
      return 3;
    default: return 0;
  }
}

static int run_rank(int rank, int nranks, int fd_in, const int *fd_out, RocJpegOutputFormat fmt, const char *prefix,
                    int n, char **files) {
  RocJpegAmdCommId id;
  if (rank == 0) {
    CHECK(rocJpegAmdCommGetUniqueId(&id));
    for (int r = 1; r < nranks; r++)
      if (write(fd_out[r], &id, sizeof(id)) != (ssize_t)sizeof(id)) return 4;
  } else if (read(fd_in, &id, sizeof(id)) != (ssize_t)sizeof(id)) {
    return 4;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) return 3;
  const int dev = rank % ndev;
  if (hipSetDevice(dev) != hipSuccess) return 3;
  RocJpegAmdComm comm;
  CHECK(rocJpegAmdCommInitRank(dev, nranks, &id, rank, &comm));
  RocJpegHandle handle;
  CHECK(rocJpegCreate(ROCJPEG_BACKEND_HARDWARE, dev, &handle));

  /* the batch as one blob every rank reads (a dataset file on the node in a real job) */
  uint64_t *offs = (uint64_t *)calloc((size_t)n, sizeof(uint64_t));
  uint32_t *sizes = (uint32_t *)calloc((size_t)n, sizeof(uint32_t));
  unsigned char **bytes = (unsigned char **)calloc((size_t)n, sizeof(unsigned char *));
  uint64_t total = 0;
  for (int i = 0; i < n; i++) {
    size_t len = 0;
    bytes[i] = read_file(files[i], &len);
    if (!bytes[i]) return 1;
    offs[i] = total;
    sizes[i] = (uint32_t)len;
    total += len;
  }
  unsigned char *blob = (unsigned char *)malloc((size_t)total);
  for (int i = 0; i < n; i++) memcpy(blob + offs[i], bytes[i], sizes[i]);

  /* destinations for every image (a rank only touches its own); sizes from a parse on this rank */
  RocJpegImage *images = (RocJpegImage *)calloc((size_t)n, sizeof(RocJpegImage));
  uint32_t (*rows)[4] = calloc((size_t)n, sizeof(*rows));
  int *nch = (int *)calloc((size_t)n, sizeof(int));
  for (int i = 0; i < n; i++) {
    RocJpegStreamHandle s;
    CHECK(rocJpegStreamCreate(&s));
    CHECK(rocJpegStreamParse(bytes[i], sizes[i], s));
    uint8_t nc;
    RocJpegChromaSubsampling css;
    uint32_t w[ROCJPEG_MAX_COMPONENT], h[ROCJPEG_MAX_COMPONENT], pitch[4];
    CHECK(rocJpegGetImageInfo(handle, s, &nc, &css, w, h));
    CHECK(rocJpegStreamDestroy(s));
    nch[i] = channel_sizes(fmt, css, w, h, rows[i], pitch);
    for (int c = 0; c < nch[i]; c++) {
      if (hipMalloc((void **)&images[i].channel[c], (size_t)pitch[c] * rows[i][c]) != hipSuccess) return 3;
      if (hipMemset(images[i].channel[c], 0xA5, (size_t)pitch[c] * rows[i][c]) != hipSuccess) return 3;
      images[i].pitch[c] = pitch[c];
    }
  }
  RocJpegDecodeParams params;
  memset(&params, 0, sizeof(params));
  params.output_format = fmt;
  RocJpegAmdWorkItem *table = (RocJpegAmdWorkItem *)calloc((size_t)n, sizeof(RocJpegAmdWorkItem));
  CHECK(rocJpegAmdDecodeBatchedSharded(handle, comm, blob, total, offs, sizes, n, &params, images, table));

  char path[4096];
  snprintf(path, sizeof(path), "%s.%d", prefix, rank);
  FILE *out = fopen(path, "wb");
  if (!out) return 1;
  int mine = 0;
  for (int i = 0; i < n; i++) {
    if (table[i].shard != rank) continue;
    const uint32_t idx = table[i].index;
    uint32_t nbytes = 0;
    for (int c = 0; c < nch[idx]; c++) nbytes += images[idx].pitch[c] * rows[idx][c];
    fwrite(&idx, 4, 1, out);
    fwrite(&nbytes, 4, 1, out);
    for (int c = 0; c < nch[idx]; c++) {
      const size_t sz = (size_t)images[idx].pitch[c] * rows[idx][c];
      unsigned char *hbuf = (unsigned char *)malloc(sz);
      if (hipMemcpy(hbuf, images[idx].channel[c], sz, hipMemcpyDeviceToHost) != hipSuccess) return 3;
      fwrite(hbuf, 1, sz, out);
      free(hbuf);
    }
    mine++;
  }
  fclose(out);
  for (int i = 0; i < n; i++)
    for (int c = 0; c < nch[i]; c++) (void)hipFree(images[i].channel[c]);
  CHECK(rocJpegDestroy(handle));
  CHECK(rocJpegAmdCommDestroy(comm));
  printf("rank %d/%d on device %d: decoded %d of %d image(s)\n", rank, nranks, dev, mine, n);
  return 0;
}

int main(int argc, char **argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: %s <nranks> <fmt> <out_prefix> <in.jpg>...\n", argv[0]);
    return 1;
  }
  const int nranks = atoi(argv[1]);
  const RocJpegOutputFormat fmt = (RocJpegOutputFormat)atoi(argv[2]);
  if (nranks < 1 || nranks > 16) return 1;
  int fds[16][2];
  int wr[16];
  for (int r = 0; r < nranks; r++) {
    if (pipe(fds[r]) != 0) return 1;
    wr[r] = fds[r][1];
  }
  pid_t pids[16];
  for (int r = 0; r < nranks; r++) {  /* fork before this process touches the GPU */
    pids[r] = fork();
    if (pids[r] < 0) return 1;
    if (pids[r] == 0) _exit(run_rank(r, nranks, fds[r][0], wr, fmt, argv[3], argc - 4, argv + 4));
  }
  int rc = 0;
  for (int r = 0; r < nranks; r++) {
    int status = 0;
    if (waitpid(pids[r], &status, 0) < 0 || !WIFEXITED(status) || WEXITSTATUS(status) != 0) rc = 5;
  }
  return rc;
}
