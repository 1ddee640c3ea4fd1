/*
 * rocjpeg_amd.h -- extensions of the MI355X-native rocJPEG drop-in.  Nothing here is needed
 * to use the reference API; these entry points exist for measurement and data staging.
 */
#ifndef ROC_JPEG_AMD_H
#define ROC_JPEG_AMD_H

#include "rocjpeg.h"

#if defined(__cplusplus)
extern "C" {
#endif

/* Parse-only image info that needs no decoder handle (rocJpegGetImageInfo requires one).
 * num_restart_intervals: baseline -- restart intervals of the scan; progressive (SOF2) -- the
 * restart intervals summed over all scans. */
RocJpegStatus rocJpegAmdStreamGetInfo(RocJpegStreamHandle stream, uint8_t *num_components,
                                      RocJpegChromaSubsampling *subsampling, uint32_t *widths, uint32_t *heights,
                                      uint32_t *num_restart_intervals);

/* Stage the entropy-coded bytes and restart-interval tables of parsed streams in the HBM of
 * the handle's device.  A later rocJpegDecode[Batched] on the same handle then reads them
 * from HBM instead of copying from host memory.  The copy is dropped when the stream is
 * re-parsed or destroyed. */
RocJpegStatus rocJpegAmdStreamsToDevice(RocJpegHandle handle, RocJpegStreamHandle *streams, int count);

/* rocJpegStreamParse of `count` streams followed by rocJpegAmdStreamsToDevice, with the O(bytes)
 * part of the parse on the handle's GPU: the host reads only the headers; one kernel
 * (rj_scan.hip) finds each entropy-coded segment's end (the first FF D9, as the reference's
 * ParseEOI, src/rocjpeg_parser.cpp:400-416) and builds the restart-interval and destuffing
 * tables in HBM.  The parsed streams are identical to host-parsed ones (same info, same tables)
 * and resident on the handle's device.  Progressive (SOF2) streams are parsed on the host.
 * Returns the first failure as rocJpegStreamParse would (BAD_JPEG). */
RocJpegStatus rocJpegAmdStreamParseDevice(RocJpegHandle handle, const unsigned char *const *data,
                                          const size_t *lengths, int count, RocJpegStreamHandle *streams);

/* Introspection of a parsed stream's restart-interval table (tests / tooling). */
typedef struct {
  uint32_t src_off, src_len;   /* raw entropy-coded bytes of the interval (ECS-relative) */
  uint32_t dst_off, dst_len;   /* destuffed bytes */
  uint32_t mcu_first, mcu_count;
  uint32_t flags;              /* 1: the interval's restart marker was missing */
  uint32_t ent_off, chunk0, reserved;
} RocJpegAmdInterval;
RocJpegStatus rocJpegAmdStreamGetIntervals(RocJpegStreamHandle stream, RocJpegAmdInterval *out, uint32_t capacity,
                                           uint32_t *count);
/* The destuffing work units: 4 x uint32 each {src_off, len | first-of-interval << 31, dst_off,
 * zero_end}; ecs_size: the entropy-coded segment length the parse found. */
RocJpegStatus rocJpegAmdStreamGetDestuffBlocks(RocJpegStreamHandle stream, uint32_t *out4, uint32_t capacity,
                                               uint32_t *count, uint32_t *ecs_size);

/* The lean K1 lookup tables of a parsed baseline stream (rj_device.h RjLeanTables: AC0, AC1
 * first levels + subtables, DC0, DC1, 32-bit entries), for tests and tooling; `bytes` is the
 * size of `out`, *needed receives the table image size. */
RocJpegStatus rocJpegAmdStreamGetLeanTables(RocJpegStreamHandle stream, void *out, size_t bytes, size_t *needed);

/* Per-stage device time of the most recent decode call, measured with HIP events on the
 * handle's internal stream (enable with rocJpegAmdSetProfiling first). */
typedef struct {
  float h2d_ms;       /* staging of non-resident bitstreams + descriptors */
  float destuff_ms;   /* K0 */
  float huffman_ms;   /* K1 */
  float idct_ms;      /* K2a (general path) or fused K2 (fast path) */
  float output_ms;    /* K2b (general path; 0 on the fused path) */
  float total_ms;
  uint64_t ecs_bytes;     /* entropy-coded bytes consumed */
  uint64_t coef_bytes;    /* int16 coefficient bytes written by K1 */
  uint64_t output_bytes;  /* bytes written to the caller's buffers */
  uint32_t images, intervals, fused_images;
  float host_ms;          /* host planning of the call (validation, layout, descriptors), wall clock */
  float entropy_chunks_ms;   /* K1 split into its launches: chunk lanes, */
  float entropy_resolve_ms;  /*   sync resolution, */
  float entropy_serial_ms;   /*   serial re-decode of intervals whose chunks did not sync */
  uint32_t chunks;           /* K1 lanes */
  uint32_t split_intervals;  /* intervals decoded in more than one chunk */
  uint32_t serial_fallbacks; /* of those, re-decoded serially (counted when profiling) */
  uint32_t pipe_groups;      /* interval length classes of a pipelined launch (1: sequential
                                K1 -> K2; >1: huffman_ms ends at the last class's K1 and idct_ms
                                is the K2 work left after it) */
  uint32_t pipe_lane_rows;   /* pipelined K2 rows taken from the K1 lane order (every interval
                                one MCU row) rather than from uploaded row lists */
  /* per-kernel launch durations (HIP events on each launch's own stream), summed over the
     call's launches of that kernel: K1 chunk/exact pass, K2 (k_rows) */
  float k1_launch_ms_sum, k2_launch_ms_sum;
  uint32_t k1_launches, k2_launches;
  uint64_t entry_bytes;      /* sparse coefficient entries K1 wrote (counted on the device) */
  /* progressive (SOF2) images of the call: K1p (all dependency levels) and their K2 rows */
  float prog_entropy_ms, prog_rows_ms;
  uint32_t prog_images, prog_intervals, prog_levels, prog_pad;
  uint64_t prog_coef_bytes;  /* dense coefficient bytes (int16 per coefficient) */
  /* rocJpegAmdStreamParseDevice (the last call on this handle): streams whose marker scan ran on
     the GPU, and those that fell back to the host scan (a scratch list overflowed) */
  uint32_t scan_device_streams, scan_host_fallbacks;
  /* progressive launches by kernel, [0] k_prog (first-scan and DC-refinement lanes), [1]
     k_prog_wave (AC scan waves: refinement, and first scans when pipelined), [2] k_prog_fold: summed launch durations (HIP events on
     each launch's stream), launch counts, and the algorithmic bytes of the call's launches
     (destuffed scan bytes read + coefficient / mask / record bytes written) */
  float prog_kernel_ms[3];
  uint32_t prog_kernel_launches[3];
  uint64_t prog_kernel_bytes[3];
  /* images whose destination was not on the handle's device (another GPU or host memory):
     decoded into device-local staging, then copied where the caller's pointers live */
  uint32_t routed_images;
  uint32_t lean_k1;          /* 1: K1 ran the lean row-interval kernel (rj_huff.hip, raw entries) */
  /* MCU rows with coefficients outside the int32 IDCT's exact domain (|coef x quant| >= 2^14:
     corrupt data with large quantisers), decoded again by the K2 fix-up launch in 64-bit */
  uint32_t wide_rows;
  /* lean K1 outlier split: intervals decoded by a head and a tail lane (rj_huff.hip) */
  uint32_t lean_split;
  /* 1: K1 ran the chunk-lane kernel on the lean machinery (rj_huff.hip k_huff_chunk) */
  uint32_t chunk_k1;
  /* the call's chunk length in bytes: intervals of at least twice this are cut into chunks */
  uint32_t chunk_bytes;
  /* MCU-phase hypotheses per speculative chunk (1: one lane per chunk; small calls: the MCU's
     block count, each speculative chunk decoded from every phase it may start in) */
  uint32_t chunk_hyp;
  /* 1: the lean K1 ran five decoder waves per CU (the overflow past one round of four as fifth
     waves, rj_huff.hip k_huff<RJ_HL_DEC5>) */
  uint32_t lean_five;
  /* live rows (K2 beside K1 inside the call): 1 when the call ran them; the rows the live K2
     decoded while K1 ran, the rows the stream-ordered K2 took after it; the live K2's launch span
     (from its stream's start, when K1 starts, to its last row) and the stream-ordered K2's span
     after K1 (rows no ticket took, synced split rows), HIP events on each launch's stream */
  uint32_t live, live_rows, rest_rows, live_pad;
  float live_ms, rest_ms;
  /* entry-buffer placement search: the K1 + K2 span (ms, HIP events) of each
     entry buffer tried on this handle's first large lean calls, how many were tried, the one kept
     (-1: the search is still running or was never started) */
  float place_ms[4];
  uint32_t place_tried;
  int32_t place_pick;
} RocJpegAmdTimings;

RocJpegStatus rocJpegAmdSetProfiling(RocJpegHandle handle, int enable);
RocJpegStatus rocJpegAmdGetLastTimings(RocJpegHandle handle, RocJpegAmdTimings *timings);

/* Select the output path: 0 = automatic (fused kernel where the output window allows it),
 * 1 = always the general two-stage path (IDCT to planes, then format conversion). */
RocJpegStatus rocJpegAmdSetPathPolicy(RocJpegHandle handle, int policy);

/* The handle's HIP stream (as void*), e.g. for external event timing. */
RocJpegStatus rocJpegAmdGetStream(RocJpegHandle handle, void **hip_stream);

/* ---- Multi-GPU batched decode: the per-image work table ----
 * The reference has one device per handle (src/rocjpeg_api.cpp:107-120) and no multi-GPU path;
 * its batched entry point (src/rocjpeg_decoder.cpp:196-292) is what each rank calls on its
 * shard.  Rank 0 reads only the headers of the batch (O(header) per image; progressive streams
 * are walked whole), builds one 64-byte record per image, assigns images to shards by greedy
 * LPT on a decode-cost estimate, and broadcasts the table (RCCL over xGMI); every rank then
 * parses and decodes the images of its own shard from the shared bitstream blob.  No pointers
 * cross ranks: `stream_offset` is an offset into the blob every rank can read. */
typedef struct {
  uint64_t stream_offset;      /* the JPEG's first byte in the caller's blob */
  uint32_t stream_bytes;       /* its length */
  uint32_t ecs_bytes;          /* entropy-coded bytes after the first SOS header (estimate) */
  uint32_t width, height;      /* luma size */
  int32_t subsampling;         /* RocJpegChromaSubsampling (-1 unknown) */
  uint32_t restart_intervals;  /* restart intervals of the scan (1 without DRI; progressive: 0) */
  uint32_t flags;              /* ROCJPEG_AMD_WORK_* */
  int32_t shard;               /* assigned shard (rank), -1 before rocJpegAmdAssignShards */
  int32_t dest_device;         /* device the decoded image is written on */
  uint32_t index;              /* position in the batch */
  uint64_t cost;               /* LPT weight: ROCJPEG_AMD_COST_BYTE x ecs_bytes + pixels
                                  + ROCJPEG_AMD_COST_INTERVAL x mean restart-interval bytes
                                  (capped at ROCJPEG_AMD_COST_INTERVAL_CAP); progressive:
                                  ROCJPEG_AMD_COST_BYTE_PROG per byte + pixels */
  uint64_t reserved;
} RocJpegAmdWorkItem;
#define ROCJPEG_AMD_WORK_PROGRESSIVE 1u
#define ROCJPEG_AMD_WORK_BAD 2u         /* header parse failed: cost 0, still assigned */
#define ROCJPEG_AMD_WORK_UNSUPPORTED 4u /* parsed, but the decode call would refuse it */
#define ROCJPEG_AMD_COST_BYTE 8u        /* measured: K1 spends ~8x per ECS byte what K2 spends per pixel */
#define ROCJPEG_AMD_COST_BYTE_PROG 120u /* progressive scans: serial refinement chains */
#define ROCJPEG_AMD_COST_INTERVAL 64u   /* per byte of the mean restart interval: K1's chain length */
#define ROCJPEG_AMD_COST_INTERVAL_CAP 12288u /* longer intervals are cut into chunk lanes (rj_entropy.hip) */

/* Fill items[0..count) from the JPEGs at blob + offsets[i] (sizes[i] bytes each, inside the
 * blob_bytes of the blob: INVALID_PARAMETER otherwise, before anything is read).  Returns
 * SUCCESS even when some images fail to parse (they are flagged ROCJPEG_AMD_WORK_BAD);
 * RUNTIME_ERROR when a header walk failed outside the JPEG rules (e.g. out of memory). */
RocJpegStatus rocJpegAmdBuildWorkTable(const unsigned char *blob, uint64_t blob_bytes, const uint64_t *offsets,
                                       const uint32_t *sizes, int count, RocJpegAmdWorkItem *items);

/* Greedy LPT (longest processing time first) over `num_shards` shards: items by decreasing
 * cost, each to the shard with the least assigned cost (ties: lower shard).  Sets `shard` and
 * `dest_device` (shard_devices[shard], or the shard index when shard_devices is NULL).
 * shard_cost (optional, num_shards entries) receives each shard's summed cost. */
RocJpegStatus rocJpegAmdAssignShards(RocJpegAmdWorkItem *items, int count, int num_shards, const int *shard_devices,
                                     uint64_t *shard_cost);

/* ---- Multi-GPU batched decode through the C ABI (csrc/rj_comm.cpp) ----
 * For a caller of the reference API with one process (or thread) per GPU, the sharded
 * counterpart of rocJpegDecodeBatched (src/rocjpeg_decoder.cpp:196-292): the reference itself
 * has no multi-GPU path (one device per handle, src/rocjpeg_api.cpp:107-120; the samples scale by
 * one handle per thread, samples/jpegDecodePerf/jpegdecodeperf.cpp:228-257).  The communicator
 * is RCCL's (loaded at run time from librccl.so.1); the work table is its only collective.
 *   1. one rank: rocJpegAmdCommGetUniqueId; the caller sends the 128-byte id to the others
 *   2. every rank: rocJpegAmdCommInitRank(its device, nranks, id, rank) -- collective
 *   3. every rank: rocJpegAmdDecodeBatchedSharded with the same blob / offsets / sizes / count:
 *      rank 0 builds the work table and assigns images by LPT (shard = rank), one RCCL broadcast
 *      sends it, each rank parses and decodes its own images into destinations[i] (only its
 *      entries are written; any destination memory: device, another GPU, host).
 * rocJpegAmdShardPlan / rocJpegAmdBroadcastWorkTable expose steps of 3 for callers that parse
 * and decode on their own (e.g. streams kept resident with rocJpegAmdStreamsToDevice). */
typedef struct { char internal[128]; } RocJpegAmdCommId; /* = ncclUniqueId */
typedef struct RocJpegAmdCommImpl *RocJpegAmdComm;
RocJpegStatus rocJpegAmdCommGetUniqueId(RocJpegAmdCommId *id);
RocJpegStatus rocJpegAmdCommInitRank(int device_id, int nranks, const RocJpegAmdCommId *id, int rank,
                                     RocJpegAmdComm *comm);
RocJpegStatus rocJpegAmdCommDestroy(RocJpegAmdComm comm);
RocJpegStatus rocJpegAmdCommInfo(RocJpegAmdComm comm, int *rank, int *nranks, int *device_id);
/* rank 0's `count` records -> every rank (each passes the same count) */
RocJpegStatus rocJpegAmdBroadcastWorkTable(RocJpegAmdComm comm, RocJpegAmdWorkItem *items, int count);
/* rank 0: rocJpegAmdBuildWorkTable + rocJpegAmdAssignShards over the ranks; then the broadcast */
RocJpegStatus rocJpegAmdShardPlan(RocJpegAmdComm comm, const unsigned char *blob, uint64_t blob_bytes,
                                  const uint64_t *offsets, const uint32_t *sizes, int count, RocJpegAmdWorkItem *items);
RocJpegStatus rocJpegAmdDecodeBatchedSharded(RocJpegHandle handle, RocJpegAmdComm comm, const unsigned char *blob,
                                             uint64_t blob_bytes, const uint64_t *offsets, const uint32_t *sizes,
                                             int count, const RocJpegDecodeParams *decode_params,
                                             RocJpegImage *destinations, RocJpegAmdWorkItem *items);

/* The resident form of the sharded call, for a caller that decodes the same batch repeatedly
 * (rocJpegAmdDecodeBatchedSharded = Create + Decode + Destroy):
 *   rocJpegAmdShardCreate   every rank, collective: the plan on rank 0, the broadcast, then this
 *                           rank parses its images with the GPU marker scan
 *                           (rocJpegAmdStreamParseDevice) and keeps their bitstreams and interval
 *                           tables resident in the HBM of `handle`'s device;
 *   rocJpegAmdShardDecode   no collective: rocJpegDecodeBatched over this rank's resident images,
 *                           image i of the batch into destinations[i] (`count` entries in batch
 *                           order, as at create; only this rank's are written);
 *   rocJpegAmdShardGetImages  this rank's batch indices;
 *   rocJpegAmdShardDestroy.
 * Collective error rules (create, plan, broadcast): every rank takes part in the broadcast on
 * every path once its communicator exists; when rank 0's plan fails every rank returns that
 * status; a rank whose own arguments are invalid returns INVALID_PARAMETER after the broadcast
 * (the other ranks still decode their shares).  A shard is used by one thread at a time. */
typedef struct RocJpegAmdShardImpl *RocJpegAmdShard;
RocJpegStatus rocJpegAmdShardCreate(RocJpegHandle handle, RocJpegAmdComm comm, const unsigned char *blob,
                                    uint64_t blob_bytes, const uint64_t *offsets, const uint32_t *sizes, int count,
                                    RocJpegAmdWorkItem *items, RocJpegAmdShard *shard);
RocJpegStatus rocJpegAmdShardDecode(RocJpegAmdShard shard, const RocJpegDecodeParams *decode_params,
                                    RocJpegImage *destinations);
RocJpegStatus rocJpegAmdShardGetImages(RocJpegAmdShard shard, int *num_images, int *indices, int capacity);
RocJpegStatus rocJpegAmdShardDestroy(RocJpegAmdShard shard);

/* Stage times of the handle's last rocJpegAmdStreamParseDevice call, in ms: [0] header walks
 * (host threads), [1] the resident allocation, [2] staging copy overlapped with the upload,
 * [3] job upload + marker-scan kernel + table read-back, [4] adopting the tables (host threads),
 * [5] the whole call.  `count` entries are written (at most 6). */
RocJpegStatus rocJpegAmdGetLastParseTimings(RocJpegHandle handle, double *ms, int count);

/* Concurrent small calls on one device are decoded together (rj_coalesce.h): counters since the
 * library was loaded -- calls that took part, combined calls (more than one caller's images in
 * one decode) and the callers' calls those covered. */
RocJpegStatus rocJpegAmdGetCoalesceStats(uint64_t *calls, uint64_t *combined, uint64_t *combined_members);

/* ABI revision of this header's extensions (rocJpegAmdGetAbiVersion returns the library's).
 * 2: rocJpegAmdBuildWorkTable takes blob_bytes; RocJpegAmdTimings as above.
 * 3: the resident sharded entry points; the work-table broadcast carries a status header.
 * 4: RocJpegAmdTimings.chunk_k1.  5: RocJpegAmdTimings.chunk_bytes (the call's chunk length).
 * 6: rocJpegAmdGetCoalesceStats, rocJpegAmdGetLastParseTimings, RocJpegAmdTimings.chunk_hyp. */
#define ROCJPEG_AMD_ABI_VERSION 8
RocJpegStatus rocJpegAmdGetAbiVersion(int *version);

#if defined(__cplusplus)
}
#endif

#endif /* ROC_JPEG_AMD_H */
