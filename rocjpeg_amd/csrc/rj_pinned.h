// rj_pinned.h -- process-wide arena of pinned (page-locked) host memory for parsed bitstreams.
//
// rocJpegStreamParse already reads every entropy-coded byte on the host (the FF D9 / RST scan
// the reference does in ParseEOI, src/rocjpeg_parser.cpp:400-416); it copies the bytes into a
// slot of this arena while it is there.  Streams parsed one after another get adjacent slots,
// so a later rocJpegDecodeBatched over them uploads a run of streams with ONE DMA straight from
// the slots: the call itself does no host copy of bitstream bytes (rj_decoder.cpp).
//
// Slots are carved from 64-MB chunks by a bump pointer; a slot holds a reference to its chunk,
// and a chunk whose slots are all released goes back to a small free list (pinned allocations
// are slow, so chunks are reused rather than freed).  Without a usable HIP device the arena
// hands out no slots and streams keep borrowing the caller's bytes, as before.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <memory>

namespace rj {

struct PinnedChunk;

struct PinnedSlot {
  uint8_t *ptr = nullptr;                // nullptr: no slot (the stream borrows the caller's bytes)
  size_t bytes = 0;
  std::shared_ptr<PinnedChunk> chunk;    // keeps the chunk alive while the slot is used
  const PinnedChunk *id() const { return chunk.get(); }
};

// A slot of at least `bytes` bytes, 256-B aligned; empty when pinned memory is unavailable
// (no device, allocation failure, or ROCJPEG_AMD_PARSE_PIN=0).
PinnedSlot PinnedAlloc(size_t bytes);

// memcpy into pinned staging memory that only a DMA or the GPU reads next: non-temporal stores
// for the bulk, so the destination lines are neither read for ownership nor kept in the host's
// caches (a plain copy of a few hundred KB uses cached stores: the host's memory then carries the
// source read, the destination's ownership read, the write and the DMA's read).  Ends with a store
// fence, so the bytes are visible before whatever the caller publishes next.
void CopyToStaging(void *dst, const void *src, size_t n);

}  // namespace rj
