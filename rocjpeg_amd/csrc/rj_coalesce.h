// rj_coalesce.h -- concurrent small decode calls on one device, decoded together.
//
// The reference's benchmark shape (samples/jpegDecodePerf/jpegdecodeperf.cpp:201-202,228-257)
// is one host thread per handle, each calling rocJpegDecodeBatched with a batch of 1.  On VCN
// those calls go to separate fixed-function cores.  Here each call is a whole K0 -> K1 -> K2
// sequence sized to fill the GPU, so concurrent calls from eight handles contend for the same
// CUs and the process's four hardware queues, and each gains little from the others.
//
// Calls of at most kSmallCall images that arrive while another call on the same device is being
// decoded wait in a per-device queue; the thread that finds the device idle (the leader) takes
// every queued call with the same decode parameters (up to kMaxImages images) and decodes them
// in ONE call on its own handle.  Each caller still returns only after its own images are
// written, with its own status, so the API stays synchronous (rocjpeg_decoder.cpp:183,290).
// The leader first waits briefly (at most RJ_COALESCE_WAIT_US = 300 us, and a quarter of the last
// group's decode time) while fewer calls are queued than threads called on the device in the last
// 10 ms: callers returning from one group call again together, and without the wait they split
// into two half groups that alternate on the device.  A lone caller (one recent thread) never
// waits.  If a combined call fails, its member calls are decoded one by one, so every caller gets
// the status of its own images.  RJ_COALESCE=0 turns it off (each call on its own handle);
// RJ_COALESCE_INFLIGHT=k lets k combined calls decode at once, each gathering 1/k of the recent
// callers (default 1).  Calls on a handle with profiling on or a forced output path are never
// combined (Decoder::Coalescable: their timings and path belong to that handle).
#pragma once
#include <stdint.h>

#include "../../include/rocjpeg.h"

namespace rj {

class Decoder;
class Stream;

// rocJpegDecode / rocJpegDecodeBatched of `n` streams on `dec` (its device), coalesced with
// concurrent small calls on the same device.
int CoalescedDecode(Decoder *dec, int device, Stream *const *streams, int n, const RocJpegDecodeParams *params,
                    RocJpegImage *dst);
// counters (rocJpegAmdGetCoalesceStats)
void CoalesceStats(uint64_t *calls, uint64_t *combined, uint64_t *members);

}  // namespace rj
