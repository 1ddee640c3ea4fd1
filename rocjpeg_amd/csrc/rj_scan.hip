// rj_scan.hip -- GPU marker scan: the O(bytes) part of rocJpegStreamParse on the device.
//
// SURVEY.md 8f rank 4.  The reference parser walks the whole entropy-coded segment on the host
// for its end (ParseEOI: the first FF D9, src/rocjpeg_parser.cpp:400-416), and this decoder's
// host parser folds the restart-interval and destuffing tables into that walk (rj_stream.cpp
// BuildIntervals).  k_scan does both for a batch of streams on the GPU, one wave per stream,
// with exactly the host's semantics (every FF is classified by the byte after it):
//   FF FF          the first FF is fill: dropped
//   FF 00          data FF; the 00 is dropped
//   FF D0..D7      restart marker (with DRI): ends interval q, interval q+1 starts after it
//   FF other       any other marker: the interval's data ends there ("cut"); the interval itself
//                  still ends at the next RST (libjpeg reads zero bits past a marker)
// An interval's data also loses the fill FFs in front of its end.  Intervals past the expected
// count are ignored; missing ones are marked RJ_SEG_MISSING.  Outputs: the RjSegDev / RjDsBlock
// tables (into the stream's resident buffers and a compact copy for the host plan) and a copy
// of the bytes into the stream's resident ECS buffer.
//
// Pass A (all lanes, 1 KB per step: 16 B per lane, the next step's chunk in flight): the copy
// into the resident ECS buffer, the FF D9 end, and the RST / other-marker / drop positions,
// compacted by wave prefix sums into per-stream lists (a step with no FF byte only copies).  Pass B (lane per interval): interval
// bounds, drops by binary search, K0 blocks, prefix sums for the destuffed / entry / chunk
// offsets.
#include <hip/hip_runtime.h>

#include "rj_device.h"
#include "rj_kernels.h"
#include "rj_math.h"

namespace rj {

__device__ __forceinline__ uint32_t lower_bound_u32(const uint32_t *a, uint32_t n, uint32_t key) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (*gp(a + mid) < key) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ uint32_t wave_prefix(uint32_t v, uint32_t lane, uint32_t &total) {
  uint32_t x = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(x, off, 64);
    if (lane >= uint32_t(off)) x += y;
  }
  total = __shfl(x, 63, 64);
  return x - v;
}

__global__ __launch_bounds__(64) void k_scan(const RjScanJob *__restrict__ jobs, const uint8_t *__restrict__ arena) {
  const RjScanJob J = jobs[blockIdx.x];
  const uint32_t lane = threadIdx.x;
  const uint8_t *src = arena + J.src_off;
  const uint32_t n = J.avail;
  RjScanOut *out = J.out;
  // ---- pass A, one sweep of 1 KB per step (a 16-B chunk per lane, the next step's chunk loaded
  // one step ahead): the bytes copied into the resident ECS buffer (+16 B of zero slack), the end
  // (the first FF D9: the reference's ParseEOI), and every FF in [0, end) whose next byte lies in
  // [0, end), classified and compacted by ballot + prefix sums into per-stream lists in byte
  // order.  The arena holds 16 zero bytes after each stream, so chunk n4 (the slack) is readable. ----
  auto byte = [&](uint32_t p) -> uint32_t { return *gp(src + p); };
  const uint32_t n4 = (n + 15) / 16;
  const uint4 *s4 = reinterpret_cast<const uint4 *>(src);  // 16-B aligned in the arena
  uint4 *d4 = reinterpret_cast<uint4 *>(J.ecs);
  const uint32_t ri = J.ri;
  uint32_t end = n;
  uint32_t nrst = 0, noth = 0, ndrop = 0;
  bool overflow = false;
  const uint4 z4 = make_uint4(0, 0, 0, 0);
  uint4 cur = z4;
  if (lane <= n4) cur = *gp(s4 + lane);
  uint32_t step = 0;
  for (;; step++) {
    const uint32_t q = step * 64u + lane;  // this lane's chunk
    if (step * 64u > n4) break;
    uint4 nxt = z4;
    if (q + 64u <= n4) nxt = *gp(s4 + q + 64u);
    if (q <= n4) *gp(d4 + q) = q < n4 ? cur : z4;
    // the byte after this lane's 16: the next lane's first (lane 63: the next step's lane 0)
    const uint32_t nb_lane = __shfl_down(cur.x & 0xFFu, 1, 64);
    const uint32_t nb_next = __shfl(nxt.x & 0xFFu, 0, 64);
    const uint32_t nb = lane == 63 ? nb_next : nb_lane;
    // and the one after that, for lane 63's last byte: an FF there followed by the next step's
    // FF D9 is a fill byte in front of the end, not a drop (the end is found only next step)
    const uint32_t nb2_next = __shfl((nxt.x >> 8) & 0xFFu, 0, 64);
    // bytes equal to 0xFF: zero bytes of ~w (exact per byte)
    auto ffb = [](uint32_t w) {
      const uint32_t t = ~w;
      return ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t | 0x7F7F7F7Fu);  // 0x80 in each 0xFF byte of w
    };
    const bool any_ff = (ffb(cur.x) | ffb(cur.y) | ffb(cur.z) | ffb(cur.w)) != 0;
    if (__builtin_amdgcn_ballot_w64(any_ff) == 0) {
      cur = nxt;
      continue;
    }
    const uint32_t w[5] = {cur.x, cur.y, cur.z, cur.w, nb};
    const uint32_t p0 = q * 16u;
    // FF at p counts when p + 1 < n (and < end, applied below once the end is known)
    // drops: an FF FF's first FF (bit j), an FF 00's 00 (bit j + 1; 16: the next lane's byte 0)
    uint32_t rst_m = 0, oth_m = 0, dff_m = 0, d00_m = 0, d9 = 0xFFFFFFFFu;
#pragma unroll
    for (uint32_t j = 0; j < 16; j++) {
      const uint32_t b = (w[j >> 2] >> (8 * (j & 3))) & 0xFFu;
      const uint32_t nx = (w[(j + 1) >> 2] >> (8 * ((j + 1) & 3))) & 0xFFu;
      const bool ff = b == 0xFFu && p0 + j + 1 < n;
      dff_m |= (ff && nx == 0xFFu) ? 1u << j : 0u;
      d00_m |= (ff && nx == 0x00u) ? 1u << (j + 1) : 0u;
      const bool rst = ff && ri != 0 && nx >= 0xD0u && nx <= 0xD7u;
      rst_m |= rst ? 1u << j : 0u;
      oth_m |= (ff && nx != 0xFFu && nx != 0x00u && !rst) ? 1u << j : 0u;
      d9 = (ff && nx == 0xD9u && d9 == 0xFFFFFFFFu) ? p0 + j : d9;
    }
    if (lane == 63 && nb == 0xFFu && nb2_next == 0xD9u) dff_m &= 0x7FFFu;  // FF | FF D9 across steps
    bool last = false;
    if (__builtin_amdgcn_ballot_w64(d9 != 0xFFFFFFFFu) != 0) {
      uint32_t m = d9;
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) m = min(m, __shfl_xor(m, off, 64));
      end = m;
      last = true;
      // only FFs at p with p + 1 < end; the 00 drop of an FF at p sits at p + 1
      const uint32_t lim = end > p0 ? end - p0 : 0u;  // positions j < lim - 1 count
      const uint32_t keep = lim >= 17u ? 0xFFFFFFFFu : (lim >= 1u ? (1u << (lim - 1u)) - 1u : 0u);
      rst_m &= keep;
      oth_m &= keep;
      dff_m &= keep;
      d00_m &= keep << 1;
    }
    const uint32_t drop_m = dff_m | d00_m;  // disjoint: a byte is not both FF and 00
    // compaction in byte order: lane-major, ascending positions within a lane
    uint32_t t;
    const uint32_t nr = __popc(rst_m), no = __popc(oth_m), nd = __popc(drop_m);
    const uint32_t pr = wave_prefix(nr, lane, t);
    const uint32_t tr = t;
    const uint32_t po = wave_prefix(no, lane, t);
    const uint32_t to = t;
    const uint32_t pd = wave_prefix(nd, lane, t);
    const uint32_t td = t;
    uint32_t k = 0;
    for (uint32_t m = rst_m; m; m &= m - 1, k++) {
      const uint32_t idx = nrst + pr + k;
      if (idx < J.rst_cap) *gp(J.rst + idx) = p0 + __builtin_ctz(m);
    }
    k = 0;
    for (uint32_t m = oth_m; m; m &= m - 1, k++) {
      const uint32_t idx = noth + po + k;
      if (idx < J.oth_cap) *gp(J.oth + idx) = p0 + __builtin_ctz(m);
    }
    k = 0;
    for (uint32_t m = drop_m; m; m &= m - 1, k++) {
      const uint32_t idx = ndrop + pd + k;
      if (idx < J.drop_cap) *gp(J.drop + idx) = p0 + __builtin_ctz(m);
    }
    nrst += tr;
    noth += to;
    ndrop += td;
    if (last) break;
    cur = nxt;
  }
  // the rest of the copy, past the step that found the end
  for (uint32_t q = (step + 1) * 64u + lane; q <= n4; q += 64u) {
    uint4 v = z4;
    if (q < n4) v = *gp(s4 + q);
    *gp(d4 + q) = v;
  }
  if (noth > J.oth_cap || ndrop > J.drop_cap) overflow = true;
  // the drop list must be sorted: a 00 drop (p + 1) of lane l's last byte may exceed lane l+1's
  // first FF drop only if byte p + 1 is both 00 and FF -- impossible; lists are ascending.
  const uint32_t expected = J.expected;
  const uint32_t nrst_used = min(nrst, min(expected, J.rst_cap));
  if (nrst > J.rst_cap && nrst < expected) overflow = true;
  __syncthreads();  // list stores visible to the wave (same wave: program order, but be explicit)
  if (overflow) {
    if (lane == 0) *gp(&out->flags) = 1u;
    return;
  }
  // ---- pass B: one lane per interval ----
  const uint32_t total = J.total_mcus, nblk = J.nblk_mcu;
  uint32_t dst_carry = 0, ent_carry = 0, ch_carry = 0, ds_carry = 0;
  uint64_t ent64_carry = 0;
  for (uint32_t q0 = 0; q0 < expected; q0 += 64) {
    const uint32_t q = q0 + lane;
    const bool valid = q < expected;
    uint32_t start = 0, stop = 0, src_len = 0, dst_len = 0, flags = 0;
    if (valid) {
      if (q <= nrst_used && !(q == nrst_used && nrst_used == expected)) {
        start = q == 0 ? 0u : *gp(J.rst + q - 1) + 2u;
        const uint32_t rawstop = q < nrst_used ? *gp(J.rst + q) : end;
        uint32_t st = rawstop;
        const uint32_t co = lower_bound_u32(J.oth, noth, start);
        if (co < noth) st = min(st, *gp(J.oth + co));
        while (st > start && byte(st - 1) == 0xFFu) st--;  // trailing fill
        stop = st;
        src_len = stop - start;
        dst_len = src_len - (lower_bound_u32(J.drop, ndrop, stop) - lower_bound_u32(J.drop, ndrop, start));
      } else {
        flags = RJ_SEG_MISSING;
        start = end;
      }
    }
    const uint32_t mcu_first = q * (ri ? ri : total);
    const uint32_t mcu_count = !valid ? 0u : (ri ? min(ri, total - mcu_first) : total);
    const uint32_t dsz = !valid ? 0u : (flags ? 16u : ((src_len + 16 + 15) & ~15u));
    const uint32_t nds = (!valid || flags) ? 0u : (src_len + RJ_DS_BLOCK - 1) / RJ_DS_BLOCK;
    const uint32_t nch = valid ? rj_chunks(src_len) : 0u;
    const uint64_t ent = valid ? rj_interval_entries(src_len, uint64_t(mcu_count) * nblk, nblk) : 0ull;
    uint32_t t;
    const uint32_t dst_off = dst_carry + wave_prefix(dsz, lane, t);
    dst_carry += t;
    const uint32_t ch0 = ch_carry + wave_prefix(nch, lane, t);
    ch_carry += t;
    const uint32_t ds0 = ds_carry + wave_prefix(nds, lane, t);
    ds_carry += t;
    // 64-bit entry offsets (the table keeps 32 bits, as the host plan does)
    uint64_t ex = ent;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint64_t y = __shfl_up(ex, off, 64);
      if (lane >= uint32_t(off)) ex += y;
    }
    const uint64_t ent_off = ent64_carry + ex - ent;
    ent64_carry += __shfl(ex, 63, 64);
    (void)ent_carry;
    if (valid) {
      RjSegDev sg;
      sg.src_off = start;
      sg.src_len = src_len;
      sg.dst_off = dst_off;
      sg.mcu_first = mcu_first;
      sg.mcu_count = mcu_count;
      sg.flags = flags;
      sg.ent_off = uint32_t(ent_off);
      sg.chunk0 = ch0;
      sg.dst_len = dst_len;
      sg.pad[0] = sg.pad[1] = sg.pad[2] = 0;
      *gp(J.segs + q) = sg;
      *gp(J.segs_copy + q) = sg;
      for (uint32_t b = 0; b < nds; b++) {
        const uint32_t o = b * RJ_DS_BLOCK;
        RjDsBlock blk;
        blk.src_off = start + o;
        blk.len = min(RJ_DS_BLOCK, src_len - o) | (o == 0 ? 0x80000000u : 0u);
        blk.dst_off = dst_off + o - (lower_bound_u32(J.drop, ndrop, start + o) - lower_bound_u32(J.drop, ndrop, start));
        blk.zero_end = b + 1 == nds ? dst_off + ((src_len + 16 + 15) & ~15u) : 0u;
        if (ds0 + b < J.ds_cap) {
          *gp(J.ds + ds0 + b) = blk;
          *gp(J.ds_copy + ds0 + b) = blk;
        }
      }
    }
  }
  if (lane == 0) {
    RjScanOut o;
    o.ecs_end = end;
    o.nds = ds_carry;
    o.flags = ds_carry > J.ds_cap ? 1u : 0u;
    o.destuff_bytes = dst_carry;
    o.entries = ent64_carry;
    o.nchunks = ch_carry;
    o.pad = 0;
    *gp(out) = o;
  }
}

hipError_t LaunchScan(hipStream_t st, const RjScanJob *jobs, uint32_t njobs, const uint8_t *arena) {
  if (njobs == 0) return hipSuccess;
  hipLaunchKernelGGL(k_scan, dim3(njobs), dim3(64), 0, st, jobs, arena);
  return hipGetLastError();
}

}  // namespace rj
