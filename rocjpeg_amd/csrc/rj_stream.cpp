// rj_stream.cpp -- host parser (see rj_stream.h).
#include "rj_stream.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "rj_common.h"

namespace rj {

namespace {

inline uint32_t Be16(const uint8_t *p) { return (uint32_t(p[0]) << 8) | p[1]; }

// rocjpeg_parser.cpp:432-470.  comp[1]/comp[2] are zero for grayscale.
int ClassifyCss(const StreamInfo &s) {
  const int h1 = s.comp[0].h, h2 = s.comp[1].h, h3 = s.comp[2].h;
  const int v1 = s.comp[0].v, v2 = s.comp[1].v, v3 = s.comp[2].v;
  auto is = [&](int a, int b, int c, int d, int e, int f) {
    return h1 == a && h2 == b && h3 == c && v1 == d && v2 == e && v3 == f;
  };
  if (is(1, 1, 1, 1, 1, 1) || is(2, 2, 2, 2, 2, 2) || is(4, 4, 4, 4, 4, 4)) return kCss444;
  if (is(1, 1, 1, 2, 1, 1)) return kCss440;
  if (is(2, 1, 1, 1, 1, 1) || is(2, 1, 1, 2, 2, 2) || is(2, 2, 2, 2, 1, 1)) return kCss422;
  if (is(2, 1, 1, 2, 1, 1)) return kCss420;
  if (is(4, 1, 1, 1, 1, 1)) return kCss411;
  if (is(1, 0, 0, 1, 0, 0) || is(4, 0, 0, 4, 0, 0)) return kCss400;
  return kCssUnknown;
}


uint64_t Fnv1a(uint64_t h, const void *p, size_t n) {
  const uint8_t *b = static_cast<const uint8_t *>(p);
  for (size_t i = 0; i < n; i++) h = (h ^ b[i]) * 1099511628211ull;
  return h;
}

}  // namespace

// Lean K1 entry of a resolved code (rj_device.h RjLeanTables), the first-symbol half.  libjpeg
// semantics: DC symbol = difference category s; AC symbol (r, s): s != 0 a coefficient after r
// zeros, (15, 0) ZRL, any other (r, 0) ends the block (decode_mcu: `if (r != 15) break`).
static uint32_t LeanEntry(uint32_t len, uint32_t sym, bool is_dc) {
  const uint32_t s = sym & 15u, r = sym >> 4;
  const uint32_t R = is_dc ? 0u : (s ? r : (r == 15 ? 15u : 63u));
  const uint32_t n = len + s;
  return (n << 16) | (s << 21) | (R << 25);
}

static void FillLeanBad(bool is_dc, uint32_t *first, uint32_t *subs) {
  const int B = is_dc ? RJ_HL_DC_BITS : RJ_HL_AC_BITS;
  const uint32_t bad = LeanEntry(17, 0, is_dc);  // libjpeg: a bad code is 17 bits of symbol 0
  for (int e = 0; e < (1 << B); e++) first[e] = bad;
  if (subs)
    for (int e = 0; e < RJ_HL_SUBS * 32; e++) subs[e] = bad;
}

// The second-symbol halves of a first level (rj_device.h): for each key of `first` (B bits)
// whose symbol leaves its block open -- a DC difference, an AC coefficient or ZRL -- with
// n1 < B, the AC code that starts at bit n1, if it is complete inside the key (its extra bits
// may run past it: the step reads them from its 32-bit peek, n1 + n2 <= 11 + 10 bits).
// `ac` (RJ_HL_AC_BITS keys, single-symbol entries): the AC table the second symbol is read with.
// The AC table each DC table's two-symbol entries are read with: the AC table of every scan
// component that uses that DC table, or -1 when none uses it or two components disagree.
static void DcPairMap(const StreamInfo &s, int (&ac_of_dc)[2]) {
  ac_of_dc[0] = ac_of_dc[1] = -1;
  bool mixed[2] = {false, false};
  for (int c = 0; c < s.scan_ncomp && c < 4; c++) {
    const int td = s.scomp[c].td & 1, ta = s.scomp[c].ta & 1;
    if (ac_of_dc[td] < 0) ac_of_dc[td] = ta;
    else if (ac_of_dc[td] != ta) mixed[td] = true;
  }
  for (int t = 0; t < 2; t++)
    if (mixed[t]) ac_of_dc[t] = -1;
}

static void AddLeanPairs(uint32_t *first, uint32_t B, bool is_dc, const uint32_t *ac) {
  const uint32_t BA = RJ_HL_AC_BITS;
  for (uint32_t key = 0; key < (1u << B); key++) {
    const uint32_t e = first[key];
    if (e & RJ_HL_ESC) continue;
    const uint32_t n1 = (e >> 16) & 31u, s1 = (e >> 21) & 15u, R1 = (e >> 25) & 63u;
    if (n1 >= B || n1 == 17u) continue;                                   // no room / bad code
    if (!is_dc && (R1 == 63u || (s1 == 0 && R1 != 15u))) continue;       // EOB: the block ends
    const uint32_t avail = B - n1;                                        // key bits after symbol 1
    const uint32_t rest = ((key << n1) & ((1u << B) - 1u)) << (BA - B);  // left-aligned AC key
    const uint32_t e2 = ac[rest];
    if (e2 & RJ_HL_ESC) continue;
    const uint32_t n2 = (e2 >> 16) & 31u, s2 = (e2 >> 21) & 15u, R2 = (e2 >> 25) & 63u;
    if (n2 == 17u || n2 - s2 > avail) continue;  // bad, or the code is not inside the key
    first[key] = e | n2 | (s2 << 5) | (R2 << 9) | RJ_HL_PAIR;
  }
}

bool BuildLeanTable(const uint8_t bits[16], const uint8_t *vals, bool is_dc, uint32_t *first, uint32_t *subs) {
  const int B = is_dc ? RJ_HL_DC_BITS : RJ_HL_AC_BITS;
  FillLeanBad(is_dc, first, subs);
  int nsub = 0;
  std::vector<int> sub_of(size_t(1) << B, -1);
  int k = 0, code = 0;
  for (int l = 1; l <= 16; l++) {
    for (int i = 0; i < bits[l - 1]; i++, k++, code++) {
      if (code >= (1 << l) || k >= (is_dc ? 12 : 162)) {  // over-subscribed: no write past the tables
        FillLeanBad(is_dc, first, subs);
        return false;
      }
      const uint32_t ent = LeanEntry(uint32_t(l), vals[k], is_dc);
      if (l <= B) {
        for (int f = 0; f < (1 << (B - l)); f++) first[(code << (B - l)) | f] = ent;
        continue;
      }
      const int prefix = code >> (l - B);
      if (sub_of[prefix] < 0) {
        sub_of[prefix] = (!is_dc && subs && nsub < RJ_HL_SUBS) ? nsub++ : RJ_HL_SUBS;
        first[prefix] = RJ_HL_ESC | (sub_of[prefix] < RJ_HL_SUBS ? uint32_t(sub_of[prefix]) : 0xFFu);
      }
      if (sub_of[prefix] < RJ_HL_SUBS) {  // the next 16 - B = 5 bits
        const int rest = code & ((1 << (l - B)) - 1);
        for (int f = 0; f < (1 << (16 - l)); f++) subs[sub_of[prefix] * 32 + ((rest << (16 - l)) | f)] = ent;
      }
    }
    code <<= 1;
  }
  return true;
}

bool BuildHuffman(const uint8_t bits[16], const uint8_t *vals, bool is_dc, RjHuffDev *t) {
  std::memset(t, 0, sizeof(*t));
  for (int e = 0; e < RJ_LUT_ENTRIES; e++) t->lut[e] = uint16_t(RJ_LUT_BAD);
  int nsub = 0;
  int sub_of_prefix[RJ_LUT_L1];
  for (int e = 0; e < RJ_LUT_L1; e++) sub_of_prefix[e] = -1;
  int k = 0, code = 0;
  for (int l = 1; l <= 16; l++) {
    const int nb = bits[l - 1];
    if (nb) {
      t->valoff[l] = k - code;
      for (int i = 0; i < nb; i++, k++, code++) {
        if (code >= (1 << l) || k >= 256) return false;  // over-subscribed: checked before any write
        const uint16_t ent = uint16_t((l << 8) | vals[k]);
        if (l <= 9) {
          const int shift = 9 - l;
          for (int f = 0; f < (1 << shift); f++) t->lut[(code << shift) | f] = ent;
        } else {
          const int prefix = code >> (l - 9);
          if (sub_of_prefix[prefix] < 0) {
            if (nsub < RJ_L2_SUBTABLES) {
              sub_of_prefix[prefix] = nsub;
              t->lut[prefix] = uint16_t(0x8000 | nsub);
              nsub++;
            } else {
              t->lut[prefix] = 0xFFFF;  // canonical search for this prefix
              sub_of_prefix[prefix] = RJ_L2_SUBTABLES;
            }
          }
          const int sub = sub_of_prefix[prefix];
          if (sub < RJ_L2_SUBTABLES) {
            const int rest = code & ((1 << (l - 9)) - 1);
            const int shift = 16 - l;
            for (int f = 0; f < (1 << shift); f++)
              t->lut[RJ_LUT_L1 + sub * 128 + ((rest << shift) | f)] = ent;
          }
        }
      }
      t->maxcode16[l] = uint32_t(code) << (16 - l);  // exclusive bound, left-justified
    } else {
      t->maxcode16[l] = 0;
    }
    if (code > (1 << l)) return false;  // over-subscribed (libjpeg JERR_BAD_HUFF_TABLE)
    code <<= 1;
  }
  if (k > 256) return false;
  std::memcpy(t->vals, vals, size_t(k));
  if (is_dc)
    for (int i = 0; i < k; i++)
      if (vals[i] > 15) return false;  // libjpeg rejects DC categories > 15
  return true;
}

bool Stream::Parse(const uint8_t *d, uint32_t n, bool defer_scan) {
  std::lock_guard<std::mutex> lock(mu_);  // rocjpeg_parser.cpp:44
  ReleaseResident();
  pin_ = PinnedSlot();
  generation_++;
  lean_.reset();
  info_ = StreamInfo();
  plan_ = DecodePlan();
  plan_.status = -3;
  scan_pending_ = false;
  StreamInfo &s = info_;
  if (d == nullptr || n < 4) return false;
  if (d[0] != 0xFF || d[1] != 0xD8) return false;  // :64-67
  if (IsProgressiveStream(d, n)) {  // SOF2: rj_prog_stream.cpp
    if (ParseProgressive(d, n)) {
      PinEcs();
      return true;
    }
    plan_ = DecodePlan();
    plan_.status = -3;
    return false;
  }
  size_t pos = 2;
  bool sos = false, dht = false, dqt = false;
  while (!sos && pos < n) {  // marker walk :74-109, bounds-checked
    while (pos < n && d[pos] == 0xFF) pos++;
    if (pos + 3 > n) return false;
    const uint32_t marker = d[pos++];
    const size_t seg = pos;
    const size_t len = Be16(d + seg);
    const size_t next = seg + len;
    if (len < 2 || next > n) return false;
    switch (marker) {
      case 0xC0: {  // SOF0 :160-207
        if (len < 8) return false;
        s.precision = d[seg + 2];
        s.height = uint16_t(Be16(d + seg + 3));
        s.width = uint16_t(Be16(d + seg + 5));
        s.ncomp = d[seg + 7];
        if (s.ncomp > 3) return false;
        if (len < 8 + 3u * s.ncomp) return false;
        for (int i = 0; i < s.ncomp; i++) {
          const uint8_t *c = d + seg + 8 + 3 * i;
          s.comp[i].id = c[0];
          if (c[2] >= 4) return false;
          s.comp[i].h = c[1] >> 4;
          s.comp[i].v = c[1] & 15;
          s.comp[i].tq = c[2];
        }
        const uint32_t hf = s.comp[0].h, vf = s.comp[0].v;
        if (hf && vf) s.num_mcus = ((s.width + hf * 8 - 1) / (hf * 8)) * ((s.height + vf * 8 - 1) / (vf * 8));
        s.css = ClassifyCss(s);
        s.sof_seen = true;
        break;
      }
      case 0xC4: {  // DHT :256-313
        long left = long(len) - 2;
        size_t p = seg + 2;
        while (left > 0) {
          if (p + 17 > next) return false;
          const uint32_t idx = d[p++];
          const uint32_t id = idx & 15;
          const bool ac = (idx & 0xF0) != 0;
          if (id >= 2) return false;
          uint32_t cnt = 0;
          for (int i = 0; i < 16; i++) cnt += d[p + i];
          std::memcpy(ac ? s.ht[id].ac_bits : s.ht[id].dc_bits, d + p, 16);
          p += 16;
          if (p + cnt > next) return false;
          if (cnt > (ac ? 162u : 12u)) return false;
          std::memcpy(ac ? s.ht[id].ac_vals : s.ht[id].dc_vals, d + p, cnt);
          s.ht_loaded[id] = 1;
          left -= 17 + long(cnt);
          p += cnt;
        }
        dht = true;
        break;
      }
      case 0xDB: {  // DQT :217-246 (8-bit tables only)
        size_t p = seg + 2;
        while (p < next) {
          const uint32_t idx = d[p++];
          if (idx >> 4) return false;
          if (idx >= 4) return false;
          if (p + 64 > n) return false;
          std::memcpy(s.qt_zz[idx], d + p, 64);
          s.qt_loaded[idx] = 1;
          p += 64;
        }
        dqt = true;
        break;
      }
      case 0xDD:  // DRI :374-390
        if (len != 4) return false;
        s.restart_interval = uint16_t(Be16(d + seg + 2));
        break;
      case 0xDA: {  // SOS :324-363
        const uint32_t ns = d[seg + 2];
        if (ns > 3) return false;
        if (len < 6 + 2 * ns) return false;
        s.scan_ncomp = uint8_t(ns);
        for (uint32_t i = 0; i < ns; i++) {
          const uint32_t cs = d[seg + 3 + 2 * i], t = d[seg + 4 + 2 * i];
          s.scomp[i].cs = uint8_t(cs);
          s.scomp[i].td = uint8_t(t >> 4);
          s.scomp[i].ta = uint8_t(t & 15);
          if ((t & 15) >= 4 || (t >> 4) >= 4) return false;
          if (cs != s.comp[i].id) return false;
        }
        sos = true;
        break;
      }
      default:
        break;
    }
    pos = next;
  }
  if (!dht || !dqt) return false;  // :111-118
  if (defer_scan && sos) {
    // GPU marker scan (Decoder::ParseOnDevice, rj_scan.hip): the device finds the FF D9 end and
    // builds the interval / K0 tables; here only what the header determines
    s.ecs = d + pos;
    s.ecs_size = n - uint32_t(pos);  // bytes available; CompleteFromDevice sets the true end
    scan_pending_ = BuildPlanHeader();
    return true;
  }
  // ParseEOI (:400-416): the entropy-coded segment runs to the first FF D9.
  size_t end = n;
  if (sos) {
    const uint8_t *p = d + pos;
    while (true) {
      p = static_cast<const uint8_t *>(std::memchr(p, 0xFF, size_t(d + n - p)));
      if (p == nullptr || p + 1 >= d + n) break;
      if (p[1] == 0xD9) { end = size_t(p - d); break; }
      p++;
    }
  }
  s.ecs = d + (sos ? pos : n);
  s.ecs_size = sos ? uint32_t(end - pos) : 0;
  BuildPlan();
  PinEcs();
  return true;
}

// While the parse is reading the bytes anyway: a copy in pinned memory, from which a later
// decode call uploads runs of consecutively parsed streams with one DMA each and no host copy
// (rj_decoder.cpp).  Streams the decoder would refuse are not copied.
void Stream::PinEcs() {
  if (plan_.status != 0 || info_.ecs_size == 0) return;
  pin_ = PinnedAlloc(size_t(info_.ecs_size) + 16);
  if (pin_.ptr == nullptr) return;
  CopyToStaging(pin_.ptr, info_.ecs, info_.ecs_size);
  std::memset(pin_.ptr + info_.ecs_size, 0, 16);  // K0 reads <= 8 B past the end
}

void Stream::BuildPlan() {
  if (BuildPlanHeader()) BuildIntervals();
}

bool Stream::BuildPlanHeader() {
  const StreamInfo &s = info_;
  DecodePlan &p = plan_;
  p.status = 0;
  // what the reference's SubmitDecode rejects (rocjpeg_vaapi_decoder.cpp:586-592, 612-636),
  // plus streams this baseline decoder cannot reconstruct.
  if (!s.sof_seen || s.ncomp == 0 || s.width < 64 || s.height < 64 || s.width > 16384 || s.height > 16384) {
    p.status = -4;  // JPEG_NOT_SUPPORTED
    return false;
  }
  if (!(s.css == kCss444 || s.css == kCss440 || s.css == kCss422 || s.css == kCss420 || s.css == kCss400)) {
    p.status = -4;
    return false;
  }
  if (s.precision != 8 || s.scan_ncomp != s.ncomp) {
    p.status = -4;
    return false;
  }
  const int nc = s.ncomp;
  p.hmax = p.vmax = 1;
  for (int c = 0; c < nc; c++) {
    if (s.comp[c].h < 1 || s.comp[c].h > 4 || s.comp[c].v < 1 || s.comp[c].v > 4) { p.status = -3; return false; }
    p.hmax = std::max(p.hmax, s.comp[c].h);
    p.vmax = std::max(p.vmax, s.comp[c].v);
  }
  p.interleaved = nc > 1;
  if (p.interleaved) {
    p.mcux = (s.width + 8u * p.hmax - 1) / (8u * p.hmax);
    p.mcuy = (s.height + 8u * p.vmax - 1) / (8u * p.vmax);
    int b = 0;
    for (int c = 0; c < nc; c++) {
      p.comp_blk0[c] = uint8_t(b);
      p.wblk[c] = p.mcux * s.comp[c].h;
      p.hblk[c] = p.mcuy * s.comp[c].v;
      for (int y = 0; y < s.comp[c].v; y++)
        for (int x = 0; x < s.comp[c].h; x++) {
          if (b >= RJ_MAX_BLK_MCU) { p.status = -3; return false; }
          p.blk_comp[b] = uint8_t(c);
          p.blk_dx[b] = uint8_t(x);
          p.blk_dy[b] = uint8_t(y);
          b++;
        }
    }
    p.nblk_mcu = uint8_t(b);
  } else {
    const uint32_t cw = (s.width * s.comp[0].h + p.hmax - 1) / p.hmax;
    const uint32_t ch = (s.height * s.comp[0].v + p.vmax - 1) / p.vmax;
    p.wblk[0] = (cw + 7) / 8;
    p.hblk[0] = (ch + 7) / 8;
    p.mcux = p.wblk[0];
    p.mcuy = p.hblk[0];
    p.nblk_mcu = 1;
  }
  // tables
  uint64_t h = 1469598103934665603ull;
  for (int c = 0; c < nc; c++) {
    const int td = s.scomp[c].td, ta = s.scomp[c].ta, tq = s.comp[c].tq;
    if (td >= 2 || ta >= 2 || !s.ht_loaded[td] || !s.ht_loaded[ta] || !s.qt_loaded[tq]) { p.status = -3; return false; }
  }
  for (int t = 0; t < 2; t++) {
    p.ht_valid[t] = 0;
    if (!s.ht_loaded[t]) continue;
    if (BuildHuffman(s.ht[t].dc_bits, s.ht[t].dc_vals, true, &p.tables.dc[t]) &&
        BuildHuffman(s.ht[t].ac_bits, s.ht[t].ac_vals, false, &p.tables.ac[t])) {
      p.ht_valid[t] = 1;
    } else {
      // only fatal when the scan actually uses this table
      for (int c = 0; c < nc; c++)
        if (s.scomp[c].td == t || s.scomp[c].ta == t) { p.status = -3; return false; }
    }
  }
  for (int q = 0; q < 4; q++) {
    p.qmax[q] = 1;
    for (int k = 0; k < 64; k++) {
      p.tables.qz[q][k] = s.qt_zz[q][k];
      p.qmax[q] = std::max<uint16_t>(p.qmax[q], s.qt_zz[q][k]);
    }
  }
  {
    static_assert(sizeof(s.ht) == 2 * (16 + 12 + 16 + 162), "raw DHT layout");
    uint8_t *kp = p.table_key;
    *kp++ = s.ht_loaded[0];
    *kp++ = s.ht_loaded[1];
    std::memcpy(kp, s.ht, sizeof(s.ht));
    kp += sizeof(s.ht);
    std::memcpy(kp, s.qt_zz, sizeof(s.qt_zz));
    kp += sizeof(s.qt_zz);
    int ac_of_dc[2];
    DcPairMap(s, ac_of_dc);
    *kp++ = uint8_t(ac_of_dc[0] < 0 ? 0xFF : ac_of_dc[0]);
    *kp++ = uint8_t(ac_of_dc[1] < 0 ? 0xFF : ac_of_dc[1]);
  }
  h = Fnv1a(h, p.table_key, sizeof(p.table_key));
  p.table_hash = h;
  return true;
}

// Restart-interval table (host marker scan; rj_scan.hip is the device version).
void Stream::BuildIntervals() {
  const StreamInfo &s = info_;
  DecodePlan &p = plan_;
  // Restart-interval table: split the ECS at RSTn markers (FF D0..D7).  Fill FFs in front
  // of a marker are excluded; FF 00 stays (the destuff kernel removes the 00).
  const uint32_t total_mcus = p.mcux * p.mcuy;
  const uint32_t ri = s.restart_interval;
  const uint32_t expected = ri ? (total_mcus + ri - 1) / ri : 1;
  p.segs.reserve(expected);
  const uint8_t *e = s.ecs;
  const uint32_t n = s.ecs_size;
  uint32_t start = 0, i = 0;
  uint64_t dst = 0, ent = 0;
  // bytes the destuffing drops (the 00 of FF 00, a fill FF followed by FF), in stream order
  std::vector<uint32_t> drops;
  size_t dq = 0;
  auto emit = [&](uint32_t b, uint32_t stop) {
    while (stop > b && e[stop - 1] == 0xFF) stop--;  // trailing fill
    if (p.segs.size() >= expected) return;
    RjSegDev sg;
    std::memset(&sg, 0, sizeof(sg));
    sg.src_off = b;
    sg.src_len = stop - b;
    sg.dst_off = uint32_t(dst);
    // K0 blocks: output offset of each = its raw offset minus the bytes dropped before it
    while (dq < drops.size() && drops[dq] < b) dq++;
    uint32_t dropped = 0;
    for (uint32_t o = 0; o < sg.src_len; o += RJ_DS_BLOCK) {
      const uint32_t blen = std::min(RJ_DS_BLOCK, sg.src_len - o);
      RjDsBlock blk;
      blk.src_off = b + o;
      blk.len = blen | (o == 0 ? 0x80000000u : 0u);  // high bit: first block of the interval
      blk.dst_off = sg.dst_off + o - dropped;
      blk.zero_end = 0;
      while (dq < drops.size() && drops[dq] < b + o + blen) { dq++; dropped++; }
      p.ds.push_back(blk);
    }
    sg.dst_len = sg.src_len - dropped;
    if (sg.src_len) p.ds.back().zero_end = uint32_t(dst + ((uint64_t(sg.src_len) + 16 + 15) & ~uint64_t(15)));
    sg.mcu_first = uint32_t(p.segs.size()) * (ri ? ri : total_mcus);
    sg.mcu_count = ri ? std::min(ri, total_mcus - sg.mcu_first) : total_mcus;
    sg.flags = 0;
    sg.ent_off = uint32_t(ent);
    sg.chunk0 = p.nchunks;
    p.nchunks += rj_chunks(sg.src_len);
    ent += rj_interval_entries(sg.src_len, uint64_t(sg.mcu_count) * p.nblk_mcu, p.nblk_mcu);
    dst += (uint64_t(sg.src_len) + 16 + 15) & ~uint64_t(15);  // >= 16 B of slack after each interval
    p.segs.push_back(sg);
  };
  // Any other marker inside an interval ends its data (a decoder reads zero bits past a
  // marker, libjpeg jdhuff.c fill_bit_buffer); the interval itself still ends at the next RST.
  uint32_t cut = UINT32_MAX;
  while (i + 1 < n) {
    const uint8_t *f = static_cast<const uint8_t *>(std::memchr(e + i, 0xFF, n - i));
    if (f == nullptr) break;
    i = uint32_t(f - e);
    if (i + 1 >= n) break;
    const uint8_t m = e[i + 1];
    if (m == 0x00) {
      drops.push_back(i + 1);
      i += 2;
    } else if (m == 0xFF) {
      drops.push_back(i);
      i += 1;
    } else if (ri && m >= 0xD0 && m <= 0xD7) {
      emit(start, std::min(i, cut));
      start = i + 2;
      cut = UINT32_MAX;
      i += 2;
    } else {
      if (cut == UINT32_MAX) cut = i;
      i += 2;
    }
  }
  emit(start, std::min(n, cut));
  while (p.segs.size() < expected) {  // intervals whose RST marker never came: zero blocks
    RjSegDev sg;
    std::memset(&sg, 0, sizeof(sg));
    sg.src_off = n;
    sg.src_len = 0;
    sg.dst_off = uint32_t(dst);
    sg.mcu_first = uint32_t(p.segs.size()) * ri;
    sg.mcu_count = std::min(ri, total_mcus - sg.mcu_first);
    sg.flags = RJ_SEG_MISSING;
    sg.ent_off = uint32_t(ent);
    sg.chunk0 = p.nchunks;
    p.nchunks += 1;
    ent += rj_interval_entries(0, uint64_t(sg.mcu_count) * p.nblk_mcu, p.nblk_mcu);
    dst += 16;
    p.segs.push_back(sg);
  }
  p.destuff_bytes = dst;
  p.entries = ent;
  FinishSegs(p);
}

void FinishSegs(DecodePlan &p) {
  p.seg_bucket.resize(p.segs.size());
  p.seg_lenblk.resize(p.segs.size());
  bool aligned = p.segs.size() == p.mcuy;
  uint32_t m = 0;
  p.src_total = 0;
  p.src_max = 0;
  for (size_t q = 0; q < p.segs.size(); q++) {
    const RjSegDev &sg = p.segs[q];
    p.src_total += sg.src_len;
    p.src_max = std::max(p.src_max, sg.src_len);
    p.seg_bucket[q] = uint16_t(std::min<uint32_t>(sg.src_len >> 5, 4095u));
    p.seg_lenblk[q] = ((sg.flags & RJ_SEG_MISSING) ? 0u : uint64_t(sg.dst_len)) |
                      (uint64_t(sg.mcu_count) * p.nblk_mcu << 32);
    aligned = aligned && sg.mcu_first == m && sg.mcu_count == p.mcux;
    m += p.mcux;
  }
  p.rows_aligned = aligned;
}

void Stream::CompleteFromDevice(uint32_t ecs_size, const RjSegDev *segs, uint32_t nsegs, const RjDsBlock *ds,
                                uint32_t nds) {
  DecodePlan &p = plan_;
  info_.ecs_size = ecs_size;
  p.segs.assign(segs, segs + nsegs);
  p.ds.assign(ds, ds + nds);
  uint64_t dst = 0, ent = 0;
  uint32_t nch = 0;
  for (const RjSegDev &sg : p.segs) {  // the totals BuildIntervals accumulates
    dst += (sg.flags & RJ_SEG_MISSING) ? 16u : ((uint64_t(sg.src_len) + 16 + 15) & ~uint64_t(15));
    ent += rj_interval_entries(sg.src_len, uint64_t(sg.mcu_count) * p.nblk_mcu, p.nblk_mcu);
    nch += rj_chunks(sg.src_len);
  }
  p.destuff_bytes = dst;
  p.entries = ent;
  p.nchunks = nch;
  FinishSegs(p);
  scan_pending_ = false;
}

const RjLeanTables *Stream::LeanTables() {
  if (!lean_) {
    auto t = std::make_unique<RjLeanTables>();
    bool ac_ok[2] = {false, false};
    for (int id = 0; id < 2; id++) {
      // only slots BuildPlanHeader accepted; an unused, invalid slot stays all 'bad' entries
      uint32_t *ac_subs = t->ac[id] + (1 << RJ_HL_AC_BITS);
      if (!plan_.ht_valid[id] ||
          !BuildLeanTable(info_.ht[id].dc_bits, info_.ht[id].dc_vals, true, t->dc[id], nullptr))
        FillLeanBad(true, t->dc[id], nullptr);
      if (!plan_.ht_valid[id] ||
          !BuildLeanTable(info_.ht[id].ac_bits, info_.ht[id].ac_vals, false, t->ac[id], ac_subs))
        FillLeanBad(false, t->ac[id], ac_subs);
      else
        ac_ok[id] = true;
    }
    // a DC table's second symbols are read with the AC table of the components that use it:
    // only when every scan component with that DC table has the same AC table (the map is part
    // of table_key, so every stream sharing these tables has the same map)
    int ac_of_dc[2];
    DcPairMap(info_, ac_of_dc);
    uint32_t single[2][1 << RJ_HL_AC_BITS];  // AC first levels before their pairs
    for (int id = 0; id < 2; id++) std::memcpy(single[id], t->ac[id], sizeof(single[id]));
    for (int id = 0; id < 2; id++) {
      if (ac_ok[id]) AddLeanPairs(t->ac[id], RJ_HL_AC_BITS, false, single[id]);
      const int ta = ac_of_dc[id];
      if (ta >= 0 && ac_ok[ta] && plan_.ht_valid[id]) AddLeanPairs(t->dc[id], RJ_HL_DC_BITS, true, single[ta]);
    }
    lean_ = std::move(t);
  }
  return lean_.get();
}

void Stream::ReleaseResident() {
  if (resident.device >= 0 && resident.block) {
    resident = Resident();  // drops this stream's share of the call's block
    return;
  }
  if (resident.device >= 0) {
    int cur = 0;
    if (hipGetDevice(&cur) == hipSuccess) {
      (void)hipSetDevice(resident.device);
      (void)hipFree(resident.ecs);
      (void)hipFree(resident.segs);
      (void)hipFree(resident.ds);
      if (resident.pscans) (void)hipFree(resident.pscans);
      if (resident.pivals) (void)hipFree(resident.pivals);
      if (resident.ptabs) (void)hipFree(resident.ptabs);
      (void)hipSetDevice(cur);
    }
  }
  resident = Resident();
}

int ImageInfo(const StreamInfo &s, uint8_t *nc, int *css, uint32_t *w, uint32_t *h) {
  if (!nc || !css || !w || !h) return -2;
  *nc = s.ncomp;
  w[0] = s.width;
  h[0] = s.height;
  w[3] = h[3] = 0;
  switch (s.css) {
    case kCss444: *css = 0; w[2] = w[1] = w[0]; h[2] = h[1] = h[0]; break;
    case kCss440: *css = 1; w[2] = w[1] = w[0]; h[2] = h[1] = h[0] >> 1; break;
    case kCss422: *css = 2; w[2] = w[1] = w[0] >> 1; h[2] = h[1] = h[0]; break;
    case kCss420: *css = 3; w[2] = w[1] = w[0] >> 1; h[2] = h[1] = h[0] >> 1; break;
    case kCss400: *css = 5; w[3] = w[2] = w[1] = 0; h[3] = h[2] = h[1] = 0; break;
    case kCss411: *css = 4; w[2] = w[1] = w[0] >> 2; h[2] = h[1] = h[0]; break;
    default: *css = -1; break;
  }
  return 0;
}

}  // namespace rj
