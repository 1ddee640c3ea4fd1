// rj_prog_stream.cpp -- host parser and planner for progressive (SOF2) streams.
//
// Beyond the reference: RocJpegStreamParser handles SOF0 only and stops at the first SOS
// (src/rocjpeg_parser.cpp:74-104, rocjpeg_parser.h:48), so a progressive stream fails to parse
// there.  SURVEY.md 8f rank 2 / BASELINE config C5 asks for it.  The marker walk restates
// libjpeg 9.4 (jdmarker.c get_sos / get_dht / get_dqt, jdinput.c latch_quant_tables,
// jdhuff.c start_pass_huff_decoder progression checks), as the CPU oracle does
// (oracle/jpeg_oracle.c make_plan_prog, pinned against libjpeg's coefficients):
//   * every scan records the Huffman tables in force at its SOS (DHT may change between scans)
//     and the DRI in force; its entropy-coded data runs to the first marker other than RSTn;
//   * a component's quant table is latched at the first scan that codes it;
//   * each scan's data is split into its restart intervals exactly like a baseline interval
//     (K0 destuffs them; a missing RST marker skips the rest of the scan's intervals).
// Planning: the dense coefficient layout, one RjHuffDev per distinct table, and a dependency
// level per scan -- a scan waits only for the earlier scans that touch one of its (component,
// coefficient) pairs, so e.g. the DC scan and the first AC scans of every component decode
// concurrently (rj_prog.hip).
#include <algorithm>
#include <cstring>

#include "rj_stream.h"

namespace rj {

namespace {

inline uint32_t Be16(const uint8_t *p) { return (uint32_t(p[0]) << 8) | p[1]; }

// End of a scan's entropy-coded data: the first marker other than RSTn (FF 00 is data, FF FF fill).
uint32_t ScanEnd(const uint8_t *d, uint32_t pos, uint32_t n) {
  while (pos + 1 < n) {
    if (d[pos] == 0xFF) {
      uint32_t q = pos + 1;
      while (q < n && d[q] == 0xFF) q++;
      if (q >= n) return pos;
      if (d[q] == 0x00 || (d[q] >= 0xD0 && d[q] <= 0xD7)) {
        pos = q + 1;
        continue;
      }
      return pos;
    }
    pos++;
  }
  return n;
}

int ClassifyCssP(const StreamInfo &s) {  // rocjpeg_parser.cpp:432-470 (same table as rj_stream.cpp)
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

// True when the frame header ahead of the first SOS is SOF2 (oracle is_progressive).
bool IsProgressiveStream(const uint8_t *d, uint32_t n) {
  if (!d || n < 4 || d[0] != 0xFF || d[1] != 0xD8) return false;
  uint32_t pos = 2;
  while (pos + 4 <= n) {
    while (pos < n && d[pos] == 0xFF) pos++;
    if (pos + 3 > n) return false;
    const uint32_t m = d[pos++];
    const uint32_t len = Be16(d + pos);
    if (m == 0xC2) return true;
    if (m == 0xDA || m == 0xC0 || m == 0xC1 || len < 2) return false;
    pos += len;
  }
  return false;
}

bool Stream::ParseProgressive(const uint8_t *d, uint32_t n) {
  StreamInfo &s = info_;
  DecodePlan &p = plan_;
  p.progressive = true;
  p.status = 0;
  struct RawTab {
    uint8_t bits[16];
    uint8_t vals[256];
    uint32_t cnt;
    bool ok;
  };
  RawTab ht[2][2];  // [ac][id]
  std::memset(ht, 0, sizeof(ht));
  uint8_t qt[4][64] = {};
  bool qt_ok[4] = {}, latched[4] = {};
  uint8_t qlat[4][64] = {};  // latched table of each component (zigzag order)
  uint32_t ri = 0;
  struct HScan {
    RjProgScanDev dev;
    uint32_t off, end;  // absolute stream offsets of the entropy-coded data
    uint8_t ah;
  };
  std::vector<HScan> scans;
  // distinct tables: raw content -> ptabs index
  struct TabKey {
    uint8_t dc;
    uint8_t bits[16];
    uint8_t vals[256];
  };
  std::vector<TabKey> keys;
  auto table_index = [&](const RawTab &t, bool dc) -> int {
    TabKey k;
    std::memset(&k, 0, sizeof(k));
    k.dc = dc;
    std::memcpy(k.bits, t.bits, 16);
    std::memcpy(k.vals, t.vals, t.cnt);
    for (size_t q = 0; q < keys.size(); q++)
      if (std::memcmp(&keys[q], &k, sizeof(k)) == 0) return int(q);
    // oracle build_htab: at most 12 DC / 162 AC symbols, no over-subscription, DC categories <= 15
    if (t.cnt > (dc ? 12u : 162u)) return -1;
    RjHuffDev h;
    if (!BuildHuffman(t.bits, t.vals, dc, &h)) return -1;
    if (p.ptabs.size() >= 0xFFFF) return -1;
    keys.push_back(k);
    p.ptabs.push_back(h);
    return int(p.ptabs.size() - 1);
  };

  uint32_t pos = 2;
  bool sof = false;
  while (pos + 1 < n) {
    if (d[pos] != 0xFF) {  // garbage between segments: skipped (libjpeg warns)
      pos++;
      continue;
    }
    while (pos < n && d[pos] == 0xFF) pos++;
    if (pos >= n) break;
    const uint32_t m = d[pos++];
    if (m == 0xD9) break;  // EOI
    if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7) || m == 0x01) continue;
    if (pos + 2 > n) break;
    const uint32_t len = Be16(d + pos), seg = pos;
    uint32_t next = pos + len;
    if (len < 2 || uint64_t(pos) + len > n) return false;
    switch (m) {
      case 0xC2: {
        if (sof || len < 8) return false;
        s.precision = d[seg + 2];
        s.height = uint16_t(Be16(d + seg + 3));
        s.width = uint16_t(Be16(d + seg + 5));
        s.ncomp = d[seg + 7];
        if (s.ncomp < 1 || s.ncomp > 3 || len < 8 + 3u * s.ncomp) return false;
        for (int i = 0; i < s.ncomp; i++) {
          const uint8_t *c = d + seg + 8 + 3 * i;
          s.comp[i].id = c[0];
          s.comp[i].h = c[1] >> 4;
          s.comp[i].v = c[1] & 15;
          s.comp[i].tq = c[2];
          if (c[2] >= 4) return false;
        }
        s.sof_seen = true;
        sof = true;
        break;
      }
      case 0xC0: case 0xC1: case 0xC3: case 0xC5: case 0xC6: case 0xC7:
      case 0xC9: case 0xCA: case 0xCB: case 0xCD: case 0xCE: case 0xCF:
        return false;  // a second frame
      case 0xC4: {
        uint32_t q = seg + 2;
        while (q < next) {
          if (q + 17 > next) return false;
          const uint32_t idx = d[q++], id = idx & 15, ac = (idx >> 4) != 0;
          if (id >= 2 || (idx >> 4) > 1) return false;
          uint32_t cnt = 0;
          for (int i = 0; i < 16; i++) cnt += d[q + i];
          std::memcpy(ht[ac][id].bits, d + q, 16);
          q += 16;
          if (cnt > 256 || q + cnt > next) return false;
          std::memset(ht[ac][id].vals, 0, 256);
          std::memcpy(ht[ac][id].vals, d + q, cnt);
          ht[ac][id].cnt = cnt;
          ht[ac][id].ok = true;
          q += cnt;
        }
        break;
      }
      case 0xDB: {
        uint32_t q = seg + 2;
        while (q < next) {
          const uint32_t idx = d[q++];
          if ((idx >> 4) || idx >= 4 || q + 64 > next) return false;  // 8-bit tables only
          std::memcpy(qt[idx], d + q, 64);
          qt_ok[idx] = true;
          q += 64;
        }
        break;
      }
      case 0xDD:
        if (len != 4) return false;
        ri = Be16(d + seg + 2);
        s.restart_interval = uint16_t(ri);
        break;
      case 0xDA: {
        if (!sof) return false;
        if (scans.size() >= 64) {  // oracle OJ_MAX_SCANS
          p.status = -4;
          return true;
        }
        HScan sc;
        std::memset(&sc, 0, sizeof(sc));
        RjProgScanDev &v = sc.dev;
        const uint32_t ns = d[seg + 2];
        if (ns < 1 || ns > 4 || len != 6 + 2 * ns) return false;
        const uint32_t ss = d[seg + 3 + 2 * ns], se = d[seg + 4 + 2 * ns];
        const uint32_t ah = d[seg + 5 + 2 * ns] >> 4, al = d[seg + 5 + 2 * ns] & 15;
        int ci_of[4] = {-1, -1, -1, -1};
        int tabs_used[2] = {-1, -1};
        for (uint32_t i = 0; i < ns; i++) {
          const uint32_t cs = d[seg + 3 + 2 * i], t = d[seg + 4 + 2 * i];
          int ci = -1;
          for (int c = 0; c < s.ncomp; c++)
            if (s.comp[c].id == cs) ci = c;
          if (ci < 0) return false;
          for (uint32_t j = 0; j < i; j++)
            if (ci_of[j] == ci) return false;
          ci_of[i] = ci;
          const uint32_t td = t >> 4, ta = t & 15;
          if (td >= 2 || ta >= 2) return false;
          int ti = -1;
          if (ss == 0 && ah == 0) {  // DC first: the DC table
            if (!ht[0][td].ok) return false;
            ti = table_index(ht[0][td], true);
          } else if (ss != 0) {      // AC scans: the AC table
            if (!ht[1][ta].ok) return false;
            ti = table_index(ht[1][ta], false);
          }
          if (ss == 0 && ah != 0) continue;  // DC refinement reads raw bits
          if (ti < 0) return false;
          // a lane holds two tables in LDS; the scan components pick one each
          if (tabs_used[0] < 0 || tabs_used[0] == ti) {
            tabs_used[0] = ti;
            v.tsel[i] = 0;
          } else if (tabs_used[1] < 0 || tabs_used[1] == ti) {
            tabs_used[1] = ti;
            v.tsel[i] = 1;
          } else {
            return false;  // three distinct tables in one scan: impossible with 2 table ids
          }
        }
        // jdhuff.c start_pass_huff_decoder: JERR_BAD_PROGRESSION
        if (ss == 0) {
          if (se != 0) return false;
        } else {
          if (se < ss || se > 63 || ns != 1) return false;
        }
        if (ah != 0 && ah - 1 != al) return false;
        if (al > 13) return false;
        for (uint32_t i = 0; i < ns; i++) {  // latch_quant_tables
          const int c = ci_of[i];
          if (!latched[c]) {
            const int tq = s.comp[c].tq;
            if (!qt_ok[tq]) return false;
            std::memcpy(qlat[c], qt[tq], 64);
            std::memcpy(s.qt_zz[tq], qt[tq], 64);
            s.qt_loaded[tq] = 1;
            latched[c] = true;
          }
        }
        v.ns = uint8_t(ns);
        v.ss = uint8_t(ss);
        v.se = uint8_t(se);
        v.al = uint8_t(al);
        sc.ah = uint8_t(ah);
        v.kind = ss == 0 ? (ah == 0 ? RJ_PK_DC_FIRST : RJ_PK_DC_REFINE) : (ah == 0 ? RJ_PK_AC_FIRST : RJ_PK_AC_REFINE);
        for (uint32_t i = 0; i < 3; i++) v.comp[i] = uint8_t(i < ns ? ci_of[i] : 0);
        v.tab[0] = uint16_t(tabs_used[0] < 0 ? 0xFFFF : tabs_used[0]);
        v.tab[1] = uint16_t(tabs_used[1] < 0 ? 0xFFFF : tabs_used[1]);
        v.ri = ri;
        sc.off = next;
        sc.end = ScanEnd(d, next, n);
        next = sc.end;
        scans.push_back(sc);
        break;
      }
      default:
        break;
    }
    pos = next;
  }
  if (!sof || scans.empty()) return false;
  if (s.precision != 8) {
    p.status = -4;
    return true;
  }
  s.css = ClassifyCssP(s);
  const int nc = s.ncomp;
  p.hmax = p.vmax = 1;
  for (int c = 0; c < nc; c++) {
    if (s.comp[c].h < 1 || s.comp[c].h > 4 || s.comp[c].v < 1 || s.comp[c].v > 4) return false;
    p.hmax = std::max(p.hmax, s.comp[c].h);
    p.vmax = std::max(p.vmax, s.comp[c].v);
  }
  p.interleaved = nc > 1;
  if (p.interleaved) {
    int bpm = 0;
    for (int c = 0; c < nc; c++) bpm += s.comp[c].h * s.comp[c].v;
    if (bpm > 10) return false;
  }
  for (int c = 0; c < nc; c++)
    if (!latched[c]) return false;  // a component no scan codes
  // the fields GetImageInfo and the output stage read
  s.scan_ncomp = s.ncomp;
  for (int c = 0; c < nc; c++) s.scomp[c].cs = s.comp[c].id;
  s.num_mcus = 0;
  {
    const uint32_t hf = s.comp[0].h, vf = s.comp[0].v;
    s.num_mcus = ((s.width + hf * 8 - 1) / (hf * 8)) * ((s.height + vf * 8 - 1) / (vf * 8));
  }
  // the ECS region handed to K0: first scan's data .. last scan's end (headers in between ride along)
  const uint32_t e0 = scans.front().off, e1 = std::max(scans.back().end, e0);
  s.ecs = d + e0;
  s.ecs_size = e1 - e0;

  // ---- geometry (oracle make_plan_prog; libjpeg jdinput.c initial_setup) ----
  p.mcux = (s.width + 8u * p.hmax - 1) / (8u * p.hmax);
  p.mcuy = (s.height + 8u * p.vmax - 1) / (8u * p.vmax);
  uint32_t hblk[3] = {};
  for (int c = 0; c < nc; c++) {
    const uint32_t cw = (uint32_t(s.width) * s.comp[c].h + p.hmax - 1) / p.hmax;
    const uint32_t ch = (uint32_t(s.height) * s.comp[c].v + p.vmax - 1) / p.vmax;
    p.cwblk[c] = (cw + 7) / 8;
    p.chblk[c] = (ch + 7) / 8;
    if (p.interleaved) {
      p.wblk[c] = p.mcux * s.comp[c].h;
      hblk[c] = p.mcuy * s.comp[c].v;
    } else {
      p.wblk[c] = p.cwblk[c];
      hblk[c] = p.chblk[c];
    }
    p.hblk[c] = hblk[c];
  }
  if (!p.interleaved) {
    p.mcux = p.wblk[0];
    p.mcuy = hblk[0];
    p.nblk_mcu = 1;
  } else {
    int b = 0;
    for (int c = 0; c < nc; c++) {
      p.comp_blk0[c] = uint8_t(b);
      for (int y = 0; y < s.comp[c].v; y++)
        for (int x = 0; x < s.comp[c].h; x++) {
          p.blk_comp[b] = uint8_t(c);
          p.blk_dx[b] = uint8_t(x);
          p.blk_dy[b] = uint8_t(y);
          b++;
        }
    }
    p.nblk_mcu = uint8_t(b);
  }
  uint64_t cb = 0, nzb = 0;
  for (int c = 0; c < nc; c++) {
    p.cblk0[c] = uint32_t(cb);
    p.nzblk0[c] = uint32_t(nzb);
    cb += uint64_t(p.wblk[c]) * hblk[c];
    nzb += uint64_t(p.cwblk[c]) * p.chblk[c];
  }
  p.coef_blocks = cb;
  p.nz_blocks = nzb;

  // ---- scans: unit geometry, dependency levels, progression checks ----
  // libjpeg warns (JWRN_BOGUS_PROGRESSION) and decodes on when a scan's Ah disagrees with the
  // bits already coded; the dense sign-magnitude accumulation equals libjpeg's two's
  // complement arithmetic only for consistent successive approximation, so such streams (and
  // first scans over already-coded coefficients) are refused with JPEG_NOT_SUPPORTED.
  int coef_bits[3][64];
  int lastlev[3][64], lastscan[3][64];
  for (int c = 0; c < 3; c++)
    for (int k = 0; k < 64; k++) coef_bits[c][k] = lastlev[c][k] = lastscan[c][k] = -1;
  bool bogus = false;
  p.plevels = 0;
  p.pscans.clear();
  for (HScan &sc : scans) {
    RjProgScanDev &v = sc.dev;
    const bool inter = v.ns > 1;
    for (int i = 0; i < 3; i++) {
      const int c = v.comp[i];
      v.hs[i] = uint8_t(inter && i < v.ns ? s.comp[c].h : 1);
      v.vs[i] = uint8_t(inter && i < v.ns ? s.comp[c].v : 1);
    }
    v.nblk = 0;
    for (int i = 0; i < v.ns; i++) v.nblk += uint32_t(v.hs[i]) * v.vs[i];
    if (inter) {
      v.units_x = p.mcux;
      v.units = p.mcux * p.mcuy;
    } else {
      v.units_x = p.cwblk[v.comp[0]];
      v.units = p.cwblk[v.comp[0]] * p.chblk[v.comp[0]];
    }
    int lev = 0;
    for (int i = 0; i < v.ns; i++) {
      const int c = v.comp[i];
      for (int k = v.ss; k <= v.se; k++) {
        const int expected = coef_bits[c][k] < 0 ? 0 : coef_bits[c][k];
        if (int(sc.ah) != expected) bogus = true;
        if (sc.ah == 0 && coef_bits[c][k] >= 0) bogus = true;  // a first scan over coded bits
        coef_bits[c][k] = v.al;
        lev = std::max(lev, lastlev[c][k] + 1);
      }
    }
    for (int i = 0; i < v.ns; i++)
      for (int k = v.ss; k <= v.se; k++) lastlev[v.comp[i]][k] = lev;
    v.level = uint8_t(std::min(lev, 255));
    p.plevels = std::max<uint32_t>(p.plevels, uint32_t(v.level) + 1);
    // producers for the pipelined launch: the latest earlier scan of each coefficient of the band
    // (that scan waited for its own producers, so its progress covers theirs)
    v.nprod = 0;
    if (v.kind == RJ_PK_AC_REFINE) {
      const int c = v.comp[0];
      for (int k = v.ss; k <= v.se && v.nprod != 0xFF; k++) {
        const int r = lastscan[c][k];
        if (r < 0) continue;  // refinement of an uncoded coefficient: bogus, refused below
        bool seen = false;
        for (int q = 0; q < v.nprod; q++) seen = seen || v.prod[q] == r;
        if (seen) continue;
        if (v.nprod < 3 && r < 0xFF) v.prod[v.nprod++] = uint8_t(r);
        else v.nprod = 0xFF;
      }
    }
    for (int i = 0; i < v.ns; i++)
      for (int k = v.ss; k <= v.se; k++) lastscan[v.comp[i]][k] = int(p.pscans.size());
    p.pscans.push_back(v);
  }
  if (bogus) {
    p.status = -4;
    return true;
  }
  std::memcpy(p.pqlat, qlat, sizeof(p.pqlat));
  p.pscan_src.clear();
  for (const HScan &sc : scans) {
    p.pscan_src.push_back(sc.off);
    p.pscan_src.push_back(std::max(sc.end, sc.off));
  }
  BuildProgressivePlan(d);
  return true;
}

// Restart intervals of every scan + K0 blocks + table set (quant tables per component).
void Stream::BuildProgressivePlan(const uint8_t *d) {
  const StreamInfo &s = info_;
  DecodePlan &p = plan_;
  if (s.width < 64 || s.height < 64 || s.width > 16384 || s.height > 16384 ||
      !(s.css == kCss444 || s.css == kCss440 || s.css == kCss422 || s.css == kCss420 || s.css == kCss400)) {
    p.status = -4;  // the SubmitDecode checks (rocjpeg_vaapi_decoder.cpp:586-592, 612-636)
    return;
  }
  // quant tables: component c's latched table in slot c (RjImageDev.comp_tq[c] = c); the
  // de-duplication key is those tables (no Huffman tables in the set: ht_loaded = 0, 0)
  std::memset(p.table_key, 0, sizeof(p.table_key));
  for (int q = 0; q < 4; q++) {
    p.qmax[q] = 1;
    for (int k = 0; k < 64; k++) {
      p.tables.qz[q][k] = q < s.ncomp ? p.pqlat[q][k] : 0;
      p.qmax[q] = std::max<uint16_t>(p.qmax[q], p.tables.qz[q][k]);
    }
  }
  std::memcpy(p.table_key + 2 + sizeof(s.ht), p.pqlat, size_t(s.ncomp) * 64);
  p.table_hash = Fnv1a(1469598103934665603ull, p.table_key, sizeof(p.table_key));

  const uint8_t *e = s.ecs;
  const uint32_t base = uint32_t(s.ecs - d);
  uint64_t dst = 0;
  std::vector<uint32_t> drops;
  p.pivals.clear();
  p.ds.clear();
  uint64_t rec = 0;  // refinement records (u64 words): AC 4 per unit, DC one bit per block
  for (size_t si = 0; si < p.pscans.size(); si++) {
    RjProgScanDev &v = p.pscans[si];
    v.ival0 = uint32_t(p.pivals.size());
    const bool refine = v.kind == RJ_PK_AC_REFINE || v.kind == RJ_PK_DC_REFINE;
    auto take_rec = [&](RjProgIvalDev &iv) {
      if (v.kind == RJ_PK_AC_REFINE) rec = (rec + 3) & ~uint64_t(3);  // 32-B records, 16-B stores
      iv.rec_off = uint32_t(rec);
      if (v.kind == RJ_PK_AC_REFINE) rec += uint64_t(iv.nunits) * 4;
      else if (v.kind == RJ_PK_DC_REFINE) rec += (uint64_t(iv.nunits) * v.nblk + 63) / 64;
      (void)refine;
    };
    const uint32_t b0 = p.pscan_src[2 * si] - base, b1 = p.pscan_src[2 * si + 1] - base;
    const uint32_t ri = v.ri, units = v.units;
    const uint32_t expected = ri ? (units + ri - 1) / ri : 1;
    uint32_t made = 0;
    drops.clear();
    size_t dq = 0;
    auto emit = [&](uint32_t b, uint32_t stop) {
      while (stop > b && e[stop - 1] == 0xFF) stop--;  // trailing fill
      if (made >= expected) return;
      RjProgIvalDev iv;
      std::memset(&iv, 0, sizeof(iv));
      const uint32_t src_len = stop - b;
      iv.dst_off = uint32_t(dst);
      while (dq < drops.size() && drops[dq] < b) dq++;
      uint32_t dropped = 0;
      for (uint32_t o = 0; o < src_len; o += RJ_DS_BLOCK) {
        const uint32_t blen = std::min(RJ_DS_BLOCK, src_len - o);
        RjDsBlock blk;
        blk.src_off = b + o;
        blk.len = blen | (o == 0 ? 0x80000000u : 0u);
        blk.dst_off = iv.dst_off + o - dropped;
        blk.zero_end = 0;
        while (dq < drops.size() && drops[dq] < b + o + blen) {
          dq++;
          dropped++;
        }
        p.ds.push_back(blk);
      }
      iv.dst_len = src_len - dropped;
      if (src_len) p.ds.back().zero_end = uint32_t(dst + ((uint64_t(src_len) + 16 + 15) & ~uint64_t(15)));
      iv.unit0 = made * (ri ? ri : units);
      iv.nunits = ri ? std::min(ri, units - iv.unit0) : units;
      iv.scan = uint16_t(si);
      take_rec(iv);
      dst += (uint64_t(src_len) + 16 + 15) & ~uint64_t(15);
      p.pivals.push_back(iv);
      made++;
    };
    uint32_t start = b0, i = b0, cut = UINT32_MAX;
    while (i + 1 < b1) {
      const uint8_t *f = static_cast<const uint8_t *>(std::memchr(e + i, 0xFF, b1 - i));
      if (f == nullptr) break;
      i = uint32_t(f - e);
      if (i + 1 >= b1) break;
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
      } else {  // RSTn without DRI: the data ends there (libjpeg reads zero bits past a marker)
        if (cut == UINT32_MAX) cut = i;
        i += 2;
      }
    }
    emit(start, std::min(b1, cut));
    while (made < expected) {  // intervals whose RST marker never came: skipped
      RjProgIvalDev iv;
      std::memset(&iv, 0, sizeof(iv));
      iv.dst_off = uint32_t(dst);
      iv.unit0 = made * ri;
      iv.nunits = std::min(ri, units - iv.unit0);
      iv.scan = uint16_t(si);
      iv.flags = RJ_SEG_MISSING;
      take_rec(iv);  // a skipped interval's records stay zero (the fold applies nothing)
      dst += 16;
      p.pivals.push_back(iv);
      made++;
    }
  }
  p.destuff_bytes = dst;
  p.prec_words = rec;
  if (rec >= (1ull << 32)) p.status = -4;  // record offsets are 32-bit
  p.segs.clear();
  p.seg_bucket.clear();
  p.seg_lenblk.clear();
  p.rows_aligned = false;
  p.entries = 0;
  p.nchunks = 0;
}

}  // namespace rj
