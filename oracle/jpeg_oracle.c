/*
 * jpeg_oracle.c -- CPU ORACLE.  TEST INFRASTRUCTURE ONLY (see jpeg_oracle.h).
 *
 * A deliberately plain, sequential restatement.  Nothing here is shared with the
 * product (rocjpeg_amd/csrc): the product has its own parser, its own table builder
 * and HIP kernels; this file exists to check them.
 */
#include "jpeg_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* RocJpegStatus values (api/rocjpeg.h:53-67) */
enum { ST_OK = 0, ST_INVALID = -2, ST_BAD_JPEG = -3, ST_NOT_SUPPORTED = -4, ST_OOM = -5 };
/* ChromaSubsampling (src/rocjpeg_parser.h:148-156) */
enum { CSS_444 = 0, CSS_440 = 1, CSS_422 = 2, CSS_420 = 3, CSS_411 = 4, CSS_400 = 5, CSS_UNKNOWN = -1 };
/* RocJpegOutputFormat (api/rocjpeg.h:124-141) */
enum { OUT_NATIVE = 0, OUT_YUV_PLANAR = 1, OUT_Y = 2, OUT_RGB = 3, OUT_RGB_PLANAR = 4 };

static unsigned be16(const uint8_t *p) { return ((unsigned)p[0] << 8) | p[1]; }

/* ---------------------------------------------------------------------------------
 * Parser: restates src/rocjpeg_parser.cpp:43-470 (same acceptance rules), but every
 * read is bounds-checked (the reference reads past the buffer on truncated input;
 * there we fail instead).
 * ------------------------------------------------------------------------------- */
static int css_of(const oj_params *p) {
  /* rocjpeg_parser.cpp:432-470 (note: comp[1]/comp[2] are zero for 1-component images) */
  int h1 = p->comp[0].h, h2 = p->comp[1].h, h3 = p->comp[2].h;
  int v1 = p->comp[0].v, v2 = p->comp[1].v, v3 = p->comp[2].v;
#define F(a, b, c, d, e, f) (h1 == a && h2 == b && h3 == c && v1 == d && v2 == e && v3 == f)
  if (F(1, 1, 1, 1, 1, 1) || F(2, 2, 2, 2, 2, 2) || F(4, 4, 4, 4, 4, 4)) return CSS_444;
  if (F(1, 1, 1, 2, 1, 1)) return CSS_440;
  if (F(2, 1, 1, 1, 1, 1) || F(2, 1, 1, 2, 2, 2) || F(2, 2, 2, 2, 1, 1)) return CSS_422;
  if (F(2, 1, 1, 2, 1, 1)) return CSS_420;
  if (F(4, 1, 1, 1, 1, 1)) return CSS_411;
  if (F(1, 0, 0, 1, 0, 0) || F(4, 0, 0, 4, 0, 0)) return CSS_400;
#undef F
  return CSS_UNKNOWN;
}

int oj_parse(const uint8_t *d, size_t n, oj_params *p) {
  memset(p, 0, sizeof(*p));
  if (!d || n < 4) return 0;
  if (d[0] != 0xFF || d[1] != 0xD8) return 0; /* :64-67 */
  size_t pos = 2;                               /* ParseSOI :133-147 */
  int sos = 0, dht = 0, dqt = 0;
  while (!sos && pos < n) { /* :74-109 */
    while (pos < n && d[pos] == 0xFF) pos++;
    if (pos + 3 > n) return 0;
    unsigned marker = d[pos++];
    size_t seg = pos; /* points at the 2-byte length */
    size_t L = be16(d + seg);
    size_t next = seg + L;
    if (L < 2 || next > n) return 0;
    switch (marker) {
      case 0xC0: { /* ParseSOF :160-207 */
        if (L < 8) return 0;
        p->precision = d[seg + 2];
        p->height = (uint16_t)be16(d + seg + 3);
        p->width = (uint16_t)be16(d + seg + 5);
        p->ncomp = d[seg + 7];
        if (p->ncomp > 3) return 0;
        if (L < 8 + 3u * p->ncomp) return 0;
        for (int i = 0; i < p->ncomp; i++) {
          const uint8_t *c = d + seg + 8 + 3 * i;
          p->comp[i].id = c[0];
          if (c[2] >= 4) return 0;
          p->comp[i].v = c[1] & 0xF;
          p->comp[i].h = c[1] >> 4;
          p->comp[i].tq = c[2];
        }
        unsigned hf = p->comp[0].h, vf = p->comp[0].v;
        if (hf && vf)
          p->num_mcus = ((p->width + hf * 8 - 1) / (hf * 8)) * ((p->height + vf * 8 - 1) / (vf * 8));
        p->css = css_of(p);
        p->sof_seen = 1;
        break;
      }
      case 0xC4: { /* ParseDHT :256-313 */
        long len = (long)L - 2;
        size_t s = seg + 2;
        while (len > 0) {
          if (s + 17 > next) return 0;
          unsigned idx = d[s++];
          unsigned ac = idx & 0xF0, id = idx & 0x0F;
          if (id >= 2) return 0;
          unsigned cnt = 0;
          for (int i = 0; i < 16; i++) cnt += d[s + i];
          if (ac) memcpy(p->ht[id].ac_bits, d + s, 16);
          else memcpy(p->ht[id].dc_bits, d + s, 16);
          s += 16;
          if (s + cnt > next) return 0;
          if (ac) {
            if (cnt > 162) return 0;
            memcpy(p->ht[id].ac_vals, d + s, cnt);
          } else {
            if (cnt > 12) return 0;
            memcpy(p->ht[id].dc_vals, d + s, cnt);
          }
          p->ht_loaded[id] = 1;
          len -= 17 + (long)cnt;
          s += cnt;
        }
        dht = 1;
        break;
      }
      case 0xDB: { /* ParseDQT :217-246 */
        size_t s = seg + 2;
        while (s < next) {
          unsigned idx = d[s++];
          if (idx >> 4) return 0;
          if (idx >= 4) return 0;
          if (s + 64 > n) return 0;
          memcpy(p->qt_zz[idx & 15], d + s, 64);
          p->qt_loaded[idx & 15] = 1;
          s += 64;
        }
        dqt = 1;
        break;
      }
      case 0xDD: /* ParseDRI :374-390 */
        if (L != 4) return 0;
        p->restart_interval = (uint16_t)be16(d + seg + 2);
        break;
      case 0xDA: { /* ParseSOS :324-363 */
        unsigned ns = d[seg + 2];
        if (ns > 3) return 0;
        if (L < 6 + 2 * ns) return 0;
        p->scan_ncomp = (uint8_t)ns;
        for (unsigned i = 0; i < ns; i++) {
          unsigned cs = d[seg + 3 + 2 * i], t = d[seg + 4 + 2 * i];
          p->scomp[i].cs = (uint8_t)cs;
          p->scomp[i].td = (uint8_t)(t >> 4);
          p->scomp[i].ta = (uint8_t)(t & 15);
          if ((t & 15) >= 4 || (t >> 4) >= 4) return 0;
          if (cs != p->comp[i].id) return 0;
        }
        sos = 1;
        break;
      }
      default:
        break;
    }
    pos = next;
  }
  if (!dht || !dqt) return 0; /* :111-118 */
  /* ParseEOI :400-416 -- first FF D9 after the SOS header */
  size_t e = pos;
  if (sos) {
    while (e + 1 < n && !(d[e] == 0xFF && d[e + 1] == 0xD9)) e++;
    if (e + 1 >= n) e = n;
  }
  p->ecs_offset = (uint32_t)(sos ? pos : n);
  p->ecs_size = (uint32_t)(sos ? e - pos : 0);
  return 1;
}

int oj_image_info(const oj_params *p, uint8_t *nc, int *css, uint32_t w[4], uint32_t h[4]) {
  /* rocjpeg_decoder.cpp:307-358 */
  if (!p || !nc || !css || !w || !h) return ST_INVALID;
  *nc = p->ncomp;
  w[0] = p->width; h[0] = p->height; w[3] = 0; h[3] = 0;
  switch (p->css) {
    case CSS_444: *css = 0; w[2] = w[1] = w[0]; h[2] = h[1] = h[0]; break;
    case CSS_440: *css = 1; w[2] = w[1] = w[0]; h[2] = h[1] = h[0] >> 1; break;
    case CSS_422: *css = 2; w[2] = w[1] = w[0] >> 1; h[2] = h[1] = h[0]; break;
    case CSS_420: *css = 3; w[2] = w[1] = w[0] >> 1; h[2] = h[1] = h[0] >> 1; break;
    case CSS_400: *css = 5; w[3] = w[2] = w[1] = 0; h[3] = h[2] = h[1] = 0; break;
    case CSS_411: *css = 4; w[2] = w[1] = w[0] >> 2; h[2] = h[1] = h[0]; break;
    default: *css = -1; break;
  }
  return ST_OK;
}

/* ---------------------------------------------------------------------------------
 * Decode core: T.81 baseline sequential Huffman (Annex C table generation, F.2.2
 * decoding procedures, F.2.1.3 DC prediction, restart handling per F.2.2.x / B.2.1)
 * with libjpeg's conventions for corrupt/truncated data (zero bits past a marker,
 * remaining MCUs of the interval left zero, bad code -> symbol 0).
 * ------------------------------------------------------------------------------- */
static const uint8_t kZigzag[80] = { /* natural index of zigzag position k (+16 pad) */
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33,
    40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36,
    29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54,
    47, 55, 62, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

typedef struct {
  int32_t maxcode[18]; /* maxcode[l] for l=1..16, [17] sentinel */
  int32_t valoff[17];  /* vals index = code + valoff[l] */
  uint8_t vals[256];
} htab;

static int build_htab(const uint8_t bits[16], const uint8_t *vals, int nvals_max, htab *t) {
  int k = 0, code = 0;
  for (int l = 1; l <= 16; l++) {
    int nb = bits[l - 1];
    if (nb) {
      t->valoff[l] = k - code;
      code += nb;
      k += nb;
      t->maxcode[l] = code - 1;
    } else {
      t->maxcode[l] = -1;
      t->valoff[l] = 0;
    }
    if (code > (1 << l)) return 0; /* over-subscribed table (libjpeg: JERR_BAD_HUFF_TABLE) */
    code <<= 1;
  }
  t->maxcode[17] = 0x7FFFFFFF;
  if (k > nvals_max) return 0;
  memset(t->vals, 0, sizeof(t->vals));
  memcpy(t->vals, vals, (size_t)k);
  if (nvals_max == 12) /* DC table: libjpeg rejects categories > 15 (jdhuff.c) */
    for (int i = 0; i < k; i++)
      if (vals[i] > 15) return 0;
  return 1;
}

typedef struct {
  const uint8_t *d;
  size_t pos, end;   /* byte cursor inside the ECS */
  uint32_t acc;      /* bit accumulator, MSB first */
  int nacc;
  int hit_marker;    /* a marker was reached: further bits are zeros */
  int insufficient;  /* a zero bit was consumed (libjpeg insufficient_data) */
} bitrd;

static int getbit(bitrd *b) {
  if (b->nacc == 0) {
    unsigned byte = 0;
    if (!b->hit_marker && b->pos < b->end) {
      byte = b->d[b->pos];
      if (byte == 0xFF) {
        size_t q = b->pos + 1;
        while (q < b->end && b->d[q] == 0xFF) q++; /* fill bytes */
        if (q < b->end && b->d[q] == 0x00) {
          b->pos = q + 1; /* stuffed FF00 -> data byte FF */
        } else {
          b->hit_marker = 1; /* pos stays on the FF so next_restart() can find the marker */
          byte = 0;
        }
      } else {
        b->pos++;
      }
    } else {
      b->hit_marker = 1;
    }
    if (b->hit_marker && byte == 0) b->insufficient = 1;
    b->acc = byte;
    b->nacc = 8;
  }
  b->nacc--;
  return (b->acc >> b->nacc) & 1;
}

static int getbits(bitrd *b, int n) {
  int v = 0;
  for (int i = 0; i < n; i++) v = (v << 1) | getbit(b);
  return v;
}

static int hdecode(bitrd *b, const htab *t) {
  int code = getbit(b), l = 1;
  while (l <= 16 && code > t->maxcode[l]) {
    code = (code << 1) | getbit(b);
    l++;
  }
  if (l > 16) return 0; /* libjpeg: JWRN_HUFF_BAD_CODE, returns 0 */
  return t->vals[(code + t->valoff[l]) & 255];
}

static int extend(int v, int s) { return (s && v < (1 << (s - 1))) ? v - (1 << s) + 1 : v; }

/* Skip to just after the next RSTn marker (discarding buffered bits).  Returns 0 when no
 * marker is left: libjpeg then keeps insufficient_data set ("smack up against a marker"),
 * so the whole interval stays zero (jdhuff.c process_restart). */
static int next_restart(bitrd *b) {
  b->nacc = 0;
  size_t q = b->pos;
  while (q + 1 < b->end) {
    if (b->d[q] == 0xFF && b->d[q + 1] >= 0xD0 && b->d[q + 1] <= 0xD7) {
      b->pos = q + 2;
      b->hit_marker = 0;
      b->insufficient = 0;
      return 1;
    }
    q++;
  }
  b->pos = b->end;
  b->hit_marker = 1;
  b->insufficient = 0;
  return 0;
}

/* One scan of a progressive (SOF2) stream: its header, the Huffman tables in force when it
 * started (DHT may change between scans), its DRI and its entropy-coded byte range. */
#define OJ_MAX_SCANS 64
typedef struct {
  int ns, comp[4];         /* component indexes (into the frame) */
  int ss, se, ah, al;
  int ri;
  htab dc[4], ac[4];       /* per scan component */
  size_t ecs_off, ecs_end;
} pscan;

typedef struct {
  oj_params p;
  int nc, hmax, vmax, mcux, mcuy, interleaved;
  int wblk[4], hblk[4];
  size_t coef_off[4], plane_off[4];
  size_t coef_total, plane_total;
  htab dc[4], ac[4];
  uint16_t q[4][64]; /* natural order */
  /* progressive */
  int progressive, nscans;
  int cwblk[4], chblk[4];  /* width/height_in_blocks: the blocks a non-interleaved scan codes */
  pscan scans[OJ_MAX_SCANS];
} plan;

static int is_progressive(const uint8_t *d, size_t n);
static int make_plan_prog(const uint8_t *d, size_t n, plan *pl);

static int make_plan(const uint8_t *data, size_t len, plan *pl) {
  memset(pl, 0, sizeof(*pl));
  if (is_progressive(data, len)) return make_plan_prog(data, len, pl);
  if (!oj_parse(data, len, &pl->p)) return ST_BAD_JPEG;
  oj_params *p = &pl->p;
  if (!p->sof_seen || p->ncomp == 0) return ST_NOT_SUPPORTED;
  if (p->precision != 8) return ST_NOT_SUPPORTED;
  if (p->scan_ncomp != p->ncomp) return ST_NOT_SUPPORTED;
  pl->nc = p->ncomp;
  for (int c = 0; c < pl->nc; c++) {
    if (p->comp[c].h < 1 || p->comp[c].h > 4 || p->comp[c].v < 1 || p->comp[c].v > 4) return ST_BAD_JPEG;
    if (p->comp[c].h > pl->hmax) pl->hmax = p->comp[c].h;
    if (p->comp[c].v > pl->vmax) pl->vmax = p->comp[c].v;
  }
  pl->interleaved = pl->nc > 1;
  if (pl->interleaved) {
    int bpm = 0;
    for (int c = 0; c < pl->nc; c++) bpm += p->comp[c].h * p->comp[c].v;
    if (bpm > 10) return ST_BAD_JPEG;
    pl->mcux = (p->width + 8 * pl->hmax - 1) / (8 * pl->hmax);
    pl->mcuy = (p->height + 8 * pl->vmax - 1) / (8 * pl->vmax);
    for (int c = 0; c < pl->nc; c++) {
      pl->wblk[c] = pl->mcux * p->comp[c].h;
      pl->hblk[c] = pl->mcuy * p->comp[c].v;
    }
  } else {
    int cw = (p->width * p->comp[0].h + pl->hmax - 1) / pl->hmax;
    int ch = (p->height * p->comp[0].v + pl->vmax - 1) / pl->vmax;
    pl->wblk[0] = (cw + 7) / 8;
    pl->hblk[0] = (ch + 7) / 8;
    pl->mcux = pl->wblk[0];
    pl->mcuy = pl->hblk[0];
  }
  size_t co = 0, po = 0;
  for (int c = 0; c < pl->nc; c++) {
    pl->coef_off[c] = co;
    pl->plane_off[c] = po;
    co += (size_t)pl->wblk[c] * pl->hblk[c] * 64;
    po += (size_t)pl->wblk[c] * pl->hblk[c] * 64;
  }
  pl->coef_total = co;
  pl->plane_total = po;
  for (int c = 0; c < pl->nc; c++) {
    int td = p->scomp[c].td, ta = p->scomp[c].ta;
    if (td >= 2 || ta >= 2 || !p->ht_loaded[td] || !p->ht_loaded[ta]) return ST_BAD_JPEG;
    if (!build_htab(p->ht[td].dc_bits, p->ht[td].dc_vals, 12, &pl->dc[c])) return ST_BAD_JPEG;
    if (!build_htab(p->ht[ta].ac_bits, p->ht[ta].ac_vals, 162, &pl->ac[c])) return ST_BAD_JPEG;
    int tq = p->comp[c].tq;
    if (!p->qt_loaded[tq]) return ST_BAD_JPEG;
    for (int k = 0; k < 64; k++) pl->q[c][kZigzag[k]] = p->qt_zz[tq][k];
  }
  return ST_OK;
}

/* ---------------------------------------------------------------------------------
 * Progressive (SOF2) decode -- SURVEY.md 8f rank 2 (config C5).  The reference parser
 * rejects SOF2 (rocjpeg_parser.cpp:74-104 handles SOF0 only), so there is no reference
 * arithmetic: this restates ITU-T T.81 Annex G and IJG libjpeg 9.4 (jdhuff.c
 * decode_mcu_DC_first / _AC_first / _DC_refine / _AC_refine, process_restart;
 * jdinput.c latch_quant_tables; jdmarker.c get_sos) and is pinned against libjpeg's own
 * jpeg_read_coefficients output (oracle/libjpeg_golden.c).  Semantics kept from libjpeg:
 *   - a needed bit past the data reads as 0 and sets insufficient_data; the MCUs after
 *     that one, up to the next restart, are skipped (their coefficients keep their values);
 *   - a restart marker that is not there keeps them skipped to the end of the interval;
 *   - each component's quant table is latched at the first scan that contains it;
 *   - block smoothing (libjpeg's output for incomplete progressions) is not applied: the
 *     planes are the ISLOW transform of the final coefficients.
 * ------------------------------------------------------------------------------- */
static int is_progressive(const uint8_t *d, size_t n) {
  if (!d || n < 4 || d[0] != 0xFF || d[1] != 0xD8) return 0;
  size_t pos = 2;
  while (pos + 4 <= n) {
    while (pos < n && d[pos] == 0xFF) pos++;
    if (pos + 3 > n) return 0;
    unsigned m = d[pos++];
    size_t len = be16(d + pos);
    if (m == 0xC2) return 1;
    if (m == 0xDA || m == 0xC0 || m == 0xC1 || len < 2) return 0;
    pos += len;
  }
  return 0;
}

/* End of a scan's entropy-coded data: the first marker other than RSTn (FF 00 is data,
 * FF FF is fill). */
static size_t scan_end(const uint8_t *d, size_t pos, size_t n) {
  while (pos + 1 < n) {
    if (d[pos] == 0xFF) {
      size_t q = pos + 1;
      while (q < n && d[q] == 0xFF) q++;
      if (q >= n) return pos;
      if (d[q] == 0x00 || (d[q] >= 0xD0 && d[q] <= 0xD7)) { pos = q + 1; continue; }
      return pos;
    }
    pos++;
  }
  return n;
}

static int make_plan_prog(const uint8_t *d, size_t n, plan *pl) {
  oj_params *p = &pl->p;
  uint8_t ht_bits[2][2][16], ht_vals[2][2][256];
  int ht_ok[2][2] = {{0, 0}, {0, 0}};
  uint8_t qt[4][64];
  int qt_ok[4] = {0, 0, 0, 0}, latched[4] = {0, 0, 0, 0};
  int ri = 0;
  pl->progressive = 1;
  size_t pos = 2;
  int sof = 0, eoi = 0;
  while (!eoi && pos + 1 < n) {
    if (d[pos] != 0xFF) { pos++; continue; } /* garbage between segments: skip (libjpeg warns) */
    while (pos < n && d[pos] == 0xFF) pos++;
    if (pos >= n) break;
    unsigned m = d[pos++];
    if (m == 0xD9) { eoi = 1; break; }
    if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7) || m == 0x01) continue;
    if (pos + 2 > n) break;
    size_t len = be16(d + pos), seg = pos, next = pos + len;
    if (len < 2 || next > n) return ST_BAD_JPEG;
    switch (m) {
      case 0xC2: {
        if (sof || len < 8) return ST_BAD_JPEG;
        p->precision = d[seg + 2];
        p->height = (uint16_t)be16(d + seg + 3);
        p->width = (uint16_t)be16(d + seg + 5);
        p->ncomp = d[seg + 7];
        if (p->ncomp < 1 || p->ncomp > 3 || len < 8 + 3u * p->ncomp) return ST_BAD_JPEG;
        for (int i = 0; i < p->ncomp; i++) {
          const uint8_t *c = d + seg + 8 + 3 * i;
          p->comp[i].id = c[0];
          p->comp[i].h = c[1] >> 4;
          p->comp[i].v = c[1] & 15;
          p->comp[i].tq = c[2];
          if (c[2] >= 4) return ST_BAD_JPEG;
        }
        p->sof_seen = 1;
        sof = 1;
        break;
      }
      case 0xC0: case 0xC1: case 0xC3: case 0xC5: case 0xC6: case 0xC7:
      case 0xC9: case 0xCA: case 0xCB: case 0xCD: case 0xCE: case 0xCF:
        return ST_BAD_JPEG; /* a second frame */
      case 0xC4: {
        size_t q = seg + 2;
        while (q < next) {
          if (q + 17 > next) return ST_BAD_JPEG;
          unsigned idx = d[q++], id = idx & 15, ac = (idx >> 4) != 0;
          if (id >= 2 || (idx >> 4) > 1) return ST_BAD_JPEG;
          unsigned cnt = 0;
          for (int i = 0; i < 16; i++) cnt += d[q + i];
          memcpy(ht_bits[ac][id], d + q, 16);
          q += 16;
          if (cnt > 256 || q + cnt > next) return ST_BAD_JPEG;
          memset(ht_vals[ac][id], 0, 256);
          memcpy(ht_vals[ac][id], d + q, cnt);
          ht_ok[ac][id] = 1;
          q += cnt;
        }
        break;
      }
      case 0xDB: {
        size_t q = seg + 2;
        while (q < next) {
          unsigned idx = d[q++];
          if ((idx >> 4) || idx >= 4 || q + 64 > next) return ST_BAD_JPEG; /* 8-bit tables only */
          memcpy(qt[idx], d + q, 64);
          qt_ok[idx] = 1;
          q += 64;
        }
        break;
      }
      case 0xDD:
        if (len != 4) return ST_BAD_JPEG;
        ri = (int)be16(d + seg + 2);
        break;
      case 0xDA: {
        if (!sof) return ST_BAD_JPEG;
        if (pl->nscans >= OJ_MAX_SCANS) return ST_NOT_SUPPORTED;
        pscan *sc = &pl->scans[pl->nscans];
        unsigned ns = d[seg + 2];
        if (ns < 1 || ns > 4 || len != 6 + 2 * ns) return ST_BAD_JPEG;
        sc->ns = (int)ns;
        for (unsigned i = 0; i < ns; i++) {
          unsigned cs = d[seg + 3 + 2 * i], t = d[seg + 4 + 2 * i];
          int ci = -1;
          for (int c = 0; c < p->ncomp; c++)
            if (p->comp[c].id == cs) ci = c;
          if (ci < 0) return ST_BAD_JPEG;
          for (unsigned j = 0; j < i; j++)
            if (sc->comp[j] == ci) return ST_BAD_JPEG;
          sc->comp[i] = ci;
          unsigned td = t >> 4, ta = t & 15;
          if (td >= 2 || ta >= 2) return ST_BAD_JPEG;
          /* tables are needed only by the scan kinds that use them */
          sc->ss = d[seg + 3 + 2 * ns];
          if (sc->ss == 0 && !(d[seg + 5 + 2 * ns] >> 4)) {
            if (!ht_ok[0][td]) return ST_BAD_JPEG;
            if (!build_htab(ht_bits[0][td], ht_vals[0][td], 12, &sc->dc[i])) return ST_BAD_JPEG;
          }
          if (sc->ss != 0) {
            if (!ht_ok[1][ta]) return ST_BAD_JPEG;
            if (!build_htab(ht_bits[1][ta], ht_vals[1][ta], 162, &sc->ac[i])) return ST_BAD_JPEG;
          }
        }
        sc->ss = d[seg + 3 + 2 * ns];
        sc->se = d[seg + 4 + 2 * ns];
        sc->ah = d[seg + 5 + 2 * ns] >> 4;
        sc->al = d[seg + 5 + 2 * ns] & 15;
        /* jdhuff.c start_pass_huff_decoder progressive checks (JERR_BAD_PROGRESSION) */
        if (sc->ss == 0) {
          if (sc->se != 0) return ST_BAD_JPEG;
        } else {
          if (sc->se < sc->ss || sc->se > 63 || sc->ns != 1) return ST_BAD_JPEG;
        }
        if (sc->ah != 0 && sc->ah - 1 != sc->al) return ST_BAD_JPEG;
        if (sc->al > 13) return ST_BAD_JPEG;
        sc->ri = ri;
        for (int i = 0; i < sc->ns; i++) { /* latch_quant_tables */
          int c = sc->comp[i];
          if (!latched[c]) {
            int tq = p->comp[c].tq;
            if (!qt_ok[tq]) return ST_BAD_JPEG;
            for (int k = 0; k < 64; k++) pl->q[c][kZigzag[k]] = qt[tq][k];
            memcpy(p->qt_zz[tq], qt[tq], 64);
            p->qt_loaded[tq] = 1;
            latched[c] = 1;
          }
        }
        sc->ecs_off = next;
        sc->ecs_end = scan_end(d, next, n);
        pl->nscans++;
        next = sc->ecs_end;
        break;
      }
      default:
        break;
    }
    pos = next;
  }
  if (!sof || pl->nscans == 0) return ST_BAD_JPEG;
  if (p->precision != 8) return ST_NOT_SUPPORTED;
  p->css = css_of(p);
  pl->nc = p->ncomp;
  for (int c = 0; c < pl->nc; c++) {
    if (p->comp[c].h < 1 || p->comp[c].h > 4 || p->comp[c].v < 1 || p->comp[c].v > 4) return ST_BAD_JPEG;
    if (p->comp[c].h > pl->hmax) pl->hmax = p->comp[c].h;
    if (p->comp[c].v > pl->vmax) pl->vmax = p->comp[c].v;
  }
  pl->interleaved = pl->nc > 1;
  if (pl->interleaved) {
    int bpm = 0;
    for (int c = 0; c < pl->nc; c++) bpm += p->comp[c].h * p->comp[c].v;
    if (bpm > 10) return ST_BAD_JPEG;
  }
  pl->mcux = (p->width + 8 * pl->hmax - 1) / (8 * pl->hmax);
  pl->mcuy = (p->height + 8 * pl->vmax - 1) / (8 * pl->vmax);
  for (int c = 0; c < pl->nc; c++) {
    int cw = (p->width * p->comp[c].h + pl->hmax - 1) / pl->hmax;
    int ch = (p->height * p->comp[c].v + pl->vmax - 1) / pl->vmax;
    pl->cwblk[c] = (cw + 7) / 8;
    pl->chblk[c] = (ch + 7) / 8;
    if (pl->interleaved) {
      pl->wblk[c] = pl->mcux * p->comp[c].h;
      pl->hblk[c] = pl->mcuy * p->comp[c].v;
    } else {
      pl->wblk[c] = pl->cwblk[c];
      pl->hblk[c] = pl->chblk[c];
      pl->mcux = pl->wblk[c];
      pl->mcuy = pl->hblk[c];
    }
  }
  for (int c = 0; c < pl->nc; c++)
    if (!latched[c]) return ST_BAD_JPEG; /* a component no scan codes */
  size_t co = 0;
  for (int c = 0; c < pl->nc; c++) {
    pl->coef_off[c] = co;
    pl->plane_off[c] = co;
    co += (size_t)pl->wblk[c] * pl->hblk[c] * 64;
  }
  pl->coef_total = pl->plane_total = co;
  /* the fields GetImageInfo and the output stage read */
  p->scan_ncomp = p->ncomp;
  for (int c = 0; c < pl->nc; c++) p->scomp[c].cs = p->comp[c].id;
  return ST_OK;
}

/* libjpeg decode_mcu_AC_refine's correction-bit step for one already-nonzero coefficient */
static void refine_coef(bitrd *b, int16_t *c, int p1, int m1) {
  if (getbit(b) && (*c & p1) == 0) *c = (int16_t)(*c >= 0 ? *c + p1 : *c + m1);
}

static void prog_block(bitrd *b, const pscan *sc, int i, int16_t *blk, int *pred, int *eobrun) {
  const int al = sc->al;
  if (sc->ss == 0) {
    if (sc->ah == 0) { /* DC first */
      int s = hdecode(b, &sc->dc[i]);
      int diff = s ? extend(getbits(b, s), s) : 0;
      *pred += diff;
      blk[0] = (int16_t)(*pred << al);
    } else if (getbit(b)) { /* DC refine */
      blk[0] = (int16_t)(blk[0] | (1 << al));
    }
    return;
  }
  if (sc->ah == 0) { /* AC first */
    if (*eobrun) { (*eobrun)--; return; }
    for (int k = sc->ss; k <= sc->se; k++) {
      int rs = hdecode(b, &sc->ac[i]), r = rs >> 4, s = rs & 15;
      if (s) {
        k += r;
        int v = extend(getbits(b, s), s);
        blk[kZigzag[k > 79 ? 79 : k]] = (int16_t)(v << al);
      } else {
        if (r != 15) {
          if (r) *eobrun = (1 << r) + getbits(b, r) - 1;
          break;
        }
        k += 15;
      }
    }
    return;
  }
  /* AC refine */
  const int p1 = 1 << al, m1 = -1 * (1 << al);
  int k = sc->ss;
  if (*eobrun == 0) {
    do {
      int rs = hdecode(b, &sc->ac[i]), r = rs >> 4, s = rs & 15;
      if (s) {
        s = getbit(b) ? p1 : m1;
      } else if (r != 15) {
        *eobrun = 1 << r;
        if (r) *eobrun += getbits(b, r);
        break;
      }
      do {
        int16_t *c = &blk[kZigzag[k > 79 ? 79 : k]];
        if (*c) refine_coef(b, c, p1, m1);
        else if (--r < 0) break;
        k++;
      } while (k <= sc->se);
      if (s) blk[kZigzag[k > 79 ? 79 : k]] = (int16_t)s;
      k++;
    } while (k <= sc->se);
  }
  if (*eobrun) {
    for (; k <= sc->se; k++) {
      int16_t *c = &blk[kZigzag[k]];
      if (*c) refine_coef(b, c, p1, m1);
    }
    (*eobrun)--;
  }
}

static int decode_progressive(const uint8_t *data, const plan *pl, int16_t *out) {
  memset(out, 0, pl->coef_total * sizeof(int16_t));
  const oj_params *p = &pl->p;
  for (int si = 0; si < pl->nscans; si++) {
    const pscan *sc = &pl->scans[si];
    bitrd b;
    memset(&b, 0, sizeof(b));
    b.d = data;
    b.pos = sc->ecs_off;
    b.end = sc->ecs_end;
    int pred[4] = {0, 0, 0, 0}, eobrun = 0, skip = 0;
    const int inter = sc->ns > 1;
    const int c0 = sc->comp[0];
    const long mx_n = inter ? pl->mcux : pl->cwblk[c0];
    const long total = inter ? (long)pl->mcux * pl->mcuy : (long)pl->cwblk[c0] * pl->chblk[c0];
    for (long m = 0; m < total; m++) {
      if (sc->ri && m > 0 && m % sc->ri == 0) {
        skip = !next_restart(&b);
        pred[0] = pred[1] = pred[2] = pred[3] = 0;
        eobrun = 0;
      }
      const long mx = m % mx_n, my = m / mx_n;
      if (!skip) {
        for (int i = 0; i < sc->ns; i++) {
          const int c = sc->comp[i];
          const int hc = inter ? p->comp[c].h : 1, vc = inter ? p->comp[c].v : 1;
          for (int by = 0; by < vc; by++)
            for (int bx = 0; bx < hc; bx++) {
              const long gx = mx * hc + bx, gy = my * vc + by;
              int16_t *blk = out + pl->coef_off[c] + ((size_t)gy * pl->wblk[c] + gx) * 64;
              prog_block(&b, sc, i, blk, &pred[c], &eobrun);
            }
        }
      }
      if (b.insufficient) skip = 1;
    }
  }
  return ST_OK;
}

static void decode_block(bitrd *b, const htab *dc, const htab *ac, int *pred, int16_t *blk, int skip) {
  memset(blk, 0, 64 * sizeof(int16_t));
  if (skip) return;
  int s = hdecode(b, dc);
  int diff = s ? extend(getbits(b, s), s) : 0;
  *pred += diff;
  blk[0] = (int16_t)*pred;
  for (int k = 1; k < 64; k++) {
    int rs = hdecode(b, ac);
    int r = rs >> 4;
    s = rs & 15;
    if (s) {
      k += r;
      int v = extend(getbits(b, s), s);
      blk[kZigzag[k > 79 ? 79 : k]] = (int16_t)v;
    } else {
      if (r != 15) break;
      k += 15;
    }
  }
}

static int decode_all_coefs(const uint8_t *data, const plan *pl, int16_t *out) {
  if (pl->progressive) return decode_progressive(data, pl, out);
  const oj_params *p = &pl->p;
  bitrd b;
  memset(&b, 0, sizeof(b));
  b.d = data;
  b.pos = p->ecs_offset;
  b.end = (size_t)p->ecs_offset + p->ecs_size;
  int pred[4] = {0, 0, 0, 0};
  long total = (long)pl->mcux * pl->mcuy;
  int ri = p->restart_interval;
  int skip = 0;
  for (long m = 0; m < total; m++) {
    if (ri && m > 0 && m % ri == 0) {
      skip = !next_restart(&b);
      pred[0] = pred[1] = pred[2] = pred[3] = 0;
    }
    int mx = (int)(m % pl->mcux), my = (int)(m / pl->mcux);
    for (int c = 0; c < pl->nc; c++) {
      int hc = pl->interleaved ? p->comp[c].h : 1, vc = pl->interleaved ? p->comp[c].v : 1;
      for (int by = 0; by < vc; by++)
        for (int bx = 0; bx < hc; bx++) {
          int gx = mx * hc + bx, gy = my * vc + by;
          int16_t *blk = out + pl->coef_off[c] + ((size_t)gy * pl->wblk[c] + gx) * 64;
          decode_block(&b, &pl->dc[c], &pl->ac[c], &pred[c], blk, skip);
        }
    }
    if (b.insufficient) skip = 1; /* libjpeg: later MCUs of this interval stay zero */
  }
  return ST_OK;
}

int oj_coef_dims(const uint8_t *data, size_t len, int32_t dims[4][2]) {
  plan *pl = malloc(sizeof(plan));
  if (!pl) return ST_OOM;
  int st = make_plan(data, len, pl);
  if (st == ST_OK)
    for (int c = 0; c < 4; c++) {
      dims[c][0] = c < pl->nc ? pl->wblk[c] : 0;
      dims[c][1] = c < pl->nc ? pl->hblk[c] : 0;
    }
  free(pl);
  return st;
}

int oj_decode_coefs(const uint8_t *data, size_t len, int16_t *out) {
  plan *pl = malloc(sizeof(plan));
  if (!pl) return ST_OOM;
  int st = make_plan(data, len, pl);
  if (st == ST_OK) st = decode_all_coefs(data, pl, out);
  free(pl);
  return st;
}

/* ISLOW inverse DCT, restating libjpeg jidctint.c (CONST_BITS 13, PASS1_BITS 2),
 * computed in 64-bit like libjpeg's INT32/JLONG on LP64. */
#define CB 13
#define P1 2
static const long FIX_0_298631336 = 2446, FIX_0_390180644 = 3196, FIX_0_541196100 = 4433,
                  FIX_0_765366865 = 6270, FIX_0_899976223 = 7373, FIX_1_175875602 = 9633,
                  FIX_1_501321110 = 12299, FIX_1_847759065 = 15137, FIX_1_961570560 = 16069,
                  FIX_2_053119869 = 16819, FIX_2_562915447 = 20995, FIX_3_072711026 = 25172;

static uint8_t range_limit(long v) {
  long w = ((v + 512) & 1023) - 512 + 128; /* libjpeg RANGE_MASK wrap, then clamp */
  return (uint8_t)(w < 0 ? 0 : w > 255 ? 255 : w);
}

static void idct_islow(const int16_t *in, const uint16_t *q, uint8_t *out, int ostride) {
  long ws[64];
  for (int c = 0; c < 8; c++) {
    const int16_t *ip = in + c;
    const uint16_t *qp = q + c;
    if (!ip[8] && !ip[16] && !ip[24] && !ip[32] && !ip[40] && !ip[48] && !ip[56]) {
      long dc = ((long)ip[0] * qp[0]) << P1;
      for (int r = 0; r < 8; r++) ws[r * 8 + c] = dc;
      continue;
    }
    long z2 = (long)ip[16] * qp[16], z3 = (long)ip[48] * qp[48];
    long z1 = (z2 + z3) * FIX_0_541196100;
    long tmp2 = z1 - z3 * FIX_1_847759065;
    long tmp3 = z1 + z2 * FIX_0_765366865;
    z2 = (long)ip[0] * qp[0];
    z3 = (long)ip[32] * qp[32];
    long tmp0 = (z2 + z3) << CB, tmp1 = (z2 - z3) << CB;
    long t10 = tmp0 + tmp3, t13 = tmp0 - tmp3, t11 = tmp1 + tmp2, t12 = tmp1 - tmp2;
    tmp0 = (long)ip[56] * qp[56];
    tmp1 = (long)ip[40] * qp[40];
    tmp2 = (long)ip[24] * qp[24];
    tmp3 = (long)ip[8] * qp[8];
    z1 = tmp0 + tmp3;
    z2 = tmp1 + tmp2;
    z3 = tmp0 + tmp2;
    long z4 = tmp1 + tmp3;
    long z5 = (z3 + z4) * FIX_1_175875602;
    tmp0 *= FIX_0_298631336;
    tmp1 *= FIX_2_053119869;
    tmp2 *= FIX_3_072711026;
    tmp3 *= FIX_1_501321110;
    z1 *= -FIX_0_899976223;
    z2 *= -FIX_2_562915447;
    z3 *= -FIX_1_961570560;
    z4 *= -FIX_0_390180644;
    z3 += z5;
    z4 += z5;
    tmp0 += z1 + z3;
    tmp1 += z2 + z4;
    tmp2 += z2 + z3;
    tmp3 += z1 + z4;
    const int sh = CB - P1;
    const long rnd = 1L << (sh - 1);
    ws[0 * 8 + c] = (t10 + tmp3 + rnd) >> sh;
    ws[7 * 8 + c] = (t10 - tmp3 + rnd) >> sh;
    ws[1 * 8 + c] = (t11 + tmp2 + rnd) >> sh;
    ws[6 * 8 + c] = (t11 - tmp2 + rnd) >> sh;
    ws[2 * 8 + c] = (t12 + tmp1 + rnd) >> sh;
    ws[5 * 8 + c] = (t12 - tmp1 + rnd) >> sh;
    ws[3 * 8 + c] = (t13 + tmp0 + rnd) >> sh;
    ws[4 * 8 + c] = (t13 - tmp0 + rnd) >> sh;
  }
  for (int r = 0; r < 8; r++) {
    const long *w = ws + r * 8;
    uint8_t *o = out + (size_t)r * ostride;
    const int sh = CB + P1 + 3;
    const long rnd = 1L << (sh - 1);
    long z2 = w[2], z3 = w[6];
    long z1 = (z2 + z3) * FIX_0_541196100;
    long tmp2 = z1 - z3 * FIX_1_847759065;
    long tmp3 = z1 + z2 * FIX_0_765366865;
    long tmp0 = (w[0] + w[4]) << CB, tmp1 = (w[0] - w[4]) << CB;
    long t10 = tmp0 + tmp3, t13 = tmp0 - tmp3, t11 = tmp1 + tmp2, t12 = tmp1 - tmp2;
    tmp0 = w[7];
    tmp1 = w[5];
    tmp2 = w[3];
    tmp3 = w[1];
    z1 = tmp0 + tmp3;
    z2 = tmp1 + tmp2;
    z3 = tmp0 + tmp2;
    long z4 = tmp1 + tmp3;
    long z5 = (z3 + z4) * FIX_1_175875602;
    tmp0 *= FIX_0_298631336;
    tmp1 *= FIX_2_053119869;
    tmp2 *= FIX_3_072711026;
    tmp3 *= FIX_1_501321110;
    z1 *= -FIX_0_899976223;
    z2 *= -FIX_2_562915447;
    z3 *= -FIX_1_961570560;
    z4 *= -FIX_0_390180644;
    z3 += z5;
    z4 += z5;
    tmp0 += z1 + z3;
    tmp1 += z2 + z4;
    tmp2 += z2 + z3;
    tmp3 += z1 + z4;
    o[0] = range_limit((t10 + tmp3 + rnd) >> sh);
    o[7] = range_limit((t10 - tmp3 + rnd) >> sh);
    o[1] = range_limit((t11 + tmp2 + rnd) >> sh);
    o[6] = range_limit((t11 - tmp2 + rnd) >> sh);
    o[2] = range_limit((t12 + tmp1 + rnd) >> sh);
    o[5] = range_limit((t12 - tmp1 + rnd) >> sh);
    o[3] = range_limit((t13 + tmp0 + rnd) >> sh);
    o[4] = range_limit((t13 - tmp0 + rnd) >> sh);
  }
}

static void planes_from_coefs(const plan *pl, const int16_t *coefs, uint8_t *planes) {
  for (int c = 0; c < pl->nc; c++) {
    int pw = pl->wblk[c] * 8;
    for (int by = 0; by < pl->hblk[c]; by++)
      for (int bx = 0; bx < pl->wblk[c]; bx++)
        idct_islow(coefs + pl->coef_off[c] + ((size_t)by * pl->wblk[c] + bx) * 64, pl->q[c],
                   planes + pl->plane_off[c] + (size_t)by * 8 * pw + bx * 8, pw);
  }
}

int oj_decode_planes(const uint8_t *data, size_t len, uint8_t *out) {
  plan *pl = malloc(sizeof(plan));
  if (!pl) return ST_OOM;
  int st = make_plan(data, len, pl);
  if (st == ST_OK) {
    int16_t *co = malloc(pl->coef_total * sizeof(int16_t));
    if (!co) st = ST_OOM;
    else {
      decode_all_coefs(data, pl, co);
      planes_from_coefs(pl, co, out);
      free(co);
    }
  }
  free(pl);
  return st;
}

/* ---------------------------------------------------------------------------------
 * Colour conversion: src/rocjpeg_hip_kernels.cpp:1431-1443 (identical in every CSC
 * kernel), packing by __builtin_amdgcn_cvt_pk_u8_f32 (:25-30).
 * ------------------------------------------------------------------------------- */
uint8_t oj_cvt_u8(float f) {
  if (!(f == f)) return 0;
  float r = rintf(f); /* default FP mode: round to nearest even */
  if (r < 0.f) return 0;
  if (r > 255.f) return 255;
  return (uint8_t)r;
}

void oj_csc_bulk(const uint8_t *y, const uint8_t *u, const uint8_t *v, size_t n, uint8_t *rgb) {
  for (size_t i = 0; i < n; i++) oj_csc_pixel(y[i], u[i], v[i], rgb + 3 * i);
}

void oj_csc_pixel(uint8_t y, uint8_t u, uint8_t v, uint8_t rgb[3]) {
  float fy = (float)y, fu = (float)u - 128.0f, fv = (float)v - 128.0f;
  rgb[0] = oj_cvt_u8(fmaf(1.5748f, fv, fy));
  rgb[1] = oj_cvt_u8(fmaf(-0.4681f, fv, fmaf(-0.1873f, fu, fy)));
  rgb[2] = oj_cvt_u8(fmaf(1.8556f, fu, fy));
}

/* ---------------------------------------------------------------------------------
 * Output stage: RocJpegDecoder::Decode (src/rocjpeg_decoder.cpp:104-185) over a model
 * of the VCN surface (fourcc per src/rocjpeg_vaapi_decoder.cpp:612-632) whose planes
 * are the decoded component planes.  Reads the reference would make outside the
 * decoded planes are undefined there; here they clamp to the plane edge.
 * ------------------------------------------------------------------------------- */
typedef struct {
  const uint8_t *pl[3];
  int pw[3], ph[3];
} planes_t;

static uint8_t px(const planes_t *P, int c, long r, long x) {
  if (r < 0) r = 0;
  if (x < 0) x = 0;
  if (r >= P->ph[c]) r = P->ph[c] - 1;
  if (x >= P->pw[c]) x = P->pw[c] - 1;
  return P->pl[c][(size_t)r * P->pw[c] + x];
}

/* byte b of row r of surface plane `sp` for the given css (0: luma/packed, 1: chroma) */
static uint8_t surf(const planes_t *P, int css, int sp, int chan, long r, long b) {
  if (css == CSS_422 && sp == 0) { /* YUYV packed */
    long q = b >> 2;
    switch (b & 3) {
      case 0: return px(P, 0, r, 2 * q);
      case 1: return px(P, 1, r, q);
      case 2: return px(P, 0, r, 2 * q + 1);
      default: return px(P, 2, r, q);
    }
  }
  if (css == CSS_420 && sp == 1) /* NV12 interleaved UV */
    return (b & 1) ? px(P, 2, r, b >> 1) : px(P, 1, r, b >> 1);
  return px(P, chan, r, b);
}

int oj_decode(const uint8_t *data, size_t len, int fmt, int16_t cl, int16_t ct, int16_t cr,
              int16_t cbm, uint8_t *ch[4], const uint32_t pitch[4]) {
  if (!ch || !pitch) return ST_INVALID;
  plan *pl = malloc(sizeof(plan));
  if (!pl) return ST_OOM;
  int st = make_plan(data, len, pl);
  const oj_params *p = &pl->p;
  if (st != ST_OK) { free(pl); return st; }
  int W = p->width, H = p->height, css = p->css;
  /* SubmitDecode checks (rocjpeg_vaapi_decoder.cpp:586-592, 612-636) */
  if (W < 64 || H < 64 || W > 16384 || H > 16384) { free(pl); return ST_NOT_SUPPORTED; }
  if (!(css == CSS_444 || css == CSS_440 || css == CSS_422 || css == CSS_420 || css == CSS_400)) {
    free(pl);
    return ST_NOT_SUPPORTED;
  }
  int16_t *co = malloc(pl->coef_total * sizeof(int16_t));
  uint8_t *pb = malloc(pl->plane_total);
  if (!co || !pb) { free(co); free(pb); free(pl); return ST_OOM; }
  decode_all_coefs(data, pl, co);
  planes_from_coefs(pl, co, pb);
  free(co);
  const uint8_t *planes[3] = {0, 0, 0};
  int32_t pw3[3] = {0, 0, 0}, ph3[3] = {0, 0, 0};
  for (int c = 0; c < pl->nc && c < 3; c++) {
    planes[c] = pb + pl->plane_off[c];
    pw3[c] = pl->wblk[c] * 8;
    ph3[c] = pl->hblk[c] * 8;
  }
  st = oj_output_stage(planes, pw3, ph3, css, W, H, fmt, cl, ct, cr, cbm, ch, pitch);
  free(pb);
  free(pl);
  return st;
}

int oj_output_stage(const uint8_t *const planes[3], const int32_t plane_w[3], const int32_t plane_h[3], int css,
                    int W, int H, int fmt, int16_t cl, int16_t ct, int16_t cr, int16_t cbm, uint8_t *ch[4],
                    const uint32_t pitch[4]) {
  if (!ch || !pitch || !planes) return ST_INVALID;
  planes_t P;
  memset(&P, 0, sizeof(P));
  for (int c = 0; c < 3; c++) {
    P.pl[c] = planes[c];
    P.pw[c] = plane_w[c];
    P.ph[c] = plane_h[c];
  }
  /* ROI (rocjpeg_decoder.cpp:124-141); gfx950 VCN has no ROI decode, so offsets apply */
  uint32_t roi_w = (uint32_t)((int)cr - (int)cl), roi_h = (uint32_t)((int)cbm - (int)ct);
  int roi = roi_w > 0 && roi_h > 0 && roi_w <= (uint32_t)W && roi_h <= (uint32_t)H;
  long pw = roi ? (long)roi_w : W, ph = roi ? (long)roi_h : H;
  long top = roi ? ct : 0, left = roi ? cl : 0;

  /* CopyChannel (rocjpeg_decoder.cpp:372-399): dst pitch bytes per row */
  for (int k = 0; k < 3; k++)
    if ((fmt == OUT_YUV_PLANAR || fmt == OUT_RGB_PLANAR || fmt == OUT_RGB || fmt == OUT_Y) &&
        (k == 0 || fmt == OUT_RGB_PLANAR || (fmt == OUT_YUV_PLANAR && css != CSS_400)) && !ch[k]) {
      return ST_INVALID; /* the reference would dereference NULL here */
    }
  #define COPY(SP, CHAN, ROWS, TOPR, LOFF, DI)                                          \
    do {                                                                              \
      if (ch[DI] && pitch[DI])                                                        \
        for (long r_ = 0; r_ < (ROWS); r_++)                                          \
          for (long b_ = 0; b_ < (long)pitch[DI]; b_++)                               \
            ch[DI][(size_t)r_ * pitch[DI] + b_] = surf(&P, css, SP, CHAN, (TOPR) + r_, (LOFF) + b_); \
    } while (0)

  long ctop_nv12 = top >> 1;
  switch (fmt) {
    case OUT_NATIVE:
      if (css == CSS_422) {
        COPY(0, 0, ph, top, 2 * left, 0);
      } else {
        COPY(0, 0, ph, top, left, 0);
        if (css == CSS_420) COPY(1, 1, ph >> 1, ctop_nv12, left, 1);
        if (css == CSS_444) { COPY(1, 1, ph, top, left, 1); COPY(1, 2, ph, top, left, 2); }
        if (css == CSS_440) { COPY(1, 1, ph >> 1, top >> 1, left, 1); COPY(1, 2, ph >> 1, top >> 1, left, 2); }
      }
      break;
    case OUT_YUV_PLANAR:
      if (css == CSS_422) {
        /* ConvertPackedYUYVToPlanarYUV (rocjpeg_hip_kernels.cpp:2186-2245): Y pw, U/V pw>>1 */
        for (long y = 0; y < ph; y++) {
          for (long x = 0; x < pw; x++) ch[0][(size_t)y * pitch[0] + x] = surf(&P, css, 0, 0, top + y, 2 * left + 2 * x);
          for (long x = 0; x < (pw >> 1); x++) {
            ch[1][(size_t)y * pitch[1] + x] = surf(&P, css, 0, 0, top + y, 2 * left + 4 * x + 1);
            ch[2][(size_t)y * pitch[1] + x] = surf(&P, css, 0, 0, top + y, 2 * left + 4 * x + 3);
          }
        }
      } else {
        COPY(0, 0, ph, top, left, 0);
        if (css == CSS_420) { /* ConvertInterleavedUVToPlanarUV (:2082-2134) */
          for (long y = 0; y < (ph >> 1); y++)
            for (long x = 0; x < (pw >> 1); x++) {
              ch[1][(size_t)y * pitch[1] + x] = surf(&P, css, 1, 1, ctop_nv12 + y, left + 2 * x);
              ch[2][(size_t)y * pitch[1] + x] = surf(&P, css, 1, 1, ctop_nv12 + y, left + 2 * x + 1);
            }
        } else if (css == CSS_444) {
          COPY(1, 1, ph, top, left, 1); COPY(1, 2, ph, top, left, 2);
        } else if (css == CSS_440) {
          COPY(1, 1, ph >> 1, top >> 1, left, 1); COPY(1, 2, ph >> 1, top >> 1, left, 2);
        }
      }
      break;
    case OUT_Y:
      if (css == CSS_422) {
        for (long y = 0; y < ph; y++)
          for (long x = 0; x < pw; x++) ch[0][(size_t)y * pitch[0] + x] = px(&P, 0, top + y, left + x);
      } else {
        COPY(0, 0, ph, top, left, 0);
      }
      break;
    case OUT_RGB:
    case OUT_RGB_PLANAR:
      for (long y = 0; y < ph; y++)
        for (long x = 0; x < pw; x++) {
          uint8_t Y = px(&P, 0, top + y, left + x), U = 128, V = 128;
          int gray = 0;
          switch (css) {
            case CSS_444: /* :464-467 -- luma ROI offset is applied twice to chroma */
              U = px(&P, 1, 2 * top + y, 2 * left + x);
              V = px(&P, 2, 2 * top + y, 2 * left + x);
              break;
            case CSS_440: /* :468-471 -- chroma offset commented out; row = top + y/2 */
              U = px(&P, 1, top + (y >> 1), left + x);
              V = px(&P, 2, top + (y >> 1), left + x);
              break;
            case CSS_422: { /* YUYV pairs read from byte 2*left */
              long b = 2 * left + 4 * (x >> 1);
              U = surf(&P, css, 0, 0, top + y, b + 1);
              V = surf(&P, css, 0, 0, top + y, b + 3);
              break;
            }
            case CSS_420: { /* UV plane + (top>>1)*pitch + left */
              long b = left + 2 * (x >> 1);
              U = surf(&P, css, 1, 1, ctop_nv12 + (y >> 1), b);
              V = surf(&P, css, 1, 1, ctop_nv12 + (y >> 1), b + 1);
              break;
            }
            default:
              gray = 1;
              break;
          }
          uint8_t rgb[3];
          if (gray) rgb[0] = rgb[1] = rgb[2] = Y;
          else oj_csc_pixel(Y, U, V, rgb);
          if (fmt == OUT_RGB) {
            uint8_t *o = ch[0] + (size_t)y * pitch[0] + 3 * x;
            o[0] = rgb[0]; o[1] = rgb[1]; o[2] = rgb[2];
          } else { /* planar: every plane uses pitch[0] (:525-544) */
            for (int k = 0; k < 3; k++) ch[k][(size_t)y * pitch[0] + x] = rgb[k];
          }
        }
      break;
    default:
      break;
  }
  #undef COPY
  return ST_OK;
}
