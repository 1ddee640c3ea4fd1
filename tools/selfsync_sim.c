/*
 * selfsync_sim.c -- CPU simulation of the wave-cooperative self-synchronising Huffman decode
 * (K1 in rj_kernels.hip): 64 "lanes" per restart interval, each speculatively decoding a
 * 1/64 chunk from a guessed state, then re-decoding from its left neighbour's end state until
 * every lane's end state is stable.  Checks the coefficients against the oracle and prints
 * how many rounds the intervals needed.  Development tool only.
 *
 *   gcc -O2 -o /tmp/sss tools/selfsync_sim.c oracle/jpeg_oracle.c -Ioracle -lm && /tmp/sss f.jpg ...
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "jpeg_oracle.h"

static const uint8_t ZZ[80] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33,
    40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36,
    29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54,
    47, 55, 62, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

typedef struct { int32_t maxcode[18], valoff[18]; uint8_t vals[256]; } htab;

static void build(const uint8_t bits[16], const uint8_t *vals, htab *t) {
  int k = 0, code = 0;
  for (int l = 1; l <= 16; l++) {
    int nb = bits[l - 1];
    t->valoff[l] = k - code;
    code += nb; k += nb;
    t->maxcode[l] = nb ? code - 1 : -1;
    code <<= 1;
  }
  memcpy(t->vals, vals, k);
}

typedef struct { const uint8_t *d; long nbits; } bits_t;
static int bit(const bits_t *s, long p) { return p < s->nbits ? (s->d[p >> 3] >> (7 - (p & 7))) & 1 : 0; }
static int getn(const bits_t *s, long *p, int n) { int v = 0; for (int i = 0; i < n; i++) v = (v << 1) | bit(s, (*p)++); return v; }
static int hdec(const bits_t *s, long *p, const htab *t) {
  int code = bit(s, (*p)++), l = 1;
  while (l <= 16 && code > t->maxcode[l]) { code = (code << 1) | bit(s, (*p)++); l++; }
  return l > 16 ? 0 : t->vals[(code + t->valoff[l]) & 255];
}
static int ext(int v, int s) { return (s && v < (1 << (s - 1))) ? v - (1 << s) + 1 : v; }

typedef struct { int nblk; int comp[10]; htab dc[3], ac[3]; } geo_t;

/* decode one block starting at *p (block-in-MCU b); returns DC diff; writes coefs if out */
static int dec_block(const bits_t *s, long *p, const geo_t *g, int b, int16_t *out) {
  int c = g->comp[b];
  int sdc = hdec(s, p, &g->dc[c]) & 15;
  int diff = sdc ? ext(getn(s, p, sdc), sdc) : 0;
  if (out) memset(out, 0, 128);
  for (int k = 1; k < 64; k++) {
    int rs = hdec(s, p, &g->ac[c]), r = rs >> 4, sz = rs & 15;
    if (sz) { k += r; int v = ext(getn(s, p, sz), sz); if (out) out[ZZ[k > 79 ? 79 : k]] = (int16_t)v; }
    else { if (r != 15) break; k += 15; }
  }
  return diff;
}

typedef struct { long p; int b; } st_t;

int main(int argc, char **argv) {
  int hist[70] = {0};
  const long chunk_target = getenv("CHUNK") ? atol(getenv("CHUNK")) : 0;
  long nint = 0, bad = 0;
  for (int a = 1; a < argc; a++) {
    FILE *f = fopen(argv[a], "rb"); fseek(f, 0, SEEK_END); long n = ftell(f); fseek(f, 0, SEEK_SET);
    uint8_t *d = malloc(n); fread(d, 1, n, f); fclose(f);
    oj_params P; if (!oj_parse(d, n, &P)) { printf("%s: parse fail\n", argv[a]); continue; }
    geo_t g; memset(&g, 0, sizeof g);
    int nc = P.ncomp, hmax = 1, vmax = 1;
    for (int c = 0; c < nc; c++) { if (P.comp[c].h > hmax) hmax = P.comp[c].h; if (P.comp[c].v > vmax) vmax = P.comp[c].v; }
    for (int c = 0; c < nc; c++) {
      build(P.ht[P.scomp[c].td].dc_bits, P.ht[P.scomp[c].td].dc_vals, &g.dc[c]);
      build(P.ht[P.scomp[c].ta].ac_bits, P.ht[P.scomp[c].ta].ac_vals, &g.ac[c]);
      for (int i = 0; i < (nc > 1 ? P.comp[c].h * P.comp[c].v : 1); i++) g.comp[g.nblk++] = c;
    }
    long mcux = nc > 1 ? (P.width + 8 * hmax - 1) / (8 * hmax) : (P.width + 7) / 8;
    long mcuy = nc > 1 ? (P.height + 8 * vmax - 1) / (8 * vmax) : (P.height + 7) / 8;
    long total = mcux * mcuy, ri = P.restart_interval ? P.restart_interval : total;
    /* oracle coefficients in MCU-major order for comparison */
    int32_t dims[4][2]; oj_coef_dims(d, n, dims);
    long ctot = 0; for (int c = 0; c < nc; c++) ctot += (long)dims[c][0] * dims[c][1] * 64;
    int16_t *oc = malloc(ctot * 2); oj_decode_coefs(d, n, oc);
    /* split + destuff */
    const uint8_t *e = d + P.ecs_offset; long en = P.ecs_size, i = 0, start = 0; long seg = 0;
    uint8_t *buf = malloc(en + 64);
    long mcu0 = 0;
    while (start <= en && mcu0 < total) {
      long end = start; while (end + 1 < en && !(e[end] == 0xFF && e[end + 1] >= 0xD0 && e[end + 1] <= 0xD7)) end++;
      if (end + 1 >= en) end = en;
      long m = 0; for (long q = start; q < end; q++) { if (e[q] == 0x00 && q > start && e[q - 1] == 0xFF) continue; buf[m++] = e[q]; }
      bits_t s = {buf, m * 8};
      long nmcu = total - mcu0 < ri ? total - mcu0 : ri, nb = nmcu * g.nblk;
      /* --- the algorithm --- */
      int L = 64;
      if (chunk_target) { L = 1; while (L < 64 && (long)L * 2 * chunk_target <= m) L *= 2; }
      long cw = (m + 4 * L - 1) / (4 * L); /* words per lane */
      st_t E[64], Eprev[64]; long nblocks[64]; int dcs[64][3];
      for (int j = 0; j < L; j++) {
        long s0 = j * cw * 32, e0 = (j + 1) * cw * 32;
        st_t x = {s0, 0};
        if (s0 < s.nbits) while (x.p < e0) { long pp = x.p; dec_block(&s, &pp, &g, x.b, NULL); x.p = pp; x.b = (x.b + 1) % g.nblk; }
        E[j] = x;
      }
      int rounds = 0;
      for (;;) {
        memcpy(Eprev, E, sizeof E);
        rounds++;
        int stable = 1;
        for (int j = 0; j < L; j++) {
          st_t x = j ? Eprev[j - 1] : (st_t){0, 0};
          long e0 = (j + 1) * cw * 32; nblocks[j] = 0; dcs[j][0] = dcs[j][1] = dcs[j][2] = 0;
          while (x.p < e0 && x.p < s.nbits + 64) { long pp = x.p; int df = dec_block(&s, &pp, &g, x.b, NULL); dcs[j][g.comp[x.b]] += df; x.p = pp; x.b = (x.b + 1) % g.nblk; nblocks[j]++; }
          E[j] = x;
          if (j < L - 1 && (E[j].p != Eprev[j].p || E[j].b != Eprev[j].b)) stable = 0;
        }
        if (stable || rounds > 65) break;
      }
      hist[rounds < 69 ? rounds : 69]++;
      nint++;
      /* output pass + compare */
      long B = 0; int pred[3] = {0, 0, 0};
      int16_t blk[64];
      for (int j = 0; j < L; j++) {
        st_t x = j ? E[j - 1] : (st_t){0, 0};
        long e0 = j == L - 1 ? (1L << 40) : (j + 1) * cw * 32;
        while (x.p < e0 && B < nb) {
          long pp = x.p; int c = g.comp[x.b];
          int df = dec_block(&s, &pp, &g, x.b, blk); pred[c] += df; blk[0] = (int16_t)pred[c];
          /* locate the oracle block */
          long mcu = mcu0 + B / g.nblk; int b = (int)(B % g.nblk);
          long mx = mcu % mcux, my = mcu / mcux;
          int cc = g.comp[b], bi = 0; for (int q = 0; q < b; q++) if (g.comp[q] == cc) bi++;
          int hc = nc > 1 ? P.comp[cc].h : 1, vc = nc > 1 ? P.comp[cc].v : 1;
          long gx = mx * hc + bi % hc, gy = my * vc + bi / hc;
          long off = 0; for (int q = 0; q < cc; q++) off += (long)dims[q][0] * dims[q][1] * 64;
          if (memcmp(blk, oc + off + (gy * dims[cc][0] + gx) * 64, 128)) bad++;
          x.p = pp; x.b = (x.b + 1) % g.nblk; B++;
        }
      }
      if (B != nb) { bad++; printf("interval %ld: %ld of %ld blocks\n", seg, B, nb); }
      mcu0 += nmcu; seg++;
      start = end + 2;
    }
    free(buf); free(oc); free(d);
  }
  printf("intervals %ld, bad blocks %ld; rounds histogram:", nint, bad);
  for (int r = 0; r < 70; r++) if (hist[r]) printf(" %d:%d", r, hist[r]);
  printf("\n");
  return 0;
}
