/*
 * libjpeg_golden.c -- TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * Independent golden-vector generator built against IJG libjpeg 9.4 (/opt/conda).
 * The reference (rocJPEG) delegates Huffman decode + dequant + IDCT to the VCN
 * fixed-function engine (src/rocjpeg_vaapi_decoder.cpp:677-689), so there is no
 * reference source for that arithmetic.  Two independent libjpegs (IJG 9.4 here,
 * libjpeg-turbo 3.1.4 inside Pillow) agree bit-for-bit on ISLOW planes, which makes
 * libjpeg's output a well-defined target for the decode core.
 *
 *   libjpeg_golden coef   in.jpg out.bin   -> quantised coefficients (jpeg_read_coefficients)
 *   libjpeg_golden planes in.jpg out.bin   -> native-resolution ISLOW planes (raw_data_out)
 *
 * coef file : "JCOF" i32 ncomp, per comp { i32 h, v, wblk, hblk; int16[wblk*hblk*64] natural order }
 *             (wblk/hblk are the coefficient arrays' dims rounded up to the MCU grid)
 * planes    : "JPLN" i32 ncomp, per comp { i32 h, v, pw, ph, rw, rh; u8[pw*ph] }
 *             pw/ph = plane padded to whole iMCU rows/cols; rw/rh = width_in_blocks*8,
 *             height_in_blocks*8 (libjpeg leaves dummy blocks beyond rw/rh un-IDCT'd: zeroed here)
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <setjmp.h>
#include <jpeglib.h>

struct err_mgr { struct jpeg_error_mgr pub; jmp_buf jb; };
static void on_error(j_common_ptr c) {
  struct err_mgr *e = (struct err_mgr *)c->err;
  (*c->err->output_message)(c);
  longjmp(e->jb, 1);
}

static void put_i32(FILE *f, int v) { fwrite(&v, 4, 1, f); }

static int dump_coef(struct jpeg_decompress_struct *ci, FILE *out) {
  jvirt_barray_ptr *arrs = jpeg_read_coefficients(ci);
  fwrite("JCOF", 1, 4, out);
  put_i32(out, ci->num_components);
  for (int c = 0; c < ci->num_components; c++) {
    jpeg_component_info *cp = &ci->comp_info[c];
    int wb = (int)((cp->width_in_blocks + cp->h_samp_factor - 1) / cp->h_samp_factor) * cp->h_samp_factor;
    int hb = (int)((cp->height_in_blocks + cp->v_samp_factor - 1) / cp->v_samp_factor) * cp->v_samp_factor;
    /* single-component (non-interleaved) scans have no dummy blocks */
    if (ci->num_components == 1) { wb = cp->width_in_blocks; hb = cp->height_in_blocks; }
    put_i32(out, cp->h_samp_factor); put_i32(out, cp->v_samp_factor);
    put_i32(out, wb); put_i32(out, hb);
    for (int by = 0; by < hb; by++) {
      JBLOCKARRAY rows = (*ci->mem->access_virt_barray)((j_common_ptr)ci, arrs[c], by, 1, FALSE);
      for (int bx = 0; bx < wb; bx++) {
        short tmp[64];
        for (int k = 0; k < 64; k++) tmp[k] = rows[0][bx][k];
        fwrite(tmp, 2, 64, out);
      }
    }
  }
  jpeg_finish_decompress(ci);
  return 0;
}

static int dump_planes(struct jpeg_decompress_struct *ci, FILE *out) {
  ci->raw_data_out = TRUE;
  ci->dct_method = JDCT_ISLOW;
  ci->do_fancy_upsampling = FALSE;
  /* progressive streams whose progression is incomplete (truncated): the planes are the
     ISLOW transform of the final coefficients, without libjpeg's block smoothing */
  ci->do_block_smoothing = FALSE;
  jpeg_start_decompress(ci);
  int nc = ci->num_components, vmax = ci->max_v_samp_factor;
  int n_imcu = (int)((ci->output_height + vmax * 8 - 1) / (vmax * 8));
  unsigned char *plane[4]; int pw[4], ph[4];
  for (int c = 0; c < nc; c++) {
    jpeg_component_info *cp = &ci->comp_info[c];
    int hb = (int)((cp->width_in_blocks + cp->h_samp_factor - 1) / cp->h_samp_factor) * cp->h_samp_factor;
    pw[c] = hb * 8 + 64; /* slack: libjpeg may touch whole MCU columns */
    ph[c] = n_imcu * cp->v_samp_factor * 8;
    plane[c] = calloc((size_t)pw[c] * ph[c], 1);
  }
  JSAMPARRAY rowp[4];
  for (int c = 0; c < nc; c++) rowp[c] = malloc(sizeof(JSAMPROW) * ci->comp_info[c].v_samp_factor * 8);
  for (int r = 0; r < n_imcu; r++) {
    for (int c = 0; c < nc; c++) {
      int vs = ci->comp_info[c].v_samp_factor * 8;
      for (int i = 0; i < vs; i++) rowp[c][i] = plane[c] + (size_t)(r * vs + i) * pw[c];
    }
    jpeg_read_raw_data(ci, rowp, vmax * 8);
  }
  fwrite("JPLN", 1, 4, out);
  put_i32(out, nc);
  for (int c = 0; c < nc; c++) {
    jpeg_component_info *cp = &ci->comp_info[c];
    int rw = (int)cp->width_in_blocks * 8, rh = (int)cp->height_in_blocks * 8;
    /* zero everything libjpeg did not IDCT (dummy blocks) so the dump is deterministic */
    for (int y = 0; y < ph[c]; y++)
      for (int x = 0; x < pw[c]; x++)
        if (x >= rw || y >= rh) plane[c][(size_t)y * pw[c] + x] = 0;
    int opw = pw[c] - 64;
    put_i32(out, cp->h_samp_factor); put_i32(out, cp->v_samp_factor);
    put_i32(out, opw); put_i32(out, ph[c]); put_i32(out, rw); put_i32(out, rh);
    for (int y = 0; y < ph[c]; y++) fwrite(plane[c] + (size_t)y * pw[c], 1, opw, out);
    free(plane[c]); free(rowp[c]);
  }
  jpeg_finish_decompress(ci);
  return 0;
}

int main(int argc, char **argv) {
  if (argc != 4) { fprintf(stderr, "usage: %s coef|planes in.jpg out.bin\n", argv[0]); return 2; }
  FILE *in = fopen(argv[2], "rb");
  if (!in) { perror(argv[2]); return 2; }
  FILE *out = fopen(argv[3], "wb");
  if (!out) { perror(argv[3]); return 2; }
  struct jpeg_decompress_struct ci;
  struct err_mgr em;
  ci.err = jpeg_std_error(&em.pub);
  em.pub.error_exit = on_error;
  if (setjmp(em.jb)) { jpeg_destroy_decompress(&ci); return 1; }
  jpeg_create_decompress(&ci);
  jpeg_stdio_src(&ci, in);
  jpeg_read_header(&ci, TRUE);
  int rc = strcmp(argv[1], "coef") == 0 ? dump_coef(&ci, out) : dump_planes(&ci, out);
  jpeg_destroy_decompress(&ci);
  fclose(in); fclose(out);
  return rc;
}
