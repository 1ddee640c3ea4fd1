// TEST INFRASTRUCTURE ONLY.  Exposes the reference's own RocJpegStreamParser
// (src/rocjpeg_parser.cpp, compiled from /root/reference by oracle/build_ref.sh into
// oracle/_ref/) through a flat C struct so tests can pin oracle/jpeg_oracle.c's
// parser restatement -- and the product parser -- against the real reference code.
#include <cstdint>
#include <cstring>
#include "rocjpeg_parser.h"

extern "C" {
struct ref_parse_out {
  int ok;
  uint16_t width, height;
  uint8_t ncomp, scan_ncomp;
  uint8_t comp_id[4], comp_h[4], comp_v[4], comp_tq[4];
  uint8_t qt_loaded[4], qt[4][64];
  uint8_t ht_loaded[2], dc_bits[2][16], dc_vals[2][12], ac_bits[2][16], ac_vals[2][162];
  uint8_t scan_cs[4], scan_td[4], scan_ta[4];
  uint16_t restart_interval;
  uint32_t num_mcus, slice_data_size;
  int64_t slice_data_offset;  // slice_data_buffer - data
  int css;
};

int ref_parse(const uint8_t *data, size_t len, ref_parse_out *o) {
  std::memset(o, 0, sizeof(*o));
  RocJpegStreamParser parser;
  o->ok = parser.ParseJpegStream(data, (uint32_t)len) ? 1 : 0;
  const JpegStreamParameters *p = parser.GetJpegStreamParameters();
  const auto &pic = p->picture_parameter_buffer;
  o->width = pic.picture_width; o->height = pic.picture_height; o->ncomp = pic.num_components;
  for (int i = 0; i < 4; i++) {
    o->comp_id[i] = pic.components[i].component_id; o->comp_h[i] = pic.components[i].h_sampling_factor;
    o->comp_v[i] = pic.components[i].v_sampling_factor; o->comp_tq[i] = pic.components[i].quantiser_table_selector;
    o->qt_loaded[i] = p->quantization_matrix_buffer.load_quantiser_table[i];
    std::memcpy(o->qt[i], p->quantization_matrix_buffer.quantiser_table[i], 64);
    o->scan_cs[i] = p->slice_parameter_buffer.components[i].component_selector;
    o->scan_td[i] = p->slice_parameter_buffer.components[i].dc_table_selector;
    o->scan_ta[i] = p->slice_parameter_buffer.components[i].ac_table_selector;
  }
  for (int t = 0; t < 2; t++) {
    const auto &h = p->huffman_table_buffer.huffman_table[t];
    o->ht_loaded[t] = p->huffman_table_buffer.load_huffman_table[t];
    std::memcpy(o->dc_bits[t], h.num_dc_codes, 16); std::memcpy(o->dc_vals[t], h.dc_values, 12);
    std::memcpy(o->ac_bits[t], h.num_ac_codes, 16); std::memcpy(o->ac_vals[t], h.ac_values, 162);
  }
  o->scan_ncomp = p->slice_parameter_buffer.num_components;
  o->restart_interval = p->slice_parameter_buffer.restart_interval;
  o->num_mcus = p->slice_parameter_buffer.num_mcus;
  o->slice_data_size = p->slice_parameter_buffer.slice_data_size;
  o->slice_data_offset = p->slice_data_buffer ? (int64_t)(p->slice_data_buffer - data) : -1;
  o->css = (int)p->chroma_subsampling;
  return o->ok;
}
}
