// CPU check of the chunk-lane layout with MCU-phase hypotheses (rj_device.h rj_chunk_lanes /
// rj_chunk_lane, the inverse k_huff_chunk and k_resolve use): every (chunk, hypothesis) of an
// interval has its own lane offset in [0, lanes), chunk 0 is the last lane, chunks are in
// reverse order, and the kernels' inverse (o -> c, h) returns the pair.  Built by
// tests/test_chunk_lanes_cpu.py.
#include <cstdio>
#include <vector>

#include "rj_device.h"

int main() {
  int bad = 0;
  for (uint32_t nch = 1; nch <= 300; nch++)
    for (uint32_t H = 1; H <= RJ_MAX_HYP; H++) {
      const uint32_t lanes = rj_chunk_lanes(nch, H);
      std::vector<int> seen(lanes, 0);
      for (uint32_t c = 0; c < nch; c++)
        for (uint32_t h = 0; h < (c ? H : 1u); h++) {
          const uint32_t o = rj_chunk_lane(nch, H, c, h);
          if (o >= lanes || seen[o]++) { bad++; continue; }
          // k_huff_chunk's inverse
          uint32_t ci = 0, hi = 0;
          if (nch > 1 && o < (nch - 1) * H) {
            ci = nch - 1 - o / H;
            hi = o - (o / H) * H;
          }
          if (ci != c || hi != h) bad++;
          // reverse order: a later chunk's lanes come before an earlier chunk's
          if (c + 1 < nch && rj_chunk_lane(nch, H, c + 1, 0) >= rj_chunk_lane(nch, H, c, 0)) bad++;
        }
      for (uint32_t o = 0; o < lanes; o++)
        if (!seen[o]) bad++;
      if (rj_chunk_lane(nch, H, 0, 0) != lanes - 1) bad++;
    }
  std::printf("%s %d\n", bad ? "FAIL" : "OK", bad);
  return bad ? 1 : 0;
}
