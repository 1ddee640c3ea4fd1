// Host-only harness for the Huffman table builders (rj_stream.cpp), built with AddressSanitizer
// by tests/test_abi_cpu.py::test_oversubscribed_tables_are_refused_without_writes.  No GPU call:
// the file given on the command line is parsed with rj::Stream::Parse and its lean K1 tables
// are built (Stream::LeanTables), which is where a crafted DHT used to write out of bounds.
// Exit 0 and one line "status=<plan status> valid=<slot0><slot1>" on success.
#include <cstdio>
#include <cstring>
#include <vector>

#include "rj_stream.h"

int main(int argc, char **argv) {
  if (argc < 2) return 2;
  FILE *f = std::fopen(argv[1], "rb");
  if (!f) return 2;
  std::vector<uint8_t> d;
  uint8_t buf[65536];
  size_t got;
  while ((got = std::fread(buf, 1, sizeof(buf), f)) > 0) d.insert(d.end(), buf, buf + got);
  std::fclose(f);
  rj::Stream s;
  if (!s.Parse(d.data(), uint32_t(d.size()))) {
    std::printf("parse=fail\n");
    return 0;
  }
  const RjLeanTables *t = s.LeanTables();
  uint64_t sum = 0;  // touch every entry so ASan sees the whole allocation read
  for (size_t i = 0; i < sizeof(RjLeanTables) / 4; i++) sum += reinterpret_cast<const uint32_t *>(t)[i];
  // the direct builders too, on the raw DHT bits of every slot
  for (int id = 0; id < 2; id++) {
    RjHuffDev h;
    uint32_t first[1 << RJ_HL_AC_BITS], subs[RJ_HL_SUBS * 32];
    (void)rj::BuildHuffman(s.info().ht[id].ac_bits, s.info().ht[id].ac_vals, false, &h);
    (void)rj::BuildLeanTable(s.info().ht[id].ac_bits, s.info().ht[id].ac_vals, false, first, subs);
    uint32_t dfirst[1 << RJ_HL_DC_BITS];
    (void)rj::BuildHuffman(s.info().ht[id].dc_bits, s.info().ht[id].dc_vals, true, &h);
    (void)rj::BuildLeanTable(s.info().ht[id].dc_bits, s.info().ht[id].dc_vals, true, dfirst, nullptr);
  }
  std::printf("status=%d valid=%d%d sum=%llu\n", s.plan().status, s.plan().ht_valid[0], s.plan().ht_valid[1],
              (unsigned long long)sum);
  return 0;
}
