"""Hand-built JPEG streams for edge cases no encoder emits (test infrastructure).

A minimal marker writer (SOI, DQT, SOF2, DHT, SOS, EOI) and an MSB-first bit writer with
T.81 F.1.2.3 byte stuffing.  Huffman tables are given as {symbol: code length}; codes are
assigned canonically (T.81 Annex C), never the all-ones code of a length (libjpeg's
jpeg_make_d_derived_tbl rejects a table that needs it).
"""
import struct


class BitWriter:
    def __init__(self):
        self.out = bytearray()
        self.acc = 0
        self.n = 0

    def put(self, code, length):
        for i in range(length - 1, -1, -1):
            self.acc = (self.acc << 1) | ((code >> i) & 1)
            self.n += 1
            if self.n == 8:
                self.out.append(self.acc)
                if self.acc == 0xFF:
                    self.out.append(0x00)  # stuffed zero byte
                self.acc, self.n = 0, 0

    def flush(self):
        if self.n:  # pad with one bits (T.81 F.1.2.3)
            self.put((1 << (8 - self.n)) - 1, 8 - self.n)
        return bytes(self.out)


def canonical_codes(lengths):
    """{symbol: length} -> ({symbol: (code, length)}, BITS[16], HUFFVAL list)."""
    by_len = sorted(lengths.items(), key=lambda kv: (kv[1], kv[0]))
    bits = [0] * 16
    for _, ln in by_len:
        bits[ln - 1] += 1
    codes, code, prev = {}, 0, by_len[0][1]
    for sym, ln in by_len:
        code <<= ln - prev
        prev = ln
        assert code < (1 << ln) - 1, "table would need an all-ones code"
        codes[sym] = (code, ln)
        code += 1
    return codes, bits, [s for s, _ in by_len]


def _seg(marker, payload):
    return bytes([0xFF, marker]) + struct.pack(">H", len(payload) + 2) + payload


def dht(tc, th, lengths):
    _, bits, vals = canonical_codes(lengths)
    return _seg(0xC4, bytes([(tc << 4) | th]) + bytes(bits) + bytes(vals))


def dqt(tq, table64):
    return _seg(0xDB, bytes([tq]) + bytes(table64))


def sof2_gray(w, h, tq=0):
    return _seg(0xC2, struct.pack(">BHHB", 8, h, w, 1) + bytes([1, 0x11, tq]))


def sos_gray(td, ta, ss, se, ah, al):
    return _seg(0xDA, bytes([1, 1, (td << 4) | ta, ss, se, (ah << 4) | al]))


def prog_gray_refine_overshoot(w=64, h=64):
    """Grayscale progressive stream whose Se = 63 AC refinement scan has a new coefficient with
    a zero run longer than the zero-history positions left: libjpeg (jdphuff.c
    decode_mcu_AC_refine) leaves the zero-run walk at k = 64 and stores the coefficient at
    jpeg_natural_order[64] == 63.  Every block:
      DC first (Al 0): DC difference 0;
      AC first 1..63, Al 1: coefficient +1 at k = 1, EOB;
      AC refine 1..63, Ah 1 Al 0: (15,1) -> new coefficient at k = 17 (one correction bit for
      k = 1 on the way), ZRL, ZRL (k = 18..49), then (15,1) with 14 zero positions left
      (k = 50..63) -> the overshoot, stored at natural index 63."""
    assert w % 8 == 0 and h % 8 == 0
    nblk = (w // 8) * (h // 8)
    dc_len = {0x00: 1}
    ac1_len = {0x01: 2, 0x00: 2}
    acr_len = {0xF1: 2, 0xF0: 2, 0x00: 2}
    dc_codes = canonical_codes(dc_len)[0]
    ac1_codes = canonical_codes(ac1_len)[0]
    acr_codes = canonical_codes(acr_len)[0]

    bw = BitWriter()
    for _ in range(nblk):
        bw.put(*dc_codes[0x00])
    scan_dc = bw.flush()

    bw = BitWriter()
    for _ in range(nblk):
        bw.put(*ac1_codes[0x01])
        bw.put(1, 1)  # +1 (x 2^Al)
        bw.put(*ac1_codes[0x00])  # EOB
    scan_ac1 = bw.flush()

    bw = BitWriter()
    for b in range(nblk):
        bw.put(*acr_codes[0xF1])
        bw.put(b & 1, 1)  # sign of the new coefficient (1: positive)
        bw.put((b >> 1) & 1, 1)  # correction bit of k = 1 (passed on the walk)
        bw.put(*acr_codes[0xF0])
        bw.put(*acr_codes[0xF0])
        bw.put(*acr_codes[0xF1])
        bw.put((b >> 2) & 1, 1)  # sign of the overshooting coefficient
    scan_acr = bw.flush()

    out = bytearray(b"\xff\xd8")
    out += dqt(0, [1] * 64)
    out += sof2_gray(w, h)
    out += dht(0, 0, dc_len)
    out += sos_gray(0, 0, 0, 0, 0, 0) + scan_dc
    out += dht(1, 0, ac1_len)
    out += sos_gray(0, 0, 1, 63, 0, 1) + scan_ac1
    out += dht(1, 0, acr_len)
    out += sos_gray(0, 0, 1, 63, 1, 0) + scan_acr
    out += b"\xff\xd9"
    return bytes(out)
