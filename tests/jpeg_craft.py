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


ZIGZAG_NAT = [0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34, 27, 20,
              13, 6, 7, 14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52,
              45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63]  # natural index of zigzag position k


def _magnitude(v):
    """(size category, extra bits) of a coefficient value (T.81 F.1.2.1)."""
    v = int(v)
    s = abs(v).bit_length()
    return s, (v if v >= 0 else v + (1 << s) - 1) & ((1 << s) - 1)


def baseline_symbols(blocks):
    """DC size categories and AC run/size symbols a block list (natural order, int) uses."""
    dcs, acs, pred = set(), set(), 0
    for blk in blocks:
        dcs.add(_magnitude(blk[0] - pred)[0])
        pred = blk[0]
        run = 0
        for k in range(1, 64):
            v = blk[ZIGZAG_NAT[k]]
            if v == 0:
                run += 1
                continue
            while run > 15:
                acs.add(0xF0)
                run -= 16
            acs.add((run << 4) | _magnitude(v)[0])
            run = 0
        if run:
            acs.add(0x00)
    return dcs, acs


def baseline_420(w, h, coefs, dims, qz, dc_len, ac_len, comp_tables):
    """Baseline interleaved 3-component JPEG (Y 2x2, Cb / Cr 1x1, no DRI) from quantised
    coefficients in natural order (tests/oracle_lib.decode_coefs layout: per component a raster
    of blocks).  qz: two quant tables in zigzag order (Y, chroma); dc_len / ac_len: two tables
    each ({symbol: code length}); comp_tables: per component (td, ta)."""
    codes_dc = [canonical_codes(t)[0] for t in dc_len]
    codes_ac = [canonical_codes(t)[0] for t in ac_len]
    comps, off = [], 0
    for (bw_, bh_) in dims:
        comps.append(coefs[off:off + bw_ * bh_ * 64].reshape(bh_, bw_, 64))
        off += bw_ * bh_ * 64
    mcux, mcuy = (w + 15) // 16, (h + 15) // 16
    bw = BitWriter()
    pred = [0, 0, 0]

    def block(c, blk):
        td, ta = comp_tables[c]
        d = int(blk[0]) - pred[c]
        pred[c] = int(blk[0])
        s, e = _magnitude(d)
        bw.put(*codes_dc[td][s])
        if s:
            bw.put(e, s)
        run = 0
        for k in range(1, 64):
            v = int(blk[ZIGZAG_NAT[k]])
            if v == 0:
                run += 1
                continue
            while run > 15:
                bw.put(*codes_ac[ta][0xF0])
                run -= 16
            s, e = _magnitude(v)
            bw.put(*codes_ac[ta][(run << 4) | s])
            bw.put(e, s)
            run = 0
        if run:
            bw.put(*codes_ac[ta][0x00])

    for my in range(mcuy):
        for mx in range(mcux):
            for by in range(2):
                for bx in range(2):
                    block(0, comps[0][2 * my + by, 2 * mx + bx])
            block(1, comps[1][my, mx])
            block(2, comps[2][my, mx])
    ecs = bw.flush()
    out = bytearray(b"\xff\xd8")
    out += dqt(0, qz[0]) + dqt(1, qz[1])
    out += _seg(0xC0, struct.pack(">BHHB", 8, h, w, 3) + bytes([1, 0x22, 0, 2, 0x11, 1, 3, 0x11, 1]))
    for t in range(2):
        out += dht(0, t, dc_len[t]) + dht(1, t, ac_len[t])
    sos = bytes([3])
    for c in range(3):
        td, ta = comp_tables[c]
        sos += bytes([c + 1, (td << 4) | ta])
    out += _seg(0xDA, sos + bytes([0, 63, 0])) + ecs
    out += b"\xff\xd9"
    return bytes(out)
