"""The lean K1's two-symbol step (rj_huff.hip RJ_HL_STEP, tables rj_device.h RjLeanTables, built by
rj_stream.cpp AddLeanPairs) restated in Python over the library's own table image
(rocJpegAmdStreamGetLeanTables), and run on every restart interval of clean baseline fixtures:
the entries and the bit position at every block end must equal those of one symbol per step
(the decode the GPU suite pins to the oracle).  This checks on the CPU that a second symbol is
only ever taken where a one-symbol decoder would decode exactly that symbol next.  (No GPU.)"""
import ctypes

import numpy as np
import pytest

import rocjpeg_amd as R
from tests import oracle_lib as O

AC_BITS, DC_BITS, SUBS = 11, 9, 8
AC_WORDS = (1 << AC_BITS) + SUBS * 32
ESC, PAIR = 0x80000000, 0x8000

NAMES = ["p420_q90_ri_256x128", "p420_opt_ri_176x144", "p444_q95_ri_128x128", "p420_q100_ri_128x64",
         "p422_q90_ri_192x96", "p400_q85_ri_96x72", "c420_q88_ri5b_144x80", "p420_q10_160x96",
         "p420_q75_nori_200x150", "c440_q90_160x120"]


def lean_tables(stream):
    need = ctypes.c_size_t()
    L = R.lib()
    assert L.rocJpegAmdStreamGetLeanTables(stream.handle, None, 0, ctypes.byref(need)) == 0
    buf = np.zeros(need.value // 4, np.uint32)
    assert L.rocJpegAmdStreamGetLeanTables(stream.handle, buf.ctypes.data, need.value, ctypes.byref(need)) == 0
    ac = [buf[i * AC_WORDS:(i + 1) * AC_WORDS] for i in range(2)]
    d0 = 2 * AC_WORDS
    dc = [buf[d0 + i * (1 << DC_BITS):d0 + (i + 1) * (1 << DC_BITS)] for i in range(2)]
    return ac, dc


def parse_headers(data):
    """DHT specs, SOF components, SOS table selectors and the ECS start (host-side, for the model)."""
    pos, dht, comps, sos_sel, ecs0 = 2, {}, [], [], None
    while pos < len(data):
        while data[pos] == 0xFF:
            pos += 1
        m = data[pos]
        ln = (data[pos + 1] << 8) | data[pos + 2]
        seg = data[pos + 3:pos + 1 + ln]
        if m == 0xC4:
            q = 0
            while q < len(seg):
                tc, th = seg[q] >> 4, seg[q] & 15
                bits = list(seg[q + 1:q + 17])
                vals = list(seg[q + 17:q + 17 + sum(bits)])
                dht[(tc, th)] = (bits, vals)
                q += 17 + sum(bits)
        elif m == 0xC0:
            nc = seg[5]
            comps = [(seg[6 + 3 * i], seg[7 + 3 * i] >> 4, seg[7 + 3 * i] & 15) for i in range(nc)]
        elif m == 0xDA:
            ns = seg[0]
            sos_sel = [(seg[1 + 2 * i], seg[2 + 2 * i] >> 4, seg[2 + 2 * i] & 15) for i in range(ns)]
            ecs0 = pos + 1 + ln
            break
        pos += 1 + ln
    return dht, comps, sos_sel, ecs0


def canonical(bits, vals, peek16):
    code, k = 0, 0
    for ln in range(1, 17):
        for _ in range(bits[ln - 1]):
            if (peek16 >> (16 - ln)) == code:
                return ln, vals[k]
            code += 1
            k += 1
        code <<= 1
    return 17, 0


def destuff(raw):
    out, i = bytearray(), 0
    while i < len(raw):
        b = raw[i]
        if b == 0xFF and i + 1 < len(raw) and raw[i + 1] == 0x00:
            out.append(0xFF)
            i += 2
        elif b == 0xFF and i + 1 < len(raw) and raw[i + 1] == 0xFF:
            i += 1  # fill byte
        else:
            out.append(b)
            i += 1
    return bytes(out)


def decode(data, blocks, nblk, blk_tabs, ac, dc, dht, pairs):
    """Entries and block-end bit positions of one interval's destuffed bytes (the kernel's step
    semantics; `pairs`: take second symbols)."""
    bitlen = len(data) * 8
    big = int.from_bytes(data + b"\0" * 8, "big")
    total = (len(data) + 8) * 8

    def peek(pos):
        if pos >= bitlen:
            return 0
        return (big >> (total - pos - 32)) & 0xFFFFFFFF

    pos, k, b, done = 0, 0, 0, 0
    ents, ends = [], []
    while done < blocks:
        td, ta = blk_tabs[b]
        p = peek(pos)
        if k == 0:
            e = int(dc[td][p >> (32 - DC_BITS)])
        else:
            e = int(ac[ta][p >> (32 - AC_BITS)])
        if e & ESC:
            sub = e & 0xFF
            if k != 0 and sub < SUBS:
                e = int(ac[ta][(1 << AC_BITS) + sub * 32 + ((p >> (32 - AC_BITS - 5)) & 31)])
            else:
                bits, vals = dht[(0, td)] if k == 0 else dht[(1, ta)]
                ln, sym = canonical(bits, vals, p >> 16)
                s, r = sym & 15, sym >> 4
                R_ = 0 if k == 0 else (r if s else (15 if r == 15 else 63))
                e = ((ln + s) << 16) | (s << 21) | (R_ << 25)
        n1, s1, R1 = (e >> 16) & 31, (e >> 21) & 15, (e >> 25) & 63
        n2, s2, R2 = e & 31, (e >> 5) & 15, (e >> 9) & 63
        k1 = k + R1 + 1
        use2 = pairs and (e & PAIR) != 0 and k1 < 64

        def ent(shift, s, kpos):
            raw = (p >> shift) if shift < 32 else 0
            xm = (1 << s) - 1
            xb = raw & xm
            xv = xb if xb > xm - xb else (xb - xm) & 0xFFFFFFFF
            return (xv & 0xFFFF) | (min(kpos, 63) << 16)

        if k == 0 or s1 != 0:
            ents.append(ent(32 - n1, s1, k + R1))
        if use2 and s2 != 0:
            ents.append(ent((32 - n1 - n2) & 31, s2, k1 + R2))
        pos += n1 + (n2 if use2 else 0)
        kn = k1 + R2 + 1 if use2 else k1
        if kn >= 64:
            k, b, done = 0, (b + 1) % nblk, done + 1
            ends.append(pos)
        else:
            k = kn
    return ents, ends


@pytest.mark.parametrize("name", NAMES)
def test_two_symbol_steps_equal_one_symbol_steps(name):
    ent = next(f for f in O.manifest() if f["name"] == name)
    data = O.fixture_bytes(ent)
    s = R.JpegStream(data)
    ac, dc = lean_tables(s)
    npair = sum(int(((t[:1 << AC_BITS] & PAIR) != 0).sum()) for t in ac)
    assert npair > 0, "no two-symbol entries built"
    assert sum(int(((t & PAIR) != 0).sum()) for t in dc) > 0, "no DC + AC entries built"
    dht, comps, sel, ecs0 = parse_headers(data)
    hmax = max(c[1] for c in comps)
    vmax = max(c[2] for c in comps)
    blk_tabs = []
    for ci, (cid, h, v) in enumerate(comps):
        td, ta = next((t_d, t_a) for (c, t_d, t_a) in sel if c == cid)
        blk_tabs += [(td, ta)] * (h * v if len(comps) > 1 else 1)
    nblk = len(blk_tabs)
    keys = [k for k, _ in R.RocJpegAmdInterval._fields_]
    ivs = [dict(zip(keys, t)) for t in s.intervals()]
    taken = 0
    for iv in ivs:
        raw = data[ecs0 + iv["src_off"]:ecs0 + iv["src_off"] + iv["src_len"]]
        ds = destuff(raw)
        blocks = iv["mcu_count"] * nblk
        e1, b1 = decode(ds, blocks, nblk, blk_tabs, ac, dc, dht, pairs=False)
        e2, b2 = decode(ds, blocks, nblk, blk_tabs, ac, dc, dht, pairs=True)
        assert e1 == e2 and b1 == b2, (iv, len(e1), len(e2))
        taken += len(e1)
    assert taken > 0
    del hmax, vmax
