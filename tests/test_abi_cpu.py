"""C-ABI checks that need no GPU: the library loads, exports exactly what include/*.h
declares, and the host parser behind rocJpegStreamParse agrees with the reference parser
(src/rocjpeg_parser.cpp, recorded per fixture in tests/golden/manifest.json)."""
import ctypes
import os
import re

import pytest

import rocjpeg_amd as R
from tests import oracle_lib as O

INCLUDE = os.path.join(O.ROOT, "include")


def declared_functions():
    names = set()
    for h in ("rocjpeg.h", "rocjpeg_amd.h"):
        src = open(os.path.join(INCLUDE, h)).read()
        names |= set(re.findall(r"\b(rocJpeg\w+)\s*\(", src))
    return names


def test_library_exports_every_declared_symbol():
    L = R.lib()
    declared = declared_functions()
    assert set(R.API_SYMBOLS) <= declared
    for name in declared:
        assert hasattr(L, name), name


def test_error_names_match_reference_strings():
    # rocjpeg_api.cpp:246-277
    for st in R.Status:
        assert R.error_name(st) == "ROCJPEG_STATUS_" + st.name
    assert R.error_name(-99) == "UNKNOWN_ERROR"


def test_null_arguments_are_invalid_parameter():
    L = R.lib()
    assert L.rocJpegStreamCreate(None) == R.Status.INVALID_PARAMETER
    assert L.rocJpegStreamParse(None, 0, None) == R.Status.INVALID_PARAMETER
    assert L.rocJpegStreamDestroy(None) == R.Status.INVALID_PARAMETER
    assert L.rocJpegCreate(0, 0, None) == R.Status.INVALID_PARAMETER
    assert L.rocJpegDestroy(None) == R.Status.INVALID_PARAMETER
    assert L.rocJpegDecode(None, None, None, None) == R.Status.INVALID_PARAMETER
    assert L.rocJpegDecodeBatched(None, None, 0, None, None) == R.Status.INVALID_PARAMETER
    assert L.rocJpegGetImageInfo(None, None, None, None, None, None) == R.Status.INVALID_PARAMETER


@pytest.mark.parametrize("ent", O.manifest(), ids=[f["name"] for f in O.manifest()])
def test_stream_parse_matches_reference_parser(ent):
    data = O.fixture_bytes(ent)
    s = R.JpegStream()
    st = s.try_parse(data)
    ref = ent["ref_parse"]
    if _sof2(data):
        # deliberate extension: the reference parser rejects SOF2 (rocjpeg_parser.cpp:74-104,
        # it records zeros); this one parses it and reports the frame header
        assert st == R.Status.SUCCESS
        fi = O.frame_info(data)
        info = s.info()
        assert (info["widths"][0], info["heights"][0], info["num_components"]) == (fi["width"], fi["height"], fi["ncomp"])
        return
    assert (st == R.Status.SUCCESS) == bool(ref["ok"])
    if st != R.Status.SUCCESS:
        assert st == R.Status.BAD_JPEG
        return
    info = s.info()
    assert info["num_components"] == ref["ncomp"]
    assert info["subsampling"] == ref["css"]
    w, h = ref["width"], ref["height"]
    assert info["widths"][0] == w and info["heights"][0] == h
    css = ref["css"]
    expect_w1 = {0: w, 1: w, 2: w >> 1, 3: w >> 1, 4: w >> 2, 5: 0}.get(css, None)
    expect_h1 = {0: h, 1: h >> 1, 2: h, 3: h >> 1, 4: h, 5: 0}.get(css, None)
    if expect_w1 is not None:  # GetImageInfo, rocjpeg_decoder.cpp:321-355
        assert info["widths"][1:3] == [expect_w1] * 2 and info["heights"][1:3] == [expect_h1] * 2
    ri = ref["restart_interval"]
    if ri and "libjpeg_coef_sha256" in ent:
        assert info["restart_intervals"] == -(-ref["num_mcus"] // ri)


def _sof2(data):
    pos = 2
    while pos + 4 <= len(data):
        while data[pos] == 0xFF:
            pos += 1
        if data[pos] == 0xC2:
            return True
        if data[pos] in (0xC0, 0xC1, 0xDA):
            return False
        pos += 1 + ((data[pos + 1] << 8) | data[pos + 2])
    return False


def test_progressive_parse_errors():
    """SOF2 streams: the marker walk's error rules (oracle make_plan_prog / libjpeg jdmarker.c)."""
    good = O.fixture_bytes(next(f for f in O.manifest() if f["name"] == "pp420_opt_200x150"))
    s = R.JpegStream()
    assert s.try_parse(good) == R.Status.SUCCESS
    # a scan naming a component the frame does not have
    i = good.index(b"\xff\xda")
    bad = bytearray(good)
    bad[i + 5] = 0x77
    assert s.try_parse(bytes(bad)) == R.Status.BAD_JPEG
    # header cut before any scan
    assert s.try_parse(good[:i]) == R.Status.BAD_JPEG
    # Ah/Al inconsistent with the first scan (Ah != 0 with Al != Ah - 1): JERR_BAD_PROGRESSION
    bad = bytearray(good)
    ns = bad[i + 4]
    bad[i + 4 + 1 + 2 * ns + 2] = 0x31
    assert s.try_parse(bytes(bad)) == R.Status.BAD_JPEG


def test_truncated_and_garbage_streams():
    s = R.JpegStream()
    assert s.try_parse(b"\xff\xd8") == R.Status.BAD_JPEG
    assert s.try_parse(b"\x00" * 64) == R.Status.BAD_JPEG
    good = O.fixture_bytes(O.manifest()[0])
    for cut in (3, 20, 100, 400):
        assert s.try_parse(good[:cut]) in (R.Status.BAD_JPEG, R.Status.SUCCESS)


def test_create_without_gpu_fails_cleanly():
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except ImportError:
        pass
    h = ctypes.c_void_p()
    st = R.lib().rocJpegCreate(0, 0, ctypes.byref(h))
    assert st in (R.Status.EXECUTION_FAILED, R.Status.NOT_INITIALIZED)
    if h:
        R.lib().rocJpegDestroy(h)


# ---- binary drop-in: the reference header and ours give identical layouts and signatures ----
_REF_API = "/root/reference/api"
_ABI_GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "abi_layout_reference.json")


def _abi_probe(include_dir, tmp_path):
    """Compile tests/c/abi_probe.c against the rocjpeg.h in `include_dir`: once -c with the
    signature checks (incompatible pointer types are errors), once linked and run for the
    layout JSON."""
    import json
    import subprocess
    src = os.path.join(os.path.dirname(os.path.abspath(__file__)), "c", "abi_probe.c")
    flags = ["-std=c11", "-Wall", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", f"-I{include_dir}"]
    subprocess.run(["gcc", *flags, "-c", "-DABI_SIGNATURES", "-Werror=incompatible-pointer-types", src,
                    "-o", str(tmp_path / "sig.o")], check=True, capture_output=True)
    exe = tmp_path / "probe"
    subprocess.run(["gcc", *flags, src, "-o", str(exe)], check=True, capture_output=True)
    return json.loads(subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout)


def test_abi_layout_matches_reference_golden(tmp_path):
    """include/rocjpeg.h vs the layout the reference header produced (committed fixture, so the
    check runs where /root/reference is absent)."""
    import json
    ours = _abi_probe(INCLUDE, tmp_path)
    assert ours == json.load(open(_ABI_GOLDEN))


@pytest.mark.skipif(not os.path.isfile(os.path.join(_REF_API, "rocjpeg.h")), reason="reference header absent")
def test_abi_layout_matches_reference_header(tmp_path):
    """Both headers compiled side by side (api/rocjpeg.h:46-343): same sizeof / offsetof / enum
    values, and every entry point type-checks against the same signature."""
    (tmp_path / "ref").mkdir()
    (tmp_path / "ours").mkdir()
    ref = _abi_probe(_REF_API, tmp_path / "ref")
    ours = _abi_probe(INCLUDE, tmp_path / "ours")
    assert ours == ref


# ---- hardening: crafted Huffman tables (rj_stream.cpp BuildLeanTable/BuildHuffman) ----
def oversubscribed_unused_slot_stream():
    """A gray row-interval fixture with an extra DHT that defines slot 1, which its scan does not
    use: DC with 12 codes of length 1, AC with 162 codes of length 2 (both over-subscribed).
    libjpeg builds derived tables only for the scan's slots (jdhuff.c start_pass_huff_decoder),
    so the stream is valid and decodes as the original."""
    import struct
    d = O.fixture_bytes(next(f for f in O.manifest() if f["name"] == "p400_q85_ri_96x72"))
    seg = bytes([0x01, 12] + [0] * 15) + bytes(range(12)) + bytes([0x11, 0, 162] + [0] * 14) + bytes(range(162))
    return d[:2] + b"\xff\xc4" + struct.pack(">H", len(seg) + 2) + seg + d[2:]


def test_oversubscribed_tables_are_refused_without_writes(tmp_path):
    """Host parse + lean-table build of the crafted stream under AddressSanitizer (host code only:
    tests/c/huff_tables_asan.cpp links rj_stream.cpp, no GPU call).  Before the fix the lean
    builder wrote past its 512-word DC table."""
    import subprocess
    csrc = os.path.join(O.ROOT, "rocjpeg_amd", "csrc")
    exe = tmp_path / "huff_asan"
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address", "-D__HIP_PLATFORM_AMD__",
                    "-I/opt/rocm/include", f"-I{csrc}", f"-I{INCLUDE}",
                    os.path.join(O.ROOT, "tests", "c", "huff_tables_asan.cpp"),
                    os.path.join(csrc, "rj_stream.cpp"), os.path.join(csrc, "rj_prog_stream.cpp"), os.path.join(csrc, "rj_pinned.cpp"),
                    "-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib", "-o", str(exe)],
                   check=True, capture_output=True)
    bad = tmp_path / "bad.jpg"
    bad.write_bytes(oversubscribed_unused_slot_stream())
    r = subprocess.run([str(exe), str(bad)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "status=0 valid=10" in r.stdout  # decodable; slot 0 valid, slot 1 refused
    # the same bad slot used by the scan: the stream is refused at decode planning
    used = bytearray(oversubscribed_unused_slot_stream())
    j = used.index(b"\xff\xda")
    used[j + 6] = 0x11  # scan component 0 -> DC/AC table 1
    bad.write_bytes(bytes(used))
    r = subprocess.run([str(exe), str(bad)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "status=-3 valid=10" in r.stdout


def test_timings_struct_matches_binding(tmp_path):
    """The ctypes mirror of RocJpegAmdTimings (rocjpeg_amd/__init__.py) has the C layout: size and
    the offset of every field, from a probe compiled against include/rocjpeg_amd.h."""
    import subprocess
    fields = [k for k, _ in R.RocJpegAmdTimings._fields_]
    src = tmp_path / "t.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "rocjpeg_amd.h"\nint main(void) {\n'
                   '  printf("%zu\\n", sizeof(RocJpegAmdTimings));\n' +
                   "".join(f'  printf("%zu\\n", offsetof(RocJpegAmdTimings, {k}));\n' for k in fields) + "  return 0;\n}\n")
    exe = tmp_path / "t"
    subprocess.run(["gcc", "-std=c11", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", f"-I{INCLUDE}", str(src),
                    "-o", str(exe)], check=True, capture_output=True)
    out = [int(x) for x in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()]
    assert out[0] == ctypes.sizeof(R.RocJpegAmdTimings)
    assert out[1:] == [getattr(R.RocJpegAmdTimings, k).offset for k in fields]
