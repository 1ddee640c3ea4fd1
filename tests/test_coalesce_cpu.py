"""The coalescing of concurrent small calls (rocjpeg_amd/csrc/rj_coalesce.cpp), on the CPU: the
unit is built against a stub decoder (tests/c/coalesce_stub/) under AddressSanitizer and driven
by 8 threads with a handle each, as jpegdecodeperf drives rocJpegDecodeBatched
(samples/jpegDecodePerf/jpegdecodeperf.cpp:228-257).  Checked: every call gets its own status
(a bad stream fails only its own call, also inside a combined call), no handle is used by two
threads at once, streams keep their destinations, calls are combined, and no memory error occurs,
for one and for several combined calls in flight and with and without the gathering wait."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def stub_exe(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    d = tmp_path_factory.mktemp("coalesce")
    # rj_coalesce.cpp includes "rj_decoder.h" from its own directory: build it beside the stub
    for f in ("rj_coalesce.cpp", "rj_coalesce.h"):
        shutil.copy(os.path.join(ROOT, "rocjpeg_amd", "csrc", f), d / f)
    for f in ("rj_decoder.h", "coalesce_main.cpp"):
        shutil.copy(os.path.join(ROOT, "tests", "c", "coalesce_stub", f), d / f)
    src = (d / "rj_coalesce.h").read_text().replace('#include "../../include/rocjpeg.h"', '#include "rocjpeg.h"')
    (d / "rj_coalesce.h").write_text(src)
    exe = d / "coalesce_stub"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-D__HIP_PLATFORM_AMD__", f"-I{d}", f"-I{os.path.join(ROOT, 'include')}", "-I/opt/rocm/include",
           str(d / "coalesce_main.cpp"), str(d / "rj_coalesce.cpp"), "-o", str(exe), "-lpthread"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    return str(exe)


@pytest.mark.parametrize("env", [{}, {"RJ_COALESCE_WAIT_US": "0"}, {"RJ_COALESCE_INFLIGHT": "2"},
                                 {"RJ_COALESCE_INFLIGHT": "3", "RJ_COALESCE_WAIT_US": "50"}])
def test_coalesced_calls_keep_their_own_status(stub_exe, env):
    e = dict(os.environ, **env)
    e.pop("RJ_COALESCE", None)
    r = subprocess.run([stub_exe, "8", "400"], capture_output=True, text=True, timeout=300, env=e)
    assert r.returncode == 0, (r.stdout, r.stderr[-3000:])
    m = re.search(r"calls (\d+) combined (\d+) members (\d+) images (\d+) wrong_status (\d+) bad_calls (\d+) "
                  r"attempts (\d+)", r.stdout)
    calls, combined, members, images, wrong, bad, attempts = map(int, m.groups())
    assert calls == 8 * 400 and wrong == 0 and bad > 0
    assert combined > 0 and members > combined  # calls were decoded together
    # members are validated before the combined call: a bad stream is never decoded and costs
    # the calls combined with it no second decode: every good image decoded once, no image
    # handed to a decode twice
    assert images == calls - bad and attempts <= calls


def test_coalescing_off(stub_exe):
    e = dict(os.environ, RJ_COALESCE="0")
    r = subprocess.run([stub_exe, "4", "50"], capture_output=True, text=True, timeout=120, env=e)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "combined 0 members 0" in r.stdout and "calls 0" in r.stdout
