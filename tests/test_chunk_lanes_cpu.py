"""The chunk-lane layout with MCU-phase hypotheses (rocjpeg_amd/csrc/rj_device.h
rj_chunk_lanes / rj_chunk_lane) is a bijection onto the interval's lanes, with chunk 0 last and
the kernels' inverse mapping exact (tests/c/chunk_lanes_check.cpp, built here with g++)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_chunk_lane_layout_is_a_bijection(tmp_path):
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    exe = tmp_path / "chunk_lanes_check"
    r = subprocess.run(["g++", "-std=c++17", "-O1", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                        f"-I{os.path.join(ROOT, 'rocjpeg_amd', 'csrc')}", f"-I{os.path.join(ROOT, 'include')}",
                        os.path.join(ROOT, "tests", "c", "chunk_lanes_check.cpp"), "-o", str(exe)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and r.stdout.startswith("OK"), r.stdout + r.stderr
