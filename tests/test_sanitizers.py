"""CPU tier: host sanitizer builds (the reference's analogue is its Debug flags,
CMakeLists.txt:17). The oracle (oracle/pb_oracle.c) and the host code of libpoissbox_gpu
(pb_runtime.cpp, pb_solver.cpp, the host side of every .hip file; device code unchanged) are built
with -fsanitize=address,undefined and driven by tests/sanitize/*.c[pp] -- every restated routine on
small odd shapes, and the library's option parsing, slab partition and argument/error paths without
a GPU. Any out-of-bounds access, leak or undefined behaviour fails the run."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(cmd, env=None, timeout=600):
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env)
    assert out.returncode == 0, (out.stdout[-3000:] + out.stderr[-3000:])
    return out.stdout


@pytest.mark.skipif(not shutil.which("gcc"), reason="gcc not in this image")
def test_oracle_asan_ubsan():
    _run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "asan"])
    out = _run([os.path.join(REPO, "oracle", "_asan", "oracle_check")])
    assert out.strip().endswith("oracle_check ok")


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="hipcc not in this image")
def test_library_host_asan_ubsan():
    csrc = os.path.join(REPO, "poissbox_amd", "csrc")
    _run(["make", "-s", "-j8", "-C", csrc, "asan"], timeout=1200)
    env = dict(os.environ, HIP_VISIBLE_DEVICES="")  # the CPU tier: no device, error paths only
    out = _run([os.path.join(csrc, "build-asan", "host_check")], env=env)
    assert "host_check ok (0 failures)" in out
