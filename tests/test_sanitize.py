"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer: `make asan` builds every
source of librt_hip.so with host-side instrumentation and runs tests/native/host_sanitize.cpp, a driver of
the host paths (scene validation and BVH build, the reference-graph flattener walking caller-owned pointers,
built-in scenes and textures, the PPM writer, and the device entry points' error paths on a GPU-less host)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(not shutil.which("/opt/rocm/bin/hipcc"), reason="needs hipcc")
def test_host_code_is_clean_under_asan_and_ubsan():
    env = dict(os.environ, HIP_VISIBLE_DEVICES=os.environ.get("HIP_VISIBLE_DEVICES", ""))
    r = subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "cudaraytracer_amd", "csrc"), "asan"],
                       capture_output=True, text=True, timeout=900, env=env)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "all checks passed" in r.stdout
