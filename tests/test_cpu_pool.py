"""ddt_pool.cpp's cross-device settling on the CPU: the pool compiled with a
mock of the HIP calls it makes (tests/native/pool_devices.cpp) -- an unknown release on device 1
is not recycled by a device-0 allocation, and the next device-1 allocation settles it."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "ompi_amd", "csrc")


def test_pool_settles_per_device(tmp_path):
    exe = str(tmp_path / "pool_devices")
    cmd = ["g++", "-std=c++17", "-O1", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", f"-I{CSRC}",
           f"-I{os.path.join(ROOT, 'include')}", os.path.join(ROOT, "tests", "native", "pool_devices.cpp"),
           os.path.join(CSRC, "ddt_pool.cpp"), "-o", exe]
    b = subprocess.run(cmd, capture_output=True, text=True)
    if b.returncode != 0 and "hip_runtime.h" in b.stderr:
        pytest.skip("no HIP headers")
    assert b.returncode == 0, b.stderr[-3000:]
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stdout + r.stderr
