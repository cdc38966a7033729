"""Host-side sanitizer run of the native sampler/optimizer helpers.

GPU AddressSanitizer is not available on the MI355X pool, so the ``__host__
__device__`` code the persistent train kernel runs per sample (``csrc/sampler.h``,
``dtp_common.h:pow_int``) is compiled for the host only, with ASan + UBSan on the
host pass, and exercised on the CPU by ``tests/native/sampler_host_test.cpp``:
Feistel bijection for awkward n, DistributedSampler coverage and padding for
W in {1,2,3,4,8}, batch geometry, and the Adam bias-correction power.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


@pytest.mark.skipif(not os.path.exists(HIPCC) and shutil.which("hipcc") is None, reason="hipcc not installed")
def test_sampler_host_code_under_asan_ubsan(tmp_path):
    exe = tmp_path / "sampler_host_test"
    hipcc = HIPCC if os.path.exists(HIPCC) else shutil.which("hipcc")
    cmd = [hipcc, "-x", "hip", "--offload-arch=gfx950", "--cuda-host-only", "-O1", "-g", "-std=c++17",
           "-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
           "-Xarch_host", "-fno-sanitize-recover=undefined",
           "-I", os.path.join(ROOT, "distributed_training_pytorch_amd", "csrc"),
           os.path.join(ROOT, "tests", "native", "sampler_host_test.cpp"), "-o", str(exe)]
    b = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert b.returncode == 0, b.stderr[-3000:]
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    assert "sampler host test OK" in r.stdout
