"""Host-code sanitizers on the native launchers.

GPU AddressSanitizer / xnack+ code objects are not available on the MI355X pool, so the
sanitized build covers the HOST side of csrc/: argument validation of every launcher runs
under AddressSanitizer + UndefinedBehaviorSanitizer (``-Xarch_host -fsanitize=...``), on a
machine without a GPU (every case is rejected before any HIP call). Device code is still
compiled for gfx950 in the same build.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_launcher_validation_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "host_check")
    srcs = [os.path.join(CSRC, "tests", "host_check.cpp")] + [
        os.path.join(CSRC, f) for f in ("gemm_skinny.hip", "attention_decode.hip", "attention_prefill32.hip",
                                         "decode_step.hip", "kv_copy.hip")]
    cmd = [HIPCC, "--offload-arch=gfx950", "-O1", "-g", "-std=c++17",
           "-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
           "-Xarch_host", "-fno-omit-frame-pointer", "-Xarch_host", "-fno-sanitize-recover=undefined",
           "-I", CSRC, *srcs, "-o", exe]
    b = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert b.returncode == 0, b.stderr[-3000:]
    nm = shutil.which("nm")
    if nm:
        syms = subprocess.run([nm, exe], capture_output=True, text=True).stdout
        assert "__asan_init" in syms and "__ubsan_handle" in syms   # the sanitizers really are linked in
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    assert "0 failure(s)" in r.stdout
    assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr
