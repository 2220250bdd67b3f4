"""Host AddressSanitizer + UBSan run of the native runtime (JSON weight IO, protobuf codec,
schedules) -- SURVEY §5 "race detection / sanitizers": host ASan on the C++ runtime; GPU ASan
is not available on this pool, so device code is covered by the numerics tests instead."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_runtime_under_asan_ubsan(tmp_path):
    exe = tmp_path / "selftest"
    srcs = [os.path.join(ROOT, "csrc", "tests", "runtime_selftest.cpp")] + [
        os.path.join(ROOT, "csrc", "runtime", f) for f in
        ("json_weights.cpp", "matrix_codec.cpp", "schedule.cpp")]
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer",
           "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
           f"-I{os.path.join(ROOT, 'csrc')}", *srcs, "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    # the environment may preload other libraries ahead of the ASan runtime; tolerate that
    env = dict(os.environ,
               ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe), str(tmp_path)], capture_output=True, text=True, timeout=300,
                       env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "runtime selftest: OK" in r.stdout
