"""SURVEY.md §5 (race detection / sanitizers): the host-side C++ -- the native table builders of
libkadgpu.so (kad_synth.cpp) and the CPU oracle -- built from source with AddressSanitizer and
UndefinedBehaviorSanitizer and run on tables of 0..60k nodes (tests/cpp/sanitize_host.cpp). CPU only:
GPU sanitizers are not available on this pool."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))


def test_host_code_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", os.path.join(HERE, "cpp"), "sanitize_host"], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([os.path.join(HERE, "cpp", "sanitize_host")], capture_output=True, text=True, timeout=600,
                       env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "PASS" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr
