"""ThreadSanitizer run of the host runtime's CPU-side threaded code (no GPU): the speculative
parallel WAL chain walk with exact stitching and the multi-device split planner, each from several
concurrent callers (tests/cpp/test_host_threads.cpp, Makefile target `tsan`)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_host_threads_clean_under_tsan():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tinykvpp_amd", "csrc"), "tsan"], check=True)
    exe = os.path.join(ROOT, "tests", "cpp", "build", "test_host_threads_tsan")
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    assert "ThreadSanitizer" not in r.stderr, r.stderr[-4000:]
    assert r.returncode == 0 and "ALL PASSED" in r.stdout, r.stdout + r.stderr[-4000:]
