"""CPU unit tests of the seal:: surface's host-side concurrency logic, each built plain and under
ThreadSanitizer and AddressSanitizer (+UBSan):
  * the cross-stream ordering rule PolyStore applies before reads, writes and frees
    (fhe-gpt-2_amd/seal/stream_order.h; tests/cpp/stream_order_test.cpp) -- the fix for blocks handed
    out again while another stream still read them, as device-side waits instead of host syncs;
  * seal::Lockstep's round logic (fhe-gpt-2_amd/seal/lockstep_core.h; tests/cpp/lockstep_test.cpp)
    with stubbed launches from 1-8 member threads, members leaving early."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SANITIZERS = {"plain": [], "tsan": ["-fsanitize=thread"], "asan": ["-fsanitize=address,undefined",
                                                                   "-fno-sanitize-recover=undefined"]}


@pytest.mark.parametrize("san", sorted(SANITIZERS))
@pytest.mark.parametrize("name", ["stream_order_test", "lockstep_test"])
def test_host_concurrency_logic(tmp_path, name, san):
    exe = os.path.join(tmp_path, name)
    subprocess.check_call(["g++", "-O1", "-g", "-std=c++17", "-Wall", "-pthread", *SANITIZERS[san], "-o", exe,
                           os.path.join(ROOT, "tests", "cpp", name + ".cpp")])
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66", ASAN_OPTIONS="detect_leaks=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "ALL PASSED" in r.stdout, r.stdout + r.stderr
    assert "Sanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr
