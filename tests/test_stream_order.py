"""CPU unit test of the cross-stream ordering rule PolyStore applies before reads, writes and frees
(fhe-gpt-2_amd/seal/stream_order.h; tests/cpp/stream_order_test.cpp): the fix for blocks handed
out again while another stream still read them, now as device-side waits instead of host syncs."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_stream_order_rule(tmp_path):
    exe = os.path.join(tmp_path, "stream_order_test")
    subprocess.check_call(["g++", "-O1", "-std=c++17", "-Wall", "-o", exe,
                           os.path.join(ROOT, "tests", "cpp", "stream_order_test.cpp")])
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "ALL PASSED" in r.stdout, r.stdout + r.stderr
