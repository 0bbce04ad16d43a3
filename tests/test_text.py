"""The CLI's bulk text formatting (csrc/host/ggp_text.h) on CPU.

put_num must append exactly what the reference's `std::ostream << double` writes under the
default stream state (predictions.h:540-602, correlation_tree.h:96-126): checked against an
ostringstream on a million values (random bit patterns, the data's scales, short decimals,
integers, NaN, +-inf, signed zero, subnormals) and against Python's '%.6g' (printf's
conversion, which libstdc++'s `<<` uses).  write_ordered must produce the serial byte stream
for any thread count.
"""
import os
import shutil
import struct
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def text_check(tmp_path_factory):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("g++ not available")
    exe = str(tmp_path_factory.mktemp("text") / "text_check")
    subprocess.run([cxx, "-O2", "-std=c++17", "-pthread", "-I", os.path.join(ROOT, "gfp_gaussian_process_amd", "csrc", "host"),
                    "-o", exe, os.path.join(ROOT, "tests", "text_check.cpp")], check=True)
    return exe


@pytest.mark.parametrize("seed", [1, 20261017])
def test_put_num_is_the_streams_default_format(text_check, seed):
    out = subprocess.run([text_check, "formats", str(seed), "1000000"], check=True, capture_output=True,
                         text=True).stdout.split("\n")
    assert int(out[0]) == 0, "put_num differs from ostream << double"
    n = 0
    for line in out[1:]:
        if not line:
            continue
        bits, text = line.split(" ")
        x = struct.unpack("<d", bytes.fromhex(bits)[::-1])[0]
        ref = "%.6g" % x
        if x != x:                                  # printf: "nan" / "-nan" by the sign bit
            ref = "-nan" if int(bits, 16) >> 63 else "nan"
        assert text == ref, (bits, text, ref)
        n += 1
    assert n == 2000


@pytest.mark.parametrize("threads", [1, 3, 16])
def test_write_ordered_is_the_serial_stream(text_check, threads):
    out = subprocess.run([text_check, "ordered", str(threads)], check=True, capture_output=True, text=True).stdout
    assert out.strip() == "same"


@pytest.mark.parametrize("threads", [1, 4])
def test_write_ordered_rethrows_a_formatting_error(text_check, threads):
    out = subprocess.run([text_check, "throws", str(threads)], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0 and out.stdout.strip() == "caught block 377", (out.stdout, out.stderr)
