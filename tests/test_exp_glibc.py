"""exp_glibc (ggp_prop.h, the GGP_EXACT engine's exp) against this process's libm, bitwise.

The reference calls glibc's exp(); on an x86-64 CPU with FMA that resolves to glibc's FMA build of
the table-driven exp, which ggp::exp_glibc restates (DESIGN.md §2 "Exact arithmetic").  The
device source is compiled for the host (GGP_HOST_SIM) by tests/exp_glibc_check.cpp and compared
on 4e6 random arguments over [-745, 710] and the special inputs.  Skipped on a CPU without FMA
(glibc then runs its other build, which rounds differently: that difference is measured in
DESIGN.md §2)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cpu_has_fma() -> bool:
    try:
        flags = open("/proc/cpuinfo").read()
    except OSError:
        return False
    return " fma " in flags or " fma\n" in flags


@pytest.mark.skipif(not _cpu_has_fma(), reason="glibc's exp resolves to its non-FMA build on this CPU")
def test_exp_glibc_bitwise_against_libm(tmp_path):
    exe = str(tmp_path / "exp_glibc_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off",
                    "-I", os.path.join(ROOT, "gfp_gaussian_process_amd", "csrc"), "-o", exe,
                    os.path.join(ROOT, "tests", "exp_glibc_check.cpp"), "-lm"], check=True)
    for seed in (1, 2):
        out = subprocess.run([exe, "1000000", str(seed)], capture_output=True, text=True, check=True).stdout.split()
        checked, bad, first = int(out[0]), int(out[1]), out[2]
        assert checked > 4_000_000
        assert bad == 0, f"{bad} mismatches, first at x = {first}"
