"""The device's restatement of glibc's expf / tanhf (csrc/glibc_math.h,
used by exact mode's attention and by every GELU) compiled for the host from
the same source and compared with the host libm -- the libm the reference is
linked against -- on EVERY float bit pattern (2^32 inputs each)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_glibc_expf_tanhf_exhaustive(tmp_path):
    exe = str(tmp_path / "glibc_math_check")
    subprocess.run(["g++", "-O2", "-mfma", "-ffp-contract=off", "-std=c++17", "-o", exe,
                    os.path.join(ROOT, "tests", "native", "glibc_math_check.cpp"), "-lpthread", "-lm"], check=True)
    r = subprocess.run([exe, str(min(os.cpu_count() or 4, 16))], capture_output=True, text=True)
    print(r.stdout)
    assert r.returncode == 0, r.stdout
    assert "expf mismatches 0, tanhf mismatches 0" in r.stdout
