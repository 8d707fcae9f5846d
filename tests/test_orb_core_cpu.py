"""mcs_orb_core.h's FAST helpers on the host (tests/native/fast_check.cpp, g++): the
doubling-window score equals the direct 16 x 9 arc scan of the specification, and the bit-mask
segment test equals score > t -- the identity mcs_orb_level's compacted scoring relies on."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_fast_score_and_segment_test(tmp_path):
    exe = str(tmp_path / "fast_check")
    subprocess.check_call(["g++", "-O2", "-std=c++17",
                           "-I" + os.path.join(ROOT, "multicamera_stitching_amd", "csrc"),
                           os.path.join(ROOT, "tests", "native", "fast_check.cpp"), "-o", exe])
    out = subprocess.run([exe, "400000"], capture_output=True, text=True)
    n, corners, bad = map(int, out.stdout.split())
    assert out.returncode == 0 and bad == 0, out.stdout
    assert corners > n // 10          # the adversarial cases do produce corners
