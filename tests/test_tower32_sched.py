"""Host check of the fp32 tower's wave-stream schedule (csrc/hip/tower32_sched.h,
shared by the kernels, the weight packing and the fused Adam's re-pack):
compiled with g++ and run over every layer shape up to 40 x 40 blocks."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_t32_schedule_positions(tmp_path):
    exe = tmp_path / "t32_sched_check"
    subprocess.run(["g++", "-O1", "-std=c++17", "-I", os.path.join(ROOT, "csrc"),
                    os.path.join(ROOT, "tests", "native", "t32_sched_check.cc"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=False)
    assert out.returncode == 0 and out.stdout.strip() == "ok", out.stdout + out.stderr
