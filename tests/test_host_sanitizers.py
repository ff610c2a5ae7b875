"""CPU: the product's host GF(2^8) code under AddressSanitizer + UBSan
(the reference's own CMake build uses -fsanitize=address,undefined,
CMakeLists.txt:23).  GPU sanitizers are not available on this pool."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_gf256_asan_ubsan(tmp_path):
    exe = str(tmp_path / "gf256_asan")
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
                    "-fno-sanitize-recover=all", "-o", exe,
                    os.path.join(ROOT, "tests", "gf256_asan_driver.cpp"),
                    os.path.join(ROOT, "udpspeeder_amd", "csrc", "gf256.cpp")], check=True)
    out = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.startswith("ok")
