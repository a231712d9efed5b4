"""AddressSanitizer + UBSan over the native host code (the CSV tokenizer/parser)
with randomised RFC-4180 inputs (GPU sanitizers are not available on this pool, host ones are)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_csv_parser_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "csv_fuzz")
    src = os.path.join(ROOT, "scripts", "asan", "csv_fuzz.cpp")
    subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
                    "-pthread", src, "-o", exe], check=True, capture_output=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([exe, "1500"], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "csv_fuzz ok" in r.stdout
