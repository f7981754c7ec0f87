"""Host sanitizer coverage of the engine's safety boundary (SURVEY.md §5:
host code under ASan/UBSan): mythril_amd/csrc/mg_host.cpp (program
validation + IR -> record translation) built with g++
-fsanitize=address,undefined and driven by tests/fuzz_translate.cpp with
valid, mutated and random programs.  CPU only."""

import json
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def fuzz_binary(tmp_path_factory):
    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    out = str(tmp_path_factory.mktemp("fuzz") / "fuzz_translate")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer",
           "-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-static-libasan",
           "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "mythril_amd", "csrc"),
           os.path.join(ROOT, "tests", "fuzz_translate.cpp"),
           os.path.join(ROOT, "mythril_amd", "csrc", "mg_host.cpp"), "-o", out]
    subprocess.run(cmd, check=True)
    return out


def test_validate_and_translate_under_asan_ubsan(fuzz_binary):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([fuzz_binary, "6000"], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    stats = json.loads(r.stdout.strip().splitlines()[-1])
    assert stats["valid_accepted"] == stats["iterations"]
    # mutations are mostly caught; random words essentially always
    assert stats["mutated_accepted"] < stats["iterations"]
    assert stats["random_accepted"] < stats["iterations"] // 100
