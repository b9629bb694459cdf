"""Host AddressSanitizer + UndefinedBehaviorSanitizer build of the native front end (SURVEY §5;
VERDICT r1 item 9): csrc/tokenizer.cpp compiled with -fsanitize=address,undefined together with
tests/host/tokenizer_sanitize.cpp, which drives every exported entry (rs_vocab_load / _size /
_free, rs_tokenize_batch incl. the threaded path and undersized buffers, rs_json_write_scores)
on adversarial inputs.  Any sanitizer report makes the run fail (-fno-sanitize-recover)."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(os.path.dirname(HERE), "asr-rescoring_amd", "csrc", "tokenizer.cpp")
DRV = os.path.join(HERE, "host", "tokenizer_sanitize.cpp")


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_tokenizer_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "tok_sanitize")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-fno-omit-frame-pointer", "-pthread", SRC, DRV, "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    if r.returncode != 0 and "asan" in (r.stderr or "").lower():
        pytest.skip("sanitizer runtime unavailable: " + r.stderr[-300:])
    assert r.returncode == 0, r.stderr[-2000:]
    # verify_asan_link_order=0: the environment may preload a library of its own ahead of the
    # ASan runtime; that is tolerated rather than removed
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe, str(tmp_path)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, (r.returncode, r.stdout[-500:], r.stderr[-3000:])
    assert "sanitize ok" in r.stdout
