"""ASan + UBSan corpus run of the native host I/O layer: Parquet footer / page
parsing, host Snappy, run tables, the device page planner, the Parquet writer and the Avro block
decoder, on valid and corrupted inputs (``scripts/sanitize_hostio.py``).  The fixes it drove:
negative page-header lengths, footer lists longer than the footer, row groups missing columns,
overflowing bit-packed group counts (csrc/runtime/hs_parquet.cpp)."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _have_sanitizers() -> bool:
    if shutil.which("g++") is None:
        return False
    for lib in ("libasan.so", "libubsan.so"):
        r = subprocess.run(["g++", f"-print-file-name={lib}"], capture_output=True, text=True)
        if not os.path.isabs(r.stdout.strip()):
            return False
    return True


@pytest.mark.skipif(not _have_sanitizers(), reason="g++ sanitizer runtimes not installed")
def test_host_io_layer_is_clean_under_asan_ubsan(tmp_path):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "sanitize_hostio.py"),
                        "--iters", "400", "--seed", "3"], capture_output=True, text=True,
                       cwd=str(tmp_path), timeout=900)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-6000:])
    assert "clean" in r.stdout


def _have_tsan() -> bool:
    if shutil.which("g++") is None:
        return False
    r = subprocess.run(["g++", "-print-file-name=libtsan.so"], capture_output=True, text=True)
    return os.path.isabs(r.stdout.strip())


@pytest.mark.skipif(not _have_tsan(), reason="g++ ThreadSanitizer runtime not installed")
def test_host_io_layer_is_race_free_under_tsan(tmp_path):
    """ThreadSanitizer build of the host runtime (csrc/runtime/hs_parquet.cpp,
    hs_parquet_write.cpp, hs_avro.cpp) driven the way the staging pool drives it: 8 threads
    decoding / planning chunks of shared and distinct files, Snappy streams, Avro blocks and
    concurrent native Parquet writes."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "sanitize_hostio.py"),
                        "--tsan", "--iters", "64", "--seed", "3"], capture_output=True,
                       text=True, cwd=str(tmp_path), timeout=900)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-6000:])
    assert "clean" in r.stdout and "verified" in r.stdout
