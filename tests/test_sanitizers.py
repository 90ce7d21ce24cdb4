"""CPU: libg2n's host code (gzip ingest: the parallel member reader and gzip.py's reader restated,
with the prefix it keeps on failure; the convert CLI's .npz / .nodes.tsv writers; the UTF-8 scan)
built with g++ under AddressSanitizer + UndefinedBehaviorSanitizer and driven by
tests/native/sancheck.cpp on clean, truncated, corrupted and garbage-tailed member chains.
Any sanitizer report aborts the driver (-fno-sanitize-recover) and fails the test."""
import os
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "gfa2network_amd" / "csrc"


@pytest.mark.skipif(shutil.which("g++") is None or not Path("/opt/rocm/include/hip/hip_runtime.h").exists(),
                    reason="needs g++ and the ROCm headers (the HIP upload path is linked, never called)")
def test_host_code_under_asan_ubsan(tmp_path):
    exe = tmp_path / "sancheck"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-fno-omit-frame-pointer", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
           str(ROOT / "tests" / "native" / "sancheck.cpp"), str(CSRC / "g2n_ingest.cpp"), str(CSRC / "g2n_pinflate.cpp"), str(CSRC / "g2n_split.cpp"),
           str(CSRC / "g2n_writers.cpp"), "-L/opt/rocm/lib", "-Wl,-rpath,/opt/rocm/lib", "-lamdhip64", "-lz",
           "-lpthread", "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", G2N_HOST_THREADS="4")
    r = subprocess.run([str(exe)], env=env, capture_output=True, timeout=300)
    assert r.returncode == 0 and r.stdout.strip() == b"OK", r.stderr.decode(errors="replace")[-4000:]
