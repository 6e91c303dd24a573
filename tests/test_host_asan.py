"""The host-only C++ of the engine (TSV ingest, model files, host merge, mAP
fold) under AddressSanitizer + UBSan: tests/asan/host_asan.cpp linked with
csrc/mr_host.cpp + csrc/mr_modelio.cpp by g++ (no HIP), run on the committed
fixtures, a malformed file and forced multi-threaded chunking."""
import os
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "musicrecommendation_amd", "csrc")


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_host_code_under_asan(tmp_path):
    exe = tmp_path / "host_asan"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=undefined", f"-I{ROOT}/include", os.path.join(ROOT, "tests", "asan", "host_asan.cpp"),
           os.path.join(CSRC, "mr_host.cpp"), os.path.join(CSRC, "mr_modelio.cpp"), "-lpthread", "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    z = np.load(os.path.join(ROOT, "tests", "golden", "synth_small.npz"))
    paths = []
    for key in ("train", "test", "labels"):
        p = tmp_path / f"{key}.txt"
        p.write_text("".join(l + "\n" for l in z[key].tolist()))
        paths.append(str(p))
    bad = tmp_path / "bad.txt"
    bad.write_text("u1\ts1\t1\nu2\ts2\n")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe), *paths, str(bad), str(tmp_path)], capture_output=True, text=True, timeout=300,
                       env=env)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "host asan: ok" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr
