"""The JNI shim's call sequences (jni/nativeengine.c, the JDK-free core of
jni/mr_jni.c) through the plain-C harness jni/build/test_shim (built by
__graft_entry__.build(), gcc, linked against libmr_engine.so): error codes on
any box; on the GPU box the single-context sequence mr_options_default ->
mr_create -> mr_load -> mr_score_dense -> mr_destroy and the shim's group
sequences, bit-identical to the fixed-point oracle on the SURVEY §4.2 KAT."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(ROOT, "jni", "build", "test_shim")


def _run():
    assert os.path.exists(HARNESS), "jni/build/test_shim missing: run __graft_entry__.build()"
    return subprocess.run([HARNESS], capture_output=True, text=True, timeout=120)


def test_shim_error_codes_cpu():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU visible: the GPU test runs the full harness")
    r = _run()
    assert r.returncode == 0, r.stdout + r.stderr
    assert "error codes: ok" in r.stdout and "gpu: skipped" in r.stdout


@pytest.mark.gpu
def test_shim_sequences_gpu():
    r = _run()
    assert r.returncode == 0, r.stdout + r.stderr
    assert "gpu KAT sequences: ok" in r.stdout
