"""Host-code sanitizer run: the CLI built with AddressSanitizer +
UndefinedBehaviorSanitizer (`make sanitize`, built by the first test that needs it, ~1 min on
8 cores) trains the reference's example configs on the CPU learner; any ASan / UBSan report
fails the test."""
import fcntl
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASAN_CLI = os.path.join(ROOT, "build_asan", "lightgbm")
EXAMPLES = "/root/reference/examples"


def _build(target, path):
    # (make is incremental: an up-to-date build returns at once, a stale one is rebuilt).  Under
    # pytest-xdist several workers get here at once: an exclusive lock makes one build while the
    # others wait, so none runs a binary another is still linking
    os.makedirs(os.path.join(ROOT, "build"), exist_ok=True)
    with open(os.path.join(ROOT, "build", ".sanitize.lock"), "w") as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)
        try:
            subprocess.run(["make", "-j" + str(min(8, os.cpu_count() or 4)), target], cwd=ROOT, check=True,
                           capture_output=True, timeout=1500)
        finally:
            fcntl.flock(lock, fcntl.LOCK_UN)
    assert os.path.isfile(path), target


@pytest.fixture(scope="module")
def asan_cli():
    _build("sanitize", ASAN_CLI)
    return ASAN_CLI


@pytest.mark.skipif(not os.path.isdir(EXAMPLES), reason="reference examples not mounted")
@pytest.mark.parametrize("example,extra", [("binary_classification", ["num_trees=10"]),
                                           ("regression", ["num_trees=10"]),
                                           ("lambdarank", ["num_trees=5"])])
def test_examples_clean_under_asan_ubsan(tmp_path, asan_cli, example, extra):
    work = tmp_path / example
    shutil.copytree(os.path.join(EXAMPLES, example), work)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    out = subprocess.run([asan_cli, "config=train.conf", "output_model=" + str(tmp_path / "m.txt")] + extra,
                         cwd=work, env=env, capture_output=True, text=True, timeout=600)
    log = out.stdout + out.stderr
    assert out.returncode == 0, log[-4000:]
    assert "AddressSanitizer" not in log and "runtime error" not in log, log[-4000:]
    assert (tmp_path / "m.txt").exists()


TSAN_DRIVER = os.path.join(ROOT, "build_tsan", "tsan_driver")


@pytest.mark.skipif(not os.path.isdir(EXAMPLES), reason="reference examples not mounted")
def test_threads_clean_under_tsan(tmp_path):
    """ThreadSanitizer (`make tsan`): two_round loading's reader thread, and training under the
    booster's exclusive lock while three threads predict and one reads evaluations through the
    C API (tests/native/tsan_driver.cpp).  Found and fixed with it: the log level written by
    every C API call, and booster getters reading the model without the lock."""
    _build("tsan", TSAN_DRIVER)
    env = dict(os.environ, OMP_NUM_THREADS="1", TSAN_OPTIONS="exitcode=66 halt_on_error=0")
    out = subprocess.run([TSAN_DRIVER, os.path.join(EXAMPLES, "binary_classification", "binary.train"), "28"],
                         cwd=tmp_path, env=env, capture_output=True, text=True, timeout=600)
    log = out.stdout + out.stderr
    assert "ThreadSanitizer" not in log, log[-6000:]
    assert out.returncode == 0 and "tsan driver ok: 15 iterations, row-wise boosters 5 / 5" in log, log[-3000:]
