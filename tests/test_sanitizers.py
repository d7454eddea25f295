"""Host-code sanitizer run: the CLI built with AddressSanitizer +
UndefinedBehaviorSanitizer (`make sanitize`) trains the reference's example configs on the
CPU learner; any ASan / UBSan report fails the test.  Skipped when the instrumented CLI has
not been built."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASAN_CLI = os.path.join(ROOT, "build_asan", "lightgbm")
EXAMPLES = "/root/reference/examples"


@pytest.mark.skipif(not os.path.isfile(ASAN_CLI), reason="make sanitize not built")
@pytest.mark.skipif(not os.path.isdir(EXAMPLES), reason="reference examples not mounted")
@pytest.mark.parametrize("example,extra", [("binary_classification", ["num_trees=10"]),
                                           ("regression", ["num_trees=10"]),
                                           ("lambdarank", ["num_trees=5"])])
def test_examples_clean_under_asan_ubsan(tmp_path, example, extra):
    work = tmp_path / example
    shutil.copytree(os.path.join(EXAMPLES, example), work)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    out = subprocess.run([ASAN_CLI, "config=train.conf", "output_model=" + str(tmp_path / "m.txt")] + extra,
                         cwd=work, env=env, capture_output=True, text=True, timeout=600)
    log = out.stdout + out.stderr
    assert out.returncode == 0, log[-4000:]
    assert "AddressSanitizer" not in log and "runtime error" not in log, log[-4000:]
    assert (tmp_path / "m.txt").exists()
