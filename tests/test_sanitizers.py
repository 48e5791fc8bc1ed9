"""Host runtime under sanitizers: builds csrc/selftest/host_selftest.cc
with the native host sources under ASan+UBSan and TSan and runs it
(multi-threaded loader, dlopen parser plugin, async dense table, dump writers)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
@pytest.mark.parametrize("mode", ["asan", "tsan"])
def test_host_selftest_under_sanitizer(mode, tmp_path):
    env = dict(os.environ, SANITIZE_OUT=str(tmp_path))
    r = subprocess.run([os.path.join(ROOT, "scripts", "sanitize_host.sh"), mode], env=env, capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "host_selftest: ok" in r.stdout
