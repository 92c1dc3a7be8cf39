"""Run one test function against a libbos.so build variant (diagnostics):
python tools/test_with_lib.py LIB.so tests/test_x.py::test_name[param-index] ..."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = os.path.abspath(sys.argv[1])
code = f"""
import sys
sys.path.insert(0, {os.path.join(ROOT, 'tests')!r}); sys.path.insert(0, {os.path.join(ROOT, 'prb-project-bearing-only-slam_amd')!r})
import bos
bos.LIB_PATH = {lib!r}
bos.ALLOW_MISSING_SYMBOLS = True
import pytest
sys.exit(pytest.main(['-x', '-q', '-p', 'no:cacheprovider', '--timeout', '300'] + {sys.argv[2:]!r}))
"""
r = subprocess.run([sys.executable, "-c", code], cwd=ROOT)
print(os.path.basename(lib), "rc", r.returncode, flush=True)
