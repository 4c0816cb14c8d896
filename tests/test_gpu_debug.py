"""The bounds-checked debug build (libppgat_debug.so, `make debug`) on the GPU: the index
validation catches out-of-range inputs with an error instead of a kernel launch, and the
GPU parity tests of the layer pass unchanged on it.  Runs in child processes with
PPGAT_LIB pointing at the debug library."""
import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]
DBG = ROOT / "plotpointe-gat-recommendation_amd" / "libppgat_debug.so"

SNIPPET = r"""
import importlib, sys, torch
sys.path.insert(0, sys.argv[1])
pkg = importlib.import_module("plotpointe-gat-recommendation_amd")
L = pkg._lib
assert L.debug_build()
dev = torch.device("cuda", 0)
t = torch.tensor([0, 5, 9, 10, -1, 3], dtype=torch.int32, device=dev)
L.check_index_range(t[:3], 0, 10, "ok")            # in range: silent
try:
    L.check_index_range(t, 0, 10, "idx")
    raise SystemExit("no error for out-of-range indices")
except RuntimeError as e:
    assert "2 of 6 indices outside [0, 10)" in str(e), e
# an out-of-range BPR triple is refused by the debug entry point before any launch
Z = torch.randn(30, 64, device=dev)
u = torch.tensor([0, 1, 2], device=dev); i = torch.tensor([0, 1, 2], device=dev)
j = torch.tensor([0, 1, 25], device=dev)          # item 25 >= n_items = 10
try:
    pkg.bpr_loss(Z, 20, u, i, j)
    raise SystemExit("no error for an out-of-range triple")
except (RuntimeError, ValueError) as e:
    assert "outside" in str(e) or "range" in str(e), e
print("DEBUG-OK")
"""


def _env():
    return dict(os.environ, PPGAT_LIB=str(DBG), HSA_ENABLE_IPC_MODE_LEGACY="0")


def test_debug_build_rejects_out_of_range_indices(cuda):
    if not DBG.exists():
        pytest.fail("libppgat_debug.so missing: build() makes it")
    p = subprocess.run([sys.executable, "-c", SNIPPET, str(ROOT)], env=_env(), capture_output=True, text=True,
                       timeout=120)
    assert p.returncode == 0 and "DEBUG-OK" in p.stdout, p.stdout[-2000:] + p.stderr[-3000:]


def test_layer_parity_on_debug_build(cuda):
    """A slice of the GPU parity suite (layer forward/backward vs the oracle, graph builds,
    dropout) with every graph view range-checked and every entry point synchronised."""
    if not DBG.exists():
        pytest.fail("libppgat_debug.so missing: build() makes it")
    cmd = [sys.executable, "-m", "pytest", str(ROOT / "tests" / "test_gpu_parity.py"), "-m", "gpu", "-x", "-q",
           "-k", "golden or dropout or hub or empty or eval", "-p", "no:cacheprovider"]
    p = subprocess.run(cmd, cwd=str(ROOT), env=_env(), capture_output=True, text=True, timeout=150)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-2000:]
    assert " passed" in p.stdout
