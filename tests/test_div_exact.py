"""The kernels' FMA-corrected division by a small integer (bq_device.h
div_exact / div_count) equals the IEEE quotient: compiled with gcc from
tests/csrc/div_exact_check.c and run over 51M random cases (n = 1..256,
exponents -300..300 and price-like decimals)."""
import shutil
import subprocess

import pytest

from pathlib import Path

SRC = Path(__file__).parent / "csrc" / "div_exact_check.c"


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc absent")
def test_fma_corrected_quotient_is_ieee(tmp_path):
    exe = tmp_path / "div_exact_check"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", str(exe), str(SRC), "-lm"], check=True)
    for seed in ("7", "11"):
        out = subprocess.run([str(exe), "256", "100000", seed], capture_output=True, text=True, timeout=120)
        assert out.returncode == 0, out.stdout
        assert "mismatches 0" in out.stdout
