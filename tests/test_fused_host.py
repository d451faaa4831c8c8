"""binquant_amd.fused program builder on the host: the bytecode a program
compiles to, interpreted with numpy, equals the direct torch evaluation of
the same expressions bit for bit (CSE, register reuse, shift push-down,
operand broadcasts, program splitting)."""

import numpy as np
import pytest
import torch

from binquant_amd import _lib
from binquant_amd import fused as F
from fused_util import assert_same, expressions, interpret, random_panel, torch_eval

S, T = 6, 40


def _operands():
    x, y, z = (random_panel(S, T, seed=k) for k in range(3))
    b = torch.rand(S, T, generator=torch.Generator().manual_seed(9)) < 0.5
    row = torch.rand(S, 1, dtype=torch.float64, generator=torch.Generator().manual_seed(4)) + 0.5
    col = torch.randn(T, dtype=torch.float64, generator=torch.Generator().manual_seed(5))
    return x, y, z, b, row, col


@pytest.mark.parametrize("block", [None, 4, 0])
def test_programs_equal_unfused_arithmetic(block):
    ex = expressions(*_operands())
    for name, e in ex.items():
        P = F.build([(name, e)], block)
        assert_same(name, interpret(P, S, T)[name], torch_eval(e, S, T).numpy())


def test_one_program_many_outputs_and_split():
    ex = expressions(*_operands())
    items = list(ex.items())
    progs = F._plan(items)
    got = {}
    for P in progs:
        assert len(P.ins) <= _lib.FUSED_MAX_INS and P.n_regs <= _lib.FUSED_MAX_REGS
        assert len(P.outputs) <= _lib.FUSED_MAX_OUT and len(P.inputs) <= _lib.FUSED_MAX_IN
        assert all((w & 0xFF) == _lib.FUSED_OPS["LD"] for w in P.ins[:P.n_loads])
        got.update(interpret(P, S, T))
    assert set(got) == set(ex)
    for name, e in ex.items():
        assert_same(name, got[name], torch_eval(e, S, T).numpy())


def test_cse_shares_work():
    x = random_panel(S, T)
    X = F.inp(x)
    s = (X + 1) * (X + 1)
    P = F.build([("a", s), ("b", s + (X + 1))])
    # X, 1, X+1, mul, add (+2 stores): X + 1 computed once
    assert sum((w & 0xFF) == _lib.FUSED_OPS["ADD"] for w in P.ins) == 2


def test_register_budget_and_errors():
    x = random_panel(S, T)
    X = F.inp(x)
    # a long chain reuses registers
    e = X
    for k in range(60):
        e = e * 1.0001 + (k % 7)
    P = F.build([("chain", e)])
    assert P.n_regs <= 2
    np.testing.assert_array_equal(interpret(P, S, T)["chain"], torch_eval(e, S, T).numpy())
    with pytest.raises(ValueError):
        F.inp(torch.zeros(2, 2, dtype=torch.float32))
    with pytest.raises(TypeError):
        bool(X > 0)
    with pytest.raises(RuntimeError):
        F.run({"y": X + 1})   # CPU tensors: no CPU fallback


def test_native_source_compiles_for_gfx950(tmp_path, monkeypatch):
    """The native form of every battery expression (and of the whole battery
    as one plan) is generated and compiled by hiprtc for gfx950 on the host;
    the source depends on the program structure only; the disk cache is
    reused."""
    from binquant_amd import _lib as L
    lib = L.load()
    lib.bq_fused_set_cache_dir(str(tmp_path).encode())
    try:
        ex = expressions(*_operands())
        srcs = F.native_source(ex, S, T)
        assert srcs and all("extern \"C\" __global__" in s and "bq_fk4" in s for s in srcs)
        # constants travel as kernel arguments: the source is the structure
        # only, so new constant values reuse the compiled kernel
        x = _operands()[0]
        a = F.native_source({"y": F.inp(x) * 2.5 + 1e-6}, S, T)
        b = F.native_source({"y": F.inp(x) * 0.1 + 3.0}, S, T)
        assert a == b and "a.c[" in a[0]
        before = F.native_stats()
        n = F.native_compile(ex, S, T)
        after = F.native_stats()
        assert after["compiles"] + after["disk_hits"] - before["compiles"] - before["disk_hits"] <= n
        assert len(list(tmp_path.glob("*.gfx950.co"))) >= 1
        assert F.native_compile(ex, S, T) == n   # process cache: no new compile
        assert F.native_stats()["compiles"] == after["compiles"]
    finally:
        lib.bq_fused_set_cache_dir(str(L.LIB_PATH.parent / "fused_cache").encode())


def test_native_source_rejects_invalid_program():
    prog = _lib.BqFusedProgram()
    prog.n_ins = 1
    prog.ins[0] = 999   # bad opcode
    n = __import__("ctypes").c_int64()
    assert _lib.load().bq_fused_source(prog, None, 0, n) == _lib.BQ_EINVAL
    assert _lib.load().bq_fused_compile(prog) == _lib.BQ_EINVAL
