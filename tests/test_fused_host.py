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


def _same_programs(a, b):
    assert len(a) == len(b)
    for p, q in zip(a, b):
        assert list(p.ins) == list(q.ins) and list(p.consts) == list(q.consts)
        assert (p.n_loads, p.n_regs, p.outputs) == (q.n_loads, q.n_regs, q.outputs)
        assert len(p.inputs) == len(q.inputs) and all(s is t for s, t in zip(p.inputs, q.inputs))


def test_plan_cache_rebinds_operands_exactly():
    """A cached plan equals a fresh build for a new request of the same
    structure (new tensors, new output names); operand aliasing and constant
    values are part of the key."""
    F.clear_plan_cache()
    items = list(expressions(*_operands()).items())
    _same_programs(F._plan_cached(items), F._plan(items))
    assert F.plan_cache_stats()["misses"] == 1
    # same structure over other tensors and names: a hit, equal to a fresh build
    ops2 = [random_panel(S, T, seed=k + 20) for k in range(3)] + list(_operands()[3:])
    items2 = [(name + "_2", e) for name, e in expressions(*ops2).items()]
    got = F._plan_cached(items2)
    assert F.plan_cache_stats()["hits"] == 1
    _same_programs(got, F._plan(items2))
    res = {}
    for P in got:
        res.update(interpret(P, S, T))
    for name, e in items2:
        assert_same(name[:-2], res[name], torch_eval(e, S, T).numpy())
    # aliasing changes the program (one operand instead of two): a miss
    x, y = random_panel(S, T, seed=1), random_panel(S, T, seed=2)
    F._plan_cached([("s", F.inp(x) + F.inp(y))])
    m = F.plan_cache_stats()["misses"]
    P = F._plan_cached([("s", F.inp(x) + F.inp(x))])
    assert F.plan_cache_stats()["misses"] == m + 1 and len(P[0].inputs) == 1
    np.testing.assert_array_equal(interpret(P[0], S, T)["s"], (x + x).numpy())
    # a new constant value is a new key
    F._plan_cached([("s", F.inp(x) * 2.0)])
    P = F._plan_cached([("s", F.inp(y) * 3.0)])
    assert F.plan_cache_stats()["misses"] == m + 3
    np.testing.assert_array_equal(interpret(P[0], S, T)["s"], (y * 3.0).numpy())
    P = F._plan_cached([("t", F.inp(x) * 3.0)])
    assert F.plan_cache_stats()["misses"] == m + 3 and P[0].inputs[0] is x
