"""bq_fused_eval on the device: every expression of the battery equals the
unfused torch evaluation of the same operations on the same device bit for
bit; one run() with all of them (several programs); the program checks."""

import ctypes

import numpy as np
import pytest
import torch

from binquant_amd import _lib
from binquant_amd import fused as F
from fused_util import assert_same, expressions, random_panel, torch_eval

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["native", "interp"])
def mode(request):
    """Both evaluations of a program: the hiprtc-compiled kernel and the
    LDS-register interpreter."""
    prev = F.set_native(request.param == "native")
    yield request.param
    F.set_native(None if prev < 0 else bool(prev))


def _operands(S, T, dev):
    x, y, z = (random_panel(S, T, seed=k).to(dev) for k in range(3))
    b = (torch.rand(S, T, generator=torch.Generator().manual_seed(9)) < 0.5).to(dev)
    row = (torch.rand(S, 1, dtype=torch.float64, generator=torch.Generator().manual_seed(4)) + 0.5).to(dev)
    col = torch.randn(T, dtype=torch.float64, generator=torch.Generator().manual_seed(5)).to(dev)
    return x, y, z, b, row, col


@pytest.mark.parametrize("S,T", [(5, 37), (70, 600)])
def test_each_expression_matches_torch(cuda, mode, S, T):
    ex = expressions(*_operands(S, T, "cuda"))
    for name, e in ex.items():
        got = F.run({name: e}, S, T)[name]
        want = torch_eval(e, S, T, device="cuda")
        assert got.dtype == want.dtype and tuple(got.shape) == (S, T), name
        assert_same(name, got.cpu().numpy(), want.cpu().numpy())


def test_all_outputs_in_one_call(cuda, mode):
    S, T = 33, 300
    ex = expressions(*_operands(S, T, "cuda"))
    got = F.run(ex, S, T)
    for name, e in ex.items():
        assert_same(name, got[name].cpu().numpy(), torch_eval(e, S, T, device="cuda").cpu().numpy())


def test_strided_operands_and_identity(cuda):
    S, T = 9, 120
    big = random_panel(S, 2 * T).cuda()
    view = big[:, ::2]                     # stride_t 2
    sl = big[:, 5:5 + T]                   # row stride 2T
    e = F.inp(view) * 2 + F.shift(F.inp(sl), 1)
    got = F.run({"y": e, "same": F.inp(sl)})
    want = view * 2 + torch.cat([torch.full((S, 1), float("nan"), device="cuda", dtype=torch.float64),
                                 sl[:, :-1]], 1)
    np.testing.assert_array_equal(got["y"].cpu().numpy(), want.cpu().numpy())
    assert got["same"] is sl


def test_invalid_programs_are_rejected(cuda):
    lib = _lib.load()
    x = torch.zeros(2, 4, dtype=torch.float64, device="cuda")
    P = F.build([("y", F.inp(x) + 1.0)])

    def launch(mut):
        prog = _lib.BqFusedProgram()
        prog.n_ins, prog.n_loads, prog.n_regs = len(P.ins), P.n_loads, P.n_regs
        prog.n_in, prog.n_out, prog.n_const = 1, 1, len(P.consts)
        for i, w in enumerate(P.ins):
            prog.ins[i] = w
        for i, v in enumerate(P.consts):
            prog.consts[i] = v
        prog.inp[0] = _lib.BqFusedOperand(ctypes.c_void_p(x.data_ptr()), 4, 1, 0, 0)
        prog.out[0] = _lib.BqFusedOperand(ctypes.c_void_p(x.data_ptr()), 4, 1, 0, 0)
        mut(prog)
        return lib.bq_fused_eval(ctypes.byref(prog), 2, 4, None)

    assert launch(lambda p: None) == 0
    torch.cuda.synchronize()
    assert launch(lambda p: setattr(p, "n_regs", _lib.FUSED_MAX_REGS + 1)) != 0
    assert launch(lambda p: setattr(p, "n_in", 0)) != 0                      # LD of a missing operand
    assert launch(lambda p: p.ins.__setitem__(0, 99)) != 0                   # unknown opcode
    assert launch(lambda p: setattr(p, "n_loads", 2)) != 0                   # a non-load in the load block
    assert launch(lambda p: setattr(p, "n_const", 0)) != 0                   # constant index out of range


@pytest.mark.parametrize("S,T", [(3, 5), (40, 1100), (24, 4099)])
def test_native_equals_interpreter_bits(cuda, S, T):
    """Long rows take the 2- and 4-candles-per-thread forms of both
    evaluations; the compiled kernel reproduces the interpreter's bits
    (signed zeros included) for every output."""
    ex = expressions(*_operands(S, T, "cuda"))
    prev = F.set_native(False)
    try:
        ref = F.run(ex, S, T)
        F.set_native(True)
        before = F.native_stats()
        got = F.run(ex, S, T)
        st = F.native_stats()
        assert st["cached"] >= 1 and st["compiles"] + st["disk_hits"] >= before["compiles"] + before["disk_hits"]
    finally:
        F.set_native(None if prev < 0 else bool(prev))
    for name in ex:
        a, b = got[name], ref[name]
        if a.dtype == torch.float64:
            # a NaN's sign bit is not a value (the compiler may fold a
            # negation into a constant): NaN where the interpreter has NaN,
            # identical bits everywhere else
            nan = torch.isnan(b)
            assert torch.equal(torch.isnan(a), nan), name
            a, b = a[~nan].view(torch.int64), b[~nan].view(torch.int64)
        assert torch.equal(a, b), name


def test_native_constants_are_arguments(cuda):
    """A stage re-run with new constant values (thresholds that change per
    message) reuses its compiled kernel and uses the new values exactly."""
    F.set_native(True)
    try:
        S, T = 16, 300
        x = random_panel(S, T, seed=3).cuda()
        X = F.inp(x)
        F.run({"y": F.where(X > 0.25, X * 1.5, -X) + 1e-3}, S, T)
        before = F.native_stats()
        for thr, k, c in ((0.5, 2.0, 0.125), (-1.0, 1.0 / 3.0, 7.0)):
            got = F.run({"y": F.where(X > thr, X * k, -X) + c}, S, T)["y"]
            want = torch.where(x > thr, x * k, -x) + c
            assert_same("y", got.cpu().numpy(), want.cpu().numpy())
        after = F.native_stats()
        assert after["compiles"] == before["compiles"] and after["cached"] == before["cached"]
    finally:
        F.set_native(None)


def test_stream_handle_is_torch_current_stream(cuda):
    """The launch stream read through the raw accessor is torch's current
    stream, including inside a `torch.cuda.stream` context."""
    from binquant_amd import engine

    h = lambda st: engine._stream_handle(st).value or 0   # noqa: E731  (c_void_p(0).value is None)
    assert h(None) == torch.cuda.current_stream().cuda_stream
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        assert h(None) == s.cuda_stream != 0
    assert h(s) == s.cuda_stream
