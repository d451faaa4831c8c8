"""Test helpers for binquant_amd.fused: a numpy interpreter of the
bq_fused_eval bytecode (checks the program builder on CPU) and a direct
torch evaluation of an Ex DAG (the unfused arithmetic the kernel must equal)."""

import numpy as np
import torch

from binquant_amd import _lib
from binquant_amd import fused as F

OPN = {v: k for k, v in _lib.FUSED_OPS.items()}


def _operand_array(t: torch.Tensor, S: int, T: int) -> np.ndarray:
    a = t.detach().cpu()
    a = a.to(torch.float64) if a.dtype == torch.bool else a
    a = a.numpy()
    if a.ndim == 1:
        a = a[None, :]
    return np.broadcast_to(a, (S, T))


def interpret(P: F.Program, S: int, T: int) -> dict:
    """Run the bytecode on the host (numpy, vectorised over elements)."""
    R = [None] * max(P.n_regs, 1)
    ins_ = [_operand_array(t, S, T) for t in P.inputs]
    tt = np.arange(T)[None, :].repeat(S, 0)
    out = {}
    with np.errstate(all="ignore"):
        for w in P.ins:
            op = OPN[w & 0xFF]
            d, a, b, c = (w >> 8) & 0xFF, (w >> 16) & 0xFF, (w >> 24) & 0xFF, (w >> 32) & 0xFF
            imm = (w >> 40) & 0xFFFFFF
            imm = imm - (1 << 24) if imm >= (1 << 23) else imm
            if op == "LD":
                ts = tt - imm
                ok = (ts >= 0) & (ts < T)
                src = ins_[b]
                v = np.where(ok, src[np.arange(S)[:, None], np.clip(ts, 0, T - 1)], P.consts[c])
            elif op == "CONST":
                v = np.full((S, T), P.consts[imm])
            elif op == "INRANGE":
                v = (((tt - imm) >= 0) & ((tt - imm) < T)).astype(np.float64)
            elif op == "ST":
                name, kind = P.outputs[imm]
                out[name] = R[a] != 0 if kind == "b" else R[a].copy()
                continue
            else:
                opd = [P.consts[i] if (imm >> k) & 1 else R[i] for k, i in enumerate((a, b, c))
                       if (imm >> k) & 1 or R[i] is not None]
                opd += [None] * (3 - len(opd))
                x, y, z = (np.broadcast_to(np.asarray(v, dtype=np.float64), (S, T)) if v is not None else None
                           for v in opd)
                v = {
                    "ADD": lambda: x + y, "SUB": lambda: x - y, "MUL": lambda: x * y, "DIV": lambda: x / y,
                    "FMAX": lambda: np.fmax(x, y), "FMIN": lambda: np.fmin(x, y),
                    "MAXIMUM": lambda: np.maximum(x, y), "MINIMUM": lambda: np.minimum(x, y),
                    "GT": lambda: (x > y) * 1.0, "GE": lambda: (x >= y) * 1.0, "LT": lambda: (x < y) * 1.0,
                    "LE": lambda: (x <= y) * 1.0, "EQ": lambda: (x == y) * 1.0, "NE": lambda: (x != y) * 1.0,
                    "AND": lambda: ((x != 0) & (y != 0)) * 1.0, "OR": lambda: ((x != 0) | (y != 0)) * 1.0,
                    "NOT": lambda: (x == 0) * 1.0, "ABS": lambda: np.abs(x), "NEG": lambda: -x,
                    "ISNAN": lambda: np.isnan(x) * 1.0, "SQRT": lambda: np.sqrt(x), "LOG": lambda: np.log(x),
                    "WHERE": lambda: np.where(x != 0, y, z),
                }[op]()
            R[d] = np.asarray(v, dtype=np.float64)
    return out


def torch_eval(e: F.Ex, S: int, T: int, device="cpu") -> torch.Tensor:
    """The unfused evaluation of an Ex with torch ops (one tensor per node)."""
    memo = {}

    def ev(n):
        if id(n) in memo:
            return memo[id(n)]
        if n.op == "LD":
            t = n.tensor.to(device)
            t = t.to(torch.float64) if t.dtype == torch.bool else t
            t = (t[None, :] if t.dim() == 1 else t).expand(S, T)
            r = torch.full((S, T), n.value, dtype=torch.float64, device=device)
            k = n.shift
            if 0 <= k < T:
                r[:, k:] = t[:, :T - k]
            elif -T < k < 0:
                r[:, :T + k] = t[:, -k:]
        elif n.op == "CONST":
            r = torch.full((S, T), n.value, dtype=torch.float64, device=device)
        elif n.op == "INRANGE":
            tt = torch.arange(T, device=device).expand(S, T) - n.shift
            r = ((tt >= 0) & (tt < T)).to(torch.float64)
        else:
            a = [ev(x) for x in n.args]
            f = {
                "ADD": lambda: a[0] + a[1], "SUB": lambda: a[0] - a[1], "MUL": lambda: a[0] * a[1],
                "DIV": lambda: a[0] / a[1], "FMAX": lambda: torch.fmax(a[0], a[1]),
                "FMIN": lambda: torch.fmin(a[0], a[1]), "MAXIMUM": lambda: torch.maximum(a[0], a[1]),
                "MINIMUM": lambda: torch.minimum(a[0], a[1]),
                "GT": lambda: (a[0] > a[1]).double(), "GE": lambda: (a[0] >= a[1]).double(),
                "LT": lambda: (a[0] < a[1]).double(), "LE": lambda: (a[0] <= a[1]).double(),
                "EQ": lambda: (a[0] == a[1]).double(), "NE": lambda: (a[0] != a[1]).double(),
                "AND": lambda: ((a[0] != 0) & (a[1] != 0)).double(),
                "OR": lambda: ((a[0] != 0) | (a[1] != 0)).double(), "NOT": lambda: (a[0] == 0).double(),
                "ABS": lambda: a[0].abs(), "NEG": lambda: -a[0], "ISNAN": lambda: torch.isnan(a[0]).double(),
                "SQRT": lambda: torch.sqrt(a[0]), "LOG": lambda: torch.log(a[0]),
                "WHERE": lambda: torch.where(a[0] != 0, a[1], a[2]),
            }[n.op]
            r = f()
        memo[id(n)] = r
        return r

    r = ev(e.node)
    return r != 0 if e.kind == "b" else r


def assert_same(name, got, want):
    """Bit-identical (the log expression: within 2 ulp — libm log is not
    correctly rounded, so two libraries may differ in the last place)."""
    got, want = np.asarray(got), np.asarray(want)
    if want.dtype == bool:
        np.testing.assert_array_equal(got, want, err_msg=name)
    elif name in ("log", "sqrt"):   # host torch uses SLEEF vector sqrt (0.5001 ulp)
        np.testing.assert_allclose(got, want, rtol=5e-16, atol=5e-16, err_msg=name)
    else:
        np.testing.assert_array_equal(got, want, err_msg=name)
        num = ~np.isnan(want)
        assert np.array_equal(np.signbit(got[num]), np.signbit(want[num])), name   # -0.0 kept


def random_panel(S, T, seed=0, nan_frac=0.05):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(S, T, generator=g, dtype=torch.float64)
    x[torch.rand(S, T, generator=g) < nan_frac] = float("nan")
    x[torch.rand(S, T, generator=g) < 0.02] = 0.0
    x[0, :3] = torch.tensor([float("inf"), -float("inf"), -0.0], dtype=torch.float64)
    return x


def expressions(x, y, z, b, row, col):
    """A battery of expressions over every op, shifts of computed values,
    broadcasts and shared subexpressions."""
    X, Y, Z, B, Rw, C = (F.inp(t) for t in (x, y, z, b, row, col))
    s = X / (Y + 1e-6)
    ex = {
        "arith": (X + Y) * Z - X / Y,
        "rev": 1 - 2.5 * X + 3 / Y,
        "minmax": F.fmax(F.fmax(X - Y, (X - F.shift(Z, 1)).abs()), (Y - F.shift(Z, 1)).abs()),
        "maxnan": F.maximum(X, Y) - F.minimum(Y, Z),
        "cmp": (X > Y) & ~(Y <= Z) | (X == 0) | (Z != Y) & (X >= 1) | (Y < -1),
        "where": F.where(X < 0.5, 0.5, X),
        "isnan": F.isnan(X) | F.isnan(s),
        "shift_expr": F.shift(s, 3) - s,
        "shift_neg": F.shift(X * Y, -2),
        "shift_bool": F.shift(B & (X > 0), 1) & ~F.shift(B, -1),
        "nested": F.shift(F.shift(X + 1, 1) * Y, 2),
        "diff": F.diff(s, 3),
        "row": X / Rw + C,
        "row_shift": F.shift(Rw * X, 1),
        "sqrt": F.sqrt(F.fmax(X, 0.0)) + Y,
        "log": F.log(F.fmax(Y, 1e-9)),   # libm log: not correctly rounded, compared to 1 ulp
        "clip": F.clip_lower(X, 0.0) / F.replace0(Y),
        "fillna": F.fillna(s, 0.0),
        "float": (X > Y).float() + (Y > Z).float(),
        "bool_in": B,
        "const_out": F.const(1.0) + 0.0,
        "shared": s * s + s,
    }
    return ex
