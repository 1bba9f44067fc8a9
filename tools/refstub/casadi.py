"""Sympy-backed stand-in for the tiny CasADi subset the reference's model code touches.

TEST TOOL ONLY (used by tools/gen_golden.py in the build container, never shipped, never on
the product path).  It lets the reference's own ``blasterModel.generateModel()`` build its
symbolic f(x, u, p) so golden vectors can be evaluated from the reference's expressions.
Covers: SX.sym/eye/zeros/SX(list)/SX(n, m), element get/set, + - * / @ (also ndarray @ SX),
sin, cos, inv, cross, vertcat, reshape (column-major), rows/columns/size.
"""
import numpy as _np
import sympy as _sp


class SX:
    __array_ufunc__ = None  # make ``ndarray @ SX`` defer to SX.__rmatmul__

    def __init__(self, *args):
        if len(args) == 0:
            self.M = _sp.zeros(1, 1)
        elif len(args) == 1:
            a = args[0]
            if isinstance(a, SX):
                self.M = a.M.copy()
            elif isinstance(a, _sp.MatrixBase):
                self.M = _sp.Matrix(a)
            elif isinstance(a, (list, tuple, _np.ndarray)):
                arr = _np.asarray(a, dtype=object)
                if arr.ndim == 1:
                    self.M = _sp.Matrix([[_sp.sympify(v)] for v in arr])
                else:
                    self.M = _sp.Matrix(arr.tolist())
            else:
                self.M = _sp.Matrix([[_sp.sympify(a)]])
        else:
            self.M = _sp.zeros(int(args[0]), int(args[1]))

    # construction -------------------------------------------------------------------------
    @staticmethod
    def sym(name, n=1, m=1):
        return SX(_sp.Matrix(n, m, lambda i, j: _sp.Dummy(f'{name}_{i}_{j}')))

    @staticmethod
    def eye(n):
        return SX(_sp.eye(n))

    @staticmethod
    def zeros(n, m=1):
        return SX(_sp.zeros(n, m))

    # shape --------------------------------------------------------------------------------
    def rows(self):
        return self.M.rows

    def columns(self):
        return self.M.cols

    def size(self):
        return (self.M.rows, self.M.cols)

    @property
    def shape(self):
        return (self.M.rows, self.M.cols)

    # element access -----------------------------------------------------------------------
    def _idx(self, k):
        if isinstance(k, tuple):
            return k
        # linear index, column-major like CasADi
        return (k % self.M.rows, k // self.M.rows)

    def __getitem__(self, k):
        i, j = self._idx(k)
        return SX(_sp.Matrix([[self.M[i, j]]]))

    def __setitem__(self, k, v):
        i, j = self._idx(k)
        self.M[i, j] = _lift(v).M[0, 0]

    # arithmetic ---------------------------------------------------------------------------
    def _bin(self, o, op):
        o = _lift(o)
        a, b = self.M, o.M
        if a.shape == (1, 1) and b.shape != (1, 1):
            return SX(b.applyfunc(lambda e: op(a[0, 0], e)))
        if b.shape == (1, 1) and a.shape != (1, 1):
            return SX(a.applyfunc(lambda e: op(e, b[0, 0])))
        return SX(_sp.Matrix(a.rows, a.cols, lambda i, j: op(a[i, j], b[i, j])))

    def __add__(self, o): return self._bin(o, lambda x, y: x + y)
    def __radd__(self, o): return _lift(o)._bin(self, lambda x, y: x + y)
    def __sub__(self, o): return self._bin(o, lambda x, y: x - y)
    def __rsub__(self, o): return _lift(o)._bin(self, lambda x, y: x - y)
    def __mul__(self, o): return self._bin(o, lambda x, y: x * y)
    def __rmul__(self, o): return _lift(o)._bin(self, lambda x, y: x * y)
    def __truediv__(self, o): return self._bin(o, lambda x, y: x / y)
    def __rtruediv__(self, o): return _lift(o)._bin(self, lambda x, y: x / y)
    def __neg__(self): return SX(-self.M)
    def __pow__(self, k): return SX(self.M.applyfunc(lambda e: e ** k))

    def __matmul__(self, o):
        return SX(self.M * _lift(o).M)

    def __rmatmul__(self, o):
        return SX(_lift(o).M * self.M)


def _lift(v):
    if isinstance(v, SX):
        return v
    if isinstance(v, _np.ndarray):
        return SX(v.astype(object) if v.ndim == 2 else v)
    return SX(v)


def sin(x): return SX(_lift(x).M.applyfunc(_sp.sin))
def cos(x): return SX(_lift(x).M.applyfunc(_sp.cos))
def inv(x): return SX(_lift(x).M.inv())


def cross(a, b):
    a, b = _lift(a).M, _lift(b).M
    return SX(_sp.Matrix([a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]]))


def vertcat(*xs):
    mats = [_lift(x).M for x in xs]
    return SX(_sp.Matrix.vstack(*mats))


def reshape(x, n, m):
    M = _lift(x).M
    flat = [M[i, j] for j in range(M.cols) for i in range(M.rows)]  # column-major
    return SX(_sp.Matrix(m, n, flat).T)


__all__ = ['SX', 'sin', 'cos', 'inv', 'cross', 'vertcat', 'reshape']
