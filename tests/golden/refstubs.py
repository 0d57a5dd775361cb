"""Stub modules that let the reference's own Python run in THIS container (fixture generation only).

The reference (/root/reference) imports cvxpy, hppfcl, pinocchio, meshcat and polytope, none
of which is installed here (ordinary ModuleNotFoundError -- nothing is refused).  To pin the
oracle against the reference's *own* code we install, in ``sys.modules``:

  * meshcat, meshcat.geometry, meshcat.transformations, polytope -- inert (display only);
  * pinocchio -- the four closed-form Lie operations the path uses (skew, skewSquare, exp3,
    unSkew) plus ``pinocchio.utils.rotate``;
  * hppfcl -- Capsule / Cylinder / Transform3f / distance, answered by the oracle's
    brute-force geometry (so hppfcl parity itself stays unpinned, as documented);
  * cvxpy -- a *tracing* modelling layer: Variables, Parameters and the affine atoms the
    reference uses are recorded; ``Problem.solve`` evaluates the model at the current
    parameter values into (P, q, A, b, G, h, cones), records it, and answers it with the
    oracle IPM (Clarabel is absent).  What this pins is the reference's own problem
    formulation and outer-loop code, not Clarabel.

This file is test infrastructure: it is imported only by ``tests/golden/make_golden.py``
(run in the dev container, never on the GPU box) and contains no reference source.
"""

from __future__ import annotations

import sys
import time
import types

import numpy as np

from oracle import forest as oforest
from oracle import ipm as oipm
from oracle import model as omodel

# ============================================================================ cvxpy tracing stub
_REGISTRY = []  # all Variables in creation order
TRACE = []      # recorded problem data of every Problem.solve
_NX = [0]       # total size of the registered Variables (kept in step with _REGISTRY)


def _nx():
    return _NX[0]


class Expr:
    __array_ufunc__ = None  # make numpy defer to our reflected operators
    __array_priority__ = 1000

    def __init__(self, shape, ev):
        self.shape = tuple(shape)
        self._ev = ev  # () -> (coef[*shape, nx], const[*shape])

    # -- evaluation
    def ev(self):
        return self._ev()

    @property
    def size(self):
        n = 1
        for d in self.shape:
            n *= int(d)
        return n

    @property
    def ndim(self):
        return len(self.shape)

    # -- arithmetic
    def __add__(self, o):
        if isinstance(o, Quad):
            return o + self
        o = _wrap(o)
        shp = np.broadcast_shapes(self.shape, o.shape)

        def ev():
            (ca, ka), (cb, kb) = self.ev(), o.ev()
            nx = _nx()
            ca, cb = _pad(ca, nx), _pad(cb, nx)
            return (np.broadcast_to(ca, shp + (nx,)) + np.broadcast_to(cb, shp + (nx,)),
                    np.broadcast_to(ka, shp) + np.broadcast_to(kb, shp))

        return Expr(shp, ev)

    __radd__ = __add__

    def __neg__(self):
        def ev():
            c, k = self.ev()
            return -c, -k

        return Expr(self.shape, ev)

    def __sub__(self, o):
        if isinstance(o, Quad):
            return o * (-1.0) + self
        return self + (-_wrap(o))

    def __rsub__(self, o):
        return _wrap(o) + (-self)

    def __mul__(self, o):
        if isinstance(o, Quad):
            return o.__rmul__(self)
        o = _wrap(o)
        if o.shape == () or self.shape == ():
            shp = np.broadcast_shapes(self.shape, o.shape)

            def ev():
                (ca, ka), (cb, kb) = self.ev(), o.ev()
                nx = _nx()
                ca, cb = _pad(ca, nx), _pad(cb, nx)
                if not np.any(cb):  # o constant
                    return ca * np.asarray(kb)[..., None], ka * kb
                if not np.any(ca):
                    return cb * np.asarray(ka)[..., None], ka * kb
                raise ValueError("non-affine product")

            return Expr(shp, ev)
        raise ValueError("use cv.multiply / @ for array products")

    __rmul__ = __mul__

    def __truediv__(self, o):
        return self * (1.0 / float(o))

    def __matmul__(self, o):
        return _matmul(self, _wrap(o))

    def __rmatmul__(self, o):
        return _matmul(_wrap(o), self)

    def __getitem__(self, idx):
        probe = np.empty(self.shape)[idx]

        def ev():
            c, k = self.ev()
            return c[idx + (slice(None),) if isinstance(idx, tuple) else (idx, slice(None))], np.asarray(k)[idx]

        return Expr(probe.shape, ev)

    @property
    def T(self):
        if self.ndim < 2:
            return self

        def ev():
            c, k = self.ev()
            return np.swapaxes(c, 0, 1), np.asarray(k).T

        return Expr(self.shape[::-1], ev)

    def reshape(self, shape, order="F"):
        def ev():
            c, k = self.ev()
            nx = c.shape[-1]
            nd = c.ndim - 1
            cf = np.transpose(c, tuple(range(nd - 1, -1, -1)) + (nd,)).reshape(-1, nx)  # F-order rows
            c2 = cf.reshape(tuple(shape)[::-1] + (nx,))
            c2 = np.transpose(c2, tuple(range(len(shape) - 1, -1, -1)) + (len(shape),))
            return c2, np.asarray(k).reshape(-1, order="F").reshape(shape, order="F")

        return Expr(shape, ev)

    # -- constraints
    def __eq__(self, o):
        return Constraint("eq", self - _wrap(o))

    def __ge__(self, o):
        return Constraint("ge", self - _wrap(o))

    def __le__(self, o):
        return Constraint("ge", _wrap(o) - self)

    __hash__ = object.__hash__


def _pad(c, nx):
    if c.shape[-1] < nx:
        c = np.concatenate([c, np.zeros(c.shape[:-1] + (nx - c.shape[-1],))], axis=-1)
    return c


def _wrap(o):
    if isinstance(o, (Expr, Quad)):
        return o
    val = np.asarray(o, dtype=float)
    return Expr(val.shape, lambda: (np.zeros(val.shape + (_nx(),)), val))


def _matmul(a: Expr, b: Expr):
    probe = np.empty(a.shape) @ np.empty(b.shape) if (a.shape and b.shape) else None
    shp = probe.shape if probe is not None else ()

    def ev():
        (ca, ka), (cb, kb) = a.ev(), b.ev()
        nx = _nx()
        ca, cb = _pad(ca, nx), _pad(cb, nx)
        if not np.any(ca):
            A = np.asarray(ka)
            if b.ndim == 1:
                coef = np.einsum("...k,kx->...x", A, cb)
            else:
                coef = np.einsum("...k,knx->...nx", A, cb)
            return coef, A @ kb
        if not np.any(cb):
            Bm = np.asarray(kb)
            if a.ndim == 1:
                coef = np.einsum("kx,k...->...x", ca, Bm)
            else:
                coef = np.einsum("mkx,k...->m...x", ca, Bm)
            return coef, ka @ Bm
        raise ValueError("non-affine matmul")

    return Expr(shp, ev)


class Variable(Expr):
    def __init__(self, shape=()):
        shape = (shape,) if isinstance(shape, int) else tuple(shape)
        self.offset = _nx()
        self._value = None
        size = int(np.prod(shape)) if shape else 1
        sz = size

        def ev():
            nx = _nx()
            c = np.zeros((sz, nx))
            c[np.arange(sz), self.offset + np.arange(sz)] = 1.0
            # variables vectorise column-major (cvxpy convention)
            if shape:
                c = c.reshape(shape[::-1] + (nx,))
                c = np.transpose(c, tuple(range(len(shape) - 1, -1, -1)) + (len(shape),))
            else:
                c = c[0]
            return c, np.zeros(shape)

        super().__init__(shape, ev)
        _REGISTRY.append(self)
        _NX[0] += self.size

    @property
    def value(self):
        return self._value

    @value.setter
    def value(self, v):
        self._value = None if v is None else np.asarray(v, float)


class Parameter(Expr):
    def __init__(self, shape=(), nonneg=False):
        shape = (shape,) if isinstance(shape, int) else tuple(shape)
        self._value = None
        super().__init__(shape, lambda: (np.zeros(tuple(shape) + (_nx(),)), np.asarray(self._value, float)))

    @property
    def value(self):
        return self._value

    @value.setter
    def value(self, v):
        self._value = np.array(v, dtype=float)


class Norm2:
    def __init__(self, e: Expr, axis=None):
        self.e, self.axis = e, axis

    def __le__(self, t):
        return Constraint("soc", (self.e, _wrap(t), self.axis))


class Quad:
    """sum_k w_k ||e_k||^2 + affine scalar."""

    def __init__(self, terms=None, lin=None):
        self.terms = terms or []
        self.lin = lin

    def __add__(self, o):
        if isinstance(o, (int, float)) and o == 0:
            return self
        if isinstance(o, Quad):
            lin = o.lin if self.lin is None else (self.lin if o.lin is None else self.lin + o.lin)
            return Quad(self.terms + o.terms, lin)
        o = _wrap(o)
        return Quad(self.terms, o if self.lin is None else self.lin + o)

    __radd__ = __add__

    def __sub__(self, o):
        return self + (-1.0) * o

    def __mul__(self, k):
        k = _wrap(k)
        return Quad([(w * k, e) for (w, e) in self.terms], None if self.lin is None else self.lin * k)

    __rmul__ = __mul__


def sum_squares(e):
    return Quad([(_wrap(1.0), _wrap(e))])


def _sum(e, axis=None):
    e = _wrap(e)

    def ev():
        c, k = e.ev()
        if axis is None:
            return c.reshape(-1, c.shape[-1]).sum(0), np.asarray(k).sum()
        return c.sum(axis), np.asarray(k).sum(axis)

    shp = () if axis is None else tuple(d for i, d in enumerate(e.shape) if i != axis)
    return Expr(shp, ev)


def multiply(a, b):
    a, b = _wrap(a), _wrap(b)
    shp = np.broadcast_shapes(a.shape, b.shape)

    def ev():
        (ca, ka), (cb, kb) = a.ev(), b.ev()
        nx = _nx()
        ca, cb = _pad(ca, nx), _pad(cb, nx)
        if not np.any(ca):
            return cb * np.asarray(ka)[..., None], ka * kb
        if not np.any(cb):
            return ca * np.asarray(kb)[..., None], ka * kb
        raise ValueError("non-affine multiply")

    return Expr(shp, ev)


class Constraint:
    def __init__(self, kind, data):
        self.kind, self.data = kind, data


class Minimize:
    def __init__(self, obj):
        self.obj = obj if isinstance(obj, Quad) else Quad([], _wrap(obj))


class _Stats:
    solve_time = 0.0


class Problem:
    def __init__(self, objective, constraints):
        self.objective, self.constraints = objective, list(constraints)
        self.status = None
        self.solver_stats = _Stats()
        self._vars = None

    def is_dcp(self):
        return True

    def data(self):
        nx = _nx()
        P = np.zeros((nx, nx))
        q = np.zeros(nx)
        for w, e in self.objective.obj.terms:
            cw, kw = w.ev()
            assert not np.any(cw)
            c, k = e.ev()
            C = _pad(c, nx).reshape(-1, nx)
            k = np.asarray(k).reshape(-1)
            P += 2.0 * float(kw) * C.T @ C
            q += 2.0 * float(kw) * C.T @ k
        if self.objective.obj.lin is not None:
            c, _ = self.objective.obj.lin.ev()
            q += _pad(c, nx).reshape(nx)
        A, b, Gl, hl, Gq, hq = [], [], [], [], [], []
        for con in self.constraints:
            if con.kind == "eq":
                c, k = con.data.ev()
                A.append(_pad(c, nx).reshape(-1, nx))
                b.append(-np.asarray(k).reshape(-1))
            elif con.kind == "ge":
                c, k = con.data.ev()
                Gl.append(-_pad(c, nx).reshape(-1, nx))
                hl.append(np.asarray(k).reshape(-1))
            else:
                e, t, axis = con.data
                ce, ke = e.ev()
                ct, kt = t.ev()
                ce, ct = _pad(ce, nx), _pad(ct, nx)
                ke, kt = np.asarray(ke), np.asarray(kt)
                if axis is None:
                    cols = [(ce.reshape(-1, nx), ke.reshape(-1), ct.reshape(nx), float(kt))]
                else:
                    cols = [(ce[:, j, :], ke[:, j], np.broadcast_to(ct, (e.shape[1], nx))[j],
                             float(np.broadcast_to(kt, (e.shape[1],))[j])) for j in range(e.shape[1])]
                for cx, kx, ctt, ktt in cols:
                    Gq.append(-np.vstack([ctt[None, :], cx]))
                    hq.append(np.concatenate([[ktt], kx]))
        # restrict to this problem's variables
        used = np.zeros(nx, bool)
        for M in [P] + A + Gl + Gq:
            used |= np.any(M != 0, axis=0)
        lo = min(np.nonzero(used)[0]) if used.any() else 0
        hi = max(np.nonzero(used)[0]) + 1 if used.any() else 0
        vs = [v for v in _REGISTRY if lo <= v.offset < hi or (v.offset < lo < v.offset + v.size)]
        lo = min(v.offset for v in vs)
        hi = max(v.offset + v.size for v in vs)
        sl = slice(lo, hi)
        self._vars = vs
        G_ = np.vstack([g[:, sl] for g in Gl] + [g[:, sl] for g in Gq])
        h_ = np.concatenate(hl + hq)
        dims = oipm.ConeDims(l=int(sum(g.shape[0] for g in Gl)), q=[g.shape[0] for g in Gq])
        return dict(P=P[sl, sl], q=q[sl], A=np.vstack(A)[:, sl], b=np.concatenate(b), G=G_, h=h_,
                    l=dims.l, q_dims=np.array(dims.q), lo=lo), dims

    def solve(self, solver=None, warm_start=True, **kw):
        d, dims = self.data()
        t0 = time.perf_counter()
        # drop rows 0'x >= 0 (no information; see oracle.model.build_qp)
        keep = np.ones(d["G"].shape[0], bool)
        keep[: dims.l] = np.any(d["G"][: dims.l] != 0, axis=1) | (d["h"][: dims.l] != 0)
        G_, h_ = d["G"][keep], d["h"][keep]
        dims2 = oipm.ConeDims(l=int(keep[: dims.l].sum()), q=list(dims.q))
        r = oipm.solve_qp(d["P"], d["q"], G_, h_, dims2, d["A"], d["b"])
        self.solver_stats.solve_time = time.perf_counter() - t0
        TRACE.append(dict(d, x=r.x, status=r.status, iters=r.iters))
        if r.status == oipm.OPTIMAL:
            self.status = OPTIMAL
            off = d["lo"]
            for v in self._vars:
                val = r.x[v.offset - off : v.offset - off + v.size]
                v.value = val.reshape(v.shape, order="F") if v.shape else val[0]
        else:
            self.status = "optimal_inaccurate" if r.status == oipm.MAX_ITER else "solver_error"
        return r.obj


OPTIMAL = "optimal"


def _make_cvxpy():
    m = types.ModuleType("cvxpy")
    m.Variable, m.Parameter, m.Problem, m.Minimize = Variable, Parameter, Problem, Minimize
    m.sum, m.sum_squares, m.multiply = _sum, sum_squares, multiply
    m.norm2 = lambda e, axis=None: Norm2(_wrap(e), axis)
    m.reshape = lambda e, shape, order="F": _wrap(e).reshape(shape, order)
    m.vstack = lambda xs: None
    m.Expression = Expr
    m.OPTIMAL = OPTIMAL
    m.CLARABEL, m.SCS, m.CVXOPT = "CLARABEL", "SCS", "CVXOPT"
    return m


# ============================================================================ pinocchio stub
def _make_pinocchio():
    m = types.ModuleType("pinocchio")
    m.skew = omodel.skew
    m.skewSquare = omodel.skew_sq
    m.exp3 = omodel.exp3
    m.unSkew = omodel.unskew
    u = types.ModuleType("pinocchio.utils")

    def rotate(axis, ang):
        v = {"x": [1.0, 0, 0], "y": [0, 1.0, 0], "z": [0, 0, 1.0]}[axis]
        return omodel.exp3(np.array(v) * ang)

    u.rotate = rotate
    m.utils = u
    return m, u


# ============================================================================ hppfcl stub
class _Capsule:
    def __init__(self, radius, lz):
        self.radius, self.lz = radius, lz


class _Cylinder:
    def __init__(self, radius, lz):
        self.radius, self.lz = radius, lz


class _Transform3f:
    def __init__(self):
        self.t = np.zeros(3)
        self.R = np.eye(3)

    def setTranslation(self, t):
        self.t = np.array(t, float)

    def setRotation(self, R):
        self.R = np.array(R, float)

    def getTranslation(self):
        return self.t


class _DistanceResult:
    def __init__(self):
        self.p1 = self.p2 = np.zeros(3)

    def getNearestPoint1(self):
        return self.p1

    def getNearestPoint2(self):
        return self.p2


def _distance(obj1, tf1, obj2, tf2, req, res):
    assert isinstance(obj1, _Capsule) and isinstance(obj2, _Cylinder)
    assert abs(obj2.radius - oforest.BARK_RADIUS) < 1e-15 and abs(obj2.lz - oforest.BARK_HEIGHT) < 1e-15
    axis = tf1.R @ np.array([0.0, 0.0, 1.0])
    x0 = tf1.t - 0.5 * obj1.lz * axis
    x1 = tf1.t + 0.5 * obj1.lz * axis
    d, p1, p2 = oforest.capsule_tree_distance(x0, x1, obj1.radius, tf2.getTranslation())
    res.p1, res.p2 = p1, p2
    return d


def _make_hppfcl():
    m = types.ModuleType("hppfcl")
    m.Capsule, m.Cylinder, m.Transform3f = _Capsule, _Cylinder, _Transform3f
    m.DistanceRequest = lambda *a, **k: object()
    m.DistanceResult = _DistanceResult
    m.distance = _distance
    return m


class _Inert:
    def __init__(self, *a, **k):
        pass

    def __call__(self, *a, **k):
        return _Inert()

    def __getattr__(self, k):
        return _Inert()

    def __getitem__(self, k):
        return _Inert()

    @classmethod
    def from_file(cls, *a, **k):
        return cls()


def _inert_module(name):
    m = types.ModuleType(name)
    m.__getattr__ = lambda k: _Inert
    return m


def install():
    """Install all stubs into sys.modules (idempotent)."""
    cv = _make_cvxpy()
    pin, pinu = _make_pinocchio()
    mods = {
        "cvxpy": cv,
        "pinocchio": pin,
        "pinocchio.utils": pinu,
        "hppfcl": _make_hppfcl(),
        "meshcat": _inert_module("meshcat"),
        "meshcat.geometry": _inert_module("meshcat.geometry"),
        "meshcat.transformations": _inert_module("meshcat.transformations"),
        "polytope": _inert_module("polytope"),
    }
    mods["meshcat"].geometry = mods["meshcat.geometry"]
    mods["meshcat"].transformations = mods["meshcat.transformations"]
    mods["meshcat"].Visualizer = _Inert
    sys.modules.update(mods)
