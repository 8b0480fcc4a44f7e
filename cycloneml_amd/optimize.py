"""Host-side first-order minimizers driving the device loss (the driver side of
LogisticRegression.train, ml/classification/LogisticRegression.scala:777-815,
999-1012).

The reference builds them from breeze 1.2 (`breeze_2.12:1.2`, pom.xml:929), an
external dependency that is not in /root/reference: `LBFGS(maxIter, 10, tol)`
for L2 / no regularization and `OWLQN(maxIter, 10, l1reg, tol)` when
elasticNetParam * regParam > 0.  This module restates breeze's published
algorithms (breeze.optimize.{FirstOrderMinimizer, LBFGS, OWLQN,
StrongWolfeLineSearch, BacktrackingLineSearch}):

- the iteration loop with one history reset after a failed step
  (FirstOrderMinimizer.infiniteIterations) and the default convergence check:
  maxIter, function values converged (|f - max of the last 20 f| <= tol |f0|),
  gradient converged (|adjGrad|_inf <= max(tol |f|, 1e-8)), search failed;
- the L-BFGS two-loop recursion over the last m (step, gradient delta) pairs
  with the sy / yy initial scaling (LBFGS.ApproximateInverseHessian);
- the strong-Wolfe line search (c1 = 1e-4, c2 = 0.9, cubic interpolation,
  10 bracketing and 10 zoom steps) from 1 / |dir| on the first iteration, 1
  afterwards;
- OWL-QN: the pseudo-gradient, the direction masked to the pseudo-gradient's
  orthant, the orthant projection of each step, and a backtracking line
  search on the adjusted objective (shrink 0.1 on the first iteration, 0.5
  afterwards, grow 2.1, Armijo 1e-4, Wolfe 0.9).

The vectors here are the model (dim = numFeatures + 1 for binary LR, 8 MB at
BASELINE config 5); the data pass behind `fn` runs on the GPU.  Iterate-level
equality with breeze is not pinned (breeze is absent); the estimator tests
pin the converged solutions against the glmnet coefficients the reference's
LogisticRegressionSuite asserts (relTol 1e-3).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Callable, List, Optional

import numpy as np


class FirstOrderException(RuntimeError):
    pass


class LineSearchFailed(FirstOrderException):
    pass


class StepSizeUnderflow(FirstOrderException):
    pass


class NaNHistory(FirstOrderException):
    pass


class CachedDiffFunction:
    """breeze CachedDiffFunction: remembers the last (x, value, gradient), so
    the line search's accepted point is not evaluated twice."""

    def __init__(self, fn: Callable[[np.ndarray], tuple]):
        self.fn = fn
        self._x = None
        self._v = None
        self._g = None
        self.evaluations = 0

    def calculate(self, x: np.ndarray):
        if self._x is not None and self._x.shape == x.shape and np.array_equal(self._x, x):
            return self._v, self._g
        v, g = self.fn(x)
        self.evaluations += 1
        self._x = np.array(x, dtype=np.float64, copy=True)
        self._v = float(v)
        self._g = np.asarray(g, dtype=np.float64)
        return self._v, self._g


@dataclass
class State:
    x: np.ndarray
    value: float
    grad: np.ndarray
    adjustedValue: float
    adjustedGradient: np.ndarray
    iter: int
    initialAdjVal: float
    history: "ApproximateInverseHessian"
    fvals: List[float] = field(default_factory=lambda: [math.inf])
    searchFailed: bool = False
    convergenceReason: Optional[str] = None


class ApproximateInverseHessian:
    """LBFGS.ApproximateInverseHessian: newest pair first, at most m pairs."""

    def __init__(self, m: int, steps=(), deltas=()):
        self.m = m
        self.steps = list(steps)
        self.deltas = list(deltas)

    def updated(self, step, delta):
        return ApproximateInverseHessian(self.m, ([step] + self.steps)[:self.m],
                                         ([delta] + self.deltas)[:self.m])

    def times(self, grad: np.ndarray) -> np.ndarray:
        h = len(self.steps)
        if h > 0:
            sy = float(self.steps[0] @ self.deltas[0])
            yy = float(self.deltas[0] @ self.deltas[0])
            if sy < 0 or math.isnan(sy):
                raise NaNHistory("sy < 0")
            diag = sy / yy
        else:
            diag = 1.0
        d = grad.copy()
        a = np.zeros(self.m)
        rho = np.zeros(self.m)
        for i in range(h):
            rho[i] = float(self.steps[i] @ self.deltas[i])
            a[i] = float(self.steps[i] @ d) / rho[i]
            if math.isnan(a[i]):
                raise NaNHistory("NaN in the history")
            d -= self.deltas[i] * a[i]
        d *= diag
        for i in range(h - 1, -1, -1):
            beta = float(self.deltas[i] @ d) / rho[i]
            d += self.steps[i] * (a[i] - beta)
        d *= -1.0
        return d


def _interp(l, r):
    """CubicLineSearch.interp (Nocedal & Wright p. 57), clamped to the middle
    80 % of the bracket.  l, r = (t, f, dd)."""
    lt, lf, ld = l
    rt, rf, rd = r
    d1 = ld + rd - 3 * (lf - rf) / (lt - rt)
    d2 = math.sqrt(max(d1 * d1 - ld * rd, 0.0))
    t = rt - (rt - lt) * (rd + d2 - d1) / (rd - ld + 2 * d2)
    lb = lt + 0.1 * (rt - lt)
    ub = lt + 0.9 * (rt - lt)
    if t < lb:
        return lb
    if t > ub:
        return ub
    return t


def strong_wolfe(phi: Callable[[float], tuple], init: float, maxZoomIter: int = 10,
                 maxLineSearchIter: int = 10, c1: float = 1e-4, c2: float = 0.9) -> float:
    """StrongWolfeLineSearch.minimize; phi(t) -> (f, dd)."""
    f0, dd0 = phi(0.0)
    if dd0 > 0:
        raise FirstOrderException(f"Line search invoked with non-descent direction: {dd0}")
    low = (0.0, f0, dd0)

    def zoom(lo, hi):
        for _ in range(maxZoomIter):
            t = _interp(hi, lo) if lo[0] > hi[0] else _interp(lo, hi)
            f, dd = phi(t)
            c = (t, f, dd)
            if f > f0 + c1 * t * dd0 or f >= lo[1]:
                hi = c
            else:
                if abs(dd) <= c2 * abs(dd0):
                    return t
                if dd * (hi[0] - lo[0]) >= 0:
                    hi = lo
                lo = c
        raise LineSearchFailed("Line search zoom failed")

    t = init
    for i in range(maxLineSearchIter):
        f, dd = phi(t)
        if math.isinf(f) or math.isnan(f):
            t /= 2.0
            continue
        c = (t, f, dd)
        if f > f0 + c1 * t * dd0 or (f >= low[1] and i > 0):
            return zoom(low, c)
        if abs(dd) <= -c2 * dd0:
            return t
        if dd >= 0:
            return zoom(c, low)
        low = c
        t *= 1.5
    raise LineSearchFailed("Line search failed")


def backtracking(phi: Callable[[float], tuple], init: float,
                 shrinkStep: float = 0.5, growStep: float = 2.1, cArmijo: float = 1e-4,
                 cWolfe: float = 0.9, maxIterations: int = 20, minAlpha: float = 1e-10,
                 maxAlpha: float = 1e10) -> float:
    """BacktrackingLineSearch with the Wolfe and strong-Wolfe conditions
    enforced; phi(alpha) -> (objective, directional derivative), both of
    OWL-QN's adjusted (L1-including) objective, Armijo against phi(0)."""
    initfval, initfderiv = phi(0.0)
    alpha = init
    fval, fderiv = phi(alpha)
    it = 0
    while True:
        if fval > initfval + alpha * initfderiv * cArmijo:
            mult = shrinkStep
        elif fderiv < cWolfe * initfderiv:
            mult = growStep
        elif fderiv > -cWolfe * initfderiv:
            mult = shrinkStep
        else:
            return alpha
        if it >= maxIterations:
            raise LineSearchFailed("Backtracking line search failed")
        alpha *= mult
        if alpha < minAlpha:
            raise StepSizeUnderflow("step size underflow")
        if alpha > maxAlpha:
            raise FirstOrderException("step size overflow")
        fval, fderiv = phi(alpha)
        it += 1


class LBFGS:
    """breeze LBFGS(maxIter, m, tolerance) with the default convergence check."""

    fvalMemory = 20

    def __init__(self, maxIter: int = 100, m: int = 10, tolerance: float = 1e-6):
        if m <= 0:
            raise ValueError("m must be positive")
        self.maxIter, self.m, self.tolerance = int(maxIter), int(m), float(tolerance)

    # -- hooks OWLQN overrides -------------------------------------------------
    def adjust(self, x, grad, value):
        return value, grad

    def chooseDescentDirection(self, state: State, f) -> np.ndarray:
        return state.history.times(state.grad)

    def takeStep(self, state: State, d: np.ndarray, stepSize: float) -> np.ndarray:
        return state.x + d * stepSize

    def determineStepSize(self, state: State, f, d: np.ndarray) -> float:
        x = state.x

        def phi(t):
            v, g = f.calculate(x + d * t)
            return v, float(g @ d)
        init = 1.0 / np.linalg.norm(d) if state.iter == 0 else 1.0
        alpha = strong_wolfe(phi, init)
        if alpha * np.linalg.norm(state.grad) < 1e-10:
            raise StepSizeUnderflow("step size underflow")
        return alpha

    # -- the loop ---------------------------------------------------------------
    def _converged(self, s: State) -> Optional[str]:
        if self.maxIter >= 0 and s.iter >= self.maxIter:
            return "max iterations reached"
        if len(s.fvals) >= 2 and abs(s.adjustedValue - max(s.fvals)) <= \
                self.tolerance * abs(s.initialAdjVal):
            return "function values converged"
        if np.max(np.abs(s.adjustedGradient), initial=0.0) <= \
                max(self.tolerance * abs(s.adjustedValue), 1e-8):
            return "gradient converged"
        if s.searchFailed:
            return "line search failed"
        return None

    def iterations(self, fn, init: np.ndarray):
        """Yields every state, the converged one last (takeUpToWhere)."""
        f = fn if isinstance(fn, CachedDiffFunction) else CachedDiffFunction(fn)
        x = np.array(init, dtype=np.float64, copy=True)
        v, g = f.calculate(x)
        av, ag = self.adjust(x, g, v)
        state = State(x, v, g, av, ag, 0, av, ApproximateInverseHessian(self.m))
        failedOnce = False
        while True:
            state.convergenceReason = self._converged(state)
            yield state
            if state.convergenceReason is not None:
                return
            try:
                d = self.chooseDescentDirection(state, f)
                step = self.determineStepSize(state, f, d)
                nx = self.takeStep(state, d, step)
                nv, ng = f.calculate(nx)
                nav, nag = self.adjust(nx, ng, nv)
                hist = state.history.updated(nx - state.x, ng - state.grad)
                fvals = (state.fvals + [nv])[-self.fvalMemory:]
                state = State(nx, nv, ng, nav, nag, state.iter + 1, state.initialAdjVal, hist,
                              fvals)
                failedOnce = False
            except FirstOrderException:
                if not failedOnce:
                    failedOnce = True
                    state = State(state.x, state.value, state.grad, state.adjustedValue,
                                  state.adjustedGradient, state.iter, state.initialAdjVal,
                                  ApproximateInverseHessian(self.m), state.fvals)
                else:
                    state = State(state.x, state.value, state.grad, state.adjustedValue,
                                  state.adjustedGradient, state.iter, state.initialAdjVal,
                                  state.history, state.fvals, searchFailed=True)

    def minimize(self, fn, init):
        s = None
        for s in self.iterations(fn, init):
            pass
        return s.x


class OWLQN(LBFGS):
    """breeze OWLQN(maxIter, m, l1reg: index -> weight, tolerance)."""

    def __init__(self, maxIter: int, m: int, l1reg, tolerance: float):
        super().__init__(maxIter, m, tolerance)
        self._l1 = l1reg
        self._w = None

    def _weights(self, n):
        if self._w is None or self._w.shape[0] != n:
            w = np.array([self._l1(i) for i in range(n)], dtype=np.float64) \
                if callable(self._l1) else np.asarray(self._l1, dtype=np.float64)
            if np.any(w < 0):
                raise ValueError("requirement failed")
            self._w = w
        return self._w

    def adjust(self, x, grad, value):
        w = self._weights(x.shape[0])
        adj = value + float(np.sum(np.abs(w * x)))
        dp, dm = grad + w, grad - w
        at0 = np.where(dm > 0, dm, np.where(dp < 0, dp, 0.0))
        res = np.where(x == 0.0, at0, grad + np.sign(x) * w)
        res = np.where(w == 0.0, grad, res)
        return adj, res

    def chooseDescentDirection(self, state: State, f):
        d = state.history.times(state.adjustedGradient)
        return np.where(d * state.adjustedGradient < 0, d, 0.0)

    def _orthant(self, x, g):
        return np.where(x != 0, np.sign(x), np.sign(-g))

    def takeStep(self, state: State, d, stepSize):
        stepped = state.x + d * stepSize
        orth = self._orthant(state.x, state.adjustedGradient)
        return np.where(np.sign(stepped) == np.sign(orth), stepped, 0.0)

    def determineStepSize(self, state: State, f, d):
        def phi(alpha):
            nx = self.takeStep(state, d, alpha)
            v, g = f.calculate(nx)
            av, ag = self.adjust(nx, g, v)
            return av, float(ag @ d)
        it = state.iter
        init = 0.5 / np.linalg.norm(state.grad) if it < 1 else 1.0
        return backtracking(phi, init, shrinkStep=0.1 if it < 1 else 0.5)


class LBFGSB:
    """breeze LBFGSB(lowerBounds, upperBounds, maxIter, m, tolerance) as
    LogisticRegression.createOptimizer builds it for bound-constrained fits
    (LogisticRegression.scala:786-789): the L-BFGS-B method of Byrd, Lu,
    Nocedal and Zhu (1995), restated -- compact limited-memory matrices
    W = [Y, theta S] and M; the generalized Cauchy point along the projected
    steepest-descent path (breakpoints in order); direct primal minimization
    of the quadratic model over the free variables, its point projected into
    the box; a backtracking Armijo search along the feasible segment
    (step <= 1 keeps every iterate in the box).  Convergence: maxIter, the
    relative function change of the default check (FunctionValuesConverged
    with tolerance), or the projected gradient's inf-norm <= max(tol |f|,
    1e-8)."""

    fvalMemory = 20

    def __init__(self, lower, upper, maxIter=100, m=10, tolerance=1e-6):
        self.l = np.asarray(lower, dtype=np.float64)
        self.u = np.asarray(upper, dtype=np.float64)
        if np.any(self.l > self.u):
            raise ValueError("requirement failed: lower bounds must not exceed upper bounds")
        self.maxIter, self.m, self.tolerance = int(maxIter), int(m), float(tolerance)

    def _proj(self, x):
        return np.minimum(np.maximum(x, self.l), self.u)

    def _pg_norm(self, x, g):
        return float(np.max(np.abs(self._proj(x - g) - x), initial=0.0))

    def _cauchy(self, x, g, W, M, theta):
        l, u = self.l, self.u
        n = x.size
        t = np.full(n, np.inf)
        neg, pos = g < 0, g > 0
        t[neg] = (x[neg] - u[neg]) / g[neg]
        t[pos] = (x[pos] - l[pos]) / g[pos]
        d = np.where(t > 0, -g, 0.0)
        xc = x.copy()
        p = W.T @ d if W.shape[1] else np.zeros(0)
        c = np.zeros_like(p)
        fp = -float(d @ d)
        fpp = -theta * fp - (float(p @ (M @ p)) if p.size else 0.0)
        fpp = max(fpp, 1e-300)
        dtmin = -fp / fpp
        told = 0.0
        order = np.argsort(t)
        order = order[(t[order] > 0) & np.isfinite(t[order])]
        for b in order:
            dt = t[b] - told
            if dtmin < dt:
                break
            xc[b] = u[b] if d[b] > 0 else l[b]
            zb = xc[b] - x[b]
            c = c + dt * p
            gb = g[b]
            wb = W[b]
            Mc = M @ c if c.size else c
            Mp = M @ p if p.size else p
            fp = fp + dt * fpp + gb * gb + theta * gb * zb - (gb * float(wb @ Mc) if c.size else 0.0)
            fpp = fpp - theta * gb * gb - (2.0 * gb * float(wb @ Mp) + gb * gb * float(wb @ (M @ wb))
                                           if p.size else 0.0)
            fpp = max(fpp, 1e-300)
            p = p + gb * wb
            d[b] = 0.0
            dtmin = -fp / fpp
            told = t[b]
        dtmin = max(dtmin, 0.0)
        told += dtmin
        free = d != 0
        xc[free] = x[free] + told * d[free]
        c = c + dtmin * p
        return self._proj(xc), c

    def _subspace(self, x, g, xc, c, W, M, theta):
        free = (xc > self.l) & (xc < self.u)
        if not np.any(free):
            return xc
        if W.shape[1] == 0:
            r = g + theta * (xc - x)
            xb = xc.copy()
            xb[free] = xc[free] - r[free] / theta
            return self._proj(xb)
        r = g + theta * (xc - x) - W @ (M @ c)
        rF = r[free]
        WF = W[free]
        v = M @ (WF.T @ rF)
        Nm = np.eye(M.shape[0]) - (M @ (WF.T @ WF)) / theta
        try:
            v = np.linalg.solve(Nm, v)
        except np.linalg.LinAlgError:
            v = np.linalg.lstsq(Nm, v, rcond=None)[0]
        du = -rF / theta - (WF @ v) / (theta * theta)
        xb = xc.copy()
        xb[free] = xc[free] + du
        return self._proj(xb)

    def iterations(self, fn, init):
        f = fn if isinstance(fn, CachedDiffFunction) else CachedDiffFunction(fn)
        x = self._proj(np.array(init, dtype=np.float64, copy=True))
        v, g = f.calculate(x)
        S, Y = [], []
        theta = 1.0
        fvals = [math.inf]
        it = 0
        v0 = v
        while True:
            reason = None
            if self.maxIter >= 0 and it >= self.maxIter:
                reason = "max iterations reached"
            elif len(fvals) >= 2 and abs(v - max(fvals)) <= self.tolerance * abs(v0):
                reason = "function values converged"
            elif self._pg_norm(x, g) <= max(self.tolerance * abs(v), 1e-8):
                reason = "projected gradient converged"
            st = State(x, v, g, v, g, it, v0, None, list(fvals), convergenceReason=reason)
            yield st
            if reason is not None:
                return
            if S:
                Sm, Ym = np.stack(S, 1), np.stack(Y, 1)
                W = np.concatenate([Ym, theta * Sm], axis=1)
                SY = Sm.T @ Ym
                D = np.diag(np.diag(SY))
                L = np.tril(SY, -1)
                K = np.block([[-D, L.T], [L, theta * (Sm.T @ Sm)]])
                M = np.linalg.inv(K)
            else:
                W = np.zeros((x.size, 0))
                M = np.zeros((0, 0))
            xc, c = self._cauchy(x, g, W, M, theta)
            xb = self._subspace(x, g, xc, c, W, M, theta)
            d = xb - x
            dg = float(d @ g)
            if not dg < 0:           # not a descent direction: restart from steepest descent
                S, Y, theta = [], [], 1.0
                d = self._proj(x - g) - x
                dg = float(d @ g)
                if not dg < 0:
                    st.convergenceReason = "no descent direction"
                    yield st
                    return
            alpha = 1.0
            for _ in range(30):
                xn = self._proj(x + alpha * d)
                vn, gn = f.calculate(xn)
                if vn <= v + 1e-4 * alpha * dg:
                    break
                alpha *= 0.5
            else:
                st.searchFailed = True
                st.convergenceReason = "line search failed"
                yield st
                return
            s, y = xn - x, gn - g
            sy = float(s @ y)
            if sy > 2.2e-16 * float(y @ y):
                S.append(s)
                Y.append(y)
                if len(S) > self.m:
                    S.pop(0)
                    Y.pop(0)
                theta = float(y @ y) / sy
            x, v, g = xn, vn, gn
            fvals = (fvals + [v])[-self.fvalMemory:]
            it += 1

    def minimize(self, fn, init):
        s = None
        for s in self.iterations(fn, init):
            pass
        return s.x
