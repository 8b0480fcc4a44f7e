"""LogisticRegression: the estimator around the device aggregators.

Host-side mirror of ml/classification/LogisticRegression.scala:
  train             :495-685  (summaries, checks, optimizer choice, the
                               solution back to the original space, centring
                               of unregularized multinomial coefficients)
  createOptimizer   :777-816  (LBFGS, or OWLQN when elasticNet * reg > 0)
  createInitialSolution :822-933
  trainImpl         :935-1035 (fitWithMean, the initial / final intercept
                               adaptation, the optimizer loop)
with the reference's parameter names, defaults and error texts, including
bound-constrained fits (createBounds :732-775, LBFGS-B).

Standardization.  The reference scales every instance by inverseStd into a
new RDD before blockifying (:962-968) and runs the aggregators on the scaled
blocks.  Here the shard stays in HBM unscaled and the scaling moves into the
model: margins of scaled rows with coefficients w equal margins of the raw
rows with w * inverseStd, scaledMean . w = featuresMean . (w * inverseStd),
and each gradient entry of the scaled problem is the raw one times
inverseStd(j).  The same loss and gradient (to rounding) without a copy or
an in-place rewrite of a 157 GB shard.
"""
from __future__ import annotations

import math
from typing import Callable, Optional, Sequence

import numpy as np

from . import _native as N
from . import optim, optimize, stat


class SparkException(RuntimeError):
    pass


def _is_multinomial(family: str, numClasses: int) -> bool:
    """checkMultinomial (:687-697)."""
    f = family.lower()
    if f == "binomial":
        if not (numClasses == 1 or numClasses == 2):
            raise N.IllegalArgumentException(
                "requirement failed: Binomial family only supports 1 or 2 outcome classes but "
                f"found {numClasses}.")
        return False
    if f == "multinomial":
        return True
    if f == "auto":
        return numClasses > 2
    raise N.IllegalArgumentException(f"Unsupported family: {family}")


class LogisticRegressionModel:
    """coefficientMatrix (numCoefficientSets x numFeatures, row-major) and
    interceptVector, as LogisticRegressionModel holds them."""

    def __init__(self, coefficientMatrix, interceptVector, numClasses, isMultinomial,
                 objectiveHistory=(), fitIntercept=True):
        self.coefficientMatrix = np.asarray(coefficientMatrix, dtype=np.float64)
        # the model's fitIntercept param (copyValues of its estimator; default true)
        self.fitIntercept = bool(fitIntercept)
        self.interceptVector = np.asarray(interceptVector, dtype=np.float64)
        self.numClasses = int(numClasses)
        self.isMultinomial = bool(isMultinomial)
        self.objectiveHistory = np.asarray(objectiveHistory, dtype=np.float64)

    @property
    def numFeatures(self) -> int:
        return int(self.coefficientMatrix.shape[1])

    def save(self, path, estimator=None, overwrite=False):
        """model.write.save(path) in Spark's format (cycloneml_amd.persist)."""
        from . import persist
        persist.save_logistic_model(self, path, estimator, getattr(self, "uid", None),
                                    overwrite=overwrite)

    @staticmethod
    def load(path) -> "LogisticRegressionModel":
        from . import persist
        return persist.load_logistic_model(path)

    @property
    def coefficients(self) -> np.ndarray:
        if self.isMultinomial:
            raise SparkException("Multinomial models contain a matrix of coefficients, use "
                                 "coefficientMatrix instead.")
        return self.coefficientMatrix[0].copy()

    @property
    def intercept(self) -> float:
        if self.isMultinomial:
            raise SparkException("Multinomial models contain a vector of intercepts, use "
                                 "interceptVector instead.")
        return float(self.interceptVector[0])

    @property
    def totalIterations(self) -> int:
        return max(len(self.objectiveHistory) - 1, 0)

    def predictRaw(self, X) -> np.ndarray:
        """Margins (:1224-1246) for host rows: binomial (-m, m), multinomial
        coefficientMatrix x + interceptVector."""
        X = np.atleast_2d(np.asarray(X, dtype=np.float64))
        m = X @ self.coefficientMatrix.T + self.interceptVector
        if self.isMultinomial:
            return m
        return np.concatenate([-m, m], axis=1)

    def predict(self, X, threshold: float = 0.5) -> np.ndarray:
        raw = self.predictRaw(X)
        if self.isMultinomial:
            return np.argmax(raw, axis=1).astype(np.float64)
        p = 1.0 / (1.0 + np.exp(-raw[:, 1]))
        return (p > threshold).astype(np.float64)


class LogisticRegression:
    """LogisticRegression estimator over device-resident DeviceInstanceBlocks
    (one rank's shard; with torch.distributed initialised every rank calls
    fit on its own shard and the per-evaluation merge is an all-reduce)."""

    def __init__(self, regParam: float = 0.0, elasticNetParam: float = 0.0, maxIter: int = 100,
                 tol: float = 1e-6, fitIntercept: bool = True, standardization: bool = True,
                 family: str = "auto", aggregationDepth: int = 2, maxBlockSizeInMB: float = 0.0):
        self.regParam = float(regParam)
        self.elasticNetParam = float(elasticNetParam)
        self.maxIter = int(maxIter)
        self.tol = float(tol)
        self.fitIntercept = bool(fitIntercept)
        self.standardization = bool(standardization)
        self.family = family
        self.aggregationDepth = int(aggregationDepth)
        self.maxBlockSizeInMB = float(maxBlockSizeInMB)
        self.initialModel: Optional[LogisticRegressionModel] = None
        self.lowerBoundsOnCoefficients = None     # (numCoefficientSets, numFeatures)
        self.upperBoundsOnCoefficients = None
        self.lowerBoundsOnIntercepts = None       # (numCoefficientSets,)
        self.upperBoundsOnIntercepts = None
        self._validate()

    @property
    def usingBoundConstrainedOptimization(self) -> bool:
        """:251-254"""
        return any(b is not None for b in (self.lowerBoundsOnCoefficients,
                                           self.upperBoundsOnCoefficients,
                                           self.lowerBoundsOnIntercepts,
                                           self.upperBoundsOnIntercepts))

    def setLowerBoundsOnCoefficients(self, M):
        self.lowerBoundsOnCoefficients = np.atleast_2d(np.asarray(M, dtype=np.float64)); return self

    def setUpperBoundsOnCoefficients(self, M):
        self.upperBoundsOnCoefficients = np.atleast_2d(np.asarray(M, dtype=np.float64)); return self

    def setLowerBoundsOnIntercepts(self, v):
        self.lowerBoundsOnIntercepts = np.atleast_1d(np.asarray(v, dtype=np.float64)); return self

    def setUpperBoundsOnIntercepts(self, v):
        self.upperBoundsOnIntercepts = np.atleast_1d(np.asarray(v, dtype=np.float64)); return self

    def _check_bounds(self, numCoefficientSets, numFeatures):
        """validateAndTransformSchema (:258-268) and
        assertBoundConstrainedOptimizationParamsValid (:442-485)."""
        def req(c, msg):
            if not c:
                raise N.IllegalArgumentException("requirement failed: " + msg)
        if not self.usingBoundConstrainedOptimization:
            return
        req(self.elasticNetParam == 0.0, "Fitting under bound constrained optimization only "
            f"supports L2 regularization, but got elasticNetParam = {self.elasticNetParam}.")
        if not self.fitIntercept:
            req(self.lowerBoundsOnIntercepts is None and self.upperBoundsOnIntercepts is None,
                "Please don't set bounds on intercepts if fitting without intercept.")
        for name, M in (("LowerBoundsOnCoefficients", self.lowerBoundsOnCoefficients),
                        ("upperBoundsOnCoefficients", self.upperBoundsOnCoefficients)):
            if M is not None:
                req(M.shape == (numCoefficientSets, numFeatures),
                    f"The shape of {name} must be compatible with (1, number of features) for "
                    "binomial regression, or (number of classes, number of features) for "
                    f"multinomial regression, but found: ({M.shape[0]}, {M.shape[1]}).")
        for name, v in (("lowerBoundsOnIntercepts", self.lowerBoundsOnIntercepts),
                        ("upperBoundsOnIntercepts", self.upperBoundsOnIntercepts)):
            if v is not None:
                req(v.shape[0] == numCoefficientSets, f"The size of {name} must be equal to 1 "
                    "for binomial regression, or the number of classes for multinomial "
                    f"regression, but found: {v.shape[0]}.")
        if self.lowerBoundsOnCoefficients is not None and \
                self.upperBoundsOnCoefficients is not None:
            req(bool(np.all(self.lowerBoundsOnCoefficients <= self.upperBoundsOnCoefficients)),
                "LowerBoundsOnCoefficients should always be less than or equal to "
                "upperBoundsOnCoefficients")
        if self.lowerBoundsOnIntercepts is not None and self.upperBoundsOnIntercepts is not None:
            req(bool(np.all(self.lowerBoundsOnIntercepts <= self.upperBoundsOnIntercepts)),
                "LowerBoundsOnIntercepts should always be less than or equal to "
                "upperBoundsOnIntercepts")

    def _create_bounds(self, numCoefficientSets, numFeatures, featuresStd):
        """createBounds (:732-775): column-major (index i -> class i % nCS,
        feature i / nCS), coefficient bounds scaled by featuresStd."""
        if not self.usingBoundConstrainedOptimization:
            return None, None
        nFPI = numFeatures + 1 if self.fitIntercept else numFeatures
        n = nFPI * numCoefficientSets
        lo = np.full(n, -np.inf)
        hi = np.full(n, np.inf)
        for i in range(n):
            cs, fi = i % numCoefficientSets, i // numCoefficientSets
            if fi < numFeatures:
                if self.lowerBoundsOnCoefficients is not None:
                    lo[i] = self.lowerBoundsOnCoefficients[cs, fi] * featuresStd[fi]
                if self.upperBoundsOnCoefficients is not None:
                    hi[i] = self.upperBoundsOnCoefficients[cs, fi] * featuresStd[fi]
            else:
                if self.lowerBoundsOnIntercepts is not None:
                    lo[i] = self.lowerBoundsOnIntercepts[cs]
                if self.upperBoundsOnIntercepts is not None:
                    hi[i] = self.upperBoundsOnIntercepts[cs]
        return lo, hi

    def _validate(self):
        if not self.regParam >= 0:
            raise N.IllegalArgumentException("regParam given invalid value " + str(self.regParam))
        if not 0.0 <= self.elasticNetParam <= 1.0:
            raise N.IllegalArgumentException(
                "elasticNetParam given invalid value " + str(self.elasticNetParam))
        if not self.maxIter >= 0:
            raise N.IllegalArgumentException("maxIter given invalid value " + str(self.maxIter))
        if not self.tol >= 0:
            raise N.IllegalArgumentException("tol given invalid value " + str(self.tol))
        if self.family.lower() not in ("auto", "binomial", "multinomial"):
            raise N.IllegalArgumentException("family given invalid value " + self.family)

    # Spark-style setters (chainable)
    def setRegParam(self, v):
        self.regParam = float(v); self._validate(); return self

    def setElasticNetParam(self, v):
        self.elasticNetParam = float(v); self._validate(); return self

    def setMaxIter(self, v):
        self.maxIter = int(v); self._validate(); return self

    def setTol(self, v):
        self.tol = float(v); self._validate(); return self

    def setFitIntercept(self, v):
        self.fitIntercept = bool(v); return self

    def setStandardization(self, v):
        self.standardization = bool(v); return self

    def setFamily(self, v):
        self.family = v; self._validate(); return self

    def setInitialModel(self, model: LogisticRegressionModel):
        self.initialModel = model; return self

    # -- fit --------------------------------------------------------------------
    def fit(self, blocks) -> LogisticRegressionModel:
        """train (:495-685) over this rank's device blocks."""
        blocks = list(blocks) if isinstance(blocks, (list, tuple)) else [blocks]
        summ, lab = stat.getClassificationSummarizers(blocks)
        numFeatures = summ.n
        histogram = lab.histogram
        if lab.countInvalid != 0:
            raise SparkException(
                f"Classification labels should be in [0 to {len(histogram) - 1}]. "
                f"Found {lab.countInvalid} invalid labels.")
        mean, std = summ.mean, summ.std
        device = blocks[0].labels.device

        def make_cost(numClasses, multinomial, fitWithMean, inverseStd):
            # kept as lastCost: its evaluations count the data passes
            self.lastCost = _DeviceCost(blocks, numFeatures, numClasses, multinomial,
                                        self.fitIntercept, fitWithMean, mean, inverseStd, device)
            return self.lastCost
        return self.train_from_summary(numFeatures, histogram, mean, std, make_cost)

    def train_from_summary(self, numFeatures: int, histogram, featuresMean, featuresStd,
                           make_cost: Callable) -> LogisticRegressionModel:
        """The driver logic of train / trainImpl once the summaries exist.
        make_cost(numClasses, multinomial, fitWithMean, inverseStd) returns a
        function: coefficients of the SCALED problem -> (loss, gradient),
        i.e. RDDLossFunction.calculate over the standardized blocks without
        the regularization term."""
        histogram = np.asarray(histogram, dtype=np.float64)
        featuresMean = np.asarray(featuresMean, dtype=np.float64)
        featuresStd = np.asarray(featuresStd, dtype=np.float64)
        numClasses = len(histogram)
        fitIntercept = self.fitIntercept
        numFeaturesPlusIntercept = numFeatures + 1 if fitIntercept else numFeatures
        isMultinomial = _is_multinomial(self.family, numClasses)
        numCoefficientSets = numClasses if isMultinomial else 1

        isConstantLabel = int(np.count_nonzero(histogram)) == 1
        if fitIntercept and isConstantLabel and not self.usingBoundConstrainedOptimization:
            # :564-577 -- all labels the same: zero coefficients, infinite intercept
            idx = int(np.argmax(histogram))
            coef = np.zeros((numCoefficientSets, numFeatures))
            if isMultinomial:
                icpt = np.zeros(numClasses)
                icpt[idx] = math.inf
            else:
                icpt = np.array([math.inf if numClasses == 2 else -math.inf])
            return LogisticRegressionModel(coef, icpt, numClasses, isMultinomial, [0.0],
                                           fitIntercept=self.fitIntercept)

        self._check_bounds(numCoefficientSets, numFeatures)
        bounded = self.usingBoundConstrainedOptimization
        regParamL2 = (1.0 - self.elasticNetParam) * self.regParam
        regularization = None
        if regParamL2 != 0.0:
            nreg = numFeatures * numCoefficientSets
            stdOf = None if self.standardization else \
                np.repeat(featuresStd, numCoefficientSets)     # j -> featuresStd(j / nCS)
            regularization = _L2(regParamL2, nreg, stdOf)

        lower, upper = self._create_bounds(numCoefficientSets, numFeatures, featuresStd)
        optimizer = self._create_optimizer(numCoefficientSets, numFeatures, featuresStd,
                                           lower, upper)
        init = self._initial_solution(numClasses, numFeatures, histogram, featuresStd,
                                      isMultinomial)
        if bounded:      # :912-930, every initial value inside its bounds
            init = np.minimum(np.maximum(init, lower), upper)
        solution, history = self._train_impl(numFeatures, featuresMean, featuresStd, numClasses,
                                             isMultinomial, init, regularization, optimizer,
                                             make_cost)
        if solution is None:
            raise SparkException(f"{type(optimizer).__name__} failed.")

        # :637-654 -- back to the original space, row-major coefficient matrix
        all_ = solution.reshape(numFeaturesPlusIntercept, numCoefficientSets).T  # col-major
        coefM = np.zeros((numCoefficientSets, numFeatures))
        nz = featuresStd != 0.0
        coefM[:, nz] = all_[:, :numFeatures][:, nz] / featuresStd[nz]
        icpt = all_[:, numFeatures].copy() if fitIntercept else np.zeros(numCoefficientSets)
        if self.regParam == 0.0 and isMultinomial and not bounded:
            # :656-674 -- mean-centred coefficients (identifiability, as glmnet)
            coefM = coefM - coefM.sum(axis=0) / numCoefficientSets
        if fitIntercept and isMultinomial and not bounded:
            icpt = icpt - icpt.sum() / len(icpt)
        return LogisticRegressionModel(coefM, icpt, numClasses, isMultinomial, history,
                                       fitIntercept=self.fitIntercept)

    def _create_optimizer(self, numCoefficientSets, numFeatures, featuresStd, lower=None,
                          upper=None):
        """createOptimizer (:777-816)."""
        regParamL1 = self.elasticNetParam * self.regParam
        if self.elasticNetParam == 0.0 or self.regParam == 0.0:
            if lower is not None and upper is not None:
                return optimize.LBFGSB(lower, upper, self.maxIter, 10, self.tol)
            return optimize.LBFGS(self.maxIter, 10, self.tol)
        n = (numFeatures + (1 if self.fitIntercept else 0)) * numCoefficientSets
        w = np.zeros(n)
        for index in range(n):
            if self.fitIntercept and index >= numFeatures * numCoefficientSets:
                w[index] = 0.0          # no L1 on the intercepts
            elif self.standardization:
                w[index] = regParamL1
            else:
                s = featuresStd[index // numCoefficientSets]
                w[index] = regParamL1 / s if s != 0.0 else 0.0
        return optimize.OWLQN(self.maxIter, 10, w, self.tol)

    def _initial_solution(self, numClasses, numFeatures, histogram, featuresStd, isMultinomial):
        """createInitialSolution (:822-933): column-major (numCoefficientSets x
        numFeaturesPlusIntercept) as a flat array."""
        nCS = numClasses if isMultinomial else 1
        nFPI = numFeatures + 1 if self.fitIntercept else numFeatures
        M = np.zeros((nCS, nFPI))
        m = self.initialModel
        # :838-844 -- shape, intercept count AND the same fitIntercept
        valid = m is not None and m.coefficientMatrix.shape == (nCS, numFeatures) and \
            m.interceptVector.shape[0] == nCS and \
            getattr(m, "fitIntercept", True) == self.fitIntercept
        if valid:
            M[:, :numFeatures] = m.coefficientMatrix * featuresStd
            if self.fitIntercept:
                M[:, numFeatures] = m.interceptVector
        elif self.fitIntercept and isMultinomial:
            raw = np.log1p(histogram)
            M[:, numFeatures] = raw - raw.sum() / len(raw)
        elif self.fitIntercept:
            M[0, numFeatures] = math.log(histogram[1] / histogram[0])
        return M.T.reshape(-1).copy()        # column-major

    def _train_impl(self, numFeatures, featuresMean, featuresStd, numClasses, multinomial,
                    init, regularization, optimizer, make_cost):
        """trainImpl (:935-1035)."""
        # :950-954: centre only without (finite) bounds on the intercepts
        fitWithMean = self.fitIntercept and \
            (self.lowerBoundsOnIntercepts is None or
             bool(np.all(np.isneginf(self.lowerBoundsOnIntercepts)))) and \
            (self.upperBoundsOnIntercepts is None or
             bool(np.all(np.isposinf(self.upperBoundsOnIntercepts))))
        inverseStd = np.where(featuresStd != 0, 1.0 / np.where(featuresStd != 0, featuresStd, 1),
                              0.0)
        scaledMean = inverseStd * featuresMean
        cost = make_cost(numClasses, multinomial, fitWithMean, inverseStd)

        def fn(coef):
            loss, grad = cost(coef)
            if regularization is not None:
                rl, rg = regularization.calculate(coef)
                loss, grad = loss + rl, grad + rg
            return loss, grad

        x0 = init.copy()
        nC = numClasses if multinomial else 1
        if fitWithMean:
            if multinomial:
                # adapt = linear (C x F col-major) . scaledMean; intercepts += adapt
                lin = x0[:nC * numFeatures].reshape(numFeatures, nC)
                x0[nC * numFeatures:] += scaledMean @ lin
            else:
                x0[numFeatures] += float(np.dot(x0[:numFeatures], scaledMean))
        history = []
        state = None
        for state in optimizer.iterations(fn, x0):
            history.append(state.adjustedValue)
        if state is None:
            return None, history
        sol = state.x.copy()
        if fitWithMean:
            if multinomial:
                lin = sol[:nC * numFeatures].reshape(numFeatures, nC)
                sol[nC * numFeatures:] -= scaledMean @ lin
            else:
                sol[numFeatures] -= float(np.dot(sol[:numFeatures], scaledMean))
        self.lastState = state
        return sol, history


class _L2:
    """L2Regularization (ml/optim/loss/DifferentiableRegularization.scala):
    the first nreg indices are regularized; with std given (standardization =
    false) coef_j / std_j^2 per the reverse-standardization branch."""

    def __init__(self, regParam, nreg, std=None):
        self.regParam, self.nreg, self.std = float(regParam), int(nreg), std

    def calculate(self, coef):
        c = coef[:self.nreg]
        g = np.zeros_like(coef)
        if self.std is None:
            s = float(np.dot(c, c))
            g[:self.nreg] = c * self.regParam
        else:
            nz = self.std != 0.0
            t = np.zeros_like(c)
            t[nz] = c[nz] / (self.std[nz] * self.std[nz])
            s = float(np.dot(c, t))
            g[:self.nreg] = self.regParam * t
        return 0.5 * s * self.regParam, g


class _DeviceCost:
    """RDDLossFunction.calculate over the device shard, for coefficients of
    the standardized problem (see the module docstring): coefficients and
    gradient are rescaled by inverseStd on the host; the data pass is one
    aggregator add over every block plus the all-reduce."""

    def __init__(self, blocks, numFeatures, numClasses, multinomial, fitIntercept, fitWithMean,
                 featuresMean, inverseStd, device):
        self.blocks = blocks
        self.F = int(numFeatures)
        self.C = int(numClasses) if multinomial else 1
        self.multinomial = multinomial
        self.fitIntercept, self.fitWithMean = fitIntercept, fitWithMean
        self.inv = np.asarray(inverseStd, dtype=np.float64)
        # per coefficient: the inverseStd of its feature, 1 for intercepts
        nlin = self.F * self.C
        s = np.ones(nlin + (self.C if fitIntercept else 0))
        s[:nlin] = np.repeat(self.inv, self.C) if multinomial else self.inv
        self.scale = s
        self.mean = np.asarray(featuresMean, dtype=np.float64) if fitWithMean else None
        self.device = device
        self.ones = np.ones(self.F)
        self.evaluations = 0

    def __call__(self, coef_scaled):
        raw = coef_scaled * self.scale
        if self.multinomial:
            agg = optim.MultinomialLogisticBlockAggregator(
                self.ones, self.mean, self.fitIntercept, self.fitWithMean, raw,
                device=self.device)
        else:
            agg = optim.BinaryLogisticBlockAggregator(
                self.ones, self.mean, self.fitIntercept, self.fitWithMean, raw,
                device=self.device)
        for b in self.blocks:
            agg.add(b)
        agg.allreduce()
        self.evaluations += 1
        return agg.loss, agg.gradient * self.scale
