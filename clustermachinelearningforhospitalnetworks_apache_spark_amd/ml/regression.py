"""Regressors of the reference (ref.py:30, ref.py:145-158): LinearRegression,
DecisionTreeRegressor, RandomForestRegressor.

LinearRegression (Spark defaults maxIter=100, regParam=0, elasticNetParam=0,
tol=1e-6, fitIntercept=True, standardization=True, solver="auto"): the normal
equations are built on the device in ONE pass (K15 Gram [X 1 y]ᵀ[X 1 y] in f64),
all-reduced (C4), and solved on the host in float64 — Cholesky, with ridge in the
standardized space like Spark's WeightedLeastSquares; L1/elastic-net by coordinate
descent on the same Gram (same optimum as Spark's OWL-QN); a singular system falls
back to the minimum-norm least-squares solution.
"""
from __future__ import annotations

import math
from typing import Optional

import numpy as np
import torch

from ..ops import glm_ops
from ..sql import types as T
from ..sql.column import ColumnData
from . import util as U
from .base import Estimator, Model
from .evaluation import RegressionEvaluator
from .feature import _replace_col
from .linalg import DenseVector, as_array
from .tree_models import (FOREST_PARAMS, GBT_PARAMS, TREE_PARAMS, GBTEstimatorMixin, GBTModelMixin,
                          TreeEstimatorMixin, TreeModelMixin, _default_seed)

_LR_PARAMS = {
    "featuresCol": ("features", "features column name", str),
    "labelCol": ("label", "label column name", str),
    "predictionCol": ("prediction", "prediction column name", str),
    "maxIter": (100, "max number of iterations (>= 0)", int),
    "regParam": (0.0, "regularization parameter (>= 0)", float),
    "elasticNetParam": (0.0, "ElasticNet mixing parameter in [0, 1]: 0 = L2, 1 = L1", float),
    "tol": (1e-6, "convergence tolerance for iterative algorithms (>= 0)", float),
    "fitIntercept": (True, "whether to fit an intercept term", bool),
    "standardization": (True, "whether to standardize the training features before fitting", bool),
    "solver": ("auto", "the solver algorithm for optimization: auto, normal, l-bfgs", str),
    "weightCol": (None, "weight column name", None),
    "aggregationDepth": (2, "suggested depth for treeAggregate (>= 2)", int),
    "loss": ("squaredError", "the loss function to be optimized: squaredError, huber", str),
    "epsilon": (1.35, "the shape parameter to control the amount of robustness (huber)", float),
    "maxBlockSizeInMB": (0.0, "maximum memory in MB for stacking input data into blocks", float),
}


def solve_wls(G: np.ndarray, d: int, reg: float, alpha: float, fit_intercept: bool, standardization: bool,
              max_iter: int = 1000, tol: float = 1e-10):
    """Solve weighted least squares from the Gram matrix of [X 1 y] (weights folded in).

    Returns (coefficients [d], intercept, diag info dict).
    """
    n = G[d, d]
    sx = G[:d, d]
    sy = G[d, d + 1]
    XtX = G[:d, :d]
    Xty = G[:d, d + 1]
    yty = G[d + 1, d + 1]
    mx = sx / n
    my = sy / n
    if fit_intercept:
        Cxx = XtX / n - np.outer(mx, mx)
        cxy = Xty / n - mx * my
        vy = yty / n - my * my
    else:
        Cxx = XtX / n
        cxy = Xty / n
        vy = yty / n
    var_x = np.maximum(np.diag(XtX) / n - mx * mx, 0.0)
    unbiased = n / (n - 1) if n > 1 else 1.0
    sigx = np.sqrt(var_x * unbiased)
    sigy = math.sqrt(max(yty / n - my * my, 0.0) * unbiased)
    info = {"n": n, "mean_x": mx, "mean_y": my, "std_x": sigx, "std_y": sigy}
    if sigy == 0.0 and fit_intercept:
        # constant label: Spark returns zero coefficients and intercept = label mean
        return np.zeros(d), my, info
    active = sigx > 0
    if reg == 0.0:
        A = Cxx[np.ix_(active, active)]
        b = cxy[active]
        w = np.zeros(d)
        try:
            L = np.linalg.cholesky(A)
            w[active] = np.linalg.solve(L.T, np.linalg.solve(L, b))
        except np.linalg.LinAlgError:
            w[active] = np.linalg.lstsq(A, b, rcond=None)[0]
    else:
        sy_ = sigy if sigy > 0 else 1.0
        s = np.where(active, sigx, 1.0)
        Z = Cxx / np.outer(s, s)                    # covariance of standardized features
        zt = cxy / s / sy_                          # covariance with standardized label
        # Spark's WeightedLeastSquares penalises in the label-standardized space with effectiveRegParam =
        # regParam / std(label) (pinned against sklearn Ridge / Lasso in tests/test_linreg_solvers.py)
        l2 = reg / sy_ * (1.0 - alpha)
        l1 = reg / sy_ * alpha
        # standardization=False penalises the original-scale coefficients: rescale per feature
        pen2 = np.full(d, l2) if standardization else l2 / (s * s)
        pen1 = np.full(d, l1) if standardization else l1 / s
        beta = np.zeros(d)
        if l1 == 0.0:
            A = Z + np.diag(pen2)
            A = A[np.ix_(active, active)]
            beta[active] = np.linalg.solve(A, zt[active])
        else:
            for _ in range(max_iter):
                maxd = 0.0
                for j in np.nonzero(active)[0]:
                    rj = zt[j] - Z[j] @ beta + Z[j, j] * beta[j]
                    new = np.sign(rj) * max(abs(rj) - pen1[j], 0.0) / (Z[j, j] + pen2[j])
                    maxd = max(maxd, abs(new - beta[j]))
                    beta[j] = new
                if maxd < tol:
                    break
        w = np.where(active, beta * sy_ / s, 0.0)
    intercept = (my - mx @ w) if fit_intercept else 0.0
    return w, float(intercept), info


class LinearRegression(Estimator):
    _params = _LR_PARAMS

    def __init__(self, featuresCol=None, labelCol=None, predictionCol=None, maxIter=None, regParam=None,
                 elasticNetParam=None, tol=None, fitIntercept=None, standardization=None, solver=None,
                 weightCol=None, aggregationDepth=None, loss=None, epsilon=None, maxBlockSizeInMB=None):
        super().__init__(featuresCol=featuresCol, labelCol=labelCol, predictionCol=predictionCol, maxIter=maxIter,
                         regParam=regParam, elasticNetParam=elasticNetParam, tol=tol, fitIntercept=fitIntercept,
                         standardization=standardization, solver=solver, weightCol=weightCol,
                         aggregationDepth=aggregationDepth, loss=loss, epsilon=epsilon,
                         maxBlockSizeInMB=maxBlockSizeInMB)
        self._defaultParamMap.pop("weightCol", None)

    # Spark's WeightedLeastSquares.MAX_NUM_FEATURES: solver "auto" takes the normal equations up to this width
    _NORMAL_MAX_FEATURES = 4096

    def _fit(self, df):
        loss = self.getLoss()
        if loss not in ("squaredError", "huber"):
            raise ValueError(f"loss must be 'squaredError' or 'huber', got {loss!r}")
        solver = self.getSolver()
        if solver not in ("auto", "normal", "l-bfgs"):
            raise ValueError(f"solver must be 'auto', 'normal' or 'l-bfgs', got {solver!r}")
        x = df._feature_matrix(self.getFeaturesCol())
        d = x.shape[1]
        y = df._column_data(self.getLabelCol()).values.to(torch.float64)
        w = df._column_data(self.getOrDefault("weightCol")).values.to(torch.float64) \
            if self.isSet("weightCol") else None
        if loss == "huber":
            if solver == "normal":
                raise ValueError("LinearRegression with huber loss only supports the l-bfgs solver")
            if self.getElasticNetParam() > 0 and self.getRegParam() > 0:
                raise ValueError("LinearRegression with huber loss only supports L2 regularization")
        # Spark LinearRegression.train: the normal equations for "normal", and for "auto" with squared
        # loss up to 4096 features; L-BFGS / OWL-QN passes over the rows otherwise (no D² Gram)
        if loss == "huber" or solver == "l-bfgs" or (solver == "auto" and d > self._NORMAL_MAX_FEATURES):
            return self._fit_iterative(df, x, d, y, w, loss)
        G = glm_ops.gram(x, d, y, w)
        df._comm.allreduce_(G)
        Gn = G.cpu().numpy()
        if Gn[d, d] == 0:
            raise ValueError("LinearRegression: empty training set")
        coef, intercept, info = solve_wls(Gn, d, self.getRegParam(), self.getElasticNetParam(),
                                          self.getFitIntercept(), self.getStandardization(),
                                          max_iter=max(self.getMaxIter(), 1) * 10, tol=self.getTol())
        model = LinearRegressionModel(coef, intercept)
        self._copyValues(model)
        model._attach_summary(LinearRegressionTrainingSummary(model, df, Gn, d, self.getRegParam() == 0.0))
        return model


    def _fit_iterative(self, df, x, d, y, w, loss):
        """Spark's "l-bfgs" path (LinearRegression.train with LeastSquaresAggregator / HuberAggregator):
        L-BFGS (OWL-QN with an L1 part) over the features scaled by their std; every objective evaluation is
        one K13 pass of the local rows ('squared' loss: margins, residuals and Xᵀr with the rows read once)
        all-reduced over the ranks. Squared error also scales the label by its std (the optimum is the
        normal equations' one); huber keeps the raw label and optimises the scale σ too (through log σ,
        which keeps it positive as Spark's L-BFGS-B bound does)."""
        from ..models.optim import lbfgs
        comm = df._comm
        n = int(x.shape[0])
        fi = self.getFitIntercept()
        reg, alpha = self.getRegParam(), self.getElasticNetParam()
        # weighted first and second moments of the features and the label, all-reduced (Spark's summarizer)
        ww = w if w is not None else None
        mom = torch.zeros(2 * d + 4, dtype=torch.float64, device=x.device)
        step = max(1, (1 << 24) // max(d, 1))
        for r0 in range(0, n, step):
            xf = x[r0:r0 + step, :d].to(torch.float64)
            yc = y[r0:r0 + step]
            wc = ww[r0:r0 + step] if ww is not None else torch.ones_like(yc)
            mom[:d] += wc @ xf
            mom[d:2 * d] += wc @ (xf * xf)
            mom[2 * d] += (wc * yc).sum()
            mom[2 * d + 1] += (wc * yc * yc).sum()
            mom[2 * d + 2] += wc.sum()
            mom[2 * d + 3] += (wc * wc).sum()
        comm.allreduce_(mom)
        m = mom.cpu().numpy()
        W, W2 = m[2 * d + 2], m[2 * d + 3]
        if W <= 0:
            raise ValueError("LinearRegression: empty training set")
        mx, my = m[:d] / W, m[2 * d] / W
        denom = W - W2 / W if W - W2 / W > 0 else W  # unbiased weighted variance (Spark's summarizer)
        sx = np.sqrt(np.maximum(m[d:2 * d] - W * mx * mx, 0.0) / denom)
        rawsy = math.sqrt(max(m[2 * d + 1] - W * my * my, 0.0) / denom)
        if loss == "squaredError" and rawsy == 0.0 and (fi or my == 0.0):
            # constant label: Spark returns zero coefficients and the label mean (or zero) as intercept
            model = LinearRegressionModel(np.zeros(d), my if fi else 0.0)
            self._copyValues(model)
            model._attach_summary(LinearRegressionTrainingSummary(model, df, None, d, False, [0.0], 0))
            return model
        sy = rawsy if rawsy > 0 else abs(my)
        inv = np.where(sx > 0, 1.0 / np.where(sx > 0, sx, 1.0), 0.0)  # constant features get no weight
        # Spark LinearRegression (l-bfgs): squared error runs on label / std(label) with effectiveRegParam =
        # regParam / std(label); huber keeps the raw label and regParam as given
        eff = reg if loss == "huber" else reg / sy
        l2, l1 = eff * (1.0 - alpha), eff * alpha
        std_pen = self.getStandardization()
        pen2 = np.full(d, l2) if std_pen else l2 * inv * inv
        pen1 = (np.full(d, l1) if std_pen else l1 * inv) if l1 > 0 else None
        huber = loss == "huber"
        eps = self.getEpsilon()
        dev = x.device
        ylab = y if huber else y / sy
        evals = [0]

        def fg(p):
            evals[0] += 1
            beta = p[:d]
            b = p[d] if fi else 0.0
            coef = torch.as_tensor(np.r_[beta * inv, b], dtype=torch.float64, device=dev)
            if not huber:
                o = glm_ops.loss_grad(x, d, ylab, coef, ww, loss="squared")
                comm.allreduce_(o)
                o = o.cpu().numpy()
                f = o[d + 1] / W + 0.5 * float(np.sum(pen2 * beta * beta))
                g = np.zeros_like(p)
                g[:d] = o[:d] * inv / W + pen2 * beta
                if fi:
                    g[d] = o[d] / W
                return f, g
            sig = math.exp(p[-1])
            mrg = glm_ops.linear_predict(x, d, coef) if n else torch.zeros(0, dtype=torch.float64, device=dev)
            r = y - mrg
            wr = ww if ww is not None else torch.ones_like(r)
            inb = r.abs() <= eps * sig
            lrow = torch.where(inb, 0.5 * (sig + r * r / sig), 0.5 * (sig + 2.0 * eps * r.abs() - sig * eps * eps))
            gm = torch.where(inb, -r / sig, -eps * torch.where(r >= 0, 1.0, -1.0).to(r.dtype))
            gs = torch.where(inb, 0.5 * (1.0 - (r / sig) ** 2), torch.full_like(r, 0.5 * (1.0 - eps * eps)))
            # Xᵀ(w·∂ℓ/∂m) through the 'squared' K13 (zero coefficients, label -(w·∂ℓ/∂m): residual = w·∂ℓ/∂m)
            o = glm_ops.loss_grad(x, d, -(wr * gm), torch.zeros(d + 1, dtype=torch.float64, device=dev),
                                  None, loss="squared")
            sc = torch.stack([(wr * lrow).sum(), (wr * gs).sum()])
            msg = torch.cat([o[:d + 1], sc])
            comm.allreduce_(msg)
            o = msg.cpu().numpy()
            f = o[d + 1] / W + 0.5 * float(np.sum(pen2 * beta * beta))
            g = np.zeros_like(p)
            g[:d] = o[:d] * inv / W + pen2 * beta
            if fi:
                g[d] = o[d] / W
            g[-1] = o[d + 2] / W * sig
            return f, g

        nv = d + 1 + (1 if huber else 0)
        p0 = np.zeros(nv)
        if fi and not huber:
            p0[d] = my / sy
        l1v = None
        if pen1 is not None:
            l1v = np.zeros(nv)
            l1v[:d] = pen1
        p, hist, iters = lbfgs(fg, p0, max(self.getMaxIter(), 0), self.getTol(), l1=l1v)
        scale_y = 1.0 if huber else sy
        coef = p[:d] * inv * scale_y
        intercept = (p[d] * scale_y) if fi else 0.0
        model = LinearRegressionModel(coef, intercept, math.exp(p[-1]) if huber else 1.0)
        self._copyValues(model)
        model._attach_summary(LinearRegressionTrainingSummary(model, df, None, d, False, hist, iters))
        return model


class LinearRegressionModel(Model):
    _params = _LR_PARAMS

    def __init__(self, coefficients=None, intercept: float = 0.0, scale: float = 1.0):
        super().__init__()
        self._coef = np.asarray(coefficients if coefficients is not None else [], dtype=np.float64)
        self._intercept = float(intercept)
        self._scale = float(scale)
        self._summary = None

    @property
    def coefficients(self) -> DenseVector:
        return DenseVector(self._coef)

    @property
    def intercept(self) -> float:
        return self._intercept

    @property
    def scale(self) -> float:
        return self._scale

    @property
    def numFeatures(self) -> int:
        return int(self._coef.shape[0])

    def predict(self, value) -> float:
        return float(as_array(value) @ self._coef + self._intercept)

    def _transform(self, df):
        x = df._feature_matrix(self.getFeaturesCol())
        coef = torch.as_tensor(np.r_[self._coef, self._intercept], device=x.device)
        pred = glm_ops.linear_predict(x, x.shape[1], coef, "identity")
        return _replace_col(df, self.getPredictionCol(), ColumnData(pred, None, T.DoubleType()))

    def evaluate(self, df) -> "LinearRegressionSummary":
        return LinearRegressionSummary(self, df)

    def _save_impl(self, path):
        import pyarrow as pa
        U.write_metadata(self, path)
        table = pa.Table.from_pylist(
            [{"intercept": self._intercept, "coefficients": U.vector_struct(self._coef), "scale": self._scale}],
            schema=pa.schema([pa.field("intercept", pa.float64(), nullable=False),
                              ("coefficients", U.vector_arrow_type()),
                              pa.field("scale", pa.float64(), nullable=False)]))
        U.write_parquet(path, "data", table)

    @classmethod
    def _load_impl(cls, path, md):
        row = U.read_parquet(path, "data").to_pylist()[0]
        m = cls(U.vector_from_struct(row["coefficients"]), row["intercept"], row.get("scale", 1.0))
        U.apply_params(m, md)
        return m


class LinearRegressionSummary:
    def __init__(self, model: LinearRegressionModel, df):
        self._model = model
        self._df = df
        self.labelCol = model.getLabelCol()
        self.predictionCol = model.getPredictionCol()
        self.featuresCol = model.getFeaturesCol()
        self._pred = None

    @property
    def predictions(self):
        if self._pred is None:
            self._pred = self._model.transform(self._df)
        return self._pred

    def _metric(self, name):
        return RegressionEvaluator(labelCol=self.labelCol, predictionCol=self.predictionCol,
                                   metricName=name).evaluate(self.predictions)

    @property
    def rootMeanSquaredError(self) -> float:
        return self._metric("rmse")

    @property
    def meanSquaredError(self) -> float:
        return self._metric("mse")

    @property
    def meanAbsoluteError(self) -> float:
        return self._metric("mae")

    @property
    def r2(self) -> float:
        return self._metric("r2")

    @property
    def explainedVariance(self) -> float:
        return self._metric("var")

    @property
    def numInstances(self) -> int:
        return self._df.count()

    @property
    def degreesOfFreedom(self) -> int:
        return self.numInstances - self._model.numFeatures - (1 if self._model.getFitIntercept() else 0)

    @property
    def r2adj(self) -> float:
        n = self.numInstances
        p = self._model.numFeatures
        k = 1 if self._model.getFitIntercept() else 0
        return 1.0 - (1.0 - self.r2) * (n - k) / max(n - p - k, 1)

    @property
    def residuals(self):
        from ..sql import functions as F
        p = self.predictions
        return p.select((F.col(self.labelCol) - F.col(self.predictionCol)).alias("residuals"))


class LinearRegressionTrainingSummary(LinearRegressionSummary):
    def __init__(self, model, df, G: Optional[np.ndarray], d: int, exact: bool, history=None, iterations: int = 1):
        super().__init__(model, df)
        self._G = G
        self._d = d
        self._exact = exact
        self.objectiveHistory = list(history) if history is not None else [0.0]
        self.totalIterations = int(iterations)

    def _cov(self):
        if self._G is None:
            raise RuntimeError("No Std. Error of coefficients available for this LinearRegressionModel "
                               "(the l-bfgs solver keeps no normal equations)")
        if not self._exact:
            raise RuntimeError("coefficient statistics need regParam=0 (normal equation solver)")
        G, d = self._G, self._d
        fi = self._model.getFitIntercept()
        idx = list(range(d)) + ([d] if fi else [])
        A = G[np.ix_(idx, idx)]
        n = G[d, d]
        dof = n - len(idx)
        coef = np.r_[self._model._coef, [self._model._intercept] if fi else []]
        # SSE from the Gram: yᵀy − 2 βᵀAᵀy + βᵀAβ
        Aty = G[idx, d + 1]
        sse = G[d + 1, d + 1] - 2 * coef @ Aty + coef @ A @ coef
        sigma2 = max(sse, 0.0) / max(dof, 1)
        cov = sigma2 * np.linalg.pinv(A)
        return coef, cov, dof

    @property
    def coefficientStandardErrors(self):
        _, cov, _ = self._cov()
        return list(np.sqrt(np.maximum(np.diag(cov), 0.0)))

    @property
    def tValues(self):
        coef, cov, _ = self._cov()
        se = np.sqrt(np.maximum(np.diag(cov), 1e-300))
        return list(coef / se)

    @property
    def pValues(self):
        from scipy import stats
        coef, cov, dof = self._cov()
        se = np.sqrt(np.maximum(np.diag(cov), 1e-300))
        t = np.abs(coef / se)
        return list(2 * stats.t.sf(t, max(dof, 1)))


# ------------------------------------------------------------------------------------------------ trees

class DecisionTreeRegressor(TreeEstimatorMixin, Estimator):
    _task = "regression"
    _params = dict(TREE_PARAMS, impurity=("variance", "criterion used for information gain (variance)", str),
                   seed=(_default_seed("org.apache.spark.ml.regression.DecisionTreeRegressor"), "random seed", int),
                   varianceCol=(None, "column name for the biased sample variance of prediction", None))

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        self._defaultParamMap.pop("weightCol", None)
        self._defaultParamMap.pop("varianceCol", None)

    def _fit(self, df):
        trees, d, _ = self._tree_fit(df)
        m = DecisionTreeRegressionModel()
        self._copyValues(m)
        m._init_trees(trees, d)
        return m


class DecisionTreeRegressionModel(TreeModelMixin, Model):
    _task = "regression"
    _params = DecisionTreeRegressor._params

    def __init__(self):
        super().__init__()
        self._init_trees([], 0)

    @staticmethod
    def _single_tree_class():
        return DecisionTreeRegressionModel


class RandomForestRegressor(TreeEstimatorMixin, Estimator):
    _task = "regression"
    _forest = True
    _params = dict(TREE_PARAMS, **FOREST_PARAMS,
                   impurity=("variance", "criterion used for information gain (variance)", str),
                   seed=(_default_seed("org.apache.spark.ml.regression.RandomForestRegressor"), "random seed", int))

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        self._defaultParamMap.pop("weightCol", None)

    def _fit(self, df):
        trees, d, _ = self._tree_fit(df)
        m = RandomForestRegressionModel()
        self._copyValues(m)
        m._init_trees(trees, d)
        return m


class RandomForestRegressionModel(TreeModelMixin, Model):
    _task = "regression"
    _forest = True
    _params = RandomForestRegressor._params

    def __init__(self):
        super().__init__()
        self._init_trees([], 0)

    @staticmethod
    def _single_tree_class():
        return DecisionTreeRegressionModel


class GBTRegressor(GBTEstimatorMixin, Estimator):
    """Gradient-boosted regression trees (Spark ``GBTRegressor``; lossType squared | absolute)."""
    _params = dict(TREE_PARAMS, **GBT_PARAMS,
                   lossType=("squared", "loss function which GBT tries to minimize (squared, absolute)", str),
                   seed=(_default_seed("org.apache.spark.ml.regression.GBTRegressor"), "random seed", int))

    def _fit(self, df):
        trees, tw, d = self._gbt_fit(df)
        m = GBTRegressionModel()
        self._copyValues(m)
        m._init_trees(trees, d, 2, tw)
        return m


class GBTRegressionModel(GBTModelMixin, Model):
    _params = GBTRegressor._params

    def __init__(self):
        super().__init__()
        self._init_trees([], 0)

    @staticmethod
    def _single_tree_class():
        return DecisionTreeRegressionModel


from .glr import (GeneralizedLinearRegression, GeneralizedLinearRegressionModel,  # noqa: E402,F401
                  GeneralizedLinearRegressionTrainingSummary)
from .regression_more import (AFTSurvivalRegression, AFTSurvivalRegressionModel,  # noqa: E402,F401
                              IsotonicRegression, IsotonicRegressionModel)
from .fm import FMRegressionModel, FMRegressor  # noqa: E402,F401
