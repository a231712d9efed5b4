"""Level-wise decision-tree / random-forest engine (Spark MLlib semantics).

Used by DecisionTreeRegressor / RandomForestRegressor (ref.py:150-158) and
DecisionTreeClassifier / RandomForestClassifier (ref.py:182-190).  Spark defaults
the reference relies on: maxDepth=5, maxBins=32,
minInstancesPerNode=1, minInfoGain=0, impurity variance (regression) / gini
(classification), RF numTrees=20 with Poisson(1) bootstrap weights and per-node
feature subsets ("auto" -> onethird for regression, sqrt for classification).

Pipeline per fit (each rank holds a row shard, all trees are grown together):
  1. split candidates: a counter-based row sample (GPU-count invariant) of
     max(maxBins², 10000) rows is all-gathered, thresholds per feature follow
     Spark's findSplitsForContinuousFeature rule (midpoints between distinct
     values, or count-stride quantiles when there are more than maxBins-1);
  2. K17 binize: bin codes [n, d] resident on the device — uint8 up to 256 bins (Spark's default
     maxBins = 32), 16-bit above (maxBins up to MAX_BINS = 32768), so large maxBins never wrap;
  3. per level: K18 histogram of (tree, node, feature, bin) stats for every tree at
     once, ONE all-reduce of the histogram buffer, best split per node on the host
     (identical on every rank), K20 routes rows to children;
  4. leaves keep the (weighted) impurity statistics Spark stores in NodeData.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np
import torch

from .. import _native
from .._native import c_dbl, c_int, c_ll, c_vp
from ..parallel.comm import Communicator, local_comm
from ..utils import rng

_native.register_kernel_sigs({
    "cml_tree_binize": (c_int, [c_vp, c_ll, c_ll, c_int, c_vp, c_int, c_vp, c_vp, c_int, c_vp]),
    "cml_tree_hist": (c_int, [c_vp, c_ll, c_int, c_int, c_vp, c_int, c_vp, c_vp, c_vp, c_int, c_int, c_vp, c_vp,
                              c_int, c_int, c_vp]),
    "cml_tree_best_split": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_vp, c_int, c_vp, c_vp, c_dbl, c_dbl,
                                    c_dbl, c_vp, c_vp]),
    "cml_tree_route": (c_int, [c_vp, c_ll, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_vp]),
    "cml_tree_predict": (c_int, [c_vp, c_ll, c_ll, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_dbl, c_vp,
                                 c_vp]),
    "cml_forest_vote": (c_int, [c_vp, c_ll, c_int, c_vp, c_vp, c_vp, c_vp]),
})


@dataclass
class Node:
    id: int = -1                       # preorder id (assigned at the end, Spark's NodeData id)
    prediction: float = 0.0
    impurity: float = 0.0
    stats: np.ndarray = None           # impurity calculator stats
    count: float = 0.0                 # weighted instance count
    gain: float = -1.0
    feature: int = -1                  # split feature (-1: leaf)
    threshold: float = 0.0
    split_bin: int = -1
    left: Optional["Node"] = None
    right: Optional["Node"] = None

    @property
    def is_leaf(self) -> bool:
        return self.feature < 0


@dataclass
class TreeParams:
    task: str = "regression"           # or "classification"
    num_classes: int = 2
    impurity: str = "variance"
    max_depth: int = 5
    max_bins: int = 32
    min_instances: int = 1
    min_weight_fraction: float = 0.0
    min_info_gain: float = 0.0
    num_trees: int = 1
    subsampling_rate: float = 1.0
    bootstrap: bool = True
    feature_subset: str = "auto"
    seed: int = 0


# ---------------------------------------------------------------------------------------------- impurity

def impurity_of(stats: np.ndarray, kind: str) -> float:
    if kind == "variance":
        w = stats[0]
        if w <= 0:
            return 0.0
        m = stats[1] / w
        return max(stats[2] / w - m * m, 0.0)
    tot = stats.sum()
    if tot <= 0:
        return 0.0
    p = stats / tot
    if kind == "gini":
        return float(1.0 - (p * p).sum())
    nz = p[p > 0]
    return float(-(nz * np.log2(nz)).sum())


def count_of(stats: np.ndarray, kind: str) -> float:
    return float(stats[0]) if kind == "variance" else float(stats.sum())


def predict_of(stats: np.ndarray, kind: str) -> float:
    if kind == "variance":
        return float(stats[1] / stats[0]) if stats[0] > 0 else 0.0
    return float(np.argmax(stats))


# ---------------------------------------------------------------------------------------------- split candidates

def continuous_splits(values: np.ndarray, num_splits: int) -> np.ndarray:
    """Spark findSplitsForContinuousFeature: midpoints of distinct values, or count-stride cut points."""
    if values.size == 0:
        return np.zeros(0)
    uniq, counts = np.unique(values, return_counts=True)
    if uniq.size - 1 <= num_splits:
        return (uniq[:-1] + uniq[1:]) / 2.0
    # Spark walks the distinct values once, cutting between values i-1 and i when the cumulative
    # count there is closer to the running target than the count after value i, i.e. when the
    # midpoint (cum[i-1] + cum[i]) / 2 lies past the target, then advancing the target by one stride.
    # The midpoints increase, so the cut for each target is a binary search — a loop over at most
    # num_splits targets instead of over the (up to ~10^4 sampled) distinct values per feature.
    # `_continuous_splits_loop` keeps the walk itself as the test oracle.
    stride = counts.sum() / (num_splits + 1)
    cum = np.cumsum(counts)
    mid2 = cum[:-1] + cum[1:]  # 2 x midpoint between distinct values i-1 and i (i = 1..u-1)
    cuts = []
    nxt = 0  # first boundary (index into mid2) still available
    target = stride
    while nxt < mid2.size:
        j = max(nxt, int(np.searchsorted(mid2, 2.0 * target, side="right")))
        if j >= mid2.size:
            break
        cuts.append(j)
        nxt = j + 1
        target += stride
    cuts = np.asarray(cuts, dtype=np.int64)
    return (uniq[cuts] + uniq[cuts + 1]) / 2.0


def _continuous_splits_loop(values: np.ndarray, num_splits: int) -> np.ndarray:
    """The value-by-value walk continuous_splits replaces (reference behaviour; tests only)."""
    if values.size == 0:
        return np.zeros(0)
    uniq, counts = np.unique(values, return_counts=True)
    if uniq.size - 1 <= num_splits:
        return (uniq[:-1] + uniq[1:]) / 2.0
    stride = counts.sum() / (num_splits + 1)
    out = []
    current = counts[0]
    target = stride
    for i in range(1, uniq.size):
        prev = current
        current += counts[i]
        if abs(prev - target) < abs(current - target):
            out.append((uniq[i - 1] + uniq[i]) / 2.0)
            target += stride
    return np.asarray(out, dtype=np.float64)


def subset_size(strategy: str, d: int, task: str, num_trees: int) -> int:
    s = strategy.lower()
    if s == "auto":
        s = "all" if num_trees == 1 else ("sqrt" if task == "classification" else "onethird")
    if s == "all":
        return d
    if s == "sqrt":
        return max(1, int(math.ceil(math.sqrt(d))))
    if s == "log2":
        return max(1, int(math.ceil(math.log2(d))))
    if s == "onethird":
        return max(1, int(math.ceil(d / 3.0)))
    try:
        v = float(s)
    except ValueError:
        raise ValueError(f"unknown featureSubsetStrategy {strategy!r}")
    if v.is_integer() and v >= 1:
        return min(d, int(v))
    return max(1, int(math.ceil(v * d)))


# ---------------------------------------------------------------------------------------------- engine

MAX_BINS = 32768  # 16-bit bin codes (int16 storage, read as uint16 by the kernels)


def bin_dtype(nbins: int) -> torch.dtype:
    """Storage type of the bin codes: one byte while every code fits (nbins <= 256), two above."""
    if nbins > MAX_BINS:
        raise ValueError(f"maxBins must be <= {MAX_BINS}, got {nbins}")
    return torch.uint8 if nbins <= 256 else torch.int16


class ForestEngine:
    def __init__(self, x: torch.Tensor, y: torch.Tensor, params: TreeParams, comm: Optional[Communicator] = None,
                 row_ids: Optional[torch.Tensor] = None, weights: Optional[torch.Tensor] = None):
        self.comm = comm or local_comm()
        self.p = params
        self.x = x.to(torch.float64).contiguous()
        self.n, self.d = int(x.shape[0]), int(x.shape[1])
        self.dev = x.device
        self.gpu = x.is_cuda
        self.y = y.to(torch.float64).contiguous()
        self.row_ids = row_ids if row_ids is not None else torch.arange(self.n, device=self.dev)
        self.sample_weight = weights
        self.kind = params.impurity
        self.S = 3 if self.kind == "variance" else params.num_classes
        if not 2 <= params.max_bins <= MAX_BINS:
            raise ValueError(f"maxBins must be in [2, {MAX_BINS}], got {params.max_bins}")

    # -------------------------------------------------------------- splits
    def find_splits(self) -> List[np.ndarray]:
        p = self.p
        gn = self.comm.sum_scalar(float(self.n))
        required = max(p.max_bins * p.max_bins, 10000)
        frac = min(required / max(gn, 1.0), 1.0)
        if self.n:
            u = rng.uniform(self.row_ids, p.seed, stream=21)
            sample = self.x[u < frac] if frac < 1.0 else self.x
        else:
            sample = self.x
        allv = self.comm.allgather_cat(sample.to(torch.float64)).cpu().numpy()
        return [continuous_splits(allv[:, j], p.max_bins - 1) for j in range(self.d)]

    def binize(self, splits: List[np.ndarray]) -> torch.Tensor:
        ms = max(1, max((len(s) for s in splits), default=1))
        thr = np.full((self.d, ms), np.inf)
        ns = np.zeros(self.d, dtype=np.int32)
        for j, s in enumerate(splits):
            thr[j, : len(s)] = s
            ns[j] = len(s)
        self.nbins = ms + 1
        bdt = bin_dtype(self.nbins)
        if not self.gpu or self.n == 0:
            t = torch.as_tensor(thr, device=self.dev)
            bins = torch.empty((self.n, self.d), dtype=bdt, device=self.dev)
            for j in range(self.d):
                bins[:, j] = torch.searchsorted(t[j, : max(ns[j], 0)].contiguous(), self.x[:, j].contiguous(),
                                                right=False).to(bdt) if ns[j] else 0
            return bins
        thr_t = torch.as_tensor(thr, device=self.dev)
        ns_t = torch.as_tensor(ns, device=self.dev)
        bins = torch.empty((self.n, self.d), dtype=bdt, device=self.dev)
        st = _native.kernels().cml_tree_binize(self.x.data_ptr(), self.n, self.x.stride(0), self.d, thr_t.data_ptr(),
                                               ms, ns_t.data_ptr(), bins.data_ptr(), bins.element_size(),
                                               _native.stream_ptr())
        _native.check(st, "tree_binize")
        return bins

    # -------------------------------------------------------------- histogram / routing
    def fixed_point_scales(self, wt) -> np.ndarray:
        """Per-statistic scales 2^e of the GPU histogram's 64-bit fixed point: the largest e for
        which n_global · max w · max|y|^p still fits 2^61 (global maxima, so every rank and every
        world size uses the same scales and the integer histograms add up exactly)."""
        ymax = float(self.y.abs().max().item()) if (self.n and self.kind == "variance") else 1.0
        wmax = float(wt.max().item()) if (wt is not None and self.n) else 1.0
        ymax = self.comm.max_scalar(max(ymax, 1e-300))
        wmax = self.comm.max_scalar(max(wmax, 1e-300))
        gn = max(self.comm.sum_scalar(float(self.n)), 1.0)
        out = np.ones(3)
        for s in range(3):
            bound = gn * wmax * (ymax ** s if self.kind == "variance" else 1.0)
            out[s] = 2.0 ** max(-1000, min(1000, 61 - math.ceil(math.log2(max(bound, 1e-300)))))
        return out

    def histogram(self, bins, node_of, wt, nodes: int) -> torch.Tensor:
        """(T, nodes, d, nbins, S) statistics of this rank's rows in int64 fixed point (scale
        ``self.scales``; converted in best_splits after the all-reduce). Both paths quantise each row's
        w, w·y, w·y² the same way (f64 product, exact power-of-two scale, round half to even), so the
        integer histograms — and every node's statistics — are bit-identical between the GPU kernel
        (K18), the CPU form and any world size."""
        T, S, d, nb = self.p.num_trees, self.S, self.d, self.nbins
        if self.gpu:
            out = torch.zeros((T, nodes, d, nb, S), dtype=torch.int64, device=self.dev)
            if self.n == 0 or nodes == 0:
                return out
            cls = self.y.to(torch.int32).contiguous() if self.kind != "variance" else None
            rb = max(1, min((self.n + 255) // 256, 1024 // max(T, 1) + 1))
            st = _native.kernels().cml_tree_hist(bins.data_ptr(), self.n, d, nb, node_of.data_ptr(), T,
                                                 wt.data_ptr() if wt is not None else 0, self.y.data_ptr(),
                                                 cls.data_ptr() if cls is not None else 0, S, nodes,
                                                 self._scales_host.data_ptr(), out.data_ptr(), rb,
                                                 bins.element_size(), _native.stream_ptr())
            _native.check(st, "tree_hist")
            return out
        out = torch.zeros((T, nodes, d, nb, S), dtype=torch.int64, device=self.dev)
        if self.n == 0 or nodes == 0:
            return out
        flat = out.view(-1)
        sc = [float(v) for v in self.scales]
        for t in range(T):
            nd = node_of[t]
            active = nd >= 0
            if wt is not None:
                active = active & (wt[t] > 0)
            idx_rows = torch.nonzero(active).flatten()
            if idx_rows.numel() == 0:
                continue
            w = wt[t][idx_rows].to(torch.float64) if wt is not None else torch.ones(idx_rows.numel(),
                                                                                   dtype=torch.float64)
            nsel = nd[idx_rows].long()
            b = bins[idx_rows].long()
            yy = self.y[idx_rows]
            feat = torch.arange(d, device=self.dev)
            base = (((t * nodes + nsel)[:, None] * d + feat[None, :]) * nb + b) * S
            if self.kind == "variance":
                wy = w * yy
                for s, v in enumerate((w, wy, wy * yy)):
                    q = torch.round(v * sc[s]).to(torch.int64)
                    flat.index_add_(0, (base + s).reshape(-1), q[:, None].expand(-1, d).reshape(-1))
            else:
                c = yy.long()
                q = torch.round(w * sc[0]).to(torch.int64)
                flat.index_add_(0, (base + c[:, None]).reshape(-1), q[:, None].expand(-1, d).reshape(-1))
        return out

    def route(self, bins, node_of, split_feat, split_bin, left_id, right_id, nodes: int) -> None:
        T = self.p.num_trees
        if self.n == 0:
            return
        sf = torch.as_tensor(split_feat, dtype=torch.int32, device=self.dev).contiguous()
        sb = torch.as_tensor(split_bin, dtype=torch.int32, device=self.dev).contiguous()
        li = torch.as_tensor(left_id, dtype=torch.int32, device=self.dev).contiguous()
        ri = torch.as_tensor(right_id, dtype=torch.int32, device=self.dev).contiguous()
        if self.gpu:
            st = _native.kernels().cml_tree_route(bins.data_ptr(), self.n, self.d, T, nodes, node_of.data_ptr(),
                                                  sf.data_ptr(), sb.data_ptr(), li.data_ptr(), ri.data_ptr(),
                                                  bins.element_size(), _native.stream_ptr())
            _native.check(st, "tree_route")
            return
        for t in range(T):
            nd = node_of[t]
            act = nd >= 0
            k = (t * nodes + nd.clamp(min=0)).long()
            f = sf[k]
            leaf = f < 0
            fb = bins.gather(1, f.clamp(min=0).long().reshape(-1, 1)).reshape(-1).to(torch.int32)
            go_left = fb <= sb[k]
            new = torch.where(go_left, li[k], ri[k])
            new = torch.where(leaf, torch.full_like(new, -1), new)
            node_of[t] = torch.where(act, new, nd)

    # -------------------------------------------------------------- fit
    def fit(self, splits: Optional[List[np.ndarray]] = None, bins: Optional[torch.Tensor] = None,
            replay: Optional[List[np.ndarray]] = None, on_level=None) -> List[Node]:
        """Grow ``num_trees`` trees level-wise.  ``splits``/``bins`` let a caller that fits many
        trees on the same rows (gradient boosting) find candidates and bin the rows once.

        Checkpoints: a level's whole outcome is its K19 result ``res`` (identical on every
        rank: it comes from the all-reduced histogram), so ``on_level(levels_done, [res_0, ...])`` after
        each level is the forest's state, and ``replay`` (those arrays) resumes a fit — completed levels
        rebuild their nodes and re-route the rows from the saved results (no histogram pass), the feature
        subset draws are replayed, and the fit continues bit for bit as the uninterrupted one."""
        p = self.p
        replay = list(replay) if replay is not None else []
        done: List[np.ndarray] = []
        T = p.num_trees
        if splits is None:
            splits = self.find_splits()
        self.splits = splits
        if bins is None:
            bins = self.binize(splits)
        self.bins = bins
        # bagging weights (Spark BaggedPoint: Poisson(rate) with replacement, Bernoulli without)
        if T > 1 and p.bootstrap:
            wt = torch.stack([rng.poisson1(self.row_ids, p.seed, 1000 + t).to(torch.float32)
                              for t in range(T)]) if p.subsampling_rate == 1.0 else torch.stack(
                [_poisson(self.row_ids, p.seed, 1000 + t, p.subsampling_rate) for t in range(T)])
        elif p.subsampling_rate < 1.0:
            wt = torch.stack([(rng.uniform(self.row_ids, p.seed, 1000 + t) < p.subsampling_rate).to(torch.float32)
                              for t in range(T)])
        else:
            wt = None
        if self.sample_weight is not None:
            sw = self.sample_weight.to(torch.float32)
            wt = sw[None, :].repeat(T, 1) if wt is None else wt * sw[None, :]
        if wt is not None:
            wt = wt.to(self.dev).contiguous()
        node_of = torch.zeros((T, self.n), dtype=torch.int32, device=self.dev)
        self.scales = self.fixed_point_scales(wt)
        if self.gpu:
            self._scales_host = torch.as_tensor(self.scales, dtype=torch.float64).contiguous()
        k_sub = subset_size(p.feature_subset, self.d, p.task, T)
        roots = [Node() for _ in range(T)]
        level_nodes: List[List[Node]] = [[r] for r in roots]
        rs = np.random.RandomState(p.seed & 0x7FFFFFFF)
        for depth in range(p.max_depth + 1):
            nodes = max(len(l) for l in level_nodes)
            if nodes == 0 or depth == p.max_depth:
                break  # nodes at maxDepth are leaves; their stats came with the parent's split
            from ..utils.fault import maybe_fail
            maybe_fail("forest.level", depth)  # crash point
            # per-node feature subsets (RF), drawn for every node of the level in order, identically on
            # every rank (same seed, same draws)
            masks = np.ones((T, nodes, self.d), dtype=np.uint8)
            if k_sub < self.d:
                masks[:] = 0
                for t in range(T):
                    for j in range(len(level_nodes[t])):
                        masks[t, j, rs.choice(self.d, k_sub, replace=False)] = 1
            if depth < len(replay):
                res = np.asarray(replay[depth], dtype=np.float64)
            else:
                hist = self.histogram(bins, node_of, wt, nodes)
                self.comm.allreduce_(hist)
                res = self.best_splits(hist, masks, nodes)  # [T, nodes, 3 + 3S] (K19)
            done.append(res)
            S = self.S
            split_feat = np.full((T, nodes), -1, dtype=np.int32)
            split_bin = np.zeros((T, nodes), dtype=np.int32)
            left_id = np.full((T, nodes), -1, dtype=np.int32)
            right_id = np.full((T, nodes), -1, dtype=np.int32)
            next_level: List[List[Node]] = [[] for _ in range(T)]
            for t in range(T):
                for j, node in enumerate(level_nodes[t]):
                    r = res[t, j]
                    if node.stats is None:
                        node.stats = r[3:3 + S].copy()
                    node.count = count_of(node.stats, self.kind)
                    node.impurity = impurity_of(node.stats, self.kind)
                    node.prediction = predict_of(node.stats, self.kind)
                    gain, f = float(r[0]), int(r[1])
                    if node.count <= 0 or f < 0 or not gain > 0:
                        continue  # leaf (Spark: isLeaf = gain <= 0)
                    b = int(r[2])
                    node.gain, node.feature, node.split_bin = gain, f, b
                    node.threshold = float(splits[f][b])
                    node.left = Node(stats=r[3 + S:3 + 2 * S].copy())
                    node.right = Node(stats=r[3 + 2 * S:3 + 3 * S].copy())
                    for child in (node.left, node.right):
                        child.count = count_of(child.stats, self.kind)
                        child.impurity = impurity_of(child.stats, self.kind)
                        child.prediction = predict_of(child.stats, self.kind)
                    split_feat[t, j] = f
                    split_bin[t, j] = b
                    left_id[t, j] = len(next_level[t])
                    next_level[t].append(node.left)
                    right_id[t, j] = len(next_level[t])
                    next_level[t].append(node.right)
            if depth < p.max_depth and any(next_level):
                self.route(bins, node_of, split_feat.reshape(-1), split_bin.reshape(-1), left_id.reshape(-1),
                           right_id.reshape(-1), nodes)
            if on_level is not None and depth >= len(replay):
                on_level(depth + 1, done)
            level_nodes = next_level
            if not any(level_nodes):
                break
        for r in roots:
            _assign_ids(r)
        return roots

    def best_splits(self, hist, masks: np.ndarray, nodes: int) -> np.ndarray:
        """K19: per (tree, node) [gain, feature, bin, total S, left S, right S] of the best split among
        candidates whose children both reach the minimum weight and whose gain reaches minInfoGain (feature
        -1: none). Spark's binsToBestSplit takes the first maximum in (feature, bin) order; exact ties (two
        features separating the same rows of a small node) are common and rounding breaks them arbitrarily,
        so both paths take the first (feature, bin) within TIE_REL·|G| of the maximum G. GPU: one workgroup
        per node on the fixed-point histogram; CPU: the same rule vectorised in numpy."""
        T, S, d, nb = self.p.num_trees, self.S, self.d, self.nbins
        p = self.p
        kind_id = {"variance": 0, "gini": 1, "entropy": 2}[self.kind]
        nsplit = np.array([len(sp) for sp in self.splits], dtype=np.int32)
        if self.gpu:
            out = torch.empty((T * nodes, 3 + 3 * S), dtype=torch.float64, device=self.dev)
            sc = torch.as_tensor(self.scales, dtype=torch.float64, device=self.dev)
            mk = torch.as_tensor(masks.reshape(-1), device=self.dev)
            ns = torch.as_tensor(nsplit, device=self.dev)
            st = _native.kernels().cml_tree_best_split(hist.data_ptr(), T * nodes, d, nb, S, sc.data_ptr(), kind_id,
                                                        mk.data_ptr(), ns.data_ptr(), float(p.min_instances),
                                                        float(p.min_weight_fraction), float(p.min_info_gain),
                                                        out.data_ptr(), _native.stream_ptr())
            _native.check(st, "tree_best_split")
            return out.cpu().numpy().reshape(T, nodes, 3 + 3 * S)
        hi = hist.cpu().numpy()                                   # [T, nodes, d, nb, S] int64
        tot_i = hi[:, :, 0].sum(axis=2) if d else np.zeros((T, nodes, S), dtype=np.int64)  # [T, nodes, S]
        left_i = np.cumsum(hi, axis=3)
        # to f64 exactly as K19 does: (double)integer / 2^e
        scv = np.asarray(self.scales[:S] if self.kind == "variance" else [self.scales[0]] * S, dtype=np.float64)
        tot = tot_i.astype(np.float64) / scv
        left = left_i.astype(np.float64) / scv
        right = (tot_i[:, :, None, None, :] - left_i).astype(np.float64) / scv
        cnt = (lambda a: a[..., 0]) if self.kind == "variance" else (lambda a: a.sum(-1))
        wtot, wl, wr = cnt(tot), cnt(left), cnt(right)
        imp_t, imp_l, imp_r = _impurity_vec(tot, self.kind), _impurity_vec(left, self.kind), _impurity_vec(right,
                                                                                                       self.kind)
        with np.errstate(divide="ignore", invalid="ignore"):
            gain = imp_t[:, :, None, None] - (wl / wtot[:, :, None, None]) * imp_l - (wr / wtot[:, :, None, None]) * imp_r
        min_w = np.maximum(p.min_instances, p.min_weight_fraction * wtot)[:, :, None, None]
        ok = (wl >= min_w) & (wr >= min_w) & (wl > 0) & (wr > 0)
        ok &= np.arange(nb)[None, None, None, :] < nsplit[None, None, :, None]
        ok &= masks[:, :, :, None].astype(bool)
        ok &= gain >= p.min_info_gain
        gain = np.where(ok, gain, -np.inf)
        flat = gain.reshape(T, nodes, d * nb)
        if d * nb:
            # order-independent tie rule (see trees.hip K19): first (feature, bin) within 1e-12·|G| of the max G
            G = flat.max(-1)
            near = flat >= (G - TIE_REL * np.abs(G))[..., None]
            arg = near.argmax(-1)
            best = np.take_along_axis(flat, arg[..., None], -1)[..., 0]
            valid = np.isfinite(G)
        else:
            arg = np.zeros((T, nodes), dtype=np.int64)
            best = np.full((T, nodes), -np.inf)
            valid = np.zeros((T, nodes), dtype=bool)
        f, b = arg // max(nb, 1), arg % max(nb, 1)
        ti, ni = np.meshgrid(np.arange(T), np.arange(nodes), indexing="ij")
        out = np.zeros((T, nodes, 3 + 3 * S))
        out[..., 0] = np.where(valid, best, -np.inf)
        out[..., 1] = np.where(valid, f, -1)
        out[..., 2] = np.where(valid, b, -1)
        out[..., 3:3 + S] = tot
        if d * nb:
            out[..., 3 + S:3 + 2 * S] = left[ti, ni, f, b]
            out[..., 3 + 2 * S:] = right[ti, ni, f, b]
        return out


TIE_REL = 1e-12  # kTreeTieRel in trees.hip


def _impurity_vec(st: np.ndarray, kind: str) -> np.ndarray:
    """impurity_of over the last axis of a stats array."""
    with np.errstate(divide="ignore", invalid="ignore"):
        if kind == "variance":
            w = st[..., 0]
            m = st[..., 1] / w
            v = np.maximum(st[..., 2] / w - m * m, 0.0)
            return np.where(w > 0, v, 0.0)
        tot = st.sum(-1)
        pr = st / tot[..., None]
        if kind == "gini":
            r = 1.0 - (pr * pr).sum(-1)
        else:
            r = -np.where(pr > 0, pr * np.log2(np.where(pr > 0, pr, 1.0)), 0.0).sum(-1)
        return np.where(tot > 0, r, 0.0)


def _poisson(row_ids, seed, stream, lam):
    u = rng.uniform(row_ids, seed, stream)
    out = torch.zeros_like(u, dtype=torch.float32)
    p = math.exp(-lam)
    cdf = p
    for k in range(1, 17):
        out += (u >= cdf).to(torch.float32)
        p = p * lam / k
        cdf += p
    return out


def _assign_ids(root: Node) -> None:
    """Spark NodeData ids: preorder numbering (root 0, then the left subtree, then the right)."""
    nid = 0
    stack = [root]
    while stack:
        n = stack.pop()
        n.id = nid
        nid += 1
        if not n.is_leaf:
            stack.append(n.right)
            stack.append(n.left)


def preorder(root: Node) -> List[Node]:
    out = []
    stack = [root]
    while stack:
        n = stack.pop()
        out.append(n)
        if not n.is_leaf:
            stack.append(n.right)
            stack.append(n.left)
    return out


def tree_depth(root: Node) -> int:
    if root.is_leaf:
        return 0
    return 1 + max(tree_depth(root.left), tree_depth(root.right))


def num_nodes(root: Node) -> int:
    return len(preorder(root))


def feature_importances(trees: List[Node], d: int, per_tree_normalization: bool = True) -> np.ndarray:
    """Spark: per tree Σ gain·count over split nodes, normalised; forest = mean, renormalised.
    GBT models sum the raw per-tree importances (``perTreeNormalization = false``)."""
    total = np.zeros(d)
    for t in trees:
        imp = np.zeros(d)
        for n in preorder(t):
            if not n.is_leaf:
                imp[n.feature] += n.gain * n.count
        s = imp.sum()
        if s > 0 and per_tree_normalization:
            imp /= s
        total += imp
    if len(trees) > 1 and per_tree_normalization:
        total /= len(trees)
    s = total.sum()
    return total / s if s > 0 else total


def predict_forest(trees: List[Node], x: torch.Tensor, kind: str, num_classes: int, average: bool,
                   normalize_leaves: bool, tree_weights: Optional[Sequence[float]] = None) -> torch.Tensor:
    """[n, S] per-row accumulated leaf values: regression -> prediction (mean if `average`),
    classification -> summed class distributions (normalised per tree when `normalize_leaves`)."""
    S = 1 if kind == "variance" else num_classes
    feats, thrs, lefts, rights, leaves, roots = [], [], [], [], [], []
    for ti, t in enumerate(trees):
        tw = 1.0 if tree_weights is None else float(tree_weights[ti])
        nodes = preorder(t)
        base = len(feats)
        roots.append(base)
        index = {id(nd): base + i for i, nd in enumerate(nodes)}
        for nd in nodes:
            feats.append(nd.feature if not nd.is_leaf else -1)
            thrs.append(nd.threshold)
            lefts.append(index[id(nd.left)] if not nd.is_leaf else -1)
            rights.append(index[id(nd.right)] if not nd.is_leaf else -1)
            if kind == "variance":
                leaves.append([nd.prediction * tw])
            else:
                st = np.asarray(nd.stats, dtype=np.float64)
                if normalize_leaves:
                    s = st.sum()
                    st = st / s if s > 0 else st
                leaves.append(list(st))
    dev = x.device
    n = x.shape[0]
    xx = x.to(torch.float64).contiguous()
    if x.is_cuda and S <= 16:
        # K21 writes every element and takes the forest mean itself: no tensor op of its own on the device
        out = torch.empty((n, S), dtype=torch.float64, device=dev)
        if n == 0:
            return out
        to = lambda a, dt: torch.as_tensor(np.asarray(a), dtype=dt, device=dev).contiguous()  # noqa: E731
        r, f, th, l, rr, lv = (to(roots, torch.int32), to(feats, torch.int32), to(thrs, torch.float64),
                               to(lefts, torch.int32), to(rights, torch.int32),
                               to(np.asarray(leaves, dtype=np.float64).reshape(-1), torch.float64))
        div = float(len(trees)) if average and len(trees) > 1 else 1.0
        st = _native.kernels().cml_tree_predict(xx.data_ptr(), n, xx.stride(0), len(trees), r.data_ptr(),
                                                f.data_ptr(), th.data_ptr(), l.data_ptr(), rr.data_ptr(),
                                                lv.data_ptr(), S, div, out.data_ptr(), _native.stream_ptr())
        _native.check(st, "tree_predict")
        return out
    out = torch.zeros((n, S), dtype=torch.float64, device=dev)
    if n == 0:
        return out
    f = torch.as_tensor(feats, dtype=torch.long, device=dev)
    th = torch.as_tensor(thrs, dtype=torch.float64, device=dev)
    l = torch.as_tensor(lefts, dtype=torch.long, device=dev)
    rr = torch.as_tensor(rights, dtype=torch.long, device=dev)
    lv = torch.as_tensor(np.asarray(leaves, dtype=np.float64), device=dev)
    for root in roots:
        k = torch.full((n,), root, dtype=torch.long, device=dev)
        for _ in range(64):
            ff = f[k]
            inner = ff >= 0
            if not bool(inner.any()):
                break
            v = xx.gather(1, ff.clamp(min=0).reshape(-1, 1)).reshape(-1)
            nxt = torch.where(v <= th[k], l[k], rr[k])
            k = torch.where(inner, nxt, k)
        out += lv[k]
    if average and len(trees) > 1:
        # true division on every device (a python-scalar divisor becomes a reciprocal multiply on the GPU)
        out /= torch.full((1,), float(len(trees)), dtype=torch.float64, device=dev)
    return out


def forest_vote(raw: torch.Tensor, thresholds: Optional[Sequence[float]] = None):
    """(probability [n, S], prediction [n] f64) of a classifier's summed leaf distributions: raw / row sum
    (uniform when the sum is not positive), prediction = first argmax of probability / thresholds. One
    K21b launch on the device (Spark ProbabilisticClassificationModel.transform)."""
    n, S = raw.shape
    if raw.is_cuda and S <= 16:
        rr = raw.to(torch.float64).contiguous()
        prob = torch.empty_like(rr)
        pred = torch.empty(n, dtype=torch.float64, device=raw.device)
        t = None
        if thresholds:
            t = torch.as_tensor(np.asarray(thresholds, dtype=np.float64), device=raw.device)
        st = _native.kernels().cml_forest_vote(rr.data_ptr(), n, S, 0 if t is None else t.data_ptr(),
                                               prob.data_ptr(), pred.data_ptr(), _native.stream_ptr())
        _native.check(st, "forest_vote")
        return prob, pred
    s = raw.sum(1, keepdim=True)
    prob = torch.where(s > 0, raw / s.clamp(min=1e-300), torch.full_like(raw, 1.0 / S))
    if thresholds:
        t = torch.as_tensor(np.asarray(thresholds, dtype=np.float64), device=prob.device)
        return prob, torch.argmax(prob / t.clamp(min=1e-300), 1).to(torch.float64)
    return prob, torch.argmax(prob, 1).to(torch.float64)


# ---------------------------------------------------------------------------------------------- boosting

GBT_LOSSES = ("squared", "absolute", "logistic")


def gbt_residual(loss: str, f: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """Pseudo-residual ``-dL/dF`` of Spark's losses (SquaredError 2(y-F), AbsoluteError sign(y-F),
    LogLoss on labels in {-1,+1}: 4y / (1 + exp(2yF)))."""
    if loss == "squared":
        return 2.0 * (y - f)
    if loss == "absolute":
        return torch.sign(y - f)
    return 4.0 * y / (1.0 + torch.exp(torch.clamp(2.0 * y * f, max=700.0)))


def gbt_loss(loss: str, f: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    if loss == "squared":
        return (y - f) ** 2
    if loss == "absolute":
        return (y - f).abs()
    m = 2.0 * y * f
    return 2.0 * torch.where(m < -30, -m, torch.log1p(torch.exp(-m)))  # Spark LogLoss: 2 log(1 + e^(-2yF))


def predict_tree(tree: Node, x: torch.Tensor) -> torch.Tensor:
    return predict_forest([tree], x, "variance", 1, average=False, normalize_leaves=False)[:, 0]


def fit_gbt(x: torch.Tensor, y: torch.Tensor, params: TreeParams, max_iter: int, step_size: float, loss: str,
            comm: Optional[Communicator] = None, row_ids: Optional[torch.Tensor] = None,
            weights: Optional[torch.Tensor] = None, valid: Optional[torch.Tensor] = None,
            validation_tol: float = 0.01, ckpt=None):
    """Gradient-boosted regression trees (Spark ``GradientBoostedTrees.boost``): tree 0 is fit on the
    labels with weight 1, tree m on the pseudo-residuals of the running margin with weight
    ``step_size``.  Candidate splits and the bin codes (K16/K17) are built once and reused by
    every tree; each tree is one level-wise pass of the K18/K19/K20 kernels plus an all-reduce
    per level; the margin is updated in place by K21.  Labels for ``logistic`` must already be
    in {-1, +1}.  ``valid`` (bool per row) holds rows out of training and stops early once the
    validation loss improves by less than ``validation_tol * max(loss, 0.01)`` (Spark's rule).
    ``ckpt`` (utils/checkpoint.FitCheckpoint): the K19 results of every completed tree are saved every
    ``checkpointInterval`` trees; a resumed fit replays those trees (nodes, margin and validation updates
    exactly as they happened) and boosts on — the uninterrupted fit bit for bit.
    Returns (trees, tree_weights)."""
    comm = comm or local_comm()
    if loss not in GBT_LOSSES:
        raise ValueError(f"unsupported GBT loss {loss!r}")
    n = int(x.shape[0])
    row_ids = row_ids if row_ids is not None else torch.arange(n, device=x.device)
    y = y.to(torch.float64)
    xv = yv = None
    if valid is not None:
        keep = ~valid
        xv, yv = x[valid].to(torch.float64).contiguous(), y[valid]
        x, y, row_ids = x[keep], y[keep], row_ids[keep]
        weights = weights[keep] if weights is not None else None
    p = TreeParams(**{**params.__dict__, "task": "regression", "impurity": "variance", "num_trees": 1,
                      "bootstrap": False})
    eng = ForestEngine(x, y, p, comm, row_ids=row_ids, weights=weights)
    splits = eng.find_splits()
    bins = eng.binize(splits)
    trees: List[Node] = []
    tw: List[float] = []
    f = torch.zeros_like(eng.y)
    fv = torch.zeros_like(yv) if yv is not None else None
    best_err, best_m = float("inf"), 0
    from ..utils.fault import maybe_fail
    saved: List[List[np.ndarray]] = []  # K19 results per level of every completed tree
    if ckpt is not None:
        got = ckpt.load()
        if got is not None:
            arrs = got[1]
            for mm in range(int(arrs["trees"][0])):
                saved.append([arrs[f"t{mm}_l{lv}"] for lv in range(int(arrs["levels"][mm]))])
    resumed = len(saved)
    for m in range(max_iter):
        if m >= resumed:
            maybe_fail("forest.tree", m)  # crash point
        w = 1.0 if m == 0 else step_size
        if m > 0:
            eng.y = gbt_residual(loss, f, y).contiguous()
        eng.p.seed = params.seed + m
        levels: List[np.ndarray] = []
        t = eng.fit(splits, bins, replay=saved[m] if m < resumed else None,
                    on_level=lambda _, done: levels.__setitem__(slice(None), list(done)))[0]
        if m >= resumed:
            saved.append(list(levels))
            if ckpt is not None and ckpt.due(m + 1):
                arrays = {"trees": np.array([m + 1]), "levels": np.array([len(v) for v in saved])}
                for mm, lv in enumerate(saved):
                    for li, r in enumerate(lv):
                        arrays[f"t{mm}_l{li}"] = r
                ckpt.save(m + 1, arrays)
        trees.append(t)
        tw.append(w)
        f += w * predict_tree(t, eng.x)
        if fv is not None:
            fv += w * predict_tree(t, xv)
            num = comm.sum_scalar(float(gbt_loss(loss, fv, yv).sum().item()))
            err = num / max(comm.sum_scalar(float(yv.numel())), 1.0)
            if m == 0:
                best_err, best_m = err, 1
            elif best_err - err < validation_tol * max(err, 0.01):
                break
            elif err < best_err:
                best_err, best_m = err, m + 1
    if fv is not None and best_m:
        trees, tw = trees[:best_m], tw[:best_m]
    return trees, tw
