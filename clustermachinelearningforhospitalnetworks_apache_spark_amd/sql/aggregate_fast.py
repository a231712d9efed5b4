"""Columnar group-by: the batch ``groupBy().agg()`` result built from device tensors end to end.

``group_fast.tensor_partials`` gives every rank its per-group partials as tensors (groups in
first-appearance order). Instead of turning them into Python tuples and merging dictionaries
(``group.gather_partials`` / ``final_row``), this path

1. all-gathers each rank's group keys (one row per local group, strings as dictionary codes) and
   codes them jointly — the global groups, in the first-seen (rank, local first appearance) order
   the row-loop merge produces;
2. all-gathers the partial tensors and merges them rank block by rank block (inside a block every
   group appears once, so each step is a duplicate-free scatter): counts and integer sums add,
   min / max reduce, first / last pick the earliest / latest rank holding a value, and
   (count, sum, mean, M2) follow the same sequential Chan et al. update as ``group._merge`` — from
   the same partials the results are the Python merge's, bit for bit (the local float partials are
   ``index_add_`` sums: on the GPU their last bits depend on atomic order);
3. finishes sum / avg / variance / stddev (the moment merge and the final division / square root
   run in numpy over one value per group and rank: IEEE-rounded f64, identical on every device)
   and places global group g on rank g % world (``rows_round_robin``'s placement) as device columns.

High-cardinality aggregations (a group per patient or per admission, not per hospital) therefore
never build per-group Python objects. Time-window and session keys, custom aggregates
(``Summarizer``) and the aggregates ``group_fast`` declines use the row-loop merge.
"""
from __future__ import annotations

from typing import List, Optional

import numpy as np
import torch

from . import types as T
from .column import ColumnData

ENABLED = True


def _concat(blocks: List[ColumnData], dtype) -> ColumnData:
    from .relational_fast import _dict_column, _merge_str
    if blocks and blocks[0].is_host:
        if isinstance(dtype, T.StringType):
            return _dict_column(*_merge_str(blocks), dtype)
        from .relational_fast import _host_values
        vals = np.concatenate([_host_values(b) for b in blocks])
        ok = np.asarray([v is not None for v in vals], dtype=bool)
        return ColumnData(vals, None if ok.all() else ok, dtype)
    v = torch.cat([b.values for b in blocks])
    ok = torch.cat([b.valid_mask().to(v.device) for b in blocks])
    return ColumnData(v, ok, dtype)


def device_aggregate(df, keys, exprs):
    """``group.aggregate`` on device columns, or None (then the row-loop merge runs)."""
    from . import group_fast
    from .group import _result_type
    from .relational_fast import _blocks, _counts, _key_kind, _rerank, _tuple_codes
    from .window import SessionWindow, TimeWindow
    if not ENABLED or not group_fast.ENABLED:
        return None
    comm, dev = df._comm, df._device
    ok = not any(isinstance(k, (TimeWindow, SessionWindow)) for k in keys)
    tp = group_fast.tensor_partials(df, keys, exprs) if ok else None
    ok = tp is not None and all(p is None or p["kind"] != "custom" for p in tp.parts) and \
        all(_key_kind(c) is not None for c in tp.key_cols)
    if comm.is_distributed:
        ok = all(comm.allgather_object(ok))
    if not ok:
        return None
    W, me = comm.world_size, comm.rank
    gl = _counts(comm, tp.G)                       # local groups per rank
    offs = np.cumsum([0] + gl)
    E = int(offs[-1])                              # gathered entries (rank-major)
    # ---- global groups, first-seen order
    kblocks = [_blocks(cd.take(tp.first_rows), comm, dev) for cd in tp.key_cols]
    if keys:
        code, card = _rerank(_tuple_codes(kblocks, dev, null_equal=True))  # dense: every code occurs
    else:
        code, card = torch.zeros(E, dtype=torch.int64, device=dev), 1 if E else 0
    pos = torch.arange(E, device=dev)
    firstpos = torch.full((card,), E, dtype=torch.int64, device=dev).scatter_reduce_(0, code, pos, "amin")
    order = torch.argsort(firstpos)
    fid_of_code = torch.empty_like(order)
    fid_of_code[order] = torch.arange(card, device=dev)
    fid = fid_of_code[code]                        # final group of every entry
    G = card
    first_entry = firstpos[order]                  # entry holding each final group's key
    mine = torch.arange(me, max(G, me), W, device=dev)  # round-robin placement (none when me >= G)
    cols, fields = {}, []

    def gathered(t):
        return comm.allgather_cat(t.contiguous()) if comm.is_distributed else t

    blk = [slice(int(offs[r]), int(offs[r + 1])) for r in range(W)]
    for sp, pt in zip(tp.specs, tp.parts):
        name = sp[1]
        if pt is None:  # grouping column
            j = sp[2]
            kd = tp.key_types[j]
            col = _concat(kblocks[j], kd).take(first_entry[mine])
            cols[name] = col
            fields.append(T.StructField(name, kd, True))
            continue
        kind, fn = pt["kind"], sp[2].fn
        rtype = _result_type(fn, sp[4], getattr(sp[2], "arg", None))
        cnt_e = gathered(pt["cnt"])
        cnt = torch.zeros(G, dtype=torch.int64, device=dev).index_add_(0, fid, cnt_e)
        has = cnt > 0
        if kind == "n":
            val, valid = cnt, None
        elif kind in ("min", "max"):
            v = gathered(pt["val"])
            if v.is_floating_point():
                fill = float("inf") if kind == "min" else float("-inf")
            else:
                info = torch.iinfo(v.dtype)
                fill = info.max if kind == "min" else info.min
            v = torch.where(cnt_e > 0, v, torch.full_like(v, fill))
            val = torch.full((G,), fill, dtype=v.dtype, device=dev)
            val.scatter_reduce_(0, fid, v, "amin" if kind == "min" else "amax", include_self=True)
            valid = has
        elif kind in ("first", "last"):
            src = pt["cd"].take(pt["rows"])
            vblocks = _blocks(src, comm, dev)
            e = torch.where(cnt_e > 0, pos, torch.full_like(pos, E if kind == "first" else -1))
            pick = torch.full((G,), E if kind == "first" else -1, dtype=torch.int64, device=dev)
            pick.scatter_reduce_(0, fid, e, "amin" if kind == "first" else "amax", include_self=True)
            from .relational_fast import _take_nullable
            allv = _concat(vblocks, pt["cd"].dtype)
            pick = torch.where(has, pick, torch.full_like(pick, -1))
            col = _take_nullable(allv, pick[mine])
            cols[name] = col
            fields.append(T.StructField(name, rtype, True))
            continue
        elif kind == "isum":
            s = torch.zeros(G, dtype=torch.int64, device=dev).index_add_(0, fid, gathered(pt["sum"]))
            val, valid = s, has
        else:
            # sequential Chan et al. merge over rank blocks (group._merge's order and arithmetic), in
            # numpy on the host: IEEE-rounded f64 division and sqrt, so the values are the Python
            # merge's bit for bit on any device (one value per group and rank crosses the link)
            s_e, mu_e, m2_e = (gathered(pt[k]).cpu().numpy() for k in ("sum", "mu", "m2"))
            ce = cnt_e.cpu().numpy().astype(np.float64)
            fid_h = fid.cpu().numpy()
            n = np.zeros(G)
            mean = np.zeros(G)
            m2 = np.zeros(G)
            s = np.zeros(G)
            for b in blk:
                if b.stop == b.start:
                    continue
                g = fid_h[b]
                nb = ce[b]
                live = nb > 0
                n0, mean0, m20 = n[g], mean[g], m2[g]
                delta = mu_e[b] - mean0
                tot = n0 + nb
                safe = np.where(live, tot, 1.0)
                n[g] = np.where(live, tot, n0)
                mean[g] = np.where(live, mean0 + delta * nb / safe, mean0)
                m2[g] = np.where(live, m20 + m2_e[b] + delta * delta * n0 * nb / safe, m20)
                s[g] = np.where(live, s[g] + s_e[b], s[g])
            has_h = n > 0
            nz = np.where(has_h, n, 1.0)
            valid = has
            if fn == "sum":
                res = s
            elif fn == "avg":
                res = s / nz
            else:
                var_pop = np.maximum(m2 / nz, 0.0)
                if fn in ("var_pop", "stddev_pop"):
                    res = var_pop if fn == "var_pop" else np.sqrt(var_pop)
                else:
                    big = n >= 2
                    var = var_pop * n / np.where(big, n - 1, 1.0)
                    res = var if fn == "variance" else np.sqrt(var)
                    valid = torch.as_tensor(big, device=dev)
            val = torch.from_numpy(res).to(dev)
        out = val[mine]
        tdt = rtype.torch_dtype
        if tdt is not None and out.dtype != tdt:
            out = out.to(tdt)
        vm = None if valid is None else valid[mine]
        cols[name] = ColumnData(out, None if vm is None or bool(vm.all()) else vm, rtype)
        fields.append(T.StructField(name, rtype, True))
    from .dataframe import DataFrame
    return DataFrame(df._session, T.StructType(fields), cols, int(mine.numel()), mine.to(torch.int64), dev)
