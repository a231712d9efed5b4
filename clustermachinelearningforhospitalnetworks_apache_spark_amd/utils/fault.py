"""Fault injection: named crash points the tests arm through ``CML_FAULT``.

``CML_FAULT`` is a comma-separated list of ``point`` or ``point=arg`` entries, e.g.
``stream.after_offsets=2`` (raise once batch 2's offsets are logged but before its commit),
``kmeans.iteration=3`` (raise at the start of Lloyd iteration 3), ``ml.save`` (raise after a
model's metadata is written, before its data). ``maybe_fail(point, arg)`` raises
``InjectedFault`` when armed for that point (and that arg, if one was given). The faults model
a process dying at the worst moment: tests then restart and check that checkpoint / resume /
exactly-once logic repairs the state.
"""
from __future__ import annotations

import os
from typing import Optional


class InjectedFault(RuntimeError):
    pass


def _armed():
    spec = os.environ.get("CML_FAULT", "")
    out = {}
    for item in spec.split(","):
        item = item.strip()
        if not item:
            continue
        if "=" in item:
            k, v = item.split("=", 1)
            out.setdefault(k.strip(), set()).add(v.strip())
        else:
            out.setdefault(item, set()).add(None)
    return out


def maybe_fail(point: str, arg: Optional[object] = None) -> None:
    armed = _armed().get(point)
    if not armed:
        return
    if None in armed or (arg is not None and str(arg) in armed):
        raise InjectedFault(f"injected fault at {point}" + ("" if arg is None else f" ({arg})"))
