"""Measured parity errors, kept on file.

``check(metric, value, bound)`` asserts ``value <= bound`` (or ``<`` with strict=True) and appends
{test, metric, value, bound, ratio} as one JSON line to ``gpurun_out/parity_metrics.jsonl`` (merged back
from the GPU box; a copy of each round's file is committed under ``profiles/rNN/``), so the margin of
every bounded comparison is on record, not only pass / fail.  ``TMAE_PARITY_LOG`` overrides the path.
"""
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _path():
    return os.environ.get("TMAE_PARITY_LOG") or os.path.join(ROOT, "gpurun_out", "parity_metrics.jsonl")


def record(metric, value, bound=None, **extra):
    test = os.environ.get("PYTEST_CURRENT_TEST", "?").split(" ")[0]
    rec = {"test": test, "metric": metric, "value": float(value)}
    if bound is not None:
        rec["bound"] = float(bound)
        rec["ratio"] = float(value) / float(bound) if bound else None
    rec.update(extra)
    try:
        p = _path()
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "a") as fh:
            fh.write(json.dumps(rec) + "\n")
    except OSError:
        pass


def check(metric, value, bound, strict=True, **extra):
    record(metric, value, bound, **extra)
    ok = value < bound if strict else value <= bound
    assert ok, f"{metric}: {value:.3e} exceeds bound {bound:.1e}"
