"""CG parity bars shared by every GPU CG test (history and solution against the oracle).

The GPU sums its reductions in another order than the oracle (per-block partials, fixed-order
tree), so CG iterates differ at rounding level: measured max relative ||z_k|| difference about
1e-13 on the 7-point operator (r01 smoke: 5.9e-14). The bars sit two orders above that, tight
enough that a wrong finalize order, null-space shift or deferred-x bug fails them.

Set PB_MARGINS_FILE to append every measured margin as a JSON line (GPU runs record them under
gpurun_out/ so the committed profiles show how much room each bar leaves).
"""
import json
import os

import numpy as np

HIST_RTOL = 1e-11   # every ||z_k|| relative to the oracle's
# SOR / MG preconditioned CG: the V-cycle is bit-identical to the oracle's, but 13 iterations take
# the norm down 10 orders, so the rounding-level residual differences weigh more (measured max
# 7.0e-12 at 64^3, gpurun_out r02 margins)
HIST_RTOL_PC = 5e-11
X_RTOL = 1e-10      # max |x - x_oracle| relative to max |x_oracle|


def _record(kind, value, bar, tag):
    path = os.environ.get("PB_MARGINS_FILE")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps({"kind": kind, "value": float(value), "bar": bar,
                                "test": os.environ.get("PYTEST_CURRENT_TEST", tag)}) + "\n")


def hist_rel(hist, ho):
    hist, ho = np.asarray(hist), np.asarray(ho)
    assert hist.shape == ho.shape, (hist.shape, ho.shape)
    return float(np.max(np.abs(hist - ho) / ho)) if ho.size else 0.0


def check_history(hist, ho, bar=HIST_RTOL, tag=""):
    rel = hist_rel(hist, ho)
    _record("history", rel, bar, tag)
    assert rel < bar, f"max relative ||z_k|| difference {rel:.3e} >= {bar:.0e} {tag}"
    return rel


def check_x(xs, xo, bar=X_RTOL, scale=None, tag=""):
    xs, xo = np.asarray(xs), np.asarray(xo)
    s = float(np.max(np.abs(xo))) if scale is None else scale
    rel = float(np.max(np.abs(xs - xo))) / s if s > 0 else float(np.max(np.abs(xs - xo)))
    _record("x", rel, bar, tag)
    assert rel <= bar, f"max |x - x_oracle| / max|x_oracle| = {rel:.3e} > {bar:.0e} {tag}"
    return rel
