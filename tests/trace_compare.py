"""Tie-aware comparison of CLEAN component traces (test harness).

The GPU computes the scale convolutions in float32 (the reference: FFTW
float) and the oracle in float64, so the two engines see the same images up
to rounding. They take the same decisions wherever the decision's two sides
differ by more than that rounding. The oracle records, for every component,
the smallest gap between the two sides of any decision taken since the
previous component (`margin`: argmax runner-up, loop-continue threshold,
scale selection/activation; oracle/oracle.h Component), and the component's
|peak| (`value`). This module finds the first component where the traces
differ and checks that the oracle's margin there, relative to that peak, is
below `rtol`: a divergence is accepted only at a near-tie.
"""
import numpy as np


class TraceComparison:
    def __init__(self, n_gpu, n_oracle, first_divergence, margin_rel):
        self.n_gpu, self.n_oracle = n_gpu, n_oracle
        self.first_divergence = first_divergence  # None: identical
        self.margin_rel = margin_rel              # oracle margin there / |peak|

    @property
    def identical(self):
        return self.first_divergence is None

    @property
    def matched(self):
        """Length of the identical prefix."""
        return min(self.n_gpu, self.n_oracle) if self.identical else self.first_divergence

    def __repr__(self):
        if self.identical:
            return f"traces identical ({self.n_gpu} components)"
        return (f"identical for {self.first_divergence} of {self.n_oracle} oracle / "
                f"{self.n_gpu} GPU components, then a decision with oracle margin "
                f"{self.margin_rel:.3g} x |peak|")


def compare(gpu, oracle, margins, values):
    """gpu, oracle: (n, k) integer traces; margins/values: len(oracle) + 1
    entries (the last one is the end-of-run decision)."""
    gpu = np.asarray(gpu).reshape(len(gpu), -1)
    oracle = np.asarray(oracle).reshape(len(oracle), -1)
    n = min(len(gpu), len(oracle))
    diff = np.nonzero(np.any(gpu[:n] != oracle[:n], axis=1))[0]
    if len(diff):
        k = int(diff[0])
    elif len(gpu) != len(oracle):
        k = n  # one engine stopped earlier: the end-of-loop decisions
    else:
        return TraceComparison(len(gpu), len(oracle), None, None)
    m = float(margins[min(k, len(margins) - 1)])
    v = float(values[min(k, len(values) - 1)])
    if k >= len(oracle) and len(oracle):
        v = float(values[len(oracle) - 1])
    return TraceComparison(len(gpu), len(oracle), k, m / max(abs(v), 1e-30))


def assert_tie_aware(gpu, oracle, margins, values, rtol, min_prefix=0):
    c = compare(gpu, oracle, margins, values)
    if not c.identical:
        assert c.margin_rel <= rtol, (
            f"trace diverges at component {c.first_divergence} where the oracle's "
            f"decision margin is {c.margin_rel:.3g} x |peak| > {rtol:g}: not a near-tie "
            f"({c})")
        assert c.first_divergence >= min_prefix, c
    return c
