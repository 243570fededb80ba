"""Drop-in for ``sctools.stats`` (reference: src/sctools/stats.py:4-27).

Only the float epilogue of ``Barcodes.effective_diversity`` lives here: the per-position
base counts are tallied on the GPU (``sct_base_frequency``, an (L, 4) table) and turned
into base-4 Shannon entropies on the host.  The arithmetic is the reference's, step for
step (normalise, natural log divided by log 4, zero probabilities contribute 0, sum,
absolute value), so the float64 results agree bit for bit with the reference's.
"""

import numpy as np

__all__ = ["base4_entropy"]


def base4_entropy(x, axis=1):
    """Base-4 entropy of the distribution(s) held in ``x`` along ``axis``; each value lies
    in [0, 1] for four outcomes (a uniform A/C/G/T column gives 1).

    :param np.array x: counts or frequencies, one or more dimensions
    :param axis: the axis holding the outcomes; 1 (default) = rows of a (positions, 4) table
    :return np.array: ``x`` with ``axis`` reduced away
    """
    totals = np.sum(x, axis=axis)
    p = np.divide(x, totals[:, None] if axis == 1 else totals)
    with np.errstate(divide='ignore'):
        log4p = np.log(p) / np.log(4)
    log4p[np.isinf(log4p)] = 0  # an outcome never seen adds nothing (not -inf * 0)
    return np.abs(-np.sum(p * log4p, axis=axis))
