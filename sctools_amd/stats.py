"""Drop-in for ``sctools.stats`` (src/sctools/stats.py).

``base4_entropy`` is the float epilogue of ``Barcodes.effective_diversity``: a
(L, 4) table of base counts comes back from the GPU (``sct_base_frequency``) and
this numpy code turns it into per-position entropies, op for op as stats.py:4-27
does so the float64 results match bit for bit.
"""

import numpy as np

__all__ = ["base4_entropy"]


def base4_entropy(x, axis=1):
    """Entropy of x in base 4 across ``axis`` (1 = across the 4 nucleotide columns).

    :param np.array x: array of dimension one or more containing numeric types
    :param axis: (default 1) axis to reduce
    :return np.array: entropies bounded in [0, 1]
    """
    if axis == 1:
        x = np.divide(x, np.sum(x, axis=axis)[:, None])
    else:
        x = np.divide(x, np.sum(x, axis=axis))

    with np.errstate(divide='ignore'):
        r = np.log(x) / np.log(4)

    # convention: 0 * log(0) = 0, != -INF.
    r[np.isinf(r)] = 0

    return np.abs(-1 * np.sum(x * r, axis=axis))
