"""Shared helpers for the golden-fixture tests (tests/golden/*.npz, made by oracle/gen_golden.py
from the reference's own head code)."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def check_array(fx, key, got, rtol, atol):
    """Compare `got` with fixture entry `key`, or with its summary (rows/cols/samples)."""
    import oracle.golden_inputs as GI
    got = np.asarray(got, dtype=np.float64)
    if key in fx:
        np.testing.assert_allclose(got.reshape(fx[key].shape), fx[key], rtol=rtol, atol=atol,
                                   err_msg=key)
        return
    summ = GI.summarize(got)
    assert np.array_equal(summ["idx"], fx[f"{key}_idx"]), key
    # row/column sums accumulate many terms: scale atol with the summed length
    n_r, n_c = (got.shape[1] if got.ndim > 1 else 1), got.shape[0]
    np.testing.assert_allclose(summ["samples"], fx[f"{key}_samples"], rtol=rtol, atol=atol,
                               err_msg=key + " samples")
    np.testing.assert_allclose(summ["rows"], fx[f"{key}_rows"], rtol=rtol, atol=atol * n_r,
                               err_msg=key + " rows")
    np.testing.assert_allclose(summ["cols"], fx[f"{key}_cols"], rtol=rtol, atol=atol * n_c,
                               err_msg=key + " cols")
